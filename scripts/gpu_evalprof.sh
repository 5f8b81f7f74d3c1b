#!/bin/bash
# GPU-box: the default bench line (C2 + CPU baseline), then rocprofv3 kernel traces of the bench for the queries
# in $QUERIES (where eval time goes outside the scan kernel).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
timeout -k 10 600 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.log || exit $?
tail -2 gpurun_out/bench_default.log
for q in $QUERIES; do
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/kt_$q -o kt --output-format csv -- python3 bench.py --query $q --steps 5 --warmup 2 --cpu-sample 0 > gpurun_out/prof/kt_$q.json 2> gpurun_out/prof/kt_$q.log || exit $?
  head -8 gpurun_out/prof/kt_$q/kt_kernel_stats.csv
done
