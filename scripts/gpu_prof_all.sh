#!/bin/bash
# GPU-box: rocprofv3 evidence for every bench config: kernel-trace stats + FETCH/WRITE PMC passes (via
# gpu_bench_prof.sh) for $QUERIES; summaries kept under gpurun_out/prof_<query>/ and gpurun_out/pmc_<query>.json.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for q in ${QUERIES:-c3 c4}; do
  QUERY=$q bash scripts/gpu_bench_prof.sh > gpurun_out/prof_$q.log 2>&1 || { tail -5 gpurun_out/prof_$q.log; exit 1; }
  rm -rf gpurun_out/prof_$q && mkdir -p gpurun_out/prof_$q
  cp gpurun_out/prof/bench_kt/kt_kernel_stats.csv gpurun_out/prof_$q/ && cp gpurun_out/prof/bench_kt.json gpurun_out/prof_$q/
  rm -rf gpurun_out/prof
  echo "$q done"; head -3 gpurun_out/prof_$q/kt_kernel_stats.csv
done
