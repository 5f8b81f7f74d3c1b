#!/bin/bash
# rocprofv3 evidence for the bench line: kernel-trace stats of the bench command itself, then FETCH_SIZE and
# WRITE_SIZE passes (separate runs, counters only), and a FETCH_SIZE pass on the dense query (every row read)
# to calibrate the counter for this kernel's access widths. Summary -> gpurun_out/pmc_<query>.json.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
Q=${QUERY:-c2}
rm -rf gpurun_out/prof/bench_kt gpurun_out/prof/bench_fetch gpurun_out/prof/bench_write gpurun_out/prof/dense_fetch
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/bench_kt -o kt --output-format csv -- python3 bench.py --query $Q --steps 10 --warmup 3 --cpu-sample 0 > gpurun_out/prof/bench_kt.json 2> gpurun_out/prof/bench_kt.log || exit $?
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/prof/bench_fetch -o pmc --output-format csv -- python3 bench.py --query $Q --steps 3 --warmup 1 --cpu-sample 0 > gpurun_out/prof/bench_fetch.json 2> gpurun_out/prof/bench_fetch.log || exit $?
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/prof/bench_write -o pmc --output-format csv -- python3 bench.py --query $Q --steps 3 --warmup 1 --cpu-sample 0 > gpurun_out/prof/bench_write.json 2> gpurun_out/prof/bench_write.log || exit $?
if [ -z "$NODENSE" ]; then
  timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/prof/dense_fetch -o pmc --output-format csv -- python3 bench.py --query dense --steps 3 --warmup 1 --cpu-sample 0 > gpurun_out/prof/dense_fetch.json 2> gpurun_out/prof/dense_fetch.log || exit $?
fi
mkdir -p gpurun_out/prof_$Q && cp -r gpurun_out/prof/bench_* gpurun_out/prof_$Q/ && python3 scripts/pmc_traffic.py gpurun_out/prof $Q > gpurun_out/pmc_$Q.json && cat gpurun_out/pmc_$Q.json
