#!/bin/bash
# GPU-box, round 6 evidence at one library build: for every query in $QUERIES a validated bench line, the rocprofv3
# kernel-trace stats of the same command, and FETCH_SIZE / WRITE_SIZE passes (separate runs, counters alone) whose
# summary carries the build's sha (scripts/pmc_traffic.py), so bench.py can attach it as roofline.traffic.
# Stops at the first failing step.  Output under gpurun_out/r6e/<query>/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for q in ${QUERIES:-c2}; do
  d=gpurun_out/r6e/$q
  rm -rf $d && mkdir -p $d/prof
  timeout -k 10 ${PER:-300} python3 bench.py --query $q --steps 10 --warmup 3 --cpu-sample -1 $BENCH_ARGS > $d/bench.json 2> $d/bench.log || exit $?
  echo "== $q"; grep -h "scan kernel\|validation" $d/bench.log | sed 's/; in the call.*//'
  if [ -z "$NOPROF" ]; then
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $d/prof/bench_kt -o kt --output-format csv -- python3 bench.py --query $q --steps 10 --warmup 3 --cpu-sample 0 > $d/prof/bench_kt.json 2> $d/prof/bench_kt.log || exit $?
    timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $d/prof/bench_fetch -o pmc --output-format csv -- python3 bench.py --query $q --steps 3 --warmup 1 --cpu-sample 0 > $d/prof/bench_fetch.json 2> $d/prof/bench_fetch.log || exit $?
    timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $d/prof/bench_write -o pmc --output-format csv -- python3 bench.py --query $q --steps 3 --warmup 1 --cpu-sample 0 > $d/prof/bench_write.json 2> $d/prof/bench_write.log || exit $?
    python3 scripts/pmc_traffic.py $d/prof $q > $d/pmc.json || exit $?
    head -4 $(ls $d/prof/bench_kt/*/kt_kernel_stats.csv $d/prof/bench_kt/kt_kernel_stats.csv 2>/dev/null | head -1)
    grep -h "hbm_bytes_per_launch\|plan_bytes" $d/pmc.json
  fi
done
exit 0
