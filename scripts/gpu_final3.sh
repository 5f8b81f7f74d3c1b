#!/bin/bash
# Round-3 closing evidence at HEAD: GPU suite, smoke, the default bench line (C2, validated against the CPU
# restatement), rocprofv3 kernel stats + PMC traffic of the same bench command.  Stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/final
export TMPDIR=/tmp
if [ -z "$NOTESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/final/tests.log 2>&1
  rc=$?; grep -E "passed|failed|error" gpurun_out/final/tests.log | tail -2; [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final/smoke.log 2>&1
rc=$?; tail -1 gpurun_out/final/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 bench.py > gpurun_out/final/bench.json 2> gpurun_out/final/bench.log
rc=$?; grep -h "scan kernel\|validation" gpurun_out/final/bench.log | sed 's/; in the call.*//'; [ $rc -eq 0 ] || exit $rc
QUERY=c2 NODENSE=1 bash scripts/gpu_bench_prof.sh > gpurun_out/final/prof.log 2>&1
rc=$?; tail -3 gpurun_out/final/prof.log; exit $rc
