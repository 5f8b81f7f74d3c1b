#!/bin/bash
# Quick iteration: parity subset + C2/C3/C4 benches (default build).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/q
export TMPDIR=/tmp
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_hash.py -x -q --timeout 400 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/q/tests.log 2>&1
  rc=$?; tail -3 gpurun_out/q/tests.log; [ $rc -eq 0 ] || exit $rc
fi
B="python3 bench.py --steps 10 --warmup 3 --cpu-sample 0"
for q in ${QUERIES:-c2 c3 c4}; do
  timeout -k 10 300 $B --query $q $BENCH_ARGS > gpurun_out/q/${q}.json 2> gpurun_out/q/${q}.log || exit $?
done
grep -H "scan kernel" gpurun_out/q/*.log | sed 's/; in the call.*//'
