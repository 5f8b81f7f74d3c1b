#!/bin/bash
# GPU-box: full GPU suite (optional), then bench lines for QUERIES (default "c2 dense"), each step time-limited.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
if [ -z "$NOTESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/tests.log 2>&1
  rc=$?; grep -E "FAIL|Error|passed|failed" gpurun_out/tests.log | tail -8; [ $rc -eq 0 ] || exit $rc
fi
for q in ${QUERIES:-c2 dense}; do
  timeout -k 10 600 python3 bench.py --query $q --steps 10 --warmup 3 --cpu-sample ${CPU_SAMPLE:-0} > gpurun_out/bench_$q.json 2> gpurun_out/bench_$q.log || exit $?
  grep "scan kernel" gpurun_out/bench_$q.log | tail -1
done
exit 0
