#!/bin/bash
# GPU-box: exemplar parity tests first, then the rest of the GPU suite (stop at the first failure).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_exemplar.py -x -v --timeout 200 --timeout-method thread > gpurun_out/ex.log 2>&1
rc=$?; grep -E "PASS|FAIL|ERROR|passed|failed|Error" gpurun_out/ex.log | tail -30; [ $rc -eq 0 ] || exit $rc
if [ -n "$FULL" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > gpurun_out/tests.log 2>&1
  rc=$?; grep -E "passed|failed|error" gpurun_out/tests.log | tail -3; [ $rc -eq 0 ] || exit $rc
fi
exit 0
