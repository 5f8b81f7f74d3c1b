#!/bin/bash
# GPU-box: run the given GPU test files (default: the whole -m gpu suite), verbose, per-test timeouts; log under
# gpurun_out/.  Usage: TESTS="tests/test_gpu_globs.py tests/test_gpu_dist.py" bash scripts/gpu_pytest.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 ${LIMIT:-1000} python -u -m pytest ${TESTS:-tests} -m gpu -x -v --timeout ${PER_TEST:-300} --timeout-method thread -p no:cacheprovider ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed|Error" gpurun_out/pytest_gpu.log | tail -40
echo "pytest rc=$rc"
exit $rc
