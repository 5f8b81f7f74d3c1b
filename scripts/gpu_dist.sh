#!/bin/bash
# GPU-box: distributed + feature GPU tests, then (unless NOBENCH) the C2 / dense bench lines.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -m gpu -x -v --timeout 800 --timeout-method thread ${TESTS:-tests/test_gpu_dist.py tests/test_gpu_features.py} > gpurun_out/tests_dist.log 2>&1
rc=$?; grep -E "PASS|FAIL|Error|passed|failed" gpurun_out/tests_dist.log | tail -24; [ $rc -eq 0 ] || exit $rc
[ -n "$NOBENCH" ] && exit 0
NOTESTS=1 bash scripts/gpu_round.sh
