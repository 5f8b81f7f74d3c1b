#!/bin/bash
# Feature tests (test_gpu_features.py), then C2/C3/C4/C5 benches (no CPU baseline) and the C3 split on/off.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/feat
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_features.py -x -v --timeout 300 --timeout-method thread > gpurun_out/feat/tests.log 2>&1
rc=$?; grep -E "PASS|FAIL|passed|failed|Error" gpurun_out/feat/tests.log | tail -12; [ $rc -eq 0 ] || exit $rc
B="python3 bench.py --steps 10 --warmup 3 --cpu-sample 0"
for q in ${QUERIES:-c2 c3 c4 c5}; do
  timeout -k 10 300 $B --query $q > gpurun_out/feat/${q}.json 2> gpurun_out/feat/${q}.log || exit $?
done
LK_NO_LEAN_SPLIT=1 timeout -k 10 300 $B --query c3 > gpurun_out/feat/c3_general.json 2> gpurun_out/feat/c3_general.log || exit $?
grep -H "scan kernel" gpurun_out/feat/*.log | sed 's/; in the call.*//'
