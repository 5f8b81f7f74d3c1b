#!/bin/bash
# Lean-kernel round: new feature tests + parity subset, then C2/C3 benches with the lean split on and off.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/lean
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_features.py tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread > gpurun_out/lean/tests.log 2>&1
rc=$?; grep -E "passed|failed|error|FAIL" gpurun_out/lean/tests.log | tail -5; [ $rc -eq 0 ] || exit $rc
B="python3 bench.py --steps 10 --warmup 3 --cpu-sample 0"
timeout -k 10 300 $B --query c2 > gpurun_out/lean/c2.json 2> gpurun_out/lean/c2.log || exit $?
LK_NO_LEAN_SPLIT=1 timeout -k 10 300 $B --query c2 > gpurun_out/lean/c2_general.json 2> gpurun_out/lean/c2_general.log || exit $?
grep -h "scan kernel" gpurun_out/lean/c2.log gpurun_out/lean/c2_general.log | sed 's/; in the call.*//'
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/lean/kt -o kt --output-format csv -- python3 bench.py --query c2 --steps 10 --warmup 3 --cpu-sample 0 > gpurun_out/lean/kt.json 2> gpurun_out/lean/kt.log || exit $?
head -4 gpurun_out/lean/kt/kt_kernel_stats.csv
