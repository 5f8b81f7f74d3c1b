#!/bin/bash
# Parity suite on the default build, then A/B benches of the software-pipeline depth (default vs depth-3 build).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab
export TMPDIR=/tmp
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/ab/tests.log 2>&1
  rc=$?; tail -3 gpurun_out/ab/tests.log; [ $rc -eq 0 ] || exit $rc
fi
B="python3 bench.py --steps 10 --warmup 3 --cpu-sample 0"
for q in ${QUERIES:-c2 c3 c4}; do
  timeout -k 10 300 $B --query $q > gpurun_out/ab/${q}_def.json 2> gpurun_out/ab/${q}_def.log || exit $?
  LK_LIB_PATH=$PWD/lakeside_amd/exp/liblakeside_gpu_d2.so timeout -k 10 300 $B --query $q > gpurun_out/ab/${q}_d2.json 2> gpurun_out/ab/${q}_d2.log || exit $?
done
grep -H "scan kernel" gpurun_out/ab/*.log | sed 's/in the call.*//'
