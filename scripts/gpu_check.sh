#!/bin/bash
# GPU-box check: parity tests, smoke, optional short bench. Stops at the first crash-like exit status.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
ok() { local rc=$1; [ "$rc" -eq 0 ] || [ "$rc" -eq 1 ]; }
timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -40 gpurun_out/pytest_gpu.log
ok $rc || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -5 gpurun_out/smoke.log
ok $rc || exit $rc
if [ -n "$BENCH_ARGS" ]; then
  timeout -k 10 900 python bench.py $BENCH_ARGS > gpurun_out/bench.json 2> gpurun_out/bench.log
  rc=$?; echo "bench rc=$rc"; tail -5 gpurun_out/bench.log; cat gpurun_out/bench.json
  exit $rc
fi
