#!/bin/bash
# GPU-box: parity tests (verbose, per-test timeouts), smoke, then optional bench queries (QUERIES="c3 c4").
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASS|FAIL|ERROR|passed|failed" gpurun_out/pytest_gpu.log | tail -60
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -3 gpurun_out/smoke.log
[ $rc -eq 0 ] || exit $rc
for q in $QUERIES; do
  timeout -k 10 600 python bench.py --query $q --steps 5 --warmup 2 --cpu-sample 0 > gpurun_out/bench_$q.json 2> gpurun_out/bench_$q.log || exit $?
  tail -2 gpurun_out/bench_$q.log
done
