#!/bin/bash
# Round-2 GPU session: parity suite, default bench line (C2, validated against the CPU restatement), rocprofv3
# kernel-trace stats of the bench command.  Each GPU step under its own time limit; stop at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
STEPS=${STEPS:-tests,bench,prof}
if [[ $STEPS == *tests* ]]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/tests.log 2>&1
  rc=$?; grep -E "passed|failed|error" gpurun_out/tests.log | tail -3; [ $rc -eq 0 ] || exit $rc
fi
if [[ $STEPS == *bench* ]]; then
  timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 ${BENCH_ARGS:-} > gpurun_out/bench.json 2> gpurun_out/bench.log
  rc=$?; tail -4 gpurun_out/bench.log; [ $rc -eq 0 ] || exit $rc
fi
if [[ $STEPS == *prof* ]]; then
  Q=${QUERY:-c2}
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/kt_$Q -o kt --output-format csv -- python3 bench.py --query $Q --steps 10 --warmup 3 --cpu-sample 0 > gpurun_out/prof/kt_$Q.json 2> gpurun_out/prof/kt_$Q.log
  rc=$?; tail -2 gpurun_out/prof/kt_$Q.log; [ $rc -eq 0 ] || exit $rc
fi
exit 0
