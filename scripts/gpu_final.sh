#!/bin/bash
# GPU-box round evidence: full GPU suite, smoke, an N=2 rehearsal of the multi-rank bench path (host transport,
# two ranks on the one GPU), the default bench line, and rocprofv3 kernel stats of the C2 bench command.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
if [ -z "$NOTESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > gpurun_out/tests.log 2>&1
  rc=$?; grep -E "FAIL|Error|passed|failed" gpurun_out/tests.log | tail -6; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
  rc=$?; tail -2 gpurun_out/smoke.log; [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 5 --warmup 2 --segments ${N2_SEGS:-16} --comm host --cpu-sample 0 > gpurun_out/bench_n2.json 2> gpurun_out/bench_n2.log
rc=$?; tail -1 gpurun_out/bench_n2.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench.json 2> gpurun_out/bench.log
rc=$?; grep -E "scan kernel|validation" gpurun_out/bench.log | tail -2; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/kt_c2 -o kt --output-format csv -- python3 bench.py --query c2 --steps 10 --warmup 3 --cpu-sample 0 > gpurun_out/prof/kt_c2.json 2> gpurun_out/prof/kt_c2.log
rc=$?; grep "scan kernel" gpurun_out/prof/kt_c2.log | tail -1; exit $rc
