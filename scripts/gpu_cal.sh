#!/bin/bash
# Calibration + A/B session: gather microbenchmark (timing, then a FETCH_SIZE pass), C2 with/without the plan-bytes
# counter, C3 with/without lean tables.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/cal
export TMPDIR=/tmp
set -o pipefail
timeout -k 10 180 tools/gather_bench 5 > gpurun_out/cal/gather.json 2>&1 || exit $?
cat gpurun_out/cal/gather.json
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/cal/pmc -o pmc --output-format csv -- tools/gather_bench 1 > gpurun_out/cal/gather_pmc.log 2>&1 || exit $?
B="python3 bench.py --steps 10 --warmup 3 --cpu-sample 0"
timeout -k 10 300 $B > gpurun_out/cal/c2_plan.json 2> gpurun_out/cal/c2_plan.log || exit $?
LK_NO_PLANBYTES=1 timeout -k 10 300 $B > gpurun_out/cal/c2_noplan.json 2> gpurun_out/cal/c2_noplan.log || exit $?
timeout -k 10 300 $B --query c3 > gpurun_out/cal/c3_lean.json 2> gpurun_out/cal/c3_lean.log || exit $?
LK_NO_LEAN=1 timeout -k 10 300 $B --query c3 > gpurun_out/cal/c3_nolean.json 2> gpurun_out/cal/c3_nolean.log || exit $?
grep -h "scan kernel" gpurun_out/cal/*.log
