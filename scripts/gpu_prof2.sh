#!/bin/bash
# Where the scan kernel's time goes: per-phase s_memtime stamps (LK_STAMPS) and SQ counters (separate --pmc pass),
# for C2 and C3 on 16 segments.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/p2
export TMPDIR=/tmp
B="python3 bench.py --steps 3 --warmup 1 --cpu-sample 0 --segments 16"
for q in c2 c3; do
  LK_STAMPS=1 timeout -k 10 200 $B --query $q > gpurun_out/p2/${q}_stamps.json 2> gpurun_out/p2/${q}_stamps.log || exit $?
  grep "lk stamps" gpurun_out/p2/${q}_stamps.log | tail -1
  timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY -d gpurun_out/p2/pmc_$q -o pmc --output-format csv -- $B --query $q > gpurun_out/p2/${q}_pmc.json 2> gpurun_out/p2/${q}_pmc.log || exit $?
  timeout -s KILL 200 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INSTS_SMEM -d gpurun_out/p2/pmc2_$q -o pmc --output-format csv -- $B --query $q > gpurun_out/p2/${q}_pmc2.json 2> gpurun_out/p2/${q}_pmc2.log || exit $?
done
