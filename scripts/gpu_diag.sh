#!/bin/bash
# Diagnostics on 16 C2-sized segments per query: ablation timings + s_memtime phase stamps, then the PMC
# instruction mix (two passes). QUERIES="c2 dense c3".
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
for q in ${QUERIES:-c2 dense c3}; do
  LK_STAMPS=1 timeout -k 10 300 python scripts/profile_scan.py --query $q --segments 16 --steps 3 --ablate ${ABLATE:-0,1} > gpurun_out/diag_$q.log 2>&1 || exit $?
  grep -v amdgpu.ids gpurun_out/diag_$q.log
  timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_WAIT_INST_ANY -d gpurun_out/prof/pmcA_$q -o pmc --output-format csv -- python3 scripts/profile_scan.py --query $q --segments 16 --steps 2 > gpurun_out/prof_pmcA_$q.log 2>&1 || exit $?
  timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_BRANCH SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_BUSY_CU_CYCLES SQ_ACTIVE_INST_ANY -d gpurun_out/prof/pmcB_$q -o pmc --output-format csv -- python3 scripts/profile_scan.py --query $q --segments 16 --steps 2 > gpurun_out/prof_pmcB_$q.log 2>&1 || exit $?
done
python3 scripts/pmc_summary.py gpurun_out/prof
