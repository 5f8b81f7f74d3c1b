#!/bin/bash
# PMC instruction mix of the scan kernel on 16 C2 segments, per ablation (ABLATE="0 1"), one counter pass each.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
for ab in ${ABLATE:-0 1}; do
  timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_WAIT_INST_ANY -d gpurun_out/prof/pmcA_${QUERY:-c2}${SUF}_$ab -o pmc --output-format csv -- python3 scripts/profile_scan.py --segments 16 --steps 2 --query ${QUERY:-c2} --ablate $ab $PS_ARGS > gpurun_out/prof_pmcA$ab.log 2>&1 || exit $?
  timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_BRANCH SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU_INT32 SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_BUSY_CU_CYCLES -d gpurun_out/prof/pmcB_${QUERY:-c2}${SUF}_$ab -o pmc --output-format csv -- python3 scripts/profile_scan.py --segments 16 --steps 2 --query ${QUERY:-c2} --ablate $ab $PS_ARGS > gpurun_out/prof_pmcB$ab.log 2>&1 || exit $?
done
python3 scripts/pmc_summary.py gpurun_out/prof > gpurun_out/pmc_mix_${QUERY:-c2}.txt; cat gpurun_out/pmc_mix_${QUERY:-c2}.txt
