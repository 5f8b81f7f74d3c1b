#!/bin/bash
# Scan-kernel front-end diagnostics on 16 C2-sized segments per query: kernel time, then instruction-cache
# counters (one PMC pass per query). QUERIES="c2 c3 c4".
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
for q in ${QUERIES:-c2 c3 c4}; do
  timeout -k 10 300 python scripts/profile_scan.py --query $q --segments 16 --steps 3 > gpurun_out/time_$q.log 2>&1 || exit $?
  grep -v amdgpu.ids gpurun_out/time_$q.log
  timeout -k 10 300 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_IFETCH SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU -d gpurun_out/prof/pmcIC_$q -o pmc --output-format csv -- python3 scripts/profile_scan.py --query $q --segments 16 --steps 2 > gpurun_out/prof_ic_$q.log 2>&1 || exit $?
done
python3 scripts/pmc_summary.py gpurun_out/prof
