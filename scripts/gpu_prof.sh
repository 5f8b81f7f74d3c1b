#!/bin/bash
# rocprofv3 kernel trace + ablations of the scan kernel on 16 C2 segments.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
timeout -k 10 300 python scripts/profile_scan.py --segments 16 --steps 5 --ablate 0,1,2,3 > gpurun_out/ablate.log 2>&1
rc=$?; cat gpurun_out/ablate.log | tail -6; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/kt -o kt --output-format csv -- python3 scripts/profile_scan.py --segments 16 --steps 5 > gpurun_out/prof_kt.log 2>&1
rc=$?; tail -3 gpurun_out/prof_kt.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY -d gpurun_out/prof/pmc1 -o pmc1 --output-format csv -- python3 scripts/profile_scan.py --segments 16 --steps 2 > gpurun_out/prof_pmc1.log 2>&1
rc=$?; tail -2 gpurun_out/prof_pmc1.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/prof/pmc2 -o pmc2 --output-format csv -- python3 scripts/profile_scan.py --segments 16 --steps 2 > gpurun_out/prof_pmc2.log 2>&1
rc=$?; tail -2 gpurun_out/prof_pmc2.log; exit $rc
