#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
LK_STAMPS=1 timeout -k 10 300 python scripts/profile_scan.py --segments 16 --steps 2 --ablate 0,1,2,3 2>&1 | grep -v amdgpu.ids
