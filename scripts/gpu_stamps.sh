#!/bin/bash
# Per-phase cycle stamps (LK_STAMPS) and ablations of the scan kernel on 16 segments of $QUERY (default c2).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
LK_STAMPS=1 timeout -k 10 300 python scripts/profile_scan.py --query ${QUERY:-c2} --segments 16 --steps 2 --ablate ${ABLATE:-0,1} 2>&1 | grep -v amdgpu.ids
