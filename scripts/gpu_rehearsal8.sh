#!/bin/bash
# World-8 rehearsal of the 8-GPU C4 / C5 paths on the one-GPU box: 8 ranks on device 0 over the host transport (gloo),
# each rank holding the full per-GPU workload (C5: 8 segments x 2^24 rows, a 10M-value container dictionary per
# rank, different on every rank).  Timings of the scan are not 8-GPU numbers (8 ranks share one GPU); the group-dim
# agreement, key-range reduce and row emission stages are the point.  Lines -> gpurun_out/rehearsal8/<q>.json
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/rehearsal8
export TMPDIR=/tmp
for q in ${QUERIES:-c5}; do
  timeout -k 10 ${PER:-900} python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
    --master-port ${PORT:-29517} bench.py --gpus 8 --query $q --comm host --steps ${NSTEPS:-5} --warmup 2 \
    --gen-workers 2 > gpurun_out/rehearsal8/$q.json 2> gpurun_out/rehearsal8/$q.log
  rc=$?; grep -h "rank 0: scan kernel" gpurun_out/rehearsal8/$q.log | tail -1; [ $rc -eq 0 ] || exit $rc
done
exit 0
