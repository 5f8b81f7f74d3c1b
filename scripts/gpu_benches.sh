#!/bin/bash
# GPU-box: bench lines for the configs (QUERIES, default c2 c3 c4 c5); c2-c4 validated at full size against the
# CPU restatement (oracle/cpu), c5 with the CPU leg skipped (CPU_SAMPLE_C5).  Lines -> gpurun_out/bench/<q>.json
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/bench
export TMPDIR=/tmp
for q in ${QUERIES:-c2 c3 c4 c5}; do
  cs=-1; [ "$q" = c5 ] && cs=${CPU_SAMPLE_C5:-0}
  [ "$q" = dense ] && cs=0
  [ "$q" = exemplar ] && cs=0
  timeout -k 10 ${PER:-400} python3 bench.py --query $q --steps ${STEPS:-10} --warmup 3 --cpu-sample $cs $BENCH_ARGS > gpurun_out/bench/$q.json 2> gpurun_out/bench/$q.log || exit $?
  grep -h "scan kernel\|load \|validation\|cpu baseline" gpurun_out/bench/$q.log | sed 's/; in the call.*//'
done
