#!/bin/bash
# GPU-box A/B of library builds: for every query in $QUERIES one bench line per library in $LIBS ("-" = the in-tree
# build, else a path for LK_LIB_PATH), interleaved per query so box drift hits both alike.  The in-tree build's line is
# validated against oracle/cpu at full size when VALIDATE is set.  Stops at the first failing step.
# Output: gpurun_out/ab/<query>_<lib tag>.json / .log
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab
export TMPDIR=/tmp
for q in ${QUERIES:-count}; do
  for lib in ${LIBS:--}; do
    tag=main; ee=""; cs=0
    if [ "$lib" != "-" ]; then tag=$(basename "$lib" .so | sed 's/^liblakeside_gpu_//'); ee="LK_LIB_PATH=$lib"
    elif [ -n "$VALIDATE" ]; then cs=-1; fi
    env $ee $BENCH_ENV timeout -k 10 ${PER:-400} python3 bench.py --query $q --steps ${STEPS:-10} --warmup 3 --cpu-sample $cs $BENCH_ARGS > gpurun_out/ab/${q}_${tag}.json 2> gpurun_out/ab/${q}_${tag}.log || exit $?
    echo "== $q [$tag] $(grep -h "scan kernel\|validation" gpurun_out/ab/${q}_${tag}.log | sed 's/; in the call.*//' | tr '\n' ' ')"
  done
done
exit 0
