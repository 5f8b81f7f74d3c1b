#!/bin/bash
# GPU-box, round 6: the GPU suite (optionally under an env such as LK_EARLY_FIRST=1 via TEST_ENV), then bench lines
# for $QUERIES under each env in $ENVS ("-" = none), then optional rocprofv3 kernel stats for $PROF_QUERIES.
# Stops at the first failing step.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r6
export TMPDIR=/tmp
if [ -z "$NOTESTS" ]; then
  env $TEST_ENV timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${TESTS:-} > gpurun_out/r6/tests.log 2>&1
  rc=$?; tail -5 gpurun_out/r6/tests.log; [ $rc -eq 0 ] || exit $rc
fi
for e in ${ENVS:--}; do
  ee=""; [ "$e" != "-" ] && ee=$(echo "$e" | tr "+" " ")
  tag=$(echo "${e}" | tr '=,+/' '____')
  for q in ${QUERIES:-}; do
    cs=0; [ -n "$VALIDATE" ] && cs=-1
    env $ee timeout -k 10 ${PER:-400} python3 bench.py --query $q --steps ${STEPS:-10} --warmup 3 --cpu-sample $cs $BENCH_ARGS > gpurun_out/r6/${q}_${tag}.json 2> gpurun_out/r6/${q}_${tag}.log || exit $?
    echo "== $q [$e]"; grep -h "scan kernel\|validation" gpurun_out/r6/${q}_${tag}.log | sed 's/; in the call.*//'
  done
done
for q in ${LOOPBACK_QUERIES:-}; do   # lk_eval_pushdown_dist on a world-1 RCCL loopback communicator
  cs=0; [ -n "$VALIDATE" ] && cs=-1
  timeout -k 10 ${PER:-400} python3 bench.py --query $q --dist-loopback --steps ${STEPS:-10} --warmup 3 --cpu-sample $cs > gpurun_out/r6/${q}_loopback.json 2> gpurun_out/r6/${q}_loopback.log || exit $?
  echo "== $q [loopback]"; grep -h "scan kernel\|validation" gpurun_out/r6/${q}_loopback.log | sed 's/; in the call.*//'
done
for spec in ${MULTI:-}; do   # N-rank bench lines: "<query>:<N>:<comm>" (bench.py launches the N rank processes itself)
  q=${spec%%:*}; rest=${spec#*:}; n=${rest%%:*}; cm=${rest#*:}
  timeout -k 10 ${PER_MULTI:-900} python3 bench.py --query $q --gpus $n --comm $cm --steps ${STEPS:-10} --warmup 3 > gpurun_out/r6/${q}_n${n}_${cm}.json 2> gpurun_out/r6/${q}_n${n}_${cm}.log || exit $?
  echo "== $q [N=$n $cm]"; grep -h "scan kernel\|validation\|communicator" gpurun_out/r6/${q}_n${n}_${cm}.log | sed 's/; in the call.*//'
done
for q in ${PROF_QUERIES:-}; do
  env $PROF_ENV timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r6/kt_$q -o kt --output-format csv -- python3 bench.py --query $q --steps 5 --warmup 2 --cpu-sample 0 > gpurun_out/r6/kt_$q.json 2> gpurun_out/r6/kt_$q.log || exit $?
  head -6 gpurun_out/r6/kt_$q/kt_kernel_stats.csv
done
exit 0
