#!/bin/bash
# Round-3 GPU session: parity suite, bench lines for QUERIES (c2 validated against the CPU restatement by default),
# optional A/B lines (AB="NAME=VAL ..." env settings, each run on AB_QUERIES), optional rocprofv3 kernel-trace stats.
# Every GPU step under its own time limit; the script stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/bench gpurun_out/prof
export TMPDIR=/tmp
STEPS=${STEPS:-tests,bench}
if [[ $STEPS == *tests* ]]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/tests.log 2>&1
  rc=$?; grep -E "passed|failed|error" gpurun_out/tests.log | tail -3; [ $rc -eq 0 ] || exit $rc
fi
if [[ $STEPS == *bench* ]]; then
  for q in ${QUERIES:-c2 c3 c4 c5 dense}; do
    cs=0; [ "$q" = c2 ] && cs=${CPU_SAMPLE_C2:--1}; [ -n "$CPU_ALL" ] && [ "$q" != dense ] && [ "$q" != exemplar ] && [ "$q" != tag ] && cs=-1; [ -n "$CPU_ALL" ] && [ "$q" = c5 ] && cs=1
    timeout -k 10 400 python3 bench.py --query $q --steps ${NSTEPS:-10} --warmup 3 --cpu-sample $cs $BENCH_ARGS > gpurun_out/bench/$q.json 2> gpurun_out/bench/$q.log
    rc=$?; grep -h "scan kernel" gpurun_out/bench/$q.log | sed 's/; in the call.*//'; [ $rc -eq 0 ] || exit $rc
  done
fi
if [[ $STEPS == *ab* ]]; then
  for setting in $AB; do
    for q in ${AB_QUERIES:-c3}; do
      tag=$(echo "$setting" | tr '=/.' '___')
      timeout -k 10 400 env $setting python3 bench.py --query $q --steps ${NSTEPS:-10} --warmup 3 --cpu-sample 0 > gpurun_out/bench/${q}_$tag.json 2> gpurun_out/bench/${q}_$tag.log
      rc=$?; echo "$setting $q: $(grep -h 'scan kernel' gpurun_out/bench/${q}_$tag.log | sed 's/; in the call.*//')"; [ $rc -eq 0 ] || exit $rc
    done
  done
fi
if [[ $STEPS == *prof* ]]; then
  for q in ${PROF_QUERIES:-c2}; do
    timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/kt_$q -o kt --output-format csv -- python3 bench.py --query $q --steps 10 --warmup 3 --cpu-sample 0 > gpurun_out/prof/kt_$q.json 2> gpurun_out/prof/kt_$q.log
    rc=$?; tail -1 gpurun_out/prof/kt_$q.log; [ $rc -eq 0 ] || exit $rc
  done
fi
exit 0
