#!/bin/bash
# Local: copy what scripts/gpu_r6_evidence.sh left under gpurun_out/r6e/<query>/ into profiles/ under the round's
# names -- the validated bench line, the rocprofv3 kernel-trace stats and the PMC summary (bench.py attaches the
# latter as roofline.traffic only to runs of the same library build).
cd "$(dirname "$0")/.."
for d in gpurun_out/r6e/*/; do
  q=$(basename "$d")
  [ -s "$d/bench.json" ] && cp "$d/bench.json" "profiles/r06_bench_$q.json"
  ks=$(ls "$d"/prof/bench_kt/*/kt_kernel_stats.csv "$d"/prof/bench_kt/kt_kernel_stats.csv 2>/dev/null | head -1)
  [ -n "$ks" ] && cp "$ks" "profiles/r06_${q}_kernel_stats.csv"
  [ -s "$d/pmc.json" ] && cp "$d/pmc.json" "profiles/r06_pmc_$q.json"
  echo "$q: $(ls profiles/r06_bench_$q.json profiles/r06_${q}_kernel_stats.csv profiles/r06_pmc_$q.json 2>/dev/null | tr '\n' ' ')"
done
