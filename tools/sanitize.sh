#!/bin/bash
# `make sanitize`: the loader harness (tools/load_check.cpp) under ASan + UBSan and under TSan over the golden,
# compressed, PLAIN-fallback, numeric-dictionary, large-dictionary and truncated fixtures, with 1 and 8 load threads;
# the digests must not depend on the thread count or on the instrumentation.  CPU only.
set -euo pipefail
cd "$(dirname "$0")/.."
FIX=build/load_fixtures
python3 tools/make_load_fixtures.py $FIX
FILES="$(ls tests/golden/segments/*.parquet) $(ls $FIX/*.parquet)"
export ASAN_OPTIONS=detect_leaks=1:abort_on_error=1 UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1
export TSAN_OPTIONS=halt_on_error=1:second_deadlock_stack=1
for bin in load_check load_check_asan load_check_tsan; do
  for t in 1 8; do
    echo "== $bin, $t thread(s)"
    build/$bin $t $FILES > build/sanitize_${bin}_$t.out
  done
done
ref=build/sanitize_load_check_1.out
for f in build/sanitize_*.out; do
  cmp -s $ref $f || { echo "digest differs: $f vs $ref"; diff $ref $f | head -20; exit 1; }
done
grep -c "error" $ref | xargs -I{} echo "files failing to load (expected: the truncated fixture): {}"
echo "sanitize: OK ($(grep -c '^dict ' $ref) dictionaries, $(echo $FILES | wc -w) files, identical digests)"
