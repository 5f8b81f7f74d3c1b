// Device helpers shared by the HIP kernels (included by kernels.hip only).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "kernels.hpp"
#include "layout.hpp"

namespace lk {

constexpr int BLOCK = 256;
constexpr int RPT = 4;                 // row slots decoded together in phase 1
constexpr int SLOTS = 8;               // row slots per thread per sub-tile
constexpr int SUBT = BLOCK * SLOTS;    // rows per sub-tile (2048)
constexpr int HCAP = 512;              // LDS hash entries
constexpr int HPROBE = 16;
constexpr int LUT_CAP = 256;           // LDS lookup entries per string column
constexpr unsigned long long EMPTY = ~0ull;
constexpr uint32_t OOB = 0x80000000u;  // buffer offset past num_records: no memory access, reads 0

typedef unsigned int v2u __attribute__((ext_vector_type(2)));

struct LRun {                          // LDS copy of a RunDesc (12 B)
  uint32_t start, off_lit, value;
};

__device__ __forceinline__ unsigned long long dbl_order(double d) {
  unsigned long long u = (unsigned long long)__double_as_longlong(d);
  if (d != d) u = 0x7ff8000000000000ull;     // NaN sorts above +inf (DuckDB orders NaN greatest)
  return (u >> 63) ? ~u : (u | 0x8000000000000000ull);
}
__device__ __forceinline__ double order_dbl(unsigned long long o) {
  if (o == MIN_NAN_ORDER) return __longlong_as_double(0x7ff8000000000000ll);
  unsigned long long u = (o >> 63) ? (o & 0x7fffffffffffffffull) : ~o;
  return __longlong_as_double((long long)u);
}
__device__ __forceinline__ void two_sum(double a, double b, double& s, double& e) {
  s = a + b;
  double bb = s - a;
  e = (a - (s - bb)) + (b - bb);
}

// ---- wave-uniform values: readfirstlane puts them in SGPRs so branches on them stay scalar ----
__device__ __forceinline__ uint32_t uni(uint32_t x) { return __builtin_amdgcn_readfirstlane(x); }
__device__ __forceinline__ const uint8_t* uni_ptr(const uint8_t* p) {
  uint64_t v = reinterpret_cast<uint64_t>(p);
  uint64_t lo = uni(uint32_t(v)), hi = uni(uint32_t(v >> 32));
  return reinterpret_cast<const uint8_t*>((hi << 32) | lo);
}
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const uint8_t* base, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)uni_ptr(base), (short)0, int(uni(bytes)), 0x00020000);
}

// Branch-free run lookup over at most RUN_CAP staged runs: last run whose start <= v.
__device__ __forceinline__ int find_run(const LRun* runs, int n, uint32_t v) {
  static_assert((RUN_CAP & (RUN_CAP - 1)) == 0, "RUN_CAP: power of two");
  int lo = 0;
#pragma unroll
  for (int step = int(RUN_CAP) / 2; step >= 1; step >>= 1) {
    const int m = lo + step;
    const uint32_t st = runs[m < n ? m : n - 1].start;
    lo = (m < n && st <= v) ? m : lo;
  }
  return lo;
}

// Branch-free hybrid RLE/bit-packed value read through a buffer descriptor over the stream: RLE runs read the
// stream's first dword (harmless) and select the run value, so no lane branches around the load.
__device__ __forceinline__ uint32_t hybrid_get_buf(__amdgpu_buffer_rsrc_t rs, const LRun& r, uint32_t v, int bw) {
  const bool lit = (r.off_lit & 0x80000000u) != 0;
  const uint32_t bit = lit ? (v - r.start) * uint32_t(bw) : 0u;
  const uint32_t byte = (lit ? (r.off_lit & 0x7fffffffu) : 0u) + (bit >> 3);
  const v2u w = __builtin_amdgcn_raw_buffer_load_b64(rs, byte & ~3u, 0, 0);
  uint64_t x = ((uint64_t)w.y << 32) | w.x;
  x >>= ((byte & 3u) * 8u + (bit & 7u));
  const uint32_t mask = bw >= 32 ? 0xffffffffu : ((1u << bw) - 1u);
  return lit ? (uint32_t(x) & mask) : r.value;
}

struct Acc {                           // one aggregation cell's partial state
  unsigned long long key;
  uint32_t rows, cnt;
  double hi, lo;                       // SUM: compensated sum
  unsigned long long ext;              // MIN/MAX: ordered bits
};

template <int AGG>
__device__ __forceinline__ void acc_add(Acc& a, bool vvalid, double v) {
  a.rows += 1;
  if (!vvalid) return;
  a.cnt += 1;
  if (AGG == AGG_SUM) {
    double s, e;
    two_sum(a.hi, v, s, e);
    a.hi = s;
    a.lo += e;
  } else if (AGG == AGG_MIN) {
    unsigned long long o = dbl_order(v);
    a.ext = o < a.ext ? o : a.ext;
  } else if (AGG == AGG_MAX) {
    unsigned long long o = dbl_order(v);
    a.ext = o > a.ext ? o : a.ext;
  }
}

// MIN over a NaN row: flagged so the host can keep cells apart whose sharing would hide an all-NaN DuckDB group from
// query-api's NaN-absorbing math.min (eval.cpp, REDO_MIN_APART).  NULL-like group values share a cell row by row,
// so the test is per row (a rarely taken branch; MIN queries only).
template <int AGG>
__device__ __forceinline__ void min_nan_check(const QParams& P, bool vvalid, double v) {
  if (AGG == AGG_MIN && vvalid && v != v) atomicOr(P.flags, FLAG_MIN_NAN);
}

template <int AGG>
__device__ __forceinline__ void acc_reset(Acc& a, unsigned long long key) {
  a.key = key;
  a.rows = 0;
  a.cnt = 0;
  a.hi = 0.0;
  a.lo = 0.0;
  a.ext = (AGG == AGG_MIN) ? ~0ull : 0ull;
}

// DDSketch bin of a value (sketches-java 0.8.2 LogarithmicMapping.index + DDSketch.accept): |v| <= dd_min -> the
// zero bin; index = (int) (ln|v| * multiplier), minus one when negative (LogLikeIndexMapping.index's floor);
// NaN / |v| > dd_max is untrackable (accept throws): FLAG_SKETCH_RANGE.
__device__ __forceinline__ uint32_t dd_bin(const QParams& P, double v) {
  const double a = fabs(v);
  if (!(a <= P.dd_max)) {
    atomicOr(P.flags, FLAG_SKETCH_RANGE);
    return 0u;
  }
  if (a <= P.dd_min) return 0u;
  const double x = log(a) * P.dd_mult;
  const int32_t i = x >= 0.0 ? int32_t(x) : int32_t(x) - 1;
  return uint32_t(1 + DD_BIAS + i) + (v < 0.0 ? DD_HALF : 0u);
}

__device__ __forceinline__ unsigned long long mix64(unsigned long long x) {   // splitmix64 finalizer
  x ^= x >> 30;
  x *= 0xbf58476d1ce4e5b9ull;
  x ^= x >> 27;
  x *= 0x94d049bb133111ebull;
  return x ^ (x >> 31);
}

// Slot of cell key `cell` in a hash-mode table (linear probing; the key is claimed by CAS).  ~0 when the probe
// limit is reached: FLAG_HASH_FULL is raised and the host re-runs the query with a larger table.
__device__ __forceinline__ unsigned long long hash_slot(unsigned long long* keys, unsigned long long mask,
                                                       uint32_t* flags, unsigned long long cell) {
  unsigned long long h = mix64(cell) & mask;
  for (uint32_t p = 0; p < HASH_MAX_PROBE; p++) {
    unsigned long long k = __hip_atomic_load(&keys[h], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (k == EMPTY) {
      k = atomicCAS(&keys[h], EMPTY, cell);
      if (k == EMPTY) return h;
    }
    if (k == cell) return h;
    h = (h + 1) & mask;
  }
  atomicOr(flags, FLAG_HASH_FULL);
  return EMPTY;
}

// Merge a partial cell into the global table (device-scope atomics).  HASH: the table is the hash-mode table
// (a compile-time choice: the probe loop would otherwise cost the dense kernels registers).
template <int AGG, bool HASH = false>
__device__ __forceinline__ void global_merge(const QParams& P, unsigned long long cell, uint32_t rows,
                                             uint32_t cnt, double hi, double lo, unsigned long long ext) {
  if (rows == 0) return;
  if (P.ablate & 4u) return;   // diagnostics only (LK_ABLATE=4): no device atomics (wrong results; the atomics' cost)
  if (HASH) {
    cell = hash_slot(P.hkeys, P.hmask, P.flags, cell);
    if (cell == EMPTY) return;
  }
  if (!(P.lean & (LEAN_NO_ROWS | LEAN_SUM_EXISTS))) atomicAdd(&P.rows[cell], (unsigned long long)rows);
  if (cnt == 0) return;
  if (!(P.lean & (LEAN_NO_CNT | LEAN_NO_ROWS | LEAN_SUM_EXISTS))) atomicAdd(&P.cnt[cell], (unsigned long long)cnt);
  if (AGG == AGG_SUM) {
    if (P.lean & LEAN_SUM_EXISTS) hi = hi + 0.0;   // never -0.0: the empty cell's marker (layout.hpp)
    if (P.exact_sum) {   // exact adds (QParams::exact_sum): no compensation, no returned value to wait for
      __hip_atomic_fetch_add(&P.hi[cell], hi, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return;
    }
    double old = atomicAdd(&P.hi[cell], hi);   // returning atomic: old is exact -> TwoSum recovers the error
    double s, e;
    two_sum(old, hi, s, e);
    // The correction is often exactly 0 (integer-valued data, a first add into an empty cell): adding 0.0 is a
    // no-op, so skip that scattered memory-side atomic (each costs one request to HBM, MI355X_MICROARCH §atomics).
    const double c = lo + e;
    if (c != 0.0) atomicAdd(&P.lo[cell], c);
  } else if (AGG == AGG_MIN) {
    if (ext == NAN_ORDER) atomicOr(P.flags, FLAG_MIN_NAN);   // the general row scan's rows (see min_nan_check)
    atomicMin(&P.ext[cell], ext);
  } else if (AGG == AGG_MAX) {
    atomicMax(&P.ext[cell], ext);
  }
}

// The tile qualifies for scan_lean with `nl` late string columns (uniform: scalar loads).  scan_tiles applies the
// same test to skip it.  Late columns (query columns 3 .. 2 + nl) must hold no NULL over the tile (value index =
// row) or be absent from the segment.
__device__ __forceinline__ bool lean_tile(const QSeg* Sp, uint32_t t, uint32_t nl, uint32_t rows_only) {
  if (!Sp->cols[0].present || !Sp->cols[2].present) return false;
  if (!Sp->cols[1].present && !rows_only) return false;   // COUNT(*) reads no value column
  const TileCol* a = Sp->cols[0].tcols + t;
  const TileCol* c = Sp->cols[2].tcols + t;
  if (Sp->cols[1].present && Sp->cols[1].tcols[t].has_nulls) return false;
  if (a->has_nulls || c->has_nulls || c->kind != PAGE_DICT || c->dict_n > 64u || c->nruns == 0u ||
      c->bw < 1u || c->bw > 6u)
    return false;
  for (uint32_t k = 0; k < nl; k++) {
    if (!Sp->cols[3 + k].present) continue;
    const TileCol* l = Sp->cols[3 + k].tcols + t;
    if (l->has_nulls || l->kind != PAGE_DICT || l->nruns == 0u || l->bw > 32u) return false;
  }
  return true;
}

}  // namespace lk
