// HIP kernels for gfx950 (MI355X): sealed-segment DataExpr scan + table finalize/compaction.
//
// scan_tiles<AGG>: one 256-thread workgroup per tile (a row range inside one page of every column).
//   1. stage each query column's run directory window and, for small dictionaries, the per-query lookup
//      table (dictionary index -> leaf bits | group-dim id) in LDS;
//   2. per 1024-row sub-tile (row = sub + k*256 + tid, so every global access of a wave is contiguous):
//      decode definition levels (ballot + popcount prefix -> value index), decode dictionary indices from
//      the hybrid RLE/bit-packed stream, fold every string column into leaf T/F bitmasks and the group id,
//      run the postfix filter under Kleene logic, and only for passing rows load timestamp + value;
//   3. aggregate: a per-thread register cell (time-sorted rows hit it almost always), spilling to an LDS
//      hash table (LDS atomics; sums as compensated hi/lo via returning-atomic TwoSum), flushed to the
//      global table at tile end with global atomics (count/min/max exact, sums within 1 ulp).
// finalize_*: per output key, combine glob slots (and the name dimension when the query has no groupBys,
//   TimeGroupedSketchAggregator.scala:148-170) and compact non-empty keys in (glob, bucket, group) order.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "kernels.hpp"
#include "layout.hpp"

namespace lk {

constexpr int BLOCK = 256;
constexpr int RPT = 4;                 // rows per thread per sub-tile
constexpr int SUB = BLOCK * RPT;       // rows per sub-tile
constexpr int HCAP = 512;              // LDS hash entries
constexpr int HPROBE = 16;
constexpr int LUT_CAP = 256;           // LDS lookup entries per string column
constexpr int POOL = 2 * MAXQCOL * 64; // LDS run-directory pool (entries)
constexpr unsigned long long EMPTY = ~0ull;

static_assert(2 * MAXQCOL * RUN_CAP <= POOL, "run windows must fit the LDS pool");

struct LRun {                          // LDS copy of a RunDesc (12 B)
  uint32_t start, off_lit, value;
};

__device__ __forceinline__ unsigned long long dbl_order(double d) {
  unsigned long long u = (unsigned long long)__double_as_longlong(d);
  if (d != d) u = 0x7ff8000000000000ull;     // NaN sorts above +inf (DuckDB orders NaN greatest)
  return (u >> 63) ? ~u : (u | 0x8000000000000000ull);
}
__device__ __forceinline__ double order_dbl(unsigned long long o) {
  unsigned long long u = (o >> 63) ? (o & 0x7fffffffffffffffull) : ~o;
  return __longlong_as_double((long long)u);
}
__device__ __forceinline__ void two_sum(double a, double b, double& s, double& e) {
  s = a + b;
  double bb = s - a;
  e = (a - (s - bb)) + (b - bb);
}

// Value at index v of a hybrid RLE/bit-packed stream, given the run that contains v.
__device__ __forceinline__ uint32_t hybrid_get(const uint8_t* stream, const LRun& r, uint32_t v, int bw) {
  if (!(r.off_lit & 0x80000000u)) return r.value;
  uint64_t bit = uint64_t(v - r.start) * uint32_t(bw);
  uintptr_t a = reinterpret_cast<uintptr_t>(stream + (r.off_lit & 0x7fffffffu) + (bit >> 3));
  const uint32_t* w = reinterpret_cast<const uint32_t*>(a & ~uintptr_t(3));
  uint64_t x = (uint64_t(w[1]) << 32) | w[0];
  x >>= ((a & 3) * 8 + (bit & 7));
  uint32_t mask = bw >= 32 ? 0xffffffffu : ((1u << bw) - 1u);
  return uint32_t(x) & mask;
}

__device__ __forceinline__ int find_run(const LRun* runs, int n, uint32_t v) {
  int lo = 0, hi = n - 1;
  while (lo < hi) {
    int mid = (lo + hi + 1) >> 1;
    if (runs[mid].start <= v) lo = mid;
    else hi = mid - 1;
  }
  return lo;
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

template <int AGG>
__device__ __forceinline__ void acc_reset(Acc& a, unsigned long long key) {
  a.key = key;
  a.rows = 0;
  a.cnt = 0;
  a.hi = 0.0;
  a.lo = 0.0;
  a.ext = (AGG == AGG_MIN) ? ~0ull : 0ull;
}

// Merge a partial cell into the global table (device-scope atomics).
template <int AGG>
__device__ __forceinline__ void global_merge(const QParams& P, unsigned long long cell, uint32_t rows,
                                             uint32_t cnt, double hi, double lo, unsigned long long ext) {
  if (rows == 0) return;
  atomicAdd(&P.rows[cell], (unsigned long long)rows);
  if (cnt == 0) return;
  atomicAdd(&P.cnt[cell], (unsigned long long)cnt);
  if (AGG == AGG_SUM) {
    double old = atomicAdd(&P.hi[cell], hi);   // returning atomic: old is exact -> TwoSum recovers the error
    double s, e;
    two_sum(old, hi, s, e);
    atomicAdd(&P.lo[cell], lo + e);
  } else if (AGG == AGG_MIN) {
    atomicMin(&P.ext[cell], ext);
  } else if (AGG == AGG_MAX) {
    atomicMax(&P.ext[cell], ext);
  }
}

struct Lds {
  LRun pool[POOL];
  uint32_t lut[MAXSTR][LUT_CAP];
  unsigned long long hkey[HCAP];
  uint32_t hrows[HCAP];
  uint32_t hcnt[HCAP];
  double hhi[HCAP];                      // SUM: hi; MIN/MAX: ordered bits (reinterpreted)
  double hlo[HCAP];
  uint32_t wsum[MAXQCOL][BLOCK / 64];    // per-wave valid counts (def-level prefix)
  // tile / segment state broadcast from thread 0
  QSeg seg;
  TileDesc tile;
  TileCol tc[MAXQCOL];
  PageDesc pg[MAXQCOL];
  uint32_t pool_off[MAXQCOL];            // value runs
  uint32_t dpool_off[MAXQCOL];           // def runs
  uint32_t lut_on[MAXSTR];
  uint32_t vrun[MAXQCOL];                // running non-null count since the tile start (nullable pages)
  int seg_idx;
};

template <int AGG>
__device__ __forceinline__ void lds_merge(Lds& L, const QParams& P, const Acc& a) {
  if (a.rows == 0) return;
  uint32_t h = uint32_t(a.key * 0x9E3779B97F4A7C15ull >> 32) & (HCAP - 1);
  for (int probe = 0; probe < HPROBE; probe++) {
    unsigned long long prev = atomicCAS(&L.hkey[h], EMPTY, a.key);
    if (prev == EMPTY || prev == a.key) {
      atomicAdd(&L.hrows[h], a.rows);
      if (a.cnt) {
        atomicAdd(&L.hcnt[h], a.cnt);
        if (AGG == AGG_SUM) {
          double old = atomicAdd(&L.hhi[h], a.hi);
          double s, e;
          two_sum(old, a.hi, s, e);
          atomicAdd(&L.hlo[h], a.lo + e);
        } else if (AGG == AGG_MIN) {
          atomicMin(reinterpret_cast<unsigned long long*>(&L.hhi[h]), a.ext);
        } else if (AGG == AGG_MAX) {
          atomicMax(reinterpret_cast<unsigned long long*>(&L.hhi[h]), a.ext);
        }
      }
      return;
    }
    h = (h + 1) & (HCAP - 1);
  }
  global_merge<AGG>(P, a.key, a.rows, a.cnt, a.hi, a.lo, a.ext);   // LDS table full: straight to HBM
}

// Value index (relative to the tile's first non-null row) of this thread's row in one k-slice of a
// nullable column: non-null rows before it in the tile.  Wave part: ballot + popcount; block part: LDS;
// the running count since the tile start lives in L.vrun[c] (read between the barriers, advanced by
// thread 0 after the second one, so the next slice's reads are ordered behind the write).
__device__ __forceinline__ uint32_t block_prefix(Lds& L, int c, bool valid) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  unsigned long long m = __ballot(valid);
  uint32_t pre = __popcll(m & ((1ull << lane) - 1ull));
  if (lane == 0) L.wsum[c][wave] = __popcll(m);
  __syncthreads();
  uint32_t base = 0, total = 0;
#pragma unroll
  for (int w = 0; w < BLOCK / 64; w++) {
    uint32_t s = L.wsum[c][w];
    base += (w < wave) ? s : 0;
    total += s;
  }
  const uint32_t run = L.vrun[c];
  __syncthreads();
  if (threadIdx.x == 0) L.vrun[c] = run + total;
  return run + base + pre;
}

template <int AGG>
__global__ __launch_bounds__(BLOCK) void scan_tiles(QParams P, const uint32_t* __restrict__ seg_begin) {
  __shared__ Lds L;
  const int tid = threadIdx.x;
  const uint32_t tile_id = blockIdx.x;

  // ---- locate the segment (binary search over the per-query tile prefix, staged in LDS) ----
  {
    uint32_t* sb = reinterpret_cast<uint32_t*>(L.pool);   // pool is free until staged below
    for (uint32_t i = tid; i < P.nsegs; i += BLOCK) sb[i] = seg_begin[i];
    __syncthreads();
    if (tid == 0) {
      int lo = 0, hi = int(P.nsegs) - 1;
      while (lo < hi) {
        int mid = (lo + hi + 1) >> 1;
        if (sb[mid] <= tile_id) lo = mid;
        else hi = mid - 1;
      }
      L.seg_idx = lo;
    }
    __syncthreads();
  }
  const QSeg* gseg = P.segs + L.seg_idx;
  {
    // copy the QSeg (432 B) cooperatively
    const uint32_t* src = reinterpret_cast<const uint32_t*>(gseg);
    uint32_t* dst = reinterpret_cast<uint32_t*>(&L.seg);
    for (uint32_t i = tid; i < sizeof(QSeg) / 4; i += BLOCK) dst[i] = src[i];
    __syncthreads();
  }
  const uint32_t local_tile = tile_id - L.seg.tile_begin;
  const int ncols = 2 + int(P.nstr);
  if (tid == 0) L.tile = L.seg.tiles[local_tile];
  if (tid < ncols && L.seg.cols[tid].present) {
    L.tc[tid] = L.seg.cols[tid].tcols[local_tile];
    L.pg[tid] = L.seg.cols[tid].pages[L.tc[tid].page];
  }
  __syncthreads();
  const TileDesc tile = L.tile;
  if (tile.ts_max < L.seg.win_lo || tile.ts_min >= L.seg.win_hi) return;   // zone map: outside the window

  // ---- stage run windows and lookup tables ----
  if (tid == 0) {
    uint32_t off = 0;
    for (int c = 0; c < ncols; c++) {
      L.pool_off[c] = off;
      if (L.seg.cols[c].present && L.pg[c].kind == PAGE_DICT) off += L.tc[c].nruns;
      L.dpool_off[c] = off;
      if (L.seg.cols[c].present && L.pg[c].has_nulls) off += L.tc[c].ndruns;
    }
  }
  __syncthreads();
  for (int c = 0; c < ncols; c++) {
    if (!L.seg.cols[c].present) continue;
    const TileCol tc = L.tc[c];
    if (L.pg[c].kind == PAGE_DICT)
      for (uint32_t i = tid; i < tc.nruns; i += BLOCK) {
        RunDesc r = L.seg.cols[c].runs[tc.run_lo + i];
        L.pool[L.pool_off[c] + i] = LRun{r.start, r.off_lit, r.value};
      }
    if (L.pg[c].has_nulls)
      for (uint32_t i = tid; i < tc.ndruns; i += BLOCK) {
        RunDesc r = L.seg.cols[c].runs[tc.drun_lo + i];
        L.pool[L.dpool_off[c] + i] = LRun{r.start, r.off_lit, r.value};
      }
  }
  for (int s = 0; s < int(P.nstr); s++) {
    const int c = 2 + s;
    L.lut_on[s] = 0;
    if (!L.seg.cols[c].present || L.pg[c].dict_n > LUT_CAP) continue;
    const uint32_t* remap = L.seg.cols[c].remap + L.pg[c].remap;
    const uint32_t* tab = P.strtab[s];
    for (uint32_t i = tid; i < L.pg[c].dict_n; i += BLOCK) {
      uint32_t g = remap[i];
      L.lut[s][i] = tab ? tab[g] : g;
    }
    L.lut_on[s] = 1;
  }
  if (tid < MAXQCOL) L.vrun[tid] = 0;
  for (int i = tid; i < HCAP; i += BLOCK) {
    L.hkey[i] = EMPTY;
    L.hrows[i] = 0;
    L.hcnt[i] = 0;
    L.hlo[i] = 0.0;
    if (AGG == AGG_MIN) reinterpret_cast<unsigned long long*>(L.hhi)[i] = ~0ull;
    else L.hhi[i] = 0.0;
  }
  __syncthreads();

  Acc acc;
  acc_reset<AGG>(acc, EMPTY);
  const uint32_t leaf_false = L.seg.leaf_false;
  const unsigned long long glob_base = (unsigned long long)L.seg.glob_slot * P.nbuckets;

  for (uint32_t sub = 0; sub < tile.nrows; sub += SUB) {
    uint32_t leafT[RPT], leafF[RPT];
    unsigned long long gid[RPT];
    bool inrow[RPT];
#pragma unroll
    for (int k = 0; k < RPT; k++) {
      leafT[k] = 0;
      leafF[k] = 0;
      gid[k] = 0;
      inrow[k] = sub + k * BLOCK + tid < tile.nrows;
    }

    // ---------------- string columns ----------------
    for (int s = 0; s < int(P.nstr); s++) {
      const int c = 2 + s;
      uint32_t packed[RPT];
      bool isnull[RPT];
      if (!L.seg.cols[c].present) {
#pragma unroll
        for (int k = 0; k < RPT; k++) isnull[k] = true, packed[k] = 0;
      } else {
        const PageDesc pg = L.pg[c];
        const TileCol tc = L.tc[c];
        const uint8_t* vstream = L.seg.base + pg.vals;
        const uint32_t row_in_page = tile.row0 - pg.first_row;
        uint32_t vidx[RPT];
        if (pg.has_nulls) {
          const uint8_t* dstream = L.seg.base + pg.defs;
          const LRun* druns = L.pool + L.dpool_off[c];
#pragma unroll
          for (int k = 0; k < RPT; k++) {
            uint32_t r = row_in_page + sub + k * BLOCK + tid;
            bool valid = false;
            if (inrow[k]) {
              int ri = find_run(druns, int(tc.ndruns), r);
              valid = hybrid_get(dstream, druns[ri], r, 1) != 0;
            }
            vidx[k] = tc.vbase + block_prefix(L, c, valid);
            isnull[k] = !valid;
          }
        } else {
#pragma unroll
          for (int k = 0; k < RPT; k++) {
            vidx[k] = tc.vbase + sub + k * BLOCK + tid;
            isnull[k] = !inrow[k];
          }
        }
        const LRun* runs = L.pool + L.pool_off[c];
        const bool lut = L.lut_on[s];
        const uint32_t* remap = L.seg.cols[c].remap + pg.remap;
        const uint32_t* tab = P.strtab[s];
#pragma unroll
        for (int k = 0; k < RPT; k++) {
          packed[k] = 0;
          if (isnull[k]) continue;
          int ri = find_run(runs, int(tc.nruns), vidx[k]);
          uint32_t idx = hybrid_get(vstream, runs[ri], vidx[k], pg.bw);
          if (lut) {
            packed[k] = L.lut[s][idx];
          } else {
            uint32_t g = remap[idx];
            packed[k] = tab ? tab[g] : g;
          }
        }
      }
      // fold: group dimension + leaves of this column
      const unsigned long long dstride = P.dim_stride[s];
      const uint32_t dnull = P.dim_null[s];
      const uint32_t lbase = P.str_lbase[s], lmask = P.str_lmask[s], hmask = P.str_hmask[s];
#pragma unroll
      for (int k = 0; k < RPT; k++) {
        if (isnull[k]) {
          gid[k] += (unsigned long long)dnull * dstride;
          leafF[k] |= hmask;                   // IS NOT NULL on NULL is FALSE; other leaves are NULL
        } else {
          gid[k] += (unsigned long long)(packed[k] & DIM_MASK) * dstride;
          uint32_t bits = (packed[k] >> 24) << lbase;
          leafT[k] |= bits & lmask;
          leafF[k] |= ~bits & lmask;
        }
      }
    }

    // ---------------- filter program (Kleene logic on T/F bit stacks) ----------------
    bool pass[RPT];
#pragma unroll
    for (int k = 0; k < RPT; k++) {
      uint32_t T = leafT[k] & ~leaf_false, F = leafF[k] | leaf_false;
      uint64_t st = 0, sf = 0;
      for (uint32_t i = 0; i < P.nprog; i++) {
        uint8_t op = P.prog[i];
        if (op < 0x80) {
          st = (st << 1) | ((T >> op) & 1u);
          sf = (sf << 1) | ((F >> op) & 1u);
        } else if (op == OP_NOT) {
          uint64_t t1 = st & 1, f1 = sf & 1;
          st = (st & ~1ull) | f1;
          sf = (sf & ~1ull) | t1;
        } else if (op == OP_TRUE) {
          st = (st << 1) | 1;
          sf = sf << 1;
        } else {
          uint64_t t2 = st & 1, f2 = sf & 1;
          st >>= 1;
          sf >>= 1;
          uint64_t t1 = st & 1, f1 = sf & 1;
          uint64_t t = (op == OP_AND) ? (t1 & t2) : (t1 | t2);
          uint64_t f = (op == OP_AND) ? (f1 | f2) : (f1 & f2);
          st = (st & ~1ull) | t;
          sf = (sf & ~1ull) | f;
        }
      }
      pass[k] = inrow[k] && (st & 1);
    }

    // ---------------- timestamp + value: only for passing rows ----------------
    int64_t ts[RPT];
    bool tsok[RPT];
    double val[RPT];
    bool vok[RPT];
#pragma unroll
    for (int c = 0; c < 2; c++) {
      const bool present = L.seg.cols[c].present;
      const PageDesc pg = L.pg[c];
      const TileCol tc = L.tc[c];
      uint32_t vidx[RPT];
      bool valid[RPT];
      if (present && pg.has_nulls) {
        const uint8_t* dstream = L.seg.base + pg.defs;
        const LRun* druns = L.pool + L.dpool_off[c];
        const uint32_t row_in_page = tile.row0 - pg.first_row;
#pragma unroll
        for (int k = 0; k < RPT; k++) {
          uint32_t r = row_in_page + sub + k * BLOCK + tid;
          bool v = false;
          if (inrow[k]) {
            int ri = find_run(druns, int(tc.ndruns), r);
            v = hybrid_get(dstream, druns[ri], r, 1) != 0;
          }
          vidx[k] = tc.vbase + block_prefix(L, c, v);
          valid[k] = v;
        }
      } else {
#pragma unroll
        for (int k = 0; k < RPT; k++) {
          vidx[k] = tc.vbase + sub + k * BLOCK + tid;
          valid[k] = present && inrow[k];
        }
      }
      const uint64_t* data = reinterpret_cast<const uint64_t*>(L.seg.base + pg.vals);
#pragma unroll
      for (int k = 0; k < RPT; k++) {
        uint64_t raw = 0;
        bool ok = valid[k] && pass[k];
        if (ok) raw = __builtin_nontemporal_load(data + vidx[k]);
        if (c == 0) {
          ts[k] = (int64_t)raw;
          tsok[k] = ok;
        } else {
          val[k] = __longlong_as_double((long long)raw);
          vok[k] = ok;
        }
      }
    }

    // ---------------- bucket + aggregate ----------------
#pragma unroll
    for (int k = 0; k < RPT; k++) {
      if (!pass[k] || !tsok[k]) continue;
      const int64_t t = ts[k];
      if (t < L.seg.win_lo || t >= L.seg.win_hi) continue;         // BaseExpr.scala:159-161
      int64_t b;
      if (P.metrics) {
        int64_t d = t - P.bucket_base;
        b = d / P.step;
        if (d - b * P.step != 0) { atomicOr(P.flags, FLAG_METRICS_UNALIGNED); continue; }
      } else {
        int64_t st = t - t % P.step;                                  // ts - ts % step (fmod, trunc)
        b = (st - P.bucket_base) / P.step;
      }
      if (b < 0 || (uint64_t)b >= P.nbuckets) { atomicOr(P.flags, FLAG_CELL_RANGE); continue; }
      unsigned long long cell = (glob_base + (unsigned long long)b) * P.ngroups + gid[k];
      if (cell != acc.key) {
        lds_merge<AGG>(L, P, acc);
        acc_reset<AGG>(acc, cell);
      }
      acc_add<AGG>(acc, vok[k], val[k]);
    }
  }
  lds_merge<AGG>(L, P, acc);
  __syncthreads();
  for (int i = tid; i < HCAP; i += BLOCK) {
    if (L.hkey[i] == EMPTY) continue;
    global_merge<AGG>(P, L.hkey[i], L.hrows[i], L.hcnt[i], L.hhi[i], L.hlo[i],
                      reinterpret_cast<unsigned long long*>(L.hhi)[i]);
  }
}

// ------------------------------------------------------------------------------------------------
// Finalize + compaction
// ------------------------------------------------------------------------------------------------
struct OutRow {
  bool exists;
  double value;
  unsigned long long gid;
  uint32_t glob;
};

__device__ __forceinline__ double cell_value(const FParams& F, unsigned long long cell) {
  unsigned long long cnt = F.cnt[cell];
  switch (F.agg) {
    case AGG_COUNT: return double(cnt);
    case AGG_SUM: return cnt ? F.hi[cell] + F.lo[cell] : 0.0;     // NULL -> 0.0 (JDBC getDouble)
    case AGG_MIN:
    case AGG_MAX: return cnt ? order_dbl(F.ext[cell]) : 0.0;
    default: return cnt ? (F.hi[cell] + F.lo[cell]) / double(cnt) : 0.0;   // avg (per-glob only)
  }
}

// Output key -> row. Per-glob: key = (glob, bucket, group). Merged: key = (bucket, group) or (bucket)
// when the name dimension collapses (no groupBys).
__device__ OutRow make_row(const FParams& F, unsigned long long key) {
  OutRow o{false, 0.0, 0, 0};
  if (F.per_glob) {
    unsigned long long cell = key;
    if (F.rows[cell] == 0) return o;
    o.exists = true;
    o.value = cell_value(F, cell);
    o.gid = cell % F.ngroups;
    o.glob = uint32_t(cell / (F.ngroups * F.nbuckets));
    return o;
  }
  const unsigned long long b = F.collapse ? key : key / F.ngroups;
  const unsigned long long g0 = F.collapse ? 0 : key % F.ngroups;
  const unsigned long long ng = F.collapse ? F.ngroups : 1;
  double hi = 0.0, lo = 0.0, ext = 0.0;
  unsigned long long cnt = 0;
  uint32_t best_rank = 0xffffffffu;
  for (uint32_t gs = 0; gs < F.nglob_slots; gs++) {
    for (unsigned long long g = g0; g < g0 + ng; g++) {
      unsigned long long cell = ((unsigned long long)gs * F.nbuckets + b) * F.ngroups + g;
      if (F.rows[cell] == 0) continue;
      unsigned long long c = F.cnt[cell];
      if (F.agg == AGG_SUM) {
        double s, e;
        two_sum(hi, F.hi[cell], s, e);
        hi = s;
        lo += e + F.lo[cell];
      } else if (F.agg == AGG_MIN || F.agg == AGG_MAX) {
        double v = c ? order_dbl(F.ext[cell]) : 0.0;   // a glob's NULL cell merges as 0.0
        if (!o.exists) ext = v;
        else ext = (F.agg == AGG_MIN) ? fmin(ext, v) : fmax(ext, v);
      }
      cnt += c;
      uint32_t rank = F.name_rank ? F.name_rank[g / F.name_stride] : 0;
      if (!o.exists || rank < best_rank) {
        best_rank = rank;
        o.gid = g;
      }
      o.exists = true;
    }
  }
  if (!o.exists) return o;
  if (F.agg == AGG_SUM) o.value = hi + lo;
  else if (F.agg == AGG_COUNT) o.value = double(cnt);
  else o.value = ext;
  return o;
}

constexpr int FB = 256;
constexpr int FITEMS = 8;

__global__ __launch_bounds__(FB) void finalize_count(FParams F, uint32_t* block_counts) {
  __shared__ uint32_t ws[FB / 64];
  uint32_t n = 0;
  const unsigned long long base = (unsigned long long)blockIdx.x * FB * FITEMS;
  for (int i = 0; i < FITEMS; i++) {
    unsigned long long key = base + (unsigned long long)i * FB + threadIdx.x;
    if (key < F.nkeys && make_row(F, key).exists) n++;
  }
  for (int o = 32; o > 0; o >>= 1) n += __shfl_down(n, o, 64);
  if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = n;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t t = 0;
    for (int w = 0; w < FB / 64; w++) t += ws[w];
    block_counts[blockIdx.x] = t;
  }
}

// Single-block exclusive scan of the per-block counts; writes the total at counts[n].
__global__ __launch_bounds__(1024) void finalize_scan(uint32_t* counts, uint32_t n) {
  __shared__ uint32_t carry;
  __shared__ uint32_t ws[16];
  if (threadIdx.x == 0) carry = 0;
  __syncthreads();
  for (uint32_t base = 0; base < n; base += 1024) {
    uint32_t i = base + threadIdx.x;
    uint32_t v = i < n ? counts[i] : 0;
    uint32_t x = v;
    for (int o = 1; o < 64; o <<= 1) {
      uint32_t y = __shfl_up(x, o, 64);
      if ((threadIdx.x & 63) >= o) x += y;
    }
    if ((threadIdx.x & 63) == 63) ws[threadIdx.x >> 6] = x;
    __syncthreads();
    uint32_t wbase = 0;
    for (int w = 0; w < int(threadIdx.x >> 6); w++) wbase += ws[w];
    uint32_t excl = carry + wbase + x - v;
    if (i < n) counts[i] = excl;
    __syncthreads();
    if (threadIdx.x == 1023) carry = excl + v;
    __syncthreads();
  }
  if (threadIdx.x == 0) counts[n] = carry;
}

__global__ __launch_bounds__(FB) void finalize_write(FParams F, const uint32_t* block_offsets, int64_t* out_ts,
                                                   double* out_val, unsigned long long* out_gid,
                                                   uint32_t* out_glob) {
  __shared__ uint32_t ws[FB / 64];
  const unsigned long long base = (unsigned long long)blockIdx.x * FB * FITEMS;
  uint32_t off = block_offsets[blockIdx.x];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int i = 0; i < FITEMS; i++) {
    unsigned long long key = base + (unsigned long long)i * FB + threadIdx.x;
    OutRow r{false, 0, 0, 0};
    if (key < F.nkeys) r = make_row(F, key);
    unsigned long long m = __ballot(r.exists);
    if (lane == 0) ws[wave] = __popcll(m);
    __syncthreads();
    uint32_t wb = 0, tot = 0;
    for (int w = 0; w < FB / 64; w++) {
      wb += (w < wave) ? ws[w] : 0;
      tot += ws[w];
    }
    if (r.exists) {
      uint32_t pos = off + wb + __popcll(m & ((1ull << lane) - 1ull));
      unsigned long long b = F.per_glob ? (key / F.ngroups) % F.nbuckets : (F.collapse ? key : key / F.ngroups);
      out_ts[pos] = F.bucket_base + (int64_t)b * F.step;
      out_val[pos] = r.value;
      out_gid[pos] = r.gid;
      out_glob[pos] = r.glob;
    }
    off += tot;
    __syncthreads();
  }
}

// Rank 0 of a sharded evaluation: add ranks 1..world-1's compensated sums (gathered as [hi | lo] blocks)
// to its own, in rank order, so the merged sum is deterministic for a given shard assignment.
__global__ __launch_bounds__(256) void merge_dd(double* hi, double* lo, const double* parts, int world, size_t nc) {
  size_t i = size_t(blockIdx.x) * 256 + threadIdx.x;
  if (i >= nc) return;
  double h = hi[i], l = lo[i];
  for (int r = 1; r < world; r++) {
    const double* p = parts + size_t(r) * nc * 2;
    double s, e;
    two_sum(h, p[i], s, e);
    h = s;
    l += e + p[nc + i];
  }
  hi[i] = h;
  lo[i] = l;
}

// ------------------------------------------------------------------------------------------------
// Host launchers
// ------------------------------------------------------------------------------------------------
hipError_t launch_merge_dd(double* hi, double* lo, const double* parts, int world, size_t nc, hipStream_t stream) {
  if (nc == 0) return hipSuccess;
  hipLaunchKernelGGL(merge_dd, dim3(uint32_t((nc + 255) / 256)), dim3(256), 0, stream, hi, lo, parts, world, nc);
  return hipGetLastError();
}

hipError_t launch_scan(const QParams& P, const uint32_t* d_seg_begin, int agg, hipStream_t stream) {
  if (P.total_tiles == 0) return hipSuccess;
  dim3 grid(P.total_tiles), block(BLOCK);
  switch (agg) {
    case AGG_SUM: hipLaunchKernelGGL(scan_tiles<AGG_SUM>, grid, block, 0, stream, P, d_seg_begin); break;
    case AGG_MIN: hipLaunchKernelGGL(scan_tiles<AGG_MIN>, grid, block, 0, stream, P, d_seg_begin); break;
    case AGG_MAX: hipLaunchKernelGGL(scan_tiles<AGG_MAX>, grid, block, 0, stream, P, d_seg_begin); break;
    default: hipLaunchKernelGGL(scan_tiles<AGG_COUNT>, grid, block, 0, stream, P, d_seg_begin); break;
  }
  return hipGetLastError();
}

uint32_t finalize_blocks(unsigned long long nkeys) {
  return uint32_t((nkeys + FB * FITEMS - 1) / (FB * FITEMS));
}

hipError_t launch_finalize(const FParams& F, uint32_t* d_counts, int64_t* ts, double* val, unsigned long long* gid,
                           uint32_t* glob, hipStream_t stream) {
  uint32_t nb = finalize_blocks(F.nkeys);
  if (nb == 0) return hipMemsetAsync(d_counts, 0, sizeof(uint32_t), stream);
  hipLaunchKernelGGL(finalize_count, dim3(nb), dim3(FB), 0, stream, F, d_counts);
  hipLaunchKernelGGL(finalize_scan, dim3(1), dim3(1024), 0, stream, d_counts, nb);
  hipLaunchKernelGGL(finalize_write, dim3(nb), dim3(FB), 0, stream, F, d_counts, ts, val, gid, glob);
  return hipGetLastError();
}

}  // namespace lk
