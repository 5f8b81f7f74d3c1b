// scan_tiles<AGG, NSTR, TT>: the fused decode -> filter -> bucket -> aggregate kernel (included by kernels.hip).
//
// grid (tile, segment); one 256-thread workgroup per tile (a row range inside one page of every column).
//   prologue: every fact about the tile's columns (stream pointers, run windows, value bases, flags) is read
//     once and staged in LDS together with the run windows, small dictionaries' lookup values (dictionary index
//     -> leaf bits | group-dim id) and the filter truth table.
//   Per 2048-row sub-tile, thread t owns rows 8t..8t+7 (wave w: rows 512w..512w+511):
//   A. definition levels of nullable columns: one packed byte per thread (bit e = row 8t+e is non-NULL); value
//      indices from a bit-sliced ballot prefix (4 ballots + mbcnt) and the per-wave totals (one barrier);
//   B. string columns: a non-NULL column's values 8t..8t+7 are the thread's rows: unpacked from one bit-packed
//      group (one 96-bit load issued a sub-tile ahead) straight into registers; a nullable column's values are
//      unpacked value-major into LDS and gathered by value index (two barriers). Every row folds its value into
//      leaf T/F bits and its group id;
//   C. the filter's truth table (Kleene logic precomputed on the host; TT=false interprets the program) -> a
//      pass byte per thread;
//   D. passing rows are compacted, in row order, into the wave's own LDS list (ballot prefix; no barrier);
//   E. the wave streams timestamp + value of its listed rows only (late materialization), buckets by exact
//      32-bit reciprocal division and accumulates in a per-thread register cell (time-sorted rows hit it),
//      spilling to an LDS hash table (LDS atomics; sums as compensated hi/lo with a returning-atomic TwoSum).
//   tile end: LDS cells -> global table with device atomics (count/min/max exact, sums within 1 ulp).
// Without nullable columns the sub-tile loop has no workgroup barrier: the four waves run independently.
#pragma once
#include <type_traits>

#include "device_common.hpp"

namespace lk {

constexpr int WAVES = BLOCK / 64;        // 4
constexpr int WROWS = SUBT / WAVES;      // rows per wave per sub-tile (512)
constexpr int PS = 4;                    // listed rows per lane loaded together in phase E

struct ColHot {                          // one column over one tile, staged once per tile
  const uint8_t* vals;                   // value stream (absolute)
  const uint8_t* defs;                   // def-level stream (absolute)
  const uint32_t* remap;                 // chunk dictionary remap (absolute)
  uint32_t vals_len, defs_len;
  uint32_t vbase, rip, nruns, ndruns;
  uint32_t bw, has_nulls, present, lut_on;
  uint32_t dict_n, pad;
};

constexpr int RS = RUN_CAP + 1;                  // staged runs per stream (+ sentinel)
// LDS hash entries: a single string column (name) has few cells per tile, so half a table buys the LDS the
// 128-run windows need while keeping four workgroups per CU
template <int NSTR>
constexpr int hcap_v = NSTR == 1 ? HCAP / 2 : HCAP;
constexpr int RBLK = TILE_ROWS / 64 + 8;         // run-block table entries per string column

// LDS aggregation table layout.  FULL: rows, non-NULL count, compensated sum (hi, lo) / ordered extreme.  SLIM
// (lean tables of min / max / count, LEAN_* in layout.hpp): one 8-B value per cell (the ordered extreme, or the
// row count), so the same LDS holds twice the cells -- high-cardinality :by queries spill half as often.
template <int NSTR, bool SLIM>
constexpr int hslots_v = hcap_v<NSTR> * (SLIM ? 2 : 1);

template <int NSTR, bool SLIM = false>
struct Lds {
  LRun pool[(2 + 2 * NSTR) * RS];        // run windows (+ sentinel): def runs of column c at c*RS, value runs of
                                         //   string column s at (2 + NSTR + s)*RS
  uint8_t rblk[NSTR][RBLK];              // per string column: run holding value index vbase + 64b (tile-relative
                                         //   64-value blocks), so a run lookup is one table read + a short search
  uint32_t lut[NSTR][LUT_CAP];
  uint32_t truth[(1u << (2 * TT_MAX_LEAVES)) / 32];
  uint32_t truth_e[NSTR > 1 ? (1u << (2 * TT_MAX_LEAVES)) / 32 : 1];   // late materialization: early / late
  uint32_t truth_l[NSTR > 1 ? (1u << (2 * TT_MAX_LEAVES)) / 32 : 1];   //   conjunct tables
  static constexpr int H = hslots_v<NSTR, SLIM>;
  unsigned long long hkey[H];
  uint32_t hrows[SLIM ? 1 : H];
  uint32_t hcnt[SLIM ? 1 : H];
  double hhi[SLIM ? 1 : H];                      // SUM: hi; MIN/MAX: ordered bits (reinterpreted)
  double hlo[SLIM ? 1 : H];
  unsigned long long hval[SLIM ? H : 1];         // SLIM: MIN/MAX ordered extreme, COUNT rows
  uint2 list[WAVES][WROWS];              // per wave: passing rows {group id, ts index | value index << 11 |
                                         //   value valid << 22} (indices relative to the sub-tile's values).
                                         // Its first 2 KB per wave double as the wave's pk slots (thread t:
                                         //   8 u32 at 8*lane): a nullable string column's lookup values,
                                         //   value-major, and the straddling-group decode's scratch.
  uint32_t wsum[2 + NSTR][WAVES];        // per nullable column: non-NULL rows of each wave in the sub-tile
  ColHot hot[2 + NSTR];                  // per-tile column state
  StrParam sp[NSTR];                     // per-query string column parameters
  int64_t win_lo, win_hi;
  uint32_t glob_slot, leaf_false;
  uint32_t hfull;                        // the LDS table refused a key: later cells go straight to HBM
  unsigned long long stamp[LK_NSTAMP];   // diagnostics only
};

// Merge a register cell into the workgroup's LDS table (any LDS layout with hkey/hrows/hcnt/hhi/hlo/hval/hfull and
// H slots); a full table sends the cell straight to the global table.
template <int AGG, bool HASH, bool SLIM, class LT>
__device__ __forceinline__ void lds_merge(LT& L, const QParams& P, const Acc& a) {
  if (a.rows == 0) return;
  constexpr int H = LT::H;
  uint32_t h = uint32_t(a.key * 0x9E3779B97F4A7C15ull >> 32) & (H - 1);
  for (int probe = 0; probe < HPROBE; probe++) {
    unsigned long long prev = atomicCAS(&L.hkey[h], EMPTY, a.key);
    if (probe == 0 && prev != EMPTY && prev != a.key && L.hfull) break;   // table known full: no more probes
    if (prev == EMPTY || prev == a.key) {
      if constexpr (SLIM) {
        if (AGG == AGG_MIN) atomicMin(&L.hval[h], a.ext);
        else if (AGG == AGG_MAX) atomicMax(&L.hval[h], a.ext);
        else atomicAdd(&L.hval[h], (unsigned long long)a.rows);
        return;
      } else {
        // lean tables whose rows / cnt the global table never accumulates (LEAN_NO_ROWS, LEAN_SUM_EXISTS; fixup_table
        // restores them): the LDS cell's rows / cnt only mark it occupied -- set once by the inserting lane, no atomics
        const bool marks = (P.lean & (LEAN_NO_ROWS | LEAN_SUM_EXISTS)) != 0u;
        if (marks) {
          if (prev == EMPTY) {
            L.hrows[h] = 1u;
            L.hcnt[h] = 1u;
          }
        } else {
          atomicAdd(&L.hrows[h], a.rows);
        }
        if (a.cnt) {
          if (!marks) atomicAdd(&L.hcnt[h], a.cnt);
          if (AGG == AGG_SUM) {
            if (P.exact_sum) {   // exact adds: nothing to compensate
              __hip_atomic_fetch_add(&L.hhi[h], a.hi, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
              return;
            }
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
    }
    h = (h + 1) & (H - 1);
  }
  L.hfull = 1u;                                                     // benign race: any writer stores 1
  global_merge<AGG, HASH>(P, a.key, a.rows, a.cnt, a.hi, a.lo, a.ext);   // LDS table full: straight to HBM
}

}  // namespace lk

#ifdef LK_INST_LEAN
#include "lean_kernel.hpp"   // scan_lean (uses lds_merge); its units only (scan_inst.hpp)
#endif

namespace lk {

// Kleene evaluation of the postfix program (filters with more than TT_MAX_LEAVES leaves).
__device__ __forceinline__ bool interpret(const QParams& P, uint32_t T, uint32_t F) {
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
  return st & 1;
}

// Uniform LDS-staged pointer -> SGPR pair.
template <class T>
__device__ __forceinline__ const T* uptr(const T* p) {
  return reinterpret_cast<const T*>(uni_ptr(reinterpret_cast<const uint8_t*>(p)));
}

// Distinct 128-B lines among the wave's gather offsets (page streams start 128-B aligned, so a stream offset >> 7
// is its HBM line; live lanes hold non-decreasing offsets, the listed rows being in row order), not counting the
// line the wave's previous gather of the same stream ended on: the plan-bytes counter's unit for a per-row gather.
__device__ __forceinline__ uint32_t new_lines(bool live, uint32_t off, uint32_t& last) {
  const uint32_t line = off >> 7;
  const uint32_t prev = __shfl_up(line, 1, 64);
  const unsigned long long m = __ballot(live);
  const bool fresh = live && (__lane_id() == 0 ? line != last : line != prev);
  const uint32_t n = uint32_t(__popcll(__ballot(fresh)));
  if (m) last = __builtin_amdgcn_readlane(line, 63 - __clzll(m));
  return n;
}

// Exclusive prefix over the wave's lanes of a count in 0..15, and the wave total (uniform): one ballot per bit.
__device__ __forceinline__ uint32_t wave_prefix16(uint32_t cnt, uint32_t& total) {
  uint32_t pre = 0, tot = 0;
#pragma unroll
  for (int k = 0; k < 4; k++) {
    const unsigned long long b = __ballot((cnt >> k) & 1u);
    pre += __builtin_amdgcn_mbcnt_hi(uint32_t(b >> 32), __builtin_amdgcn_mbcnt_lo(uint32_t(b), 0u)) << k;
    tot += uint32_t(__popcll(b)) << k;
  }
  total = tot;
  return pre;
}

// 8 consecutive values [v, v+8) of a hybrid RLE/bit-packed stream (runs staged in LDS: `n` runs + a sentinel
// holding the end of the last one), in two steps so the load latency overlaps other work:
//   g8_issue: run lookup; when [v, v+8) lies inside one bit-packed run with bw <= 8, load the 96 bits from the
//             dword enclosing its first bit (8*bw <= 64 bits + <= 31 bits of misalignment);
//   g8_unpack / g8_bits: unpack (an RLE run: its value; a group straddling runs or bw > 8: per-value reads).
struct G8 {
  v2u w01;
  uint32_t w2;
  uint32_t ri;   // run index
};

// Run holding value v through the run-block table: runs blk[b] .. blk[b+1] bracket the 64-value block of v
// (v >= vbase; values past the tile clamp to the last block — their lanes are masked by the caller).
__device__ __forceinline__ int find_run_blk(const LRun* runs, const uint8_t* blk, uint32_t nb, uint32_t vbase,
                                            uint32_t v) {
  uint32_t b = (v - vbase) >> 6;
  b = b < nb ? b : nb - 1u;
  int lo = blk[b], hi = blk[b + 1];
  while (lo < hi) {
    const int m = (lo + hi + 1) >> 1;
    if (runs[m].start <= v) lo = m;
    else hi = m - 1;
  }
  return lo;
}

__device__ __forceinline__ G8 g8_issue(__amdgpu_buffer_rsrc_t rs, const LRun* runs, int n, uint32_t v, int bw,
                                       bool wide, const uint8_t* blk = nullptr, uint32_t nb = 0, uint32_t vbase = 0) {
  G8 g;
  g.ri = n == 1 ? 0 : (blk ? find_run_blk(runs, blk, nb, vbase, v) : find_run(runs, n, v));   // n: uniform
  const LRun r = runs[g.ri];
  const bool fast = (r.off_lit & 0x80000000u) != 0 && v + 8 <= runs[g.ri + 1].start && bw <= 8;
  const uint32_t byte = (r.off_lit & 0x7fffffffu) + (((v - r.start) * uint32_t(bw)) >> 3);
  g.w01 = __builtin_amdgcn_raw_buffer_load_b64(rs, fast ? (byte & ~3u) : OOB, 0, 0);
  g.w2 = wide ? __builtin_amdgcn_raw_buffer_load_b32(rs, fast ? (byte & ~3u) + 8u : OOB, 0, 0) : 0u;
  return g;
}

// the 64 bits starting at value v's first bit (fast case)
__device__ __forceinline__ uint64_t g8_window(const G8& g, const LRun& r, uint32_t v, int bw) {
  const uint32_t bit = (v - r.start) * uint32_t(bw);
  const uint32_t sh = (((r.off_lit & 0x7fffffffu) + (bit >> 3)) & 3u) * 8u + (bit & 7u);   // <= 31
  const uint64_t lo = ((uint64_t)g.w01.y << 32) | g.w01.x;
  return sh ? ((lo >> sh) | ((uint64_t)g.w2 << (64 - sh))) : lo;
}

// Unpack the group through `look` (dictionary index -> lookup value) into out[0..8); values at or past `left`
// are looked up as index 0. An RLE run looks its value up once. The straddling / wide case is a rolled loop
// through the thread's own 8 LDS slots `own` (no other thread reads them).
template <class Look>
__device__ __forceinline__ void g8_unpack(const G8& g, __amdgpu_buffer_rsrc_t rs, const LRun* runs, int n, uint32_t v,
                                          int bw, uint32_t left, uint32_t* own, Look look, uint32_t out[8]) {
  const LRun r = runs[g.ri];
  const bool lit = (r.off_lit & 0x80000000u) != 0;
  const bool whole = v + 8 <= runs[g.ri + 1].start;
  if (whole && !lit) {
    const uint32_t x = look(r.value);
#pragma unroll
    for (int e = 0; e < 8; e++) out[e] = x;
  } else if (whole && bw <= 8) {
    const uint64_t x = g8_window(g, r, v, bw);
    const uint32_t mask = (1u << bw) - 1u;
#pragma unroll
    for (int e = 0; e < 8; e++) out[e] = look(uint32_t(e) < left ? uint32_t(x >> (e * bw)) & mask : 0u);
  } else {
#pragma unroll 1
    for (int e = 0; e < 8; e++) {
      const uint32_t ve = v + e;
      own[e] = look(uint32_t(e) < left ? hybrid_get_buf(rs, runs[find_run(runs, n, ve)], ve, bw) : 0u);
    }
#pragma unroll
    for (int e = 0; e < 8; e++) out[e] = own[e];
  }
}

// definition levels (bw 1): the 8 levels as bits, row v + e at bit e
__device__ __forceinline__ uint32_t g8_bits(const G8& g, __amdgpu_buffer_rsrc_t rs, const LRun* runs, int n,
                                            uint32_t v) {
  const LRun r = runs[g.ri];
  const bool lit = (r.off_lit & 0x80000000u) != 0;
  const bool whole = v + 8 <= runs[g.ri + 1].start;
  if (whole && !lit) return r.value ? 0xffu : 0u;
  if (whole) {
    const uint32_t bit = v - r.start;
    const uint32_t sh = (((r.off_lit & 0x7fffffffu) + (bit >> 3)) & 3u) * 8u + (bit & 7u);
    const uint64_t lo = ((uint64_t)g.w01.y << 32) | g.w01.x;
    return uint32_t(lo >> sh) & 0xffu;
  }
  uint32_t bits = 0;
#pragma unroll 1
  for (int e = 0; e < 8; e++) {
    const uint32_t ve = v + e;
    bits |= (hybrid_get_buf(rs, runs[find_run(runs, n, ve)], ve, 1) & 1u) << e;
  }
  return bits;
}

#ifndef LK_DEPTH   // software-pipeline depth per string-column count (ring of pending chunks, see the main loop)
#define LK_DEPTH(nstr) 1
#endif

// Listed rows of a wave whose timestamp/value loads are in flight: NS slots of 64 rows (one row per lane per slot).
template <int NS>
struct ChunkT {
  static constexpr int kSlots = NS;
  v2u ts[NS], v[NS];
  uint32_t gid[NS];
  uint32_t vok;    // bit j: value j is non-NULL
  uint32_t live;   // bit j: slot j holds a row
  uint32_t n;      // listed rows in the chunk (uniform; 0: none)
};

template <int AGG, int NSTR, bool TT, bool HASH, bool SLIM = false>
__global__ __launch_bounds__(BLOCK) __attribute__((amdgpu_waves_per_eu(NSTR == 1 ? 4 : (NSTR <= 3 ? 3 : 2)))) void scan_tiles(QParams P) {
  __shared__ Lds<NSTR, SLIM> L;
  constexpr int HS = hslots_v<NSTR, SLIM>;
  constexpr int NC = 2 + NSTR;
  auto druns = [&](int c) { return L.pool + c * RS; };                  // def-level runs of column c
  auto vruns = [&](int c) { return L.pool + (NSTR + c) * RS; };         // value runs of string column c >= 2
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const unsigned long long st0 = P.stamps ? __builtin_amdgcn_s_memtime() : 0;   // diagnostics only

  // ---- segment (grid.y) and tile (grid.x): uniform addresses -> scalar loads, once ----
  const QSeg* Sp = P.segs + blockIdx.y;
  const uint32_t t = blockIdx.x;
  if (t >= Sp->ntiles) return;
  const TileDesc* tdp = Sp->tiles + t;
  if (tdp->ts_max < Sp->win_lo || tdp->ts_min >= Sp->win_hi) return;   // zone map: outside the glob window
  if (P.lean_split && lean_tile(Sp, t, P.nstr - 1, P.rows_only)) return;             // scan_lean's tile
  const uint32_t tile_nrows = tdp->nrows;

  // ---- stage per-tile column state, run windows, lookup values, truth table; clear the LDS table ----
  if (tid < NC) {
    const int c = tid;
    ColHot h{};
    h.present = Sp->cols[c].present;
    if (h.present) {
      const TileCol tc = Sp->cols[c].tcols[t];
      h.vals = Sp->base + tc.vals;
      h.defs = Sp->base + tc.defs;
      h.remap = Sp->cols[c].remap + tc.remap;
      h.vals_len = tc.vals_len;
      h.defs_len = tc.defs_len;
      h.vbase = tc.vbase;
      h.rip = tc.row_in_page;
      h.nruns = tc.kind == PAGE_DICT ? tc.nruns : 0u;
      h.ndruns = tc.has_nulls ? tc.ndruns : 0u;
      h.bw = tc.bw;
      h.has_nulls = tc.has_nulls;
      h.lut_on = c >= 2 && tc.dict_n <= LUT_CAP;
      h.dict_n = tc.dict_n;
    }
    L.hot[c] = h;
    if (c >= 2) L.sp[c - 2] = uint32_t(c - 2) < P.nstr ? P.strp[c - 2] : StrParam{};   // generic: unused columns
  }
  if (tid == 0) {
    L.win_lo = Sp->win_lo;
    L.win_hi = Sp->win_hi;
    L.glob_slot = Sp->glob_slot;
    L.leaf_false = Sp->leaf_false;
    L.hfull = 0u;
  }
  __syncthreads();
#pragma unroll
  for (int c = 0; c < NC; c++) {
    if (!uni(L.hot[c].present)) continue;
    const TileCol* tc = Sp->cols[c].tcols + t;
    const RunDesc* runs = Sp->cols[c].runs;
    const uint32_t nr = c >= 2 ? uni(L.hot[c].nruns) : 0u, nd = uni(L.hot[c].ndruns);
    const uint32_t rlo = tc->run_lo, dlo = tc->drun_lo;
    if (c >= 2) {
      LRun* vp = vruns(c);
      for (uint32_t i = tid; i < nr; i += BLOCK) {
        const RunDesc r = runs[rlo + i];
        vp[i] = LRun{r.start, r.off_lit, r.value};
        if (i == nr - 1) vp[nr] = LRun{r.start + r.count, 0u, 0u};        // sentinel: end of the last run
      }
    }
    LRun* dp = druns(c);
    for (uint32_t i = tid; i < nd; i += BLOCK) {
      const RunDesc r = runs[dlo + i];
      dp[i] = LRun{r.start, r.off_lit, r.value};
      if (i == nd - 1) dp[nd] = LRun{r.start + r.count, 0u, 0u};
    }
  }
  // run-block tables of the string columns' value runs (the runs just staged)
  const uint32_t nblk = (tile_nrows + 63u) / 64u;
  __syncthreads();
#pragma unroll
  for (int s = 0; s < NSTR; s++) {
    const int c = 2 + s;
    const uint32_t nr = ((uni(L.hot[c].present)) ? uni(L.hot[c].nruns) : 0u);
    if (!nr) continue;
    const uint32_t vb = uni(L.hot[c].vbase);
    for (uint32_t b = tid; b <= nblk; b += BLOCK) L.rblk[s][b] = uint8_t(find_run(vruns(c), int(nr), vb + 64u * b));
  }
#pragma unroll
  for (int s = 0; s < NSTR; s++) {
    const int c = 2 + s;
    if (!uni(L.hot[c].lut_on)) continue;
    const uint32_t* remap = uptr(L.hot[c].remap);
    const uint32_t* tab = uptr(L.sp[s].strtab);
    const uint32_t dict_n = Sp->cols[c].tcols[t].dict_n;
    for (uint32_t i = tid; i < dict_n; i += BLOCK) {
      const uint32_t g = remap[i];
      L.lut[s][i] = tab ? tab[g] : g;
    }
  }
  if (TT) {
    const uint32_t words = ((1u << (2 * P.nleaves)) + 31) / 32;
    for (uint32_t i = tid; i < words; i += BLOCK) L.truth[i] = P.truth[i];
    if (NSTR > 1 && P.late_mask)
      for (uint32_t i = tid; i < words; i += BLOCK) {
        L.truth_e[i] = P.truth_early[i];
        L.truth_l[i] = P.truth_late[i];
      }
  }
  for (int i = tid; i < HS; i += BLOCK) {
    L.hkey[i] = EMPTY;
    if constexpr (SLIM) {
      L.hval[i] = AGG == AGG_MIN ? ~0ull : 0ull;
    } else {
      L.hrows[i] = 0;
      L.hcnt[i] = 0;
      L.hlo[i] = 0.0;
      if (AGG == AGG_MIN) reinterpret_cast<unsigned long long*>(L.hhi)[i] = ~0ull;
      else L.hhi[i] = 0.0;
    }
  }
  const bool stamp = P.stamps != nullptr;   // diagnostics only
  if (stamp && tid == 0)
    for (int k = 0; k < LK_NSTAMP; k++) L.stamp[k] = 0;
  __syncthreads();

  // s_memtime section totals (wave 0): 0 prologue, 1 def levels, 2 decode, 3 fold, 4 filter, 5 compaction,
  // 6 prefetch, 7 streaming
  unsigned long long st_mark = stamp ? __builtin_amdgcn_s_memtime() : 0;
  if (stamp && tid == 0) L.stamp[0] = st_mark - st0;
#define LK_STAMP(k)                                                \
  if (stamp && tid == 0) {                                         \
    const unsigned long long now_ = __builtin_amdgcn_s_memtime();   \
    L.stamp[k] += now_ - st_mark;                                  \
    st_mark = now_;                                                \
  }

  // plan bytes of this wave (uniform): wave 0 accounts the tile's metadata reads (TileDesc, TileCols, staged
  // runs, dictionary lookups); every wave its own gathers
  uint64_t pbytes = 0;
  const bool count_plan = P.plan_bytes != nullptr;   // uniform
  if (wave == 0 && count_plan) {
    pbytes += sizeof(TileDesc);
#pragma unroll
    for (int c = 0; c < NC; c++) {
      if (!uni(L.hot[c].present)) continue;
      pbytes += sizeof(TileCol) + uint64_t(c >= 2 ? uni(L.hot[c].nruns) : 0u) * sizeof(RunDesc) +
                uint64_t(uni(L.hot[c].ndruns)) * sizeof(RunDesc) + (uni(L.hot[c].lut_on) ? uint64_t(uni(L.hot[c].dict_n)) * 8u : 0u);
    }
  }
  uint32_t last_ts_line = ~0u, last_v_line = ~0u;

  // per-tile column flags as scalar bit masks (bit c): present, has NULLs, small-dictionary lookup in LDS
  uint32_t presm = 0, nullm = 0, lutm = 0;
#pragma unroll
  for (int c = 0; c < NC; c++) {
    presm |= (uni(L.hot[c].present) ? 1u : 0u) << c;
    nullm |= (uni(L.hot[c].present) && uni(L.hot[c].has_nulls) ? 1u : 0u) << c;
    lutm |= (uni(L.hot[c].lut_on) ? 1u : 0u) << c;
  }
  presm = uni(presm), nullm = uni(nullm), lutm = uni(lutm);
  // Late materialization on this tile: late string columns are decoded per listed row (value index = row, so
  // neither they nor the timestamps may hold NULLs here); otherwise every column is decoded up front.
  const uint32_t latem = (TT && NSTR > 1) ? P.late_mask : 0u;
  const bool late_ok = latem != 0 && (nullm & ((latem << 2) | 1u)) == 0;
  const uint32_t skipm = late_ok ? latem : 0u;   // string columns not decoded in phase B

  // Fast early filter: when phase B decodes a single string column (the only one, or the early column of a
  // late tile) that has no NULLs here and at most 64 dictionary entries, its filter outcome depends on the code
  // alone: a 64-bit mask over the codes (this tile's chunk dictionary) replaces the lookup + fold + truth table
  // per row, and listed rows carry the code until the compaction, where it becomes their group-dim term.
  const int ecol = (NSTR > 1 && late_ok) ? __builtin_ctz(~latem & ((1u << NSTR) - 1u)) : 0;
  // (NSTR <= 3: with more columns the extra live state pushes the kernel past its VGPR budget.)
  const bool fast = TT && NSTR <= 3 && (NSTR == 1 || late_ok) && ((presm >> (2 + ecol)) & 1u) &&
                    !((nullm >> (2 + ecol)) & 1u) && ((lutm >> (2 + ecol)) & 1u) &&
                    uni(L.hot[2 + ecol].dict_n) <= 64u && uni(L.hot[2 + ecol].nruns) > 0u;
  unsigned long long emask = 0;
  if (fast) {
    const uint32_t* tt = (NSTR > 1 && late_ok) ? L.truth_e : L.truth;
    const uint32_t lbase = uni(L.sp[ecol].lbase), lmask = uni(L.sp[ecol].lmask), lf = uni(L.leaf_false);
    bool pass = false;
    if (uint32_t(lane) < uni(L.hot[2 + ecol].dict_n)) {
      const uint32_t bits = (L.lut[ecol][lane] >> 24) << lbase;
      const uint32_t T = bits & lmask & ~lf, F = (~bits & lmask) | lf;
      const uint32_t ix = T | (F << P.nleaves);
      pass = (tt[ix >> 5] >> (ix & 31)) & 1u;
    }
    emask = __ballot(pass);
  }
  const bool emask32 = fast && uni(L.hot[2 + ecol].dict_n) <= 32u;   // uniform
  const uint32_t emask_lo = uint32_t(emask);

  // Per column: index (tile-relative) of the sub-tile's first value: its first row for a column without
  // NULLs, the running non-NULL count for a nullable one.
  uint32_t vrun[NC];
#pragma unroll
  for (int c = 0; c < NC; c++) vrun[c] = 0;

  // Packed groups of a sub-tile (first row s0, first values vfirst_next[c]): def levels of rows s0+8t..,
  // dictionary indices of its values 8t.. (nullable: value-major). Issued one sub-tile ahead.
  G8 gd[NC], gv[NSTR];
  auto prefetch = [&](uint32_t s0, const uint32_t* vnext) {
#pragma unroll
    for (int c = 0; c < NC; c++) {
      gd[c] = G8{};
      if (!((nullm >> c) & 1u)) continue;
      const __amdgpu_buffer_rsrc_t drs = make_rsrc(L.hot[c].defs, L.hot[c].defs_len + 8);
      gd[c] = g8_issue(drs, druns(c), int(uni(L.hot[c].ndruns)), uni(L.hot[c].rip) + s0 + 8 * tid, 1, false);
    }
#pragma unroll
    for (int s = 0; s < NSTR; s++) {
      const int c = 2 + s;
      gv[s] = G8{};
      const uint32_t nr = ((presm >> c) & 1u) ? uni(L.hot[c].nruns) : 0u;
      if (!nr || ((skipm >> s) & 1u)) continue;
      const __amdgpu_buffer_rsrc_t vrs = make_rsrc(L.hot[c].vals, L.hot[c].vals_len + 8);
      const uint32_t vb = uni(L.hot[c].vbase);
      gv[s] = g8_issue(vrs, vruns(c), int(nr), vb + vnext[c] + 8 * tid, int(uni(L.hot[c].bw)), true, L.rblk[s],
                       nblk, vb);
    }
  };
  prefetch(0, vrun);

  // streaming state: timestamp/value buffers of the tile's pages, window, glob cell base
  const bool pres1 = (presm >> 1) & 1u;
  const __amdgpu_buffer_rsrc_t rs0 = make_rsrc(L.hot[0].vals, L.hot[0].vals_len);
  const __amdgpu_buffer_rsrc_t rs1 = make_rsrc(L.hot[1].vals, pres1 ? L.hot[1].vals_len : 0u);
  const uint32_t vbase0 = uni(L.hot[0].vbase), vbase1 = uni(L.hot[1].vbase);
  const int64_t win_lo = L.win_lo, win_hi = L.win_hi;
  const unsigned long long glob_base = (unsigned long long)uni(L.glob_slot) * P.nbuckets;
  const uint32_t step32 = uint32_t(P.step);
  // Zone-map bucket: when the tile's timestamps (exact min/max of its non-NULL values) all lie in the window
  // and in one step bucket, every listed row's bucket is known without reading its timestamp.
  int64_t tile_b = -1;
  {
    const int64_t tmin = tdp->ts_min, tmax = tdp->ts_max;
    if (tmin >= win_lo && tmax < win_hi) {
      if (P.metrics) {
        if (tmin == tmax && (tmin - P.bucket_base) % P.step == 0) tile_b = (tmin - P.bucket_base) / P.step;
      } else {
        const int64_t b0 = ((tmin - tmin % P.step) - P.bucket_base) / P.step;
        const int64_t b1 = ((tmax - tmax % P.step) - P.bucket_base) / P.step;
        if (b0 == b1) tile_b = b0;
      }
      if (tile_b >= int64_t(P.nbuckets)) tile_b = -1;   // out of the cell space: the per-row path flags it
    }
  }
  const bool one_bucket = tile_b >= 0;
  const bool sketch = AGG == AGG_COUNT && P.sketch != 0u;   // uniform

  Acc acc;
  acc_reset<AGG>(acc, EMPTY);
  uint2* wlist = L.list[wave];
  uint32_t* own = reinterpret_cast<uint32_t*>(wlist) + 8 * lane;   // the thread's 8 pk slots

  // One chunk: up to PSN*64 listed rows of a wave, loads in flight (2 slots with 3+ string columns: VGPRs).
  constexpr int PSN = NSTR >= 3 ? 2 : PS;
  // Late columns: slot k = the k-th set bit of latem (at most NSTR - 1: the early column is never late).
  constexpr int NLS = NSTR > 1 ? NSTR - 1 : 1;
  uint32_t late_col[NLS];
#pragma unroll
  for (int k = 0; k < NLS; k++) {
    uint32_t m = latem;
    for (int q = 0; q < k && m; q++) m &= m - 1;
    late_col[k] = m ? uint32_t(__builtin_ctz(m)) : 0xffu;   // string column index, 0xff: slot unused
  }
  using Chunk = ChunkT<PSN>;
  auto issue = [&](auto& ch, uint32_t cb, uint32_t nlist, uint32_t vb0, uint32_t vb1) {
    constexpr int NS = std::remove_reference_t<decltype(ch)>::kSlots;
    ch.n = min(nlist - cb, uint32_t(NS * 64));
    ch.vok = 0;
    ch.live = 0;
#pragma unroll
    for (int j = 0; j < NS; j++) {
      ch.ts[j] = v2u{0u, 0u};
      ch.v[j] = v2u{0u, 0u};
      ch.gid[j] = 0;
      if (uint32_t(j * 64) >= ch.n) continue;                                  // uniform
      const uint32_t i = j * 64 + lane;
      const bool live = i < ch.n;
      const uint2 en = live ? wlist[cb + i] : make_uint2(0u, 0u);
      ch.gid[j] = en.x;
      const uint32_t tv = en.y & 0x7ffu, vv = (en.y >> 11) & 0x7ffu;
      const bool vok = live && ((en.y >> 22) & 1u);
      ch.vok |= uint32_t(vok) << j;
      ch.live |= uint32_t(live) << j;
      if (!one_bucket) {
        ch.ts[j] = __builtin_amdgcn_raw_buffer_load_b64(rs0, live ? (vb0 + tv) * 8u : OOB, 0, 0);
        if (count_plan) pbytes += 128u * new_lines(live, (vb0 + tv) * 8u, last_ts_line);
      }
      if (AGG != AGG_COUNT || sketch) {
        ch.v[j] = __builtin_amdgcn_raw_buffer_load_b64(rs1, vok ? (vb1 + vv) * 8u : OOB, 0, 0);
        if (count_plan) pbytes += 128u * new_lines(vok, (vb1 + vv) * 8u, last_v_line);
      }
    }
  };
  // One row per lane (the late stage's survivors, in place: no compaction), slot 0.
  auto issue_one = [&](auto& ch, bool live, uint32_t gid, uint32_t ey, uint32_t vb0, uint32_t vb1) {
    constexpr int NS = std::remove_reference_t<decltype(ch)>::kSlots;
    ch.n = 64;
#pragma unroll
    for (int j = 0; j < NS; j++) {
      ch.ts[j] = v2u{0u, 0u};
      ch.v[j] = v2u{0u, 0u};
      ch.gid[j] = 0;
    }
    ch.gid[0] = gid;
    const uint32_t tv = ey & 0x7ffu, vv = (ey >> 11) & 0x7ffu;
    const bool vok = live && ((ey >> 22) & 1u);
    ch.vok = uint32_t(vok);
    ch.live = uint32_t(live);
    if (!one_bucket) {
      ch.ts[0] = __builtin_amdgcn_raw_buffer_load_b64(rs0, live ? (vb0 + tv) * 8u : OOB, 0, 0);
      if (count_plan) pbytes += 128u * new_lines(live, (vb0 + tv) * 8u, last_ts_line);
    }
    if (AGG != AGG_COUNT || sketch) {
      ch.v[0] = __builtin_amdgcn_raw_buffer_load_b64(rs1, vok ? (vb1 + vv) * 8u : OOB, 0, 0);
      if (count_plan) pbytes += 128u * new_lines(vok, (vb1 + vv) * 8u, last_v_line);
    }
  };
  auto consume = [&](const auto& ch) {
    constexpr int NS = std::remove_reference_t<decltype(ch)>::kSlots;
#pragma unroll
    for (int j = 0; j < NS; j++) {
      if (uint32_t(j * 64) >= ch.n) break;                                     // uniform
      const int64_t ts = (int64_t)(((uint64_t)ch.ts[j].y << 32) | ch.ts[j].x);
      bool ok = ((ch.live >> j) & 1u) && (one_bucket || (ts >= win_lo && ts < win_hi));   // BaseExpr.scala:159-161
      int64_t b = 0;
      if (one_bucket) {
        b = tile_b;
      } else if (P.fast_div) {
        // d < 2^32: q from the double reciprocal is off by at most one; fix with the remainder
        const uint32_t d = uint32_t(ts - P.bucket_base);
        uint32_t q = uint32_t(double(d) * P.inv_step);
        int64_t rm = int64_t(d) - int64_t(q) * step32;
        q = rm < 0 ? q - 1 : (rm >= int64_t(step32) ? q + 1 : q);
        rm = int64_t(d) - int64_t(q) * step32;
        if (P.metrics && rm != 0 && ok) {
          atomicOr(P.flags, FLAG_METRICS_UNALIGNED);
          ok = false;
        }
        b = q;
      } else if (ok) {
        if (P.metrics) {
          const int64_t d = ts - P.bucket_base;
          b = d / P.step;
          if (d - b * P.step != 0) {
            atomicOr(P.flags, FLAG_METRICS_UNALIGNED);
            ok = false;
          }
        } else {
          b = ((ts - ts % P.step) - P.bucket_base) / P.step;        // ts - ts % step (fmod, truncation)
        }
      }
      if (!ok) continue;
      if (b < 0 || (uint64_t)b >= P.nbuckets) {
        atomicOr(P.flags, FLAG_CELL_RANGE);
        continue;
      }
      unsigned long long cell = (glob_base + (unsigned long long)b) * P.ngroups + ch.gid[j];
      const double v = __longlong_as_double((long long)(((uint64_t)ch.v[j].y << 32) | ch.v[j].x));
      bool vvalid = (ch.vok >> j) & 1u;
      if constexpr (AGG == AGG_COUNT) {
        if (sketch) {   // DDSketch bin of the value (NULL: 0.0, counted); every passing row counts
          cell = cell * DD_NBINS + dd_bin(P, vvalid ? v : 0.0);
          vvalid = true;
        }
      }
      if (cell != acc.key) {
        lds_merge<AGG, HASH, SLIM>(L, P, acc);
        acc_reset<AGG>(acc, cell);
      }
      min_nan_check<AGG>(P, vvalid, v);
      acc_add<AGG>(acc, vvalid, v);
    }
  };
  // Software pipeline: the first 64 listed rows of sub-tile k are issued into ring slot k % DEPTH and consumed
  // DEPTH sub-tiles later, after that many decodes have overlapped their timestamp/value (or late-column) loads:
  // the loop is unrolled DEPTH times so every ring slot keeps its own registers (moving a register a load is still
  // writing would wait for the load).  Further listed rows of a sub-tile (dense filters) stream at once.
  constexpr int DEPTH = LK_DEPTH(NSTR);
  const bool stream_on = !(P.ablate & 1);

  // Late stage (late_ok tiles), one row per lane: the listed row's late columns' packed words in flight.
  // Pipelined: the loads of a sub-tile's first 64 listed rows land during the next sub-tile's decode; the
  // survivors' timestamp/value loads land during the one after (through `pend`).
  struct LPend {
    uint2 en;              // list entry
    v2u w[NLS];            // packed words of the late columns
    uint32_t meta[NLS];    // bit 31: bit-packed (bits 0..5: bit shift), else the RLE run's value
    uint32_t n;            // listed rows in the chunk (uniform; 0: none)
    uint32_t vb0, vb1;     // timestamp / value bases of the chunk's sub-tile (uniform)
  };
  auto late_issue = [&](LPend& lp, uint32_t cb, uint32_t nlist, uint32_t sub, uint32_t vb0, uint32_t vb1) {
    lp.n = min(nlist - cb, 64u);
    lp.vb0 = vb0;
    lp.vb1 = vb1;
    const bool live = uint32_t(lane) < lp.n;
    lp.en = live ? wlist[cb + lane] : make_uint2(0u, 0u);
    const uint32_t row = lp.en.y & 0x7ffu;   // = the timestamp value index (no NULL timestamps here)
#pragma unroll
    for (int k = 0; k < NLS; k++) {
      lp.w[k] = v2u{0u, 0u};
      lp.meta[k] = 0;
      const uint32_t sl = late_col[k];
      if (sl == 0xffu) continue;                                             // uniform
      const uint32_t c = 2 + sl;
      const uint32_t nr = ((presm >> c) & 1u) ? uni(L.hot[c].nruns) : 0u;
      if (!nr) continue;                                                     // absent column
      const LRun* runs = vruns(int(c));
      const uint32_t vb = uni(L.hot[c].vbase);
      const uint32_t v = vb + sub + row;                                    // no NULLs: value index = row
      const LRun r = runs[nr == 1 ? 0 : find_run_blk(runs, L.rblk[sl], nblk, vb, v)];
      const bool lit = (r.off_lit & 0x80000000u) != 0;
      const uint32_t bit = (v - r.start) * uni(L.hot[c].bw);
      const uint32_t byte = (r.off_lit & 0x7fffffffu) + (bit >> 3);
      const __amdgpu_buffer_rsrc_t vrs = make_rsrc(L.hot[c].vals, L.hot[c].vals_len + 8);
      lp.w[k] = __builtin_amdgcn_raw_buffer_load_b64(vrs, (live && lit) ? (byte & ~3u) : OOB, 0, 0);
      uint32_t no_carry = ~0u;   // late columns' packed words: lines of this chunk (runs revisit lines rarely)
      if (count_plan) pbytes += 128u * new_lines(live && lit, byte & ~3u, no_carry);
      lp.meta[k] = lit ? (0x80000000u | ((byte & 3u) * 8u + (bit & 7u))) : r.value;
    }
  };
  // Late conjuncts + late group dims of the chunk's rows; returns whether the lane's row passes.
  auto late_eval = [&](const LPend& lp, uint32_t& gid) -> bool {
    gid = lp.en.x;
    uint32_t T = 0, F = 0;
#pragma unroll
    for (int k = 0; k < NLS; k++) {
      const uint32_t sl = late_col[k];
      if (sl == 0xffu) continue;                                             // uniform
      const uint32_t c = 2 + sl;
      const uint32_t dstride = uni(L.sp[sl].dim_stride), lbase = uni(L.sp[sl].lbase);
      const uint32_t lmask = uni(L.sp[sl].lmask);
      if (!((presm >> c) & 1u) || !uni(L.hot[c].nruns)) {                   // absent: NULL in every row
        gid += uni(L.sp[sl].dim_null) * dstride;
        F |= uni(L.sp[sl].hmask);
        continue;
      }
      const uint32_t bw = uni(L.hot[c].bw);
      const uint64_t x = ((uint64_t)lp.w[k].y << 32) | lp.w[k].x;
      const uint32_t idx = (lp.meta[k] >> 31) ? uint32_t(x >> (lp.meta[k] & 63u)) & (bw >= 32 ? ~0u : ((1u << bw) - 1u))
                                              : lp.meta[k];
      uint32_t packed;
      if ((lutm >> c) & 1u) {
        packed = L.lut[sl][idx < LUT_CAP ? idx : 0u];
      } else {
        const uint32_t g = uptr(L.hot[c].remap)[idx];
        const uint32_t* tab = uptr(L.sp[sl].strtab);
        packed = tab ? tab[g] : g;
      }
      const uint32_t bits = (packed >> 24) << lbase;
      gid += (packed & DIM_MASK) * dstride;
      T |= bits & lmask;
      F |= ~bits & lmask;
    }
    const uint32_t leaf_false = uni(L.leaf_false);
    T &= ~leaf_false;
    F |= leaf_false;
    const uint32_t ix = T | (F << P.nleaves);
    return uint32_t(lane) < lp.n && ((L.truth_l[ix >> 5] >> (ix & 31)) & 1u);
  };
  LPend lpend;
  lpend.n = 0;

  auto step = [&](auto& ring, uint32_t sub) __attribute__((always_inline)) {
    const uint32_t nsub = min(uint32_t(SUBT), tile_nrows - sub);
    const uint32_t r0 = 8u * tid;   // the thread's first row in the sub-tile
    const uint32_t inb = r0 < nsub ? (nsub - r0 >= 8 ? 0xffu : (1u << (nsub - r0)) - 1u) : 0u;

    // ============ A. validity bytes and value indices ============
    uint32_t vb[NC], vfirst[NC], ctot[NC];   // non-NULL rows (bit e = row r0+e), first value index, count
#pragma unroll
    for (int c = 0; c < NC; c++) {
      vb[c] = ((presm >> c) & 1u) ? inb : 0u;
      vfirst[c] = r0;
      ctot[c] = nsub;
      if ((nullm >> c) & 1u) {
        const __amdgpu_buffer_rsrc_t drs = make_rsrc(L.hot[c].defs, L.hot[c].defs_len + 8);
        vb[c] = g8_bits(gd[c], drs, druns(c), int(uni(L.hot[c].ndruns)),
                        uni(L.hot[c].rip) + sub + r0) & inb;
        uint32_t wt;
        vfirst[c] = wave_prefix16(__popc(vb[c]), wt);
        if (lane == 0) L.wsum[c][wave] = wt;
      }
    }
    if (nullm) {
      __syncthreads();
#pragma unroll
      for (int c = 0; c < NC; c++) {
        if (!((nullm >> c) & 1u)) continue;
        uint32_t before = 0, all = 0;
#pragma unroll
        for (int w = 0; w < WAVES; w++) {
          const uint32_t x = L.wsum[c][w];
          before += w < wave ? x : 0u;
          all += x;
        }
        vfirst[c] += before;
        ctot[c] = uni(all);
      }
      __syncthreads();   // wsum is rewritten by the next sub-tile
    }
    LK_STAMP(1)

    // ============ B. string columns -> leaf T/F bits and group id per row ============
    uint32_t leafT[8], leafF[8], gid[8];
#pragma unroll
    for (int e = 0; e < 8; e++) leafT[e] = 0, leafF[e] = 0, gid[e] = 0;
    uint32_t passf = 0;   // fast early filter: pass bits straight from the codes
#pragma unroll
    for (int s = 0; s < NSTR; s++) {
      const int c = 2 + s;
      if ((skipm >> s) & 1u) continue;   // late column: decoded per listed row in phase E
      if (fast && s == ecol) {           // uniform: codes only (gid[] carries them to the compaction)
        uint32_t dec[8];
        g8_unpack(gv[s], make_rsrc(L.hot[c].vals, L.hot[c].vals_len + 8), vruns(c),
                  int(uni(L.hot[c].nruns)), uni(L.hot[c].vbase) + vrun[c] + r0, int(uni(L.hot[c].bw)),
                  ctot[c] > r0 ? ctot[c] - r0 : 0u, own, [](uint32_t i) { return i; }, dec);
        if (emask32) {   // <= 32 codes: one 32-bit shift per row
#pragma unroll
          for (int e = 0; e < 8; e++) {
            gid[e] = dec[e];
            passf |= ((emask_lo >> (dec[e] & 31u)) & 1u) << e;
          }
        } else {
#pragma unroll
          for (int e = 0; e < 8; e++) {
            gid[e] = dec[e];
            passf |= uint32_t((emask >> (dec[e] & 63u)) & 1ull) << e;
          }
        }
        continue;
      }
      const uint32_t nr = ((presm >> c) & 1u) ? uni(L.hot[c].nruns) : 0u;
      uint32_t packed[8];
#pragma unroll
      for (int e = 0; e < 8; e++) packed[e] = 0;
      if (nr) {
        const __amdgpu_buffer_rsrc_t vrs = make_rsrc(L.hot[c].vals, L.hot[c].vals_len + 8);
        const LRun* runs = vruns(c);
        const int bw = int(uni(L.hot[c].bw));
        const uint32_t v0 = uni(L.hot[c].vbase) + vrun[c] + r0;   // this thread's group: values r0.. of the sub-tile
        const uint32_t left = ctot[c] > r0 ? ctot[c] - r0 : 0u;
        uint32_t dec[8];
        if ((lutm >> c) & 1u) {
          const uint32_t* lt = L.lut[s];
          g8_unpack(gv[s], vrs, runs, int(nr), v0, bw, left, own, [&](uint32_t i) { return lt[i < LUT_CAP ? i : 0u]; },
                    dec);
        } else {
          const uint32_t* remap = uptr(L.hot[c].remap);
          const uint32_t* tab = uptr(L.sp[s].strtab);
          g8_unpack(gv[s], vrs, runs, int(nr), v0, bw, left, own, [&](uint32_t i) {
            const uint32_t g = remap[i];
            return tab ? tab[g] : g;
          }, dec);
        }
        if (!((nullm >> c) & 1u)) {
#pragma unroll
          for (int e = 0; e < 8; e++) packed[e] = dec[e];
        } else {
          // values are value-major: publish them (value i lives in wave i/512's list area), then gather each
          // row's value by its value index
#pragma unroll
          for (int e = 0; e < 8; e++) own[e] = dec[e];
          __syncthreads();
          const uint32_t* pkw = reinterpret_cast<const uint32_t*>(L.list);
          uint32_t vi = vfirst[c];
#pragma unroll
          for (int e = 0; e < 8; e++) {
            const bool valid = (vb[c] >> e) & 1u;
            packed[e] = valid ? pkw[((vi >> 9) << 10) | (vi & 511u)] : 0u;
            vi += valid;
          }
          __syncthreads();   // the area is rewritten by the next column / the wave's list
        }
      }
      LK_STAMP(2)
      const uint32_t dstride = uni(L.sp[s].dim_stride), dnull = uni(L.sp[s].dim_null);
      const uint32_t lbase = uni(L.sp[s].lbase), lmask = uni(L.sp[s].lmask), hmask = uni(L.sp[s].hmask);
      const uint32_t valid = nr ? vb[c] : 0u;
#pragma unroll
      for (int e = 0; e < 8; e++) {
        const bool ok = (valid >> e) & 1u;
        const uint32_t bits = (packed[e] >> 24) << lbase;
        gid[e] += (ok ? (packed[e] & DIM_MASK) : dnull) * dstride;
        leafT[e] |= ok ? (bits & lmask) : 0u;
        leafF[e] |= ok ? (~bits & lmask) : hmask;   // IS NOT NULL on NULL: FALSE; others NULL
      }
      LK_STAMP(3)
    }

    // plan bytes of the streams decoded in full for this sub-tile (wave 0): def levels, early string columns
    if (wave == 0 && count_plan) {
#pragma unroll
      for (int c = 0; c < NC; c++)
        if ((nullm >> c) & 1u) pbytes += (nsub + 7u) / 8u;
#pragma unroll
      for (int s2 = 0; s2 < NSTR; s2++) {
        const int c = 2 + s2;
        if (((skipm >> s2) & 1u) || !((presm >> c) & 1u) || !uni(L.hot[c].nruns)) continue;
        pbytes += (uint64_t(ctot[c]) * uni(L.hot[c].bw) + 7u) / 8u;
      }
    }

    // ============ C. filter -> pass byte (NULL / absent timestamps fail the window) ============
    uint32_t passb = 0;
    if (fast) {
      passb = passf & vb[0];
    } else {
      const uint32_t leaf_false = uni(L.leaf_false);
      const uint32_t nleaves = P.nleaves;
#pragma unroll
      for (int e = 0; e < 8; e++) {
        const uint32_t T = leafT[e] & ~leaf_false, F = leafF[e] | leaf_false;
        bool ok;
        if (TT) {
          const uint32_t ix = T | (F << nleaves);
          ok = ((late_ok ? L.truth_e : L.truth)[ix >> 5] >> (ix & 31)) & 1u;
        } else {
          ok = interpret(P, T, F);
        }
        passb |= uint32_t(ok) << e;
      }
      passb &= vb[0];
    }
    LK_STAMP(4)

    // ============ D. compact the wave's passing rows into its list, in row order ============
    uint32_t nlist;
    {
      uint32_t k = wave_prefix16(__popc(passb), nlist);
      if (!(nullm & 3u)) {
        // no NULL timestamps / values here: value index = row; a loop over the set pass bits (sparse filters
        // write few entries; the loop runs max-popcount times, not 8)
        const uint32_t vok_all = (vb[1] != 0u) ? 1u : 0u;   // value column present on this tile
        uint32_t m = passb;
        while (m) {
          const uint32_t e = uint32_t(__builtin_ctz(m));
          m &= m - 1u;
          uint32_t g = gid[0];
#pragma unroll
          for (int q = 1; q < 8; q++) g = (e == uint32_t(q)) ? gid[q] : g;
          const uint32_t r = r0 + e;
          wlist[k++] = make_uint2(g, r | (r << 11) | (vok_all << 22));
        }
      } else {
        uint32_t tv = vfirst[0], vv = vfirst[1];
#pragma unroll
        for (int e = 0; e < 8; e++) {
          const uint32_t vok = (vb[1] >> e) & 1u;
          if ((passb >> e) & 1u) {
            wlist[k] = make_uint2(gid[e], tv | (vv << 11) | (vok << 22));
            k++;
          }
          tv += (vb[0] >> e) & 1u;
          vv += vok;
        }
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (fast) {   // listed rows only: the early column's code -> its group-dim term
      const uint32_t dstride = uni(L.sp[ecol].dim_stride);
      const uint32_t* lt = L.lut[ecol];
      for (uint32_t cb = 0; cb < nlist; cb += 64) {                           // uniform
        const uint32_t i = cb + lane;
        if (i < nlist) wlist[i].x = (lt[wlist[i].x & (LUT_CAP - 1)] & DIM_MASK) * dstride;
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
    LK_STAMP(5)

    // next sub-tile's packed groups: in flight while this sub-tile streams
    uint32_t vnext[NC];
#pragma unroll
    for (int c = 0; c < NC; c++) vnext[c] = vrun[c] + ctot[c];
    if (sub + SUBT < tile_nrows) prefetch(sub + SUBT, vnext);
    LK_STAMP(6)

    // ============ E. stream timestamp + value of the wave's listed rows, bucket, aggregate ============
    const uint32_t vb0 = vbase0 + vrun[0], vb1 = vbase1 + vrun[1];
    bool late_done = false;
    if constexpr (NSTR > 1) {
      if (late_ok) {
        // E'. late tiles, three stages in flight across sub-tiles:
        //   stream rows of sub-tile k-2's survivors (loads issued one decode ago) -> aggregate;
        //   late columns of sub-tile k-1's first 64 listed rows -> survivors' timestamp/value loads;
        //   late-column loads of this sub-tile's first 64 listed rows.
        // Further listed rows (dense early filters) run the late stage and stream at once.
        late_done = true;
        if (stream_on) consume(ring);
        ring.n = 0;
        if (lpend.n) {
          uint32_t g;
          const bool pass = late_eval(lpend, g);
          if (stream_on) issue_one(ring, pass, g, lpend.en.y, lpend.vb0, lpend.vb1);
          lpend.n = 0;
        }
        if (nlist) late_issue(lpend, 0, nlist, sub, vb0, vb1);
        for (uint32_t cb = 64; cb < nlist; cb += 64) {                          // uniform
          LPend lp;
          late_issue(lp, cb, nlist, sub, vb0, vb1);
          uint32_t g;
          const bool pass = late_eval(lp, g);
          if (stream_on) {
            ChunkT<1> ch;
            issue_one(ch, pass, g, lp.en.y, vb0, vb1);
            consume(ch);
          }
        }
      }
    }
    // The ring slot's chunk (issued DEPTH sub-tiles ago) has had DEPTH decodes to land; this sub-tile's first
    // 64 listed rows take its place.  Further chunks (dense filters) stream at once.
    if (stream_on && !late_done) {
      consume(ring);
      ring.n = 0;
      if (nlist) issue(ring, 0, nlist, vb0, vb1);
      for (uint32_t cb = 64; cb < nlist; cb += PSN * 64) {
        Chunk ch;
        issue(ch, cb, nlist, vb0, vb1);
        consume(ch);
      }
    }
#pragma unroll
    for (int c = 0; c < NC; c++) vrun[c] = vnext[c];
    // the list entries were copied to registers; the wave rewrites its list only after this point
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    LK_STAMP(7)
  };
  ChunkT<1> q0, q1, q2;
  q0.n = q1.n = q2.n = 0;
  for (uint32_t sub = 0; sub < tile_nrows; sub += DEPTH * SUBT) {
    step(q0, sub);
    if constexpr (DEPTH > 1) {
      if (sub + SUBT < tile_nrows) step(q1, sub + SUBT);
    }
    if constexpr (DEPTH > 2) {
      if (sub + 2 * SUBT < tile_nrows) step(q2, sub + 2 * SUBT);
    }
  }
  // drain: the ring's chunks still in flight, then the last late chunk's survivors
  if (stream_on) {
    consume(q0);
    if constexpr (DEPTH > 1) consume(q1);
    if constexpr (DEPTH > 2) consume(q2);
  }
  if constexpr (NSTR > 1) {
    if (lpend.n) {
      uint32_t g;
      const bool pass = late_eval(lpend, g);
      if (stream_on) {
        ChunkT<1> ch;
        issue_one(ch, pass, g, lpend.en.y, lpend.vb0, lpend.vb1);
        consume(ch);
      }
    }
  }
#undef LK_STAMP
  if (stamp && tid == 0) {
    unsigned long long* o = P.stamps + LK_NSTAMP * (size_t(blockIdx.y) * P.max_tiles + blockIdx.x);
#pragma unroll
    for (int k = 0; k < LK_NSTAMP; k++) o[k] = L.stamp[k] | (k == 0 ? 1ull << 63 : 0ull);   // bit 63: block ran
  }
  if (P.plan_bytes && lane == 0 && pbytes) atomicAdd(P.plan_bytes, (unsigned long long)pbytes);
  lds_merge<AGG, HASH, SLIM>(L, P, acc);
  __syncthreads();
  for (int i = tid; i < HS; i += BLOCK) {
    if (L.hkey[i] == EMPTY) continue;
    if constexpr (SLIM) {   // lean table: MIN/MAX existence via the extreme, COUNT rows == non-NULL count
      const unsigned long long v = L.hval[i];
      if (AGG == AGG_COUNT) global_merge<AGG, HASH>(P, L.hkey[i], uint32_t(v), uint32_t(v), 0.0, 0.0, 0ull);
      else global_merge<AGG, HASH>(P, L.hkey[i], 1u, 1u, 0.0, 0.0, v);
    } else {
      global_merge<AGG, HASH>(P, L.hkey[i], L.hrows[i], L.hcnt[i], L.hhi[i], L.hlo[i],
                              reinterpret_cast<unsigned long long*>(L.hhi)[i]);
    }
  }
}

}  // namespace lk
