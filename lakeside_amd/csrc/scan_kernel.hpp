// scan_tiles<AGG, NSTR>: the fused decode -> filter -> bucket -> aggregate kernel (included by kernels.hip).
//
// grid (tile, segment); one 256-thread workgroup per tile (a row range inside one page of every column).
//   prologue: every fact about the tile's columns (stream pointers, run windows, value bases, flags) is read
//     once and staged in LDS together with the run windows, small dictionaries' lookup values (dictionary index
//     -> leaf bits | group-dim id) and the filter truth table.
//   Per 2048-row sub-tile:
//   1. definition levels of every nullable column, run-major: thread i unpacks the byte of rows 8i..8i+7
//      (one bit-packed byte, or the RLE value) into an LDS validity bitmap; one wave per column turns the
//      bitmap into per-64-row prefix counts (value index of every row);
//   2. string columns, one at a time, value-major: thread i unpacks the 8 dictionary indices 8i..8i+7 of the
//      sub-tile's values from one bit-packed group (one or two dword loads, shifts) and writes their lookup
//      values to LDS; then every row (k-major: row j*256 + tid) folds its value into leaf T/F bits and its
//      group id, in registers;
//   3. the filter's truth table (Kleene logic precomputed on the host) gives the pass bit of every row
//      (one ballot per 64 rows); passing rows are compacted, in row order, into an LDS list;
//   4. streaming: timestamps and values are loaded only for listed rows, all loads of a thread issued before
//      the first use; bucket by exact 32-bit reciprocal division; accumulate in a per-thread register cell
//      (time-sorted rows hit it), spilling to an LDS hash table (LDS atomics; sums as compensated hi/lo with a
//      returning-atomic TwoSum).
//   tile end: LDS cells -> global table with device atomics (count/min/max exact, sums within 1 ulp).
#pragma once
#include "device_common.hpp"

namespace lk {

constexpr int WORDS = SUBT / 64;         // 64-row groups per sub-tile (32)
constexpr int PS = 4;                    // listed rows per thread loaded together in phase 4

struct ColHot {                          // one column over one tile, staged once per tile
  const uint8_t* vals;                   // value stream (absolute)
  const uint8_t* defs;                   // def-level stream (absolute)
  const uint32_t* remap;                 // chunk dictionary remap (absolute)
  uint32_t vals_len, defs_len;
  uint32_t vbase, rip, nruns, ndruns;
  uint32_t bw, has_nulls, present, lut_on;
};

template <int NSTR>
struct Lds {
  LRun pool[(2 + NSTR) * 2 * (RUN_CAP + 1)];   // run windows: [column][value runs | def runs], + sentinel
  uint32_t lut[NSTR][LUT_CAP];
  uint32_t truth[(1u << (2 * TT_MAX_LEAVES)) / 32];
  unsigned long long hkey[HCAP];
  uint32_t hrows[HCAP];
  uint32_t hcnt[HCAP];
  double hhi[HCAP];                      // SUM: hi; MIN/MAX: ordered bits (reinterpreted)
  double hlo[HCAP];
  uint32_t pk[SUBT];                     // decoded lookup values of one string column (value-major); after the
                                         //   last column's fold: the group id of every row (phases 3-4)
  uint16_t list[SUBT];                   // passing rows, in row order
  unsigned long long passw[WORDS];       // pass bitmap
  uint32_t ppre[WORDS + 1];              // its exclusive prefix (+ total)
  unsigned long long nv[2 + NSTR][WORDS];  // validity bitmaps (nullable columns)
  uint32_t npre[2 + NSTR][WORDS + 1];    // their exclusive prefix within the sub-tile (+ total)
  uint32_t vrun[2 + NSTR];               // non-null values of the column before this sub-tile (tile-relative)
  ColHot hot[2 + NSTR];                  // per-tile column state
  StrParam sp[NSTR];                     // per-query string column parameters
  int64_t win_lo, win_hi;
  uint32_t glob_slot, leaf_false;
};

template <int AGG, int NSTR>
__device__ __forceinline__ void lds_merge(Lds<NSTR>& L, const QParams& P, const Acc& a) {
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

// 8 consecutive values [v, v+8) of a hybrid stream (runs staged in LDS, `n` runs + sentinel), bit width
// bw <= 8: one bit-packed group (bw bytes) or the RLE value; other cases fall back to per-value reads.
__device__ __forceinline__ void hybrid_get8(__amdgpu_buffer_rsrc_t rs, const LRun* runs, int n, uint32_t v, int bw,
                                            uint32_t out[8]) {
  const int ri = find_run64(runs, n, v);
  const LRun r = runs[ri];
  const uint32_t end = runs[ri + 1].start;   // sentinel past the last run
  const bool lit = (r.off_lit & 0x80000000u) != 0;
  const bool whole = v + 8 <= end;
  if (whole && !lit) {
#pragma unroll
    for (int e = 0; e < 8; e++) out[e] = r.value;
    return;
  }
  if (whole && bw <= 8) {
    // 8 values = 8*bw <= 64 bits starting at bit `bit`; the 96 bits from the enclosing dword cover them
    const uint32_t bit = (v - r.start) * uint32_t(bw);
    const uint32_t byte = (r.off_lit & 0x7fffffffu) + (bit >> 3);
    const uint32_t al = byte & ~3u;
    const v2u w01 = __builtin_amdgcn_raw_buffer_load_b64(rs, al, 0, 0);
    const uint32_t w2 = __builtin_amdgcn_raw_buffer_load_b32(rs, al + 8, 0, 0);
    const uint32_t sh = (byte & 3u) * 8u + (bit & 7u);                       // <= 31
    const uint64_t lo = ((uint64_t)w01.y << 32) | w01.x;
    const uint64_t x = sh ? ((lo >> sh) | ((uint64_t)w2 << (64 - sh))) : lo;
    const uint32_t mask = (1u << bw) - 1u;
#pragma unroll
    for (int e = 0; e < 8; e++) out[e] = uint32_t(x >> (e * bw)) & mask;
    return;
  }
#pragma unroll
  for (int e = 0; e < 8; e++) {
    const uint32_t ve = v + e;
    out[e] = hybrid_get_buf(rs, runs[find_run64(runs, n, ve)], ve, bw);
  }
}

template <int AGG, int NSTR>
__global__ __launch_bounds__(BLOCK) void scan_tiles(QParams P) {
  __shared__ Lds<NSTR> L;
  constexpr int NC = 2 + NSTR;
  constexpr int PSTRIDE = 2 * (RUN_CAP + 1);
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const unsigned long long lane_lt = (1ull << lane) - 1ull;
  const unsigned long long st0 = P.stamps ? __builtin_amdgcn_s_memtime() : 0;   // diagnostics only

  // ---- segment (grid.y) and tile (grid.x): uniform addresses -> scalar loads, once ----
  const QSeg* Sp = P.segs + blockIdx.y;
  const uint32_t t = blockIdx.x;
  if (t >= Sp->ntiles) return;
  const TileDesc* tdp = Sp->tiles + t;
  if (tdp->ts_max < Sp->win_lo || tdp->ts_min >= Sp->win_hi) return;   // zone map: outside the glob window
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
    }
    L.hot[c] = h;
    L.vrun[c] = 0;
    if (c >= 2) L.sp[c - 2] = P.strp[c - 2];
  }
  if (tid == 0) {
    L.win_lo = Sp->win_lo;
    L.win_hi = Sp->win_hi;
    L.glob_slot = Sp->glob_slot;
    L.leaf_false = Sp->leaf_false;
  }
  __syncthreads();
#pragma unroll
  for (int c = 0; c < NC; c++) {
    if (!uni(L.hot[c].present)) continue;
    const TileCol* tc = Sp->cols[c].tcols + t;
    const RunDesc* runs = Sp->cols[c].runs;
    LRun* vp = L.pool + c * PSTRIDE;
    const uint32_t nr = uni(L.hot[c].nruns), nd = uni(L.hot[c].ndruns);
    const uint32_t rlo = tc->run_lo, dlo = tc->drun_lo;
    for (uint32_t i = tid; i < nr; i += BLOCK) {
      const RunDesc r = runs[rlo + i];
      vp[i] = LRun{r.start, r.off_lit, r.value};
      if (i == nr - 1) vp[nr] = LRun{r.start + r.count, 0u, 0u};          // sentinel: end of the last run
    }
    for (uint32_t i = tid; i < nd; i += BLOCK) {
      const RunDesc r = runs[dlo + i];
      vp[RUN_CAP + 1 + i] = LRun{r.start, r.off_lit, r.value};
      if (i == nd - 1) vp[RUN_CAP + 1 + nd] = LRun{r.start + r.count, 0u, 0u};
    }
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
  if (P.truth) {
    const uint32_t words = ((1u << (2 * P.nleaves)) + 31) / 32;
    for (uint32_t i = tid; i < words; i += BLOCK) L.truth[i] = P.truth[i];
  }
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
  const bool stamp = P.stamps != nullptr;   // diagnostics only
  unsigned long long st_pro = stamp ? __builtin_amdgcn_s_memtime() : 0, st_p1 = 0, st_p2 = 0, st_mark = st_pro;

  for (uint32_t sub = 0; sub < tile_nrows; sub += SUBT) {
    const uint32_t nsub = min(uint32_t(SUBT), tile_nrows - sub);

    // ============ 1. validity bitmaps of nullable columns (run-major, 8 rows per thread) ============
    bool any_nulls = false;
#pragma unroll
    for (int c = 0; c < NC; c++) {
      if (!(uni(L.hot[c].present) && uni(L.hot[c].has_nulls))) continue;
      any_nulls = true;
      const __amdgpu_buffer_rsrc_t drs = make_rsrc(L.hot[c].defs, L.hot[c].defs_len + 8);
      const LRun* druns = L.pool + c * PSTRIDE + RUN_CAP + 1;
      const int nd = int(uni(L.hot[c].ndruns));
      const uint32_t r0 = uni(L.hot[c].rip) + sub + 8 * tid;    // rows 8*tid .. 8*tid+7 of the sub-tile
      uint32_t bits = 0;
      if (8 * uint32_t(tid) < nsub) {
        uint32_t d[8];
        hybrid_get8(drs, druns, nd, r0, 1, d);
#pragma unroll
        for (int e = 0; e < 8; e++) bits |= (d[e] & 1u) << e;
        const uint32_t left = nsub - 8 * tid;
        if (left < 8) bits &= (1u << left) - 1u;
      }
      reinterpret_cast<uint8_t*>(L.nv[c])[tid] = uint8_t(bits);
    }
    if (any_nulls) {
      __syncthreads();
      // per-64-row prefix counts (one wave per column; WORDS = 32 <= 64 lanes)
      for (int c = wave; c < NC; c += BLOCK / 64) {
        if (!(uni(L.hot[c].present) && uni(L.hot[c].has_nulls))) continue;
        const uint32_t cnt = lane < WORDS ? __popcll(L.nv[c][lane]) : 0u;
        uint32_t x = cnt;
        for (int o = 1; o < 64; o <<= 1) {
          const uint32_t y = __shfl_up(x, o, 64);
          if (lane >= o) x += y;
        }
        if (lane < WORDS) L.npre[c][lane] = x - cnt;
        if (lane == WORDS - 1) L.npre[c][WORDS] = x;
      }
      __syncthreads();
    }

    // ============ 2. string columns: value-major decode to LDS, then fold per row ============
    uint32_t leafT[SLOTS], leafF[SLOTS], gid[SLOTS];
#pragma unroll
    for (int j = 0; j < SLOTS; j++) leafT[j] = 0, leafF[j] = 0, gid[j] = 0;
#pragma unroll
    for (int s = 0; s < NSTR; s++) {
      const int c = 2 + s;
      const bool present = uni(L.hot[c].present) != 0;
      const bool nullable = present && uni(L.hot[c].has_nulls) != 0;
      const uint32_t nr = present ? uni(L.hot[c].nruns) : 0u;
      if (nr) {
        // values of this sub-tile: [vs, vs + nvals)
        const uint32_t vs = uni(L.hot[c].vbase) + (nullable ? uni(L.vrun[c]) : sub);
        const uint32_t nvals = nullable ? uni(L.npre[c][WORDS]) : nsub;
        const __amdgpu_buffer_rsrc_t vrs = make_rsrc(L.hot[c].vals, L.hot[c].vals_len + 8);
        const LRun* runs = L.pool + c * PSTRIDE;
        const int bw = int(uni(L.hot[c].bw));
        const bool lut = uni(L.hot[c].lut_on) != 0;
        if (8 * uint32_t(tid) < nvals) {
          uint32_t idx[8];
          hybrid_get8(vrs, runs, int(nr), vs + 8 * tid, bw, idx);
          if (lut) {
#pragma unroll
            for (int e = 0; e < 8; e++) L.pk[8 * tid + e] = L.lut[s][idx[e] < LUT_CAP ? idx[e] : 0];
          } else {
            const uint32_t* remap = uptr(L.hot[c].remap);
            const uint32_t* tab = uptr(L.sp[s].strtab);
            const uint32_t left = nvals - 8 * tid;
#pragma unroll
            for (int e = 0; e < 8; e++) {
              const uint32_t g = remap[e < int(left) ? idx[e] : idx[0]];
              L.pk[8 * tid + e] = tab ? tab[g] : g;
            }
          }
        }
        __syncthreads();
      }
      const uint32_t dstride = uni(L.sp[s].dim_stride), dnull = uni(L.sp[s].dim_null);
      const uint32_t lbase = uni(L.sp[s].lbase), lmask = uni(L.sp[s].lmask), hmask = uni(L.sp[s].hmask);
#pragma unroll
      for (int j = 0; j < SLOTS; j++) {
        const uint32_t r = j * BLOCK + tid;   // row within the sub-tile
        const int w = r >> 6;
        bool valid = false;
        uint32_t vi = 0;
        if (nr && nullable) {
          const unsigned long long m = L.nv[c][w];
          valid = (m >> lane) & 1ull;
          vi = L.npre[c][w] + __popcll(m & lane_lt);
        } else if (nr) {
          valid = r < nsub;
          vi = r;
        }
        const uint32_t packed = valid ? L.pk[vi] : 0u;
        const uint32_t bits = (packed >> 24) << lbase;
        const uint32_t dim = valid ? (packed & DIM_MASK) : dnull;
        gid[j] += dim * dstride;
        leafT[j] |= valid ? (bits & lmask) : 0u;
        leafF[j] |= valid ? (~bits & lmask) : hmask;   // IS NOT NULL on NULL: FALSE; others NULL
      }
      if (nr) __syncthreads();   // the next column reuses pk
    }

    // ============ 3. filter (truth table) -> pass bitmap, group ids; compaction ============
    {
      const uint32_t leaf_false = uni(L.leaf_false);
      const uint32_t nleaves = P.nleaves;
      const bool use_truth = P.truth != nullptr;
      const bool ts_null = uni(L.hot[0].has_nulls) != 0 && uni(L.hot[0].present) != 0;
      const bool ts_present = uni(L.hot[0].present) != 0;
#pragma unroll
      for (int j = 0; j < SLOTS; j++) {
        const uint32_t r = j * BLOCK + tid;
        const uint32_t T = leafT[j] & ~leaf_false, F = leafF[j] | leaf_false;
        bool ok;
        if (use_truth) {
          const uint32_t ix = T | (F << nleaves);
          ok = (L.truth[ix >> 5] >> (ix & 31)) & 1u;
        } else {
          ok = interpret(P, T, F);
        }
        if (P.ablate & 2) ok = (tid & 15) == 0;
        bool pass = ok && r < nsub && ts_present;
        if (ts_null) pass = pass && ((L.nv[0][r >> 6] >> lane) & 1ull);   // NULL timestamp fails the window
        const unsigned long long pm = __ballot(pass);
        if (lane == 0) L.passw[r >> 6] = pm;
        L.pk[r] = gid[j];   // pk is free: every fold that read it ended with a barrier
      }
    }
    __syncthreads();
    if (wave == 0) {
      const uint32_t cnt = lane < WORDS ? __popcll(L.passw[lane]) : 0u;
      uint32_t x = cnt;
      for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
      }
      if (lane < WORDS) L.ppre[lane] = x - cnt;
      if (lane == WORDS - 1) L.ppre[WORDS] = x;
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < SLOTS; j++) {
      const uint32_t r = j * BLOCK + tid;
      const unsigned long long m = L.passw[r >> 6];
      if ((m >> lane) & 1ull) L.list[L.ppre[r >> 6] + __popcll(m & lane_lt)] = uint16_t(r);
    }
    __syncthreads();
    if (stamp) {
      const unsigned long long now = __builtin_amdgcn_s_memtime();
      st_p1 += now - st_mark;
      st_mark = now;
    }

    // ============ 4. stream timestamp + value of listed rows, bucket, aggregate ============
    const uint32_t nlist = uni(L.ppre[WORDS]);
    if (!(P.ablate & 1) && nlist) {
      const bool pres1 = uni(L.hot[1].present) != 0;
      const bool nn0 = uni(L.hot[0].has_nulls) != 0, nn1 = pres1 && uni(L.hot[1].has_nulls) != 0;
      const __amdgpu_buffer_rsrc_t rs0 = make_rsrc(L.hot[0].vals, L.hot[0].vals_len);
      const __amdgpu_buffer_rsrc_t rs1 = make_rsrc(L.hot[1].vals, pres1 ? L.hot[1].vals_len : 0u);
      const uint32_t vb0 = uni(L.hot[0].vbase) + (nn0 ? uni(L.vrun[0]) : sub);
      const uint32_t vb1 = uni(L.hot[1].vbase) + (nn1 ? uni(L.vrun[1]) : sub);
      const int64_t win_lo = L.win_lo, win_hi = L.win_hi;
      const unsigned long long glob_base = (unsigned long long)uni(L.glob_slot) * P.nbuckets;
      const uint32_t step32 = uint32_t(P.step);
      for (uint32_t cb = 0; cb < nlist; cb += PS * BLOCK) {
      v2u tsr[PS], vr[PS];
      uint32_t rows[PS];
      bool vok[PS];
#pragma unroll
      for (int j = 0; j < PS; j++) {
        tsr[j] = v2u{0u, 0u};
        vr[j] = v2u{0u, 0u};
        rows[j] = 0;
        vok[j] = false;
        if (cb + j * BLOCK >= nlist) continue;                                // uniform
        const uint32_t e = cb + j * BLOCK + tid;
        const bool live = e < nlist;
        const uint32_t r = live ? L.list[e] : 0u;
        rows[j] = r;
        const int w = r >> 6, ln = r & 63;
        const unsigned long long below = (1ull << ln) - 1ull;
        const uint32_t tv = nn0 ? L.npre[0][w] + __popcll(L.nv[0][w] & below) : r;
        tsr[j] = __builtin_amdgcn_raw_buffer_load_b64(rs0, live ? (vb0 + tv) * 8u : OOB, 0, 0);
        bool vv = pres1;
        uint32_t vi = r;
        if (nn1) {
          const unsigned long long m = L.nv[1][w];
          vv = (m >> ln) & 1ull;
          vi = L.npre[1][w] + __popcll(m & below);
        }
        vok[j] = vv && live;
        if (AGG != AGG_COUNT) vr[j] = __builtin_amdgcn_raw_buffer_load_b64(rs1, (live && vv) ? (vb1 + vi) * 8u : OOB, 0, 0);
        else vr[j] = v2u{0u, 0u};
      }
#pragma unroll
      for (int j = 0; j < PS; j++) {
        if (cb + j * BLOCK >= nlist) break;                                   // uniform
        const int64_t ts = (int64_t)(((uint64_t)tsr[j].y << 32) | tsr[j].x);
        bool ok = (cb + j * BLOCK + tid < nlist) && ts >= win_lo && ts < win_hi;   // BaseExpr.scala:159-161
        int64_t b = 0;
        if (P.fast_div) {
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
        const unsigned long long cell = (glob_base + (unsigned long long)b) * P.ngroups + L.pk[rows[j]];
        if (cell != acc.key) {
          lds_merge<AGG>(L, P, acc);
          acc_reset<AGG>(acc, cell);
        }
        const double v = __longlong_as_double((long long)(((uint64_t)vr[j].y << 32) | vr[j].x));
        acc_add<AGG>(acc, vok[j], v);
      }
      }
    }
    __syncthreads();   // the next sub-tile overwrites the bitmaps, pk, list
    // advance the per-column non-null counters (read next after the next sub-tile's validity barriers)
    if (any_nulls && tid < NC && L.hot[tid].present && L.hot[tid].has_nulls) L.vrun[tid] += L.npre[tid][WORDS];
    if (stamp) {
      const unsigned long long now = __builtin_amdgcn_s_memtime();
      st_p2 += now - st_mark;
      st_mark = now;
    }
  }
  if (stamp && tid == 0) {
    unsigned long long* o = P.stamps + 4 * (size_t(blockIdx.y) * P.max_tiles + blockIdx.x);
    o[0] = st_pro - st0;
    o[1] = st_p1;
    o[2] = st_p2;
    o[3] = __builtin_amdgcn_s_memtime() - st0;
  }
  lds_merge<AGG>(L, P, acc);
  __syncthreads();
  for (int i = tid; i < HCAP; i += BLOCK) {
    if (L.hkey[i] == EMPTY) continue;
    global_merge<AGG>(P, L.hkey[i], L.hrows[i], L.hcnt[i], L.hhi[i], L.hlo[i],
                      reinterpret_cast<unsigned long long*>(L.hhi)[i]);
  }
}

}  // namespace lk
