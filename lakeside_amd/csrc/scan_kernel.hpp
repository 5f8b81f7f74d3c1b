// scan_tiles<AGG, NSTR>: the fused decode -> filter -> bucket -> aggregate kernel (included by kernels.hip).
//
// grid (tile, segment); one 256-thread workgroup per tile (a row range inside one page of every column).
//   prologue: every fact about the tile's columns (stream pointers, run windows, value bases, flags) is read
//     once and staged in LDS together with the run windows, small dictionaries' lookup values (dictionary index
//     -> leaf bits | group-dim id) and the filter truth table;
//   per 2048-row sub-tile (thread owns rows j*256 + tid, j < 8: every 64-row group is one wave, contiguous)
//   phase 1, one string column at a time: definition levels (ballot + popcount + LDS prefix -> value index),
//     dictionary indices (branch-free buffer loads, all 8 in flight, run lookup in LDS), folded into the row's
//     leaf T/F bits and group id held in registers; then the truth table (Kleene logic precomputed on the host)
//     gives the pass bitmap (one ballot per 64 rows) and the group ids, both to LDS;
//   phase 2: every timestamp/value load of the sub-tile is issued before the first use; non-passing lanes use
//     an out-of-range buffer offset, which the hardware drops (late materialization without branches); bucket
//     by exact 32-bit reciprocal division; accumulate in a per-thread register cell (time-sorted rows hit it),
//     spilling to an LDS hash table (LDS atomics; sums as compensated hi/lo via returning-atomic TwoSum);
//   tile end: LDS cells -> global table with device atomics (count/min/max exact, sums within 1 ulp).
#pragma once
#include "device_common.hpp"

namespace lk {

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
  LRun pool[(2 + NSTR) * 2 * RUN_CAP];   // run windows: [column][value runs | def runs]
  uint32_t lut[NSTR][LUT_CAP];
  uint32_t truth[(1u << (2 * TT_MAX_LEAVES)) / 32];
  unsigned long long hkey[HCAP];
  uint32_t hrows[HCAP];
  uint32_t hcnt[HCAP];
  double hhi[HCAP];                      // SUM: hi; MIN/MAX: ordered bits (reinterpreted)
  double hlo[HCAP];
  unsigned long long passw[SUBT / 64];   // phase 1 -> 2: predicate bitmap of the sub-tile
  uint32_t gidl[SUBT];                   // phase 1 -> 2: group id per row
  unsigned long long nvw[2][SUBT / 64];  // timestamp / value validity bits (nullable pages)
  uint32_t npre[2][SUBT / 64];           // their exclusive prefix (+ running base)
  uint32_t wsum[2 + NSTR][BLOCK / 64];   // per-wave valid counts (string def-level prefix)
  uint32_t vrun[2 + NSTR];               // running non-null count since the tile start (nullable pages)
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

// Value index (relative to the tile's first non-null row) of this thread's row in one slice of a nullable
// string column: non-null rows before it in the tile.  Wave part: ballot + popcount; block part: LDS; the
// running count since the tile start lives in L.vrun[c] (read between the barriers, advanced by thread 0 after
// the second one, so the next slice's reads are ordered behind the write).
template <int NSTR>
__device__ __forceinline__ uint32_t block_prefix(Lds<NSTR>& L, int c, bool valid) {
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

template <int AGG, int NSTR>
__global__ __launch_bounds__(BLOCK) void scan_tiles(QParams P) {
  __shared__ Lds<NSTR> L;
  constexpr int NC = 2 + NSTR;
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
    LRun* vp = L.pool + c * 2 * RUN_CAP;
    const uint32_t nr = uni(L.hot[c].nruns), nd = uni(L.hot[c].ndruns);
    const uint32_t rlo = tc->run_lo, dlo = tc->drun_lo;
    for (uint32_t i = tid; i < nr; i += BLOCK) {
      const RunDesc r = runs[rlo + i];
      vp[i] = LRun{r.start, r.off_lit, r.value};
    }
    for (uint32_t i = tid; i < nd; i += BLOCK) {
      const RunDesc r = runs[dlo + i];
      vp[RUN_CAP + i] = LRun{r.start, r.off_lit, r.value};
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
    // ============ phase 1: one string column at a time ============
    uint32_t leafT[SLOTS], leafF[SLOTS], gid[SLOTS];
    bool inrow[SLOTS];
#pragma unroll
    for (int j = 0; j < SLOTS; j++) {
      leafT[j] = 0;
      leafF[j] = 0;
      gid[j] = 0;
      inrow[j] = sub + j * BLOCK + tid < tile_nrows;
    }
#pragma unroll
    for (int s = 0; s < NSTR; s++) {
      const int c = 2 + s;
      uint32_t packed[SLOTS];
      bool isnull[SLOTS];
#pragma unroll
      for (int j = 0; j < SLOTS; j++) isnull[j] = true, packed[j] = 0;
      if (uni(L.hot[c].present)) {
        const uint32_t vbase = uni(L.hot[c].vbase);
        uint32_t vidx[SLOTS];
        if (uni(L.hot[c].has_nulls)) {
          const __amdgpu_buffer_rsrc_t drs = make_rsrc(L.hot[c].defs, L.hot[c].defs_len + 8);
          const LRun* druns = L.pool + c * 2 * RUN_CAP + RUN_CAP;
          const int nd = int(uni(L.hot[c].ndruns));
          const uint32_t rip = uni(L.hot[c].rip);
          bool valid[SLOTS];
#pragma unroll
          for (int j = 0; j < SLOTS; j++) {
            const uint32_t r = rip + min(sub + j * BLOCK + tid, tile_nrows - 1);
            valid[j] = inrow[j] && hybrid_get_buf(drs, druns[find_run64(druns, nd, r)], r, 1) != 0;
          }
#pragma unroll
          for (int j = 0; j < SLOTS; j++) {
            vidx[j] = vbase + block_prefix(L, c, valid[j]);
            isnull[j] = !valid[j];
          }
        } else {
#pragma unroll
          for (int j = 0; j < SLOTS; j++) {
            vidx[j] = vbase + sub + j * BLOCK + tid;
            isnull[j] = !inrow[j];
          }
        }
        const uint32_t nr = uni(L.hot[c].nruns);
        if (nr) {
          const __amdgpu_buffer_rsrc_t vrs = make_rsrc(L.hot[c].vals, L.hot[c].vals_len + 8);
          const LRun* runs = L.pool + c * 2 * RUN_CAP;
          const int bw = int(uni(L.hot[c].bw));
          uint32_t idx[SLOTS];
#pragma unroll
          for (int j = 0; j < SLOTS; j++) {
            const uint32_t v = isnull[j] ? vbase : vidx[j];      // branch-free: NULL rows decode a valid value
            idx[j] = hybrid_get_buf(vrs, runs[find_run64(runs, int(nr), v)], v, bw);
          }
          if (uni(L.hot[c].lut_on)) {
#pragma unroll
            for (int j = 0; j < SLOTS; j++) packed[j] = isnull[j] ? 0u : L.lut[s][idx[j]];
          } else {
            const uint32_t* remap = uptr(L.hot[c].remap);
            const uint32_t* tab = uptr(L.sp[s].strtab);
#pragma unroll
            for (int j = 0; j < SLOTS; j++) {
              const uint32_t g = remap[idx[j]];
              packed[j] = isnull[j] ? 0u : (tab ? tab[g] : g);
            }
          }
        }
      }
      // fold: group dimension + leaves of this column
      const uint32_t dstride = uni(L.sp[s].dim_stride), dnull = uni(L.sp[s].dim_null);
      const uint32_t lbase = uni(L.sp[s].lbase), lmask = uni(L.sp[s].lmask), hmask = uni(L.sp[s].hmask);
#pragma unroll
      for (int j = 0; j < SLOTS; j++) {
        const uint32_t bits = (packed[j] >> 24) << lbase;
        const uint32_t dim = isnull[j] ? dnull : (packed[j] & DIM_MASK);
        gid[j] += dim * dstride;
        leafT[j] |= isnull[j] ? 0u : (bits & lmask);
        leafF[j] |= isnull[j] ? hmask : (~bits & lmask);   // IS NOT NULL on NULL: FALSE; others NULL
      }
    }
    // filter: truth table over the leaves' (T, F) bits (Kleene logic precomputed on the host)
    {
      const uint32_t leaf_false = uni(L.leaf_false);
      const uint32_t nleaves = P.nleaves;
      const bool use_truth = P.truth != nullptr;
#pragma unroll
      for (int j = 0; j < SLOTS; j++) {
        const uint32_t T = leafT[j] & ~leaf_false, F = leafF[j] | leaf_false;
        bool ok;
        if (use_truth) {
          const uint32_t ix = T | (F << nleaves);
          ok = (L.truth[ix >> 5] >> (ix & 31)) & 1u;
        } else {
          ok = interpret(P, T, F);
        }
        const bool pass = (P.ablate & 2) ? (inrow[j] && (tid & 15) == 0) : (inrow[j] && ok);
        const unsigned long long pm = __ballot(pass);
        if (lane == 0) L.passw[j * (BLOCK / 64) + wave] = pm;
        L.gidl[j * BLOCK + tid] = gid[j];
      }
    }
    // timestamp / value validity (nullable pages): one bit per row
    const bool nn0 = uni(L.hot[0].has_nulls) != 0, nn1 = uni(L.hot[1].has_nulls) != 0;
#pragma unroll
    for (int c = 0; c < 2; c++) {
      if (!(c == 0 ? nn0 : nn1)) continue;
      const __amdgpu_buffer_rsrc_t drs = make_rsrc(L.hot[c].defs, L.hot[c].defs_len + 8);
      const LRun* druns = L.pool + c * 2 * RUN_CAP + RUN_CAP;
      const int nd = int(uni(L.hot[c].ndruns));
      const uint32_t rip = uni(L.hot[c].rip);
#pragma unroll
      for (int j = 0; j < SLOTS; j++) {
        const uint32_t r = rip + min(sub + j * BLOCK + tid, tile_nrows - 1);
        const bool v = inrow[j] && hybrid_get_buf(drs, druns[find_run64(druns, nd, r)], r, 1) != 0;
        const unsigned long long vm = __ballot(v);
        if (lane == 0) L.nvw[c][j * (BLOCK / 64) + wave] = vm;
      }
    }
    __syncthreads();
    // exclusive prefix of valid rows per 64-row group (nullable timestamp / value pages)
    if (nn0 || nn1) {
      if ((wave == 0 && nn0) || (wave == 1 && nn1)) {
        const int c = wave;
        uint32_t cnt = lane < SUBT / 64 ? __popcll(L.nvw[c][lane]) : 0;
        uint32_t x = cnt;
        for (int o = 1; o < 64; o <<= 1) {
          uint32_t y = __shfl_up(x, o, 64);
          if (lane >= o) x += y;
        }
        const uint32_t rb = L.vrun[c];
        if (lane < SUBT / 64) L.npre[c][lane] = rb + x - cnt;
        const uint32_t tot = __shfl(x, 63, 64);
        if (lane == 0) L.vrun[c] = rb + tot;
      }
      __syncthreads();
    }
    if (stamp) {
      const unsigned long long now = __builtin_amdgcn_s_memtime();
      st_p1 += now - st_mark;
      st_mark = now;
    }
    if (P.ablate & 1) {
      __syncthreads();
      continue;
    }

    // ============ phase 2: stream timestamp + value of passing rows, bucket, aggregate ============
    {
      const bool pres0 = uni(L.hot[0].present) != 0, pres1 = uni(L.hot[1].present) != 0;
      const __amdgpu_buffer_rsrc_t rs0 = make_rsrc(L.hot[0].vals, pres0 ? L.hot[0].vals_len : 0u);
      const __amdgpu_buffer_rsrc_t rs1 = make_rsrc(L.hot[1].vals, pres1 ? L.hot[1].vals_len : 0u);
      const uint32_t vb0 = uni(L.hot[0].vbase), vb1 = uni(L.hot[1].vbase);
      v2u tsr[SLOTS], vr[SLOTS];
      bool pass[SLOTS], vok[SLOTS];
#pragma unroll
      for (int j = 0; j < SLOTS; j++) {
        const int w = j * (BLOCK / 64) + wave;
        bool p = ((L.passw[w] >> lane) & 1ull) && pres0;
        uint32_t tv = vb0 + sub + j * BLOCK + tid;
        if (nn0) {
          const unsigned long long m = L.nvw[0][w];
          p = p && ((m >> lane) & 1ull);
          tv = vb0 + L.npre[0][w] + __popcll(m & lane_lt);
        }
        pass[j] = p;
        tsr[j] = __builtin_amdgcn_raw_buffer_load_b64(rs0, p ? tv * 8u : OOB, 0, 0);
        bool vv = pres1;
        uint32_t vi = vb1 + sub + j * BLOCK + tid;
        if (nn1) {
          const unsigned long long m = L.nvw[1][w];
          vv = vv && ((m >> lane) & 1ull);
          vi = vb1 + L.npre[1][w] + __popcll(m & lane_lt);
        }
        vok[j] = vv;
        if (AGG != AGG_COUNT) vr[j] = __builtin_amdgcn_raw_buffer_load_b64(rs1, (p && vv) ? vi * 8u : OOB, 0, 0);
        else vr[j] = v2u{0u, 0u};
      }
      const int64_t win_lo = L.win_lo, win_hi = L.win_hi;
      const unsigned long long glob_base = (unsigned long long)uni(L.glob_slot) * P.nbuckets;
      const uint32_t step32 = uint32_t(P.step);
#pragma unroll
      for (int j = 0; j < SLOTS; j++) {
        const int64_t ts = (int64_t)(((uint64_t)tsr[j].y << 32) | tsr[j].x);
        bool ok = pass[j] && ts >= win_lo && ts < win_hi;            // BaseExpr.scala:159-161
        int64_t b = 0;
        if (P.fast_div) {
          // d < 2^32: q from the double reciprocal is off by at most one; fix with the remainder
          const uint32_t d = uint32_t(ts - P.bucket_base);
          uint32_t q = uint32_t(double(d) * P.inv_step);
          int64_t r = int64_t(d) - int64_t(q) * step32;
          q = r < 0 ? q - 1 : (r >= int64_t(step32) ? q + 1 : q);
          r = int64_t(d) - int64_t(q) * step32;
          if (P.metrics && r != 0 && ok) {
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
        const unsigned long long cell = (glob_base + (unsigned long long)b) * P.ngroups + L.gidl[j * BLOCK + tid];
        if (cell != acc.key) {
          lds_merge<AGG>(L, P, acc);
          acc_reset<AGG>(acc, cell);
        }
        const double v = __longlong_as_double((long long)(((uint64_t)vr[j].y << 32) | vr[j].x));
        acc_add<AGG>(acc, vok[j], v);
      }
    }
    __syncthreads();   // phase 1 of the next sub-tile overwrites passw / gidl
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
