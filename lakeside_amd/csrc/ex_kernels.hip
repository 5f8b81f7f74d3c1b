// Exemplar scans (raw rows, no chart): per glob the worker runs
//   SELECT <projection>, * FROM (SELECT * FROM {table} WHERE <window>) WHERE <filter>
//   ORDER BY "_cardinalhq.timestamp" <DESC|ASC> LIMIT <n>
// (BaseExpr.getBaseQuery, core/src/main/scala/com/cardinal/utils/ast/BaseExpr.scala:234-239).  Top-n by time is a
// selection problem, solved here without sorting the glob:
//   ex_scan (HIST): every tile whose zone map meets a glob's open range decodes its filter columns row by row,
//     evaluates the filter (Kleene truth table / program) and counts passing rows per time bin of that range
//     (LDS histogram, one device atomic per non-empty bin per tile);
//   host: per glob, the bins from the ordered end until n rows are covered give a narrower range (refined again
//     while its candidates exceed the emit capacity);
//   ex_scan (EMIT): the same decode over the tiles meeting the narrowed ranges; passing rows inside them are
//     appended as (timestamp, segment | tile | row) records (wave-aggregated atomics);
//   host: sort the few candidates, keep n per glob;
//   ex_gather: one thread per (selected row, output column) decodes that row's value of every column of the
//     glob's union (def-level prefix over the tile's def runs, then PLAIN / bit-packed / dictionary value) -> raw
//     payload + valid flag; the host formats the tag strings (Commons.toDataPoint, Commons.scala:428-459).
// HBM traffic is the filter columns of the tiles in the window (HIST) plus the tiles near the ordered end (EMIT);
// the gather is a few KB.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "device_common.hpp"
#include "kernels.hpp"
#include "layout.hpp"

namespace lk {

namespace {

struct XHot {
  const uint8_t* vals;
  const uint8_t* defs;
  const uint32_t* remap;
  const uint32_t* tab;
  uint32_t vals_len, defs_len, vbase, rip, nruns, ndruns, bw, kind, nulls, present;
};

__device__ __forceinline__ bool x_interpret(const XParams& X, uint32_t T, uint32_t F) {
  uint64_t st = 0, sf = 0;
  for (uint32_t i = 0; i < X.nprog; i++) {
    const uint8_t op = X.prog[i];
    if (op < 0x80) {
      st = (st << 1) | ((T >> op) & 1u);
      sf = (sf << 1) | ((F >> op) & 1u);
    } else if (op == OP_NOT) {
      const uint64_t t1 = st & 1, f1 = sf & 1;
      st = (st & ~1ull) | f1;
      sf = (sf & ~1ull) | t1;
    } else if (op == OP_TRUE) {
      st = (st << 1) | 1;
      sf = sf << 1;
    } else {
      const uint64_t t2 = st & 1, f2 = sf & 1;
      st >>= 1;
      sf >>= 1;
      const uint64_t t1 = st & 1, f1 = sf & 1;
      st = (st & ~1ull) | ((op == OP_AND) ? (t1 & t2) : (t1 | t2));
      sf = (sf & ~1ull) | ((op == OP_AND) ? (f1 | f2) : (f1 & f2));
    }
  }
  return st & 1;
}

__device__ __forceinline__ uint32_t lanes_below(unsigned long long m) {
  return __builtin_amdgcn_mbcnt_hi(uint32_t(m >> 32), __builtin_amdgcn_mbcnt_lo(uint32_t(m), 0u));
}

// Canonical group key of a tag value (pad: Parquet physical type | glob union type << 8), as DuckDB groups the
// union_by_name column: integers as BIGINT / INTEGER, FLOAT / DOUBLE unions with every NaN as one value and -0.0 as
// +0.0, BOOLEAN as 0 / 1.
__device__ __forceinline__ unsigned long long tag_key(unsigned long long raw, uint32_t pad) {
  const uint32_t pt = pad & 0xffu, ut = (pad >> 8) & 0xffu;
  const long long iv = pt == 2u ? (long long)raw : (long long)int32_t(uint32_t(raw));
  if (ut == 2u || ut == 1u) return (unsigned long long)iv;
  if (ut == 0u) return raw & 1ull;
  if (ut == 4u) {
    float f = pt == 4u ? __uint_as_float(uint32_t(raw)) : float(iv);
    if (f != f) return 0x7fc00000ull;
    const uint32_t b = __float_as_uint(f);
    return (b & 0x7fffffffu) == 0u ? 0ull : (unsigned long long)b;
  }
  const double d = pt == 5u ? __longlong_as_double((long long)raw) : (pt == 4u ? double(__uint_as_float(uint32_t(raw))) : double(iv));
  if (d != d) return 0x7ff8000000000000ull;
  const unsigned long long b = (unsigned long long)__double_as_longlong(d);
  return (b & 0x7fffffffffffffffull) == 0ull ? 0ull : b;
}

__device__ __forceinline__ unsigned long long tag_hash(unsigned long long k) {
  k ^= k >> 33;
  k *= 0xff51afd7ed558ccdull;
  k ^= k >> 33;
  k *= 0xc4ceb9fe1a85ec53ull;
  k ^= k >> 33;
  return k;
}

// (key, c) into glob g's device table (linear probing; a table without room sets FLAG_HASH_FULL: the host regrows)
__device__ void tag_global_add(const XParams& X, uint32_t g, unsigned long long k, unsigned long long c) {
  const unsigned long long mask = X.tcap - 1, base = (unsigned long long)g * X.tcap;
  unsigned long long s = tag_hash(k) & mask;
  for (unsigned long long i = 0; i <= mask && i < 4096; i++, s = (s + 1) & mask) {
    const unsigned long long prev = atomicCAS(X.tkeys + base + s, TAG_EMPTY, k);
    if (prev == TAG_EMPTY || prev == k) {
      atomicAdd(X.tcnt + base + s, c);
      return;
    }
  }
  atomicOr(X.tflags, FLAG_HASH_FULL);
}

constexpr uint32_t TAG_LDS_SLOTS = 512;   // per workgroup (aliases the HIST bins)

}  // namespace

template <int AGG, bool HASH>
__device__ __forceinline__ void ex_merge(const QParams& q, unsigned long long cell, bool vok, double v) {
  global_merge<AGG, HASH>(q, cell, 1u, vok ? 1u : 0u, vok ? v : 0.0, 0.0, vok ? dbl_order(v) : (AGG == AGG_MIN ? ~0ull : 0ull));
}

__global__ __launch_bounds__(BLOCK) void ex_scan(XParams X) {
  // column state by query column: 0 timestamp, 1 value (AGG), 2 .. 2+nstr strings, then numeric filter columns
  __shared__ XHot H[MAXQCOL];
  __shared__ LRun vr[MAXQCOL][RUN_CAP];
  __shared__ LRun dr[MAXQCOL][RUN_CAP];
  __shared__ uint32_t truth[(1u << (2 * TT_MAX_LEAVES)) / 32];
  __shared__ uint32_t wsum[MAXQCOL][BLOCK / 64];
  __shared__ __attribute__((aligned(16))) uint32_t hist[XBINS];   // HIST bins, or the TAGNUM table (64-bit keys)

  const QSeg* Sp = X.segs + blockIdx.y;
  const uint32_t t = blockIdx.x;
  if (t >= Sp->ntiles) return;
  const uint32_t g = Sp->glob_slot;
  const bool aggm = X.mode == XMODE_AGG;
  const int64_t lo = aggm ? Sp->win_lo : X.rlo[g], hi = aggm ? Sp->win_hi : X.rhi[g];
  const TileDesc* tdp = Sp->tiles + t;
  if (lo >= hi || tdp->ts_max < lo || tdp->ts_min >= hi) return;   // zone map outside the glob's open range
  const uint32_t nrows = tdp->nrows;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int ns = int(X.nstr);
  const int nc = 2 + ns + int(X.nnum);

  if (tid < nc) {
    const int qc = tid;
    XHot h{};
    h.present = (qc == 1 && !aggm) ? 0u : Sp->cols[qc].present;
    if (h.present) {
      const TileCol tc = Sp->cols[qc].tcols[t];
      h.vals = Sp->base + tc.vals;
      h.defs = Sp->base + tc.defs;
      h.remap = Sp->cols[qc].remap + tc.remap;
      h.tab = (qc >= 2 && qc < 2 + ns) ? X.strp[qc - 2].strtab : nullptr;
      h.vals_len = tc.vals_len;
      h.defs_len = tc.defs_len;
      h.vbase = tc.vbase;
      h.rip = tc.row_in_page;
      h.nruns = tc.kind == PAGE_DICT ? tc.nruns : 0u;
      h.ndruns = tc.has_nulls ? tc.ndruns : 0u;
      h.bw = tc.bw;
      h.kind = tc.kind;
      h.nulls = tc.has_nulls;
    }
    H[qc] = h;
  }
  if (X.truth)
    for (uint32_t i = tid; i < ((1u << (2 * X.nleaves)) + 31) / 32; i += BLOCK) truth[i] = X.truth[i];
  if (X.mode == XMODE_HIST)
    for (uint32_t i = tid; i < X.nbins; i += BLOCK) hist[i] = 0;
  // TAGNUM: the workgroup's table in the bins' LDS: [512 keys (u64) | 512 counts | NULL rows | all-ones-key rows]
  unsigned long long* tk = reinterpret_cast<unsigned long long*>(hist);
  uint32_t* tc = hist + 2 * TAG_LDS_SLOTS;
  if (X.mode == XMODE_TAGNUM) {
    for (uint32_t i = tid; i < TAG_LDS_SLOTS; i += BLOCK) {
      tk[i] = TAG_EMPTY;
      tc[i] = 0;
    }
    if (tid < 2) tc[TAG_LDS_SLOTS + tid] = 0;
  }
  __syncthreads();
  for (int qc = 0; qc < nc; qc++) {
    if (!H[qc].present) continue;
    const TileCol* tc = Sp->cols[qc].tcols + t;
    const RunDesc* runs = Sp->cols[qc].runs;
    for (uint32_t i = tid; i < H[qc].nruns; i += BLOCK) {
      const RunDesc r = runs[tc->run_lo + i];
      vr[qc][i] = LRun{r.start, r.off_lit, r.value};
    }
    for (uint32_t i = tid; i < H[qc].ndruns; i += BLOCK) {
      const RunDesc r = runs[tc->drun_lo + i];
      dr[qc][i] = LRun{r.start, r.off_lit, r.value};
    }
  }
  __syncthreads();

  const uint32_t leaf_false = Sp->leaf_false;
  const int64_t hbase = X.mode == XMODE_HIST ? X.hbase[g] : 0;
  const int64_t hwidth = X.mode == XMODE_HIST ? X.hwidth[g] : 1;
  uint32_t carry[MAXQCOL];
#pragma unroll
  for (int k = 0; k < MAXQCOL; k++) carry[k] = 0;

  for (uint32_t c0 = 0; c0 < nrows; c0 += BLOCK) {
    const uint32_t r = c0 + uint32_t(tid);
    const bool inb = r < nrows;
    uint32_t T = 0, F = 0;
    bool ts_ok = false, v_ok = false, tag_ok = false;
    unsigned long long tag_raw = 0;
    int64_t ts = 0;
    double v = 0.0;
    unsigned long long gid = 0;
#pragma unroll
    for (int qc = 0; qc < MAXQCOL; qc++) {
      if (qc >= nc) break;
      const XHot& h = H[qc];
      bool ok = inb && h.present;
      uint32_t vi = h.vbase + r;
      if (h.present && h.nulls) {   // block-uniform
        const __amdgpu_buffer_rsrc_t drs = make_rsrc(h.defs, h.defs_len + 8);
        const uint32_t row = h.rip + r;
        const int ri = find_run(dr[qc], int(h.ndruns), row);
        const bool bit = inb && (hybrid_get_buf(drs, dr[qc][ri], row, 1) & 1u);
        const unsigned long long m = __ballot(bit);
        const uint32_t below = lanes_below(m);
        if (lane == 0) wsum[qc][wave] = uint32_t(__popcll(m));
        __syncthreads();
        uint32_t before = 0, all = 0;
#pragma unroll
        for (int w = 0; w < BLOCK / 64; w++) {
          before += w < wave ? wsum[qc][w] : 0u;
          all += wsum[qc][w];
        }
        __syncthreads();
        vi = h.vbase + carry[qc] + before + below;
        carry[qc] += all;
        ok = bit;
      }
      if (qc < 2 || qc >= 2 + ns) {   // PLAIN numeric: timestamp, value, numeric filter column
        const bool w8 = h.kind == PAGE_PLAIN64;
        const bool bl = h.kind == PAGE_BOOL && uint32_t(qc) == X.tag_qc;   // BOOLEAN: a numeric tag only
        if (!w8 && h.kind != PAGE_PLAIN32 && !bl) ok = false;
        // (BOOLEAN: bit-packed bytes read as whole dwords -- the slack keeps the stream's last dword in range)
        const __amdgpu_buffer_rsrc_t rs = make_rsrc(h.vals, h.vals_len + (bl ? 4u : 0u));
        uint64_t raw = 0;
        if (w8) {
          const v2u w = __builtin_amdgcn_raw_buffer_load_b64(rs, ok ? vi * 8u : OOB, 0, 0);
          raw = (uint64_t(w.y) << 32) | w.x;
        } else if (bl) {
          raw = (__builtin_amdgcn_raw_buffer_load_b32(rs, ok ? (vi >> 5) * 4u : OOB, 0, 0) >> (vi & 31u)) & 1u;
        } else {
          raw = __builtin_amdgcn_raw_buffer_load_b32(rs, ok ? vi * 4u : OOB, 0, 0);
        }
        if (uint32_t(qc) == X.tag_qc) {
          tag_raw = raw;
          tag_ok = ok;
        }
        if (qc == 0) {   // BIGINT over INT64 / INT32 files (union_by_name)
          ts = w8 ? int64_t(raw) : int64_t(int32_t(uint32_t(raw)));
          ts_ok = ok;
        } else if (qc == 1) {
          // the value as the glob's union_by_name type, then as double (JDBC getDouble of the aggregate):
          // DOUBLE as is, INT64 / INT32 / FLOAT exactly widened; integers in a FLOAT union rounded to float first
          const uint32_t pad = Sp->cols[1].pad, pt = pad & 0xffu;
          if (pt == 5u) {
            v = __longlong_as_double((long long)raw);
          } else if (pt == 4u) {
            v = double(__uint_as_float(uint32_t(raw)));
          } else {
            const long long iv = pt == 2u ? (long long)raw : (long long)int32_t(uint32_t(raw));
            v = (pad & VCONV_VIA_FLOAT) ? double(float(iv)) : double(iv);
          }
          v_ok = ok;
        } else {
          const uint32_t pt = Sp->cols[qc].pad;   // Parquet physical type of this segment's column
          const bool is_int = pt == 1u || pt == 2u;
          const long long iv = pt == 2u ? (long long)raw : (long long)int32_t(uint32_t(raw));
          const double dv = pt == 5u ? __longlong_as_double((long long)raw) : double(__uint_as_float(uint32_t(raw)));
          for (uint32_t k = 0; k < X.nnl; k++) {
            const NumLeaf& L = X.nl[k];
            if (int(L.col) != qc - 2 - ns) continue;
            if (L.pad & NUMLEAF_NOTNULL) {   // IS NOT NULL: never UNKNOWN
              T |= uint32_t(ok) << L.leaf;
              F |= uint32_t(!ok) << L.leaf;
              continue;
            }
            if (!ok) continue;   // NULL: UNKNOWN
            bool pass;
            const double x = is_int ? double(iv) : dv;   // integers vs a DOUBLE (scientific) literal: cast first
            if (is_int && !L.pad) {
              pass = iv >= L.ilo && iv <= L.ihi;        // integers vs a decimal literal: exact
            } else if (x != x) {
              pass = L.nan_pass != 0;
            } else {
              pass = (x > L.dlo || (L.lo_incl && x == L.dlo)) && (x < L.dhi || (L.hi_incl && x == L.dhi));
            }
            T |= uint32_t(pass) << L.leaf;
            F |= uint32_t(!pass) << L.leaf;
          }
        }
        continue;
      }
      const StrParam& sp = X.strp[qc - 2];
      if (!h.present || h.nruns == 0u) ok = false;   // absent / no value in this tile: NULL
      if (ok) {
        const __amdgpu_buffer_rsrc_t rs = make_rsrc(h.vals, h.vals_len + 8);
        const int ri = find_run(vr[qc], int(h.nruns), vi);
        const uint32_t idx = hybrid_get_buf(rs, vr[qc][ri], vi, int(h.bw));
        const uint32_t gl = h.remap[idx];
        const uint32_t packed = h.tab ? h.tab[gl] : gl;
        const uint32_t bits = (packed >> 24) << sp.lbase;
        T |= bits & sp.lmask;
        F |= ~bits & sp.lmask;
        gid += (unsigned long long)(packed & DIM_MASK) * sp.dim_stride;
      } else {
        F |= sp.hmask;   // IS NOT NULL on NULL: FALSE; other leaves NULL
        gid += (unsigned long long)sp.dim_null * sp.dim_stride;
      }
    }
    T &= ~leaf_false;
    F |= leaf_false;
    bool pass;
    if (X.truth) {
      const uint32_t ix = T | (F << X.nleaves);
      pass = (truth[ix >> 5] >> (ix & 31)) & 1u;
    } else {
      pass = x_interpret(X, T, F);
    }
    pass = pass && ts_ok && ts >= lo && ts < hi;
    if (X.mode == XMODE_AGG) {
      if (pass) {
        const QParams& q = X.q;
        int64_t b;
        bool ok = true;
        if (q.metrics) {   // BaseExpr.scala:376-394: the raw timestamp, on the step grid
          const int64_t d = ts - q.bucket_base;
          b = d / q.step;
          if (d - b * q.step != 0) {
            atomicOr(q.flags, FLAG_METRICS_UNALIGNED);
            ok = false;
          }
        } else {           // BaseExpr.scala:163-165: ts - ts % step
          b = ((ts - ts % q.step) - q.bucket_base) / q.step;
        }
        if (ok && (b < 0 || (uint64_t)b >= q.nbuckets)) {
          atomicOr(q.flags, FLAG_CELL_RANGE);
          ok = false;
        }
        if (ok) {
          unsigned long long cell = ((unsigned long long)g * q.nbuckets + (unsigned long long)b) * q.ngroups + gid;
          // percentiles: rows per (cell, DDSketch bin of the value; NULL reads 0.0), as scan_tiles keys them
          if (q.sketch) cell = cell * DD_NBINS + dd_bin(q, v_ok ? v : 0.0);
          switch (X.agg * 2 + (X.hash ? 1 : 0)) {
            case AGG_SUM * 2: ex_merge<AGG_SUM, false>(q, cell, v_ok, v); break;
            case AGG_SUM * 2 + 1: ex_merge<AGG_SUM, true>(q, cell, v_ok, v); break;
            case AGG_MIN * 2: ex_merge<AGG_MIN, false>(q, cell, v_ok, v); break;
            case AGG_MIN * 2 + 1: ex_merge<AGG_MIN, true>(q, cell, v_ok, v); break;
            case AGG_MAX * 2: ex_merge<AGG_MAX, false>(q, cell, v_ok, v); break;
            case AGG_MAX * 2 + 1: ex_merge<AGG_MAX, true>(q, cell, v_ok, v); break;
            case AGG_COUNT * 2: ex_merge<AGG_COUNT, false>(q, cell, v_ok, v); break;
            default: ex_merge<AGG_COUNT, true>(q, cell, v_ok, v); break;
          }
        }
      }
    } else if (X.mode == XMODE_TAGNUM) {
      // every passing row of the glob window: NULL tags and the all-ones key counted apart; the other keys deduplicated
      // across the wave (one leader per distinct key) and added into the workgroup's LDS table
      const int cls = !pass ? 0 : (!tag_ok ? 2 : 1);
      const unsigned long long key = cls == 1 ? tag_key(tag_raw, Sp->cols[X.tag_qc].pad) : 0ull;
      const int cl2 = (cls == 1 && key == TAG_EMPTY) ? 3 : cls;
      const unsigned long long mn = __ballot(cl2 == 2), mo = __ballot(cl2 == 3);
      if (lane == 0 && mn) atomicAdd(&tc[TAG_LDS_SLOTS], uint32_t(__popcll(mn)));
      if (lane == 0 && mo) atomicAdd(&tc[TAG_LDS_SLOTS + 1], uint32_t(__popcll(mo)));
      unsigned long long act = __ballot(cl2 == 1);
      while (act) {
        const int leader = __ffsll((long long)act) - 1;
        const uint32_t lo32 = __shfl(uint32_t(key), leader), hi32 = __shfl(uint32_t(key >> 32), leader);
        const unsigned long long lk = (unsigned long long)hi32 << 32 | lo32;
        const unsigned long long m = __ballot(cl2 == 1 && key == lk);
        if (lane == leader) {
          const uint32_t c = uint32_t(__popcll(m));
          uint32_t s = uint32_t(tag_hash(lk)) & (TAG_LDS_SLOTS - 1);
          bool done = false;
          for (uint32_t i = 0; i < TAG_LDS_SLOTS; i++, s = (s + 1) & (TAG_LDS_SLOTS - 1)) {
            const unsigned long long prev = atomicCAS(&tk[s], TAG_EMPTY, lk);
            if (prev == TAG_EMPTY || prev == lk) {
              atomicAdd(&tc[s], c);
              done = true;
              break;
            }
          }
          if (!done) tag_global_add(X, g, lk, c);   // the workgroup's table is full
        }
        act &= ~m;
      }
    } else if (X.mode == XMODE_HIST) {
      if (pass) {
        int64_t b = (ts - hbase) / hwidth;
        b = b < 0 ? 0 : (b >= int64_t(X.nbins) ? int64_t(X.nbins) - 1 : b);
        atomicAdd(&hist[b], 1u);
      }
    } else {
      const unsigned long long m = __ballot(pass);
      if (m) {
        uint32_t base = 0;
        if (lane == 0) base = atomicAdd(X.out_n, uint32_t(__popcll(m)));
        base = __shfl(base, 0) + lanes_below(m);
        if (pass && base < X.cap) {
          X.out[2 * size_t(base)] = (unsigned long long)ts;
          X.out[2 * size_t(base) + 1] = ((unsigned long long)blockIdx.y << 48) | ((unsigned long long)t << 16) | r;
        }
      }
    }
  }
  if (X.mode == XMODE_HIST) {
    __syncthreads();
    for (uint32_t i = tid; i < X.nbins; i += BLOCK)
      if (hist[i]) atomicAdd(&X.hist[size_t(g) * X.nbins + i], hist[i]);
  }
  if (X.mode == XMODE_TAGNUM) {   // flush: one device atomic per distinct key of the tile
    __syncthreads();
    for (uint32_t i = tid; i < TAG_LDS_SLOTS; i += BLOCK)
      if (tk[i] != TAG_EMPTY) tag_global_add(X, g, tk[i], tc[i]);
    if (tid < 2 && tc[TAG_LDS_SLOTS + tid]) atomicAdd(X.tspec + 2 * size_t(g) + tid, (unsigned long long)tc[TAG_LDS_SLOTS + tid]);
  }
}

__global__ __launch_bounds__(256) void tag_compact(const unsigned long long* keys, const unsigned long long* cnt,
                                                   unsigned long long n, unsigned long long tcap,
                                                   unsigned long long* out, uint32_t* out_n) {
  const unsigned long long i = (unsigned long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= n || keys[i] == TAG_EMPTY) return;
  const uint32_t o = atomicAdd(out_n, 1u);
  out[3 * size_t(o)] = keys[i];
  out[3 * size_t(o) + 1] = cnt[i];
  out[3 * size_t(o) + 2] = i / tcap;
}

hipError_t launch_tag_compact(const unsigned long long* keys, const unsigned long long* cnt, unsigned long long tcap,
                              uint32_t nglobs, unsigned long long* out, uint32_t* out_n, hipStream_t stream) {
  const unsigned long long n = tcap * nglobs;
  if (!n) return hipSuccess;
  hipLaunchKernelGGL(tag_compact, dim3(uint32_t((n + 255) / 256)), dim3(256), 0, stream, keys, cnt, n, tcap, out, out_n);
  return hipGetLastError();
}

namespace {

// Bits [a, b) of a little-endian bit stream: how many are set.
__device__ uint32_t popcount_range(const uint8_t* p, uint32_t a, uint32_t b) {
  uint32_t n = 0;
  while (a < b && (a & 7u)) {
    n += (p[a >> 3] >> (a & 7u)) & 1u;
    a++;
  }
  while (a + 8 <= b) {
    n += __popc(p[a >> 3]);
    a += 8;
  }
  while (a < b) {
    n += (p[a >> 3] >> (a & 7u)) & 1u;
    a++;
  }
  return n;
}

// `bw` bits at bit offset `bit` of a little-endian bit-packed stream of `len` bytes.
__device__ uint32_t packed_get(const uint8_t* p, uint32_t len, uint64_t bit, uint32_t bw) {
  uint64_t x = 0;
  const uint64_t byte = bit >> 3;
  for (uint32_t i = 0; i < 5; i++)
    if (byte + i < len) x |= uint64_t(p[byte + i]) << (8 * i);
  x >>= (bit & 7u);
  return bw >= 32 ? uint32_t(x) : uint32_t(x) & ((1u << bw) - 1u);
}

}  // namespace

__global__ __launch_bounds__(256) void ex_gather(GParams G) {
  const uint64_t i = uint64_t(blockIdx.x) * 256 + threadIdx.x;
  if (i >= uint64_t(G.nsel) * G.ncols) return;
  const uint32_t j = uint32_t(i / G.ncols), k = uint32_t(i % G.ncols);
  const unsigned long long ref = G.sel[j];
  const uint32_t seg = uint32_t(ref >> 48), tile = uint32_t((ref >> 16) & 0xffffffffu), r = uint32_t(ref & 0xffffu);
  const GCol& C = G.cols[size_t(seg) * G.ncols + k];
  G.ok[i] = 0;
  G.val[i] = 0;
  if (!C.present) return;
  const TileCol tc = C.tcols[tile];
  const uint32_t row = tc.row_in_page + r;   // page-relative
  uint32_t vi = tc.vbase + r;
  if (tc.has_nulls) {
    const uint8_t* defs = C.base + tc.defs;
    uint32_t cnt = 0;
    bool bit = false;
    for (uint32_t q = 0; q < tc.ndruns; q++) {
      const RunDesc rd = C.runs[tc.drun_lo + q];
      const uint32_t s = rd.start, e = rd.start + rd.count;
      const uint32_t a = s > tc.row_in_page ? s : tc.row_in_page, b = e < row ? e : row;
      const bool lit = (rd.off_lit & 0x80000000u) != 0;
      const uint32_t off = rd.off_lit & 0x7fffffffu;
      if (a < b) cnt += lit ? popcount_range(defs + off, a - s, b - s) : (rd.value ? b - a : 0u);
      if (row >= s && row < e) bit = lit ? ((defs[off + ((row - s) >> 3)] >> ((row - s) & 7u)) & 1u) : rd.value != 0;
    }
    if (!bit) return;
    vi = tc.vbase + cnt;
  }
  const uint8_t* vals = C.base + tc.vals;
  unsigned long long v = 0;
  switch (tc.kind) {
    case PAGE_PLAIN64:
      if (uint64_t(vi) * 8 + 8 > tc.vals_len) return;
      for (int b = 0; b < 8; b++) v |= (unsigned long long)vals[size_t(vi) * 8 + b] << (8 * b);
      break;
    case PAGE_PLAIN32:
      if (uint64_t(vi) * 4 + 4 > tc.vals_len) return;
      for (int b = 0; b < 4; b++) v |= (unsigned long long)vals[size_t(vi) * 4 + b] << (8 * b);
      break;
    case PAGE_BOOL:
      if ((vi >> 3) >= tc.vals_len) return;
      v = (vals[vi >> 3] >> (vi & 7u)) & 1u;
      break;
    case PAGE_DICT: {
      if (tc.nruns == 0) return;
      uint32_t a = tc.run_lo, b = tc.run_lo + tc.nruns - 1;   // last run whose start <= vi
      while (a < b) {
        const uint32_t m = (a + b + 1) / 2;
        if (C.runs[m].start <= vi) a = m;
        else b = m - 1;
      }
      const RunDesc rd = C.runs[a];
      const uint32_t idx = (rd.off_lit & 0x80000000u)
                               ? packed_get(vals + (rd.off_lit & 0x7fffffffu), tc.vals_len - (rd.off_lit & 0x7fffffffu),
                                            uint64_t(vi - rd.start) * tc.bw, tc.bw)
                               : rd.value;
      if (idx >= tc.dict_n) return;
      v = C.remap[tc.remap + idx];
      break;
    }
    default:
      return;
  }
  G.val[i] = v;
  G.ok[i] = 1;
}

hipError_t launch_ex_scan(const XParams& X, hipStream_t stream) {
  if (!X.nsegs || !X.max_tiles) return hipSuccess;
  hipLaunchKernelGGL(ex_scan, dim3(X.max_tiles, X.nsegs), dim3(BLOCK), 0, stream, X);
  return hipGetLastError();
}

hipError_t launch_ex_gather(const GParams& G, hipStream_t stream) {
  const uint64_t n = uint64_t(G.nsel) * G.ncols;
  if (!n) return hipSuccess;
  hipLaunchKernelGGL(ex_gather, dim3(uint32_t((n + 255) / 256)), dim3(256), 0, stream, G);
  return hipGetLastError();
}

}  // namespace lk
