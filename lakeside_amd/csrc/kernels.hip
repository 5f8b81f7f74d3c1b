// HIP kernels for gfx950 (MI355X): sealed-segment DataExpr scan + table finalize/compaction.
//
// scan_tiles<AGG, NSTR>: grid (tile, segment), one 256-thread workgroup per tile (a row range inside one page
// of every column).  Per-tile column state (page stream offsets, run windows, flags) is read with scalar loads
// into SGPRs; NSTR (string columns of the query) is a template parameter so every column loop unrolls.
//   prologue: stage each string column's run window and, for small dictionaries, the per-query lookup values
//     (dictionary index -> leaf bits | group-dim id) and the filter truth table in LDS;
//   per 2048-row sub-tile, phase 1: decode definition levels (ballot + popcount + LDS prefix -> value index)
//     and dictionary indices (branch-free buffer loads, run lookup in LDS), fold every string column into leaf
//     T/F bits and the group id, look the row up in the filter's truth table (Kleene logic precomputed on the
//     host) -> pass bitmap + group ids in LDS;
//   phase 2: every timestamp/value load of the sub-tile is issued before the first use, non-passing lanes use
//     an out-of-range buffer offset (the hardware drops them: late materialization without branches); bucket
//     by exact 32-bit reciprocal division; accumulate in a per-thread register cell (time-sorted rows hit it),
//     spilling to an LDS hash table (LDS atomics, sums as compensated hi/lo via returning-atomic TwoSum);
//   tile end: LDS cells -> global table with device atomics (count/min/max exact, sums within 1 ulp).
// finalize_*: per output key, combine glob slots (and the name dimension when the query has no groupBys,
//   TimeGroupedSketchAggregator.scala:148-170) and compact non-empty keys in (glob, bucket, group) order.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "device_common.hpp"
#include "kernels.hpp"
#include "layout.hpp"
#include "scan_kernel.hpp"

namespace lk {

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
    case AGG_ROWS: return double(F.rows[cell]);
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
  unsigned long long cnt = 0, nrows = 0;
  uint32_t best_rank = 0xffffffffu;
  for (uint32_t gs = 0; gs < F.nglob_slots; gs++) {
    for (unsigned long long g = g0; g < g0 + ng; g++) {
      unsigned long long cell = ((unsigned long long)gs * F.nbuckets + b) * F.ngroups + g;
      if (F.rows[cell] == 0) continue;
      unsigned long long c = F.cnt[cell];
      if (F.agg == AGG_SUM || F.agg == AGG_AVG) {
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
      nrows += F.rows[cell];
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
  else if (F.agg == AGG_AVG) o.value = (hi + lo) / double(cnt);   // merged {sum, count} map: 0/0 = NaN
  else if (F.agg == AGG_COUNT) o.value = double(cnt);
  else if (F.agg == AGG_ROWS) o.value = double(nrows);
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
      if (out_glob) out_glob[pos] = r.glob;   // null: merged rows (glob 0, a shared zero block on the host)
    }
    off += tot;
    __syncthreads();
  }
}

// Rank 0 of a sharded evaluation: fold ranks 1..world-1's partial tables (gathered whole, one [rows | cnt | hi |
// lo | ext] block of nc cells each, in rank order) into its own. rows/cnt add, min/max compare the
// order-preserving bits (exact), compensated sums add hi by TwoSum in rank order, so the merged sum is
// deterministic for a given shard assignment.
__global__ __launch_bounds__(256) void merge_tables(TableRef T, const unsigned long long* parts, int world, size_t nc,
                                                    int agg) {
  size_t i = size_t(blockIdx.x) * 256 + threadIdx.x;
  if (i >= nc) return;
  unsigned long long rows = T.rows[i], cnt = T.cnt[i], ext = T.ext[i];
  double h = T.hi[i], l = T.lo[i];
  for (int r = 1; r < world; r++) {
    const unsigned long long* p = parts + size_t(r) * nc * 5;
    rows += p[i];
    cnt += p[nc + i];
    if (agg == AGG_SUM) {
      double s, e;
      two_sum(h, __longlong_as_double((long long)p[2 * nc + i]), s, e);
      h = s;
      l += e + __longlong_as_double((long long)p[3 * nc + i]);
    } else if (agg == AGG_MIN) {
      ext = min(ext, p[4 * nc + i]);
    } else if (agg == AGG_MAX) {
      ext = max(ext, p[4 * nc + i]);
    }
  }
  T.rows[i] = rows;
  T.cnt[i] = cnt;
  T.hi[i] = h;
  T.lo[i] = l;
  T.ext[i] = ext;
}

// Merged min/max when values can be NULL: per-glob cells keep NULL, "null" and "" group values apart (DuckDB
// groups them separately and a group whose values are all NULL reads back 0.0, Commons.scala:427); the
// query-api then merges rows whose tag maps are equal (the three drop to the same map, Commons.scala:433).
// Re-key every per-glob cell to its collapsed group and fold its SQL value in with exact min/max.
__global__ __launch_bounds__(256) void rekey_minmax(RParams R) {
  size_t i = size_t(blockIdx.x) * 256 + threadIdx.x;
  if (i >= R.ncells_in) return;
  unsigned long long rows = R.in_rows[i];
  if (rows == 0) return;
  unsigned long long g = i % R.ngroups;
  unsigned long long b = (i / R.ngroups) % R.nbuckets;
  unsigned long long cg = 0;
  for (int d = 0; d < R.ndims; d++) {
    unsigned long long v = (g / R.stride[d]) % R.ndim[d];
    if (R.map[d]) v = R.map[d][v];
    cg += v * R.stride[d];
  }
  unsigned long long o = b * R.ngroups + cg;
  unsigned long long v = R.in_cnt[i] ? R.in_ext[i] : dbl_order(0.0);
  atomicAdd(&R.out_rows[o], rows);
  atomicMax(&R.out_cnt[o], 1ull);
  if (R.agg == AGG_MIN) atomicMin(&R.out_ext[o], v);
  else atomicMax(&R.out_ext[o], v);
}

// ------------------------------------------------------------------------------------------------
// Host launchers
// ------------------------------------------------------------------------------------------------
hipError_t launch_rekey_minmax(const RParams& R, hipStream_t stream) {
  if (R.ncells_in == 0) return hipSuccess;
  hipLaunchKernelGGL(rekey_minmax, dim3(uint32_t((R.ncells_in + 255) / 256)), dim3(256), 0, stream, R);
  return hipGetLastError();
}

hipError_t launch_merge_tables(const TableRef& T, const unsigned long long* parts, int world, size_t nc, int agg,
                              hipStream_t stream) {
  if (nc == 0 || world <= 1) return hipSuccess;
  hipLaunchKernelGGL(merge_tables, dim3(uint32_t((nc + 255) / 256)), dim3(256), 0, stream, T, parts, world, nc, agg);
  return hipGetLastError();
}

template <int AGG>
static void launch_agg(const QParams& P, dim3 grid, hipStream_t st) {
  const dim3 block(BLOCK);
  if (!P.truth) {   // > TT_MAX_LEAVES leaves: one generic instantiation interprets the Kleene program per row
    hipLaunchKernelGGL((scan_tiles<AGG, MAXSTR, false>), grid, block, 0, st, P);
    return;
  }
  switch (P.nstr) {
    case 1: hipLaunchKernelGGL((scan_tiles<AGG, 1, true>), grid, block, 0, st, P); break;
    case 2: hipLaunchKernelGGL((scan_tiles<AGG, 2, true>), grid, block, 0, st, P); break;
    case 3: hipLaunchKernelGGL((scan_tiles<AGG, 3, true>), grid, block, 0, st, P); break;
    case 4: hipLaunchKernelGGL((scan_tiles<AGG, 4, true>), grid, block, 0, st, P); break;
    case 5: hipLaunchKernelGGL((scan_tiles<AGG, 5, true>), grid, block, 0, st, P); break;
    default: hipLaunchKernelGGL((scan_tiles<AGG, 6, true>), grid, block, 0, st, P); break;
  }
}

hipError_t launch_scan(const QParams& P, int agg, hipStream_t stream) {
  if (P.total_tiles == 0 || P.nsegs == 0) return hipSuccess;
  if (P.nstr < 1 || P.nstr > MAXSTR) return hipErrorInvalidValue;
  const dim3 grid(P.max_tiles, P.nsegs);
  switch (agg) {
    case AGG_SUM: launch_agg<AGG_SUM>(P, grid, stream); break;
    case AGG_MIN: launch_agg<AGG_MIN>(P, grid, stream); break;
    case AGG_MAX: launch_agg<AGG_MAX>(P, grid, stream); break;
    default: launch_agg<AGG_COUNT>(P, grid, stream); break;
  }
  return hipGetLastError();
}

uint32_t finalize_blocks(unsigned long long nkeys) {
  return uint32_t((nkeys + FB * FITEMS - 1) / (FB * FITEMS));
}

hipError_t launch_finalize_count(const FParams& F, uint32_t* d_counts, hipStream_t stream) {
  uint32_t nb = finalize_blocks(F.nkeys);
  if (nb == 0) return hipMemsetAsync(d_counts, 0, sizeof(uint32_t), stream);
  hipLaunchKernelGGL(finalize_count, dim3(nb), dim3(FB), 0, stream, F, d_counts);
  hipLaunchKernelGGL(finalize_scan, dim3(1), dim3(1024), 0, stream, d_counts, nb);
  return hipGetLastError();
}

hipError_t launch_finalize_write(const FParams& F, const uint32_t* d_counts, int64_t* ts, double* val,
                                 unsigned long long* gid, uint32_t* glob, hipStream_t stream) {
  uint32_t nb = finalize_blocks(F.nkeys);
  if (nb == 0) return hipSuccess;
  hipLaunchKernelGGL(finalize_write, dim3(nb), dim3(FB), 0, stream, F, d_counts, ts, val, gid, glob);
  return hipGetLastError();
}

hipError_t launch_finalize(const FParams& F, uint32_t* d_counts, int64_t* ts, double* val, unsigned long long* gid,
                           uint32_t* glob, hipStream_t stream) {
  hipError_t e = launch_finalize_count(F, d_counts, stream);
  if (e != hipSuccess) return e;
  return launch_finalize_write(F, d_counts, ts, val, gid, glob, stream);
}

}  // namespace lk
