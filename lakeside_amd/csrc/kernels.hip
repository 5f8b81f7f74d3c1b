// HIP kernels for gfx950 (MI355X): sealed-segment DataExpr scan + table finalize/compaction.
// (The scan kernel's instantiations live in scan_<agg>.hip, one translation unit per aggregate, built in parallel.)
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
#include "scan_inst.hpp"   // launch_scan_agg (host dispatch; the kernels live in the scan_*.hip units)
#include "layout.hpp"

#include <hipcub/device/device_radix_sort.hpp>

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

// query-api's merge of per-glob min/max values: Scala math.min / math.max = java.lang.Math (a NaN argument gives NaN;
// -0.0 < +0.0), TimeGroupedSketchAggregator.scala:79-88.  (fmin/fmax would drop the NaN.)
__device__ __forceinline__ double java_min(double a, double b) {
  if (a != a || b != b) return __longlong_as_double(0x7ff8000000000000ll);
  if (a == 0.0 && b == 0.0) return signbit(a) ? a : b;
  return a < b ? a : b;
}
__device__ __forceinline__ double java_max(double a, double b) {
  if (a != a || b != b) return __longlong_as_double(0x7ff8000000000000ll);
  if (a == 0.0 && b == 0.0) return signbit(a) ? b : a;
  return a > b ? a : b;
}

// Output key -> row. Per-glob: key = (glob, bucket, group). Merged: key = (bucket, group) or (bucket)
// when the name dimension collapses (no groupBys).
__device__ OutRow make_row(const FParams& F, unsigned long long key) {
  OutRow o{false, 0.0, 0, 0};
  if (F.per_glob) {   // key = (bucket, glob, group): rows ascending in time, ties by glob (Commons.scala:391-392)
    const unsigned long long g = key % F.ngroups, t = key / F.ngroups;
    const unsigned long long gs = t % F.nglob_slots, b = t / F.nglob_slots;
    const unsigned long long cell = (gs * F.nbuckets + b) * F.ngroups + g - F.cell_base;
    if (F.rows[cell] == 0) return o;
    o.exists = true;
    o.value = cell_value(F, cell);
    o.gid = g;
    o.glob = uint32_t(gs);
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
      unsigned long long cell = ((unsigned long long)gs * F.nbuckets + b) * F.ngroups + g - F.cell_base;
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
        else ext = (F.agg == AGG_MIN) ? java_min(ext, v) : java_max(ext, v);
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
    const bool ex = key < F.nkeys && make_row(F, F.key_base + key).exists;
    n += ex ? 1u : 0u;
    if (F.key_bits) {   // one 64-key word per wave (keys 64-aligned: base is a multiple of FB * FITEMS)
      const unsigned long long w = __ballot(ex);
      if ((threadIdx.x & 63) == 0) F.key_bits[(key - (threadIdx.x & 63)) >> 6] = w;
    }
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
                                                   double* out_val, uint32_t* out_gid,
                                                   uint32_t* out_glob) {
  __shared__ uint32_t ws[FB / 64];
  const unsigned long long base = (unsigned long long)blockIdx.x * FB * FITEMS;
  uint32_t off = block_offsets[blockIdx.x];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int i = 0; i < FITEMS; i++) {
    const unsigned long long local = base + (unsigned long long)i * FB + threadIdx.x;
    const unsigned long long key = F.key_base + local;
    OutRow r{false, 0, 0, 0};
    if (local < F.nkeys) r = make_row(F, key);
    unsigned long long m = __ballot(r.exists);
    if (lane == 0) ws[wave] = __popcll(m);
    __syncthreads();
    uint32_t wb = 0, tot = 0;
    for (int w = 0; w < FB / 64; w++) {
      wb += (w < wave) ? ws[w] : 0;
      tot += ws[w];
    }
    if (r.exists) {
      const uint32_t pos = off + wb + __popcll(m & ((1ull << lane) - 1ull));
      const unsigned long long b = F.per_glob ? key / F.ngroups / F.nglob_slots : (F.collapse ? key : key / F.ngroups);
      if (out_ts) out_ts[pos] = F.bucket_base + (int64_t)b * F.step;   // null: expanded on the host
      out_val[pos] = r.value;
      if (out_gid) out_gid[pos] = uint32_t(r.gid);   // null: derived on the host (key_bits)
      if (out_glob) out_glob[pos] = r.glob;   // null: merged rows (glob 0, a shared zero block on the host)
    }
    off += tot;
    __syncthreads();
  }
}

// Large results (FParams::bucket_pos, whole key space): the row position of every bucket's first row -- rows are
// bucket-major, so it is the scanned count of the block holding the bucket's first key plus the existing keys ahead of
// it in that block -- and bucket_pos[nbuckets] = the row count.  One workgroup per bucket; enqueued before
// finalize_write, so the host expands the timestamps while the other columns cross the host link.
__global__ __launch_bounds__(FB) void finalize_bucket_pos(FParams F, const uint32_t* block_offsets, uint32_t nb) {
  __shared__ uint32_t ws[FB / 64];
  const unsigned long long per = F.per_glob ? F.ngroups * F.nglob_slots : (F.collapse ? 1ull : F.ngroups);
  const unsigned long long b = blockIdx.x;
  const unsigned long long K = b * per;
  const unsigned long long blk = K / (FB * FITEMS);
  uint32_t n = 0;
  for (unsigned long long k = blk * FB * FITEMS + threadIdx.x; k < K; k += FB) n += make_row(F, k).exists ? 1u : 0u;
  for (int o = 32; o > 0; o >>= 1) n += __shfl_down(n, o, 64);
  if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = n;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t t = 0;
    for (int w = 0; w < FB / 64; w++) t += ws[w];
    F.bucket_pos[b] = block_offsets[blk] + t;
    if (b == 0) F.bucket_pos[F.nbuckets] = block_offsets[nb];
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
// Re-key every per-glob cell to its collapsed group and fold its SQL value in with math.min / math.max (order bits;
// for MIN a NaN value re-orders below everything, MIN_NAN_ORDER, so it absorbs like java.lang.Math.min).
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
  if (R.agg == AGG_MIN && v == NAN_ORDER) v = MIN_NAN_ORDER;   // math.min: a NaN row absorbs the merge
  atomicAdd(&R.out_rows[o], rows);
  atomicMax(&R.out_cnt[o], 1ull);
  if (R.agg == AGG_MIN) atomicMin(&R.out_ext[o], v);
  else atomicMax(&R.out_ext[o], v);
}


// ------------------------------------------------------------------------------------------------
// Hash mode: record exchange (multi-GPU) and sparse finalize
// ------------------------------------------------------------------------------------------------
constexpr int SB = 256;
constexpr int SITEMS = 8;

__device__ __forceinline__ bool slot_live(const SParams& S, unsigned long long i) {
  return S.keys[i] != EMPTY && S.rows[i] != 0;
}

__global__ __launch_bounds__(SB) void sparse_count(SParams S, uint32_t* block_counts) {
  __shared__ uint32_t ws[SB / 64];
  uint32_t n = 0;
  const unsigned long long base = (unsigned long long)blockIdx.x * SB * SITEMS;
  for (int i = 0; i < SITEMS; i++) {
    const unsigned long long k = base + (unsigned long long)i * SB + threadIdx.x;
    if (k < S.cap && slot_live(S, k)) n++;
  }
  for (int o = 32; o > 0; o >>= 1) n += __shfl_down(n, o, 64);
  if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = n;
  __syncthreads();
  if (threadIdx.x == 0) block_counts[blockIdx.x] = ws[0] + ws[1] + ws[2] + ws[3];
}

// Output key of a cell key (see SParams): per-glob (bucket, glob, group); merged (bucket, group) with the group
// folded under the rekey maps, or (bucket) when the name dimension collapses.
__device__ __forceinline__ unsigned long long out_key(const SParams& S, unsigned long long cell) {
  const unsigned long long g = cell % S.ngroups, t = cell / S.ngroups;
  const unsigned long long b = t % S.nbuckets, gs = t / S.nbuckets;
  if (S.per_glob) return (b * S.nslots + gs) * S.ngroups + g;
  if (S.collapse) return b;
  if (!S.rekey) return b * S.ngroups + g;
  unsigned long long cg = 0;
  for (int d = 0; d < S.ndims; d++) {
    unsigned long long v = (g / S.stride[d]) % S.ndim[d];
    if (S.map[d]) v = S.map[d][v];
    cg += v * S.stride[d];
  }
  return b * S.ngroups + cg;
}

// Compact (output key, slot) of occupied slots at their block's scanned offset.
__global__ __launch_bounds__(SB) void sparse_emit(SParams S, const uint32_t* block_offsets, unsigned long long* okey,
                                                  uint32_t* oslot) {
  __shared__ uint32_t ws[SB / 64];
  const unsigned long long base = (unsigned long long)blockIdx.x * SB * SITEMS;
  uint32_t off = block_offsets[blockIdx.x];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int i = 0; i < SITEMS; i++) {
    const unsigned long long k = base + (unsigned long long)i * SB + threadIdx.x;
    const bool live = k < S.cap && slot_live(S, k);
    const unsigned long long m = __ballot(live);
    if (lane == 0) ws[wave] = __popcll(m);
    __syncthreads();
    uint32_t wb = 0, tot = 0;
    for (int w = 0; w < SB / 64; w++) {
      wb += (w < wave) ? ws[w] : 0;
      tot += ws[w];
    }
    if (live) {
      const uint32_t pos = off + wb + __popcll(m & ((1ull << lane) - 1ull));
      okey[pos] = out_key(S, S.keys[k]);
      oslot[pos] = uint32_t(k);
    }
    off += tot;
    __syncthreads();
  }
}

// Run heads of the sorted output keys, counted per block.
__global__ __launch_bounds__(SB) void runs_count(const unsigned long long* k, unsigned long long n, uint32_t* block_counts) {
  __shared__ uint32_t ws[SB / 64];
  uint32_t c = 0;
  const unsigned long long base = (unsigned long long)blockIdx.x * SB * SITEMS;
  for (int i = 0; i < SITEMS; i++) {
    const unsigned long long j = base + (unsigned long long)i * SB + threadIdx.x;
    if (j < n && (j == 0 || k[j] != k[j - 1])) c++;
  }
  for (int o = 32; o > 0; o >>= 1) c += __shfl_down(c, o, 64);
  if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) block_counts[blockIdx.x] = ws[0] + ws[1] + ws[2] + ws[3];
}

// One row per run of equal output keys: the run's cells combined as make_row combines dense cells.
__global__ __launch_bounds__(SB) void runs_write(SParams S, const unsigned long long* k, const uint32_t* slot,
                                                 unsigned long long n, const uint32_t* block_offsets, int64_t* out_ts,
                                                 double* out_val, uint32_t* out_gid, uint32_t* out_glob) {
  __shared__ uint32_t ws[SB / 64];
  const unsigned long long base = (unsigned long long)blockIdx.x * SB * SITEMS;
  uint32_t off = block_offsets[blockIdx.x];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int i = 0; i < SITEMS; i++) {
    const unsigned long long j = base + (unsigned long long)i * SB + threadIdx.x;
    const bool head = j < n && (j == 0 || k[j] != k[j - 1]);
    const unsigned long long m = __ballot(head);
    if (lane == 0) ws[wave] = __popcll(m);
    __syncthreads();
    uint32_t wb = 0, tot = 0;
    for (int w = 0; w < SB / 64; w++) {
      wb += (w < wave) ? ws[w] : 0;
      tot += ws[w];
    }
    if (head) {
      const unsigned long long key = k[j];
      double hi = 0.0, lo = 0.0, ext = 0.0;
      unsigned long long cnt = 0, nrows = 0, oext = (S.agg == AGG_MIN) ? ~0ull : 0ull, gid = 0;
      uint32_t best_rank = 0xffffffffu, glob = 0;
      bool any = false;
      for (unsigned long long e = j; e < n && k[e] == key; e++) {
        const uint32_t c = slot[e];
        const unsigned long long cell = S.keys[c];
        const unsigned long long g = cell % S.ngroups;
        const unsigned long long cc = S.cnt[c];
        if (S.agg == AGG_SUM || S.agg == AGG_AVG) {
          double s2, e2;
          two_sum(hi, S.hi[c], s2, e2);
          hi = s2;
          lo += e2 + S.lo[c];
        } else if (S.agg == AGG_MIN || S.agg == AGG_MAX) {
          if (S.rekey) {   // per-glob SQL value: NULL cell -> 0.0 (Commons.scala:427), exact min/max on order bits
            unsigned long long v = cc ? S.ext[c] : dbl_order(0.0);
            if (S.agg == AGG_MIN && v == NAN_ORDER) v = MIN_NAN_ORDER;   // math.min: NaN absorbs
            oext = (S.agg == AGG_MIN) ? (v < oext ? v : oext) : (v > oext ? v : oext);
          } else {
            const double v = cc ? order_dbl(S.ext[c]) : 0.0;
            if (!any) ext = v;
            else ext = (S.agg == AGG_MIN) ? java_min(ext, v) : java_max(ext, v);
          }
        }
        cnt += cc;
        nrows += S.rows[c];
        const uint32_t rank = (S.collapse && S.name_rank) ? S.name_rank[g / S.name_stride] : 0u;
        if (!any || rank < best_rank) {
          best_rank = rank;
          gid = S.rekey ? key % S.ngroups : g;
          glob = uint32_t(cell / S.ngroups / S.nbuckets);
        }
        any = true;
      }
      double value;
      if (S.agg == AGG_COUNT) value = double(cnt);
      else if (S.agg == AGG_ROWS) value = double(nrows);
      else if (S.agg == AGG_SUM) value = cnt ? hi + lo : 0.0;
      else if (S.agg == AGG_AVG) value = S.per_glob ? (cnt ? (hi + lo) / double(cnt) : 0.0) : (hi + lo) / double(cnt);
      else if (S.rekey) value = order_dbl(oext);
      else value = ext;
      const unsigned long long b = S.per_glob ? key / S.ngroups / S.nslots : (S.collapse ? key : key / S.ngroups);
      const uint32_t pos = off + wb + __popcll(m & ((1ull << lane) - 1ull));
      out_ts[pos] = S.bucket_base + (int64_t)b * S.step;
      out_val[pos] = value;
      out_gid[pos] = uint32_t(gid);
      if (out_glob) out_glob[pos] = S.per_glob ? glob : 0u;
    }
    off += tot;
    __syncthreads();
  }
}

// Rank 0: fold records [key | rows | cnt | hi | lo | ext] of another rank's hash table into its own.
template <int AGG>
__global__ __launch_bounds__(256) void merge_records(QParams P, const unsigned long long* recs, size_t n) {
  const size_t i = size_t(blockIdx.x) * 256 + threadIdx.x;
  if (i >= n) return;
  const unsigned long long rows = recs[n + i];
  if (!rows) return;
  const unsigned long long slot = hash_slot(P.hkeys, P.hmask, P.flags, recs[i]);   // merge target: hash table
  if (slot == EMPTY) return;
  atomicAdd(&P.rows[slot], rows);
  const unsigned long long cnt = recs[2 * n + i];
  if (!cnt) return;
  atomicAdd(&P.cnt[slot], cnt);
  if (AGG == AGG_SUM) {
    const double h = __longlong_as_double((long long)recs[3 * n + i]);
    const double l = __longlong_as_double((long long)recs[4 * n + i]);
    const double old = atomicAdd(&P.hi[slot], h);
    double s, e;
    two_sum(old, h, s, e);
    atomicAdd(&P.lo[slot], l + e);
  } else if (AGG == AGG_MIN) {
    atomicMin(&P.ext[slot], recs[5 * n + i]);
  } else if (AGG == AGG_MAX) {
    atomicMax(&P.ext[slot], recs[5 * n + i]);
  }
}

// Occupied slots of a hash-mode table -> compact records (offsets from the sparse count + scan).
__global__ __launch_bounds__(SB) void table_records(SParams S, const uint32_t* block_offsets, unsigned long long* recs,
                                                    size_t n) {
  __shared__ uint32_t ws[SB / 64];
  const unsigned long long base = (unsigned long long)blockIdx.x * SB * SITEMS;
  uint32_t off = block_offsets[blockIdx.x];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int i = 0; i < SITEMS; i++) {
    const unsigned long long k = base + (unsigned long long)i * SB + threadIdx.x;
    const bool live = k < S.cap && slot_live(S, k);
    const unsigned long long m = __ballot(live);
    if (lane == 0) ws[wave] = __popcll(m);
    __syncthreads();
    uint32_t wb = 0, tot = 0;
    for (int w = 0; w < SB / 64; w++) {
      wb += (w < wave) ? ws[w] : 0;
      tot += ws[w];
    }
    if (live) {
      const size_t pos = off + wb + __popcll(m & ((1ull << lane) - 1ull));
      recs[pos] = S.keys[k];
      recs[n + pos] = S.rows[k];
      recs[2 * n + pos] = S.cnt[k];
      recs[3 * n + pos] = (unsigned long long)__double_as_longlong(S.hi[k]);
      recs[4 * n + pos] = (unsigned long long)__double_as_longlong(S.lo[k]);
      recs[5 * n + pos] = S.ext[k];
    }
    off += tot;
    __syncthreads();
  }
}

// Lean tables (LEAN_*): restore rows / cnt after the scan.  NO_ROWS (min/max, no NULL values): a cell exists iff
// its extreme left the identity; its SQL count is then >= 1 (only existence is read downstream).  NO_CNT: cnt = rows.
__global__ __launch_bounds__(256) void fixup_table(QParams P, unsigned long long nc, int agg) {
  const unsigned long long i = (unsigned long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= nc) return;
  if (P.hkeys && P.hkeys[i] == EMPTY) return;
  if (P.lean & LEAN_SUM_EXISTS) {
    const bool e = (unsigned long long)__double_as_longlong(P.hi[i]) != NEG_ZERO_BITS;
    P.rows[i] = e ? 1ull : 0ull;
    P.cnt[i] = e ? 1ull : 0ull;
    if (!e) P.hi[i] = 0.0;
  } else if (P.lean & LEAN_NO_ROWS) {
    const unsigned long long ident = agg == AGG_MIN ? ~0ull : 0ull;
    const unsigned long long e = P.ext[i] != ident ? 1ull : 0ull;
    P.rows[i] = e;
    P.cnt[i] = e;
  } else if (P.lean & LEAN_NO_CNT) {
    P.cnt[i] = P.rows[i];
  }
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


hipError_t launch_merge_records(const QParams& P, const unsigned long long* recs, size_t n, int agg, hipStream_t st) {
  if (n == 0) return hipSuccess;
  const dim3 g(uint32_t((n + 255) / 256)), b(256);
  switch (agg) {
    case AGG_SUM: hipLaunchKernelGGL(merge_records<AGG_SUM>, g, b, 0, st, P, recs, n); break;
    case AGG_MIN: hipLaunchKernelGGL(merge_records<AGG_MIN>, g, b, 0, st, P, recs, n); break;
    case AGG_MAX: hipLaunchKernelGGL(merge_records<AGG_MAX>, g, b, 0, st, P, recs, n); break;
    default: hipLaunchKernelGGL(merge_records<AGG_COUNT>, g, b, 0, st, P, recs, n); break;
  }
  return hipGetLastError();
}

__global__ __launch_bounds__(256) void fill_u64(unsigned long long* p, unsigned long long n, unsigned long long v) {
  for (unsigned long long i = (unsigned long long)blockIdx.x * 256 + threadIdx.x; i < n; i += (unsigned long long)gridDim.x * 256)
    p[i] = v;
}

__global__ __launch_bounds__(256) void fill_many(FillList L) {
  const unsigned long long stride = (unsigned long long)gridDim.x * 256;
  for (int k = 0; k < L.count; k++) {
    unsigned long long* p = L.p[k];
    const unsigned long long n = L.n[k], v = L.v[k];
    for (unsigned long long i = (unsigned long long)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) p[i] = v;
  }
}

hipError_t launch_fill_many(const FillList& L, hipStream_t st) {
  unsigned long long mx = 0;
  for (int k = 0; k < L.count; k++) mx = std::max(mx, L.n[k]);
  if (mx == 0) return hipSuccess;
  const unsigned long long blocks = std::min<unsigned long long>((mx + 255) / 256, 8192);
  hipLaunchKernelGGL(fill_many, dim3(uint32_t(blocks)), dim3(256), 0, st, L);
  return hipGetLastError();
}

// One workgroup: fixup (as fixup_table) -> barrier -> rows in key order (as finalize_count / scan / write, the block
// walking the keys 1024 at a time with a running offset) -> flags and row count to the host.  The barrier makes the
// fixup's table writes visible to every wave of the workgroup (HIP __syncthreads semantics for global memory).
constexpr int EB = 1024;
__global__ __launch_bounds__(EB) void epilogue_small(QParams P, FParams F, unsigned long long nc, int agg, int64_t* out_ts,
                                                   double* out_val, uint32_t* out_gid, uint32_t* out_glob,
                                                   const uint32_t* dflags, uint32_t* host_tail) {
  __shared__ uint32_t ws[EB / 64];
  if (P.lean)
    for (unsigned long long i = threadIdx.x; i < nc; i += EB) {
      if (P.lean & LEAN_SUM_EXISTS) {
        const bool e = (unsigned long long)__double_as_longlong(P.hi[i]) != NEG_ZERO_BITS;
        P.rows[i] = e ? 1ull : 0ull;
        P.cnt[i] = e ? 1ull : 0ull;
        if (!e) P.hi[i] = 0.0;
      } else if (P.lean & LEAN_NO_ROWS) {
        const unsigned long long ident = agg == AGG_MIN ? ~0ull : 0ull;
        const unsigned long long e = P.ext[i] != ident ? 1ull : 0ull;
        P.rows[i] = e;
        P.cnt[i] = e;
      } else if (P.lean & LEAN_NO_CNT) {
        P.cnt[i] = P.rows[i];
      }
    }
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  uint32_t off = 0;
  for (unsigned long long base = 0; base < F.nkeys; base += EB) {   // uniform trip count
    const unsigned long long local = base + threadIdx.x;
    const unsigned long long key = F.key_base + local;
    OutRow r{false, 0, 0, 0};
    if (local < F.nkeys) r = make_row(F, key);
    const unsigned long long m = __ballot(r.exists);
    if (lane == 0) ws[wave] = uint32_t(__popcll(m));
    __syncthreads();
    uint32_t wb = 0, tot = 0;
    for (int w = 0; w < EB / 64; w++) {
      wb += (w < wave) ? ws[w] : 0u;
      tot += ws[w];
    }
    if (r.exists) {
      const uint32_t pos = off + wb + uint32_t(__popcll(m & ((1ull << lane) - 1ull)));
      const unsigned long long b = F.per_glob ? key / F.ngroups / F.nglob_slots : (F.collapse ? key : key / F.ngroups);
      out_ts[pos] = F.bucket_base + (int64_t)b * F.step;
      out_val[pos] = r.value;
      out_gid[pos] = uint32_t(r.gid);
      if (out_glob) out_glob[pos] = r.glob;
    }
    off += tot;
    __syncthreads();
  }
  if (threadIdx.x < 4) host_tail[threadIdx.x] = dflags[threadIdx.x];
  if (threadIdx.x == 0) host_tail[4] = off;
}

hipError_t launch_epilogue_small(const QParams& P, const FParams& F, unsigned long long nc, int agg, int64_t* ts,
                                 double* val, uint32_t* gid, uint32_t* glob, const uint32_t* dflags,
                                 uint32_t* host_tail, hipStream_t st) {
  if (nc > kEpilogueMax || F.nkeys > kEpilogueMax) return hipErrorInvalidValue;
  hipLaunchKernelGGL(epilogue_small, dim3(1), dim3(EB), 0, st, P, F, nc, agg, ts, val, gid, glob, dflags, host_tail);
  return hipGetLastError();
}

// Dictionary compaction (Engine::compact_locked): a segment's chunk remap, old engine id -> new id.
__global__ __launch_bounds__(256) void remap_ids(uint32_t* p, unsigned long long n, const uint32_t* map) {
  for (unsigned long long i = (unsigned long long)blockIdx.x * 256 + threadIdx.x; i < n; i += (unsigned long long)gridDim.x * 256)
    p[i] = map[p[i]];
}

hipError_t launch_remap_ids(uint32_t* p, unsigned long long n, const uint32_t* map, hipStream_t st) {
  if (n == 0) return hipSuccess;
  const unsigned long long blocks = std::min<unsigned long long>((n + 255) / 256, 4096);
  hipLaunchKernelGGL(remap_ids, dim3(uint32_t(blocks)), dim3(256), 0, st, p, n, map);
  return hipGetLastError();
}

hipError_t launch_fill_u64(unsigned long long* p, unsigned long long n, unsigned long long v, hipStream_t st) {
  if (n == 0) return hipSuccess;
  const unsigned long long blocks = std::min<unsigned long long>((n + 255) / 256, 8192);
  hipLaunchKernelGGL(fill_u64, dim3(uint32_t(blocks)), dim3(256), 0, st, p, n, v);
  return hipGetLastError();
}

hipError_t launch_fixup_table(const QParams& P, unsigned long long nc, int agg, hipStream_t st) {
  if (!P.lean || nc == 0) return hipSuccess;
  hipLaunchKernelGGL(fixup_table, dim3(uint32_t((nc + 255) / 256)), dim3(256), 0, st, P, nc, agg);
  return hipGetLastError();
}

uint32_t sparse_blocks(unsigned long long cap) { return uint32_t((cap + SB * SITEMS - 1) / (SB * SITEMS)); }

hipError_t launch_sparse_count(const SParams& S, uint32_t* d_counts, hipStream_t st) {
  const uint32_t nb = sparse_blocks(S.cap);
  if (nb == 0) return hipMemsetAsync(d_counts, 0, sizeof(uint32_t), st);
  hipLaunchKernelGGL(sparse_count, dim3(nb), dim3(SB), 0, st, S, d_counts);
  hipLaunchKernelGGL(finalize_scan, dim3(1), dim3(1024), 0, st, d_counts, nb);
  return hipGetLastError();
}

hipError_t launch_table_records(const QParams& P, unsigned long long cap, uint32_t* d_counts, unsigned long long* recs,
                                size_t n, hipStream_t st) {
  SParams S{};
  S.keys = P.hkeys;
  S.rows = P.rows;
  S.cnt = P.cnt;
  S.hi = P.hi;
  S.lo = P.lo;
  S.ext = P.ext;
  S.cap = cap;
  const uint32_t nb = sparse_blocks(cap);
  if (nb == 0 || n == 0) return hipSuccess;
  hipLaunchKernelGGL(table_records, dim3(nb), dim3(SB), 0, st, S, d_counts, recs, n);
  return hipGetLastError();
}

// sparse workspace: okey[2n] | oslot[2n] | run counts | sort temp
namespace {
struct SparseWs {
  unsigned long long *k0, *k1;
  uint32_t *s0, *s1, *counts;
  void* temp;
  size_t temp_bytes;
};
size_t sort_temp_bytes(unsigned long long n, int end_bit) {
  size_t t = 0;
  (void)hipcub::DeviceRadixSort::SortPairs(nullptr, t, (unsigned long long*)nullptr, (unsigned long long*)nullptr,
                                           (uint32_t*)nullptr, (uint32_t*)nullptr, int(n), 0, end_bit, hipStream_t(0));
  return t;
}
SparseWs carve(void* ws, unsigned long long n, int end_bit) {
  auto al = [](size_t x) { return (x + 255) / 256 * 256; };
  uint8_t* p = static_cast<uint8_t*>(ws);
  SparseWs w;
  w.k0 = reinterpret_cast<unsigned long long*>(p);
  p += al(n * 8);
  w.k1 = reinterpret_cast<unsigned long long*>(p);
  p += al(n * 8);
  w.s0 = reinterpret_cast<uint32_t*>(p);
  p += al(n * 4);
  w.s1 = reinterpret_cast<uint32_t*>(p);
  p += al(n * 4);
  w.counts = reinterpret_cast<uint32_t*>(p);
  p += al((size_t(sparse_blocks(n)) + 2) * 4);
  w.temp = p;
  w.temp_bytes = sort_temp_bytes(n, end_bit);
  return w;
}
}  // namespace

size_t sparse_workspace_bytes(unsigned long long n, int end_bit) {
  auto al = [](size_t x) { return (x + 255) / 256 * 256; };
  return al(n * 8) * 2 + al(n * 4) * 2 + al((size_t(sparse_blocks(n)) + 2) * 4) + al(sort_temp_bytes(n, end_bit)) + 256;
}

hipError_t launch_sparse_sort(const SParams& S, const uint32_t* d_counts, unsigned long long n, int end_bit, void* ws,
                              uint32_t** d_nrows, hipStream_t st) {
  SparseWs w = carve(ws, n, end_bit);
  *d_nrows = w.counts + sparse_blocks(n);
  if (n == 0) return hipMemsetAsync(*d_nrows, 0, 4, st);
  hipLaunchKernelGGL(sparse_emit, dim3(sparse_blocks(S.cap)), dim3(SB), 0, st, S, d_counts, w.k0, w.s0);
  size_t tb = w.temp_bytes;
  hipError_t e = hipcub::DeviceRadixSort::SortPairs(w.temp, tb, w.k0, w.k1, w.s0, w.s1, int(n), 0, end_bit, st);
  if (e != hipSuccess) return e;
  const uint32_t nb = sparse_blocks(n);
  hipLaunchKernelGGL(runs_count, dim3(nb), dim3(SB), 0, st, w.k1, n, w.counts);
  hipLaunchKernelGGL(finalize_scan, dim3(1), dim3(1024), 0, st, w.counts, nb);
  return hipGetLastError();
}

hipError_t launch_sparse_write(const SParams& S, unsigned long long n, void* ws, int64_t* ts, double* val,
                               uint32_t* gid, uint32_t* glob, hipStream_t st) {
  if (n == 0) return hipSuccess;
  SparseWs w = carve(ws, n, 64);
  hipLaunchKernelGGL(runs_write, dim3(sparse_blocks(n)), dim3(SB), 0, st, S, w.k1, w.s1, n, w.counts, ts, val, gid, glob);
  return hipGetLastError();
}

hipError_t launch_scan(const QParams& P, int agg, hipStream_t stream) {
  if (P.total_tiles == 0 || P.nsegs == 0) return hipSuccess;
  if (P.nstr < 1 || P.nstr > MAXSTR) return hipErrorInvalidValue;
  const dim3 grid(P.max_tiles, P.nsegs);
  switch (agg) {
    case AGG_SUM: launch_scan_agg<AGG_SUM>(P, grid, stream); break;
    case AGG_MIN: launch_scan_agg<AGG_MIN>(P, grid, stream); break;
    case AGG_MAX: launch_scan_agg<AGG_MAX>(P, grid, stream); break;
    default: launch_scan_agg<AGG_COUNT>(P, grid, stream); break;
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
                                 uint32_t* gid, uint32_t* glob, hipStream_t stream) {
  uint32_t nb = finalize_blocks(F.nkeys);
  if (nb == 0) return hipSuccess;
  hipLaunchKernelGGL(finalize_write, dim3(nb), dim3(FB), 0, stream, F, d_counts, ts, val, gid, glob);
  return hipGetLastError();
}

hipError_t launch_finalize_bucket_pos(const FParams& F, const uint32_t* d_counts, hipStream_t stream) {
  const uint32_t nb = finalize_blocks(F.nkeys);
  if (nb == 0 || F.nbuckets == 0 || !F.bucket_pos || F.key_base) return hipErrorInvalidValue;
  hipLaunchKernelGGL(finalize_bucket_pos, dim3(uint32_t(F.nbuckets)), dim3(FB), 0, stream, F, d_counts, nb);
  return hipGetLastError();
}

hipError_t launch_finalize(const FParams& F, uint32_t* d_counts, int64_t* ts, double* val, uint32_t* gid,
                           uint32_t* glob, hipStream_t stream) {
  hipError_t e = launch_finalize_count(F, d_counts, stream);
  if (e != hipSuccess) return e;
  return launch_finalize_write(F, d_counts, ts, val, gid, glob, stream);
}

}  // namespace lk
