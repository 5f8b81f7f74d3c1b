// Host-visible interface of the HIP kernels (kernels.hip).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "layout.hpp"

namespace lk {

struct FParams {
  const unsigned long long* rows;
  const unsigned long long* cnt;
  const double* hi;
  const double* lo;
  const unsigned long long* ext;
  unsigned long long nkeys;        // output key space
  unsigned long long ngroups;
  unsigned long long nbuckets;
  unsigned long long name_stride;  // group-id stride of the name dimension (most significant)
  const uint32_t* name_rank;       // name dim id -> rank in string order (merged + collapse), or null
  uint32_t nglob_slots;
  int agg;                         // Agg, or 4 = avg
  int per_glob;                    // 1: one output row per (glob, bucket, group) cell
  int collapse;                    // merged without groupBys: one row per bucket (S19)
  int64_t bucket_base;
  int64_t step;
};

constexpr int AGG_AVG = 4;
constexpr int AGG_ROWS = 5;        // COUNT(*): passing rows, NULL values included (tag queries)

struct RParams {                   // rekey_minmax: per-glob uncollapsed table -> merged collapsed table
  const unsigned long long* in_rows;
  const unsigned long long* in_cnt;
  const unsigned long long* in_ext;
  unsigned long long ncells_in;
  unsigned long long* out_rows;
  unsigned long long* out_cnt;
  unsigned long long* out_ext;
  unsigned long long nbuckets;
  unsigned long long ngroups;
  int ndims;
  int agg;
  unsigned long long stride[MAXSTR];
  unsigned long long ndim[MAXSTR];
  const uint32_t* map[MAXSTR];     // dim id -> collapsed dim id (null: identity)
};

hipError_t launch_rekey_minmax(const RParams& R, hipStream_t stream);

// The aggregation table: one contiguous block [rows | cnt | hi | lo | ext] of nc cells each.
struct TableRef {
  unsigned long long* rows;
  unsigned long long* cnt;
  double* hi;
  double* lo;
  unsigned long long* ext;
};
hipError_t launch_merge_tables(const TableRef& T, const unsigned long long* parts, int world, size_t nc, int agg,
                               hipStream_t stream);
hipError_t launch_scan(const QParams& P, int agg, hipStream_t stream);
uint32_t finalize_blocks(unsigned long long nkeys);
// d_counts must hold finalize_blocks(nkeys) + 1 entries; the row total lands in d_counts[nblocks].
// Split form: count + scan (row total at d_counts[nblocks]), then write -- the write may target mapped pinned host
// memory (hipHostMalloc) directly, so no device->host copy follows.
hipError_t launch_finalize_count(const FParams& F, uint32_t* d_counts, hipStream_t stream);
hipError_t launch_finalize_write(const FParams& F, const uint32_t* d_counts, int64_t* ts, double* val,
                                 unsigned long long* gid, uint32_t* glob, hipStream_t stream);
hipError_t launch_finalize(const FParams& F, uint32_t* d_counts, int64_t* ts, double* val, unsigned long long* gid,
                           uint32_t* glob, hipStream_t stream);

}  // namespace lk
