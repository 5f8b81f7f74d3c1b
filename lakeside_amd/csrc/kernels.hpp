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
  // key-range finalize (distributed): output keys [key_base, key_base + nkeys); the table arrays hold
  // cells [cell_base, ...) of the full table (0, 0: the whole table)
  unsigned long long key_base;
  unsigned long long cell_base;
  // large results (whole key space): finalize_bucket_pos writes the row position of every bucket's first row here
  // (rows are in bucket-major order) and finalize_write is given no timestamp column -- the host expands it (8 of the
  // 20-24 bytes per row that cross the host link)
  uint32_t* bucket_pos;
  // large results with a group key (not collapsed): finalize_count also writes one existence bit per output key here
  // (mapped pinned memory), from which the host derives every row's timestamp, group id and glob -- finalize_write then
  // sends the values alone (8 of 20-24 bytes per row)
  unsigned long long* key_bits;
};

constexpr int AGG_AVG = 4;
constexpr int AGG_ROWS = 5;        // COUNT(*): passing rows, NULL values included (tag queries)
constexpr int AGG_SKETCH = 6;      // percentiles: COUNT per (cell, DDSketch bin) (P.sketch), sketches on the host
constexpr int AGG_CES = 7;         // cardinality estimates: distinct (cell) set, HLL per step on the host

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
// Hash-mode table of a rank merged into rank 0's: `n` gathered records [key | rows | cnt | hi | lo | ext] (n each).
hipError_t launch_merge_records(const QParams& P, const unsigned long long* recs, size_t n, int agg, hipStream_t stream);
// Hash-mode table -> compact records [key | rows | cnt | hi | lo | ext] (cap = slots; count first with
// launch_finalize_sparse's counting pass: rows land at d_counts offsets).
hipError_t launch_table_records(const QParams& P, unsigned long long cap, uint32_t* d_counts, unsigned long long* recs,
                                size_t n, hipStream_t stream);

// Sparse finalize (hash mode): occupied slots -> (output key, slot) -> radix sort -> one row per output key,
// cells of one key combined exactly as the dense finalize combines them.
struct SParams {
  const unsigned long long* keys;  // slot keys (EMPTY = ~0)
  const unsigned long long* rows;
  const unsigned long long* cnt;
  const double* hi;
  const double* lo;
  const unsigned long long* ext;
  unsigned long long cap;          // slots
  unsigned long long ngroups, nbuckets;
  uint32_t nslots;                 // glob slots of the cell keys
  int agg;
  int per_glob;                    // output key (bucket, glob, group)
  int collapse;                    // output key (bucket): the name dimension folds (no groupBys, merged)
  int rekey;                       // merged min/max with NULL-able values: per-glob SQL values fold under `map`
  int ndims;
  unsigned long long stride[MAXSTR];
  unsigned long long ndim[MAXSTR];
  const uint32_t* map[MAXSTR];
  unsigned long long name_stride;
  const uint32_t* name_rank;
  int64_t bucket_base;
  int64_t step;
};
// Workspace bytes launch_finalize_sparse needs for `n` occupied slots (sort buffers + scan + sort temp).
size_t sparse_workspace_bytes(unsigned long long n, int end_bit);
// Count occupied slots: total at d_counts[sparse_blocks(cap)] after the scan.
uint32_t sparse_blocks(unsigned long long cap);
hipError_t launch_sparse_count(const SParams& S, uint32_t* d_counts, hipStream_t stream);
// Build + sort (output key, slot) pairs of the `n` occupied slots and count the output rows: the row total lands
// at the returned device pointer (uint32).  `end_bit`: bits of the largest output key.
hipError_t launch_sparse_sort(const SParams& S, const uint32_t* d_counts, unsigned long long n, int end_bit, void* ws,
                              uint32_t** d_nrows, hipStream_t stream);
hipError_t launch_sparse_write(const SParams& S, unsigned long long n, void* ws, int64_t* ts, double* val,
                               uint32_t* gid, uint32_t* glob, hipStream_t stream);

// Exemplar scans (ex_kernels.hip).  ex_scan decodes the filter columns (QSeg cols 0 = timestamp, 2.. = strings) of
// every tile meeting its glob's open range [rlo, rhi) and either counts passing rows per time bin (HIST) or appends
// them as (timestamp, segment << 48 | tile << 16 | row) records (EMIT).
constexpr uint32_t XBINS = 2048;
enum XMode : uint32_t { XMODE_HIST = 0, XMODE_EMIT = 1, XMODE_AGG = 2, XMODE_TAGNUM = 3 };
// XMODE_TAGNUM (tag queries over a numeric tag column): passing rows counted per (glob, canonical tag value) in a
// per-glob open-addressing table (wave dedup -> LDS table -> device atomics); NULL tags and the one value whose
// canonical key is the empty marker (all ones) are counted apart.  NumLeaf.pad bit 1 (NUMLEAF_NOTNULL): the leaf is
// `IS NOT NULL` on that column (query-api's `exists` on the tag).
constexpr uint32_t NUMLEAF_NOTNULL = 2u;
constexpr unsigned long long TAG_EMPTY = ~0ull;
// A numeric comparison leaf (`gt/ge/lt/le`, BaseExpr.scala:488-498) on numeric filter column `col` (QSeg column
// 2 + nstr + col, its Parquet physical type in QCol.pad): TRUE iff the value lies in the interval, FALSE otherwise,
// UNKNOWN on NULL.  Integer columns test [ilo, ihi] (exact); floating columns the double interval, NaN (ordered
// greatest by DuckDB) passing iff nan_pass.
struct NumLeaf {
  uint32_t col, leaf;
  uint32_t lo_incl, hi_incl, nan_pass;
  uint32_t pad;                    // 1: integer columns compare as double (|literal| >= 1e7 prints in E notation)
  double dlo, dhi;
  long long ilo, ihi;
};
struct XParams {
  const QSeg* segs;
  uint32_t nsegs;
  uint32_t max_tiles;
  const StrParam* strp;            // [nstr]: strtab = global id -> leaf bits << 24
  uint32_t nstr;
  uint32_t nleaves;
  uint32_t nprog;
  uint8_t prog[MAXPROG];
  const uint32_t* truth;           // null: interpret prog
  const int64_t* rlo;              // per glob slot: the open range
  const int64_t* rhi;
  uint32_t mode;
  uint32_t nbins;                  // HIST: bins per glob (<= XBINS)
  uint32_t* hist;                  // HIST: [glob][nbins] passing rows
  const int64_t* hbase;            // HIST: per glob: bin b covers [hbase + b*hwidth, + hwidth)
  const int64_t* hwidth;
  unsigned long long* out;         // EMIT: 2 words per record
  uint32_t* out_n;                 // EMIT: records appended (may exceed cap: only the first cap are written)
  uint32_t cap;
  uint32_t nnum;                   // numeric filter columns
  uint32_t nnl;                    // numeric leaves
  NumLeaf nl[MAXLEAF];
  // AGG (general scan: the queries the fused kernels do not take, e.g. numeric leaves): rows in the glob window
  // aggregate into q's table (q.segs..q.strp as above; value column = QSeg column 1) with device atomics
  int agg;                         // Agg (kernel aggregate)
  int hash;                        // q's table is the hash-mode table
  QParams q;
  // TAGNUM: the tag's query column (its QCol.pad: Parquet type | glob union type << 8), per-glob tables of tcap slots
  // (keys TAG_EMPTY-initialised, 64-bit counts), per-glob [NULL rows, all-ones-key rows], overflow flag
  uint32_t tag_qc;
  unsigned long long tcap;
  unsigned long long* tkeys;
  unsigned long long* tcnt;
  unsigned long long* tspec;
  uint32_t* tflags;
};
// TAGNUM tables -> records [key, count, glob] of the occupied slots (unordered); count at *out_n.
hipError_t launch_tag_compact(const unsigned long long* keys, const unsigned long long* cnt, unsigned long long tcap,
                              uint32_t nglobs, unsigned long long* out, uint32_t* out_n, hipStream_t stream);
hipError_t launch_ex_scan(const XParams& X, hipStream_t stream);

struct GCol {                      // one (segment, output column) of an exemplar gather
  const uint8_t* base;             // segment streams
  const RunDesc* runs;
  const TileCol* tcols;
  const uint32_t* remap;
  uint32_t present;
  uint32_t pad;
};
struct GParams {
  const unsigned long long* sel;   // selected rows: segment << 48 | tile << 16 | row
  uint32_t nsel;
  uint32_t ncols;
  const GCol* cols;                // [segment][ncols]
  unsigned long long* val;         // [nsel][ncols]: raw value (8/4-B PLAIN, BOOLEAN bit, or string global id)
  uint8_t* ok;                     // [nsel][ncols]: 1 = non-NULL
};
hipError_t launch_ex_gather(const GParams& G, hipStream_t stream);

hipError_t launch_merge_tables(const TableRef& T, const unsigned long long* parts, int world, size_t nc, int agg,
                               hipStream_t stream);
hipError_t launch_scan(const QParams& P, int agg, hipStream_t stream);
// lean tables: restore the rows / cnt fields the scan did not accumulate (LEAN_* in layout.hpp)
hipError_t launch_remap_ids(uint32_t* p, unsigned long long n, const uint32_t* map, hipStream_t stream);
hipError_t launch_fixup_table(const QParams& P, unsigned long long nc, int agg, hipStream_t stream);
// p[0 .. n) = v (64-bit pattern fill: LEAN_SUM_EXISTS's -0.0)
hipError_t launch_fill_u64(unsigned long long* p, unsigned long long n, unsigned long long v, hipStream_t stream);
// Several 64-bit pattern fills in one launch (a table's planes and the scan flags before a scan).
struct FillList {
  static constexpr int kMax = 8;
  unsigned long long* p[kMax];
  unsigned long long n[kMax];
  unsigned long long v[kMax];
  int count;
};
hipError_t launch_fill_many(const FillList& L, hipStream_t stream);
// Small dense tables (nc, out_keys <= kEpilogueMax): the whole epilogue of a single-GPU scan in one single-workgroup
// launch -- the lean-table fixup, the output rows compacted in key order straight into the (mapped pinned) result
// columns, and the scan's flags (flags[0..3]) plus the row count written to host_tail[0..3] / host_tail[4] (mapped
// pinned host memory), so the host reads everything after one stream synchronization.
constexpr unsigned long long kEpilogueMax = 1ull << 16;
hipError_t launch_epilogue_small(const QParams& P, const FParams& F, unsigned long long nc, int agg, int64_t* ts,
                                 double* val, uint32_t* gid, uint32_t* glob, const uint32_t* dflags,
                                 uint32_t* host_tail, hipStream_t stream);
// one aggregate's scan instantiations (scan_<agg>.hip)
template <int AGG>
void launch_scan_agg(const QParams& P, dim3 grid, hipStream_t st);
uint32_t finalize_blocks(unsigned long long nkeys);
// d_counts must hold finalize_blocks(nkeys) + 1 entries; the row total lands in d_counts[nblocks].
// Split form: count + scan (row total at d_counts[nblocks]), then write -- the write may target mapped pinned host
// memory (hipHostMalloc) directly, so no device->host copy follows.
hipError_t launch_finalize_count(const FParams& F, uint32_t* d_counts, hipStream_t stream);
hipError_t launch_finalize_bucket_pos(const FParams& F, const uint32_t* d_counts, hipStream_t stream);
hipError_t launch_finalize_write(const FParams& F, const uint32_t* d_counts, int64_t* ts, double* val,
                                 uint32_t* gid, uint32_t* glob, hipStream_t stream);
hipError_t launch_finalize(const FParams& F, uint32_t* d_counts, int64_t* ts, double* val, uint32_t* gid,
                           uint32_t* glob, hipStream_t stream);

}  // namespace lk
