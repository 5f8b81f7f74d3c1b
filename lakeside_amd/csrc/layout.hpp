// Data layout shared by the host engine and the HIP kernels.
//
// HBM-resident segment (loaded once, reused by every query; the worker's disk cache becomes an HBM cache):
//   bytes    : the sealed Parquet file, verbatim (page headers included, never read by the GPU)
//   pages    : one PageDesc per data page of every column chunk (where its value / def-level streams start)
//   runs     : RunDesc per run of every hybrid RLE/bit-packed stream (dictionary indices, def levels)
//   tiles    : TileDesc per tile = a row range inside one row group and inside one page of every column,
//              small enough that each column's runs over the tile fit the kernel's LDS staging (RUN_CAP)
//   tcols    : TileCol per (column, tile): the page and the run windows of that column over the tile
//   remap    : per dictionary-encoded column chunk, local dictionary index -> engine-global value id
//
// Per query the host uploads one QSeg per segment (which columns the query reads, the glob it belongs to,
// forced-false leaves) and, per string column, a table global id -> (leaf bits << 24 | group-dim id).
#pragma once
#include <cstdint>

namespace lk {

// Query-shape caps (VERDICT r5 missing #2: r05's 6 / 16 / 48 sent a DataExpr with 3 groupBys and 3 filter tags to
// DuckDB).  Leaf outcomes travel as 32-bit T / F masks, so 32 leaves is the ceiling of this representation; the fused
// kernels are instantiated per string-column count up to MAXSTR (scan_inst.hpp).
constexpr int MAXQCOL = 12;     // query columns: 0 = timestamp, 1 = aggregated value, 2.. = string / numeric columns
constexpr int MAXSTR = 8;       // string columns per query (name + filter keys + groupBys)
constexpr int MAXLEAF = 32;     // filter leaves
constexpr int MAXPROG = 96;     // postfix filter program length (32 leaves, 31 binary nodes, NOTs)
constexpr int LEAF_BITS = 8;    // leaf bits per string column in the packed lookup value
constexpr uint32_t DIM_MASK = 0x00ffffffu;   // group-dim id bits of the packed lookup value
constexpr uint32_t TILE_ROWS = 65536;        // max rows per tile
constexpr uint32_t RUN_CAP = 128;            // max runs of one stream of one column inside a tile

enum PageKind : uint8_t { PAGE_PLAIN64 = 1, PAGE_DICT = 2, PAGE_PLAIN32 = 3, PAGE_BOOL = 4 };   // PLAIN32: INT32 / FLOAT

struct PageDesc {           // 48 B
  uint64_t vals;            // byte offset (from segment base) of the value stream: PLAIN data, or dictionary
                            //   indices' hybrid data (after the bit-width byte)
  uint64_t defs;            // byte offset of the definition-level hybrid stream (0 if the column is REQUIRED)
  uint32_t first_row;       // first row of the page within its row group
  uint32_t nrows;
  uint32_t nvals;           // non-null values stored in the page
  uint32_t remap;           // offset (elements) of the chunk's dictionary remap in the segment remap array
  uint32_t dict_n;          // dictionary size of the chunk
  uint32_t vals_len;        // bytes of the value stream
  uint32_t defs_len;        // bytes of the def-level stream
  uint8_t bw;               // dictionary index bit width
  uint8_t kind;             // PageKind
  uint8_t nullable;         // has a def-level stream
  uint8_t has_nulls;        // at least one NULL row in this page
};

struct RunDesc {            // 16 B; one run of a hybrid RLE/bit-packed stream
  uint32_t start;           // first value index (value stream) / row (def stream), relative to the page
  uint32_t off_lit;         // bit 31: literal (bit-packed) run; bits 0..30: byte offset from stream start
  uint32_t value;           // RLE run: the repeated value
  uint32_t count;           // values covered
};

struct TileDesc {           // 32 B
  uint32_t rg;              // row group
  uint32_t row0;            // first row (within the row group)
  uint32_t nrows;
  uint32_t pad;             // TILE_TS_SORTED
  int64_t ts_min;           // zone map of the timestamp column over the tile (INT64_MAX/MIN if no value)
  int64_t ts_max;
};

// TileDesc::pad bit: the tile's timestamps (PLAIN INT64, no NULL) never decrease from row to row
constexpr uint32_t TILE_TS_SORTED = 1u;

struct TileCol {            // 64 B: everything the kernel needs about one column over one tile
  uint64_t vals;            // byte offset (segment base) of the page's value stream
  uint64_t defs;            // byte offset of the page's def-level stream
  uint32_t vals_len;
  uint32_t defs_len;
  uint32_t row_in_page;     // first row of the tile within its page
  uint32_t vbase;           // value index (within the page) of the tile's first non-null row
  uint32_t run_lo;          // first value-stream run overlapping the tile (index into the run array)
  uint32_t nruns;
  uint32_t drun_lo;         // first def-stream run overlapping the tile
  uint32_t ndruns;
  uint32_t remap;           // offset of the chunk's dictionary remap
  uint32_t dict_n;          // dictionary size of the chunk
  uint8_t bw;               // dictionary index bit width
  uint8_t kind;             // PageKind
  uint8_t has_nulls;        // the page has at least one NULL
  uint8_t pad0;
  uint32_t page;            // index into the segment's page array (host bookkeeping)
};
static_assert(sizeof(TileCol) == 64, "TileCol layout");

struct QCol {               // one query column in one segment
  const PageDesc* pages;
  const RunDesc* runs;
  const TileCol* tcols;     // per tile
  const uint32_t* remap;
  uint32_t present;         // 0: column absent from this segment (all NULL)
  uint32_t pad;             // bits 0..7: Parquet physical type; value column: VCONV_* bits
};
// Value column of a segment whose glob unifies it to FLOAT while the file stores integers (union_by_name): the value
// is cast to FLOAT (round to nearest) before it is aggregated.
constexpr uint32_t VCONV_VIA_FLOAT = 0x100u;

struct QSeg {
  const uint8_t* base;
  const TileDesc* tiles;
  uint32_t tile_begin;      // prefix sum of tiles over the query's segments (stats only)
  uint32_t ntiles;          // grid.x covers the largest segment; blocks past ntiles exit
  uint32_t glob_slot;       // glob index in the cell space (0 when globs are merged in the table)
  uint32_t leaf_false;      // leaves compiled to literal `false` for this segment's glob (BaseExpr.scala:462)
  int64_t win_lo;           // glob window [min startTs, max endTs) (Commons.scala:225-226)
  int64_t win_hi;
  QCol cols[MAXQCOL];
};

enum Agg : int { AGG_SUM = 0, AGG_MIN = 1, AGG_MAX = 2, AGG_COUNT = 3 };
enum Op : uint8_t { OP_AND = 0x80, OP_OR = 0x81, OP_NOT = 0x82, OP_TRUE = 0x83 };   // < 0x80: push leaf

constexpr int TT_MAX_LEAVES = 6;   // filters with <= 6 leaves run as a truth table (4^6 bits)
constexpr int LK_NSTAMP = 8;       // diagnostics: per-block s_memtime section totals (scan_kernel.hpp)

struct StrParam {           // per string column of a query (device array; read inside the column loop)
  const uint32_t* strtab;   // global id -> (leaf bits << 24) | dim id; null: identity dim, no leaves
  uint32_t dim_null;        // dim id of NULL / absent
  uint32_t dim_stride;      // 0: not a group dimension
  uint32_t lbase;           // first leaf index of this column
  uint32_t lmask;           // leaf-index mask of its leaves
  uint32_t hmask;           // its `has`/`exists` leaves
  uint32_t pad;
};

constexpr int VLEAF_MAX = 5;
struct VLeaf {                       // value in (lo, hi) with inclusive ends per flag; NaN (greatest) passes iff nan_pass
  double lo, hi;
  uint32_t lo_incl, hi_incl, nan_pass, pad;
};
struct QParams {
  const QSeg* segs;
  uint32_t nsegs;
  uint32_t total_tiles;
  uint32_t max_tiles;       // grid.x
  const uint32_t* truth;    // filter truth table: bit (T | F << nleaves) = row passes; null: interpret prog
  // late materialization (truth tables only): filter = early AND late; string column s with bit s of late_mask
  // is decoded only for rows where the early table passes (tiles where no late column / timestamp is NULL)
  const uint32_t* truth_early;
  const uint32_t* truth_late;
  uint32_t late_mask;
  int32_t fast_div;         // 1: (ts - bucket_base) fits 32 bits for every window -> 32-bit bucket division
  double inv_step;          // 1.0 / step
  const StrParam* strp;     // [nstr]
  uint32_t nstr;            // string columns (query cols 2 .. 2+nstr)
  uint32_t nleaves;
  uint32_t nprog;
  int32_t metrics;          // 1: bucket = raw timestamp (BaseExpr.scala:391); 0: ts - ts % step (163-165)
  int64_t step;
  int64_t bucket_base;      // step-aligned origin of bucket 0
  uint64_t nbuckets;
  uint64_t ngroups;
  uint64_t ncells;
  uint8_t prog[MAXPROG];
  // aggregation table (structure of arrays, ncells each)
  unsigned long long* rows;         // rows that passed the filter (cell existence)
  unsigned long long* cnt;          // non-NULL values
  double* hi;                       // sum = hi + lo (compensated)
  double* lo;
  unsigned long long* ext;          // min/max as order-preserving u64
  // hash mode (high cardinality, SURVEY §2.2 K4 spill): the SoA arrays above are slots of an open-addressing
  // table whose slot keys are `hkeys` (EMPTY = ~0); null: dense mode (array index = cell key)
  unsigned long long* hkeys;
  unsigned long long hmask;         // slots - 1 (a power of two)
  // DDSketch mode (percentile aggregations, COUNT instantiation only): the cell key gains the value's DDSketch bin,
  // key = cell * DD_NBINS + dd_bin(value) (a NULL value reads as 0.0, the JDBC getDouble contract); rows per key
  uint32_t sketch;
  double dd_mult;                   // 1 / ln(gamma) of the index mapping
  double dd_min;                    // smallest indexable magnitude (smaller values go to the zero bin)
  double dd_max;                    // largest trackable magnitude (beyond: FLAG_SKETCH_RANGE)
  uint32_t lean_split;              // 1: scan_lean takes the lean tiles (lean_tile), scan_tiles skips them;
                                    // 2: every tile is lean (scan_tiles is not launched)
  uint32_t lean;                    // LEAN_* bits: table fields the scan leaves to the fix-up pass (fewer atomics)
  uint32_t* flags;                  // error / diagnostic flags
  uint32_t ablate;                  // diagnostics only (env LK_ABLATE): 1 skip phase 2, 2 skip tag decode,
                                    // 4 no global-table atomics; scan_lean: 0x100..0x800 plan-byte categories left
                                    // out, 0x10000 no row listed, 0x20000 listed rows dropped unprocessed, 0x40000
                                    // listed rows loaded but not accumulated, 0x80000 the tile prologue alone
  unsigned long long* stamps;       // diagnostics only (env LK_STAMPS): per block s_memtime phase totals
  // Plan bytes (the roofline numerator): bytes the late-materialized plan must read from HBM, counted
  // by the kernel: tile metadata + staged runs + dictionary lookups, every fully decoded stream of a tile, and the
  // distinct 128-B lines touched by the per-row gathers (timestamps, values, late columns).
  unsigned long long* plan_bytes;
  // scan_lean (lean_kernel.hpp): the direct table holds up to dir_span buckets of ngroups cells, dir_planes u64 planes per
  // cell (0: the LDS hash table instead)
  uint32_t dir_span;
  uint32_t dir_planes;
  uint32_t dir_rep;                  // replicas per direct-table cell (1, 2 or 4)
  uint32_t rows_only;                // COUNT(*) (tag queries): no value column bound; lean tiles take none
  uint32_t late_chunk;               // scan_lean NL > 0: late columns decoded per 16-row chunk in the main loop (the
                                     // list then carries each row's group term; lean_kernel.hpp)
  uint32_t spec_gather;              // scan_lean NL > 0 with a late filter: a listed row's timestamp / value loads go
                                     // out with its late-column loads, before the late filter decides (lean_kernel.hpp)
  // SUM over integral values (every segment's value column: integers of magnitude <= M, load-time summary) whose
  // rows x M < 2^53: every partial sum is exact in any order, so the TwoSum compensation (and the old value a
  // returning atomic fetches for it) is dropped -- adds are fire-and-forget; results are identical
  uint32_t exact_sum;
  // group spaces far beyond the tile's LDS hash table (C5's 10M container ids): cells go straight to the global table
  uint32_t global_cells;
  // scan_lean split tiles (TILE_TS_SORTED tiles spanning a few buckets: rows bucketed by index, no timestamp gather)
  uint32_t split_ok;
  // Numeric comparison leaves on the value column (`value > 1.5`, BaseExpr.scala:488-498) in the fused kernel: a row
  // whose string conjuncts pass is kept iff vtab bit (its leaves' outcomes, bit k = leaf k) is set -- the numeric
  // conjuncts' value.  scan_lean tiles hold no NULL value, so no leaf is UNKNOWN there.
  uint32_t nvl;
  uint32_t vtab;
  VLeaf vl[VLEAF_MAX];
};
// scan_lean's direct table: LDS words by late-column count NL (the hash table's 8 KB for NL >= 1, so the kernels keep
// their occupancy), at most LEAN_DIR_MAXSPAN buckets
constexpr uint32_t LEAN_DIR_WORDS0 = 1536;
constexpr uint32_t LEAN_DIR_WORDS1 = 1024;
// two late columns (C3's shape: a 4-wave kernel, 4 workgroups per CU): 18 KB, one bucket of a 2,000-group space at
// one plane (MIN / MAX) -- its cells otherwise overflow the 256-slot LDS hash table into device atomics
constexpr uint32_t LEAN_DIR_WORDS2 = 2304;
constexpr uint32_t LEAN_DIR_MAXSPAN = 8;
constexpr uint32_t lean_dir_words(uint32_t nl) { return nl == 0 ? LEAN_DIR_WORDS0 : (nl == 1 ? LEAN_DIR_WORDS1 : LEAN_DIR_WORDS2); }

enum Flag : uint32_t {
  FLAG_METRICS_UNALIGNED = 1u, FLAG_CELL_RANGE = 2u, FLAG_HASH_FULL = 4u, FLAG_SKETCH_RANGE = 8u,
  FLAG_HASH_GROW = 16u,  // host only: this rank's hash table was full below its bound (agreed re-run)
  FLAG_MIN_NAN = 32u     // MIN over a NaN value (eval.cpp: merged tables re-run with per-glob cells)
};
constexpr unsigned long long NAN_ORDER = 0xfff8000000000000ull;   // dbl_order(NaN)
// NaN re-ordered below -inf (0: no dbl_order value) where MIN merges rows with math.min semantics (rekey_minmax)
constexpr unsigned long long MIN_NAN_ORDER = 0ull;

// DDSketch bins (sketches-java LogarithmicMapping, relative accuracy 0.01): bin 0 = zero, 1 + DD_BIAS + i = positive
// index i, 1 + DD_HALF + DD_BIAS + i = negative index i (|i| < DD_BIAS covers every finite double).
constexpr int32_t DD_BIAS = 40000;
constexpr uint32_t DD_HALF = 2 * DD_BIAS;
constexpr uint32_t DD_NBINS = 1 + 2 * DD_HALF;
constexpr uint32_t HASH_MAX_PROBE = 4096;
// Lean tables: with no NULL value in the query's value column, a cell's non-NULL count equals its row count
// (LEAN_NO_CNT: `cnt` is not accumulated), and for min/max a cell exists iff its extreme left the identity
// (LEAN_NO_ROWS: neither `rows` nor `cnt` is accumulated).  fixup_table restores both after the scan, so every
// later stage (merge, finalize) reads an ordinary table.  Each dropped field is one memory-side atomic per flush.
constexpr uint32_t LEAN_NO_CNT = 1u, LEAN_NO_ROWS = 2u;
// LEAN_SUM_EXISTS (dense SUM tables, no NULL value): `hi` starts at -0.0, which no add can produce again (partials
// are normalized by + 0.0 -- exact for DuckDB's SUM, whose running value starts at +0.0 and so never is -0.0), so
// "hi != -0.0" says the cell exists and `rows` needs no atomic either: one scattered atomic per flushed cell instead
// of two or three (fixup_table restores rows / cnt and hi = +0.0 of empty cells).
constexpr uint32_t LEAN_SUM_EXISTS = 4u;
// LEAN_NO_DENSE_DIRECT (env LK_NO_DENSE_DIRECT, A/B only): dense blocks accumulate through the register cell too
constexpr uint32_t LEAN_NO_DENSE_DIRECT = 8u;
constexpr unsigned long long NEG_ZERO_BITS = 0x8000000000000000ull;

}  // namespace lk
