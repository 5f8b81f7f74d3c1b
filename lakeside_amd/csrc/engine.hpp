// Engine state shared by engine.cpp (segment cache), eval.cpp (query evaluation), comm.cpp (RCCL).
#pragma once
#include <atomic>
#include <hip/hip_runtime.h>

#include <condition_variable>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <set>
#include <shared_mutex>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "ddsketch.hpp"
#include "hll.hpp"
#include "layout.hpp"
#include "plan.hpp"
#include "segment.hpp"

namespace lk {

void set_error(const std::string& m);

struct Segment : SegmentData {
  TileDesc* d_tiles = nullptr;
  uint8_t* d_data = nullptr;                     // page streams (def levels / values), 16-B aligned
  void* d_meta = nullptr;
  size_t meta_bytes = 0;
  bool from_put = false;                         // registered by lk_segment_put (its key is not a file path)
  std::atomic<uint64_t> last_use{0};             // LRU clock value of the last lookup (cache eviction)
  struct Engine* engine = nullptr;               // whose dictionaries its remaps reference (refs released at ~Segment)
  ~Segment();
};

struct Workspace {
  void* p = nullptr;
  size_t cap = 0;
};

// Device resources of one evaluation in flight: its own stream, timing events, device workspaces and pinned
// staging.  The engine keeps a small pool, so calls from several dispatcher threads run concurrently on their own
// streams (the reference keeps up to 8 glob queries in flight, Commons.scala:371-372).
struct CallCtx {
  int device = 0;
  hipStream_t stream = nullptr;
  hipEvent_t ev_scan0 = nullptr, ev_scan1 = nullptr;
  hipEvent_t ev_rows = nullptr;   // large results: bucket_pos written (host expands timestamps meanwhile)
  std::map<std::string, Workspace> ws;
  void* pinned = nullptr;
  size_t pinned_cap = 0;
  void* comm_pin = nullptr;   // distributed calls: pinned slots of the small all-gathers (comm.cpp, kCommPinBytes)
  // Distributed calls: a rank-local failure met after a collective step, held until the next agreement point (an
  // all-gather every rank takes) so that every rank fails together instead of leaving peers inside a collective.
  int pend_code = 0;
  std::string pend_msg;
  explicit CallCtx(int dev);
  ~CallCtx();
  CallCtx(const CallCtx&) = delete;
  CallCtx& operator=(const CallCtx&) = delete;
  void* workspace(const std::string& name, size_t bytes);
  void* pinned_buf(size_t bytes);
};

struct Comm;   // comm.cpp

// A column's engine dictionary (its first n values) keyed by value hash: every value's 128-bit MurmurHash3 key,
// sorted, and a fingerprint of the sorted keys.  Ranks agree on a distributed group-dim space through these keys
// (DimUnion) instead of exchanging and sorting strings; ranks holding the same value set compare fingerprints only.
struct Key128 {
  uint64_t hi = 0, lo = 0;
  bool operator<(const Key128& o) const { return hi != o.hi ? hi < o.hi : lo < o.lo; }
  bool operator==(const Key128& o) const { return hi == o.hi && lo == o.lo; }
};
struct DictOrder {
  size_t n = 0;
  std::vector<Key128> keys;     // sorted (position = dim id of the value set alone)
  std::vector<uint32_t> perm;   // position -> engine global id
  std::vector<uint32_t> rank;   // engine global id -> position
  uint64_t fp[2] = {0, 0};
};

// The agreed group-dim space of an unrestricted dimension over the ranks of a distributed evaluation: the sorted
// union U of every rank's value keys (dim id = position in U; U's size = NULL's dim id).  Built collectively once
// per set of rank dictionaries and cached (agree_key = every rank's (n, fingerprint)), so a steady-state query
// agrees with one small all-gather.
struct DimUnion {
  std::string agree_key;
  size_t dict_n = 0;
  uint32_t size = 0;                          // |U|
  std::shared_ptr<const std::vector<uint32_t>> dim_of_gid;   // this rank: engine global id -> dim id
  std::shared_ptr<std::vector<const char*>> text;            // dim id -> value (nullptr: null-like or unknown here);
                                                             // [size] = nullptr (NULL); complete on rank 0
  std::deque<std::string> owned;              // values this rank received from the ranks that hold them
  std::shared_ptr<const DictOrder> order;
  std::shared_ptr<StableStrs> strs;           // the dictionary block `text` points into
  uint32_t* d_dim_of_gid = nullptr;           // device copy (the scan's lookup table for this dim)
  int device = 0;
  ~DimUnion();
};

// Process-wide pool of pinned host blocks for result columns (engine.cpp).
struct HostBlock {
  void* p = nullptr;
  size_t cap = 0;
  bool pinned = false;
};
HostBlock pinned_acquire(size_t bytes);
// A process-wide read-only block of at least `bytes` zero bytes (calloc: untouched pages map the zero page).
std::shared_ptr<void> zero_block(size_t bytes);
void pinned_release(HostBlock b);

// Per (column, leaf) cache of leaf outcomes over the column's engine dictionary: bit j of byte i = leaf j of the
// column on dictionary value i.  Extended incrementally as the dictionary grows, so a regex over a 10M-value
// dictionary is matched once per value, not once per value per query.
struct LeafBits {
  std::mutex mu;
  std::vector<uint8_t> hit;   // one byte per evaluated dictionary value
};

struct Engine {
  int device = 0;
  size_t max_calls = 4;                          // evaluation contexts (streams) in flight
  std::mutex ctx_mu;
  std::condition_variable ctx_cv;
  std::vector<std::unique_ptr<CallCtx>> ctx_free;
  size_t ctx_made = 0;
  std::mutex comm_mu;                            // distributed calls: collectives in one order on every rank
  std::mutex dev_mu;                             // segment upload
  std::mutex cache_mu;
  std::unordered_map<std::string, std::shared_ptr<Segment>> cache;
  size_t cache_bytes = 0;
  // HBM budget of the segment cache (lk_engine_create {"hbm_budget_bytes": N}; 0 = none): inserting past it evicts
  // the least recently used segments, as the worker's weighted Caffeine cache does (WorkerApi.scala:53-64).  A
  // segment an evaluation still holds is freed when that evaluation drops it.
  size_t hbm_budget = 0;
  std::atomic<uint64_t> use_clock{0};
  size_t evictions = 0;
  // Keys registered with lk_segment_put that the LRU policy evicted since: an evaluation naming one fails with
  // LK_ERR_EVICTED (the caller re-puts it) instead of treating the key as a missing file.  Cleared per key
  // by a re-put or lk_segment_evict; bounded.
  std::unordered_set<std::string> evicted_puts;
  // Segment ingest: host threads of build_segment (lk_engine_create {"load_threads": N}; 0 = OMP_NUM_THREADS or the
  // hardware threads, at most 16) and the pinned staging area its upload goes through (under dev_mu).
  int load_threads = 0;
  int load_thread_count() const;
  // Result-path host work (large results' rows expanded on the host while their values cross the link): threads
  // spawned per call, the job's whole thread share.  A persistent pool measured slower (C5 eval 2.66 vs 1.94 ms,
  // profiles/r06_ab_c5_pool.json / _spawned_threads.json) and was removed.
  template <class F>
  void host_parallel(size_t n, F&& fn) {
    parallel_for(n, load_thread_count(), fn);
  }
  void* load_pinned = nullptr;
  size_t load_pinned_cap = 0;
  hipStream_t load_stream = nullptr;
  double load_host_ms_total = 0, load_ms_total = 0;   // cumulative (lk_engine_stats)
  // evict LRU segments (never `keep`) until cache_bytes + extra <= budget; caller holds cache_mu
  size_t evict_lru_locked(size_t target_bytes, const std::string& keep, std::vector<std::shared_ptr<Segment>>* out);
  std::mutex dict_mu;
  std::unordered_map<std::string, std::unique_ptr<GlobalDict>> dicts;
  // Dictionary generations: loads and evaluations hold gen_mu shared (at the C ABI); a compaction holds it exclusive,
  // so no evaluation or load sees ids change under it.
  std::shared_mutex gen_mu;
  size_t compact_min_dead = 1024;                // compact a column once dead ids >= max(live ids, this)
  size_t compactions = 0;
  void maybe_compact();                          // caller holds no engine lock
  void compact_locked(const std::string& col);   // caller holds gen_mu exclusive
  void dict_ref(const std::string& col, const uint32_t* ids, size_t n, int delta);
  std::mutex leaf_mu;
  std::map<std::string, std::shared_ptr<LeafBits>> leaf_cache;   // key: column \x1f op \x1f values
  std::shared_ptr<LeafBits> leaf_bits(const std::string& key);
  Comm* comm = nullptr;                          // set once by lk_comm_init* (under comm_init_mu), never replaced
  std::mutex comm_init_mu;                       //   guards the set-once check and comm_desc
  std::string comm_desc = "null";                //   comm->describe() taken at init: lk_engine_stats reads this copy
  std::mutex order_mu;
  std::unordered_map<std::string, std::shared_ptr<const DictOrder>> orders;   // per column, latest size
  std::shared_ptr<const DictOrder> dict_order(const std::string& col, size_t n);
  // Bulk tag export (lk_result_tag_dictionary): the column's first n dictionary values as C strings (nullptr for the
  // null-like "" / "null", which drop the tag) plus a trailing nullptr (the dim id of NULL).  Cached per column and
  // rebuilt (prefix copied) only when the dictionary has grown, so in steady state a result's dictionary costs O(1).
  std::mutex ptrs_mu;
  struct PtrTable {
    std::shared_ptr<StableStrs> strs;              // the dictionary block the pointers point into
    std::shared_ptr<const std::vector<const char*>> tab;
  };
  std::unordered_map<std::string, PtrTable> ptrs;
  std::shared_ptr<const std::vector<const char*>> dict_ptrs(const std::string& col, size_t n,
                                                           const std::shared_ptr<StableStrs>& strs);
  // Parsed requests by their JSON text (a dashboard re-issues the same pushdown every refresh): parsing a 64-segment
  // request is a third of the host planning.  Bounded; a parsed Request is immutable.
  std::mutex parsed_mu;
  std::unordered_map<std::string, std::shared_ptr<const Request>> parsed;
  std::shared_ptr<const Request> parse_cached(const std::string& json);
  // distributed group-dim unions, latest per column (DimUnion); used under comm_mu
  std::unordered_map<std::string, std::shared_ptr<DimUnion>> unions;

  // Lifetime token: results hold a weak reference, so a result read after its engine was destroyed builds its own
  // pointer tables instead of dereferencing the engine.
  std::shared_ptr<const char> life = std::make_shared<const char>('\0');
  explicit Engine(int dev);
  ~Engine();
  GlobalDict& dict(const std::string& col);
  std::shared_ptr<Segment> build_segment(const std::string& key, const uint8_t* data, size_t size);
  int put_segment(const std::string& key, const uint8_t* data, size_t size, bool from_put = true);
  std::shared_ptr<Segment> get_segment(const std::string& key, bool load_on_miss);
  std::unique_ptr<CallCtx> acquire_ctx();
  void release_ctx(std::unique_ptr<CallCtx> c);
  void comm_destroy();
};

// RAII: a call context for the duration of one evaluation.
class CtxLease {
 public:
  explicit CtxLease(Engine& e) : e_(e), c_(e.acquire_ctx()) {}
  ~CtxLease() { e_.release_ctx(std::move(c_)); }
  CallCtx& operator*() { return *c_; }
  CallCtx* operator->() { return c_.get(); }

 private:
  Engine& e_;
  std::unique_ptr<CallCtx> c_;
};

}  // namespace lk

struct lk_engine {
  std::unique_ptr<lk::Engine> e;
};

// Rows of one evaluation, columnar: timestamps, values, glob and group id per row.  Tag strings are decoded
// from the group id on demand (lk_result_tag_value), so emitting millions of rows costs no per-row host work.
// Tag values point into the engine's dictionaries: free results before destroying their engine.
struct lk_result {
  size_t nrows = 0;
  int64_t* ts = nullptr;                         // columns carved out of one pinned host block (pinned_acquire):
  double* val = nullptr;                         //   device-to-host copies run at full link rate and a freed
  uint32_t* glob = nullptr;                      //   result hands the block to the next one
  uint32_t* gid = nullptr;                       // group id: Σ dim id × stride over the group dims (< 2^32)
  lk::HostBlock blk;
  std::vector<std::string> tag_names;            // "name", groupBys, then queryTags keys
  struct TagCol {                                // a "name" / groupBy tag column
    unsigned long long stride = 1, ndim = 1;
    uint32_t dim_null = 0;                       // dim id of NULL: tag absent
    std::vector<const char*> local;              // dim id -> string (nullptr: absent); empty: read `dict`
    std::shared_ptr<const std::vector<const char*>> shared;   // distributed union dim: dim id -> string (DimUnion)
    std::shared_ptr<const void> keep;            // keeps the strings `shared` points to alive
    const lk::StableStrs* dict = nullptr;        // the engine dictionary (dim id = global id, or perm[dim id])
    std::shared_ptr<lk::StableStrs> dict_keep;   // ... kept alive across dictionary compactions
    std::shared_ptr<const lk::DictOrder> order;  // distributed dims agreed by fingerprint: dim id -> global id
    bool hidden = false;                         // tag name dropped by NoisyTagsDropper (tag queries)
    const char* null_value = nullptr;            // the tag's value for dim_null (nullptr: tag dropped)
    lk::Engine* engine = nullptr;                // bulk export of an engine-dictionary column: its name and the
    std::string col;                             //   dictionary size of this evaluation
    std::weak_ptr<const char> engine_life;       // expires with the engine: the export then builds its own table
    size_t dict_n = 0;
  };
  std::vector<TagCol> tcols;
  // Bulk tag export (lk_result_tag_dictionary): per tag column, dim id -> string (nullptr: tag absent), built on first
  // use (engine-dictionary columns share the engine's cached table).
  mutable std::mutex bulk_mu;
  mutable std::vector<std::shared_ptr<const std::vector<const char*>>> bulk;
  const std::vector<const char*>* tag_dictionary(size_t c) const;
  // Commons.scala:450-452: a row whose own tags are all absent takes its glob head's queryTags
  std::vector<std::vector<std::pair<size_t, const char*>>> qt_of_glob;   // (tag column, value) per glob
  bool per_glob = false;
  int count_col = -1;                            // tag queries: the "count" tag column
  std::vector<std::string> count_str;            //   and its per-row value (COUNT(*) as text)
  std::deque<std::string> owned;                 // strings not owned by a dictionary
  std::vector<std::shared_ptr<const void>> keep; // dictionary blocks tag pointers point into
  std::string stats;
  std::vector<std::string> sketches;             // percentile rows: the serialized DDSketch of each row
  // internal (evaluate_mixed_steps): the rows' sketches as objects, so rows of globs with different steps can be
  // merged per (timestamp, tags) as query-api merges sketches (TimeGroupedSketchAggregator.scala:34-43)
  bool keep_sketches = false;
  std::vector<lk::dd::Sketch> dd_objs;           // percentile rows
  std::vector<lk::hll::Sketch> hll_objs;         // cardinality rows

  lk_result() = default;
  lk_result(const lk_result&) = delete;
  lk_result& operator=(const lk_result&) = delete;
  ~lk_result() { lk::pinned_release(blk); }
  // with_glob = false (merged rows: every glob index is 0): the glob column is a shared read-only block of
  // zeros, so the device writes 20 instead of 24 bytes per row over the host link.
  void alloc_rows(size_t n, bool with_glob = true) {
    lk::pinned_release(blk);   // a re-run evaluation (metrics / MIN re-runs) allocates again
    blk = lk::HostBlock{};
    blk = lk::pinned_acquire(n * (with_glob ? 24 : 20) + 64);
    nrows = n;
    auto* b = static_cast<uint8_t*>(blk.p);
    ts = reinterpret_cast<int64_t*>(b);
    val = reinterpret_cast<double*>(b + n * 8);
    gid = reinterpret_cast<uint32_t*>(b + n * 16);
    if (with_glob) {
      glob = reinterpret_cast<uint32_t*>(b + n * 20);
    } else {
      zeros = lk::zero_block(n * 4);
      glob = static_cast<uint32_t*>(zeros.get());
    }
  }
  std::shared_ptr<void> zeros;                   // glob column of merged rows (see alloc_rows)
  std::shared_ptr<void> shared_block;            // rows adopted from a shared host block (adopt_rows)
  // Merged rows another party wrote into a host block laid out [ts | value | group id] x n (the distributed key-range
  // emit, comm_emit_begin): the result reads them in place and holds `lease` until it is freed.
  void adopt_rows(void* host, size_t n, std::shared_ptr<void> lease) {
    auto* b = static_cast<uint8_t*>(host);
    nrows = n;
    ts = reinterpret_cast<int64_t*>(b);
    val = reinterpret_cast<double*>(b + n * 8);
    gid = reinterpret_cast<uint32_t*>(b + n * 16);
    zeros = lk::zero_block(n * 4);
    glob = static_cast<uint32_t*>(zeros.get());
    shared_block = std::move(lease);
  }

  // exemplar rows: every row's tag strings, materialized ([row][tag column]; nullptr: tag absent)
  bool exemplar = false;
  std::vector<const char*> ex_tags;

  const char* tag(size_t row, size_t col) const {
    if (exemplar) return ex_tags[row * tag_names.size() + col];
    if (int(col) == count_col) return count_str[row].c_str();
    if (col < tcols.size()) return own_tag(row, col);
    for (size_t c = 0; c < tcols.size(); c++)
      if (own_tag(row, c)) return nullptr;
    for (auto& kv : qt_of_glob[per_glob ? glob[row] : 0])
      if (kv.first == col) return kv.second;
    return nullptr;
  }
  // S15 (Commons.scala:433): NULL, "null" and "" drop the tag
  const char* own_tag(size_t row, size_t c) const {
    const TagCol& t = tcols[c];
    if (t.hidden) return nullptr;
    const uint32_t d = uint32_t((gid[row] / t.stride) % t.ndim);
    if (d == t.dim_null) return t.null_value;
    if (t.shared) return (*t.shared)[d];
    if (!t.local.empty()) return t.local[d];
    const std::string& s = (*t.dict)[t.order ? t.order->perm[d] : d];
    return (s.empty() || s == "null") ? nullptr : s.c_str();
  }
};
