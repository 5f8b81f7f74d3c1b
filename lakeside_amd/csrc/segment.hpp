// Host-side segment model and engine dictionaries (no HIP): what the Parquet loader (loader.cpp) builds on the host
// before a segment is uploaded (engine.cpp), so the loader can also run -- and be sanitized -- without a GPU
// (tools/load_check.cpp, `make sanitize`).
#pragma once
#include <atomic>
#include <cstdint>
#include <exception>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <set>
#include <stdexcept>
#include <string>
#include <string_view>
#include <thread>
#include <unordered_map>
#include <utility>
#include <vector>

#include "layout.hpp"

namespace lk {

// fn(0..n-1) on up to `threads` threads (the calling thread among them); the first exception is rethrown after every
// worker has finished.  Not nested: a caller inside a parallel_for passes threads = 1 (the load's thread bound holds).
template <class F>
void parallel_for(size_t n, int threads, F&& fn) {
  const size_t T = std::max<size_t>(1, std::min<size_t>(size_t(threads > 0 ? threads : 1), n));
  if (T <= 1) {
    for (size_t i = 0; i < n; i++) fn(i);
    return;
  }
  std::atomic<size_t> next{0};
  std::exception_ptr err;
  std::mutex err_mu;
  auto work = [&]() {
    for (;;) {
      const size_t i = next.fetch_add(1);
      if (i >= n) return;
      try {
        fn(i);
      } catch (...) {
        std::lock_guard<std::mutex> g(err_mu);
        if (!err) err = std::current_exception();
        next.store(n);
      }
    }
  };
  std::vector<std::thread> pool;
  for (size_t t = 1; t < T; t++) pool.emplace_back(work);
  work();
  for (auto& th : pool) th.join();
  if (err) std::rethrow_exception(err);
}

// Append-only string array in fixed 64K-entry blocks behind a fixed block table: an element never moves, and
// reading an element published before (under the owner's mutex) needs no lock, so results keep reading tag
// strings while loads append to the dictionary.
class StableStrs {
 public:
  static constexpr uint32_t kShift = 16, kBlock = 1u << kShift, kMaxBlocks = 1u << 14;   // 2^30 entries
  size_t size() const { return n_; }
  const std::string& operator[](size_t i) const { return blocks_[i >> kShift][i & (kBlock - 1)]; }
  void push_back(const std::string& s) {
    grow(n_ + 1);
    blocks_[(n_ - 1) >> kShift][(n_ - 1) & (kBlock - 1)] = s;
  }
  // n entries (new ones empty), then `slot` fills them -- distinct slots from several threads at once
  void grow(size_t n) {
    if (n <= n_) return;
    if (((n - 1) >> kShift) >= kMaxBlocks) throw std::length_error("dictionary exceeds 2^30 values");
    for (size_t b = n_ >> kShift; b <= ((n - 1) >> kShift); b++)
      if (!blocks_[b]) blocks_[b].reset(new std::string[kBlock]);
    n_ = n;
  }
  std::string& slot(size_t i) { return blocks_[i >> kShift][i & (kBlock - 1)]; }
  const std::string& back() const { return (*this)[n_ - 1]; }

 private:
  std::unique_ptr<std::unique_ptr<std::string[]>[]> blocks_{new std::unique_ptr<std::string[]>[kMaxBlocks]};
  size_t n_ = 0;
};

// value -> id of one dictionary: open addressing over 64 hash shards (a shard per thread when a large batch of new
// values is indexed), each slot one word -- a 31-bit hash tag and the id -- so a lookup costs one slot read and, on a
// tag match, one string compare against the dictionary's own entry (no node chasing, no key copies).
class IdMap {
 public:
  static constexpr size_t kShards = 64;
  static constexpr uint32_t kNone = UINT32_MAX;
  explicit IdMap(const StableStrs* strs = nullptr) : strs_(strs), m_(kShards) {}
  static uint64_t hash(std::string_view s) {   // FNV-1a 64 + a final mix (the shard takes the low bits)
    uint64_t h = 1469598103934665603ull;
    for (char c : s) h = (h ^ uint8_t(c)) * 1099511628211ull;
    h ^= h >> 33;
    h *= 0xff51afd7ed558ccdull;
    return h ^ (h >> 29);
  }
  static size_t shard_of(uint64_t h) { return size_t(h & (kShards - 1)); }
  uint32_t find(std::string_view s) const { return find_h(s, hash(s)); }
  uint32_t find_h(std::string_view s, uint64_t h) const {
    const Shard& sh = m_[shard_of(h)];
    if (sh.slots.empty()) return kNone;
    const uint64_t tag = tag_of(h), mask = sh.slots.size() - 1;
    for (size_t i = size_t(h >> 6) & mask;; i = (i + 1) & mask) {
      const uint64_t v = sh.slots[i];
      if (!v) return kNone;
      if ((v >> 32) == tag && (*strs_)[uint32_t(v)] == s) return uint32_t(v);
    }
  }
  size_t count(std::string_view s) const { return find(s) != kNone ? 1 : 0; }
  void prefetch(uint64_t h) const {
    const Shard& sh = m_[shard_of(h)];
    if (!sh.slots.empty()) __builtin_prefetch(&sh.slots[size_t(h >> 6) & (sh.slots.size() - 1)]);
  }
  // second stage (the home slot prefetched earlier): the stored string of a tag-matching home slot, which the
  // lookup's compare reads next (short values live inside the string object)
  void prefetch_str(uint64_t h) const {
    const Shard& sh = m_[shard_of(h)];
    if (sh.slots.empty()) return;
    const uint64_t v = sh.slots[size_t(h >> 6) & (sh.slots.size() - 1)];
    if (v && (v >> 32) == tag_of(h)) __builtin_prefetch(&(*strs_)[uint32_t(v)]);
  }
  // id -> its value (*strs)[id] must not be in the map yet
  void emplace(uint32_t id) { emplace_h(id, hash((*strs_)[id])); }
  void emplace_h(uint32_t id, uint64_t h) {
    Shard& sh = m_[shard_of(h)];
    if ((sh.n + 1) * 10 > sh.slots.size() * 7) grow(sh, std::max<size_t>(64, sh.slots.size() * 2));
    insert(sh, id, h);
  }
  // room for n more entries in shard k (a batch of new values indexed by one thread per shard)
  void reserve_shard(size_t k, size_t n) {
    Shard& sh = m_[k];
    size_t cap = std::max<size_t>(64, sh.slots.size());
    while ((sh.n + n) * 10 > cap * 7) cap *= 2;
    if (cap != sh.slots.size()) grow(sh, cap);
  }
  void reserve(size_t n) {
    for (size_t k = 0; k < kShards; k++) reserve_shard(k, n / kShards + 1);
  }
  void swap(IdMap& o) {
    std::swap(strs_, o.strs_);
    m_.swap(o.m_);
  }

 private:
  struct Shard {
    std::vector<uint64_t> slots;   // 0: empty; else (tag | 2^31) << 32 | id
    size_t n = 0;
  };
  static uint64_t tag_of(uint64_t h) { return ((h >> 32) & 0x7fffffffull) | 0x80000000ull; }
  static void insert(Shard& sh, uint32_t id, uint64_t h) {
    const uint64_t mask = sh.slots.size() - 1;
    size_t i = size_t(h >> 6) & mask;
    while (sh.slots[i]) i = (i + 1) & mask;
    sh.slots[i] = (tag_of(h) << 32) | id;
    sh.n++;
  }
  void grow(Shard& sh, size_t cap) {
    std::vector<uint64_t> old;
    old.swap(sh.slots);
    sh.slots.assign(cap, 0);
    sh.n = 0;
    for (uint64_t v : old)
      if (v) insert(sh, uint32_t(v), hash((*strs_)[uint32_t(v)]));
  }
  const StableStrs* strs_;
  std::vector<Shard> m_;
};

// Engine-global dictionary of one column name.  Values get dense ids in first-seen order, at stable
// addresses (result tag values point into it).  Every id counts the chunk-dictionary entries of cached segments
// that map to it (`refs`); when evictions have left as many dead ids as live ones, Engine::maybe_compact renumbers
// the live values densely (old order kept), rewrites the cached segments' remaps and starts a new `vals` block --
// results keep the block they were built from (shared ownership), so the group-dim space of a long-lived worker
// tracks its cached segments, as the worker's bounded disk cache does (WorkerApi.scala:53-64).
struct GlobalDict {
  std::mutex mu;
  std::shared_ptr<StableStrs> vals = std::make_shared<StableStrs>();
  IdMap ids{vals.get()};                   // over `vals` (a compaction swaps both)
  std::vector<uint32_t> refs;              // per id: cached chunk-dictionary entries mapping to it
  size_t live = 0;                         // ids with refs > 0
  uint64_t gen = 0;                        // compactions so far (ids are renumbered by each)
  uint32_t intern(std::string_view s);     // caller holds mu
  // ids of values[i] in order (caller holds mu): known values looked up, new ones interned in first-occurrence order
  // -- the ids equal those of interning the values one by one -- on up to `threads` threads.
  void intern_all(const std::vector<std::string_view>& values, uint32_t* ids_out, int threads);
  // scratch of the parallel path (caller holds mu), kept across loads: a 10M-value column's passes would otherwise
  // fault in ~0.45 GB of fresh pages per segment (hashes, first occurrences, the chunk dictionaries' views)
  std::vector<uint64_t> sc_hash;
  std::vector<uint32_t> sc_first;
  std::vector<std::string_view> sc_views;
  size_t size() const { return vals->size(); }
  const std::string& operator[](size_t i) const { return (*vals)[i]; }
};

struct HostCol {
  std::string name;
  int ptype = -1;
  bool nullable = false;
  bool is_string = false;
  bool unsupported = false;
  bool any_nulls = false;
  // page summaries (load time), so a query's lean-tile test costs O(1) per column instead of a walk over its pages:
  bool pages_lean_name = false;           // every page: dictionary indices, chunk dictionary <= 64 values, 1..6 bits
  bool pages_lean_late = false;           // every page: dictionary indices of <= 32 bits
  uint64_t compressed_bytes = 0;          // Σ ColumnMetaData.total_compressed_size (algorithmic bytes)
  // DOUBLE / INT64 columns with PLAIN pages: the largest magnitude when every value is an integer, else -1 (a
  // non-integral or non-finite value, another encoding, another type) -- QParams::exact_sum
  double int_abs_max = -1.0;
  std::vector<PageDesc> pages;            // host copy (planner reads dict sizes / null flags)
  std::vector<RunDesc> runs;              // load-time only
  std::vector<TileCol> tcols;             // load-time only
  std::vector<uint32_t> remap;            // load-time only
  size_t nremap = 0;                      // entries of d_remap counted in the column dictionary's refs
  PageDesc* d_pages = nullptr;
  RunDesc* d_runs = nullptr;
  TileCol* d_tcols = nullptr;
  uint32_t* d_remap = nullptr;
};

// The host part of a cached segment (the loader's output; engine.hpp's Segment adds the device copies).
struct SegmentData {
  std::string key;
  int64_t num_rows = 0;
  std::vector<int64_t> rg_rows;
  std::vector<HostCol> cols;                     // loadable columns
  std::set<std::string> all_columns;             // every column of the file (DESCRIBE, Commons.scala:214-221)
  // columns of the file the engine does not decode (nested / repeated, INT96 / FIXED_LEN_BYTE_ARRAY, an encoding or
  // codec outside the implemented set) -> why; a query referencing one fails with LK_ERR_UNSUPPORTED
  std::map<std::string, std::string> unloaded;
  double load_host_ms = 0, load_ms = 0;          // build_segment: host walk / total (stats)
  std::vector<std::pair<std::string, int>> schema;   // (name, Parquet physical type) in file order (SELECT *)
  std::unordered_map<std::string, int> by_name;
  std::vector<TileDesc> tiles;
  size_t data_bytes = 0;                         // the page-stream area (device: d_data)
  int col_index(const std::string& name) const;
};

}  // namespace lk
