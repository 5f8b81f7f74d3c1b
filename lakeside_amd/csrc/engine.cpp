// lakeside_gpu engine: HBM segment cache, engine-global dictionaries, plan compile, evaluation, results.
//
// Replaces, for the hot query shape, the worker evaluator's DuckDB seam:
//   Commons.evaluatePushDownRequest / toGlobResultSet / resultSetToSource / toDataPoint
//   (core/src/main/scala/com/cardinal/utils/Commons.scala:200-462)
// and the query-api cross-glob merge (core/src/main/scala/com/cardinal/eval/TimeGroupedSketchAggregator.scala:57-177).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <climits>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <exception>
#include <string_view>
#include <thread>
#include <deque>
#include <fstream>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/lakeside_gpu.h"
#include "engine.hpp"
#include "hll.hpp"
#include "kernels.hpp"
#include "layout.hpp"
#include "codec.hpp"
#include "parquet.hpp"
#include "plan.hpp"
#include "thrift.hpp"

namespace lk {

// ------------------------------------------------------------------------------------------------
// errors
// ------------------------------------------------------------------------------------------------
struct DeviceError : std::runtime_error {
  using std::runtime_error::runtime_error;
};

#define HIP_CHECK(x)                                                                          \
  do {                                                                                        \
    hipError_t _e = (x);                                                                      \
    if (_e != hipSuccess) {                                                                   \
      (void)hipGetLastError(); /* a failed allocation must not poison the next launch */      \
      throw DeviceError(std::string("HIP: ") + #x + ": " + hipGetErrorString(_e));            \
    }                                                                                         \
  } while (0)

// Call-context failures (workspace sync / free) surface as PlanError(LK_ERR_DEVICE): the distributed paths agree
// on PlanErrors before the next collective, so no rank is left waiting.
#define CTX_CHECK(x)                                                                            \
  do {                                                                                          \
    hipError_t _e = (x);                                                                        \
    if (_e != hipSuccess) {                                                                     \
      (void)hipGetLastError();                                                                  \
      throw PlanError(LK_ERR_DEVICE, std::string("HIP: ") + #x + ": " + hipGetErrorString(_e)); \
    }                                                                                           \
  } while (0)

static constexpr size_t kAlign = 256;
static inline size_t align_up(size_t x, size_t a = kAlign) { return (x + a - 1) / a * a; }

// fn(0..n-1) on up to `threads` threads (the calling thread among them); the first exception is rethrown
template <class F>
static void parallel_for(size_t n, int threads, F&& fn) {
  const size_t T = std::max<size_t>(1, std::min<size_t>(size_t(threads), n));
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


// ------------------------------------------------------------------------------------------------
// engine-global dictionaries: one per column name; chunk dictionaries remap into them at load
// ------------------------------------------------------------------------------------------------
uint32_t GlobalDict::intern(const std::string& s) {
  auto it = ids.find(s);
  if (it != ids.end()) return it->second;
  uint32_t id = uint32_t(vals->size());
  vals->push_back(s);
  refs.push_back(0);
  ids.emplace(vals->back(), id);
  return id;
}

// ------------------------------------------------------------------------------------------------
// pinned host blocks for result columns: allocated on first need, recycled by freed results
// ------------------------------------------------------------------------------------------------
namespace {
std::mutex g_pool_mu;
std::vector<HostBlock> g_pool;            // free blocks
constexpr size_t kPoolKeep = 8;
}  // namespace

HostBlock pinned_acquire(size_t bytes) {
  {
    std::lock_guard<std::mutex> g(g_pool_mu);
    size_t best = SIZE_MAX;
    for (size_t i = 0; i < g_pool.size(); i++)
      if (g_pool[i].cap >= bytes && (best == SIZE_MAX || g_pool[i].cap < g_pool[best].cap)) best = i;
    if (best != SIZE_MAX) {
      HostBlock b = g_pool[best];
      g_pool.erase(g_pool.begin() + long(best));
      return b;
    }
  }
  HostBlock b;
  b.cap = std::max<size_t>(align_up(bytes, size_t(1) << 20), size_t(1) << 20);
  if (hipHostMalloc(&b.p, b.cap, hipHostMallocDefault) == hipSuccess) {
    b.pinned = true;
  } else {
    (void)hipGetLastError();
    b.p = std::malloc(b.cap);
    if (!b.p) throw std::bad_alloc();
  }
  return b;
}

std::shared_ptr<void> zero_block(size_t bytes) {
  static std::mutex mu;
  static std::shared_ptr<void> blk;
  static size_t cap = 0;
  std::lock_guard<std::mutex> g(mu);
  if (!blk || cap < bytes) {
    const size_t n = std::max<size_t>(align_up(bytes, size_t(1) << 20), size_t(1) << 20);
    void* p = std::calloc(n, 1);
    if (!p) throw std::bad_alloc();
    blk = std::shared_ptr<void>(p, [](void* q) { std::free(q); });   // earlier results keep the old block alive
    cap = n;
  }
  return blk;
}

void pinned_release(HostBlock b) {
  if (!b.p) return;
  std::lock_guard<std::mutex> g(g_pool_mu);
  g_pool.push_back(b);
  if (g_pool.size() > kPoolKeep) {   // drop the smallest
    auto it = std::min_element(g_pool.begin(), g_pool.end(),
                               [](const HostBlock& x, const HostBlock& y) { return x.cap < y.cap; });
    if (it->pinned) (void)hipHostFree(it->p);
    else std::free(it->p);
    g_pool.erase(it);
  }
}

// LSD radix sort of (key, payload) pairs by the 128-bit key (16-bit digits, lo then hi word: stable, so the result
// is ordered by (hi, lo)).
static void radix_sort_keys(std::vector<Key128>& k, std::vector<uint32_t>& v) {
  const size_t n = k.size();
  std::vector<Key128> k2(n);
  std::vector<uint32_t> v2(n);
  std::vector<size_t> cnt(65537);
  for (int pass = 0; pass < 8; pass++) {
    const int word = pass / 4, shift = (pass % 4) * 16;   // lo word first
    auto digit = [&](const Key128& x) { return size_t(((word ? x.hi : x.lo) >> shift) & 0xffffu); };
    std::fill(cnt.begin(), cnt.end(), 0);
    for (size_t i = 0; i < n; i++) cnt[digit(k[i]) + 1]++;
    if (cnt[1] == n) continue;   // one digit value everywhere: the pass is the identity
    for (size_t d = 1; d <= 65536; d++) cnt[d] += cnt[d - 1];
    for (size_t i = 0; i < n; i++) {
      const size_t o = cnt[digit(k[i])]++;
      k2[o] = k[i];
      v2[o] = v[i];
    }
    k.swap(k2);
    v.swap(v2);
  }
}

Key128 value_key(const std::string& s) {
  uint64_t h[2];
  hll::murmur3_x64_128(s.data(), s.size(), 0x6c616b65ull /* "lake" */, h);
  return Key128{h[0], h[1]};
}

std::shared_ptr<const DictOrder> Engine::dict_order(const std::string& col, size_t n) {
  std::lock_guard<std::mutex> g(order_mu);
  auto& slot = orders[col];
  if (slot && slot->n == n) return slot;
  GlobalDict& gd = dict(col);
  std::vector<const std::string*> v(n);
  {
    std::lock_guard<std::mutex> dg(gd.mu);
    for (size_t i = 0; i < n; i++) v[i] = &gd[i];   // stable addresses (StableStrs)
  }
  auto o = std::make_shared<DictOrder>();
  o->n = n;
  o->keys.resize(n);
  o->perm.resize(n);
  const int T = n >= (size_t(1) << 16) ? load_thread_count() : 1;
  const size_t hb = (n + size_t(T) * 4 - 1) / (size_t(T) * 4);
  parallel_for(n ? (n + hb - 1) / hb : 0, T, [&](size_t b) {
    for (size_t i = b * hb; i < std::min(n, (b + 1) * hb); i++) {
      o->keys[i] = value_key(*v[i]);
      o->perm[i] = uint32_t(i);
    }
  });
  if (T > 1) {
    // uniform 128-bit hash keys: one scatter into 2^16 buckets by the top bits of `hi`, then every bucket sorted on
    // its own (in parallel) -- instead of the radix sort's 8 scatter passes
    // per-range bucket counts, then each range scatters into its own slice of every bucket (parallel, stable)
    const size_t R = size_t(T), per = (n + R - 1) / R;
    std::vector<std::vector<size_t>> rc(R, std::vector<size_t>(65536, 0));
    parallel_for(R, T, [&](size_t r) {
      for (size_t i = r * per; i < std::min(n, (r + 1) * per); i++) rc[r][o->keys[i].hi >> 48]++;
    });
    std::vector<size_t> cnt(65537, 0);
    for (size_t d = 0; d < 65536; d++) {
      size_t at = cnt[d];
      for (size_t r = 0; r < R; r++) {
        const size_t c = rc[r][d];
        rc[r][d] = at;   // range r's first slot in bucket d
        at += c;
      }
      cnt[d + 1] = at;
    }
    std::vector<std::pair<Key128, uint32_t>> kv(n);
    parallel_for(R, T, [&](size_t r) {
      std::vector<size_t>& pos = rc[r];
      for (size_t i = r * per; i < std::min(n, (r + 1) * per); i++) kv[pos[o->keys[i].hi >> 48]++] = {o->keys[i], o->perm[i]};
    });
    parallel_for(256, T, [&](size_t g) {
      for (size_t d = g * 256; d < (g + 1) * 256; d++)
        std::sort(kv.begin() + long(cnt[d]), kv.begin() + long(cnt[d + 1]),
                  [](const std::pair<Key128, uint32_t>& a, const std::pair<Key128, uint32_t>& b) { return a.first < b.first; });
    });
    parallel_for(R, T, [&](size_t r) {
      for (size_t i = r * per; i < std::min(n, (r + 1) * per); i++) {
        o->keys[i] = kv[i].first;
        o->perm[i] = kv[i].second;
      }
    });
  } else {
    radix_sort_keys(o->keys, o->perm);
  }
  for (size_t i = 1; i < n; i++)   // two distinct values of one dictionary on one 128-bit key: refuse, never merge
    if (o->keys[i] == o->keys[i - 1])
      throw PlanError(LK_ERR_UNSUPPORTED, "dictionary of " + col + ": 128-bit value-key collision");
  o->rank.resize(n);
  {
    const size_t per = (n + size_t(T) - 1) / size_t(T);
    parallel_for(size_t(T), T, [&](size_t r) {   // disjoint writes (perm is a permutation)
      for (size_t d = r * per; d < std::min(n, (r + 1) * per); d++) o->rank[o->perm[d]] = uint32_t(d);
    });
  }
  // Fingerprint of the value set: MurmurHash3_x64_128 over the sorted keys, chained over 1 MiB blocks.
  uint64_t fp[2] = {uint64_t(n), 0x9e3779b97f4a7c15ull};
  const char* base = reinterpret_cast<const char*>(o->keys.data());
  const size_t bytes = n * sizeof(Key128), blk = size_t(1) << 20;
  for (size_t off = 0; off < bytes || off == 0; off += blk) {
    uint64_t h[2];
    hll::murmur3_x64_128(base + off, std::min(blk, bytes - off), fp[0] ^ (fp[1] << 1), h);
    fp[0] ^= h[0];
    fp[1] = fp[1] * 0x100000001b3ull ^ h[1];
    if (bytes == 0) break;
  }
  o->fp[0] = fp[0];
  o->fp[1] = fp[1];
  slot = o;
  return slot;
}

DimUnion::~DimUnion() {
  if (d_dim_of_gid) {
    (void)hipSetDevice(device);
    (void)hipFree(d_dim_of_gid);
  }
}

std::shared_ptr<const std::vector<const char*>> Engine::dict_ptrs(const std::string& col, size_t n,
                                                                  const std::shared_ptr<StableStrs>& strs) {
  std::lock_guard<std::mutex> g(ptrs_mu);
  PtrTable& slot = ptrs[col];
  if (slot.strs != strs) slot = PtrTable{strs, nullptr};   // another generation of the dictionary: start over
  if (slot.tab && slot.tab->size() == n + 1) return slot.tab;
  auto v = std::make_shared<std::vector<const char*>>(n + 1, nullptr);
  size_t from = 0;
  if (slot.tab && slot.tab->size() <= n + 1) {   // the dictionary grew: values [0, old n) are unchanged (StableStrs)
    from = slot.tab->size() - 1;
    memcpy(v->data(), slot.tab->data(), from * sizeof(const char*));
  }
  for (size_t i = from; i < n; i++) {   // values [0, n) of one block never change (stable addresses)
    const std::string& x = (*strs)[i];
    (*v)[i] = (x.empty() || x == "null") ? nullptr : x.c_str();
  }
  if (!slot.tab || slot.tab->size() < v->size()) slot.tab = v;
  return v;
}

}  // namespace lk

const std::vector<const char*>* lk_result::tag_dictionary(size_t c) const {
  if (c >= tcols.size() || tcols[c].hidden) return nullptr;
  std::lock_guard<std::mutex> g(bulk_mu);
  if (bulk.size() < tcols.size()) bulk.resize(tcols.size());
  if (bulk[c]) return bulk[c].get();
  const TagCol& t = tcols[c];
  if (t.shared && !t.null_value && t.shared->size() == t.ndim) {   // an agreed union dim: its shared text table
    bulk[c] = t.shared;
    return bulk[c].get();
  }
  if (t.local.empty() && !t.order && t.engine && t.dict_keep && !t.null_value && t.dim_null == t.dict_n &&
      t.ndim == t.dict_n + 1) {
    if (const auto alive = t.engine_life.lock()) {   // the engine still exists: its cached table
      bulk[c] = t.engine->dict_ptrs(t.col, t.dict_n, t.dict_keep);   // dim id = engine global id: the shared table
      return bulk[c].get();
    }
  }
  auto v = std::make_shared<std::vector<const char*>>(size_t(t.ndim), nullptr);
  if (t.shared) {
    for (size_t d = 0; d < v->size() && d < t.shared->size(); d++) (*v)[d] = (*t.shared)[d];
  } else if (!t.local.empty()) {
    for (size_t d = 0; d < v->size() && d < t.local.size(); d++) (*v)[d] = t.local[d];
  } else if (t.dict) {
    for (size_t d = 0; d < v->size(); d++) {
      if (d == t.dim_null) continue;
      const std::string& s = (*t.dict)[t.order ? t.order->perm[d] : d];
      (*v)[d] = (s.empty() || s == "null") ? nullptr : s.c_str();
    }
  }
  if (t.dim_null < v->size()) (*v)[t.dim_null] = t.null_value;
  bulk[c] = v;
  return v.get();
}

namespace lk {

GlobalDict& Engine::dict(const std::string& col) {
  std::lock_guard<std::mutex> g(dict_mu);
  auto& p = dicts[col];
  if (!p) p = std::make_unique<GlobalDict>();
  return *p;
}

std::shared_ptr<const Request> Engine::parse_cached(const std::string& json) {
  {
    std::lock_guard<std::mutex> g(parsed_mu);
    auto it = parsed.find(json);
    if (it != parsed.end()) return it->second;
  }
  auto r = std::make_shared<const Request>(parse_request(json));   // throws on a malformed request: nothing cached
  std::lock_guard<std::mutex> g(parsed_mu);
  if (parsed.size() >= 64) parsed.clear();
  parsed.emplace(json, r);
  return r;
}

void Engine::dict_ref(const std::string& col, const uint32_t* ids, size_t n, int delta) {
  GlobalDict& gd = dict(col);
  std::lock_guard<std::mutex> g(gd.mu);
  for (size_t i = 0; i < n; i++) {
    const uint32_t id = ids[i];
    if (id >= gd.refs.size()) continue;
    if (delta > 0) {
      if (gd.refs[id]++ == 0) gd.live++;
    } else if (gd.refs[id] > 0 && --gd.refs[id] == 0) {
      gd.live--;
    }
  }
}

// Columns whose dead ids (no cached segment references them) are at least as many as the live ones get renumbered.
// Called at the C ABI before a load or an evaluation takes gen_mu shared.
void Engine::maybe_compact() {
  std::vector<std::string> cols;
  {
    std::lock_guard<std::mutex> g(dict_mu);
    for (auto& kv : dicts) {
      GlobalDict& gd = *kv.second;
      std::lock_guard<std::mutex> dg(gd.mu);
      const size_t dead = gd.size() - gd.live;
      if (dead > 0 && dead >= std::max(gd.live, compact_min_dead)) cols.push_back(kv.first);
    }
  }
  if (cols.empty()) return;
  std::unique_lock<std::shared_mutex> g(gen_mu);
  for (auto& c : cols) compact_locked(c);
}

void Engine::compact_locked(const std::string& col) {
  GlobalDict& gd = dict(col);
  std::vector<uint32_t> map;
  auto nv = std::make_shared<StableStrs>();
  std::unordered_map<std::string, uint32_t> ids;
  std::vector<uint32_t> refs;
  {
    std::lock_guard<std::mutex> dg(gd.mu);
    const size_t n = gd.size();
    if (n - gd.live == 0 || n - gd.live < std::max(gd.live, compact_min_dead)) return;
    map.assign(n, UINT32_MAX);
    ids.reserve(gd.live);
    refs.reserve(gd.live);
    for (size_t i = 0; i < n; i++) {
      if (gd.refs[i] == 0) continue;
      map[i] = uint32_t(nv->size());
      nv->push_back(gd[i]);
      ids.emplace(nv->back(), map[i]);
      refs.push_back(gd.refs[i]);
    }
  }
  // every cached segment's remap of this column: old id -> new id, on the GPU
  std::vector<std::pair<uint32_t*, size_t>> remaps;
  {
    std::lock_guard<std::mutex> g(cache_mu);
    for (auto& kv : cache) {
      const int c = kv.second->col_index(col);
      if (c < 0) continue;
      const HostCol& hc = kv.second->cols[size_t(c)];
      if (hc.is_string && hc.nremap) remaps.emplace_back(hc.d_remap, hc.nremap);
    }
  }
  if (!remaps.empty()) {
    CtxLease X(*this);
    uint32_t* d_map = static_cast<uint32_t*>(X->workspace("compact_map", map.size() * sizeof(uint32_t)));
    HIP_CHECK(hipMemcpyAsync(d_map, map.data(), map.size() * sizeof(uint32_t), hipMemcpyHostToDevice, X->stream));
    for (auto& r : remaps) HIP_CHECK(launch_remap_ids(r.first, r.second, d_map, X->stream));
    HIP_CHECK(hipStreamSynchronize(X->stream));
  }
  {
    std::lock_guard<std::mutex> dg(gd.mu);
    gd.live = refs.size();
    gd.vals = nv;          // results built before keep the old block (lk_result::TagCol::dict_keep / keep)
    gd.ids.swap(ids);
    gd.refs.swap(refs);
    gd.gen++;
  }
  // caches keyed by the old ids
  {
    std::lock_guard<std::mutex> g(leaf_mu);
    const std::string pre = col + '\x1f';
    for (auto it = leaf_cache.begin(); it != leaf_cache.end();)
      it = it->first.compare(0, pre.size(), pre) == 0 ? leaf_cache.erase(it) : std::next(it);
  }
  {
    std::lock_guard<std::mutex> g(order_mu);
    orders.erase(col);
  }
  {
    std::lock_guard<std::mutex> g(ptrs_mu);
    ptrs.erase(col);
  }
  unions.erase(col);   // (used under comm_mu by distributed evaluations, none of which runs now)
  compactions++;
}

// ------------------------------------------------------------------------------------------------
// segment load: footer + page walk + run directories + tiles + zone maps -> HBM
// ------------------------------------------------------------------------------------------------
namespace {

struct PageStreams {
  const uint8_t* defs = nullptr;
  size_t defs_len = 0;
  const uint8_t* vals = nullptr;
  size_t vals_len = 0;
  uint32_t nrows = 0;
  int encoding = 0;
};

struct HostPage {
  PageDesc d{};
  uint32_t rg = 0;
  uint32_t run_lo = 0, run_n = 0, drun_lo = 0, drun_n = 0;
  std::vector<uint32_t> vprefix;   // nullable pages with NULLs: non-null rows before row i (size nrows+1)
  const uint8_t* host_vals = nullptr;
};

// A byte range of one page stream: copied from `src` (the file, or a decompressed / re-encoded page buffer) to `off`
// in its chunk's stream area.
struct StreamRef {
  const uint8_t* src;
  size_t len;
  size_t off;
};

// One column chunk (column, row group) walked on the host: page descriptors, run tables and the byte ranges of its
// page streams.  Chunks are independent, so the walk runs on several threads (Engine::load_threads); string
// dictionary values are interned into the engine dictionaries afterwards, per column in row-group order, so the
// engine-global ids do not depend on thread timing.
struct ChunkOut {
  std::vector<StreamRef> streams;
  size_t bytes = 0;                       // the chunk's stream area (every stream 128-B aligned: one HBM line start)
  std::vector<HostPage> pages;            // d.vals / d.defs: offsets in the chunk's area; run_lo / drun_lo: indices into
                                          // `runs`; d.remap: index into `dict`
  std::vector<RunDesc> runs;
  // strings: the dictionary page's values, then every PLAIN page's own values -- views into the file bytes or `plain`
  // (both outlive the load), so a 10M-value dictionary is not copied string by string before interning
  std::vector<std::string_view> dict;
  // decompressed / re-encoded pages (streams, zone maps and dictionary views point into them): heap-held so the
  // buffers stay put when the ChunkOut moves
  std::vector<std::unique_ptr<std::vector<uint8_t>>> plain;
  uint64_t compressed = 0;
  int code = 0;                           // LK_ERR_IO: the file is corrupt; LK_ERR_UNSUPPORTED: this column's shape
  std::string msg;
  size_t put(const uint8_t* p, size_t n) {
    const size_t off = (bytes + 127) / 128 * 128;
    if (n) streams.push_back(StreamRef{p, n, off});
    bytes = off + n;
    return off;
  }
};

// A vector<ChunkOut> that reallocates must move its elements (a copy would re-allocate `plain` and leave every
// StreamRef / host_vals / dictionary view pointing at freed buffers).
static_assert(std::is_nothrow_move_constructible<ChunkOut>::value, "ChunkOut must move without copying");

PageStreams split_page(const pq::PageHeader& h, const uint8_t* data, size_t n, bool nullable) {
  PageStreams s;
  if (h.type == pq::DATA_PAGE) {
    s.nrows = uint32_t(h.num_values);
    s.encoding = h.encoding;
    size_t off = 0;
    if (nullable) {
      if (h.def_encoding != pq::RLE) throw PlanError(LK_ERR_UNSUPPORTED, "parquet: BIT_PACKED definition levels");
      if (n < 4) throw PlanError(LK_ERR_IO, "parquet: truncated page");
      uint32_t L;
      memcpy(&L, data, 4);
      if (size_t(L) + 4 > n) throw PlanError(LK_ERR_IO, "parquet: bad def-level length");
      s.defs = data + 4;
      s.defs_len = L;
      off = 4 + L;
    }
    s.vals = data + off;
    s.vals_len = n - off;
  } else {  // DATA_PAGE_V2
    s.nrows = uint32_t(h.num_rows >= 0 ? h.num_rows : h.num_values);
    s.encoding = h.encoding;
    if (h.rep_len) throw PlanError(LK_ERR_UNSUPPORTED, "parquet: repeated columns");
    size_t off = size_t(h.rep_len);
    if (size_t(h.def_len) + off > n) throw PlanError(LK_ERR_IO, "parquet: bad v2 level lengths");
    if (nullable) {
      s.defs = data + off;
      s.defs_len = size_t(h.def_len);
    }
    off += size_t(h.def_len);
    s.vals = data + off;
    s.vals_len = n - off;
  }
  return s;
}

// Walks one column chunk's pages (thread-safe: reads only `col`'s schema fields and the file bytes).
void walk_column_chunk(const uint8_t* F, size_t size, const HostCol& col, uint32_t rg, int64_t rg_rows,
                       const pq::ColumnMeta& m, ChunkOut& C) {
  if (!pq::codec_supported(m.codec))
    throw PlanError(LK_ERR_UNSUPPORTED, "parquet: compression codec " + std::to_string(m.codec) + " in column " +
                                            col.name + " is not supported");
  int64_t start = m.data_page_offset;
  if (m.dictionary_page_offset > 0 && m.dictionary_page_offset < start) start = m.dictionary_page_offset;
  if (start < 4 || size_t(start) >= size) throw PlanError(LK_ERR_IO, "parquet: bad page offset");
  C.compressed += uint64_t(m.total_compressed);
  size_t pos = size_t(start);
  int64_t seen = 0;
  uint32_t dict_n = 0;
  bool have_dict = false;
  // numeric columns: fixed width of a PLAIN value (BOOLEAN: bit-packed) and the chunk's dictionary, if any (its
  // pages are materialized to PLAIN at load, so the kernels only ever see PLAIN numeric pages)
  const size_t width = col.ptype == pq::INT64 || col.ptype == pq::DOUBLE ? 8 : (col.ptype == pq::BOOLEAN ? 0 : 4);
  std::vector<uint8_t> ndict;
  uint32_t first_row = 0;
  while (seen < m.num_values) {
    if (pos >= size) throw PlanError(LK_ERR_IO, "parquet: page walk ran past the file");
    pq::PageHeader h = pq::parse_page_header(F + pos, size - pos);
    const uint8_t* data = F + pos + h.header_len;
    size_t n = size_t(h.compressed);
    if (pos + h.header_len + n > size) throw PlanError(LK_ERR_IO, "parquet: page overruns the file");
    pos += h.header_len + n;
    if (m.codec != pq::CODEC_UNCOMPRESSED &&
        (h.type == pq::DICTIONARY_PAGE || h.type == pq::DATA_PAGE || h.type == pq::DATA_PAGE_V2)) {
      // v1 and dictionary pages: the whole payload is compressed; v2: the levels stay plain, the values are
      // compressed unless is_compressed = false (parquet.thrift DataPageHeaderV2)
      const size_t lv = h.type == pq::DATA_PAGE_V2 ? size_t(h.rep_len) + size_t(h.def_len) : 0;
      if (h.uncompressed < 0 || lv > n || lv > size_t(h.uncompressed))
        throw PlanError(LK_ERR_IO, "parquet: bad page sizes");
      if (h.type != pq::DATA_PAGE_V2 || h.v2_compressed) {
        C.plain.push_back(std::make_unique<std::vector<uint8_t>>(size_t(h.uncompressed)));
        std::vector<uint8_t>& out = *C.plain.back();
        if (lv) memcpy(out.data(), data, lv);
        pq::decompress(m.codec, data + lv, n - lv, out.data() + lv, out.size() - lv);
        data = out.data();
        n = out.size();
      }
    }
    if (h.type == pq::DICTIONARY_PAGE && !col.is_string) {
      if (width == 0) throw PlanError(LK_ERR_UNSUPPORTED, "parquet: dictionary-encoded BOOLEAN column " + col.name);
      if (h.dict_num_values < 0 || size_t(h.dict_num_values) * width > n)
        throw PlanError(LK_ERR_IO, "parquet: truncated dictionary page in " + col.name);
      ndict.assign(data, data + size_t(h.dict_num_values) * width);
      dict_n = uint32_t(h.dict_num_values);
      have_dict = true;
      continue;
    }
    if (h.type == pq::DICTIONARY_PAGE) {
      if (h.dict_num_values < 0) throw PlanError(LK_ERR_IO, "parquet: bad dictionary page in " + col.name);
      if (have_dict) throw PlanError(LK_ERR_IO, "parquet: second dictionary page in " + col.name);
      size_t p = 0;
      C.dict.reserve(size_t(h.dict_num_values));
      for (int32_t i = 0; i < h.dict_num_values; i++) {
        if (p + 4 > n) throw PlanError(LK_ERR_IO, "parquet: truncated dictionary page");
        uint32_t L;
        memcpy(&L, data + p, 4);
        p += 4;
        if (p + L > n) throw PlanError(LK_ERR_IO, "parquet: truncated dictionary entry");
        C.dict.emplace_back(reinterpret_cast<const char*>(data + p), L);
        p += L;
      }
      dict_n = uint32_t(h.dict_num_values);
      have_dict = true;
      continue;
    }
    if (h.type != pq::DATA_PAGE && h.type != pq::DATA_PAGE_V2) continue;   // index pages: skip
    PageStreams st = split_page(h, data, n, col.nullable);
    HostPage hp;
    hp.rg = rg;
    PageDesc& d = hp.d;
    d.first_row = first_row;
    d.nrows = st.nrows;
    d.nullable = col.nullable ? 1 : 0;
    // definition levels
    uint32_t nvals = st.nrows;
    if (col.nullable) {
      auto druns = pq::hybrid_runs(st.defs, st.defs_len, 1, st.nrows);
      // non-null count from the runs: RLE runs by their value, bit-packed runs by popcount of their bytes
      nvals = 0;
      bool any_null = false;
      for (auto& r : druns) {
        if (!r.literal) {
          if (r.value) nvals += r.count;
          else any_null = any_null || r.count;
          continue;
        }
        const uint8_t* b = st.defs + r.off;
        uint32_t k = 0, c = 0;
        for (; k + 8 <= r.count; k += 8) c += uint32_t(__builtin_popcount(b[k >> 3]));
        for (; k < r.count; k++) c += (b[k >> 3] >> (k & 7)) & 1u;
        nvals += c;
      }
      (void)any_null;
      d.has_nulls = nvals < st.nrows;
      if (d.has_nulls) {
        std::vector<uint32_t> defv(st.nrows);
        pq::hybrid_decode(st.defs, st.defs_len, 1, st.nrows, defv.data());
        hp.vprefix.resize(st.nrows + 1);
        uint32_t acc = 0;
        for (uint32_t i = 0; i < st.nrows; i++) {
          hp.vprefix[i] = acc;
          acc += defv[i] ? 1 : 0;
        }
        hp.vprefix[st.nrows] = acc;
        hp.drun_lo = uint32_t(C.runs.size());
        for (auto& r : druns) C.runs.push_back(RunDesc{r.start, (r.literal ? 0x80000000u : 0u) | r.off, r.value, r.count});
        hp.drun_n = uint32_t(druns.size());
        d.defs = C.put(st.defs, st.defs_len);
        d.defs_len = uint32_t(st.defs_len);
      }
    }
    d.nvals = nvals;
    if (col.is_string) {
      uint32_t page_remap = 0, page_dict_n = dict_n;
      if (st.encoding == pq::PLAIN) {
        // PLAIN BYTE_ARRAY page (a writer's dictionary fallback, or no dictionary at all): the page gets its own
        // dictionary -- its distinct values in first-seen order, interned with the chunk -- and its values are
        // re-encoded as one bit-packed literal run of indices, so the kernels see a dictionary page.
        std::unordered_map<std::string_view, uint32_t> local;
        std::vector<uint32_t> idx(nvals);
        page_remap = uint32_t(C.dict.size());
        size_t p = 0;
        for (uint32_t i = 0; i < nvals; i++) {
          if (p + 4 > st.vals_len) throw PlanError(LK_ERR_IO, "parquet: truncated PLAIN BYTE_ARRAY page in " + col.name);
          uint32_t L;
          memcpy(&L, st.vals + p, 4);
          p += 4;
          if (p + L > st.vals_len) throw PlanError(LK_ERR_IO, "parquet: truncated PLAIN BYTE_ARRAY value in " + col.name);
          auto ins = local.emplace(std::string_view(reinterpret_cast<const char*>(st.vals + p), L), uint32_t(local.size()));
          if (ins.second) C.dict.emplace_back(ins.first->first);
          idx[i] = ins.first->second;
          p += L;
        }
        page_dict_n = uint32_t(local.size());
        int pbw = 1;
        while (pbw < 32 && (1ull << pbw) < page_dict_n) pbw++;
        const size_t ngroups = (size_t(nvals) + 7) / 8;
        C.plain.push_back(std::make_unique<std::vector<uint8_t>>());
        std::vector<uint8_t>& enc = *C.plain.back();
        enc.push_back(uint8_t(pbw));
        for (uint64_t hdr = (uint64_t(ngroups) << 1) | 1u;; hdr >>= 7) {   // literal-run header (ULEB128)
          enc.push_back(uint8_t((hdr & 0x7f) | (hdr >= 0x80 ? 0x80 : 0)));
          if (hdr < 0x80) break;
        }
        const size_t base = enc.size();
        enc.resize(base + ngroups * size_t(pbw), 0);
        for (size_t i = 0; i < size_t(nvals); i++) {
          const uint64_t bit = uint64_t(i) * uint64_t(pbw);
          for (int b = 0; b < pbw; b++)
            if ((idx[i] >> b) & 1u) enc[base + ((bit + b) >> 3)] |= uint8_t(1u << ((bit + b) & 7));
        }
        st.vals = enc.data();
        st.vals_len = enc.size();
      } else if (st.encoding != pq::RLE_DICTIONARY && st.encoding != pq::PLAIN_DICTIONARY) {
        throw PlanError(LK_ERR_UNSUPPORTED, "parquet: string page encoding " + std::to_string(st.encoding) + " in " +
                                                col.name);
      } else if (!have_dict) {
        throw PlanError(LK_ERR_IO, "parquet: dictionary page missing for " + col.name);
      }
      const uint32_t pdict = page_dict_n;
      if (st.vals_len < 1 && nvals) throw PlanError(LK_ERR_IO, "parquet: empty dictionary-index page");
      int bw = st.vals_len ? st.vals[0] : 0;
      if (bw > 32) throw PlanError(LK_ERR_IO, "parquet: bad dictionary index bit width");
      const uint8_t* stream = st.vals_len ? st.vals + 1 : st.vals;
      size_t slen = st.vals_len ? st.vals_len - 1 : 0;
      auto runs = pq::hybrid_runs(stream, slen, bw, nvals);
      // validate every index against the dictionary so a corrupt page can never index out of bounds on the GPU:
      // RLE runs by their value, bit-packed runs by their largest index
      if (!runs.empty() && pdict < (bw >= 32 ? 0xffffffffu : (1u << bw))) {
        for (auto& r : runs) {
          const uint32_t mx = r.literal ? pq::hybrid_literal_max(stream + r.off, slen - r.off, bw, r.count) : r.value;
          if (r.count && mx >= pdict) throw PlanError(LK_ERR_IO, "parquet: dictionary index out of range in " + col.name);
        }
      }
      hp.run_lo = uint32_t(C.runs.size());
      for (auto& r : runs) C.runs.push_back(RunDesc{r.start, (r.literal ? 0x80000000u : 0u) | r.off, r.value, r.count});
      hp.run_n = uint32_t(runs.size());
      d.kind = PAGE_DICT;
      d.bw = uint8_t(bw);
      d.remap = page_remap;
      d.dict_n = pdict;
      d.vals = C.put(stream, slen);
      d.vals_len = uint32_t(slen);
    } else {
      if ((st.encoding == pq::RLE_DICTIONARY || st.encoding == pq::PLAIN_DICTIONARY) && width) {
        // dictionary-encoded numeric page (e.g. a writer's default dictionary for every column): materialized to
        // PLAIN values here
        if (!have_dict) throw PlanError(LK_ERR_IO, "parquet: dictionary page missing for " + col.name);
        if (st.vals_len < 1 && nvals) throw PlanError(LK_ERR_IO, "parquet: empty dictionary-index page");
        const int bw = st.vals_len ? st.vals[0] : 0;
        if (bw > 32) throw PlanError(LK_ERR_IO, "parquet: bad dictionary index bit width");
        std::vector<uint32_t> idx(nvals);
        pq::hybrid_decode(st.vals_len ? st.vals + 1 : st.vals, st.vals_len ? st.vals_len - 1 : 0, bw, nvals, idx.data());
        C.plain.push_back(std::make_unique<std::vector<uint8_t>>(size_t(nvals) * width));
        std::vector<uint8_t>& out = *C.plain.back();
        for (uint32_t i = 0; i < nvals; i++) {
          if (idx[i] >= dict_n) throw PlanError(LK_ERR_IO, "parquet: dictionary index out of range in " + col.name);
          memcpy(out.data() + size_t(i) * width, ndict.data() + size_t(idx[i]) * width, width);
        }
        st.vals = out.data();
        st.vals_len = out.size();
      } else if (st.encoding != pq::PLAIN) {
        throw PlanError(LK_ERR_UNSUPPORTED, "parquet: numeric page encoding " + std::to_string(st.encoding) + " in " + col.name);
      }
      // PLAIN: 8-B (INT64 / DOUBLE) or 4-B (INT32 / FLOAT) values; BOOLEAN bit-packed, LSB first
      const size_t bytes = width ? size_t(nvals) * width : (size_t(nvals) + 7) / 8;
      if (st.vals_len < bytes) throw PlanError(LK_ERR_IO, "parquet: truncated PLAIN page in " + col.name);
      d.kind = width == 8 ? PAGE_PLAIN64 : (width == 4 ? PAGE_PLAIN32 : PAGE_BOOL);
      d.vals = C.put(st.vals, bytes);
      d.vals_len = uint32_t(bytes);
      hp.host_vals = st.vals;
    }
    C.pages.push_back(std::move(hp));
    first_row += st.nrows;
    seen += h.type == pq::DATA_PAGE ? h.num_values : st.nrows;
  }
  if (int64_t(first_row) != rg_rows)
    throw PlanError(LK_ERR_IO, "parquet: column " + col.name + " row count disagrees with its row group");
}

// value index within page of row r (relative to page)
inline uint32_t vindex(const HostPage& p, uint32_t r) { return p.vprefix.empty() ? r : p.vprefix[r]; }
// first row (relative to page) whose value index is >= v
inline uint32_t row_of_vindex(const HostPage& p, uint32_t v) {
  if (p.vprefix.empty()) return v;
  return uint32_t(std::lower_bound(p.vprefix.begin(), p.vprefix.end() - 1, v) - p.vprefix.begin());
}

// run index (within [lo, lo+n)) containing position x; runs sorted by start
inline uint32_t run_containing(const std::vector<RunDesc>& runs, uint32_t lo, uint32_t n, uint32_t x) {
  uint32_t a = lo, b = lo + n - 1;
  while (a < b) {
    uint32_t mid = (a + b + 1) / 2;
    if (runs[mid].start <= x) a = mid;
    else b = mid - 1;
  }
  return a;
}

// Tiles of one row group: row ranges inside one page of every column, clipped so each stream's runs over a tile fit
// RUN_CAP; the timestamp zone map per tile.  `page0[c]`: index of column c's first page of this row group.
void build_tiles_rg(const Segment& S, const std::vector<std::vector<HostPage>>& pages, uint32_t rg,
                    const std::vector<size_t>& page0, std::vector<TileDesc>& tiles, std::vector<std::vector<TileCol>>& tcols) {
  const int nc = int(S.cols.size());
  const int ts_col = S.col_index(kTimestamp);
  std::vector<size_t> cursor(page0);
  const uint32_t nrows = uint32_t(S.rg_rows[rg]);
  tcols.assign(size_t(nc), {});
  uint32_t a = 0;
  std::vector<size_t> pidx(static_cast<size_t>(nc));
  while (a < nrows) {
    uint32_t e = std::min<uint64_t>(nrows, uint64_t(a) + TILE_ROWS);
    // page of every column containing row a; clip e to that page's end and to the run caps
    for (int c = 0; c < nc; c++) {
      auto& pg = pages[size_t(c)];
      size_t& k = cursor[size_t(c)];
      while (k < pg.size() && pg[k].rg == rg && pg[k].d.first_row + pg[k].d.nrows <= a) k++;
      if (k >= pg.size() || pg[k].rg != rg) throw PlanError(LK_ERR_IO, "parquet: page index inconsistent");
      pidx[size_t(c)] = k;
      const HostPage& p = pg[k];
      e = std::min(e, p.d.first_row + p.d.nrows);
      uint32_t ra = a - p.d.first_row, re = e - p.d.first_row;
      if (p.d.kind == PAGE_DICT && p.run_n) {
        uint32_t va = vindex(p, ra), ve = vindex(p, re);
        if (ve > va) {
          uint32_t r0 = run_containing(S.cols[size_t(c)].runs, p.run_lo, p.run_n, va);
          uint32_t r1 = run_containing(S.cols[size_t(c)].runs, p.run_lo, p.run_n, ve - 1);
          if (r1 - r0 + 1 > RUN_CAP) {
            uint32_t vcut = S.cols[size_t(c)].runs[r0 + RUN_CAP].start;
            e = std::min(e, p.d.first_row + row_of_vindex(p, vcut));
          }
        }
      }
      if (p.d.has_nulls) {
        re = e - p.d.first_row;
        uint32_t r0 = run_containing(S.cols[size_t(c)].runs, p.drun_lo, p.drun_n, ra);
        uint32_t r1 = run_containing(S.cols[size_t(c)].runs, p.drun_lo, p.drun_n, re - 1);
        if (r1 - r0 + 1 > RUN_CAP) e = std::min(e, p.d.first_row + S.cols[size_t(c)].runs[r0 + RUN_CAP].start);
      }
    }
    if (e <= a) throw PlanError(LK_ERR_IO, "parquet: tile construction made no progress");
    TileDesc t{};
    t.rg = rg;
    t.row0 = a;
    t.nrows = e - a;
    t.ts_min = INT64_MAX;
    t.ts_max = INT64_MIN;
    for (int c = 0; c < nc; c++) {
      const HostPage& p = pages[size_t(c)][pidx[size_t(c)]];
      TileCol tc{};
      tc.page = uint32_t(pidx[size_t(c)]);
      uint32_t ra = a - p.d.first_row, re = e - p.d.first_row;
      uint32_t va = vindex(p, ra), ve = vindex(p, re);
      tc.vbase = va;
      tc.vals = p.d.vals;
      tc.defs = p.d.defs;
      tc.vals_len = p.d.vals_len;
      tc.defs_len = p.d.defs_len;
      tc.row_in_page = ra;
      tc.remap = p.d.remap;
      tc.dict_n = p.d.dict_n;
      tc.bw = p.d.bw;
      tc.kind = p.d.kind;
      tc.has_nulls = p.d.has_nulls;
      if (p.d.kind == PAGE_DICT && p.run_n && ve > va) {
        uint32_t r0 = run_containing(S.cols[size_t(c)].runs, p.run_lo, p.run_n, va);
        uint32_t r1 = run_containing(S.cols[size_t(c)].runs, p.run_lo, p.run_n, ve - 1);
        tc.run_lo = r0;
        tc.nruns = r1 - r0 + 1;
      }
      if (p.d.has_nulls) {
        uint32_t r0 = run_containing(S.cols[size_t(c)].runs, p.drun_lo, p.drun_n, ra);
        uint32_t r1 = run_containing(S.cols[size_t(c)].runs, p.drun_lo, p.drun_n, re - 1);
        tc.drun_lo = r0;
        tc.ndruns = r1 - r0 + 1;
      }
      tcols[size_t(c)].push_back(tc);
      if (c == ts_col && p.d.kind == PAGE_PLAIN64 && !S.cols[size_t(c)].is_string) {
        const int64_t* v = reinterpret_cast<const int64_t*>(p.host_vals);   // (host_vals: 8-B PLAIN values)
        int64_t lo = INT64_MAX, hi = INT64_MIN;
        for (uint32_t i = va; i < ve; i++) {
          int64_t x;
          memcpy(&x, v + i, 8);
          lo = std::min(lo, x);
          hi = std::max(hi, x);
        }
        t.ts_min = lo;
        t.ts_max = hi;
      } else if (c == ts_col && p.d.kind == PAGE_PLAIN32 && S.cols[size_t(c)].ptype == pq::INT32) {
        for (uint32_t v = va; v < ve; v++) {   // INT32 timestamps (BIGINT in a union_by_name glob)
          int32_t x;
          memcpy(&x, p.host_vals + size_t(v) * 4, 4);
          t.ts_min = std::min<int64_t>(t.ts_min, x);
          t.ts_max = std::max<int64_t>(t.ts_max, x);
        }
      }
    }
    tiles.push_back(t);
    a = e;
  }
}

// Runs fn(i) for i in [0, n) on up to `threads` threads (the calling thread included); the first exception is
// rethrown after every worker has finished.

}  // namespace

int Segment::col_index(const std::string& name) const {
  auto it = by_name.find(name);
  return it == by_name.end() ? -1 : it->second;
}

Segment::~Segment() {
  // release this segment's references to dictionary ids (read back from its remaps: the host copy is dropped after
  // upload), so a later compaction can reclaim ids no cached segment uses any more
  if (engine && d_meta)
    for (const HostCol& c : cols) {
      if (!c.is_string || c.nremap == 0 || !c.d_remap) continue;
      std::vector<uint32_t> ids(c.nremap);
      if (hipMemcpy(ids.data(), c.d_remap, c.nremap * sizeof(uint32_t), hipMemcpyDeviceToHost) != hipSuccess) {
        (void)hipGetLastError();
        continue;   // the ids stay referenced (never reclaimed): safe
      }
      engine->dict_ref(c.name, ids.data(), ids.size(), -1);
    }
  if (d_data) (void)hipFree(d_data);
  if (d_meta) (void)hipFree(d_meta);
}

// Physical types the engine loads: BYTE_ARRAY strings, INT64 / DOUBLE (the scan's timestamp and value columns), and
// INT32 / FLOAT / BOOLEAN (read by exemplar rows).  INT96 / FIXED_LEN_BYTE_ARRAY are not loaded.
static bool loadable_type(int ptype) {
  return ptype == pq::BYTE_ARRAY || ptype == pq::INT64 || ptype == pq::DOUBLE || ptype == pq::INT32 ||
         ptype == pq::FLOAT || ptype == pq::BOOLEAN;
}

int Engine::load_thread_count() const {
  if (load_threads > 0) return load_threads;
  int t = int(std::thread::hardware_concurrency());
  if (const char* o = getenv("OMP_NUM_THREADS")) t = std::min(t > 0 ? t : 16, std::max(1, atoi(o)));
  return std::max(1, std::min(t > 0 ? t : 8, 16));
}

// Parquet bytes -> an HBM segment.  Host: footer, schema walk, then every column chunk walked on its own thread
// (pages, run tables, decompression, index validation), string dictionaries interned per column in row-group order,
// tiles built per row group in parallel; device: the page streams copied once into a pinned staging area (in
// parallel) and uploaded with one DMA, then one metadata blob.
// A column the engine cannot decode (nested / repeated, INT96 / FIXED_LEN_BYTE_ARRAY, a page encoding or codec
// outside the implemented set) is left unloaded with its reason (Segment::unloaded): the segment still serves every
// query that does not reference it, and a query that does fails with LK_ERR_UNSUPPORTED -- a capability gap, not an
// empty glob.  A corrupt file is LK_ERR_IO.
std::shared_ptr<Segment> Engine::build_segment(const std::string& key, const uint8_t* F, size_t size) {
  const auto t0 = std::chrono::steady_clock::now();
  auto S = std::make_shared<Segment>();
  S->key = key;
  pq::FileMeta fm = pq::parse_footer(F, size);
  if (fm.schema.empty()) throw PlanError(LK_ERR_IO, "parquet: empty schema");
  // Schema walk: top-level primitive fields are columns; a group (struct / list / map) is one top-level name whose
  // leaves occupy column chunks but are not loaded.  leaf_col[i] = index into S->cols of the i-th leaf, or -1.
  std::vector<int> leaf_col;
  {
    size_t i = 1;
    const int ntop = fm.schema[0].num_children > 0 ? fm.schema[0].num_children : int(fm.schema.size()) - 1;
    for (int f = 0; f < ntop && i < fm.schema.size(); f++) {
      const auto& e = fm.schema[i];
      if (e.num_children > 0) {   // nested group: skip its subtree, counting its leaves
        S->all_columns.insert(e.name);
        S->unloaded[e.name] = "nested column " + e.name + " (struct / list / map) is not loaded";
        S->schema.emplace_back(e.name, -1);   // SELECT * names it (a query that reads it fails: unloaded)
        size_t pending = 1;
        while (pending && i < fm.schema.size()) {
          const auto& g = fm.schema[i++];
          pending--;
          if (g.num_children > 0) pending += size_t(g.num_children);
          else leaf_col.push_back(-1);
        }
        continue;
      }
      i++;
      S->all_columns.insert(e.name);
      S->schema.emplace_back(e.name, e.type);
      if (e.repetition == pq::REPEATED) {
        S->unloaded[e.name] = "repeated column " + e.name + " is not loaded";
        leaf_col.push_back(-1);
        continue;
      }
      if (!loadable_type(e.type)) {
        S->unloaded[e.name] = "column " + e.name + " of Parquet physical type " + std::to_string(e.type) +
                              " (INT96 / FIXED_LEN_BYTE_ARRAY) is not loaded";
        leaf_col.push_back(-1);
        continue;
      }
      HostCol c;
      c.name = e.name;
      c.ptype = e.type;
      c.nullable = e.repetition == pq::OPTIONAL;
      c.is_string = e.type == pq::BYTE_ARRAY;
      leaf_col.push_back(int(S->cols.size()));
      S->cols.push_back(std::move(c));
    }
  }
  S->num_rows = fm.num_rows;
  const size_t nrg = fm.row_groups.size();
  for (auto& g : fm.row_groups) {
    if (g.columns.size() != leaf_col.size()) throw PlanError(LK_ERR_IO, "parquet: row group column count mismatch");
    S->rg_rows.push_back(g.num_rows);
  }
  const int threads = load_thread_count();

  // ---- 1. every (column, row group) chunk walked in parallel ----
  const size_t ncol = S->cols.size();
  std::vector<int> leaf_of(ncol);
  for (size_t l = 0; l < leaf_col.size(); l++)
    if (leaf_col[l] >= 0) leaf_of[size_t(leaf_col[l])] = int(l);
  std::vector<ChunkOut> chunks(ncol * nrg);   // [column][row group]
  parallel_for(chunks.size(), threads, [&](size_t k) {
    const size_t ci = k / std::max<size_t>(nrg, 1), rg = k % std::max<size_t>(nrg, 1);
    ChunkOut& C = chunks[k];
    try {
      walk_column_chunk(F, size, S->cols[ci], uint32_t(rg), S->rg_rows[rg], fm.row_groups[rg].columns[size_t(leaf_of[ci])], C);
    } catch (const PlanError& e) {
      C.code = e.code;
      C.msg = e.what();
    } catch (const std::bad_alloc&) {
      throw;
    } catch (const std::exception& e) {   // thrift / codec parse errors: the file is corrupt
      C.code = LK_ERR_IO;
      C.msg = e.what();
    }
  });
  // a corrupt chunk fails the segment (LK_ERR_IO); a chunk outside the implemented shapes unloads its column
  std::vector<char> keep(ncol, 1);
  for (size_t ci = 0; ci < ncol; ci++)
    for (size_t rg = 0; rg < nrg; rg++) {
      const ChunkOut& C = chunks[ci * nrg + rg];
      if (C.code == LK_ERR_IO) throw PlanError(LK_ERR_IO, C.msg);
      if (C.code && keep[ci]) {
        keep[ci] = 0;
        S->unloaded[S->cols[ci].name] = C.code == LK_ERR_UNSUPPORTED ? C.msg : ("column " + S->cols[ci].name + ": " + C.msg);
      }
    }
  {   // drop unloaded columns (and their chunks) from the index
    std::vector<HostCol> kept;
    std::vector<ChunkOut> kept_chunks;
    kept_chunks.reserve(chunks.size());
    S->by_name.clear();
    for (size_t ci = 0; ci < ncol; ci++) {
      if (!keep[ci]) continue;
      S->by_name[S->cols[ci].name] = int(kept.size());
      kept.push_back(std::move(S->cols[ci]));
      for (size_t rg = 0; rg < nrg; rg++) kept_chunks.push_back(std::move(chunks[ci * nrg + rg]));
    }
    S->cols = std::move(kept);
    chunks = std::move(kept_chunks);
  }
  const size_t nc = S->cols.size();

  // ---- 2. per column, in row-group order: intern dictionaries, concatenate runs and pages, place streams ----
  // Byte offset of each chunk's stream area in the segment: row-group major (a row group's columns side by side, as
  // in the file), so the streams one tile reads lie close together (column-major placement measured ~1.8x slower
  // scans; LK_COLMAJOR=1 keeps it for A/B).
  std::vector<size_t> chunk_base(chunks.size());
  {
    const bool colmajor = getenv("LK_COLMAJOR") != nullptr;
    size_t off = 0;
    for (size_t i = 0; i < chunks.size(); i++) {
      const size_t k = colmajor || nrg == 0 ? i : (i % nc) * nrg + i / nc;   // i = rg * nc + column
      off = (off + 127) / 128 * 128;
      chunk_base[k] = off;
      off += chunks[k].bytes;
    }
    S->data_bytes = align_up(off + 64);
  }
  std::vector<std::vector<HostPage>> pages(nc);
  std::vector<std::vector<size_t>> page0(nc, std::vector<size_t>(nrg, 0));   // first page of (column, row group)
  parallel_for(nc, threads, [&](size_t ci) {
    HostCol& col = S->cols[ci];
    size_t npages = 0, nruns = 0, ndict = 0;
    for (size_t rg = 0; rg < nrg; rg++) {
      npages += chunks[ci * nrg + rg].pages.size();
      nruns += chunks[ci * nrg + rg].runs.size();
      ndict += chunks[ci * nrg + rg].dict.size();
    }
    pages[ci].reserve(npages);
    col.runs.reserve(nruns);
    col.remap.reserve(ndict);
    if (col.is_string && ndict) {
      GlobalDict& gd = dict(col.name);
      std::lock_guard<std::mutex> g(gd.mu);
      std::vector<const std::string_view*> sv;
      sv.reserve(ndict);
      for (size_t rg = 0; rg < nrg; rg++)
        for (const std::string_view& v : chunks[ci * nrg + rg].dict) sv.push_back(&v);
      col.remap.assign(ndict, UINT32_MAX);
      if (ndict >= (size_t(1) << 16) && threads > 1) {
        // large dictionaries (a 10M-value group column): values already known are looked up in parallel -- reads
        // only, under this thread's lock -- and only the new ones interned below, in order (ids stay deterministic)
        const size_t blk = (ndict + size_t(threads) * 4 - 1) / (size_t(threads) * 4);
        parallel_for((ndict + blk - 1) / blk, threads, [&](size_t b) {
          for (size_t i = b * blk; i < std::min(ndict, (b + 1) * blk); i++) {
            auto it = gd.ids.find(std::string(*sv[i]));
            if (it != gd.ids.end()) col.remap[i] = it->second;
          }
        });
      }
      for (size_t i = 0; i < ndict; i++)
        if (col.remap[i] == UINT32_MAX) col.remap[i] = gd.intern(std::string(*sv[i]));
    }
    uint32_t remap_base = 0;
    for (size_t rg = 0; rg < nrg; rg++) {
      ChunkOut& C = chunks[ci * nrg + rg];
      const uint32_t run_base = uint32_t(col.runs.size());
      const uint64_t base = chunk_base[ci * nrg + rg];
      page0[ci][rg] = pages[ci].size();
      col.runs.insert(col.runs.end(), C.runs.begin(), C.runs.end());
      col.compressed_bytes += C.compressed;
      for (HostPage& hp : C.pages) {
        hp.run_lo += run_base;
        hp.drun_lo += run_base;
        hp.d.vals += base;
        if (hp.d.has_nulls) hp.d.defs += base;
        if (hp.d.kind == PAGE_DICT) hp.d.remap += remap_base;
        pages[ci].push_back(std::move(hp));
      }
      remap_base += uint32_t(C.dict.size());
      std::vector<RunDesc>().swap(C.runs);
    }
  });

  // ---- 3. tiles, per row group in parallel ----
  std::vector<std::vector<TileDesc>> rg_tiles(nrg);
  std::vector<std::vector<std::vector<TileCol>>> rg_tcols(nrg);
  if (S->num_rows > 0 && nc) {
    parallel_for(nrg, threads, [&](size_t rg) {
      std::vector<size_t> p0(nc);
      for (size_t c = 0; c < nc; c++) p0[c] = page0[c][rg];
      build_tiles_rg(*S, pages, uint32_t(rg), p0, rg_tiles[rg], rg_tcols[rg]);
    });
    for (size_t rg = 0; rg < nrg; rg++) {
      S->tiles.insert(S->tiles.end(), rg_tiles[rg].begin(), rg_tiles[rg].end());
      for (size_t c = 0; c < nc; c++)
        S->cols[c].tcols.insert(S->cols[c].tcols.end(), rg_tcols[rg][c].begin(), rg_tcols[rg][c].end());
    }
  }
  for (size_t ci = 0; ci < nc; ci++) {
    auto& col = S->cols[ci];
    col.pages.reserve(pages[ci].size());
    for (auto& hp : pages[ci]) col.pages.push_back(hp.d);
  }
  const double host_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();

  // ---- 4. upload: the streams through the pinned staging area (filled in parallel), then the metadata blob ----
  std::lock_guard<std::mutex> dg(dev_mu);
  HIP_CHECK(hipSetDevice(device));
  if (!load_stream) HIP_CHECK(hipStreamCreateWithFlags(&load_stream, hipStreamNonBlocking));
  HIP_CHECK(hipMalloc(&S->d_data, S->data_bytes));
  {
    // every stream, with its destination offset, cut at staging-piece boundaries
    struct Copy {
      const uint8_t* src;
      size_t len;
      size_t dst;
    };
    std::vector<Copy> copies;
    for (size_t k = 0; k < chunks.size(); k++)
      for (const StreamRef& r : chunks[k].streams) copies.push_back(Copy{r.src, r.len, chunk_base[k] + r.off});
    // (the piece walk below needs them in destination order)
    std::sort(copies.begin(), copies.end(), [](const Copy& a, const Copy& b) { return a.dst < b.dst; });
    const size_t piece = std::min<size_t>(S->data_bytes, size_t(1) << 30);
    if (load_pinned_cap < piece) {
      if (load_pinned) HIP_CHECK(hipHostFree(load_pinned));
      load_pinned = nullptr;
      load_pinned_cap = 0;
      HIP_CHECK(hipHostMalloc(&load_pinned, piece));
      load_pinned_cap = piece;
    }
    uint8_t* pin = static_cast<uint8_t*>(load_pinned);
    size_t ci0 = 0;
    for (size_t lo = 0; lo < S->data_bytes; lo += piece) {
      const size_t hi = std::min(S->data_bytes, lo + piece);
      // the copies overlapping [lo, hi): split into ~8 MB work items
      std::vector<Copy> work;
      while (ci0 < copies.size() && copies[ci0].dst + copies[ci0].len <= lo) ci0++;
      size_t cur = lo;   // the alignment gaps are zeroed (src == nullptr): reads past a stream's end see zeros
      for (size_t c = ci0; c < copies.size() && copies[c].dst < hi; c++) {
        size_t a = std::max(lo, copies[c].dst), b = std::min(hi, copies[c].dst + copies[c].len);
        if (a > cur) work.push_back(Copy{nullptr, a - cur, cur - lo});
        for (size_t x = a; x < b; x += size_t(8) << 20) {
          const size_t y = std::min(b, x + (size_t(8) << 20));
          work.push_back(Copy{copies[c].src + (x - copies[c].dst), y - x, x - lo});
        }
        cur = std::max(cur, b);
      }
      if (cur < hi) work.push_back(Copy{nullptr, hi - cur, cur - lo});
      parallel_for(work.size(), threads, [&](size_t w) {
        if (work[w].src) memcpy(pin + work[w].dst, work[w].src, work[w].len);
        else memset(pin + work[w].dst, 0, work[w].len);
      });
      // explicit stream + synchronize: a copy from pinned memory may still be reading `pin` when a plain hipMemcpy
      // returns, and the next piece (or segment) rewrites it
      HIP_CHECK(hipMemcpyAsync(S->d_data + lo, pin, hi - lo, hipMemcpyHostToDevice, load_stream));
      HIP_CHECK(hipStreamSynchronize(load_stream));
    }
  }
  size_t meta = align_up(S->tiles.size() * sizeof(TileDesc));
  for (auto& c : S->cols) {
    meta += align_up(c.pages.size() * sizeof(PageDesc)) + align_up(c.runs.size() * sizeof(RunDesc)) +
            align_up(c.tcols.size() * sizeof(TileCol)) + align_up(c.remap.size() * sizeof(uint32_t));
  }
  S->meta_bytes = std::max<size_t>(meta, kAlign);
  HIP_CHECK(hipMalloc(&S->d_meta, S->meta_bytes));
  std::vector<uint8_t> blob(S->meta_bytes, 0);
  size_t off = 0;
  auto place = [&](const void* src, size_t n) -> size_t {
    size_t o = off;
    if (n) memcpy(blob.data() + o, src, n);
    off += align_up(n);
    return o;
  };
  uint8_t* base = static_cast<uint8_t*>(S->d_meta);
  S->d_tiles = reinterpret_cast<TileDesc*>(base + place(S->tiles.data(), S->tiles.size() * sizeof(TileDesc)));
  for (auto& c : S->cols) {
    c.d_pages = reinterpret_cast<PageDesc*>(base + place(c.pages.data(), c.pages.size() * sizeof(PageDesc)));
    c.d_runs = reinterpret_cast<RunDesc*>(base + place(c.runs.data(), c.runs.size() * sizeof(RunDesc)));
    c.d_tcols = reinterpret_cast<TileCol*>(base + place(c.tcols.data(), c.tcols.size() * sizeof(TileCol)));
    c.d_remap = reinterpret_cast<uint32_t*>(base + place(c.remap.data(), c.remap.size() * sizeof(uint32_t)));
    c.any_nulls = false;
    c.pages_lean_name = c.pages_lean_late = !c.pages.empty();
    for (auto& p : c.pages) {
      c.any_nulls |= p.has_nulls != 0;
      if (p.kind != PAGE_DICT || p.dict_n > 64 || p.bw < 1 || p.bw > 6) c.pages_lean_name = false;
      if (p.kind != PAGE_DICT || p.bw > 32) c.pages_lean_late = false;
    }
  }
  HIP_CHECK(hipMemcpyAsync(S->d_meta, blob.data(), off, hipMemcpyHostToDevice, load_stream));
  HIP_CHECK(hipStreamSynchronize(load_stream));   // `blob` is freed on return
  // the segment now references its chunk dictionaries' ids (released by ~Segment)
  S->engine = this;
  for (auto& c : S->cols)
    if (c.is_string && !c.remap.empty()) {
      dict_ref(c.name, c.remap.data(), c.remap.size(), +1);
      c.nremap = c.remap.size();
    }
  // host copies no longer needed except what the planner reads
  for (auto& c : S->cols) {
    std::vector<RunDesc>().swap(c.runs);
    std::vector<TileCol>().swap(c.tcols);
    std::vector<uint32_t>().swap(c.remap);
  }
  S->load_host_ms = host_ms;
  S->load_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  return S;
}

size_t Engine::evict_lru_locked(size_t target_bytes, const std::string& keep, std::vector<std::shared_ptr<Segment>>* out) {
  size_t freed = 0;
  while (cache_bytes > target_bytes) {
    auto victim = cache.end();
    for (auto it = cache.begin(); it != cache.end(); ++it)
      if (it->first != keep && (victim == cache.end() || it->second->last_use < victim->second->last_use)) victim = it;
    if (victim == cache.end()) break;
    const size_t b = victim->second->data_bytes + victim->second->meta_bytes;
    cache_bytes -= b;
    freed += b;
    evictions++;
    if (victim->second->from_put) {
      if (evicted_puts.size() >= (size_t(1) << 20)) evicted_puts.clear();   // bounded (then: a missing-file error)
      evicted_puts.insert(victim->first);
    }
    if (out) out->push_back(std::move(victim->second));   // destroyed by the caller after cache_mu
    cache.erase(victim);
  }
  return freed;
}

// build_segment with the file's own faults as LK_ERR_IO: a truncated / corrupt footer, page or run (thrift and
// Parquet parse errors) is a property of that one file -- the evaluation empties only its glob, as DuckDB's failing
// read_parquet does (Commons.scala:249-253) -- while HIP failures and host OOM stay what they are.
static std::shared_ptr<Segment> build_checked(Engine& E, const std::string& key, const uint8_t* data, size_t size) {
  try {
    return E.build_segment(key, data, size);
  } catch (const DeviceError&) {
    throw;
  } catch (const PlanError&) {
    throw;
  } catch (const std::bad_alloc&) {
    throw;
  } catch (const std::exception& e) {
    throw PlanError(LK_ERR_IO, std::string(e.what()) + " (" + key + ")");
  }
}

int Engine::put_segment(const std::string& key, const uint8_t* data, size_t size, bool from_put) {
  std::shared_ptr<Segment> S;
  try {
    S = build_checked(*this, key, data, size);
  } catch (const DeviceError&) {
    // HBM exhausted: make room by evicting least recently used segments (about twice the file), then retry once.
    // The failed hipMalloc left HIP's thread-local last error set: clear it, or the next launch on this thread
    // would report it.
    (void)hipGetLastError();
    std::vector<std::shared_ptr<Segment>> dead;
    {
      std::lock_guard<std::mutex> g(cache_mu);
      const size_t want = 2 * size + (64u << 20);
      if (evict_lru_locked(cache_bytes > want ? cache_bytes - want : 0, key, &dead) == 0) throw;
    }
    dead.clear();   // their HBM is freed (and dictionary references returned) before the retry
    S = build_checked(*this, key, data, size);
  }
  S->last_use = ++use_clock;
  S->from_put = from_put;
  std::vector<std::shared_ptr<Segment>> dead;   // replaced / evicted segments, destroyed after cache_mu
  std::lock_guard<std::mutex> g(cache_mu);
  evicted_puts.erase(key);
  load_host_ms_total += S->load_host_ms;
  load_ms_total += S->load_ms;
  auto it = cache.find(key);
  if (it != cache.end()) {
    cache_bytes -= it->second->data_bytes + it->second->meta_bytes;
    dead.push_back(std::move(it->second));
  }
  cache_bytes += S->data_bytes + S->meta_bytes;
  cache[key] = S;
  if (hbm_budget) evict_lru_locked(hbm_budget, key, &dead);
  return LK_OK;
}

std::shared_ptr<Segment> Engine::get_segment(const std::string& key, bool load_on_miss) {
  {
    std::lock_guard<std::mutex> g(cache_mu);
    auto it = cache.find(key);
    if (it != cache.end()) {
      it->second->last_use = ++use_clock;
      return it->second;
    }
  }
  if (!load_on_miss) return nullptr;
  {
    std::lock_guard<std::mutex> g(cache_mu);
    if (evicted_puts.count(key))
      throw PlanError(LK_ERR_EVICTED, "segment " + key + " was evicted from the HBM cache (lk_segment_put it again)");
  }
  std::ifstream f(key, std::ios::binary);
  if (!f) throw PlanError(LK_ERR_IO, "cannot open segment " + key);
  std::vector<uint8_t> buf((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
  put_segment(key, buf.data(), buf.size(), false);
  std::lock_guard<std::mutex> g(cache_mu);
  return cache[key];
}

// ------------------------------------------------------------------------------------------------
// engine lifecycle + workspace
// ------------------------------------------------------------------------------------------------
Engine::Engine(int dev) : device(dev) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) throw DeviceError("no HIP device available");
  if (dev < 0 || dev >= n) throw DeviceError("device index out of range");
  HIP_CHECK(hipSetDevice(device));
  ctx_free.push_back(std::make_unique<CallCtx>(device));   // one context up front: fail here, not mid-query
  ctx_made = 1;
}

Engine::~Engine() {
  life.reset();   // results' weak references expire first
  (void)hipSetDevice(device);
  comm_destroy();
  ctx_free.clear();
  cache.clear();
  if (load_pinned) (void)hipHostFree(load_pinned);
  if (load_stream) (void)hipStreamDestroy(load_stream);
}

std::unique_ptr<CallCtx> Engine::acquire_ctx() {
  std::unique_lock<std::mutex> g(ctx_mu);
  for (;;) {
    if (!ctx_free.empty()) {
      auto c = std::move(ctx_free.back());
      ctx_free.pop_back();
      return c;
    }
    if (ctx_made < max_calls) {
      ctx_made++;
      g.unlock();
      try {
        return std::make_unique<CallCtx>(device);
      } catch (...) {
        std::lock_guard<std::mutex> g2(ctx_mu);
        ctx_made--;
        throw;
      }
    }
    ctx_cv.wait(g);
  }
}

void Engine::release_ctx(std::unique_ptr<CallCtx> c) {
  if (!c) return;
  {
    std::lock_guard<std::mutex> g(ctx_mu);
    ctx_free.push_back(std::move(c));
  }
  ctx_cv.notify_one();
}

std::shared_ptr<LeafBits> Engine::leaf_bits(const std::string& key) {
  std::lock_guard<std::mutex> g(leaf_mu);
  auto& slot = leaf_cache[key];
  if (!slot) {
    slot = std::make_shared<LeafBits>();
    if (leaf_cache.size() > 256) {   // bounded: drop entries nobody holds (a query re-fills what it needs)
      for (auto it = leaf_cache.begin(); it != leaf_cache.end() && leaf_cache.size() > 128;) {
        if (it->first != key && it->second.use_count() == 1) it = leaf_cache.erase(it);
        else ++it;
      }
    }
  }
  return slot;
}

CallCtx::CallCtx(int dev) : device(dev) {
  HIP_CHECK(hipSetDevice(device));
  HIP_CHECK(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
  HIP_CHECK(hipEventCreate(&ev_scan0));
  HIP_CHECK(hipEventCreate(&ev_scan1));
  HIP_CHECK(hipHostMalloc(&pinned, pinned_cap = 1 << 20));
}

CallCtx::~CallCtx() {
  (void)hipSetDevice(device);
  if (stream) (void)hipStreamSynchronize(stream);
  for (auto& w : ws)
    if (w.second.p) (void)hipFree(w.second.p);
  if (pinned) (void)hipHostFree(pinned);
  if (comm_pin) (void)hipHostFree(comm_pin);
  if (ev_scan0) (void)hipEventDestroy(ev_scan0);
  if (ev_scan1) (void)hipEventDestroy(ev_scan1);
  if (stream) (void)hipStreamDestroy(stream);
}

void* CallCtx::workspace(const std::string& name, size_t bytes) {
  auto& w = ws[name];
  if (w.cap < bytes) {
    const size_t old_cap = w.cap;   // growth is 1.5x of the old capacity, so a growing workspace reallocates rarely
    if (w.p) {
      CTX_CHECK(hipStreamSynchronize(stream));   // earlier work of this call may still read it
      CTX_CHECK(hipFree(w.p));
      w.p = nullptr;
      w.cap = 0;
    }
    const size_t cap = align_up(std::max(bytes, old_cap * 3 / 2), 1 << 20);
    hipError_t e = hipMalloc(&w.p, cap);
    if (e != hipSuccess) {
      (void)hipGetLastError();
      w.p = nullptr;
      throw PlanError(LK_ERR_MEMORY, "HBM: cannot allocate " + std::to_string(cap) + " bytes of workspace '" + name + "'");
    }
    w.cap = cap;
  }
  return w.p;
}

void* CallCtx::pinned_buf(size_t bytes) {
  if (pinned_cap < bytes) {
    CTX_CHECK(hipStreamSynchronize(stream));
    CTX_CHECK(hipHostFree(pinned));
    pinned = nullptr;
    pinned_cap = 0;
    const size_t cap = align_up(bytes, 1 << 20);
    CTX_CHECK(hipHostMalloc(&pinned, cap));
    pinned_cap = cap;
  }
  return pinned;
}

}  // namespace lk
