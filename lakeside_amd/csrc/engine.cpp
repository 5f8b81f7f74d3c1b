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
#include "loader.hpp"
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

// ------------------------------------------------------------------------------------------------
// engine-global dictionaries: one per column name; chunk dictionaries remap into them at load
// ------------------------------------------------------------------------------------------------

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
  IdMap ids(nv.get());
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
      ids.emplace(map[i]);
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
  HostLoad H = load_host(key, F, size, load_thread_count(), [this](const std::string& c) -> GlobalDict& { return dict(c); });
  auto S = std::make_shared<Segment>();
  static_cast<SegmentData&>(*S) = std::move(H.seg);
  const int threads = load_thread_count();
  // ---- 4. upload: the streams through the pinned staging area (filled in parallel), then the metadata blob ----
  std::lock_guard<std::mutex> dg(dev_mu);
  HIP_CHECK(hipSetDevice(device));
  if (!load_stream) HIP_CHECK(hipStreamCreateWithFlags(&load_stream, hipStreamNonBlocking));
  HIP_CHECK(hipMalloc(&S->d_data, S->data_bytes));
  {
    const size_t piece = std::min<size_t>(S->data_bytes, size_t(1) << 30);
    if (load_pinned_cap < piece) {
      if (load_pinned) HIP_CHECK(hipHostFree(load_pinned));
      load_pinned = nullptr;
      load_pinned_cap = 0;
      HIP_CHECK(hipHostMalloc(&load_pinned, piece));
      load_pinned_cap = piece;
    }
    uint8_t* pin = static_cast<uint8_t*>(load_pinned);
    StagePlan plan(H);
    for (size_t lo = 0; lo < S->data_bytes; lo += piece) {
      const size_t hi = std::min(S->data_bytes, lo + piece);
      plan.stage(pin, lo, hi, threads);   // [lo, hi) of the stream area into the pinned piece (gaps zeroed)
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
  S->load_host_ms = H.host_ms;
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
  std::ifstream f(key, std::ios::binary);
  if (!f) {
    // an evicted lk_segment_put key that is not a readable file: the caller must put it again (LK_ERR_EVICTED); a put
    // key that is also a real path is simply reloaded from the file below, as any cache miss
    std::lock_guard<std::mutex> g(cache_mu);
    if (evicted_puts.count(key))
      throw PlanError(LK_ERR_EVICTED, "segment " + key + " was evicted from the HBM cache (lk_segment_put it again)");
    throw PlanError(LK_ERR_IO, "cannot open segment " + key);
  }
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
  // results' weak references expire first; a result still reading through the engine (lk_result_tag_dictionary holds
  // the token while it calls dict_ptrs) finishes before anything is torn down
  {
    std::weak_ptr<const char> w = life;
    life.reset();
    while (!w.expired()) std::this_thread::yield();
  }
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
  HIP_CHECK(hipEventCreateWithFlags(&ev_rows, hipEventDisableTiming));
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
  if (ev_rows) (void)hipEventDestroy(ev_rows);
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
