// Distributed group-dim agreement for unrestricted group dimensions.
//
// Reference: segments go to worker pods by Math.floorMod(segmentId.hashCode, pods) (core/.../discovery/
// WorkerManager.scala:150-156), every pod answers per (timestamp, tags) and the query-api merges rows whose tag maps
// are equal (TimeGroupedSketchAggregator.scala:74-114).  Here the ranks' partial tables must share one cell space, so
// a group column's values get dim ids every rank agrees on -- without shipping and sorting dictionaries of strings:
//   * each rank keys its dictionary values by 128-bit MurmurHash3 (Engine::dict_order: radix-sorted keys, cached
//     per dictionary size) and fingerprints the sorted key set;
//   * one all-gather of (n, fingerprint) per query; when it matches the cached agreement on every rank the cached
//     union is reused (steady state: a few tens of microseconds);
//   * otherwise, the sorted key arrays are all-gathered and merged into their sorted union U (dim id = position in
//     U; identical on every rank), each rank maps its global ids to U positions by a merge walk, and each value that
//     rank 0 lacks is shipped once, by the lowest rank holding it, so every rank can print every dim's tag text.
// Ties within a timestamp are unordered in the reference (S17), so hash order is as good an order as string order.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "../../include/lakeside_gpu.h"
#include "comm.hpp"
#include "engine.hpp"
#include "plan.hpp"

namespace lk {

namespace {
// fn(a, b) over [0, n) cut into ranges on up to `threads` threads (the calling thread among them); small n inline
template <class F>
void par_ranges(size_t n, int threads, F&& fn) {
  const size_t T = n < (size_t(1) << 16) ? 1 : size_t(std::max(1, threads));
  if (T <= 1) {
    fn(size_t(0), n);
    return;
  }
  const size_t per = (n + T - 1) / T;
  std::vector<std::thread> pool;
  for (size_t t = 1; t < T; t++)
    if (t * per < n) pool.emplace_back([&, t] { fn(t * per, std::min(n, (t + 1) * per)); });
  fn(size_t(0), std::min(n, per));
  for (auto& th : pool) th.join();
}
}  // namespace

namespace {

double ms_since_d(std::chrono::steady_clock::time_point t0) {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

// sorted-unique union of sorted-unique key arrays (pairwise tree of merges)
std::vector<Key128> union_of(std::vector<std::vector<Key128>> parts) {
  if (parts.empty()) return {};
  while (parts.size() > 1) {
    std::vector<std::vector<Key128>> next;
    for (size_t i = 0; i + 1 < parts.size(); i += 2) {
      std::vector<Key128> m;
      m.reserve(parts[i].size() + parts[i + 1].size());
      std::set_union(parts[i].begin(), parts[i].end(), parts[i + 1].begin(), parts[i + 1].end(), std::back_inserter(m));
      next.push_back(std::move(m));
    }
    if (parts.size() % 2) next.push_back(std::move(parts.back()));
    parts.swap(next);
  }
  return std::move(parts[0]);
}

}  // namespace

std::shared_ptr<DimUnion> agree_dim_union(Engine& E, CallCtx& X, const std::string& col, uint32_t dict_n,
                                          double& agree_ms, bool& rebuilt) {
  const auto t0 = std::chrono::steady_clock::now();
  rebuilt = false;
  const int W = comm_world(E), me = comm_rank(E);
  // 1. every rank's (status, n, fingerprint): a rank-local failure (a 128-bit key collision) fails every rank here
  std::shared_ptr<const DictOrder> order;
  int err = 0;
  std::string msg;
  try {
    order = E.dict_order(col, dict_n);
  } catch (const PlanError& e) {
    err = e.code;
    msg = e.what();
  }
  // payload: n (8) | fingerprint (16) | this rank's cached agreement key (the exact string, W x 24 bytes); the status
  // travels in front (comm_allgather_status)
  std::shared_ptr<DimUnion>& slot = E.unions[col];
  std::string mine(24, '\0');
  {
    const uint64_t n = dict_n, f0 = order ? order->fp[0] : 0, f1 = order ? order->fp[1] : 0;
    memcpy(&mine[0], &n, 8);
    memcpy(&mine[8], &f0, 8);
    memcpy(&mine[16], &f1, 8);
  }
  const std::string fp_mine = mine;
  if (slot) mine += slot->agree_key;
  const std::vector<std::string> all = comm_allgather_status(E, X, err, msg, mine);
  std::string agree_key;
  bool same = true;
  for (int r = 0; r < W; r++) {
    if (all[size_t(r)].size() < 24) throw PlanError(LK_ERR_DEVICE, "internal: short dictionary fingerprint");
    agree_key += all[size_t(r)].substr(0, 24);
    if (all[size_t(r)].substr(0, 24) != fp_mine) same = false;
  }
  // 2. the cached agreement is reused only when every rank holds exactly this one: decided from exchanged data alone
  // (each rank's cached key travelled in full), so every rank reaches the same decision without another collective
  // (a local-only comparison could split the ranks)
  bool all_hit = true;
  for (int r = 0; r < W; r++) all_hit = all_hit && all[size_t(r)].compare(24, std::string::npos, agree_key) == 0;
  (void)me;
  if (all_hit) {
    agree_ms = ms_since_d(t0);
    return slot;
  }
  rebuilt = true;
  auto u = std::make_shared<DimUnion>();
  u->agree_key = agree_key;
  u->dict_n = dict_n;
  u->order = order;
  u->device = E.device;
  GlobalDict& gd = E.dict(col);
  auto dim_of_gid = std::make_shared<std::vector<uint32_t>>(dict_n);
  std::vector<const std::string*> own(dict_n);
  {
    std::lock_guard<std::mutex> g(gd.mu);
    for (uint32_t i = 0; i < dict_n; i++) own[i] = &gd[i];   // stable addresses
    u->strs = gd.vals;   // `text` points into this block: it outlives a dictionary compaction with the union
  }
  auto text_of = [](const std::string* s) -> const char* {
    return (s->empty() || *s == "null") ? nullptr : s->c_str();
  };
  if (same) {
    // every rank holds the same value set: U = this rank's sorted keys, nothing to exchange
    u->size = dict_n;
    u->text = std::make_shared<std::vector<const char*>>(size_t(dict_n) + 1, nullptr);
    // (10M values: one cache miss per string, so the walk runs on the load threads)
    std::vector<const char*>& text = *u->text;
    const DictOrder& o = *order;
    par_ranges(dict_n, E.load_thread_count(), [&](size_t a, size_t b) {
      for (size_t d = a; d < b; d++) text[d] = text_of(own[o.perm[d]]);
    });
    *dim_of_gid = order->rank;
  } else {
    // 3. all-gather the sorted key sets, merge them into U
    const std::string keys_blob(reinterpret_cast<const char*>(order->keys.data()), order->keys.size() * sizeof(Key128));
    const std::vector<std::string> kall = comm_allgather_bytes(E, X, keys_blob);
    std::vector<std::vector<Key128>> parts(static_cast<size_t>(W));
    for (int r = 0; r < W; r++) {
      const std::string& b = kall[size_t(r)];
      parts[size_t(r)].resize(b.size() / sizeof(Key128));
      if (!b.empty()) memcpy(parts[size_t(r)].data(), b.data(), parts[size_t(r)].size() * sizeof(Key128));
    }
    const std::vector<Key128> U = union_of(parts);
    if (U.size() + 1 > DIM_MASK) throw PlanError(LK_ERR_UNSUPPORTED, "group dimension " + col + " too large");
    u->size = uint32_t(U.size());
    u->text = std::make_shared<std::vector<const char*>>(U.size() + 1, nullptr);
    // 4. this rank's global ids -> U positions (merge walk: both sorted); its own values' text
    std::vector<uint32_t> pos_of_key(order->keys.size());
    {
      const DictOrder& o = *order;
      std::vector<uint32_t>& dg = *dim_of_gid;
      std::vector<const char*>& text = *u->text;
      par_ranges(o.keys.size(), E.load_thread_count(), [&](size_t a, size_t b) {   // each range: its own merge walk
        size_t j = a < b ? size_t(std::lower_bound(U.begin(), U.end(), o.keys[a]) - U.begin()) : 0;
        for (size_t i = a; i < b; i++) {
          while (U[j] < o.keys[i]) j++;
          pos_of_key[i] = uint32_t(j);
          dg[o.perm[i]] = uint32_t(j);
          text[j] = text_of(own[o.perm[i]]);
        }
      });
    }
    // 5. the values rank 0 lacks, each shipped once by its lowest holder: (position, length, bytes) records
    std::string ship;
    if (me > 0) {
      std::vector<size_t> cur(static_cast<size_t>(me), 0);
      for (size_t i = 0; i < order->keys.size(); i++) {
        const Key128& k = order->keys[i];
        bool lower = false;
        for (int r = 0; r < me && !lower; r++) {   // held by a lower rank? (merge walk per lower rank)
          const std::vector<Key128>& p = parts[size_t(r)];
          size_t& c = cur[size_t(r)];
          while (c < p.size() && p[c] < k) c++;
          lower = c < p.size() && p[c] == k;
        }
        if (lower) continue;
        const std::string& s = *own[order->perm[i]];
        const uint32_t pos = pos_of_key[i], len = uint32_t(s.size());
        ship.append(reinterpret_cast<const char*>(&pos), 4);
        ship.append(reinterpret_cast<const char*>(&len), 4);
        ship.append(s);
      }
    }
    for (const std::string& b : comm_allgather_bytes(E, X, ship)) {
      size_t o = 0;
      while (o + 8 <= b.size()) {
        uint32_t pos, len;
        memcpy(&pos, b.data() + o, 4);
        memcpy(&len, b.data() + o + 4, 4);
        o += 8;
        if (pos >= U.size() || o + len > b.size()) throw PlanError(LK_ERR_DEVICE, "internal: bad dictionary shipment");
        if (!(*u->text)[pos]) {
          u->owned.emplace_back(b, o, len);
          const std::string& s = u->owned.back();
          if (!s.empty() && s != "null") (*u->text)[pos] = s.c_str();
        }
        o += len;
      }
    }
  }
  u->dim_of_gid = dim_of_gid;
  // 6. the scan's lookup table (global id -> dim id) stays resident in HBM with the agreement; a rank that cannot
  // place it fails every rank (one status all-gather: nobody is left in a later collective)
  int up_err = 0;
  if (dict_n) {
    if (hipMalloc(&u->d_dim_of_gid, size_t(dict_n) * 4) != hipSuccess) {
      (void)hipGetLastError();
      u->d_dim_of_gid = nullptr;
      up_err = LK_ERR_MEMORY;
    } else if (hipMemcpy(u->d_dim_of_gid, dim_of_gid->data(), size_t(dict_n) * 4, hipMemcpyHostToDevice) != hipSuccess) {
      (void)hipGetLastError();
      up_err = LK_ERR_DEVICE;
    }
  }
  comm_agree(E, X, up_err, "HBM: group-dim table of " + col);
  slot = u;
  agree_ms = ms_since_d(t0);
  return u;
}

}  // namespace lk
