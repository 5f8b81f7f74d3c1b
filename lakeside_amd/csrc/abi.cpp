// extern "C" surface of include/lakeside_gpu.h: argument checks, exception -> status translation.
#include <cstring>
#include <exception>
#include <new>
#include <shared_mutex>
#include <string>

#include "../../include/lakeside_gpu.h"
#include "comm.hpp"
#include "engine.hpp"
#include "json.hpp"
#include "plan.hpp"

namespace lk {
int evaluate(Engine& E, const std::string& json, const char* const* paths, size_t n_paths, int glob_size,
             unsigned flags, const int32_t* shard, bool dist, lk_result* res);
}

namespace {
thread_local std::string t_err;

template <class F>
int guarded(F&& f) {
  try {
    return f();
  } catch (const lk::PlanError& e) {
    t_err = e.what();
    return e.code;
  } catch (const lk::JsonError& e) {
    t_err = e.what();
    return LK_ERR_ARG;
  } catch (const std::bad_alloc&) {
    t_err = "out of host memory";
    return LK_ERR_MEMORY;
  } catch (const std::exception& e) {
    t_err = e.what();
    std::string m = e.what();
    if (m.rfind("HIP", 0) == 0 || m.find("device") != std::string::npos) return LK_ERR_DEVICE;
    if (m.rfind("parquet", 0) == 0 || m.rfind("thrift", 0) == 0) return LK_ERR_IO;
    return LK_ERR_ARG;
  }
}
}  // namespace

namespace lk {
void set_error(const std::string& m) { t_err = m; }
}

extern "C" {

const char* lk_last_error(void) { return t_err.c_str(); }

int lk_engine_create(const char* options_json, lk_engine** out) {
  if (!out) return LK_ERR_ARG;
  *out = nullptr;
  return guarded([&] {
    int dev = 0;
    if (options_json && *options_json) {
      lk::Json o = lk::Json::parse(options_json);
      if (const lk::Json* d = o.get("device")) dev = int(d->as_i64());
    }
    auto* e = new lk_engine();
    try {
      e->e = std::make_unique<lk::Engine>(dev);
      if (options_json && *options_json) {
        lk::Json o = lk::Json::parse(options_json);
        if (const lk::Json* b = o.get("hbm_budget_bytes")) e->e->hbm_budget = size_t(b->as_i64());
        if (const lk::Json* c = o.get("max_calls")) e->e->max_calls = size_t(std::max<int64_t>(1, c->as_i64()));
        if (const lk::Json* d = o.get("dict_compact_min_dead"))
          e->e->compact_min_dead = size_t(std::max<int64_t>(1, d->as_i64()));
        if (const lk::Json* t = o.get("load_threads"))
          e->e->load_threads = int(std::min<int64_t>(64, std::max<int64_t>(0, t->as_i64())));
      }
    } catch (...) {
      delete e;
      throw;
    }
    *out = e;
    return LK_OK;
  });
}

void lk_engine_destroy(lk_engine* e) { delete e; }

// Loads, evictions and evaluations hold the engine's dictionary generation shared (a compaction renumbers ids only
// between them); each first compacts dictionaries that evictions have left mostly dead.
int lk_segment_put(lk_engine* e, const char* key, const uint8_t* data, size_t size) {
  if (!e || !key || (!data && size)) return LK_ERR_ARG;
  return guarded([&] {
    e->e->maybe_compact();
    std::shared_lock<std::shared_mutex> gen(e->e->gen_mu);
    return e->e->put_segment(key, data, size);
  });
}

int lk_segment_load(lk_engine* e, const char* path) {
  if (!e || !path) return LK_ERR_ARG;
  return guarded([&] {
    e->e->maybe_compact();
    std::shared_lock<std::shared_mutex> gen(e->e->gen_mu);
    e->e->get_segment(path, true);
    return LK_OK;
  });
}

int lk_segment_evict(lk_engine* e, const char* key) {
  if (!e || !key) return LK_ERR_ARG;
  return guarded([&] {
    std::shared_lock<std::shared_mutex> gen(e->e->gen_mu);
    std::shared_ptr<lk::Segment> victim;   // released after cache_mu (~Segment returns its dictionary references)
    {
      std::lock_guard<std::mutex> g(e->e->cache_mu);
      e->e->evicted_puts.erase(key);   // the caller dropped the key itself
      auto it = e->e->cache.find(key);
      if (it == e->e->cache.end()) return int(LK_ERR_ARG);
      e->e->cache_bytes -= it->second->data_bytes + it->second->meta_bytes;
      victim = std::move(it->second);
      e->e->cache.erase(it);
    }
    return int(LK_OK);
  });
}

const char* lk_engine_stats(lk_engine* e) {
  if (!e) return nullptr;
  lk::Engine& E = *e->e;
  std::string o = "{";
  {
    std::lock_guard<std::mutex> g(E.cache_mu);
    o += "\"segments\":" + std::to_string(E.cache.size()) + ",\"segment_bytes\":" + std::to_string(E.cache_bytes) +
         ",\"evictions\":" + std::to_string(E.evictions) + ",\"load_ms\":" + std::to_string(E.load_ms_total) +
         ",\"load_host_ms\":" + std::to_string(E.load_host_ms_total);
  }
  o += ",\"dict_compactions\":" + std::to_string(E.compactions) + ",\"dictionaries\":{";
  {
    std::lock_guard<std::mutex> g(E.dict_mu);
    bool first = true;
    for (auto& kv : E.dicts) {
      std::lock_guard<std::mutex> dg(kv.second->mu);
      if (!first) o += ",";
      first = false;
      std::string name;
      for (char c : kv.first) {
        if (c == '"' || c == '\\') name += '\\';
        if (static_cast<unsigned char>(c) >= 0x20) name += c;
      }
      o += "\"" + name + "\":{\"size\":" + std::to_string(kv.second->size()) + ",\"live\":" +
           std::to_string(kv.second->live) + ",\"generation\":" + std::to_string(kv.second->gen) + "}";
    }
  }
  o += "}";
  o += ",\"comm\":" + lk::comm_describe(E);   // the description cached at lk_comm_init* (not under comm_mu)
  o += "}";
  t_err.clear();
  static thread_local std::string t_stats;
  t_stats = o;
  return t_stats.c_str();
}

int lk_engine_drop_caches(lk_engine* e) {
  if (!e) return LK_ERR_ARG;
  lk::Engine& E = *e->e;
  std::unique_lock<std::shared_mutex> gen(E.gen_mu);   // no evaluation in flight
  std::lock_guard<std::mutex> cm(E.comm_mu);
  {
    std::lock_guard<std::mutex> g(E.parsed_mu);
    E.parsed.clear();
  }
  {
    std::lock_guard<std::mutex> g(E.leaf_mu);
    E.leaf_cache.clear();
  }
  {
    std::lock_guard<std::mutex> g(E.order_mu);
    E.orders.clear();
  }
  {
    std::lock_guard<std::mutex> g(E.ptrs_mu);
    E.ptrs.clear();
  }
  E.unions.clear();
  t_err.clear();
  return LK_OK;
}

size_t lk_segment_count(const lk_engine* e) {
  if (!e) return 0;
  std::lock_guard<std::mutex> g(e->e->cache_mu);
  return e->e->cache.size();
}
size_t lk_segment_bytes(const lk_engine* e) {
  if (!e) return 0;
  std::lock_guard<std::mutex> g(e->e->cache_mu);
  return e->e->cache_bytes;
}

static int eval_common(lk_engine* e, const char* json, const char* const* paths, size_t n_paths, const int32_t* shard,
                       int glob_size, unsigned flags, bool dist, lk_result** out) {
  if (!e || !json || !out || (n_paths && !paths)) return LK_ERR_ARG;
  *out = nullptr;
  return guarded([&] {
    e->e->maybe_compact();
    std::shared_lock<std::shared_mutex> gen(e->e->gen_mu);
    auto* r = new lk_result();
    try {
      lk::evaluate(*e->e, json, paths, n_paths, glob_size, flags, shard, dist, r);
    } catch (...) {
      delete r;
      throw;
    }
    *out = r;
    return LK_OK;
  });
}

int lk_eval_pushdown(lk_engine* e, const char* push_down_json, const char* const* paths, size_t n_paths, int glob_size,
                     unsigned flags, lk_result** out) {
  return eval_common(e, push_down_json, paths, n_paths, nullptr, glob_size, flags, false, out);
}

int lk_eval_pushdown_dist(lk_engine* e, const char* push_down_json, const char* const* paths, size_t n_paths,
                          const int32_t* shard, int glob_size, lk_result** out) {
  return eval_common(e, push_down_json, paths, n_paths, shard, glob_size, LK_MERGED, true, out);
}

size_t lk_result_num_rows(const lk_result* r) { return r ? r->nrows : 0; }
const int64_t* lk_result_timestamps(const lk_result* r) { return r ? r->ts : nullptr; }
const double* lk_result_values(const lk_result* r) { return r ? r->val : nullptr; }
const uint32_t* lk_result_globs(const lk_result* r) { return r ? r->glob : nullptr; }
size_t lk_result_num_tag_columns(const lk_result* r) { return r ? r->tag_names.size() : 0; }
const char* lk_result_tag_name(const lk_result* r, size_t col) {
  return (r && col < r->tag_names.size()) ? r->tag_names[col].c_str() : nullptr;
}
const char* lk_result_tag_value(const lk_result* r, size_t row, size_t col) {
  if (!r || row >= r->nrows || col >= r->tag_names.size()) return nullptr;
  return r->tag(row, col);
}
const uint32_t* lk_result_group_ids(const lk_result* r) { return r ? r->gid : nullptr; }
size_t lk_result_num_group_columns(const lk_result* r) { return (r && !r->exemplar) ? r->tcols.size() : 0; }
const char* const* lk_result_tag_dictionary(const lk_result* r, size_t col, uint64_t* stride, uint64_t* ndim) {
  if (stride) *stride = 1;
  if (ndim) *ndim = 0;
  if (!r || r->exemplar || col >= r->tcols.size()) return nullptr;
  try {
    const std::vector<const char*>* v = r->tag_dictionary(col);
    if (!v) return nullptr;
    if (stride) *stride = r->tcols[col].stride;
    if (ndim) *ndim = r->tcols[col].ndim;
    return v->data();
  } catch (const std::exception& e) {
    t_err = e.what();
    return nullptr;
  }
}
const char* lk_result_stats(const lk_result* r) { return r ? r->stats.c_str() : nullptr; }
const uint8_t* lk_result_sketch(const lk_result* r, size_t row, size_t* len) {
  if (len) *len = 0;
  if (!r || row >= r->sketches.size()) return nullptr;
  if (len) *len = r->sketches[row].size();
  return reinterpret_cast<const uint8_t*>(r->sketches[row].data());
}
void lk_result_free(lk_result* r) { delete r; }

}  // extern "C"
