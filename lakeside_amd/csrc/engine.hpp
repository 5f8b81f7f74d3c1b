// Engine state shared by engine.cpp (segment cache), eval.cpp (query evaluation), comm.cpp (RCCL).
#pragma once
#include <hip/hip_runtime.h>

#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <set>
#include <string>
#include <unordered_map>
#include <vector>

#include "layout.hpp"
#include "plan.hpp"

namespace lk {

void set_error(const std::string& m);

// Engine-global dictionary of one column name.  Values get dense ids in first-seen order; a deque keeps
// every string at a stable address (result tag values point into it).
struct GlobalDict {
  std::mutex mu;
  std::unordered_map<std::string, uint32_t> ids;
  std::deque<std::string> vals;
  uint32_t intern(const std::string& s);   // caller holds mu
};

struct HostCol {
  std::string name;
  int ptype = -1;
  bool nullable = false;
  bool is_string = false;
  bool unsupported = false;
  bool any_nulls = false;
  uint64_t compressed_bytes = 0;          // Σ ColumnMetaData.total_compressed_size (algorithmic bytes)
  std::vector<PageDesc> pages;            // host copy (planner reads dict sizes / null flags)
  std::vector<RunDesc> runs;              // load-time only
  std::vector<TileCol> tcols;             // load-time only
  std::vector<uint32_t> remap;            // load-time only
  PageDesc* d_pages = nullptr;
  RunDesc* d_runs = nullptr;
  TileCol* d_tcols = nullptr;
  uint32_t* d_remap = nullptr;
};

struct Segment {
  std::string key;
  int64_t num_rows = 0;
  std::vector<int64_t> rg_rows;
  std::vector<HostCol> cols;                     // loadable columns
  std::set<std::string> all_columns;             // every column of the file (DESCRIBE, Commons.scala:214-221)
  std::unordered_map<std::string, int> by_name;
  std::vector<TileDesc> tiles;
  TileDesc* d_tiles = nullptr;
  uint8_t* d_data = nullptr;                     // page streams (def levels / values), 16-B aligned
  size_t data_bytes = 0;
  void* d_meta = nullptr;
  size_t meta_bytes = 0;
  int col_index(const std::string& name) const;
  ~Segment();
};

struct Workspace {
  void* p = nullptr;
  size_t cap = 0;
};

struct Comm;   // comm.cpp

struct Engine {
  int device = 0;
  hipStream_t stream = nullptr;
  hipEvent_t ev_scan0 = nullptr, ev_scan1 = nullptr;
  std::mutex eval_mu;                            // one evaluation at a time per engine (round 1)
  std::mutex dev_mu;
  std::mutex cache_mu;
  std::unordered_map<std::string, std::shared_ptr<Segment>> cache;
  size_t cache_bytes = 0;
  std::mutex dict_mu;
  std::unordered_map<std::string, std::unique_ptr<GlobalDict>> dicts;
  std::map<std::string, Workspace> ws;
  void* pinned = nullptr;
  size_t pinned_cap = 0;
  Comm* comm = nullptr;

  explicit Engine(int dev);
  ~Engine();
  GlobalDict& dict(const std::string& col);
  std::shared_ptr<Segment> build_segment(const std::string& key, const uint8_t* data, size_t size);
  int put_segment(const std::string& key, const uint8_t* data, size_t size);
  std::shared_ptr<Segment> get_segment(const std::string& key, bool load_on_miss);
  void* workspace(const std::string& name, size_t bytes);
  void* pinned_buf(size_t bytes);
  void comm_destroy();
};

}  // namespace lk

struct lk_engine {
  std::unique_ptr<lk::Engine> e;
};

struct lk_result {
  std::vector<int64_t> ts;
  std::vector<double> val;
  std::vector<uint32_t> glob;
  std::vector<std::string> tag_names;
  std::vector<const char*> tag_vals;             // row-major: rows x tag columns
  std::deque<std::string> owned;                 // strings not owned by a dictionary
  std::string stats;
};
