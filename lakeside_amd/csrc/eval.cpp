// Query evaluation: PushDownRequest -> per-glob plan -> scan kernel -> (RCCL merge) -> finalize -> rows.
//
// Semantics: globs of `glob_size` segments in request order (Commons.scala:361-366);
// per glob the column union decides nonExistentFields (Commons.scala:214-224) -> literal `false` leaves
// (BaseExpr.scala:462-464) and dropped groupBys (338-346); a column the SQL references that no file of the
// glob has is a DuckDB Binder Error -> empty glob (Commons.scala:249-253); window [min startTs, max endTs)
// (Commons.scala:225-226); step of the glob head (Commons.scala:232); bucket ts - ts % step (logs/traces,
// BaseExpr.scala:163-165) or raw ts (metrics, 376-394); sum/min/max/count ignore NULL values, a group whose
// values are all NULL reads back 0.0 (Commons.scala:427); tags drop NULL/"null"/"" (Commons.scala:433) and
// fall back to the glob head's queryTags (450-452).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <climits>
#include <cmath>
#include <cstring>
#include <unordered_set>
#include <string>
#include <vector>

#include "../../include/lakeside_gpu.h"
#include "comm.hpp"
#include "engine.hpp"
#include "kernels.hpp"
#include "layout.hpp"
#include "parquet.hpp"
#include "plan.hpp"
#include "ddsketch.hpp"
#include "hll.hpp"
#include "regex.hpp"
#include "evalutil.hpp"

namespace lk {

#define HIP_TRY(x)                                                                              \
  do {                                                                                          \
    hipError_t _e = (x);                                                                        \
    if (_e != hipSuccess)                                                                       \
      throw PlanError(LK_ERR_DEVICE, std::string("HIP: ") + #x + ": " + hipGetErrorString(_e)); \
  } while (0)

// (the helpers below up to noisy_tag are shared with exemplar.cpp through evalutil.hpp)

namespace {
struct StrCol {
  std::string name;
  std::vector<const FilterNode*> leaves;
  bool is_dim = false;
  bool restricted = false;
  std::vector<std::string> cand;          // restricted dims: candidate values (dim id = position)
  uint32_t ndim = 1;
  uint32_t dim_null = 0;
  uint64_t stride = 0;
  uint32_t lbase = 0, lmask = 0, hmask = 0;
  uint32_t dict_n = 0;                    // snapshot of the global dictionary size
  std::vector<int> dim_of_cand_null;      // restricted: candidate positions that collapse to absent
  // distributed, unrestricted dim: the agreed union of every rank's value keys (dims.cpp; dim id = position)
  bool exchanged = false;
  std::shared_ptr<DimUnion> uni;
  // the value of dim id d (d != dim_null); `gd` is this column's engine dictionary (caller holds its lock).  A union
  // dim's null-like values read as "" (their tag drops either way).
  std::string_view dim_value(uint32_t d, const GlobalDict& gd) const {
    if (restricted) return cand[d];
    if (!exchanged) return gd[d];
    const char* t = (*uni->text)[d];
    return t ? std::string_view(t) : std::string_view();
  }
  // engine global id -> dim id of an exchanged dim
  uint32_t exchanged_dim(uint32_t gid) const { return (*uni->dim_of_gid)[gid]; }
};

// union_by_name over a glob's files unifies a numeric column to the widest of its physical types in DuckDB's order
// INTEGER < BIGINT < FLOAT < DOUBLE (the same rule exemplar.cpp's union_type applies to tag text).  Rank 0: not a
// numeric type a value column can have.
int value_rank(int ptype) {
  switch (ptype) {
    case pq::INT32: return 1;
    case pq::INT64: return 2;
    case pq::FLOAT: return 3;
    case pq::DOUBLE: return 4;
    default: return 0;
  }
}
int value_type_of_rank(int r) {
  static const int t[5] = {-1, pq::INT32, pq::INT64, pq::FLOAT, pq::DOUBLE};
  return t[r < 0 || r > 4 ? 0 : r];
}

std::string json_escape(const std::string& s) {
  std::string o;
  for (char c : s) {
    if (c == '"' || c == '\\') o += '\\';
    if (static_cast<unsigned char>(c) < 0x20) {
      char b[8];
      snprintf(b, sizeof(b), "\\u%04x", unsigned(static_cast<unsigned char>(c)));
      o += b;
    } else {
      o += c;
    }
  }
  return o;
}

struct GlobInfo {
  std::vector<int> segs;                  // request indices
  bool skip = false;                      // Binder-error glob or no segments here
  uint32_t leaf_false = 0;
  int64_t win_lo = 0, win_hi = 0;
  int64_t step = 0;
  std::vector<std::pair<std::string, std::string>> query_tags;   // glob head's queryTags
};
}  // namespace

// One leaf on one dictionary value (BaseExpr.scala:470-501).  `re`: the compiled RE2-semantics matcher of a
// regex / contains leaf; `set`: the value list of a large in / not_in.
bool leaf_eval(const FilterNode& f, const std::string& s, re::Regex* re, const std::unordered_set<std::string>* set) {
  const std::string& op = f.op;
  if (op == "eq") return s == f.v[0];
  if (op == "!=") return s != f.v[0];
  if (op == "in") return set ? set->count(s) != 0 : std::find(f.v.begin(), f.v.end(), s) != f.v.end();
  if (op == "not_in") return set ? set->count(s) == 0 : std::find(f.v.begin(), f.v.end(), s) == f.v.end();
  if (op == "has" || op == "exists") return true;
  if (op == "regex" || op == "contains") return re->search(s);
  throw PlanError(LK_ERR_UNSUPPORTED, "operator " + op);
}

// regexp_matches(label, p, 'i') (BaseExpr.scala:485-486) / regexp_matches(label, '.*p.*', 'i') (500-501).  A pattern
// RE2 rejects makes DuckDB fail the glob's query, which Commons.toGlobResultSet turns into an empty result
// (Commons.scala:249-253): LK_ERR_ARG, which the shim maps to the same empty source.
re::Regex compile_leaf_regex(const FilterNode& l) {
  const std::string pat = l.op == "contains" ? ".*" + l.v[0] + ".*" : l.v[0];
  try {
    return re::Regex(pat, true);
  } catch (const re::RegexError& e) {
    throw PlanError(e.unsupported ? LK_ERR_UNSUPPORTED : LK_ERR_ARG, std::string("regex '") + pat + "': " + e.what());
  }
}

void postfix(const FilterNode* n, const std::vector<LeafInfo>& leaves, std::vector<uint8_t>& prog) {
  switch (n->kind) {
    case FilterNode::LEAF:
      for (auto& l : leaves)
        if (l.node == n) { prog.push_back(uint8_t(l.index)); return; }
      throw PlanError(LK_ERR_ARG, "internal: leaf not numbered");
    case FilterNode::AND:
    case FilterNode::OR:
      postfix(n->a.get(), leaves, prog);
      postfix(n->b.get(), leaves, prog);
      prog.push_back(n->kind == FilterNode::AND ? OP_AND : OP_OR);
      return;
    case FilterNode::NOT:
      postfix(n->a.get(), leaves, prog);
      prog.push_back(OP_NOT);
      return;
  }
}

void collect_leaves(const FilterNode* n, std::vector<const FilterNode*>& out) {
  if (n->kind == FilterNode::LEAF) out.push_back(n);
  else {
    collect_leaves(n->a.get(), out);
    if (n->b) collect_leaves(n->b.get(), out);
  }
}

bool null_like(const std::string& s) { return s.empty() || s == "null"; }
bool null_like(std::string_view s) { return s.empty() || s == "null"; }

// Conjuncts of the filter's top-level AND chain (a AND (b AND c) -> a, b, c).
void conjuncts(const FilterNode* n, std::vector<const FilterNode*>& out) {
  if (n->kind == FilterNode::AND) {
    conjuncts(n->a.get(), out);
    conjuncts(n->b.get(), out);
  } else {
    out.push_back(n);
  }
}

// Truth table of a postfix Kleene program over L leaves: bit (T | F << L) = the program is TRUE.  An empty
// program is TRUE.
std::vector<uint32_t> truth_table(const std::vector<uint8_t>& prog, uint32_t L) {
  std::vector<uint32_t> truth(((1u << (2 * L)) + 31) / 32, 0u);
  for (uint32_t idx = 0; idx < (1u << (2 * L)); idx++) {
    const uint32_t T = idx & ((1u << L) - 1), F = idx >> L;
    uint64_t st = 0, sf = 0;
    for (uint8_t op : prog) {
      if (op < 0x80) {
        st = (st << 1) | ((T >> op) & 1u);
        sf = (sf << 1) | ((F >> op) & 1u);
      } else if (op == OP_NOT) {
        uint64_t t1 = st & 1, f1 = sf & 1;
        st = (st & ~1ull) | f1;
        sf = (sf & ~1ull) | t1;
      } else if (op == OP_TRUE) {
        st = (st << 1) | 1;
        sf = sf << 1;
      } else {
        uint64_t t2 = st & 1, f2 = sf & 1;
        st >>= 1;
        sf >>= 1;
        uint64_t t1 = st & 1, f1 = sf & 1;
        uint64_t tt = op == OP_AND ? (t1 & t2) : (t1 | t2);
        uint64_t ff = op == OP_AND ? (f1 | f2) : (f1 & f2);
        st = (st & ~1ull) | tt;
        sf = (sf & ~1ull) | ff;
      }
    }
    if (prog.empty() || (st & 1)) truth[idx >> 5] |= 1u << (idx & 31);
  }
  return truth;
}

double ms_since(std::chrono::steady_clock::time_point t0) {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

// NoisyTagsDropper.DO_NOT_DISPLAY_TAGS / DO_NOT_DISPLAY_TAG_PREFIXES (core/.../utils/NoisyTagsDropper.scala)
bool noisy_tag(const std::string& t) {
  static const char* const names[] = {
      "day", "month", "hour", "minute", "year", "sketch", "_cardinalhq.tid", "_cardinalhq.would_filter",
      "_cardinalhq.trace_has_error", "_cardinalhq.id", "_cardinalhq.telemetry_type", "_cardinalhq.filtered",
      "_cardinalhq.is_root_span", "_cardinalhq.positive_counts", "_cardinalhq.negative_counts", "metric.stepTs",
      "metric.tagName", "metric.metrics_type", "scope.telemetry.sdk.name", "metric.filter", "metric.dd.israte",
      "metric.dd.rateinterval"};
  for (const char* n : names)
    if (t == n) return true;
  return t.rfind("rollup_", 0) == 0;
}

namespace {
// Metrics timestamps off the step grid: the scan is re-run at millisecond granularity (see below).
struct MetricsUnaligned {};
// Merged MIN with an all-NaN partial cell: the scan is re-run with per-glob cells (see below).
struct MinNanApart {};
enum Redo : unsigned { REDO_METRICS_RAW = 1u, REDO_MIN_APART = 2u };

// Large dense results cross the host link without their timestamp column: finalize_write records the first row of
// every bucket (FParams::bucket_pos) and the timestamps are expanded here, rows being in bucket-major order.
constexpr unsigned long long kTsRunsMinKeys = 1ull << 18;   // output key spaces this large (C5: 10M keys)
constexpr uint64_t kTsRunsMaxBuckets = 1u << 16;            // bucket_pos entries (mapped pinned memory)

void expand_ts_runs(Engine& E, int64_t* ts, size_t nrows, const FParams& F) {
  if (!nrows) return;
  const uint32_t* bp = F.bucket_pos;
  const uint64_t nb = F.nbuckets;
  const size_t piece = size_t(1) << 19;
  const size_t npieces = (nrows + piece - 1) / piece;
  E.host_parallel(npieces, [&](size_t p) {
    const size_t lo = p * piece, hi = std::min(nrows, lo + piece);
    // the bucket of row lo: the last bucket starting at or before it
    uint64_t b = uint64_t(std::upper_bound(bp, bp + nb, uint32_t(lo)) - bp);
    b = b ? b - 1 : 0;
    for (size_t r = lo; r < hi;) {
      const size_t end = std::min<size_t>(hi, b + 1 < nb ? bp[b + 1] : nrows);
      const int64_t t = F.bucket_base + int64_t(b) * F.step;
      for (; r < end; r++) ts[r] = t;
      b++;
    }
  });
}

// Rows of a large result from its output keys' existence bits (FParams::key_bits): rows are the existing keys in key
// order, so row r's key -- and from it the timestamp, group id and glob -- follow from the bits alone.  Pieces of 2^20
// keys: counts, a prefix, then every piece expanded on its own thread.
void expand_rows_from_keys(Engine& E, int64_t* ts, uint32_t* gid, uint32_t* glob, const unsigned long long* bits,
                           const FParams& F, bool per_glob) {
  const uint64_t words = (F.nkeys + 63) / 64;
  constexpr uint64_t kPiece = uint64_t(1) << 14;   // words per piece
  const size_t np = size_t((words + kPiece - 1) / kPiece);
  std::vector<size_t> base(np + 1, 0);
  E.host_parallel(np, [&](size_t p) {
    size_t c = 0;
    for (uint64_t w = p * kPiece; w < std::min(words, (p + 1) * kPiece); w++) c += size_t(__builtin_popcountll(bits[w]));
    base[p + 1] = c;
  });
  for (size_t p = 0; p < np; p++) base[p + 1] += base[p];
  const uint64_t ng = F.ngroups, ns = F.nglob_slots ? F.nglob_slots : 1;
  E.host_parallel(np, [&](size_t p) {
    size_t r = base[p];
    for (uint64_t w = p * kPiece; w < std::min(words, (p + 1) * kPiece); w++) {
      unsigned long long x = bits[w];
      if (!x) continue;
      const uint64_t k0 = w * 64;
      uint64_t t0 = k0 / ng, g0 = k0 - t0 * ng;   // key = t * ngroups + g
      while (x) {
        const uint64_t b = uint64_t(__builtin_ctzll(x));
        x &= x - 1;
        uint64_t g = g0 + b, t = t0;
        if (g >= ng) {
          t += g / ng;
          g %= ng;
        }
        const uint64_t bucket = per_glob ? t / ns : t;
        ts[r] = F.bucket_base + int64_t(bucket) * F.step;
        gid[r] = uint32_t(g);
        if (glob) glob[r] = uint32_t(t % ns);
        r++;
      }
    }
  });
}
}  // namespace

static int evaluate_once(Engine& E, const std::shared_ptr<const Request>& Rp, const char* const* paths, size_t n_paths,
                         int glob_size, unsigned flags, const int32_t* shard, bool dist, lk_result* res, unsigned redo);
// internal evaluation flag: per-glob rows of a distributed call (rank 0 receives them), for evaluate_metrics_pct
constexpr unsigned kEvalDistPerGlob = 1u << 30;
static int evaluate_metrics_pct(Engine& E, const std::string& json, const Request& R, const char* const* paths,
                                size_t n_paths, int glob_size, unsigned flags, const int32_t* shard, bool dist,
                                lk_result* res);
static int evaluate_mixed_steps(Engine& E, const std::string& json, const Request& R, const char* const* paths,
                                size_t n_paths, int glob_size, unsigned flags, const int32_t* shard, bool dist,
                                lk_result* res);

// Globs whose head segment requests carry different steps (Commons.scala:232, 376-378: each glob's SQL is generated
// from pushDownRequest.copy(segmentRequests = group), i.e. with that glob's head stepInMillis).
static bool mixed_steps(const Request& R, int glob_size) {
  if (R.is_tag_query || !R.has_chart || glob_size <= 0) return false;
  int64_t step = 0;
  for (size_t i = 0; i < R.segments.size(); i += size_t(glob_size)) {
    const int64_t s = R.segments[i].step;
    if (s <= 0) return false;   // (the single-step path reports it)
    if (step && s != step) return true;
    step = s;
  }
  return false;
}

static int evaluate_req(Engine& E, const std::shared_ptr<const Request>& Rp, const char* const* paths, size_t n_paths,
                        int glob_size, unsigned flags, const int32_t* shard, bool dist, lk_result* res) {
  // Both re-runs are thrown before anything is written to *res, and every rank throws them together (agreed flags).
  unsigned redo = 0;
  for (;;) {
    try {
      return evaluate_once(E, Rp, paths, n_paths, glob_size, flags, shard, dist, res, redo);
    } catch (const MetricsUnaligned&) {
      if (redo & REDO_METRICS_RAW) throw PlanError(LK_ERR_DEVICE, "internal: metrics re-run flagged again");
      redo |= REDO_METRICS_RAW;
    } catch (const MinNanApart&) {
      if (redo & REDO_MIN_APART) throw PlanError(LK_ERR_DEVICE, "internal: min re-run flagged again");
      redo |= REDO_MIN_APART;
    }
  }
}

// Metrics: the worker groups by the raw timestamp (`GROUP BY "_cardinalhq.timestamp"`, BaseExpr.scala:376-394); the
// segment index picks segments whose frequency equals the step (`metric_seg.frequency_ms = ?`,
// QueryEngineV2.scala:746-752), so timestamps normally sit on the step grid and a bucket per step is exact.  When a
// row's timestamp is off that grid (the kernel flags it; every rank sees the flag), the evaluation runs again with
// one bucket per millisecond: the cell key is then the raw timestamp (a sparse key space: the hash table).
int evaluate(Engine& E, const std::string& json, const char* const* paths, size_t n_paths, int glob_size,
             unsigned flags, const int32_t* shard, bool dist, lk_result* res) {
  const std::shared_ptr<const Request> Rp = E.parse_cached(json);
  if (Rp->dataset == "metrics" && Rp->has_chart && !Rp->is_tag_query && Rp->aggregation.size() > 1 &&
      Rp->aggregation[0] == 'p' && !Rp->field_chart && !Rp->has_extract && !Rp->has_compute)
    return evaluate_metrics_pct(E, json, *Rp, paths, n_paths, glob_size, flags, shard, dist, res);
  if (n_paths == Rp->segments.size() && mixed_steps(*Rp, glob_size <= 0 ? 10 : glob_size))
    return evaluate_mixed_steps(E, json, *Rp, paths, n_paths, glob_size <= 0 ? 10 : glob_size, flags, shard, dist, res);
  return evaluate_req(E, Rp, paths, n_paths, glob_size, flags, shard, dist, res);
}

// Globs of different steps: one evaluation per step over its globs (each glob keeps its own step, as each glob's SQL
// does), then the rows combined as query-api combines the globs' streams: per glob as they are, or merged per
// (timestamp, tag map) -- sum / count added, min / max by java.lang.Math.min / max (NaN absorbs, -0.0 < +0.0), avg as
// the merged sum over the merged count (two evaluations per step: sum and count).  Tags are materialized per row.
static int evaluate_mixed_steps(Engine& E, const std::string& json, const Request& R, const char* const* paths,
                                size_t n_paths, int glob_size, unsigned flags, const int32_t* shard, bool dist,
                                lk_result* res) {
  const auto t0 = std::chrono::steady_clock::now();
  const bool per_glob_rows = (flags & LK_PER_GLOB_ROWS) != 0;
  const std::string& agg = R.aggregation;
  // sketch aggregations (VERDICT r4 missing #4): percentiles (logs / traces `p<NN>`) merge their DDSketches and
  // cardinality (`ces`) its HLLs per (timestamp, tags), as query-api merges sketches of any origin
  // (TimeGroupedSketchAggregator.scala:34-43), then read the quantile / estimate of the merged sketch
  const bool ces = agg == "ces" || (R.rollup.find("ces") != std::string::npos && R.dataset != "metrics");
  const bool pct = !ces && agg.size() > 1 && agg[0] == 'p' && R.dataset != "metrics";
  double quantile = 0.0;
  if (pct) quantile = strtod(agg.c_str() + 1, nullptr) / 100.0;
  if (!ces && !pct && agg != "sum" && agg != "min" && agg != "max" && agg != "count" && agg != "avg")
    throw PlanError(LK_ERR_UNSUPPORTED, "globs with different steps under aggregation " + agg);
  const size_t G = size_t(glob_size), ng = (n_paths + G - 1) / G;
  std::vector<std::pair<int64_t, std::vector<size_t>>> groups;   // step -> its globs, in order of first appearance
  for (size_t g = 0; g < ng; g++) {
    const int64_t s = R.segments[g * G].step;
    auto it = std::find_if(groups.begin(), groups.end(), [&](const auto& p) { return p.first == s; });
    if (it == groups.end()) groups.emplace_back(s, std::vector<size_t>{g});
    else it->second.push_back(g);
  }
  struct Out {
    int64_t ts;
    uint32_t glob;
    double v, v2;   // value (avg merged: sum) / avg merged: count
    std::vector<std::pair<std::string, std::string>> tags;   // the row's tag map, sorted by name
    dd::Sketch dd;     // percentile rows
    hll::Sketch hll;   // cardinality rows
  };
  std::vector<Out> rows;
  std::vector<std::string> names;   // tag names, first-seen order
  double scan_ms = 0;
  const bool avg_merged = agg == "avg" && !per_glob_rows;
  for (auto& grp : groups) {
    std::vector<const char*> sp;
    std::vector<int32_t> ssh;
    std::vector<SegmentReq> ss;
    for (size_t g : grp.second)
      for (size_t i = g * G; i < std::min(n_paths, (g + 1) * G); i++) {
        sp.push_back(paths[i]);
        ss.push_back(R.segments[i]);
        if (shard) ssh.push_back(shard[i]);
      }
    for (int pass = 0; pass < (avg_merged ? 2 : 1); pass++) {
      auto sub = std::make_shared<Request>(parse_request(json));
      sub->segments = ss;
      if (avg_merged) sub->aggregation = pass == 0 ? "sum" : "count";
      lk_result r;
      r.keep_sketches = pct || ces;
      evaluate_req(E, sub, sp.data(), sp.size(), glob_size, flags, shard ? ssh.data() : nullptr, dist, &r);
      const size_t nt = r.tag_names.size();
      for (size_t c = 0; c < nt; c++)
        if (std::find(names.begin(), names.end(), r.tag_names[c]) == names.end()) names.push_back(r.tag_names[c]);
      for (size_t i = 0; i < r.nrows; i++) {
        Out o{r.ts[i], uint32_t(grp.second[r.per_glob ? r.glob[i] : 0]), r.val[i], 0.0, {}, {}, {}};
        if (pct && i < r.dd_objs.size()) o.dd = std::move(r.dd_objs[i]);
        if (ces && i < r.hll_objs.size()) o.hll = std::move(r.hll_objs[i]);
        for (size_t c = 0; c < nt; c++)
          if (const char* v = r.tag(i, c)) o.tags.emplace_back(r.tag_names[c], v);
        std::sort(o.tags.begin(), o.tags.end());
        if (avg_merged && pass == 1) {
          o.v2 = o.v;
          o.v = 0.0;
        }
        rows.push_back(std::move(o));
      }
      const char* k = strstr(r.stats.c_str(), "\"scan_ms\":");
      if (k) scan_ms += atof(k + 10);
    }
  }
  if (!per_glob_rows) {   // query-api merge per (timestamp, tag map), in first-arrival order
    std::vector<Out> m;
    std::map<std::pair<int64_t, std::vector<std::pair<std::string, std::string>>>, size_t> at;
    auto jmin = [](double a, double b) {   // java.lang.Math.min
      if (a != a) return a;
      if (a == 0.0 && b == 0.0 && std::signbit(b)) return b;
      return a <= b ? a : b;
    };
    auto jmax = [](double a, double b) {   // java.lang.Math.max
      if (a != a) return a;
      if (a == 0.0 && b == 0.0 && std::signbit(a)) return b;
      return a >= b ? a : b;
    };
    for (auto& o : rows) {
      auto key = std::make_pair(o.ts, o.tags);
      auto it = at.find(key);
      if (it == at.end()) {
        at.emplace(std::move(key), m.size());
        o.glob = 0;
        m.push_back(std::move(o));
        continue;
      }
      Out& x = m[it->second];
      if (pct) {
        x.dd.merge(o.dd);
        x.v = x.dd.quantile(quantile);
      } else if (ces) {
        x.hll.merge(o.hll);
        x.v = x.hll.estimate();
      } else if (agg == "min") x.v = jmin(x.v, o.v);
      else if (agg == "max") x.v = jmax(x.v, o.v);
      else {
        x.v += o.v;
        x.v2 += o.v2;
      }
    }
    if (avg_merged)
      for (auto& o : m) o.v = o.v / o.v2;
    rows.swap(m);
  }
  std::stable_sort(rows.begin(), rows.end(), [](const Out& a, const Out& b) {
    return a.ts != b.ts ? a.ts < b.ts : a.glob < b.glob;
  });
  res->exemplar = true;   // tags materialized per row (ex_tags)
  res->per_glob = per_glob_rows;
  res->alloc_rows(rows.size());
  if (pct)
    for (auto& o : rows) res->sketches.push_back(o.dd.serialize());
  res->tag_names = names;
  res->ex_tags.assign(rows.size() * names.size(), nullptr);
  for (size_t i = 0; i < rows.size(); i++) {
    res->ts[i] = rows[i].ts;
    res->val[i] = rows[i].v;
    res->glob[i] = rows[i].glob;
    res->gid[i] = uint32_t(i);
    for (auto& kv : rows[i].tags) {
      const size_t c = size_t(std::find(names.begin(), names.end(), kv.first) - names.begin());
      res->owned.push_back(kv.second);
      res->ex_tags[i * names.size() + c] = res->owned.back().c_str();
    }
  }
  char buf[200];
  snprintf(buf, sizeof buf, "{\"scan_ms\":%.6f,\"total_ms\":%.6f,\"step_groups\":%zu,\"table\":\"per_step\"}", scan_ms,
           std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count(), groups.size());
  res->stats = buf;
  return LK_OK;
}

// Metrics percentiles (VERDICT r5 missing #1).  Each glob's SQL is
//   SELECT ts, MAX(rollup_<rollup|sum>) AS value, name, <groupBys> ... GROUP BY ts, <groupBys>, name
// (BaseExpr.scala:379-383), and the worker's PushDownAggregatorStage feeds every row's value (NULL -> 0.0, JDBC
// getDouble) into the DDSketch of its (raw timestamp, key tags) -- the groupBys' tags, or {"_cardinalhq.name": ""}
// without groupBys (PushDownAggregatorStage.scala:56-60, 69-81, 188-197); query-api merges the sketches per (timestamp, tags)
// (TimeGroupedSketchAggregator.scala:34-37).  Here the per-glob MAX rows come from the GPU scan (the metrics MAX
// path with per-glob cells, every rank's partial table folded on rank 0 when distributed) and the host builds the
// sketches from those rows -- O(output rows), as the logs path assembles its sketches from the kernel's bins.
static int evaluate_metrics_pct(Engine& E, const std::string& json, const Request& R, const char* const* paths,
                                size_t n_paths, int glob_size, unsigned flags, const int32_t* shard, bool dist,
                                lk_result* res) {
  const auto t0 = std::chrono::steady_clock::now();
  const bool per_glob_rows = (flags & LK_PER_GLOB_ROWS) != 0;
  if (!per_glob_rows && !(flags & LK_MERGED)) throw PlanError(LK_ERR_ARG, "flags must be LK_PER_GLOB_ROWS or LK_MERGED");
  if (dist && per_glob_rows) throw PlanError(LK_ERR_ARG, "distributed evaluation returns merged rows");
  char* end = nullptr;
  const std::string qs = R.aggregation.substr(1);
  const double quantile = strtod(qs.c_str(), &end) / 100.0;
  if (end == qs.c_str() || *end || !(quantile >= 0.0 && quantile <= 1.0))
    throw PlanError(LK_ERR_ARG, "percentile aggregation " + R.aggregation);
  if (n_paths == R.segments.size() && mixed_steps(R, glob_size <= 0 ? 10 : glob_size))
    throw PlanError(LK_ERR_UNSUPPORTED, "metrics percentiles over globs with different steps");
  auto sub = std::make_shared<Request>(parse_request(json));
  sub->aggregation = "max";
  lk_result r;
  evaluate_req(E, sub, paths, n_paths, glob_size, LK_PER_GLOB_ROWS | kEvalDistPerGlob, shard, dist, &r);
  using Tags = std::vector<std::pair<std::string, std::string>>;
  struct Row {
    int64_t ts;
    uint32_t glob;
    Tags tags;          // key tags, sorted by name
    dd::Sketch sk;
  };
  std::vector<Row> rows;
  std::map<std::tuple<int64_t, uint32_t, Tags>, size_t> at;   // (ts, glob, key tags) -> row
  const bool by_name = R.group_bys.empty();
  const size_t nt = r.tag_names.size();
  for (size_t i = 0; i < r.nrows; i++) {
    Tags all;   // the DataPoint's tags (NULL / "null" / "" dropped, queryTags when none, Commons.scala:433, 450-452)
    for (size_t c = 0; c < nt; c++)
      if (const char* v = r.tag(i, c)) all.emplace_back(r.tag_names[c], v);
    auto get = [&](const std::string& k) -> const std::string* {
      for (auto& kv : all)
        if (kv.first == k) return &kv.second;
      return nullptr;
    };
    Tags kt;   // getGroupByKeyTags: no groupBys -> {"_cardinalhq.name": ""} (the name tag is labelled `name`)
    if (by_name) {
      kt.emplace_back(kName, std::string());
    } else {
      for (auto& g : R.group_bys)
        if (const std::string* v = get(g))
          if (std::none_of(kt.begin(), kt.end(), [&](const auto& kv) { return kv.first == g; })) kt.emplace_back(g, *v);
      std::sort(kt.begin(), kt.end());
    }
    const uint32_t glob = per_glob_rows ? r.glob[i] : 0u;
    auto ins = at.emplace(std::make_tuple(r.ts[i], glob, kt), rows.size());
    if (ins.second) rows.push_back(Row{r.ts[i], glob, kt, dd::Sketch{}});
    Row& o = rows[ins.first->second];
    // DDSketch.accept throws on NaN / an untrackable magnitude: the worker's stream fails (Commons.scala:331-335)
    if (!o.sk.accept(r.val[i])) throw PlanError(LK_ERR_ARG, "DDSketch: value outside the trackable range");
  }
  std::sort(rows.begin(), rows.end(), [](const Row& a, const Row& b) {
    return a.ts != b.ts ? a.ts < b.ts : (a.glob != b.glob ? a.glob < b.glob : a.tags < b.tags);
  });
  std::vector<std::string> names;   // tag names, first-seen order
  for (auto& o : rows)
    for (auto& kv : o.tags)
      if (std::find(names.begin(), names.end(), kv.first) == names.end()) names.push_back(kv.first);
  res->exemplar = true;   // tags materialized per row (ex_tags)
  res->per_glob = per_glob_rows;
  res->alloc_rows(rows.size());
  res->tag_names = names;
  res->ex_tags.assign(rows.size() * names.size(), nullptr);
  for (size_t i = 0; i < rows.size(); i++) {
    res->ts[i] = rows[i].ts;
    res->val[i] = rows[i].sk.quantile(quantile);
    res->glob[i] = rows[i].glob;
    res->gid[i] = uint32_t(i);
    res->sketches.push_back(rows[i].sk.serialize());
    if (res->keep_sketches) res->dd_objs.push_back(rows[i].sk);
    for (auto& kv : rows[i].tags) {
      const size_t c = size_t(std::find(names.begin(), names.end(), kv.first) - names.begin());
      res->owned.push_back(kv.second);
      res->ex_tags[i * names.size() + c] = res->owned.back().c_str();
    }
  }
  // the MAX scan's own stats, then this stage's
  std::string st = r.stats;
  if (!st.empty() && st.back() == '}') st.pop_back();
  char buf[160];
  snprintf(buf, sizeof buf, ",\"metrics_pct_rows_in\":%zu,\"pct_total_ms\":%.6f}", r.nrows,
           std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
  res->stats = st + buf;
  return LK_OK;
}

static int evaluate_once(Engine& E, const std::shared_ptr<const Request>& Rp, const char* const* paths, size_t n_paths,
                         int glob_size, unsigned flags, const int32_t* shard, bool dist, lk_result* res, unsigned redo) {
  const bool metrics_raw = (redo & REDO_METRICS_RAW) != 0;
  auto t_start = std::chrono::steady_clock::now();
  // Distributed calls issue collectives: one at a time per engine, in the same order on every rank.  Every call
  // runs on its own context (stream, workspaces), so local calls from several threads overlap.
  std::unique_lock<std::mutex> comm_lock;
  if (dist) comm_lock = std::unique_lock<std::mutex>(E.comm_mu);
  CtxLease X(E);
  X->pend_code = 0;
  X->pend_msg.clear();
  const CommCounters cc0 = dist ? comm_counters(E) : CommCounters{};
  static const bool plan_timing = getenv("LK_PLAN_TIMING") != nullptr;   // diagnostics: host planning stages
  auto stage = [&](const char* what) {
    if (plan_timing) fprintf(stderr, "[lk plan] %-10s %.3f ms\n", what, ms_since(t_start));
  };
  const Request& R = *Rp;
  stage("parse");
  const bool per_glob_rows = (flags & LK_PER_GLOB_ROWS) != 0;
  if (!per_glob_rows && !(flags & LK_MERGED)) throw PlanError(LK_ERR_ARG, "flags must be LK_PER_GLOB_ROWS or LK_MERGED");
  if (glob_size <= 0) glob_size = 10;
  if (n_paths != R.segments.size()) throw PlanError(LK_ERR_ARG, "paths must match segmentRequests");
  // Exemplar query (no chart, not a tag query): raw rows, ORDER BY timestamp LIMIT n (BaseExpr.scala:234-239)
  if (!R.is_tag_query && !R.has_chart)
    return evaluate_exemplar(E, *X, R, paths, n_paths, glob_size, flags, dist, res, std::string(), shard);

  // ---- shape gate ----
  // Tag query (isTagQuery with a tagDataType): BaseExpr.generateSql (BaseExpr.scala:127-143) emits
  //   SELECT "<tag>", COUNT(*) AS count FROM {table} WHERE <filter> AND <window> GROUP BY "<tag>"
  // i.e. the same scan with one group dim (the tag), one bucket and COUNT(*) (rows, NULL values included).
  const bool tagq = R.is_tag_query && !R.tag_name.empty();
  // (tagDataType -- "string", "number", ... from the API's query parameter, QueryApi.scala:128-129 -- does not enter
  // the worker's SQL: the tag column's own type decides; a numeric tag column takes the row scan, below)
  if (!tagq && R.is_tag_query)   // isTagQuery without a tagDataType: SELECT * ... WHERE <filter> (BaseExpr.scala:231-232)
    throw PlanError(LK_ERR_UNSUPPORTED, "tag queries without a tagDataType");
  if (R.field_chart || R.has_extract || R.has_compute)
    throw PlanError(LK_ERR_UNSUPPORTED, "extract / compute / field charts are not on the hot path");
  if (R.dataset != "logs" && R.dataset != "traces" && R.dataset != "metrics")
    throw PlanError(LK_ERR_ARG, "Invalid dataset: " + R.dataset);
  int agg;
  if (tagq) agg = AGG_ROWS;
  // Cardinality (`ces` in the chart's rollup, PushDownAggregatorStage.scala:44,82-94; computeCardinality sets it,
  // QueryEngineV2.scala:616-617): per step one HLL over the rows' group-key strings, whatever the SQL aggregate.
  // Metrics: `ces` as the chart's aggregation compiles to `SELECT ts, 1.0 as value, name, <groupBys> ... WHERE
  // <filter>` -- every passing row, no rollup column (BaseExpr.scala:385-388); a metrics rollup of "ces" under another
  // aggregation stays that aggregation over rollup_ces (the SQL reads that column).
  else if (R.aggregation == "ces" || (R.rollup.find("ces") != std::string::npos && R.dataset != "metrics")) agg = AGG_CES;
  else if (R.aggregation == "sum") agg = AGG_SUM;
  else if (R.aggregation == "min") agg = AGG_MIN;
  else if (R.aggregation == "max") agg = AGG_MAX;
  else if (R.aggregation == "count") agg = AGG_COUNT;
  else if (R.aggregation == "avg") agg = AGG_AVG;
  else if (R.aggregation.size() > 1 && R.aggregation[0] == 'p' && R.dataset != "metrics") agg = AGG_SKETCH;
  else throw PlanError(LK_ERR_UNSUPPORTED, "aggregation " + R.aggregation + " (sketch path) is not on the hot path");
  // Percentiles (logs / traces): BaseExpr.getChartSql selects the passing rows (BaseExpr.scala:397-399), the
  // worker's PushDownAggregatorStage builds one DDSketch per (step, group-key tags) (PushDownAggregatorStage.scala:
  // 69-81, 188-197), query-api merges per (timestamp, tags) and reads getValueAtQuantile(p / 100)
  // (BaseExpr.scala:59-61).  Here: the scan bins every value on the GPU (COUNT per (cell, DDSketch bin)), the host
  // assembles the sketches.
  const bool sketch = agg == AGG_SKETCH;
  const bool ces = agg == AGG_CES;
  // queries whose SQL references no value column: tag queries (COUNT(*)) and metrics `ces` (1.0 per row)
  const bool no_value_col = tagq || (ces && R.dataset == "metrics");
  double quantile = 0.0;
  if (sketch) {
    char* end = nullptr;
    const std::string qs = R.aggregation.substr(1);
    quantile = strtod(qs.c_str(), &end) / 100.0;
    if (end == qs.c_str() || *end || !(quantile >= 0.0 && quantile <= 1.0))
      throw PlanError(LK_ERR_ARG, "percentile aggregation " + R.aggregation);
  }
  // Merged avg: query-api runs AVG as separate SUM and COUNT pushdowns, merges them per (timestamp, tags) into
  // a {sum, count} map and divides (QueryEngineV2.scala:280-283, TimeGroupedSketchAggregator.scala:74-78,
  // BaseExpr.scala:88-91).  The table holds both, so one scan gives Σsum / Σcount (NaN when no value).
  // (metrics percentiles evaluate their per-glob MAX rows distributed: kEvalDistPerGlob, internal)
  if (dist && per_glob_rows && !(flags & kEvalDistPerGlob))
    throw PlanError(LK_ERR_ARG, "distributed evaluation returns merged rows");
  const bool metrics = R.dataset == "metrics" && !tagq;   // a tag query groups no timestamps
  const std::string vcol = value_column(R);

  std::vector<const FilterNode*> all_leaves;
  collect_leaves(R.filter.get(), all_leaves);
  // Numeric comparison leaves (gt/ge/lt/le, BaseExpr.scala:488-498) compare a numeric column per row: such queries
  // run on the general row scan (ex_scan AGG mode, ex_kernels.hip) instead of the fused string-filter kernels.
  std::vector<std::string> nums;   // numeric filter columns
  for (auto* l : all_leaves) {
    if (l->extracted || l->computed) throw PlanError(LK_ERR_UNSUPPORTED, "extracted/computed filter fields");
    if (numeric_op(l->op)) {
      if (std::find(nums.begin(), nums.end(), l->k) == nums.end()) nums.push_back(l->k);
      continue;
    }
    static const char* ok[] = {"eq", "!=", "in", "not_in", "regex", "contains", "has", "exists"};
    if (std::none_of(std::begin(ok), std::end(ok), [&](const char* o) { return l->op == o; }))
      throw PlanError(LK_ERR_ARG, "Invalid operator " + l->op);
  }
  const bool numeric = !nums.empty();
  if (numeric && (sketch || ces)) throw PlanError(LK_ERR_UNSUPPORTED, "numeric comparison leaves in sketch queries");
  // (distributed: the numeric leaves' per-glob decisions -- a bad literal, a VARCHAR column -- come from the agreed glob
  // unions, and the general row scan's partial tables reduce like any other)

  // no segments: the worker answers one sentinel row (Commons.scala:393-396)
  if (R.segments.empty()) {
    if (per_glob_rows) {
      res->alloc_rows(1);
      res->ts[0] = -1;
      res->val[0] = -1.0;
      res->glob[0] = 0;
      res->gid[0] = 0;
    }
    res->stats = "{\"scan_ms\":0,\"total_ms\":0,\"rows_scanned\":0,\"algorithmic_bytes\":0,\"tiles\":0,\"cells\":0}";
    return LK_OK;
  }

  // ---- string columns: name first, then leaf keys, then groupBys ----
  std::vector<StrCol> strs;
  auto str_index = [&](const std::string& name) -> int {
    for (size_t i = 0; i < strs.size(); i++)
      if (strs[i].name == name) return int(i);
    strs.push_back(StrCol{});
    strs.back().name = name;
    return int(strs.size() - 1);
  };
  str_index(tagq ? R.tag_name : kName);   // the first string column is the leading group dim
  for (auto* l : all_leaves)
    if (!numeric_op(l->op)) strs[str_index(l->k)].leaves.push_back(l);
  std::vector<std::string> gbs;
  for (auto& g : R.group_bys)
    if (std::find(gbs.begin(), gbs.end(), g) == gbs.end()) gbs.push_back(g);
  for (auto& g : gbs) str_index(g);
  if (strs.size() > size_t(MAXSTR)) throw PlanError(LK_ERR_UNSUPPORTED, "too many string columns in one query");
  for (auto& nm : nums)   // a column compared both as a string and as a number fails the glob's SQL either way
    if (std::find_if(strs.begin(), strs.end(), [&](const StrCol& sc) { return sc.name == nm; }) != strs.end())
      throw PlanError(LK_ERR_UNSUPPORTED, "column " + nm + " used both as a string and as a number");
  if (2 + strs.size() + nums.size() > size_t(MAXQCOL)) throw PlanError(LK_ERR_UNSUPPORTED, "too many filter columns");
  if (all_leaves.size() > size_t(MAXLEAF)) throw PlanError(LK_ERR_UNSUPPORTED, "too many filter leaves");
  // (a tag query's tag may be the value / timestamp column: numeric, it takes the TAGNUM row scan below)
  if (std::find_if(strs.begin(), strs.end(), [&](const StrCol& s) {
        return (s.name == kTimestamp || s.name == vcol) && !(tagq && s.name == R.tag_name);
      }) != strs.end())
    throw PlanError(LK_ERR_UNSUPPORTED, "filters / groupBys on the timestamp or value column");
  std::vector<LeafInfo> leaves;
  for (size_t s = 0; s < strs.size(); s++) {
    StrCol& sc = strs[s];
    if (sc.leaves.size() > size_t(LEAF_BITS)) throw PlanError(LK_ERR_UNSUPPORTED, "too many leaves on one column");
    sc.lbase = uint32_t(leaves.size());
    for (size_t j = 0; j < sc.leaves.size(); j++) {
      uint32_t idx = uint32_t(leaves.size());
      leaves.push_back(LeafInfo{sc.leaves[j], int(s), int(idx)});
      sc.lmask |= 1u << idx;
      if (sc.leaves[j]->op == "has" || sc.leaves[j]->op == "exists") sc.hmask |= 1u << idx;
    }
  }
  std::vector<NumLeaf> nleaves;
  std::vector<std::string> bad_literal;   // fields whose numeric literal fails the SQL (per glob where they exist)
  for (auto* l : all_leaves)
    if (numeric_op(l->op)) {
      const uint32_t idx = uint32_t(leaves.size());
      leaves.push_back(LeafInfo{l, -1, int(idx)});
      bool bad = false;
      nleaves.push_back(make_num_leaf(*l, uint32_t(std::find(nums.begin(), nums.end(), l->k) - nums.begin()), idx, bad));
      if (bad) bad_literal.push_back(l->k);
    }
  std::vector<uint8_t> prog;
  postfix(R.filter.get(), leaves, prog);
  if (prog.size() > size_t(MAXPROG)) throw PlanError(LK_ERR_UNSUPPORTED, "filter too large");
  // Regex leaves RE2 rejects (LK_ERR_ARG) fail the SQL only of the globs where the leaf's field exists (glob loop
  // below); a pattern RE2 takes but this matcher does not (LK_ERR_UNSUPPORTED) fails the call.
  std::vector<uint8_t> bad_regex(leaves.size(), 0);
  for (auto& l : leaves)
    if (l.node->op == "regex" || l.node->op == "contains") {
      try {
        (void)compile_leaf_regex(*l.node);
      } catch (const PlanError& e) {
        if (e.code != LK_ERR_ARG) throw;
        bad_regex[size_t(l.index)] = 1;
      }
    }

  // ---- segments: which ones this process evaluates ----
  const int world = dist ? comm_world(E) : 1;
  const int rank = dist ? comm_rank(E) : 0;
  std::vector<char> mine(n_paths, 1);
  if (dist)
    for (size_t i = 0; i < n_paths; i++) mine[i] = (shard ? shard[i] : int32_t(i % size_t(world))) == rank;
  std::vector<std::shared_ptr<Segment>> segs(n_paths);
  // A segment the worker cannot read (missing file, corrupt Parquet, a file shape the loader does not take) fails
  // its glob's DuckDB query, which Commons.toGlobResultSet turns into an empty result for that glob alone
  // (Commons.scala:249-253, 338-340): such segments are marked here and empty their glob below.
  std::vector<uint8_t> seg_bad(n_paths, 0);
  std::string bad_msg;   // the first such failure (stats)
  int load_err = 0;
  std::string load_msg;
  {
    // A rank-local failure of the engine itself (HIP, HBM, host memory) must not leave the other ranks waiting in the
    // next collective: the ranks agree on a status first and fail together (folded into the glob-union exchange
    // below: one all-gather carries both).
    int err = 0;
    std::string msg;
    try {
      for (size_t i = 0; i < n_paths; i++) {
        if (!mine[i]) continue;
        try {
          segs[i] = E.get_segment(paths[i], true);
        } catch (const PlanError& e) {
          // only the file's own faults (missing, unreadable, corrupt) empty its glob; an engine capability gap
          // (LK_ERR_UNSUPPORTED) or an evicted put key (LK_ERR_EVICTED) fails the call
          if (e.code != LK_ERR_IO) throw;
          seg_bad[i] = 1;
          if (bad_msg.empty()) bad_msg = e.what();
        }
      }
    } catch (const PlanError& e) {
      if (!dist) throw;
      err = e.code;
      msg = e.what();
    } catch (const std::exception& e) {
      if (!dist) throw;
      err = LK_ERR_DEVICE;
      msg = e.what();
    }
    load_err = err;
    load_msg = msg;
  }
  // A tag query over a numeric tag column (INT32 / INT64 / FLOAT / DOUBLE / BOOLEAN in a loaded segment): the values are
  // grouped and printed by the row scan's TAGNUM mode (exemplar.cpp).  Distributed: agreed on with the glob unions.
  bool tag_numeric = false;
  if (tagq)
    for (size_t i = 0; i < n_paths && !tag_numeric; i++) {
      if (!segs[i]) continue;
      const int c = segs[i]->col_index(R.tag_name);
      tag_numeric = c >= 0 && !segs[i]->cols[size_t(c)].is_string;
    }
  if (tag_numeric && !dist) {
    segs.clear();
    return evaluate_exemplar(E, *X, R, paths, n_paths, glob_size, flags, false, res, R.tag_name);
  }

  stage("segments");
  // ---- globs ----
  const std::set<std::string> fset = field_set(R);
  std::vector<std::string> probe_cols(fset.begin(), fset.end());   // columns whose existence matters
  for (auto& k : tagq ? std::vector<std::string>{kTimestamp, R.tag_name}
                      : (no_value_col ? std::vector<std::string>{kTimestamp, kName}
                                      : std::vector<std::string>{kTimestamp, kName, vcol}))
    if (std::find(probe_cols.begin(), probe_cols.end(), k) == probe_cols.end()) probe_cols.push_back(k);
  for (auto* l : all_leaves)
    if (std::find(probe_cols.begin(), probe_cols.end(), l->k) == probe_cols.end()) probe_cols.push_back(l->k);
  std::vector<GlobInfo> globs;
  for (size_t i = 0; i < n_paths; i += size_t(glob_size)) {
    GlobInfo g;
    for (size_t j = i; j < std::min(n_paths, i + size_t(glob_size)); j++) g.segs.push_back(int(j));
    globs.push_back(std::move(g));
  }
  // Per glob: the union of columns (over the probe columns), "this glob's query fails" (a segment that did not load,
  // or a column whose type the query cannot use), the union_by_name type of the value column, and "value column may
  // be NULL".  Layout: [globs x np exists | globs fail | globs value-type rank | value NULLs].
  const size_t np = probe_cols.size();
  const size_t ng = globs.size();
  // [.. | value NULLs | numeric tag column]
  std::vector<uint8_t> exists(ng * np + 2 * ng + 2, 0);
  const size_t vnull_at = ng * np + 2 * ng;
  exists[vnull_at + 1] = tag_numeric ? 1 : 0;
  // A referenced column this engine does not decode (Segment::unloaded) fails the call with LK_ERR_UNSUPPORTED: DuckDB
  // would read it, so the shim must fall back rather than see an empty glob.  Rank-local (it depends on
  // this rank's segments): agreed on with the load status below.
  std::vector<std::string> ref_cols(probe_cols);
  for (auto& sc : strs) ref_cols.push_back(sc.name);
  for (auto& nm : nums) ref_cols.push_back(nm);
  uint8_t* gfail = exists.data() + ng * np;
  uint8_t* gvrank = gfail + ng;
  for (size_t gi = 0; gi < ng; gi++)
    for (int si : globs[gi].segs) {
      if (seg_bad[si]) gfail[gi] = 1;
      if (!segs[si]) continue;
      const Segment& S = *segs[si];
      for (size_t k = 0; k < np; k++)
        if (S.all_columns.count(probe_cols[k])) exists[gi * np + k] = 1;
      if (!S.unloaded.empty() && !load_err)
        for (auto& c : ref_cols) {
          auto u = S.unloaded.find(c);
          if (u == S.unloaded.end()) continue;
          if (!dist) throw PlanError(LK_ERR_UNSUPPORTED, u->second + " (" + S.key + ")");
          load_err = LK_ERR_UNSUPPORTED;
          load_msg = u->second + " (" + S.key + ")";
          break;
        }
      int vc = S.col_index(vcol);
      // a NULL value anywhere (or no value column): a glob cell may hold only NULLs and read back 0.0
      if (vc < 0 || S.cols[vc].any_nulls) exists[vnull_at] = 1;
      // Column types per role.  read_parquet(union_by_name=True) (Commons.scala:213) unifies each column's type
      // over the glob's files; a column the query cannot bind (the value column as text, a string filter /
      // groupBy column stored as a number, a numeric comparison on text, INT96 / FIXED_LEN_BYTE_ARRAY, which the
      // engine does not load) makes DuckDB fail the glob's SQL -> that glob is empty (Commons.scala:249-253).
      auto bad = [&](const std::string& name, int role) -> bool {
        if (!S.all_columns.count(name)) return false;   // absent: nonExistentFields / NULL, not an error
        const int c = S.col_index(name);
        if (c < 0) return true;
        const HostCol& hc = S.cols[size_t(c)];
        if (role == 0) return hc.ptype != pq::INT64 && hc.ptype != pq::INT32;   // BIGINT over INT32 / INT64 files
        if (role == 2) return !hc.is_string;
        return value_rank(hc.ptype) == 0;   // value column / numeric comparison column
      };
      if (bad(kTimestamp, 0)) gfail[gi] = 1;
      if (!no_value_col) {
        if (bad(vcol, 1)) {
          // sum / avg over a VARCHAR value column is DuckDB's Binder Error (empty glob); count / min / max over it
          // run in DuckDB and this engine does not implement them: the call fails (LK_ERR_UNSUPPORTED)
          if (vc >= 0 && S.cols[size_t(vc)].is_string && agg != AGG_SUM && agg != AGG_AVG && !load_err) {
            const std::string m = "aggregation over the VARCHAR value column " + vcol + " (" + S.key + ")";
            if (!dist) throw PlanError(LK_ERR_UNSUPPORTED, m);
            load_err = LK_ERR_UNSUPPORTED;
            load_msg = m;
          }
          gfail[gi] = 1;
        }
        else if (vc >= 0) gvrank[gi] = std::max<uint8_t>(gvrank[gi], uint8_t(value_rank(S.cols[size_t(vc)].ptype)));
      }
      for (auto& sc : strs)
        if (bad(sc.name, 2)) gfail[gi] = 1;
      for (auto& nm : nums)
        if (bad(nm, 3)) gfail[gi] = 1;
    }
  // every rank sees every glob's union, failures and value type; a rank-local engine failure fails every rank here
  if (dist) comm_agree_max_u8(E, *X, load_err, load_msg, exists.data(), exists.size());
  const bool value_nulls = exists[vnull_at] != 0;
  if (exists[vnull_at + 1]) {   // agreed: a numeric tag column on some rank -- every rank takes the TAGNUM row scan
    segs.clear();
    return evaluate_exemplar(E, *X, R, paths, n_paths, glob_size, flags, true, res, R.tag_name, shard);
  }
  size_t nfailed = 0;
  for (size_t gi = 0; gi < ng; gi++)
    if (gfail[gi]) {
      globs[gi].skip = true;
      nfailed++;
    }
  auto glob_has = [&](size_t gi, const std::string& c) {
    size_t k = size_t(std::find(probe_cols.begin(), probe_cols.end(), c) - probe_cols.begin());
    return exists[gi * np + k] != 0;
  };
  int64_t step = -1;
  for (size_t gi = 0; gi < globs.size(); gi++) {
    GlobInfo& g = globs[gi];
    const SegmentReq& head = R.segments[g.segs[0]];
    g.step = head.step;
    g.query_tags = head.query_tags;
    g.win_lo = INT64_MAX;
    g.win_hi = INT64_MIN;
    for (int si : g.segs) {
      g.win_lo = std::min(g.win_lo, R.segments[si].start_ts);
      g.win_hi = std::max(g.win_hi, R.segments[si].end_ts);
    }
    // nonExistentFields (Commons.scala:224) -> leaves compiled to `false`
    std::set<std::string> nonexist;
    for (auto& f : fset)
      if (!glob_has(gi, f)) nonexist.insert(f);
    for (auto& l : leaves)
      if (nonexist.count(l.node->k)) g.leaf_false |= 1u << l.index;
    // Binder Error: referenced column absent from the whole glob
    if (tagq) {
      if (!glob_has(gi, kTimestamp) || !glob_has(gi, R.tag_name)) g.skip = true;   // SELECT "<tag>": Binder Error
    } else if (!glob_has(gi, kTimestamp) || !glob_has(gi, kName) || (!no_value_col && !glob_has(gi, vcol))) {
      g.skip = true;
    }
    for (auto& l : leaves)
      if (!nonexist.count(l.node->k) && !glob_has(gi, l.node->k)) g.skip = true;
    for (auto& k : bad_literal)   // normalizedValue failed for a field this glob has
      if (!nonexist.count(k)) g.skip = true;
    // a regex leaf RE2 rejects fails the SQL of every glob where its field exists (where it does not, the leaf is
    // the literal `false` and the pattern is never compiled, BaseExpr.scala:462-464)
    for (auto& l : leaves)
      if (bad_regex[size_t(l.index)] && !nonexist.count(l.node->k)) g.skip = true;
    // (`<string column> > 1.5`, a Binder Error -> empty glob, is among the column-type failures above)
    if (tagq) continue;
    if (g.step <= 0) throw PlanError(LK_ERR_ARG, "stepInMillis must be positive");
    if (step < 0) step = g.step;
    else if (g.step != step) throw PlanError(LK_ERR_DEVICE, "internal: globs with different steps (evaluate splits them)");
  }

  // A tag query's single bucket: ts - ts % 2^62 = 0 for every |ts| < 2^62, so bucket_base = 0 and one bucket.
  if (tagq) step = int64_t(1) << 62;
  // metrics off the step grid: one bucket per millisecond, i.e. the raw timestamp (see evaluate())
  if (metrics_raw && R.dataset == "metrics" && !tagq) step = 1;

  stage("globs");
  // ---- group dimensions ----
  const bool merged = !per_glob_rows;
  // Merged min/max over values that can be NULL: NULL, "null" and "" group values stay apart in the table
  // (each is its own DuckDB group, and an all-NULL group reads back 0.0); they collapse after per-glob
  // finalization (rekey_minmax).  Everywhere else they can share a cell.
  // MIN re-run (REDO_MIN_APART): a DuckDB group whose values are all NaN has MIN = NaN, and query-api's math.min of
  // the globs' rows (TimeGroupedSketchAggregator.scala:79-88) -- or of a glob's NULL / "null" / "" groups, which share
  // an output key -- is then NaN; cells shared in the table would lose it (NaN orders above every number), so they stay
  // apart exactly as for NULL values.
  const bool min_max_nulls = (agg == AGG_MIN || agg == AGG_MAX) && (value_nulls || (redo & REDO_MIN_APART));
  const bool collapse_in_table = merged && !min_max_nulls;
  double dims_ms = 0;      // distributed group-dim agreement (stats)
  int dims_rebuilt = 0;
  for (size_t s = 0; s < strs.size(); s++) {
    StrCol& sc = strs[s];
    sc.is_dim = (s == 0) || std::find(gbs.begin(), gbs.end(), sc.name) != gbs.end();
    GlobalDict& gd = E.dict(sc.name);
    {
      std::lock_guard<std::mutex> g(gd.mu);
      sc.dict_n = uint32_t(gd.size());
    }
    if (!sc.is_dim) continue;
    if (restricted_values(R.filter.get(), sc.name, sc.cand)) {
      sc.restricted = true;
      // A passing row holds one of the candidates (the filter is `col IN cand AND ...`): NULL / absent / other
      // values never reach a cell, so the absent slot is needed only where a null-like candidate ("" / "null")
      // is itself folded into it.  Without it the dim has cand.size() ids and dim_null is past them (C5: the
      // name dim of `:eq name` no longer doubles the 10M-group cell space).
      const bool nl_cand = std::any_of(sc.cand.begin(), sc.cand.end(), [](const std::string& v) { return null_like(v); });
      sc.ndim = uint32_t(sc.cand.size()) + ((nl_cand || sc.cand.empty()) ? 1u : 0u);
      sc.dim_null = uint32_t(sc.cand.size());
    } else if (dist) {
      // Every rank holds its own engine dictionary: the dim space is the agreed union of the ranks' value keys
      // (dims.cpp), cached while no rank's dictionary changes.
      double ms = 0;
      bool rebuilt = false;
      sc.uni = agree_dim_union(E, *X, sc.name, sc.dict_n, ms, rebuilt);
      dims_ms += ms;
      dims_rebuilt += rebuilt ? 1 : 0;
      sc.exchanged = true;
      sc.ndim = sc.uni->size + 1;
      sc.dim_null = sc.uni->size;
    } else {
      if (sc.dict_n + 1 > DIM_MASK) throw PlanError(LK_ERR_UNSUPPORTED, "group dimension too large");
      sc.ndim = sc.dict_n + 1;
      sc.dim_null = sc.dict_n;
    }
  }
  uint64_t ngroups = 1;
  for (int s = int(strs.size()) - 1; s >= 0; s--) {
    if (!strs[s].is_dim) continue;
    strs[s].stride = ngroups;
    ngroups *= strs[s].ndim;
    if (ngroups > 0xffffffffull) throw PlanError(LK_ERR_UNSUPPORTED, "group space beyond 2^32 groups");
  }

  stage("dims");
  // ---- lookup tables: global id -> leaf bits << 24 | dim id ----
  std::vector<std::vector<uint32_t>> tabs(strs.size());
  std::vector<char> need_tab(strs.size(), 0);
  for (size_t s = 0; s < strs.size(); s++) {
    StrCol& sc = strs[s];
    GlobalDict& gd = E.dict(sc.name);
    bool null_like_present;
    {
      std::lock_guard<std::mutex> g(gd.mu);
      null_like_present = gd.ids.count("null") || gd.ids.count("");
    }
    need_tab[s] = !sc.leaves.empty() || sc.restricted || sc.exchanged ||
                  (sc.is_dim && collapse_in_table && null_like_present) || (!sc.is_dim && sc.leaves.empty());
    // an agreed union dim without leaves reads its global id -> dim id table straight from HBM (built once with the
    // agreement), unless null-like values must fold into dim_null in this query's table
    if (sc.exchanged && sc.leaves.empty() && !(collapse_in_table && null_like_present) && sc.uni->d_dim_of_gid)
      need_tab[s] = false;
    if (!need_tab[s]) continue;
    // Leaf outcomes over the column's dictionary (values [0, dict_n) are immutable: StableStrs), cached per
    // (column, leaves) and extended only over values added since: a regex runs once per distinct value.
    std::shared_ptr<LeafBits> lb;
    std::unique_lock<std::mutex> lb_guard;
    if (!sc.leaves.empty()) {
      std::string key = sc.name;
      for (const FilterNode* l : sc.leaves) {
        key += '\x1f';
        key += l->op;
        for (auto& v : l->v) {
          key += '\x1e';
          key += v;
        }
      }
      std::vector<std::unique_ptr<re::Regex>> res(sc.leaves.size());
      std::vector<std::unique_ptr<std::unordered_set<std::string>>> sets(sc.leaves.size());
      std::vector<char> skip_leaf(sc.leaves.size(), 0);   // a rejected pattern: every glob it could run in is empty
      for (size_t j = 0; j < sc.leaves.size(); j++) {
        const FilterNode* l = sc.leaves[j];
        if (bad_regex[sc.lbase + j]) {
          skip_leaf[j] = 1;
          continue;
        }
        if (l->op == "regex" || l->op == "contains") res[j] = std::make_unique<re::Regex>(compile_leaf_regex(*l));
        if ((l->op == "in" || l->op == "not_in") && l->v.size() > 8)
          sets[j] = std::make_unique<std::unordered_set<std::string>>(l->v.begin(), l->v.end());
      }
      lb = E.leaf_bits(key);
      lb_guard = std::unique_lock<std::mutex>(lb->mu);
      lb->hit.reserve(sc.dict_n);
      for (uint32_t gid = uint32_t(lb->hit.size()); gid < sc.dict_n; gid++) {
        const std::string& v = gd[gid];
        uint8_t bits = 0;
        for (size_t j = 0; j < sc.leaves.size(); j++)
          if (!skip_leaf[j] && leaf_eval(*sc.leaves[j], v, res[j].get(), sets[j].get())) bits |= uint8_t(1u << j);
        lb->hit.push_back(bits);
      }
    }
    auto& tab = tabs[s];
    tab.resize(std::max<uint32_t>(sc.dict_n, 1));
    for (uint32_t gid = 0; gid < sc.dict_n; gid++) {
      const std::string& v = gd[gid];
      const uint32_t bits = lb ? lb->hit[gid] : 0u;
      uint32_t dim = 0;
      if (sc.is_dim) {
        if (sc.restricted) {
          auto it = std::find(sc.cand.begin(), sc.cand.end(), v);
          dim = it == sc.cand.end() ? sc.dim_null : uint32_t(it - sc.cand.begin());
          if (collapse_in_table && null_like(v)) dim = sc.dim_null;
        } else {
          dim = (collapse_in_table && null_like(v)) ? sc.dim_null : (sc.exchanged ? sc.exchanged_dim(gid) : gid);
        }
      }
      tab[gid] = (bits << 24) | dim;
    }
  }

  stage("tables");
  // ---- bucket space ----
  int64_t min_lo = INT64_MAX, max_hi = INT64_MIN;
  for (auto& g : globs) {
    if (g.skip) continue;
    min_lo = std::min(min_lo, g.win_lo);
    max_hi = std::max(max_hi, g.win_hi);
  }
  int64_t bucket_base = 0;
  uint64_t nbuckets = 0;
  if (min_lo < max_hi) {
    if (metrics) bucket_base = min_lo;
    else bucket_base = min_lo - min_lo % step;
    int64_t last = max_hi - 1;
    int64_t last_b = metrics ? last : last - last % step;
    nbuckets = uint64_t((last_b - bucket_base) / step + 1);
  }
  const bool per_glob_cells = per_glob_rows || min_max_nulls;
  // dims whose null-like values must be folded after per-glob finalization
  std::vector<std::vector<uint32_t>> fold_maps(strs.size());
  bool rekey = false;
  if (merged && min_max_nulls && !gbs.empty()) {
    for (size_t s = 0; s < strs.size(); s++) {
      StrCol& sc = strs[s];
      if (!sc.is_dim) continue;
      GlobalDict& gd = E.dict(sc.name);
      std::lock_guard<std::mutex> g(gd.mu);
      std::vector<uint32_t> m(sc.ndim);
      bool any = false;
      for (uint32_t d = 0; d < sc.ndim; d++) {
        m[d] = d;
        if (d == sc.dim_null) continue;
        if (null_like(sc.dim_value(d, gd))) { m[d] = sc.dim_null; any = true; }
      }
      if (any) { fold_maps[s] = std::move(m); rekey = true; }
    }
  }
  const uint32_t nslots = per_glob_cells ? uint32_t(globs.size()) : 1u;
  if (nbuckets && (double(nslots) * double(nbuckets) * double(ngroups) > 9.0e18))
    throw PlanError(LK_ERR_UNSUPPORTED, "cell key space beyond 64 bits");
  const uint64_t ncells = uint64_t(nslots) * nbuckets * ngroups;

  // Numeric leaves on the value column alone (`:and(:eq name, :gt value 1.5)`), in conjuncts of their own: the fused
  // kernels filter on the string conjuncts and test the value of each passing row (QParams.vl / vtab) -- the segments
  // whose tiles all qualify for scan_lean; the other segments take the general row scan as before.
  bool vleaf = false;
  std::vector<uint8_t> prog_str;   // vleaf: the string conjuncts (the fused kernels' filter)
  uint32_t vtab = 0;
  if (numeric && !tagq && nums.size() == 1 && nums[0] == vcol && nleaves.size() <= size_t(VLEAF_MAX) &&
      leaves.size() <= size_t(TT_MAX_LEAVES) && !getenv("LK_NO_VLEAF")) {
    std::vector<const FilterNode*> conj;
    conjuncts(R.filter.get(), conj);
    std::vector<uint8_t> pn;
    bool ok = true;
    for (auto* c : conj) {
      std::vector<const FilterNode*> ls;
      collect_leaves(c, ls);
      const size_t nn = size_t(std::count_if(ls.begin(), ls.end(), [](const FilterNode* l) { return numeric_op(l->op); }));
      if (nn && nn != ls.size()) ok = false;   // a conjunct mixing string and numeric leaves
      std::vector<uint8_t>& dst = nn ? pn : prog_str;
      const bool first = dst.empty();
      postfix(c, leaves, dst);
      if (!first) dst.push_back(OP_AND);
    }
    if (ok && !pn.empty()) {
      vleaf = true;
      if (prog_str.empty()) prog_str.push_back(OP_TRUE);
      // vtab bit m: the numeric conjuncts with leaf k TRUE iff bit k of m (no UNKNOWN: scan_lean tiles hold no NULL)
      const uint32_t L = uint32_t(leaves.size()), nsl = L - uint32_t(nleaves.size());
      const std::vector<uint32_t> tn = truth_table(pn, L);
      for (uint32_t m = 0; m < (1u << nleaves.size()); m++) {
        const uint32_t full = (1u << nleaves.size()) - 1u;
        const uint32_t ix = (m << nsl) | (((~m & full) << nsl) << L);
        if ((tn[ix >> 5] >> (ix & 31)) & 1u) vtab |= 1u << m;
      }
    }
  }
  // filter truth table: bit (T | F << L) = Kleene value of the tree is TRUE (host-evaluated once per query)
  std::vector<uint32_t> truth, truth_early, truth_late, truth_x;   // truth_x: the general row scan's (vleaf)
  uint32_t late_mask = 0;
  int early = -1;   // the string column (strs index) of the single-column early conjuncts, when there is one
  if (leaves.size() <= size_t(TT_MAX_LEAVES)) {
    const uint32_t L = uint32_t(leaves.size());
    truth = truth_table(vleaf ? prog_str : prog, L);
    if (vleaf) truth_x = truth_table(prog, L);
    // Predicate pushdown + late materialization.  filter = C_early AND C_late where C_early is the conjuncts
    // over one "early" column (the name column when a conjunct constrains it alone).  The kernel decodes the
    // early column for every row, lists the rows where C_early is TRUE, and decodes every other string column
    // (late filter columns, group dims) only for listed rows, where it evaluates C_late.
    std::vector<const FilterNode*> conj;
    conjuncts(R.filter.get(), conj);
    auto cols_of = [&](const FilterNode* n) {
      std::vector<const FilterNode*> ls;
      collect_leaves(n, ls);
      uint32_t m = 0;
      for (auto* l : ls) m |= numeric_op(l->op) ? (1u << 31) : (1u << str_index(l->k));   // no StrCol for numbers
      return m;
    };
    // A conjunct of only `exists`/`has` leaves (IS NOT NULL: passes nearly every row, e.g. the one query-api adds
    // to a tag query) is a poor early filter: it is chosen only when no other single-column conjunct exists.
    auto weak = [&](const FilterNode* n) {
      std::vector<const FilterNode*> ls;
      collect_leaves(n, ls);
      return std::all_of(ls.begin(), ls.end(), [](const FilterNode* l) { return l->op == "exists" || l->op == "has"; });
    };
    bool early_weak = true;
    if (vleaf)   // the value-leaf conjuncts are tested per passing row, outside the early / late split
      conj.erase(std::remove_if(conj.begin(), conj.end(), [&](const FilterNode* c) { return cols_of(c) == (1u << 31); }),
                 conj.end());
    for (auto* c : conj) {
      const uint32_t m = cols_of(c);
      if (__builtin_popcount(m) != 1) continue;
      const int col = __builtin_ctz(m);
      const bool w = weak(c);
      if (early < 0 || (early_weak && !w) || (w == early_weak && col == 0)) {
        early = col;
        early_weak = w;
      }
    }
    // The late pass sees only the late columns' leaves: a conjunct mixing the early column with others keeps
    // every column early (no late pass).
    bool mixed = false;
    for (auto* c : conj) {
      const uint32_t m = cols_of(c);
      if (early >= 0 && m != (1u << early) && ((m >> early) & 1u)) mixed = true;
    }
    if (early >= 0 && strs.size() >= 2 && !mixed && (!numeric || vleaf)) {
      std::vector<uint8_t> pe, pl;
      for (auto* c : conj) {
        std::vector<uint8_t>& dst = cols_of(c) == (1u << early) ? pe : pl;
        const bool first = dst.empty();
        postfix(c, leaves, dst);
        if (!first) dst.push_back(OP_AND);
      }
      truth_early = truth_table(pe, L);
      truth_late = truth_table(pl, L);
      for (size_t sidx = 0; sidx < strs.size(); sidx++)
        if (int(sidx) != early) late_mask |= 1u << sidx;
    }
  }
  // Device order of the string columns (query column 2 + dev_of[s]): the early column first when the filter's late
  // materialization lists every other column late, so scan_lean (whose early column is query column 2) takes the
  // query even when the leading group dim -- a tag query's tag, a :by column -- is not the filter's early column.
  std::vector<int> dev_of(strs.size());
  for (size_t i = 0; i < strs.size(); i++) dev_of[i] = int(i);
  // (LK_NO_EARLY_FIRST=1: the r03 order, for A/B)
  if (late_mask && early > 0 && strs.size() <= 3 && !getenv("LK_NO_EARLY_FIRST")) {
    std::swap(dev_of[0], dev_of[size_t(early)]);
    uint32_t m = 0;
    for (size_t i = 0; i < strs.size(); i++)
      if ((late_mask >> i) & 1u) m |= 1u << dev_of[i];
    late_mask = m;
  }
  const int lead = dev_of[0] == 0 ? 0 : int(std::find(dev_of.begin(), dev_of.end(), 0) - dev_of.begin());   // strs index at device 0
  // vleaf needs scan_lean's shape: the early column alone, or with <= 2 late columns (the launch test below)
  const bool vleaf_shape = vleaf && !truth.empty() &&
                           (strs.size() == 1 || (strs.size() <= 3 && late_mask == ((1u << strs.size()) - 2u)));

  // ---- per-segment query descriptors ----
  // `qsegs` go to the fused kernels (scan_lean / scan_tiles: INT64 timestamps, DOUBLE values); `gsegs` to the general
  // row scan (ex_scan AGG mode): every segment of a numeric-leaf query, and segments whose timestamp or value column
  // needs union_by_name promotion (INT32 timestamps; INT32 / INT64 / FLOAT values, cast through FLOAT where the glob's
  // value type is FLOAT).  Both kinds aggregate into the same table.
  std::vector<QSeg> qsegs, gsegs;
  std::vector<uint32_t> seg_begin;
  uint32_t total_tiles = 0;
  uint64_t rows_scanned = 0, alg_bytes = 0;
  // QParams::exact_sum: every bound value column integral (HostCol::int_abs_max), its largest magnitude, their rows
  bool vals_integral = true;
  double vals_abs_max = 0.0, vals_rows = 0.0;
  bool all_lean = true;       // every fused-kernel tile is scan_lean's (the general kernel need not run)
  int local_err = 0;          // distributed: a rank-local failure, agreed on with the other ranks after the scan
  std::string local_msg;
  try {
  for (size_t gi = 0; gi < globs.size() && nbuckets; gi++) {
    const GlobInfo& g = globs[gi];
    if (g.skip) continue;
    const int vunion = value_type_of_rank(gvrank[gi]);   // the glob's union_by_name value type (-1: no value column)
    for (int si : g.segs) {
      if (!segs[si]) continue;
      const Segment& S = *segs[si];
      rows_scanned += uint64_t(S.num_rows);
      QSeg q{};
      q.base = S.d_data;
      q.tiles = S.d_tiles;
      q.ntiles = uint32_t(S.tiles.size());
      q.glob_slot = per_glob_cells ? uint32_t(gi) : 0;
      q.leaf_false = g.leaf_false;
      q.win_lo = g.win_lo;
      q.win_hi = g.win_hi;
      bool general = numeric && !vleaf;
      // (column types were checked per glob above: a type the query cannot bind emptied the glob)
      auto bind = [&](int qc, const std::string& name, bool want_string) {
        int c = S.col_index(name);
        if (c < 0) {
          if (S.all_columns.count(name))
            throw PlanError(LK_ERR_DEVICE, "internal: column " + name + " of an unloaded type in a live glob");
          return;
        }
        const HostCol& hc = S.cols[c];
        if (want_string != hc.is_string)
          throw PlanError(LK_ERR_DEVICE, "internal: column " + name + " of an unexpected type in a live glob");
        uint32_t pad = uint32_t(hc.ptype);
        if (qc == 0 && hc.ptype != pq::INT64) general = true;   // INT32 timestamps: sign-extended
        if (qc == 1) {
          if (hc.ptype != pq::DOUBLE) general = true;
          // an integer value column in a glob whose value type is FLOAT is cast to FLOAT first (DuckDB's implicit
          // BIGINT -> FLOAT of the union column), then aggregated as a float
          if (vunion == pq::FLOAT && hc.ptype != pq::FLOAT) pad |= VCONV_VIA_FLOAT;
          if (hc.int_abs_max < 0.0) vals_integral = false;
          vals_abs_max = std::max(vals_abs_max, hc.int_abs_max);
          vals_rows += double(S.num_rows);
        }
        q.cols[qc] = QCol{hc.d_pages, hc.d_runs, hc.d_tcols, hc.d_remap, 1u, pad};
        alg_bytes += hc.compressed_bytes;
      };
      bind(0, kTimestamp, false);
      if (!q.cols[0].present) continue;            // no timestamps: every row fails the window
      if (!no_value_col) bind(1, vcol, false);     // COUNT(*) / metrics `ces` read no value column
      for (size_t s = 0; s < strs.size(); s++) bind(2 + dev_of[s], strs[s].name, true);
      for (size_t n = 0; n < nums.size(); n++) bind(int(2 + strs.size() + n), nums[n], false);
      // scan_lean takes every tile of this segment when no page of its three columns holds a NULL and every
      // name page has a small dictionary (lean_tile's test at page granularity)
      bool seg_lean = !general;
      if (seg_lean) {
        const int ct = S.col_index(kTimestamp), cv = no_value_col ? -1 : S.col_index(vcol);
        const int cn = strs.size() <= 3 ? S.col_index(strs[size_t(lead)].name) : -1;
        seg_lean = ct >= 0 && (cv >= 0 || no_value_col) && cn >= 0 && !S.cols[ct].any_nulls &&
                   (no_value_col || !S.cols[cv].any_nulls) &&
                   !S.cols[cn].any_nulls;
        for (size_t s2 = 0; s2 < strs.size() && seg_lean; s2++) {   // late columns: absent, or NULL-free dictionaries
          if (int(s2) == lead) continue;
          const int cl = S.col_index(strs[s2].name);
          if (cl < 0) continue;
          if (S.cols[cl].any_nulls || !S.cols[cl].pages_lean_late) seg_lean = false;
        }
        if (seg_lean && !S.cols[cn].pages_lean_name) seg_lean = false;
      }
      // vleaf: only scan_lean tests the value leaves -- a segment it does not take whole goes to the general row scan
      if (vleaf && (!seg_lean || !vleaf_shape)) general = true;
      if (general) {
        q.tile_begin = total_tiles;
        seg_begin.push_back(total_tiles);
        total_tiles += q.ntiles;
        gsegs.push_back(q);
        continue;
      }
      all_lean = all_lean && seg_lean;
      q.tile_begin = total_tiles;
      seg_begin.push_back(total_tiles);
      total_tiles += q.ntiles;
      qsegs.push_back(q);
    }
  }

  if (seg_begin.size() > 65535) throw PlanError(LK_ERR_UNSUPPORTED, "more than 65535 segments in one evaluation");
  if (total_tiles >= (1u << 31)) throw PlanError(LK_ERR_UNSUPPORTED, "too many tiles");
  } catch (const PlanError& e) {
    if (!dist) throw;
    local_err = e.code;
    local_msg = e.what();
    qsegs.clear();
    gsegs.clear();
    total_tiles = 0;
  }
  stage("qsegs");
  uint32_t max_tiles = 0, gmax_tiles = 0;
  for (auto& q : qsegs) max_tiles = std::max(max_tiles, q.ntiles);
  for (auto& q : gsegs) gmax_tiles = std::max(gmax_tiles, q.ntiles);
  // ---- table mode ----
  // Dense: array index = cell key = (glob slot, bucket, group).  Hash (SURVEY §2.2 K4 spill, high cardinality):
  // an open-addressing table keyed by the cell key, first sized from a bound on the distinct cells and grown
  // (the scan re-run) when the bound was optimistic.  Every passing row lands in one cell, so the distinct cells
  // never exceed the rows scanned.
  const uint64_t dense_max = getenv("LK_DENSE_MAX_CELLS") ? uint64_t(atoll(getenv("LK_DENSE_MAX_CELLS")))
                                                          : (uint64_t(1) << 26);
  const bool hash_mode = sketch || ces || ncells > dense_max;   // sketch keys: (cell, bin), sparse
  if (sketch && double(ncells) * double(DD_NBINS) > 9.0e18) throw PlanError(LK_ERR_UNSUPPORTED, "sketch key space beyond 64 bits");
  auto pow2 = [](uint64_t x) {
    uint64_t p = 1;
    while (p < x) p <<= 1;
    return p;
  };
  const double key_space = double(ncells) * (sketch ? double(DD_NBINS) : 1.0);   // distinct keys <= both
  const uint64_t hash_bound = std::max<uint64_t>(1, key_space < double(rows_scanned) ? uint64_t(key_space) : rows_scanned);
  const uint64_t cap_max = std::max<uint64_t>(pow2(2 * hash_bound), 1 << 16);
  uint64_t cap = hash_mode ? std::min<uint64_t>(cap_max, std::max<uint64_t>(1 << 16, std::min<uint64_t>(pow2(2 * hash_bound), 1 << 25))) : 0;
  if (hash_mode && getenv("LK_HASH_INIT_SLOTS"))   // tests only: a deliberately small first table (regrowth path)
    cap = std::min<uint64_t>(cap_max, pow2(std::max<uint64_t>(64, uint64_t(atoll(getenv("LK_HASH_INIT_SLOTS"))))));

  // ---- device: upload, zero table, scan ----
  stage("truth");
  const double plan_ms = ms_since(t_start);
  hipStream_t st = X->stream;
  QParams P{};
  P.nsegs = uint32_t(qsegs.size());
  P.total_tiles = total_tiles;
  P.max_tiles = max_tiles;
  P.fast_div = (step > 0 && step < (int64_t(1) << 31) && nbuckets &&
                max_hi - bucket_base < (int64_t(1) << 32)) ? 1 : 0;
  P.inv_step = 1.0 / double(step > 0 ? step : 1);
  P.nstr = uint32_t(strs.size());
  P.nleaves = uint32_t(leaves.size());
  P.nprog = uint32_t(prog.size());
  P.metrics = metrics ? 1 : 0;
  P.step = step > 0 ? step : 1;
  P.bucket_base = bucket_base;
  P.nbuckets = nbuckets;
  P.ngroups = ngroups;
  P.ncells = ncells;
  std::vector<StrParam> strp(strs.size());
  for (size_t s = 0; s < strs.size(); s++) {
    StrParam& sp = strp[size_t(dev_of[s])];   // device order (query column 2 + dev_of[s])
    sp.dim_null = strs[s].dim_null;
    sp.dim_stride = strs[s].is_dim ? uint32_t(strs[s].stride) : 0u;
    sp.lbase = strs[s].lbase;
    sp.lmask = strs[s].lmask;
    sp.hmask = strs[s].hmask;
  }
  memcpy(P.prog, prog.data(), prog.size());
  if (const char* ab = getenv("LK_ABLATE")) P.ablate = uint32_t(atoi(ab));   // diagnostics only

  // staging layout in one pinned buffer + one device workspace
  size_t off = 0;
  auto reserve = [&](size_t n) { size_t o = (off + 255) / 256 * 256; off = o + n; return o; };
  const size_t o_segs = reserve(qsegs.size() * sizeof(QSeg));
  const size_t o_gsegs = reserve(gsegs.size() * sizeof(QSeg));
  const size_t o_truth = reserve(truth.size() * 4);
  const size_t o_truth_x = reserve(truth_x.size() * 4);
  const size_t o_truth_e = reserve(truth_early.size() * 4);
  const size_t o_truth_l = reserve(truth_late.size() * 4);
  std::vector<size_t> o_tab(strs.size());
  for (size_t s = 0; s < strs.size(); s++) o_tab[s] = need_tab[s] ? reserve(tabs[s].size() * 4) : 0;
  const size_t o_flags = reserve(sizeof(uint32_t) * 4);
  const size_t o_strp = reserve(strp.size() * sizeof(StrParam));
  std::vector<uint32_t> name_rank;
  const bool collapse = merged && gbs.empty() && !tagq;
  if (collapse && strs[0].is_dim) {
    // "tags of the first input" (TimeGroupedSketchAggregator.scala:57-60) is arrival-order dependent in the
    // reference; we pick the smallest name string among the merged cells, deterministically.
    // Order = the row's resulting tag map as a sorted (key, value) list: {"name": v}, or the first glob's
    // queryTags when the name is NULL / "null" / "" (Commons.scala:433, 450-452).
    using TagList = std::vector<std::pair<std::string, std::string>>;
    TagList qt = globs[0].query_tags;
    std::sort(qt.begin(), qt.end());
    std::vector<std::pair<TagList, uint32_t>> order;
    GlobalDict& gd = E.dict(kName);
    std::lock_guard<std::mutex> g(gd.mu);
    for (uint32_t d = 0; d < strs[0].ndim; d++) {
      const std::string_view v = d == strs[0].dim_null ? std::string_view() : strs[0].dim_value(d, gd);
      if (!null_like(v)) order.emplace_back(TagList{{"name", std::string(v)}}, d);
      else order.emplace_back(qt, d);
    }
    std::sort(order.begin(), order.end());
    name_rank.assign(strs[0].ndim, 0);
    for (uint32_t r = 0; r < order.size(); r++) name_rank[order[r].second] = r;
  }
  const size_t o_rank = reserve(name_rank.size() * 4);
  // null-like group values folded after per-glob aggregation (merged min/max over NULL-able values)
  std::vector<uint32_t> flat;
  std::vector<size_t> map_off(strs.size(), SIZE_MAX);
  if (rekey)
    for (size_t s = 0; s < strs.size(); s++)
      if (!fold_maps[s].empty()) {
        map_off[s] = flat.size();
        flat.insert(flat.end(), fold_maps[s].begin(), fold_maps[s].end());
      }
  const size_t o_maps = reserve(flat.size() * 4);
  const size_t stage_bytes = off;
  const size_t o_tail = reserve(64);   // host side only: the small-table epilogue's flags and row count (mapped)
  // host side only (mapped): the first row of every bucket, when a large result's timestamps are expanded on the host
  const bool ts_runs_ok = nbuckets <= kTsRunsMaxBuckets && !getenv("LK_NO_TS_RUNS");
  const size_t o_bpos = reserve(ts_runs_ok ? (size_t(nbuckets) + 1) * 4 : 0);
  // host side only (mapped): the existence bit of every output key of a large grouped result (FParams::key_bits)
  const uint64_t okeys = per_glob_rows ? ncells : (collapse ? nbuckets : nbuckets * ngroups);
  // default since r06 (LK_NO_KEY_ROWS=1 for A/B): with the row expansion on the job's whole thread share it runs while
  // the values cross the host link -- C5 eval 2.64 -> 1.93 ms (profiles/r06_ab_c5_*); r05's 8-thread expansion measured
  // slower (2.28 vs 2.13 ms)
  const bool key_rows_ok = !collapse && okeys >= kTsRunsMinKeys && !getenv("LK_NO_KEY_ROWS");
  const size_t o_kbits = reserve(key_rows_ok ? size_t((okeys + 2047) / 2048) * 2048 / 8 : 0);
  // staging buffers: a rank-local failure here is agreed on after the scan stage (no scan runs on this rank)
  uint8_t* hbuf = nullptr;
  uint8_t* dbuf = nullptr;
  try {
    HIP_TRY(hipSetDevice(E.device));
    hbuf = static_cast<uint8_t*>(X->pinned_buf(off + 64));
    dbuf = static_cast<uint8_t*>(X->workspace("query", stage_bytes));
  } catch (const PlanError& e) {
    if (!dist) throw;
    if (!local_err) {
      local_err = e.code;
      local_msg = e.what();
    }
  }
  if (hbuf && dbuf) {
  memcpy(hbuf + o_segs, qsegs.data(), qsegs.size() * sizeof(QSeg));
  memcpy(hbuf + o_gsegs, gsegs.data(), gsegs.size() * sizeof(QSeg));
  if (!truth.empty()) memcpy(hbuf + o_truth, truth.data(), truth.size() * 4);
  if (!truth_x.empty()) memcpy(hbuf + o_truth_x, truth_x.data(), truth_x.size() * 4);
  if (late_mask) {
    memcpy(hbuf + o_truth_e, truth_early.data(), truth_early.size() * 4);
    memcpy(hbuf + o_truth_l, truth_late.data(), truth_late.size() * 4);
  }
  for (size_t s = 0; s < strs.size(); s++)
    if (need_tab[s]) {
      memcpy(hbuf + o_tab[s], tabs[s].data(), tabs[s].size() * 4);
      strp[size_t(dev_of[s])].strtab = reinterpret_cast<const uint32_t*>(dbuf + o_tab[s]);
    } else if (strs[s].exchanged) {
      strp[size_t(dev_of[s])].strtab = strs[s].uni->d_dim_of_gid;   // resident (dims.cpp)
    }
  memcpy(hbuf + o_strp, strp.data(), strp.size() * sizeof(StrParam));
  memset(hbuf + o_flags, 0, 16);
  if (!name_rank.empty()) memcpy(hbuf + o_rank, name_rank.data(), name_rank.size() * 4);
  if (!flat.empty()) memcpy(hbuf + o_maps, flat.data(), flat.size() * 4);
  const hipError_t up = hipMemcpyAsync(dbuf, hbuf, stage_bytes, hipMemcpyHostToDevice, st);
  if (up != hipSuccess) {
    (void)hipGetLastError();
    if (!dist) throw PlanError(LK_ERR_DEVICE, std::string("HIP: query upload: ") + hipGetErrorString(up));
    if (!local_err) {
      local_err = LK_ERR_DEVICE;
      local_msg = std::string("HIP: query upload: ") + hipGetErrorString(up);
    }
  }
  }
  P.segs = reinterpret_cast<const QSeg*>(dbuf + o_segs);
  P.flags = reinterpret_cast<uint32_t*>(dbuf + o_flags);
  P.truth = truth.empty() ? nullptr : reinterpret_cast<const uint32_t*>(dbuf + o_truth);
  P.late_mask = getenv("LK_NO_LATE") ? 0u : late_mask;   // env: diagnostics only (A/B of the late path)
  P.truth_early = late_mask ? reinterpret_cast<const uint32_t*>(dbuf + o_truth_e) : nullptr;
  P.truth_late = late_mask ? reinterpret_cast<const uint32_t*>(dbuf + o_truth_l) : nullptr;
  P.strp = reinterpret_cast<const StrParam*>(dbuf + o_strp);
  const uint32_t* d_maps = reinterpret_cast<const uint32_t*>(dbuf + o_maps);
  const int kagg = agg == AGG_AVG ? AGG_SUM : ((agg == AGG_ROWS || agg == AGG_SKETCH || agg == AGG_CES) ? AGG_COUNT : agg);
  // lean tables: no NULL value anywhere in the value column -> cnt == rows; min/max also imply rows
  if (!value_nulls && !no_value_col && !getenv("LK_NO_LEAN"))
    P.lean = (kagg == AGG_MIN || kagg == AGG_MAX) ? LEAN_NO_ROWS : LEAN_NO_CNT;
  // dense SUM (not AVG, which needs the row counts): existence from the -0.0 marker, no rows atomics at all
  if (P.lean == LEAN_NO_CNT && agg == AGG_SUM && !hash_mode && !sketch && !ces && !getenv("LK_NO_SUM_EXISTS"))
    P.lean |= LEAN_SUM_EXISTS;
  // single string column (filter and group dim on `name` only): NULL-free tiles with a small chunk dictionary go
  // to scan_lean (lean_kernel.hpp), the rest to scan_tiles
  // single string column (filter and group dim on `name` only), or name early with every other string column late
  // (<= 2 of them): NULL-free tiles with a small name dictionary go to scan_lean (lean_kernel.hpp), the rest to
  // scan_tiles
  const bool lean_shape = P.nstr == 1 || (P.nstr <= 3 && P.late_mask == ((1u << P.nstr) - 2u));
  P.rows_only = no_value_col ? 1u : 0u;   // COUNT(*) / metrics ces: no value column is bound (lean tiles need none)
  bool dense_shape = false;               // the single-column dense-code scan_lean shape was picked (stats)
  // late columns decoded per chunk (scan_lean<..., EARLY>) where a late filter leaf exists: the late filter then runs
  // before the rows are listed, and a listed row waits only on its value.  Opt-in (LK_LATE_CHUNK=1): measured slower
  // than the per-row late stage on C3 (3.47 vs 1.97 ms) and the tag query (2.28 vs 1.06 ms) -- every chunk pays a
  // run search and a window load per late column before its filter outcome is known
  {
    bool late_leaves = false;
    for (size_t s = 0; s < strs.size(); s++)
      if (((late_mask >> dev_of[s]) & 1u) && !strs[s].leaves.empty()) late_leaves = true;
    // tag queries: COUNT(*) counted in the chunk loop from the late window (A/B: LK_TAG_DIRECT=1)
    const bool tag_direct = tagq && getenv("LK_TAG_DIRECT") && *getenv("LK_TAG_DIRECT") == '1';
    P.late_chunk = ((late_leaves || tag_direct) && ngroups <= 65536u && (getenv("LK_LATE_CHUNK") || tag_direct)) ? 1u : 0u;
    // speculative value gather for late-filtered rows (lean_kernel.hpp rowsN): opt-in
    // (LK_SPEC_GATHER=1) -- measured slower on C3, 2.155 vs 1.968 ms: the loads of the rows the late filter drops
    // (half of C3's listed rows) cost more than the round trip they save (profiles/r05_bench_c3*.json)
    const char* sg = getenv("LK_SPEC_GATHER");
    P.spec_gather = (late_leaves && sg && *sg == '1') ? 1u : 0u;
    // one string column whose eq / in filter passes a quarter or more of its values (the dense query): the 5-wave
    // per-lane scan_lean<..., 0, EARLY> -- its dense-code tiles lose ~0.3 ms in C2's 4-wave listed shape
    // (LK_NO_DENSE_SHAPE=1: A/B).  Against the dictionary's live ids (values some cached segment references), not
    // its size, which also counts ids evicted segments left behind; the pick is in stats.lean_dense_shape.
    if (P.nstr == 1 && !strs[0].cand.empty() && !getenv("LK_NO_DENSE_SHAPE")) {
      GlobalDict& gd = E.dict(strs[0].name);
      size_t nv = 0;
      {
        std::lock_guard<std::mutex> g(gd.mu);
        nv = gd.live;
      }
      if (strs[0].cand.size() * 4 >= nv) {
        P.late_chunk = 1u;
        dense_shape = true;
      }
    }
  }
  P.lean_split = (lean_shape && P.truth && (agg != AGG_ROWS || tagq) && !sketch && (!numeric || vleaf) && !getenv("LK_NO_LEAN_SPLIT"))
                    ? (all_lean ? 2u : 1u) : 0u;
  if (numeric && !(vleaf && gsegs.empty())) P.lean = 0;   // the general row scan accumulates every table field
  if (P.lean && getenv("LK_NO_DENSE_DIRECT")) P.lean |= LEAN_NO_DENSE_DIRECT;   // env: A/B only
  // exact integer sums: every partial sum of <= vals_rows integers of magnitude <= vals_abs_max is <= 2^52 (a margin for
  // the FLOAT cast of union_by_name integer columns), so it is
  // exact in any order and the compensated sum equals the plain one bit for bit (LK_NO_EXACT_SUM=1: A/B)
  P.exact_sum = (kagg == AGG_SUM && !sketch && !ces && vals_integral && vals_abs_max * vals_rows <= 4503599627370496.0 &&
                 !getenv("LK_NO_EXACT_SUM")) ? 1u : 0u;
  // a group space far beyond scan_lean's LDS hash table (1M+ cells): register cells go straight to the global table
  P.global_cells = (uint64_t(ngroups) * nbuckets >= (1ull << 20) && !getenv("LK_LDS_CELLS")) ? 1u : 0u;
  P.split_ok = getenv("LK_NO_SPLIT") ? 0u : 1u;   // env: A/B only
  if (vleaf && !qsegs.empty()) {   // scan_lean tests the value leaves of every row its string conjuncts pass
    P.nvl = uint32_t(nleaves.size());
    P.vtab = vtab;
    for (size_t k = 0; k < nleaves.size(); k++) {
      const NumLeaf& nl = nleaves[k];
      P.vl[k] = VLeaf{nl.dlo, nl.dhi, nl.lo_incl, nl.hi_incl, nl.nan_pass, 0u};
    }
  }
  // scan_lean: a dense table whose group space fits LDS for the few buckets a tile spans is aggregated in the tile's
  // direct table (lean_kernel.hpp) instead of the LDS hash table: dir_span = the most buckets it holds
  if (P.lean_split && !hash_mode && !getenv("LK_NO_DIRECT")) {
    const uint64_t words = lean_dir_words(P.nstr - 1);
    const bool rows_plane = kagg != AGG_COUNT && !(P.lean & (LEAN_SUM_EXISTS | LEAN_NO_ROWS));
    const uint32_t cw = (kagg == AGG_SUM ? 2u : 1u) + (rows_plane ? 1u : 0u);
    // the most replicas per cell (spreading lanes that add into the same cells over more LDS addresses) that still
    // leave room for a tile spanning two buckets
    const uint32_t rep_max = getenv("LK_DIRECT_REPMAX") ? uint32_t(atoi(getenv("LK_DIRECT_REPMAX"))) : 4u;   // env: A/B
    for (uint32_t rep = rep_max >= 64 ? 64u : rep_max >= 16 ? 16u : rep_max >= 8 ? 8u : 4u; rep >= 1; rep /= 2) {
      const uint64_t w = std::min<uint64_t>(LEAN_DIR_MAXSPAN, words / (uint64_t(cw) * rep * std::max<uint64_t>(ngroups, 1)));
      if (w >= 2 || (rep == 1 && w >= 1)) {
        P.dir_span = uint32_t(w);
        P.dir_planes = cw;
        P.dir_rep = getenv("LK_DIRECT_REP1") ? 1u : rep;   // env: A/B only
        if (P.dir_rep == 1u && rep != 1u)
          P.dir_span = uint32_t(std::min<uint64_t>(LEAN_DIR_MAXSPAN, words / (uint64_t(cw) * std::max<uint64_t>(ngroups, 1))));
        break;
      }
    }
  }
  if (sketch) {
    P.sketch = 1;
    P.dd_mult = dd::mapping().multiplier;
    P.dd_min = dd::mapping().min_indexable;
    P.dd_max = dd::mapping().max_indexable;
  }

  // Single-GPU dense tables with a bounded output: the finalize is enqueued right behind the scan -- rows written by
  // the kernel into the (pinned) result block sized for every output key -- so the flags, the row count and the rows
  // come back with one stream synchronization instead of three (scan flags, row count, rows).  A re-run (metrics off
  // the step grid, MIN over NaN) discards the speculative rows.
  const uint64_t out_keys = ncells == 0 ? 0 : (per_glob_rows ? ncells : (collapse ? nbuckets : nbuckets * ngroups));
  const bool fast_final = !dist && !hash_mode && !sketch && !ces && !rekey && ncells && out_keys <= (uint64_t(1) << 20) &&
                          !getenv("LK_NO_FAST_FINAL");
  auto setup_final = [&](FParams& Fp, uint32_t fslots) {
    Fp.ngroups = ngroups;
    Fp.nbuckets = nbuckets;
    Fp.nglob_slots = fslots;
    Fp.agg = agg;
    Fp.per_glob = per_glob_rows ? 1 : 0;
    Fp.collapse = collapse ? 1 : 0;
    Fp.name_stride = strs[0].stride ? strs[0].stride : 1;
    Fp.name_rank = name_rank.empty() ? nullptr : reinterpret_cast<const uint32_t*>(dbuf + o_rank);
    Fp.bucket_base = bucket_base;
    Fp.step = P.step;
    Fp.nkeys = out_keys;
  };
  bool fast_done = false;         // rows already written by the speculative finalize
  uint32_t fast_rows = 0;

  // Zero the table (SoA [rows | cnt | hi | lo | ext (| keys)]) and scan; returns the kernel's flags.
  size_t nc = 0;
  double launch_ms = 0;
  unsigned long long plan_bytes = 0;
  auto zero_table = [&](size_t ncl, bool hashed) {
    uint8_t* tb = static_cast<uint8_t*>(X->workspace("table", ncl * 8 * (hashed ? 6 : 5) + 4 * 256));
    P.rows = reinterpret_cast<unsigned long long*>(tb);
    P.cnt = reinterpret_cast<unsigned long long*>(tb + ncl * 8);
    P.hi = reinterpret_cast<double*>(tb + ncl * 16);
    P.lo = reinterpret_cast<double*>(tb + ncl * 24);
    P.ext = reinterpret_cast<unsigned long long*>(tb + ncl * 32);
    P.hkeys = hashed ? reinterpret_cast<unsigned long long*>(tb + ncl * 40) : nullptr;
    P.hmask = hashed ? ncl - 1 : 0;
    // one launch: the planes this aggregate reads, and the scan flags + plan-bytes counter (4 x u32)
    FillList F{};
    auto add = [&](void* p, size_t n, unsigned long long v) {
      F.p[F.count] = static_cast<unsigned long long*>(p);
      F.n[F.count] = n;
      F.v[F.count] = v;
      F.count++;
    };
    add(tb, ncl * 2, 0ull);                                           // rows | cnt
    if (kagg == AGG_SUM) {
      add(P.hi, ncl, (P.lean & LEAN_SUM_EXISTS) ? NEG_ZERO_BITS : 0ull);
      add(P.lo, ncl, 0ull);
    }
    if (kagg == AGG_MIN) add(P.ext, ncl, ~0ull);
    if (kagg == AGG_MAX) add(P.ext, ncl, 0ull);
    if (hashed) add(P.hkeys, ncl, ~0ull);
    add(P.flags, 2, 0ull);                                            // flags + the 64-bit plan-bytes counter
    HIP_TRY(launch_fill_many(F, st));
  };
  // Multi-GPU reduce shape (decided before the scan: its receive buffers are placed before the scan's agreement
  // point, so no rank can fail alone between that agreement and the first point-to-point transfer).
  const char* kr_env = getenv("LK_KEYRANGE_MIN_CELLS");
  const uint64_t kr_min = kr_env ? uint64_t(atoll(kr_env)) : (uint64_t(1) << 20);
  const bool keyrange = dist && (comm_world(E) > 1 || comm_loopback(E)) && !hash_mode && !per_glob_rows && !collapse && !rekey && !sketch &&
                        !ces && nslots == 1 && ncells >= std::max<uint64_t>(kr_min, 1);
  const int W = dist ? comm_world(E) : 1;
  std::vector<uint64_t> kb(size_t(W) + 1);   // key-range bounds: rank j owns cells [kb[j], kb[j+1])
  for (int j = 0; j <= W; j++) kb[size_t(j)] = j == W ? ncells : (ncells * uint64_t(j) / uint64_t(W)) & ~63ull;
  const size_t kr_len = size_t(kb[size_t(rank) + 1] - kb[size_t(rank)]);
  auto run_scan = [&]() -> uint32_t {
    nc = hash_mode ? size_t(cap) : size_t(std::max<uint64_t>(ncells, 1));
    if (dist && !hash_mode) {   // the reduce stage's buffers
      fault_point(E, "reduce");
      if (keyrange) {
        (void)X->workspace("kr_parts", size_t(W) * 5 * kr_len * 8 + 64);
        (void)X->workspace("kr_counts", (size_t(finalize_blocks(kr_len)) + 2) * 4);
      } else {
        comm_reduce_prepare(E, *X, nc);
      }
    }
    zero_table(nc, hash_mode);   // (and the flags)
    P.plan_bytes = (flags & LK_PLAN_BYTES) ? reinterpret_cast<unsigned long long*>(P.flags + 2) : nullptr;
    HIP_TRY(hipEventRecord(X->ev_scan0, st));
    const size_t nstamp = size_t(P.max_tiles) * P.nsegs * LK_NSTAMP;
    if (getenv("LK_STAMPS") && nstamp) {   // diagnostics only: per-block phase cycle totals
      P.stamps = static_cast<unsigned long long*>(X->workspace("stamps", nstamp * 8));
      HIP_TRY(hipMemsetAsync(P.stamps, 0, nstamp * 8, st));
    }
    launch_ms = ms_since(t_start);   // host staging done, scan enqueued
    if (ncells && !qsegs.empty()) HIP_TRY(launch_scan(P, kagg, st));
    if (ncells && !gsegs.empty()) {   // general row scan (numeric comparison leaves, union_by_name promotion)
      XParams XG{};
      XG.segs = reinterpret_cast<const QSeg*>(dbuf + o_gsegs);
      XG.nsegs = uint32_t(gsegs.size());
      XG.max_tiles = gmax_tiles;
      XG.strp = P.strp;
      XG.nstr = P.nstr;
      XG.nleaves = P.nleaves;
      XG.nprog = P.nprog;
      memcpy(XG.prog, P.prog, sizeof(XG.prog));
      XG.truth = truth_x.empty() ? P.truth : reinterpret_cast<const uint32_t*>(dbuf + o_truth_x);
      XG.mode = XMODE_AGG;
      XG.nnum = uint32_t(nums.size());
      XG.nnl = uint32_t(nleaves.size());
      for (size_t i = 0; i < nleaves.size(); i++) XG.nl[i] = nleaves[i];
      XG.agg = kagg;
      XG.hash = hash_mode ? 1 : 0;
      XG.q = P;
      HIP_TRY(launch_ex_scan(XG, st));
    }
    HIP_TRY(hipEventRecord(X->ev_scan1, st));
    // small dense single-GPU tables: fixup, rows and flags in one single-workgroup launch (launch_epilogue_small),
    // read after one synchronization from mapped pinned memory -- no fixup / count / scan / write launches, no copies
    const bool epilogue = fast_final && !fast_done && !P.stamps && nc <= kEpilogueMax && out_keys <= kEpilogueMax &&
                          !getenv("LK_NO_EPILOGUE");
    if (epilogue) {
      res->alloc_rows(size_t(out_keys), per_glob_rows);
      if (res->blk.pinned) {
        FParams Fs{};
        Fs.rows = P.rows;
        Fs.cnt = P.cnt;
        Fs.hi = P.hi;
        Fs.lo = P.lo;
        Fs.ext = P.ext;
        setup_final(Fs, nslots);
        uint32_t* tail = reinterpret_cast<uint32_t*>(hbuf + o_tail);
        memset(tail, 0, 32);
        HIP_TRY(launch_epilogue_small(P, Fs, nc, kagg, res->ts, res->val, res->gid, per_glob_rows ? res->glob : nullptr,
                                      P.flags, tail, st));
        HIP_TRY(hipStreamSynchronize(st));
        fast_rows = tail[4];
        fast_done = true;
        memcpy(&plan_bytes, tail + 2, 8);
        return tail[0];
      }
    }
    if (ncells) HIP_TRY(launch_fixup_table(P, nc, kagg, st));
    if (P.stamps) {
      std::vector<unsigned long long> h(nstamp);
      HIP_TRY(hipMemcpyAsync(h.data(), P.stamps, nstamp * 8, hipMemcpyDeviceToHost, st));
      HIP_TRY(hipStreamSynchronize(st));
      static const char* names[LK_NSTAMP] = {"prologue", "defs", "decode", "fold", "filter", "compact", "prefetch", "stream"};
      double sm[LK_NSTAMP] = {};
      size_t n = 0;
      for (size_t i = 0; i < nstamp; i += LK_NSTAMP) {
        if (!(h[i] >> 63)) continue;   // block exited early (zone map / past the segment's tiles)
        h[i] &= ~(1ull << 63);
        for (int k = 0; k < LK_NSTAMP; k++) sm[k] += double(h[i + k]);
        n++;
      }
      if (n) {
        double tot = 0;
        std::string line;
        for (int k = 0; k < LK_NSTAMP; k++) {
          tot += sm[k] / n;
          line += std::string(" ") + names[k] + "=" + std::to_string(long(sm[k] / n));
        }
        fprintf(stderr, "[lk stamps] blocks=%zu mean cycles:%s total=%.0f\n", n, line.c_str(), tot);
      }
    }
    uint32_t fl[4] = {0, 0, 0, 0};
    if (fast_final && !fast_done) {
      res->alloc_rows(size_t(out_keys), per_glob_rows);
      if (res->blk.pinned) {
        FParams Fs{};
        Fs.rows = P.rows;
        Fs.cnt = P.cnt;
        Fs.hi = P.hi;
        Fs.lo = P.lo;
        Fs.ext = P.ext;
        setup_final(Fs, nslots);
        const uint32_t nb = finalize_blocks(Fs.nkeys);
        uint32_t* cnts = static_cast<uint32_t*>(X->workspace("counts", (size_t(nb) + 2) * 4));
        if (ts_runs_ok && out_keys >= kTsRunsMinKeys) Fs.bucket_pos = reinterpret_cast<uint32_t*>(hbuf + o_bpos);
        HIP_TRY(launch_finalize_count(Fs, cnts, st));
        if (Fs.bucket_pos) {
          HIP_TRY(launch_finalize_bucket_pos(Fs, cnts, st));
          HIP_TRY(hipEventRecord(X->ev_rows, st));
        }
        HIP_TRY(launch_finalize_write(Fs, cnts, Fs.bucket_pos ? nullptr : res->ts, res->val, res->gid,
                                      per_glob_rows ? res->glob : nullptr, st));
        HIP_TRY(hipMemcpyAsync(&fast_rows, cnts + nb, 4, hipMemcpyDeviceToHost, st));
        fast_done = true;
        if (Fs.bucket_pos) {   // timestamps expanded here while finalize_write's rows cross the host link
          HIP_TRY(hipMemcpyAsync(fl, P.flags, 16, hipMemcpyDeviceToHost, st));
          HIP_TRY(hipEventSynchronize(X->ev_rows));
          expand_ts_runs(E, res->ts, Fs.bucket_pos[nbuckets], Fs);
          HIP_TRY(hipStreamSynchronize(st));
          memcpy(&plan_bytes, fl + 2, 8);
          return fl[0];
        }
      }
    }
    HIP_TRY(hipMemcpyAsync(fl, P.flags, 16, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    memcpy(&plan_bytes, fl + 2, 8);
    return fl[0];
  };
  // Every rank reports (error, flags); a failure anywhere fails every rank (no rank is left in a collective),
  // and every rank sees the OR of the flags (so they re-run a too-small hash table together).
  auto agree = [&](int err, const std::string& msg, uint32_t fl) -> uint32_t {
    if (!dist) {
      if (err) throw PlanError(err, msg);
      return fl;
    }
    uint32_t all_fl = 0;
    const std::vector<std::string> all =
        comm_allgather_status(E, *X, err, msg, std::string(reinterpret_cast<const char*>(&fl), 4));
    for (const std::string& b : all) {
      uint32_t f = 0;
      memcpy(&f, b.data(), std::min<size_t>(4, b.size()));
      all_fl |= f;
    }
    return all_fl;
  };
  uint32_t hflags = 0;
  int attempts = 0;
  for (;;) {
    attempts++;
    int err = local_err;
    std::string msg = local_msg;
    uint32_t fl = 0;
    if (!err) {
      try {
        fl = run_scan();
      } catch (const PlanError& e) {
        if (!dist) throw;
        err = e.code;
        msg = e.what();
      }
    }
    // A full hash table is reported as "full, can grow" or "full at its bound" (cap and cap_max are rank-local):
    // the ranks agree on both, re-run together while any rank can grow -- each growing only its own full table --
    // and fail together when any table is full at its bound (a rank must not leave while another
    // re-runs into the next collective).
    const bool my_full = hash_mode && (fl & FLAG_HASH_FULL);
    if (my_full && cap < cap_max) fl = (fl & ~uint32_t(FLAG_HASH_FULL)) | FLAG_HASH_GROW;
    hflags = agree(err, msg, fl);
    if (hash_mode && !(hflags & FLAG_HASH_FULL) && (hflags & FLAG_HASH_GROW)) {
      if (my_full) cap = std::min<uint64_t>(cap_max, cap * 4);
      continue;
    }
    break;
  }
  const double scan_agreed_ms = ms_since(t_start);   // every rank's scan done and its status agreed
  if (hflags & FLAG_METRICS_UNALIGNED) {
    if (step == 1) throw PlanError(LK_ERR_DEVICE, "internal: metrics timestamp off a 1 ms grid");
    throw MetricsUnaligned{};
  }
  if ((hflags & FLAG_MIN_NAN) && agg == AGG_MIN && merged && !min_max_nulls) throw MinNanApart{};
  if (hflags & FLAG_CELL_RANGE) throw PlanError(LK_ERR_DEVICE, "internal: bucket outside the table");
  if (hflags & FLAG_HASH_FULL) throw PlanError(LK_ERR_MEMORY, "aggregation hash table full at its bound");
  // DDSketch.accept on NaN / a magnitude beyond the mapping's range throws in the worker's stream stage: the
  // stream fails (Commons.scala:331-335) and query-api sees an empty source
  if (hflags & FLAG_SKETCH_RANGE) throw PlanError(LK_ERR_ARG, "DDSketch: value outside the trackable range");

  // ---- multi-GPU: reduce partial tables to rank 0 over RCCL ----
  uint32_t nrows_out = 0;
  bool rows_done = false;   // key-range path: rank 0's result rows are already in place
  const char* emit_mode = "local";
  const double t_reduce0 = ms_since(t_start);
  if (dist) {
    if (hash_mode) {
      unsigned long long cap0 = cap;
      comm_reduce_hash(E, *X, P, kagg, cap0);
      cap = cap0;
      nc = size_t(cap);
    } else if (keyrange) {
      // Large dense tables (C5: 10M-key group dims), SURVEY §8(e): the merged output key is the cell index, so the
      // key space is cut into one contiguous range per rank.  All-to-all: every rank sends range j of its partial
      // table to rank j (grouped send/recv: all xGMI links at once, 7/8 of a table per rank instead of every table
      // into rank 0); rank j folds the W slices in rank order (merge_tables: the same deterministic fold) and
      // finalizes its range; the ranges' rows, already in key order, are concatenated on rank 0 in rank order.
      // (buffers placed before the scan's agreement: nothing between it and the exchange fails on one rank)
      const size_t len = kr_len;
      uint8_t* tb = reinterpret_cast<uint8_t*>(P.rows);   // [rows | cnt | hi | lo | ext], nc cells each
      uint8_t* parts = static_cast<uint8_t*>(X->workspace("kr_parts", size_t(W) * 5 * len * 8 + 64));
      std::vector<Piece> sends, recvs;
      for (int p2 = 0; p2 < W; p2++)
        for (int a = 0; a < 5; a++) {
          const size_t l2 = size_t(kb[size_t(p2) + 1] - kb[size_t(p2)]);
          sends.push_back(Piece{p2, tb + (size_t(a) * nc + kb[size_t(p2)]) * 8, l2 * 8});
          recvs.push_back(Piece{p2, parts + (size_t(p2) * 5 + size_t(a)) * len * 8, len * 8});
        }
      comm_exchange(E, *X, sends, recvs);
      TableRef T{reinterpret_cast<unsigned long long*>(parts), reinterpret_cast<unsigned long long*>(parts + len * 8),
                 reinterpret_cast<double*>(parts + 2 * len * 8), reinterpret_cast<double*>(parts + 3 * len * 8),
                 reinterpret_cast<unsigned long long*>(parts + 4 * len * 8)};
      FParams Fk{};
      Fk.rows = T.rows;
      Fk.cnt = T.cnt;
      Fk.hi = T.hi;
      Fk.lo = T.lo;
      Fk.ext = T.ext;
      Fk.ngroups = ngroups;
      Fk.nbuckets = nbuckets;
      Fk.nglob_slots = 1;
      Fk.agg = agg;
      Fk.name_stride = strs[0].stride ? strs[0].stride : 1;
      Fk.bucket_base = bucket_base;
      Fk.step = P.step;
      Fk.key_base = kb[size_t(rank)];
      Fk.cell_base = kb[size_t(rank)];
      Fk.nkeys = len;
      const uint32_t nfk = finalize_blocks(len);
      uint32_t* kc = static_cast<uint32_t*>(X->workspace("kr_counts", (size_t(nfk) + 2) * 4));
      uint32_t mine_n = 0;
      // fold + count this rank's range; a failure travels with the row-count all-gather (every rank fails there)
      comm_local(*X, [&] {
        fault_point(E, "keyrange_merge");
        if (!len) return;
        HIP_TRY(launch_merge_tables(T, reinterpret_cast<const unsigned long long*>(parts), W, len, kagg, st));
        HIP_TRY(launch_finalize_count(Fk, kc, st));
        HIP_TRY(hipMemcpyAsync(&mine_n, kc + nfk, 4, hipMemcpyDeviceToHost, st));
        HIP_TRY(hipStreamSynchronize(st));
      });
      const uint64_t n64 = mine_n;
      std::vector<uint64_t> ncnt(static_cast<size_t>(W)), noff(static_cast<size_t>(W));
      uint64_t total_rows = 0;
      {
        const std::vector<std::string> all =
            comm_allgather_status(E, *X, 0, std::string(), std::string(reinterpret_cast<const char*>(&n64), 8));
        for (int j = 0; j < W; j++) {
          memcpy(&ncnt[size_t(j)], all[size_t(j)].data(), 8);
          noff[size_t(j)] = total_rows;
          total_rows += ncnt[size_t(j)];
        }
      }
      if (total_rows >= (uint64_t(1) << 32)) throw PlanError(LK_ERR_UNSUPPORTED, "more than 2^32 result rows");
      // Parallel emission: every rank's GPU writes its range's rows straight into rank 0's result -- a shared host
      // block, columns [ts | value | group id] of total_rows each -- at the range's row offset, so the rows cross
      // every PCIe link of the node at once (otherwise: all rows into rank 0's device, then over its one link).
      const char* se = getenv("LK_SHM_EMIT");
      EmitTarget ET;
      if (total_rows && !(se && *se == '0')) ET = comm_emit_begin(E, *X, size_t(total_rows) * 20);
      if (ET.ok) {
        const size_t N = size_t(total_rows), o = size_t(noff[size_t(rank)]);
        int wst = ET.mapped ? 0 : LK_ERR_DEVICE;
        if (ET.mapped && mine_n) {
          if (launch_finalize_write(Fk, kc, reinterpret_cast<int64_t*>(ET.dev) + o,
                                    reinterpret_cast<double*>(ET.dev + N * 8) + o,
                                    reinterpret_cast<uint32_t*>(ET.dev + N * 16) + o, nullptr, st) != hipSuccess)
            wst = LK_ERR_DEVICE;
        }
        if (hipStreamSynchronize(st) != hipSuccess) wst = LK_ERR_DEVICE;
        std::string wmsg = "shared result block: mapping or write failed";
        if (!wst && getenv("LK_FAULT")) {   // tests only: an injected failure of the row write
          try {
            fault_point(E, "emit");
          } catch (const PlanError& e) {
            wst = LK_ERR_DEVICE;
            wmsg = e.what();
          }
        }
        try {
          comm_agree(E, *X, wst, wmsg);   // every range written
        } catch (...) {
          comm_emit_end(E, ET, false);     // rank 0: retire the block (a rank may not have mapped it)
          throw;
        }
        comm_emit_end(E, ET, true);   // every rank holds its mapping: this block's name can go
        if (rank == 0) {
          nrows_out = uint32_t(total_rows);
          res->adopt_rows(ET.host, N, ET.lease);
          rows_done = true;
        }
        emit_mode = "shared_host_block";
      } else {
      uint8_t* ob = nullptr;
      uint8_t* rb = nullptr;
      comm_local(*X, [&] {   // this rank's rows (and rank 0's receive buffer), agreed on before they move
        ob = static_cast<uint8_t*>(X->workspace("kr_rows_mine", size_t(mine_n) * 20 + 64));
        if (mine_n)
          HIP_TRY(launch_finalize_write(Fk, kc, reinterpret_cast<int64_t*>(ob), reinterpret_cast<double*>(ob + size_t(mine_n) * 8),
                                        reinterpret_cast<uint32_t*>(ob + size_t(mine_n) * 16), nullptr, st));
        HIP_TRY(hipStreamSynchronize(st));   // rows complete before they are sent
        if (rank == 0) rb = static_cast<uint8_t*>(X->workspace("kr_rows_all", size_t(total_rows) * 20 + 64));
      });
      comm_agree(E, *X, 0, std::string());
      std::vector<Piece> s2, r2;   // [ts 8 B | value 8 B | group id 4 B] per row, column by column
      const size_t wcol[3] = {8, 8, 4};
      for (int a = 0; a < 3; a++) s2.push_back(Piece{0, ob + size_t(a) * mine_n * 8, size_t(mine_n) * wcol[a]});
      if (rank == 0)
        for (int j = 0; j < W; j++)
          for (int a = 0; a < 3; a++)
            r2.push_back(Piece{j, rb + size_t(a) * total_rows * 8 + noff[size_t(j)] * wcol[a], size_t(ncnt[size_t(j)]) * wcol[a]});
      comm_exchange(E, *X, s2, r2);
      comm_throw_pending(*X);   // (host transport) a failed unpacking of the last round; no collective follows
      if (rank == 0) {
        nrows_out = uint32_t(total_rows);
        res->alloc_rows(nrows_out, false);
        if (nrows_out) {
          HIP_TRY(hipMemcpyAsync(res->ts, rb, size_t(nrows_out) * 8, hipMemcpyDeviceToHost, st));
          HIP_TRY(hipMemcpyAsync(res->val, rb + size_t(nrows_out) * 8, size_t(nrows_out) * 8, hipMemcpyDeviceToHost, st));
          HIP_TRY(hipMemcpyAsync(res->gid, rb + size_t(nrows_out) * 16, size_t(nrows_out) * 4, hipMemcpyDeviceToHost, st));
        }
        HIP_TRY(hipStreamSynchronize(st));
        rows_done = true;
      }
      emit_mode = "gather_to_root";
      }
    } else {
      comm_reduce_table(E, *X, P, kagg, nc);
    }
    comm_throw_pending(*X);   // past the last collective: a rank-local failure unwinds this rank alone
  }
  const double reduce_ms = ms_since(t_start) - t_reduce0;   // dist: table reduce (+ key-range emission)
  const bool emit = (!dist || rank == 0) && !rows_done;

  FParams F{};
  SParams S{};
  uint32_t nfb = 0;
  uint32_t* d_counts = nullptr;
  void* sws = nullptr;
  unsigned long long nocc = 0;
  // Percentiles: one DDSketch per (glob, step, group-key tags) -- the groupBys' values, or {"_cardinalhq.name": ""}
  // without groupBys (PushDownAggregatorStage.getGroupByKeyTags, 188-197: see below); NULL / "null" / "" values drop
  // out of the tags (Commons.scala:433).  Merged: per (step, tags).
  struct SkRow {
    int64_t ts;
    uint32_t glob;
    unsigned long long gid;
    dd::Sketch sk;
  };
  std::vector<SkRow> sk_rows;
  struct CesRow {
    int64_t ts;
    uint32_t glob;
    hll::Sketch h;
  };
  std::vector<CesRow> ces_rows;
  if (ces && emit) {
    // occupied cells -> (glob, step) -> the set of group-key strings, one HLL each
    SParams S2{};
    S2.keys = P.hkeys;
    S2.rows = P.rows;
    S2.cnt = P.cnt;
    S2.hi = P.hi;
    S2.lo = P.lo;
    S2.ext = P.ext;
    S2.cap = cap;
    const uint32_t nsb = sparse_blocks(cap);
    uint32_t* occ = static_cast<uint32_t*>(X->workspace("occ_counts", (size_t(nsb) + 2) * 4));
    HIP_TRY(launch_sparse_count(S2, occ, st));
    uint32_t n32 = 0;
    HIP_TRY(hipMemcpyAsync(&n32, occ + nsb, 4, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    nocc = n32;
    std::vector<unsigned long long> keys(nocc);
    if (nocc) {
      auto* recs = static_cast<unsigned long long*>(X->workspace("ces_recs", size_t(nocc) * 48 + 64));
      HIP_TRY(launch_table_records(P, cap, occ, recs, nocc, st));
      HIP_TRY(hipMemcpyAsync(keys.data(), recs, nocc * 8, hipMemcpyDeviceToHost, st));
      HIP_TRY(hipStreamSynchronize(st));
    }
    // key string of each cell: groupBys.map(g => tags.getOrElse(g, "")).mkString(":") (Aggregator.scala:53-56)
    std::vector<std::string> kstr(nocc);
    for (size_t gi2 = 0; gi2 < R.group_bys.size(); gi2++) {
      StrCol& sc = strs[size_t(str_index(R.group_bys[gi2]))];
      GlobalDict& gd = E.dict(sc.name);
      std::lock_guard<std::mutex> g(gd.mu);
      for (size_t i = 0; i < nocc; i++) {
        const uint32_t d = uint32_t((keys[i] % ngroups) / (sc.stride ? sc.stride : 1) % sc.ndim);
        if (gi2) kstr[i] += ':';
        if (d != sc.dim_null && sc.stride) {
          const std::string_view v = sc.dim_value(d, gd);
          if (!null_like(v)) kstr[i] += v;
        }
      }
    }
    std::map<std::pair<uint64_t, uint32_t>, size_t> at;   // (step, glob) -> row
    for (size_t i = 0; i < nocc; i++) {
      const unsigned long long cell = keys[i];
      const uint64_t b = (cell / ngroups) % nbuckets;
      const uint32_t slot = per_glob_rows ? uint32_t(cell / ngroups / nbuckets) : 0u;
      auto ins = at.emplace(std::make_pair(b, slot), ces_rows.size());
      if (ins.second) ces_rows.push_back(CesRow{bucket_base + int64_t(b) * P.step, slot, hll::Sketch{}});
      ces_rows[ins.first->second].h.update(kstr[i]);
    }
    std::vector<CesRow> sorted;   // std::map order: (step, glob) ascending
    sorted.reserve(ces_rows.size());
    for (auto& kv : at) sorted.push_back(std::move(ces_rows[kv.second]));
    ces_rows.swap(sorted);
    nrows_out = uint32_t(ces_rows.size());
  }
  if (ces) {
  } else if (sketch) {
    if (emit) {
      SParams S2{};
      S2.keys = P.hkeys;
      S2.rows = P.rows;
      S2.cnt = P.cnt;
      S2.hi = P.hi;
      S2.lo = P.lo;
      S2.ext = P.ext;
      S2.cap = cap;
      const uint32_t nsb = sparse_blocks(cap);
      uint32_t* occ = static_cast<uint32_t*>(X->workspace("occ_counts", (size_t(nsb) + 2) * 4));
      HIP_TRY(launch_sparse_count(S2, occ, st));
      uint32_t n32 = 0;
      HIP_TRY(hipMemcpyAsync(&n32, occ + nsb, 4, hipMemcpyDeviceToHost, st));
      HIP_TRY(hipStreamSynchronize(st));
      nocc = n32;
      std::vector<unsigned long long> keys(nocc), cnts(nocc);
      if (nocc) {
        auto* recs = static_cast<unsigned long long*>(X->workspace("sketch_recs", size_t(nocc) * 48 + 64));
        HIP_TRY(launch_table_records(P, cap, occ, recs, nocc, st));
        HIP_TRY(hipMemcpyAsync(keys.data(), recs, nocc * 8, hipMemcpyDeviceToHost, st));
        HIP_TRY(hipMemcpyAsync(cnts.data(), recs + nocc, nocc * 8, hipMemcpyDeviceToHost, st));
        HIP_TRY(hipStreamSynchronize(st));
      }
      // group term of each record's key tags
      std::vector<unsigned long long> kg(nocc, 0);
      std::vector<unsigned long long> cellv(nocc);
      for (size_t i = 0; i < nocc; i++) cellv[i] = keys[i] / DD_NBINS;
      const bool by_name = gbs.empty();
      const bool name_grouped = std::find(gbs.begin(), gbs.end(), std::string(kName)) != gbs.end();
      for (size_t si = 0; si < strs.size(); si++) {
        StrCol& sc = strs[si];
        if (!sc.is_dim || !sc.stride) continue;
        const bool drop = si == 0 && !by_name && !name_grouped;   // name is no key tag when groupBys exist
        if (drop) continue;   // the name is no key tag (its column is hidden): no group term
        if (si == 0 && by_name) {
          // no groupBys: getGroupByKeyTags reads `datapoint.tags.getOrElse(NAME, "")` with NAME = "_cardinalhq.name"
          // (PushDownAggregatorStage.scala:188-197, Commons.scala:45), but the row's name tag is labelled `name` (the
          // SQL's `"_cardinalhq.name" as name`): every row's key tags are {"_cardinalhq.name": ""} -- one sketch per
          // step, every name in it: no group term (the tag column reads "" for every row: tcols[0] below).
          continue;
        }
        GlobalDict& gd = E.dict(sc.name);
        std::lock_guard<std::mutex> g(gd.mu);
        std::unordered_map<uint32_t, bool> nl;
        for (size_t i = 0; i < nocc; i++) {
          uint32_t d = uint32_t((cellv[i] % ngroups) / sc.stride % sc.ndim);
          if (d != sc.dim_null) {
            auto it = nl.find(d);
            if (it == nl.end()) it = nl.emplace(d, null_like(sc.dim_value(d, gd))).first;
            if (it->second) d = sc.dim_null;
          }
          kg[i] += (unsigned long long)d * sc.stride;
        }
      }
      std::map<std::tuple<uint64_t, uint32_t, unsigned long long>, size_t> at;   // (bucket, glob, key) -> row
      for (size_t i = 0; i < nocc; i++) {
        const unsigned long long cell = cellv[i];
        const uint64_t b = (cell / ngroups) % nbuckets;
        const uint32_t slot = uint32_t(cell / ngroups / nbuckets);
        auto ins = at.emplace(std::make_tuple(b, per_glob_rows ? slot : 0u, kg[i]), sk_rows.size());
        if (ins.second)
          sk_rows.push_back(SkRow{bucket_base + int64_t(b) * P.step, per_glob_rows ? slot : 0u, kg[i], dd::Sketch{}});
        sk_rows[ins.first->second].sk.add_bin(uint32_t(keys[i] % DD_NBINS), double(cnts[i]));
      }
      std::vector<size_t> ord(sk_rows.size());
      for (size_t i = 0; i < ord.size(); i++) ord[i] = i;
      std::sort(ord.begin(), ord.end(), [&](size_t a, size_t b) {
        const SkRow &x = sk_rows[a], &y = sk_rows[b];
        return x.ts != y.ts ? x.ts < y.ts : (x.glob != y.glob ? x.glob < y.glob : x.gid < y.gid);
      });
      std::vector<SkRow> sorted;
      sorted.reserve(ord.size());
      for (size_t i : ord) sorted.push_back(std::move(sk_rows[i]));
      sk_rows.swap(sorted);
      nrows_out = uint32_t(sk_rows.size());
    }
  } else if (!hash_mode) {
    // ---- merged min/max with NULL-able values: fold null-like group values per glob-cell SQL value ----
    F.rows = P.rows;
    F.cnt = P.cnt;
    F.hi = P.hi;
    F.lo = P.lo;
    F.ext = P.ext;
    uint32_t fslots = nslots;
    if (rekey && emit && ncells) {
      const size_t n2 = size_t(nbuckets * ngroups);
      uint8_t* t2 = static_cast<uint8_t*>(X->workspace("table2", n2 * 24 + 256));
      RParams RP{};
      RP.in_rows = P.rows;
      RP.in_cnt = P.cnt;
      RP.in_ext = P.ext;
      RP.ncells_in = ncells;
      RP.out_rows = reinterpret_cast<unsigned long long*>(t2);
      RP.out_cnt = reinterpret_cast<unsigned long long*>(t2 + n2 * 8);
      RP.out_ext = reinterpret_cast<unsigned long long*>(t2 + n2 * 16);
      RP.nbuckets = nbuckets;
      RP.ngroups = ngroups;
      RP.agg = kagg;
      for (size_t s = 0; s < strs.size(); s++) {
        if (!strs[s].is_dim) continue;
        RP.stride[RP.ndims] = strs[s].stride;
        RP.ndim[RP.ndims] = strs[s].ndim;
        RP.map[RP.ndims] = map_off[s] == SIZE_MAX ? nullptr : d_maps + map_off[s];
        RP.ndims++;
      }
      HIP_TRY(hipMemsetAsync(t2, 0, n2 * 16, st));
      HIP_TRY(hipMemsetAsync(RP.out_ext, kagg == AGG_MIN ? 0xff : 0, n2 * 8, st));
      HIP_TRY(launch_rekey_minmax(RP, st));
      F.rows = RP.out_rows;
      F.cnt = RP.out_cnt;
      F.ext = RP.out_ext;
      fslots = 1;
    }

    // ---- finalize + compaction ----
    setup_final(F, fslots);
    nfb = finalize_blocks(F.nkeys);
    d_counts = static_cast<uint32_t*>(X->workspace("counts", (size_t(nfb) + 2) * 4));
    if (fast_done) {
      nrows_out = fast_rows;   // rows already in the result block (speculative finalize behind the scan)
    } else if (emit && F.nkeys) {
      if (key_rows_ok && F.nkeys == okeys && !F.key_base) F.key_bits = reinterpret_cast<unsigned long long*>(hbuf + o_kbits);
      HIP_TRY(launch_finalize_count(F, d_counts, st));
      HIP_TRY(hipMemcpyAsync(&nrows_out, d_counts + nfb, 4, hipMemcpyDeviceToHost, st));
    }
  } else if (emit) {
    // ---- sparse finalize: occupied slots -> (output key, slot) -> radix sort -> one row per output key ----
    S.keys = P.hkeys;
    S.rows = P.rows;
    S.cnt = P.cnt;
    S.hi = P.hi;
    S.lo = P.lo;
    S.ext = P.ext;
    S.cap = cap;
    S.ngroups = ngroups;
    S.nbuckets = nbuckets;
    S.nslots = nslots;
    S.agg = agg;
    S.per_glob = per_glob_rows ? 1 : 0;
    S.collapse = collapse ? 1 : 0;
    S.rekey = rekey ? 1 : 0;
    for (size_t s = 0; s < strs.size() && rekey; s++) {
      if (!strs[s].is_dim) continue;
      S.stride[S.ndims] = strs[s].stride;
      S.ndim[S.ndims] = strs[s].ndim;
      S.map[S.ndims] = map_off[s] == SIZE_MAX ? nullptr : d_maps + map_off[s];
      S.ndims++;
    }
    S.name_stride = strs[0].stride ? strs[0].stride : 1;
    S.name_rank = name_rank.empty() ? nullptr : reinterpret_cast<const uint32_t*>(dbuf + o_rank);
    S.bucket_base = bucket_base;
    S.step = P.step;
    const uint32_t nsb = sparse_blocks(cap);
    uint32_t* occ = static_cast<uint32_t*>(X->workspace("occ_counts", (size_t(nsb) + 2) * 4));
    HIP_TRY(launch_sparse_count(S, occ, st));
    uint32_t n32 = 0;
    HIP_TRY(hipMemcpyAsync(&n32, occ + nsb, 4, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    nocc = n32;
    const unsigned long long max_key =
        per_glob_rows ? nbuckets * nslots * ngroups : (collapse ? nbuckets : nbuckets * ngroups);
    int end_bit = 1;
    while (end_bit < 64 && (1ull << end_bit) < max_key) end_bit++;
    sws = X->workspace("sparse", sparse_workspace_bytes(nocc, end_bit));
    uint32_t* d_nrows = nullptr;
    HIP_TRY(launch_sparse_sort(S, occ, nocc, end_bit, sws, &d_nrows, st));
    HIP_TRY(hipMemcpyAsync(&nrows_out, d_nrows, 4, hipMemcpyDeviceToHost, st));
  }
  if (!fast_done) HIP_TRY(hipStreamSynchronize(st));
  const double sync_ms = ms_since(t_start);     // scan + merge + finalize done
  if (fast_done) res->nrows = nrows_out;       // the block holds out_keys rows' room; nrows_out of them are written
  else if (!rows_done) res->alloc_rows(nrows_out, per_glob_rows);
  const double alloc_ms = ms_since(t_start);
  if (ces) {
    for (size_t r = 0; r < nrows_out; r++) {
      res->ts[r] = ces_rows[r].ts;
      res->val[r] = ces_rows[r].h.estimate();
      res->gid[r] = 0;
      if (per_glob_rows) res->glob[r] = ces_rows[r].glob;
      if (res->keep_sketches) res->hll_objs.push_back(ces_rows[r].h);
    }
  } else if (sketch) {
    res->sketches.reserve(nrows_out);
    for (size_t r = 0; r < nrows_out; r++) {
      const SkRow& k = sk_rows[r];
      res->ts[r] = k.ts;
      res->val[r] = k.sk.quantile(quantile);
      res->gid[r] = uint32_t(k.gid);
      if (per_glob_rows) res->glob[r] = k.glob;
      res->sketches.push_back(k.sk.serialize());
      if (res->keep_sketches) res->dd_objs.push_back(k.sk);
    }
  } else if (nrows_out && !rows_done && !fast_done) {
    // Rows written by the kernel straight into the mapped pinned result block when it is pinned: no device->host
    // copies (small async D2H copies cost ~1 ms of completion latency each call on this stack, measured in C4).
    const bool direct = res->blk.pinned;
    const size_t nk = direct ? 1 : nrows_out;
    uint8_t* ob = static_cast<uint8_t*>(X->workspace("out", nk * (8 + 8 + 8 + 4) + 1024));
    int64_t* o_ts = direct ? res->ts : reinterpret_cast<int64_t*>(ob);
    double* o_val = direct ? res->val : reinterpret_cast<double*>(ob + nk * 8);
    uint32_t* o_gid = direct ? res->gid : reinterpret_cast<uint32_t*>(ob + nk * 16);
    uint32_t* o_glob = per_glob_rows ? (direct ? res->glob : reinterpret_cast<uint32_t*>(ob + nk * 24)) : nullptr;
    // large grouped results: values only; timestamps, group ids and globs from the key bits (finalize_count's, already
    // on the host) while the values cross the host link
    const bool key_rows = direct && !hash_mode && F.key_bits;
    const bool ts_runs = direct && !hash_mode && !key_rows && ts_runs_ok && F.nkeys >= kTsRunsMinKeys;
    if (ts_runs) {
      F.bucket_pos = reinterpret_cast<uint32_t*>(hbuf + o_bpos);
      HIP_TRY(launch_finalize_bucket_pos(F, d_counts, st));
      HIP_TRY(hipEventRecord(X->ev_rows, st));
    }
    if (hash_mode) HIP_TRY(launch_sparse_write(S, nocc, sws, o_ts, o_val, o_gid, o_glob, st));
    else if (key_rows) HIP_TRY(launch_finalize_write(F, d_counts, nullptr, o_val, nullptr, nullptr, st));
    else HIP_TRY(launch_finalize_write(F, d_counts, ts_runs ? nullptr : o_ts, o_val, o_gid, o_glob, st));
    if (!direct) {
      HIP_TRY(hipMemcpyAsync(res->ts, o_ts, size_t(nrows_out) * 8, hipMemcpyDeviceToHost, st));
      HIP_TRY(hipMemcpyAsync(res->val, o_val, size_t(nrows_out) * 8, hipMemcpyDeviceToHost, st));
      HIP_TRY(hipMemcpyAsync(res->gid, o_gid, size_t(nrows_out) * 4, hipMemcpyDeviceToHost, st));
      if (per_glob_rows) HIP_TRY(hipMemcpyAsync(res->glob, o_glob, size_t(nrows_out) * 4, hipMemcpyDeviceToHost, st));
    }
    if (ts_runs) {   // timestamps expanded here while finalize_write's rows cross the host link
      HIP_TRY(hipEventSynchronize(X->ev_rows));
      expand_ts_runs(E, res->ts, nrows_out, F);
    }
    if (key_rows)
      expand_rows_from_keys(E, res->ts, res->gid, per_glob_rows ? res->glob : nullptr, F.key_bits, F, per_glob_rows);
    HIP_TRY(hipStreamSynchronize(st));
  }
  const double copy_ms = ms_since(t_start);
  const double device_ms = copy_ms - plan_ms;
  float scan_ms = 0;
  if (!local_err && ncells) HIP_TRY(hipEventElapsedTime(&scan_ms, X->ev_scan0, X->ev_scan1));

  // ---- tags: "name", groupBys (as written), then queryTags keys (rows whose own tags are all absent) ----
  std::vector<int> col_str;   // tag column -> string column index
  res->tag_names.push_back(tagq ? R.tag_name : std::string("name"));
  col_str.push_back(0);
  if (!tagq)
    for (auto& g : R.group_bys) {
      res->tag_names.push_back(g);
      col_str.push_back(str_index(g));
    }
  const size_t nreg = res->tag_names.size();
  std::vector<std::string> qt_keys;
  for (auto& g : globs)
    for (auto& kv : g.query_tags)
      if (!tagq && !sketch && !ces && std::find(qt_keys.begin(), qt_keys.end(), kv.first) == qt_keys.end()) qt_keys.push_back(kv.first);
  for (auto& k : qt_keys) res->tag_names.push_back(k);
  // Per tag column: how a row's group id decodes to the tag string (lk_result::tag; nullptr: tag dropped,
  // Commons.scala:433).  Strings local to this call (filter candidates, the distributed union) move into the
  // result once; engine-dictionary strings are read in place (stable addresses, StableStrs).
  res->per_glob = per_glob_rows;
  res->tcols.resize(nreg);
  for (size_t c = 0; c < nreg; c++) {
    StrCol& sc = strs[col_str[c]];
    lk_result::TagCol& tc = res->tcols[c];
    tc.stride = sc.stride ? sc.stride : 1;
    tc.ndim = sc.ndim;
    tc.dim_null = sc.dim_null;
    {
      GlobalDict& gd = E.dict(sc.name);
      std::lock_guard<std::mutex> g(gd.mu);
      tc.dict_keep = gd.vals;   // this generation's block stays alive with the result
      tc.dict = tc.dict_keep.get();
    }
    tc.engine = &E;
    tc.engine_life = E.life;
    tc.col = sc.name;
    tc.dict_n = sc.dict_n;
    if (sc.exchanged) {   // the agreed union's text table, shared (no copy): 10M-value dims cost nothing here
      tc.shared = sc.uni->text;
      tc.keep = sc.uni;
      continue;
    }
    if (!sc.restricted) continue;
    auto& m = tc.local;
    bool shared = false;
    for (size_t c2 = 0; c2 < c && !shared; c2++)   // a groupBy listed twice shares the first column's strings
      if (col_str[c2] == col_str[c] && !res->tcols[c2].local.empty()) {
        m = res->tcols[c2].local;
        shared = true;
      }
    if (shared) continue;
    m.assign(sc.ndim, nullptr);
    for (uint32_t d = 0; d < sc.ndim; d++) {
      if (d == sc.dim_null) continue;
      const std::string& v = sc.cand[d];
      if (null_like(v)) continue;
      res->owned.push_back(v);                                 // a few filter candidates: copied
      m[d] = res->owned.back().c_str();
    }
  }
  if (sketch && gbs.empty()) {   // key tags {"_cardinalhq.name": ""} (getOrElse(NAME, ""): see the sketch rows above)
    res->tag_names[0] = kName;
    lk_result::TagCol& tc = res->tcols[0];
    tc = lk_result::TagCol{};    // one dim id, whose text is ""
    tc.ndim = 1;
    tc.dim_null = 1;
    res->owned.push_back(std::string());
    tc.local.assign(1, res->owned.back().c_str());
  }
  if (sketch && !gbs.empty()) res->tcols[0].hidden = true;     // key tags: the groupBys only
  if (ces)   // the HLL SketchInput carries no tags (Aggregator.scala:58)
    for (auto& tc : res->tcols) tc.hidden = true;
  if (tagq) {
    // Tag-query rows (Commons.toDataPoint, Commons.scala:406-423): every column becomes a tag -- the tag and
    // "count" (COUNT(*) via getString) -- then NoisyTagsDropper.remove (NoisyTagsDropper.scala) drops hidden
    // tag names and NULL / "" / "null" values; timestamp = System.currentTimeMillis(), value 0.0 in the
    // reference (unused downstream: the payload is the tag map, QueryEngineV2.scala:473-477).  Here `value`
    // carries the count.
    res->tcols[0].hidden = noisy_tag(R.tag_name);
    res->tag_names.push_back("count");
    res->count_col = int(res->tag_names.size() - 1);
    res->count_str.reserve(nrows_out);
    const int64_t now_ms = std::chrono::duration_cast<std::chrono::milliseconds>(
                               std::chrono::system_clock::now().time_since_epoch()).count();
    for (size_t r = 0; r < nrows_out; r++) {
      res->ts[r] = now_ms;
      res->count_str.push_back(std::to_string((unsigned long long)res->val[r]));
    }
  }
  res->qt_of_glob.resize(globs.size());
  for (size_t gi = 0; gi < globs.size() && !sketch && !ces; gi++)
    for (auto& kv : globs[gi].query_tags) {
      size_t c = nreg + size_t(std::find(qt_keys.begin(), qt_keys.end(), kv.first) - qt_keys.begin());
      res->owned.push_back(kv.second);
      res->qt_of_glob[gi].emplace_back(c, res->owned.back().c_str());
    }
  char buf[1280];
  snprintf(buf, sizeof(buf),
           "{\"scan_ms\":%.6f,\"total_ms\":%.6f,\"plan_ms\":%.6f,\"device_ms\":%.6f,\"launch_ms\":%.6f,"
           "\"sync_ms\":%.6f,\"alloc_ms\":%.6f,\"copy_ms\":%.6f,\"rows_scanned\":%llu,"
           "\"algorithmic_bytes\":%llu,\"tiles\":%u,\"cells\":%llu,\"segments\":%zu,\"general_segments\":%zu,"
           "\"failed_globs\":%zu,\"table\":\"%s\","
           "\"slots\":%llu,\"occupied\":%llu,\"attempts\":%d,\"plan_bytes\":%llu,\"reduce\":\"%s\","
           "\"dims_ms\":%.6f,\"dims_rebuilt\":%d,\"emit\":\"%s\",\"exact_sum\":%u,\"global_cells\":%u",
           double(scan_ms), ms_since(t_start), plan_ms, device_ms, launch_ms, sync_ms, alloc_ms, copy_ms, (unsigned long long)rows_scanned,
           (unsigned long long)alg_bytes, total_tiles, (unsigned long long)ncells, qsegs.size() + gsegs.size(), gsegs.size(),
           nfailed, hash_mode ? "hash" : "dense", (unsigned long long)(hash_mode ? cap : ncells), nocc, attempts, plan_bytes,
           !dist ? "none" : (keyrange ? "keyrange" : (hash_mode ? "records_to_root" : "gather_to_root")), dims_ms,
           dims_rebuilt, emit_mode, P.exact_sum, P.global_cells);
  res->stats = buf;
  if (dist) {   // the distributed call's stages and collectives (this rank)
    const CommCounters cc = comm_counters(E);
    char b2[384];
    snprintf(b2, sizeof(b2),
             ",\"reduce_ms\":%.6f,\"scan_agreed_ms\":%.6f,\"collectives\":%llu,\"allgathers\":%llu,"
             "\"allgather_bytes\":%llu,\"p2p_groups\":%llu,\"p2p_bytes\":%llu",
             reduce_ms, scan_agreed_ms, (unsigned long long)(cc.allgathers - cc0.allgathers + cc.p2p_groups - cc0.p2p_groups),
             (unsigned long long)(cc.allgathers - cc0.allgathers), (unsigned long long)(cc.allgather_bytes - cc0.allgather_bytes),
             (unsigned long long)(cc.p2p_groups - cc0.p2p_groups), (unsigned long long)(cc.p2p_bytes - cc0.p2p_bytes));
    res->stats += b2;
  }
  if (!bad_msg.empty()) res->stats += ",\"first_glob_error\":\"" + json_escape(bad_msg) + "\"";
  if (redo) res->stats += ",\"redo\":" + std::to_string(redo);   // 1: metrics at 1 ms, 2: MIN cells kept per glob
  if (dense_shape) res->stats += ",\"lean_dense_shape\":1";
  res->stats += "}";
  return LK_OK;
}

}  // namespace lk
