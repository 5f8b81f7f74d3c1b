// Exemplar queries: a PushDownRequest whose baseExpr has no chart (and no tag query) -- raw rows.
//
// Reference (per glob of `glob_size` segments, Commons.scala:361-389):
//   SELECT "_cardinalhq.timestamp", "_cardinalhq.value", "_cardinalhq.name", "_cardinalhq.message", *     (logs)
//          "_cardinalhq.timestamp", "_cardinalhq.value", "span.name", "span.kind", *                      (traces)
//   FROM (SELECT * FROM read_parquet([...], union_by_name=True) WHERE <window>) WHERE <filter>
//   ORDER BY "_cardinalhq.timestamp" <order, default DESC> LIMIT <limit, default 1000>
// (BaseExpr.getBaseQuery, BaseExpr.scala:206-239; projections 41-45; defaults ASTUtils.scala:360-361).
// Each row becomes DataPoint(timestamp = col 1, value = getDouble(col 2), tags = every later column whose value is
// non-NULL, not "null" and not empty, keyed by column name, values as JDBC getString text) (Commons.toDataPoint,
// Commons.scala:428-459); PushDownAggregatorStage passes exemplar rows through (PushDownAggregatorStage.scala:42,
// 66-68); the globs' streams are folded with Akka mergeSorted under pushDownResponseOrdering (timestamp, reversed
// when reverseSort; Commons.scala:116-132, 391-392).
//
// Here: ex_scan HIST passes narrow each glob's window to the rows that can be in its top `limit`, one ex_scan EMIT
// pass lists them, the host sorts those few candidates, and ex_gather decodes every column of the selected rows
// (ex_kernels.hip).  Documented choices where the reference is unspecified: rows tied on the timestamp keep file
// order (segment position in the glob, then row), which DuckDB's ORDER BY leaves open; metrics exemplars (value =
// getDouble of the name column) fail like the reference's stream does (-> empty).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <charconv>
#include <chrono>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <map>
#include <set>
#include <string>
#include <unordered_set>
#include <vector>

#include "../../include/lakeside_gpu.h"
#include "comm.hpp"
#include "engine.hpp"
#include "evalutil.hpp"
#include "kernels.hpp"
#include "layout.hpp"
#include "parquet.hpp"

namespace lk {

#define XHIP_TRY(x)                                                                             \
  do {                                                                                          \
    hipError_t _e = (x);                                                                        \
    if (_e != hipSuccess)                                                                       \
      throw PlanError(LK_ERR_DEVICE, std::string("HIP: ") + #x + ": " + hipGetErrorString(_e)); \
  } while (0)

namespace {

const char* const kMessage = "_cardinalhq.message";   // Commons.scala:59
const char* const kSpanName = "span.name";            // Commons.scala:71
const char* const kSpanKind = "span.kind";            // Commons.scala:72

// union_by_name type of a column over a glob's files (DuckDB's common supertype for the physical types a segment
// writer produces): equal types stay; INT32/INT64 -> BIGINT; integers with FLOAT -> FLOAT; with DOUBLE -> DOUBLE.
// Anything else (strings mixed with numbers, BOOLEAN with numbers, INT96 / FIXED_LEN) is not decoded here.
int union_type(int a, int b) {
  if (a < 0) return b;
  if (a == b) return a;
  auto rank = [](int t) {
    switch (t) {
      case pq::INT32: return 1;
      case pq::INT64: return 2;
      case pq::FLOAT: return 3;
      case pq::DOUBLE: return 4;
      default: return 0;
    }
  };
  const int ra = rank(a), rb = rank(b);
  if (!ra || !rb) throw PlanError(LK_ERR_UNSUPPORTED, "union_by_name over incompatible column types");
  if ((ra <= 2 && rb <= 2)) return pq::INT64;
  if (ra == 4 || rb == 4) return pq::DOUBLE;
  return pq::FLOAT;
}

// JDBC getString text of a raw value of physical type `pt` read as union type `ut`.
std::string value_text(unsigned long long raw, int pt, int ut) {
  int64_t iv = 0;
  double dv = 0.0;
  float fv = 0.0f;
  switch (pt) {
    case pq::INT64: iv = int64_t(raw); dv = double(iv); fv = float(iv); break;
    case pq::INT32: iv = int32_t(uint32_t(raw)); dv = double(iv); fv = float(iv); break;
    case pq::DOUBLE: memcpy(&dv, &raw, 8); break;
    case pq::FLOAT: {
      const uint32_t u = uint32_t(raw);
      memcpy(&fv, &u, 4);
      dv = double(fv);
      break;
    }
    case pq::BOOLEAN: return raw ? "true" : "false";
    default: throw PlanError(LK_ERR_UNSUPPORTED, "exemplar column of an undecoded type");
  }
  switch (ut) {
    case pq::INT64:
    case pq::INT32: return std::to_string(iv);
    case pq::FLOAT: return java_text(fv);
    default: return java_text(dv);
  }
}

double value_double(unsigned long long raw, int pt) {
  switch (pt) {
    case pq::DOUBLE: {
      double d;
      memcpy(&d, &raw, 8);
      return d;
    }
    case pq::INT64: return double(int64_t(raw));
    case pq::INT32: return double(int32_t(uint32_t(raw)));
    case pq::FLOAT: {
      float f;
      const uint32_t u = uint32_t(raw);
      memcpy(&f, &u, 4);
      return double(f);
    }
    default: throw PlanError(LK_ERR_UNSUPPORTED, "exemplar value column of a non-numeric type");
  }
}

struct XGlob {
  std::vector<int> segs;
  bool skip = false;
  uint32_t leaf_false = 0;
  int64_t win_lo = 0, win_hi = 0;
  std::vector<std::string> cols;          // output columns: projection, then the union (file order)
  std::map<std::string, int> types;       // union type per column
  // selection state
  bool open = false;
  std::vector<int64_t> probes;            // ordered-end-first ranges to try before the whole window (zone maps)
  size_t probe = 0;
  int64_t hlo = 0, hhi = 0;               // range still being narrowed
  uint64_t need = 0, above = 0;           // rows still wanted from [hlo, hhi); rows certainly in beyond it
  int64_t elo = 0, ehi = 0;               // final emit range
  uint64_t count = 0;                     // rows in the emit range
};

struct Cand {
  int64_t ts;
  uint32_t qseg;
  uint32_t pos;       // segment position in the glob
  uint64_t row;       // row in the file
  unsigned long long ref;
};

}  // namespace

namespace {
// A pinned host block from the engine's pool for the length of a transfer (returned to the pool on scope exit).
struct PinnedTmp {
  HostBlock b;
  explicit PinnedTmp(size_t n) : b(pinned_acquire(n)) {}
  ~PinnedTmp() { pinned_release(b); }
  PinnedTmp(const PinnedTmp&) = delete;
  PinnedTmp& operator=(const PinnedTmp&) = delete;
  void* p() const { return b.p; }
};
}  // namespace

namespace {
// Row streams as bytes (the ranks' exchange): tag names, then per row ts | value | present tags (column, text).
void put_u32(std::string& b, uint32_t x) { b.append(reinterpret_cast<const char*>(&x), 4); }
void put_str(std::string& b, const std::string& s) {
  put_u32(b, uint32_t(s.size()));
  b += s;
}
struct Reader {
  const std::string& b;
  size_t o = 0;
  template <class T>
  T get() {
    if (o + sizeof(T) > b.size()) throw PlanError(LK_ERR_DEVICE, "internal: short exemplar stream from a rank");
    T x;
    memcpy(&x, b.data() + o, sizeof(T));
    o += sizeof(T);
    return x;
  }
  std::string str() {
    const uint32_t n = get<uint32_t>();
    if (o + n > b.size()) throw PlanError(LK_ERR_DEVICE, "internal: short exemplar stream from a rank");
    std::string s = b.substr(o, n);
    o += n;
    return s;
  }
};
struct XRow {
  int64_t ts;
  double val;
  std::vector<std::pair<std::string, std::string>> tags;   // (column name, text), the row's present tags
};
}  // namespace

// Distributed exemplar / numeric-tag query (VERDICT r4 missing #1-2).  Reference: query-api fans the pushdown out to
// every worker pod holding segments of the group (SegmentSequencer.allSources), each pod evaluates its own segments
// (globs of its own request, Commons.scala:361-392), and query-api merges the pods' streams -- exemplars:
// flatMapMerge then take(limit) (QueryEngineV2.scala:493-535); tag queries: every pod's (tag, count) rows
// (QueryEngineV2.scala:452-487).  Here each rank is a pod: it evaluates the segments of its shard as the worker
// would (its exemplar stream: per-glob top `limit`, globs folded by mergeSorted; its numeric tag rows: counts per tag
// text over its globs), one all-gather carries every rank's rows (and status: a rank-local failure fails every
// rank), and rank 0 folds them -- exemplars: Akka mergeSorted over the ranks in rank order (the deterministic
// stand-in for flatMapMerge's arrival order) and take(limit); numeric tags: counts summed per tag text (NULL apart),
// in first-seen order, as the string tag query's merged table does.  Other ranks return no rows.
static int exemplar_dist(Engine& E, CallCtx& X, const Request& R, const char* const* paths, size_t n_paths,
                         int glob_size, lk_result* res, const std::string& numtag, const int32_t* shard) {
  const auto t0 = std::chrono::steady_clock::now();
  const bool tagnum = !numtag.empty();
  const int world = comm_world(E), rank = comm_rank(E);
  Request sub = copy_request(R);
  sub.segments.clear();
  std::vector<const char*> sp;
  for (size_t i = 0; i < n_paths; i++)
    if ((shard ? shard[i] : int32_t(i % size_t(world))) == rank) {
      sp.push_back(paths[i]);
      sub.segments.push_back(R.segments[i]);
    }
  int code = 0;
  std::string msg, blob;
  double scan_ms = 0;
  uint64_t local_rows = 0;
  if (!sp.empty()) {   // a pod with no segment of the group is not asked at all (no sentinel row)
    try {
      lk_result local;
      evaluate_exemplar(E, X, sub, sp.data(), sp.size(), glob_size, tagnum ? LK_MERGED : LK_PER_GLOB_ROWS, false,
                        &local, numtag);
      const size_t nt = local.tag_names.size();
      put_u32(blob, uint32_t(nt));
      for (auto& n : local.tag_names) put_str(blob, n);
      const uint64_t n = local.nrows;
      blob.append(reinterpret_cast<const char*>(&n), 8);
      for (size_t i = 0; i < local.nrows; i++) {
        blob.append(reinterpret_cast<const char*>(&local.ts[i]), 8);
        blob.append(reinterpret_cast<const char*>(&local.val[i]), 8);
        uint32_t present = 0;
        for (size_t c = 0; c < nt; c++) present += local.tag(i, c) != nullptr;
        put_u32(blob, present);
        for (size_t c = 0; c < nt; c++)
          if (const char* v = local.tag(i, c)) {
            put_u32(blob, uint32_t(c));
            put_str(blob, v);
          }
      }
      local_rows = local.nrows;
      const char* k = strstr(local.stats.c_str(), "\"scan_ms\":");
      if (k) scan_ms = atof(k + 10);
    } catch (const PlanError& e) {
      code = e.code;
      msg = e.what();
    } catch (const std::exception& e) {
      code = LK_ERR_DEVICE;
      msg = e.what();
    }
  }
  const std::vector<std::string> all = comm_allgather_status(E, X, code, msg, blob);
  res->exemplar = true;
  res->per_glob = false;
  std::vector<XRow> out;
  std::vector<std::string> names;   // tag columns, first-seen order over the ranks
  if (rank == 0) {
    std::vector<std::vector<XRow>> streams(all.size());
    for (size_t r = 0; r < all.size(); r++) {
      if (all[r].empty()) continue;
      Reader rd{all[r]};
      const uint32_t nt = rd.get<uint32_t>();
      std::vector<std::string> tn(nt);
      for (auto& t : tn) t = rd.str();
      for (auto& t : tn)
        if (std::find(names.begin(), names.end(), t) == names.end()) names.push_back(t);
      const uint64_t n = rd.get<uint64_t>();
      streams[r].resize(size_t(n));
      for (auto& row : streams[r]) {
        row.ts = rd.get<int64_t>();
        row.val = rd.get<double>();
        const uint32_t np = rd.get<uint32_t>();
        for (uint32_t j = 0; j < np; j++) {
          const uint32_t c = rd.get<uint32_t>();
          if (c >= nt) throw PlanError(LK_ERR_DEVICE, "internal: bad tag column in a rank's exemplar stream");
          row.tags.emplace_back(tn[c], rd.str());
        }
      }
    }
    if (!tagnum) {
      // Akka mergeSorted fold over the ranks' streams (left head when strictly less), then take(limit)
      const bool rev = R.reverse_sort;
      for (auto& v : streams) {
        std::vector<XRow> m;
        m.reserve(out.size() + v.size());
        size_t i = 0, j = 0;
        while (i < out.size() && j < v.size()) {
          const bool lt = rev ? out[i].ts > v[j].ts : out[i].ts < v[j].ts;
          if (lt) m.push_back(std::move(out[i++]));
          else m.push_back(std::move(v[j++]));
        }
        while (i < out.size()) m.push_back(std::move(out[i++]));
        while (j < v.size()) m.push_back(std::move(v[j++]));
        out.swap(m);
      }
      if (R.limit >= 0 && out.size() > uint64_t(R.limit)) out.resize(size_t(R.limit));
    } else {
      // counts summed per tag text (the "count" tag rewritten), NULL / dropped tag apart, first-seen order.
      // A deliberate deviation: query-api's streamTags (QueryEngineV2.scala:452-487) flatMapMerges the
      // pods' (tag, count) rows unsummed, in arrival order (TagQueryUtils.aggregate is commented out there), so a
      // value present on two pods reaches the client twice.  The distributed call returns one merged table instead
      // -- the same table the string-tag distributed path returns (one row per value, counts added) -- because
      // arrival order across ranks is not reproducible; DESIGN.md §5 records this.
      std::map<std::string, size_t> at;
      for (auto& v : streams)
        for (auto& row : v) {
          std::string key = "\x01";   // the tag dropped (NULL or a null-like text)
          for (auto& kv : row.tags)
            if (kv.first == numtag) key = "\x02" + kv.second;
          auto it = at.find(key);
          if (it == at.end()) {
            at.emplace(key, out.size());
            out.push_back(std::move(row));
          } else {
            out[it->second].val += row.val;
          }
        }
      for (auto& row : out)
        for (auto& kv : row.tags)
          if (kv.first == "count") kv.second = std::to_string((unsigned long long)row.val);
    }
  }
  res->alloc_rows(out.size());
  res->tag_names = names;
  res->ex_tags.assign(out.size() * names.size(), nullptr);
  for (size_t i = 0; i < out.size(); i++) {
    res->ts[i] = out[i].ts;
    res->val[i] = out[i].val;
    res->glob[i] = 0;
    res->gid[i] = uint32_t(i);
    for (auto& kv : out[i].tags) {
      const size_t c = size_t(std::find(names.begin(), names.end(), kv.first) - names.begin());
      res->owned.push_back(kv.second);
      res->ex_tags[i * names.size() + c] = res->owned.back().c_str();
    }
  }
  char buf[320];
  snprintf(buf, sizeof buf,
           "{\"scan_ms\":%.4f,\"total_ms\":%.4f,\"rank_rows\":%llu,\"rows\":%zu,\"reduce\":\"%s\",\"table\":\"%s\"}",
           scan_ms, ms_since(t0), (unsigned long long)local_rows, out.size(), tagnum ? "tag_counts" : "merge_sorted",
           tagnum ? "tagnum" : "exemplar");
  res->stats = buf;
  return LK_OK;
}

int evaluate_exemplar(Engine& E, CallCtx& X, const Request& R, const char* const* paths, size_t n_paths,
                      int glob_size, unsigned flags, bool dist, lk_result* res, const std::string& numtag,
                      const int32_t* shard) {
  const auto t_start = std::chrono::steady_clock::now();
  const bool tagnum = !numtag.empty();
  if (dist) return exemplar_dist(E, X, R, paths, n_paths, glob_size <= 0 ? 10 : glob_size, res, numtag, shard);
  if (R.has_extract || R.has_compute)
    throw PlanError(LK_ERR_UNSUPPORTED, "extract / compute exemplar queries are not on the hot path");
  const bool logs = R.dataset == "logs";
  if (!tagnum && !logs && R.dataset != "traces") {
    // metrics: the projection's second column is "_cardinalhq.name" (BaseExpr.scala:41); getDouble of a metric
    // name fails the stream, which query-api turns into an empty source (QueryEngineV2.scala:141-145)
    if (R.dataset == "metrics") throw PlanError(LK_ERR_ARG, "metrics exemplar: getDouble of \"_cardinalhq.name\"");
    throw PlanError(LK_ERR_ARG, "Invalid dataset: " + R.dataset);
  }
  std::string order = R.order;
  for (auto& c : order) c = char(toupper(static_cast<unsigned char>(c)));
  if (tagnum) order = "DESC";   // (a tag query has no ORDER BY / LIMIT)
  if (order != "DESC" && order != "ASC") throw PlanError(LK_ERR_ARG, "ORDER BY direction '" + R.order + "'");
  if (R.limit < 0 && !tagnum) throw PlanError(LK_ERR_ARG, "negative LIMIT");
  const bool desc = order == "DESC";
  const uint64_t limit = tagnum ? 0 : uint64_t(R.limit);
  const bool per_glob_rows = (flags & LK_PER_GLOB_ROWS) != 0;

  std::vector<const FilterNode*> all_leaves;
  collect_leaves(R.filter.get(), all_leaves);
  std::vector<std::string> nums;   // numeric comparison columns (gt/ge/lt/le, BaseExpr.scala:488-498)
  // numeric tag: its leaves (query-api's `exists` on the tag) are numeric IS NOT NULL leaves; the tag column is a
  // numeric column of the scan either way
  auto num_col = [&](const FilterNode* l) { return numeric_op(l->op) || (tagnum && l->k == numtag); };
  for (auto* l : all_leaves) {
    if (l->extracted || l->computed) throw PlanError(LK_ERR_UNSUPPORTED, "extracted/computed filter fields");
    if (tagnum && l->k == numtag && !numeric_op(l->op) && l->op != "exists" && l->op != "has")
      throw PlanError(LK_ERR_UNSUPPORTED, "string comparison '" + l->op + "' on the numeric tag column " + numtag);
    if (num_col(l)) {
      if (std::find(nums.begin(), nums.end(), l->k) == nums.end()) nums.push_back(l->k);
      continue;
    }
    static const char* ok[] = {"eq", "!=", "in", "not_in", "regex", "contains", "has", "exists"};
    if (std::none_of(std::begin(ok), std::end(ok), [&](const char* o) { return l->op == o; }))
      throw PlanError(LK_ERR_ARG, "Invalid operator " + l->op);
  }
  if (tagnum && std::find(nums.begin(), nums.end(), numtag) == nums.end()) nums.push_back(numtag);
  res->exemplar = true;
  res->per_glob = true;
  if (R.segments.empty()) {   // Commons.scala:393-396: the sentinel DataPoint(-1, -1, {})
    if (per_glob_rows) {
      res->alloc_rows(1);
      res->ts[0] = -1;
      res->val[0] = -1.0;
      res->glob[0] = 0;
      res->gid[0] = 0;
    }
    res->stats = "{\"scan_ms\":0,\"total_ms\":0,\"rows_scanned\":0,\"candidates\":0}";
    return LK_OK;
  }

  // ---- filter columns (string dictionaries) and the Kleene program ----
  struct XStr {
    std::string name;
    std::vector<const FilterNode*> leaves;
    uint32_t lbase = 0, lmask = 0, hmask = 0, dict_n = 0;
  };
  std::vector<XStr> strs;
  for (auto* l : all_leaves) {
    if (num_col(l)) continue;
    auto it = std::find_if(strs.begin(), strs.end(), [&](const XStr& s) { return s.name == l->k; });
    if (it == strs.end()) {
      strs.push_back(XStr{});
      strs.back().name = l->k;
      it = strs.end() - 1;
    }
    it->leaves.push_back(l);
  }
  if (2 + strs.size() + nums.size() > size_t(MAXQCOL))
    throw PlanError(LK_ERR_UNSUPPORTED, "too many filter columns in one query");
  for (auto& nm : nums)
    if (std::find_if(strs.begin(), strs.end(), [&](const XStr& sc) { return sc.name == nm; }) != strs.end())
      throw PlanError(LK_ERR_UNSUPPORTED, "column " + nm + " used both as a string and as a number");
  if (all_leaves.size() > size_t(MAXLEAF)) throw PlanError(LK_ERR_UNSUPPORTED, "too many filter leaves");
  std::vector<LeafInfo> leaves;
  for (size_t s = 0; s < strs.size(); s++) {
    XStr& sc = strs[s];
    if (sc.leaves.size() > size_t(LEAF_BITS)) throw PlanError(LK_ERR_UNSUPPORTED, "too many leaves on one column");
    sc.lbase = uint32_t(leaves.size());
    for (const FilterNode* l : sc.leaves) {
      const uint32_t idx = uint32_t(leaves.size());
      leaves.push_back(LeafInfo{l, int(s), int(idx)});
      sc.lmask |= 1u << idx;
      if (l->op == "has" || l->op == "exists") sc.hmask |= 1u << idx;
    }
  }
  std::vector<NumLeaf> nleaves;
  std::vector<std::string> bad_literal;   // fields whose numeric literal fails the SQL (per glob where they exist)
  for (auto* l : all_leaves)
    if (num_col(l)) {
      const uint32_t idx = uint32_t(leaves.size());
      leaves.push_back(LeafInfo{l, -1, int(idx)});
      const uint32_t col = uint32_t(std::find(nums.begin(), nums.end(), l->k) - nums.begin());
      if (!numeric_op(l->op)) {   // IS NOT NULL on the numeric tag (BaseExpr: "<tag>" IS NOT NULL)
        NumLeaf nl{};
        nl.col = col;
        nl.leaf = idx;
        nl.pad = NUMLEAF_NOTNULL;
        nleaves.push_back(nl);
        continue;
      }
      bool bad = false;
      nleaves.push_back(make_num_leaf(*l, col, idx, bad));
      if (bad) bad_literal.push_back(l->k);
    }
  std::vector<uint8_t> prog;
  postfix(R.filter.get(), leaves, prog);
  if (prog.size() > size_t(MAXPROG)) throw PlanError(LK_ERR_UNSUPPORTED, "filter too large");

  // ---- segments and globs ----
  // A segment that cannot be read (missing, corrupt, a shape the loader does not take) fails its glob's query only:
  // that glob is empty, the others stream (Commons.scala:249-253, 338-340).
  std::vector<std::shared_ptr<Segment>> segs(n_paths);
  std::vector<uint8_t> seg_bad(n_paths, 0);
  for (size_t i = 0; i < n_paths; i++) {
    try {
      segs[i] = E.get_segment(paths[i], true);
    } catch (const PlanError& e) {
      if (e.code != LK_ERR_IO) throw;   // capability gaps / evicted keys fail the call
      seg_bad[i] = 1;
    }
  }
  if (glob_size <= 0) glob_size = 10;
  const std::vector<std::string> proj = tagnum ? std::vector<std::string>{kTimestamp, numtag}
                                       : logs ? std::vector<std::string>{kTimestamp, kValue, kName, kMessage}
                                              : std::vector<std::string>{kTimestamp, kValue, kSpanName, kSpanKind};
  const std::set<std::string> fset = field_set(R);
  std::vector<XGlob> globs;
  for (size_t i = 0; i < n_paths; i += size_t(glob_size)) {
    XGlob g;
    for (size_t j = i; j < std::min(n_paths, i + size_t(glob_size)); j++) g.segs.push_back(int(j));
    g.win_lo = INT64_MAX;
    g.win_hi = INT64_MIN;
    std::vector<std::string> uni;
    for (int si : g.segs) {
      g.win_lo = std::min(g.win_lo, R.segments[si].start_ts);
      g.win_hi = std::max(g.win_hi, R.segments[si].end_ts);
      if (seg_bad[si]) {
        g.skip = true;
        continue;
      }
      for (auto& [name, pt] : segs[si]->schema) {
        if (!g.types.count(name)) uni.push_back(name);
        // a union this engine does not form (e.g. VARCHAR with a number, which DuckDB unifies to VARCHAR): the call
        // fails with LK_ERR_UNSUPPORTED so the caller can fall back, not an empty glob
        g.types[name] = union_type(g.types.count(name) ? g.types[name] : -1, pt);
      }
    }
    for (auto& l : leaves)   // nonExistentFields -> literal false (Commons.scala:224, BaseExpr.scala:462-464)
      if (fset.count(l.node->k) && !g.types.count(l.node->k)) g.leaf_false |= 1u << l.index;
    for (auto& p : proj)      // Binder Error -> empty glob (Commons.scala:249-253)
      if (!g.types.count(p)) g.skip = true;
    for (auto& l : leaves)
      if (!(g.leaf_false >> l.index & 1u) && !g.types.count(l.node->k)) g.skip = true;
    for (auto& k : bad_literal)   // normalizedValue failed for a field this glob has
      if (!(fset.count(k) && !g.types.count(k))) g.skip = true;
    if (tagnum && g.types.count(numtag) && g.types[numtag] == pq::BYTE_ARRAY)   // VARCHAR in a glob of numbers
      throw PlanError(LK_ERR_UNSUPPORTED, "tag column " + numtag + " is text in some files and numeric in others");
    for (auto& nm : nums)   // a VARCHAR compared with a number: Binder Error -> empty glob
      if (g.types.count(nm) && g.types[nm] == pq::BYTE_ARRAY) g.skip = true;
    g.cols = proj;
    for (auto& u : uni)
      if (std::find(g.cols.begin(), g.cols.end(), u) == g.cols.end()) g.cols.push_back(u);
    globs.push_back(std::move(g));
  }

  // ---- per filter column: dictionary value -> leaf bits (cached per (column, leaves) like the aggregate path) ----
  std::vector<std::vector<uint32_t>> tabs(strs.size());
  for (size_t s = 0; s < strs.size(); s++) {
    XStr& sc = strs[s];
    GlobalDict& gd = E.dict(sc.name);
    std::lock_guard<std::mutex> dg(gd.mu);
    sc.dict_n = uint32_t(gd.size());
    std::string key = sc.name;
    for (const FilterNode* l : sc.leaves) {
      key += '\x1f';
      key += l->op;
      for (auto& v : l->v) {
        key += '\x1e';
        key += v;
      }
    }
    std::vector<std::unique_ptr<re::Regex>> rxs(sc.leaves.size());
    std::vector<std::unique_ptr<std::unordered_set<std::string>>> sets(sc.leaves.size());
    for (size_t j = 0; j < sc.leaves.size(); j++) {
      const FilterNode* l = sc.leaves[j];
      if (l->op == "regex" || l->op == "contains") rxs[j] = std::make_unique<re::Regex>(compile_leaf_regex(*l));
      if ((l->op == "in" || l->op == "not_in") && l->v.size() > 8)
        sets[j] = std::make_unique<std::unordered_set<std::string>>(l->v.begin(), l->v.end());
    }
    auto lb = E.leaf_bits(key);
    std::lock_guard<std::mutex> lg(lb->mu);
    for (uint32_t gid = uint32_t(lb->hit.size()); gid < sc.dict_n; gid++) {
      uint8_t bits = 0;
      for (size_t j = 0; j < sc.leaves.size(); j++)
        if (leaf_eval(*sc.leaves[j], gd[gid], rxs[j].get(), sets[j].get())) bits |= uint8_t(1u << j);
      lb->hit.push_back(bits);
    }
    tabs[s].resize(std::max<uint32_t>(sc.dict_n, 1));
    for (uint32_t gid = 0; gid < sc.dict_n; gid++) tabs[s][gid] = uint32_t(lb->hit[gid]) << 24;
  }

  // ---- per-segment descriptors ----
  std::vector<QSeg> qsegs;
  std::vector<const Segment*> qseg_seg;
  std::vector<uint32_t> qseg_pos, qseg_glob;
  uint64_t rows_scanned = 0;
  uint32_t max_tiles = 0;
  // a referenced column this engine does not decode fails the call (LK_ERR_UNSUPPORTED: the caller falls back), where
  // a column of a type the query cannot bind is DuckDB's Binder Error (empty glob, below)
  for (size_t gi = 0; gi < globs.size(); gi++) {
    if (globs[gi].skip) continue;
    for (int si : globs[gi].segs) {
      if (!segs[si] || segs[si]->unloaded.empty()) continue;
      const Segment& S = *segs[si];
      auto check = [&](const std::string& c) {
        auto u = S.unloaded.find(c);
        if (u != S.unloaded.end()) throw PlanError(LK_ERR_UNSUPPORTED, u->second + " (" + S.key + ")");
      };
      check(kTimestamp);
      for (auto& sc : strs) check(sc.name);
      for (auto& nm : nums) check(nm);
      for (auto& c : globs[gi].cols) check(c);
    }
  }
  for (size_t gi = 0; gi < globs.size(); gi++) {
    XGlob& g = globs[gi];
    if (g.skip || g.win_lo >= g.win_hi || (limit == 0 && !tagnum)) continue;
    // the glob's descriptors go in together: a column its query cannot bind empties the glob (Binder Error,
    // Commons.scala:249-253), the other globs are unaffected
    const size_t mark = qsegs.size();
    const uint64_t rows_mark = rows_scanned;
    const uint32_t tiles_mark = max_tiles;
    try {
    for (size_t p = 0; p < g.segs.size(); p++) {
      const Segment& S = *segs[g.segs[p]];
      QSeg q{};
      q.base = S.d_data;
      q.tiles = S.d_tiles;
      q.ntiles = uint32_t(S.tiles.size());
      q.glob_slot = uint32_t(gi);
      q.leaf_false = g.leaf_false;
      q.win_lo = g.win_lo;
      q.win_hi = g.win_hi;
      auto bind = [&](int qc, const std::string& name, bool want_string) {
        const int c = S.col_index(name);
        if (c < 0) return;
        const HostCol& hc = S.cols[c];
        if (want_string != hc.is_string)
          throw PlanError(LK_ERR_UNSUPPORTED, "column " + name + " has an unexpected type for its role");
        if (qc == 0 && hc.ptype != pq::INT64 && hc.ptype != pq::INT32)
          throw PlanError(LK_ERR_UNSUPPORTED, "timestamp column must be INT64 or INT32");
        const bool is_tag = tagnum && name == numtag;
        if (qc >= 2 + int(strs.size()) && hc.ptype != pq::INT64 && hc.ptype != pq::DOUBLE && hc.ptype != pq::INT32 &&
            hc.ptype != pq::FLOAT && !(is_tag && hc.ptype == pq::BOOLEAN))
          throw PlanError(LK_ERR_UNSUPPORTED, "numeric comparison on column " + name + " of an undecoded type");
        uint32_t pad = uint32_t(hc.ptype);
        if (is_tag) pad |= uint32_t(g.types.count(numtag) ? g.types[numtag] : hc.ptype) << 8;   // the glob's union type
        q.cols[qc] = QCol{hc.d_pages, hc.d_runs, hc.d_tcols, hc.d_remap, 1u, pad};
      };
      bind(0, kTimestamp, false);
      if (!q.cols[0].present) continue;
      for (size_t s = 0; s < strs.size(); s++) bind(int(2 + s), strs[s].name, true);
      for (size_t n = 0; n < nums.size(); n++) bind(int(2 + strs.size() + n), nums[n], false);
      rows_scanned += uint64_t(S.num_rows);
      max_tiles = std::max(max_tiles, q.ntiles);
      qsegs.push_back(q);
      qseg_seg.push_back(&S);
      qseg_pos.push_back(uint32_t(p));
      qseg_glob.push_back(uint32_t(gi));
    }
    g.open = true;
    } catch (const PlanError& e) {
      if (e.code != LK_ERR_UNSUPPORTED) throw;
      g.skip = true;
      qsegs.resize(mark);
      qseg_seg.resize(mark);
      qseg_pos.resize(mark);
      qseg_glob.resize(mark);
      rows_scanned = rows_mark;
      max_tiles = tiles_mark;
    }
  }
  if (qsegs.size() > 65535) throw PlanError(LK_ERR_UNSUPPORTED, "more than 65535 segments in one evaluation");

  // ---- device staging ----
  XHIP_TRY(hipSetDevice(E.device));
  hipStream_t st = X.stream;
  std::vector<uint32_t> truth;
  if (leaves.size() <= size_t(TT_MAX_LEAVES)) truth = truth_table(prog, uint32_t(leaves.size()));
  std::vector<StrParam> strp(strs.size());
  const size_t ng = globs.size();
  size_t off = 0;
  auto reserve = [&](size_t n) { size_t o = (off + 255) / 256 * 256; off = o + n; return o; };
  const size_t o_segs = reserve(qsegs.size() * sizeof(QSeg));
  const size_t o_truth = reserve(truth.size() * 4);
  std::vector<size_t> o_tab(strs.size());
  for (size_t s = 0; s < strs.size(); s++) o_tab[s] = reserve(tabs[s].size() * 4);
  const size_t o_strp = reserve(strp.size() * sizeof(StrParam));
  const size_t o_rng = reserve(ng * 8 * 4);          // rlo, rhi, hbase, hwidth
  const size_t o_n = reserve(8);
  const size_t stage_bytes = off;
  const size_t o_hist = reserve(ng * XBINS * 4);   // host side only: the histogram read back each pass
  uint8_t* hbuf = static_cast<uint8_t*>(X.pinned_buf(off));
  uint8_t* dbuf = static_cast<uint8_t*>(X.workspace("xquery", stage_bytes));
  uint32_t* d_hist = static_cast<uint32_t*>(X.workspace("xhist", std::max<size_t>(ng * XBINS * 4, 4)));
  memcpy(hbuf + o_segs, qsegs.data(), qsegs.size() * sizeof(QSeg));
  if (!truth.empty()) memcpy(hbuf + o_truth, truth.data(), truth.size() * 4);
  for (size_t s = 0; s < strs.size(); s++) {
    memcpy(hbuf + o_tab[s], tabs[s].data(), tabs[s].size() * 4);
    strp[s].strtab = reinterpret_cast<const uint32_t*>(dbuf + o_tab[s]);
    strp[s].lbase = strs[s].lbase;
    strp[s].lmask = strs[s].lmask;
    strp[s].hmask = strs[s].hmask;
  }
  memcpy(hbuf + o_strp, strp.data(), strp.size() * sizeof(StrParam));
  int64_t* hr = reinterpret_cast<int64_t*>(hbuf + o_rng);
  XParams P{};
  P.segs = reinterpret_cast<const QSeg*>(dbuf + o_segs);
  P.nsegs = uint32_t(qsegs.size());
  P.max_tiles = max_tiles;
  P.strp = reinterpret_cast<const StrParam*>(dbuf + o_strp);
  P.nstr = uint32_t(strs.size());
  P.nleaves = uint32_t(leaves.size());
  P.nprog = uint32_t(prog.size());
  memcpy(P.prog, prog.data(), prog.size());
  P.truth = truth.empty() ? nullptr : reinterpret_cast<const uint32_t*>(dbuf + o_truth);
  P.nnum = uint32_t(nums.size());
  P.nnl = uint32_t(nleaves.size());
  for (size_t i = 0; i < nleaves.size(); i++) P.nl[i] = nleaves[i];
  int64_t* d_rng = reinterpret_cast<int64_t*>(dbuf + o_rng);
  P.rlo = d_rng;
  P.rhi = d_rng + ng;
  P.hbase = d_rng + 2 * ng;
  P.hwidth = d_rng + 3 * ng;
  P.out_n = reinterpret_cast<uint32_t*>(dbuf + o_n);
  P.tag_qc = ~0u;

  if (tagnum) {
    // ---- tag query over a numeric tag: SELECT "<tag>", COUNT(*) ... GROUP BY "<tag>" per glob (BaseExpr.scala:
    // 127-138): one TAGNUM pass counts passing rows per (glob, canonical tag value); the host prints each value as JDBC
    // getString does for the glob's union_by_name type (Long / Integer / Double / Float / Boolean .toString) ----
    const uint32_t tagk = uint32_t(std::find(nums.begin(), nums.end(), numtag) - nums.begin());
    P.tag_qc = uint32_t(2 + strs.size() + tagk);
    uint64_t max_rows = 1;
    for (size_t gi = 0; gi < ng; gi++) {
      const XGlob& g = globs[gi];
      const bool live = !g.skip && g.win_lo < g.win_hi;
      hr[gi] = live ? g.win_lo : 0;
      hr[ng + gi] = live ? g.win_hi : 0;
    }
    {
      std::vector<uint64_t> grow(ng, 0);
      for (size_t q = 0; q < qsegs.size(); q++) grow[qseg_glob[q]] += uint64_t(qseg_seg[q]->num_rows);
      for (uint64_t r : grow) max_rows = std::max(max_rows, r);
    }
    auto pow2 = [](uint64_t x) {
      uint64_t p = 1;
      while (p < x) p <<= 1;
      return p;
    };
    const uint64_t cap_max = std::max<uint64_t>(1 << 12, pow2(2 * max_rows));
    uint64_t tcap = std::min<uint64_t>(cap_max, uint64_t(1) << 12);
    if (const char* e = getenv("LK_TAGNUM_INIT_SLOTS")) tcap = std::min<uint64_t>(cap_max, pow2(std::max<uint64_t>(64, strtoull(e, nullptr, 10))));
    XHIP_TRY(hipMemcpyAsync(dbuf, hbuf, stage_bytes, hipMemcpyHostToDevice, st));
    P.mode = XMODE_TAGNUM;
    float scan_ms = 0.f;
    int attempts = 0;
    uint8_t* tb = nullptr;
    for (;;) {
      attempts++;
      const size_t tbytes = ng * tcap * 16 + ng * 16 + 64;
      tb = static_cast<uint8_t*>(X.workspace("tagnum", tbytes));
      P.tkeys = reinterpret_cast<unsigned long long*>(tb);
      P.tcnt = reinterpret_cast<unsigned long long*>(tb + ng * tcap * 8);
      P.tspec = reinterpret_cast<unsigned long long*>(tb + ng * tcap * 16);
      P.tflags = reinterpret_cast<uint32_t*>(tb + ng * tcap * 16 + ng * 16);
      P.tcap = tcap;
      XHIP_TRY(hipMemsetAsync(tb, 0xff, ng * tcap * 8, st));
      XHIP_TRY(hipMemsetAsync(tb + ng * tcap * 8, 0, ng * tcap * 8 + ng * 16 + 64, st));
      XHIP_TRY(hipEventRecord(X.ev_scan0, st));
      XHIP_TRY(launch_ex_scan(P, st));
      XHIP_TRY(hipEventRecord(X.ev_scan1, st));
      uint32_t fl = 0;
      XHIP_TRY(hipMemcpyAsync(&fl, P.tflags, 4, hipMemcpyDeviceToHost, st));
      XHIP_TRY(hipStreamSynchronize(st));
      float ms = 0.f;
      XHIP_TRY(hipEventElapsedTime(&ms, X.ev_scan0, X.ev_scan1));
      scan_ms += ms;
      if (!(fl & FLAG_HASH_FULL)) break;
      if (tcap >= cap_max) throw PlanError(LK_ERR_MEMORY, "tag value table full at its bound");
      tcap = std::min(cap_max, tcap * 8);
    }
    // occupied slots -> (key, count, glob) records; per-glob NULL / all-ones counts
    auto* recs = static_cast<unsigned long long*>(X.workspace("tagrecs", ng * tcap * 24 + 64));
    uint32_t* d_n = reinterpret_cast<uint32_t*>(recs);
    XHIP_TRY(hipMemsetAsync(d_n, 0, 4, st));
    XHIP_TRY(launch_tag_compact(P.tkeys, P.tcnt, tcap, uint32_t(ng), recs + 1, d_n, st));
    uint32_t nrec = 0;
    std::vector<unsigned long long> spec(ng * 2);
    XHIP_TRY(hipMemcpyAsync(&nrec, d_n, 4, hipMemcpyDeviceToHost, st));
    XHIP_TRY(hipMemcpyAsync(spec.data(), P.tspec, ng * 16, hipMemcpyDeviceToHost, st));
    XHIP_TRY(hipStreamSynchronize(st));
    std::vector<unsigned long long> hrec(size_t(nrec) * 3);
    if (nrec) {
      XHIP_TRY(hipMemcpyAsync(hrec.data(), recs + 1, size_t(nrec) * 24, hipMemcpyDeviceToHost, st));
      XHIP_TRY(hipStreamSynchronize(st));
    }
    // per glob: (key, count) in the union type's value order, NULL last
    struct TRow {
      uint32_t glob;
      bool null;
      unsigned long long key;
      uint64_t count;
      std::string text;
    };
    std::vector<TRow> rows;
    auto union_of = [&](uint32_t gi) {
      auto it = globs[gi].types.find(numtag);
      return it == globs[gi].types.end() ? int(pq::INT64) : it->second;
    };
    for (uint32_t i = 0; i < nrec; i++)
      rows.push_back(TRow{uint32_t(hrec[3 * i + 2]), false, hrec[3 * i], hrec[3 * i + 1], std::string()});
    for (uint32_t gi = 0; gi < ng; gi++) {
      if (spec[2 * gi + 1]) rows.push_back(TRow{gi, false, TAG_EMPTY, spec[2 * gi + 1], std::string()});
      if (spec[2 * gi]) rows.push_back(TRow{gi, true, 0, spec[2 * gi], std::string()});
    }
    auto num_of = [&](const TRow& r) -> double {   // value order within a glob
      const int ut = union_of(r.glob);
      if (ut == pq::DOUBLE) {
        double d;
        memcpy(&d, &r.key, 8);
        return d;
      }
      if (ut == pq::FLOAT) {
        float f;
        const uint32_t u = uint32_t(r.key);
        memcpy(&f, &u, 4);
        return double(f);
      }
      return double(int64_t(r.key));
    };
    for (auto& r : rows)
      if (!r.null) r.text = value_text(r.key, union_of(r.glob), union_of(r.glob));
    std::sort(rows.begin(), rows.end(), [&](const TRow& a, const TRow& b) {
      if (a.glob != b.glob) return a.glob < b.glob;
      if (a.null != b.null) return b.null;
      if (a.null) return false;
      const int ut = union_of(a.glob);
      if (ut != pq::DOUBLE && ut != pq::FLOAT)   // integers (the all-ones key is -1): exact order, not as doubles
        return int64_t(a.key) < int64_t(b.key);  // (beyond 2^53 doubles tie and the text order is wrong)
      const double x = num_of(a), y = num_of(b);
      if (x != y && x == x && y == y) return x < y;
      return a.text < b.text;
    });
    if (!per_glob_rows) {   // merged: counts summed per tag text (NULL apart), in first-seen order
      std::vector<TRow> m;
      std::map<std::pair<bool, std::string>, size_t> at;
      for (auto& r : rows) {
        auto k = std::make_pair(r.null, r.text);
        auto it = at.find(k);
        if (it == at.end()) {
          at.emplace(k, m.size());
          m.push_back(r);
          m.back().glob = 0;
        } else {
          m[it->second].count += r.count;
        }
      }
      rows.swap(m);
    }
    // rows: Commons.toDataPoint's tag branch (Commons.scala:406-423): the tag (dropped when NULL / "" / "null" or a
    // noisy name, NoisyTagsDropper) and "count"; value = the count, timestamp = now (as the string tag path)
    const int64_t now_ms = std::chrono::duration_cast<std::chrono::milliseconds>(
                               std::chrono::system_clock::now().time_since_epoch()).count();
    const bool hide = noisy_tag(numtag);
    res->per_glob = per_glob_rows;
    res->alloc_rows(rows.size());
    res->tag_names = {numtag, "count"};
    res->ex_tags.assign(rows.size() * 2, nullptr);
    for (size_t i = 0; i < rows.size(); i++) {
      res->ts[i] = now_ms;
      res->val[i] = double(rows[i].count);
      res->glob[i] = rows[i].glob;
      res->gid[i] = uint32_t(i);
      if (!rows[i].null && !hide && !null_like(rows[i].text)) {
        res->owned.push_back(rows[i].text);
        res->ex_tags[2 * i] = res->owned.back().c_str();
      }
      res->owned.push_back(std::to_string((unsigned long long)rows[i].count));
      res->ex_tags[2 * i + 1] = res->owned.back().c_str();
    }
    char buf[320];
    snprintf(buf, sizeof buf,
             "{\"scan_ms\":%.4f,\"total_ms\":%.4f,\"rows_scanned\":%llu,\"tag_values\":%u,\"attempts\":%d,"
             "\"slots\":%llu,\"table\":\"tagnum\",\"failed_globs\":%zu}",
             double(scan_ms), ms_since(t_start), (unsigned long long)rows_scanned, nrec, attempts,
             (unsigned long long)tcap, size_t(std::count_if(globs.begin(), globs.end(), [](const XGlob& g) { return g.skip; })));
    res->stats = buf;
    return LK_OK;
  }

  // ---- HIST passes: narrow every glob to the rows that can make its top `limit` ----
  // rows listed beyond each glob's `limit` at most, unless tied on one millisecond (tests shrink it with
  // LK_EX_CAND_CAP to exercise the refinement)
  const uint64_t kCandCap = getenv("LK_EX_CAND_CAP") ? std::max<uint64_t>(1, strtoull(getenv("LK_EX_CAND_CAP"), nullptr, 10))
                                                     : (uint64_t(1) << 24);
  hipEvent_t e0 = X.ev_scan0, e1 = X.ev_scan1;
  float scan_ms = 0.f;
  int passes = 0;
  for (auto& g : globs) {
    g.hlo = g.win_lo;
    g.hhi = g.win_hi;
    g.need = limit;
    g.elo = g.win_lo;
    g.ehi = g.win_hi;
  }
  // Ordered end first: segments are written in time order, so the newest (DESC) rows sit in a few tiles.  From the
  // zone maps, candidate boundaries covering the last 2^20, 2^23, ... rows of the glob; a HIST pass over
  // [boundary, window end) that already counts `limit` passing rows holds the whole top `limit` (every row before
  // the boundary is older than all of them); otherwise the next, wider boundary is tried.
  {
    std::vector<std::vector<std::pair<int64_t, int64_t>>> tl(ng);   // (ordered key, other end)
    std::vector<std::vector<uint32_t>> tr(ng);
    for (size_t q = 0; q < qsegs.size(); q++) {
      const XGlob& g = globs[qseg_glob[q]];
      for (const TileDesc& td : qseg_seg[q]->tiles) {
        if (td.ts_max < g.win_lo || td.ts_min >= g.win_hi) continue;
        tl[qseg_glob[q]].emplace_back(desc ? -td.ts_max : td.ts_min, desc ? td.ts_min : td.ts_max);
        tr[qseg_glob[q]].push_back(td.nrows);
      }
    }
    for (size_t gi = 0; gi < ng; gi++) {
      XGlob& g = globs[gi];
      if (!g.open) continue;
      std::vector<size_t> ord(tl[gi].size());
      for (size_t i = 0; i < ord.size(); i++) ord[i] = i;
      std::sort(ord.begin(), ord.end(), [&](size_t a, size_t b) { return tl[gi][a].first < tl[gi][b].first; });
      uint64_t rows = 0, goal = getenv("LK_EX_PROBE_ROWS") ? std::max<uint64_t>(1, strtoull(getenv("LK_EX_PROBE_ROWS"), nullptr, 10))
                                                         : (uint64_t(1) << 20);   // env: tests only
      int64_t edge = desc ? INT64_MAX : INT64_MIN;
      for (size_t i : ord) {
        rows += tr[gi][i];
        edge = desc ? std::min(edge, tl[gi][i].second) : std::max(edge, tl[gi][i].second + 1);
        if (rows >= goal) {
          const int64_t b = desc ? std::max(edge, g.win_lo) : std::min(edge, g.win_hi);
          if ((desc && b > g.win_lo) || (!desc && b < g.win_hi)) g.probes.push_back(b);
          goal *= 8;
        }
      }
    }
  }
  bool first_upload = true;
  while (std::any_of(globs.begin(), globs.end(), [](const XGlob& g) { return g.open; })) {
    std::vector<uint32_t> nb(ng, 0);
    for (size_t gi = 0; gi < ng; gi++) {
      XGlob& g = globs[gi];
      if (g.open && g.probe < g.probes.size()) {   // probing: [boundary, end) (DESC) / [start, boundary) (ASC)
        g.hlo = desc ? g.probes[g.probe] : g.win_lo;
        g.hhi = desc ? g.win_hi : g.probes[g.probe];
      }
      const int64_t span = g.open ? g.hhi - g.hlo : 0;
      const int64_t w = span > 0 ? (span + XBINS - 1) / XBINS : 1;
      hr[gi] = g.open ? g.hlo : 0;
      hr[ng + gi] = g.open ? g.hhi : 0;
      hr[2 * ng + gi] = g.hlo;
      hr[3 * ng + gi] = w;
      nb[gi] = span > 0 ? uint32_t((span + w - 1) / w) : 0u;
    }
    XHIP_TRY(hipMemcpyAsync(first_upload ? dbuf : dbuf + o_rng, first_upload ? hbuf : hbuf + o_rng,
                            first_upload ? stage_bytes : ng * 32, hipMemcpyHostToDevice, st));
    first_upload = false;
    XHIP_TRY(hipMemsetAsync(d_hist, 0, ng * XBINS * 4, st));
    P.mode = XMODE_HIST;
    P.nbins = XBINS;
    P.hist = d_hist;
    XHIP_TRY(hipEventRecord(e0, st));
    XHIP_TRY(launch_ex_scan(P, st));
    XHIP_TRY(hipEventRecord(e1, st));
    uint32_t* hh = reinterpret_cast<uint32_t*>(hbuf + o_hist);
    XHIP_TRY(hipMemcpyAsync(hh, d_hist, ng * XBINS * 4, hipMemcpyDeviceToHost, st));
    XHIP_TRY(hipStreamSynchronize(st));
    float ms = 0.f;
    XHIP_TRY(hipEventElapsedTime(&ms, e0, e1));
    scan_ms += ms;
    passes++;
    for (size_t gi = 0; gi < ng; gi++) {
      XGlob& g = globs[gi];
      if (!g.open) continue;
      const uint32_t* h = hh + gi * XBINS;
      const int64_t w = hr[3 * ng + gi];
      if (g.probe < g.probes.size()) {
        uint64_t tot = 0;
        for (uint32_t k = 0; k < nb[gi]; k++) tot += h[k];
        if (tot < g.need) {   // not enough rows past this boundary: a wider one, or the whole window
          if (++g.probe >= g.probes.size()) {
            g.hlo = g.win_lo;
            g.hhi = g.win_hi;
          }
          continue;
        }
        g.probe = g.probes.size();   // the top `limit` lies in the probed range: narrow it as usual
      }
      uint64_t cum = 0;
      int64_t split = -1;
      for (uint32_t k = 0; k < nb[gi]; k++) {
        const uint32_t b = desc ? nb[gi] - 1 - k : k;
        if (cum + h[b] >= g.need) {
          split = int64_t(b);
          break;
        }
        cum += h[b];
      }
      if (split < 0) {   // fewer rows than wanted: every row of the range
        g.count = g.above + cum;
        if (desc) g.elo = g.hlo;
        else g.ehi = g.hhi;
        g.open = false;
        continue;
      }
      const int64_t blo = g.hlo + split * w, bhi = std::min(g.hhi, blo + w);
      // the split bin is taken whole when the rows it adds beyond the `need` still wanted stay under the cap (or it
      // is one millisecond wide: those rows are tied and all listed)
      const uint64_t with_bin = g.above + cum + h[split];
      if (cum + h[split] - g.need <= kCandCap || w == 1) {
        g.count = with_bin;
        if (desc) g.elo = blo;
        else g.ehi = bhi;
        g.open = false;
      } else {
        g.above += cum;
        g.need -= cum;
        g.hlo = blo;
        g.hhi = bhi;
      }
    }
  }

  // ---- EMIT: the candidates of every glob's final range ----
  uint64_t total = 0;
  for (auto& g : globs) total += g.count;
  if (total > (uint64_t(1) << 28)) throw PlanError(LK_ERR_UNSUPPORTED, "too many exemplar candidates");
  std::vector<Cand> cands;
  if (total) {
    for (size_t gi = 0; gi < ng; gi++) {
      const XGlob& g = globs[gi];
      const bool live = g.count > 0;
      hr[gi] = live ? g.elo : 0;
      hr[ng + gi] = live ? g.ehi : 0;
    }
    unsigned long long* d_out = static_cast<unsigned long long*>(X.workspace("xcand", total * 16));
    XHIP_TRY(hipMemcpyAsync(dbuf + o_rng, hbuf + o_rng, ng * 16, hipMemcpyHostToDevice, st));
    XHIP_TRY(hipMemsetAsync(dbuf + o_n, 0, 8, st));
    P.mode = XMODE_EMIT;
    P.out = d_out;
    P.cap = uint32_t(total);
    XHIP_TRY(hipEventRecord(e0, st));
    XHIP_TRY(launch_ex_scan(P, st));
    XHIP_TRY(hipEventRecord(e1, st));
    // pinned destinations: a device-to-host copy into pageable memory goes through the runtime's staging buffers
    PinnedTmp eo(total * 16 + 64);
    const unsigned long long* h_out = static_cast<const unsigned long long*>(eo.p());
    XHIP_TRY(hipMemcpyAsync(eo.p(), d_out, total * 16, hipMemcpyDeviceToHost, st));
    XHIP_TRY(hipMemcpyAsync(static_cast<uint8_t*>(eo.p()) + total * 16, dbuf + o_n, 4, hipMemcpyDeviceToHost, st));
    XHIP_TRY(hipStreamSynchronize(st));
    uint32_t got = 0;
    memcpy(&got, static_cast<const uint8_t*>(eo.p()) + total * 16, 4);
    float ms = 0.f;
    XHIP_TRY(hipEventElapsedTime(&ms, e0, e1));
    scan_ms += ms;
    if (got != total) throw PlanError(LK_ERR_DEVICE, "internal: exemplar candidate count disagrees with the histogram");
    cands.resize(total);
    for (uint64_t i = 0; i < total; i++) {
      const unsigned long long ref = h_out[2 * i + 1];
      const uint32_t qs = uint32_t(ref >> 48), tile = uint32_t((ref >> 16) & 0xffffffffu), r = uint32_t(ref & 0xffffu);
      const Segment& S = *qseg_seg[qs];
      const TileDesc& td = S.tiles[tile];
      uint64_t row = uint64_t(td.row0) + r;
      for (uint32_t k = 0; k < td.rg; k++) row += uint64_t(S.rg_rows[k]);
      cands[i] = Cand{int64_t(h_out[2 * i]), qs, qseg_pos[qs], row, ref};
    }
  }

  // ---- per glob: the top `limit` in ORDER BY order (ties: file order) ----
  std::vector<std::vector<const Cand*>> per(ng);
  for (auto& c : cands) per[qseg_glob[c.qseg]].push_back(&c);
  for (auto& v : per) {
    std::sort(v.begin(), v.end(), [&](const Cand* a, const Cand* b) {
      if (a->ts != b->ts) return desc ? a->ts > b->ts : a->ts < b->ts;
      if (a->pos != b->pos) return a->pos < b->pos;
      return a->row < b->row;
    });
    if (v.size() > limit) v.resize(size_t(limit));
  }
  // Akka mergeSorted fold over the globs' streams (Commons.scala:391-392): merge(merge(merge([], g0), g1), g2)...,
  // each merge emitting the left head when it is strictly less under the ordering, the right head otherwise.
  const bool rev = R.reverse_sort;   // rollupAgg is empty for exemplars (Commons.scala:125-129)
  auto less = [&](const Cand* a, const Cand* b) { return rev ? a->ts > b->ts : a->ts < b->ts; };
  std::vector<const Cand*> stream;
  for (auto& v : per) {
    std::vector<const Cand*> m;
    m.reserve(stream.size() + v.size());
    size_t i = 0, j = 0;
    while (i < stream.size() && j < v.size()) {
      if (less(stream[i], v[j])) m.push_back(stream[i++]);
      else m.push_back(v[j++]);
    }
    while (i < stream.size()) m.push_back(stream[i++]);
    while (j < v.size()) m.push_back(v[j++]);
    stream.swap(m);
  }

  // ---- gather every output column of the selected rows ----
  std::vector<std::string> out_cols;
  for (auto& g : globs) {
    if (g.skip) continue;
    for (auto& c : g.cols)
      if (std::find(out_cols.begin(), out_cols.end(), c) == out_cols.end()) out_cols.push_back(c);
  }
  const size_t nsel = stream.size(), ncols = out_cols.size();
  std::vector<unsigned long long> gval(nsel * ncols);
  std::vector<uint8_t> gok(nsel * ncols);
  if (nsel && ncols) {
    std::vector<GCol> gcols(qsegs.size() * ncols);
    for (size_t q = 0; q < qsegs.size(); q++) {
      const Segment& S = *qseg_seg[q];
      for (size_t k = 0; k < ncols; k++) {
        GCol& gc = gcols[q * ncols + k];
        const int c = S.col_index(out_cols[k]);
        if (c < 0) {
          if (S.all_columns.count(out_cols[k]))
            throw PlanError(LK_ERR_UNSUPPORTED, "column " + out_cols[k] + " has a physical type the engine does not load");
          continue;
        }
        const HostCol& hc = S.cols[c];
        gc = GCol{S.d_data, hc.d_runs, hc.d_tcols, hc.d_remap, 1u, 0u};
      }
    }
    const size_t gb = gcols.size() * sizeof(GCol), sb = nsel * 8, vb = nsel * ncols * 8, ob = nsel * ncols;
    PinnedTmp gio(gb + sb + vb + ob + 64);   // pinned staging both ways: [columns | selected refs | values | ok]
    uint8_t* hg = static_cast<uint8_t*>(gio.p());
    memcpy(hg, gcols.data(), gb);
    for (size_t i = 0; i < nsel; i++) reinterpret_cast<unsigned long long*>(hg + gb)[i] = stream[i]->ref;
    uint8_t* dg = static_cast<uint8_t*>(X.workspace("xgather", gb + sb + vb + ob + 1024));
    XHIP_TRY(hipMemcpyAsync(dg, hg, gb + sb, hipMemcpyHostToDevice, st));
    GParams G{};
    G.cols = reinterpret_cast<const GCol*>(dg);
    G.sel = reinterpret_cast<const unsigned long long*>(dg + gb);
    G.nsel = uint32_t(nsel);
    G.ncols = uint32_t(ncols);
    G.val = reinterpret_cast<unsigned long long*>(dg + gb + sb);
    G.ok = dg + gb + sb + vb;
    XHIP_TRY(launch_ex_gather(G, st));
    XHIP_TRY(hipMemcpyAsync(hg + gb + sb, G.val, vb + ob, hipMemcpyDeviceToHost, st));   // values and ok flags
    XHIP_TRY(hipStreamSynchronize(st));
    memcpy(gval.data(), hg + gb + sb, vb);
    memcpy(gok.data(), hg + gb + sb + vb, ob);
  }

  // ---- rows: timestamp, getDouble(value) (SQL NULL -> 0.0), tags as JDBC getString text ----
  res->alloc_rows(nsel);
  res->tag_names = out_cols;
  res->ex_tags.assign(nsel * ncols, nullptr);
  const size_t vcol = size_t(std::find(out_cols.begin(), out_cols.end(), std::string(kValue)) - out_cols.begin());
  for (size_t i = 0; i < nsel; i++) {
    const Cand& c = *stream[i];
    res->ts[i] = c.ts;
    res->glob[i] = qseg_glob[c.qseg];
    res->gid[i] = uint32_t(i);
    res->val[i] = 0.0;
  }
  // column by column: each (segment, column)'s physical / union type looked up once, each dictionary locked once
  std::vector<const HostCol*> qcol(qsegs.size());
  std::vector<int> qut(qsegs.size());
  for (size_t k = 0; k < ncols; k++) {
    const std::string& name = out_cols[k];
    bool any_string = false;
    for (size_t q = 0; q < qsegs.size(); q++) {
      const Segment& S = *qseg_seg[q];
      const int ci = S.col_index(name);
      qcol[q] = ci < 0 ? nullptr : &S.cols[size_t(ci)];
      if (!qcol[q]) continue;
      const XGlob& g = globs[qseg_glob[q]];
      const auto ut = g.types.find(name);
      qut[q] = ut == g.types.end() ? qcol[q]->ptype : ut->second;
      any_string = any_string || qcol[q]->is_string;
    }
    GlobalDict* gd = any_string ? &E.dict(name) : nullptr;
    std::unique_lock<std::mutex> dl;
    if (gd) {
      dl = std::unique_lock<std::mutex>(gd->mu);
      res->keep.push_back(gd->vals);   // tag text outlives a compaction
    }
    for (size_t i = 0; i < nsel; i++) {
      if (!gok[i * ncols + k]) continue;
      const uint32_t q = stream[i]->qseg;
      const HostCol& hc = *qcol[q];
      const unsigned long long raw = gval[i * ncols + k];
      if (k == vcol) res->val[i] = value_double(raw, hc.ptype);
      if (hc.is_string) {
        if (qut[q] != pq::BYTE_ARRAY) throw PlanError(LK_ERR_UNSUPPORTED, "union_by_name over string and numeric " + name);
        const std::string& s = (*gd)[size_t(raw)];
        if (!null_like(s)) res->ex_tags[i * ncols + k] = s.c_str();   // Commons.scala:433
      } else {
        res->owned.push_back(value_text(raw, hc.ptype, qut[q]));
        res->ex_tags[i * ncols + k] = res->owned.back().c_str();
      }
    }
  }
  char buf[256];
  snprintf(buf, sizeof buf,
           "{\"scan_ms\":%.4f,\"total_ms\":%.4f,\"rows_scanned\":%llu,\"candidates\":%llu,\"hist_passes\":%d}",
           double(scan_ms), ms_since(t_start), (unsigned long long)rows_scanned, (unsigned long long)total, passes);
  res->stats = buf;
  return LK_OK;
}

}  // namespace lk
