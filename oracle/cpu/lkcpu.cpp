// lkcpu — multi-core CPU restatement of the sealed-segment DataExpr evaluation (TEST INFRASTRUCTURE ONLY).
//
// The parity oracle's fast twin: the same semantics as oracle/dataexpr.py, written from
// scratch in C++17 + OpenMP over the same in-memory Parquet bytes, so that
//   * bench.py times the reference algorithm on every host core (cpu_baseline, kind "port": the reference's
//     JVM + DuckDB 1.3.2 cannot run here), and
//   * bench.py validates the GPU's merged rows at the full BASELINE size (64 x 2^24 rows), where the Python
//     oracle would take minutes.
// Only tests/, bench.py's cpu_baseline / validation leg and __graft_entry__.smoke() may load it; the product path
// (lakeside_amd/) never does.
//
// What it restates (reference file:line):
//   globs of glob_size segments in request order                       Commons.scala:361-366
//   per-glob column union, nonExistentFields -> leaf `false`          Commons.scala:214-224, BaseExpr.scala:462-464
//   referenced column missing from the whole glob -> empty glob       Commons.scala:249-253 (DuckDB Binder Error)
//   window [min startTs, max endTs), step of the glob head            Commons.scala:225-226, 232
//   bucket ts - fmod(ts, step) (logs/traces) or ts (metrics)          BaseExpr.scala:163-165, 376-394
//   Kleene filter over eq / != / in / not_in / has / exists / regex   BaseExpr.scala:470-511
//   GROUP BY bucket, groupBys present in the glob, name; NULL key     BaseExpr.scala:338-346, 400-404
//   sum / min / max / count (NULL values ignored), avg = sum / count  BaseExpr.scala:319-405
//   tag queries: COUNT(*) per tag value (NULL its own group)          BaseExpr.scala:127-143
// Regex leaves use POSIX ERE (regcomp, REG_ICASE): identical to RE2 on the ASCII patterns of the bench configs
// (the exact RE2 semantics are tested separately, tests/test_regex.py).  Pages must be uncompressed (the bench's
// synthetic segments are); anything else is refused.
#include <regex.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <vector>

#ifdef _OPENMP
#include <omp.h>
#endif

namespace {

struct Err : std::runtime_error {
  using std::runtime_error::runtime_error;
};

// ---------------------------------------------------------------------------------------------------------
// Thrift compact protocol (the subset Parquet footers / page headers use)
// ---------------------------------------------------------------------------------------------------------
struct TReader {
  const uint8_t* p;
  const uint8_t* e;
  uint8_t byte() {
    if (p >= e) throw Err("thrift: truncated");
    return *p++;
  }
  uint64_t varint() {
    uint64_t v = 0;
    for (int sh = 0; sh < 64; sh += 7) {
      const uint8_t b = byte();
      v |= uint64_t(b & 0x7f) << sh;
      if (!(b & 0x80)) return v;
    }
    throw Err("thrift: bad varint");
  }
  int64_t zz() {
    const uint64_t v = varint();
    return int64_t(v >> 1) ^ -int64_t(v & 1);
  }
  std::string bin() {
    const uint64_t n = varint();
    if (uint64_t(e - p) < n) throw Err("thrift: truncated binary");
    std::string s(reinterpret_cast<const char*>(p), n);
    p += n;
    return s;
  }
  void skip(int t) {
    switch (t) {
      case 1: case 2: return;
      case 3: byte(); return;
      case 4: case 5: case 6: varint(); return;
      case 7: if (e - p < 8) throw Err("thrift: truncated"); p += 8; return;
      case 8: bin(); return;
      case 9: case 10: {
        const uint8_t h = byte();
        uint64_t n = h >> 4;
        if (n == 15) n = varint();
        for (uint64_t i = 0; i < n; i++) skip_elem(h & 15);
        return;
      }
      case 11: {
        const uint64_t n = varint();
        if (!n) return;
        const uint8_t kv = byte();
        for (uint64_t i = 0; i < n; i++) {
          skip_elem(kv >> 4);
          skip_elem(kv & 15);
        }
        return;
      }
      case 12: skip_struct(); return;
      default: throw Err("thrift: bad type");
    }
  }
  void skip_elem(int t) {
    if (t == 1 || t == 2) byte();
    else skip(t);
  }
  void skip_struct() {
    int16_t id = 0;
    for (;;) {
      int t;
      if (!field(id, t)) return;
      skip(t);
    }
  }
  // next field of the current struct; false at STOP
  bool field(int16_t& id, int& t) {
    const uint8_t h = byte();
    if (h == 0) return false;
    t = h & 15;
    const int d = h >> 4;
    id = d ? int16_t(id + d) : int16_t(zz());
    return true;
  }
  // list header -> (count, element type)
  uint64_t list(int& et) {
    const uint8_t h = byte();
    et = h & 15;
    uint64_t n = h >> 4;
    if (n == 15) n = varint();
    return n;
  }
};

struct SchemaElem {
  int type = -1, rep = 0, nchild = 0;
  std::string name;
};
struct ColMeta {
  int type = -1, codec = 0;
  int64_t num_values = 0, data_off = -1, dict_off = -1, total_compressed = 0;
};
struct RowGroupMeta {
  int64_t num_rows = 0;
  std::vector<ColMeta> cols;
};
struct FileMeta {
  std::vector<SchemaElem> schema;
  int64_t num_rows = 0;
  std::vector<RowGroupMeta> rgs;
};

ColMeta read_colmeta(TReader& r) {
  ColMeta m;
  int16_t id = 0;
  int t;
  while (r.field(id, t)) {
    if (id == 1 && t == 5) m.type = int(r.zz());
    else if (id == 4 && t == 5) m.codec = int(r.zz());
    else if (id == 5 && t == 6) m.num_values = r.zz();
    else if (id == 7 && t == 6) m.total_compressed = r.zz();
    else if (id == 9 && t == 6) m.data_off = r.zz();
    else if (id == 11 && t == 6) m.dict_off = r.zz();
    else r.skip(t);
  }
  return m;
}

FileMeta read_footer(const uint8_t* f, size_t n) {
  if (n < 12 || memcmp(f, "PAR1", 4) || memcmp(f + n - 4, "PAR1", 4)) throw Err("parquet: not a Parquet file");
  uint32_t flen;
  memcpy(&flen, f + n - 8, 4);
  if (size_t(flen) + 8 > n) throw Err("parquet: bad footer length");
  TReader r{f + n - 8 - flen, f + n - 8};
  FileMeta fm;
  int16_t id = 0;
  int t;
  while (r.field(id, t)) {
    if (id == 2 && t == 9) {
      int et;
      const uint64_t k = r.list(et);
      for (uint64_t i = 0; i < k; i++) {
        SchemaElem s;
        int16_t sid = 0;
        int st;
        while (r.field(sid, st)) {
          if (sid == 1 && st == 5) s.type = int(r.zz());
          else if (sid == 3 && st == 5) s.rep = int(r.zz());
          else if (sid == 4 && st == 8) s.name = r.bin();
          else if (sid == 5 && st == 5) s.nchild = int(r.zz());
          else r.skip(st);
        }
        fm.schema.push_back(s);
      }
    } else if (id == 3 && t == 6) {
      fm.num_rows = r.zz();
    } else if (id == 4 && t == 9) {
      int et;
      const uint64_t k = r.list(et);
      for (uint64_t i = 0; i < k; i++) {
        RowGroupMeta g;
        int16_t gid = 0;
        int gt;
        while (r.field(gid, gt)) {
          if (gid == 1 && gt == 9) {
            int ct;
            const uint64_t nc = r.list(ct);
            for (uint64_t c = 0; c < nc; c++) {
              ColMeta m;
              int16_t cid = 0;
              int cty;
              while (r.field(cid, cty)) {
                if (cid == 3 && cty == 12) m = read_colmeta(r);
                else r.skip(cty);
              }
              g.cols.push_back(m);
            }
          } else if (gid == 3 && gt == 6) {
            g.num_rows = r.zz();
          } else {
            r.skip(gt);
          }
        }
        fm.rgs.push_back(std::move(g));
      }
    } else {
      r.skip(t);
    }
  }
  return fm;
}

struct PageHdr {
  int type = -1;
  int32_t usize = 0, csize = 0;
  int32_t nvals = 0, enc = 0, nrows = -1, def_len = 0, rep_len = 0;
  size_t hlen = 0;
};

PageHdr read_page_header(const uint8_t* p, const uint8_t* e) {
  TReader r{p, e};
  PageHdr h;
  int16_t id = 0;
  int t;
  while (r.field(id, t)) {
    if (id == 1 && t == 5) h.type = int(r.zz());
    else if (id == 2 && t == 5) h.usize = int32_t(r.zz());
    else if (id == 3 && t == 5) h.csize = int32_t(r.zz());
    else if ((id == 5 || id == 7 || id == 8) && t == 12) {   // data page v1 / dictionary / data page v2 header
      int16_t sid = 0;
      int st;
      while (r.field(sid, st)) {
        if (sid == 1 && st == 5) h.nvals = int32_t(r.zz());
        else if (id == 5 && sid == 2 && st == 5) h.enc = int32_t(r.zz());
        else if (id == 8 && sid == 3 && st == 5) h.nrows = int32_t(r.zz());
        else if (id == 8 && sid == 4 && st == 5) h.enc = int32_t(r.zz());
        else if (id == 8 && sid == 5 && st == 5) h.def_len = int32_t(r.zz());
        else if (id == 8 && sid == 6 && st == 5) h.rep_len = int32_t(r.zz());
        else r.skip(st);
      }
    } else {
      r.skip(t);
    }
  }
  h.hlen = size_t(r.p - p);
  return h;
}

// RLE / bit-packed hybrid: n values of bit width bw
void hybrid(const uint8_t* p, const uint8_t* e, int bw, size_t n, int32_t* out) {
  TReader r{p, e};
  size_t i = 0;
  const int vb = (bw + 7) / 8;
  while (i < n) {
    const uint64_t h = r.varint();
    if (h & 1) {
      const size_t groups = size_t(h >> 1), cnt = groups * 8;
      const uint8_t* d = r.p;
      if (size_t(e - d) < groups * size_t(bw)) throw Err("parquet: truncated bit-packed run");
      const uint64_t mask = bw >= 32 ? 0xffffffffull : ((1ull << bw) - 1);
      const size_t bytes = groups * size_t(bw);
      for (size_t k = 0; k < cnt && i < n; k++, i++) {
        const uint64_t bit = uint64_t(k) * uint64_t(bw);
        const size_t b0 = size_t(bit >> 3);
        uint64_t w = 0;
        memcpy(&w, d + b0, std::min<size_t>(8, bytes - b0));   // bw <= 32: the value lies in these 8 bytes
        out[i] = int32_t((w >> (bit & 7)) & mask);
      }
      r.p = d + groups * size_t(bw);
    } else {
      const size_t cnt = size_t(h >> 1);
      uint32_t v = 0;
      for (int b = 0; b < vb; b++) v |= uint32_t(r.byte()) << (8 * b);
      for (size_t k = 0; k < cnt && i < n; k++) out[i++] = int32_t(v);
    }
  }
}

// One column chunk decoded: numeric values (+ validity) or dictionary codes (-1 = NULL) + the chunk dictionary.
struct Chunk {
  std::vector<int64_t> i64;
  std::vector<double> f64;
  std::vector<uint8_t> valid;
  std::vector<int32_t> codes;
  std::vector<std::string> dict;
};

void decode_chunk(const uint8_t* f, size_t fsize, const ColMeta& m, bool optional, int64_t nrows, bool is_string,
                  Chunk& c) {
  if (m.codec != 0) throw Err("lkcpu: compressed pages are not supported by the CPU restatement");
  int64_t pos = m.data_off;
  if (m.dict_off > 0 && m.dict_off < pos) pos = m.dict_off;
  if (is_string) c.codes.assign(size_t(nrows), -1);
  else c.valid.assign(size_t(nrows), 0);
  if (!is_string) {
    if (m.type == 2) c.i64.assign(size_t(nrows), 0);
    else c.f64.assign(size_t(nrows), 0.0);
  }
  int64_t row = 0;
  std::vector<int32_t> defs, idx;
  while (row < nrows) {
    if (pos < 0 || size_t(pos) >= fsize) throw Err("parquet: page offset past the file");
    const PageHdr h = read_page_header(f + pos, f + fsize);
    const uint8_t* d = f + pos + h.hlen;
    const uint8_t* de = d + h.csize;
    if (de > f + fsize) throw Err("parquet: page past the file");
    pos += int64_t(h.hlen) + h.csize;
    if (h.type == 2) {   // dictionary page: PLAIN byte arrays
      c.dict.clear();
      const uint8_t* q = d;
      for (int32_t k = 0; k < h.nvals; k++) {
        uint32_t L;
        memcpy(&L, q, 4);
        q += 4;
        c.dict.emplace_back(reinterpret_cast<const char*>(q), L);
        q += L;
      }
      continue;
    }
    if (h.type != 0 && h.type != 3) continue;
    const int64_t n = h.type == 3 ? (h.nrows >= 0 ? h.nrows : h.nvals) : h.nvals;
    const uint8_t* v = d;
    defs.assign(size_t(n), 1);
    if (h.type == 0) {
      if (optional) {
        uint32_t L;
        memcpy(&L, v, 4);
        hybrid(v + 4, v + 4 + L, 1, size_t(n), defs.data());
        v += 4 + L;
      }
    } else {
      if (h.rep_len) throw Err("lkcpu: repeated columns");
      if (optional) hybrid(v, v + h.def_len, 1, size_t(n), defs.data());
      v += h.def_len;
    }
    size_t nn = 0;
    for (int64_t k = 0; k < n; k++) nn += defs[size_t(k)] != 0;
    if (is_string) {
      idx.assign(nn, 0);
      if (h.enc == 0) {   // PLAIN byte arrays: a page-local dictionary appended to the chunk's
        const uint8_t* q = v;
        std::unordered_map<std::string, int32_t> local;
        for (size_t k = 0; k < nn; k++) {
          uint32_t L;
          memcpy(&L, q, 4);
          q += 4;
          std::string s(reinterpret_cast<const char*>(q), L);
          q += L;
          auto it = local.find(s);
          if (it == local.end()) {
            it = local.emplace(s, int32_t(c.dict.size())).first;
            c.dict.push_back(s);
          }
          idx[k] = it->second;
        }
      } else {   // RLE_DICTIONARY / PLAIN_DICTIONARY
        const int bw = *v;
        hybrid(v + 1, de, bw, nn, idx.data());
      }
      size_t k = 0;
      for (int64_t r = 0; r < n; r++) c.codes[size_t(row + r)] = defs[size_t(r)] ? idx[k++] : -1;
    } else {
      if (h.enc != 0) throw Err("lkcpu: non-PLAIN numeric page");
      const uint8_t* q = v;
      for (int64_t r = 0; r < n; r++) {
        if (!defs[size_t(r)]) continue;
        if (m.type == 2) memcpy(&c.i64[size_t(row + r)], q, 8);
        else memcpy(&c.f64[size_t(row + r)], q, 8);
        c.valid[size_t(row + r)] = 1;
        q += 8;
      }
    }
    row += n;
  }
}

// ---------------------------------------------------------------------------------------------------------
// plan
// ---------------------------------------------------------------------------------------------------------
struct Leaf {
  int col;                       // string column index (-1: a numeric comparison on the value column)
  double c = 0;                  // numeric leaf: the normalized literal
  std::string op;
  std::vector<std::string> v;
  std::unique_ptr<regex_t> re;   // regex / contains
};

enum { OP_AND = -1, OP_OR = -2, OP_NOT = -3 };

struct Plan {
  bool metrics = false;
  bool tag = false;                        // tag query: strcols[0] is the tag, the only key; COUNT(*), one bucket
  std::string agg, vcol;
  int glob_size = 10;
  std::vector<int64_t> start, end, step;   // per segment request
  std::vector<std::string> strcols;        // 0 = name, then filter keys / groupBys
  std::vector<int> gby;                    // groupBy string column indices, request order (deduplicated)
  std::vector<Leaf> leaves;
  std::vector<int> prog;                   // postfix: >= 0 leaf, < 0 op
  std::vector<std::string> fieldset;       // BaseExpr.fieldSet: filter keys outside NOT + groupBys
};

// ---------------------------------------------------------------------------------------------------------
// aggregation
// ---------------------------------------------------------------------------------------------------------
struct Acc {
  uint64_t rows = 0, cnt = 0;
  double hi = 0, lo = 0;   // double-double sum (TwoSum)
  double mn = INFINITY, mx = -INFINITY;
  bool any_nan = false;
  int nonnan = 0;
  void add(bool valid, double v) {
    rows++;
    if (!valid) return;
    cnt++;
    const double s = hi + v, bb = s - hi;
    lo += (hi - (s - bb)) + (v - bb);
    hi = s;
    if (std::isnan(v)) {
      any_nan = true;
    } else {
      mn = std::min(mn, v);
      mx = std::max(mx, v);
      nonnan = 1;
    }
  }
  void merge(const Acc& o) {
    rows += o.rows;
    cnt += o.cnt;
    const double s = hi + o.hi, bb = s - hi;
    lo += (hi - (s - bb)) + (o.hi - bb) + o.lo;
    hi = s;
    mn = std::min(mn, o.mn);
    mx = std::max(mx, o.mx);
    any_nan |= o.any_nan;
    nonnan |= o.nonnan;
  }
};

// cell key: bucket index + up to 6 group ids (global ids per column, -1 NULL)
struct Key {
  int64_t ts;
  int32_t g[7];
  bool operator==(const Key& o) const { return ts == o.ts && memcmp(g, o.g, sizeof(g)) == 0; }
};
struct KeyHash {
  size_t operator()(const Key& k) const {
    uint64_t h = uint64_t(k.ts) * 0x9E3779B97F4A7C15ull;
    for (int i = 0; i < 7; i++) h = (h ^ uint32_t(k.g[i])) * 0xff51afd7ed558ccdull;
    return size_t(h ^ (h >> 29));
  }
};
using CellMap = std::unordered_map<Key, Acc, KeyHash>;

// engine-global ids of string values per column (chunks remap into these)
struct GlobalIds {
  std::mutex mu;
  std::unordered_map<std::string, int32_t> ids;
  std::vector<std::string> vals;
  int32_t id(const std::string& s) {
    auto it = ids.find(s);
    if (it != ids.end()) return it->second;
    const int32_t i = int32_t(vals.size());
    vals.push_back(s);
    ids.emplace(s, i);
    return i;
  }
};

struct Segment {
  const uint8_t* data;
  size_t size;
  FileMeta fm;
  std::map<std::string, int> col;   // column name -> schema leaf index
};

bool leaf_hit(const Leaf& l, const std::string& s) {
  if (l.op == "eq") return s == l.v[0];
  if (l.op == "!=") return s != l.v[0];
  if (l.op == "in") return std::find(l.v.begin(), l.v.end(), s) != l.v.end();
  if (l.op == "not_in") return std::find(l.v.begin(), l.v.end(), s) == l.v.end();
  if (l.op == "has" || l.op == "exists") return true;
  return regexec(l.re.get(), s.c_str(), 0, nullptr, 0) == 0;
}

struct Result {
  // per-glob cells
  std::vector<int32_t> glob;
  std::vector<int64_t> ts;
  std::vector<uint64_t> rows, cnt;
  std::vector<double> hi, lo, mn, mx;
  std::vector<uint8_t> nan_flag;   // bit0: some NaN value, bit1: some non-NaN value
  std::vector<int32_t> keys;       // ncol per cell: global id (-1 NULL / absent column)
  int ncol = 0;
  std::vector<std::vector<std::string>> dict;   // per key column: global id -> string
  std::string err;
};

thread_local std::string t_err;

}  // namespace

// ---------------------------------------------------------------------------------------------------------
// C ABI
// ---------------------------------------------------------------------------------------------------------
extern "C" {

struct lkcpu_result;

// plan: newline-separated tokens (strings percent-encoded), see oracle/cpu.py:_plan_text
// segments: n_segs (pointer, size) pairs of in-memory Parquet files, in request order.
void* lkcpu_eval(const char* plan_text, const uint8_t* const* seg_ptrs, const size_t* seg_sizes, size_t n_segs,
                 int threads);
const char* lkcpu_error(void);
size_t lkcpu_ncells(void* r);
int lkcpu_ncols(void* r);
void lkcpu_cells(void* r, int32_t* glob, int64_t* ts, uint64_t* rows, uint64_t* cnt, double* hi, double* lo,
                 double* mn, double* mx, uint8_t* nanf, int32_t* keys);
const char* lkcpu_key_string(void* r, int col, int32_t id);
void lkcpu_free(void* r);
// Exemplar rows (no chart): per glob ORDER BY timestamp <desc|asc> LIMIT limit (ties in file order), tags = every
// column's text, globs folded by Akka mergeSorted (reverse: timestamp descending).  Numbers print as JDBC getString:
// INT64 in decimal, DOUBLE only when integral and below 1e7 ("N.0", Java Double.toString) -- anything else is refused
// (the restatement does not carry a Java double formatter; the bench's synthetic values are integers).
void* lkcpu_exemplar(const char* plan_text, const uint8_t* const* seg_ptrs, const size_t* seg_sizes, size_t n_segs,
                     int threads, int64_t limit, int desc, int reverse);
size_t lkcpu_ex_rows(void* r);
void lkcpu_ex_row(void* r, size_t i, int64_t* ts, double* val, int32_t* glob);
const char* lkcpu_ex_tags(void* r, size_t i);   // canonical tag key: items sorted by name, "k\x1ev" joined by "\x1f"
void lkcpu_ex_free(void* r);

}  // extern "C"

namespace {

std::string pct_decode(const std::string& s) {
  std::string o;
  for (size_t i = 0; i < s.size(); i++) {
    if (s[i] == '%' && i + 2 < s.size()) {
      o += char(std::stoi(s.substr(i + 1, 2), nullptr, 16));
      i += 2;
    } else {
      o += s[i];
    }
  }
  return o;
}

Plan parse_plan(const char* text) {
  std::vector<std::string> tok;
  {
    std::string cur;
    for (const char* p = text; *p; p++) {
      if (*p == '\n') {
        tok.push_back(pct_decode(cur));
        cur.clear();
      } else {
        cur += *p;
      }
    }
    if (!cur.empty()) tok.push_back(pct_decode(cur));
  }
  size_t i = 0;
  auto next = [&]() -> const std::string& {
    if (i >= tok.size()) throw Err("lkcpu: truncated plan");
    return tok[i++];
  };
  auto num = [&]() { return std::stoll(next()); };
  Plan P;
  {
    const std::string ds = next();
    P.metrics = ds == "metrics";
    P.tag = ds == "tag";
  }
  P.agg = next();
  P.vcol = next();
  P.glob_size = int(num());
  const int nseg = int(num());
  for (int s = 0; s < nseg; s++) {
    P.start.push_back(num());
    P.end.push_back(num());
    P.step.push_back(num());
  }
  const int nstr = int(num());
  for (int s = 0; s < nstr; s++) P.strcols.push_back(next());
  const int ngb = int(num());
  for (int g = 0; g < ngb; g++) P.gby.push_back(int(num()));
  const int nl = int(num());
  for (int l = 0; l < nl; l++) {
    Leaf L;
    L.col = int(num());
    L.op = next();
    const int nv = int(num());
    for (int k = 0; k < nv; k++) L.v.push_back(next());
    if (L.col < 0) L.c = std::stod(L.v.at(0));
    if (L.op == "regex" || L.op == "contains") {
      const std::string pat = L.op == "contains" ? ".*" + L.v[0] + ".*" : L.v[0];
      L.re.reset(new regex_t);
      if (regcomp(L.re.get(), pat.c_str(), REG_EXTENDED | REG_ICASE | REG_NOSUB) != 0)
        throw Err("lkcpu: regex " + pat + " not compilable as POSIX ERE");
    }
    P.leaves.push_back(std::move(L));
  }
  const int np = int(num());
  for (int k = 0; k < np; k++) P.prog.push_back(int(num()));
  const int nf = int(num());
  for (int k = 0; k < nf; k++) P.fieldset.push_back(next());
  return P;
}

// Kleene evaluation of the postfix program on (T, F) leaf bit masks: TRUE?
bool kleene(const std::vector<int>& prog, uint32_t T, uint32_t F) {
  uint64_t st = 0, sf = 0;
  for (int op : prog) {
    if (op >= 0) {
      st = (st << 1) | ((T >> op) & 1u);
      sf = (sf << 1) | ((F >> op) & 1u);
    } else if (op == OP_NOT) {
      const uint64_t t1 = st & 1, f1 = sf & 1;
      st = (st & ~1ull) | f1;
      sf = (sf & ~1ull) | t1;
    } else {
      const uint64_t t2 = st & 1, f2 = sf & 1;
      st >>= 1;
      sf >>= 1;
      const uint64_t t1 = st & 1, f1 = sf & 1;
      st = (st & ~1ull) | (op == OP_AND ? (t1 & t2) : (t1 | t2));
      sf = (sf & ~1ull) | (op == OP_AND ? (f1 | f2) : (f1 & f2));
    }
  }
  return prog.empty() || (st & 1);
}

Result* evaluate(const Plan& P, const uint8_t* const* ptrs, const size_t* sizes, size_t nseg, int threads) {
  auto* R = new Result();
  std::vector<Segment> segs(nseg);
  for (size_t s = 0; s < nseg; s++) {
    segs[s].data = ptrs[s];
    segs[s].size = sizes[s];
    segs[s].fm = read_footer(ptrs[s], sizes[s]);
    for (size_t k = 1; k < segs[s].fm.schema.size(); k++) segs[s].col[segs[s].fm.schema[k].name] = int(k - 1);
  }
  const size_t nglobs = (nseg + size_t(P.glob_size) - 1) / size_t(P.glob_size);
  const int nstr = int(P.strcols.size());
  // per glob: union of columns -> nonexistent fields, skipped globs, present group-by columns
  std::vector<uint32_t> leaf_false(nglobs, 0);
  std::vector<char> skip(nglobs, 0);
  std::vector<std::vector<int>> keycols(nglobs);   // string column indices forming the key: name + present groupBys
  std::vector<int64_t> wlo(nglobs), whi(nglobs), gstep(nglobs);
  for (size_t g = 0; g < nglobs; g++) {
    std::map<std::string, int> uni;
    const size_t a = g * size_t(P.glob_size), b = std::min(nseg, a + size_t(P.glob_size));
    wlo[g] = INT64_MAX;
    whi[g] = INT64_MIN;
    for (size_t s = a; s < b; s++) {
      for (auto& kv : segs[s].col) uni[kv.first] = 1;
      wlo[g] = std::min(wlo[g], P.start[s]);
      whi[g] = std::max(whi[g], P.end[s]);
    }
    gstep[g] = P.step[a];
    std::map<std::string, int> nonexist;
    for (auto& f : P.fieldset)
      if (!uni.count(f)) nonexist[f] = 1;
    auto leaf_col = [&](const Leaf& l) -> const std::string& { return l.col < 0 ? P.vcol : P.strcols[size_t(l.col)]; };
    for (size_t l = 0; l < P.leaves.size(); l++)
      if (nonexist.count(leaf_col(P.leaves[l]))) leaf_false[g] |= 1u << l;
    // DuckDB Binder Error: a referenced column no file of the glob has (leaf columns not compiled to false,
    // timestamp, name, value)
    for (auto& l : P.leaves)
      if (!nonexist.count(leaf_col(l)) && !uni.count(leaf_col(l))) skip[g] = 1;
    if (P.tag) {   // SELECT "<tag>", COUNT(*) ... GROUP BY "<tag>" (BaseExpr.scala:127-143): the tag must exist
      if (!uni.count("_cardinalhq.timestamp") || !uni.count(P.strcols[0])) skip[g] = 1;
      keycols[g].push_back(0);
      continue;
    }
    if (!uni.count("_cardinalhq.timestamp") || !uni.count("_cardinalhq.name") || !uni.count(P.vcol)) skip[g] = 1;
    keycols[g].push_back(0);
    for (int c : P.gby)
      if (!nonexist.count(P.strcols[size_t(c)])) keycols[g].push_back(c);
  }
  std::vector<std::unique_ptr<GlobalIds>> gids(static_cast<size_t>(nstr));
  for (auto& x : gids) x.reset(new GlobalIds);

  // tasks: (segment, row group)
  std::vector<std::pair<int, int>> tasks;
  for (size_t s = 0; s < nseg; s++)
    if (!skip[s / size_t(P.glob_size)])
      for (size_t r = 0; r < segs[s].fm.rgs.size(); r++) tasks.emplace_back(int(s), int(r));
#ifdef _OPENMP
  if (threads > 0) omp_set_num_threads(threads);
  const int nthreads = omp_get_max_threads();
#else
  const int nthreads = 1;
#endif
  std::vector<std::vector<CellMap>> part(static_cast<size_t>(nthreads), std::vector<CellMap>(nglobs));
  std::atomic<int> failed{0};
  std::mutex err_mu;
  std::string err;

#pragma omp parallel for schedule(dynamic, 1)
  for (size_t ti = 0; ti < tasks.size(); ti++) {
    if (failed.load()) continue;
    try {
#ifdef _OPENMP
      const int tid = omp_get_thread_num();
#else
      const int tid = 0;
#endif
      const Segment& S = segs[size_t(tasks[ti].first)];
      const RowGroupMeta& RG = S.fm.rgs[size_t(tasks[ti].second)];
      const size_t g = size_t(tasks[ti].first) / size_t(P.glob_size);
      const int64_t nrows = RG.num_rows;
      auto load = [&](const std::string& name, bool is_string, Chunk& c) -> bool {
        auto it = S.col.find(name);
        if (it == S.col.end()) return false;
        const SchemaElem& se = S.fm.schema[size_t(it->second) + 1];
        decode_chunk(S.data, S.size, RG.cols[size_t(it->second)], se.rep == 1, nrows, is_string, c);
        return true;
      };
      Chunk tsc, vc;
      const bool has_ts = load("_cardinalhq.timestamp", false, tsc);
      const bool has_v = !P.tag && load(P.vcol, false, vc);
      std::vector<Chunk> sc(static_cast<size_t>(nstr));
      std::vector<char> has_s(static_cast<size_t>(nstr));
      // per string column: chunk code -> (leaf T bits, global id)
      std::vector<std::vector<uint32_t>> tbits(static_cast<size_t>(nstr));
      std::vector<std::vector<int32_t>> gidmap(static_cast<size_t>(nstr));
      std::vector<uint32_t> colmask(static_cast<size_t>(nstr), 0);
      uint32_t nummask = 0;   // numeric leaves on the value column
      for (size_t l = 0; l < P.leaves.size(); l++) {
        if (P.leaves[l].col < 0) nummask |= 1u << l;
        else colmask[size_t(P.leaves[l].col)] |= 1u << l;
      }
      for (int c = 0; c < nstr; c++) {
        has_s[size_t(c)] = load(P.strcols[size_t(c)], true, sc[size_t(c)]);
        const auto& dict = sc[size_t(c)].dict;
        tbits[size_t(c)].assign(dict.size(), 0);
        gidmap[size_t(c)].assign(dict.size(), -1);
        for (size_t d = 0; d < dict.size(); d++)
          for (size_t l = 0; l < P.leaves.size(); l++)
            if (P.leaves[l].col == c && leaf_hit(P.leaves[l], dict[d])) tbits[size_t(c)][d] |= 1u << l;
        std::lock_guard<std::mutex> lg(gids[size_t(c)]->mu);
        for (size_t d = 0; d < dict.size(); d++) gidmap[size_t(c)][d] = gids[size_t(c)]->id(dict[d]);
      }
      if (!has_ts) continue;
      CellMap& cells = part[size_t(tid)][g];
      const uint32_t lf = leaf_false[g];
      const int64_t lo = wlo[g], hi = whi[g], step = gstep[g];
      Acc* last = nullptr;   // unordered_map references stay valid across inserts
      Key last_key{};
      for (int64_t r = 0; r < nrows; r++) {
        if (!tsc.valid[size_t(r)]) continue;
        const int64_t t = tsc.i64[size_t(r)];
        if (t < lo || t >= hi) continue;
        uint32_t T = 0, F = 0;
        for (int c = 0; c < nstr; c++) {
          const uint32_t m = colmask[size_t(c)];
          if (!m) continue;
          const int32_t code = has_s[size_t(c)] ? sc[size_t(c)].codes[size_t(r)] : -1;
          if (code < 0) {   // NULL: has/exists FALSE, the others NULL
            for (size_t l = 0; l < P.leaves.size(); l++)
              if (((m >> l) & 1u) && (P.leaves[l].op == "has" || P.leaves[l].op == "exists")) F |= 1u << l;
            continue;
          }
          const uint32_t b = tbits[size_t(c)][size_t(code)];
          T |= b & m;
          F |= ~b & m;
        }
        if (nummask && has_v && vc.valid[size_t(r)]) {   // value NULL: the comparison is NULL (neither bit)
          const double x = vc.f64[size_t(r)];
          for (size_t l = 0; l < P.leaves.size(); l++) {
            if (!((nummask >> l) & 1u)) continue;
            const Leaf& L = P.leaves[l];
            const bool up = L.op == "gt" || L.op == "ge";
            const bool pass = std::isnan(x) ? up   // NaN sorts greatest (DuckDB)
                              : L.op == "gt" ? x > L.c : L.op == "ge" ? x >= L.c : L.op == "lt" ? x < L.c : x <= L.c;
            (pass ? T : F) |= 1u << l;
          }
        }
        T &= ~lf;
        F |= lf;
        if (!kleene(P.prog, T, F)) continue;
        Key k;
        k.ts = P.tag ? 0 : P.metrics ? t : t - int64_t(std::fmod(double(t), double(step)));
        for (int j = 0; j < 7; j++) k.g[j] = -1;
        for (size_t j = 0; j < keycols[g].size(); j++) {
          const int c = keycols[g][j];
          const int32_t code = has_s[size_t(c)] ? sc[size_t(c)].codes[size_t(r)] : -1;
          k.g[j] = code < 0 ? -1 : gidmap[size_t(c)][size_t(code)];
        }
        const bool vv = has_v && vc.valid[size_t(r)];
        if (!last || !(last_key == k)) {   // time-sorted rows: runs of one cell
          last = &cells[k];
          last_key = k;
        }
        last->add(vv, vv ? vc.f64[size_t(r)] : 0.0);
      }
    } catch (const std::exception& e) {
      failed = 1;
      std::lock_guard<std::mutex> lg(err_mu);
      err = e.what();
    }
  }
  if (failed) throw Err(err);
  // merge the threads' partial maps per glob (thread order; the sums are compensated)
  int ncol = 1 + int(P.gby.size());
  R->ncol = ncol;
  for (size_t g = 0; g < nglobs; g++) {
    CellMap all;
    for (int t = 0; t < nthreads; t++)
      for (auto& kv : part[size_t(t)][g]) all[kv.first].merge(kv.second);
    for (auto& kv : all) {
      R->glob.push_back(int32_t(g));
      R->ts.push_back(kv.first.ts);
      R->rows.push_back(kv.second.rows);
      R->cnt.push_back(kv.second.cnt);
      R->hi.push_back(kv.second.hi);
      R->lo.push_back(kv.second.lo);
      R->mn.push_back(kv.second.mn);
      R->mx.push_back(kv.second.mx);
      R->nan_flag.push_back(uint8_t((kv.second.any_nan ? 1 : 0) | (kv.second.nonnan ? 2 : 0)));
      // key columns in request order: name, then every groupBy (-1 when absent from this glob)
      std::vector<int32_t> row(static_cast<size_t>(ncol), -1);
      row[0] = kv.first.g[0];
      for (size_t j = 1; j < keycols[g].size(); j++) {
        const int c = keycols[g][j];
        const size_t pos = size_t(std::find(P.gby.begin(), P.gby.end(), c) - P.gby.begin()) + 1;
        row[pos] = kv.first.g[j];
      }
      R->keys.insert(R->keys.end(), row.begin(), row.end());
    }
  }
  R->dict.resize(size_t(ncol));
  R->dict[0] = gids[0]->vals;
  for (size_t j = 0; j < P.gby.size(); j++) R->dict[j + 1] = gids[size_t(P.gby[j])]->vals;
  return R;
}

struct ExResult {
  std::vector<int64_t> ts;
  std::vector<double> val;
  std::vector<int32_t> glob;
  std::vector<std::string> key;
};

// Java Double.toString of an integral double below 1e7 in magnitude ("123.0", "-0.0"); refuses the rest.
std::string java_integral_text(double v) {
  if (!(std::fabs(v) < 1e7) || v != std::trunc(v)) throw Err("lkcpu exemplar: non-integral double text is not restated");
  if (v == 0.0) return std::signbit(v) ? "-0.0" : "0.0";
  return std::to_string((long long)v) + ".0";
}

ExResult* exemplar(const Plan& P, const uint8_t* const* ptrs, const size_t* sizes, size_t nseg, int threads,
                   int64_t limit, bool desc, bool reverse) {
  std::unique_ptr<ExResult> R(new ExResult());
  std::vector<Segment> segs(nseg);
  for (size_t s = 0; s < nseg; s++) {
    segs[s].data = ptrs[s];
    segs[s].size = sizes[s];
    segs[s].fm = read_footer(ptrs[s], sizes[s]);
    for (size_t k = 1; k < segs[s].fm.schema.size(); k++) segs[s].col[segs[s].fm.schema[k].name] = int(k - 1);
  }
  const std::vector<std::string> proj = P.metrics ? std::vector<std::string>{}
                                                  : std::vector<std::string>{"_cardinalhq.timestamp", "_cardinalhq.value",
                                                                             "_cardinalhq.name", "_cardinalhq.message"};
  if (P.metrics) throw Err("lkcpu exemplar: logs only");
  const size_t G = size_t(P.glob_size), nglobs = (nseg + G - 1) / G;
  const int nstr = int(P.strcols.size());
  std::vector<uint32_t> leaf_false(nglobs, 0);
  std::vector<char> skip(nglobs, 0);
  std::vector<int64_t> wlo(nglobs), whi(nglobs);
  for (size_t g = 0; g < nglobs; g++) {
    std::map<std::string, int> uni;
    wlo[g] = INT64_MAX;
    whi[g] = INT64_MIN;
    for (size_t s = g * G; s < std::min(nseg, (g + 1) * G); s++) {
      for (auto& kv : segs[s].col) uni[kv.first] = 1;
      wlo[g] = std::min(wlo[g], P.start[s]);
      whi[g] = std::max(whi[g], P.end[s]);
    }
    std::map<std::string, int> nonexist;
    for (auto& f : P.fieldset)
      if (!uni.count(f)) nonexist[f] = 1;
    for (size_t l = 0; l < P.leaves.size(); l++) {
      const std::string& c = P.strcols[size_t(P.leaves[l].col)];
      if (nonexist.count(c)) leaf_false[g] |= 1u << l;
      else if (!uni.count(c)) skip[g] = 1;   // Binder Error: the glob's query fails (empty)
    }
    for (auto& c : proj)
      if (!uni.count(c)) skip[g] = 1;
  }
  for (auto& l : P.leaves)
    if (l.col < 0) throw Err("lkcpu exemplar: numeric leaves are not restated");
  // candidates per (segment, row group): (ts, segment position in glob, row in file)
  struct Cand {
    int64_t ts;
    uint32_t seg;
    int64_t row;   // row in the file
  };
  std::vector<std::pair<int, int>> tasks;
  for (size_t s = 0; s < nseg; s++)
    if (!skip[s / G])
      for (size_t r = 0; r < segs[s].fm.rgs.size(); r++) tasks.emplace_back(int(s), int(r));
#ifdef _OPENMP
  if (threads > 0) omp_set_num_threads(threads);
#endif
  std::vector<std::vector<Cand>> part(tasks.size());
  std::atomic<int> failed{0};
  std::mutex err_mu;
  std::string err;
  auto before = [&](const Cand& a, const Cand& b) {   // ORDER BY ts <dir>, then file order (segment, row)
    if (a.ts != b.ts) return desc ? a.ts > b.ts : a.ts < b.ts;
    if (a.seg != b.seg) return a.seg < b.seg;
    return a.row < b.row;
  };
#pragma omp parallel for schedule(dynamic, 1)
  for (size_t ti = 0; ti < tasks.size(); ti++) {
    if (failed.load()) continue;
    try {
      const Segment& S = segs[size_t(tasks[ti].first)];
      const int rg = tasks[ti].second;
      const RowGroupMeta& RG = S.fm.rgs[size_t(rg)];
      const size_t g = size_t(tasks[ti].first) / G;
      int64_t row0 = 0;
      for (int k = 0; k < rg; k++) row0 += S.fm.rgs[size_t(k)].num_rows;
      auto load = [&](const std::string& name, bool is_string, Chunk& c) -> bool {
        auto it = S.col.find(name);
        if (it == S.col.end()) return false;
        const SchemaElem& se = S.fm.schema[size_t(it->second) + 1];
        decode_chunk(S.data, S.size, RG.cols[size_t(it->second)], se.rep == 1, RG.num_rows, is_string, c);
        return true;
      };
      Chunk tsc;
      if (!load("_cardinalhq.timestamp", false, tsc)) continue;
      std::vector<Chunk> sc(static_cast<size_t>(nstr));
      std::vector<char> has(static_cast<size_t>(nstr), 0);
      std::vector<std::vector<uint32_t>> tbits(static_cast<size_t>(nstr));
      std::vector<uint32_t> colmask(static_cast<size_t>(nstr), 0);
      for (size_t l = 0; l < P.leaves.size(); l++) colmask[size_t(P.leaves[l].col)] |= 1u << l;
      for (int c = 0; c < nstr; c++) {
        if (!colmask[size_t(c)]) continue;
        has[size_t(c)] = load(P.strcols[size_t(c)], true, sc[size_t(c)]);
        tbits[size_t(c)].assign(sc[size_t(c)].dict.size(), 0);
        for (size_t d = 0; d < sc[size_t(c)].dict.size(); d++)
          for (size_t l = 0; l < P.leaves.size(); l++)
            if (P.leaves[l].col == c && leaf_hit(P.leaves[l], sc[size_t(c)].dict[d])) tbits[size_t(c)][d] |= 1u << l;
      }
      std::vector<Cand>& out = part[ti];
      for (int64_t r = 0; r < RG.num_rows; r++) {
        if (!tsc.valid[size_t(r)]) continue;
        const int64_t t = tsc.i64[size_t(r)];
        if (t < wlo[g] || t >= whi[g]) continue;
        uint32_t T = 0, F = 0;
        for (int c = 0; c < nstr; c++) {
          const uint32_t m = colmask[size_t(c)];
          if (!m) continue;
          const int32_t code = has[size_t(c)] ? sc[size_t(c)].codes[size_t(r)] : -1;
          if (code < 0) {
            for (size_t l = 0; l < P.leaves.size(); l++)
              if (((m >> l) & 1u) && (P.leaves[l].op == "has" || P.leaves[l].op == "exists")) F |= 1u << l;
            continue;
          }
          const uint32_t b = tbits[size_t(c)][size_t(code)];
          T |= b & m;
          F |= ~b & m;
        }
        T &= ~leaf_false[g];
        F |= leaf_false[g];
        if (!kleene(P.prog, T, F)) continue;
        out.push_back(Cand{t, uint32_t(tasks[ti].first), row0 + r});
      }
      if (limit >= 0 && out.size() > size_t(limit)) {   // a task keeps at most its own top `limit`
        std::nth_element(out.begin(), out.begin() + limit, out.end(), before);
        out.resize(size_t(limit));
      }
    } catch (const std::exception& e) {
      failed = 1;
      std::lock_guard<std::mutex> lg(err_mu);
      err = e.what();
    }
  }
  if (failed) throw Err(err);
  // per glob: its top `limit` in ORDER BY order
  std::vector<std::vector<Cand>> per(nglobs);
  for (size_t ti = 0; ti < tasks.size(); ti++) {
    auto& v = per[size_t(tasks[ti].first) / G];
    v.insert(v.end(), part[ti].begin(), part[ti].end());
  }
  for (auto& v : per) {
    std::sort(v.begin(), v.end(), before);
    if (limit >= 0 && v.size() > size_t(limit)) v.resize(size_t(limit));
  }
  // Akka mergeSorted fold over the globs: the left head when strictly less
  struct Sel {
    Cand c;
    int32_t glob;
  };
  std::vector<Sel> stream;
  for (size_t g = 0; g < nglobs; g++) {
    std::vector<Sel> m;
    size_t i = 0, j = 0;
    while (i < stream.size() && j < per[g].size()) {
      const bool lt = reverse ? stream[i].c.ts > per[g][j].ts : stream[i].c.ts < per[g][j].ts;
      if (lt) m.push_back(stream[i++]);
      else m.push_back(Sel{per[g][j++], int32_t(g)});
    }
    while (i < stream.size()) m.push_back(stream[i++]);
    while (j < per[g].size()) m.push_back(Sel{per[g][j++], int32_t(g)});
    stream.swap(m);
  }
  // every column of the selected rows, decoded per (segment, row group) once
  std::map<std::pair<uint32_t, int>, std::map<std::string, Chunk>> cache;
  for (const Sel& x : stream) {
    const Segment& S = segs[x.c.seg];
    int rg = 0;
    int64_t r = x.c.row;
    while (rg < int(S.fm.rgs.size()) && r >= S.fm.rgs[size_t(rg)].num_rows) r -= S.fm.rgs[size_t(rg++)].num_rows;
    auto& cols = cache[std::make_pair(x.c.seg, rg)];
    if (cols.empty())
      for (auto& kv : S.col) {
        const SchemaElem& se = S.fm.schema[size_t(kv.second) + 1];
        Chunk& c = cols[kv.first];
        if (se.type != 6 && se.type != 2 && se.type != 5) throw Err("lkcpu exemplar: column type not restated: " + kv.first);
        decode_chunk(S.data, S.size, S.fm.rgs[size_t(rg)].cols[size_t(kv.second)], se.rep == 1,
                     S.fm.rgs[size_t(rg)].num_rows, se.type == 6, c);
      }
    std::map<std::string, std::string> tags;
    double value = 0.0;
    for (auto& kv : cols) {
      const SchemaElem& se = S.fm.schema[size_t(S.col.at(kv.first)) + 1];
      const Chunk& c = kv.second;
      if (se.type == 6) {
        const int32_t code = c.codes[size_t(r)];
        if (code < 0) continue;
        const std::string& v = c.dict[size_t(code)];
        if (!v.empty() && v != "null") tags[kv.first] = v;   // Commons.scala:433
      } else if (c.valid[size_t(r)]) {
        if (se.type == 2) {
          tags[kv.first] = std::to_string((long long)c.i64[size_t(r)]);
        } else {
          const double d = c.f64[size_t(r)];
          if (kv.first == "_cardinalhq.value") value = d;
          tags[kv.first] = java_integral_text(d);
        }
      }
    }
    std::string key;
    for (auto& kv : tags) {
      if (!key.empty()) key += '\x1f';
      key += kv.first;
      key += '\x1e';
      key += kv.second;
    }
    R->ts.push_back(x.c.ts);
    R->val.push_back(value);
    R->glob.push_back(x.glob);
    R->key.push_back(std::move(key));
  }
  return R.release();
}

}  // namespace

extern "C" {

void* lkcpu_exemplar(const char* plan_text, const uint8_t* const* seg_ptrs, const size_t* seg_sizes, size_t n_segs,
                     int threads, int64_t limit, int desc, int reverse) {
  try {
    Plan P = parse_plan(plan_text);
    return exemplar(P, seg_ptrs, seg_sizes, n_segs, threads, limit, desc != 0, reverse != 0);
  } catch (const std::exception& e) {
    t_err = e.what();
    return nullptr;
  }
}
size_t lkcpu_ex_rows(void* r) { return static_cast<ExResult*>(r)->ts.size(); }
void lkcpu_ex_row(void* r, size_t i, int64_t* ts, double* val, int32_t* glob) {
  const ExResult& R = *static_cast<ExResult*>(r);
  *ts = R.ts[i];
  *val = R.val[i];
  *glob = R.glob[i];
}
const char* lkcpu_ex_tags(void* r, size_t i) { return static_cast<ExResult*>(r)->key[i].c_str(); }
void lkcpu_ex_free(void* r) { delete static_cast<ExResult*>(r); }

void* lkcpu_eval(const char* plan_text, const uint8_t* const* seg_ptrs, const size_t* seg_sizes, size_t n_segs,
                 int threads) {
  try {
    Plan P = parse_plan(plan_text);
    return evaluate(P, seg_ptrs, seg_sizes, n_segs, threads);
  } catch (const std::exception& e) {
    t_err = e.what();
    return nullptr;
  }
}
const char* lkcpu_error(void) { return t_err.c_str(); }
size_t lkcpu_ncells(void* r) { return static_cast<Result*>(r)->ts.size(); }
int lkcpu_ncols(void* r) { return static_cast<Result*>(r)->ncol; }
void lkcpu_cells(void* r, int32_t* glob, int64_t* ts, uint64_t* rows, uint64_t* cnt, double* hi, double* lo,
                 double* mn, double* mx, uint8_t* nanf, int32_t* keys) {
  const Result& R = *static_cast<Result*>(r);
  const size_t n = R.ts.size();
  std::copy(R.glob.begin(), R.glob.end(), glob);
  std::copy(R.ts.begin(), R.ts.end(), ts);
  std::copy(R.rows.begin(), R.rows.end(), rows);
  std::copy(R.cnt.begin(), R.cnt.end(), cnt);
  std::copy(R.hi.begin(), R.hi.end(), hi);
  std::copy(R.lo.begin(), R.lo.end(), lo);
  std::copy(R.mn.begin(), R.mn.end(), mn);
  std::copy(R.mx.begin(), R.mx.end(), mx);
  std::copy(R.nan_flag.begin(), R.nan_flag.end(), nanf);
  std::copy(R.keys.begin(), R.keys.begin() + long(n * size_t(R.ncol)), keys);
}
const char* lkcpu_key_string(void* r, int col, int32_t id) {
  const Result& R = *static_cast<Result*>(r);
  if (id < 0 || col < 0 || col >= R.ncol || size_t(id) >= R.dict[size_t(col)].size()) return nullptr;
  return R.dict[size_t(col)][size_t(id)].c_str();
}
void lkcpu_free(void* r) { delete static_cast<Result*>(r); }

}  // extern "C"
