// Synthetic sealed-segment writer (bench / test tooling, not product code).
//
// Writes an uncompressed Parquet file with the lakeside logs schema of SURVEY.md §8(d):
//   _cardinalhq.timestamp INT64 PLAIN (sorted, evenly spread over [t0, t0 + span); with ts_shuffle the same
//                         values permuted within each row group: no tile is sorted or pinned to one bucket)
//   _cardinalhq.value     DOUBLE PLAIN ("exact": integers in [0,1000); "real": lognormal(0, 2))
//   _cardinalhq.name               dict, 16 values  metric_00..metric_15
//   resource.service.name          dict, 100 values svc-000..svc-099
//   resource.k8s.namespace.name    dict, 20 values  ns-00..ns-19
//   _cardinalhq.level              dict, 5 values
//   resource.container.id          dict, N values c%07d (only when highcard_n > 0; config C5)
// OPTIONAL columns, v1 data pages, RLE/bit-packed definition levels, RLE_DICTIONARY indices, the layout
// pyarrow produces with compression="NONE", data_page_version="1.0".  Row groups are written in parallel.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "../lakeside_amd/csrc/thrift.hpp"

extern "C" {
typedef struct {
  uint64_t rows;
  uint64_t seed;
  int64_t t0_ms;
  int64_t span_ms;
  uint32_t rg_rows;
  uint32_t page_rows;
  int32_t value_mode;     // 0: exact integers, 1: lognormal(0,2)
  double null_frac;       // NULL probability of tag and value cells
  uint32_t highcard_n;    // 0: no resource.container.id column
  int32_t threads;        // 0: one per row group (capped at 32)
  int32_t ts_shuffle;     // 0: timestamps sorted; 1: the sorted timestamps permuted within each row group
} lk_synth_spec;

int lk_synth_segment(const lk_synth_spec* spec, uint8_t** out, size_t* out_len);
void lk_synth_free(uint8_t* p);
}

namespace {

using lk::TWriter;

struct Rng {
  uint64_t s;
  explicit Rng(uint64_t seed) : s(seed * 0x9E3779B97F4A7C15ull + 0xD1B54A32D192ED03ull) {}
  uint64_t next() {
    uint64_t z = (s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
  }
  double uniform() { return double(next() >> 11) * (1.0 / 9007199254740992.0); }
  uint32_t below(uint32_t n) { return uint32_t((next() >> 32) * uint64_t(n) >> 32); }
  double normal() {
    double u1 = uniform(), u2 = uniform();
    if (u1 < 1e-300) u1 = 1e-300;
    return std::sqrt(-2.0 * std::log(u1)) * std::cos(6.283185307179586 * u2);
  }
};

enum ColKind { TS, VAL, DICT };

struct ColSpec {
  std::string name;
  ColKind kind;
  uint32_t card = 0;
  std::vector<std::string> values;
};

void put_varint(std::vector<uint8_t>& o, uint64_t v) {
  while (v >= 0x80) { o.push_back(uint8_t(v | 0x80)); v >>= 7; }
  o.push_back(uint8_t(v));
}

// Hybrid RLE/bit-packed: RLE runs for repeats >= 8 of one value, else bit-packed runs of up to 512 values.
void hybrid_encode(const uint32_t* v, size_t n, int bw, std::vector<uint8_t>& o) {
  size_t i = 0;
  const int vbytes = (bw + 7) / 8;
  std::vector<uint32_t> lit;
  auto flush_lit = [&]() {
    size_t k = 0;
    while (k < lit.size()) {
      size_t cnt = std::min<size_t>(512, lit.size() - k);
      size_t groups = (cnt + 7) / 8;
      put_varint(o, (groups << 1) | 1);
      size_t nbytes = groups * size_t(bw);
      size_t base = o.size();
      o.resize(base + nbytes, 0);
      uint8_t* dst = o.data() + base;
      unsigned __int128 acc = 0;
      int nacc = 0;
      size_t w = 0;
      for (size_t j = 0; j < groups * 8; j++) {
        uint64_t x = j < cnt ? lit[k + j] : 0;
        acc |= (unsigned __int128)x << nacc;
        nacc += bw;
        while (nacc >= 8) {
          dst[w++] = uint8_t(acc);
          acc >>= 8;
          nacc -= 8;
        }
      }
      k += cnt;
    }
    lit.clear();
  };
  while (i < n) {
    size_t j = i + 1;
    while (j < n && v[j] == v[i]) j++;
    size_t rep = j - i;
    if (rep >= 8 && lit.size() % 8 == 0) {
      flush_lit();
      put_varint(o, uint64_t(rep) << 1);
      for (int b = 0; b < vbytes; b++) o.push_back(uint8_t(v[i] >> (8 * b)));
      i = j;
    } else {
      lit.push_back(v[i]);
      i++;
    }
  }
  flush_lit();
}

int bit_width(uint32_t maxv) {
  int b = 0;
  while (b < 32 && (uint64_t(1) << b) <= maxv) b++;
  return b;
}

struct ChunkOut {
  std::vector<uint8_t> bytes;
  int64_t dict_off = -1;    // relative to chunk start
  int64_t data_off = 0;
  int64_t num_values = 0;
};

std::vector<uint8_t> page_header_data(int32_t nvals, int32_t size, int enc) {
  TWriter w;
  w.struct_begin();
  w.i32(1, 0);          // DATA_PAGE
  w.i32(2, size);
  w.i32(3, size);
  w.field(5, lk::T_STRUCT);
  w.struct_begin();
  w.i32(1, nvals);
  w.i32(2, enc);
  w.i32(3, 3);          // RLE definition levels
  w.i32(4, 3);
  w.struct_end();
  w.struct_end();
  return w.out;
}

std::vector<uint8_t> page_header_dict(int32_t nvals, int32_t size) {
  TWriter w;
  w.struct_begin();
  w.i32(1, 2);          // DICTIONARY_PAGE
  w.i32(2, size);
  w.i32(3, size);
  w.field(7, lk::T_STRUCT);
  w.struct_begin();
  w.i32(1, nvals);
  w.i32(2, 0);          // PLAIN
  w.struct_end();
  w.struct_end();
  return w.out;
}

void append(std::vector<uint8_t>& a, const std::vector<uint8_t>& b) { a.insert(a.end(), b.begin(), b.end()); }

void encode_defs(const std::vector<uint8_t>& valid, size_t lo, size_t hi, std::vector<uint8_t>& page) {
  std::vector<uint32_t> d(hi - lo);
  for (size_t i = lo; i < hi; i++) d[i - lo] = valid.empty() ? 1 : valid[i];
  std::vector<uint8_t> enc;
  hybrid_encode(d.data(), d.size(), 1, enc);
  uint32_t L = uint32_t(enc.size());
  page.insert(page.end(), reinterpret_cast<uint8_t*>(&L), reinterpret_cast<uint8_t*>(&L) + 4);
  append(page, enc);
}

struct RgOut {
  std::vector<ChunkOut> chunks;
  uint64_t rows = 0;
};

void build_rg(const lk_synth_spec& sp, const std::vector<ColSpec>& cols, uint64_t rg, uint64_t row0, uint64_t nrows,
              RgOut& out) {
  out.rows = nrows;
  out.chunks.resize(cols.size());
  const uint32_t prow = sp.page_rows ? sp.page_rows : 131072;
  for (size_t c = 0; c < cols.size(); c++) {
    // independent stream per (segment, row group, column): the seed goes through a full 64-bit mix, so streams
    // of neighbouring row groups / columns are not shifted copies of one another
    Rng rng(Rng(Rng(sp.seed).next() ^ (rg * 0xA24BAED4963EE407ull)).next() ^ (c * 0x9FB21C651E98DF25ull + 1));
    const ColSpec& cs = cols[c];
    std::vector<uint8_t> valid;
    if (cs.kind != TS && sp.null_frac > 0) {
      valid.resize(nrows);
      for (uint64_t i = 0; i < nrows; i++) valid[i] = rng.uniform() >= sp.null_frac;
    }
    ChunkOut& ch = out.chunks[c];
    ch.num_values = int64_t(nrows);
    if (cs.kind == DICT) {
      std::vector<uint32_t> vals(nrows);
      for (uint64_t i = 0; i < nrows; i++) vals[i] = rng.below(cs.card);
      // chunk dictionary in first-appearance order (as arrow does)
      std::vector<int32_t> local(cs.card, -1);
      std::vector<uint32_t> order;
      std::vector<uint32_t> idx;
      idx.reserve(nrows);
      for (uint64_t i = 0; i < nrows; i++) {
        if (!valid.empty() && !valid[i]) continue;
        uint32_t v = vals[i];
        if (local[v] < 0) { local[v] = int32_t(order.size()); order.push_back(v); }
        idx.push_back(uint32_t(local[v]));
      }
      std::vector<uint8_t> dict;
      for (uint32_t v : order) {
        std::string s;
        if (cs.values.empty()) {
          char buf[16];
          snprintf(buf, sizeof buf, "c%07u", v);
          s = buf;
        } else {
          s = cs.values[v];
        }
        uint32_t L = uint32_t(s.size());
        dict.insert(dict.end(), reinterpret_cast<uint8_t*>(&L), reinterpret_cast<uint8_t*>(&L) + 4);
        dict.insert(dict.end(), s.begin(), s.end());
      }
      ch.dict_off = 0;
      append(ch.bytes, page_header_dict(int32_t(order.size()), int32_t(dict.size())));
      append(ch.bytes, dict);
      ch.data_off = int64_t(ch.bytes.size());
      const int bw = bit_width(order.empty() ? 0 : uint32_t(order.size() - 1));
      size_t vpos = 0;
      for (uint64_t p = 0; p < nrows; p += prow) {
        uint64_t pe = std::min<uint64_t>(nrows, p + prow);
        std::vector<uint8_t> page;
        encode_defs(valid, p, pe, page);
        size_t nv = 0;
        for (uint64_t i = p; i < pe; i++) nv += valid.empty() || valid[i];
        page.push_back(uint8_t(bw));
        hybrid_encode(idx.data() + vpos, nv, bw, page);
        vpos += nv;
        append(ch.bytes, page_header_data(int32_t(pe - p), int32_t(page.size()), 8));
        append(ch.bytes, page);
      }
    } else {
      ch.data_off = 0;
      std::vector<uint64_t> perm;   // ts_shuffle: row i of the row group takes sorted timestamp perm[i]
      if (cs.kind == TS && sp.ts_shuffle) {
        perm.resize(nrows);
        for (uint64_t i = 0; i < nrows; i++) perm[i] = i;
        for (uint64_t i = nrows; i > 1; i--) std::swap(perm[i - 1], perm[rng.next() % i]);
      }
      for (uint64_t p = 0; p < nrows; p += prow) {
        uint64_t pe = std::min<uint64_t>(nrows, p + prow);
        std::vector<uint8_t> page;
        encode_defs(valid, p, pe, page);
        size_t base = page.size();
        page.resize(base + (pe - p) * 8);
        uint8_t* dst = page.data() + base;
        size_t nv = 0;
        for (uint64_t i = p; i < pe; i++) {
          uint64_t g = row0 + (perm.empty() ? i : perm[i]);
          if (cs.kind == TS) {
            int64_t t = sp.t0_ms + int64_t((unsigned __int128)g * uint64_t(sp.span_ms) / sp.rows);
            memcpy(dst + 8 * nv++, &t, 8);
          } else {
            double x = sp.value_mode == 0 ? double(rng.below(1000)) : std::exp(2.0 * rng.normal());
            if (!valid.empty() && !valid[i]) continue;
            memcpy(dst + 8 * nv++, &x, 8);
          }
        }
        page.resize(base + nv * 8);
        append(ch.bytes, page_header_data(int32_t(pe - p), int32_t(page.size()), 0));
        append(ch.bytes, page);
      }
    }
  }
}

}  // namespace

extern "C" int lk_synth_segment(const lk_synth_spec* spec, uint8_t** out, size_t* out_len) {
  if (!spec || !out || !out_len || spec->rows == 0) return -1;
  const lk_synth_spec& sp = *spec;
  std::vector<ColSpec> cols;
  cols.push_back({"_cardinalhq.timestamp", TS, 0, {}});
  cols.push_back({"_cardinalhq.value", VAL, 0, {}});
  auto dict_col = [&](const char* name, uint32_t n, const char* fmt) {
    ColSpec c{name, DICT, n, {}};
    for (uint32_t i = 0; i < n; i++) {
      char buf[32];
      snprintf(buf, sizeof buf, fmt, i);
      c.values.push_back(buf);
    }
    cols.push_back(c);
  };
  dict_col("_cardinalhq.name", 16, "metric_%02u");
  dict_col("resource.service.name", 100, "svc-%03u");
  dict_col("resource.k8s.namespace.name", 20, "ns-%02u");
  {
    ColSpec c{"_cardinalhq.level", DICT, 5, {"INFO", "WARN", "ERROR", "DEBUG", "TRACE"}};
    cols.push_back(c);
  }
  if (sp.highcard_n) cols.push_back({"resource.container.id", DICT, sp.highcard_n, {}});
  dict_col("_cardinalhq.message", 64, "request %02u handled");   // logs projection column (exemplar rows)

  const uint64_t rgr = sp.rg_rows ? sp.rg_rows : (1u << 20);
  const uint64_t nrg = (sp.rows + rgr - 1) / rgr;
  std::vector<RgOut> rgs(nrg);
  int nt = sp.threads > 0 ? sp.threads : int(std::min<uint64_t>(nrg, 32));
  std::vector<std::thread> th;
  for (int t = 0; t < nt; t++)
    th.emplace_back([&, t] {
      for (uint64_t g = uint64_t(t); g < nrg; g += uint64_t(nt)) {
        uint64_t r0 = g * rgr;
        build_rg(sp, cols, g, r0, std::min(rgr, sp.rows - r0), rgs[g]);
      }
    });
  for (auto& x : th) x.join();

  size_t total = 4;
  for (auto& g : rgs)
    for (auto& ch : g.chunks) total += ch.bytes.size();
  std::vector<std::vector<int64_t>> offs(nrg, std::vector<int64_t>(cols.size()));
  TWriter w;
  w.struct_begin();
  w.i32(1, 1);
  w.list_begin(2, lk::T_STRUCT, uint32_t(cols.size() + 1));
  w.struct_begin();
  w.bin(4, "schema");
  w.i32(5, int32_t(cols.size()));
  w.struct_end();
  for (auto& c : cols) {
    w.struct_begin();
    w.i32(1, c.kind == TS ? 2 : c.kind == VAL ? 5 : 6);
    w.i32(3, 1);            // OPTIONAL
    w.bin(4, c.name);
    if (c.kind == DICT) w.i32(6, 0);   // UTF8
    w.struct_end();
  }
  w.i64(3, int64_t(sp.rows));
  w.list_begin(4, lk::T_STRUCT, uint32_t(nrg));
  int64_t pos = 4;
  for (uint64_t g = 0; g < nrg; g++) {
    w.struct_begin();
    w.list_begin(1, lk::T_STRUCT, uint32_t(cols.size()));
    int64_t rg_bytes = 0;
    for (size_t c = 0; c < cols.size(); c++) {
      const ChunkOut& ch = rgs[g].chunks[c];
      int64_t base = pos;
      offs[g][c] = base;
      w.struct_begin();
      w.i64(2, base);
      w.field(3, lk::T_STRUCT);
      w.struct_begin();
      w.i32(1, cols[c].kind == TS ? 2 : cols[c].kind == VAL ? 5 : 6);
      if (cols[c].kind == DICT) {
        w.list_begin(2, lk::T_I32, 3);
        w.list_i32(0);
        w.list_i32(3);
        w.list_i32(8);
      } else {
        w.list_begin(2, lk::T_I32, 2);
        w.list_i32(0);
        w.list_i32(3);
      }
      w.list_begin(3, lk::T_BINARY, 1);
      w.list_bin(cols[c].name);
      w.i32(4, 0);
      w.i64(5, ch.num_values);
      w.i64(6, int64_t(ch.bytes.size()));
      w.i64(7, int64_t(ch.bytes.size()));
      w.i64(9, base + ch.data_off);
      if (ch.dict_off >= 0) w.i64(11, base + ch.dict_off);
      w.struct_end();
      w.struct_end();
      pos += int64_t(ch.bytes.size());
      rg_bytes += int64_t(ch.bytes.size());
    }
    w.i64(2, rg_bytes);
    w.i64(3, int64_t(rgs[g].rows));
    w.struct_end();
  }
  w.bin(6, "lakeside-mi355x synth");
  w.struct_end();
  total += w.out.size() + 8;
  uint8_t* buf = static_cast<uint8_t*>(malloc(total));
  if (!buf) return -2;
  memcpy(buf, "PAR1", 4);
  size_t p = 4;
  for (auto& g : rgs)
    for (auto& ch : g.chunks) {
      memcpy(buf + p, ch.bytes.data(), ch.bytes.size());
      p += ch.bytes.size();
    }
  memcpy(buf + p, w.out.data(), w.out.size());
  p += w.out.size();
  uint32_t flen = uint32_t(w.out.size());
  memcpy(buf + p, &flen, 4);
  memcpy(buf + p + 4, "PAR1", 4);
  *out = buf;
  *out_len = total;
  return 0;
}

extern "C" void lk_synth_free(uint8_t* p) { free(p); }
