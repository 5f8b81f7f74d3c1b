#include "parquet.hpp"

#include <algorithm>
#include <cstring>
#include <stdexcept>

#include "thrift.hpp"

namespace lk {
namespace pq {

static void parse_schema_element(TReader& r, SchemaElement& e) {
  r.struct_begin();
  int16_t id; uint8_t t;
  while (r.field(id, t)) {
    switch (id) {
      case 1: e.type = int(r.zigzag()); break;
      case 3: e.repetition = int(r.zigzag()); break;
      case 4: e.name = r.binary(); break;
      case 5: e.num_children = int(r.zigzag()); break;
      default: r.skip(t);
    }
  }
  r.struct_end();
}

static void parse_statistics(TReader& r, ColumnMeta& m) {
  r.struct_begin();
  int16_t id; uint8_t t;
  while (r.field(id, t)) {
    if (id == 3) m.null_count = r.zigzag();
    else r.skip(t);
  }
  r.struct_end();
}

static void parse_column_meta(TReader& r, ColumnMeta& m) {
  r.struct_begin();
  int16_t id; uint8_t t;
  while (r.field(id, t)) {
    switch (id) {
      case 1: m.type = int(r.zigzag()); break;
      case 3: {
        uint8_t et; uint32_t n;
        r.list_begin(et, n);
        for (uint32_t i = 0; i < n; i++) m.path.push_back(r.binary());
        break;
      }
      case 4: m.codec = int(r.zigzag()); break;
      case 5: m.num_values = r.zigzag(); break;
      case 6: m.total_uncompressed = r.zigzag(); break;
      case 7: m.total_compressed = r.zigzag(); break;
      case 9: m.data_page_offset = r.zigzag(); break;
      case 11: m.dictionary_page_offset = r.zigzag(); break;
      case 12: parse_statistics(r, m); break;
      default: r.skip(t);
    }
  }
  r.struct_end();
}

static void parse_column_chunk(TReader& r, ColumnMeta& m) {
  r.struct_begin();
  int16_t id; uint8_t t;
  bool have_meta = false;
  while (r.field(id, t)) {
    if (id == 3) { parse_column_meta(r, m); have_meta = true; }
    else if (id == 1) { r.binary(); throw std::runtime_error("parquet: external column chunks are not supported"); }
    else r.skip(t);
  }
  r.struct_end();
  if (!have_meta) throw std::runtime_error("parquet: column chunk without meta_data");
}

static void parse_row_group(TReader& r, RowGroupMeta& g) {
  r.struct_begin();
  int16_t id; uint8_t t;
  while (r.field(id, t)) {
    if (id == 1) {
      uint8_t et; uint32_t n;
      r.list_begin(et, n);
      g.columns.resize(n);
      for (uint32_t i = 0; i < n; i++) parse_column_chunk(r, g.columns[i]);
    } else if (id == 3) {
      g.num_rows = r.zigzag();
    } else {
      r.skip(t);
    }
  }
  r.struct_end();
}

FileMeta parse_footer(const uint8_t* file, size_t size) {
  if (size < 12 || memcmp(file, "PAR1", 4) != 0 || memcmp(file + size - 4, "PAR1", 4) != 0)
    throw std::runtime_error("parquet: missing PAR1 magic");
  uint32_t flen;
  memcpy(&flen, file + size - 8, 4);
  if (size_t(flen) + 12 > size) throw std::runtime_error("parquet: bad footer length");
  TReader r(file + size - 8 - flen, flen);
  FileMeta fm;
  r.struct_begin();
  int16_t id; uint8_t t;
  while (r.field(id, t)) {
    switch (id) {
      case 2: {
        uint8_t et; uint32_t n;
        r.list_begin(et, n);
        fm.schema.resize(n);
        for (uint32_t i = 0; i < n; i++) parse_schema_element(r, fm.schema[i]);
        break;
      }
      case 3: fm.num_rows = r.zigzag(); break;
      case 4: {
        uint8_t et; uint32_t n;
        r.list_begin(et, n);
        fm.row_groups.resize(n);
        for (uint32_t i = 0; i < n; i++) parse_row_group(r, fm.row_groups[i]);
        break;
      }
      default: r.skip(t);
    }
  }
  r.struct_end();
  return fm;
}

static void parse_data_page_header(TReader& r, PageHeader& h) {
  r.struct_begin();
  int16_t id; uint8_t t;
  while (r.field(id, t)) {
    switch (id) {
      case 1: h.num_values = int32_t(r.zigzag()); break;
      case 2: h.encoding = int(r.zigzag()); break;
      case 3: h.def_encoding = int(r.zigzag()); break;
      default: r.skip(t);
    }
  }
  r.struct_end();
}

static void parse_data_page_header_v2(TReader& r, PageHeader& h) {
  r.struct_begin();
  int16_t id; uint8_t t;
  while (r.field(id, t)) {
    switch (id) {
      case 1: h.num_values = int32_t(r.zigzag()); break;
      case 2: h.num_nulls = int32_t(r.zigzag()); break;
      case 3: h.num_rows = int32_t(r.zigzag()); break;
      case 4: h.encoding = int(r.zigzag()); break;
      case 5: h.def_len = int32_t(r.zigzag()); break;
      case 6: h.rep_len = int32_t(r.zigzag()); break;
      case 7: h.v2_compressed = r.bool_val(t); break;
      default: r.skip(t);
    }
  }
  r.struct_end();
}

static void parse_dictionary_page_header(TReader& r, PageHeader& h) {
  r.struct_begin();
  int16_t id; uint8_t t;
  while (r.field(id, t)) {
    if (id == 1) h.dict_num_values = int32_t(r.zigzag());
    else if (id == 2) h.encoding = int(r.zigzag());
    else r.skip(t);
  }
  r.struct_end();
}

PageHeader parse_page_header(const uint8_t* p, size_t n) {
  TReader r(p, n);
  PageHeader h;
  r.struct_begin();
  int16_t id; uint8_t t;
  while (r.field(id, t)) {
    switch (id) {
      case 1: h.type = int(r.zigzag()); break;
      case 2: h.uncompressed = int32_t(r.zigzag()); break;
      case 3: h.compressed = int32_t(r.zigzag()); break;
      case 5: parse_data_page_header(r, h); break;
      case 7: parse_dictionary_page_header(r, h); break;
      case 8: parse_data_page_header_v2(r, h); break;
      default: r.skip(t);
    }
  }
  r.struct_end();
  h.header_len = r.consumed();
  return h;
}

static inline uint64_t read_varint(const uint8_t*& p, const uint8_t* end) {
  uint64_t v = 0;
  for (int s = 0; s < 64; s += 7) {
    if (p >= end) throw std::runtime_error("parquet: truncated hybrid run header");
    uint8_t b = *p++;
    v |= uint64_t(b & 0x7f) << s;
    if (!(b & 0x80)) return v;
  }
  throw std::runtime_error("parquet: bad varint");
}

std::vector<HRun> hybrid_runs(const uint8_t* p, size_t len, int bw, uint32_t nvalues) {
  std::vector<HRun> runs;
  const uint8_t* s = p;
  const uint8_t* end = p + len;
  uint32_t v = 0;
  const int vbytes = (bw + 7) / 8;
  while (v < nvalues) {
    uint64_t h = read_varint(s, end);
    HRun r{};
    r.start = v;
    if (h & 1) {
      uint64_t groups = h >> 1;
      uint64_t bytes = groups * uint64_t(bw);
      if (uint64_t(end - s) < bytes) throw std::runtime_error("parquet: truncated bit-packed run");
      uint64_t cnt = groups * 8;
      if (cnt == 0) continue;
      r.literal = true;
      r.off = uint32_t(s - p);
      r.count = uint32_t(std::min<uint64_t>(cnt, nvalues - v));
      s += bytes;
    } else {
      uint64_t cnt = h >> 1;
      if (end - s < vbytes) throw std::runtime_error("parquet: truncated RLE run");
      uint32_t val = 0;
      for (int i = 0; i < vbytes; i++) val |= uint32_t(s[i]) << (8 * i);
      s += vbytes;
      if (cnt == 0) continue;
      r.literal = false;
      r.value = val;
      r.count = uint32_t(std::min<uint64_t>(cnt, nvalues - v));
    }
    v += r.count;
    runs.push_back(r);
  }
  return runs;
}

// The i-th bw-bit value of a bit-packed group stream (LSB first) of `avail` bytes: one unaligned 8-byte load where
// it fits, else byte by byte at the stream's end.
static inline uint32_t unpack_at(const uint8_t* d, size_t avail, int bw, uint64_t mask, uint64_t i) {
  const uint64_t bit = i * uint64_t(bw);
  const size_t b0 = size_t(bit >> 3);
  uint64_t w = 0;
  if (b0 + 8 <= avail) {
    memcpy(&w, d + b0, 8);
  } else {
    for (size_t k = 0; k < 8 && b0 + k < avail; k++) w |= uint64_t(d[b0 + k]) << (8 * k);
  }
  return uint32_t((w >> (bit & 7)) & mask);
}

void hybrid_decode(const uint8_t* p, size_t len, int bw, uint32_t nvalues, uint32_t* out) {
  auto runs = hybrid_runs(p, len, bw, nvalues);
  const uint64_t mask = bw >= 32 ? 0xffffffffull : ((1ull << bw) - 1);
  for (const auto& r : runs) {
    if (!r.literal) {
      for (uint32_t i = 0; i < r.count; i++) out[r.start + i] = r.value;
    } else {
      for (uint32_t i = 0; i < r.count; i++) out[r.start + i] = unpack_at(p + r.off, len - r.off, bw, mask, i);
    }
  }
}

uint32_t hybrid_literal_max(const uint8_t* d, size_t avail, int bw, uint32_t count) {
  const uint64_t mask = bw >= 32 ? 0xffffffffull : ((1ull << bw) - 1);
  uint32_t mx = 0;
  for (uint32_t i = 0; i < count; i++) mx = std::max(mx, unpack_at(d, avail, bw, mask, i));
  return mx;
}


// ---- value encodings materialized at load (parquet-format Encodings.md) ----
namespace {
struct Reader {
  const uint8_t* p;
  const uint8_t* end;
  uint64_t uleb() {
    uint64_t v = 0;
    for (int sh = 0; sh < 64; sh += 7) {
      if (p >= end) throw std::runtime_error("parquet: truncated DELTA header");
      const uint8_t b = *p++;
      v |= uint64_t(b & 0x7f) << sh;
      if (!(b & 0x80)) return v;
    }
    throw std::runtime_error("parquet: bad varint in a DELTA stream");
  }
  int64_t zigzag() {
    const uint64_t u = uleb();
    return int64_t(u >> 1) ^ -int64_t(u & 1);
  }
};
}  // namespace

size_t delta_binary_decode(const uint8_t* p, size_t len, size_t n, int bits, int64_t* out) {
  Reader r{p, p + len};
  const uint64_t block = r.uleb(), nmini = r.uleb(), total = r.uleb();
  int64_t prev = r.zigzag();
  if (block == 0 || block % 128 || nmini == 0 || block % nmini || (block / nmini) % 32)
    throw std::runtime_error("parquet: bad DELTA_BINARY_PACKED block layout");
  if (total < n) throw std::runtime_error("parquet: DELTA_BINARY_PACKED page holds fewer values than its rows");
  const uint64_t per_mini = block / nmini;
  const uint64_t mask = bits == 32 ? 0xffffffffull : ~0ull;
  auto wrap = [&](uint64_t v) -> int64_t {   // the column's width: INT32 sign-extends its low 32 bits
    return bits == 32 ? int64_t(int32_t(uint32_t(v & mask))) : int64_t(v);
  };
  size_t i = 0;
  if (n) out[i++] = wrap(uint64_t(prev));
  while (i < n) {
    const uint64_t min_delta = uint64_t(r.zigzag());
    if (uint64_t(r.end - r.p) < nmini) throw std::runtime_error("parquet: truncated DELTA_BINARY_PACKED block");
    const uint8_t* widths = r.p;
    r.p += nmini;
    for (uint64_t m = 0; m < nmini && i < n; m++) {
      const int w = widths[m];
      if (w > 64) throw std::runtime_error("parquet: bad DELTA_BINARY_PACKED bit width");
      const uint64_t bytes = per_mini * uint64_t(w) / 8;
      if (uint64_t(r.end - r.p) < bytes) throw std::runtime_error("parquet: truncated DELTA_BINARY_PACKED miniblock");
      const uint8_t* d = r.p;
      for (uint64_t k = 0; k < per_mini && i < n; k++) {
        uint64_t v = 0;
        if (w) {   // LSB-first, bit k * w .. k * w + w - 1
          const uint64_t bit = k * uint64_t(w);
          unsigned __int128 acc = 0;
          const uint64_t b0 = bit >> 3, nb = (uint64_t(bit & 7) + uint64_t(w) + 7) / 8;
          for (uint64_t j = 0; j < nb; j++) acc |= (unsigned __int128)d[b0 + j] << (8 * j);
          v = uint64_t(acc >> (bit & 7));
          if (w < 64) v &= (uint64_t(1) << w) - 1;
        }
        prev = int64_t(uint64_t(prev) + min_delta + v);   // two's-complement wrap, then the column's width
        prev = wrap(uint64_t(prev));
        out[i++] = prev;
      }
      r.p += bytes;
    }
  }
  return size_t(r.p - p);
}

size_t delta_length_decode(const uint8_t* p, size_t len, size_t n, std::vector<ByteView>& views) {
  std::vector<int64_t> lens(n);
  size_t pos = n ? delta_binary_decode(p, len, n, 32, lens.data()) : 0;
  if (!n) {   // an empty page still carries a (value-less) header
    Reader r{p, p + len};
    if (len) {
      r.uleb(), r.uleb(), r.uleb(), r.zigzag();
      pos = size_t(r.p - p);
    }
  }
  views.clear();
  views.reserve(n);
  for (size_t i = 0; i < n; i++) {
    if (lens[i] < 0 || uint64_t(lens[i]) > len - pos) throw std::runtime_error("parquet: truncated DELTA_LENGTH_BYTE_ARRAY");
    views.push_back(ByteView{p + pos, uint32_t(lens[i])});
    pos += size_t(lens[i]);
  }
  return pos;
}

void delta_byte_array_decode(const uint8_t* p, size_t len, size_t n, std::vector<uint8_t>& store,
                             std::vector<ByteView>& views) {
  std::vector<int64_t> pre(n);
  const size_t used = n ? delta_binary_decode(p, len, n, 32, pre.data()) : 0;
  std::vector<ByteView> suf;
  delta_length_decode(p + used, len - used, n, suf);
  size_t total = 0, last = 0;
  for (size_t i = 0; i < n; i++) {
    if (pre[i] < 0 || uint64_t(pre[i]) > last) throw std::runtime_error("parquet: bad DELTA_BYTE_ARRAY prefix length");
    last = size_t(pre[i]) + suf[i].len;
    total += last;
  }
  store.clear();
  store.reserve(total);
  views.clear();
  views.reserve(n);
  for (size_t i = 0; i < n; i++) {   // (reserved: no reallocation, so earlier views stay valid)
    const size_t at = store.size(), pl = size_t(pre[i]);   // pre[0] == 0 (checked above)
    store.resize(at + pl + suf[i].len);
    if (pl) memcpy(store.data() + at, views[i - 1].p, pl);
    if (suf[i].len) memcpy(store.data() + at + pl, suf[i].p, suf[i].len);
    views.push_back(ByteView{store.data() + at, uint32_t(pl + suf[i].len)});
  }
}

void byte_stream_split_decode(const uint8_t* p, size_t len, size_t n, size_t width, uint8_t* out) {
  if (len < n * width) throw std::runtime_error("parquet: truncated BYTE_STREAM_SPLIT page");
  for (size_t k = 0; k < width; k++) {
    const uint8_t* s = p + k * n;
    for (size_t i = 0; i < n; i++) out[i * width + k] = s[i];
  }
}

}  // namespace pq
}  // namespace lk
