// Parquet segment loader, host part: see loader.hpp.  Moved out of engine.cpp so it builds and runs without HIP
// (tools/load_check.cpp under ASan / UBSan / TSan, `make sanitize`).
#include "loader.hpp"

#include <cmath>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <climits>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <string_view>
#include <thread>
#include <unordered_map>
#include <vector>

#include "../../include/lakeside_gpu.h"
#include "codec.hpp"
#include "parquet.hpp"
#include "plan.hpp"

namespace lk {

static constexpr size_t kAlign = 256;
static inline size_t align_up(size_t x, size_t a = kAlign) { return (x + a - 1) / a * a; }

// ------------------------------------------------------------------------------------------------
// engine-global dictionaries: one per column name; chunk dictionaries remap into them at load
// ------------------------------------------------------------------------------------------------
uint32_t GlobalDict::intern(std::string_view s) {
  const uint64_t h = IdMap::hash(s);
  const uint32_t f = ids.find_h(s, h);
  if (f != IdMap::kNone) return f;
  const uint32_t id = uint32_t(vals->size());
  vals->push_back(std::string(s));
  refs.push_back(0);
  ids.emplace_h(id, h);
  return id;
}

// Parallel interning with the sequential result (a 10M-value dictionary interned one value at a
// time ran C5 ingest at 0.41 GB/s): known values are looked up in parallel (reads only); the unknown ones are
// partitioned by hash shard with their positions in order, each shard finds its values' first occurrences on its own,
// a prefix count over the first occurrences in position order gives them the ids the one-by-one walk would give, the
// strings are stored and the repeats take their first occurrence's id, and every shard indexes its new values.
void GlobalDict::intern_all(const std::vector<std::string_view>& v, uint32_t* out, int threads) {
  const size_t n = v.size();
  if (n < (size_t(1) << 16) || threads <= 1) {
    for (size_t i = 0; i < n; i++) out[i] = intern(v[i]);
    return;
  }
  static const bool timing = getenv("LK_LOAD_TIMING") != nullptr;
  const auto t0 = std::chrono::steady_clock::now();
  auto mark = [&](const char* w) {
    if (timing) fprintf(stderr, "[lk intern] %-8s %8.1f ms (%zu values)\n", w, std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count(), n);
  };
  constexpr size_t K = IdMap::kShards;
  const size_t B = std::min<size_t>(size_t(threads) * 8, (n + 4095) / 4096), bs = (n + B - 1) / B;
  if (sc_hash.size() < n) sc_hash.resize(n);
  if (sc_first.size() < n) sc_first.resize(n);
  uint64_t* const h = sc_hash.data();
  uint32_t* const first = sc_first.data();   // unknown positions: the first position of the same value
  parallel_for(B, threads, [&](size_t b) {
    const size_t lo = b * bs, hi = std::min(n, (b + 1) * bs);
    std::fill(first + lo, first + hi, UINT32_MAX);
    constexpr size_t D = 16;   // lookups in flight: slot lines prefetched D values ahead (each lookup is a cache miss)
    for (size_t i = lo; i < std::min(hi, lo + D); i++) {
      h[i] = IdMap::hash(v[i]);
      ids.prefetch(h[i]);
    }
    for (size_t i = lo; i < hi; i++) {
      if (i + D < hi) {
        h[i + D] = IdMap::hash(v[i + D]);
        ids.prefetch(h[i + D]);
      }
      if (i + D / 2 < hi) ids.prefetch_str(h[i + D / 2]);   // its slot arrived: the string it points at next
      out[i] = ids.find_h(v[i], h[i]);   // kNone (UINT32_MAX) when unknown
    }
  });
  mark("lookup");
  std::vector<std::vector<uint32_t>> lists(B * K);   // [block][shard]: positions of unknown values, ascending
  parallel_for(B, threads, [&](size_t b) {
    for (size_t i = b * bs; i < std::min(n, (b + 1) * bs); i++)
      if (out[i] == UINT32_MAX) lists[b * K + IdMap::shard_of(h[i])].push_back(uint32_t(i));
  });
  mark("lists");
  parallel_for(K, threads, [&](size_t k) {
    // open addressing over this shard's positions (slot: hash tag | position), walked in position order
    size_t m = 0;
    for (size_t b = 0; b < B; b++) m += lists[b * K + k].size();
    size_t cap = 64;
    while (cap * 7 < m * 10) cap <<= 1;
    std::vector<uint64_t> tab(cap, 0);
    const size_t mask = cap - 1;
    for (size_t b = 0; b < B; b++)
      for (uint32_t i : lists[b * K + k]) {
        const uint64_t tag = ((h[i] >> 32) & 0x7fffffffull) | 0x80000000ull;
        for (size_t j = size_t(h[i] >> 6) & mask;; j = (j + 1) & mask) {
          const uint64_t x = tab[j];
          if (!x) {
            tab[j] = (tag << 32) | i;
            first[i] = i;
            break;
          }
          if ((x >> 32) == tag && v[uint32_t(x)] == v[i]) {
            first[i] = uint32_t(x);
            break;
          }
        }
      }
  });
  mark("dedup");
  std::vector<size_t> base(B + 1, 0);
  parallel_for(B, threads, [&](size_t b) {
    size_t c = 0;
    for (size_t i = b * bs; i < std::min(n, (b + 1) * bs); i++) c += out[i] == UINT32_MAX && first[i] == i;
    base[b + 1] = c;
  });
  for (size_t b = 0; b < B; b++) base[b + 1] += base[b];
  mark("count");
  const size_t old = vals->size(), added = base[B];
  if (old + added > size_t(UINT32_MAX)) throw std::length_error("dictionary exceeds 2^32 values");
  vals->grow(old + added);
  refs.resize(old + added, 0);
  mark("grow");
  parallel_for(B, threads, [&](size_t b) {   // first occurrences: ids in position order, strings stored
    uint32_t id = uint32_t(old + base[b]);
    for (size_t i = b * bs; i < std::min(n, (b + 1) * bs); i++)
      if (out[i] == UINT32_MAX && first[i] == i) {
        vals->slot(id).assign(v[i].data(), v[i].size());
        out[i] = id++;
      }
  });
  mark("store");
  parallel_for(B, threads, [&](size_t b) {   // repeats (their first occurrence is final after the previous pass)
    for (size_t i = b * bs; i < std::min(n, (b + 1) * bs); i++)
      if (first[i] != UINT32_MAX && first[i] != i) out[i] = out[first[i]];
  });
  mark("repeats");
  parallel_for(K, threads, [&](size_t k) {   // index the new values, one thread per shard
    size_t nk = 0;
    for (size_t b = 0; b < B; b++)
      for (uint32_t i : lists[b * K + k]) nk += first[i] == i;
    ids.reserve_shard(k, nk);
    for (size_t b = 0; b < B; b++)
      for (uint32_t i : lists[b * K + k])
        if (first[i] == i) ids.emplace_h(out[i], h[i]);
  });
  mark("index");
}

int SegmentData::col_index(const std::string& name) const {
  auto it = by_name.find(name);
  return it == by_name.end() ? -1 : it->second;
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
      if (st.encoding == pq::PLAIN || st.encoding == pq::DELTA_LENGTH_BYTE_ARRAY || st.encoding == pq::DELTA_BYTE_ARRAY) {
        // PLAIN BYTE_ARRAY page (a writer's dictionary fallback, or no dictionary at all), or its DELTA_LENGTH_BYTE_ARRAY
        // / DELTA_BYTE_ARRAY forms (decoded here; the rebuilt DELTA_BYTE_ARRAY values are held with the chunk): the
        // page gets its own dictionary -- its distinct values in first-seen order, interned with the chunk -- and its
        // values are re-encoded as one bit-packed literal run of indices, so the kernels see a dictionary page.
        std::vector<pq::ByteView> vals;
        if (st.encoding == pq::PLAIN) {
          vals.reserve(nvals);
          size_t p = 0;
          for (uint32_t i = 0; i < nvals; i++) {
            if (p + 4 > st.vals_len) throw PlanError(LK_ERR_IO, "parquet: truncated PLAIN BYTE_ARRAY page in " + col.name);
            uint32_t L;
            memcpy(&L, st.vals + p, 4);
            p += 4;
            if (p + L > st.vals_len) throw PlanError(LK_ERR_IO, "parquet: truncated PLAIN BYTE_ARRAY value in " + col.name);
            vals.push_back(pq::ByteView{st.vals + p, L});
            p += L;
          }
        } else if (st.encoding == pq::DELTA_LENGTH_BYTE_ARRAY) {
          pq::delta_length_decode(st.vals, st.vals_len, nvals, vals);
        } else {
          C.plain.push_back(std::make_unique<std::vector<uint8_t>>());
          pq::delta_byte_array_decode(st.vals, st.vals_len, nvals, *C.plain.back(), vals);
        }
        std::unordered_map<std::string_view, uint32_t> local;
        std::vector<uint32_t> idx(nvals);
        page_remap = uint32_t(C.dict.size());
        for (uint32_t i = 0; i < nvals; i++) {
          auto ins = local.emplace(std::string_view(reinterpret_cast<const char*>(vals[i].p), vals[i].len),
                                   uint32_t(local.size()));
          if (ins.second) C.dict.emplace_back(ins.first->first);
          idx[i] = ins.first->second;
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
      } else if (st.encoding == pq::DELTA_BINARY_PACKED && (col.ptype == pq::INT32 || col.ptype == pq::INT64)) {
        // DELTA_BINARY_PACKED integers (e.g. a writer's sorted timestamps): materialized to PLAIN here
        std::vector<int64_t> v(nvals);
        pq::delta_binary_decode(st.vals, st.vals_len, nvals, col.ptype == pq::INT32 ? 32 : 64, v.data());
        C.plain.push_back(std::make_unique<std::vector<uint8_t>>(size_t(nvals) * width));
        std::vector<uint8_t>& out = *C.plain.back();
        for (uint32_t i = 0; i < nvals; i++) {
          if (width == 8) {
            memcpy(out.data() + size_t(i) * 8, &v[i], 8);
          } else {
            const int32_t x = int32_t(v[i]);
            memcpy(out.data() + size_t(i) * 4, &x, 4);
          }
        }
        st.vals = out.data();
        st.vals_len = out.size();
      } else if (st.encoding == pq::BYTE_STREAM_SPLIT && width) {
        // BYTE_STREAM_SPLIT (FLOAT / DOUBLE, and INT32 / INT64 in format 2.11): the byte streams interleaved back
        C.plain.push_back(std::make_unique<std::vector<uint8_t>>(size_t(nvals) * width));
        pq::byte_stream_split_decode(st.vals, st.vals_len, nvals, width, C.plain.back()->data());
        st.vals = C.plain.back()->data();
        st.vals_len = C.plain.back()->size();
      } else if (st.encoding == pq::RLE && width == 0) {
        // RLE BOOLEAN values (data page v2 writers): a 4-byte length, then the hybrid stream at bit width 1 -> the
        // PLAIN bit-packed layout (LSB first)
        if (st.vals_len < 4) throw PlanError(LK_ERR_IO, "parquet: truncated RLE BOOLEAN page in " + col.name);
        uint32_t L;
        memcpy(&L, st.vals, 4);
        if (size_t(L) + 4 > st.vals_len) throw PlanError(LK_ERR_IO, "parquet: bad RLE BOOLEAN length in " + col.name);
        std::vector<uint32_t> b(nvals);
        pq::hybrid_decode(st.vals + 4, L, 1, nvals, b.data());
        C.plain.push_back(std::make_unique<std::vector<uint8_t>>((size_t(nvals) + 7) / 8, 0));
        std::vector<uint8_t>& out = *C.plain.back();
        for (uint32_t i = 0; i < nvals; i++)
          if (b[i]) out[i >> 3] |= uint8_t(1u << (i & 7));
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
void build_tiles_rg(const SegmentData& S, const std::vector<std::vector<HostPage>>& pages, uint32_t rg,
                    const std::vector<size_t>& page0, std::vector<TileDesc>& tiles, std::vector<std::vector<TileCol>>& tcols,
                    std::vector<double>& imax) {
  const int nc = int(S.cols.size());
  const int ts_col = S.col_index(kTimestamp);
  std::vector<size_t> cursor(page0);
  const uint32_t nrows = uint32_t(S.rg_rows[rg]);
  tcols.assign(size_t(nc), {});
  imax.assign(size_t(nc), 0.0);   // HostCol::int_abs_max over this row group
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
      const int pt = S.cols[size_t(c)].ptype;
      if (c != ts_col && imax[size_t(c)] >= 0.0) {   // integral-value summary (a tile's values: indices [va, ve))
        if (p.d.kind != PAGE_PLAIN64 || (pt != pq::DOUBLE && pt != pq::INT64)) {
          imax[size_t(c)] = -1.0;
        } else {
          bool integral = true;
          double m = imax[size_t(c)];
          for (uint32_t i = va; i < ve; i++) {
            double x;
            if (pt == pq::DOUBLE) {
              memcpy(&x, p.host_vals + size_t(i) * 8, 8);
              integral &= x == std::trunc(x);   // NaN fails; +-inf fails the bound below
            } else {
              int64_t y;
              memcpy(&y, p.host_vals + size_t(i) * 8, 8);
              x = double(y);
            }
            m = std::max(m, std::fabs(x));
          }
          imax[size_t(c)] = integral ? m : -1.0;
        }
      }
      if (c == ts_col && p.d.kind == PAGE_PLAIN64 && !S.cols[size_t(c)].is_string) {
        const int64_t* v = reinterpret_cast<const int64_t*>(p.host_vals);   // (host_vals: 8-B PLAIN values)
        int64_t lo = INT64_MAX, hi = INT64_MIN, prev = INT64_MIN;
        bool sorted = true;
        for (uint32_t i = va; i < ve; i++) {
          int64_t x;
          memcpy(&x, v + i, 8);
          lo = std::min(lo, x);
          hi = std::max(hi, x);
          sorted &= x >= prev;
          prev = x;
        }
        t.ts_min = lo;
        t.ts_max = hi;
        // every row has a timestamp and they never decrease: a query's bucket boundaries inside the tile can be found
        // by searching the timestamps (scan_lean's split tiles)
        if (sorted && ve - va == e - a && !p.d.has_nulls) t.pad |= TILE_TS_SORTED;
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

}  // namespace


// Physical types the engine loads: BYTE_ARRAY strings, INT64 / DOUBLE (the scan's timestamp and value columns), and
// INT32 / FLOAT / BOOLEAN (read by exemplar rows).  INT96 / FIXED_LEN_BYTE_ARRAY are not loaded.
static bool loadable_type(int ptype) {
  return ptype == pq::BYTE_ARRAY || ptype == pq::INT64 || ptype == pq::DOUBLE || ptype == pq::INT32 ||
         ptype == pq::FLOAT || ptype == pq::BOOLEAN;
}

// Parquet bytes -> a segment's host part.  Footer, schema walk, then every column chunk walked on its own thread
// (pages, run tables, decompression, index validation), string dictionaries interned per column in row-group order,
// tiles built per row group in parallel.
// A column the engine cannot decode (nested / repeated, INT96 / FIXED_LEN_BYTE_ARRAY, a page encoding or codec
// outside the implemented set) is left unloaded with its reason (SegmentData::unloaded): the segment still serves every
// query that does not reference it, and a query that does fails with LK_ERR_UNSUPPORTED -- a capability gap, not an
// empty glob.  A corrupt file is LK_ERR_IO.
HostLoad load_host(const std::string& key, const uint8_t* F, size_t size, int threads,
                   const std::function<GlobalDict&(const std::string&)>& dict) {
  const auto t0 = std::chrono::steady_clock::now();
  HostLoad H;
  SegmentData* S = &H.seg;
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

  static const bool timing = getenv("LK_LOAD_TIMING") != nullptr;   // diagnostics: stage times on stderr
  auto mark = [&](const char* what) {
    if (timing)
      fprintf(stderr, "[lk load] %-8s %9.1f ms  %s\n", what,
              std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count(), key.c_str());
  };
  mark("footer");
  // ---- 1. every (column, row group) chunk walked in parallel ----
  const size_t ncol = S->cols.size();
  std::vector<int> leaf_of(ncol);
  for (size_t l = 0; l < leaf_col.size(); l++)
    if (leaf_col[l] >= 0) leaf_of[size_t(leaf_col[l])] = int(l);
  std::vector<ChunkOut>& chunks = H.chunks;
  chunks.resize(ncol * nrg);   // [column][row group]
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

  mark("walk");
  // ---- 2. per column, in row-group order: intern dictionaries, concatenate runs and pages, place streams ----
  // Byte offset of each chunk's stream area in the segment: row-group major (a row group's columns side by side, as
  // in the file), so the streams one tile reads lie close together (column-major placement measured ~1.8x slower
  // scans; LK_COLMAJOR=1 keeps it for A/B).
  std::vector<size_t>& chunk_base = H.chunk_base;
  chunk_base.assign(chunks.size(), 0);
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
  // A column's chunk dictionaries, in row-group order, through its engine dictionary (GlobalDict::intern_all: the ids
  // are those of interning the values one by one, whatever the thread count).  Large dictionaries (a 10M-value group
  // column) first, one column at a time with every load thread; then the other columns one thread each -- no nested
  // parallel_for, so a load never runs more than `threads` threads.
  auto intern_column = [&](size_t ci, int t) {
    HostCol& col = S->cols[ci];
    GlobalDict& gd = dict(col.name);
    std::lock_guard<std::mutex> g(gd.mu);
    std::vector<std::string_view>& sv = gd.sc_views;   // (reused across loads)
    std::vector<size_t> at(nrg + 1, 0);
    for (size_t rg = 0; rg < nrg; rg++) at[rg + 1] = at[rg] + chunks[ci * nrg + rg].dict.size();
    sv.resize(at[nrg]);
    parallel_for(nrg, t, [&](size_t rg) {   // the row groups' chunk dictionaries side by side (16M views: C5)
      const auto& d = chunks[ci * nrg + rg].dict;
      std::copy(d.begin(), d.end(), sv.begin() + std::ptrdiff_t(at[rg]));
    });
    col.remap.resize(sv.size());
    if (t > 1) mark("  views");
    gd.intern_all(sv, col.remap.data(), t);
    if (t <= 1 || sv.size() < (size_t(1) << 16)) std::vector<std::string_view>().swap(sv);   // small: not kept
    if (t > 1) mark("  interned");
  };
  mark("layout");
  std::vector<char> big(nc, 0);
  for (size_t ci = 0; ci < nc; ci++) {
    size_t ndict = 0;
    for (size_t rg = 0; rg < nrg; rg++) ndict += chunks[ci * nrg + rg].dict.size();
    if (S->cols[ci].is_string && ndict >= (size_t(1) << 16) && threads > 1) {
      big[ci] = 1;
      intern_column(ci, threads);
    }
  }
  mark("intern");
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
    if (col.is_string && ndict && !big[ci]) intern_column(ci, 1);
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

  mark("concat");
  // ---- 3. tiles, per row group in parallel ----
  std::vector<std::vector<TileDesc>> rg_tiles(nrg);
  std::vector<std::vector<std::vector<TileCol>>> rg_tcols(nrg);
  std::vector<std::vector<double>> rg_imax(nrg);
  if (S->num_rows > 0 && nc) {
    parallel_for(nrg, threads, [&](size_t rg) {
      std::vector<size_t> p0(nc);
      for (size_t c = 0; c < nc; c++) p0[c] = page0[c][rg];
      build_tiles_rg(*S, pages, uint32_t(rg), p0, rg_tiles[rg], rg_tcols[rg], rg_imax[rg]);
    });
    for (size_t rg = 0; rg < nrg; rg++) {
      S->tiles.insert(S->tiles.end(), rg_tiles[rg].begin(), rg_tiles[rg].end());
      for (size_t c = 0; c < nc; c++)
        S->cols[c].tcols.insert(S->cols[c].tcols.end(), rg_tcols[rg][c].begin(), rg_tcols[rg][c].end());
    }
    for (size_t c = 0; c < nc; c++) {   // integral-value summary over the row groups (HostCol::int_abs_max)
      double m = 0.0;
      for (size_t rg = 0; rg < nrg && m >= 0.0; rg++) m = rg_imax[rg][c] < 0.0 ? -1.0 : std::max(m, rg_imax[rg][c]);
      S->cols[c].int_abs_max = S->cols[c].is_string ? -1.0 : m;
    }
  }
  for (size_t ci = 0; ci < nc; ci++) {
    auto& col = S->cols[ci];
    col.pages.reserve(pages[ci].size());
    for (auto& hp : pages[ci]) col.pages.push_back(hp.d);
  }
  mark("tiles");
  H.host_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  S->load_host_ms = H.host_ms;
  return H;
}

StagePlan::StagePlan(const HostLoad& H) {
  for (size_t k = 0; k < H.chunks.size(); k++)
    for (const StreamRef& r : H.chunks[k].streams) copies_.push_back(Copy{r.src, r.len, H.chunk_base[k] + r.off});
  std::sort(copies_.begin(), copies_.end(), [](const Copy& a, const Copy& b) { return a.dst < b.dst; });
}

void StagePlan::stage(uint8_t* dst, size_t lo, size_t hi, int threads) {
  // the copies overlapping [lo, hi), split into ~8 MB work items; the gaps between them are zeroed (src == nullptr)
  std::vector<Copy> work;
  while (next_ < copies_.size() && copies_[next_].dst + copies_[next_].len <= lo) next_++;
  size_t cur = lo;
  for (size_t c = next_; c < copies_.size() && copies_[c].dst < hi; c++) {
    const size_t a = std::max(lo, copies_[c].dst), b = std::min(hi, copies_[c].dst + copies_[c].len);
    if (a > cur) work.push_back(Copy{nullptr, a - cur, cur - lo});
    for (size_t x = a; x < b; x += size_t(8) << 20) {
      const size_t y = std::min(b, x + (size_t(8) << 20));
      work.push_back(Copy{copies_[c].src + (x - copies_[c].dst), y - x, x - lo});
    }
    cur = std::max(cur, b);
  }
  if (cur < hi) work.push_back(Copy{nullptr, hi - cur, cur - lo});
  parallel_for(work.size(), threads, [&](size_t w) {
    if (work[w].src) memcpy(dst + work[w].dst, work[w].src, work[w].len);
    else memset(dst + work[w].dst, 0, work[w].len);
  });
}

}  // namespace lk
