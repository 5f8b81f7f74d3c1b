// Test tool (tests/test_codec_cpu.py): walk every page of every column chunk of a Parquet file, decompress it
// with lakeside_amd/csrc/codec.cpp the way the segment loader does, and print one FNV-1a hash per column over
// the plain page payloads (v2: levels + values).  A compressed file and the same table written uncompressed
// must print the same hashes.
#include <cstdio>
#include <cstring>
#include <fstream>
#include <iterator>
#include <vector>

#include "codec.hpp"
#include "parquet.hpp"

using namespace lk;

int main(int argc, char** argv) {
  if (argc != 2) return 2;
  std::ifstream f(argv[1], std::ios::binary);
  std::vector<uint8_t> d((std::istreambuf_iterator<char>(f)), {});
  try {
    const pq::FileMeta fm = pq::parse_footer(d.data(), d.size());
    const size_t ncol = fm.row_groups.empty() ? 0 : fm.row_groups[0].columns.size();
    std::vector<uint64_t> hash(ncol, 1469598103934665603ull);
    for (const auto& rg : fm.row_groups)
      for (size_t c = 0; c < rg.columns.size(); c++) {
        const pq::ColumnMeta& m = rg.columns[c];
        size_t pos = size_t(m.dictionary_page_offset > 0 && m.dictionary_page_offset < m.data_page_offset
                                ? m.dictionary_page_offset : m.data_page_offset);
        int64_t seen = 0;
        while (seen < m.num_values) {
          const pq::PageHeader h = pq::parse_page_header(d.data() + pos, d.size() - pos);
          const uint8_t* p = d.data() + pos + h.header_len;
          pos += h.header_len + size_t(h.compressed);
          std::vector<uint8_t> out(size_t(h.compressed));
          memcpy(out.data(), p, out.size());
          if (m.codec != pq::CODEC_UNCOMPRESSED) {
            const size_t lv = h.type == pq::DATA_PAGE_V2 ? size_t(h.rep_len + h.def_len) : 0;
            out.assign(size_t(h.uncompressed), 0);
            memcpy(out.data(), p, lv);
            if (h.type != pq::DATA_PAGE_V2 || h.v2_compressed)
              pq::decompress(m.codec, p + lv, size_t(h.compressed) - lv, out.data() + lv, out.size() - lv);
            else
              memcpy(out.data() + lv, p + lv, size_t(h.compressed) - lv);
          }
          if (h.type == pq::DATA_PAGE || h.type == pq::DATA_PAGE_V2) seen += h.num_values;
          for (uint8_t b : out) hash[c] = (hash[c] ^ b) * 1099511628211ull;
        }
      }
    for (size_t c = 0; c < ncol; c++) printf("%016llx\n", (unsigned long long)hash[c]);
  } catch (const std::exception& e) {
    fprintf(stderr, "error: %s\n", e.what());
    return 1;
  }
  return 0;
}
