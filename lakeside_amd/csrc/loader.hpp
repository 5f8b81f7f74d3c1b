// Parquet segment loader, host part (no HIP): footer and schema walk, every column chunk's pages walked on its own
// thread (decompression, PLAIN string pages re-encoded, numeric dictionaries materialized, run tables, index
// validation), string dictionaries interned into the engine dictionaries per column in row-group order, tiles and
// zone maps per row group -- and the byte plan that stages the page streams for upload.  engine.cpp uploads the
// result (Engine::build_segment); tools/load_check.cpp runs it alone under the sanitizers (`make sanitize`).
#pragma once
#include <cstddef>
#include <cstdint>
#include <functional>
#include <memory>
#include <string>
#include <string_view>
#include <vector>

#include "layout.hpp"
#include "segment.hpp"

namespace lk {

struct HostPage {
  PageDesc d{};
  uint32_t rg = 0;
  uint32_t run_lo = 0, run_n = 0, drun_lo = 0, drun_n = 0;
  std::vector<uint32_t> vprefix;   // nullable pages with NULLs: non-null rows before row i (size nrows+1)
  const uint8_t* host_vals = nullptr;
};

// A byte range of one page stream: copied from `src` (the file, or a decompressed / re-encoded page buffer) to `off`
// in its chunk's stream area.
struct StreamRef {
  const uint8_t* src;
  size_t len;
  size_t off;
};

// One column chunk (column, row group) walked on the host: page descriptors, run tables and the byte ranges of its
// page streams.  Chunks are independent, so the walk runs on several threads (Engine::load_threads); string
// dictionary values are interned into the engine dictionaries afterwards, per column in row-group order, so the
// engine-global ids do not depend on thread timing.
struct ChunkOut {
  std::vector<StreamRef> streams;
  size_t bytes = 0;                       // the chunk's stream area (every stream 128-B aligned: one HBM line start)
  std::vector<HostPage> pages;            // d.vals / d.defs: offsets in the chunk's area; run_lo / drun_lo: indices into
                                          // `runs`; d.remap: index into `dict`
  std::vector<RunDesc> runs;
  // strings: the dictionary page's values, then every PLAIN page's own values -- views into the file bytes or `plain`
  // (both outlive the load), so a 10M-value dictionary is not copied string by string before interning
  std::vector<std::string_view> dict;
  // decompressed / re-encoded pages (streams, zone maps and dictionary views point into them): heap-held so the
  // buffers stay put when the ChunkOut moves
  std::vector<std::unique_ptr<std::vector<uint8_t>>> plain;
  uint64_t compressed = 0;
  int code = 0;                           // LK_ERR_IO: the file is corrupt; LK_ERR_UNSUPPORTED: this column's shape
  std::string msg;
  size_t put(const uint8_t* p, size_t n) {
    const size_t off = (bytes + 127) / 128 * 128;
    if (n) streams.push_back(StreamRef{p, n, off});
    bytes = off + n;
    return off;
  }
};

// The loader's output: the segment's host part, the chunks whose streams are still to be staged (their buffers and
// the file bytes must outlive the staging), and each chunk's offset in the stream area.
struct HostLoad {
  SegmentData seg;
  std::vector<ChunkOut> chunks;
  std::vector<size_t> chunk_base;
  double host_ms = 0;
};

// Steps 1-3 of a segment load on up to `threads` threads; `dict(column)` is the engine dictionary strings intern into.
HostLoad load_host(const std::string& key, const uint8_t* F, size_t size, int threads,
                   const std::function<GlobalDict&(const std::string&)>& dict);

// The stream area's bytes in destination order: stage(dst, lo, hi) writes bytes [lo, hi) of it into dst (the page
// streams, alignment gaps zeroed, so reads past a stream's end see zeros), in ~8 MB pieces on up to `threads` threads.
class StagePlan {
 public:
  explicit StagePlan(const HostLoad& H);
  void stage(uint8_t* dst, size_t lo, size_t hi, int threads);

 private:
  struct Copy {
    const uint8_t* src;
    size_t len;
    size_t dst;
  };
  std::vector<Copy> copies_;   // sorted by destination
  size_t next_ = 0;            // first copy not wholly below the last piece staged
};

}  // namespace lk
