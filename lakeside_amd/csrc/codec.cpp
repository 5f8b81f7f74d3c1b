// Parquet page decompression at segment load (host): the HBM cache holds decompressed page streams, so the
// scan kernels are codec-agnostic.  SURVEY.md §8(f) f2: the production writer's codec is not in the reference
// repo, so every codec a Parquet writer commonly emits is accepted.
//
//   SNAPPY (1)  — decoded here (raw snappy block format, as Parquet stores it: no framing)
//   GZIP (2)    — zlib inflate, gzip or zlib header auto-detected
//   ZSTD (6)    — the system libzstd (runtime library only in this image: the two entry points are declared below)
//   LZ4_RAW (7) — the system liblz4 block decoder; LZ4 (5, deprecated): Hadoop framing, else one raw block
//   BROTLI (4)  — the system libbrotlidec one-shot decoder (r06)
// LZO (3) is rejected with LK_ERR_UNSUPPORTED.
#include "codec.hpp"

#include <zlib.h>

#include <cstring>
#include <string>

#include "../../include/lakeside_gpu.h"
#include "plan.hpp"

extern "C" {
// libzstd.so.1 / liblz4.so.1 (stable C ABIs; their headers are not installed in this image)
size_t ZSTD_decompress(void* dst, size_t dst_capacity, const void* src, size_t compressed_size);
unsigned ZSTD_isError(size_t code);
const char* ZSTD_getErrorName(size_t code);
int LZ4_decompress_safe(const char* src, char* dst, int compressed_size, int dst_capacity);
// libbrotlidec.so.1: BrotliDecoderResult BrotliDecoderDecompress(...); BROTLI_DECODER_RESULT_SUCCESS = 1
int BrotliDecoderDecompress(size_t encoded_size, const uint8_t* encoded_buffer, size_t* decoded_size,
                            uint8_t* decoded_buffer);
}

namespace lk {
namespace pq {

namespace {

[[noreturn]] void bad(const char* codec, const std::string& why) {
  throw PlanError(LK_ERR_IO, std::string("parquet: ") + codec + " page: " + why);
}

void snappy(const uint8_t* src, size_t n, uint8_t* dst, size_t cap) {
  size_t i = 0;
  uint64_t len = 0;
  for (int shift = 0;; shift += 7) {           // preamble: uncompressed length, varint
    if (i >= n || shift > 35) bad("SNAPPY", "bad length preamble");
    const uint8_t b = src[i++];
    len |= uint64_t(b & 0x7f) << shift;
    if (!(b & 0x80)) break;
  }
  if (len != cap) bad("SNAPPY", "length mismatch");
  size_t o = 0;
  while (i < n) {
    const uint8_t tag = src[i++];
    size_t l, off;
    if ((tag & 3) == 0) {                      // literal
      l = tag >> 2;
      if (l >= 60) {
        const size_t k = l - 59;               // 1..4 length bytes
        if (i + k > n) bad("SNAPPY", "truncated literal length");
        l = 0;
        for (size_t j = 0; j < k; j++) l |= size_t(src[i + j]) << (8 * j);
        i += k;
      }
      l += 1;
      if (i + l > n || o + l > cap) bad("SNAPPY", "literal out of bounds");
      memcpy(dst + o, src + i, l);
      i += l;
      o += l;
      continue;
    }
    if ((tag & 3) == 1) {                      // copy, 1-byte offset
      if (i + 1 > n) bad("SNAPPY", "truncated copy");
      l = ((tag >> 2) & 7) + 4;
      off = (size_t(tag >> 5) << 8) | src[i];
      i += 1;
    } else if ((tag & 3) == 2) {               // copy, 2-byte offset
      if (i + 2 > n) bad("SNAPPY", "truncated copy");
      l = (tag >> 2) + 1;
      off = size_t(src[i]) | (size_t(src[i + 1]) << 8);
      i += 2;
    } else {                                   // copy, 4-byte offset
      if (i + 4 > n) bad("SNAPPY", "truncated copy");
      l = (tag >> 2) + 1;
      off = size_t(src[i]) | (size_t(src[i + 1]) << 8) | (size_t(src[i + 2]) << 16) | (size_t(src[i + 3]) << 24);
      i += 4;
    }
    if (off == 0 || off > o || o + l > cap) bad("SNAPPY", "copy out of bounds");
    for (size_t j = 0; j < l; j++, o++) dst[o] = dst[o - off];   // byte order: overlapping copies repeat
  }
  if (o != cap) bad("SNAPPY", "short output");
}

void gzip(const uint8_t* src, size_t n, uint8_t* dst, size_t cap) {
  z_stream z{};
  if (inflateInit2(&z, 15 + 32) != Z_OK) bad("GZIP", "inflateInit2");
  z.next_in = const_cast<Bytef*>(src);
  z.avail_in = uInt(n);
  z.next_out = dst;
  z.avail_out = uInt(cap);
  const int rc = inflate(&z, Z_FINISH);
  const size_t out = z.total_out;
  inflateEnd(&z);
  if (rc != Z_STREAM_END || out != cap) bad("GZIP", "inflate failed");
}

}  // namespace

void decompress(int codec, const uint8_t* src, size_t n, uint8_t* dst, size_t cap) {
  uint8_t empty[1];
  if (!dst) dst = empty;   // an empty page (e.g. an all-NULL column's dictionary): zlib refuses a null output
  switch (codec) {
    case CODEC_SNAPPY: snappy(src, n, dst, cap); return;
    case CODEC_GZIP: gzip(src, n, dst, cap); return;
    case CODEC_ZSTD: {
      const size_t r = ZSTD_decompress(dst, cap, src, n);
      if (ZSTD_isError(r)) bad("ZSTD", ZSTD_getErrorName(r));
      if (r != cap) bad("ZSTD", "short output");
      return;
    }
    case CODEC_LZ4_RAW: {
      const int r = LZ4_decompress_safe(reinterpret_cast<const char*>(src), reinterpret_cast<char*>(dst), int(n),
                                        int(cap));
      if (r < 0 || size_t(r) != cap) bad("LZ4_RAW", "decode failed");
      return;
    }
    case CODEC_LZ4: {
      // deprecated LZ4: Hadoop framing (big-endian decompressed size, compressed size, block)*; writers that
      // emitted raw blocks under this id exist, so fall back to one raw block (as Arrow's reader does)
      size_t i = 0, o = 0;
      bool framed = true;
      while (i < n && framed) {
        if (i + 8 > n) { framed = false; break; }
        const size_t dl = (size_t(src[i]) << 24) | (size_t(src[i + 1]) << 16) | (size_t(src[i + 2]) << 8) | src[i + 3];
        const size_t cl = (size_t(src[i + 4]) << 24) | (size_t(src[i + 5]) << 16) | (size_t(src[i + 6]) << 8) | src[i + 7];
        if (i + 8 + cl > n || o + dl > cap) { framed = false; break; }
        const int r = LZ4_decompress_safe(reinterpret_cast<const char*>(src + i + 8), reinterpret_cast<char*>(dst + o),
                                          int(cl), int(dl));
        if (r < 0 || size_t(r) != dl) { framed = false; break; }
        i += 8 + cl;
        o += dl;
      }
      if (framed && o == cap) return;
      const int r = LZ4_decompress_safe(reinterpret_cast<const char*>(src), reinterpret_cast<char*>(dst), int(n),
                                        int(cap));
      if (r < 0 || size_t(r) != cap) bad("LZ4", "decode failed");
      return;
    }
    case CODEC_BROTLI: {
      size_t out = cap;
      if (BrotliDecoderDecompress(n, src, &out, dst) != 1) bad("BROTLI", "decode failed");
      if (out != cap) bad("BROTLI", "short output");
      return;
    }
    default:
      throw PlanError(LK_ERR_UNSUPPORTED, "parquet: compression codec " + std::to_string(codec) + " is not supported");
  }
}

bool codec_supported(int codec) {
  return codec == CODEC_UNCOMPRESSED || codec == CODEC_SNAPPY || codec == CODEC_GZIP || codec == CODEC_ZSTD ||
         codec == CODEC_LZ4 || codec == CODEC_LZ4_RAW || codec == CODEC_BROTLI;
}

}  // namespace pq
}  // namespace lk
