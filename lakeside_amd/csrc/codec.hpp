// Parquet page decompression (host, at segment load); codec.cpp.
#pragma once
#include <cstddef>
#include <cstdint>

namespace lk {
namespace pq {

// parquet.thrift CompressionCodec
enum Codec { CODEC_UNCOMPRESSED = 0, CODEC_SNAPPY = 1, CODEC_GZIP = 2, CODEC_LZO = 3, CODEC_BROTLI = 4,
             CODEC_LZ4 = 5, CODEC_ZSTD = 6, CODEC_LZ4_RAW = 7 };

// Decompress exactly `cap` bytes (the page header's uncompressed size) from src[0..n) into dst.
// Throws PlanError (LK_ERR_IO on corrupt input, LK_ERR_UNSUPPORTED on an unsupported codec).
void decompress(int codec, const uint8_t* src, size_t n, uint8_t* dst, size_t cap);
bool codec_supported(int codec);

}  // namespace pq
}  // namespace lk
