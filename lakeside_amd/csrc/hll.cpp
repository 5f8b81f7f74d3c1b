// HLL host side (see hll.hpp).
#include "hll.hpp"

#include <cmath>
#include <cstring>

namespace lk::hll {

namespace {
inline uint64_t rotl(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }
inline uint64_t fmix(uint64_t k) {
  k ^= k >> 33;
  k *= 0xff51afd7ed558ccdull;
  k ^= k >> 33;
  k *= 0xc4ceb9fe1a85ec53ull;
  k ^= k >> 33;
  return k;
}
}  // namespace

// MurmurHash3_x64_128 (Austin Appleby, public domain): 16-byte blocks, little-endian, tail, finalization.
void murmur3_x64_128(const void* data, size_t len, uint64_t seed, uint64_t out[2]) {
  const uint8_t* p = static_cast<const uint8_t*>(data);
  const size_t nblocks = len / 16;
  uint64_t h1 = seed, h2 = seed;
  const uint64_t c1 = 0x87c37b91114253d5ull, c2 = 0x4cf5ad432745937full;
  for (size_t i = 0; i < nblocks; i++) {
    uint64_t k1, k2;
    memcpy(&k1, p + 16 * i, 8);
    memcpy(&k2, p + 16 * i + 8, 8);
    k1 *= c1; k1 = rotl(k1, 31); k1 *= c2; h1 ^= k1;
    h1 = rotl(h1, 27); h1 += h2; h1 = h1 * 5 + 0x52dce729;
    k2 *= c2; k2 = rotl(k2, 33); k2 *= c1; h2 ^= k2;
    h2 = rotl(h2, 31); h2 += h1; h2 = h2 * 5 + 0x38495ab5;
  }
  const uint8_t* tail = p + nblocks * 16;
  uint64_t k1 = 0, k2 = 0;
  switch (len & 15) {
    case 15: k2 ^= uint64_t(tail[14]) << 48; [[fallthrough]];
    case 14: k2 ^= uint64_t(tail[13]) << 40; [[fallthrough]];
    case 13: k2 ^= uint64_t(tail[12]) << 32; [[fallthrough]];
    case 12: k2 ^= uint64_t(tail[11]) << 24; [[fallthrough]];
    case 11: k2 ^= uint64_t(tail[10]) << 16; [[fallthrough]];
    case 10: k2 ^= uint64_t(tail[9]) << 8; [[fallthrough]];
    case 9:
      k2 ^= uint64_t(tail[8]);
      k2 *= c2; k2 = rotl(k2, 33); k2 *= c1; h2 ^= k2;
      [[fallthrough]];
    case 8: k1 ^= uint64_t(tail[7]) << 56; [[fallthrough]];
    case 7: k1 ^= uint64_t(tail[6]) << 48; [[fallthrough]];
    case 6: k1 ^= uint64_t(tail[5]) << 40; [[fallthrough]];
    case 5: k1 ^= uint64_t(tail[4]) << 32; [[fallthrough]];
    case 4: k1 ^= uint64_t(tail[3]) << 24; [[fallthrough]];
    case 3: k1 ^= uint64_t(tail[2]) << 16; [[fallthrough]];
    case 2: k1 ^= uint64_t(tail[1]) << 8; [[fallthrough]];
    case 1:
      k1 ^= uint64_t(tail[0]);
      k1 *= c1; k1 = rotl(k1, 31); k1 *= c2; h1 ^= k1;
      break;
    default: break;
  }
  h1 ^= uint64_t(len);
  h2 ^= uint64_t(len);
  h1 += h2;
  h2 += h1;
  h1 = fmix(h1);
  h2 = fmix(h2);
  h1 += h2;
  h2 += h1;
  out[0] = h1;
  out[1] = h2;
}

uint32_t coupon(const std::string& s) {
  if (s.empty()) return 0;
  uint64_t h[2];
  murmur3_x64_128(s.data(), s.size(), 9001, h);
  const uint32_t lz = h[1] ? uint32_t(__builtin_clzll(h[1])) : 64u;
  return ((lz > 62 ? 62u : lz) + 1u) << 26 | uint32_t(h[0] & 0x3FFFFFFull);
}

void Sketch::update(const std::string& s) {
  const uint32_t c = coupon(s);
  if (c) coupons.insert(c);
}

void Sketch::merge(const Sketch& o) { coupons.insert(o.coupons.begin(), o.coupons.end()); }

double Sketch::estimate() const {
  constexpr uint32_t m = 1u << kLgK;
  if (coupons.size() <= 384) return double(coupons.size());
  std::vector<uint8_t> reg(m, 0);
  for (uint32_t c : coupons) {
    const uint32_t slot = c & (m - 1), v = c >> 26;
    if (v > reg[slot]) reg[slot] = uint8_t(v);
  }
  double sum = 0.0;
  uint32_t zeros = 0;
  for (uint8_t r : reg) {
    sum += std::ldexp(1.0, -int(r));
    zeros += r == 0;
  }
  const double alpha = 0.7213 / (1.0 + 1.079 / double(m));
  const double e = alpha * double(m) * double(m) / sum;
  if (e <= 2.5 * double(m) && zeros) return double(m) * std::log(double(m) / double(zeros));
  return e;
}

}  // namespace lk::hll
