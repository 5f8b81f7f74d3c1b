// Cardinality estimates (`ces`): the host side.
//
// The reference keeps one datasketches HllSketch(lgConfigK = 12, HLL_4) per time step and feeds it every row's
// group-key string groupBys.map(g => tags.getOrElse(g, "")).mkString(":") (Aggregator.scala:43-60,
// PushDownAggregatorStage.scala:82-94,183-186); query-api unions the per-step sketches and reads getEstimate
// (TimeGroupedSketchAggregator.scala:38-43, BaseExpr.scala:56-58).  An HLL's state depends only on the SET of
// strings fed to it, so the GPU scan computes the exact distinct (step, group key) set (a COUNT table over the
// groupBys) and the host hashes each distinct key once.
//
// Library: org.apache.datasketches:datasketches-java 4.2.0 (not vendored, no JVM).  Restated: update(String)
// ignores an empty string, hashes the UTF-8 bytes with MurmurHash3_x64_128 (seed 9001) and forms the coupon
// (min(nlz(h2), 62) + 1) << 26 | (h1 & 0x3FFFFFF); the register of slot (coupon & (2^12 - 1)) keeps the largest
// value.  Estimate (parity unpinned: datasketches' coupon-interpolation and HIP estimators are not restated):
// up to 384 distinct coupons (the sketch's LIST/SET modes) the coupon count; beyond, the HLL estimate
// alpha_m m^2 / sum 2^-M[j] with linear counting m ln(m / V) below 5m/2.
#pragma once
#include <cstdint>
#include <string>
#include <unordered_set>
#include <vector>

namespace lk::hll {

constexpr int kLgK = 12;

void murmur3_x64_128(const void* data, size_t len, uint64_t seed, uint64_t out[2]);
uint32_t coupon(const std::string& s);   // 0 for the empty string (not counted)

struct Sketch {
  std::unordered_set<uint32_t> coupons;
  void update(const std::string& s);
  void merge(const Sketch& o);
  double estimate() const;
};

}  // namespace lk::hll
