// DDSketch host side (see ddsketch.hpp).
#include "ddsketch.hpp"

#include <cfloat>
#include <cmath>
#include <cstring>

#include "layout.hpp"

namespace lk::dd {

const Mapping& mapping() {
  static const Mapping m = [] {
    Mapping x{};
    const double mantissa = 2.0 * kRelativeAccuracy / (1.0 - kRelativeAccuracy);
    x.gamma = 1.0 + mantissa;
    x.multiplier = 1.0 / std::log1p(mantissa);
    x.relative_accuracy = (x.gamma - 1.0) / (x.gamma + 1.0);
    x.min_indexable = DBL_MIN * x.gamma;
    x.max_indexable = DBL_MAX / x.gamma;
    return x;
  }();
  return m;
}

double Mapping::value(int32_t index) const { return std::exp(double(index) / multiplier) * (1.0 + relative_accuracy); }

void Sketch::add_bin(uint32_t bin, double count) {
  if (bin == 0) {
    zero += count;
  } else if (bin <= DD_HALF) {
    pos[int32_t(bin) - 1 - DD_BIAS] += count;
  } else {
    neg[int32_t(bin - DD_HALF) - 1 - DD_BIAS] += count;
  }
}

bool Sketch::accept(double v) {
  const Mapping& m = mapping();
  const double a = std::fabs(v);
  if (!(a <= m.max_indexable)) return false;
  if (a <= m.min_indexable) {
    zero += 1.0;
    return true;
  }
  const double x = std::log(a) * m.multiplier;
  const int32_t i = x >= 0.0 ? int32_t(x) : int32_t(x) - 1;
  (v < 0.0 ? neg : pos)[i] += 1.0;
  return true;
}

void Sketch::merge(const Sketch& o) {
  for (auto& kv : o.pos) pos[kv.first] += kv.second;
  for (auto& kv : o.neg) neg[kv.first] += kv.second;
  zero += o.zero;
}

double Sketch::count() const {
  double n = zero;
  for (auto& kv : neg) n += kv.second;
  for (auto& kv : pos) n += kv.second;
  return n;
}

double Sketch::quantile(double q) const {
  const Mapping& m = mapping();
  const double rank = q * (count() - 1.0);
  double n = 0.0;
  for (auto it = neg.rbegin(); it != neg.rend(); ++it)
    if ((n += it->second) > rank) return -m.value(it->first);
  if ((n += zero) > rank) return 0.0;
  for (auto& kv : pos)
    if ((n += kv.second) > rank) return m.value(kv.first);
  return pos.empty() ? 0.0 : m.value(pos.rbegin()->first);
}

namespace {
void varint(std::string& o, uint64_t v) {
  while (v >= 0x80) {
    o.push_back(char(uint8_t(v) | 0x80));
    v >>= 7;
  }
  o.push_back(char(v));
}
void fixed64(std::string& o, double d) {
  uint64_t u;
  memcpy(&u, &d, 8);
  for (int i = 0; i < 8; i++) o.push_back(char(uint8_t(u >> (8 * i))));
}
std::string store(const std::map<int32_t, double>& bins) {
  std::string s;
  if (bins.empty()) return s;
  const int32_t lo = bins.begin()->first, hi = bins.rbegin()->first;
  std::string packed;
  for (int32_t i = lo; i <= hi; i++) {
    auto it = bins.find(i);
    fixed64(packed, it == bins.end() ? 0.0 : it->second);
  }
  s.push_back(char(0x12));   // field 2 contiguousBinCounts, packed doubles
  varint(s, packed.size());
  s += packed;
  if (lo != 0) {
    s.push_back(char(0x18));   // field 3 contiguousBinIndexOffset, sint32 (zigzag)
    varint(s, uint32_t((uint32_t(lo) << 1) ^ uint32_t(lo >> 31)));
  }
  return s;
}
}  // namespace

std::string Sketch::serialize() const {
  std::string o, mp;
  mp.push_back(char(0x09));    // IndexMapping.gamma (field 1, fixed64); indexOffset 0 and NONE interpolation omitted
  fixed64(mp, mapping().gamma);
  o.push_back(char(0x0a));     // DDSketch.mapping (field 1)
  varint(o, mp.size());
  o += mp;
  const std::string p = store(pos), n = store(neg);
  o.push_back(char(0x12));     // positiveValues (field 2)
  varint(o, p.size());
  o += p;
  o.push_back(char(0x1a));     // negativeValues (field 3)
  varint(o, n.size());
  o += n;
  if (zero != 0.0) {
    o.push_back(char(0x21));   // zeroCount (field 4, fixed64)
    fixed64(o, zero);
  }
  return o;
}

}  // namespace lk::dd
