// Java 17 Double.toString / Float.toString: the text DuckDB's JDBC getString hands the reference for DOUBLE / FLOAT
// exemplar columns (the worker runs on eclipse-temurin:17, query-worker/Dockerfile:20).
//
// JDK 17 formats with sun.misc.FloatingDecimal (BinaryToASCIIBuffer.dtoa + getChars), which is NOT the shortest
// round-trip digit algorithm JDK 19 adopted: integers below 2^63 print through a long with only the provably
// insignificant low digits dropped (2.82879384806159E17 -> "2.82879384806159008E17"), and the digit loop's stopping
// test is strict in the int / long branches but not in the big-integer branch (2e23 -> "1.9999999999999998E23").
// Restated here from the algorithm (Steele & White free-format digit generation with an estimated decimal exponent);
// every branch runs on one small big-integer type, which gives the same digits as the JDK's int / long arithmetic
// since those branches are only taken when nothing overflows.  oracle/exemplar.py holds the same restatement in
// Python; tests/test_jdtoa.py checks the two against each other and against the JDK's documented outputs.
#include <cmath>
#include <cstdint>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/lakeside_text.h"
#include "evalutil.hpp"

namespace lk {
namespace {

// Bits of 5^i for small i (FloatingDecimal.N_5_BITS): sizes the branch choice, not the arithmetic.
constexpr int kN5Bits[] = {0,  3,  5,  7,  10, 12, 14, 17, 19, 21, 24, 26, 28, 31,
                           33, 35, 38, 40, 42, 45, 47, 49, 52, 54, 56, 59, 61};
constexpr int kN5Len = int(sizeof kN5Bits / sizeof kN5Bits[0]);
// Decimal digits of 2^k that cannot matter when printing a value with k more bits than it has significant
// (FloatingDecimal.insignificantDigitsNumber).
constexpr int kInsignificant[] = {0,  0,  0,  0,  1,  1,  1,  2,  2,  2,  3,  3,  3,  3,  4,  4,  4,  5,  5,  5,  6,  6,
                                  6,  6,  7,  7,  7,  8,  8,  8,  9,  9,  9,  9,  10, 10, 10, 11, 11, 11, 12, 12, 12, 12,
                                  13, 13, 13, 14, 14, 14, 15, 15, 15, 15, 16, 16, 16, 17, 17, 17, 18, 18, 18, 19};
constexpr int kInsLen = int(sizeof kInsignificant / sizeof kInsignificant[0]);
constexpr int kExpShift = 52;

// Non-negative integer, little-endian 32-bit limbs (at most ~1200 bits here: 5^325 << ~1100).
struct Big {
  std::vector<uint32_t> d;
  explicit Big(uint64_t v = 0) {
    if (v) d.push_back(uint32_t(v));
    if (v >> 32) d.push_back(uint32_t(v >> 32));
  }
  void trim() {
    while (!d.empty() && d.back() == 0) d.pop_back();
  }
  void mul(uint32_t k) {
    uint64_t c = 0;
    for (auto& x : d) {
      const uint64_t t = uint64_t(x) * k + c;
      x = uint32_t(t);
      c = t >> 32;
    }
    if (c) d.push_back(uint32_t(c));
  }
  void mul_pow5(int e) {
    for (; e >= 13; e -= 13) mul(1220703125u);   // 5^13
    uint32_t p = 1;
    while (e-- > 0) p *= 5;
    if (p > 1) mul(p);
  }
  void shl(int s) {
    if (d.empty() || s == 0) return;
    const int w = s / 32, b = s % 32;
    if (b) {
      uint32_t c = 0;
      for (auto& x : d) {
        const uint32_t nx = (x << b) | c;
        c = x >> (32 - b);
        x = nx;
      }
      if (c) d.push_back(c);
    }
    d.insert(d.begin(), size_t(w), 0u);
  }
  void sub(const Big& o) {   // *this >= o
    int64_t br = 0;
    for (size_t i = 0; i < d.size(); i++) {
      int64_t t = int64_t(d[i]) - br - (i < o.d.size() ? int64_t(o.d[i]) : 0);
      br = t < 0;
      d[i] = uint32_t(t + (br << 32));
    }
    trim();
  }
  static Big add(const Big& a, const Big& b) {
    Big r;
    const size_t n = std::max(a.d.size(), b.d.size());
    r.d.resize(n + 1);
    uint64_t c = 0;
    for (size_t i = 0; i < n; i++) {
      c += (i < a.d.size() ? a.d[i] : 0u);
      c += (i < b.d.size() ? b.d[i] : 0u);
      r.d[i] = uint32_t(c);
      c >>= 32;
    }
    r.d[n] = uint32_t(c);
    r.trim();
    return r;
  }
  static int cmp(const Big& a, const Big& b) {
    if (a.d.size() != b.d.size()) return a.d.size() < b.d.size() ? -1 : 1;
    for (size_t i = a.d.size(); i-- > 0;)
      if (a.d[i] != b.d[i]) return a.d[i] < b.d[i] ? -1 : 1;
    return 0;
  }
};

// quotient (< 10 by construction of the scaling) and remainder of b / s
int div_digit(Big& b, const Big& s) {
  int q = 0;
  while (Big::cmp(b, s) >= 0) {
    b.sub(s);
    q++;
  }
  return q;
}

// FloatingDecimal.estimateDecExp: floor(log10(value)) estimated from the mantissa's first bits, maybe one too high.
int estimate_dec_exp(uint64_t fract_bits, int bin_exp) {
  const uint64_t bits = (uint64_t(0x3ff) << 52) | (fract_bits & ((uint64_t(1) << 52) - 1));
  double d2;
  memcpy(&d2, &bits, 8);
  const double d = (d2 - 1.5) * 0.289529654 + 0.176091259 + double(bin_exp) * 0.301029995663981;
  return int(std::floor(d));
}

// BinaryToASCIIBuffer.dtoa (compatible format): digits and the decimal exponent (value = 0.d1d2... x 10^dec_exponent).
void dtoa(int bin_exp, uint64_t fract_bits, int n_sig, std::string& digits, int& dec_exponent) {
  const int tail_zeros = __builtin_ctzll(fract_bits);
  const int n_fract_bits = kExpShift + 1 - tail_zeros;
  const int n_tiny_bits = std::max(0, n_fract_bits - bin_exp - 1);
  digits.clear();
  if (bin_exp <= 62 && bin_exp >= -21 && n_tiny_bits == 0 && n_fract_bits + kN5Bits[0] < 64) {
    // the easy case: an integer that fits a long, printed with its provably insignificant low digits rounded off
    const int k = bin_exp - n_sig - 1;
    const int insignificant = (bin_exp > n_sig && k > 1 && k < kInsLen) ? kInsignificant[k] : 0;
    uint64_t lv = bin_exp >= kExpShift ? fract_bits << (bin_exp - kExpShift) : fract_bits >> (kExpShift - bin_exp);
    int dexp = 0;
    if (insignificant) {
      uint64_t p10 = 1;
      for (int i = 0; i < insignificant; i++) p10 *= 10;
      const uint64_t residue = lv % p10;
      lv /= p10;
      dexp += insignificant;
      if (residue >= (p10 >> 1)) lv++;
    }
    std::string s = std::to_string(lv);
    dexp += int(s.size()) - 1;
    while (s.size() > 1 && s.back() == '0') s.pop_back();
    digits = s;
    dec_exponent = dexp + 1;
    return;
  }
  int dec_exp = estimate_dec_exp(fract_bits, bin_exp);
  const int b5 = std::max(0, -dec_exp);
  int b2 = b5 + n_tiny_bits + bin_exp;
  const int s5 = std::max(0, dec_exp);
  int s2 = s5 + n_tiny_bits;
  const int m5 = b5;
  int m2 = b2 - n_sig;
  fract_bits >>= tail_zeros;
  b2 -= n_fract_bits - 1;
  const int common = std::min(b2, s2);
  b2 -= common;
  s2 -= common;
  m2 -= common;
  if (n_fract_bits == 1) m2 -= 1;
  if (m2 < 0) {
    b2 -= m2;
    s2 -= m2;
    m2 = 0;
  }
  const int b_bits = n_fract_bits + b2 + (b5 < kN5Len ? kN5Bits[b5] : b5 * 3);
  const int ten_s_bits = s2 + 1 + (s5 + 1 < kN5Len ? kN5Bits[s5 + 1] : (s5 + 1) * 3);
  const bool small = b_bits < 64 && ten_s_bits < 64;   // the JDK's int / long branches: high = b + m > 10 s

  Big b(fract_bits), s(1), m(1);
  b.mul_pow5(b5);
  b.shl(b2);
  s.mul_pow5(s5);
  s.shl(s2);
  m.mul_pow5(m5);
  m.shl(m2);
  Big tens = s;
  tens.mul(10);
  auto is_high = [&](const Big& bb, const Big& mm) {
    const int c = Big::cmp(Big::add(bb, mm), tens);
    return small ? c > 0 : c >= 0;   // big branch: FDBigInteger.addAndCmp(B, M) <= 0
  };

  int q = div_digit(b, s);
  b.mul(10);
  m.mul(10);
  bool low = Big::cmp(b, m) < 0, high = is_high(b, m);
  if (q == 0 && !high)
    dec_exp--;   // the estimate was one too high: drop the leading zero
  else
    digits.push_back(char('0' + q));
  if (dec_exp < -3 || dec_exp >= 8) low = high = false;   // E-form prints at least two digits
  while (!low && !high) {
    q = div_digit(b, s);
    b.mul(10);
    m.mul(10);
    low = Big::cmp(b, m) < 0;
    high = is_high(b, m);
    digits.push_back(char('0' + q));
  }
  dec_exponent = dec_exp + 1;
  bool up = false;
  if (high) {
    if (!low) {
      up = true;
    } else {
      Big b2x = b;
      b2x.shl(1);
      const int ld = Big::cmp(b2x, tens);   // sign of 2b - 10s: which neighbour is nearer
      up = ld > 0 || (ld == 0 && ((digits.back() - '0') & 1));
    }
  }
  if (up) {   // roundup(): carry through trailing nines; an all-nine string becomes 1 followed by zeros
    size_t i = digits.size() - 1;
    while (digits[i] == '9' && i > 0) digits[i--] = '0';
    if (digits[i] == '9') {
      dec_exponent++;
      digits[0] = '1';
    } else {
      digits[i]++;
    }
  }
}

// BinaryToASCIIBuffer.getChars: plain for 10^-3 <= |x| < 10^7, d.ddddE<exp> otherwise.
std::string java_chars(bool neg, const std::string& digits, int dec_exponent) {
  std::string out = neg ? "-" : "";
  const int nd = int(digits.size());
  if (dec_exponent > 0 && dec_exponent < 8) {
    const int n = std::min(nd, dec_exponent);
    out.append(digits, 0, size_t(n));
    if (n < dec_exponent) return out + std::string(size_t(dec_exponent - n), '0') + ".0";
    return out + "." + (n < nd ? digits.substr(size_t(n)) : std::string("0"));
  }
  if (dec_exponent <= 0 && dec_exponent > -3) return out + "0." + std::string(size_t(-dec_exponent), '0') + digits;
  out += digits[0];
  out += '.';
  out += nd > 1 ? digits.substr(1) : std::string("0");
  out += 'E';
  out += dec_exponent <= 0 ? "-" + std::to_string(-dec_exponent + 1) : std::to_string(dec_exponent - 1);
  return out;
}

}  // namespace

std::string java_text(double x) {
  uint64_t bits;
  memcpy(&bits, &x, 8);
  const bool neg = bits >> 63;
  uint64_t fract = bits & ((uint64_t(1) << 52) - 1);
  int bexp = int((bits >> 52) & 0x7ff);
  if (bexp == 0x7ff) return fract ? "NaN" : (neg ? "-Infinity" : "Infinity");
  int nsig;
  if (bexp == 0) {
    if (fract == 0) return neg ? "-0.0" : "0.0";
    const int lz = __builtin_clzll(fract);
    const int shift = lz - (63 - kExpShift);
    fract <<= shift;
    bexp = 1 - shift;
    nsig = 64 - lz;
  } else {
    fract |= uint64_t(1) << 52;
    nsig = 53;
  }
  std::string digits;
  int dexp = 0;
  dtoa(bexp - 1023, fract, nsig, digits, dexp);
  return java_chars(neg, digits, dexp);
}

std::string java_text(float x) {
  uint32_t bits;
  memcpy(&bits, &x, 4);
  const bool neg = bits >> 31;
  uint32_t fract = bits & ((1u << 23) - 1);
  int bexp = int((bits >> 23) & 0xff);
  if (bexp == 0xff) return fract ? "NaN" : (neg ? "-Infinity" : "Infinity");
  int nsig;
  if (bexp == 0) {
    if (fract == 0) return neg ? "-0.0" : "0.0";
    const int lz = __builtin_clz(fract);
    const int shift = lz - (31 - 23);
    fract <<= shift;
    bexp = 1 - shift;
    nsig = 32 - lz;
  } else {
    fract |= 1u << 23;
    nsig = 24;
  }
  std::string digits;
  int dexp = 0;
  dtoa(bexp - 127, uint64_t(fract) << (kExpShift - 23), nsig, digits, dexp);
  return java_chars(neg, digits, dexp);
}

}  // namespace lk

// Host-only test hook (liblakeside_text.so, include/lakeside_text.h): the text, NUL-terminated; returns its length,
// or -1 when `cap` is too small.
extern "C" int lk_java_double_text(double x, char* buf, size_t cap) {
  const std::string s = lk::java_text(x);
  if (s.size() + 1 > cap) return -1;
  memcpy(buf, s.c_str(), s.size() + 1);
  return int(s.size());
}
extern "C" int lk_java_float_text(float x, char* buf, size_t cap) {
  const std::string s = lk::java_text(x);
  if (s.size() + 1 > cap) return -1;
  memcpy(buf, s.c_str(), s.size() + 1);
  return int(s.size());
}
