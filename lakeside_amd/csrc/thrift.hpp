// Thrift compact protocol: the subset Parquet metadata uses (reader + writer).
// Parquet stores FileMetaData and every PageHeader in this encoding (parquet-format's parquet.thrift).
#pragma once
#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

namespace lk {

enum TType : uint8_t {
  T_STOP = 0, T_TRUE = 1, T_FALSE = 2, T_BYTE = 3, T_I16 = 4, T_I32 = 5, T_I64 = 6,
  T_DOUBLE = 7, T_BINARY = 8, T_LIST = 9, T_SET = 10, T_MAP = 11, T_STRUCT = 12
};

struct ThriftError : std::runtime_error {
  using std::runtime_error::runtime_error;
};

class TReader {
 public:
  TReader(const uint8_t* p, size_t n) : p_(p), end_(p + n), begin_(p) {}
  size_t consumed() const { return size_t(p_ - begin_); }

  uint8_t byte() {
    if (p_ >= end_) throw ThriftError("thrift: truncated");
    return *p_++;
  }
  uint64_t varint() {
    uint64_t v = 0;
    for (int s = 0; s < 64; s += 7) {
      uint8_t b = byte();
      v |= uint64_t(b & 0x7f) << s;
      if (!(b & 0x80)) return v;
    }
    throw ThriftError("thrift: bad varint");
  }
  int64_t zigzag() {
    uint64_t v = varint();
    return int64_t(v >> 1) ^ -int64_t(v & 1);
  }
  std::string binary() {
    uint64_t n = varint();
    if (n > uint64_t(end_ - p_)) throw ThriftError("thrift: binary overflow");
    std::string s(reinterpret_cast<const char*>(p_), n);
    p_ += n;
    return s;
  }
  double dbl() {
    if (end_ - p_ < 8) throw ThriftError("thrift: truncated double");
    double d;
    memcpy(&d, p_, 8);
    p_ += 8;
    return d;
  }

  // Struct field iteration. Returns false at STOP. `type` is the field's compact type.
  void struct_begin() { last_.push_back(0); }
  void struct_end() { last_.pop_back(); }
  bool field(int16_t& id, uint8_t& type) {
    uint8_t h = byte();
    if (h == T_STOP) return false;
    type = h & 0x0f;
    int16_t delta = h >> 4;
    if (delta) id = int16_t(last_.back() + delta);
    else id = int16_t(zigzag());
    last_.back() = id;
    return true;
  }
  void list_begin(uint8_t& etype, uint32_t& n) {
    uint8_t h = byte();
    etype = h & 0x0f;
    n = h >> 4;
    if (n == 15) n = uint32_t(varint());
  }
  bool bool_val(uint8_t type) { return type == T_TRUE; }
  void skip(uint8_t type) {
    switch (type) {
      case T_TRUE: case T_FALSE: return;
      case T_BYTE: byte(); return;
      case T_I16: case T_I32: case T_I64: varint(); return;
      case T_DOUBLE: dbl(); return;
      case T_BINARY: binary(); return;
      case T_LIST: case T_SET: {
        uint8_t et; uint32_t n;
        list_begin(et, n);
        for (uint32_t i = 0; i < n; i++) {
          if (et == T_TRUE || et == T_FALSE) byte();
          else skip(et);
        }
        return;
      }
      case T_MAP: {
        uint64_t n = varint();
        if (n == 0) return;
        uint8_t kv = byte();
        for (uint64_t i = 0; i < n; i++) { skip(kv >> 4); skip(kv & 0xf); }
        return;
      }
      case T_STRUCT: {
        struct_begin();
        int16_t id; uint8_t t;
        while (field(id, t)) skip(t);
        struct_end();
        return;
      }
      default: throw ThriftError("thrift: bad type");
    }
  }

 private:
  const uint8_t* p_;
  const uint8_t* end_;
  const uint8_t* begin_;
  std::vector<int16_t> last_;
};

class TWriter {
 public:
  std::vector<uint8_t> out;
  void byte(uint8_t b) { out.push_back(b); }
  void varint(uint64_t v) {
    while (v >= 0x80) { out.push_back(uint8_t(v | 0x80)); v >>= 7; }
    out.push_back(uint8_t(v));
  }
  void zigzag(int64_t v) { varint((uint64_t(v) << 1) ^ uint64_t(v >> 63)); }
  void struct_begin() { last_.push_back(0); }
  void struct_end() { byte(T_STOP); last_.pop_back(); }
  void field(int16_t id, uint8_t type) {
    int16_t d = int16_t(id - last_.back());
    if (d > 0 && d <= 15) byte(uint8_t((d << 4) | type));
    else { byte(type); zigzag(id); }
    last_.back() = id;
  }
  void i32(int16_t id, int32_t v) { field(id, T_I32); zigzag(v); }
  void i64(int16_t id, int64_t v) { field(id, T_I64); zigzag(v); }
  void boolean(int16_t id, bool v) { field(id, v ? T_TRUE : T_FALSE); }
  void bin(int16_t id, const std::string& s) { field(id, T_BINARY); varint(s.size()); out.insert(out.end(), s.begin(), s.end()); }
  void list_begin(int16_t id, uint8_t etype, uint32_t n) {
    field(id, T_LIST);
    if (n < 15) byte(uint8_t((n << 4) | etype));
    else { byte(uint8_t(0xf0 | etype)); varint(n); }
  }
  void list_i32(int32_t v) { zigzag(v); }
  void list_bin(const std::string& s) { varint(s.size()); out.insert(out.end(), s.begin(), s.end()); }

 private:
  std::vector<int16_t> last_;
};

}  // namespace lk
