// Minimal JSON DOM (order-preserving objects) for PushDownRequest / engine options.
#pragma once
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <memory>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

namespace lk {

struct JsonError : std::runtime_error {
  using std::runtime_error::runtime_error;
};

class Json {
 public:
  enum Kind { Null, Bool, Number, String, Array, Object };
  Kind kind = Null;
  bool b = false;
  double num = 0;
  std::string num_text;  // exact digits (int64 timestamps must not go through double)
  std::string str;
  std::vector<Json> arr;
  std::vector<std::pair<std::string, Json>> obj;

  bool is_null() const { return kind == Null; }
  bool is_str() const { return kind == String; }
  bool is_arr() const { return kind == Array; }
  bool is_obj() const { return kind == Object; }
  const Json* get(const std::string& k) const {
    if (kind != Object) return nullptr;
    for (auto& kv : obj)
      if (kv.first == k) return &kv.second;
    return nullptr;
  }
  int64_t as_i64() const {
    if (kind == Number) {
      if (num_text.find_first_of(".eE") == std::string::npos) return std::strtoll(num_text.c_str(), nullptr, 10);
      return int64_t(num);
    }
    if (kind == String) return std::strtoll(str.c_str(), nullptr, 10);
    throw JsonError("json: expected a number");
  }
  bool as_bool() const {
    if (kind == Bool) return b;
    throw JsonError("json: expected a boolean");
  }
  // JSON scalar rendered the way Scala's String.valueOf would show it (queryTags values).
  std::string scalar_text() const {
    switch (kind) {
      case String: return str;
      case Number: return num_text;
      case Bool: return b ? "true" : "false";
      case Null: return "null";
      default: return "";
    }
  }

  static Json parse(const std::string& s) {
    size_t i = 0;
    Json j = parse_value(s, i);
    skip_ws(s, i);
    if (i != s.size()) throw JsonError("json: trailing characters");
    return j;
  }

 private:
  static void skip_ws(const std::string& s, size_t& i) {
    while (i < s.size() && (s[i] == ' ' || s[i] == '\n' || s[i] == '\r' || s[i] == '\t')) i++;
  }
  static void put_utf8(std::string& o, uint32_t cp) {
    if (cp < 0x80) o += char(cp);
    else if (cp < 0x800) { o += char(0xC0 | (cp >> 6)); o += char(0x80 | (cp & 0x3F)); }
    else if (cp < 0x10000) { o += char(0xE0 | (cp >> 12)); o += char(0x80 | ((cp >> 6) & 0x3F)); o += char(0x80 | (cp & 0x3F)); }
    else { o += char(0xF0 | (cp >> 18)); o += char(0x80 | ((cp >> 12) & 0x3F)); o += char(0x80 | ((cp >> 6) & 0x3F)); o += char(0x80 | (cp & 0x3F)); }
  }
  static std::string parse_string(const std::string& s, size_t& i) {
    if (s[i] != '"') throw JsonError("json: expected string");
    i++;
    std::string o;
    while (i < s.size() && s[i] != '"') {
      if (s[i] != '\\') {   // a run of plain characters: appended at once
        size_t j = i + 1;
        while (j < s.size() && s[j] != '"' && s[j] != '\\') j++;
        o.append(s, i, j - i);
        i = j;
        continue;
      }
      i++;
      if (i >= s.size()) throw JsonError("json: bad escape");
      char e = s[i++];
      switch (e) {
        case '"': o += '"'; break;
        case '\\': o += '\\'; break;
        case '/': o += '/'; break;
        case 'b': o += '\b'; break;
        case 'f': o += '\f'; break;
        case 'n': o += '\n'; break;
        case 'r': o += '\r'; break;
        case 't': o += '\t'; break;
        case 'u': {
          if (i + 4 > s.size()) throw JsonError("json: bad \\u");
          uint32_t cp = uint32_t(std::strtoul(s.substr(i, 4).c_str(), nullptr, 16));
          i += 4;
          if (cp >= 0xD800 && cp < 0xDC00 && i + 6 <= s.size() && s[i] == '\\' && s[i + 1] == 'u') {
            uint32_t lo = uint32_t(std::strtoul(s.substr(i + 2, 4).c_str(), nullptr, 16));
            if (lo >= 0xDC00 && lo < 0xE000) { cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00); i += 6; }
          }
          put_utf8(o, cp);
          break;
        }
        default: throw JsonError("json: bad escape");
      }
    }
    if (i >= s.size()) throw JsonError("json: unterminated string");
    i++;
    return o;
  }
  static Json parse_value(const std::string& s, size_t& i) {
    skip_ws(s, i);
    if (i >= s.size()) throw JsonError("json: unexpected end");
    Json j;
    char c = s[i];
    if (c == '{') {
      j.kind = Object;
      i++;
      skip_ws(s, i);
      if (i < s.size() && s[i] == '}') { i++; return j; }
      while (true) {
        skip_ws(s, i);
        std::string k = parse_string(s, i);
        skip_ws(s, i);
        if (i >= s.size() || s[i] != ':') throw JsonError("json: expected ':'");
        i++;
        j.obj.emplace_back(std::move(k), parse_value(s, i));
        skip_ws(s, i);
        if (i < s.size() && s[i] == ',') { i++; continue; }
        if (i < s.size() && s[i] == '}') { i++; break; }
        throw JsonError("json: expected ',' or '}'");
      }
    } else if (c == '[') {
      j.kind = Array;
      i++;
      skip_ws(s, i);
      if (i < s.size() && s[i] == ']') { i++; return j; }
      while (true) {
        j.arr.push_back(parse_value(s, i));
        skip_ws(s, i);
        if (i < s.size() && s[i] == ',') { i++; continue; }
        if (i < s.size() && s[i] == ']') { i++; break; }
        throw JsonError("json: expected ',' or ']'");
      }
    } else if (c == '"') {
      j.kind = String;
      j.str = parse_string(s, i);
    } else if (s.compare(i, 4, "true") == 0) {
      j.kind = Bool; j.b = true; i += 4;
    } else if (s.compare(i, 5, "false") == 0) {
      j.kind = Bool; j.b = false; i += 5;
    } else if (s.compare(i, 4, "null") == 0) {
      j.kind = Null; i += 4;
    } else {
      size_t st = i;
      while (i < s.size() && (isdigit((unsigned char)s[i]) || s[i] == '-' || s[i] == '+' || s[i] == '.' ||
                              s[i] == 'e' || s[i] == 'E'))
        i++;
      if (st == i) throw JsonError("json: unexpected character");
      j.kind = Number;
      j.num_text = s.substr(st, i - st);
      j.num = std::strtod(j.num_text.c_str(), nullptr);
    }
    return j;
  }
};

}  // namespace lk
