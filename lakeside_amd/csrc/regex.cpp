// RE2-semantics matcher (see regex.hpp).  Parser -> Thompson NFA -> lazy DFA / NFA simulation.
//
// Syntax and its corner cases follow RE2's documented grammar (github.com/google/re2/wiki/Syntax) with the
// options DuckDB's regexp_matches(..., 'i') passes: Perl-like syntax, ^/$ at text boundaries unless (?m), '.'
// excludes \n unless (?s), negated classes include \n, \d \s \w \b ASCII, case folding over Unicode simple-folding
// orbits (tables generated from unicodedata by tools/gen_unicode_tables.py).  Verified differentially against
// RE2 itself (pyarrow.compute.match_substring_regex) in tests/test_regex.py.
#include "regex.hpp"

#include <algorithm>
#include <cstring>
#include <string>
#include <unordered_map>
#include <utility>
#include <vector>

namespace lk {
namespace re {
namespace {

#include "unicode_tables.inc"

constexpr uint32_t kMaxRune = 0x10FFFF;
constexpr uint32_t kBadRune = 0x110000;   // an invalid UTF-8 byte of the text: in no class
constexpr int kMaxRepeat = 1000;          // RE2: counted repetition limit (and of nested products)
constexpr size_t kMaxInst = 400000;       // RE2 fails to compile programs beyond its memory budget
constexpr size_t kMaxDfaStates = 4096;    // lazy DFA cache (reset when full, as RE2 does)

using Range = std::pair<uint32_t, uint32_t>;
using Ranges = std::vector<Range>;

[[noreturn]] void syntax(const std::string& m) { throw RegexError(false, m); }
[[noreturn]] void unsupported(const std::string& m) { throw RegexError(true, m); }

void normalize(Ranges& r) {
  std::sort(r.begin(), r.end());
  Ranges out;
  for (auto& x : r) {
    if (!out.empty() && x.first <= out.back().second + 1) out.back().second = std::max(out.back().second, x.second);
    else out.push_back(x);
  }
  r.swap(out);
}

Ranges negate(const Ranges& in) {   // in: normalized
  Ranges out;
  uint32_t next = 0;
  for (auto& x : in) {
    if (x.first > next) out.emplace_back(next, x.first - 1);
    next = x.second + 1;
  }
  if (next <= kMaxRune) out.emplace_back(next, kMaxRune);
  return out;
}

// [lo, hi] plus every code point fold-equivalent to one in it (RE2 AddFoldedRange).
void add_folded(Ranges& out, uint32_t lo, uint32_t hi) {
  out.emplace_back(lo, hi);
  const size_t n = sizeof(kFoldNext) / sizeof(kFoldNext[0]);
  const uint32_t(*b)[2] = std::lower_bound(kFoldNext, kFoldNext + n, lo,
                                           [](const uint32_t(&e)[2], uint32_t v) { return e[0] < v; });
  for (; b != kFoldNext + n && (*b)[0] <= hi; ++b) {
    uint32_t c = (*b)[1];
    for (int guard = 0; c != (*b)[0] && guard < 8; guard++) {   // walk the orbit
      if (c < lo || c > hi) out.emplace_back(c, c);
      const uint32_t(*e)[2] = std::lower_bound(kFoldNext, kFoldNext + n, c,
                                               [](const uint32_t(&x)[2], uint32_t v) { return x[0] < v; });
      if (e == kFoldNext + n || (*e)[0] != c) break;
      c = (*e)[1];
    }
  }
}

struct Flags {
  bool fold = false;    // i
  bool multi = false;   // m: ^ $ at line boundaries
  bool dotnl = false;   // s
};

// ---- UTF-8 ----
// Decode one code point; invalid sequences (bad lead/continuation, overlong, > U+10FFFF) -> kBadRune, 1 byte.
inline uint32_t utf8(const uint8_t* s, size_t n, size_t& len) {
  const uint8_t c = s[0];
  len = 1;
  if (c < 0x80) return c;
  if (c < 0xC2) return kBadRune;
  if (c < 0xE0) {
    if (n < 2 || (s[1] & 0xC0) != 0x80) return kBadRune;
    len = 2;
    return (uint32_t(c & 0x1F) << 6) | (s[1] & 0x3F);
  }
  if (c < 0xF0) {
    if (n < 3 || (s[1] & 0xC0) != 0x80 || (s[2] & 0xC0) != 0x80) return kBadRune;
    const uint32_t r = (uint32_t(c & 0x0F) << 12) | (uint32_t(s[1] & 0x3F) << 6) | (s[2] & 0x3F);
    if (r < 0x800) return kBadRune;
    len = 3;
    return r;
  }
  if (c < 0xF5) {
    if (n < 4 || (s[1] & 0xC0) != 0x80 || (s[2] & 0xC0) != 0x80 || (s[3] & 0xC0) != 0x80) return kBadRune;
    const uint32_t r = (uint32_t(c & 0x07) << 18) | (uint32_t(s[1] & 0x3F) << 12) | (uint32_t(s[2] & 0x3F) << 6) |
                       (s[3] & 0x3F);
    if (r < 0x10000 || r > kMaxRune) return kBadRune;
    len = 4;
    return r;
  }
  return kBadRune;
}

inline bool is_word(uint32_t c) {
  return (c >= '0' && c <= '9') || (c >= 'A' && c <= 'Z') || (c >= 'a' && c <= 'z') || c == '_';
}

// ---- parse tree ----
enum AssertKind : uint8_t { A_BOT, A_EOT, A_BOL, A_EOL, A_WB, A_NWB };

struct Node {
  enum Kind : uint8_t { EMPTY, CLASS, CAT, ALT, REP, ASSERT } k = EMPTY;
  uint8_t a = 0;          // ASSERT kind
  int cls = -1;           // CLASS: index into Parser::classes
  int min = 0, max = 0;   // REP; max -1 = unbounded
  std::vector<int> kids;
};

struct PosixGroup {
  const char* name;
  Ranges r;
};

const std::vector<PosixGroup>& posix_groups() {
  static const std::vector<PosixGroup> g = {
      {"alnum", {{'0', '9'}, {'A', 'Z'}, {'a', 'z'}}},
      {"alpha", {{'A', 'Z'}, {'a', 'z'}}},
      {"ascii", {{0, 0x7F}}},
      {"blank", {{'\t', '\t'}, {' ', ' '}}},
      {"cntrl", {{0, 0x1F}, {0x7F, 0x7F}}},
      {"digit", {{'0', '9'}}},
      {"graph", {{'!', '~'}}},
      {"lower", {{'a', 'z'}}},
      {"print", {{' ', '~'}}},
      {"punct", {{'!', '/'}, {':', '@'}, {'[', '`'}, {'{', '~'}}},
      {"space", {{'\t', '\r'}, {' ', ' '}}},
      {"upper", {{'A', 'Z'}}},
      {"word", {{'0', '9'}, {'A', 'Z'}, {'a', 'z'}, {'_', '_'}}},
      {"xdigit", {{'0', '9'}, {'A', 'F'}, {'a', 'f'}}},
  };
  return g;
}

// Unicode script names RE2 knows (\p{Greek} ...): valid syntax this matcher does not implement.
bool is_script_name(const std::string& n) {
  static const char* const names[] = {
      "Adlam", "Ahom", "Anatolian_Hieroglyphs", "Arabic", "Armenian", "Avestan", "Balinese", "Bamum", "Bassa_Vah",
      "Batak", "Bengali", "Bhaiksuki", "Bopomofo", "Brahmi", "Braille", "Buginese", "Buhid", "Canadian_Aboriginal",
      "Carian", "Caucasian_Albanian", "Chakma", "Cham", "Cherokee", "Chorasmian", "Common", "Coptic", "Cuneiform",
      "Cypriot", "Cypro_Minoan", "Cyrillic", "Deseret", "Devanagari", "Dives_Akuru", "Dogra", "Duployan",
      "Egyptian_Hieroglyphs", "Elbasan", "Elymaic", "Ethiopic", "Georgian", "Glagolitic", "Gothic", "Grantha", "Greek",
      "Gujarati", "Gunjala_Gondi", "Gurmukhi", "Han", "Hangul", "Hanifi_Rohingya", "Hanunoo", "Hatran", "Hebrew",
      "Hiragana", "Imperial_Aramaic", "Inherited", "Inscriptional_Pahlavi", "Inscriptional_Parthian", "Javanese",
      "Kaithi", "Kannada", "Katakana", "Kawi", "Kayah_Li", "Kharoshthi", "Khitan_Small_Script", "Khmer", "Khojki",
      "Khudawadi", "Lao", "Latin", "Lepcha", "Limbu", "Linear_A", "Linear_B", "Lisu", "Lycian", "Lydian", "Mahajani",
      "Makasar", "Malayalam", "Mandaic", "Manichaean", "Marchen", "Masaram_Gondi", "Medefaidrin", "Meetei_Mayek",
      "Mende_Kikakui", "Meroitic_Cursive", "Meroitic_Hieroglyphs", "Miao", "Modi", "Mongolian", "Mro", "Multani",
      "Myanmar", "Nabataean", "Nag_Mundari", "Nandinagari", "New_Tai_Lue", "Newa", "Nko", "Nushu", "Nyiakeng_Puachue_Hmong",
      "Ogham", "Ol_Chiki", "Old_Hungarian", "Old_Italic", "Old_North_Arabian", "Old_Permic", "Old_Persian",
      "Old_Sogdian", "Old_South_Arabian", "Old_Turkic", "Old_Uyghur", "Oriya", "Osage", "Osmanya", "Pahawh_Hmong",
      "Palmyrene", "Pau_Cin_Hau", "Phags_Pa", "Phoenician", "Psalter_Pahlavi", "Rejang", "Runic", "Samaritan",
      "Saurashtra", "Sharada", "Shavian", "Siddham", "SignWriting", "Sinhala", "Sogdian", "Sora_Sompeng", "Soyombo",
      "Sundanese", "Syloti_Nagri", "Syriac", "Tagalog", "Tagbanwa", "Tai_Le", "Tai_Tham", "Tai_Viet", "Takri", "Tamil",
      "Tangsa", "Tangut", "Telugu", "Thaana", "Thai", "Tibetan", "Tifinagh", "Tirhuta", "Toto", "Ugaritic", "Vai",
      "Vithkuqi", "Wancho", "Warang_Citi", "Yezidi", "Yi", "Zanabazar_Square"};
  for (const char* s : names)
    if (n == s) return true;
  return false;
}

class Parser {
 public:
  Parser(const std::string& p, bool fold) : s_(p) { flags_.fold = fold; }

  int parse() {
    const int root = parse_alt();
    if (pos_ < s_.size()) syntax("unexpected ): " + s_);   // parse_alt stops only at an unmatched ')'
    return root;
  }

  std::vector<Node> nodes;
  std::vector<Ranges> classes;

 private:
  const std::string& s_;
  size_t pos_ = 0;
  Flags flags_;
  int depth_ = 0;

  bool eof() const { return pos_ >= s_.size(); }
  char peek(size_t k = 0) const { return pos_ + k < s_.size() ? s_[pos_ + k] : '\0'; }

  int add(Node n) {
    nodes.push_back(std::move(n));
    return int(nodes.size() - 1);
  }
  int add_class(Ranges r) {
    normalize(r);
    classes.push_back(std::move(r));
    Node n;
    n.k = Node::CLASS;
    n.cls = int(classes.size() - 1);
    return add(std::move(n));
  }
  int add_assert(AssertKind a) {
    Node n;
    n.k = Node::ASSERT;
    n.a = a;
    return add(std::move(n));
  }

  uint32_t next_rune() {   // from the pattern; invalid UTF-8 is an RE2 syntax error
    size_t len;
    const uint32_t r = utf8(reinterpret_cast<const uint8_t*>(s_.data()) + pos_, s_.size() - pos_, len);
    if (r == kBadRune) syntax("invalid UTF-8 in regex");
    pos_ += len;
    return r;
  }

  int literal(uint32_t r) {
    Ranges rr;
    if (flags_.fold) add_folded(rr, r, r);
    else rr.emplace_back(r, r);
    return add_class(std::move(rr));
  }

  // a range of an explicit class item / group under the current flags (RE2 AddRangeFlags with ClassNL)
  void add_range(Ranges& out, uint32_t lo, uint32_t hi) const {
    if (flags_.fold) add_folded(out, lo, hi);
    else out.emplace_back(lo, hi);
  }
  // a named group (Perl, POSIX, Unicode) with sign: folded positive set, negated when sign < 0 (RE2 AddUGroup)
  void add_group(Ranges& out, const Ranges& g, bool negated) const {
    Ranges pos;
    for (auto& x : g) add_range(pos, x.first, x.second);
    normalize(pos);
    if (negated) pos = negate(pos);
    out.insert(out.end(), pos.begin(), pos.end());
  }

  int parse_alt() {
    std::vector<int> alts{parse_concat()};
    while (peek() == '|' && !eof()) {
      pos_++;
      alts.push_back(parse_concat());
    }
    if (alts.size() == 1) return alts[0];
    Node n;
    n.k = Node::ALT;
    n.kids = std::move(alts);
    return add(std::move(n));
  }

  int parse_concat() {
    std::vector<int> items;
    while (!eof() && peek() != '|' && peek() != ')') {
      int atom = parse_atom(items);
      if (atom < 0) {   // flag group / empty \Q\E: pushes nothing, so a repetition after it applies to the previous item
        if (!items.empty()) items.back() = parse_repeat(items.back());
        continue;
      }
      atom = parse_repeat(atom);
      items.push_back(atom);
    }
    if (items.size() == 1) return items[0];
    Node n;
    n.k = items.empty() ? Node::EMPTY : Node::CAT;
    n.kids = std::move(items);
    return add(std::move(n));
  }

  static bool parse_int(const std::string& s, size_t& p, int& v) {
    if (p >= s.size() || !isdigit(static_cast<unsigned char>(s[p]))) return false;
    if (p + 1 < s.size() && s[p] == '0' && isdigit(static_cast<unsigned char>(s[p + 1]))) return false;   // no leading 0
    long n = 0;
    while (p < s.size() && isdigit(static_cast<unsigned char>(s[p]))) {
      if (n >= 100000000) return false;
      n = n * 10 + (s[p] - '0');
      p++;
    }
    v = int(n);
    return true;
  }
  // {n} {n,} {n,m} at pos_; on success advances pos_ past '}'
  bool maybe_counted(int& lo, int& hi) {
    if (peek() != '{') return false;
    size_t p = pos_ + 1;
    if (!parse_int(s_, p, lo)) return false;
    if (p < s_.size() && s_[p] == ',') {
      p++;
      if (p < s_.size() && s_[p] == '}') hi = -1;
      else if (!parse_int(s_, p, hi)) return false;
    } else {
      hi = lo;
    }
    if (p >= s_.size() || s_[p] != '}') return false;
    pos_ = p + 1;
    return true;
  }

  // RE2 RepetitionWalker: the product of nested counted repetitions may not exceed kMaxRepeat.
  int rep_budget(int n, int budget) const {
    const Node& x = nodes[size_t(n)];
    if (x.k == Node::REP && !(x.min == 0 && x.max == -1) && !(x.min == 1 && x.max == -1) && !(x.min == 0 && x.max == 1)) {
      int m = x.max < 0 ? x.min : x.max;
      if (m > 0) budget /= m;
    }
    int out = budget;
    for (int k : x.kids) out = std::min(out, rep_budget(k, budget));
    return out;
  }

  int parse_repeat(int atom) {
    bool repeated = false;
    for (;;) {
      const char c = peek();
      int lo = 0, hi = 0;
      bool counted = false;
      if (eof()) break;
      if (c == '*') { lo = 0; hi = -1; pos_++; }
      else if (c == '+') { lo = 1; hi = -1; pos_++; }
      else if (c == '?') { lo = 0; hi = 1; pos_++; }
      else if (c == '{') {
        if (!maybe_counted(lo, hi)) break;   // a literal '{'
        counted = true;
      } else {
        break;
      }
      if (peek() == '?' && !eof()) pos_++;   // non-greedy: same language
      if (repeated) syntax("bad repetition operator in " + s_);
      repeated = true;
      if (counted && ((hi != -1 && hi < lo) || lo > kMaxRepeat || hi > kMaxRepeat))
        syntax("bad repetition operator in " + s_);
      Node n;
      n.k = Node::REP;
      n.min = lo;
      n.max = hi;
      n.kids = {atom};
      atom = add(std::move(n));
      if (counted && (lo >= 2 || hi >= 2) && rep_budget(atom, kMaxRepeat) == 0)
        syntax("bad repetition operator (nested counts) in " + s_);
    }
    return atom;
  }

  // Perl classes \d \D \s \S \w \W (ASCII) at pos_ ('\\' already checked); false if not one
  bool maybe_perl(Ranges& out) {
    if (peek() != '\\') return false;
    const char c = peek(1);
    static const Ranges d = {{'0', '9'}}, s = {{'\t', '\n'}, {'\f', '\r'}, {' ', ' '}},
                        w = {{'0', '9'}, {'A', 'Z'}, {'_', '_'}, {'a', 'z'}};
    const Ranges* g = nullptr;
    switch (c) {
      case 'd': case 'D': g = &d; break;
      case 's': case 'S': g = &s; break;
      case 'w': case 'W': g = &w; break;
      default: return false;
    }
    pos_ += 2;
    add_group(out, *g, isupper(static_cast<unsigned char>(c)) != 0);
    return true;
  }

  // \pN \p{Name} \PN \P{^Name}; false if not at one
  bool maybe_unicode(Ranges& out) {
    if (peek() != '\\' || (peek(1) != 'p' && peek(1) != 'P')) return false;
    bool neg = peek(1) == 'P';
    pos_ += 2;
    if (eof()) syntax("invalid character class range in " + s_);
    std::string name;
    if (peek() == '{') {
      const size_t e = s_.find('}', pos_);
      if (e == std::string::npos) syntax("invalid character class range in " + s_);
      name = s_.substr(pos_ + 1, e - pos_ - 1);
      pos_ = e + 1;
    } else {
      const size_t p0 = pos_;
      next_rune();
      name = s_.substr(p0, pos_ - p0);
    }
    if (!name.empty() && name[0] == '^') {
      neg = !neg;
      name.erase(0, 1);
    }
    if (name == "Any") {
      add_group(out, Ranges{{0, kMaxRune}}, neg);
      return true;
    }
    for (const UGroup& g : kUGroups) {
      if (name != g.name) continue;
      Ranges r;
      for (size_t i = 0; i < g.n; i++) r.emplace_back(g.ranges[i][0], g.ranges[i][1]);
      add_group(out, r, neg);
      return true;
    }
    if (is_script_name(name)) unsupported("Unicode script class \\p{" + name + "} is not implemented");
    syntax("invalid character class range: \\p{" + name + "}");
  }

  // RE2 ParseEscape: one code point from an escape at pos_ (which holds '\\')
  uint32_t parse_escape() {
    pos_++;   // '\\'
    if (eof()) syntax("trailing \\ in " + s_);
    const uint32_t c = next_rune();
    if (c >= '1' && c <= '7') {
      if (eof() || peek() < '0' || peek() > '7') syntax("invalid escape sequence (backreference) in " + s_);
    }
    if (c >= '0' && c <= '7') {
      uint32_t code = c - '0';
      for (int k = 0; k < 2 && !eof() && peek() >= '0' && peek() <= '7'; k++) code = code * 8 + uint32_t(s_[pos_++] - '0');
      return code;
    }
    auto hexv = [](uint32_t h) -> int {
      if (h >= '0' && h <= '9') return int(h - '0');
      if (h >= 'a' && h <= 'f') return int(h - 'a' + 10);
      if (h >= 'A' && h <= 'F') return int(h - 'A' + 10);
      return -1;
    };
    switch (c) {
      case 'x': {
        if (eof()) syntax("invalid escape sequence in " + s_);
        uint32_t h = next_rune();
        if (h == '{') {
          int nhex = 0;
          uint32_t code = 0;
          if (eof()) syntax("invalid escape sequence in " + s_);
          h = next_rune();
          while (hexv(h) >= 0) {
            nhex++;
            code = code * 16 + uint32_t(hexv(h));
            if (code > kMaxRune || eof()) syntax("invalid escape sequence in " + s_);
            h = next_rune();
          }
          if (h != '}' || nhex == 0) syntax("invalid escape sequence in " + s_);
          return code;
        }
        if (eof()) syntax("invalid escape sequence in " + s_);
        const uint32_t h2 = next_rune();
        if (hexv(h) < 0 || hexv(h2) < 0) syntax("invalid escape sequence in " + s_);
        return uint32_t(hexv(h) * 16 + hexv(h2));
      }
      case 'a': return 7;
      case 'f': return 12;
      case 'n': return 10;
      case 'r': return 13;
      case 't': return 9;
      case 'v': return 11;
      default: break;
    }
    if (c < 0x80 && !isalnum(static_cast<int>(c))) return c;   // escaped punctuation (and \_) is itself
    syntax("invalid escape sequence in " + s_);
  }

  int parse_class() {
    pos_++;   // '['
    bool neg = false;
    if (peek() == '^' && !eof()) {
      neg = true;
      pos_++;
    }
    Ranges cc;
    bool first = true;
    while (!eof() && (peek() != ']' || first)) {
      first = false;
      if (peek() == '[' && peek(1) == ':') {   // [:alpha:] [:^alpha:]
        const size_t e = s_.find(":]", pos_ + 2);
        if (e != std::string::npos) {
          std::string name = s_.substr(pos_ + 2, e - pos_ - 2);
          bool pneg = false;
          if (!name.empty() && name[0] == '^') {
            pneg = true;
            name.erase(0, 1);
          }
          const PosixGroup* g = nullptr;
          for (auto& x : posix_groups())
            if (name == x.name) g = &x;
          if (!g) syntax("invalid character class range: [:" + name + ":]");
          pos_ = e + 2;
          add_group(cc, g->r, pneg);
          continue;
        }
      }
      if (peek() == '\\' && (peek(1) == 'p' || peek(1) == 'P') && pos_ + 2 < s_.size() && maybe_unicode(cc)) continue;
      if (maybe_perl(cc)) continue;
      uint32_t lo = peek() == '\\' ? parse_escape() : next_rune(), hi = lo;
      if (peek() == '-' && pos_ + 1 < s_.size() && peek(1) != ']') {
        pos_++;
        hi = peek() == '\\' ? parse_escape() : next_rune();
        if (hi < lo) syntax("invalid character class range in " + s_);
      }
      add_range(cc, lo, hi);
    }
    if (eof()) syntax("missing closing ] in " + s_);
    pos_++;   // ']'
    normalize(cc);
    if (neg) cc = negate(cc);
    return add_class(std::move(cc));
  }

  int group(bool capture_ok) {
    const Flags saved = flags_;
    if (++depth_ > 1000) syntax("regex nests too deeply");
    const int inner = parse_alt();
    if (peek() != ')' || eof()) syntax("missing ): " + s_);
    pos_++;
    depth_--;
    flags_ = saved;
    (void)capture_ok;
    return inner;
  }

  // one atom; -1 when the construct matches nothing to repeat (a flag group)
  int parse_atom(std::vector<int>& items) {
    const char c = peek();
    switch (c) {
      case '(': {
        if (peek(1) != '?') {
          pos_++;
          return group(true);
        }
        // named capture (?P<name>re) / (?<name>re)
        if (peek(2) == 'P' || (peek(2) == '<' && peek(3) != '=' && peek(3) != '!')) {
          const size_t nb = peek(2) == 'P' ? pos_ + 3 : pos_ + 2;
          if (peek(2) == 'P' && (nb >= s_.size() || s_[nb] != '<')) syntax("invalid or unsupported Perl syntax in " + s_);
          const size_t e = s_.find('>', nb);
          if (e == std::string::npos) syntax("invalid named capture group in " + s_);
          const std::string name = s_.substr(nb + 1, e - nb - 1);
          if (name.empty() || !std::all_of(name.begin(), name.end(), [](char ch) {
                return isalnum(static_cast<unsigned char>(ch)) || ch == '_';
              }))
            syntax("invalid named capture group in " + s_);
          pos_ = e + 1;
          return group(true);
        }
        // flags: (?i) (?i-s) (?i:re) (?:re)
        size_t p = pos_ + 2;
        Flags nf = flags_;
        bool neg = false, sawneg = false, sawflag = false;
        for (;;) {
          if (p >= s_.size()) syntax("missing ) / invalid Perl flags in " + s_);
          const char f = s_[p++];
          if (f == 'i' || f == 'm' || f == 's' || f == 'U') {
            sawflag = true;
            if (f == 'i') nf.fold = !neg;
            if (f == 'm') nf.multi = !neg;
            if (f == 's') nf.dotnl = !neg;
            continue;
          }
          if (f == '-') {
            if (sawneg) syntax("invalid or unsupported Perl syntax in " + s_);
            sawneg = neg = true;
            sawflag = false;
            continue;
          }
          if (f == ':' || f == ')') {
            if (neg && !sawflag) syntax("invalid or unsupported Perl syntax in " + s_);
            pos_ = p;
            if (f == ')') {   // flags for the rest of the enclosing group
              flags_ = nf;
              return -1;
            }
            const Flags saved = flags_;
            flags_ = nf;
            const int inner = group(false);
            flags_ = saved;
            return inner;
          }
          syntax("invalid or unsupported Perl syntax in " + s_);
        }
      }
      case '*':
      case '+':
      case '?':
        syntax("missing argument to repetition operator in " + s_);
      case '{': {
        int lo, hi;
        const size_t save = pos_;
        if (maybe_counted(lo, hi)) syntax("missing argument to repetition operator in " + s_);
        pos_ = save + 1;
        return literal('{');
      }
      case '[':
        return parse_class();
      case '.': {
        pos_++;
        Ranges r;
        if (flags_.dotnl) r.emplace_back(0, kMaxRune);
        else r = {{0, '\n' - 1}, {'\n' + 1, kMaxRune}};
        return add_class(std::move(r));
      }
      case '^':
        pos_++;
        return add_assert(flags_.multi ? A_BOL : A_BOT);
      case '$':
        pos_++;
        return add_assert(flags_.multi ? A_EOL : A_EOT);
      case '\\': {
        const char e = peek(1);
        if (e == 'b' || e == 'B') {
          pos_ += 2;
          return add_assert(e == 'b' ? A_WB : A_NWB);
        }
        if (e == 'A' || e == 'z') {
          pos_ += 2;
          return add_assert(e == 'A' ? A_BOT : A_EOT);
        }
        if (e == 'C') unsupported("\\C (any byte) is not implemented");
        if (e == 'Q') {   // \Q...\E literal text; a following repetition applies to its last code point
          pos_ += 2;
          int last = -1;
          while (!eof()) {
            if (peek() == '\\' && peek(1) == 'E') {
              pos_ += 2;
              break;
            }
            if (last >= 0) items.push_back(last);
            last = literal(next_rune());
          }
          return last;
        }
        Ranges r;
        if ((e == 'p' || e == 'P') && maybe_unicode(r)) {
          normalize(r);
          return add_class(std::move(r));
        }
        if (maybe_perl(r)) {
          normalize(r);
          return add_class(std::move(r));
        }
        return literal(parse_escape());
      }
      default:
        return literal(next_rune());
    }
  }
};

// ---- program ----
enum Op : uint8_t { I_CLS, I_SPLIT, I_JMP, I_MATCH, I_ASSERT };

struct Inst {
  Op op;
  uint8_t a = 0;   // assert kind
  int x = 0, y = 0;
  int cls = -1;
};

struct Class {
  uint64_t ascii[2] = {0, 0};
  Ranges r;
  bool has(uint32_t c) const {
    if (c < 128) return (ascii[c >> 6] >> (c & 63)) & 1u;
    size_t lo = 0, hi = r.size();
    while (lo < hi) {
      const size_t m = (lo + hi) / 2;
      if (r[m].second < c) lo = m + 1;
      else hi = m;
    }
    return lo < r.size() && r[lo].first <= c;
  }
};

class Compiler {
 public:
  Compiler(const std::vector<Node>& nodes, std::vector<Inst>& prog) : nodes_(nodes), prog_(prog) {}
  void emit(int n) {
    const Node& x = nodes_[size_t(n)];
    switch (x.k) {
      case Node::EMPTY: break;
      case Node::CLASS: push(Inst{I_CLS, 0, 0, 0, x.cls}); break;
      case Node::ASSERT: push(Inst{I_ASSERT, x.a, 0, 0, -1}); break;
      case Node::CAT:
        for (int k : x.kids) emit(k);
        break;
      case Node::ALT: {
        std::vector<size_t> jumps;
        for (size_t i = 0; i + 1 < x.kids.size(); i++) {
          const size_t sp = push(Inst{I_SPLIT, 0, 0, 0, -1});
          prog_[sp].x = int(prog_.size());
          emit(x.kids[i]);
          jumps.push_back(push(Inst{I_JMP, 0, 0, 0, -1}));
          prog_[sp].y = int(prog_.size());
        }
        emit(x.kids.back());
        for (size_t j : jumps) prog_[j].x = int(prog_.size());
        break;
      }
      case Node::REP: {
        const int kid = x.kids[0];
        for (int i = 0; i < x.min; i++) emit(kid);
        if (x.max < 0) {   // kid*
          const size_t sp = push(Inst{I_SPLIT, 0, 0, 0, -1});
          prog_[sp].x = int(prog_.size());
          emit(kid);
          push(Inst{I_JMP, 0, int(sp), 0, -1});
          prog_[sp].y = int(prog_.size());
        } else {           // (kid(kid(...)?)?)?  max - min optional copies
          std::vector<size_t> splits;
          for (int i = x.min; i < x.max; i++) {
            const size_t sp = push(Inst{I_SPLIT, 0, 0, 0, -1});
            prog_[sp].x = int(prog_.size());
            splits.push_back(sp);
            emit(kid);
          }
          for (size_t sp : splits) prog_[sp].y = int(prog_.size());
        }
        break;
      }
    }
  }

 private:
  size_t push(Inst i) {
    if (prog_.size() >= kMaxInst) throw RegexError(false, "pattern too large - compile failed");
    prog_.push_back(i);
    return prog_.size() - 1;
  }
  const std::vector<Node>& nodes_;
  std::vector<Inst>& prog_;
};

}  // namespace

struct Regex::Impl {
  std::vector<Inst> prog;
  std::vector<Class> classes;
  bool dfa_ok = true;   // no line / word-boundary assertions: the lazy DFA applies

  // ---- closure (shared by the DFA builder and the NFA simulation) ----
  std::vector<uint32_t> mark;   // generation per pc
  uint32_t gen = 0;
  std::vector<int> stack;

  struct Ctx {
    bool bot, eot, bol, eol, wb;
    bool keep_eot;   // DFA: do not evaluate EOT, keep the assert pc in the kernel
  };

  bool assert_ok(uint8_t a, const Ctx& c) const {
    switch (a) {
      case A_BOT: return c.bot;
      case A_EOT: return c.eot;
      case A_BOL: return c.bol;
      case A_EOL: return c.eol;
      case A_WB: return c.wb;
      default: return !c.wb;
    }
  }

  void next_gen() {
    if (++gen == 0) {
      std::fill(mark.begin(), mark.end(), 0u);
      gen = 1;
    }
  }
  // Add the closure of pc to `out` (kernel pcs: CLS, MATCH, and with keep_eot pending EOT asserts).
  void closure(int pc0, const Ctx& c, std::vector<int>& out) {
    stack.push_back(pc0);
    while (!stack.empty()) {
      const int pc = stack.back();
      stack.pop_back();
      if (mark[size_t(pc)] == gen) continue;
      mark[size_t(pc)] = gen;
      const Inst& in = prog[size_t(pc)];
      switch (in.op) {
        case I_CLS:
        case I_MATCH: out.push_back(pc); break;
        case I_JMP: stack.push_back(in.x); break;
        case I_SPLIT:
          stack.push_back(in.y);
          stack.push_back(in.x);
          break;
        case I_ASSERT:
          if (c.keep_eot && in.a == A_EOT) out.push_back(pc);
          else if (assert_ok(in.a, c)) stack.push_back(pc + 1);
          break;
      }
    }
  }

  // ---- lazy DFA (dfa_ok programs: only BOT / EOT assertions) ----
  struct DState {
    std::vector<int> pcs;     // sorted kernel
    bool match = false;
    int8_t end_match = -1;    // lazily: MATCH reachable through pending EOT asserts at the end of the text
    int ascii[128];
  };
  std::vector<DState> states;
  std::unordered_map<std::string, int> index;
  std::unordered_map<uint64_t, int> wide;   // (state << 21 | rune) -> state for runes >= 128
  std::vector<int> restart;                  // closure of pc 0 away from the text start
  std::vector<int> tmp;

  int intern(std::vector<int>& pcs) {
    std::sort(pcs.begin(), pcs.end());
    pcs.erase(std::unique(pcs.begin(), pcs.end()), pcs.end());
    std::string key(reinterpret_cast<const char*>(pcs.data()), pcs.size() * sizeof(int));
    auto it = index.find(key);
    if (it != index.end()) return it->second;
    if (states.size() >= kMaxDfaStates) return -1;
    DState s;
    s.pcs = pcs;
    for (int pc : pcs)
      if (prog[size_t(pc)].op == I_MATCH) s.match = true;
    std::fill(std::begin(s.ascii), std::end(s.ascii), -1);
    states.push_back(std::move(s));
    index.emplace(std::move(key), int(states.size() - 1));
    return int(states.size() - 1);
  }

  void reset_dfa() {
    states.clear();
    index.clear();
    wide.clear();
  }

  int step(int s, uint32_t c) {
    if (c < 128) {
      const int t = states[size_t(s)].ascii[c];
      if (t >= 0) return t;
    } else {
      auto it = wide.find((uint64_t(s) << 21) | c);
      if (it != wide.end()) return it->second;
    }
    tmp.clear();
    next_gen();
    const Ctx ctx{false, false, false, false, false, true};
    const std::vector<int> pcs = states[size_t(s)].pcs;   // copy: states may reallocate
    for (int pc : pcs) {
      const Inst& in = prog[size_t(pc)];
      if (in.op == I_CLS && classes[size_t(in.cls)].has(c)) closure(pc + 1, ctx, tmp);
    }
    closure(0, ctx, tmp);   // unanchored: a match may start at the next position
    int t = intern(tmp);
    if (t < 0) {            // cache full: start over from this state's kernel
      std::vector<int> keep = tmp;
      reset_dfa();
      t = intern(keep);
      return t;             // (the caller re-reads its state index)
    }
    if (c < 128) states[size_t(s)].ascii[c] = t;
    else wide.emplace((uint64_t(s) << 21) | c, t);
    return t;
  }

  bool end_match(int s, bool bot) {
    DState& st = states[size_t(s)];
    if (!bot && st.end_match >= 0) return st.end_match != 0;
    tmp.clear();
    next_gen();
    const Ctx ctx{bot, true, false, false, false, false};
    const std::vector<int> pcs = st.pcs;
    for (int pc : pcs)
      if (prog[size_t(pc)].op == I_ASSERT) closure(pc + 1, ctx, tmp);
    bool m = false;
    for (int pc : tmp) m |= prog[size_t(pc)].op == I_MATCH;
    if (!bot) states[size_t(s)].end_match = m ? 1 : 0;
    return m;
  }

  int start_state() {
    tmp.clear();
    next_gen();
    closure(0, Ctx{true, false, false, false, false, true}, tmp);
    return intern(tmp);
  }

  bool dfa_search(const uint8_t* s, size_t n) {
    if (states.empty()) reset_dfa();
    int st = start_state();
    if (st < 0) {
      reset_dfa();
      st = start_state();
    }
    if (states[size_t(st)].match) return true;
    size_t i = 0;
    while (i < n) {
      uint32_t c;
      size_t len = 1;
      if (s[i] < 0x80) c = s[i];
      else c = utf8(s + i, n - i, len);
      const size_t before = states.size();
      st = step(st, c);
      (void)before;
      if (states[size_t(st)].match) return true;
      i += len;
    }
    return end_match(st, n == 0);
  }

  // RE2 searches bytes: an unanchored match may start inside a multi-byte character, where only empty-width
  // paths can succeed (no class matches a continuation byte) and the context is: not at a text / line edge,
  // no word boundary (bytes >= 0x80 are non-word).  E.g. \\B matches inside "é".
  int mid_char_match = -1;
  bool mid_match() {
    if (mid_char_match < 0) {
      tmp.clear();
      next_gen();
      closure(0, Ctx{false, false, false, false, false, false}, tmp);
      mid_char_match = 0;
      for (int pc : tmp) mid_char_match |= prog[size_t(pc)].op == I_MATCH;
    }
    return mid_char_match != 0;
  }

  // ---- NFA simulation (any program) ----
  bool nfa_search(const uint8_t* s, size_t n) {
    std::vector<int> cur, nxt;
    size_t len0 = 0;
    uint32_t prev = kBadRune;   // "no character"
    uint32_t c = n ? utf8(s, n, len0) : kBadRune;
    size_t i = 0;
    auto ctx_at = [&](size_t pos, uint32_t p, uint32_t nx) {
      Ctx x;
      x.bot = pos == 0;
      x.eot = pos == n;
      x.bol = pos == 0 || p == '\n';
      x.eol = pos == n || nx == '\n';
      x.wb = (pos > 0 && is_word(p)) != (pos < n && is_word(nx));
      x.keep_eot = false;
      return x;
    };
    next_gen();
    closure(0, ctx_at(0, prev, c), cur);
    for (;;) {
      for (int pc : cur)
        if (prog[size_t(pc)].op == I_MATCH) return true;
      if (i >= n) return false;
      const size_t len = len0;
      const uint32_t pc_rune = c;
      if (len > 1 && mid_match()) return true;
      i += len;
      prev = pc_rune;
      c = i < n ? utf8(s + i, n - i, len0) : kBadRune;
      const Ctx ctx = ctx_at(i, prev, c);
      nxt.clear();
      next_gen();
      for (int pc : cur) {
        const Inst& in = prog[size_t(pc)];
        if (in.op == I_CLS && classes[size_t(in.cls)].has(pc_rune)) closure(pc + 1, ctx, nxt);
      }
      closure(0, ctx, nxt);
      cur.swap(nxt);
    }
  }
};

Regex::Regex(const std::string& pattern, bool case_insensitive) : p_(new Impl) {
  Parser ps(pattern, case_insensitive);
  const int root = ps.parse();
  Compiler cc(ps.nodes, p_->prog);
  cc.emit(root);
  p_->prog.push_back(Inst{I_MATCH, 0, 0, 0, -1});
  p_->classes.reserve(ps.classes.size());
  for (auto& r : ps.classes) {
    Class k;
    k.r = r;
    for (auto& x : r)
      for (uint32_t c = x.first; c <= std::min<uint32_t>(x.second, 127); c++) k.ascii[c >> 6] |= 1ull << (c & 63);
    p_->classes.push_back(std::move(k));
  }
  for (auto& in : p_->prog)
    if (in.op == I_ASSERT && in.a != A_BOT && in.a != A_EOT) p_->dfa_ok = false;
  p_->mark.assign(p_->prog.size(), 0u);
}

Regex::~Regex() = default;
Regex::Regex(Regex&&) noexcept = default;
Regex& Regex::operator=(Regex&&) noexcept = default;

bool Regex::search(const char* s, size_t n) {
  const uint8_t* u = reinterpret_cast<const uint8_t*>(s);
  return p_->dfa_ok ? p_->dfa_search(u, n) : p_->nfa_search(u, n);
}

size_t Regex::program_size() const { return p_->prog.size(); }

}  // namespace re
}  // namespace lk
