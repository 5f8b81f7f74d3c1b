// RE2-semantics regular expressions for the filter leaves `regex` / `contains`.
//
// Reference: BaseExpr.filterSqlAndAccumulateFields compiles `regex` to regexp_matches(label, 'v', 'i') and
// `contains` to regexp_matches(label, '.*v.*', 'i') (core/src/main/scala/com/cardinal/utils/ast/BaseExpr.scala:
// 485-486, 500-501); DuckDB 1.3.2 runs that through RE2: unanchored search (PartialMatch), UTF-8 code points,
// case-insensitive by Unicode simple case folding ('i' = RE2::Options::set_case_sensitive(false)).
//
// This is a from-scratch matcher for that contract: RE2 syntax (Perl-like, no backreferences / lookaround),
// Thompson NFA compiled from the parse tree, run as a lazily built DFA (state = NFA state set, transitions cached
// per code point) with an NFA-simulation fallback for word-boundary / multi-line assertions.  Linear in the text
// for every pattern (no backtracking).  The engine evaluates each leaf once per distinct dictionary value on the
// host, never per row.
//
// Errors: syntax RE2 rejects -> RegexError{unsupported=false}; RE2 syntax this matcher does not implement
// (Unicode script classes \p{Greek}, \C) -> RegexError{unsupported=true}.
#pragma once
#include <cstddef>
#include <cstdint>
#include <memory>
#include <stdexcept>
#include <string>

namespace lk {
namespace re {

struct RegexError : std::runtime_error {
  bool unsupported;
  RegexError(bool u, const std::string& m) : std::runtime_error(m), unsupported(u) {}
};

class Regex {
 public:
  // pattern: RE2 syntax.  case_insensitive: regexp_matches' 'i' option.
  Regex(const std::string& pattern, bool case_insensitive);
  ~Regex();
  Regex(Regex&&) noexcept;
  Regex& operator=(Regex&&) noexcept;
  // RE2::PartialMatch(text, re): does some substring of the UTF-8 text match?  Not thread-safe (the DFA cache
  // grows during searches): one Regex per thread.
  bool search(const char* s, size_t n);
  bool search(const std::string& s) { return search(s.data(), s.size()); }
  size_t program_size() const;

 private:
  struct Impl;
  std::unique_ptr<Impl> p_;
};

}  // namespace re
}  // namespace lk
