// extern "C" surface of include/lakeside_regex.h (host-only test/diagnostic library around regex.cpp).
#include <new>
#include <string>

#include "../../include/lakeside_regex.h"
#include "regex.hpp"

struct lkre {
  lk::re::Regex re;
};

namespace {
thread_local std::string t_err;
}

extern "C" {

int lkre_compile(const char* pattern, size_t len, int case_insensitive, lkre** out) {
  if (!out || (!pattern && len)) return -1;
  *out = nullptr;
  try {
    *out = new lkre{lk::re::Regex(std::string(pattern ? pattern : "", len), case_insensitive != 0)};
    return 0;
  } catch (const lk::re::RegexError& e) {
    t_err = e.what();
    return e.unsupported ? -2 : -1;
  } catch (const std::exception& e) {
    t_err = e.what();
    return -1;
  }
}

int lkre_search(lkre* re, const char* text, size_t len) {
  if (!re) return 0;
  return re->re.search(text ? text : "", text ? len : 0) ? 1 : 0;
}

void lkre_free(lkre* re) { delete re; }

const char* lkre_last_error(void) { return t_err.c_str(); }

}  // extern "C"
