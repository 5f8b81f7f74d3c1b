/* lakeside_regex.h — the host-side RE2-semantics matcher behind the `regex` / `contains` filter leaves, as a
 * standalone C ABI (liblakeside_regex.so, no GPU needed).
 *
 * The evaluator (liblakeside_gpu.so) evaluates every regex/contains leaf once per distinct dictionary value
 * with this matcher; this separate library exists so the matcher can be checked on a CPU box against RE2 itself,
 * the engine behind DuckDB's regexp_matches(label, pattern, 'i') that the reference SQL calls
 * (core/src/main/scala/com/cardinal/utils/ast/BaseExpr.scala:485-486, 500-501).
 */
#ifndef LAKESIDE_REGEX_H
#define LAKESIDE_REGEX_H

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct lkre lkre;

/* Compile `pattern` (RE2 syntax; case_insensitive = the 'i' option).  Returns 0 and *out, or
 * -1 (syntax RE2 rejects) / -2 (valid RE2 syntax not implemented here); message in lkre_last_error(). */
int lkre_compile(const char* pattern, size_t len, int case_insensitive, lkre** out);
/* 1 if some substring of the UTF-8 text matches (RE2::PartialMatch), else 0. */
int lkre_search(lkre* re, const char* text, size_t len);
void lkre_free(lkre* re);
const char* lkre_last_error(void);

#ifdef __cplusplus
}
#endif
#endif /* LAKESIDE_REGEX_H */
