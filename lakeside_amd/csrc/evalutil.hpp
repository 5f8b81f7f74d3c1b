// Plan helpers shared by the aggregate evaluator (eval.cpp) and the exemplar path (exemplar.cpp).
#pragma once
#include <chrono>
#include <cstdint>
#include <string>
#include <unordered_set>
#include <vector>

#include "engine.hpp"
#include "kernels.hpp"
#include "plan.hpp"
#include "regex.hpp"

namespace lk {

struct LeafInfo {
  const FilterNode* node;
  int str;      // string column index
  int index;    // global leaf index
};

// One leaf on one dictionary value (BaseExpr.scala:470-501).
bool leaf_eval(const FilterNode& f, const std::string& s, re::Regex* re, const std::unordered_set<std::string>* set);
// regexp_matches(label, p, 'i') / contains' '.*p.*' as an RE2-semantics matcher (PlanError on a bad pattern).
re::Regex compile_leaf_regex(const FilterNode& l);
// Postfix Kleene program of the filter over numbered leaves.
void postfix(const FilterNode* n, const std::vector<LeafInfo>& leaves, std::vector<uint8_t>& prog);
void collect_leaves(const FilterNode* n, std::vector<const FilterNode*>& out);
// Truth table of a postfix program over L leaves: bit (T | F << L) = TRUE.
std::vector<uint32_t> truth_table(const std::vector<uint8_t>& prog, uint32_t L);
bool null_like(const std::string& s);
// NoisyTagsDropper: tag names dropped from tag-query rows
bool noisy_tag(const std::string& t);
double ms_since(std::chrono::steady_clock::time_point t0);

// Exemplar queries (no chart): exemplar.cpp.
// numtag: a tag query (isTagQuery) whose tag column is numeric -- the same row scan planning (filter, globs,
// union_by_name types), counting passing rows per canonical tag value instead of selecting rows (ex_scan TAGNUM).
// dist: every rank evaluates the segments of its shard (shard[i] == rank; default i % world) as the worker of its pod
// would, and rank 0 folds the ranks' streams (exemplar: Akka mergeSorted in rank order, then query-api's take(limit);
// numeric tag: counts summed per tag text).
int evaluate_exemplar(Engine& E, CallCtx& X, const Request& R, const char* const* paths, size_t n_paths,
                      int glob_size, unsigned flags, bool dist, lk_result* res, const std::string& numtag = std::string(),
                      const int32_t* shard = nullptr);
// Numeric comparison leaves (numleaf.cpp): gt / ge / lt / le; the normalized literal (PlanError(LK_ERR_ARG) where the
// reference's SQL fails); the leaf's interval on numeric filter column `col`.
bool numeric_op(const std::string& op);
double normalized_value(const FilterNode& f);
NumLeaf make_num_leaf(const FilterNode& f, uint32_t col, uint32_t leaf, bool& bad);
// Java 17 Double.toString / Float.toString text (jdtoa.cpp).
std::string java_text(double d);
std::string java_text(float f);

}  // namespace lk
