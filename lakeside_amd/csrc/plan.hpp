// PushDownRequest JSON -> evaluation plan (host).
//
// Parsing restates ASTUtils.toBaseExpr / handleFilter / toBinaryClauseFromFilterJsonNode / toBasicFilter
// (core/src/main/scala/com/cardinal/utils/ast/ASTUtils.scala:276-417) and PushDownRequest.fromJson
// (core/src/main/scala/com/cardinal/model/SegmentRequest.scala:45-60).  Semantics of the compiled plan
// follow BaseExpr.generateSql (BaseExpr.scala:108-513); see SURVEY.md Appendix A.
#pragma once
#include <cstdint>
#include <map>
#include <memory>
#include <set>
#include <stdexcept>
#include <string>
#include <vector>

#include "json.hpp"

namespace lk {

extern const char* const kTimestamp;   // "_cardinalhq.timestamp"  Commons.scala:55
extern const char* const kValue;       // "_cardinalhq.value"      Commons.scala:57
extern const char* const kName;        // "_cardinalhq.name"       Commons.scala:47

struct FilterNode {
  enum Kind { LEAF, AND, OR, NOT } kind = LEAF;
  // leaf
  std::string k;
  std::vector<std::string> v;
  std::string op;
  bool extracted = false, computed = false;
  std::string data_type = "string";
  // children
  std::unique_ptr<FilterNode> a, b;
};

struct SegmentReq {
  std::string segment_id;
  std::string dataset;
  std::vector<std::pair<std::string, std::string>> query_tags;   // scalar values only
  int64_t step = 0, start_ts = 0, end_ts = 0;
};

struct Request {
  std::string expr_id, dataset;
  std::unique_ptr<FilterNode> filter;
  bool has_chart = false;
  std::string aggregation = "sum";
  std::vector<std::string> group_bys;
  std::string chart_type = "count";
  std::string rollup;            // empty = none
  bool field_chart = false, has_extract = false, has_compute = false;
  // exemplar queries (no chart): ORDER BY "_cardinalhq.timestamp" <order> LIMIT <limit> (BaseExpr.scala:234-239;
  // defaults ASTUtils.scala:360-361)
  int64_t limit = 1000;
  std::string order = "DESC";
  bool is_tag_query = false, reverse_sort = false;
  std::string tag_name, tag_data_type = "string";   // PushDownRequest.tagDataType (SegmentRequest.scala:55-58)
  std::vector<SegmentReq> segments;
};

struct PlanError : std::runtime_error {
  int code;
  PlanError(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};

Request parse_request(const std::string& json);   // throws PlanError(LK_ERR_ARG, ...)
// A deep copy (the filter tree cloned), e.g. to narrow `segments` to one rank's shard.
Request copy_request(const Request& r);

// Fields: BaseExpr.fieldSet (BaseExpr.scala:648-663): filter keys outside NOT + groupBys.
std::set<std::string> field_set(const Request& r);
// Every leaf key, including those under NOT (the generated SQL references all of them).
void leaf_keys(const FilterNode* n, std::vector<std::string>& out);
// Aggregated column: logs/traces `_cardinalhq.value`; metrics rollup_<rollup|sum> (BaseExpr.scala:349-394).
std::string value_column(const Request& r);
// Column restricted to a finite value list by an eq/in leaf on the top-level AND chain (so every
// passing row carries one of those values); empty if none.
bool restricted_values(const FilterNode* n, const std::string& col, std::vector<std::string>& vals);

}  // namespace lk
