#include "plan.hpp"

#include <algorithm>

#include "../../include/lakeside_gpu.h"

namespace lk {

const char* const kTimestamp = "_cardinalhq.timestamp";
const char* const kValue = "_cardinalhq.value";
const char* const kName = "_cardinalhq.name";

static std::unique_ptr<FilterNode> handle_filter(const Json& j);

// ASTUtils.toBasicFilter (ASTUtils.scala:276-288)
static std::unique_ptr<FilterNode> basic_filter(const Json& j) {
  auto n = std::make_unique<FilterNode>();
  n->kind = FilterNode::LEAF;
  const Json* k = j.get("k");
  if (!k || !k->is_str()) throw PlanError(LK_ERR_ARG, "No `k` provided in filter!");
  const Json* op = j.get("op");
  if (!op || !op->is_str()) throw PlanError(LK_ERR_ARG, "No op provided for filter!");
  n->k = k->str;
  n->op = op->str;
  if (const Json* v = j.get("v"); v && v->is_arr())
    for (auto& e : v->arr) n->v.push_back(e.is_str() ? e.str : e.scalar_text());
  if (n->v.empty() && n->op != "exists")
    throw PlanError(LK_ERR_ARG, "No value for key = " + n->k + " provided in filter!");
  if (const Json* x = j.get("extracted"); x && x->kind == Json::Bool) n->extracted = x->b;
  if (const Json* x = j.get("computed"); x && x->kind == Json::Bool) n->computed = x->b;
  if (const Json* x = j.get("dataType"); x && x->is_str()) n->data_type = x->str;
  return n;
}

// ASTUtils.toBinaryClauseFromFilterJsonNode (ASTUtils.scala:379-404): non-textual members in JSON order,
// folded left-associatively.
static std::unique_ptr<FilterNode> binary_clause(const Json& j) {
  const Json* op = j.get("op");
  if (!op) throw PlanError(LK_ERR_ARG, "No `op` provided in binary query clause!");
  std::vector<std::unique_ptr<FilterNode>> kids;
  for (auto& kv : j.obj)
    if (!kv.second.is_str()) kids.push_back(handle_filter(kv.second));
  if (kids.size() < 2) throw PlanError(LK_ERR_ARG, "Atleast two clauses required in a binary clause!");
  std::string o = op->str;
  if (o != "and" && o != "or") throw PlanError(LK_ERR_ARG, "unknown binary op " + o);
  std::unique_ptr<FilterNode> acc = std::move(kids[0]);
  for (size_t i = 1; i < kids.size(); i++) {
    auto n = std::make_unique<FilterNode>();
    n->kind = o == "and" ? FilterNode::AND : FilterNode::OR;
    n->a = std::move(acc);
    n->b = std::move(kids[i]);
    acc = std::move(n);
  }
  return acc;
}

// ASTUtils.handleFilter (ASTUtils.scala:406-417)
static std::unique_ptr<FilterNode> handle_filter(const Json& j) {
  if (!j.is_obj()) throw PlanError(LK_ERR_ARG, "filter must be an object");
  if (const Json* n = j.get("not"); n && !n->is_null()) {
    auto node = std::make_unique<FilterNode>();
    node->kind = FilterNode::NOT;
    node->a = handle_filter(*n);
    return node;
  }
  if (const Json* k = j.get("k"); k && !k->is_null()) return basic_filter(j);
  return binary_clause(j);
}

Request parse_request(const std::string& text) {
  Json p;
  try {
    p = Json::parse(text);
  } catch (const JsonError& e) {
    throw PlanError(LK_ERR_ARG, e.what());
  }
  Request r;
  const Json* be = p.get("baseExpr");
  if (!be || !be->is_obj()) throw PlanError(LK_ERR_ARG, "missing baseExpr");
  // ASTUtils.toBaseExpr (ASTUtils.scala:290-377)
  r.expr_id = be->get("id") && be->get("id")->is_str() ? be->get("id")->str : "_";
  r.dataset = be->get("dataset") && be->get("dataset")->is_str() ? be->get("dataset")->str : "metrics";
  if (const Json* c = be->get("chart"); c && c->is_obj()) {
    r.has_chart = true;
    if (const Json* g = c->get("groupBys"); g && g->is_arr())
      for (auto& e : g->arr) r.group_bys.push_back(e.is_str() ? e.str : e.scalar_text());
    if (const Json* a = c->get("aggregation"); a && a->is_str()) r.aggregation = a->str;
    if (const Json* ro = c->get("rollup"); ro && ro->is_str()) r.rollup = ro->str;
    if (const Json* t = c->get("type"); t && t->is_str()) r.chart_type = t->str;
    if (const Json* f = c->get("fieldName"); f && !f->is_null()) r.field_chart = true;
  }
  if (const Json* x = be->get("extract"); x && !x->is_null()) r.has_extract = true;
  if (const Json* x = be->get("compute"); x && !x->is_null()) r.has_compute = true;
  // ASTUtils.scala:360-361: Option(node.get("order")).map(_.textValue), Option(node.get("limit")).map(_.intValue)
  if (const Json* o = be->get("order"); o && o->is_str()) r.order = o->str;
  if (const Json* l = be->get("limit"))
    r.limit = l->kind == Json::Number ? l->as_i64() : 0;   // JSON null: NullNode.intValue = 0
  const Json* f = be->get("filter");
  if (!f || f->is_null()) throw PlanError(LK_ERR_ARG, "No filter provided!");
  r.filter = handle_filter(*f);
  if (const Json* x = p.get("isTagQuery"); x && x->kind == Json::Bool) r.is_tag_query = x->b;
  if (const Json* td = p.get("tagDataType"); td && td->is_obj()) {   // TagDataType(tagName, dataType)
    if (const Json* n = td->get("tagName"); n && n->is_str()) r.tag_name = n->str;
    if (const Json* d = td->get("dataType"); d && d->is_str()) r.tag_data_type = d->str;
  }
  if (const Json* x = p.get("reverseSort"); x && x->kind == Json::Bool) r.reverse_sort = x->b;
  const Json* segs = p.get("segmentRequests");
  if (!segs || !segs->is_arr()) throw PlanError(LK_ERR_ARG, "missing segmentRequests");
  for (auto& s : segs->arr) {
    SegmentReq q;
    if (const Json* x = s.get("segmentId")) q.segment_id = x->scalar_text();
    q.dataset = s.get("dataset") && s.get("dataset")->is_str() ? s.get("dataset")->str : r.dataset;
    const Json* st = s.get("stepInMillis");
    const Json* a = s.get("startTs");
    const Json* b = s.get("endTs");
    if (!st || !a || !b) throw PlanError(LK_ERR_ARG, "segmentRequest needs stepInMillis/startTs/endTs");
    q.step = st->as_i64();
    q.start_ts = a->as_i64();
    q.end_ts = b->as_i64();
    if (const Json* qt = s.get("queryTags"); qt && qt->is_obj())
      for (auto& kv : qt->obj)
        if (kv.second.kind == Json::String || kv.second.kind == Json::Number || kv.second.kind == Json::Bool)
          q.query_tags.emplace_back(kv.first, kv.second.scalar_text());
    r.segments.push_back(std::move(q));
  }
  return r;
}

static void filter_fields(const FilterNode* n, std::set<std::string>& out) {
  // BaseExpr.filterFieldSet (BaseExpr.scala:652-663): NotClause contributes nothing.
  if (n->kind == FilterNode::LEAF) out.insert(n->k);
  else if (n->kind == FilterNode::AND || n->kind == FilterNode::OR) {
    filter_fields(n->a.get(), out);
    filter_fields(n->b.get(), out);
  }
}

std::set<std::string> field_set(const Request& r) {
  std::set<std::string> s;
  filter_fields(r.filter.get(), s);
  for (auto& g : r.group_bys) s.insert(g);
  return s;
}

void leaf_keys(const FilterNode* n, std::vector<std::string>& out) {
  if (n->kind == FilterNode::LEAF) {
    if (std::find(out.begin(), out.end(), n->k) == out.end()) out.push_back(n->k);
  } else {
    leaf_keys(n->a.get(), out);
    if (n->b) leaf_keys(n->b.get(), out);
  }
}

std::string value_column(const Request& r) {
  if (r.dataset == "metrics") return "rollup_" + (r.rollup.empty() ? std::string("sum") : r.rollup);
  return kValue;
}

bool restricted_values(const FilterNode* n, const std::string& col, std::vector<std::string>& vals) {
  if (n->kind == FilterNode::LEAF) {
    if (n->k != col || n->extracted || n->computed) return false;
    if (n->op == "eq") { vals = {n->v[0]}; return true; }
    if (n->op == "in") {
      vals.clear();
      for (auto& v : n->v)
        if (std::find(vals.begin(), vals.end(), v) == vals.end()) vals.push_back(v);
      return true;
    }
    return false;
  }
  if (n->kind == FilterNode::AND) {
    std::vector<std::string> va, vb;
    bool ra = restricted_values(n->a.get(), col, va);
    bool rb = restricted_values(n->b.get(), col, vb);
    if (ra && rb) {   // intersection, keeping the first list's order
      vals.clear();
      for (auto& v : va)
        if (std::find(vb.begin(), vb.end(), v) != vb.end()) vals.push_back(v);
      return true;
    }
    if (ra) { vals = va; return true; }
    if (rb) { vals = vb; return true; }
  }
  return false;
}

static std::unique_ptr<FilterNode> clone_filter(const FilterNode* n) {
  if (!n) return nullptr;
  auto c = std::make_unique<FilterNode>();
  c->kind = n->kind;
  c->k = n->k;
  c->v = n->v;
  c->op = n->op;
  c->extracted = n->extracted;
  c->computed = n->computed;
  c->data_type = n->data_type;
  c->a = clone_filter(n->a.get());
  c->b = clone_filter(n->b.get());
  return c;
}

Request copy_request(const Request& r) {
  Request c;
  c.expr_id = r.expr_id;
  c.dataset = r.dataset;
  c.filter = clone_filter(r.filter.get());
  c.has_chart = r.has_chart;
  c.aggregation = r.aggregation;
  c.group_bys = r.group_bys;
  c.chart_type = r.chart_type;
  c.rollup = r.rollup;
  c.field_chart = r.field_chart;
  c.has_extract = r.has_extract;
  c.has_compute = r.has_compute;
  c.limit = r.limit;
  c.order = r.order;
  c.is_tag_query = r.is_tag_query;
  c.reverse_sort = r.reverse_sort;
  c.tag_name = r.tag_name;
  c.tag_data_type = r.tag_data_type;
  c.segments = r.segments;
  return c;
}

}  // namespace lk
