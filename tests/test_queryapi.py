"""query-api final evaluation (lakeside_amd/queryapi.py) on the host: label / transformer / group-key strings
pinned from the Scala (file:line in each test), and the product's eval of merged rows checked against the
oracle's independent restatement (oracle/dataexpr.py::final_eval) on the committed golden merged rows."""
import json
import math
import os

import numpy as np
import pytest

from lakeside_amd import queryapi as qa
from oracle import dataexpr as dx
from tests.parity import from_jsonable

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
NAME, SVC, NS = "_cardinalhq.name", "resource.service.name", "resource.k8s.namespace.name"


def leaf(k, op, *v):
    return {"k": k, "v": list(v), "op": op}


def base_expr(filt, agg="sum", group_bys=(), chart_type="count", dataset="logs", metric_type=None):
    be = {"id": "A", "dataset": dataset, "filter": filt,
          "chart": {"aggregation": agg, "groupBys": list(group_bys), "type": chart_type}}
    if metric_type is not None:
        be["metricType"] = metric_type
    return be


def test_label_strings():
    """BaseExpr.label (BaseExpr.scala:697-716) over QueryClause.toString (ASTUtils.scala:102-122)."""
    c3 = {"op": "and", "q1": leaf(NAME, "eq", "metric_07"), "q2": leaf(SVC, "regex", "^svc-0[0-4]")}
    be = base_expr(c3)
    want = "((_cardinalhq.name = metric_07 and regexMatches(resource.service.name, ^svc-0[0-4])))"
    assert qa.label(be, {"name": "metric_07"}) == want
    assert dx.clause_label(dx.handle_filter(c3)) == want[1:-1]
    assert qa.label(base_expr({"not": leaf(NS, "in", "a", "b")}), {}) == "(not(resource.k8s.namespace.name in (a, b)))"
    assert qa.label(base_expr(leaf(SVC, "contains", "api")), {}) == "(resource.service.name contains api)"
    # operators without a toString case print "" (ASTUtils.scala:115)
    assert qa.label(base_expr({"op": "or", "a": leaf(SVC, "!=", "x"), "b": leaf(NS, "eq", "y")}), {}) == \
        "(( or resource.k8s.namespace.name = y))"
    # three children fold left (ASTUtils.scala:395-402)
    three = {"op": "or", "q1": leaf("a", "eq", "1"), "q2": leaf("b", "eq", "2"), "q3": leaf("c", "eq", "3")}
    assert qa.clause_string(three) == "((a = 1 or b = 2) or c = 3)"
    # with groupBys: sorted keys present in the tags (BaseExpr.scala:700-710)
    be = base_expr(leaf(NAME, "eq", "m"), group_bys=[SVC, NS])
    assert qa.label(be, {NS: "ns-01", SVC: "svc-003", "name": "m"}) == \
        "(resource.k8s.namespace.name = ns-01, resource.service.name = svc-003)"
    assert qa.label(be, {SVC: "svc-003"}) == "(resource.service.name = svc-003)"


def test_group_by_key():
    """ASTUtils.toGroupByKey (ASTUtils.scala:87-89): sorted keys, missing -> ""."""
    assert qa.group_by_key([], {"a": "1"}) == "default"
    assert qa.group_by_key(["b", "a", "b"], {"a": "1", "b": "2"}) == "1:2"
    assert qa.group_by_key(["b", "a"], {"b": "2"}) == ":2"


def test_transformers():
    """ASTUtils.getTransformerFunc (ASTUtils.scala:190-219): step seconds = stepInMillis / 1000 on Longs."""
    v = np.array([120.0, 0.0, -3.0])
    f = qa.transformer(base_expr(leaf(NAME, "eq", "m"), chart_type="rate"), 60000)
    assert f(v).tolist() == [2.0, 0.0, -0.05]
    assert qa.transformer(base_expr(leaf(NAME, "eq", "m")), 60000)(v).tolist() == v.tolist()
    m = base_expr(leaf(NAME, "eq", "m"), dataset="metrics", metric_type="rate")
    assert qa.transformer(m, 10000)(v).tolist() == [1200.0, 0.0, -30.0]
    m = base_expr(leaf(NAME, "eq", "m"), chart_type="rate", dataset="metrics", metric_type="count")
    assert qa.transformer(m, 10000)(v).tolist() == [12.0, 0.0, -0.3]
    m = base_expr(leaf(NAME, "eq", "m"), chart_type="rate", dataset="metrics", metric_type="gauge")
    assert qa.transformer(m, 10000)(v).tolist() == v.tolist()
    # sub-second step: Long 500 / 1000 = 0 -> IEEE division by zero, as on the JVM
    r = qa.transformer(base_expr(leaf(NAME, "eq", "m"), chart_type="rate"), 500)(v)
    assert r[0] == math.inf and math.isnan(r[1]) and r[2] == -math.inf
    with pytest.raises(ValueError):
        qa.transformer(base_expr(leaf(NAME, "eq", "m"), chart_type="bar"), 60000)


def _payloads_equal(got, want):
    assert len(got) == len(want)
    for g, w in zip(got, want):
        gm, wm = g["message"], w["message"]
        assert (g["id"], g["type"], gm["timestamp"], gm["tags"], gm["label"]) == \
               (w["id"], w["type"], wm["timestamp"], wm["tags"], wm["label"])
        assert gm["value"] == wm["value"] or (math.isnan(gm["value"]) and math.isnan(wm["value"]))


def _golden():
    with open(os.path.join(GOLDEN, "cases.json")) as f:
        return [c for c in json.load(f) if c["expected_merged"] is not None]


@pytest.mark.parametrize("chart_type,metric_type", [("count", None), ("rate", None), ("count", "rate"),
                                                    ("rate", "counter")])
@pytest.mark.parametrize("case", _golden(), ids=lambda c: c["name"])
def test_eval_merged_rows_matches_oracle(case, chart_type, metric_type):
    be = dict(case["request"]["baseExpr"])
    be["chart"] = dict(be["chart"], type=chart_type)
    if metric_type:
        be["metricType"] = metric_type
    rows = from_jsonable(case["expected_merged"])
    step = case["request"]["segmentRequests"][0]["stepInMillis"]
    now = max([r[0] for r in rows], default=0) - 1      # the last timestamp is "in the future": dropped
    got = qa.eval_merged_rows(be, np.array([r[0] for r in rows], np.int64), np.array([r[1] for r in rows]),
                              [r[2] for r in rows], step, now)
    _payloads_equal(got, dx.final_eval(be, rows, step, now))
    assert all(p["message"]["timestamp"] <= now for p in got)


def test_group_key_collision_keeps_one_row_per_key():
    """Rows of one timestamp whose tags differ outside the groupBys (here: name) collapse to one result per
    group key (BaseExpr.scala:689-690); the smallest tag list wins (deterministic stand-in for hash order)."""
    be = base_expr(leaf(NAME, "in", "m1", "m2"), group_bys=[SVC])
    rows = [(1000, 5.0, {"name": "m2", SVC: "s"}), (1000, 7.0, {"name": "m1", SVC: "s"}),
            (1000, 1.0, {"name": "m1", SVC: "t"}), (2000, 2.0, {"name": "m2"})]
    got = qa.eval_merged_rows(be, np.array([r[0] for r in rows]), np.array([r[1] for r in rows]),
                              [r[2] for r in rows], 60000, 10 ** 13)
    assert [(p["message"]["timestamp"], p["message"]["value"]) for p in got] == [(1000, 7.0), (1000, 1.0), (2000, 2.0)]
    assert got[2]["message"]["label"] == "()"
    _payloads_equal(got, dx.final_eval(be, rows, 60000, 10 ** 13))
