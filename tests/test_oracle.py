"""The oracle itself: pinned to the reference's SQL plan strings, cross-checked by SQLite, and the committed
golden rows reproduce (CPU)."""
import json
import os

import pytest

from oracle import dataexpr as dx
from oracle import sqlplan
from tests.parity import assert_rows_equal, from_jsonable

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = os.path.join(HERE, "golden")


def _ref_cases():
    with open(os.path.join(GOLDEN, "ref_sql_cases.json")) as f:
        return json.load(f)


def _cases():
    with open(os.path.join(GOLDEN, "cases.json")) as f:
        return json.load(f)


@pytest.mark.parametrize("case", _ref_cases(), ids=lambda c: c["name"])
def test_sql_plan_matches_reference_test_strings(case):
    """BaseExpr.generateSql restated in oracle/sqlplan.py reproduces the reference's own expected SQL
    (ASTUtilsBaseExprTest.scala) character for character, except the extract sub-query, which is outside
    the hot path and is spliced in from the expected string."""
    node = case["payload"]["baseExpressions"][case["expr"]]
    be = dx.to_base_expr(node, case["expr"])
    pr = dx.PushDownRequest(baseExpr=be, segmentRequests=[])
    exp = case["expected"]
    if case["kind"] == "tag_filter_sql":
        got = sqlplan.generate_tag_sql(pr, "resource.container.name", case["start"], case["end"], set())
        assert got == exp
    else:
        lo = exp.index("FROM (") + len("FROM (")
        hi = exp.rindex(")  WHERE true AND ")
        sub = exp[lo:hi]
        assert sqlplan.timestamp_filter(case["start"], case["end"]) in sub
        got = sqlplan.generate_sql(pr, case["start"], case["end"], case["step"], set(), sub_query=sub)
        assert got == exp


@pytest.mark.parametrize("case", _cases(), ids=lambda c: c["name"])
def test_oracle_matches_sqlite_running_reference_sql(case):
    pr = dx.parse_pushdown(json.dumps(case["request"]))
    paths = [os.path.join(GOLDEN, p) for p in case["segments"]]
    per_glob = dx.evaluate_per_glob(pr, paths, case["glob_size"])
    agg = pr.baseExpr.chart.aggregation
    for g, rows in zip(dx.globs_of(pr, case["glob_size"]), per_glob):
        ref = sqlplan.run_sql(pr, g, [paths[i] for i in g])
        # SQLite 3.37 sums naively in row order: compare sums with a relative bound, the rest exactly
        assert len(rows) == len(ref)
        for a, b in zip(rows, ref):
            assert a[0] == b[0] and a[2] == b[2]
            if agg in ("sum", "avg"):
                assert a[1] == pytest.approx(b[1], rel=1e-12, abs=0)
            else:
                assert a[1] == b[1]


@pytest.mark.parametrize("case", _cases(), ids=lambda c: c["name"])
def test_committed_golden_rows_reproduce(case):
    pr = dx.parse_pushdown(json.dumps(case["request"]))
    paths = [os.path.join(GOLDEN, p) for p in case["segments"]]
    agg = pr.baseExpr.chart.aggregation
    cells = dx.evaluate_glob_cells(pr, case["glob_size"], paths)
    for rows, want in zip([[(c.ts, c.agg_value(agg), c.tags) for c in cs] for cs in cells],
                          case["expected_per_glob"]):
        assert_rows_equal(rows, from_jsonable(want), "exact", case["name"])
    if case["expected_merged"] is not None:
        assert_rows_equal(dx.merge_glob_cells(pr, cells), from_jsonable(case["expected_merged"]), "exact",
                          case["name"])


def test_no_segments_sentinel_shape():
    """Commons.scala:393-396: no segments -> one DataPoint(timestamp=-1, value=-1) (checked on the GPU path
    in test_gpu_parity)."""
    req = {"baseExpr": {"id": "A", "dataset": "logs", "filter": {"k": dx.NAME, "v": ["x"], "op": "eq"},
                        "chart": {"aggregation": "sum", "groupBys": []}},
           "segmentRequests": [], "reverseSort": False, "isTagQuery": False}
    pr = dx.parse_pushdown(json.dumps(req))
    assert dx.globs_of(pr, 10) == []


def test_binary_clause_folds_left_in_json_order():
    node = {"op": "or", "q1": {"k": "a", "v": ["1"], "op": "eq"}, "q2": {"k": "b", "v": ["2"], "op": "eq"},
            "q3": {"k": "c", "v": ["3"], "op": "eq"}}
    f = dx.handle_filter(node)
    assert isinstance(f, dx.BinaryClause) and f.op == "or"
    assert isinstance(f.q1, dx.BinaryClause) and f.q2.k == "c"
    assert sqlplan.filter_sql(f, {"b"}) == "((a = '1' or false) or c = '3')"


def _tag_cases():
    out = []
    for fn in ("tag_cases.json", "numtag_cases.json"):   # string tags; numeric tags (make_numtag_cases.py)
        with open(os.path.join(GOLDEN, fn)) as f:
            out += json.load(f)
    return out


@pytest.mark.parametrize("case", _tag_cases(), ids=lambda c: c["name"])
def test_tag_query_oracle_matches_golden(case):
    """Tag queries (BaseExpr.scala:127-143): the oracle reproduces the committed rows, and for every glob agrees
    with the reference's tag SQL run on SQLite."""
    text = json.dumps(case["request"])
    pr = dx.parse_pushdown(text)
    tag = dx.parse_tag_data_type(text)
    paths = [os.path.join(GOLDEN, p) for p in case["segments"]]
    assert dx.evaluate_tag_per_glob(pr, tag, paths, case["glob_size"]) == case["expected_per_glob"]
    assert dx.evaluate_tag_merged(pr, tag, paths, case["glob_size"]) == case["expected_merged"]
    g = dx.globs_of(pr, case["glob_size"])[-1]
    assert dx.evaluate_tag_glob(pr, tag, g, [paths[i] for i in g]) == sqlplan.run_tag_sql(pr, tag, g, [paths[i] for i in g])


def test_tag_row_noisy_tags_dropped():
    """NoisyTagsDropper.remove: hidden names / rollup_ prefix / NULL, "" and "null" values drop the tag; the count
    column stays (Commons.scala:406-423)."""
    assert dx.tag_row_tags("resource.service.name", "svc-001", 7) == {"resource.service.name": "svc-001", "count": "7"}
    for name in ("_cardinalhq.id", "hour", "rollup_sum", "metric.filter"):
        assert dx.tag_row_tags(name, "x", 3) == {"count": "3"}
    for v in (None, "", "null"):
        assert dx.tag_row_tags("a", v, 1) == {"count": "1"}
