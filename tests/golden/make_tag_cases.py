"""Golden tag-query cases (TEST ONLY): isTagQuery requests over the committed golden segments.

Each case's expected rows come from oracle/dataexpr.py (evaluate_tag_glob) and are cross-checked, glob by glob,
against the reference's own tag-query SQL (BaseExpr.scala:127-143, restated by oracle/sqlplan.generate_tag_sql
and pinned by ASTUtilsBaseExprTest.scala:71-74) executed on SQLite.  Writes tests/golden/tag_cases.json.

    python tests/golden/make_tag_cases.py
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from oracle import dataexpr as dx          # noqa: E402
from oracle import sqlplan                 # noqa: E402
from tests.golden.make_fixtures import T0, NAME, SVC, NS, LEVEL, _hour, leaf, seg_req   # noqa: E402


def tag_request(filt, tag, segs):
    # QueryEngineV2.evaluateTagQuery (QueryEngineV2.scala:418-441): chartOpts = None
    return {"baseExpr": {"id": "A", "dataset": "logs", "filter": filt, "limit": 1000, "order": "DESC",
                         "returnResults": True},
            "segmentRequests": segs, "reverseSort": False, "isTagQuery": True,
            "tagDataType": {"tagName": tag, "dataType": "string"}}


def exists_and(filt, tag):
    # evaluateTagQuery adds `tag IS NOT NULL` for a non-synthetic tag (QueryEngineV2.scala:430-437)
    return {"op": "and", "q1": filt, "q2": leaf(tag, "exists")}


def main():
    files = {i: f"segments/seg{i:02d}.parquet" for i in range(12)}
    all_logs = list(range(12))

    def segs(ids, **kw):
        return [seg_req(i, _hour(i), **kw) for i in ids]

    name07 = leaf(NAME, "eq", "metric_07")
    cases = []

    def add(name, req, ids, glob_size=10):
        cases.append({"name": name, "request": req, "segments": [files[i] for i in ids], "glob_size": glob_size})

    add("svc_of_name07", tag_request(exists_and(name07, SVC), SVC, segs(all_logs)), all_logs)
    add("level_nulls_no_exists", tag_request(leaf(NAME, "in", "metric_01", "metric_02"), LEVEL, segs(all_logs)),
        all_logs, 5)
    add("ns_missing_glob", tag_request(exists_and(leaf(SVC, "regex", "^svc-0[0-4]"), NS), NS, segs([1, 5, 11, 0])),
        [1, 5, 11, 0], 2)
    add("name_of_not_svc", tag_request({"not": leaf(SVC, "eq", "svc-001")}, NAME, segs(all_logs)), all_logs)
    add("svc_window_cut", tag_request(exists_and(leaf(NS, "in", "ns-01", "ns-02", "ns-03"), SVC),
                                      SVC, segs([0, 4, 7], start=T0 + 600_000, end=T0 + 1_800_000)), [0, 4, 7])
    add("level_or_missing_col", tag_request({"op": "or", "q1": leaf(NS, "eq", "ns-07"),
                                             "q2": leaf(LEVEL, "eq", "WARN")}, LEVEL, segs(all_logs)), all_logs, 3)

    for c in cases:
        text = json.dumps(c["request"])
        pr = dx.parse_pushdown(text)
        tag = dx.parse_tag_data_type(text)
        paths = [os.path.join(HERE, p) for p in c["segments"]]
        per_glob = []
        for g in dx.globs_of(pr, c["glob_size"]):
            rows = dx.evaluate_tag_glob(pr, tag, g, [paths[i] for i in g])
            ref = sqlplan.run_tag_sql(pr, tag, g, [paths[i] for i in g])
            if rows != ref:
                raise AssertionError(f"{c['name']}: oracle {rows} vs sqlite {ref}")
            per_glob.append([dx.tag_row_tags(tag, v, n) for v, n in rows])
        c["expected_per_glob"] = per_glob
        c["expected_merged"] = dx.evaluate_tag_merged(pr, tag, paths, c["glob_size"])
        print(f"{c['name']}: globs={len(per_glob)} rows={sum(map(len, per_glob))} merged={len(c['expected_merged'])}",
              file=sys.stderr)
    with open(os.path.join(HERE, "tag_cases.json"), "w") as f:
        json.dump(cases, f, indent=0)


if __name__ == "__main__":
    main()
