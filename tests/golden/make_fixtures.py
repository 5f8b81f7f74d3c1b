"""Generate the committed parity fixtures: small sealed segments + PushDownRequests + expected rows.

Segments are written with pyarrow exactly as SURVEY.md §8(d) prescribes for in-container fixtures
(compression NONE, dictionary tag columns, PLAIN timestamp/value, v1 data pages; two segments use v2
pages), with 5% NULLs, missing columns, multiple row groups and small pages.  Expected rows come from
``oracle/dataexpr.py`` and every case is cross-checked here against the reference's generated SQL run on
SQLite (``oracle/sqlplan.py``) before it is written.

Run:  python tests/golden/make_fixtures.py     (writes tests/golden/segments/*.parquet, cases.json)
"""
import json
import os
import sys

import numpy as np
import pyarrow as pa
import pyarrow.parquet as pq

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from oracle import dataexpr as dx          # noqa: E402
from oracle import sqlplan                 # noqa: E402

T0 = 1704067200000
TS, VAL, NAME = dx.TIMESTAMP, dx.VALUE, dx.NAME
SVC, NS, LEVEL = "resource.service.name", "resource.k8s.namespace.name", "_cardinalhq.level"
SEGDIR = os.path.join(HERE, "segments")


def make_segment(idx, n, *, hour, nulls=0.05, drop=(), int_values=False, v2=False, rg=2048, page=4096,
                 all_null=(), ts_nulls=0, metrics=False, step=60000):
    rng = np.random.default_rng(20240101 + idx)
    start = T0 + hour * 3_600_000
    if metrics:
        ts = np.sort(start + step * rng.integers(0, 60, n))
    else:
        ts = np.sort(start + rng.integers(0, 3_600_000, n))
    if int_values:
        vals = rng.integers(0, 1000, n).astype(np.float64)
    else:
        vals = rng.lognormal(0.0, 2.0, n)
    cols = {
        TS: pa.array(ts, pa.int64(), mask=_mask(rng, n, ts_nulls)),
        VAL: pa.array(vals, pa.float64(), mask=_mask(rng, n, nulls)),
        NAME: pa.array([f"metric_{i:02d}" for i in rng.integers(0, 16, n)], pa.string(), mask=_mask(rng, n, nulls)),
        SVC: pa.array([f"svc-{i:03d}" for i in rng.integers(0, 100, n)], pa.string(), mask=_mask(rng, n, nulls)),
        NS: pa.array([f"ns-{i:02d}" for i in rng.integers(0, 20, n)], pa.string(), mask=_mask(rng, n, nulls)),
        LEVEL: pa.array([["INFO", "WARN", "ERROR", "DEBUG", "null", ""][i] for i in rng.integers(0, 6, n)],
                        pa.string(), mask=_mask(rng, n, nulls)),
    }
    if metrics:
        cols.pop(VAL)
        cols["rollup_sum"] = pa.array(vals, pa.float64(), mask=_mask(rng, n, nulls))
        cols["rollup_max"] = pa.array(vals * 2, pa.float64())
    for c in all_null:
        cols[c] = pa.nulls(n, pa.string())
    for c in drop:
        cols.pop(c)
    table = pa.table(cols)
    strings = [c for c in table.column_names if pa.types.is_string(table.schema.field(c).type)]
    path = os.path.join(SEGDIR, f"seg{idx:02d}.parquet")
    pq.write_table(table, path, compression="NONE", use_dictionary=strings,
                   column_encoding={c: "PLAIN" for c in table.column_names if c not in strings},
                   data_page_version="2.0" if v2 else "1.0", row_group_size=rg, data_page_size=page,
                   write_statistics=True)
    return os.path.relpath(path, HERE)


def _mask(rng, n, p):
    if not p:
        return None
    return rng.random(n) < p


def seg_req(i, hour, step=60000, qtags=None, start=None, end=None):
    s = T0 + hour * 3_600_000
    return {"hour": f"{hour:02d}", "dateInt": "20240101", "segmentId": f"seg{i:02d}", "sealedStatus": True,
            "dataset": "logs", "queryTags": qtags or {}, "stepInMillis": step, "customerId": "c",
            "collectorId": "k", "bucketName": "b", "cName": "",
            "startTs": s if start is None else start, "endTs": s + 3_600_000 if end is None else end}


def leaf(k, op, *v):
    return {"k": k, "v": list(v), "op": op, "extracted": False, "computed": False, "dataType": "string"}


def request(filt, agg="sum", group_bys=(), segs=(), dataset="logs", rollup=None):
    chart = {"aggregation": agg, "groupBys": list(group_bys), "type": "count"}
    if rollup:
        chart["rollup"] = rollup
    return {"baseExpr": {"id": "A", "dataset": dataset, "filter": filt, "chart": chart, "limit": 1000,
                         "order": "DESC", "metricType": "gauge", "returnResults": True},
            "segmentRequests": list(segs), "reverseSort": False, "isTagQuery": False}


def main():
    os.makedirs(SEGDIR, exist_ok=True)
    files = {}
    files[0] = make_segment(0, 3000, hour=0)
    files[1] = make_segment(1, 2500, hour=0, drop=(NS,))
    files[2] = make_segment(2, 4000, hour=1, int_values=True, nulls=0.0)
    files[3] = make_segment(3, 1500, hour=1, v2=True, rg=700, page=1024)
    files[4] = make_segment(4, 2000, hour=0, all_null=(SVC,), ts_nulls=0.02)
    files[5] = make_segment(5, 3000, hour=2, drop=(SVC, NS), int_values=True)
    files[6] = make_segment(6, 1200, hour=2, v2=True, nulls=0.2)
    files[7] = make_segment(7, 5000, hour=0, int_values=True, nulls=0.0, rg=5000, page=1 << 20)
    files[8] = make_segment(8, 2200, hour=3)
    files[9] = make_segment(9, 1800, hour=3, drop=(LEVEL,))
    files[10] = make_segment(10, 2600, hour=1, rg=1024, page=2048)
    files[11] = make_segment(11, 900, hour=2, drop=(NS, LEVEL), nulls=0.1)
    files[12] = make_segment(12, 3000, hour=0, metrics=True)
    files[13] = make_segment(13, 2000, hour=1, metrics=True, nulls=0.0)

    def segs(ids, step=60000, qtags=None, **kw):
        return [seg_req(i, _hour(i), step, qtags, **kw) for i in ids]

    all_logs = list(range(12))
    cases = []

    def add(name, req, paths_ids, glob_size=10):
        cases.append({"name": name, "request": req, "segments": [files[i] for i in paths_ids],
                      "glob_size": glob_size})

    name07 = leaf(NAME, "eq", "metric_07")
    add("c1_eq_sum", request(name07, "sum", segs=segs([7], qtags={NAME: "metric_07"})), [7])
    add("eq_sum_all", request(name07, "sum", segs=segs(all_logs, qtags={NAME: "metric_07"})), all_logs)
    add("eq_sum_glob5", request(name07, "sum", segs=segs(all_logs)), all_logs, 5)
    add("c3_and_regex_by2_max",
        request({"op": "and", "q1": name07, "q2": leaf(SVC, "regex", "^svc-0[0-4]")}, "max", (SVC, NS),
                segs=segs(all_logs)), all_logs)
    add("in_by_level_min", request(leaf(NAME, "in", "metric_01", "metric_02", "metric_03"), "min", (LEVEL,),
                                   segs=segs(all_logs)), all_logs, 5)
    add("or_not_count", request({"op": "or", "q1": {"not": leaf(SVC, "eq", "svc-001")},
                                 "q2": leaf(NS, "in", "ns-01", "ns-02")}, "count", (NS,),
                                segs=segs(all_logs, step=300000)), all_logs, 4)
    add("neq_notin_sum_by_svc", request({"op": "and", "q1": leaf(NAME, "!=", "metric_00"),
                                         "q2": leaf(NS, "not_in", "ns-03", "ns-04", "ns-05"),
                                         "q3": leaf(LEVEL, "has", "")}, "sum", (SVC,),
                                        segs=segs(all_logs, step=10000)), all_logs, 3)
    add("contains_avg", request(leaf(SVC, "contains", "VC-09"), "avg", segs=segs(all_logs)), all_logs, 6)
    add("missing_col_not", request({"op": "and", "q1": {"not": leaf(NS, "eq", "ns-01")},
                                    "q2": {"op": "or", "q1": leaf(NAME, "eq", "metric_03"),
                                           "q2": leaf(NS, "eq", "ns-02")}}, "sum", (NS,),
                                   segs=segs([1, 5, 11, 0])), [1, 5, 11, 0], 3)
    add("not_only_field_binder_error", request({"op": "and", "q1": {"not": leaf("resource.missing", "eq", "x")},
                                                "q2": leaf(NAME, "eq", "metric_03")}, "sum",
                                               segs=segs([1, 0])), [1, 0], 1)
    add("missing_col_leaf_false", request({"op": "or", "q1": leaf(NS, "eq", "ns-07"),
                                           "q2": leaf(NAME, "eq", "metric_05")}, "max",
                                          segs=segs([1, 5, 11, 2, 3])), [1, 5, 11, 2, 3], 2)
    add("window_clip", request(name07, "sum", segs=segs([0, 4, 7], start=T0 + 600_000, end=T0 + 1_800_000)),
        [0, 4, 7])
    add("null_group_key_count", request(leaf(NAME, "eq", "metric_09"), "count", (SVC, LEVEL),
                                        segs=segs([4, 6, 0])), [4, 6, 0])
    add("metrics_rollup_sum", request(name07, "sum", (SVC,), dataset="metrics",
                                      segs=[dict(seg_req(12, 0), dataset="metrics"),
                                            dict(seg_req(13, 1), dataset="metrics")]), [12, 13])
    add("metrics_rollup_max", request(leaf(NAME, "in", "metric_01", "metric_02"), "max", dataset="metrics",
                                      rollup="max", segs=[dict(seg_req(12, 0), dataset="metrics"),
                                                          dict(seg_req(13, 1), dataset="metrics")]), [12, 13])

    for c in cases:
        pr = dx.parse_pushdown(json.dumps(c["request"]))
        paths = [os.path.join(HERE, p) for p in c["segments"]]
        glob_cells = dx.evaluate_glob_cells(pr, c["glob_size"], paths)
        agg = pr.baseExpr.chart.aggregation
        per_glob = [[(x.ts, x.agg_value(agg), x.tags) for x in cells] for cells in glob_cells]
        for g, rows in zip(dx.globs_of(pr, c["glob_size"]), per_glob):
            ref = sqlplan.run_sql(pr, g, [paths[i] for i in g])
            check_same(c["name"], rows, ref)
        c["expected_per_glob"] = [dx.rows_to_jsonable(r) for r in per_glob]
        c["expected_merged"] = None if pr.baseExpr.chart.aggregation == dx.AVG else \
            dx.rows_to_jsonable(dx.merge_glob_cells(pr, glob_cells))
        print(f"{c['name']}: globs={len(per_glob)} rows={sum(map(len, per_glob))} "
              f"merged={len(c['expected_merged'] or [])}", file=sys.stderr)
    with open(os.path.join(HERE, "cases.json"), "w") as f:
        json.dump(cases, f, indent=0)


def _hour(i):
    return {0: 0, 1: 0, 2: 1, 3: 1, 4: 0, 5: 2, 6: 2, 7: 0, 8: 3, 9: 3, 10: 1, 11: 2, 12: 0, 13: 1}[i]


def check_same(name, rows, ref):
    """Oracle vs SQLite running the reference SQL: ts/tags exact, counts/min/max exact, sums <= 1e-12 rel
    (SQLite 3.37 sums naively in row order; the oracle is correctly rounded)."""
    if len(rows) != len(ref):
        raise AssertionError(f"{name}: {len(rows)} rows vs sqlite {len(ref)}")
    for (t1, v1, g1), (t2, v2, g2) in zip(rows, ref):
        if t1 != t2 or g1 != g2:
            raise AssertionError(f"{name}: key mismatch {(t1, g1)} vs {(t2, g2)}")
        if not (v1 == v2 or abs(v1 - v2) <= 1e-12 * max(abs(v1), abs(v2))):
            raise AssertionError(f"{name}: value {v1!r} vs sqlite {v2!r} at {t1} {g1}")


if __name__ == "__main__":
    main()
