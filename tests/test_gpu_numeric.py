"""Numeric comparison leaves (`gt/ge/lt/le`, BaseExpr.scala:450-459, 488-498) on the MI355X through the C ABI vs the
oracle: DOUBLE / FLOAT / INT64 / INT32 filter columns (NULLs, NaN, union_by_name INT32+INT64), duration / datasize /
number literals, the value column itself, a decimal vs a scientific literal on integers near 2^60, a VARCHAR column
(Binder Error -> empty glob), a bad literal (-> empty globs where the field exists), combinations with string leaves
under and / or / not; aggregate rows per glob and merged, tag queries and exemplar rows."""
import json

import numpy as np
import pytest

from tests.parity import assert_rows_equal

pytestmark = pytest.mark.gpu

SVC = "resource.service.name"


def _files(tmp_path, nfiles=4, rows=30_000):
    import pyarrow as pa
    import pyarrow.parquet as pq
    from lakeside_amd import synth
    from oracle import dataexpr as dx
    rng = np.random.default_rng(11)
    paths, blobs = [], []
    for i in range(nfiles):
        n = rows + 313 * i
        ts = np.sort(synth.T0 + rng.integers(0, synth.HOUR, n))
        val = rng.lognormal(0, 2, n)
        val[rng.random(n) < 0.02] = np.nan
        cols = {
            dx.TIMESTAMP: pa.array(ts, pa.int64()),
            dx.VALUE: pa.array(val, pa.float64(), mask=rng.random(n) < 0.05),
            dx.NAME: pa.array([f"metric_{k:02d}" for k in rng.integers(0, 4, n)], pa.string()),
            SVC: pa.array([f"svc-{k}" for k in rng.integers(0, 5, n)], pa.string(), mask=rng.random(n) < 0.1),
            "_cardinalhq.message": pa.array([f"m{k}" for k in rng.integers(0, 9, n)], pa.string()),
            "attr.dur": pa.array(rng.integers(0, 5_000_000, n), pa.int64(), mask=rng.random(n) < 0.1),
            "attr.size": pa.array(rng.integers(0, 4096, n).astype(np.int32 if i % 2 else np.int64),
                                  mask=rng.random(n) < 0.1),
            "attr.ratio": pa.array(rng.random(n).astype(np.float32), pa.float32()),
            "attr.big": pa.array((1 << 60) + rng.integers(-3, 4, n), pa.int64()),
            "attr.txt": pa.array([str(k) for k in rng.integers(0, 100, n)], pa.string()),
        }
        t = pa.table(cols)
        path = str(tmp_path / f"num{i}.parquet")
        if i % 2:
            pq.write_table(t, path, row_group_size=10_000)                      # dictionaries everywhere
        else:
            strings = [c for c in t.column_names if t.schema.field(c).type == pa.string()]
            pq.write_table(t, path, compression="NONE", use_dictionary=strings, row_group_size=12_000,
                           column_encoding={c: "PLAIN" for c in t.column_names if c not in strings})
        paths.append(path)
        blobs.append(open(path, "rb").read())
    return paths, blobs


def _num(k, op, v, dt="number"):
    return {"k": k, "v": [v], "op": op, "extracted": False, "computed": False, "dataType": dt}


CASES = [
    ("value_gt", _num("_cardinalhq.value", "gt", "10"), "sum", []),
    ("dur_ge_ms", _num("attr.dur", "ge", "1.5ms", "duration"), "count", [SVC]),
    ("and_size_lt_kb", {"q1": {"k": "_cardinalhq.name", "v": ["metric_01"], "op": "eq"},
                        "q2": _num("attr.size", "lt", "2kb", "datasize"), "op": "and"}, "max", []),
    ("ratio_le_or_svc", {"q1": _num("attr.ratio", "le", "0.25"), "q2": {"k": SVC, "v": ["svc-3"], "op": "eq"},
                         "op": "or"}, "min", [SVC]),
    ("not_value_gt", {"not": _num("_cardinalhq.value", "gt", "5")}, "avg", []),
    ("big_decimal_vs_sci", {"q1": _num("attr.big", "ge", "1152921504606846976"), "q2": _num("attr.dur", "lt", "2e6"),
                            "op": "and"}, "count", []),
    ("string_column", _num("attr.txt", "gt", "50"), "count", []),
    ("bad_literal", _num("attr.dur", "gt", "abc"), "count", []),
    ("bad_literal_missing_field", {"q1": _num("no.such", "gt", "abc"), "q2": _num("attr.dur", "le", "1000000"),
                                   "op": "or"}, "sum", []),
]


def test_numeric_leaves_aggregates(engine, tmp_path):
    from lakeside_amd import LK_MERGED, LK_PER_GLOB_ROWS, synth
    from oracle import dataexpr as dx
    paths, blobs = _files(tmp_path)
    for p in paths:
        engine.load_segment(p)
    segs = [synth.segment_request(i, hour=0) for i in range(len(paths))]
    for label, filt, agg, gbs in CASES:
        req = json.dumps(synth.pushdown(filt, segs, agg, gbs))
        pr = dx.parse_pushdown(req)
        cells = dx.evaluate_glob_cells(pr, 2, paths, sources=blobs)
        got = engine.eval_pushdown(req, paths, 2, LK_PER_GLOB_ROWS).per_glob(len(cells))
        for gi, (g, cs) in enumerate(zip(got, cells)):
            assert_rows_equal(g, [(c.ts, c.agg_value(agg), c.tags) for c in cs], agg, f"{label} glob {gi}")
        merged = engine.eval_pushdown(req, paths, 2, LK_MERGED).rows()
        assert_rows_equal(merged, dx.merge_glob_cells(pr, cells), agg, f"{label} merged")
        if label in ("string_column", "bad_literal"):
            assert merged == []
        elif label != "bad_literal_missing_field":
            assert len(merged) > 0, label


def test_numeric_leaves_tag_and_exemplar(engine, tmp_path):
    from lakeside_amd import LK_MERGED, LK_PER_GLOB_ROWS, synth
    from oracle import dataexpr as dx
    from oracle import exemplar as ex
    paths, blobs = _files(tmp_path, nfiles=3, rows=20_000)
    for p in paths:
        engine.load_segment(p)
    segs = [synth.segment_request(i, hour=0) for i in range(len(paths))]
    # tag query: values of the service among rows with a long duration
    filt = {"q1": _num("attr.dur", "gt", "4ms", "duration"), "q2": {"k": SVC, "v": [], "op": "exists"}, "op": "and"}
    req = json.dumps(synth.pushdown(filt, segs, tag=SVC))
    pr = dx.parse_pushdown(req)
    want = dx.evaluate_tag_merged(pr, SVC, paths, 2, sources=blobs)
    got = engine.eval_pushdown(req, paths, 2, LK_MERGED)
    key = lambda t: sorted(t.items())   # noqa: E731
    assert sorted(got.tags, key=key) == sorted(want, key=key)
    # exemplar rows filtered on a FLOAT column and the value column
    be = {"id": "A", "dataset": "logs", "limit": 200,
          "filter": {"q1": _num("attr.ratio", "ge", "0.5"), "q2": _num("_cardinalhq.value", "lt", "0.1"), "op": "and"}}
    req = json.dumps({"baseExpr": be, "segmentRequests": segs})
    want = ex.evaluate_exemplar(dx.parse_pushdown(req), paths, 2, sources=blobs)
    res = engine.eval_pushdown(req, paths, 2, LK_PER_GLOB_ROWS)
    rows = list(zip(res.ts.tolist(), res.values.tolist(), res.tags, res.globs.tolist()))
    assert len(rows) == len(want) > 0
    for g, w in zip(rows, want):
        assert (g[0], g[3], g[2]) == (w[0], w[3], w[2])


@pytest.mark.parametrize("mixed", [False, True])
def test_value_leaf_on_scan_lean(engine, mixed):
    """numeric leaves on the value column run inside scan_lean (string conjuncts early, the value
    tested per passing row), with the general row scan taking only segments scan_lean cannot take whole (mixed: one
    segment with NULL values).  GPU == oracle per glob and merged."""
    from lakeside_amd import LK_MERGED, LK_PER_GLOB_ROWS, synth
    from oracle import dataexpr as dx
    keys, blobs = [], []
    for i in range(4):
        nf = 0.05 if (mixed and i == 2) else 0.0
        s = synth.make_segment(synth.segment_spec(i, rows=1 << 17, null_frac=nf, rg_rows=1 << 16, page_rows=1 << 14))
        blobs.append(s.bytes())
        engine.put_segment_ptr(f"vleaf/{mixed}/{i}", s.ptr, s.size)
        s.free()
        keys.append(f"vleaf/{mixed}/{i}")
    segs = [synth.segment_request(i) for i in range(4)]
    v = lambda op, x: _num(dx.VALUE, op, x)   # noqa: E731
    for filt, agg, gbs in [({"op": "and", "q1": synth.leaf(synth.NAME, "eq", "metric_07"), "q2": v("gt", "1.5")}, "sum", []),
                           ({"op": "and", "q1": synth.leaf(synth.NAME, "in", "metric_01", "metric_07"),
                             "q2": {"op": "or", "q1": v("le", "0.25"), "q2": v("gt", "100")}}, "count", [SVC]),
                           ({"op": "and", "q1": {"op": "and", "q1": synth.leaf(synth.NAME, "eq", "metric_03"),
                                                 "q2": synth.leaf(SVC, "regex", "^svc-0[0-4]")},
                             "q2": {"not": v("ge", "2")}}, "max", [SVC]),
                           ({"op": "and", "q1": synth.leaf(synth.NAME, "eq", "metric_05"), "q2": v("lt", "1e3")}, "avg", [])]:
        req = json.dumps(synth.pushdown(filt, segs, agg, gbs))
        pr = dx.parse_pushdown(req)
        got = engine.eval_pushdown(req, keys, 2, LK_MERGED)
        assert_rows_equal(got.rows(), dx.evaluate_merged(pr, keys, 2, sources=blobs), agg, f"vleaf {agg} merged")
        assert got.stats["general_segments"] == (1 if mixed else 0), got.stats
        pg = engine.eval_pushdown(req, keys, 2, LK_PER_GLOB_ROWS).per_glob(2)
        for gi, (g, w) in enumerate(zip(pg, dx.evaluate_per_glob(pr, keys, 2, sources=blobs))):
            assert_rows_equal(g, w, agg, f"vleaf {agg} glob {gi}")
