"""Exemplar (raw-row) queries on the MI355X through the C ABI vs the oracle restatement (oracle/exemplar.py):
ORDER BY timestamp DESC/ASC LIMIT n per glob (BaseExpr.scala:234-239), every column of the glob's union as tags
(Commons.toDataPoint, Commons.scala:428-459), Akka mergeSorted fold over globs (Commons.scala:391-392).

Exact equality: timestamps, values (bit-exact: the value is read, not computed), tag maps (every string), and the
ROW ORDER of the merged stream (the test does not sort)."""
import json
import math
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SVC = "resource.service.name"


def _logs_files(tmp_path, nfiles=5, rows=40_000, seed=5):
    """Logs segments written by pyarrow with a mix of physical types, NULLs, dictionary-encoded numerics (pyarrow's
    default), differing schemas (union_by_name: a column missing from some files, INT32 in one file and INT64 in
    another), duplicate timestamps (ties), and one file without the message column."""
    import pyarrow as pa
    import pyarrow.parquet as pq
    from lakeside_amd import synth
    from oracle import dataexpr as dx
    rng = np.random.default_rng(seed)
    paths, blobs = [], []
    for i in range(nfiles):
        n = rows + 997 * i
        t0 = synth.T0 + (i % 2) * synth.HOUR
        ts = np.sort(t0 + rng.integers(0, synth.HOUR // 50, n))          # ~1 row / 90 ms: ties exist
        cols = {
            dx.TIMESTAMP: pa.array(ts, pa.int64(), mask=rng.random(n) < 0.01),
            dx.VALUE: pa.array(rng.lognormal(0, 3, n) * np.where(rng.random(n) < 0.1, -1, 1), pa.float64(),
                               mask=rng.random(n) < 0.05),
            dx.NAME: pa.array([f"metric_{k:02d}" for k in rng.integers(0, 6, n)], pa.string()),
            SVC: pa.array([["svc-a", "svc-b", "null", "", "Svc-A"][k] for k in rng.integers(0, 5, n)], pa.string(),
                          mask=rng.random(n) < 0.1),
            "attr.count": pa.array(rng.integers(-5, 50, n).astype(np.int32 if i % 2 else np.int64),
                                   mask=rng.random(n) < 0.2),
            "attr.ratio": pa.array(rng.random(n).astype(np.float32) * 1e8, pa.float32()),
            "attr.flag": pa.array(rng.random(n) < 0.5, pa.bool_(), mask=rng.random(n) < 0.3),
            "attr.big": pa.array(rng.integers(-2**40, 2**40, n), pa.int64()),
        }
        if i != 3:
            cols["_cardinalhq.message"] = pa.array([f"msg {k} ü" for k in rng.integers(0, 300, n)], pa.string())
        if i % 3 == 1:
            cols["extra.only.some"] = pa.array([f"x{k}" for k in rng.integers(0, 9, n)], pa.string())
            del cols["attr.ratio"]
        t = pa.table(cols)
        path = str(tmp_path / f"logs{i}.parquet")
        if i % 2:
            pq.write_table(t, path, row_group_size=15_000, data_page_size=32_768)        # dictionaries everywhere
        else:
            strings = [c for c in t.column_names if t.schema.field(c).type == pa.string()]
            pq.write_table(t, path, compression="NONE", use_dictionary=strings, row_group_size=20_000,
                           column_encoding={c: "PLAIN" for c in t.column_names if c not in strings},
                           data_page_size=65_536, data_page_version="2.0" if i == 2 else "1.0")
        paths.append(path)
        blobs.append(open(path, "rb").read())
    return paths, blobs


def _request(filt, nfiles, limit=None, order=None, reverse=False, dataset="logs", hour=None):
    from lakeside_amd import synth
    segs = [synth.segment_request(i, hour=i % 2 if hour is None else hour, dataset=dataset) for i in range(nfiles)]
    be = {"id": "A", "dataset": dataset, "filter": filt}
    if limit is not None:
        be["limit"] = limit
    if order is not None:
        be["order"] = order
    return json.dumps({"baseExpr": be, "segmentRequests": segs, "reverseSort": reverse})


def _check(engine, req, paths, blobs, glob_size, label):
    from lakeside_amd import LK_PER_GLOB_ROWS
    from oracle import dataexpr as dx
    from oracle import exemplar as ex
    pr = dx.parse_pushdown(req)
    want = ex.evaluate_exemplar(pr, paths, glob_size, sources=blobs)
    got = engine.eval_pushdown(req, paths, glob_size, LK_PER_GLOB_ROWS)
    rows = list(zip(got.ts.tolist(), got.values.tolist(), got.tags, got.globs.tolist()))
    assert len(rows) == len(want), f"{label}: {len(rows)} rows vs {len(want)}"
    for i, (g, w) in enumerate(zip(rows, want)):
        assert g[0] == w[0] and g[3] == w[3], f"{label}: row {i}: (ts, glob) {g[0], g[3]} vs {w[0], w[3]}"
        assert g[1] == w[1] or (math.isnan(g[1]) and math.isnan(w[1])), f"{label}: row {i} value {g[1]} vs {w[1]}"
        assert g[2] == w[2], f"{label}: row {i} tags\n{g[2]}\nvs\n{w[2]}"
    return got


def test_exemplar_shapes(engine, tmp_path):
    from lakeside_amd import synth
    from oracle import dataexpr as dx
    paths, blobs = _logs_files(tmp_path)
    for p in paths:
        engine.load_segment(p)
    name_eq = synth.leaf(dx.NAME, "eq", "metric_02")
    svc_re = synth.leaf(SVC, "regex", "^svc-a")
    cases = [
        ("default", name_eq, {}, 2),
        ("limit7_asc", {"q1": svc_re, "q2": {"not": synth.leaf(dx.NAME, "eq", "metric_01")}, "op": "or"},
         {"limit": 7, "order": "asc"}, 2),
        ("reverse_sort", svc_re, {"limit": 50, "reverse": True}, 3),
        ("nonexistent_or", {"q1": synth.leaf("no.such.col", "eq", "x"), "q2": name_eq, "op": "or"}, {"limit": 25}, 10),
        ("limit0", name_eq, {"limit": 0}, 2),
        ("everything", {"k": SVC, "v": [], "op": "exists", "extracted": False, "computed": False, "dataType": "string"},
         {"limit": 100_000}, 4),
        ("contains_unicode", synth.leaf("_cardinalhq.message", "contains", "MSG 1"), {"limit": 333}, 1),
    ]
    # second round: zone-map probing from the ordered end (LK_EX_PROBE_ROWS, tests only: probe boundaries every few
    # thousand rows instead of 2^20, so these small globs go through it)
    for probe in (None, "3000"):
        if probe:
            os.environ["LK_EX_PROBE_ROWS"] = probe
        try:
            for label, filt, kw, gs in cases:
                req = _request(filt, len(paths), limit=kw.get("limit"), order=kw.get("order"),
                               reverse=kw.get("reverse", False))
                got = _check(engine, req, paths, blobs, gs, f"{label} probe={probe}")
                _shape_asserts(label, got)
        finally:
            os.environ.pop("LK_EX_PROBE_ROWS", None)


def _shape_asserts(label, got):
    if label == "everything":
        assert len(got) > 40_000                       # all passing rows of every glob
    if label == "default":
        assert len(got) > 1000 and {"attr.flag", "attr.ratio", "attr.count", "attr.big"} <= set(got.tag_names)


def test_exemplar_refinement_and_ties(engine, tmp_path):
    """A small candidate cap (LK_EX_CAND_CAP, tests only) forces the histogram refinement down to single
    milliseconds, with hundreds of rows tied on the boundary timestamp."""
    import pyarrow as pa
    import pyarrow.parquet as pq
    from lakeside_amd import synth
    from oracle import dataexpr as dx
    rng = np.random.default_rng(9)
    paths, blobs = [], []
    for i in range(3):
        n = 200_000
        ts = np.sort(synth.T0 + 100 * rng.integers(0, 2000, n))   # a 100 ms grid: ~100 rows per timestamp
        t = pa.table({dx.TIMESTAMP: pa.array(ts, pa.int64()),
                      dx.VALUE: pa.array(np.arange(n, dtype=np.float64) + i * 1e6),
                      dx.NAME: pa.array([f"metric_{k:02d}" for k in rng.integers(0, 3, n)], pa.string()),
                      "_cardinalhq.message": pa.array([f"m{k}" for k in rng.integers(0, 5, n)], pa.string())})
        path = str(tmp_path / f"ties{i}.parquet")
        pq.write_table(t, path, compression="NONE", use_dictionary=[dx.NAME, "_cardinalhq.message"],
                       column_encoding={dx.TIMESTAMP: "PLAIN", dx.VALUE: "PLAIN"}, row_group_size=65_536)
        engine.load_segment(path)
        paths.append(path)
        blobs.append(open(path, "rb").read())
    os.environ["LK_EX_CAND_CAP"] = "50"
    try:
        for limit, order in [(777, "desc"), (450, "asc"), (5, "desc")]:
            req = _request(synth.leaf(dx.NAME, "!=", "metric_00"), 3, limit=limit, order=order, hour=0)
            got = _check(engine, req, paths, blobs, 2, f"ties {limit} {order}")
            assert got.stats["hist_passes"] >= 2
    finally:
        del os.environ["LK_EX_CAND_CAP"]


def test_exemplar_errors(engine, tmp_path):
    """Metrics exemplars fail (getDouble of the name column) and a bad ORDER direction is an error; the Python
    mirror of evaluatePushDownRequest turns both into an empty result like the reference."""
    from lakeside_amd import LK_PER_GLOB_ROWS, LakesideError, synth
    from lakeside_amd.evaluator import evaluate_push_down_request
    from oracle import dataexpr as dx
    paths, _ = _logs_files(tmp_path, nfiles=2, rows=5000)
    for p in paths:
        engine.load_segment(p)
    for req in [_request(synth.leaf(dx.NAME, "eq", "metric_02"), 2, dataset="metrics"),
                _request(synth.leaf(dx.NAME, "eq", "metric_02"), 2, order="sideways")]:
        with pytest.raises(LakesideError):
            engine.eval_pushdown(req, paths, 10, LK_PER_GLOB_ROWS)
        assert evaluate_push_down_request(engine, "q", True, req, paths) == [[]]


def test_exemplar_java17_number_text(engine, tmp_path):
    """DOUBLE / FLOAT tag text is Java 17's Double.toString / Float.toString (the reference runs on
    eclipse-temurin:17): values whose JDK 17 digits are not the shortest round-trip ones (2e23, 2.82879384806159E17,
    Float.MIN_NORMAL, integers below 2^63 with noise digits) print as JDK 17 prints them, next to random bit patterns;
    every row is checked against the oracle and the pinned values against the JDK's documented strings."""
    import pyarrow as pa
    import pyarrow.parquet as pq
    from lakeside_amd import synth
    from oracle import dataexpr as dx
    from tests.test_jdtoa import PINNED_DOUBLE, PINNED_FLOAT
    rng = np.random.default_rng(17)
    n = 4000
    dv = rng.integers(0, 2 ** 64, n, dtype=np.uint64).view(np.float64).copy()
    fv = rng.integers(0, 2 ** 32, n, dtype=np.uint64).astype(np.uint32).view(np.float32).copy()
    dv[: len(PINNED_DOUBLE)] = [v for v, _ in PINNED_DOUBLE]
    fv[: len(PINNED_FLOAT)] = [v for v, _ in PINNED_FLOAT]
    dv[len(PINNED_DOUBLE): 200] = rng.integers(1, 2 ** 62, 200 - len(PINNED_DOUBLE)).astype(np.float64)
    dv[np.isnan(dv)] = 1.5
    fv[np.isnan(fv)] = 2.5
    ts = synth.T0 + np.arange(n, dtype=np.int64) * 10
    t = pa.table({dx.TIMESTAMP: pa.array(ts), dx.VALUE: pa.array(dv),
                  dx.NAME: pa.array(["m"] * n, pa.string()), "_cardinalhq.message": pa.array(["msg"] * n, pa.string()),
                  "attr.d": pa.array(dv), "attr.f": pa.array(fv)})
    path = str(tmp_path / "jdk17.parquet")
    strings = [dx.NAME, "_cardinalhq.message"]   # the logs projection needs the message column (a Binder Error without)
    pq.write_table(t, path, compression="NONE", use_dictionary=strings,
                   column_encoding={c: "PLAIN" for c in t.column_names if c not in strings})
    engine.load_segment(path)
    blobs = [open(path, "rb").read()]
    req = _request(synth.leaf(dx.NAME, "eq", "m"), 1, limit=n, order="asc", hour=0)
    got = _check(engine, req, [path], blobs, 1, "jdk17 text")
    assert len(got) == n
    texts_d = {got.tags[r]["attr.d"] for r in range(len(got))}
    texts_f = {got.tags[r]["attr.f"] for r in range(len(got))}
    for _, s in PINNED_DOUBLE:
        assert s in texts_d, s
    for _, s in PINNED_FLOAT:
        assert s in texts_f, s
