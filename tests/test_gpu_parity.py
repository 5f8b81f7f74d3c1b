"""Parity of the HIP path (through the C ABI) with the oracle and the committed golden rows (MI355X)."""
import json
import math
import os

import numpy as np
import pytest

from tests.parity import assert_rows_equal, check_columns, from_jsonable

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = os.path.join(HERE, "golden")

pytestmark = pytest.mark.gpu


def _cases():
    with open(os.path.join(GOLDEN, "cases.json")) as f:
        return json.load(f)


@pytest.fixture(scope="module")
def golden_engine(engine):
    for c in _cases():
        for p in c["segments"]:
            path = os.path.join(GOLDEN, p)
            if not _cached(engine, path):
                engine.load_segment(path)
    return engine


_loaded = set()


def _cached(engine, path):
    if path in _loaded:
        return True
    _loaded.add(path)
    return False


@pytest.mark.parametrize("case", _cases(), ids=lambda c: c["name"])
def test_golden_per_glob(golden_engine, case):
    from lakeside_amd import LK_PER_GLOB_ROWS
    paths = [os.path.join(GOLDEN, p) for p in case["segments"]]
    res = golden_engine.eval_pushdown(json.dumps(case["request"]), paths, case["glob_size"], LK_PER_GLOB_ROWS)
    agg = case["request"]["baseExpr"]["chart"]["aggregation"]
    got = res.per_glob(len(case["expected_per_glob"]))
    for gi, (g, w) in enumerate(zip(got, case["expected_per_glob"])):
        assert_rows_equal(g, from_jsonable(w), agg, f"{case['name']} glob {gi}")


@pytest.mark.parametrize("case", [c for c in _cases() if c["expected_merged"] is not None],
                         ids=lambda c: c["name"])
def test_golden_merged(golden_engine, case):
    from lakeside_amd import LK_MERGED
    paths = [os.path.join(GOLDEN, p) for p in case["segments"]]
    res = golden_engine.eval_pushdown(json.dumps(case["request"]), paths, case["glob_size"], LK_MERGED)
    agg = case["request"]["baseExpr"]["chart"]["aggregation"]
    assert_rows_equal(res.rows(), from_jsonable(case["expected_merged"]), agg, case["name"])


def _tag_cases():
    out = []
    for fn in ("tag_cases.json", "numtag_cases.json"):   # string tags; numeric tags (make_numtag_cases.py)
        with open(os.path.join(GOLDEN, fn)) as f:
            out += json.load(f)
    return out


def _tag_key(t):
    return sorted(t.items())


@pytest.mark.parametrize("case", _tag_cases(), ids=lambda c: c["name"])
def test_golden_tag_query(golden_engine, case):
    """Tag queries (isTagQuery + tagDataType; BaseExpr.scala:127-143): per-glob rows {tag, count} and merged
    counts equal the golden rows (oracle pinned by the reference's tag SQL on SQLite).  Numeric tag columns
    (numtag_cases.json: INT64 / INT32 / DOUBLE / FLOAT / BOOLEAN and their union_by_name unions) print as JDBC
    getString of the glob's union type (ex_scan TAGNUM)."""
    from lakeside_amd import LK_MERGED, LK_PER_GLOB_ROWS
    paths = [os.path.join(GOLDEN, p) for p in case["segments"]]
    for p in paths:
        if not _cached(golden_engine, p):
            golden_engine.load_segment(p)
    req = json.dumps(case["request"])
    tag = case["request"]["tagDataType"]["tagName"]
    res = golden_engine.eval_pushdown(req, paths, case["glob_size"], LK_PER_GLOB_ROWS)
    assert res.tag_names == [tag, "count"]
    assert all(int(v) == int(t["count"]) for v, t in zip(res.values, res.tags))
    got = res.per_glob(len(case["expected_per_glob"]))
    for gi, (g, w) in enumerate(zip(got, case["expected_per_glob"])):
        assert sorted((r[2] for r in g), key=_tag_key) == sorted(w, key=_tag_key), f"{case['name']} glob {gi}"
    res = golden_engine.eval_pushdown(req, paths, case["glob_size"], LK_MERGED)
    assert sorted(res.tags, key=_tag_key) == sorted(case["expected_merged"], key=_tag_key)


def test_no_segments_sentinel(engine):
    from lakeside_amd.evaluator import evaluate_push_down_request
    req = {"baseExpr": {"id": "A", "dataset": "logs", "filter": {"k": "_cardinalhq.name", "v": ["x"], "op": "eq"},
                        "chart": {"aggregation": "sum", "groupBys": []}},
           "segmentRequests": [], "reverseSort": False, "isTagQuery": False}
    rows = evaluate_push_down_request(engine, "q", True, json.dumps(req), [])
    assert rows == [[(-1, -1.0, {})]]


def _synth_case(engine, nseg, rows, value_mode, null_frac, filt, agg, group_bys, step=60000, glob_size=10,
                window=None, highcard_n=0, hour=None):
    """Synthetic segments written by tools/synth.cpp, evaluated by the GPU and by the oracle on the same bytes.
    window=(lo, hi): the segment requests' [startTs, endTs) narrowed by lo ms at the start and hi ms at the end."""
    import pyarrow as pa  # noqa: F401
    from lakeside_amd import LK_MERGED, LK_PER_GLOB_ROWS
    from lakeside_amd import synth
    from oracle import dataexpr as dx
    keys, blobs, segs = [], [], []
    for i in range(nseg):
        s = synth.make_segment(synth.segment_spec(i, rows=rows, value_mode=value_mode, null_frac=null_frac,
                                                  rg_rows=1 << 18, page_rows=1 << 15, highcard_n=highcard_n,
                                                  hour=hour))
        key = f"synth/{rows}/{value_mode}/{null_frac}/{highcard_n}/{hour}/{i}"
        engine.put_segment_ptr(key, s.ptr, s.size)
        blobs.append(s.bytes())
        s.free()
        keys.append(key)
        segs.append(synth.segment_request(i, step=step, hour=hour))
        if window:
            segs[-1]["startTs"] += window[0]
            segs[-1]["endTs"] -= window[1]
    req = json.dumps(synth.pushdown(filt, segs, agg, group_bys))
    if highcard_n >= 20_000 and not null_frac:   # 10^5-10^6 result rows: column-wise vs the C++ restatement
        return check_columns(engine, req, keys, blobs, glob_size)["merged"]
    pr = dx.parse_pushdown(req)
    cells = dx.evaluate_glob_cells(pr, glob_size, keys, sources=blobs)
    want_pg = [[(c.ts, c.agg_value(agg), c.tags) for c in cs] for cs in cells]
    got = engine.eval_pushdown(req, keys, glob_size, LK_PER_GLOB_ROWS).per_glob(len(want_pg))
    for gi, (g, w) in enumerate(zip(got, want_pg)):
        assert_rows_equal(g, w, agg, f"glob {gi}")
    merged = engine.eval_pushdown(req, keys, glob_size, LK_MERGED)
    assert_rows_equal(merged.rows(), dx.merge_glob_cells(pr, cells), agg, "merged")
    return merged


def test_c1_shape_eq_sum(engine):
    """C1: 1 segment x 2^20 rows, :eq name :sum, 1m step (bit-exact on integer values)."""
    from lakeside_amd import synth
    res = _synth_case(engine, 1, 1 << 20, 0, 0.0, synth.leaf(synth.NAME, "eq", "metric_07"), "sum", [])
    assert len(res) == 60


def test_real_values_sum_within_one_ulp(engine):
    from lakeside_amd import synth
    _synth_case(engine, 3, 1 << 19, 1, 0.0, synth.leaf(synth.NAME, "in", "metric_01", "metric_02"), "sum", [])


def test_avg_merged_single_scan(engine):
    """Merged avg = Σsum / Σcount of the SUM and COUNT pushdowns query-api would send (one scan here), with
    NULL values (all-NULL cells: 0/0 = NaN), with and without groupBys."""
    from lakeside_amd import synth
    _synth_case(engine, 3, 1 << 19, 1, 0.05, synth.leaf(synth.NAME, "in", "metric_01", "metric_02"), "avg", [])
    _synth_case(engine, 2, 1 << 18, 1, 0.3, synth.leaf(synth.NAME, "eq", "metric_04"), "avg",
                [synth.SERVICE, synth.NAMESPACE], step=10000)


def test_c3_shape_and_regex_by2_max_with_nulls(engine):
    from lakeside_amd import synth
    filt = {"op": "and", "q1": synth.leaf(synth.NAME, "eq", "metric_07"),
            "q2": synth.leaf(synth.SERVICE, "regex", "^svc-0[0-4]")}
    _synth_case(engine, 4, 1 << 19, 1, 0.05, filt, "max", [synth.SERVICE, synth.NAMESPACE])


@pytest.mark.parametrize("late_chunk", [False, True], ids=["per_row", "late_chunk"])
def test_late_materialization_paths(engine, late_chunk, monkeypatch):
    """NULL-free tiles take the late path: the early column (a conjunct on one column alone, name first) is
    decoded for every row, every other string column only for rows the early conjuncts pass -- per listed row
    (default) or per 16-row chunk (LK_LATE_CHUNK=1: scan_lean<..., EARLY>)."""
    from lakeside_amd import synth
    if late_chunk:
        monkeypatch.setenv("LK_LATE_CHUNK", "1")
    c3 = {"op": "and", "q1": synth.leaf(synth.NAME, "eq", "metric_07"),
          "q2": synth.leaf(synth.SERVICE, "regex", "^svc-0[0-4]")}
    _synth_case(engine, 3, 1 << 19, 1, 0.0, c3, "max", [synth.SERVICE, synth.NAMESPACE])          # C3 shape
    _synth_case(engine, 3, 1 << 19, 0, 0.0, synth.leaf(synth.NAME, "eq", "metric_07"), "sum",
                [synth.SERVICE])                                                                   # C4 shape
    late_or = {"op": "and", "q1": synth.leaf(synth.NAME, "in", "metric_01", "metric_02"),
               "q2": {"op": "or", "q1": synth.leaf(synth.SERVICE, "!=", "svc-003"),
                      "q2": {"not": synth.leaf(synth.NAMESPACE, "eq", "ns-01")}}}
    _synth_case(engine, 2, 1 << 19, 1, 0.0, late_or, "count", [synth.NAMESPACE])
    # early column other than name: name becomes a late group dim
    _synth_case(engine, 2, 1 << 19, 1, 0.0, synth.leaf(synth.SERVICE, "in", "svc-010", "svc-011"), "min",
                [synth.NAME])
    # a conjunct mixing the early column with another: no late pass
    mixed = {"op": "and", "q1": synth.leaf(synth.NAME, "in", "metric_01", "metric_02"),
             "q2": {"op": "or", "q1": synth.leaf(synth.NAME, "eq", "metric_01"),
                    "q2": synth.leaf(synth.SERVICE, "eq", "svc-003")}}
    _synth_case(engine, 2, 1 << 19, 1, 0.0, mixed, "sum", [synth.SERVICE])


def test_groupby_count_min_with_nulls(engine):
    from lakeside_amd import synth
    filt = {"op": "or", "q1": {"not": synth.leaf(synth.SERVICE, "eq", "svc-001")},
            "q2": synth.leaf(synth.NAMESPACE, "in", "ns-01")}
    _synth_case(engine, 2, 1 << 18, 1, 0.05, filt, "count", [synth.NAMESPACE], step=300000)
    _synth_case(engine, 2, 1 << 18, 1, 0.05, filt, "min", [synth.NAMESPACE], step=10000)


def test_zone_map_bucket_paths(engine):
    """Tiles whose timestamps fall in one step bucket skip the timestamp read (zone-map bucket); the others read
    it. 2^22 rows/hour at a 1m step: most 32K-row tiles sit inside one minute, some straddle a boundary; a 1h
    step puts every tile in one bucket; a 7s step none."""
    from lakeside_amd import synth
    filt = synth.leaf(synth.NAME, "in", "metric_03", "metric_11")
    _synth_case(engine, 2, 1 << 22, 1, 0.05, filt, "sum", [synth.NAME])
    _synth_case(engine, 1, 1 << 22, 0, 0.0, filt, "count", [], step=3600000)
    _synth_case(engine, 1, 1 << 21, 1, 0.0, filt, "max", [], step=7000)


@pytest.mark.parametrize("split", [True, False], ids=["split", "no_split"])
def test_split_tiles_sorted_timestamps(engine, split, monkeypatch):
    """Tiles whose timestamps never decrease (TILE_TS_SORTED) and span 2-3 buckets take the split path: bucket and
    window boundaries found by searching the timestamps, rows bucketed by index with no timestamp gather.  Steps
    putting 1-4 boundaries inside a 32K-row tile (~56 s of data), a window cutting tiles at both ends, and a 7 s step
    whose tiles span too many buckets (per-row timestamps again) -- each against the oracle, with and without it."""
    from lakeside_amd import synth
    if not split:
        monkeypatch.setenv("LK_NO_SPLIT", "1")
    filt = synth.leaf(synth.NAME, "in", "metric_03", "metric_11")
    _synth_case(engine, 2, 1 << 21, 1, 0.0, filt, "sum", [synth.NAME], step=20000)
    _synth_case(engine, 1, 1 << 21, 0, 0.0, filt, "count", [], step=30000, window=(7 * 60000 + 123, 11 * 60000 - 17))
    _synth_case(engine, 1, 1 << 21, 1, 0.0, filt, "max", [synth.SERVICE], step=60000, window=(45_000, 1_001))
    _synth_case(engine, 1, 1 << 21, 1, 0.0, filt, "min", [], step=7000)


def test_window_cuts_tiles(engine):
    """A glob window narrower than the data: tiles crossing either edge filter rows by timestamp, tiles outside
    are skipped by their zone map."""
    from lakeside_amd import synth
    filt = synth.leaf(synth.NAME, "eq", "metric_05")
    _synth_case(engine, 2, 1 << 21, 1, 0.02, filt, "sum", [], window=(7 * 60000 + 123, 11 * 60000 - 17))
    _synth_case(engine, 1, 1 << 21, 0, 0.0, filt, "count", [], step=3600000, window=(60000, 0))


@pytest.mark.parametrize("rows_mode", ["key_rows", "ts_runs"])
def test_c5_shape_high_cardinality_group_by(engine, rows_mode, monkeypatch):
    """C5 shape: a high-cardinality group key (resource.container.id, 300k-value dictionary, ~2^18 distinct per
    row group) over segments of one hour, 1h step: groups far beyond the LDS table spill to the global table.  Large
    results cross the host link as values + key bits (default since r06) or values + group ids with the timestamps
    expanded on the host (LK_NO_KEY_ROWS=1)."""
    from lakeside_amd import synth
    if rows_mode == "ts_runs":
        monkeypatch.setenv("LK_NO_KEY_ROWS", "1")
    filt = synth.leaf(synth.NAME, "eq", "metric_07")
    res = _synth_case(engine, 2, 1 << 20, 0, 0.0, filt, "sum", [synth.CONTAINER], step=3600000, highcard_n=300000,
                      hour=0)
    assert len(res) > 50000
    _synth_case(engine, 2, 1 << 19, 1, 0.05, filt, "max", [synth.CONTAINER], step=600000, highcard_n=100000,
                hour=0)
    # 60 buckets x 20k groups (1.2M output keys): the timestamps of a result this large are expanded on the host from
    # each bucket's first row (FParams::bucket_pos); most buckets' first keys are empty cells
    _synth_case(engine, 1, 1 << 20, 0, 0.0, filt, "count", [synth.CONTAINER], step=60000, highcard_n=20000, hour=0)


def test_large_result_rows_from_key_bits(engine):
    """Key-bit rows (default since r06): a large grouped result's rows carry only their values over the host link;
    timestamps, group ids and globs come from finalize_count's per-key existence bits -- per glob and merged, one and
    60 buckets."""
    from lakeside_amd import synth
    filt = synth.leaf(synth.NAME, "eq", "metric_07")
    _synth_case(engine, 2, 1 << 20, 0, 0.0, filt, "sum", [synth.CONTAINER], step=3600000, highcard_n=300000, hour=0)
    _synth_case(engine, 1, 1 << 20, 0, 0.0, filt, "count", [synth.CONTAINER], step=60000, highcard_n=20000, hour=0)


@pytest.mark.parametrize("exact", [True, False], ids=["exact_sum", "compensated"])
def test_integral_sums_exact_and_compensated(engine, exact, monkeypatch):
    """Integer values (load-time summary: every value integral, |v| <= 999): SUM adds are fire-and-forget
    (QParams::exact_sum) -- on the direct LDS table, the LDS hash table and the global table (C5 shape, global
    cells) -- and equal the compensated path (LK_NO_EXACT_SUM=1) and the oracle bit for bit.  Real values never
    take it."""
    from lakeside_amd import synth
    if not exact:
        monkeypatch.setenv("LK_NO_EXACT_SUM", "1")
    filt = synth.leaf(synth.NAME, "in", "metric_03", "metric_09")
    res = _synth_case(engine, 2, 1 << 20, 0, 0.0, filt, "sum", [synth.SERVICE])
    assert res.stats["exact_sum"] == (1 if exact else 0)
    res = _synth_case(engine, 2, 1 << 19, 0, 0.0, filt, "avg", [synth.NAMESPACE], step=10000)
    assert res.stats["exact_sum"] == (1 if exact else 0)
    res = _synth_case(engine, 2, 1 << 20, 0, 0.0, synth.leaf(synth.NAME, "eq", "metric_07"), "sum", [synth.CONTAINER],
                      step=3600000, highcard_n=2_000_000, hour=0)
    assert res.stats["exact_sum"] == (1 if exact else 0) and res.stats["global_cells"] == 1
    res = _synth_case(engine, 2, 1 << 19, 1, 0.0, filt, "sum", [synth.SERVICE])
    assert res.stats["exact_sum"] == 0   # real values


def test_full_size_properties(engine):
    """At a BASELINE-sized segment (2^24 rows): counts are exact, every row lands in one bucket, and the
    per-name counts over all buckets add up to the rows of the segment (no row lost or double counted)."""
    from lakeside_amd import LK_MERGED
    from lakeside_amd import synth
    s = synth.make_segment(synth.segment_spec(0, rows=1 << 24))
    engine.put_segment_ptr("synth/full/0", s.ptr, s.size)
    s.free()
    seg = synth.segment_request(0)
    names = [f"metric_{i:02d}" for i in range(16)]
    req = json.dumps(synth.pushdown(synth.leaf(synth.NAME, "in", *names), [seg], "count", [synth.NAME]))
    res = engine.eval_pushdown(req, ["synth/full/0"], 10, LK_MERGED)
    assert len(res) == 60 * 16
    assert int(res.values.sum()) == 1 << 24
    req = json.dumps(synth.pushdown(synth.leaf(synth.NAME, "eq", "metric_03"), [seg], "count", []))
    part = engine.eval_pushdown(req, ["synth/full/0"], 10, LK_MERGED)
    by_ts = {}
    for t, v, tags in res.rows():
        if tags["name"] == "metric_03":
            by_ts[t] = v
    assert {t: v for t, v, _ in part.rows()} == by_ts


def test_queryapi_end_to_end(engine):
    """query-api over the engine (lakeside_amd/queryapi.py: merged table -> drop future -> transformer ->
    group-key collapse -> payload) vs the oracle's merge + final_eval: merged avg in one scan with a rate chart,
    a :by whose rows collide on the group key (name differs), and :and/:re :max with a rate chart."""
    from lakeside_amd import queryapi, synth
    from oracle import dataexpr as dx
    keys, blobs, segs = [], [], []
    for i in range(3):
        s = synth.make_segment(synth.segment_spec(i, rows=1 << 19, value_mode=1, null_frac=0.05, rg_rows=1 << 18,
                                                  page_rows=1 << 15))
        key = f"queryapi/{i}"
        engine.put_segment_ptr(key, s.ptr, s.size)
        blobs.append(s.bytes())
        s.free()
        keys.append(key)
        segs.append(synth.segment_request(i, step=60000))
    names = synth.leaf(synth.NAME, "in", "metric_01", "metric_02")
    c3 = {"op": "and", "q1": synth.leaf(synth.NAME, "eq", "metric_03"),
          "q2": synth.leaf(synth.SERVICE, "regex", "^svc-0[0-4]")}
    now = synth.T0 + 2 * synth.HOUR + 30 * 60000          # the last half hour is "in the future": dropped
    for filt, agg, gbs, ctype in [(names, "avg", [], "rate"), (names, "sum", [synth.NAMESPACE], "count"),
                                  (c3, "max", [synth.SERVICE], "rate")]:
        req = synth.pushdown(filt, segs, agg, gbs)
        be = req["baseExpr"]
        be["chart"]["type"] = ctype
        got = queryapi.evaluate_base_expr(engine, be, segs, keys, 60000, now_ms=now)
        pr = dx.parse_pushdown(json.dumps(req))
        merged = dx.merge_glob_cells(pr, dx.evaluate_glob_cells(pr, 10, keys, sources=blobs))
        want = dx.final_eval(be, merged, 60000, now)
        assert len(got) == len(want) > 0, (agg, len(got), len(want))
        for g, w in zip(got, want):
            gm, wm = g["message"], w["message"]
            assert (gm["timestamp"], gm["tags"], gm["label"]) == (wm["timestamp"], wm["tags"], wm["label"])
            gv, wv = gm["value"], wm["value"]
            tol = 2 * math.ulp(wv) if agg in ("sum", "avg") else 0.0     # <= 1 ulp sum, then one division
            assert gv == wv or (math.isnan(gv) and math.isnan(wv)) or abs(gv - wv) <= tol, (agg, gm, wm)


@pytest.mark.parametrize("codec", ["snappy", "gzip", "zstd", "lz4"])
def test_compressed_segments(engine, tmp_path, codec):
    """Compressed column chunks: the golden segments rewritten with each codec (v1 and v2
    pages as in the originals), loaded through the engine (pages decompressed at load, HBM holds plain
    streams), give the golden rows."""
    import pyarrow.parquet as pq
    from lakeside_amd import LK_MERGED, LK_PER_GLOB_ROWS
    cases = {c["name"]: c for c in _cases()}
    for name in ["c1_eq_sum", "c3_and_regex_by2_max", "null_group_key_count", "metrics_rollup_sum",
                 "window_clip"]:
        case = cases[name]
        paths = []
        for p in case["segments"]:
            src = os.path.join(GOLDEN, p)
            dst = os.path.join(str(tmp_path), f"{codec}_{os.path.basename(p)}")
            if not os.path.exists(dst):
                f = pq.ParquetFile(src)
                t = f.read()
                strings = [c for c in t.column_names if str(t.schema.field(c).type) == "string"]
                v2 = codec in ("snappy", "zstd")       # v2 pages: levels stay plain, values compressed
                pq.write_table(t, dst, compression=codec, use_dictionary=strings,
                               column_encoding={c: "PLAIN" for c in t.column_names if c not in strings},
                               data_page_version="2.0" if v2 else "1.0",
                               row_group_size=f.metadata.row_group(0).num_rows, data_page_size=4096)
            paths.append(dst)
        req = json.dumps(case["request"])
        agg = case["request"]["baseExpr"]["chart"]["aggregation"]
        got = engine.eval_pushdown(req, paths, case["glob_size"], LK_PER_GLOB_ROWS).per_glob(len(case["expected_per_glob"]))
        for gi, (g, w) in enumerate(zip(got, case["expected_per_glob"])):
            assert_rows_equal(g, from_jsonable(w), agg, f"{codec} {name} glob {gi}")
        if case["expected_merged"] is not None:
            res = engine.eval_pushdown(req, paths, case["glob_size"], LK_MERGED)
            assert_rows_equal(res.rows(), from_jsonable(case["expected_merged"]), agg, f"{codec} {name} merged")


def test_plain_string_pages(engine, tmp_path):
    """PLAIN BYTE_ARRAY string pages: a writer's dictionary fallback mid-chunk (tiny
    dictionary page limit on a high-cardinality column) and columns written without dictionaries, compressed
    and not; each fallback page gets its own dictionary at load."""
    import pyarrow as pa
    import pyarrow.parquet as pq
    from lakeside_amd import LK_MERGED, LK_PER_GLOB_ROWS, synth
    from oracle import dataexpr as dx
    rng = np.random.default_rng(11)
    keys, blobs, segs = [], [], []
    for i, (dicts, codec) in enumerate([([synth.NAME, synth.SERVICE, synth.CONTAINER], "NONE"),
                                        ([synth.NAME], "zstd"), ([], "snappy")]):
        n = 200_000
        t0 = synth.T0 + i * synth.HOUR
        t = pa.table({
            dx.TIMESTAMP: pa.array(np.sort(rng.integers(t0, t0 + synth.HOUR, n)), pa.int64()),
            dx.VALUE: pa.array(rng.integers(0, 1000, n).astype(np.float64), pa.float64(), mask=rng.random(n) < 0.05),
            synth.NAME: pa.array([f"metric_{k:02d}" for k in rng.integers(0, 16, n)], pa.string()),
            synth.SERVICE: pa.array([f"svc-{k:03d}" for k in rng.integers(0, 100, n)], pa.string(),
                                    mask=rng.random(n) < 0.05),
            synth.CONTAINER: pa.array([f"c{k:07d}" for k in rng.integers(0, 60_000, n)], pa.string()),
        })
        path = str(tmp_path / f"plain{i}.parquet")
        pq.write_table(t, path, compression=codec, use_dictionary=dicts, dictionary_pagesize_limit=16384,
                       column_encoding={c: "PLAIN" for c in t.column_names if c not in dicts},
                       row_group_size=100_000, data_page_size=32768)
        engine.load_segment(path)
        keys.append(path)
        blobs.append(open(path, "rb").read())
        segs.append(synth.segment_request(i))
    for filt, agg, gbs in [(synth.leaf(synth.NAME, "eq", "metric_07"), "sum", [synth.CONTAINER]),
                           (synth.leaf(synth.SERVICE, "regex", "^svc-0[0-4]"), "count", [synth.SERVICE]),
                           (synth.leaf(synth.CONTAINER, "in", "c0000001", "c0000002", "c0059999"), "max", [])]:
        req = json.dumps(synth.pushdown(filt, segs, agg, gbs))
        pr = dx.parse_pushdown(req)
        cells = dx.evaluate_glob_cells(pr, 2, keys, sources=blobs)
        got = engine.eval_pushdown(req, keys, 2, LK_PER_GLOB_ROWS).per_glob(len(cells))
        for gi, (g, cs) in enumerate(zip(got, cells)):
            assert_rows_equal(g, [(c.ts, c.agg_value(agg), c.tags) for c in cs], agg, f"plain glob {gi}")
        merged = engine.eval_pushdown(req, keys, 2, LK_MERGED)
        assert_rows_equal(merged.rows(), dx.merge_glob_cells(pr, cells), agg, "plain merged")


def test_tag_query_synthetic_with_nulls(engine):
    """Tag query over synthetic segments (NULL tags, a window cutting tiles, globs of 2): per-glob {tag, count}
    rows and merged counts equal the oracle on the same bytes."""
    from lakeside_amd import LK_MERGED, LK_PER_GLOB_ROWS
    from lakeside_amd import synth
    from oracle import dataexpr as dx
    keys, blobs, segs = [], [], []
    for i in range(3):
        s = synth.make_segment(synth.segment_spec(i, rows=1 << 20, null_frac=0.05, rg_rows=1 << 18,
                                                  page_rows=1 << 15))
        key = f"synth-tag/{i}"
        engine.put_segment_ptr(key, s.ptr, s.size)
        blobs.append(s.bytes())
        s.free()
        keys.append(key)
        segs.append(synth.segment_request(i))
        segs[-1]["startTs"] += 123_457
        segs[-1]["endTs"] -= 654_321
    filt = {"op": "and", "q1": synth.leaf(synth.NAME, "in", "metric_03", "metric_07"),
            "q2": {"not": synth.leaf(synth.NAMESPACE, "eq", "ns-03")}}
    for tag in (synth.SERVICE, synth.NAME):
        req = json.dumps(synth.pushdown(filt, segs, tag=tag))
        pr = dx.parse_pushdown(req)
        want = dx.evaluate_tag_per_glob(pr, tag, keys, 2, sources=blobs)
        got = engine.eval_pushdown(req, keys, 2, LK_PER_GLOB_ROWS).per_glob(len(want))
        key = lambda t: sorted(t.items())   # noqa: E731
        for gi, (g, w) in enumerate(zip(got, want)):
            assert sorted((r[2] for r in g), key=key) == sorted(w, key=key), f"{tag} glob {gi}"
        merged = engine.eval_pushdown(req, keys, 2, LK_MERGED)
        assert sorted(merged.tags, key=key) == sorted(dx.evaluate_tag_merged(pr, tag, keys, 2, sources=blobs), key=key)


def test_concurrent_calls_from_threads(golden_engine):
    """The ABI is called from several dispatcher threads at once (re-entrant, thread-safe):
    four threads evaluate golden chart and tag cases concurrently on one engine, while another thread re-puts a
    segment into the HBM cache; every result equals the golden rows."""
    import threading
    from lakeside_amd import LK_MERGED, LK_PER_GLOB_ROWS
    cases = [c for c in _cases() if c["expected_merged"] is not None]
    tag_cases = _tag_cases()
    errors = []

    def worker(k):
        try:
            for it in range(3):
                for case in cases[k::4]:
                    paths = [os.path.join(GOLDEN, p) for p in case["segments"]]
                    res = golden_engine.eval_pushdown(json.dumps(case["request"]), paths, case["glob_size"], LK_MERGED)
                    agg = case["request"]["baseExpr"]["chart"]["aggregation"]
                    assert_rows_equal(res.rows(), from_jsonable(case["expected_merged"]), agg, f"thread {k} {case['name']}")
                for case in tag_cases[k::4]:
                    paths = [os.path.join(GOLDEN, p) for p in case["segments"]]
                    res = golden_engine.eval_pushdown(json.dumps(case["request"]), paths, case["glob_size"],
                                                      LK_PER_GLOB_ROWS)
                    got = sorted((sorted(t.items()) for t in res.tags))
                    want = sorted(sorted(t.items()) for g in case["expected_per_glob"] for t in g)
                    assert got == want, f"thread {k} tag {case['name']}"
        except Exception as e:   # noqa: BLE001 - reported below
            errors.append(e)

    def loader():
        try:
            p = os.path.join(GOLDEN, "segments", "seg13.parquet")
            with open(p, "rb") as f:
                data = f.read()
            for _ in range(5):
                golden_engine.put_segment("concurrent/seg13", data)
        except Exception as e:   # noqa: BLE001
            errors.append(e)

    ts = [threading.Thread(target=worker, args=(k,)) for k in range(4)] + [threading.Thread(target=loader)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=240)
    assert not any(t.is_alive() for t in ts), "a thread did not finish"
    assert not errors, errors[0]


@pytest.mark.parametrize("pattern", ["(?i)^SVC-0[0-4]", "\\Asvc-0[0-4]", "(?P<id>svc-0[1-3])[0-9]\\z", "[]x]|svc-09",
                                     "\\Qsvc-01\\E", "\\pL{3}-0[[:digit:]]1", "[[:digit:]a]\\z", "(?-i:SVC)|svc-0(?:0|4)7",
                                     "^(svc-0[0-2]){1}\\d$", "\\bsvc-0[0-4]\\B"])
def test_regex_re2_spellings(golden_engine, pattern):
    """RE2 syntax (flags, \\A / \\z, named groups, \\Q..\\E, Unicode and POSIX classes, word boundaries) through
    the evaluator's RE2-semantics matcher equals RE2 (oracle: pyarrow's RE2, the engine behind DuckDB's
    regexp_matches)."""
    from lakeside_amd import LK_MERGED
    from oracle import dataexpr as dx
    case = next(c for c in _cases() if c["name"] == "c3_and_regex_by2_max")
    req = json.loads(json.dumps(case["request"]))
    req["baseExpr"]["filter"]["q2"]["v"] = [pattern]
    paths = [os.path.join(GOLDEN, p) for p in case["segments"]]
    text = json.dumps(req)
    got = golden_engine.eval_pushdown(text, paths, case["glob_size"], LK_MERGED)
    want = dx.evaluate_merged(dx.parse_pushdown(text), paths, case["glob_size"])
    assert len(want) > 0
    assert_rows_equal(got.rows(), want, "max", pattern)


def test_regex_non_ascii_dictionary_values(engine, tmp_path):
    """regex / contains over non-ASCII tag values (case-fold orbits: sigma, Kelvin sign, long s; accents; CJK):
    the leaf outcome per dictionary value equals RE2's (pyarrow), so the GPU rows equal the oracle's."""
    import pyarrow as pa
    import pyarrow.parquet as pq
    from lakeside_amd import LK_MERGED, synth
    from oracle import dataexpr as dx
    rng = np.random.default_rng(5)
    vocab = ["Σίσυφος", "σίσυφος", "ΣΊΣΥΦΟΣ", "KELVIN-K", "kelvin-k", "ſtraße", "STRASSE", "école", "ÉCOLE",
             "日本語", "naïve café", "svc-001", "İstanbul", "istanbul", "ǅungla", "null", ""]
    n = 100_000
    t0 = synth.T0
    t = pa.table({
        dx.TIMESTAMP: pa.array(np.sort(rng.integers(t0, t0 + synth.HOUR, n)), pa.int64()),
        dx.VALUE: pa.array(rng.integers(0, 1000, n).astype(np.float64), pa.float64()),
        synth.NAME: pa.array([f"metric_{k:02d}" for k in rng.integers(0, 4, n)], pa.string()),
        synth.SERVICE: pa.array([vocab[k] for k in rng.integers(0, len(vocab), n)], pa.string(),
                                mask=rng.random(n) < 0.03),
    })
    path = str(tmp_path / "nonascii.parquet")
    pq.write_table(t, path, compression="NONE", use_dictionary=[synth.NAME, synth.SERVICE],
                   column_encoding={dx.TIMESTAMP: "PLAIN", dx.VALUE: "PLAIN"}, row_group_size=50_000)
    engine.load_segment(path)
    segs = [synth.segment_request(0)]
    for op, pat in [("regex", "σίσυφος"), ("regex", "^kelvin"), ("regex", "STRASSE|ſtr"), ("contains", "É"),
                    ("regex", "^.{3}$"), ("regex", "\\p{Lu}"), ("regex", "i̇|^ist"), ("contains", "ǆ"),
                    ("regex", "[^\\x00-\\x7f]"), ("regex", "\\bcaf")]:
        req = json.dumps(synth.pushdown(synth.leaf(synth.SERVICE, op, pat), segs, "count", [synth.SERVICE]))
        got = engine.eval_pushdown(req, [path], 10, LK_MERGED)
        want = dx.evaluate_merged(dx.parse_pushdown(req), [path], 10)
        assert_rows_equal(got.rows(), want, "count", f"{op} {pat}")


def test_numeric_tag_high_cardinality_regrowth(engine):
    """A tag query over a DOUBLE column whose values are nearly all distinct (the value column itself): workgroup
    LDS tables overflow to the device table, which starts at 64 slots (LK_TAGNUM_INIT_SLOTS) and is regrown; every
    (value text, count) equals the oracle's."""
    from lakeside_amd import LK_MERGED, synth
    from oracle import dataexpr as dx
    blobs, keys = [], []
    for i in range(2):
        s = synth.make_segment(synth.segment_spec(i, rows=1 << 16, rg_rows=1 << 15, page_rows=1 << 13))
        blobs.append(s.bytes())
        engine.put_segment_ptr(f"numtag_hc/{i}", s.ptr, s.size)
        s.free()
        keys.append(f"numtag_hc/{i}")
    tag = dx.VALUE
    req = {"baseExpr": {"id": "A", "dataset": "logs", "limit": 1000, "order": "DESC", "returnResults": True,
                        "filter": {"op": "and", "q1": synth.leaf(synth.NAME, "eq", "metric_07"),
                                   "q2": synth.leaf(tag, "exists")}},
           "segmentRequests": [synth.segment_request(i) for i in range(2)], "reverseSort": False,
           "isTagQuery": True, "tagDataType": {"tagName": tag, "dataType": "number"}}
    text = json.dumps(req)
    os.environ["LK_TAGNUM_INIT_SLOTS"] = "64"
    try:
        res = engine.eval_pushdown(text, keys, 10, LK_MERGED)
    finally:
        os.environ.pop("LK_TAGNUM_INIT_SLOTS")
    assert res.stats["attempts"] > 1 and res.stats["table"] == "tagnum", res.stats
    want = dx.evaluate_tag_merged(dx.parse_pushdown(text), tag, keys, 10, sources=blobs)
    assert len(want) >= 1000   # (synthetic values: 1000 distinct integers)
    assert sorted(res.tags, key=_tag_key) == sorted(want, key=_tag_key)
