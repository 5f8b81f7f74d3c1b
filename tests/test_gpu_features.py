"""GPU parity of the §8(f) widenings (metrics specifics, other worker query shapes) against the oracle, through
the C ABI on the MI355X."""
import json
import os

import numpy as np
import pytest

from tests.parity import assert_rows_equal

pytestmark = pytest.mark.gpu


def _metrics_segments(engine, tmp_path, specs, n=150_000):
    """Metrics segments (rollup_sum / rollup_max value columns) written by pyarrow; specs = [(hour, aligned)]:
    aligned timestamps sit on the 60 s step grid, unaligned ones on arbitrary milliseconds."""
    import pyarrow as pa
    import pyarrow.parquet as pq
    from lakeside_amd import synth
    from oracle import dataexpr as dx
    rng = np.random.default_rng(77)
    keys, blobs, segs = [], [], []
    for i, (hour, aligned) in enumerate(specs):
        t0 = synth.T0 + hour * synth.HOUR
        ts = t0 + (60_000 * rng.integers(0, 60, n) if aligned else rng.integers(0, synth.HOUR, n))
        vals = rng.integers(0, 1000, n).astype(np.float64)
        t = pa.table({
            dx.TIMESTAMP: pa.array(np.sort(ts), pa.int64()),
            "rollup_sum": pa.array(vals, pa.float64(), mask=rng.random(n) < 0.03),
            "rollup_max": pa.array(vals * 2, pa.float64()),
            synth.NAME: pa.array([f"metric_{k:02d}" for k in rng.integers(0, 4, n)], pa.string()),
            synth.SERVICE: pa.array([f"svc-{k:03d}" for k in rng.integers(0, 7, n)], pa.string(),
                                    mask=rng.random(n) < 0.05),
        })
        path = str(tmp_path / f"metrics{i}.parquet")
        strings = [synth.NAME, synth.SERVICE]
        pq.write_table(t, path, compression="NONE", use_dictionary=strings,
                       column_encoding={c: "PLAIN" for c in t.column_names if c not in strings},
                       row_group_size=n // 3, data_page_size=65536)
        engine.load_segment(path)
        keys.append(path)
        blobs.append(open(path, "rb").read())
        segs.append(synth.segment_request(i, hour=hour, dataset="metrics"))
    return keys, blobs, segs


def test_metrics_unaligned_timestamps(engine, tmp_path):
    """Metrics group by the raw timestamp (BaseExpr.scala:376-394).  Off-grid timestamps (a segment whose
    frequency is not the step) give one row per distinct timestamp, as the worker's SQL does; the engine re-runs
    the scan at millisecond granularity (hash table).  On-grid segments alongside keep their rows."""
    from lakeside_amd import LK_MERGED, LK_PER_GLOB_ROWS, synth
    from oracle import dataexpr as dx
    keys, blobs, segs = _metrics_segments(engine, tmp_path, [(0, True), (1, False), (0, False)])
    for filt, agg, gbs, rollup in [(synth.leaf(synth.NAME, "eq", "metric_01"), "sum", [synth.SERVICE], None),
                                   (synth.leaf(synth.NAME, "in", "metric_02", "metric_03"), "max", [], "max")]:
        req = synth.pushdown(filt, segs, agg, gbs, dataset="metrics")
        if rollup:
            req["baseExpr"]["chart"]["rollup"] = rollup
        req = json.dumps(req)
        pr = dx.parse_pushdown(req)
        cells = dx.evaluate_glob_cells(pr, 2, keys, sources=blobs)
        got = engine.eval_pushdown(req, keys, 2, LK_PER_GLOB_ROWS).per_glob(len(cells))
        assert sum(len(cs) for cs in cells) > 10_000           # raw timestamps: many rows
        for gi, (g, cs) in enumerate(zip(got, cells)):
            assert_rows_equal(g, [(c.ts, c.agg_value(agg), c.tags) for c in cs], agg, f"metrics glob {gi}")
        merged = engine.eval_pushdown(req, keys, 2, LK_MERGED)
        assert_rows_equal(merged.rows(), dx.merge_glob_cells(pr, cells), agg, "metrics merged")
        ts = [r[0] for r in merged.rows()]
        assert ts == sorted(ts)


def test_lean_kernel_shapes(engine, tmp_path):
    """scan_lean (single string column, NULL-free tiles, chunk dictionaries of <= 64 codes): every code width 1..6,
    RLE runs (sorted names), SWAR (<= 4 passing codes of a power-of-two width) and per-code filters, multi-bucket
    tiles (1 s step), a window cutting tiles, every aggregate; GPU == oracle, and == the general kernel
    (LK_NO_LEAN_SPLIT) bit for bit."""
    import os
    import pyarrow as pa
    import pyarrow.parquet as pq
    from lakeside_amd import LK_MERGED, LK_PER_GLOB_ROWS, synth
    from oracle import dataexpr as dx
    rng = np.random.default_rng(5)
    keys, blobs, segs = [], [], []
    for i, (card, sort) in enumerate([(2, False), (5, False), (8, False), (16, False), (40, False), (64, False),
                                      (16, True)]):
        n = 120_000
        t0 = synth.T0 + (i % 4) * synth.HOUR
        codes = rng.integers(0, card, n)
        if sort:   # long RLE runs
            codes = np.sort(codes)
        t = pa.table({
            dx.TIMESTAMP: pa.array(np.sort(rng.integers(t0, t0 + synth.HOUR, n)), pa.int64()),
            dx.VALUE: pa.array(rng.lognormal(0.0, 2.0, n), pa.float64()),
            synth.NAME: pa.array([f"metric_{k:02d}" for k in codes], pa.string()),
        })
        path = str(tmp_path / f"lean{i}.parquet")
        pq.write_table(t, path, compression="NONE", use_dictionary=[synth.NAME],
                       column_encoding={c: "PLAIN" for c in t.column_names if c != synth.NAME},
                       row_group_size=60_000, data_page_size=1 << 20)
        engine.load_segment(path)
        keys.append(path)
        blobs.append(open(path, "rb").read())
        segs.append(synth.segment_request(i, hour=i % 4))
    filters = [synth.leaf(synth.NAME, "eq", "metric_01"),
               synth.leaf(synth.NAME, "in", "metric_00", "metric_03", "metric_04"),
               synth.leaf(synth.NAME, "in", *[f"metric_{k:02d}" for k in range(0, 40, 3)]),
               synth.leaf(synth.NAME, "!=", "metric_02"),
               synth.leaf(synth.NAME, "regex", "metric_1[0-5]")]
    cases = [(f, agg, gbs, step) for f in filters for agg, gbs, step in
             [("sum", [], 60_000), ("max", [synth.NAME], 1_000), ("count", [], 60_000), ("min", [], 60_000),
              ("avg", [synth.NAME], 60_000)]]
    for ci, (filt, agg, gbs, step) in enumerate(cases):
        segs_s = [dict(s, stepInMillis=step) for s in segs]
        if ci % 3 == 0:   # a window cutting tiles
            segs_s = [dict(s, startTs=s["startTs"] + 123_457, endTs=s["endTs"] - 777_001) for s in segs_s]
        req = json.dumps(synth.pushdown(filt, segs_s, agg, gbs))
        pr = dx.parse_pushdown(req)
        cells = dx.evaluate_glob_cells(pr, 3, keys, sources=blobs)
        got = engine.eval_pushdown(req, keys, 3, LK_PER_GLOB_ROWS)
        for gi, (g, cs) in enumerate(zip(got.per_glob(len(cells)), cells)):
            assert_rows_equal(g, [(c.ts, c.agg_value(agg), c.tags) for c in cs], agg, f"lean case {ci} glob {gi}")
        merged = engine.eval_pushdown(req, keys, 3, LK_MERGED)
        assert_rows_equal(merged.rows(), dx.merge_glob_cells(pr, cells), agg, f"lean case {ci} merged")
        os.environ["LK_NO_LEAN_SPLIT"] = "1"
        try:
            general = engine.eval_pushdown(req, keys, 3, LK_MERGED)
        finally:
            del os.environ["LK_NO_LEAN_SPLIT"]
        assert list(general.ts) == list(merged.ts) and general.tags == merged.tags
        if agg not in ("sum", "avg"):   # compensated sums: each path within 1 ulp of the exact sum (checked above)
            assert np.array_equal(general.values.view(np.uint64), merged.values.view(np.uint64))


def _pct_rows_equal(got_rows, want_rows, q, label):
    """Percentile rows: (ts, tags) in ascending time (ties compared as sorted tag lists), DDSketch bins identical,
    value == the oracle sketch's getValueAtQuantile(q) bit for bit."""
    from oracle import ddsketch
    key = lambda r: (r[0], sorted(r[1].items()))
    got_rows = sorted(got_rows, key=key)
    want_rows = sorted(want_rows, key=key)
    assert [key(r) for r in got_rows] == [key(r) for r in want_rows], label
    for (ts, tags, val, blob), (_, _, sk) in zip(got_rows, want_rows):
        gs = ddsketch.decode(blob)
        assert gs.bins() == sk.bins(), (label, ts, tags)
        assert val == sk.quantile(q), (label, ts, tags, val, sk.quantile(q))


def test_percentile_sketches(engine, tmp_path):
    """`p<NN>` aggregations (logs): per-glob DDSketches per (step, key tags) and query-api's merged quantiles equal
    the oracle's restatement of sketches-java (bins exact, quantile values bit for bit); NULL values count as 0.0;
    negative values and zeros; key tags = groupBys, or {"name": v} without groupBys."""
    import pyarrow as pa
    import pyarrow.parquet as pq
    from lakeside_amd import LK_MERGED, LK_PER_GLOB_ROWS, synth
    from oracle import dataexpr as dx
    rng = np.random.default_rng(9)
    keys, blobs, segs = [], [], []
    for i in range(5):
        n = 80_000
        t0 = synth.T0 + (i % 2) * synth.HOUR
        v = rng.lognormal(0.0, 2.0, n) * np.where(rng.random(n) < 0.2, -1.0, 1.0)
        v[rng.random(n) < 0.02] = 0.0
        t = pa.table({
            dx.TIMESTAMP: pa.array(np.sort(rng.integers(t0, t0 + synth.HOUR, n)), pa.int64()),
            dx.VALUE: pa.array(v, pa.float64(), mask=rng.random(n) < 0.05),
            synth.NAME: pa.array([f"metric_{k:02d}" for k in rng.integers(0, 4, n)], pa.string(),
                                 mask=rng.random(n) < 0.03),
            synth.SERVICE: pa.array([["svc-a", "svc-b", "null", ""][k] for k in rng.integers(0, 4, n)], pa.string(),
                                    mask=rng.random(n) < 0.05),
        })
        path = str(tmp_path / f"pct{i}.parquet")
        pq.write_table(t, path, compression="NONE", use_dictionary=[synth.NAME, synth.SERVICE],
                       column_encoding={dx.TIMESTAMP: "PLAIN", dx.VALUE: "PLAIN"}, row_group_size=40_000)
        engine.load_segment(path)
        keys.append(path)
        blobs.append(open(path, "rb").read())
        segs.append(synth.segment_request(i, hour=i % 2, step=300_000))
    for filt, agg, gbs in [(synth.leaf(synth.NAME, "in", "metric_01", "metric_02"), "p95", []),
                           (synth.leaf(synth.NAME, "!=", "metric_03"), "p50", [synth.SERVICE]),
                           ({"op": "or", "q1": synth.leaf(synth.NAME, "eq", "metric_00"),
                             "q2": synth.leaf(synth.SERVICE, "eq", "svc-a")}, "p99.9", [synth.SERVICE, synth.NAME])]:
        q = float(agg[1:]) / 100.0
        req_d = synth.pushdown(filt, segs, agg, gbs)
        req_d["baseExpr"]["chart"]["rollup"] = agg
        req = json.dumps(req_d)
        pr = dx.parse_pushdown(req)
        want = dx.evaluate_percentile_per_glob(pr, 2, keys, sources=blobs)
        res = engine.eval_pushdown(req, keys, 2, LK_PER_GLOB_ROWS)
        assert list(res.ts) == sorted(res.ts)
        for gi in range(len(want)):
            got = [(int(res.ts[r]), res.tags[r], float(res.values[r]), res.sketch(r))
                   for r in range(len(res)) if int(res.globs[r]) == gi]
            _pct_rows_equal(got, want[gi], q, f"{agg} glob {gi}")
        merged = engine.eval_pushdown(req, keys, 2, LK_MERGED)
        got = [(int(merged.ts[r]), merged.tags[r], float(merged.values[r]), merged.sketch(r)) for r in range(len(merged))]
        _pct_rows_equal(got, dx.merge_percentile(pr, want), q, f"{agg} merged")


def test_cardinality_estimates(engine):
    """`ces` (cardinality, HLL per step): per-glob and merged (union) estimates equal the oracle's HLL over the
    distinct group-key strings per step -- exact key counts below 384 coupons, the HLL estimate above (a 10K-value
    container key); NULL group values join as ""; no groupBys: every key is "" (ignored) -> 0."""
    from lakeside_amd import LK_MERGED, LK_PER_GLOB_ROWS, synth
    from oracle import dataexpr as dx, hll
    keys, blobs, segs = [], [], []
    for i in range(4):
        s = synth.make_segment(synth.segment_spec(i, rows=1 << 19, null_frac=0.05, highcard_n=10_000,
                                                  rg_rows=1 << 18, page_rows=1 << 15))
        key = f"ces/{i}"
        engine.put_segment_ptr(key, s.ptr, s.size)
        blobs.append(s.bytes())
        s.free()
        keys.append(key)
        segs.append(synth.segment_request(i, step=600_000))
    for filt, gbs, agg, rollup in [(synth.leaf(synth.NAME, "eq", "metric_03"), [synth.SERVICE, synth.NAMESPACE], "count", "ces"),
                                   (synth.leaf(synth.NAME, "in", "metric_01", "metric_02"), [synth.CONTAINER], "ces", None),
                                   (synth.leaf(synth.SERVICE, "regex", "svc-00[0-4]"), [], "ces", None)]:
        req_d = synth.pushdown(filt, segs, agg, gbs)
        if rollup:
            req_d["baseExpr"]["chart"]["rollup"] = rollup
        req = json.dumps(req_d)
        pr = dx.parse_pushdown(req)
        want = dx.evaluate_ces_per_glob(pr, 2, keys, sources=blobs)
        res = engine.eval_pushdown(req, keys, 2, LK_PER_GLOB_ROWS)
        got = [[(int(res.ts[r]), float(res.values[r])) for r in range(len(res)) if int(res.globs[r]) == gi]
               for gi in range(len(want))]
        assert got == [[(ts, hll.estimate(ks)) for ts, ks in w] for w in want], (gbs, agg)
        assert all(t == {} for t in res.tags)
        merged = engine.eval_pushdown(req, keys, 2, LK_MERGED)
        assert [(int(t), float(v)) for t, v in zip(merged.ts, merged.values)] == \
            [(ts, hll.estimate(ks)) for ts, ks in dx.merge_ces(want)], (gbs, agg)


def test_metrics_percentiles_and_cardinality(engine, tmp_path):
    """Metrics `p<NN>` (VERDICT r5 missing #1): per glob MAX(rollup_<r>) per (raw ts, groupBys, name) (BaseExpr.scala:
    379-383), each row's value (NULL -> 0.0) into the DDSketch of its (raw ts, key tags); metrics `ces`: every passing
    row (`1.0 as value`, no rollup column read, 385-388) into the HLL of its raw timestamp.  On-grid and off-grid
    segments (the 1 ms re-run), NULL rollup values and NULL group values; per glob and merged vs the oracle."""
    from lakeside_amd import LK_MERGED, LK_PER_GLOB_ROWS, synth
    from oracle import dataexpr as dx, hll
    keys, blobs, segs = _metrics_segments(engine, tmp_path, [(0, True), (1, True), (0, False)], n=60_000)
    for filt, agg, gbs, rollup in [(synth.leaf(synth.NAME, "in", "metric_01", "metric_02"), "p95", [], None),
                                   (synth.leaf(synth.NAME, "!=", "metric_03"), "p50", [synth.SERVICE], "max"),
                                   (synth.leaf(synth.SERVICE, "regex", "svc-00[0-3]"), "p99.9", [synth.SERVICE, synth.NAME], None)]:
        q = float(agg[1:]) / 100.0
        req_d = synth.pushdown(filt, segs, agg, gbs, dataset="metrics")
        if rollup:
            req_d["baseExpr"]["chart"]["rollup"] = rollup
        req = json.dumps(req_d)
        pr = dx.parse_pushdown(req)
        want = dx.evaluate_percentile_per_glob(pr, 2, keys, sources=blobs)
        assert sum(len(w) for w in want) > 1000
        res = engine.eval_pushdown(req, keys, 2, LK_PER_GLOB_ROWS)
        assert list(res.ts) == sorted(res.ts)
        per = [[] for _ in want]   # one pass over the rows, bucketed by glob
        for r, g in enumerate(np.asarray(res.globs).tolist()):
            per[g].append((int(res.ts[r]), res.tags[r], float(res.values[r]), res.sketch(r)))
        for gi in range(len(want)):
            _pct_rows_equal(per[gi], want[gi], q, f"metrics {agg} glob {gi}")
        merged = engine.eval_pushdown(req, keys, 2, LK_MERGED)
        got = [(int(merged.ts[r]), merged.tags[r], float(merged.values[r]), merged.sketch(r)) for r in range(len(merged))]
        _pct_rows_equal(got, dx.merge_percentile(pr, want), q, f"metrics {agg} merged")
    for filt, gbs in [(synth.leaf(synth.NAME, "eq", "metric_01"), [synth.SERVICE]),
                      (synth.leaf(synth.SERVICE, "exists"), [synth.NAME, synth.SERVICE]),
                      (synth.leaf(synth.NAME, "in", "metric_02", "metric_03"), [])]:
        req = json.dumps(synth.pushdown(filt, segs, "ces", gbs, dataset="metrics"))
        pr = dx.parse_pushdown(req)
        want = dx.evaluate_ces_per_glob(pr, 2, keys, sources=blobs)
        res = engine.eval_pushdown(req, keys, 2, LK_PER_GLOB_ROWS)
        got = [[(int(res.ts[r]), float(res.values[r])) for r in range(len(res)) if int(res.globs[r]) == gi]
               for gi in range(len(want))]
        assert got == [[(ts, hll.estimate(ks)) for ts, ks in w] for w in want], gbs
        assert sum(len(w) for w in want) > 100
        merged = engine.eval_pushdown(req, keys, 2, LK_MERGED)
        assert [(int(t), float(v)) for t, v in zip(merged.ts, merged.values)] == \
            [(ts, hll.estimate(ks)) for ts, ks in dx.merge_ces(want)], gbs


def test_query_shape_caps(engine, tmp_path):
    """VERDICT r5 missing #2: a DataExpr with 4 groupBys and 4 filter tags (8 string columns) and one with 18 filter
    leaves (the Kleene program, beyond the 6-leaf truth tables) run on the GPU path and equal the oracle, per glob
    and merged; 9 string columns or 33 leaves still fail with LK_ERR_UNSUPPORTED (the caller falls back)."""
    import pyarrow as pa
    import pyarrow.parquet as pq
    from lakeside_amd import LK_MERGED, LK_PER_GLOB_ROWS, synth
    from lakeside_amd._lib import LK_ERR_UNSUPPORTED, LakesideError
    from oracle import dataexpr as dx
    rng = np.random.default_rng(31)
    tags = [f"attr.t{k}" for k in range(1, 9)]
    keys, blobs, segs = [], [], []
    for i in range(4):
        n = 90_000
        t0 = synth.T0 + (i % 2) * synth.HOUR
        cols = {dx.TIMESTAMP: pa.array(np.sort(rng.integers(t0, t0 + synth.HOUR, n)), pa.int64()),
                dx.VALUE: pa.array(rng.lognormal(0.0, 2.0, n), pa.float64(), mask=rng.random(n) < 0.02),
                synth.NAME: pa.array([f"metric_{k:02d}" for k in rng.integers(0, 6, n)], pa.string())}
        for j, t in enumerate(tags):
            card = 3 + j
            cols[t] = pa.array([f"v{k}" for k in rng.integers(0, card, n)], pa.string(), mask=rng.random(n) < 0.04)
        tbl = pa.table(cols)
        path = str(tmp_path / f"caps{i}.parquet")
        pq.write_table(tbl, path, compression="NONE", use_dictionary=[synth.NAME] + tags,
                       column_encoding={dx.TIMESTAMP: "PLAIN", dx.VALUE: "PLAIN"}, row_group_size=45_000)
        engine.load_segment(path)
        keys.append(path)
        blobs.append(open(path, "rb").read())
        segs.append(synth.segment_request(i, hour=i % 2, step=600_000))
    lf = synth.leaf
    wide = {"op": "and", "q1": {"op": "and", "q1": lf(synth.NAME, "in", "metric_01", "metric_02", "metric_03"),
                                "q2": lf(tags[0], "regex", "v[0-1]")},
            "q2": {"op": "and", "q1": lf(tags[1], "!=", "v2"), "q2": lf(tags[2], "in", "v0", "v1", "v3")}}
    many = {"op": "or", "q1": lf(synth.NAME, "eq", "metric_00"), "q2": lf(synth.NAME, "eq", "metric_04")}
    for k in range(16):   # 18 leaves over 5 columns
        many = {"op": "or" if k % 3 else "and", "q1": many,
                "q2": lf(tags[k % 4], "eq" if k % 2 else "!=", f"v{k % 3}")}
    for filt, agg, gbs in [(wide, "sum", tags[4:8]), (many, "max", [tags[0], tags[5]]), (wide, "count", tags[3:7])]:
        req = json.dumps(synth.pushdown(filt, segs, agg, gbs))
        pr = dx.parse_pushdown(req)
        cells = dx.evaluate_glob_cells(pr, 2, keys, sources=blobs)
        assert sum(len(c) for c in cells) > 50
        got = engine.eval_pushdown(req, keys, 2, LK_PER_GLOB_ROWS)
        for gi, (g, cs) in enumerate(zip(got.per_glob(len(cells)), cells)):
            assert_rows_equal(g, [(c.ts, c.agg_value(agg), c.tags) for c in cs], agg, f"caps {agg} glob {gi}")
        merged = engine.eval_pushdown(req, keys, 2, LK_MERGED)
        assert_rows_equal(merged.rows(), dx.merge_glob_cells(pr, cells), agg, f"caps {agg} merged")
    over_str = {"op": "and", "q1": wide, "q2": lf(tags[3], "eq", "v1")}   # name + t1..t8 = 9 string columns
    over_leaf = many
    for k in range(15):
        over_leaf = {"op": "or", "q1": over_leaf, "q2": lf(tags[k % 4], "eq", f"v{k}")}   # 33 leaves
    for filt, gbs in [(over_str, tags[4:8]), (over_leaf, [])]:
        with pytest.raises(LakesideError) as ei:
            engine.eval_pushdown(json.dumps(synth.pushdown(filt, segs, "sum", gbs)), keys, 2, LK_MERGED)
        assert ei.value.code == LK_ERR_UNSUPPORTED, ei.value


def test_value_encodings(engine, tmp_path):
    """VERDICT r5 missing #4: DELTA_BINARY_PACKED (timestamps, INT32), BYTE_STREAM_SPLIT (values, timestamps),
    DELTA_LENGTH_BYTE_ARRAY / DELTA_BYTE_ARRAY (tags) and RLE-boolean pages, data page v1 and v2, materialized at load:
    the aggregate and a numeric leaf on the DELTA-encoded INT32 column equal the oracle (pyarrow's decoders)."""
    import sys
    import pyarrow.parquet as pq
    from lakeside_amd import LK_MERGED, LK_PER_GLOB_ROWS, synth
    from oracle import dataexpr as dx
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
    from make_load_fixtures import table
    encs = [{"_cardinalhq.timestamp": "DELTA_BINARY_PACKED", "attr.count": "DELTA_BINARY_PACKED",
             "_cardinalhq.value": "BYTE_STREAM_SPLIT", "_cardinalhq.name": "DELTA_LENGTH_BYTE_ARRAY",
             "resource.service.name": "DELTA_BYTE_ARRAY", "attr.flag": "PLAIN"},
            {"_cardinalhq.timestamp": "BYTE_STREAM_SPLIT", "attr.count": "BYTE_STREAM_SPLIT",
             "_cardinalhq.value": "BYTE_STREAM_SPLIT", "_cardinalhq.name": "DELTA_BYTE_ARRAY",
             "resource.service.name": "DELTA_LENGTH_BYTE_ARRAY", "attr.flag": "RLE"}]
    keys, blobs, segs = [], [], []
    for i in range(4):
        path = str(tmp_path / f"enc{i}.parquet")
        pq.write_table(table(60_000, 100 + i), path, compression="NONE" if i < 2 else "zstd", use_dictionary=False,
                       data_page_version="1.0" if i % 2 == 0 else "2.0", row_group_size=25_000,
                       data_page_size=1 << 16, column_encoding=encs[i % 2])
        engine.load_segment(path)
        keys.append(path)
        blobs.append(open(path, "rb").read())
        segs.append(synth.segment_request(i, hour=0, step=300_000))
    num = {"k": "attr.count", "v": ["20"], "op": "gt", "dataType": "number"}
    for filt, agg, gbs in [(synth.leaf(synth.NAME, "in", "metric_01", "metric_02", "metric_09"), "sum", [synth.SERVICE]),
                           ({"op": "and", "q1": synth.leaf(synth.SERVICE, "regex", "svc-0[0-4]"), "q2": num}, "max",
                            [synth.NAME]),
                           (synth.leaf(synth.SERVICE, "exists"), "count", [])]:
        req = json.dumps(synth.pushdown(filt, segs, agg, gbs))
        pr = dx.parse_pushdown(req)
        cells = dx.evaluate_glob_cells(pr, 2, keys, sources=blobs)
        assert sum(len(c) for c in cells) > 10
        got = engine.eval_pushdown(req, keys, 2, LK_PER_GLOB_ROWS)
        for gi, (g, cs) in enumerate(zip(got.per_glob(len(cells)), cells)):
            assert_rows_equal(g, [(c.ts, c.agg_value(agg), c.tags) for c in cs], agg, f"encodings {agg} glob {gi}")
        merged = engine.eval_pushdown(req, keys, 2, LK_MERGED)
        assert_rows_equal(merged.rows(), dx.merge_glob_cells(pr, cells), agg, f"encodings {agg} merged")


def test_hbm_budget_lru_eviction():
    """HBM segment cache with a weight bound (lk_engine_create hbm_budget_bytes; the worker's weighted Caffeine
    cache, WorkerApi.scala:53-64): inserts past the budget evict the least recently used segments; a segment used
    by a query is recent; an evicted key is re-loaded on demand (here: put again) and answers identically."""
    from lakeside_amd import LK_MERGED, synth
    from lakeside_amd._lib import LK_ERR_EVICTED, LakesideError
    from lakeside_amd.evaluator import Engine
    blobs = []
    for i in range(4):
        s = synth.make_segment(synth.segment_spec(i, rows=1 << 18, rg_rows=1 << 17, page_rows=1 << 15))
        blobs.append(s.bytes())
        s.free()
    probe = Engine(0)
    probe.put_segment("p", blobs[0])
    one = probe.segment_bytes
    probe.close()
    e = Engine(0, hbm_budget_bytes=int(2.5 * one))
    try:
        req = json.dumps(synth.pushdown(synth.leaf(synth.NAME, "eq", "metric_07"), [synth.segment_request(0)]))
        e.put_segment("s0", blobs[0])
        e.put_segment("s1", blobs[1])
        want = e.eval_pushdown(req, ["s0"], 10, LK_MERGED).rows()   # s0 becomes the most recent
        e.put_segment("s2", blobs[2])                              # over budget: s1 (LRU) goes
        assert e.segment_count == 2 and e.segment_bytes <= int(2.5 * one)
        assert e.eval_pushdown(req, ["s0"], 10, LK_MERGED).rows() == want
        # evicted put key: the call fails with LK_ERR_EVICTED so the caller re-puts it -- it is not a
        # missing file, whose glob alone would be empty
        with pytest.raises(LakesideError) as ei:
            e.eval_pushdown(req, ["s1"], 10, LK_MERGED)
        assert ei.value.code == LK_ERR_EVICTED, ei.value
        e.put_segment("s1", blobs[1])                              # re-put: answers again (s2 goes, LRU)
        req1 = json.dumps(synth.pushdown(synth.leaf(synth.NAME, "eq", "metric_07"), [synth.segment_request(1)]))
        assert len(e.eval_pushdown(req1, ["s1"], 10, LK_MERGED)) == 60
        e.put_segment("s3", blobs[3])                              # s0 is now the LRU
        assert e.segment_count == 2
        e.put_segment("s0", blobs[0])
        assert e.eval_pushdown(req, ["s0"], 10, LK_MERGED).rows() == want
        # a put key that is also a readable file path is reloaded from the file once evicted (a cache miss
        # like any other), not LK_ERR_EVICTED
        import tempfile
        with tempfile.TemporaryDirectory() as td:
            path = os.path.join(td, "seg0.parquet")
            with open(path, "wb") as f:
                f.write(blobs[0])
            e.put_segment(path, blobs[0])
            e.put_segment("s2", blobs[2])
            e.put_segment("s3", blobs[3])                          # the path key is evicted (LRU)
            assert e.segment_count == 2
            assert e.eval_pushdown(req, [path], 10, LK_MERGED).rows() == want
    finally:
        e.close()


def test_load_threads_identical_segments(tmp_path):
    """The parallel ingest (lk_engine_create load_threads) builds the same segment as a single-threaded load: a
    multi-row-group, compressed, multi-page file answers identically (rows, values, tags) with 1 and 8 threads."""
    import pyarrow.parquet as pq
    from lakeside_amd import LK_MERGED, synth
    from lakeside_amd.evaluator import Engine
    s = synth.make_segment(synth.segment_spec(0, rows=1 << 18, rg_rows=1 << 15, page_rows=1 << 12))
    raw = tmp_path / "raw.parquet"
    raw.write_bytes(s.bytes())
    s.free()
    t = pq.read_table(str(raw))
    path = str(tmp_path / "zstd.parquet")
    strings = [c for c in t.column_names if str(t.schema.field(c).type) == "string"]
    pq.write_table(t, path, compression="zstd", use_dictionary=strings, row_group_size=1 << 15, data_page_size=8192)
    req = json.dumps(synth.pushdown(synth.leaf(synth.NAME, "in", "metric_03", "metric_07"), [synth.segment_request(0)],
                                    group_bys=[synth.SERVICE]))
    out = []
    for threads in (1, 8):
        e = Engine(0, load_threads=threads)
        try:
            e.load_segment(path)
            r = e.eval_pushdown(req, [path], 10, LK_MERGED)
            out.append((r.rows(), r.stats.get("tiles")))
        finally:
            e.close()
    assert len(out[0][0]) > 0 and out[0][1] == out[1][1]
    assert_rows_equal(out[1][0], out[0][0], "sum", "load_threads 8 vs 1")


def test_lean_kernel_late_columns(engine):
    """scan_lean with late string columns (name early; the others decoded per listed row): a group dim only
    (every listed row passes, loads issued together), a late regex filter + 2 group dims, a high-cardinality late
    column (lookup values outside LDS), a late column absent from one segment; GPU == oracle, and == scan_tiles
    (LK_NO_LEAN_SPLIT)."""
    import os
    from lakeside_amd import LK_MERGED, LK_PER_GLOB_ROWS, synth
    from oracle import dataexpr as dx
    keys, blobs, segs = [], [], []
    for i in range(5):
        s = synth.make_segment(synth.segment_spec(i, rows=1 << 19, null_frac=0.0, highcard_n=5000 if i != 2 else 0,
                                                  rg_rows=1 << 18, page_rows=1 << 15, value_mode=1))
        key = f"late/{i}"
        engine.put_segment_ptr(key, s.ptr, s.size)
        blobs.append(s.bytes())
        s.free()
        keys.append(key)
        segs.append(synth.segment_request(i))
    re_f = {"op": "and", "q1": synth.leaf(synth.NAME, "eq", "metric_07"),
            "q2": synth.leaf(synth.SERVICE, "regex", "^svc-0[0-4]")}
    for filt, agg, gbs in [(synth.leaf(synth.NAME, "eq", "metric_07"), "sum", [synth.SERVICE]),
                           (re_f, "max", [synth.SERVICE, synth.NAMESPACE]),
                           (synth.leaf(synth.NAME, "in", "metric_01", "metric_09"), "count", [synth.CONTAINER]),
                           ({"op": "and", "q1": synth.leaf(synth.NAME, "eq", "metric_03"),
                             "q2": synth.leaf(synth.CONTAINER, "in", "c0000001", "c0000007", "c0004999")},
                            "min", [synth.NAMESPACE])]:
        req = json.dumps(synth.pushdown(filt, segs, agg, gbs))
        pr = dx.parse_pushdown(req)
        cells = dx.evaluate_glob_cells(pr, 2, keys, sources=blobs)
        got = engine.eval_pushdown(req, keys, 2, LK_PER_GLOB_ROWS)
        for gi, (g, cs) in enumerate(zip(got.per_glob(len(cells)), cells)):
            assert_rows_equal(g, [(c.ts, c.agg_value(agg), c.tags) for c in cs], agg, f"late {gbs} glob {gi}")
        merged = engine.eval_pushdown(req, keys, 2, LK_MERGED)
        assert_rows_equal(merged.rows(), dx.merge_glob_cells(pr, cells), agg, f"late {gbs} merged")
        os.environ["LK_NO_LEAN_SPLIT"] = "1"
        try:
            general = engine.eval_pushdown(req, keys, 2, LK_MERGED)
        finally:
            del os.environ["LK_NO_LEAN_SPLIT"]
        assert list(general.ts) == list(merged.ts) and general.tags == merged.tags
        if agg not in ("sum", "avg"):
            assert np.array_equal(general.values.view(np.uint64), merged.values.view(np.uint64))


def test_sums_subnormal_and_cancelling(engine, tmp_path):
    """The compensated device sums (returning-atomic TwoSum, built with -munsafe-fp-atomics) on subnormal values,
    near-cancelling magnitudes and values past 2^53: GPU sums stay within 1 ulp of the correctly rounded sum
    (math.fsum), per glob and merged."""
    import pyarrow as pa
    import pyarrow.parquet as pq
    from lakeside_amd import LK_MERGED, LK_PER_GLOB_ROWS, synth
    from oracle import dataexpr as dx
    rng = np.random.default_rng(5)
    paths, blobs = [], []
    for i in range(3):
        n = 120_000
        kind = rng.integers(0, 4, n)
        v = np.where(kind == 0, rng.uniform(-1, 1, n) * 4.9e-322,                  # subnormals
            np.where(kind == 1, rng.choice([1e300, -1e300], n) * (1 + rng.uniform(0, 1e-15, n)),   # cancelling
            np.where(kind == 2, 2.0 ** 53 + rng.integers(0, 8, n), rng.lognormal(0, 5, n))))       # > 2^53, wide
        t = pa.table({dx.TIMESTAMP: pa.array(np.sort(synth.T0 + rng.integers(0, synth.HOUR, n)), pa.int64()),
                      dx.VALUE: pa.array(v, pa.float64()),
                      dx.NAME: pa.array([f"metric_{k:02d}" for k in kind], pa.string())})   # one kind per name
        path = str(tmp_path / f"sums{i}.parquet")
        pq.write_table(t, path, compression="NONE", use_dictionary=[dx.NAME],
                       column_encoding={dx.TIMESTAMP: "PLAIN", dx.VALUE: "PLAIN"})
        engine.load_segment(path)
        paths.append(path)
        blobs.append(open(path, "rb").read())
    segs = [synth.segment_request(i, step=600_000, hour=0) for i in range(3)]
    for agg, gbs in (("sum", [synth.NAME]), ("avg", [synth.NAME])):
        req = json.dumps(synth.pushdown(synth.leaf(synth.NAME, "!=", "metric_99"), segs, agg, gbs))
        pr = dx.parse_pushdown(req)
        cells = dx.evaluate_glob_cells(pr, 2, paths, sources=blobs)
        got = engine.eval_pushdown(req, paths, 2, LK_PER_GLOB_ROWS).per_glob(len(cells))
        for gi, (g, cs) in enumerate(zip(got, cells)):
            assert_rows_equal(g, [(c.ts, c.agg_value(agg), c.tags) for c in cs], agg, f"{agg} glob {gi}")
        merged = engine.eval_pushdown(req, paths, 2, LK_MERGED).rows()
        assert_rows_equal(merged, dx.merge_glob_cells(pr, cells), agg, f"{agg} merged")


def test_lean_direct_table_planes(engine):
    """scan_lean's per-tile direct table in every layout: segments with NULL values next to NULL-free ones (the table
    keeps a rows plane: no lean bits), NULL-free sets (SUM's -0.0 marker, MIN/MAX existence by the extreme), replicas
    per cell, per-glob rows and merged rows, the dense path (every name passes), and LK_NO_DIRECT (the LDS hash) giving
    the same rows."""
    import os
    from lakeside_amd import LK_MERGED, LK_PER_GLOB_ROWS, synth
    from oracle import dataexpr as dx
    sets = {}
    for label, nulls in (("clean", [0.0, 0.0, 0.0]), ("mixed", [0.0, 0.05, 0.0])):
        keys, blobs, segs = [], [], []
        for i, nf in enumerate(nulls):
            s = synth.make_segment(synth.segment_spec(40 + i, rows=1 << 19, null_frac=nf, rg_rows=1 << 18,
                                                      page_rows=1 << 15, value_mode=1, hour=0))
            key = f"dt/{label}/{i}"
            engine.put_segment_ptr(key, s.ptr, s.size)
            blobs.append(s.bytes())
            s.free()
            keys.append(key)
            segs.append(synth.segment_request(40 + i, hour=0))
        sets[label] = (keys, blobs, segs)
    for label, (keys, blobs, segs) in sets.items():
        for filt, agg, gbs in [(synth.leaf(synth.NAME, "eq", "metric_07"), "sum", []),
                               (synth.leaf(synth.NAME, "in", *[f"metric_{k:02d}" for k in range(16)]), "sum", []),
                               (synth.leaf(synth.NAME, "in", *[f"metric_{k:02d}" for k in range(16)]), "max", []),
                               (synth.leaf(synth.NAME, "in", "metric_01", "metric_05"), "min", [synth.SERVICE]),
                               (synth.leaf(synth.NAME, "eq", "metric_03"), "avg", [synth.SERVICE]),
                               (synth.leaf(synth.NAME, "in", "metric_02", "metric_09"), "count", [])]:
            req = json.dumps(synth.pushdown(filt, segs, agg, gbs))
            pr = dx.parse_pushdown(req)
            cells = dx.evaluate_glob_cells(pr, 2, keys, sources=blobs)
            got = engine.eval_pushdown(req, keys, 2, LK_PER_GLOB_ROWS)
            for gi, (g, cs) in enumerate(zip(got.per_glob(len(cells)), cells)):
                assert_rows_equal(g, [(c.ts, c.agg_value(agg), c.tags) for c in cs], agg, f"{label} {agg} {gbs} glob {gi}")
            merged = engine.eval_pushdown(req, keys, 2, LK_MERGED)
            assert_rows_equal(merged.rows(), dx.merge_glob_cells(pr, cells), agg, f"{label} {agg} {gbs} merged")
            os.environ["LK_NO_DIRECT"] = "1"
            try:
                hashed = engine.eval_pushdown(req, keys, 2, LK_MERGED)
            finally:
                del os.environ["LK_NO_DIRECT"]
            assert list(hashed.ts) == list(merged.ts) and hashed.tags == merged.tags
            if agg not in ("sum", "avg"):
                assert np.array_equal(hashed.values.view(np.uint64), merged.values.view(np.uint64))


def test_result_outlives_engine():
    """a result's tags (bulk export of an engine-dictionary column) are readable after its engine was
    destroyed -- the result keeps the dictionary block and builds its own pointer table."""
    from lakeside_amd import LK_MERGED, synth
    from lakeside_amd.evaluator import Engine
    e = Engine(0)
    s = synth.make_segment(synth.segment_spec(3, rows=1 << 16, rg_rows=1 << 15, page_rows=1 << 13))
    e.put_segment_ptr("outlive/0", s.ptr, s.size)
    s.free()
    req = json.dumps(synth.pushdown(synth.leaf(synth.NAME, "in", "metric_01", "metric_02"), [synth.segment_request(3)],
                                    "sum", [synth.SERVICE]))
    res = e.eval_pushdown(req, ["outlive/0"], 10, LK_MERGED)
    n = len(res)
    e.close()
    tags = res.tags
    assert n > 0 and len(tags) == n
    assert sum(1 for t in tags if t.get(synth.SERVICE, "").startswith("svc-")) > n // 2
