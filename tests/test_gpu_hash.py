"""High-cardinality path on the GPU: hash-mode aggregation table (SURVEY §2.2 K4 "spill path"), sparse finalize,
per-glob time order, C5 at the real 10M-value dictionary, concurrent calls.

Hash mode is chosen when the dense cell space (glob slots x buckets x groups) exceeds LK_DENSE_MAX_CELLS (default
2^26): the golden cases are re-run with LK_DENSE_MAX_CELLS=0 so every shape (per-glob rows, merged rows, the
name-collapse of queries without groupBys, merged min/max over NULL-able values, avg, tag queries) also goes
through the hash table + radix-sorted finalize, and must give the committed golden rows.
"""
import json
import os
import threading
import time

import numpy as np
import pytest

from tests.parity import assert_rows_equal, from_jsonable

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = os.path.join(HERE, "golden")

pytestmark = pytest.mark.gpu


def _cases():
    with open(os.path.join(GOLDEN, "cases.json")) as f:
        return json.load(f)


def _tag_cases():
    with open(os.path.join(GOLDEN, "tag_cases.json")) as f:
        return json.load(f)


class _Env:
    def __init__(self, **kv):
        self.kv = kv

    def __enter__(self):
        self.old = {k: os.environ.get(k) for k in self.kv}
        os.environ.update({k: str(v) for k, v in self.kv.items()})

    def __exit__(self, *a):
        for k, v in self.old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


@pytest.fixture(scope="module")
def golden_engine(engine):
    for c in _cases() + _tag_cases():
        for p in c["segments"]:
            engine.load_segment(os.path.join(GOLDEN, p))
    return engine


@pytest.mark.parametrize("init_slots", [None, 64])
def test_golden_cases_through_hash_mode(golden_engine, init_slots):
    """Every golden case through the hash table (and, with 64 initial slots, through table regrowth)."""
    from lakeside_amd import LK_MERGED, LK_PER_GLOB_ROWS
    env = {"LK_DENSE_MAX_CELLS": 0}
    if init_slots:
        env["LK_HASH_INIT_SLOTS"] = init_slots
    with _Env(**env):
        for case in _cases():
            paths = [os.path.join(GOLDEN, p) for p in case["segments"]]
            req = json.dumps(case["request"])
            agg = case["request"]["baseExpr"]["chart"]["aggregation"]
            res = golden_engine.eval_pushdown(req, paths, case["glob_size"], LK_PER_GLOB_ROWS)
            if len(res):
                assert res.stats["table"] == "hash", res.stats
            got = res.per_glob(len(case["expected_per_glob"]))
            for gi, (g, w) in enumerate(zip(got, case["expected_per_glob"])):
                assert_rows_equal(g, from_jsonable(w), agg, f"hash {case['name']} glob {gi}")
            if case["expected_merged"] is not None:
                res = golden_engine.eval_pushdown(req, paths, case["glob_size"], LK_MERGED)
                assert_rows_equal(res.rows(), from_jsonable(case["expected_merged"]), agg, f"hash {case['name']} merged")
                if init_slots and len(res) > 64:
                    assert res.stats["attempts"] > 1, res.stats
        key = lambda t: sorted(t.items())   # noqa: E731
        for case in _tag_cases():
            paths = [os.path.join(GOLDEN, p) for p in case["segments"]]
            res = golden_engine.eval_pushdown(json.dumps(case["request"]), paths, case["glob_size"], LK_MERGED)
            assert sorted(res.tags, key=key) == sorted(case["expected_merged"], key=key), case["name"]


def test_per_glob_rows_ascending_without_sorting(golden_engine):
    """lakeside_gpu.h: lk_result_timestamps ascending (ties: glob, then group) for LK_PER_GLOB_ROWS too: the
    worker merge-sorts its globs by timestamp (Commons.scala:391-392).  Checked on the raw row order, dense and
    hash mode."""
    from lakeside_amd import LK_MERGED, LK_PER_GLOB_ROWS
    for dense_max in (None, 0):
        with _Env(**({"LK_DENSE_MAX_CELLS": dense_max} if dense_max is not None else {})):
            multi = 0
            for case in _cases():
                paths = [os.path.join(GOLDEN, p) for p in case["segments"]]
                req = json.dumps(case["request"])
                for flags in (LK_PER_GLOB_ROWS, LK_MERGED):
                    res = golden_engine.eval_pushdown(req, paths, case["glob_size"], flags)
                    ts, gl = np.asarray(res.ts), np.asarray(res.globs)
                    assert np.all(np.diff(ts) >= 0), f"{case['name']} flags {flags}: timestamps not ascending"
                    same = np.diff(ts) == 0
                    assert np.all(np.diff(gl.astype(np.int64))[same] >= 0), f"{case['name']}: glob order within a ts"
                    if flags == LK_PER_GLOB_ROWS and len(set(gl.tolist())) > 1:
                        multi += 1
            assert multi > 0   # some case really interleaves several globs


def _synth(engine, tag, nseg, rows, **spec):
    from lakeside_amd import synth
    keys, blobs = [], []
    for i in range(nseg):
        s = synth.make_segment(synth.segment_spec(i, rows=rows, **spec))
        key = f"{tag}/{i}"
        engine.put_segment_ptr(key, s.ptr, s.size)
        blobs.append(s.bytes())
        s.free()
        keys.append(key)
    return keys, blobs


def _check(engine, keys, blobs, filt, agg, gbs, step, hour, glob_size=10, flags=("per_glob", "merged")):
    from lakeside_amd import LK_MERGED, LK_PER_GLOB_ROWS, synth
    from oracle import dataexpr as dx
    segs = [synth.segment_request(i, step=step, hour=hour) for i in range(len(keys))]
    req = json.dumps(synth.pushdown(filt, segs, agg, gbs))
    pr = dx.parse_pushdown(req)
    cells = dx.evaluate_glob_cells(pr, glob_size, keys, sources=blobs)
    out = {}
    if "per_glob" in flags:
        res = engine.eval_pushdown(req, keys, glob_size, LK_PER_GLOB_ROWS)
        got = res.per_glob(len(cells))
        for gi, (g, cs) in enumerate(zip(got, cells)):
            assert_rows_equal(g, [(c.ts, c.agg_value(agg), c.tags) for c in cs], agg, f"glob {gi}")
        out["per_glob"] = res
    if "merged" in flags:
        res = engine.eval_pushdown(req, keys, glob_size, LK_MERGED)
        assert_rows_equal(res.rows(), dx.merge_glob_cells(pr, cells), agg, "merged")
        out["merged"] = res
    return out


def _check_columns(engine, keys, blobs, filt, agg, gbs, step, hour, glob_size=10, flags=("per_glob", "merged")):
    """_check for results of ~10^5-10^6 rows, compared column-wise against the C++ restatement (tests/parity.py)."""
    from lakeside_amd import synth
    from tests.parity import check_columns
    segs = [synth.segment_request(i, step=step, hour=hour) for i in range(len(keys))]
    return check_columns(engine, json.dumps(synth.pushdown(filt, segs, agg, gbs)), keys, blobs, glob_size, flags)


@pytest.mark.timeout(600)
def test_c5_real_10m_dictionary(engine):
    """C5 (BASELINE configs[4]) at its real dictionary: resource.container.id drawn from 10,000,000 values
    (c%07d), 2 segments x 2^22 rows in hour 0, :eq name :sum :by container.  At a 1h step (dense table, 20M
    cells) and at a 1m step (60 buckets x 20M groups = 1.2B cells: the hash table), against the C++ restatement
    column-wise (half a million rows per result: the Python oracle took ~60 s per check)."""
    from lakeside_amd import synth
    keys, blobs = _synth(engine, "c5real", 2, 1 << 22, hour=0, highcard_n=10_000_000)
    filt = synth.leaf(synth.NAME, "eq", "metric_07")
    r = _check_columns(engine, keys, blobs, filt, "sum", [synth.CONTAINER], 3_600_000, 0, flags=("merged",))
    assert r["merged"].stats["table"] == "dense" and len(r["merged"]) > 400_000
    r = _check_columns(engine, keys, blobs, filt, "sum", [synth.CONTAINER], 60_000, 0)
    assert r["merged"].stats["table"] == "hash", r["merged"].stats
    assert len(r["merged"]) > 400_000
    _check_columns(engine, keys, blobs, filt, "max", [synth.CONTAINER], 600_000, 0, glob_size=1, flags=("merged",))


def test_hash_mode_nulls_minmax_avg(engine):
    """Hash mode with NULL tags/values: merged min/max over NULL-able values (the rekey fold), avg, count."""
    from lakeside_amd import synth
    keys, blobs = _synth(engine, "hashnull", 3, 1 << 19, value_mode=1, null_frac=0.05, rg_rows=1 << 18,
                         page_rows=1 << 15)
    filt = {"op": "and", "q1": synth.leaf(synth.NAME, "in", "metric_01", "metric_02"),
            "q2": synth.leaf(synth.SERVICE, "regex", "^svc-0[0-4]")}
    with _Env(LK_DENSE_MAX_CELLS=0):
        for agg, gbs in [("max", [synth.SERVICE, synth.NAMESPACE]), ("min", [synth.NAMESPACE]), ("avg", []),
                         ("count", [synth.NAME]), ("sum", [])]:
            r = _check(engine, keys, blobs, filt, agg, gbs, 60_000, None, glob_size=2)
            assert r["merged"].stats["table"] == "hash"


@pytest.mark.timeout(300)
def test_concurrent_slow_and_fast_calls(golden_engine):
    """Calls run on their own streams (no per-engine lock): while one thread evaluates a slow high-cardinality
    query, other threads keep completing golden queries, and every result is right."""
    from lakeside_amd import LK_MERGED, synth
    keys, _ = _synth(golden_engine, "slow", 4, 1 << 22, hour=0, highcard_n=2_000_000)
    segs = [synth.segment_request(i, step=60_000, hour=0) for i in range(len(keys))]
    slow_req = json.dumps(synth.pushdown(synth.leaf(synth.NAME, "in", "metric_01", "metric_02", "metric_03"), segs,
                                         "sum", [synth.CONTAINER]))
    golden_engine.eval_pushdown(slow_req, keys, 10, LK_MERGED)   # warm
    cases = [c for c in _cases() if c["expected_merged"] is not None]
    errors, fast_done, slow_done = [], [], []

    def slow():
        try:
            for _ in range(3):
                golden_engine.eval_pushdown(slow_req, keys, 10, LK_MERGED)
            slow_done.append(time.perf_counter())
        except Exception as e:   # noqa: BLE001
            errors.append(e)

    def fast(k):
        try:
            for case in cases[k::3]:
                paths = [os.path.join(GOLDEN, p) for p in case["segments"]]
                res = golden_engine.eval_pushdown(json.dumps(case["request"]), paths, case["glob_size"], LK_MERGED)
                agg = case["request"]["baseExpr"]["chart"]["aggregation"]
                assert_rows_equal(res.rows(), from_jsonable(case["expected_merged"]), agg, case["name"])
                fast_done.append(time.perf_counter())
        except Exception as e:   # noqa: BLE001
            errors.append(e)

    ts = [threading.Thread(target=slow)] + [threading.Thread(target=fast, args=(k,)) for k in range(3)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=240)
    assert not any(t.is_alive() for t in ts)
    assert not errors, errors[0]
    assert len(fast_done) == len(cases)
