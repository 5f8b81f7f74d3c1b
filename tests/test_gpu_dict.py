"""Engine dictionary lifecycle on the MI355X: ids no cached segment references are reclaimed, so the
group-dim space of an unrestricted :by follows the segments in the HBM cache -- as the worker's bounded disk cache does
(WorkerApi.scala:53-64) -- instead of everything a long-lived worker ever loaded.  Results built before a compaction
keep reading their own tag strings."""
import json

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SVC = "resource.service.name"


def _files(tmp_path, prefix, nfiles, rows=30_000, seed=0):
    import pyarrow as pa
    import pyarrow.parquet as pq
    from lakeside_amd import synth
    from oracle import dataexpr as dx
    rng = np.random.default_rng(seed)
    paths, blobs = [], []
    for i in range(nfiles):
        t = pa.table({dx.TIMESTAMP: pa.array(np.sort(synth.T0 + rng.integers(0, synth.HOUR, rows)), pa.int64()),
                      dx.VALUE: pa.array(rng.integers(0, 1000, rows).astype(np.float64)),
                      dx.NAME: pa.array([f"metric_{k:02d}" for k in rng.integers(0, 4, rows)], pa.string()),
                      SVC: pa.array([f"{prefix}-{k:03d}" for k in rng.integers(0, 150, rows)], pa.string())})
        path = str(tmp_path / f"{prefix}{i}.parquet")
        pq.write_table(t, path, compression="NONE", use_dictionary=[dx.NAME, SVC], row_group_size=rows // 2)
        paths.append(path)
        blobs.append(open(path, "rb").read())
    return paths, blobs


def _query(eng, paths, blobs, label):
    from lakeside_amd import LK_MERGED, synth
    from oracle import dataexpr as dx
    from tests.parity import assert_rows_equal
    req = json.dumps(synth.pushdown(synth.leaf(synth.NAME, "eq", "metric_02"),
                                    [synth.segment_request(i, hour=0) for i in range(len(paths))], "sum", [SVC]))
    got = eng.eval_pushdown(req, paths, 10, LK_MERGED)
    want = dx.evaluate_merged(dx.parse_pushdown(req), paths, 10, sources=blobs)
    assert_rows_equal(got.rows(), want, "sum", label)
    return got


def test_dictionary_compaction_tracks_cached_segments(tmp_path):
    from lakeside_amd.evaluator import Engine
    pa_, ba = _files(tmp_path, "alpha", 3, seed=1)
    pb, bb = _files(tmp_path, "beta", 3, seed=2)
    eng = Engine(0, dict_compact_min_dead=1)
    try:
        for p in pa_:
            eng.load_segment(p)
        ra = _query(eng, pa_, ba, "alpha")
        cells_a = ra.stats["cells"]
        tags_a = list(ra.tags)
        assert eng.stats["dictionaries"][SVC]["size"] == 150
        for p in pa_:
            eng.evict(p)
        st = eng.stats["dictionaries"][SVC]
        assert st["live"] == 0 and st["size"] == 150          # dead ids wait for the next load / evaluation
        for p in pb:
            eng.load_segment(p)                               # compacts first: alpha's ids are gone
        st = eng.stats
        assert st["dict_compactions"] >= 1
        assert st["dictionaries"][SVC]["size"] == 150 and st["dictionaries"][SVC]["live"] == 150
        rb = _query(eng, pb, bb, "beta after compaction")
        assert rb.stats["cells"] == cells_a                   # the cell space did not grow with the evicted values
        assert list(ra.tags) == tags_a                        # the earlier result still reads its own strings
        assert all(t[SVC].startswith("alpha-") for t in tags_a)
        # the same value sets again, both cached: the dictionary holds their union and queries stay exact
        for p in pa_:
            eng.load_segment(p)
        assert eng.stats["dictionaries"][SVC]["size"] == 300
        _query(eng, pa_, ba, "alpha reloaded")
        _query(eng, pb, bb, "beta with alpha cached")
    finally:
        eng.close()


def test_dictionary_compaction_rewrites_remaps_of_cached_segments(tmp_path):
    """Only some segments are evicted: the survivors' chunk remaps are rewritten to the new ids on the GPU, and
    their rows (tags included) are unchanged."""
    from lakeside_amd.evaluator import Engine
    pa_, ba = _files(tmp_path, "gamma", 2, seed=3)
    pb, bb = _files(tmp_path, "delta", 2, seed=4)
    eng = Engine(0, dict_compact_min_dead=1)
    try:
        for p in pa_ + pb:
            eng.load_segment(p)
        before = _query(eng, pb, bb, "delta before").rows()
        for p in pa_:                                         # gamma's values (interned first) die
            eng.evict(p)
        after = _query(eng, pb, bb, "delta after compaction")  # evaluation entry compacts
        assert eng.stats["dict_compactions"] >= 1
        assert eng.stats["dictionaries"][SVC]["size"] == 150
        assert sorted(after.rows(), key=repr) == sorted(before, key=repr)
    finally:
        eng.close()
