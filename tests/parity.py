"""Row comparison used by the parity tests (GPU rows vs oracle / golden rows).

Bar (BASELINE.json north_star): timestamps and tags exact; count/min/max bit-exact; sums (and avg) within
1 ulp of the correctly rounded value.
"""
import math

SUM_LIKE = ("sum", "avg")


def _key(r):
    v = r[1]
    return (r[0], sorted(r[2].items()), (1, 0.0) if v != v else (0, v))   # NaN last: a total order


def assert_rows_equal(got, want, agg, label=""):
    got = sorted(got, key=_key)
    want = sorted(want, key=_key)
    assert len(got) == len(want), f"{label}: {len(got)} rows vs expected {len(want)}"
    for i, (g, w) in enumerate(zip(got, want)):
        assert g[0] == w[0], f"{label}: row {i} ts {g[0]} vs {w[0]}"
        assert g[2] == w[2], f"{label}: row {i} tags {g[2]} vs {w[2]}"
        gv, wv = g[1], w[1]
        if agg in SUM_LIKE:
            ok = gv == wv or (math.isnan(gv) and math.isnan(wv)) or abs(gv - wv) <= math.ulp(wv)
        else:
            ok = (gv == wv and math.copysign(1, gv) == math.copysign(1, wv)) or (math.isnan(gv) and math.isnan(wv))
        assert ok, f"{label}: row {i} at ts={g[0]} tags={g[2]}: value {gv!r} vs expected {wv!r} (agg {agg})"


def from_jsonable(rows):
    return [(int(t), float.fromhex(v), dict(tags)) for t, v, tags in rows]


def result_columns(res):
    """A GPU Result as (ts, value, canonical tag key) arrays (oracle.cpu.tag_key), built column-wise from the bulk
    export (lk_result_group_ids + lk_result_tag_dictionary) -- the full-size bench validation compares millions of
    rows this way; rows whose group tags are all dropped take their per-row tags (the queryTags fallback)."""
    import ctypes

    import numpy as np

    from lakeside_amd import _lib
    from lakeside_amd.evaluator import _View
    from oracle.cpu import join_tag_columns, tag_key

    L = _lib.lib()
    h = res._owner.h
    n = len(res.ts)
    ng = L.lk_result_num_group_columns(h) if n else 0
    names, cols = [], []
    if ng:
        gid = np.asarray(_View(res._owner, L.lk_result_group_ids(h), n, "<u4")).astype(np.uint64)
        for c in range(ng):
            stride, nd = ctypes.c_uint64(), ctypes.c_uint64()
            p = L.lk_result_tag_dictionary(h, c, ctypes.byref(stride), ctypes.byref(nd))
            if not p or nd.value == 0:
                continue
            d = (gid // np.uint64(stride.value)) % np.uint64(nd.value)
            uniq, inv = np.unique(d, return_inverse=True)
            text = [ctypes.string_at(p[int(u)]) if p[int(u)] else b"" for u in uniq]
            names.append(res.tag_names[c])
            cols.append(np.array(text, dtype=object)[inv])
    fallback = np.full(n, b"", dtype=object)
    if len(res.tag_names) > ng:   # rows without own tags: their tag map from the library, row by row (few)
        own = join_tag_columns(names, cols, fallback) if names else fallback
        for r in np.nonzero(own == b"")[0].tolist():
            m = {}
            for c in range(ng, len(res.tag_names)):
                v = L.lk_result_tag_value(h, r, c)
                if v is not None:
                    m[res.tag_names[c]] = v.decode()
            fallback[r] = tag_key(m)
    key = join_tag_columns(names, cols, fallback) if names else fallback
    return np.array(res.ts, dtype=np.int64), np.array(res.values, dtype=np.float64), key


def check_columns(engine, req, keys, blobs, glob_size, flags=("per_glob", "merged")):
    """GPU rows of a request (per glob and / or merged) vs the C++ restatement (oracle/cpu, the bench's full-size
    validator; itself checked against oracle/dataexpr and the golden rows in tests/test_oracle_cpu.py), compared
    column-wise with numpy: the bar of assert_rows_equal without a Python object per row, for results of 10^5-10^6
    rows.  Returns {"per_glob": Result, "merged": Result} for the flags run."""
    import os

    import numpy as np

    from lakeside_amd import LK_MERGED, LK_PER_GLOB_ROWS
    from oracle import cpu as lkcpu
    from oracle import dataexpr as dx
    pr = dx.parse_pushdown(req)
    agg = pr.baseExpr.chart.aggregation
    table = lkcpu.evaluate_cell_table(pr, glob_size, blobs, min(16, os.cpu_count() or 1))
    out = {}
    if "per_glob" in flags:
        res = engine.eval_pushdown(req, keys, glob_size, LK_PER_GLOB_ROWS)
        ts, val, key = result_columns(res)
        globs = np.asarray(res.globs)
        assert len(ts) == len(table), f"per-glob rows {len(ts)} vs expected {len(table)}"
        for g in range(int(table.glob.max()) + 1 if len(table) else 0):
            sel = table.glob == g
            cnt = table.count[sel]
            if agg == dx.COUNT:
                want = cnt.astype(np.float64)
            elif agg in (dx.SUM, dx.AVG):   # CpuCell.agg_value: hi + lo is the double-double's rounded sum
                s = table.hi[sel] + table.lo[sel]
                want = np.where(cnt > 0, s if agg == dx.SUM else s / np.maximum(cnt, 1), 0.0)
            else:
                want = np.where(cnt > 0, (table.vmin if agg == dx.MIN else table.vmax)[sel], 0.0)
            m = globs == g
            lkcpu.assert_columns_equal((ts[m], val[m], key[m]), (table.ts[sel], want, table.key[sel]), agg,
                                       f"glob {g}")
        out["per_glob"] = res
    if "merged" in flags:
        res = engine.eval_pushdown(req, keys, glob_size, LK_MERGED)
        lkcpu.assert_columns_equal(result_columns(res), lkcpu.merge_cell_table(table, agg, bool(pr.baseExpr.chart.groupBys)),
                                   agg, "merged")
        out["merged"] = res
    return out
