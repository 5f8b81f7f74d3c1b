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
