"""CPU: the DDSketch restatement (oracle/ddsketch.py) keeps its relative-accuracy guarantee, merges exactly and
its wire decoder reads what it is given (SURVEY.md §8(f) f4 percentiles)."""
import numpy as np

from oracle import ddsketch as dd


def _exact(v, q):
    s = np.sort(v)
    return s[int(np.floor(q * (len(s) - 1)))]


def test_quantiles_within_relative_accuracy():
    rng = np.random.default_rng(3)
    v = np.concatenate([rng.lognormal(0, 3, 20000), -rng.lognormal(1, 2, 5000), np.zeros(300),
                        rng.integers(0, 1000, 4000).astype(float)])
    sk = dd.Sketch().accept_all(v)
    assert sk.count() == len(v)
    for q in np.linspace(0, 1, 101):
        e = _exact(v, q)
        got = sk.quantile(q)
        assert abs(got - e) <= dd.RELATIVE_ACCURACY * abs(e) + 1e-300, (q, got, e)


def test_merge_is_union():
    rng = np.random.default_rng(4)
    a, b = rng.lognormal(0, 2, 5000), rng.lognormal(2, 1, 7000)
    m = dd.Sketch().accept_all(a).merge(dd.Sketch().accept_all(b))
    u = dd.Sketch().accept_all(np.concatenate([a, b]))
    assert m.bins() == u.bins()


def test_index_boundaries_and_zero():
    # bin i holds (gamma^i, gamma^(i+1)]-ish magnitudes: index(gamma^k * 1.0000001) == k, tiny values are zero
    for k in (-300, -1, 0, 1, 7, 500):
        x = np.array([dd.GAMMA ** k * (1 + 1e-7)])
        assert dd.index(x)[0] == k
    sk = dd.Sketch().accept_all(np.array([0.0, 1e-310, -1e-310, 5.0]))
    assert sk.zero == 3.0 and sum(sk.pos.values()) == 1.0


def test_untrackable_values_raise():
    import pytest
    with pytest.raises(ValueError):
        dd.Sketch().accept_all(np.array([1.0, np.nan]))
