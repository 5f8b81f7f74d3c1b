"""Numeric comparison leaves in the oracle (BaseExpr.scala:450-459, 488-498): the literal normalization restated from
QuantityParser (core/src/main/scala/com/cardinal/utils/QuantityParser.scala) and Double.parseDouble, pinned by hand
from the Scala source (unit tables, left-to-right Double arithmetic, .getOrElse(0.0) on a missing unit)."""
import math

import pytest

from oracle import dataexpr as dx


def _f(v, dt, op="gt"):
    return dx.Filter(k="x", v=tuple(v) if isinstance(v, list) else (v,), op=op, dataType=dt)


@pytest.mark.parametrize("v,dt,want", [
    ("1.5ms", "duration", 1500000.0), ("10m", "duration", 600000000000.0), ("2h", "duration", 7200000000000.0),
    ("3µs", "duration", 3000.0), ("1d", "duration", 86400000000000.0), ("250ns", "duration", 250.0),
    ("10m", "datasize", 1e7), ("2kb", "datasize", 2000.0), ("1.5GiB", "datasize", 1.5 * 134200000),
    ("3KiB", "datasize", 384.0), ("latency 5s", "duration", 5e9),
    ("5", "duration", 0.0),            # no unit: the regex needs a word after the digits -> 0.0
    ("50", "duration", 0.0),           # digits split "5" + unit "0": unknown unit -> 0.0
    ("7parsecs", "duration", 0.0),     # unknown unit -> 0.0
    ("1e3", "number", 1000.0), ("1.5f", "number", 1.5), (" -2.25 ", "number", -2.25), (".5", "number", 0.5),
])
def test_normalized_value(v, dt, want):
    assert dx.normalized_value(_f(v, dt)) == want


@pytest.mark.parametrize("v,dt", [("abc", "number"), ("NaN", "number"), ("Infinity", "number"), ("1_000", "number"),
                                  ("5", "string"), ("0x10", "number")])
def test_normalized_value_sql_errors(v, dt):
    with pytest.raises(dx.GlobSqlError):
        dx.normalized_value(_f(v, dt))


def test_literal_checks_per_glob():
    bad = dx.Filter(k="x", v=("abc",), op="gt", dataType="number")
    assert not dx._check_numeric_literals(bad, set())          # the field exists: the SQL fails
    assert dx._check_numeric_literals(bad, {"x"})              # nonexistent: `false`, the literal is never built
    lst = dx.Filter(k="x", v=("1", "2"), op="gt", dataType="number")
    assert not dx._check_numeric_literals(lst, {"x"})          # a list for a normalized type throws regardless


def test_num_leaf_semantics():
    col = dx._NumCol([None, 1, 2, 3, 2 ** 60 + 1], "int")
    t, f = dx._num_leaf(_f("2", "number", "ge"), col, 5)
    assert t.tolist() == [False, False, True, True, True] and f.tolist() == [False, True, False, False, False]
    # a scientific literal (|c| >= 1e7) is a DOUBLE: 2^60 + 1 casts to 2^60, which is not > 2^60
    t, _ = dx._num_leaf(_f(repr(float(2 ** 60)), "number", "gt"), col, 5)
    assert not t[4]
    fc = dx._NumCol([float("nan"), -0.5, 0.25, None], "float")
    t, f = dx._num_leaf(_f("0.25", "number", "lt"), fc, 4)
    assert t.tolist() == [False, True, False, False] and f.tolist() == [True, False, True, False]
    t, _ = dx._num_leaf(_f("0", "number", "gt"), fc, 4)
    assert t[0] and math.isnan(fc.vals[0])                     # NaN sorts greatest
