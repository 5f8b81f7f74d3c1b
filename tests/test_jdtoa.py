"""Java 17 Double.toString / Float.toString (CPU, no GPU): the exemplar path's text (lakeside_amd/csrc/jdtoa.cpp via
liblakeside_text.so) against the oracle's restatement (oracle/exemplar.py), both pinned by outputs the JDK documents.

The reference runs on eclipse-temurin:17 (query-worker/Dockerfile:20), whose FloatingDecimal prints some values with
more digits than the shortest round-trip form; no JDK is in this image, so the pins are the JDK's own published
strings: the Javadoc of the Double / Float constants and the examples of JDK-4511638 (the bug JDK 19 fixed by
switching to shortest digits)."""
import ctypes
import os
import random
import struct

import numpy as np
import pytest

from oracle import exemplar as ex

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "lakeside_amd", "liblakeside_text.so")

# (value, JDK 17 text)
PINNED_DOUBLE = [
    (4.9e-324, "4.9E-324"),                                  # Double.MIN_VALUE Javadoc
    (2.2250738585072014e-308, "2.2250738585072014E-308"),    # Double.MIN_NORMAL Javadoc
    (1.7976931348623157e308, "1.7976931348623157E308"),      # Double.MAX_VALUE Javadoc
    (2e23, "1.9999999999999998E23"),                         # JDK-4511638 (JDK 19: "2.0E23")
    (2.82879384806159e17, "2.82879384806159008E17"),         # JDK-4511638: the long path keeps a noise digit
    (1.0e23, "9.999999999999999E22"),                        # same tie as 2e23 (strict stop in the long branch)
    (0.001, "0.001"), (1.0e-4, "1.0E-4"), (9999999.0, "9999999.0"), (1.0e7, "1.0E7"),
    (0.1 + 0.2, "0.30000000000000004"), (2.0 ** 53, "9.007199254740992E15"), (-0.0, "-0.0"),
]
PINNED_FLOAT = [
    (1.4e-45, "1.4E-45"),                 # Float.MIN_VALUE Javadoc
    (1.17549435e-38, "1.17549435E-38"),   # Float.MIN_NORMAL Javadoc (nine digits: not the shortest "1.1754944E-38")
    (3.4028235e38, "3.4028235E38"),       # Float.MAX_VALUE Javadoc
    (0.1, "0.1"), (1.0e10, "1.0E10"), (16777216.0, "1.6777216E7"), (-2.5, "-2.5"),
]


class Text:
    _L = None

    @classmethod
    def lib(cls):
        if cls._L is None:
            L = ctypes.CDLL(LIB)
            for f, t in ((L.lk_java_double_text, ctypes.c_double), (L.lk_java_float_text, ctypes.c_float)):
                f.argtypes = [t, ctypes.c_char_p, ctypes.c_size_t]
                f.restype = ctypes.c_int
            cls._L = L
        return cls._L

    @classmethod
    def double(cls, x: float) -> str:
        buf = ctypes.create_string_buffer(64)
        n = cls.lib().lk_java_double_text(x, buf, 64)
        assert n > 0
        return buf.value.decode()

    @classmethod
    def float(cls, x: float) -> str:
        buf = ctypes.create_string_buffer(64)
        n = cls.lib().lk_java_float_text(x, buf, 64)
        assert n > 0
        return buf.value.decode()


def test_oracle_pinned():
    for v, s in PINNED_DOUBLE:
        assert ex.java_double_text(v) == s, (v, s)
    for v, s in PINNED_FLOAT:
        assert ex.java_float_text(v) == s, (v, s)


def test_native_pinned():
    for v, s in PINNED_DOUBLE:
        assert Text.double(v) == s, (v, s)
    for v, s in PINNED_FLOAT:
        assert Text.float(v) == s, (v, s)
    assert Text.double(float("nan")) == "NaN" and Text.double(float("-inf")) == "-Infinity"
    buf = ctypes.create_string_buffer(4)
    assert Text.lib().lk_java_double_text(1.2345, buf, 4) == -1


def _doubles(rng, n):
    out = []
    for _ in range(n):
        k = rng.randrange(6)
        if k == 0:     # any bit pattern
            x = struct.unpack("<d", struct.pack("<Q", rng.getrandbits(64)))[0]
        elif k == 1:   # integers in the long ("easy") path
            x = float(rng.getrandbits(rng.randrange(1, 64))) * rng.choice((1, -1))
        elif k == 2:   # subnormals
            x = struct.unpack("<d", struct.pack("<Q", rng.getrandbits(rng.randrange(1, 52))))[0]
        elif k == 3:   # around the plain / E-form boundaries and typical metric values
            x = rng.choice((1e-3, 1e7, 1.0, 100.0)) * (1 + rng.uniform(-1e-9, 1e-9))
        elif k == 4:   # short decimals
            x = round(rng.uniform(-1e6, 1e6), rng.randrange(0, 6))
        else:          # decimal ties like 1e23 / 2e23
            x = float(f"{rng.randrange(1, 10)}e{rng.randrange(-320, 308)}")
        if x == x:
            out.append(x)
    return out


@pytest.mark.parametrize("seed", [1, 2])
def test_native_matches_oracle_double(seed):
    rng = random.Random(seed)
    for x in _doubles(rng, 20000):
        a, b = ex.java_double_text(x), Text.double(x)
        assert a == b, (repr(x), a, b)
        if "Infinity" not in a:
            assert float(a) == x, (repr(x), a)   # every JDK 17 string still reads back as the same double


@pytest.mark.parametrize("seed", [3, 4])
def test_native_matches_oracle_float(seed):
    rng = random.Random(seed)
    for _ in range(20000):
        k = rng.randrange(3)
        if k == 0:
            bits = rng.getrandbits(32)
        elif k == 1:
            bits = struct.unpack("<I", struct.pack("<f", float(rng.getrandbits(rng.randrange(1, 40)))))[0]
        else:
            bits = rng.getrandbits(rng.randrange(1, 23))
        x = struct.unpack("<f", struct.pack("<I", bits))[0]
        if x != x:
            continue
        a, b = ex.java_float_text(x), Text.float(x)
        assert a == b, (repr(x), a, b)
        if "Infinity" not in a:
            assert np.float32(float(a)) == np.float32(x), (repr(x), a)
