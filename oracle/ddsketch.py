"""ORACLE (test infrastructure only): DDSketch restatement for the percentile path.

The reference builds `DDSketches.unboundedDense(0.01)` per (step, group-key tags) in the worker
(core/src/main/scala/com/cardinal/utils/PushDownAggregatorStage.scala:69-81,188-197;
core/src/main/scala/com/cardinal/utils/ast/Aggregator.scala:28-41), merges per (timestamp, tags) in query-api
(core/src/main/scala/com/cardinal/eval/TimeGroupedSketchAggregator.scala:34-37) and reads
getValueAtQuantile(p / 100) (core/src/main/scala/com/cardinal/utils/ast/BaseExpr.scala:59-61).

Third-party algorithm: com.datadoghq:sketches-java 0.8.2 (core/build.gradle), not vendored and not runnable here
(no JVM).  Restated from its published algorithm (Masson, Rim, Lee, "DDSketch: a fast and fully-mergeable quantile
sketch with relative-error guarantees", VLDB 2019) and the library's LogarithmicMapping / DenseStore / quantile walk:
  gamma = 1 + 2a/(1-a), multiplier = 1/log1p(2a/(1-a)), index(v) = int(ln v * multiplier) (minus 1 when negative),
  value(i) = exp(i / multiplier) * (1 + relativeAccuracy), relativeAccuracy = (gamma-1)/(gamma+1);
  |v| <= MIN_NORMAL*gamma counts as zero; quantile q: rank = q*(count-1), walk negative bins by descending index,
  zero, positive bins ascending; first running count > rank.
Parity unpinned against the library (no reference vectors exist for sketches); pinned here by the accuracy
guarantee (tests/test_oracle_sketch.py: every quantile within relative accuracy 0.01 of the exact order statistic).
"""
import math
import struct
import sys
from typing import Dict

import numpy as np

RELATIVE_ACCURACY = 0.01
_MANT = 2.0 * RELATIVE_ACCURACY / (1.0 - RELATIVE_ACCURACY)
GAMMA = 1.0 + _MANT
MULTIPLIER = 1.0 / math.log1p(_MANT)
REL_ACC = (GAMMA - 1.0) / (GAMMA + 1.0)
MIN_INDEXABLE = sys.float_info.min * GAMMA
MAX_INDEXABLE = sys.float_info.max / GAMMA


def index(v: np.ndarray) -> np.ndarray:
    """LogLikeIndexMapping.index for positive magnitudes (vectorised; math.log per value near a bin boundary)."""
    x = np.log(v) * MULTIPLIER
    near = np.abs(x - np.round(x)) < 1e-9
    if np.any(near):
        x = x.copy()
        for i in np.nonzero(near)[0]:
            x[i] = math.log(float(v[i])) * MULTIPLIER
    t = np.trunc(x).astype(np.int64)
    return np.where(x >= 0, t, t - 1)


def value(i: int) -> float:
    return math.exp(i / MULTIPLIER) * (1.0 + REL_ACC)


class Sketch:
    def __init__(self):
        self.pos: Dict[int, float] = {}
        self.neg: Dict[int, float] = {}
        self.zero = 0.0

    def accept_all(self, v: np.ndarray):
        """DDSketch.accept over an array (raises on NaN / out-of-range values, like checkValueTrackable)."""
        v = np.asarray(v, dtype=np.float64)
        a = np.abs(v)
        if np.any(~(a <= MAX_INDEXABLE)):
            raise ValueError("value outside the trackable range")
        z = a <= MIN_INDEXABLE
        self.zero += float(np.count_nonzero(z))
        for store, sel in ((self.pos, (v > 0) & ~z), (self.neg, (v < 0) & ~z)):
            if np.any(sel):
                ks, cs = np.unique(index(a[sel]), return_counts=True)
                for k, c in zip(ks.tolist(), cs.tolist()):
                    store[k] = store.get(k, 0.0) + float(c)
        return self

    def merge(self, o: "Sketch"):
        for src, dst in ((o.pos, self.pos), (o.neg, self.neg)):
            for k, c in src.items():
                dst[k] = dst.get(k, 0.0) + c
        self.zero += o.zero
        return self

    def count(self) -> float:
        return self.zero + sum(self.pos.values()) + sum(self.neg.values())

    def quantile(self, q: float) -> float:
        rank = q * (self.count() - 1.0)
        n = 0.0
        for k in sorted(self.neg, reverse=True):
            n += self.neg[k]
            if n > rank:
                return -value(k)
        n += self.zero
        if n > rank:
            return 0.0
        for k in sorted(self.pos):
            n += self.pos[k]
            if n > rank:
                return value(k)
        return value(max(self.pos)) if self.pos else 0.0

    def bins(self):
        return (dict(self.pos), dict(self.neg), self.zero)


def decode(buf: bytes) -> Sketch:
    """Parse the DDSketch protobuf message (mapping=1, positiveValues=2, negativeValues=3, zeroCount=4; Store:
    binCounts map=1, contiguousBinCounts=2 packed doubles, contiguousBinIndexOffset=3 sint32)."""
    def varint(b, i):
        r = s = 0
        while True:
            x = b[i]
            i += 1
            r |= (x & 0x7F) << s
            s += 7
            if x < 0x80:
                return r, i

    def fields(b):
        i = 0
        while i < len(b):
            key, i = varint(b, i)
            f, wt = key >> 3, key & 7
            if wt == 0:
                v, i = varint(b, i)
            elif wt == 1:
                v = b[i:i + 8]
                i += 8
            elif wt == 2:
                n, i = varint(b, i)
                v = b[i:i + n]
                i += n
            elif wt == 5:
                v = b[i:i + 4]
                i += 4
            else:
                raise ValueError(f"wire type {wt}")
            yield f, wt, v

    def store(b, dst):
        counts, off = [], 0
        for f, wt, v in fields(b):
            if f == 2:
                counts = list(struct.unpack(f"<{len(v) // 8}d", v))
            elif f == 3:
                off = (v >> 1) ^ -(v & 1)
            elif f == 1:   # map entry {key sint32 = 1, value double = 2}
                k, c = 0, 0.0
                for f2, _, v2 in fields(v):
                    if f2 == 1:
                        k = (v2 >> 1) ^ -(v2 & 1)
                    else:
                        c = struct.unpack("<d", v2)[0]
                dst[k] = dst.get(k, 0.0) + c
        for j, c in enumerate(counts):
            if c:
                dst[off + j] = dst.get(off + j, 0.0) + c

    s = Sketch()
    for f, wt, v in fields(buf):
        if f == 1:
            for f2, _, v2 in fields(v):
                if f2 == 1 and struct.unpack("<d", v2)[0] != GAMMA:
                    raise ValueError("unexpected gamma")
        elif f == 2:
            store(v, s.pos)
        elif f == 3:
            store(v, s.neg)
        elif f == 4:
            s.zero = struct.unpack("<d", v)[0]
    return s
