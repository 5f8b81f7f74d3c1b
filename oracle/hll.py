"""ORACLE (test infrastructure only): HLL restatement for the cardinality path (`ces`).

Reference: one org.apache.datasketches HllSketch(12, HLL_4) per time step over every row's group-key string
groupBys.map(g => tags.getOrElse(g, "")).mkString(":")
(core/src/main/scala/com/cardinal/utils/ast/Aggregator.scala:43-60,
core/src/main/scala/com/cardinal/utils/PushDownAggregatorStage.scala:82-94,183-186); query-api unions them and reads
getEstimate (core/src/main/scala/com/cardinal/eval/TimeGroupedSketchAggregator.scala:38-43,
core/src/main/scala/com/cardinal/utils/ast/BaseExpr.scala:56-58).

Third-party: datasketches-java 4.2.0 (not vendored, no JVM).  Restated: empty strings are ignored; UTF-8 bytes ->
MurmurHash3_x64_128(seed 9001) -> coupon (min(nlz(h2), 62) + 1) << 26 | (h1 & 0x3FFFFFF).  The estimator is the
published HLL (Flajolet et al. 2007) over the 2^12 registers with linear counting, and the exact coupon count while
the sketch would be in its LIST/SET modes (<= 384 coupons); datasketches' interpolation / HIP estimators are not
restated (parity of the estimate unpinned; the distinct key set per step -- the GPU's product -- is exact).
"""
import math
from typing import Iterable

M64 = (1 << 64) - 1


def _rotl(x, r):
    return ((x << r) | (x >> (64 - r))) & M64


def _fmix(k):
    k ^= k >> 33
    k = (k * 0xFF51AFD7ED558CCD) & M64
    k ^= k >> 33
    k = (k * 0xC4CEB9FE1A85EC53) & M64
    k ^= k >> 33
    return k


def murmur3_x64_128(data: bytes, seed: int = 0):
    c1, c2 = 0x87C37B91114253D5, 0x4CF5AD432745937F
    h1 = h2 = seed & M64
    n = len(data)
    nb = n // 16
    for i in range(nb):
        k1 = int.from_bytes(data[16 * i:16 * i + 8], "little")
        k2 = int.from_bytes(data[16 * i + 8:16 * i + 16], "little")
        k1 = (_rotl((k1 * c1) & M64, 31) * c2) & M64
        h1 ^= k1
        h1 = (_rotl(h1, 27) + h2) & M64
        h1 = (h1 * 5 + 0x52DCE729) & M64
        k2 = (_rotl((k2 * c2) & M64, 33) * c1) & M64
        h2 ^= k2
        h2 = (_rotl(h2, 31) + h1) & M64
        h2 = (h2 * 5 + 0x38495AB5) & M64
    tail = data[16 * nb:]
    k1 = int.from_bytes(tail[:8], "little") if tail else 0
    k2 = int.from_bytes(tail[8:16], "little") if len(tail) > 8 else 0
    if len(tail) > 8:
        h2 ^= (_rotl((k2 * c2) & M64, 33) * c1) & M64
    if tail:
        h1 ^= (_rotl((k1 * c1) & M64, 31) * c2) & M64
    h1 ^= n
    h2 ^= n
    h1 = (h1 + h2) & M64
    h2 = (h2 + h1) & M64
    h1, h2 = _fmix(h1), _fmix(h2)
    h1 = (h1 + h2) & M64
    h2 = (h2 + h1) & M64
    return h1, h2


def coupon(s: str) -> int:
    if not s:
        return 0
    h1, h2 = murmur3_x64_128(s.encode("utf-8"), 9001)
    lz = 64 - h2.bit_length()
    return ((min(lz, 62) + 1) << 26) | (h1 & 0x3FFFFFF)


def estimate(keys: Iterable[str], lg_k: int = 12) -> float:
    cs = {c for c in (coupon(k) for k in keys) if c}
    if len(cs) <= 384:
        return float(len(cs))
    m = 1 << lg_k
    reg = [0] * m
    for c in cs:
        slot, v = c & (m - 1), c >> 26
        reg[slot] = max(reg[slot], v)
    s = sum(2.0 ** -r for r in reg)
    zeros = reg.count(0)
    e = 0.7213 / (1.0 + 1.079 / m) * m * m / s
    if e <= 2.5 * m and zeros:
        return m * math.log(m / zeros)
    return e
