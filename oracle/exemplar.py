"""CPU restatement of the worker's exemplar (raw-row) queries -- TEST INFRASTRUCTURE ONLY (the checker for
tests/ and smoke(); never imported by the product path).

Per glob (Commons.scala:361-389) the worker runs
    SELECT "_cardinalhq.timestamp", "_cardinalhq.value", "_cardinalhq.name", "_cardinalhq.message", *   (logs)
    FROM (SELECT * FROM read_parquet([...], union_by_name=True) WHERE <window>) WHERE <filter>
    ORDER BY "_cardinalhq.timestamp" <order> LIMIT <limit>
(BaseExpr.getBaseQuery, BaseExpr.scala:206-239; traces project "span.name", "span.kind" instead, 41-45), turns
every row into DataPoint(ts, getDouble(col 2), tags = later columns that are non-NULL, not "null", not "") with
JDBC getString text (Commons.toDataPoint, Commons.scala:428-459), passes the rows through
PushDownAggregatorStage (exemplarsOnly, PushDownAggregatorStage.scala:42,66-68), and folds the globs' streams
with Akka mergeSorted under pushDownResponseOrdering (Commons.scala:116-132, 391-392).

Choices where the reference is unspecified (same in the GPU path): rows tied on the timestamp keep file order
(segment position in the glob, then row) -- DuckDB's ORDER BY leaves tie order open.  DOUBLE / FLOAT text is
Java 17's Double.toString / Float.toString (the reference's runtime: query-worker/Dockerfile:20, eclipse-temurin:17),
restated below.  Parity pinned by the restatement only (the reference holds no exemplar result vectors).
"""
import math
import struct
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from . import dataexpr as dx

MESSAGE = "_cardinalhq.message"   # Commons.scala:59
SPAN_NAME = "span.name"           # Commons.scala:71
SPAN_KIND = "span.kind"           # Commons.scala:72


# ----------------------------------------------------------------------------------------------
# JDK 17 java.lang.Double.toString / Float.toString: sun.misc.FloatingDecimal's BinaryToASCIIBuffer.dtoa +
# getChars (the reference runs on Java 17, query-worker/Dockerfile:20; JDK 19 replaced this algorithm by a
# shortest-digit one, which differs for rare values: 2e23 prints 1.9999999999999998E23 here, 2.0E23 on JDK 19).  Restated from the algorithm (Steele & White / dtoa digit generation with a
# symmetric half-ulp stopping test, an estimated decimal exponent, the "easy" long-integer case, and the int / long /
# big-integer branches with their own `high` comparisons); Python integers make the big-integer branch exact.
# No JDK in this image and the reference holds no printed vectors: pinned by the JDK's documented outputs
# (tests/test_oracle_exemplar.py: Javadoc constants such as Float.MIN_NORMAL = 1.17549435E-38, and the JDK-4511638
# examples that JDK 17 prints with non-shortest digits).
# ----------------------------------------------------------------------------------------------
_N_5_BITS = [0, 3, 5, 7, 10, 12, 14, 17, 19, 21, 24, 26, 28, 31, 33, 35, 38, 40, 42, 45, 47, 49, 52, 54, 56, 59, 61]
_INSIGNIFICANT = [0, 0, 0, 0, 1, 1, 1, 2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 5, 5, 5, 6, 6, 6, 6, 7, 7, 7, 8, 8, 8, 9, 9, 9,
                  9, 10, 10, 10, 11, 11, 11, 12, 12, 12, 12, 13, 13, 13, 14, 14, 14, 15, 15, 15, 15, 16, 16, 16, 17,
                  17, 17, 18, 18, 18, 19]
_EXP_SHIFT = 52


def _estimate_dec_exp(fract_bits: int, bin_exp: int) -> int:
    """FloatingDecimal.estimateDecExp: floor((d2 - 1.5) * 0.289529654 + 0.176091259 + binExp * log10(2))."""
    d2 = struct.unpack("<d", struct.pack("<Q", (0x3ff << 52) | (fract_bits & ((1 << 52) - 1))))[0]
    d = (d2 - 1.5) * 0.289529654 + 0.176091259 + float(bin_exp) * 0.301029995663981
    return math.floor(d)


def _dtoa(bin_exp: int, fract_bits: int, n_sig: int):
    """BinaryToASCIIBuffer.dtoa (isCompatibleFormat = true): (digits, decExponent)."""
    tail_zeros = (fract_bits & -fract_bits).bit_length() - 1
    n_fract_bits = _EXP_SHIFT + 1 - tail_zeros
    n_tiny_bits = max(0, n_fract_bits - bin_exp - 1)
    if -21 <= bin_exp <= 62 and n_tiny_bits < 27 and n_fract_bits + _N_5_BITS[n_tiny_bits] < 64 and n_tiny_bits == 0:
        # the easy case: an integer value that fits a long (developLongDigits)
        insignificant = _INSIGNIFICANT[bin_exp - n_sig - 1] if bin_exp > n_sig and 1 < bin_exp - n_sig - 1 < 64 else 0
        lvalue = fract_bits << (bin_exp - _EXP_SHIFT) if bin_exp >= _EXP_SHIFT else fract_bits >> (_EXP_SHIFT - bin_exp)
        dec_exp = 0
        if insignificant:
            pow10 = 10 ** insignificant
            residue = lvalue % pow10
            lvalue //= pow10
            dec_exp += insignificant
            if residue >= (pow10 >> 1):
                lvalue += 1
        s = str(lvalue)
        stripped = s.rstrip("0")
        dec_exp += len(s) - 1
        return list(stripped), dec_exp + 1
    dec_exp = _estimate_dec_exp(fract_bits, bin_exp)
    b5 = max(0, -dec_exp)
    b2 = b5 + n_tiny_bits + bin_exp
    s5 = max(0, dec_exp)
    s2 = s5 + n_tiny_bits
    m5 = b5
    m2 = b2 - n_sig
    fract_bits >>= tail_zeros
    b2 -= n_fract_bits - 1
    common = min(b2, s2)
    b2 -= common
    s2 -= common
    m2 -= common
    if n_fract_bits == 1:
        m2 -= 1
    if m2 < 0:
        b2 -= m2
        s2 -= m2
        m2 = 0
    b_bits = n_fract_bits + b2 + (_N_5_BITS[b5] if b5 < len(_N_5_BITS) else b5 * 3)
    ten_s_bits = s2 + 1 + (_N_5_BITS[s5 + 1] if s5 + 1 < len(_N_5_BITS) else (s5 + 1) * 3)
    small = b_bits < 64 and ten_s_bits < 64        # int / long branches: high = b + m > tens
    b = fract_bits * 5 ** b5 << b2
    s = 5 ** s5 << s2
    m = 5 ** m5 << m2
    tens = s * 10
    digits = []

    def is_high(b, m):
        return b + m > tens if small else b + m >= tens   # FDBigInteger.addAndCmp(B, M) <= 0 in the big branch

    q, b = divmod(b, s)
    b *= 10
    m *= 10
    low, high = b < m, is_high(b, m)
    if q == 0 and not high:
        dec_exp -= 1
    else:
        digits.append(chr(48 + q))
    if dec_exp < -3 or dec_exp >= 8:
        low = high = False
    while not low and not high:
        q, b = divmod(b, s)
        b *= 10
        m *= 10
        low, high = b < m, is_high(b, m)
        digits.append(chr(48 + q))
    low_diff = 2 * b - tens
    dec_exponent = dec_exp + 1
    if high and (not low or low_diff > 0 or (low_diff == 0 and (ord(digits[-1]) & 1))):
        i = len(digits) - 1
        while digits[i] == "9" and i > 0:   # roundup()
            digits[i] = "0"
            i -= 1
        if digits[i] == "9":
            dec_exponent += 1
            digits[0] = "1"
        else:
            digits[i] = chr(ord(digits[i]) + 1)
    return digits, dec_exponent


def _java_chars(neg: bool, digits, dec_exponent: int) -> str:
    """BinaryToASCIIBuffer.getChars."""
    out = "-" if neg else ""
    nd = len(digits)
    if 0 < dec_exponent < 8:
        n = min(nd, dec_exponent)
        out += "".join(digits[:n])
        if n < dec_exponent:
            return out + "0" * (dec_exponent - n) + ".0"
        return out + "." + ("".join(digits[n:]) if n < nd else "0")
    if -3 < dec_exponent <= 0:
        return out + "0." + "0" * (-dec_exponent) + "".join(digits)
    out += digits[0] + "." + ("".join(digits[1:]) if nd > 1 else "0") + "E"
    return out + ("-" + str(-dec_exponent + 1) if dec_exponent <= 0 else str(dec_exponent - 1))


def java_double_text(x: float) -> str:
    """java.lang.Double.toString on JDK 17 (FloatingDecimal.toJavaFormatString)."""
    bits = struct.unpack("<Q", struct.pack("<d", x))[0]
    neg = bits >> 63 != 0
    fract = bits & ((1 << 52) - 1)
    bexp = (bits >> 52) & 0x7ff
    if bexp == 0x7ff:
        return "NaN" if fract else ("-Infinity" if neg else "Infinity")
    if bexp == 0:
        if fract == 0:
            return "-0.0" if neg else "0.0"
        lz = 64 - fract.bit_length()
        shift = lz - (63 - _EXP_SHIFT)
        fract <<= shift
        bexp = 1 - shift
        nsig = 64 - lz
    else:
        fract |= 1 << 52
        nsig = 53
    digits, dexp = _dtoa(bexp - 1023, fract, nsig)
    return _java_chars(neg, digits, dexp)


def java_float_text(x: float) -> str:
    """java.lang.Float.toString on JDK 17 (the same dtoa over the float's 24 significant bits)."""
    bits = struct.unpack("<I", struct.pack("<f", x))[0]
    neg = bits >> 31 != 0
    fract = bits & ((1 << 23) - 1)
    bexp = (bits >> 23) & 0xff
    if bexp == 0xff:
        return "NaN" if fract else ("-Infinity" if neg else "Infinity")
    if bexp == 0:
        if fract == 0:
            return "-0.0" if neg else "0.0"
        lz = 32 - fract.bit_length()
        shift = lz - (31 - 23)
        fract <<= shift
        bexp = 1 - shift
        nsig = 32 - lz
    else:
        fract |= 1 << 23
        nsig = 24
    digits, dexp = _dtoa(bexp - 127, fract << (_EXP_SHIFT - 23), nsig)
    return _java_chars(neg, digits, dexp)


_RANK = {"int32": 1, "int64": 2, "float": 3, "double": 4}


def _kind(t) -> str:
    import pyarrow as pa
    if pa.types.is_dictionary(t):
        t = t.value_type
    if pa.types.is_int32(t):
        return "int32"
    if pa.types.is_int64(t):
        return "int64"
    if pa.types.is_float32(t):
        return "float"
    if pa.types.is_float64(t):
        return "double"
    if pa.types.is_boolean(t):
        return "bool"
    if pa.types.is_string(t) or pa.types.is_large_string(t):
        return "string"
    raise NotImplementedError(f"column type {t}")


def union_type(a: Optional[str], b: str) -> str:
    """union_by_name common type (the build's restated subset: equal types; INT32/INT64 -> BIGINT; with FLOAT ->
    FLOAT; with DOUBLE -> DOUBLE)."""
    if a is None or a == b:
        return b
    ra, rb = _RANK.get(a, 0), _RANK.get(b, 0)
    if not ra or not rb:
        raise NotImplementedError("union_by_name over incompatible types")
    if ra <= 2 and rb <= 2:
        return "int64"
    return "double" if 4 in (ra, rb) else "float"


def _text(v, kind: str, utype: str) -> str:
    """JDBC getString of a value read as the union type."""
    if kind == "string":
        return v
    if kind == "bool":
        return "true" if v else "false"
    if utype in ("int32", "int64"):
        return str(int(v))
    if utype == "float":
        return java_float_text(float(v))
    return java_double_text(float(np.float32(v)) if kind == "float" else float(v))


def evaluate_exemplar_glob(pr: dx.PushDownRequest, seg_idx: Sequence[int], paths: Sequence[str], sources=None):
    """One glob's rows [(ts, value, tags)] in ORDER BY order, LIMIT applied."""
    import pyarrow as pa
    import pyarrow.parquet as pq
    be = pr.baseExpr
    segs = [pr.segmentRequests[i] for i in seg_idx]
    proj = [dx.TIMESTAMP, dx.VALUE] + ([dx.NAME, MESSAGE] if be.dataset == dx.LOGS else [SPAN_NAME, SPAN_KIND])
    tables, union, types = [], [], {}
    try:
        for i, p in enumerate(paths):
            t = pq.read_table(p if sources is None else pa.BufferReader(sources[i]))
            tables.append(t)
            for f in t.schema:
                if f.name not in types:
                    union.append(f.name)
                types[f.name] = union_type(types.get(f.name), _kind(f.type))
    except Exception:   # unreadable file / a union DuckDB cannot form: the glob's query fails -> empty
        return []       # (Commons.scala:249-253)
    fs = dx.field_set(be)
    nonexistent = fs - set(union)
    leafcols = dx._leaf_columns(be.filter)
    if any(c not in types for c in proj) or any(c not in types for c in set(leafcols) - nonexistent):
        return []                                                    # Binder Error -> empty (Commons.scala:249-253)
    start = min(s.startTs for s in segs)
    end = max(s.endTs for s in segs)
    numcols = sorted({l.k for l in dx._leaves(be.filter) if l.op in dx.NUMERIC_OPS} - nonexistent)
    if any(types.get(c) == "string" for c in numcols) or not dx._check_numeric_literals(be.filter, nonexistent):
        return []                                                    # VARCHAR vs number / bad literal: SQL error
    strings = sorted(set(leafcols) - nonexistent - set(numcols))
    _, nums, strs = dx._read_glob(paths, [dx.TIMESTAMP], strings, sources)
    strs.update(dx._read_numeric(paths, [c for c in numcols if c in types], sources))
    ts, tsv = nums[dx.TIMESTAMP]
    ts = ts.astype(np.int64)
    n = len(ts)
    try:
        t, _ = dx._eval_filter(be.filter, strs, nonexistent, n)
    except dx.GlobSqlError:   # a regex RE2 rejects fails the glob's SQL
        return []
    keep = np.nonzero(tsv & (ts >= start) & (ts < end) & t)[0]
    desc = be.order.upper() == "DESC"
    order = np.argsort(-ts[keep] if desc else ts[keep], kind="stable")   # ties: file order
    sel = keep[order][:max(be.limit, 0)]
    offs = np.cumsum([0] + [tb.num_rows for tb in tables])
    cols = proj + [u for u in union if u not in proj]
    out = []
    for gi in sel:
        f = int(np.searchsorted(offs, gi, side="right") - 1)
        r = int(gi - offs[f])
        tb = tables[f]
        tags: Dict[str, str] = {}
        value = 0.0
        for c in cols:
            if c not in tb.column_names:
                continue
            v = tb.column(c)[r].as_py()
            if v is None:
                continue
            kind = _kind(tb.schema.field(c).type)
            if c == dx.VALUE:
                value = float(np.float32(v)) if kind == "float" else float(v)
            s = _text(v, kind, types[c])
            if s != "null" and s != "":
                tags[c] = s
        out.append((int(ts[gi]), value, tags))
    return out


def evaluate_exemplar_per_glob(pr: dx.PushDownRequest, paths: Sequence[str], glob_size: int = 10, sources=None):
    return [evaluate_exemplar_glob(pr, g, [paths[i] for i in g], None if sources is None else [sources[i] for i in g])
            for g in dx.globs_of(pr, glob_size)]


def merge_sorted_fold(per_glob, reverse: bool) -> List[Tuple[int, float, Dict[str, str]]]:
    """sources.fold(Source.empty)(_ mergeSorted _) (Commons.scala:391-392): Akka MergeSorted emits the left head
    when it is strictly less under the ordering (timestamp; negated when reverseSort, Commons.scala:116-132),
    the right head otherwise."""
    def less(a, b):
        return a[0] > b[0] if reverse else a[0] < b[0]
    stream: list = []
    for g in per_glob:
        m, i, j = [], 0, 0
        while i < len(stream) and j < len(g):
            if less(stream[i], g[j]):
                m.append(stream[i])
                i += 1
            else:
                m.append(g[j])
                j += 1
        m.extend(stream[i:])
        m.extend(g[j:])
        stream = m
    return stream


def evaluate_exemplar(pr: dx.PushDownRequest, paths: Sequence[str], glob_size: int = 10, sources=None):
    """evaluatePushDownRequest's exemplar stream: [(ts, value, tags, glob index)]."""
    per = evaluate_exemplar_per_glob(pr, paths, glob_size, sources)
    tagged = [[(r[0], r[1], r[2], gi) for r in g] for gi, g in enumerate(per)]
    return merge_sorted_fold(tagged, pr.reverseSort)
