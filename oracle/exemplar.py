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
(segment position in the glob, then row) -- DuckDB's ORDER BY leaves tie order open; DOUBLE / FLOAT text is
Java's Double.toString / Float.toString over the shortest round-trip digits (JDK >= 19; JDK 17 differs in rare
non-shortest cases).  Parity pinned by the restatement only (the reference holds no exemplar result vectors).
"""
from decimal import Decimal
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from . import dataexpr as dx

MESSAGE = "_cardinalhq.message"   # Commons.scala:59
SPAN_NAME = "span.name"           # Commons.scala:71
SPAN_KIND = "span.kind"           # Commons.scala:72


def _java_layout(neg: bool, digits: str, exp: int, mag: float) -> str:
    """Double.toString layout: digits d1d2... with value d1.d2... x 10^exp."""
    out = "-" if neg else ""
    if 1e-3 <= mag < 1e7:
        if exp >= 0:
            ip = digits[:exp + 1].ljust(exp + 1, "0")
            fp = digits[exp + 1:] or "0"
            return out + ip + "." + fp
        return out + "0." + "0" * (-exp - 1) + digits
    return out + digits[0] + "." + (digits[1:] or "0") + "E" + str(exp)


def java_double_text(x: float) -> str:
    """java.lang.Double.toString (shortest round-trip digits)."""
    if x != x:
        return "NaN"
    if x in (float("inf"), float("-inf")):
        return "Infinity" if x > 0 else "-Infinity"
    if x == 0:
        return "-0.0" if str(x).startswith("-") else "0.0"
    t = Decimal(repr(x)).as_tuple()
    digits = "".join(map(str, t.digits)).rstrip("0") or "0"
    exp = len(t.digits) - 1 + t.exponent
    if len(digits) == 1:   # Java prints >= 2 significant digits: the 2-digit decimal closest to the exact value
        digits, exp = _two_digits(Decimal(x))
    return _java_layout(bool(t.sign), digits, exp, abs(x))


def _two_digits(exact: Decimal):
    from decimal import Context, ROUND_HALF_EVEN
    q = Context(prec=2, rounding=ROUND_HALF_EVEN).plus(abs(exact)).as_tuple()
    d = "".join(map(str, q.digits))
    return (d.rstrip("0") or "0"), len(q.digits) - 1 + q.exponent


def java_float_text(x: float) -> str:
    """java.lang.Float.toString of a float32 value (shortest digits that round-trip as float32)."""
    f = np.float32(x)
    if f != f:
        return "NaN"
    if np.isinf(f):
        return "Infinity" if f > 0 else "-Infinity"
    if f == 0:
        return "-0.0" if np.signbit(f) else "0.0"
    sci = np.format_float_scientific(f, unique=True, trim="-")   # e.g. '1.5e-04', '1e+07'
    mant, e = sci.split("e")
    neg = mant.startswith("-")
    digits = mant.lstrip("-").replace(".", "").rstrip("0") or "0"
    exp = int(e)
    if len(digits) == 1:
        digits, exp = _two_digits(Decimal(float(f)))
    return _java_layout(neg, digits, exp, abs(float(f)))


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
