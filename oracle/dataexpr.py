"""CPU restatement of lakeside's sealed-segment DataExpr evaluation (TEST INFRASTRUCTURE ONLY).

This module is the parity oracle.  Only ``tests/``, ``__graft_entry__.smoke()`` and
``bench.py``'s ``cpu_baseline`` leg may import it, and only as the checker: the product path
(``lakeside_amd``) never routes through it.

Pinning.  The reference's arithmetic runs inside DuckDB 1.3.2 (``org.duckdb:duckdb_jdbc:1.3.2.0``,
``ext.gradle:24``), which is neither vendored nor installed; the reference is Scala/JVM and cannot run
here.  The reference pins no numeric result.  What IS pinned:
  * the plan: ``oracle/sqlplan.py`` restates ``BaseExpr.generateSql`` and is checked against the exact
    SQL strings of ``query-api/src/test/scala/com/cardinal/queryapi/utils/ASTUtilsBaseExprTest.scala``;
  * the numbers: this numpy restatement is cross-checked, fixture by fixture, against that generated SQL
    executed by an independent SQL engine (SQLite, ``oracle/sqlplan.py::run_sql``).
Counts/min/max are exact; sums are the correctly rounded sum (``math.fsum``), which is the
order-independent target the reference's parallel DuckDB sum approximates.

Semantics follow SURVEY.md Appendix A (S1-S22); each function cites the reference file:line it restates.
"""
from __future__ import annotations

import functools
import json
import math
import re
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional, Sequence, Tuple

import numpy as np

TIMESTAMP = "_cardinalhq.timestamp"   # core/.../utils/Commons.scala:55
VALUE = "_cardinalhq.value"           # Commons.scala:57
NAME = "_cardinalhq.name"             # Commons.scala:47
LOGS, TRACES, METRICS = "logs", "traces", "metrics"  # Commons.scala:48-50

# Operator vocabulary, core/.../logs/LogCommons.scala:21-44
EXISTS, NOT_EQUALS, REGEX, IN, NOT_IN, CONTAINS = "exists", "!=", "regex", "in", "not_in", "contains"
EQ, HAS, GT, GE, LT, LE = "eq", "has", "gt", "ge", "lt", "le"
SUM, MIN, MAX, COUNT, AVG = "sum", "min", "max", "count", "avg"


# ----------------------------------------------------------------------------------------------
# Model + JSON parsing (ASTUtils.scala:124-137, 222-229, 276-417; SegmentRequest.scala:45-98)
# ----------------------------------------------------------------------------------------------
@dataclass(frozen=True)
class Filter:
    k: str
    v: Tuple[str, ...]
    op: str
    extracted: bool = False
    computed: bool = False
    dataType: str = "string"


@dataclass(frozen=True)
class BinaryClause:
    q1: Any
    q2: Any
    op: str


@dataclass(frozen=True)
class NotClause:
    inner: Any


@dataclass
class ChartOptions:
    aggregation: str = SUM
    groupBys: List[str] = field(default_factory=list)
    type: str = "count"
    rollup: Optional[str] = None
    fieldName: Optional[str] = None
    fieldType: Optional[str] = None


@dataclass
class BaseExpr:
    id: str
    dataset: str
    filter: Any
    chart: Optional[ChartOptions]
    extract: Any = None
    compute: Any = None
    limit: int = 1000          # exemplar queries (ASTUtils.scala:360-361)
    order: str = "DESC"


@dataclass
class SegmentRequest:
    hour: str
    dateInt: str
    segmentId: str
    sealedStatus: bool
    dataset: str
    queryTags: Dict[str, Any]
    stepInMillis: int
    customerId: str
    collectorId: str
    bucketName: str
    cName: str
    startTs: int
    endTs: int


@dataclass
class PushDownRequest:
    baseExpr: BaseExpr
    segmentRequests: List[SegmentRequest]
    reverseSort: bool = False
    isTagQuery: bool = False
    processor: Optional[dict] = None


def _basic_filter(node: dict) -> Filter:
    """ASTUtils.toBasicFilter (ASTUtils.scala:276-288)."""
    if node.get("k") is None:
        raise ValueError("No `k` provided in filter!")
    op = node.get("op")
    if op is None:
        raise ValueError("No op provided for filter!")
    values = tuple(node.get("v") or [])
    if not values and op != EXISTS:
        raise ValueError(f"No value for key = {node['k']} provided in filter!")
    return Filter(k=node["k"], v=values, op=op, extracted=bool(node.get("extracted", False)),
                  computed=bool(node.get("computed", False)), dataType=node.get("dataType", "string"))


def _binary_clause(node: dict):
    """ASTUtils.toBinaryClauseFromFilterJsonNode (ASTUtils.scala:379-404): every non-textual member of
    the object (JSON order) is a child; children fold left-associatively."""
    op = node.get("op")
    if op is None:
        raise ValueError("No `op` provided in binary query clause!")
    clauses = [handle_filter(v) for v in node.values() if not isinstance(v, str)]
    if len(clauses) < 2:
        raise ValueError("Atleast two clauses required in a binary clause!")
    acc = clauses[0]
    for c in clauses[1:]:
        acc = BinaryClause(acc, c, op)
    return acc


def handle_filter(node: dict):
    """ASTUtils.handleFilter (ASTUtils.scala:406-417)."""
    if "not" in node and node["not"] is not None:
        return NotClause(handle_filter(node["not"]))
    if node.get("k") is not None:
        return _basic_filter(node)
    return _binary_clause(node)


def to_base_expr(node: dict, id_: Optional[str] = None) -> BaseExpr:
    """ASTUtils.toBaseExpr (ASTUtils.scala:290-377)."""
    chart = None
    if node.get("chart") is not None:
        c = node["chart"]
        gb = c.get("groupBys")
        agg = c.get("aggregation")
        chart = ChartOptions(aggregation=agg if isinstance(agg, str) else SUM,
                             groupBys=list(gb) if isinstance(gb, list) else [],
                             type=c.get("type", "count"), rollup=c.get("rollup"),
                             fieldName=c.get("fieldName"), fieldType=c.get("fieldType"))
    if node.get("filter") is None:
        raise ValueError("No filter provided!")
    return BaseExpr(id=id_ if id_ is not None else node.get("id", "_"),
                    dataset=node.get("dataset", METRICS), filter=handle_filter(node["filter"]),
                    chart=chart, extract=node.get("extract"), compute=node.get("compute"),
                    limit=(node["limit"] if isinstance(node.get("limit"), int) else 0) if "limit" in node else 1000,
                    order=node["order"] if isinstance(node.get("order"), str) else "DESC")


def parse_pushdown(text: str) -> PushDownRequest:
    """PushDownRequest.fromJson (SegmentRequest.scala:45-60)."""
    p = json.loads(text)
    be = to_base_expr(p["baseExpr"])
    segs = []
    for s in p["segmentRequests"]:
        segs.append(SegmentRequest(hour=str(s.get("hour", "")), dateInt=str(s.get("dateInt", "")),
                                   segmentId=str(s.get("segmentId", "")),
                                   sealedStatus=bool(s.get("sealedStatus", True)),
                                   dataset=s.get("dataset", be.dataset), queryTags=s.get("queryTags") or {},
                                   stepInMillis=int(s["stepInMillis"]), customerId=s.get("customerId", ""),
                                   collectorId=s.get("collectorId", ""), bucketName=s.get("bucketName", ""),
                                   cName=s.get("cName", ""), startTs=int(s["startTs"]), endTs=int(s["endTs"])))
    return PushDownRequest(baseExpr=be, segmentRequests=segs, reverseSort=bool(p.get("reverseSort", False)),
                           isTagQuery=bool(p.get("isTagQuery", False)), processor=p.get("processor"))


# ----------------------------------------------------------------------------------------------
# Plan helpers
# ----------------------------------------------------------------------------------------------
def filter_field_set(q) -> set:
    """BaseExpr.filterFieldSet (BaseExpr.scala:652-663).  NOTE: a NotClause contributes nothing
    (the reference's match has no NotClause case), so a field used only under `not` is never put in
    nonExistentFields and compiles to a column reference even when absent."""
    if isinstance(q, Filter):
        return {q.k}
    if isinstance(q, BinaryClause):
        return filter_field_set(q.q1) | filter_field_set(q.q2)
    return set()


def field_set(be: BaseExpr) -> set:
    """BaseExpr.fieldSet (BaseExpr.scala:648-650)."""
    return filter_field_set(be.filter) | set(be.chart.groupBys if be.chart else [])


def exact_tags(q) -> Dict[str, Any]:
    """BaseExpr.queryTags/exactTags (BaseExpr.scala:623-646)."""
    out: Dict[str, Any] = {}
    if isinstance(q, Filter):
        if q.op == EQ:
            out[q.k] = q.v[0]
        elif q.op == IN:
            out[q.k] = list(q.v)
    elif isinstance(q, BinaryClause) and q.op == "and":
        out.update(exact_tags(q.q1))
        out.update(exact_tags(q.q2))
    return out


def value_column(be: BaseExpr) -> str:
    """Aggregated column: logs/traces `_cardinalhq.value` (BaseExpr.scala:349-351);
    metrics `rollup_<rollup|sum>` (BaseExpr.scala:376-394)."""
    if be.dataset == METRICS:
        return "rollup_" + ((be.chart.rollup if be.chart else None) or SUM)
    return VALUE


def check_hot_path(pr: PushDownRequest) -> None:
    """Raise for query shapes outside the hot path."""
    be = pr.baseExpr
    if pr.isTagQuery or be.chart is None:
        raise NotImplementedError("tag/exemplar queries are outside the hot path")
    agg = be.chart.aggregation
    if is_percentile(agg) or is_ces(be):   # logs / traces and metrics (BaseExpr.scala:379-388, 397-399)
        pass
    elif agg not in (SUM, MIN, MAX, COUNT, AVG):
        raise NotImplementedError(f"aggregation {agg} (sketch path) is outside the hot path")
    if be.chart.fieldName is not None or be.extract is not None or be.compute is not None:
        raise NotImplementedError("extract/compute/field charts are outside the hot path")
    if be.dataset not in (LOGS, TRACES, METRICS):
        raise ValueError(f"Invalid dataset: {be.dataset}")

    def walk(q):
        if isinstance(q, Filter):
            if q.extracted or q.computed:
                raise NotImplementedError("extracted/computed filter fields are outside the hot path")
            if q.op not in (EQ, NOT_EQUALS, IN, NOT_IN, REGEX, CONTAINS, HAS, EXISTS, GT, GE, LT, LE):
                raise ValueError(f"Invalid operator {q.op}")
        elif isinstance(q, BinaryClause):
            if q.op not in ("and", "or"):
                raise ValueError(f"unknown binary op {q.op}")
            walk(q.q1)
            walk(q.q2)
        else:
            walk(q.inner)
    walk(be.filter)


# ----------------------------------------------------------------------------------------------
# Regex: DuckDB regexp_matches(l, p, 'i') = RE2 partial match, case-insensitive (BaseExpr.scala:485-501)
# ----------------------------------------------------------------------------------------------
def re2_search(values: Sequence[Optional[str]], pattern: str) -> List[Optional[bool]]:
    """RE2 search over the values; a pattern RE2 rejects fails the glob's SQL (GlobSqlError) whether or not the
    glob holds any value (DuckDB compiles the constant pattern when it binds the query)."""
    import pyarrow as pa
    import pyarrow.compute as pc
    try:
        return pc.match_substring_regex(pa.array(list(values) or [""], type=pa.string()), pattern,
                                        ignore_case=True).to_pylist()[:len(values)]
    except pa.ArrowInvalid as e:
        raise GlobSqlError(f"regexp_matches: {e}") from e


# ----------------------------------------------------------------------------------------------
# Glob evaluation (Commons.toGlobResultSet 200-254 + generateSql semantics, BaseExpr.scala:319-513)
# ----------------------------------------------------------------------------------------------
class _Col:
    """A string column of a glob: dictionary codes (-1 = NULL) plus the dictionary."""

    def __init__(self, codes: np.ndarray, dictionary: List[str]):
        self.codes = codes
        self.dictionary = dictionary


def _tag_kind(typ) -> str:
    import pyarrow as pa
    if pa.types.is_dictionary(typ):
        typ = typ.value_type
    if pa.types.is_boolean(typ):
        return "bool"
    if pa.types.is_integer(typ):
        return "int"
    if pa.types.is_float32(typ):
        return "float32"
    if pa.types.is_floating(typ):
        return "float64"
    return "text"


def numeric_tag_text(kinds: set, v) -> Optional[str]:
    """JDBC getString of a numeric tag value read as the glob's union_by_name type (Commons.scala:406-423 via
    DuckDBResultSet.getString = getObject(i).toString()): BIGINT / INTEGER -> Long / Integer.toString, FLOAT ->
    Float.toString (integers of a FLOAT union cast to FLOAT first), DOUBLE -> Double.toString, BOOLEAN ->
    Boolean.toString.  Grouping is by value: every NaN is one group and -0.0 groups (and prints) as 0.0 (this
    repo's choice; DuckDB's representative of the 0.0 / -0.0 group is not pinned)."""
    from oracle.exemplar import java_double_text, java_float_text
    if v is None:
        return None
    if kinds == {"bool"}:
        return "true" if v else "false"
    if kinds <= {"int"}:
        return str(int(v))
    if "float64" in kinds:
        x = float(v)
        return "NaN" if x != x else java_double_text(0.0 if x == 0 else x)
    x = float(np.float32(v))
    return "NaN" if x != x else java_float_text(0.0 if x == 0 else x)


def _read_glob(paths: Sequence[str], numeric: Sequence[str], strings: Sequence[str], sources=None,
               numeric_tags: Sequence[str] = ()):
    """union_by_name=True read of the glob (Commons.scala:210-213): a column missing from a file is NULL
    for that file's rows.  Returns (union column names, numeric arrays + validity, string columns).
    `numeric_tags`: string-role columns (a tag query's tag) that may be numeric: their values become the JDBC
    getString text of the glob's union type (numeric_tag_text) before they are coded."""
    import pyarrow as pa
    import pyarrow.parquet as pq
    union: List[str] = []
    tables = []
    for i, p in enumerate(paths):
        src = p if sources is None else pa.BufferReader(sources[i])
        pf = pq.ParquetFile(src)
        names = pf.schema_arrow.names
        for n in names:
            if n not in union:
                union.append(n)
        want = [c for c in list(numeric) + list(strings) if c in names]
        tables.append((pf.read(columns=want, use_threads=True), pf.metadata.num_rows))
    for c in numeric_tags:
        kinds = {_tag_kind(t.schema.field(c).type) for t, _ in tables if c in t.column_names}
        if not kinds or kinds == {"text"}:
            continue
        if "text" in kinds or ("bool" in kinds and kinds != {"bool"}):
            raise NotImplementedError(f"tag column {c}: union of {sorted(kinds)} (VARCHAR / BOOLEAN with numbers)")
        conv = []
        for t, n in tables:
            if c in t.column_names:
                vals = t.column(c).to_pylist()
                col = pa.array([numeric_tag_text(kinds, v) for v in vals], pa.string())
                t = t.set_column(t.column_names.index(c), c, col)
            conv.append((t, n))
        tables = conv
    nums = {}
    for c in numeric:
        # union_by_name type of the column over the glob's files (DuckDB's common supertype, INTEGER < BIGINT <
        # FLOAT < DOUBLE); text cannot be summed / bucketed: the glob's SQL fails (Binder Error)
        kinds = set()
        for t, _ in tables:
            if c in t.column_names:
                typ = t.schema.field(c).type
                if pa.types.is_dictionary(typ):
                    typ = typ.value_type
                if pa.types.is_integer(typ):
                    kinds.add("int")
                elif pa.types.is_float32(typ):
                    kinds.add("float32")
                elif pa.types.is_floating(typ):
                    kinds.add("float64")
                else:
                    raise GlobSqlError(f"column {c} of type {typ} in a numeric role")
        via_f32 = "float32" in kinds and "float64" not in kinds   # integers of a FLOAT union are cast to FLOAT
        parts, valid = [], []
        for t, n in tables:
            if c in t.column_names:
                a = t.column(c).combine_chunks() if t.num_rows else pa.array([], pa.float64())
                arr = a.to_numpy(zero_copy_only=False)
                if via_f32:
                    arr = np.asarray(arr).astype(np.float32).astype(np.float64)
                v = np.asarray(a.is_valid().to_numpy(zero_copy_only=False), dtype=bool) if a.null_count else \
                    np.ones(n, dtype=bool)
                arr = np.where(v, arr, 0) if a.null_count else arr
                parts.append(np.asarray(arr))
                valid.append(v)
            else:
                parts.append(np.zeros(n, dtype=np.float64))
                valid.append(np.zeros(n, dtype=bool))
        nums[c] = (np.concatenate(parts) if parts else np.zeros(0), np.concatenate(valid) if valid else
                   np.zeros(0, dtype=bool))
    strs = {}
    for c in strings:
        vocab: Dict[str, int] = {}
        parts = []
        for t, n in tables:
            if c in t.column_names:
                a = t.column(c).combine_chunks()
                if pa.types.is_dictionary(a.type):
                    a = a.cast(a.type.value_type)
                d = a.dictionary_encode()
                local = d.dictionary.to_pylist()
                remap = np.array([vocab.setdefault(s, len(vocab)) for s in local] + [-1], dtype=np.int64)
                idx = d.indices.to_numpy(zero_copy_only=False)
                idx = np.where(np.asarray(d.indices.is_valid().to_numpy(zero_copy_only=False), dtype=bool),
                               idx, len(local)).astype(np.int64) if d.indices.null_count else \
                    np.asarray(idx, dtype=np.int64)
                parts.append(remap[idx])
            else:
                parts.append(np.full(n, -1, dtype=np.int64))
        inv = [None] * len(vocab)
        for s, i in vocab.items():
            inv[i] = s
        strs[c] = _Col(np.concatenate(parts) if parts else np.zeros(0, dtype=np.int64), inv)
    return union, nums, strs


# ----------------------------------------------------------------------------------------------
# Numeric comparison leaves (BaseExpr.scala:450-459, 488-498): `<label> > <normalizedValue>`
# ----------------------------------------------------------------------------------------------
NUMERIC_OPS = (GT, GE, LT, LE)


class GlobSqlError(Exception):
    """The glob's generated SQL fails (DuckDB error / exception in generateSql): an empty glob
    (Commons.scala:249-253)."""


_JAVA_DOUBLE = re.compile(r"[+-]?(NaN|Infinity|([0-9]+\.?[0-9]*|\.[0-9]+)([eE][+-]?[0-9]+)?[fFdD]?)")


def java_parse_double(text: str) -> float:
    """java.lang.Double.parseDouble (decimal grammar; surrounding whitespace, f/F/d/D suffix)."""
    t = text.strip(" \t\n\r\x0b\x0c\x00")
    if not _JAVA_DOUBLE.fullmatch(t):
        raise GlobSqlError(f"NumberFormatException: {text!r}")
    if t[-1] in "fFdD" and "Infinity" not in t:
        t = t[:-1]
    if "NaN" in t:
        return float("nan")
    if "Infinity" in t:
        return float("-inf") if t.startswith("-") else float("inf")
    return float(t)


_QUANTITY = re.compile("([0-9]+(.[0-9]+)?)(\\w+|\u00b5s)", re.ASCII)
_DUR = {**{u: lambda x: x * 1000000000.0 for u in ("s", "sec", "secs", "second", "seconds")},
        **{u: lambda x: (x * 60) * 1000000000.0 for u in ("m", "min", "mins", "minute", "minutes")},
        **{u: lambda x: x * 1000000.0 for u in ("ms", "milli", "millis", "millisecond", "milliseconds")},
        **{u: lambda x: x * 1000.0 for u in ("\u00b5s", "micro", "micros", "microsecond", "microseconds")},
        "ns": lambda x: x,
        **{u: lambda x: (x * 3600) * 1000000000.0 for u in ("h", "hr", "hrs", "hour", "hours")},
        **{u: lambda x: ((x * 24) * 3600) * 1000000000.0 for u in ("d", "day", "days")}}
_SIZE = {**dict.fromkeys(("b", "byte", "bytes"), 1.0), **dict.fromkeys(("k", "kb", "kilobyte", "kilobytes"), 1000.0),
         **dict.fromkeys(("m", "mb", "mbs", "megabyte"), 1e6),
         **dict.fromkeys(("g", "gb", "gbs", "gigabyte", "gigabytes"), 1e9),
         **dict.fromkeys(("t", "tb", "tbs", "terabyte", "terabytes"), 1e12),
         **dict.fromkeys(("pb", "pbs", "petabyte", "petabytes"), 1e15),
         **dict.fromkeys(("mib", "mibs", "mebibyte", "mebibytes"), 131072.0),
         **dict.fromkeys(("kib", "kibs", "kibibyte", "kibibytes"), 128.0),
         **dict.fromkeys(("gib", "gibs", "gibibyte", "gibibytes"), 134200000.0),
         **dict.fromkeys(("tib", "tibs", "tibibyte", "tibibytes"), 137400000000.0),
         **dict.fromkeys(("pib", "pibs", "pibibyte", "pibibytes"), 1126000000000000.0)}


def parse_quantity(value: str, duration: bool) -> Optional[float]:
    """QuantityParser.parseQuantity (core/.../utils/QuantityParser.scala:124-141): first match of
    ([0-9]+(.[0-9]+)?)(\\w+|µs), unit lower-cased, normalized left to right in Double arithmetic."""
    m = _QUANTITY.search(value)
    if not m:
        return None
    x = java_parse_double(m.group(1))
    unit = m.group(3).lower()
    if duration:
        f = _DUR.get(unit)
        return None if f is None else f(x)
    k = _SIZE.get(unit)
    return None if k is None else x * k


def normalized_value(f: Filter) -> float:
    """BaseExpr.scala:450-459: the literal of a numeric comparison (NaN / Infinity print as identifiers: an error)."""
    if f.dataType in ("duration", "datasize", "number") and len(f.v) != 1:
        raise GlobSqlError("filter value is a list of values")
    if f.dataType == "number":
        c = java_parse_double(f.v[0])
    elif f.dataType in ("duration", "datasize"):
        q = parse_quantity(f.v[0], f.dataType == "duration")
        c = 0.0 if q is None else q
    else:
        c = float("nan")
    if not math.isfinite(c):
        raise GlobSqlError(f"{f.k} {f.op} {c}")
    return c


class _NumCol:
    """A numeric column of a glob: Python values (None = NULL) and its union kind ('int' / 'float')."""

    def __init__(self, vals: list, kind: str):
        self.vals = vals
        self.kind = kind


def _read_numeric(paths: Sequence[str], names: Sequence[str], sources=None):
    """union_by_name read of numeric filter columns; a column stored as a string anywhere in the glob makes the
    comparison a Binder Error (GlobSqlError)."""
    import pyarrow as pa
    import pyarrow.parquet as pq
    out = {}
    files = []
    for i, p in enumerate(paths):
        pf = pq.ParquetFile(p if sources is None else pa.BufferReader(sources[i]))
        want = [c for c in names if c in pf.schema_arrow.names]
        files.append((pf.read(columns=want), pf.metadata.num_rows))
    for c in names:
        vals, kinds = [], set()
        for t, n in files:
            if c not in t.column_names:
                vals.extend([None] * n)
                continue
            typ = t.schema.field(c).type
            if pa.types.is_dictionary(typ):
                typ = typ.value_type
            if pa.types.is_integer(typ):
                kinds.add("int")
            elif pa.types.is_floating(typ):
                kinds.add("float")
            else:
                raise GlobSqlError(f"cannot compare {typ} column {c} with a number")
            vals.extend(t.column(c).to_pylist())
        out[c] = _NumCol(vals, "int" if kinds <= {"int"} else "float")
    return out


def _num_leaf(f: Filter, col: Optional[_NumCol], n: int):
    """x > c etc.: NULL -> UNKNOWN; NaN ordered greatest (DuckDB); an integer column compares exactly against a
    decimal literal (|c| < 1e7: Double.toString prints it plain) and as DOUBLE against a scientific one."""
    c = normalized_value(f)
    t = np.zeros(n, bool)
    fl = np.zeros(n, bool)
    if col is None:
        return t, fl
    exact = col.kind == "int" and abs(c) < 1e7
    for i, x in enumerate(col.vals):
        if x is None:
            continue
        if not exact:
            x = float(x)
        if x != x:
            ok = f.op in (GT, GE)
        elif f.op == GT:
            ok = x > c
        elif f.op == GE:
            ok = x >= c
        elif f.op == LT:
            ok = x < c
        else:
            ok = x <= c
        t[i] = ok
        fl[i] = not ok
    return t, fl


def _leaf(f: Filter, col: Optional[_Col], nonexistent: set, n: int):
    """One filter leaf under SQL three-valued logic -> (is_true, is_false) masks.
    Leaf compile: BaseExpr.scala:461-504; NULL semantics: SURVEY.md Appendix A S7."""
    if f.k in nonexistent:                       # BaseExpr.scala:462-464 -> literal `false`
        return np.zeros(n, bool), np.ones(n, bool)
    if f.op in NUMERIC_OPS:
        return _num_leaf(f, col, n)
    if col is None:                              # absent column referenced only under NOT: all NULL
        codes, dictionary = np.full(n, -1, np.int64), []
    else:
        codes, dictionary = col.codes, col.dictionary
    notnull = codes >= 0
    if f.op in (HAS, EXISTS):                    # IS NOT NULL never yields NULL
        return notnull.copy(), ~notnull
    if f.op == EQ:
        hit = [s == f.v[0] for s in dictionary]
    elif f.op == NOT_EQUALS:
        hit = [s != f.v[0] for s in dictionary]
    elif f.op == IN:
        hit = [s in f.v for s in dictionary]
    elif f.op == NOT_IN:
        hit = [s not in f.v for s in dictionary]
    elif f.op == REGEX:
        hit = [bool(b) for b in re2_search(dictionary, f.v[0])]
    elif f.op == CONTAINS:
        hit = [bool(b) for b in re2_search(dictionary, ".*" + f.v[0] + ".*")]
    else:
        raise NotImplementedError(f.op)
    lut = np.array(list(hit) + [False], dtype=bool)
    h = lut[np.where(notnull, codes, len(hit))]
    return h & notnull, (~h) & notnull


def _eval_filter(q, cols: Dict[str, _Col], nonexistent: set, n: int):
    """Kleene AND/OR/NOT over (is_true, is_false) masks (BaseExpr.scala:505-511)."""
    if isinstance(q, Filter):
        return _leaf(q, cols.get(q.k), nonexistent, n)
    if isinstance(q, NotClause):
        t, f = _eval_filter(q.inner, cols, nonexistent, n)
        return f, t
    t1, f1 = _eval_filter(q.q1, cols, nonexistent, n)
    t2, f2 = _eval_filter(q.q2, cols, nonexistent, n)
    if q.op == "and":
        return t1 & t2, f1 | f2
    return t1 | t2, f1 & f2


def _check_numeric_literals(q, nonexistent: set) -> bool:
    """generateSql's numeric leaves (BaseExpr.scala:450-459): a list of values for a normalized dataType throws for
    every glob; the literal itself (normalizedValue, a lazy def) is computed only for fields that exist -- a bad
    one fails that glob's SQL.  False: the glob's query fails."""
    try:
        for l in _leaves(q):
            if l.op in NUMERIC_OPS:
                if l.dataType in ("duration", "datasize", "number") and len(l.v) != 1:
                    return False
                if l.k not in nonexistent:
                    normalized_value(l)
    except GlobSqlError:
        return False
    return True


def _leaf_columns(q) -> List[str]:
    if isinstance(q, Filter):
        return [q.k]
    if isinstance(q, NotClause):
        return _leaf_columns(q.inner)
    return _leaf_columns(q.q1) + _leaf_columns(q.q2)


@dataclass
class Cell:
    """One (bucket, tags) aggregate cell: raw aggregation state, exact."""
    ts: int
    tags: Dict[str, str]
    rows: int = 0
    count: int = 0
    values: Optional[np.ndarray] = None      # non-null values (for exact sum)
    vmin: float = math.inf
    vmax: float = -math.inf
    gkey: Tuple = ()                          # the SQL group's raw key values (None = NULL), name first

    def agg_value(self, agg: str) -> float:
        """SQL aggregate of the cell, NULL -> 0.0 via JDBC getDouble (Commons.scala:427)."""
        if agg == COUNT:
            return float(self.count)
        if self.count == 0:
            return 0.0
        if agg == SUM:
            return exact_sum(self.values)
        if agg == MIN:
            return self.vmin
        if agg == MAX:
            return self.vmax
        if agg == AVG:
            return exact_sum(self.values) / self.count
        raise NotImplementedError(agg)


def exact_sum(v: np.ndarray) -> float:
    """Correctly rounded sum; NaN/Inf follow IEEE."""
    if v is None or len(v) == 0:
        return 0.0
    if not np.all(np.isfinite(v)):
        return float(np.sum(v))
    return math.fsum(v.tolist())


def evaluate_glob(pr: PushDownRequest, seg_idx: Sequence[int], paths: Sequence[str], sources=None,
                  only: Optional[Sequence[int]] = None, union: Optional[Sequence[str]] = None):
    """Rows of ONE glob = one DuckDB query (Commons.toGlobResultSet, Commons.scala:200-254, then
    resultSetToSource/toDataPoint 280-341, 399-462).  Returns list of (ts, value, tags) in ascending ts
    order (ties ordered by tags for determinism; the reference's tie order is arbitrary, S17).

    Partial evaluation (the sharded protocol's decomposition, checked by tests/test_dist_cpu.py): `only`
    = positions within the glob whose files are read here; `union` = the glob's column union agreed over
    every shard.  Window and step still come from the whole glob."""
    be = pr.baseExpr
    chart = be.chart
    segs = [pr.segmentRequests[i] for i in seg_idx]
    vcol = value_column(be)
    # metrics `ces`: `SELECT ts, 1.0 as value, name, <groupBys> ... WHERE <filter>` reads no rollup column
    # (BaseExpr.scala:385-388)
    no_value = be.dataset == METRICS and is_ces(be)
    fs = field_set(be)
    numcols = sorted({l.k for l in _leaves(be.filter) if l.op in NUMERIC_OPS})
    strings = sorted((set(_leaf_columns(be.filter)) - set(numcols)) | set(chart.groupBys) | {NAME})
    if only is not None:
        paths = [paths[j] for j in only]
        sources = None if sources is None else [sources[j] for j in only]
    try:
        read_union, nums, strs = _read_glob(paths, [TIMESTAMP] + ([] if no_value else [vcol]), strings, sources)
        strs.update(_read_numeric(paths, [c for c in numcols if c in read_union], sources))
    except Exception:   # missing / unreadable file, a column DuckDB cannot bind: that glob alone is empty
        return []       # (Commons.scala:249-253: any exception -> (null, null, null) -> Source.empty)
    union = list(union) if union is not None else read_union
    nonexistent = fs - set(union)                                   # Commons.scala:224
    if not _check_numeric_literals(be.filter, nonexistent):
        return []
    # Columns the generated SQL references but that no file of the glob has: DuckDB raises a Binder
    # Error, which Commons.toGlobResultSet turns into an empty result (Commons.scala:249-253).  This
    # happens for a field used only under `not` (not in fieldSet), and for ts/name/value columns.
    referenced = (set(_leaf_columns(be.filter)) - nonexistent) | {TIMESTAMP, NAME} | (set() if no_value else {vcol})
    if not referenced <= set(union):
        return []
    start = min(s.startTs for s in segs)                            # Commons.scala:225-226
    end = max(s.endTs for s in segs)
    step = segs[0].stepInMillis                                     # Commons.scala:232 (glob head)
    ts, ts_valid = nums[TIMESTAMP]
    ts = ts.astype(np.int64)
    n = len(ts)
    win = ts_valid & (ts >= start) & (ts < end)                     # BaseExpr.scala:159-161
    try:
        t, _ = _eval_filter(be.filter, strs, nonexistent, n)
    except GlobSqlError:   # a regex RE2 rejects, on a field the glob has: the glob's SQL fails
        return []
    keep = win & t
    if be.dataset == METRICS:
        bucket = ts                                                  # BaseExpr.scala:391-394
    else:
        bucket = ts - np.fmod(ts, step)                              # BaseExpr.scala:163-165 (fmod)
    gcols = [g for g in chart.groupBys if g not in nonexistent]      # BaseExpr.scala:338-346 (S12)
    keycols = [("name", strs[NAME])] + [(g, strs[g]) for g in gcols]
    vals, vvalid = (np.zeros(n), np.zeros(n, dtype=bool)) if no_value else nums[vcol]
    idx = np.nonzero(keep)[0]
    if len(idx) == 0:
        return []
    key = np.stack([bucket[idx]] + [c.codes[idx] for _, c in keycols], axis=1)
    order = np.lexsort(key.T[::-1])
    key = key[order]
    idx = idx[order]
    brk = np.nonzero(np.any(key[1:] != key[:-1], axis=1))[0] + 1
    starts = np.concatenate([[0], brk])
    ends = np.concatenate([brk, [len(idx)]])
    qtags = {k: (v if isinstance(v, str) else str(v)) for k, v in segs[0].queryTags.items()}
    out = []
    for s, e in zip(starts, ends):
        rows = idx[s:e]
        ok = vvalid[rows]
        v = vals[rows][ok].astype(np.float64)
        cell = Cell(ts=int(key[s, 0]), tags={}, rows=len(rows), count=int(ok.sum()), values=v)
        if len(v):
            cell.vmin = float(_sql_min(v))
            cell.vmax = float(_sql_max(v))
        cell.gkey = tuple(c.dictionary[key[s, j + 1]] if key[s, j + 1] >= 0 else None
                          for j, (_, c) in enumerate(keycols))
        tags = {}
        for j, (name, c) in enumerate(keycols):
            code = key[s, j + 1]
            if code >= 0:
                sv = c.dictionary[code]
                if sv is not None and sv != "null" and sv != "":   # Commons.scala:433 (S15)
                    tags[name] = sv
        if not tags:
            tags = dict(qtags)                                        # Commons.scala:450-452
        cell.tags = tags
        out.append(cell)
    std = chart.aggregation in (SUM, MIN, MAX, COUNT, AVG) and not is_ces(be)
    out.sort(key=lambda c: (c.ts, sorted(c.tags.items()), c.agg_value(chart.aggregation) if std else 0.0))
    return out


def _sql_min(v):
    """DuckDB orders NaN above every other double: min ignores NaN unless all are NaN."""
    nn = v[~np.isnan(v)]
    return np.min(nn) if len(nn) else np.nan


def _sql_max(v):
    return np.nan if np.any(np.isnan(v)) else np.max(v)


def globs_of(pr: PushDownRequest, glob_size: int) -> List[List[int]]:
    """Segments chunked in request order (Commons.scala:361-366)."""
    n = len(pr.segmentRequests)
    return [list(range(i, min(n, i + glob_size))) for i in range(0, n, glob_size)]


def evaluate_glob_cells(pr: PushDownRequest, glob_size: int, paths: Sequence[str], sources=None):
    """Cells (with their raw non-NULL values) of every glob."""
    check_hot_path(pr)
    out = []
    for g in globs_of(pr, glob_size):
        out.append(evaluate_glob(pr, g, [paths[i] for i in g], None if sources is None else [sources[i] for i in g]))
    return out


def evaluate_per_glob(pr: PushDownRequest, paths: Sequence[str], glob_size: int = 10, sources=None):
    """Worker level (S17): list over globs of the glob's rows [(ts, value, tags)]."""
    agg = pr.baseExpr.chart.aggregation
    return [[(c.ts, c.agg_value(agg), c.tags) for c in cells]
            for cells in evaluate_glob_cells(pr, glob_size, paths, sources)]


def java_min(a: float, b: float) -> float:
    """Scala math.min = java.lang.Math.min (TimeGroupedSketchAggregator.scala:79-83): NaN if either is NaN,
    -0.0 below +0.0."""
    if a != a or b != b:
        return math.nan
    if a == 0.0 and b == 0.0:
        return -0.0 if (math.copysign(1, a) < 0 or math.copysign(1, b) < 0) else 0.0
    return a if a < b else b


def java_max(a: float, b: float) -> float:
    """Scala math.max = java.lang.Math.max (TimeGroupedSketchAggregator.scala:84-88)."""
    if a != a or b != b:
        return math.nan
    if a == 0.0 and b == 0.0:
        return 0.0 if (math.copysign(1, a) > 0 or math.copysign(1, b) > 0) else -0.0
    return a if a > b else b


def merge_glob_cells(pr: PushDownRequest, glob_cells) -> List[Tuple[int, float, Dict[str, str]]]:
    """query-api merge (S19): TimeGroupedSketchAggregator (TimeGroupedSketchAggregator.scala:57-114,
    148-170).  Cells merge by exact timestamp; with groupBys by the full tag map, otherwise all cells of a
    timestamp merge into one.  sum/count add, min/max by min/max of the per-glob values (a glob cell whose
    values are all NULL contributes its JDBC 0.0, Commons.scala:427).

    Order-dependent details of the reference are pinned to a deterministic choice:
      * sums: the correctly rounded sum of every underlying value (the reference adds per-glob DuckDB sums
        in arrival order; SURVEY.md Appendix A S14 makes the correctly rounded sum the parity target);
      * without groupBys the merged row takes "the first input's" tags (TimeGroupedSketchAggregator.scala:
        57-60, arrival order); we take the smallest tag map."""
    agg = pr.baseExpr.chart.aggregation
    # AVG: query-api sends SUM and COUNT pushdowns (QueryEngineV2.scala:280-283); their rows merge per
    # (timestamp, tags) into one {sum, count} map (TimeGroupedSketchAggregator.scala:74-78) and the value is
    # sum / count (BaseExpr.scala:88-91; 0/0 = NaN).
    has_gb = bool(pr.baseExpr.chart.groupBys)
    merged: Dict[Any, list] = {}
    for cells in glob_cells:
        for c in cells:
            k = (c.ts, tuple(sorted(c.tags.items()))) if has_gb else c.ts
            merged.setdefault(k, []).append(c)
    out = []
    for k, cs in merged.items():
        tags = min((c.tags for c in cs), key=lambda t: sorted(t.items()))
        if agg == SUM:
            val = exact_sum(np.concatenate([c.values for c in cs]))
        elif agg == COUNT:
            val = float(sum(c.count for c in cs))
        elif agg == AVG:
            n = sum(c.count for c in cs)
            s = exact_sum(np.concatenate([c.values for c in cs]))
            val = s / n if n else math.nan
        elif agg == MIN:
            val = functools.reduce(java_min, (c.agg_value(MIN) for c in cs))
        else:
            val = functools.reduce(java_max, (c.agg_value(MAX) for c in cs))
        out.append((cs[0].ts, val, tags))
    out.sort(key=lambda r: (r[0], sorted(r[2].items()), r[1]))
    return out


def merge_partial_cells(parts) -> list:
    """Fold one glob's partial cells from several shards (lists of Cell) into the glob's cells: cells of the
    same SQL group (bucket, raw key values) add rows/counts/values and take min/max, exactly as rank 0's
    table merge does (lakeside_amd/csrc/kernels.hip merge_tables)."""
    merged: Dict[Any, Cell] = {}
    for cells in parts:
        for c in cells:
            k = (c.ts, c.gkey)
            m = merged.get(k)
            if m is None:
                merged[k] = Cell(ts=c.ts, tags=dict(c.tags), rows=c.rows, count=c.count,
                                 values=np.array(c.values, dtype=np.float64), vmin=c.vmin, vmax=c.vmax, gkey=c.gkey)
                continue
            m.rows += c.rows
            m.count += c.count
            m.values = np.concatenate([m.values, c.values])
            if m.count:
                m.vmin = float(_sql_min(m.values))
                m.vmax = float(_sql_max(m.values))
    return list(merged.values())


def evaluate_merged(pr: PushDownRequest, paths: Sequence[str], glob_size: int = 10, sources=None):
    return merge_glob_cells(pr, evaluate_glob_cells(pr, glob_size, paths, sources))


# ----------------------------------------------------------------------------------------------
# Tag queries (isTagQuery + tagDataType): BaseExpr.generateSql tag branch (BaseExpr.scala:127-143)
# ----------------------------------------------------------------------------------------------
# NoisyTagsDropper (core/src/main/scala/com/cardinal/utils/NoisyTagsDropper.scala): hidden tag names / prefixes
NOISY_TAGS = {"day", "month", "hour", "minute", "year", "sketch", "_cardinalhq.tid", "_cardinalhq.would_filter",
              "_cardinalhq.trace_has_error", "_cardinalhq.id", "_cardinalhq.telemetry_type", "_cardinalhq.filtered",
              "_cardinalhq.is_root_span", "_cardinalhq.positive_counts", "_cardinalhq.negative_counts",
              "metric.stepTs", "metric.tagName", "metric.metrics_type", "scope.telemetry.sdk.name", "metric.filter",
              "metric.dd.israte", "metric.dd.rateinterval"}


def noisy_tag(name: str) -> bool:
    return name in NOISY_TAGS or name.startswith("rollup_")


def tag_row_tags(tag: str, value: Optional[str], count: int) -> Dict[str, str]:
    """Commons.toDataPoint's tag branch (Commons.scala:406-423): every column becomes a tag, then
    NoisyTagsDropper.remove drops hidden names and NULL / "" / "null" values."""
    tags = {"count": str(count)}
    if value is not None and value != "" and value != "null" and not noisy_tag(tag):
        tags[tag] = value
    return tags


def parse_tag_data_type(text: str) -> Optional[str]:
    """PushDownRequest.fromJson's tagDataType (SegmentRequest.scala:55-58) -> tagName (None: no tag query)."""
    p = json.loads(text)
    td = p.get("tagDataType")
    return td.get("tagName") if p.get("isTagQuery") and isinstance(td, dict) else None


def evaluate_tag_glob(pr: PushDownRequest, tag: str, seg_idx: Sequence[int], paths: Sequence[str], sources=None):
    """One glob of a tag query:  SELECT "<tag>", COUNT(*) AS count FROM {table} WHERE <filter> AND <window>
    GROUP BY "<tag>"  (BaseExpr.scala:127-143; the filter/nonExistentFields compile as for charts, 170-180).
    Returns [(raw tag value or None, COUNT(*))] sorted by value (None first); the SQL has no ORDER BY."""
    be = pr.baseExpr
    if any(f.extracted or f.computed for f in _leaves(be.filter)):
        raise NotImplementedError("synthetic (extracted/computed) tag queries are outside the hot path")
    segs = [pr.segmentRequests[i] for i in seg_idx]
    fs = filter_field_set(be.filter) | set(be.chart.groupBys if be.chart else [])
    numcols = sorted({l.k for l in _leaves(be.filter) if l.op in NUMERIC_OPS})
    strings = sorted((set(_leaf_columns(be.filter)) - set(numcols)) | {tag})
    try:
        union, nums, strs = _read_glob(paths, [TIMESTAMP], strings, sources, numeric_tags=[tag])
        strs.update(_read_numeric(paths, [c for c in numcols if c in union], sources))
    except NotImplementedError:
        raise
    except Exception:   # Commons.scala:249-253: the glob's query fails -> empty
        return []
    nonexistent = fs - set(union)
    if not _check_numeric_literals(be.filter, nonexistent):
        return []
    referenced = (set(_leaf_columns(be.filter)) - nonexistent) | {TIMESTAMP, tag}
    if not referenced <= set(union):                                  # Binder Error -> empty glob
        return []
    start = min(s.startTs for s in segs)
    end = max(s.endTs for s in segs)
    ts, ts_valid = nums[TIMESTAMP]
    ts = ts.astype(np.int64)
    n = len(ts)
    try:
        t, _ = _eval_filter(be.filter, strs, nonexistent, n)
    except GlobSqlError:   # a regex RE2 rejects, on a field the glob has: the glob's SQL fails
        return []
    keep = ts_valid & (ts >= start) & (ts < end) & t
    col = strs[tag]
    codes = col.codes[keep]
    if len(codes) == 0:
        return []
    u, cnt = np.unique(codes, return_counts=True)
    out = [(col.dictionary[c] if c >= 0 else None, int(k)) for c, k in zip(u, cnt)]
    out.sort(key=lambda r: (r[0] is not None, r[0] or ""))
    return out


def _leaves(q):
    if isinstance(q, Filter):
        return [q]
    if isinstance(q, NotClause):
        return _leaves(q.inner)
    return _leaves(q.q1) + _leaves(q.q2)


def evaluate_tag_per_glob(pr: PushDownRequest, tag: str, paths: Sequence[str], glob_size: int = 10, sources=None):
    """Worker rows of a tag query per glob: [[tags map]] (values: the DataPoint tags; timestamp =
    System.currentTimeMillis() and value 0.0 in the reference, not compared)."""
    out = []
    for g in globs_of(pr, glob_size):
        rows = evaluate_tag_glob(pr, tag, g, [paths[i] for i in g], None if sources is None else [sources[i] for i in g])
        out.append([tag_row_tags(tag, v, c) for v, c in rows])
    return out


def evaluate_tag_merged(pr: PushDownRequest, tag: str, paths: Sequence[str], glob_size: int = 10, sources=None):
    """Counts summed per tag value over the globs (the engine's LK_MERGED for tag queries; query-api streams the
    per-glob rows unmerged, its TagQueryUtils.aggregate is commented out, QueryEngineV2.scala:487).  NULL, "" and
    "null" give the same tag map and merge into one row."""
    acc: Dict[Optional[str], int] = {}
    for g in globs_of(pr, glob_size):
        for v, c in evaluate_tag_glob(pr, tag, g, [paths[i] for i in g], None if sources is None else [sources[i] for i in g]):
            k = None if (v is None or v == "" or v == "null") else v
            acc[k] = acc.get(k, 0) + c
    return [tag_row_tags(tag, v, c) for v, c in sorted(acc.items(), key=lambda r: (r[0] is not None, r[0] or ""))]


def rows_to_jsonable(rows):
    return [[int(ts), float(v).hex(), dict(sorted(tags.items()))] for ts, v, tags in rows]


# ----------------------------------------------------------------------------------------------
# query-api final evaluation of merged rows (§8(f) f1)
# ----------------------------------------------------------------------------------------------
def clause_label(q) -> str:
    """QueryClause.toString (ASTUtils.scala:102-122)."""
    if isinstance(q, Filter):
        sym = {EQ: "=", GT: ">", GE: ">=", LT: "<", LE: "<="}
        if q.op in sym:
            return f"{q.k} {sym[q.op]} {q.v[0]}"
        if q.op == REGEX:
            return f"regexMatches({q.k}, {q.v[0]})"
        if q.op == CONTAINS:
            return f"{q.k} contains {q.v[0]}"
        if q.op == IN:
            return f"{q.k} in ({', '.join(q.v)})"
        return ""
    if isinstance(q, BinaryClause):
        return f"({clause_label(q.q1)} {q.op} {clause_label(q.q2)})"
    return f"not({clause_label(q.inner)})"


def _jvm_div(a: float, b: float) -> float:
    """Double division as on the JVM (IEEE: x/0 = +-Infinity, 0/0 = NaN)."""
    if b != 0:
        return a / b
    if a != a or a == 0:
        return math.nan
    return math.copysign(math.inf, a) * math.copysign(1.0, b)


def final_eval(base_expr: dict, merged_rows, step_ms: int, now_ms: int) -> List[dict]:
    """Merged rows (S19) -> timeseries payloads:
      * drop ts > now (TimeGroupedSketchAggregator.scala:204-207);
      * value = transformer(map[agg]) (BaseExpr.scala:677-687; ASTUtils.getTransformerFunc 190-219, step in
        whole seconds = stepInMillis / 1000 on Longs; MetricType "count"/"counter" -> COUNTER,
        MetricType.scala:65-73, Commons.scala:49-52);
      * results of one timestamp keyed by toGroupByKey (ASTUtils.scala:87-89) or "default"
        (BaseExpr.scala:689-690), a later row overwriting an earlier one; the reference's order is a hash
        map's, here the smallest sorted tag list wins;
      * label: BaseExpr.label (BaseExpr.scala:697-716); payload: QueryEngineV2.toGenericSSEPayload (400-417)."""
    be = to_base_expr(base_expr)
    ctype = (be.chart.type if be.chart.type is not None else "count").lower().strip()
    mtype = (base_expr.get("metricType") or "gauge").lower().strip()
    secs = float(int(step_ms) // 1000)

    def transform(v: float) -> float:
        if be.dataset == METRICS:
            if ctype == "count" and mtype == "rate":
                return v * secs
            if ctype == "rate" and mtype in ("count", "counter"):
                return _jvm_div(v, secs)
            return v
        return _jvm_div(v, secs) if ctype == "rate" else v

    keys = sorted(set(be.chart.groupBys))
    by_ts: Dict[int, list] = {}
    for ts, v, tags in merged_rows:
        if ts > now_ms:
            continue
        by_ts.setdefault(int(ts), []).append((float(v), dict(tags)))
    out = []
    for ts in sorted(by_ts):
        chosen = {}
        for v, tags in sorted(by_ts[ts], key=lambda x: sorted(x[1].items()), reverse=True):
            gk = ":".join(str(tags.get(k, "")) for k in keys) if keys else "default"
            chosen[gk] = (v, tags)
        for gk in sorted(chosen):
            v, tags = chosen[gk]
            if keys:
                lab = "(" + ", ".join(f"{k} = {tags[k]}" for k in keys if k in tags) + ")"
            else:
                lab = "(" + clause_label(be.filter) + ")"
            out.append({"id": base_expr.get("id", "_"), "type": "timeseries",
                        "message": {"timestamp": ts, "tags": tags, "value": transform(v), "label": lab}})
    return out


# ----------------------------------------------------------------------------------------------
# Percentiles: DDSketch per (step, group-key tags)
# ----------------------------------------------------------------------------------------------
def is_percentile(agg: Optional[str]) -> bool:
    return agg is not None and len(agg) > 1 and agg[0] == "p"


def _key_tags(pr: PushDownRequest, tags: Dict[str, str]) -> Dict[str, str]:
    """PushDownAggregatorStage.getGroupByKeyTags (PushDownAggregatorStage.scala:188-197) over the DataPoint's tags
    (Commons.toDataPoint: NULL / "null" / "" dropped, Commons.scala:433).  Without groupBys it reads
    `tags.getOrElse(NAME, "")` with NAME = "_cardinalhq.name" (Commons.scala:45), while the row's name tag is labelled
    `name` (the SQL's `"_cardinalhq.name" as name`, BaseExpr.scala:397-399): the key tags are {"_cardinalhq.name": ""}
    for every row -- one sketch per step."""
    gbs = pr.baseExpr.chart.groupBys
    if not gbs:
        return {NAME: tags.get(NAME, "")}
    return {g: tags[g] for g in gbs if g in tags}


def evaluate_percentile_per_glob(pr: PushDownRequest, glob_size: int, paths: Sequence[str], sources=None):
    """Per glob: [(ts, key tags, Sketch)] ascending in ts (ties: sorted tags).  The worker's SQL returns the passing
    rows (BaseExpr.scala:397-399); each row's value (NULL -> 0.0, JDBC getDouble) goes into the sketch of its
    (ts - ts % step, key tags) (PushDownAggregatorStage.scala:56-60, 69-81).  Metrics: the SQL returns one row per
    (raw ts, groupBys, name) with MAX(rollup_<r>) (BaseExpr.scala:379-383), whose value (NULL -> 0.0) goes into the
    sketch of its (raw ts, key tags) -- moduloTs is the raw timestamp for metrics (PushDownAggregatorStage.scala:
    56-60)."""
    from oracle import ddsketch
    check_hot_path(pr)
    out = []
    for g in globs_of(pr, glob_size):
        cells = evaluate_glob(pr, g, [paths[i] for i in g], None if sources is None else [sources[i] for i in g])
        acc: Dict[Tuple, Tuple[Dict[str, str], Any]] = {}
        for c in cells:
            kt = _key_tags(pr, c.tags)
            if pr.baseExpr.dataset == METRICS:
                vals = np.array([c.agg_value(MAX)])
            else:
                vals = np.concatenate([c.values, np.zeros(c.rows - c.count)])
            sk = ddsketch.Sketch().accept_all(vals)
            key = (c.ts, tuple(sorted(kt.items())))
            if key in acc:
                acc[key][1].merge(sk)
            else:
                acc[key] = (kt, sk)
        out.append([(k[0], acc[k][0], acc[k][1]) for k in sorted(acc)])
    return out


def merge_percentile(pr: PushDownRequest, per_glob) -> List[Tuple[int, Dict[str, str], Any]]:
    """query-api merge of DD sketches (TimeGroupedSketchAggregator.scala:34-37, 101-114): per (timestamp, tags) (without
    groupBys every key-tag map is {"_cardinalhq.name": ""}: one sketch per timestamp)."""
    from oracle import ddsketch
    acc: Dict[Tuple, Tuple[Dict[str, str], Any]] = {}
    for rows in per_glob:
        for ts, kt, sk in rows:
            key = (ts, tuple(sorted(kt.items())))
            if key not in acc:
                acc[key] = (dict(kt), ddsketch.Sketch().merge(sk))
            else:
                acc[key][1].merge(sk)
    return [(k[0], acc[k][0], acc[k][1]) for k in sorted(acc)]


# ----------------------------------------------------------------------------------------------
# Cardinality estimates (`ces`): one HLL per step over the group-key strings
# ----------------------------------------------------------------------------------------------
def is_ces(be: BaseExpr) -> bool:
    """`ces` as the aggregation, or (logs / traces) in the rollup; a metrics rollup of "ces" under another
    aggregation stays that aggregation over the rollup_ces column (BaseExpr.scala:376-395)."""
    c = be.chart
    return c is not None and (c.aggregation == "ces" or ("ces" in (c.rollup or "") and be.dataset != METRICS))


def evaluate_ces_per_glob(pr: PushDownRequest, glob_size: int, paths: Sequence[str], sources=None):
    """Per glob: [(ts, key set)] ascending in ts.  Each passing row feeds its step's HLL the string
    groupBys.map(g => tags.getOrElse(g, "")).mkString(":") (Aggregator.scala:53-56; tags after toDataPoint's
    NULL / "null" / "" drop, Commons.scala:433).  The set of strings determines the HLL state."""
    gbs = pr.baseExpr.chart.groupBys
    out = []
    for g in globs_of(pr, glob_size):
        cells = evaluate_glob(pr, g, [paths[i] for i in g], None if sources is None else [sources[i] for i in g])
        acc: Dict[int, set] = {}
        for c in cells:
            acc.setdefault(c.ts, set()).add(":".join(c.tags.get(x, "") for x in gbs))
        out.append([(ts, acc[ts]) for ts in sorted(acc)])
    return out


def merge_ces(per_glob) -> List[Tuple[int, set]]:
    """query-api: HLL union per timestamp (TimeGroupedSketchAggregator.scala:38-43) = the union of the key sets."""
    acc: Dict[int, set] = {}
    for rows in per_glob:
        for ts, ks in rows:
            acc.setdefault(ts, set()).update(ks)
    return [(ts, acc[ts]) for ts in sorted(acc)]
