"""ctypes wrapper of oracle/liblkcpu.so: the multi-core C++ restatement of the evaluator (TEST INFRASTRUCTURE ONLY).

Same contract as oracle/dataexpr.py (per-glob rows at the worker, S17; merged rows at query-api, S19), computed by
oracle/cpu/lkcpu.cpp over in-memory Parquet bytes on every host core.  Used by bench.py (timed CPU baseline,
full-size validation of the GPU rows) and checked against oracle/dataexpr.py in tests/test_oracle_cpu.py.
Only tests/, bench.py and __graft_entry__.smoke() may import it; the product path never does.
"""
import ctypes
import math
import os
import time
from typing import Dict, List, Optional, Sequence, Tuple
from urllib.parse import quote

import numpy as np

from . import dataexpr as dx

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "liblkcpu.so")
_L = None


def lib():
    global _L
    if _L is None:
        L = ctypes.CDLL(LIB)
        L.lkcpu_eval.restype = ctypes.c_void_p
        L.lkcpu_eval.argtypes = [ctypes.c_char_p, ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_size_t),
                                 ctypes.c_size_t, ctypes.c_int]
        L.lkcpu_error.restype = ctypes.c_char_p
        L.lkcpu_ncells.restype = ctypes.c_size_t
        L.lkcpu_ncells.argtypes = [ctypes.c_void_p]
        L.lkcpu_ncols.restype = ctypes.c_int
        L.lkcpu_ncols.argtypes = [ctypes.c_void_p]
        L.lkcpu_cells.argtypes = [ctypes.c_void_p] + [ctypes.c_void_p] * 10
        L.lkcpu_key_string.restype = ctypes.c_char_p
        L.lkcpu_key_string.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int32]
        L.lkcpu_free.argtypes = [ctypes.c_void_p]
        _L = L
    return _L


def _leaves(q, out):
    if isinstance(q, dx.Filter):
        out.append(q)
    elif isinstance(q, dx.NotClause):
        _leaves(q.inner, out)
    else:
        _leaves(q.q1, out)
        _leaves(q.q2, out)
    return out


def _postfix(q, leaves, out):
    if isinstance(q, dx.Filter):
        out.append(next(i for i, l in enumerate(leaves) if l is q))
    elif isinstance(q, dx.NotClause):
        _postfix(q.inner, leaves, out)
        out.append(-3)
    else:
        _postfix(q.q1, leaves, out)
        _postfix(q.q2, leaves, out)
        out.append(-1 if q.op == "and" else -2)
    return out


def plan_text(pr: dx.PushDownRequest, glob_size: int) -> Tuple[str, List[str], List[str]]:
    """Flatten the parsed request into lkcpu's line format; returns (text, string columns, groupBys)."""
    be = pr.baseExpr
    dx.check_hot_path(pr)
    leaves = _leaves(be.filter, [])
    vcol = dx.value_column(be)
    strcols = [dx.NAME]
    for l in leaves:
        if l.op in dx.NUMERIC_OPS:   # numeric comparison leaves: on the value column only (BaseExpr.scala:488-498)
            if l.k != vcol:
                raise NotImplementedError("lkcpu: numeric comparison leaves on a column other than the value column")
            continue
        if l.k not in strcols:
            strcols.append(l.k)
    gbs = []
    for g in be.chart.groupBys:
        if g not in gbs:
            gbs.append(g)
    for g in gbs:
        if g not in strcols:
            strcols.append(g)
    if len(strcols) > 7:
        raise NotImplementedError("lkcpu: at most 7 string columns")
    t = ["metrics" if be.dataset == dx.METRICS else be.dataset, be.chart.aggregation, dx.value_column(be),
         str(glob_size), str(len(pr.segmentRequests))]
    for s in pr.segmentRequests:
        t += [str(s.startTs), str(s.endTs), str(s.stepInMillis)]
    t += [str(len(strcols))] + strcols
    t += [str(len(gbs))] + [str(strcols.index(g)) for g in gbs]
    t += [str(len(leaves))]
    for l in leaves:
        if l.op in dx.NUMERIC_OPS:   # column -1 = the value column; the literal normalized (BaseExpr.scala:450-459)
            t += ["-1", l.op, "1", repr(dx.normalized_value(l))]
        else:
            t += [str(strcols.index(l.k)), l.op, str(len(l.v))] + list(l.v)
    prog = _postfix(be.filter, leaves, [])
    t += [str(len(prog))] + [str(x) for x in prog]
    fs = sorted(dx.field_set(be))
    t += [str(len(fs))] + fs
    return "\n".join(quote(x, safe="") for x in t) + "\n", strcols, gbs


def plan_text_tag(pr: dx.PushDownRequest, tag: str, glob_size: int) -> str:
    """A tag query (isTagQuery + tagDataType, BaseExpr.scala:127-143) in lkcpu's line format: the tag is string column
    0 and the only key; rows are counted (COUNT(*), NULL values included) in one bucket."""
    leaves = _leaves(pr.baseExpr.filter, []) if pr.baseExpr.filter is not None else []
    strcols = [tag]
    for l in leaves:
        if l.op in dx.NUMERIC_OPS:
            raise NotImplementedError("lkcpu: numeric leaves in a tag query")
        if l.k not in strcols:
            strcols.append(l.k)
    if len(strcols) > 7:
        raise NotImplementedError("lkcpu: at most 7 string columns")
    t = ["tag", "count", dx.VALUE, str(glob_size), str(len(pr.segmentRequests))]
    for s in pr.segmentRequests:
        t += [str(s.startTs), str(s.endTs), str(s.stepInMillis)]
    t += [str(len(strcols))] + strcols + ["0"]
    t += [str(len(leaves))]
    for l in leaves:
        t += [str(strcols.index(l.k)), l.op, str(len(l.v))] + list(l.v)
    prog = _postfix(pr.baseExpr.filter, leaves, []) if leaves else []
    t += [str(len(prog))] + [str(x) for x in prog]
    fs = sorted(dx.field_set(pr.baseExpr))
    t += [str(len(fs))] + fs
    return "\n".join(quote(x, safe="") for x in t) + "\n"


def evaluate_tag_counts(pr: dx.PushDownRequest, tag: str, glob_size: int, blobs: Sequence, threads: int = 0,
                        timing: Optional[list] = None) -> Dict[Optional[str], int]:
    """Tag query counts merged over the globs (the engine's LK_MERGED tag table, oracle/dataexpr.evaluate_tag_merged):
    {tag text (None: NULL / "" / "null") -> COUNT(*)}."""
    text = plan_text_tag(pr, tag, glob_size)
    n = len(blobs)
    ptrs = (ctypes.c_void_p * max(1, n))()
    sizes = (ctypes.c_size_t * max(1, n))()
    keep = []
    for i, b in enumerate(blobs):
        if isinstance(b, (bytes, bytearray)):
            buf = ctypes.create_string_buffer(bytes(b), len(b))
            keep.append(buf)
            ptrs[i], sizes[i] = ctypes.cast(buf, ctypes.c_void_p), len(b)
        else:
            ptrs[i], sizes[i] = ctypes.cast(b[0], ctypes.c_void_p), b[1]
    L = lib()
    t0 = time.perf_counter()
    h = L.lkcpu_eval(text.encode(), ptrs, sizes, n, threads)
    if timing is not None:
        timing.append(time.perf_counter() - t0)
    if not h:
        raise RuntimeError(L.lkcpu_error().decode())
    try:
        m = L.lkcpu_ncells(h)
        nc = L.lkcpu_ncols(h)
        arrs = [np.zeros(m, t) for t in (np.int32, np.int64, np.uint64, np.uint64, np.float64, np.float64, np.float64,
                                          np.float64, np.uint8)]
        keys = np.zeros(max(1, m * nc), np.int32)
        L.lkcpu_cells(h, *[a.ctypes.data for a in arrs + [keys]])
        rows = arrs[2]
        out: Dict[Optional[str], int] = {}
        for i in range(m):
            kid = int(keys[i * nc])
            v = L.lkcpu_key_string(h, 0, kid) if kid >= 0 else None
            s = None if v is None or v in (b"", b"null") else v.decode()
            out[s] = out.get(s, 0) + int(rows[i])
        return out
    finally:
        L.lkcpu_free(h)


def plan_text_exemplar(pr: dx.PushDownRequest, glob_size: int) -> str:
    """An exemplar request (no chart, BaseExpr.scala:206-239) in lkcpu's line format: the filter's string columns,
    no group keys."""
    be = pr.baseExpr
    leaves = _leaves(be.filter, []) if be.filter is not None else []
    strcols = [dx.NAME]
    for l in leaves:
        if l.op in dx.NUMERIC_OPS:
            raise NotImplementedError("lkcpu exemplar: numeric leaves")
        if l.k not in strcols:
            strcols.append(l.k)
    t = [be.dataset, "sum", dx.VALUE, str(glob_size), str(len(pr.segmentRequests))]
    for s in pr.segmentRequests:
        t += [str(s.startTs), str(s.endTs), str(s.stepInMillis)]
    t += [str(len(strcols))] + strcols + ["0"]
    t += [str(len(leaves))]
    for l in leaves:
        t += [str(strcols.index(l.k)), l.op, str(len(l.v))] + list(l.v)
    prog = _postfix(be.filter, leaves, []) if leaves else []
    t += [str(len(prog))] + [str(x) for x in prog]
    fs = sorted(dx.field_set(be))
    t += [str(len(fs))] + fs
    return "\n".join(quote(x, safe="") for x in t) + "\n"


def evaluate_exemplar_rows(pr: dx.PushDownRequest, glob_size: int, blobs: Sequence, threads: int = 0,
                           timing: Optional[list] = None):
    """The worker's exemplar stream (per glob ORDER BY ts LIMIT n, globs folded by mergeSorted) from the C++
    restatement: [(ts, value, canonical tag key, glob)] in stream order."""
    text = plan_text_exemplar(pr, glob_size)
    n = len(blobs)
    ptrs = (ctypes.c_void_p * max(1, n))()
    sizes = (ctypes.c_size_t * max(1, n))()
    keep = []
    for i, b in enumerate(blobs):
        if isinstance(b, (bytes, bytearray)):
            buf = ctypes.create_string_buffer(bytes(b), len(b))
            keep.append(buf)
            ptrs[i], sizes[i] = ctypes.cast(buf, ctypes.c_void_p), len(b)
        else:
            ptrs[i], sizes[i] = ctypes.cast(b[0], ctypes.c_void_p), b[1]
    L = lib()
    if not getattr(L, "_ex_bound", False):
        L.lkcpu_exemplar.restype = ctypes.c_void_p
        L.lkcpu_exemplar.argtypes = [ctypes.c_char_p, ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_size_t),
                                     ctypes.c_size_t, ctypes.c_int, ctypes.c_int64, ctypes.c_int, ctypes.c_int]
        L.lkcpu_ex_rows.restype = ctypes.c_size_t
        L.lkcpu_ex_rows.argtypes = [ctypes.c_void_p]
        L.lkcpu_ex_row.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.POINTER(ctypes.c_int64),
                                   ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_int32)]
        L.lkcpu_ex_tags.restype = ctypes.c_char_p
        L.lkcpu_ex_tags.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
        L.lkcpu_ex_free.argtypes = [ctypes.c_void_p]
        L._ex_bound = True
    be = pr.baseExpr
    t0 = time.perf_counter()
    h = L.lkcpu_exemplar(text.encode(), ptrs, sizes, n, threads, int(be.limit), 1 if be.order.upper() == "DESC" else 0,
                         1 if pr.reverseSort else 0)
    if timing is not None:
        timing.append(time.perf_counter() - t0)
    if not h:
        raise RuntimeError(L.lkcpu_error().decode())
    try:
        out = []
        ts, val, g = ctypes.c_int64(), ctypes.c_double(), ctypes.c_int32()
        for i in range(L.lkcpu_ex_rows(h)):
            L.lkcpu_ex_row(h, i, ctypes.byref(ts), ctypes.byref(val), ctypes.byref(g))
            out.append((ts.value, val.value, L.lkcpu_ex_tags(h, i), g.value))
        return out
    finally:
        L.lkcpu_ex_free(h)


def _dd(*xs):
    """Correctly rounded sum of double-double parts (IEEE propagation for non-finite values)."""
    return math.fsum(xs) if all(math.isfinite(x) for x in xs) else float(np.sum(np.array(xs)))


class CpuCell:
    """One per-glob (bucket, group) cell of the CPU restatement."""
    __slots__ = ("ts", "tags", "rows", "count", "hi", "lo", "vmin", "vmax", "glob")

    def agg_value(self, agg: str) -> float:
        if agg == dx.COUNT:
            return float(self.count)
        if self.count == 0:
            return 0.0
        if agg == dx.SUM:
            return _dd(self.hi, self.lo)
        if agg == dx.AVG:
            return _dd(self.hi, self.lo) / self.count
        return self.vmin if agg == dx.MIN else self.vmax


def evaluate_glob_cells(pr: dx.PushDownRequest, glob_size: int, blobs: Sequence, threads: int = 0):
    """Per-glob cells over in-memory Parquet `blobs` (bytes or (pointer, size)), in request order."""
    text, strcols, gbs = plan_text(pr, glob_size)
    n = len(blobs)
    ptrs = (ctypes.c_void_p * max(1, n))()
    sizes = (ctypes.c_size_t * max(1, n))()
    keep = []
    for i, b in enumerate(blobs):
        if isinstance(b, (bytes, bytearray)):
            buf = ctypes.create_string_buffer(bytes(b), len(b))
            keep.append(buf)
            ptrs[i] = ctypes.cast(buf, ctypes.c_void_p)
            sizes[i] = len(b)
        else:
            ptrs[i] = ctypes.cast(b[0], ctypes.c_void_p)
            sizes[i] = b[1]
    L = lib()
    h = L.lkcpu_eval(text.encode(), ptrs, sizes, n, threads)
    if not h:
        raise RuntimeError(L.lkcpu_error().decode())
    try:
        m = L.lkcpu_ncells(h)
        nc = L.lkcpu_ncols(h)
        glob = np.zeros(m, np.int32)
        ts = np.zeros(m, np.int64)
        rows = np.zeros(m, np.uint64)
        cnt = np.zeros(m, np.uint64)
        hi = np.zeros(m, np.float64)
        lo = np.zeros(m, np.float64)
        mn = np.zeros(m, np.float64)
        mx = np.zeros(m, np.float64)
        nanf = np.zeros(m, np.uint8)
        keys = np.zeros(m * nc, np.int32)
        L.lkcpu_cells(h, *[a.ctypes.data for a in (glob, ts, rows, cnt, hi, lo, mn, mx, nanf, keys)])
        names = ["name"] + gbs
        strings: List[Dict[int, Optional[str]]] = [dict() for _ in range(nc)]

        def key_string(c, i):
            d = strings[c]
            if i not in d:
                v = L.lkcpu_key_string(h, c, int(i))
                d[i] = None if v is None else v.decode()
            return d[i]

        nglobs = (len(pr.segmentRequests) + glob_size - 1) // glob_size
        out = [[] for _ in range(nglobs)]
        globs = dx.globs_of(pr, glob_size)
        qtags = [{k: (v if isinstance(v, str) else str(v)) for k, v in pr.segmentRequests[g[0]].queryTags.items()}
                 for g in globs]
        keys = keys.reshape(m, nc) if m else keys.reshape(0, nc)
        for i in range(m):
            c = CpuCell()
            c.glob = int(glob[i])
            c.ts = int(ts[i])
            c.rows = int(rows[i])
            c.count = int(cnt[i])
            c.hi = float(hi[i])
            c.lo = float(lo[i])
            c.vmin = float(mn[i]) if nanf[i] & 2 else math.nan
            c.vmax = math.nan if nanf[i] & 1 else float(mx[i])
            tags = {}
            for j in range(nc):
                if keys[i, j] < 0:
                    continue
                sv = key_string(j, keys[i, j])
                if sv is not None and sv != "null" and sv != "":   # Commons.scala:433 (S15)
                    tags[names[j]] = sv
            c.tags = tags if tags else dict(qtags[c.glob])          # Commons.scala:450-452
            out[c.glob].append(c)
        for cells in out:
            cells.sort(key=lambda c: (c.ts, sorted(c.tags.items())))
        return out
    finally:
        L.lkcpu_free(h)


def merge_glob_cells(pr: dx.PushDownRequest, glob_cells) -> List[Tuple[int, float, Dict[str, str]]]:
    """query-api merge (S19), as oracle/dataexpr.merge_glob_cells, over the CPU cells."""
    agg = pr.baseExpr.chart.aggregation
    has_gb = bool(pr.baseExpr.chart.groupBys)
    merged: Dict = {}
    for cells in glob_cells:
        for c in cells:
            k = (c.ts, tuple(sorted(c.tags.items()))) if has_gb else c.ts
            merged.setdefault(k, []).append(c)
    out = []
    for k, cs in merged.items():
        tags = min((c.tags for c in cs), key=lambda t: sorted(t.items()))
        if agg == dx.SUM:
            val = _dd(*[x for c in cs for x in (c.hi, c.lo)]) if any(c.count for c in cs) else 0.0
        elif agg == dx.COUNT:
            val = float(sum(c.count for c in cs))
        elif agg == dx.AVG:
            n = sum(c.count for c in cs)
            s = _dd(*[x for c in cs for x in (c.hi, c.lo)])
            val = s / n if n else math.nan
        elif agg == dx.MIN:
            val = min(c.agg_value(dx.MIN) for c in cs)
        else:
            val = max(c.agg_value(dx.MAX) for c in cs)
        out.append((cs[0].ts, val, tags))
    out.sort(key=lambda r: (r[0], sorted(r[2].items()), r[1]))
    return out


def evaluate_merged(pr: dx.PushDownRequest, blobs: Sequence, glob_size: int = 10, threads: int = 0):
    return merge_glob_cells(pr, evaluate_glob_cells(pr, glob_size, blobs, threads))


# ---------------------------------------------------------------------------------------------------------------
# Columnar form (bench validation at full size: millions of cells, and partial tables of several ranks).  A row's tag
# map is one canonical byte string, `tag_key(tags)`: its items sorted by key, key and value joined by 0x1e, items by
# 0x1f -- equal maps give equal keys, so the query-api merge and the comparison run on numpy arrays.
# ---------------------------------------------------------------------------------------------------------------
def tag_key(tags: Dict[str, str]) -> bytes:
    return "\x1f".join(f"{k}\x1e{v}" for k, v in sorted(tags.items())).encode()


def tags_of_key(key: bytes) -> Dict[str, str]:
    if not key:
        return {}
    return dict(item.split("\x1e", 1) for item in key.decode().split("\x1f"))


def join_tag_columns(names: Sequence[str], cols: Sequence[np.ndarray], fallback: np.ndarray) -> np.ndarray:
    """Per-row canonical tag keys from per-column value arrays (bytes; b"" = the tag is dropped, S15) in any column
    order; rows with no tag left take `fallback` (their queryTags key, Commons.scala:450-452)."""
    order = sorted(range(len(names)), key=lambda c: names[c])
    n = len(fallback)
    out = np.full(n, b"", dtype=object)
    for c in order:
        v = np.asarray(cols[c], dtype=object)
        has = v != b""
        piece = np.full(n, b"", dtype=object)
        if has.any():
            piece[has] = names[c].encode() + b"\x1e" + v[has]
        both = has & (out != b"")
        out[both] = out[both] + b"\x1f"
        out = out + piece
    empty = out == b""
    out[empty] = fallback[empty]
    return out


class CellTable:
    """Per-glob (bucket, group) cells as numpy columns: ts, glob, count, hi, lo, vmin, vmax (count == 0: no value),
    key (canonical tag key, object array of bytes)."""

    FIELDS = ("ts", "glob", "count", "hi", "lo", "vmin", "vmax", "key")

    def __init__(self, **cols):
        for f in self.FIELDS:
            setattr(self, f, cols[f])

    def __len__(self):
        return len(self.ts)

    def to_dict(self):
        return {f: getattr(self, f) for f in self.FIELDS}

    @staticmethod
    def concat(tables: Sequence["CellTable"]) -> "CellTable":
        return CellTable(**{f: np.concatenate([getattr(t, f) for t in tables]) if tables else np.zeros(0)
                            for f in CellTable.FIELDS})


def evaluate_cell_table(pr: dx.PushDownRequest, glob_size: int, blobs: Sequence, threads: int = 0,
                        timing: Optional[list] = None) -> CellTable:
    """evaluate_glob_cells in columnar form: the same cells, tags already materialized per S15 into canonical keys.
    `timing` (a list) receives the C++ evaluation's wall time in seconds (the CPU baseline's timed part)."""
    text, strcols, gbs = plan_text(pr, glob_size)
    n = len(blobs)
    ptrs = (ctypes.c_void_p * max(1, n))()
    sizes = (ctypes.c_size_t * max(1, n))()
    keep = []
    for i, b in enumerate(blobs):
        if isinstance(b, (bytes, bytearray)):
            buf = ctypes.create_string_buffer(bytes(b), len(b))
            keep.append(buf)
            ptrs[i], sizes[i] = ctypes.cast(buf, ctypes.c_void_p), len(b)
        else:
            ptrs[i], sizes[i] = ctypes.cast(b[0], ctypes.c_void_p), b[1]
    L = lib()
    t0 = time.perf_counter()
    h = L.lkcpu_eval(text.encode(), ptrs, sizes, n, threads)
    if timing is not None:
        timing.append(time.perf_counter() - t0)
    if not h:
        raise RuntimeError(L.lkcpu_error().decode())
    try:
        m = L.lkcpu_ncells(h)
        nc = L.lkcpu_ncols(h)
        glob = np.zeros(m, np.int32)
        ts = np.zeros(m, np.int64)
        rows = np.zeros(m, np.uint64)
        cnt = np.zeros(m, np.uint64)
        hi = np.zeros(m, np.float64)
        lo = np.zeros(m, np.float64)
        mn = np.zeros(m, np.float64)
        mx = np.zeros(m, np.float64)
        nanf = np.zeros(m, np.uint8)
        keys = np.zeros(max(1, m * nc), np.int32)
        L.lkcpu_cells(h, *[a.ctypes.data for a in (glob, ts, rows, cnt, hi, lo, mn, mx, nanf, keys)])
        keys = keys[:m * nc].reshape(m, nc)
        names = ["name"] + gbs
        cols = []
        for j in range(nc):
            uniq, inv = np.unique(keys[:, j], return_inverse=True)
            text_u = []
            for u in uniq.tolist():
                v = L.lkcpu_key_string(h, j, int(u)) if u >= 0 else None
                text_u.append(b"" if v is None or v in (b"null", b"") else v)   # Commons.scala:433 (S15)
            cols.append(np.array(text_u, dtype=object)[inv] if m else np.zeros(0, object))
        globs = dx.globs_of(pr, glob_size)
        qkeys = np.array([tag_key({k: (v if isinstance(v, str) else str(v))
                                   for k, v in pr.segmentRequests[g[0]].queryTags.items()}) for g in globs] or [b""],
                         dtype=object)
        key = join_tag_columns(names, cols, qkeys[glob] if m else np.zeros(0, object))
        vmin = np.where(nanf & 2, mn, np.nan)
        vmax = np.where(nanf & 1, np.nan, mx)
        return CellTable(ts=ts, glob=glob, count=cnt, hi=hi, lo=lo, vmin=vmin, vmax=vmax, key=key)
    finally:
        L.lkcpu_free(h)


def _two_sum(a, b):
    s = a + b
    bb = s - a
    return s, (a - (s - bb)) + (b - bb)


def merge_cell_table(t: CellTable, agg: str, has_group_bys: bool):
    """query-api merge (S19) of cells (any number of globs and ranks) -> (ts, value, key) arrays sorted by (ts, key):
    with groupBys one row per (ts, tag map), else one per ts with the smallest tag map (deterministic stand-in for
    the first arrival, as merge_glob_cells).  sum: hi / lo parts accumulated in double-double, rounded once (within
    1 ulp of the correctly rounded sum, the test bar); min / max: java.lang.Math semantics, a NaN absorbs."""
    n = len(t)
    if n == 0:
        return np.zeros(0, np.int64), np.zeros(0), np.zeros(0, object)
    kid_u, kid = np.unique(t.key.astype(bytes), return_inverse=True)
    if has_group_bys:
        order = np.lexsort((kid, t.ts))
        ts_s, k_s = t.ts[order], kid[order]
        start = np.ones(n, bool)
        start[1:] = (ts_s[1:] != ts_s[:-1]) | (k_s[1:] != k_s[:-1])
    else:
        order = np.lexsort((kid, t.ts))
        ts_s, k_s = t.ts[order], kid[order]
        start = np.ones(n, bool)
        start[1:] = ts_s[1:] != ts_s[:-1]
    g = np.cumsum(start) - 1
    G = int(g[-1]) + 1
    first = np.nonzero(start)[0]
    pos = np.arange(n) - first[g]
    out_ts = ts_s[first]
    out_key = kid_u[k_s[first]].astype(object)   # (sorted by key within a ts: the first is the smallest map)
    cnt = t.count[order]
    total = np.zeros(G, np.uint64)
    np.add.at(total, g, cnt)
    if agg in (dx.SUM, dx.AVG):
        hi, lo = t.hi[order], t.lo[order]
        acc_hi, acc_lo = np.zeros(G), np.zeros(G)
        for k in range(int(pos.max()) + 1):
            sel = pos == k
            idx = g[sel]
            for x in (hi[sel], lo[sel]):
                s, e = _two_sum(acc_hi[idx], x)
                acc_hi[idx] = s
                acc_lo[idx] += e
        with np.errstate(invalid="ignore"):
            ssum = np.where(np.isfinite(acc_hi), acc_hi + acc_lo, acc_hi)
        if agg == dx.SUM:
            val = np.where(total > 0, ssum, 0.0)
        else:
            with np.errstate(invalid="ignore", divide="ignore"):
                val = np.where(total > 0, ssum / np.maximum(total, 1).astype(np.float64), np.nan)
    elif agg == dx.COUNT:
        val = total.astype(np.float64)
    else:
        src = (t.vmin if agg == dx.MIN else t.vmax)[order]
        cell = np.where(cnt > 0, src, 0.0)   # a cell without values reads 0.0 (S15 getDouble of NULL)
        val = np.full(G, np.inf if agg == dx.MIN else -np.inf)
        (np.minimum if agg == dx.MIN else np.maximum).at(val, g, cell)
    return out_ts, val, out_key


def assert_columns_equal(got, want, agg: str, label: str = ""):
    """(ts, value, key) arrays, each side in any order: the same rows; count / min / max bit-exact, sum / avg within
    1 ulp (tests/parity.py's bar, vectorized)."""
    def srt(cols):
        ts, val, key = cols
        key = np.asarray(key, dtype=object).astype(bytes)
        o = np.lexsort((key, ts))
        return ts[o], val[o], key[o]
    gt, gv, gk = srt(got)
    wt, wv, wk = srt(want)
    assert len(gt) == len(wt), f"{label}: {len(gt)} rows vs expected {len(wt)}"
    bad = np.nonzero(gt != wt)[0]
    assert not len(bad), f"{label}: row {bad[0]} ts {gt[bad[0]]} vs {wt[bad[0]]}"
    bad = np.nonzero(gk != wk)[0]
    assert not len(bad), f"{label}: row {bad[0]} tags {tags_of_key(gk[bad[0]])} vs {tags_of_key(wk[bad[0]])}"
    both_nan = np.isnan(gv) & np.isnan(wv)
    if agg in (dx.SUM, dx.AVG):
        with np.errstate(invalid="ignore"):
            ok = (gv == wv) | both_nan | (np.abs(gv - wv) <= np.spacing(np.abs(wv)))
    else:
        ok = ((gv == wv) & (np.signbit(gv) == np.signbit(wv))) | both_nan
    bad = np.nonzero(~ok)[0]
    assert not len(bad), (f"{label}: row {bad[0]} at ts={gt[bad[0]]} tags={tags_of_key(gk[bad[0]])}: value "
                          f"{gv[bad[0]]!r} vs expected {wv[bad[0]]!r} (agg {agg})")


def evaluate_per_glob(pr: dx.PushDownRequest, blobs: Sequence, glob_size: int = 10, threads: int = 0):
    agg = pr.baseExpr.chart.aggregation
    return [[(c.ts, c.agg_value(agg), c.tags) for c in cells]
            for cells in evaluate_glob_cells(pr, glob_size, blobs, threads)]
