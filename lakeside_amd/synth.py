"""Synthetic sealed segments (bench/test tooling): ctypes wrapper of tools/synth.cpp."""
import ctypes
import os

from ._lib import SYNTH_PATH

T0 = 1704067200000          # 2024-01-01T00:00:00Z
HOUR = 3_600_000


class Spec(ctypes.Structure):
    _fields_ = [("rows", ctypes.c_uint64), ("seed", ctypes.c_uint64), ("t0_ms", ctypes.c_int64),
                ("span_ms", ctypes.c_int64), ("rg_rows", ctypes.c_uint32), ("page_rows", ctypes.c_uint32),
                ("value_mode", ctypes.c_int32), ("null_frac", ctypes.c_double), ("highcard_n", ctypes.c_uint32),
                ("threads", ctypes.c_int32), ("ts_shuffle", ctypes.c_int32)]


_L = None


def _lib():
    global _L
    if _L is None:
        if not os.path.exists(SYNTH_PATH):
            raise ImportError(f"{SYNTH_PATH} missing: run `make`")
        _L = ctypes.CDLL(SYNTH_PATH)
        _L.lk_synth_segment.argtypes = [ctypes.POINTER(Spec), ctypes.POINTER(ctypes.POINTER(ctypes.c_uint8)),
                                        ctypes.POINTER(ctypes.c_size_t)]
        _L.lk_synth_segment.restype = ctypes.c_int
        _L.lk_synth_free.argtypes = [ctypes.POINTER(ctypes.c_uint8)]
    return _L


class Segment:
    """Owns a malloc'd Parquet buffer; ``ptr``/``size`` feed Engine.put_segment_ptr without a copy."""

    def __init__(self, ptr, size):
        self.ptr = ptr
        self.size = size

    def bytes(self) -> bytes:
        return ctypes.string_at(self.ptr, self.size)

    def free(self):
        if self.ptr:
            _lib().lk_synth_free(self.ptr)
            self.ptr = None

    def __del__(self):
        self.free()


def segment_spec(index: int, rows: int = 1 << 24, hour: int = None, value_mode: int = 0, null_frac: float = 0.0,
                 rg_rows: int = 1 << 20, page_rows: int = 131072, highcard_n: int = 0, threads: int = 0,
                 ts_shuffle: int = 0) -> Spec:
    """Segment `index` of the bench configs: seed 20240101 + index, covering hour (index mod 4) of T0.
    value_mode 0: integer values in [0, 1000); 1: lognormal(0, 2) reals (SURVEY §8(d) "real").  ts_shuffle 1: the
    timestamps permuted within each row group (no sorted tile, no tile pinned to one bucket by its zone map)."""
    h = index % 4 if hour is None else hour
    return Spec(rows=rows, seed=20240101 + index, t0_ms=T0 + h * HOUR, span_ms=HOUR, rg_rows=rg_rows,
                page_rows=page_rows, value_mode=value_mode, null_frac=null_frac, highcard_n=highcard_n,
                threads=threads, ts_shuffle=ts_shuffle)


def make_segment(spec: Spec) -> Segment:
    p = ctypes.POINTER(ctypes.c_uint8)()
    n = ctypes.c_size_t()
    rc = _lib().lk_synth_segment(ctypes.byref(spec), ctypes.byref(p), ctypes.byref(n))
    if rc != 0:
        raise RuntimeError(f"lk_synth_segment failed: {rc}")
    return Segment(p, n.value)


def segment_request(index: int, step: int = 60000, hour: int = None, query_tags=None, dataset="logs") -> dict:
    h = index % 4 if hour is None else hour
    start = T0 + h * HOUR
    return {"hour": f"{h:02d}", "dateInt": "20240101", "segmentId": f"tbl_{index}", "sealedStatus": True,
            "dataset": dataset, "queryTags": query_tags or {}, "stepInMillis": step, "customerId": "c",
            "collectorId": "k", "bucketName": "b", "cName": "", "startTs": start, "endTs": start + HOUR}


def pushdown(filter_, segs, agg="sum", group_bys=(), dataset="logs", tag=None) -> dict:
    """A PushDownRequest; with `tag`, a tag query (no chart, isTagQuery + tagDataType, as
    QueryEngineV2.evaluateTagQuery sends it)."""
    be = {"id": "A", "dataset": dataset, "filter": filter_,
          "chart": {"aggregation": agg, "groupBys": list(group_bys), "type": "count"},
          "limit": 1000, "order": "DESC", "metricType": "gauge", "returnResults": True}
    req = {"baseExpr": be, "segmentRequests": list(segs), "reverseSort": False, "isTagQuery": False}
    if tag is not None:
        del be["chart"]
        req["isTagQuery"] = True
        req["tagDataType"] = {"tagName": tag, "dataType": "string"}
    return req


def leaf(k, op, *v):
    return {"k": k, "v": list(v), "op": op, "extracted": False, "computed": False, "dataType": "string"}


NAME = "_cardinalhq.name"
SERVICE = "resource.service.name"
NAMESPACE = "resource.k8s.namespace.name"
CONTAINER = "resource.container.id"
