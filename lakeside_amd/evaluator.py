"""Host-side mirror of the worker's per-segment evaluator over the HIP engine.

``evaluate_push_down_request`` mirrors ``Commons.evaluatePushDownRequest(queryId, localParquet,
pushDownRequest)`` (core/src/main/scala/com/cardinal/utils/Commons.scala:343-397): same arguments, globs
of 10 (local) or 5 (remote) segments, rows ascending by timestamp per glob, errors swallowed into an empty
result as the reference does (Commons.scala:249-253, 338-340).  ``Engine`` is the lower-level API that
raises ``LakesideError`` instead.
"""
import ctypes
import json
import logging
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from . import _lib
from ._lib import LK_MERGED, LK_PER_GLOB_ROWS, LakesideError, check

log = logging.getLogger("lakeside_amd")

Row = Tuple[int, float, Dict[str, str]]


class _Handle:
    """Owns an lk_result; freed when the last Result / array view referencing it goes away."""

    def __init__(self, h):
        self.h = h

    def __del__(self):
        try:
            if self.h is not None:
                _lib.lib().lk_result_free(self.h)
                self.h = None
        except Exception:
            pass


class _View:
    """numpy array interface over a result column (zero copy; keeps the owning handle alive)."""

    def __init__(self, owner: _Handle, ptr, n: int, typestr: str):
        self._owner = owner
        self.__array_interface__ = {"shape": (n,), "typestr": typestr, "version": 3,
                                    "data": (ctypes.cast(ptr, ctypes.c_void_p).value, True)}


class Result:
    """Rows of one evaluation.  Timestamps, values and glob indices are read-only numpy views of the library
    result (no copy); tag strings are decoded from the library result on first use."""

    def __init__(self, handle):
        self._owner = _Handle(handle)
        self._cols = None
        self._tag_names = None
        self._stats = None
        self._tags = None

    def _columns(self):
        """Timestamps, values and glob indices as numpy views of the library result (built on first use: a caller
        that only needs the row count or the stats pays one C call)."""
        if self._cols is None:
            L = _lib.lib()
            h = self._owner.h
            n = L.lk_result_num_rows(h)

            def col(ptr, typestr, dtype):
                return np.asarray(_View(self._owner, ptr, n, typestr)) if n else np.zeros(0, dtype)

            self._cols = (col(L.lk_result_timestamps(h), "<i8", np.int64), col(L.lk_result_values(h), "<f8", np.float64),
                          col(L.lk_result_globs(h), "<u4", np.uint32))
        return self._cols

    @property
    def ts(self):
        return self._columns()[0]

    @property
    def values(self):
        return self._columns()[1]

    @property
    def globs(self):
        return self._columns()[2]

    @property
    def tag_names(self) -> List[str]:
        if self._tag_names is None:
            L = _lib.lib()
            h = self._owner.h
            self._tag_names = [L.lk_result_tag_name(h, c).decode() for c in range(L.lk_result_num_tag_columns(h))]
        return self._tag_names

    def stats_text(self) -> str:
        """The library's stats JSON text, unparsed (the bench's timed loop keeps these and parses them afterwards)."""
        return _lib.lib().lk_result_stats(self._owner.h).decode()

    @property
    def stats(self) -> dict:
        if self._stats is None:
            self._stats = json.loads(self.stats_text())
        return self._stats

    @property
    def tags(self) -> List[Dict[str, str]]:
        """Per-row tag maps, decoded through the bulk export (lk_result_group_ids + lk_result_tag_dictionary: one
        array read per row and group column, each distinct string decoded once); only the queryTags fallback and
        a tag query's count column go through lk_result_tag_value, per row."""
        if self._tags is None:
            if self._owner is None:
                raise ValueError("result closed before its tags were read")
            L = _lib.lib()
            h = self._owner.h
            n = len(self.ts)
            out: List[Dict[str, str]] = [{} for _ in range(n)]
            ng = L.lk_result_num_group_columns(h) if n else 0
            own = np.zeros(n, dtype=bool)
            if ng:
                gid = np.asarray(_View(self._owner, L.lk_result_group_ids(h), n, "<u4")).astype(np.uint64)
                for c in range(ng):
                    stride, nd = ctypes.c_uint64(), ctypes.c_uint64()
                    p = L.lk_result_tag_dictionary(h, c, ctypes.byref(stride), ctypes.byref(nd))
                    if not p or nd.value == 0:
                        continue
                    d = (gid // np.uint64(stride.value)) % np.uint64(nd.value)
                    uniq, inv = np.unique(d, return_inverse=True)
                    text = [ctypes.string_at(p[int(u)]).decode() if p[int(u)] else None for u in uniq]
                    name = self.tag_names[c]
                    present = np.array([s is not None for s in text], dtype=bool)[inv]
                    own |= present
                    for r in np.nonzero(present)[0].tolist():
                        out[r][name] = text[inv[r]]
            for c in range(ng, len(self.tag_names)):
                name = self.tag_names[c]
                for r in range(n):
                    if own[r] and name != "count":
                        continue   # queryTags apply only to rows whose own tags are all absent
                    v = L.lk_result_tag_value(h, r, c)
                    if v is not None:
                        out[r][name] = v.decode()
            self._tags = out
        return self._tags

    def sketch(self, row: int) -> bytes:
        """The row's serialized DDSketch (percentile aggregations); b"" otherwise."""
        L = _lib.lib()
        n = ctypes.c_size_t()
        p = L.lk_result_sketch(self._owner.h, row, ctypes.byref(n))
        return ctypes.string_at(p, n.value) if n.value else b""

    def close(self):
        """Drop this object's reference; the library result is freed once no array view remains (the columns,
        tag names and stats are read before, so they stay usable)."""
        if self._owner is not None:
            self._columns()
            _ = self.tag_names, self.stats
        self._owner = None

    def __len__(self):
        return int(_lib.lib().lk_result_num_rows(self._owner.h)) if self._cols is None else len(self._cols[0])

    def rows(self) -> List[Row]:
        return [(int(t), float(v), g) for t, v, g in zip(self.ts, self.values, self.tags)]

    def per_glob(self, nglobs: int) -> List[List[Row]]:
        out: List[List[Row]] = [[] for _ in range(nglobs)]
        for t, v, g, tags in zip(self.ts, self.values, self.globs, self.tags):
            out[int(g)].append((int(t), float(v), tags))
        return out


class Engine:
    """One per process per GPU: HIP device, stream, HBM segment cache, optional RCCL communicator."""

    def __init__(self, device: int = 0, hbm_budget_bytes: int = 0, max_calls: int = 4, dict_compact_min_dead: int = 0,
                 load_threads: int = 0):
        L = _lib.lib()
        h = ctypes.c_void_p()
        opts = {"device": device, "hbm_budget_bytes": int(hbm_budget_bytes), "max_calls": int(max_calls)}
        if dict_compact_min_dead:
            opts["dict_compact_min_dead"] = int(dict_compact_min_dead)
        if load_threads:
            opts["load_threads"] = int(load_threads)
        check(L.lk_engine_create(json.dumps(opts).encode(), ctypes.byref(h)))
        self._h = h
        self.device = device

    def close(self):
        if getattr(self, "_h", None):
            _lib.lib().lk_engine_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---- HBM segment cache ----
    def put_segment(self, key: str, data) -> None:
        buf = (ctypes.c_uint8 * len(data)).from_buffer_copy(data) if not isinstance(data, ctypes.Array) else data
        check(_lib.lib().lk_segment_put(self._h, key.encode(), ctypes.cast(buf, ctypes.c_void_p), len(data)))

    def put_segment_ptr(self, key: str, ptr, size: int) -> None:
        check(_lib.lib().lk_segment_put(self._h, key.encode(), ptr, size))

    def load_segment(self, path: str) -> None:
        check(_lib.lib().lk_segment_load(self._h, path.encode()))

    def evict(self, key: str) -> None:
        check(_lib.lib().lk_segment_evict(self._h, key.encode()))

    @property
    def segment_count(self) -> int:
        return int(_lib.lib().lk_segment_count(self._h))

    @property
    def segment_bytes(self) -> int:
        return int(_lib.lib().lk_segment_bytes(self._h))

    @property
    def stats(self) -> dict:
        """Engine counters: cached segments, evictions, dictionary sizes / live ids / compactions."""
        return json.loads(_lib.lib().lk_engine_stats(self._h).decode())

    def drop_caches(self):
        """Forget parsed requests, leaf outcomes, value-key orders and group-dim unions (segments stay cached): the
        next evaluation runs cold."""
        check(_lib.lib().lk_engine_drop_caches(self._h))

    # ---- evaluation ----
    def _path_array(self, paths: Sequence[str]):
        """The C array of encoded paths, reused while the caller passes the same path list (a dashboard's refresh).
        Key and array live in one tuple swapped in by a single assignment, and the call returns the array it built
        or checked itself, so concurrent callers with different path lists never see each other's array."""
        key = tuple(paths)
        c = getattr(self, "_paths_cache", None)
        if c is None or c[0] != key:
            c = (key, (ctypes.c_char_p * len(paths))(*[p.encode() for p in paths]))
            self._paths_cache = c
        return c[1]

    def eval_pushdown(self, request_json: str, paths: Sequence[str], glob_size: int = 10,
                      flags: int = LK_PER_GLOB_ROWS) -> Result:
        L = _lib.lib()
        arr = self._path_array(paths)
        h = ctypes.c_void_p()
        check(L.lk_eval_pushdown(self._h, request_json.encode(), arr, len(paths), glob_size, flags, ctypes.byref(h)))
        return Result(h)

    # ---- multi-GPU ----
    @staticmethod
    def unique_id() -> bytes:
        buf = (ctypes.c_uint8 * _lib.LK_UNIQUE_ID_BYTES)()
        check(_lib.lib().lk_comm_unique_id(buf))
        return bytes(buf)

    def comm_init(self, uid: bytes, world: int, rank: int) -> None:
        buf = (ctypes.c_uint8 * _lib.LK_UNIQUE_ID_BYTES).from_buffer_copy(uid)
        check(_lib.lib().lk_comm_init(self._h, buf, world, rank))

    def comm_init_host(self, world: int, rank: int, group=None, allgather=None) -> None:
        """Host transport (lk_comm_init_host) over a torch.distributed group (default: the gloo world), or over
        `allgather(bytes) -> [bytes per rank]`.  The callback object lives as long as the engine."""
        from . import dist as _dist
        self._allgather_cb = _dist.make_callback(allgather or _dist.gloo_allgather(group))
        check(_lib.lib().lk_comm_init_host(self._h, world, rank, self._allgather_cb, None))

    def eval_pushdown_dist(self, request_json: str, paths: Sequence[str], shard: Optional[Sequence[int]] = None,
                           glob_size: int = 10) -> Result:
        L = _lib.lib()
        arr = self._path_array(paths)
        sh = (ctypes.c_int32 * len(paths))(*shard) if shard is not None else None
        h = ctypes.c_void_p()
        check(L.lk_eval_pushdown_dist(self._h, request_json.encode(), arr, len(paths), sh, glob_size,
                                      ctypes.byref(h)))
        return Result(h)


def evaluate_push_down_request(engine: Engine, query_id: str, local_parquet: bool, push_down_request: str,
                               paths: Sequence[str]) -> List[List[Row]]:
    """Commons.evaluatePushDownRequest (Commons.scala:343-397): per-glob rows; a failing glob/request
    yields no rows (Commons.scala:249-253) and is logged; no segments -> one sentinel row ts=-1."""
    glob_size = 10 if local_parquet else 5
    nglobs = max(1, (len(paths) + glob_size - 1) // glob_size)
    try:
        res = engine.eval_pushdown(push_down_request, paths, glob_size, LK_PER_GLOB_ROWS)
    except LakesideError as e:
        log.error("[%s] Error in reading glob: %s", query_id, e)
        return [[] for _ in range(nglobs)]
    return res.per_glob(nglobs)


def merge_sorted_fold(streams: Sequence[Sequence[Row]], reverse: bool) -> List[Row]:
    """`sources.fold(Source.empty)(_ mergeSorted _)` under Commons.pushDownResponseOrdering (Commons.scala:116-132,
    391-392; WorkerApi.scala:169-173): timestamp order (negated when reverseSort); Akka's MergeSorted emits the
    left head when it is strictly less, the right head otherwise."""
    out: List[Row] = []
    for s in streams:
        m: List[Row] = []
        i = j = 0
        while i < len(out) and j < len(s):
            a, b = out[i][0], s[j][0]
            if (a > b) if reverse else (a < b):
                m.append(out[i])
                i += 1
            else:
                m.append(s[j])
                j += 1
        m.extend(out[i:])
        m.extend(s[j:])
        out = m
    return out


def stream_cached_segment(engine: Engine, payload: str, is_cached, path_of, query_id: str = "") -> List[Row]:
    """WorkerApi.streamCachedSegment (query-worker/src/main/scala/com/cardinal/queryworker/WorkerApi.scala:121-182),
    the worker's HTTP entry, over the engine:
      * the request's segments split into locally cached ones (`is_cached(segment_request)` -- the Caffeine cache
        lookup, 131-147) and sealed ones;
      * each non-empty part runs streamDataRoute -> evaluatePushDownRequest (101-119) with localParquet = true
        (globs of 10) or false (globs of 5); `path_of(segment_request, local)` resolves its Parquet path
        (Commons.toParquetFilePath, Commons.scala:256-278);
      * the two streams fold with mergeSorted (169-173): List(lcSource, sealedSource).fold(Source.empty)(_ mergeSorted _).
    Returns the worker's row stream [(ts, value, tags)] in emission order (wire.worker_sse frames it as SSE).  A part
    with no segments contributes nothing (no sentinel: that is only evaluatePushDownRequest's own empty case)."""
    req = json.loads(payload)
    chart = req.get("baseExpr", {}).get("chart") or {}
    reverse = bool(req.get("reverseSort", False)) and chart.get("rollup") is None   # pushDownResponseOrdering
    segs = req.get("segmentRequests", [])
    parts = ([s for s in segs if is_cached(s)], True), ([s for s in segs if not is_cached(s)], False)
    streams = []
    for part, local in parts:
        if not part:
            continue
        sub = dict(req)
        sub["segmentRequests"] = part
        per_glob = evaluate_push_down_request(engine, query_id, local, json.dumps(sub), [path_of(s, local) for s in part])
        streams.append(merge_sorted_fold(per_glob, reverse))   # evaluatePushDownRequest's fold over its globs
    return merge_sorted_fold(streams, reverse)


__all__ = ["Engine", "Result", "LakesideError", "evaluate_push_down_request", "stream_cached_segment",
           "merge_sorted_fold", "LK_MERGED", "LK_PER_GLOB_ROWS"]
