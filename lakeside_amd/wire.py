"""Worker <-> query-api wire format around the evaluator.

  * PushDownAggregatorStage map branch (core/src/main/scala/com/cardinal/utils/PushDownAggregatorStage.scala:95-106):
    every worker row becomes a SketchInput with a "map" sketch {aggregation: value};
  * Commons.dataPointResponseToSSE (core/src/main/scala/com/cardinal/utils/Commons.scala:474-502) +
    GenericSSEPayload.toChunkStreamPart (core/src/main/scala/com/cardinal/model/SSEMessage.scala:27-34):
    `data: {"id":"_","type":"data","message":{...}}\\r\\n\\r\\n`; the no-segment sentinel DataPoint(-1, -1, {})
    (Commons.scala:393-396) goes out as an "exemplar" message;
  * SegmentSequencer.decode (query-api/src/main/scala/com/cardinal/queryapi/engine/SegmentSequencer.scala:35-101):
    the query-api side, tolerant of "NaN"/"Infinity" strings for values.

Non-finite doubles are written as the strings "NaN" / "Infinity" / "-Infinity" (Jackson's quoted non-numeric
numbers); key order inside an object is not significant.
"""
import json
import math
from typing import Dict, Iterable, Iterator, Tuple

SEP = "\r\n\r\n"


def _num(v: float):
    v = float(v)
    if math.isnan(v):
        return "NaN"
    if math.isinf(v):
        return "Infinity" if v > 0 else "-Infinity"
    return v


def _sse(obj: dict) -> str:
    return "data: " + json.dumps(obj, separators=(",", ":"), allow_nan=False) + SEP


def worker_message(ts: int, value: float, tags: Dict[str, str], aggregation: str) -> dict:
    """One worker output row -> the SSE message body (PushDownAggregatorStage map wrap + dataPointResponseToSSE);
    the sentinel row (ts -1) is the exemplar DataPoint(-1, -1, {})."""
    if ts == -1 and not tags:
        return {"timestamp": -1, "value": _num(value), "tags": {}, "type": "exemplar"}
    return {"timestamp": int(ts), "tags": dict(tags), "type": "sketch", "sketchType": "map",
            "sketch": {aggregation: _num(value)}}


def worker_sse(rows: Iterable[Tuple[int, float, Dict[str, str]]], aggregation: str) -> Iterator[str]:
    """Rows (ascending time, as lk_eval_pushdown returns them) -> SSE chunks of the worker stream."""
    for ts, v, tags in rows:
        yield _sse({"id": "_", "type": "data", "message": worker_message(ts, v, tags, aggregation)})


def _as_double(v) -> float:
    """SegmentSequencer.asDouble (SegmentSequencer.scala:35-45)."""
    if isinstance(v, (int, float)) and not isinstance(v, bool):
        return float(v)
    if isinstance(v, str):
        if v in ("NaN", "nan"):
            return math.nan
        if v in ("Infinity", "+Infinity"):
            return math.inf
        if v == "-Infinity":
            return -math.inf
        try:
            return float(v)
        except ValueError:
            return math.nan
    return math.nan


def _as_long(v) -> int:
    """SegmentSequencer.asLong (SegmentSequencer.scala:47-51)."""
    if isinstance(v, (int, float)) and not isinstance(v, bool):
        return int(v)
    if isinstance(v, str):
        try:
            return int(v)
        except ValueError:
            return 0
    return 0


def decode_message(text: str):
    """SegmentSequencer.decode (SegmentSequencer.scala:65-101) for the map-sketch and exemplar messages:
    -> ("sketch", ts, tags, {agg: value}) or ("exemplar", ts, tags, value)."""
    m = json.loads(text)
    tags = {k: str(v) for k, v in m["tags"].items()}
    if m["type"] == "exemplar":
        return "exemplar", _as_long(m["timestamp"]), tags, _as_double(m["value"])
    if m["sketchType"] != "map":
        raise NotImplementedError("hll / dd sketches are not on the hot path")
    return "sketch", _as_long(m["timestamp"]), tags, {k: _as_double(v) for k, v in m["sketch"].items()}


def parse_sse(stream: str) -> Iterator[dict]:
    """Split an SSE stream into its `data:` payloads (heartbeats included)."""
    for chunk in stream.split(SEP):
        if chunk.startswith("data: "):
            yield json.loads(chunk[len("data: "):])


def timeseries_sse(payloads: Iterable[dict]) -> Iterator[str]:
    """query-api payloads (queryapi.eval_merged_rows) -> the client stream (QueryEngineV2.scala:400-417)."""
    for p in payloads:
        m = dict(p["message"])
        m["value"] = _num(m["value"])
        yield _sse({"id": p["id"], "type": p["type"], "message": m})


__all__ = ["worker_message", "worker_sse", "decode_message", "parse_sse", "timeseries_sse"]
