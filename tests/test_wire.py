"""Worker / query-api wire format (lakeside_amd/wire.py): the SSE framing of Commons.dataPointResponseToSSE +
PushDownAggregatorStage (pinned from the Scala, file:line in the module) and the SegmentSequencer.decode
round trip, including non-finite values and the no-segment sentinel."""
import json
import math

from lakeside_amd import wire


def test_worker_sse_frame():
    (chunk,) = list(wire.worker_sse([(1704067200000, 12.5, {"name": "metric_07"})], "sum"))
    assert chunk.startswith("data: ") and chunk.endswith("\r\n\r\n")
    body = json.loads(chunk[6:-4])
    assert body == {"id": "_", "type": "data",
                    "message": {"timestamp": 1704067200000, "tags": {"name": "metric_07"}, "type": "sketch",
                                "sketchType": "map", "sketch": {"sum": 12.5}}}


def test_round_trip_with_non_finite_values():
    rows = [(1000, 1.0, {"name": "a"}), (2000, math.nan, {"name": "b", "svc": "x"}), (3000, math.inf, {}),
            (4000, -math.inf, {"k": "v"}), (5000, -0.0, {"name": "z"})]
    out = [wire.decode_message(json.dumps(p["message"])) for p in wire.parse_sse("".join(wire.worker_sse(rows, "max")))]
    assert len(out) == len(rows)
    for (kind, ts, tags, sk), (t, v, g) in zip(out, rows):
        assert kind == "sketch" and ts == t and tags == g
        w = sk["max"]
        assert (math.isnan(w) and math.isnan(v)) or (w == v and math.copysign(1, w) == math.copysign(1, v))


def test_sentinel_is_an_exemplar():
    (chunk,) = list(wire.worker_sse([(-1, -1.0, {})], "sum"))
    kind, ts, tags, v = wire.decode_message(json.dumps(json.loads(chunk[6:-4])["message"]))
    assert (kind, ts, tags, v) == ("exemplar", -1, {}, -1.0)


def test_decode_tolerates_strings():
    """SegmentSequencer.asDouble / asLong (SegmentSequencer.scala:35-51)."""
    m = {"timestamp": "17", "tags": {}, "type": "sketch", "sketchType": "map",
         "sketch": {"a": "Infinity", "b": "nan", "c": "2.5", "d": "junk", "e": 3}}
    kind, ts, _, sk = wire.decode_message(json.dumps(m))
    assert ts == 17 and sk["a"] == math.inf and math.isnan(sk["b"]) and sk["c"] == 2.5 and math.isnan(sk["d"])
    assert sk["e"] == 3.0


def test_timeseries_payload_frame():
    p = {"id": "A", "type": "timeseries", "message": {"timestamp": 5, "tags": {"name": "m"}, "value": math.nan,
                                                       "label": "(x = 1)"}}
    (chunk,) = list(wire.timeseries_sse([p]))
    assert json.loads(chunk[6:-4]) == {"id": "A", "type": "timeseries",
                                       "message": {"timestamp": 5, "tags": {"name": "m"}, "value": "NaN",
                                                   "label": "(x = 1)"}}
