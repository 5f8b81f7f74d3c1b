"""query-api side of an aggregate DataExpr over the HIP evaluator.

Mirrors, for one chart DataExpr over one SegmentGroup:
  QueryEngineV2.evaluateBaseExpr      query-api/src/main/scala/com/cardinal/queryapi/engine/QueryEngineV2.scala:271-308
  (fan-out + K-way mergeSortedSource  QueryEngineV2.scala:76-97, SegmentSequencer.scala:53-160)
  TimeGroupedSketchAggregator         core/src/main/scala/com/cardinal/eval/TimeGroupedSketchAggregator.scala:57-258
  BaseExpr.eval / getFromSketch       core/src/main/scala/com/cardinal/utils/ast/BaseExpr.scala:665-695, 86-93
  ASTUtils.getTransformerFunc / toGroupByKey / QueryClause.toString
                                      core/src/main/scala/com/cardinal/utils/ast/ASTUtils.scala:190-219, 87-89, 102-122
  BaseExpr.label                      BaseExpr.scala:697-716
  toGenericSSEPayload                 QueryEngineV2.scala:400-417

MI355X design: the worker fan-out, the K-way stream merge and the time-grouped sketch merge collapse into the
engine's merged table (LK_MERGED: one cell per (bucket, tags), globs and GPUs folded on the device, emitted in
ascending time).  AVG, which the reference runs as two pushdowns (SUM and COUNT) merged per (timestamp, tags)
into a {sum, count} map, is one scan: the table carries both and the merged value is Σsum / Σcount.  What is
left for the host is O(output rows): the future-timestamp drop, the chart transformer (vectorised), the
group-key collapse of BaseExpr.eval and the payload.
"""
import json
import time
from typing import Callable, Dict, List, Optional, Sequence

import numpy as np

from ._lib import LK_MERGED

SUM, COUNT, MIN, MAX, AVG = "sum", "count", "min", "max", "avg"


def clause_string(q: dict) -> str:
    """QueryClause.toString (ASTUtils.scala:102-122) of a filter JSON node (parsed as ASTUtils.handleFilter,
    ASTUtils.scala:379-417: `not`, leaf, or a binary node whose non-text members fold left)."""
    if q.get("not") is not None:
        return f"not({clause_string(q['not'])})"
    if q.get("k") is not None:
        k, v, op = q["k"], list(q.get("v") or []), q.get("op")
        if op in ("eq", "gt", "ge", "lt", "le"):
            sym = {"eq": "=", "gt": ">", "ge": ">=", "lt": "<", "le": "<="}[op]
            return f"{k} {sym} {v[0]}"
        if op == "regex":
            return f"regexMatches({k}, {v[0]})"
        if op == "contains":
            return f"{k} contains {v[0]}"
        if op == "in":
            return f"{k} in ({', '.join(v)})"
        return ""
    children = [c for c in q.values() if not isinstance(c, str)]
    s = clause_string(children[0])
    for c in children[1:]:
        s = f"({s} {q['op']} {clause_string(c)})"
    return s


def label(base_expr: dict, tags: Dict[str, str]) -> str:
    """BaseExpr.label (BaseExpr.scala:697-716)."""
    gbs = sorted(set((base_expr.get("chart") or {}).get("groupBys") or []))
    if gbs:
        inner = ", ".join(f"{k} = {tags[k]}" for k in gbs if k in tags)
    else:
        inner = clause_string(base_expr["filter"])
    return f"({inner})"


def group_by_key(group_bys: Sequence[str], tags: Dict[str, str]) -> str:
    """ASTUtils.toGroupByKey (ASTUtils.scala:87-89); "default" without groupBys (BaseExpr.scala:689-690)."""
    gbs = sorted(set(group_bys))
    if not gbs:
        return "default"
    return ":".join(str(tags.get(k, "")) for k in gbs)


def _chart_type(s: Optional[str]) -> str:
    """ChartType.fromStr (core/.../model/query/common/ChartType.scala:41-47); default "count"
    (ASTUtils.scala:350)."""
    t = (s if s is not None else "count").lower().strip()
    if t not in ("count", "rate"):
        raise ValueError(f"Unknown chart type {s}!")
    return t


def _metric_type(s: Optional[str]) -> str:
    """MetricType.fromStr (core/.../model/query/common/MetricType.scala:65-73; METRIC_TYPE_* at
    core/.../utils/Commons.scala:49-52); default gauge (ASTUtils.scala:298-303)."""
    t = (s if s is not None else "gauge").lower().strip()
    if t == "rate":
        return "rate"
    if t in ("count", "counter"):
        return "counter"
    if t in ("gauge", "histogram"):
        return t
    raise ValueError(f"Unknown metric type {s}!")


def transformer(base_expr: dict, step_ms: int) -> Callable[[np.ndarray], np.ndarray]:
    """ASTUtils.getTransformerFunc (ASTUtils.scala:190-219), vectorised.  The step in seconds is the Long
    quotient stepInMillis / 1000; IEEE division (x / 0 = ±inf / NaN) as on the JVM."""
    chart = base_expr.get("chart") or {}
    ct = _chart_type(chart.get("type"))
    mt = _metric_type(base_expr.get("metricType"))
    secs = np.float64(int(step_ms) // 1000)

    def div(v):
        with np.errstate(divide="ignore", invalid="ignore"):
            return np.asarray(v, np.float64) / secs

    if base_expr.get("dataset", "metrics") == "metrics":
        if ct == "count" and mt == "rate":
            return lambda v: np.asarray(v, np.float64) * secs
        if ct == "rate" and mt == "counter":
            return div
        return lambda v: np.asarray(v, np.float64)
    if ct == "rate":
        return div
    return lambda v: np.asarray(v, np.float64)


def eval_merged_rows(base_expr: dict, ts: np.ndarray, values: np.ndarray, tags: Sequence[Dict[str, str]],
                     step_ms: int, now_ms: Optional[int] = None) -> List[dict]:
    """Merged (timestamp, value, tags) rows, ascending in time (one per time-grouped sketch merger cell) ->
    the `timeseries` payloads query-api streams to the client.

      * TimeGroupedSketchAggregator.onPush (TimeGroupedSketchAggregator.scala:200-222): a timestamp later than
        now is dropped ("future"); with ascending input the "old" drop never fires;
      * BaseExpr.eval (BaseExpr.scala:665-695): value = transformer(getFromSketch(map, aggregation)); results of
        one timestamp are keyed by toGroupByKey (sorted groupBy values joined with ":") or "default", a later
        row overwriting an earlier one under the same key.  The reference's order among rows of one
        timestamp is the iteration order of a hash map; here the row with the smallest sorted tag list wins
        (deterministic), and payloads of one timestamp come out in key order.
    """
    now = int(time.time() * 1000) if now_ms is None else int(now_ms)
    gbs = (base_expr.get("chart") or {}).get("groupBys") or []
    expr_id = base_expr.get("id", "_")
    vals = transformer(base_expr, step_ms)(values)
    out: List[dict] = []
    n = len(ts)
    i = 0
    while i < n:
        t = int(ts[i])
        j = i
        while j < n and int(ts[j]) == t:
            j += 1
        if t <= now:
            best: Dict[str, tuple] = {}
            for r in range(i, j):
                key = group_by_key(gbs, tags[r])
                rank = sorted(tags[r].items())
                if key not in best or rank < best[key][0]:
                    best[key] = (rank, r)
            for key in sorted(best):
                r = best[key][1]
                out.append({"id": expr_id, "type": "timeseries",
                            "message": {"timestamp": t, "tags": dict(tags[r]), "value": float(vals[r]),
                                        "label": label(base_expr, tags[r])}})
        i = j
    return out


def evaluate_base_expr(engine, base_expr: dict, segment_requests: Sequence[dict], paths: Sequence[str],
                       step_ms: int, glob_size: int = 10, now_ms: Optional[int] = None,
                       shard: Optional[Sequence[int]] = None, distributed: bool = False) -> List[dict]:
    """QueryEngineV2.evaluateBaseExpr (QueryEngineV2.scala:271-308) for one SegmentGroup, then
    toGenericSSEPayload (400-417): one merged evaluation on the engine (lk_eval_pushdown LK_MERGED, or the
    sharded lk_eval_pushdown_dist whose rank 0 alone gets rows), then eval_merged_rows."""
    req = json.dumps({"baseExpr": base_expr, "segmentRequests": list(segment_requests), "reverseSort": False,
                      "isTagQuery": False})
    if distributed:
        res = engine.eval_pushdown_dist(req, list(paths), shard, glob_size)
    else:
        res = engine.eval_pushdown(req, list(paths), glob_size, LK_MERGED)
    return eval_merged_rows(base_expr, res.ts, res.values, res.tags, step_ms, now_ms)


__all__ = ["clause_string", "label", "group_by_key", "transformer", "eval_merged_rows", "evaluate_base_expr"]
