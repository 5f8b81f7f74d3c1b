"""Restatement of the reference's DataExpr -> SQL compiler + an independent SQL executor (TEST ONLY).

``generate_sql`` restates ``BaseExpr.generateSql`` (core/src/main/scala/com/cardinal/utils/ast/
BaseExpr.scala:108-144, getBaseQuery 181-242, getChartSql 319-405, filterSqlAndAccumulateFields
433-513) for chart queries without extract/compute.  Its output is pinned character-for-character by
the SQL strings of the reference's own test ``ASTUtilsBaseExprTest.scala`` (fixtures in
``tests/golden/ref_sql_cases.json``).

``run_sql`` executes that exact SQL text on SQLite (stdlib) over the glob's Parquet rows, which gives
an engine-independent check of ``oracle/dataexpr.py``: the reference's own plan, run by a second SQL
engine.  Differences DuckDB vs SQLite that matter here are handled explicitly: ``regexp_matches`` is
registered as a UDF backed by RE2 (pyarrow), and SQLite's ``%`` casts to INTEGER, which equals
DuckDB's ``BIGINT % DOUBLE`` fmod for integral timestamps below 2**53.
"""
from __future__ import annotations

import sqlite3
from typing import Dict, List, Optional, Sequence

from .dataexpr import (BinaryClause, Filter, NotClause, PushDownRequest, METRICS, NAME, TIMESTAMP, VALUE,
                       SUM, field_set, re2_search, HAS, EXISTS, EQ, NOT_EQUALS, IN, NOT_IN, REGEX, CONTAINS,
                       GT, GE, LT, LE)

STEP_TS = "step_ts"   # Commons.scala:56


def filter_sql(q, nonexistent: set) -> str:
    """BaseExpr.filterSqlAndAccumulateFields (BaseExpr.scala:433-513)."""
    if isinstance(q, Filter):
        label = q.k
        if label in nonexistent and not q.extracted and not q.computed:
            return "false"
        if "." in label:
            label = f'"{label}"'
        op = q.op
        if op in (HAS, EXISTS):
            return f"{label} IS NOT NULL"
        if op == EQ:
            return f"{label} = '{q.v[0]}'"
        if op == NOT_EQUALS:
            return f"{label} != '{q.v[0]}'"
        if op == IN:
            return f"{label} IN ({', '.join(repr_sql(v) for v in q.v)})"
        if op == NOT_IN:
            return f"{label} NOT IN ({', '.join(repr_sql(v) for v in q.v)})"
        if op == REGEX:
            return f"regexp_matches({label}, '{q.v[0]}','i')"
        if op == CONTAINS:
            return f"regexp_matches({label}, '.*{q.v[0]}.*','i')"
        if op in (GT, GE, LT, LE):
            sym = {GT: ">", GE: ">=", LT: "<", LE: "<="}[op]
            return f"{label} {sym} {float(q.v[0])!r}"
        raise ValueError(f"Invalid operator {op}")
    if isinstance(q, BinaryClause):
        return f"({filter_sql(q.q1, nonexistent)} {q.op} {filter_sql(q.q2, nonexistent)})"
    return f"NOT ({filter_sql(q.inner, nonexistent)})"


def repr_sql(v: str) -> str:
    return f"'{v}'"


def timestamp_filter(start: int, end: int) -> str:
    """BaseExpr.timestampFilter (BaseExpr.scala:159-161)."""
    return f'"{TIMESTAMP}" >= {start} AND "{TIMESTAMP}" < {end}'


def generate_sql(pr: PushDownRequest, start: int, end: int, step: int, nonexistent: set,
                 sub_query: Optional[str] = None) -> str:
    """BaseExpr.generateSql for a chart query (BaseExpr.scala:108-144 -> getChartSql 319-405).
    ``sub_query`` overrides the inner projection query (used to pin the wrapper against the reference
    test strings, whose inner query is an extract pipeline that is outside the hot path)."""
    be = pr.baseExpr
    chart = be.chart
    fsql = filter_sql(be.filter, nonexistent)
    sub = sub_query if sub_query is not None else f"SELECT * FROM {{tableName}} WHERE {timestamp_filter(start, end)}"
    existing = [g for g in chart.groupBys if g not in nonexistent]           # 338 (no synthetic fields)
    gb = (", " + ", ".join(f'"{g}"' for g in existing)) if (chart.groupBys and existing) else ""
    agg = chart.aggregation
    chart_field_filter = "true"                                               # 407-426 (no fieldName)
    if be.dataset == METRICS:
        rollup = chart.rollup or SUM
        if len(agg) > 1 and agg[0] == "p":   # BaseExpr.scala:379-383: MAX of the rollup per (ts, groupBys, name)
            return (f'SELECT "{TIMESTAMP}", MAX(rollup_{rollup}) as value,'
                    f' "{NAME}" as name  {gb} FROM ({sub}) '
                    f" WHERE {chart_field_filter}"
                    f' AND {fsql} GROUP BY "{TIMESTAMP}" {gb}, name ORDER BY "{TIMESTAMP}" ASC')
        if agg == "ces":                      # BaseExpr.scala:385-388: every passing row, 1.0, no rollup column
            return (f'SELECT "{TIMESTAMP}", 1.0 as value, "{NAME}" as name  {gb} FROM ({sub}) '
                    f" WHERE {chart_field_filter}"
                    f' AND {fsql} ORDER BY "{TIMESTAMP}" ASC')
        return (f'SELECT "{TIMESTAMP}", {agg}(rollup_{rollup}) as value,'
                f' "{NAME}" as name  {gb} FROM ({sub}) '
                f" WHERE {chart_field_filter}"
                f' AND {fsql} GROUP BY "{TIMESTAMP}" {gb}, name  ORDER BY "{TIMESTAMP}" ASC')
    step_sql = f'("{TIMESTAMP}" - ("{TIMESTAMP}" % {step}.0)) as {STEP_TS}'  # 163-165
    calc = f'{agg}("{VALUE}")'
    return (f'SELECT {step_sql}, {calc}, "{NAME}" as name {gb} FROM ({sub}) '
            f" WHERE {chart_field_filter} AND {fsql}"
            f" GROUP BY {STEP_TS} {gb}, name ORDER BY {STEP_TS} ASC")


def _load_glob(paths: Sequence[str]):
    """The glob's rows (union_by_name) in an in-memory SQLite table `t`, with regexp_matches bound to RE2."""
    import pyarrow.parquet as pq
    tables, union = [], []
    for p in paths:
        t = pq.read_table(p)
        for c in t.column_names:
            if c not in union:
                union.append(c)
        tables.append(t)
    con = sqlite3.connect(":memory:")
    cache: Dict[tuple, Optional[bool]] = {}

    def regexp_matches(s, pattern, flags):
        if s is None or pattern is None:
            return None
        k = (s, pattern)
        if k not in cache:
            cache[k] = re2_search([s], pattern)[0]
        r = cache[k]
        return None if r is None else int(r)

    con.create_function("regexp_matches", 3, regexp_matches, deterministic=True)
    cols = ", ".join(f'"{c}"' for c in union)
    con.execute(f"CREATE TABLE t ({cols})")
    for t in tables:
        data = {c: (t.column(c).to_pylist() if c in t.column_names else [None] * t.num_rows) for c in union}
        rows = list(zip(*[data[c] for c in union])) if union else []
        con.executemany(f"INSERT INTO t VALUES ({', '.join('?' * len(union))})", rows)
    return con, union


def generate_tag_sql(pr: PushDownRequest, tag: str, start: int, end: int, nonexistent: set) -> str:
    """BaseExpr.generateSql tag branch for a non-synthetic tag (BaseExpr.scala:127-143)."""
    fsql = filter_sql(pr.baseExpr.filter, nonexistent)
    return (f'SELECT "{tag}" as "{tag}", COUNT(*) AS count FROM {{tableName}} WHERE {fsql} AND '
            f'{timestamp_filter(start, end)} GROUP BY "{tag}"')


def run_tag_sql(pr: PushDownRequest, tag: str, seg_idx: Sequence[int], paths: Sequence[str]):
    """Run the reference's tag-query SQL for one glob on SQLite -> [(raw tag value or None, count)] sorted as
    oracle.dataexpr.evaluate_tag_glob sorts."""
    segs = [pr.segmentRequests[i] for i in seg_idx]
    con, union = _load_glob(paths)
    be = pr.baseExpr
    fs = field_set(be) if be.chart is not None else _filter_fields(be.filter)
    nonexistent = fs - set(union)
    sql = generate_tag_sql(pr, tag, min(s.startTs for s in segs), max(s.endTs for s in segs),
                           nonexistent).replace("{tableName}", "t")
    import re
    if not set(re.findall(r'"([^"]+)"', sql)) <= set(union):   # DuckDB Binder Error -> empty glob
        con.close()
        return []
    out = [(v, int(c)) for v, c in con.execute(sql).fetchall()]
    con.close()
    # a numeric tag column: SQLite groups the values; the row's tag is JDBC getString of the glob's union type
    import pyarrow.parquet as pq
    from oracle.dataexpr import _tag_kind, numeric_tag_text
    kinds = set()
    for p in paths:
        sch = pq.read_schema(p)
        if tag in sch.names:
            kinds.add(_tag_kind(sch.field(tag).type))
    if kinds and "text" not in kinds:
        acc = {}
        for v, c in out:
            k = numeric_tag_text(kinds, v)
            acc[k] = acc.get(k, 0) + c
        out = list(acc.items())
    out.sort(key=lambda r: (r[0] is not None, r[0] or ""))
    return out


def _filter_fields(q) -> set:
    from oracle.dataexpr import filter_field_set
    return filter_field_set(q)


def run_sql(pr: PushDownRequest, seg_idx: Sequence[int], paths: Sequence[str]):
    """Run the reference's generated SQL for one glob on SQLite; returns rows materialized as
    Commons.toDataPoint does (Commons.scala:399-462): [(ts, value, tags)]."""
    segs = [pr.segmentRequests[i] for i in seg_idx]
    con, union = _load_glob(paths)
    nonexistent = field_set(pr.baseExpr) - set(union)
    start = min(s.startTs for s in segs)
    end = max(s.endTs for s in segs)
    step = segs[0].stepInMillis
    sql = generate_sql(pr, start, end, step, nonexistent).replace("{tableName}", "t")
    # SQLite reads an unknown double-quoted identifier as a string literal; DuckDB raises a Binder Error
    # that the worker turns into an empty glob (Commons.scala:249-253).  Mirror DuckDB.
    import re
    metrics_ces = pr.baseExpr.dataset == METRICS and pr.baseExpr.chart.aggregation == "ces"
    idents = set(re.findall(r'"([^"]+)"', sql)) | (set() if metrics_ces else
                                                   {"rollup_" + (pr.baseExpr.chart.rollup or SUM)
                                                    if pr.baseExpr.dataset == METRICS else VALUE})
    if not idents <= set(union):
        con.close()
        return []
    cur = con.execute(sql)
    names = [d[0] for d in cur.description]
    out = []
    qtags = {k: str(v) for k, v in segs[0].queryTags.items()}
    for r in cur.fetchall():
        ts = int(r[0])
        v = 0.0 if r[1] is None else float(r[1])
        tags = {}
        for name, val in zip(names[2:], r[2:]):
            if val is not None and str(val) != "null" and str(val) != "":
                tags[name] = str(val)
        out.append((ts, v, tags or dict(qtags)))
    out.sort(key=lambda x: (x[0], sorted(x[2].items()), x[1]))
    con.close()
    return out
