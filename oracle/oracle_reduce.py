"""Combine / broker-reduce restatement for the CPU oracle. TEST INFRASTRUCTURE ONLY.

Restated from the reference independently of pinot_amd.query (the product's host mirror), so the
oracle's cross-segment combine and its final rows do not share code with what they check:

* merge(): AggregationFunction.merge of each function, null handling disabled
  (pinot-core/.../query/aggregation/function/): COUNT `a + b` (CountAggregationFunction.java:193-195);
  SUM / SUMLONG `a + b` (SumAggregationFunction.merge); MIN `a < b ? a : b`
  (MinAggregationFunction.java:353-367) and MAX `a > b ? a : b` (MaxAggregationFunction.java:353-367) —
  Java's comparison order, so a NaN on the left loses and on the right wins; AVG AvgPair sums
  (AvgAggregationFunction.java:271-285); MINMAXRANGE MinMaxRangePair.apply with < / >
  (MinMaxRangeAggregationFunction.java:278-292); DISTINCTCOUNT set union.
* final(): extractFinalResult — AVG sum / count, DEFAULT_FINAL_RESULT (-inf) when count is 0
  (AvgAggregationFunction.java:306-316); MINMAXRANGE max - min (:313-318); DISTINCTCOUNT set size.
* rows(): GroupByDataTableReducer's final rows: group values then final results, ORDER BY applied
  stably right to left (the comparator chain of the select list), LIMIT (default 10).
* Value identity of group keys and DISTINCTCOUNT elements: Double.doubleToLongBits /
  Float.floatToIntBits (every NaN one value, -0.0 != 0.0), as the fastutil maps and sets compare.

Queries come from the oracle's own SQL front end (oracle_sql.parse); nothing here imports product code
(the functions read a compiled query's attributes only).
"""
from __future__ import annotations

import math
import struct

_NAN_BITS = 0x7FF8000000000000


def java_identity(v):
    """Value identity in a group key / DISTINCTCOUNT set (doubleToLongBits for floating values)."""
    if isinstance(v, float) or type(v).__name__ in ("float64", "float32"):
        f = float(v)
        return ("f", _NAN_BITS if math.isnan(f) else struct.unpack("<q", struct.pack("<d", f))[0])
    return v


def identity_key(key) -> tuple:
    return tuple(java_identity(v) for v in key)


class JDouble(float):
    """A FLOAT/DOUBLE group-key value that compares and hashes by Java's Double.equals identity."""
    __slots__ = ()

    def __eq__(self, other):
        if isinstance(other, float):
            return java_identity(float(self)) == java_identity(float(other))
        return float.__eq__(self, other)

    def __ne__(self, other):
        r = self.__eq__(other)
        return r if r is NotImplemented else not r

    def __hash__(self):
        return hash(_NAN_BITS) if math.isnan(self) else float.__hash__(self)

    def __repr__(self):
        return float.__repr__(self)


def merge(func: str, a, b):
    """AggregationFunction.merge(a, b) (a: the combined result so far, b: the next segment's)."""
    if func in ("COUNT", "SUM", "SUMLONG"):
        return a + b
    if func == "MIN":
        return a if a < b else b
    if func == "MAX":
        return a if a > b else b
    if func == "AVG":
        return (a[0] + b[0], a[1] + b[1])
    if func == "MINMAXRANGE":
        mn = b[0] if b[0] < a[0] else a[0]
        mx = b[1] if b[1] > a[1] else a[1]
        return (mn, mx)
    if func == "DISTINCTCOUNT":
        return a | b
    raise ValueError(func)


def final(func: str, partial):
    """AggregationFunction.extractFinalResult."""
    if func == "AVG":
        s, c = partial
        return s / c if c else float("-inf")
    if func == "MINMAXRANGE":
        return partial[1] - partial[0]
    if func == "DISTINCTCOUNT":
        return len(partial)
    return partial


def rows(qc, groups: dict) -> list:
    """Final rows: (group values..., final results...), ORDER BY then LIMIT."""
    out = [tuple(k) + tuple(final(a.func, p) for a, p in zip(qc.aggregations, parts)) for k, parts in groups.items()]
    names = [g.lower() for g in qc.group_by] + [a.name.lower() for a in qc.aggregations]
    alt = [g.lower() for g in qc.group_by] + [f"{a.func.lower()}({a.column})".lower() for a in qc.aggregations]
    for expr, asc in reversed(qc.order_by):
        e = expr.lower()
        hits = [i for i in range(len(names)) if e in (names[i], alt[i])]
        if not hits:
            raise ValueError(f"ORDER BY {expr} not in select list")
        i = hits[-1]
        out.sort(key=lambda r: r[i], reverse=not asc)
    return out[: qc.limit]


def _value_order(v):
    """Sort key of a group-by value in dictionary order: numbers ascending (Double.compare for floating
    values: -0.0 < 0.0, NaN last), strings in String.compareTo order (UTF-16 code units)."""
    if isinstance(v, str):
        return (0, v.encode("utf-16-be"))
    if isinstance(v, float):
        if math.isnan(v):
            return (1, float("inf"), 1)
        return (1, v, 1 if math.copysign(1.0, v) > 0 else 0)
    return (1, v, 0)


def _final_order(x):
    """Double.compare order of a final aggregation value."""
    x = float(x)
    if math.isnan(x):
        return (1, 0.0, 0)
    return (0, x, 1 if math.copysign(1.0, x) > 0 else 0)


def server_table(qc, groups: dict) -> dict:
    """The server's combine table (GroupByUtils.createIndexedTableForCombineOperator, GroupByUtils.java:104-149;
    IndexedTable.finish) over the combined groups: without ORDER BY the first LIMIT groups (taken in
    ascending group-key order: the key compares its last group-by column first, each column in dictionary
    order); with ORDER BY the top trimSize = max(5 * LIMIT, minServerGroupTrimSize) groups by the ORDER BY
    on final values (ties in ascending key order), none dropped when minServerGroupTrimSize <= 0. Two cases
    keep LIMIT groups instead: serverReturnFinalResult without HAVING (GroupByUtils.java:134-139), and a safe
    trim -- ORDER BY expressions = GROUP BY expressions as sets, QueryContext.java:746-747 -- with LIMIT below
    sortAggregateLimitThreshold, where CombinePlanNode.java:150-154 picks the sorted combine whose merger keeps
    LIMIT records (SortedGroupByCombineOperator, GroupByUtils.getSortedReduceMerger).
    Returns the kept groups (a dict in the table's order)."""
    keys = sorted(groups, key=lambda k: tuple(_value_order(v) for v in reversed(k)))
    if not qc.order_by:
        return {k: groups[k] for k in keys[:qc.limit]}
    targets = qc.order_by_targets()
    rank = {k: i for i, k in enumerate(keys)}

    def sort_key(k):
        parts = []
        for kind, idx, asc in targets:
            if kind == 0:
                o = _value_order(k[idx])
            else:
                o = _final_order(final(qc.aggregations[idx].func, groups[k][idx]))
            parts.append(o if asc else _Desc(o))
        return tuple(parts) + (rank[k],)
    ordered = sorted(keys, key=sort_key)
    same_keys = all(kind == 0 for kind, _, _ in targets) and \
        sorted({idx for _, idx, _ in targets}) == list(range(len(qc.group_by)))
    if (same_keys and qc.limit < getattr(qc, "sort_aggregate_limit_threshold", 10_000)) or \
            getattr(qc, "server_return_final_result", False):
        trim = qc.limit
    else:
        trim = max(5 * qc.limit, qc.min_server_group_trim_size) if qc.min_server_group_trim_size > 0 else len(ordered)
    return {k: groups[k] for k in ordered[:trim]}


def segment_trim(qc, per_segment: list) -> dict:
    """The segments' own trim, then the combine's merge of what they keep (GroupByOperator.java:152-172): a
    segment holding more groups than trimSize keeps its top trimSize by the ORDER BY (TableResizer), trimSize from
    QueryContext.calculateEffectiveSegmentGroupTrimSize (QueryContext.java:568-580):
    * a safe trim -- ORDER BY expressions = GROUP BY expressions as sets, no HAVING (QueryContext.java:746-747) --
      keeps LIMIT groups, ordered by the group values;
    * an unsafe trim with minSegmentGroupTrimSize > 0 keeps max(5 * LIMIT, minSegmentGroupTrimSize) groups
      (GroupByUtils.getTableCapacity, GroupByUtils.java:63-66), ordered by the ORDER BY on group values and final
      aggregation values (extractFinalResult, Double.compare order); groups tied on every ORDER BY expression
      in ascending group-key order (the order server_table breaks ties in: TableResizer's heap leaves them
      unspecified, this restatement and the device both pin it);
    * otherwise (minSegmentGroupTrimSize <= 0, the default: CommonConstants.java:1436) no segment trims.
    Groups outside the global top LIMIT can thus carry partial results (only the segments whose top they made).
    per_segment: one {key: [partials]} dict per segment. Returns the combined {key: [partials]}."""
    targets = qc.order_by_targets() if qc.order_by else []
    safe = bool(targets) and all(kind == 0 for kind, _, _ in targets) and \
        sorted({idx for _, idx, _ in targets}) == list(range(len(qc.group_by)))
    min_seg = getattr(qc, "min_segment_group_trim_size", -1)
    if safe:
        trim = qc.limit
    elif targets and min_seg > 0:
        trim = max(5 * qc.limit, min_seg)
    else:
        trim = -1
    out = {}
    for groups in per_segment:
        keep = list(groups)
        if trim > 0 and len(groups) > trim:
            def sk(k):
                parts = []
                for kind, idx, asc in targets:
                    if kind == 0:
                        o = _value_order(k[idx])
                    else:
                        o = _final_order(final(qc.aggregations[idx].func, groups[k][idx]))
                    parts.append(o if asc else _Desc(o))
                return tuple(parts) + (tuple(_value_order(v) for v in reversed(k)),)
            keep = sorted(groups, key=sk)[:trim]
        for k in keep:
            if k not in out:
                out[k] = list(groups[k])
            else:
                out[k] = [merge(a.func, x, y) for a, x, y in zip(qc.aggregations, out[k], groups[k])]
    return out


class _Desc:
    """Reverses the order of a sort key component (descending ORDER BY)."""
    __slots__ = ("v",)

    def __init__(self, v):
        self.v = v

    def __lt__(self, other):
        return other.v < self.v

    def __eq__(self, other):
        return self.v == other.v
