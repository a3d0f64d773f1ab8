"""Host-side reduce semantics of the aggregations composed above the device accumulators
(AggregationFunction.merge / extractFinalResult): AVG, MINMAXRANGE, DISTINCTCOUNT, and the
DISTINCTCOUNT query split (one grouped query per DISTINCTCOUNT column)."""
from pinot_amd.query import final_value, fold_distinct_count, merge_partial, parse_sql, split_distinct_count


def test_merge_and_final_values():
    assert final_value("AVG", merge_partial("AVG", (3.0, 1), (5.0, 3))) == 2.0
    assert final_value("AVG", (0.0, 0)) == float("-inf")
    assert final_value("MINMAXRANGE", merge_partial("MINMAXRANGE", (2.0, 9.0), (-1.0, 4.0))) == 10.0
    assert final_value("MINMAXRANGE", (float("inf"), float("-inf"))) == float("-inf")
    assert final_value("DISTINCTCOUNT", merge_partial("DISTINCTCOUNT", frozenset({1, 2}), frozenset({2, 3}))) == 3


def test_distinct_count_split_and_fold():
    qc = parse_sql("SELECT g, DISTINCTCOUNT(a), SUM(b), DISTINCTCOUNT(c) FROM t WHERE b > 1 GROUP BY g")
    base, subs = split_distinct_count(qc)
    assert [a.func for a in base.aggregations] == ["SUM"] and base.group_by == ["g"]
    assert [(i, s.group_by, [a.func for a in s.aggregations]) for i, s in subs] == \
        [(0, ["g", "a"], ["COUNT"]), (2, ["g", "c"], ["COUNT"])]
    assert all(s.filter == qc.filter for _, s in subs)
    groups = fold_distinct_count(qc, {(1,): [10.0], (2,): [4.0]},
                                 [(0, {(1, 5): [2], (1, 6): [1], (2, 5): [1]}), (2, {(1, 0): [3], (2, 7): [1]})])
    assert groups == {(1,): [frozenset({5, 6}), 10.0, frozenset({0})], (2,): [frozenset({5}), 4.0, frozenset({7})]}


def test_server_table_restatement():
    """oracle_reduce.server_table: LIMIT groups in key order without ORDER BY; the top
    max(5 * LIMIT, minServerGroupTrimSize) by the ORDER BY otherwise (ties by key)."""
    import sys, os
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
    from oracle_reduce import server_table
    from oracle_sql import parse as parse_sql
    groups = {(k % 5, k // 5): [k, float(100 - k)] for k in range(40)}
    qc = parse_sql("SELECT a, b, COUNT(*), SUM(x) FROM t GROUP BY a, b LIMIT 3")
    kept = server_table(qc, groups)
    assert list(kept) == [(0, 0), (1, 0), (2, 0)]  # key order: last column first
    qc = parse_sql("SET minServerGroupTrimSize = 2; SELECT a, b, COUNT(*), SUM(x) FROM t GROUP BY a, b "
                   "ORDER BY SUM(x) DESC LIMIT 1")
    assert list(server_table(qc, groups)) == [(0, 0), (1, 0), (2, 0), (3, 0), (4, 0)]  # max(5 * 1, 2)
    qc = parse_sql("SET minServerGroupTrimSize = 7; SELECT a, b, COUNT(*), SUM(x) FROM t GROUP BY a, b "
                   "ORDER BY a DESC, COUNT(*) LIMIT 1")
    assert list(server_table(qc, groups))[:3] == [(4, 0), (4, 1), (4, 2)] and len(server_table(qc, groups)) == 7
