"""The oracle's restatement of the segment-level trim (oracle_reduce.segment_trim; GroupByOperator.java:157-175,
QueryContext.calculateEffectiveSegmentGroupTrimSize :568-580) on hand-made per-segment results."""
import oracle_sql
from oracle_reduce import segment_trim, server_table


def _qc(sql):
    return oracle_sql.parse(sql)


def test_safe_trim_keeps_each_segments_top_limit():
    qc = _qc("SET sortAggregateLimitThreshold = 1; SELECT a, COUNT(*) FROM t GROUP BY a ORDER BY a LIMIT 2")
    s0 = {(1,): [5], (2,): [1], (3,): [7]}   # keeps 1, 2
    s1 = {(2,): [4], (3,): [2], (4,): [9]}   # keeps 2, 3
    s2 = {(3,): [1]}                          # one group: nothing to trim
    got = segment_trim(qc, [s0, s1, s2])
    assert got == {(1,): [5], (2,): [5], (3,): [3]}   # group 3: the partials of s1 and s2 only; 4 dropped
    # the top LIMIT groups are exact: the combine table over the trimmed union keeps them first
    assert list(server_table(qc, got))[:2] == [(1,), (2,)]


def test_desc_and_multi_column_order():
    qc = _qc("SET sortAggregateLimitThreshold = 1; SELECT a, b, SUM(x) FROM t GROUP BY a, b ORDER BY b DESC, a LIMIT 2")
    s0 = {(1, 1): [1], (2, 1): [2], (1, 2): [3], (3, 2): [4]}
    # order: b DESC then a ASC -> (1,2), (3,2), (1,1), (2,1): keeps (1,2), (3,2)
    assert segment_trim(qc, [s0]) == {(1, 2): [3], (3, 2): [4]}


def test_unsafe_order_does_not_trim_segments():
    # ORDER BY an aggregation: unsafe trim, minSegmentGroupTrimSize -1 (default): segments keep everything
    qc = _qc("SELECT a, COUNT(*) FROM t GROUP BY a ORDER BY COUNT(*) DESC LIMIT 1")
    s0 = {(1,): [5], (2,): [1]}
    s1 = {(2,): [4]}
    assert segment_trim(qc, [s0, s1]) == {(1,): [5], (2,): [5]}
