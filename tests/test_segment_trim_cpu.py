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


def test_unsafe_trim_keeps_max_of_min_and_five_limits():
    # minSegmentGroupTrimSize 3 > 5 x LIMIT 0? no: LIMIT 1 -> 5 x 1 = 5 > 3 -> each segment keeps 5 groups by COUNT DESC
    qc = _qc("SET minSegmentGroupTrimSize = 3; SELECT a, COUNT(*) FROM t GROUP BY a ORDER BY COUNT(*) DESC LIMIT 1")
    s0 = {(i,): [10 - i] for i in range(8)}      # keeps 0..4 (counts 10..6)
    s1 = {(7,): [100], (6,): [1]}                 # two groups: nothing trimmed
    got = segment_trim(qc, [s0, s1])
    assert got == {(0,): [10], (1,): [9], (2,): [8], (3,): [7], (4,): [6], (7,): [100], (6,): [1]}
    # minSegmentGroupTrimSize above 5 x LIMIT wins
    qc = _qc("SET minSegmentGroupTrimSize = 7; SELECT a, COUNT(*) FROM t GROUP BY a ORDER BY COUNT(*) DESC LIMIT 1")
    assert set(segment_trim(qc, [s0])) == {(i,) for i in range(7)}


def test_unsafe_trim_final_values_and_ties():
    # AVG final values (sum / count) order the trim; ties (equal AVG) in ascending group-key order
    qc = _qc("SET minSegmentGroupTrimSize = 2; SELECT a, b, AVG(x) FROM t GROUP BY a, b ORDER BY AVG(x) LIMIT 0")
    s0 = {(5, 1): [(10.0, 2)], (1, 2): [(5.0, 1)], (2, 1): [(4.0, 1)], (0, 0): [(1.0, 1)]}
    # AVG: (5,1) 5.0, (1,2) 5.0, (2,1) 4.0, (0,0) 1.0 -> ascending keeps (0,0), (2,1)
    assert set(segment_trim(qc, [s0])) == {(0, 0), (2, 1)}
    qc = _qc("SET minSegmentGroupTrimSize = 3; SELECT a, b, AVG(x) FROM t GROUP BY a, b ORDER BY AVG(x) DESC LIMIT 0")
    # DESC: 5.0, 5.0 tied -> ascending key (last column first): (5,1) before (1,2); then 4.0
    assert set(segment_trim(qc, [s0])) == {(5, 1), (1, 2), (2, 1)}
    qc = _qc("SET minSegmentGroupTrimSize = 1; SELECT a, b, AVG(x) FROM t GROUP BY a, b ORDER BY AVG(x) DESC LIMIT 0")
    assert set(segment_trim(qc, [s0])) == {(5, 1)}


def test_unsafe_trim_mixed_key_and_aggregation_order():
    qc = _qc("SET minSegmentGroupTrimSize = 2; SELECT a, MAX(x) FROM t GROUP BY a ORDER BY MAX(x) DESC, a DESC LIMIT 0")
    s0 = {(1,): [3.0], (2,): [3.0], (3,): [1.0], (4,): [2.0]}
    assert set(segment_trim(qc, [s0])) == {(2,), (1,)}
