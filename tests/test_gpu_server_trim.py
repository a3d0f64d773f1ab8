"""The server's combine table on the device (pinot_amd_query_set_result_limit / add_order_by: GroupByUtils
.createIndexedTableForCombineOperator + IndexedTable.finish) against the oracle's restatement
(oracle_reduce.server_table): LIMIT groups without ORDER BY; the top max(5 * LIMIT, minServerGroupTrimSize)
by ORDER BY on group columns and final aggregation values (AVG, MIN, SUM) otherwise; trimming disabled
with minServerGroupTrimSize <= 0; LIMIT groups under a safe trim (ORDER BY = GROUP BY) below
sortAggregateLimitThreshold and with serverReturnFinalResult; DISTINCTCOUNT folded before the table;
through the dense and hash plans; and every SSB query (their ORDER BYs are mostly safe trims)."""
import numpy as np
import pytest

import oracle
from helpers import random_segment
from oracle_reduce import server_table
from pinot_amd.query import parse_sql

pytestmark = pytest.mark.gpu

from test_gpu_parity import assert_same_groups  # noqa: E402

QUERIES = [
    "SELECT d0, COUNT(*), SUM(r_long) FROM t WHERE r_int > 0 GROUP BY d0 LIMIT 7",
    "SET minServerGroupTrimSize = 4; SELECT d0, d1, SUM(r_long), AVG(r_int) FROM t GROUP BY d0, d1 "
    "ORDER BY SUM(r_long) DESC LIMIT 3",
    "SET minServerGroupTrimSize = 30; SELECT d1, MIN(r_double), COUNT(*) FROM t GROUP BY d1 "
    "ORDER BY d1 DESC, MIN(r_double) LIMIT 2",
    "SET minServerGroupTrimSize = 20; SELECT d0, AVG(r_int), MAX(r_double) FROM t GROUP BY d0 "
    "ORDER BY AVG(r_int) LIMIT 5",
    "SET minServerGroupTrimSize = -1; SELECT d1, COUNT(*) FROM t GROUP BY d1 ORDER BY COUNT(*) DESC LIMIT 1",
    # safe trim (ORDER BY keys = GROUP BY keys): the sorted combine keeps LIMIT groups
    "SELECT d0, d1, COUNT(*), SUM(r_long) FROM t GROUP BY d0, d1 ORDER BY d1, d0 DESC LIMIT 6",
    "SET serverReturnFinalResult = true; SELECT d0, SUM(r_long), COUNT(*) FROM t GROUP BY d0 "
    "ORDER BY SUM(r_long) DESC LIMIT 4",
    # DISTINCTCOUNT: the value sets are folded first, then the table (round-3 advisor: a LIMIT on the
    # (group, value) sub-queries cut the sets)
    "SET minServerGroupTrimSize = 3; SELECT d0, DISTINCTCOUNT(d1), COUNT(*) FROM t GROUP BY d0 "
    "ORDER BY DISTINCTCOUNT(d1) DESC LIMIT 2",
    "SELECT d0, DISTINCTCOUNT(d1) FROM t GROUP BY d0 LIMIT 5",
]


@pytest.mark.parametrize("plan", ["auto", "hash"])
@pytest.mark.parametrize("qi", range(len(QUERIES)))
def test_server_table_vs_oracle(qi, plan, monkeypatch):
    import torch
    assert torch.cuda.is_available()
    from pinot_amd import engine as E
    if plan == "hash":
        monkeypatch.setenv("PINOT_AMD_GROUP_PLAN", "hash")
    rng = np.random.default_rng(50 + qi)
    bufs = [random_segment(rng, 30_000 + 1_000 * i, name=f"st{i}", bits_cards=(300, 37)) for i in range(3)]
    segs = [E.ImmutableSegment(b) for b in bufs]
    qc = parse_sql(QUERIES[qi])
    got = E.ServerQueryExecutor(server_trim=True).execute(qc, segs).groups()
    _, full = oracle.execute(QUERIES[qi], bufs)
    exp = server_table(oracle.parse_sql(QUERIES[qi]), full)
    assert len(got) == len(exp) <= len(full)
    fsum = {i for i, a in enumerate(qc.aggregations) if a.func in ("SUM", "AVG") and a.column == "r_double"}
    assert_same_groups(got, exp, fsum)
    if qc.order_by:  # the table is sorted by the ORDER BY
        assert list(got) == list(exp)


SEG_TRIM_QUERIES = [
    # safe trim (ORDER BY = GROUP BY) with LIMIT >= sortAggregateLimitThreshold: each segment keeps its top LIMIT
    # groups (GroupByOperator.java:157-175), the combine table the top max(5 x LIMIT, minServerGroupTrimSize) of
    # what they kept -- groups past the global top LIMIT carry the partials of the segments that kept them
    "SET sortAggregateLimitThreshold = 5; SET minServerGroupTrimSize = 50; SELECT d0, COUNT(*), SUM(r_long) FROM t "
    "GROUP BY d0 ORDER BY d0 LIMIT 8",
    "SET sortAggregateLimitThreshold = 5; SET minServerGroupTrimSize = 200; SELECT d0, d1, COUNT(*), MIN(r_double), "
    "AVG(r_int) FROM t WHERE r_int > 0 GROUP BY d0, d1 ORDER BY d1 DESC, d0 LIMIT 20",
    "SET sortAggregateLimitThreshold = 10; SET minServerGroupTrimSize = -1; SELECT d1, d0, MAX(r_long) FROM t "
    "GROUP BY d1, d0 ORDER BY d0 DESC, d1 DESC LIMIT 30",
    # and with numGroupsLimit trimming first (each segment admits its first 500 groups, then trims to LIMIT)
    "SET numGroupsLimit = 500; SET sortAggregateLimitThreshold = 5; SET minServerGroupTrimSize = 100; "
    "SELECT d0, d1, COUNT(*) FROM t GROUP BY d0, d1 ORDER BY d0, d1 LIMIT 12",
]


@pytest.mark.parametrize("plan", ["auto", "partitioned"])
@pytest.mark.parametrize("qi", range(len(SEG_TRIM_QUERIES)))
def test_segment_level_safe_trim_vs_oracle(qi, plan, monkeypatch):
    """The segment-level safe trim on the device (a presence pass over ORDER BY ranks, each segment's LIMIT-th
    rank as its cutoff, the aggregation keeping the docs within it) against the oracle's restatement: every
    segment trimmed to its top LIMIT by the ORDER BY (oracle_reduce.segment_trim), then the combine table."""
    import torch
    assert torch.cuda.is_available()
    from oracle_reduce import segment_trim
    from pinot_amd import engine as E
    if plan == "partitioned":  # the key space leaves the LDS: the partitioned count / scatter passes trim
        monkeypatch.setenv("PINOT_AMD_WIDE_LDS", "0")
    rng = np.random.default_rng(90 + qi)
    bufs = [random_segment(rng, 25_000 + 3_000 * i, name=f"sg{i}", bits_cards=(300, 37)) for i in range(3)]
    segs = [E.ImmutableSegment(b) for b in bufs]
    q = SEG_TRIM_QUERIES[qi]
    qc = parse_sql(q)
    res = E.ServerQueryExecutor(server_trim=True).execute(qc, segs)
    got = res.groups()
    oq = oracle.parse_sql(q)
    per_seg = [oracle.execute(q, [b])[1] for b in bufs]
    assert max(len(g) for g in per_seg) > qc.limit  # some segment trims
    exp = server_table(oq, segment_trim(oq, per_seg))
    _, full = oracle.execute(q, bufs)
    assert exp != server_table(oq, full)  # the segment trim changes the server's result
    assert len(got) == len(exp)
    assert_same_groups(got, exp, set())
    assert list(got) == list(exp)
    if plan == "partitioned" and len(qc.group_by) > 1:
        assert "partitioned" in res.kernel_info()


def test_segment_level_safe_trim_untrimmed_segments():
    """No segment can hold more than LIMIT groups: nothing to trim (the plan takes no presence pass)."""
    import torch
    assert torch.cuda.is_available()
    from pinot_amd import engine as E
    rng = np.random.default_rng(7)
    bufs = [random_segment(rng, 20_000, name="sf0", bits_cards=(300, 37))]
    segs = [E.ImmutableSegment(b) for b in bufs]
    q2 = "SET sortAggregateLimitThreshold = 5; SELECT d0, COUNT(*) FROM t WHERE d0 < 3 GROUP BY d0 ORDER BY d0 LIMIT 5"
    got = E.ServerQueryExecutor(server_trim=True).execute(q2, segs).groups()
    _, full = oracle.execute(q2, bufs)
    assert got == server_table(oracle.parse_sql(q2), full)


UNSAFE_TRIM_QUERIES = [
    # unsafe trim (an ORDER BY other than the GROUP BY keys) with minSegmentGroupTrimSize > 0: each segment keeps its
    # top max(minSegmentGroupTrimSize, 5 x LIMIT) groups by the ORDER BY on final values (QueryContext.java:568-580)
    "SET minSegmentGroupTrimSize = 10; SELECT d0, COUNT(*) FROM t GROUP BY d0 ORDER BY COUNT(*) DESC LIMIT 2",
    "SET minSegmentGroupTrimSize = 40; SET minServerGroupTrimSize = 60; SELECT d0, d1, SUM(r_long), AVG(r_int) FROM t "
    "GROUP BY d0, d1 ORDER BY SUM(r_long) DESC LIMIT 3",
    "SET minSegmentGroupTrimSize = 5; SELECT d0, AVG(r_int), MAX(r_double) FROM t WHERE r_int > 0 GROUP BY d0 "
    "ORDER BY AVG(r_int) LIMIT 6",
    "SET minSegmentGroupTrimSize = 25; SELECT d1, d0, MIN(r_double), COUNT(*) FROM t GROUP BY d1, d0 "
    "ORDER BY d1 DESC, MIN(r_double) LIMIT 4",
    "SET minSegmentGroupTrimSize = 30; SELECT d0, MINMAXRANGE(r_int), SUMLONG(r_long) FROM t GROUP BY d0 "
    "ORDER BY MINMAXRANGE(r_int) DESC, SUMLONG(r_long) LIMIT 5",
    # after numGroupsLimit admission (each segment's first 500 groups, then its top 50 by COUNT)
    "SET numGroupsLimit = 500; SET minSegmentGroupTrimSize = 50; SELECT d0, d1, COUNT(*), SUM(r_long) FROM t "
    "GROUP BY d0, d1 ORDER BY COUNT(*) DESC, SUM(r_long) LIMIT 3",
]


@pytest.mark.parametrize("plan", ["auto", "hash"])
@pytest.mark.parametrize("qi", range(len(UNSAFE_TRIM_QUERIES)))
def test_unsafe_segment_trim_vs_oracle(qi, plan, monkeypatch):
    """The unsafe segment trim on the device (the (key, segment) hash plan, then per segment a radix selection of
    its top entries over the ORDER BY's stage keys -- group ids, final aggregation values in Double.compare order,
    the key words for ties) against oracle_reduce.segment_trim then server_table. Ties on every ORDER BY
    expression go in ascending group-key order on both sides (TableResizer's heap leaves them unspecified)."""
    import torch
    assert torch.cuda.is_available()
    from oracle_reduce import segment_trim
    from pinot_amd import engine as E
    if plan == "hash":
        monkeypatch.setenv("PINOT_AMD_GROUP_PLAN", "hash")
    rng = np.random.default_rng(130 + qi)
    bufs = [random_segment(rng, 20_000 + 2_000 * i, name=f"su{i}", bits_cards=(300, 37)) for i in range(3)]
    segs = [E.ImmutableSegment(b) for b in bufs]
    q = UNSAFE_TRIM_QUERIES[qi]
    qc = parse_sql(q)
    got = E.ServerQueryExecutor(server_trim=True).execute(qc, segs).groups()
    oq = oracle.parse_sql(q)
    per_seg = [oracle.execute(q, [b])[1] for b in bufs]
    keep = max(5 * qc.limit, oq.min_segment_group_trim_size)
    assert max(len(g) for g in per_seg) > keep  # some segment trims
    trimmed = segment_trim(oq, per_seg)
    exp = server_table(oq, trimmed)
    _, full = oracle.execute(q, bufs)
    assert trimmed != full  # the segment trim drops or cuts groups
    assert len(got) == len(exp)
    assert_same_groups(got, exp, set())
    assert list(got) == list(exp)


def test_unsafe_segment_trim_untrimmed_segments():
    """minSegmentGroupTrimSize above every segment's group count: nothing to trim (the plan keeps its kind)."""
    import torch
    assert torch.cuda.is_available()
    from pinot_amd import engine as E
    rng = np.random.default_rng(9)
    bufs = [random_segment(rng, 20_000, name="su0", bits_cards=(300, 37))]
    segs = [E.ImmutableSegment(b) for b in bufs]
    q2 = "SET minSegmentGroupTrimSize = 1000; SELECT d0, COUNT(*) FROM t GROUP BY d0 ORDER BY COUNT(*) DESC LIMIT 2"
    got = E.ServerQueryExecutor(server_trim=True).execute(q2, segs).groups()
    _, full = oracle.execute(q2, bufs)
    assert list(got) == list(server_table(oracle.parse_sql(q2), full))


@pytest.mark.parametrize("plan", ["hash", "cap"])
@pytest.mark.parametrize("qi", range(len(SEG_TRIM_QUERIES)))
def test_segment_level_safe_trim_hash_plan_vs_oracle(qi, plan, monkeypatch):
    """The segment-level safe trim over a hash plan's key space (forced, or a key space past the dense cap): the
    (key, segment) scan table, each segment's top LIMIT entries by the ORDER BY's group ids (segsel), against the
    oracle's segment_trim then server_table."""
    import torch
    assert torch.cuda.is_available()
    from oracle_reduce import segment_trim
    from pinot_amd import engine as E
    if plan == "hash":
        monkeypatch.setenv("PINOT_AMD_GROUP_PLAN", "hash")
    else:
        monkeypatch.setenv("PINOT_AMD_DENSE_MAX_KEYS", "64")
    rng = np.random.default_rng(90 + qi)
    bufs = [random_segment(rng, 25_000 + 3_000 * i, name=f"sg{i}", bits_cards=(300, 37)) for i in range(3)]
    segs = [E.ImmutableSegment(b) for b in bufs]
    q = SEG_TRIM_QUERIES[qi]
    qc = parse_sql(q)
    got = E.ServerQueryExecutor(server_trim=True).execute(qc, segs).groups()
    oq = oracle.parse_sql(q)
    per_seg = [oracle.execute(q, [b])[1] for b in bufs]
    assert max(len(g) for g in per_seg) > qc.limit
    exp = server_table(oq, segment_trim(oq, per_seg))
    assert len(got) == len(exp)
    assert_same_groups(got, exp, set())
    assert list(got) == list(exp)


def test_ssb_server_table_vs_oracle():
    """Every SSB query with the server's combine table on the device, over segments with different
    dictionaries, against oracle_reduce.server_table of the oracle's groups."""
    import torch
    assert torch.cuda.is_available()
    from pinot_amd import engine as E
    from pinot_amd import ssb
    bufs = [ssb.lineorder_flat_segment(f"st{i}", 200_003 + i, seed=40 + i) for i in range(3)]
    segs = [E.ImmutableSegment(b) for b in bufs]
    for name, sql in ssb.SSB_QUERIES:
        qc = parse_sql(sql)
        if not qc.group_by:
            continue
        got = E.ServerQueryExecutor(server_trim=True).execute(qc, segs).groups()
        _, full = oracle.execute(sql, bufs)
        exp = server_table(oracle.parse_sql(sql), full)
        assert list(got) == list(exp), name
        assert_same_groups(got, exp, set(range(len(qc.aggregations))))
