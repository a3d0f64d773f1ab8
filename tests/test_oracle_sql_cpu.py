"""The oracle's own SQL front end (oracle/oracle_sql.py) against the product's (pinot_amd.query.parse_sql):
two independent compilations of every query the tests and benchmarks run must agree on the filter's CNF
leaves, aggregations, GROUP BY, ORDER BY, LIMIT and query options; and the product's host-mirror server
table (used for folded DISTINCTCOUNT groups) must keep what the oracle's restatement keeps."""
import random

import pytest

import oracle_sql
from oracle_reduce import server_table as oracle_server_table
from pinot_amd import datagen, ssb
from pinot_amd.query import parse_sql, server_table

CORPUS = [
    datagen.BENCH_QUERY, datagen.README_QUERY, datagen.HIGHCARD_QUERY, datagen.HIGHCARD_DEFAULT_QUERY,
    datagen.WIDEKEYS_QUERY, *[datagen.inverted_query(s) for s in datagen.INVERTED_SELECTIVITIES],
    *[sql for _, sql in ssb.SSB_QUERIES],
    "SELECT COUNT(*) FROM t",
    "SELECT d0, COUNT(*), SUM(r_long) FROM t WHERE NOT (d0 < 5 OR d1 IN (1, 2, 3)) GROUP BY d0 LIMIT 7",
    "SET minServerGroupTrimSize = 4; SELECT d0, d1, SUM(r_long), AVG(r_int) FROM t GROUP BY d0, d1 "
    "ORDER BY SUM(r_long) DESC LIMIT 3",
    "SET serverReturnFinalResult = true; SET sortAggregateLimitThreshold = 5; SELECT d0, MINMAXRANGE(x) AS r "
    "FROM t WHERE s NOT BETWEEN 'a' AND 'b''c' AND f >= -1.5e3 GROUP BY d0 ORDER BY d0 DESC",
    "SELECT SUMLONG(a * b), SUM(a - b), MIN(a + b), DISTINCTCOUNT(c) FROM t WHERE x <> 3 OR y != 'q' "
    "OPTION(numGroupsLimit=77)",
    "SELECT a, MAX(b) m FROM t WHERE a NOT IN ('x', 'y') AND (b > 1 AND (c = 2 OR NOT d <= 9)) GROUP BY a",
]


def _leaf(p, neg):
    return (p.type, p.column, tuple(p.values), p.lower, p.upper, p.lower_inclusive, p.upper_inclusive, neg)


@pytest.mark.parametrize("sql", CORPUS)
def test_two_front_ends_agree(sql):
    a, b = parse_sql(sql), oracle_sql.parse(sql)
    assert [[_leaf(*x) for x in cl] for cl in a.cnf] == [[_leaf(*x) for x in cl] for cl in b.cnf]
    assert [(x.func, x.column, x.expr, x.name) for x in a.aggregations] == \
           [(x.func, x.column, x.expr, x.name) for x in b.aggregations]
    assert a.group_by == b.group_by and a.limit == b.limit
    assert [(e.lower(), asc) for e, asc in a.order_by] == [(e.lower(), asc) for e, asc in b.order_by]
    if a.order_by:
        assert a.order_by_targets() == b.order_by_targets()
    for k in ("num_groups_limit", "min_server_group_trim_size", "group_trim_threshold",
              "server_return_final_result", "sort_aggregate_limit_threshold"):
        assert getattr(a, k) == getattr(b, k), k


@pytest.mark.parametrize("sql", [
    "SELECT a, b, COUNT(*), SUM(x) FROM t GROUP BY a, b LIMIT 3",
    "SET minServerGroupTrimSize = 2; SELECT a, b, COUNT(*), SUM(x) FROM t GROUP BY a, b ORDER BY SUM(x) DESC LIMIT 1",
    "SELECT a, b, COUNT(*), SUM(x) FROM t GROUP BY a, b ORDER BY b DESC, a LIMIT 4",
    "SET serverReturnFinalResult = true; SELECT a, b, COUNT(*), SUM(x) FROM t GROUP BY a, b ORDER BY COUNT(*) LIMIT 2",
    "SET sortAggregateLimitThreshold = 3; SET minServerGroupTrimSize = 6; SELECT a, b, COUNT(*), SUM(x) FROM t "
    "GROUP BY a, b ORDER BY a, b LIMIT 4",
])
def test_host_mirror_server_table_matches_oracle(sql):
    rnd = random.Random(sql)
    groups = {(rnd.randrange(6), rnd.choice(["p", "q", "é", "\U0001f600"])): [rnd.randrange(5), rnd.random()]
              for _ in range(40)}
    got = server_table(parse_sql(sql), groups)
    exp = oracle_server_table(oracle_sql.parse(sql), groups)
    assert list(got) == list(exp)
