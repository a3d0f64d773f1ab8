"""Pin the CPU oracle to the reference: expected values hard-coded in Pinot's own query tests
(tests/golden/sv_queries_expected.json, transcribed from InnerSegmentAggregationSingleValueQueriesTest,
InterSegmentAggregationSingleValueQueriesTest and InterSegmentGroupBySingleValueQueriesTest) over the
segment BaseSingleValueQueriesTest builds from test_data-sv.avro."""
import math

import pytest

import oracle
from helpers import SV_FILTER, load_expected, sv_segment

EXP = load_expected()
INNER_QUERY = "SELECT COUNT(*), SUM(column1), MAX(column3), MIN(column6), AVG(column7) FROM testTable"


@pytest.fixture(scope="module")
def seg():
    return sv_segment()


def _inner_tuple(parts):
    cnt, s1, mx3, mn6, avg7 = parts
    return [cnt, int(s1), int(mx3), int(mn6), int(avg7[0]), avg7[1]]


@pytest.mark.parametrize("use_inverted", [True, False])
@pytest.mark.parametrize("with_filter", [False, True])
def test_inner_aggregation(seg, with_filter, use_inverted):
    e = EXP["inner_aggregation"]["filter" if with_filter else "no_filter"]
    n, groups = oracle.execute(INNER_QUERY + (SV_FILTER if with_filter else ""), [seg], use_inverted)
    got = _inner_tuple(groups[()])
    assert got == [e["count"], e["sum_column1"], e["max_column3"], e["min_column6"], e["avg_column7_sum"],
                   e["avg_column7_count"]]
    assert n == e["count"]
    if with_filter:
        # numEntriesScannedPostFilter = matched docs x projected columns (4)
        assert n * 4 == EXP["inner_aggregation"]["filter_stats"]["num_entries_scanned_post_filter"]


@pytest.mark.parametrize("case", EXP["inner_group_by"]["cases"], ids=lambda c: f"{len(c['group_by'])}cols-f{int(c['filter'])}")
def test_inner_group_by(seg, case):
    q = INNER_QUERY + (SV_FILTER if case["filter"] else "") + " GROUP BY " + ", ".join(case["group_by"])
    _, groups = oracle.execute(q, [seg])
    key = tuple(case["key"])
    assert key in groups, f"group {key} missing"
    assert _inner_tuple(groups[key]) == case["values"]


def _inter_query(case):
    names = []
    for i, (f, c) in enumerate(case["aggs"]):
        names.append(f"{f}({c})" + ("" if f == "COUNT" and len(case["aggs"]) == 1 and "group_by" not in case
                                   else f" AS v{i + 1}"))
    q = "SELECT " + ", ".join(names) + " FROM testTable" + (SV_FILTER if case["filter"] else "")
    if "group_by" in case:
        order = case["order"].replace("COUNT", "v1") if case["aggs"][0][0] == "COUNT" else case["order"]
        q += f" GROUP BY {case['group_by']} ORDER BY {order} LIMIT 1"
    return q


@pytest.mark.parametrize("case", EXP["inter"]["cases"], ids=lambda c: _inter_query(c)[7:60])
def test_inter_segment(seg, case):
    segs = [seg] * EXP["inter"]["num_segments"]
    rows = oracle.rows(_inter_query(case), segs)
    assert len(rows) == 1
    got = list(rows[0][1 if "group_by" in case else 0:])
    tol = case.get("rel_tol", 0.0)
    for g, e in zip(got, case["result"]):
        if tol:
            assert math.isclose(g, e, rel_tol=tol)
        else:
            assert g == e


@pytest.mark.parametrize("case", EXP["inter_group_by"]["cases"], ids=lambda c: ",".join(c["group_by"]))
def test_inter_group_by_order_by(seg, case):
    q = ("SELECT " + ", ".join(case["group_by"]) + f", SUM({case['agg'][1]}) FROM testTable GROUP BY "
         + ", ".join(case["group_by"]) + " ORDER BY " + ", ".join(case["group_by"]))
    rows = oracle.rows(q, [seg] * EXP["inter_group_by"]["num_segments"])
    assert [list(r) for r in rows] == case["rows"]
