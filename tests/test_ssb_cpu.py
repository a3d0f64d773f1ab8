"""SSB (denormalized lineorder) on the CPU oracle against the golden results restated from the
reference's SSB quickstart data and query set (tests/golden/make_ssb_golden.py): pins the oracle's
expression aggregations (times / minus transforms), STRING dictionary predicates and multi-column
STRING/INT group keys before the GPU path is compared with it."""
import math

import pytest

import oracle
from helpers import load_ssb_expected, ssb_flat_segment
from pinot_amd.query import parse_sql

EXP = load_ssb_expected()


@pytest.fixture(scope="module")
def flat():
    return ssb_flat_segment()


@pytest.mark.parametrize("qi", range(len(EXP["queries"])), ids=[q["name"] for q in EXP["queries"]])
def test_ssb_oracle_matches_golden(flat, qi):
    q = EXP["queries"][qi]
    nm, groups = oracle.execute(q["sql"], flat)
    exp = {tuple(g[:-1]): g[-1] for g in q["groups"]}
    if not q["group_by"]:
        assert math.isclose(groups[()][0], exp[()], rel_tol=1e-12) if nm else exp == {}
        return
    got = {k: v[0] for k, v in groups.items()}
    assert set(got) == set(exp)
    for k in exp:
        assert got[k] == exp[k], (k, got[k], exp[k])


def test_ssb_parse_expressions():
    qc = parse_sql("select sum(CAST(LO_EXTENDEDPRICE AS DOUBLE) * LO_DISCOUNT) as revenue from t")
    a = qc.aggregations[0]
    assert a.expr == ("MUL", "LO_EXTENDEDPRICE", "LO_DISCOUNT") and a.name == "revenue"
    assert a.column == "times(LO_EXTENDEDPRICE,LO_DISCOUNT)"
    qc = parse_sql("select D_YEAR, sum(LO_REVENUE - LO_SUPPLYCOST) profit from t group by D_YEAR")
    assert qc.aggregations[0].expr == ("SUB", "LO_REVENUE", "LO_SUPPLYCOST")
    assert qc.aggregations[0].alias == "profit"
    assert parse_sql("select sum(CAST(a AS DOUBLE)), b from t group by b").aggregations[0].expr is None
