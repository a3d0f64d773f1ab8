"""GPU parity for the Star Schema Benchmark on the denormalized lineorder (BASELINE.json configs[4]):
the 13 queries of the reference's ssb_query_set.yaml in flat form over the reference's SSB
quickstart data, against the golden results (tests/golden/make_ssb_golden.py) and the CPU oracle:
expression aggregations (times / minus), STRING dictionary predicates (EQ, RANGE, OR of EQs) and
STRING/INT multi-column group keys, on one segment and split into segments with different
dictionaries (merged key space)."""
import pytest

import oracle
from helpers import load_ssb_expected, ssb_flat_segment
from pinot_amd import ssb
from pinot_amd.query import parse_sql

pytestmark = pytest.mark.gpu

EXP = load_ssb_expected()


@pytest.fixture(scope="module")
def engine():
    import torch
    assert torch.cuda.is_available(), "GPU tests need a visible MI355X"
    from pinot_amd import engine as E
    return E


@pytest.fixture(scope="module", params=[1, 3], ids=["one_segment", "three_segments"])
def flat(request, engine):
    bufs = ssb_flat_segment(split=request.param if request.param > 1 else None)
    return bufs, [engine.ImmutableSegment(b) for b in bufs]


@pytest.mark.parametrize("qi", range(len(EXP["queries"])), ids=[q["name"] for q in EXP["queries"]])
def test_ssb_golden(engine, flat, qi, monkeypatch):
    bufs, segs = flat
    q = EXP["queries"][qi]
    res = engine.ServerQueryExecutor().execute(q["sql"], segs)
    assert res.kernel_info().startswith("jit")
    nm, og = oracle.execute(q["sql"], bufs)
    assert res.num_docs_matched() == nm
    got = {k: v[0] for k, v in res.groups().items()}
    exp = {tuple(g[:-1]): g[-1] for g in q["groups"]}
    if not q["group_by"]:
        assert got[()] == exp.get((), 0.0)
    else:
        assert got == exp
    assert got == {k: v[0] for k, v in og.items()} or not q["group_by"]


@pytest.mark.parametrize("name", ["Q1.1", "Q2.1", "Q3.1", "Q3.3", "Q4.1"])
def test_ssb_through_hash_plan(engine, flat, name, monkeypatch):
    """The same queries through the hash-table GROUP BY plan (forced), against the oracle."""
    monkeypatch.setenv("PINOT_AMD_GROUP_PLAN", "hash")
    bufs, segs = flat
    sql = dict(ssb.SSB_QUERIES)[name]
    res = engine.ServerQueryExecutor().execute(sql, segs)
    if parse_sql(sql).group_by:
        assert "hash" in res.kernel_info()
    nm, og = oracle.execute(sql, bufs)
    got = res.groups()
    if not parse_sql(sql).group_by and nm == 0:
        og = {(): og[()]}
    assert got == og


def test_ssb_synthetic_segment_vs_oracle(engine, monkeypatch):
    """The SF-scaled generator's segments (bench input) through every query, against the oracle."""
    bufs = [ssb.lineorder_flat_segment(f"lf{i}", 150_001 + i, seed=i) for i in range(2)]
    segs = [engine.ImmutableSegment(b) for b in bufs]
    for name, sql in ssb.SSB_QUERIES:
        res = engine.ServerQueryExecutor().execute(sql, segs)
        nm, og = oracle.execute(sql, bufs)
        assert res.num_docs_matched() == nm, name
        got = res.groups()
        if not parse_sql(sql).group_by and nm == 0:
            og = {(): og[()]}
        assert got == og, name
