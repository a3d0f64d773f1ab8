"""GPU parity of filter-gated fused scans (JitPlan::filter_gate: the filter columns load two steps ahead, the
whole CNF is evaluated a step ahead into a per-lane mask, and the group-key / value columns load only for
lanes holding a matching doc). Forced with PINOT_AMD_FILTER_GATE=1 (and the selection-vector plan off, so the
fused scan runs) over the random-query sweep, multi-segment dictionaries and the 13 SSB queries, against the
CPU oracle and the SSB golden results; and the planner's own choice on the SF-scaled SSB segments."""
import numpy as np
import pytest

import oracle
from helpers import load_ssb_expected, random_segment, ssb_flat_segment
from pinot_amd import ssb
from pinot_amd.query import parse_sql

pytestmark = pytest.mark.gpu

from test_gpu_parity import QUERIES, assert_same_groups  # noqa: E402

EXP = load_ssb_expected()


@pytest.fixture(scope="module")
def engine():
    import torch
    assert torch.cuda.is_available(), "GPU tests need a visible MI355X"
    from pinot_amd import engine as E
    return E


@pytest.fixture
def gate(monkeypatch):
    monkeypatch.setenv("PINOT_AMD_FILTER_GATE", "1")
    monkeypatch.setenv("PINOT_AMD_SELECT", "never")
    monkeypatch.setenv("PINOT_AMD_INV_POLICY", "never")  # column filters (docId-bitset leaves take their own gate)


def _gated(res, qc):
    info = res.kernel_info()
    assert info.startswith("jit"), info
    # dense plans with a filter and an aggregation take the gate when forced
    if qc.filter is not None and "hash" not in info and "partitioned" not in info:
        assert "+fgate" in info, info


@pytest.mark.parametrize("qi", range(len(QUERIES)))
@pytest.mark.parametrize("n", [1, 1000, 250_007])
def test_gated_random_queries_vs_oracle(engine, gate, qi, n):
    rng = np.random.default_rng(qi * 31 + n)
    bufs = random_segment(rng, n, inverted=("d1",))
    seg = engine.ImmutableSegment(bufs)
    q = QUERIES[qi]
    qc = parse_sql(q)
    fsum = {i for i, a in enumerate(qc.aggregations) if a.func in ("SUM", "AVG") and a.column == "r_double"}
    res = engine.ServerQueryExecutor(False).execute(qc, [seg])
    _gated(res, qc)
    nm, og = oracle.execute(q, [bufs], False)
    assert res.num_docs_matched() == nm
    got = res.groups()
    if not qc.group_by and nm == 0:
        og = {(): og[()]}
    assert_same_groups(got, og, fsum)


def test_gated_multi_segment_ragged(engine, gate):
    """Segments of ragged sizes (tiles straddling segment ends, a one-doc segment) with different
    dictionaries: the gate's segment walk runs two tiles ahead of the processing."""
    rng = np.random.default_rng(5)
    bufs = [random_segment(rng, n, name=f"g{i}", inverted=()) for i, n in enumerate((1, 1023, 1025, 70_001, 4096, 3))]
    segs = [engine.ImmutableSegment(b) for b in bufs]
    for q in QUERIES[1:7]:
        qc = parse_sql(q)
        fsum = {i for i, a in enumerate(qc.aggregations) if a.func in ("SUM", "AVG") and a.column == "r_double"}
        res = engine.ServerQueryExecutor(False).execute(qc, segs)
        _gated(res, qc)
        nm, og = oracle.execute(q, bufs, False)
        assert res.num_docs_matched() == nm, q
        got = res.groups()
        if not qc.group_by and nm == 0:
            og = {(): og[()]}
        assert_same_groups(got, og, fsum)


@pytest.mark.parametrize("split", [1, 3], ids=["one_segment", "three_segments"])
def test_gated_ssb_golden(engine, gate, split):
    bufs = ssb_flat_segment(split=split if split > 1 else None)
    segs = [engine.ImmutableSegment(b) for b in bufs]
    for q in EXP["queries"]:
        res = engine.ServerQueryExecutor().execute(q["sql"], segs)
        _gated(res, parse_sql(q["sql"]))
        got = {k: v[0] for k, v in res.groups().items()}
        exp = {tuple(g[:-1]): g[-1] for g in q["groups"]}
        if not q["group_by"]:
            assert got[()] == exp.get((), 0.0), q["name"]
        else:
            assert got == exp, q["name"]


def test_planner_choice_on_ssb_segments(engine, monkeypatch):
    """The opt-in cost model's choice (PINOT_AMD_FILTER_GATE=auto: gate or not, select or not) on the SF-scaled
    generator's segments."""
    monkeypatch.setenv("PINOT_AMD_FILTER_GATE", "auto")
    bufs = [ssb.lineorder_flat_segment(f"fg{i}", 200_003 + i, seed=10 + i) for i in range(2)]
    segs = [engine.ImmutableSegment(b) for b in bufs]
    for name, sql in ssb.SSB_QUERIES:
        res = engine.ServerQueryExecutor().execute(sql, segs)
        nm, og = oracle.execute(sql, bufs)
        assert res.num_docs_matched() == nm, name
        got = res.groups()
        if not parse_sql(sql).group_by and nm == 0:
            og = {(): og[()]}
        assert got == og, (name, res.kernel_info())
