"""Selection-vector plans (late materialisation): a select pass over the filter columns appends the
matching docIds, a gather pass decodes only the group-by / aggregated columns of those docs by random
access and aggregates them. Forced on (PINOT_AMD_SELECT=always) for every plan kind it serves —
aggregation only, LDS table, CU-wide LDS table, HBM table, hash table — across segment boundaries,
sorted / raw / fixed-bit / inverted-index columns and expressions, against the oracle; and chosen by
the planner's cost model for a selective query over wide value columns."""
import os
import sys

import numpy as np
import pytest

from pinot_amd import segment as S
from helpers import random_segment

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle  # noqa: E402
from test_gpu_parity import assert_same_groups  # noqa: E402


@pytest.fixture(scope="module")
def engine():
    import torch
    assert torch.cuda.is_available()
    from pinot_amd import engine as E
    return E


@pytest.fixture(scope="module")
def data(engine):
    rng = np.random.default_rng(2024)
    bufs = [random_segment(rng, n, name=f"sel{i}", bits_cards=(3000, 37, 9000), inverted=("d1",), sorted_col=True,
                           float_col=True)
            for i, n in enumerate([1, 70_001, 255, 256, 257, 131_072, 99_999])]
    return bufs, [engine.ImmutableSegment(b) for b in bufs]


QUERIES = [
    # aggregation only (register accumulators)
    "SELECT COUNT(*), SUM(r_long), MIN(r_double), MAX(r_int), AVG(r_int) FROM t WHERE d0 < 40",
    # LDS table (37 groups), filter on a raw column and a dictionary column
    "SELECT d1, COUNT(*), SUM(r_int), MAX(r_double), SUM(r_long) FROM t WHERE r_int BETWEEN 0 AND 30000 AND d0 < 900 GROUP BY d1",
    # inverted-index leaf + raw IN, group by the sorted column
    "SELECT ts, COUNT(*), SUM(r_double), MIN(r_long) FROM t WHERE d1 IN (10, 17, 73) OR r_int IN (5, 77, 1000) GROUP BY ts",
    # CU-wide LDS table (37 x 300 keys) and an expression
    "SELECT d1, fd, COUNT(*), SUM(r_int * d1), MAX(r_long) FROM t WHERE d2 < 700 GROUP BY d1, fd",
    # HBM table (3000 x 37 keys)
    "SELECT d0, d1, COUNT(*), SUM(r_long), MIN(r_int) FROM t WHERE d2 BETWEEN 100 AND 600 AND r_double > 0 GROUP BY d0, d1",
    # nothing matches / everything matches
    "SELECT d1, COUNT(*), SUM(r_int) FROM t WHERE r_int > 2000000000 GROUP BY d1",
    "SELECT COUNT(*), SUM(r_int) FROM t WHERE r_int > -2000000000",
]


@pytest.mark.parametrize("qi", range(len(QUERIES)))
@pytest.mark.parametrize("plan", ["auto", "hash"])
def test_forced_select_vs_oracle(engine, data, monkeypatch, qi, plan):
    monkeypatch.setenv("PINOT_AMD_SELECT", "always")
    if plan == "hash":
        monkeypatch.setenv("PINOT_AMD_GROUP_PLAN", "hash")
    else:  # the HBM-table query's 111k keys would otherwise take the partitioned plan
        monkeypatch.setenv("PINOT_AMD_PARTITIONED", "0")
    bufs, segs = data
    q = QUERIES[qi]
    res = engine.ServerQueryExecutor().execute(q, segs)
    assert "select" in res.kernel_info(), res.kernel_info()
    nm, og = oracle.execute(q, bufs)
    assert res.num_docs_matched() == nm
    from pinot_amd.query import parse_sql
    qc = parse_sql(q)
    fs = {i for i, a in enumerate(qc.aggregations) if a.func in ("SUM", "AVG") and
          (a.column == "r_double" or (a.expr is not None and a.expr[0] != "COL"))}
    assert_same_groups(res.groups(), og, fs)
    res.execute_again()
    assert_same_groups(res.groups(), og, fs)  # idempotent re-execution (vector counters reset)
    assert res.algorithmic_bytes() > 0


@pytest.mark.parametrize("group", ["1", "2"])
@pytest.mark.parametrize("qi", range(len(QUERIES)))
def test_select_tile_groups_vs_oracle(engine, data, monkeypatch, qi, group):
    """The select pass walks G tiles of one segment per loop step (default 4) over tile ranges padded to
    multiples of G; 1 and 2 here, on the same ragged segments (1 .. 131072 docs: padding tiles in most
    of them), must give the oracle's result too."""
    monkeypatch.setenv("PINOT_AMD_SELECT", "always")
    monkeypatch.setenv("PINOT_AMD_PARTITIONED", "0")
    monkeypatch.setenv("PINOT_AMD_SEL_GROUP", group)
    bufs, segs = data
    q = QUERIES[qi]
    res = engine.ServerQueryExecutor().execute(q, segs)
    assert "select" in res.kernel_info(), res.kernel_info()
    nm, og = oracle.execute(q, bufs)
    assert res.num_docs_matched() == nm
    from pinot_amd.query import parse_sql
    qc = parse_sql(q)
    fs = {i for i, a in enumerate(qc.aggregations) if a.func in ("SUM", "AVG") and
          (a.column == "r_double" or (a.expr is not None and a.expr[0] != "COL"))}
    assert_same_groups(res.groups(), og, fs)


def test_cost_model_picks_select_for_selective_wide_rows(engine, monkeypatch):
    """0.3 % of docs pass a filter on a 6-bit column while the query aggregates three wide raw columns:
    the planner takes the selection-vector plan on its own; at 50 % it keeps the fused scan."""
    monkeypatch.delenv("PINOT_AMD_SELECT", raising=False)
    rng = np.random.default_rng(8)
    n = 2_000_000
    f = rng.integers(0, 1000, n).astype(np.int32)
    bufs = S.build_segment("wide", {
        "f": (f, S.INT, {}),
        "g": (rng.integers(0, 50, n).astype(np.int32), S.INT, {}),
        "a": (rng.integers(-(1 << 40), 1 << 40, n), S.LONG, {"dictionary": False}),
        "b": (rng.normal(0, 1, n), S.DOUBLE, {"dictionary": False}),
        "c": (rng.integers(0, 1 << 30, n).astype(np.int32), S.INT, {"dictionary": False})})
    seg = engine.ImmutableSegment(bufs)
    ex = engine.ServerQueryExecutor()
    for where, expect in (("f < 3", True), ("f < 500", False)):
        q = f"SELECT g, COUNT(*), SUM(a), MAX(b), SUM(c) FROM t WHERE {where} GROUP BY g"
        res = ex.execute(q, [seg])
        assert ("select" in res.kernel_info()) == expect, (where, res.kernel_info())
        _, og = oracle.execute(q, [bufs])
        assert_same_groups(res.groups(), og, {2})


WORD_QUERIES = [
    "SELECT COUNT(*), SUM(r_long), MAX(r_double), MIN(r_int) FROM t WHERE d1 IN (10, 17, 73) AND ts BETWEEN 5 AND 40",
    "SELECT d0, COUNT(*), SUM(r_int) FROM t WHERE d1 NOT IN (3, 10) OR ts < 3 GROUP BY d0",
    "SELECT ts, COUNT(*), SUM(r_double) FROM t WHERE d1 = 24 GROUP BY ts",
    "SELECT COUNT(*), SUM(r_int) FROM t WHERE d1 IN (10, 17) AND ts > 100",  # nothing matches
]


@pytest.mark.parametrize("fused", ["1", "0"], ids=["fused", "expand+wselect"])
@pytest.mark.parametrize("qi", range(len(WORD_QUERIES)))
def test_word_select_vs_oracle(engine, data, monkeypatch, qi, fused):
    """Filters that read no column (inverted-index bitsets, sorted-index docId ranges, constants) select
    on 64-doc words: ragged segment sizes (1 .. 131072 docs, partial last words), negation, OR/AND --
    fused with the roaring expansion (roaring_select_kernel, the default) and as expansion + word select."""
    monkeypatch.setenv("PINOT_AMD_SELECT", "always")
    monkeypatch.setenv("PINOT_AMD_INV_POLICY", "always")
    monkeypatch.setenv("PINOT_AMD_FUSED_INV_SELECT", fused)
    bufs, segs = data
    q = WORD_QUERIES[qi]
    res = engine.ServerQueryExecutor().execute(q, segs)
    assert "wselect" in res.kernel_info(), res.kernel_info()
    nm, og = oracle.execute(q, bufs)
    assert res.num_docs_matched() == nm
    from pinot_amd.query import parse_sql
    qc = parse_sql(q)
    fs = {i for i, a in enumerate(qc.aggregations) if a.func == "SUM" and a.column == "r_double"}
    assert_same_groups(res.groups(), og, fs)
    res.execute_again()
    assert_same_groups(res.groups(), og, fs)


_D2_SET = ", ".join(str(7 * v + 3) for v in range(0, 9000, 29))  # 311 values of the 9000-entry dictionary
SET_QUERIES = [
    f"SELECT COUNT(*), SUM(r_long), MAX(r_double) FROM t WHERE d2 IN ({_D2_SET})",
    f"SELECT d1, COUNT(*), SUM(r_int) FROM t WHERE d2 NOT IN ({_D2_SET}) AND d0 < 2000 GROUP BY d1",
    f"SELECT d0, COUNT(*), MIN(r_long) FROM t WHERE d2 IN ({_D2_SET}) OR r_int > 900000 GROUP BY d0",
]


@pytest.mark.parametrize("sel", ["never", "always"])
@pytest.mark.parametrize("qi", range(len(SET_QUERIES)))
def test_lds_dictid_sets_vs_oracle(engine, data, monkeypatch, qi, sel):
    """IN / NOT IN over a 9000-entry dictionary (282 bitmap words: above the lane-register tables) read
    from an LDS copy of the segment's dictId set, in the fused scan (aggregation only, LDS table, HBM
    table) and in the select pass, across segment changes inside a block's tile range."""
    monkeypatch.setenv("PINOT_AMD_SELECT", sel)
    monkeypatch.setenv("PINOT_AMD_PARTITIONED", "0")
    bufs, segs = data
    q = SET_QUERIES[qi]
    res = engine.ServerQueryExecutor().execute(q, segs)
    nm, og = oracle.execute(q, bufs)
    assert res.num_docs_matched() == nm
    from pinot_amd.query import parse_sql
    qc = parse_sql(q)
    fs = {i for i, a in enumerate(qc.aggregations) if a.func == "SUM" and a.column == "r_double"}
    assert_same_groups(res.groups(), og, fs)
