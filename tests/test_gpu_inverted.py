"""GPU parity for inverted-index filters (BASELINE.json configs[2]): EQ/IN predicates evaluated
through the bitmap inverted index (BitmapBasedFilterOperator over BitmapInvertedIndexReader,
pinot-core/.../operator/filter/BitmapBasedFilterOperator.java) or through the forward index, as the
cost model (or PINOT_AMD_INV_POLICY) picks, combined with AND/OR across columns; RoaringBitmap
array, bitmap and run containers; aggregation and filter-only docId sets against the CPU oracle."""
import numpy as np
import pytest

import oracle
from pinot_amd import datagen
from pinot_amd import segment as S
from pinot_amd.query import parse_sql

pytestmark = pytest.mark.gpu

from test_gpu_parity import assert_same_groups  # noqa: E402


@pytest.fixture(scope="module")
def engine():
    import torch
    assert torch.cuda.is_available(), "GPU tests need a visible MI355X"
    from pinot_amd import engine as E
    return E


@pytest.fixture(scope="module")
def inv_segments(engine):
    bufs = [datagen.inverted_segment(f"inv{i}", n, seed=i) for i, n in enumerate((200_003, 65_536, 131_071))]
    return bufs, [engine.ImmutableSegment(b) for b in bufs]


@pytest.mark.parametrize("policy", ["always", "never", "cost"])
@pytest.mark.parametrize("sel", datagen.INVERTED_SELECTIVITIES)
def test_inverted_sweep_vs_oracle(engine, inv_segments, policy, sel, monkeypatch):
    monkeypatch.setenv("PINOT_AMD_INV_POLICY", policy)
    bufs, segs = inv_segments
    q = datagen.inverted_query(sel)
    res = engine.ServerQueryExecutor().execute(q, segs)
    nm, og = oracle.execute(q, bufs)
    assert res.num_docs_matched() == nm
    if nm == 0:
        og = {(): og[()]}
    assert_same_groups(res.groups(), og, {2})
    # filter-only: ascending docIds per segment (FilterPlanNode -> BlockDocIdSet)
    ids = engine.ServerQueryExecutor().filter_doc_ids(q, segs)
    qc = parse_sql(q)
    for b, got in zip(bufs, ids):
        bits, cnt = oracle.OracleSegment(b).filter_bitset(qc)
        exp = np.nonzero(np.unpackbits(bits.view(np.uint8), bitorder="little")[:b.num_docs])[0]
        assert np.array_equal(got, exp)


def _container_segment(n, seed):
    """Columns whose bitmaps hold bitmap containers (2-value column), run containers (clustered
    values) and array containers (sparse values)."""
    rng = np.random.default_rng(seed)
    cols = {
        "two": (rng.integers(0, 2, n).astype(np.int32), S.INT, {"inverted": True}),
        "clustered": ((np.arange(n) // 5000 % 40).astype(np.int32), S.INT, {"inverted": True, "detect_sorted": False}),
        "sparse": (rng.integers(0, 3000, n).astype(np.int32), S.INT, {"inverted": True}),
        "m": (rng.integers(-500, 500, n).astype(np.int64), S.LONG, {"dictionary": False}),
    }
    return S.build_segment(f"cont{seed}", cols)


@pytest.mark.parametrize("q", [
    "SELECT COUNT(*), SUM(m) FROM t WHERE two = 1",
    "SELECT COUNT(*), SUM(m) FROM t WHERE clustered IN (0, 3, 17, 39) OR sparse IN (5, 77, 2999)",
    "SELECT COUNT(*), SUM(m) FROM t WHERE two = 0 AND clustered NOT IN (1, 2) AND sparse BETWEEN 100 AND 2000",
    "SELECT clustered, COUNT(*), MAX(m) FROM t WHERE two <> 1 OR sparse = 12 GROUP BY clustered",
])
def test_roaring_container_kinds(engine, q, monkeypatch):
    monkeypatch.setenv("PINOT_AMD_INV_POLICY", "always")
    bufs = [_container_segment(n, i) for i, n in enumerate((300_001, 70_000))]
    segs = [engine.ImmutableSegment(b) for b in bufs]
    res = engine.ServerQueryExecutor().execute(q, segs)
    nm, og = oracle.execute(q, bufs)
    assert res.num_docs_matched() == nm
    assert_same_groups(res.groups(), og)


def test_leaf_cache_reissued_filters(engine, inv_segments, monkeypatch):
    """Predicate leaves resolved once per segment (the segment's leaf cache) serve re-issued filters: the
    same queries interleaved, re-executed through fresh results while earlier results are still alive and
    after they are destroyed (their blocks back in the device pool), each against the oracle."""
    monkeypatch.setenv("PINOT_AMD_INV_POLICY", "always")
    bufs, segs = inv_segments
    ex = engine.ServerQueryExecutor()
    qs = [datagen.inverted_query(s) for s in datagen.INVERTED_SELECTIVITIES[:3]]
    exp = {q: oracle.execute(q, bufs) for q in qs}
    alive = []
    for rnd in range(3):
        for q in qs:
            res = ex.execute(q, segs)
            nm, og = exp[q]
            assert res.num_docs_matched() == nm
            assert_same_groups(res.groups(), og if nm else {(): og[()]}, {2})
            if rnd == 1:
                alive.append(res)  # held across the next round's executions of the same leaves
            else:
                res.destroy()
    for res in alive:
        res.destroy()


@pytest.mark.parametrize("plan", ["scan", "select"])
@pytest.mark.parametrize("q", [
    "SELECT COUNT(*), SUM(m) FROM t WHERE NOT two = 1",
    "SELECT COUNT(*), SUM(m) FROM t WHERE sparse IN (5, 77, 2999) OR m > 400",
    "SELECT clustered, COUNT(*), SUM(m) FROM t WHERE NOT clustered IN (0, 3) AND two = 0 GROUP BY clustered",
])
def test_bitset_leaves_outside_gates_with_tile_groups(engine, q, plan, monkeypatch):
    """DocId-bitset leaves that are not gates (negated, OR-ed with a column leaf) read their bitset words per lane
    in every step of a 4-tile group, padding tiles and steps past the block's range included: segments whose
    tile counts are not multiples of 4 (1, 5, 7 tiles), fused scan and tile-level select, against the oracle
    (the bitsets carry slack behind their words for those reads)."""
    monkeypatch.setenv("PINOT_AMD_INV_POLICY", "always")
    if plan == "scan":
        monkeypatch.setenv("PINOT_AMD_SELECT", "never")
        monkeypatch.setenv("PINOT_AMD_SCAN_GROUP", "4")
        monkeypatch.setenv("PINOT_AMD_FILTER_GATE", "0")
    else:
        monkeypatch.setenv("PINOT_AMD_SELECT", "always")
        monkeypatch.setenv("PINOT_AMD_SEL_GROUP", "4")
    bufs = [_container_segment(n, 20 + i) for i, n in enumerate((300, 5000, 7 * 1024 + 3))]
    segs = [engine.ImmutableSegment(b) for b in bufs]
    res = engine.ServerQueryExecutor().execute(q, segs)
    nm, og = oracle.execute(q, bufs)
    assert res.num_docs_matched() == nm
    assert_same_groups(res.groups(), og if nm else {(): og[()]})
