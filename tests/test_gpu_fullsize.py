"""Parity at BASELINE.json's full size (configs[1]: 1B rows in 100 segments of 10M rows, the bench
table and query) through size-independent properties, since the oracle cannot run 1B rows in a test:

* combine linearity: the result over all 100 segments equals the AggregationFunction.merge of the
  results over two disjoint segment subsets (GroupByCombineOperator's merge; exact for COUNT, integer
  SUM and MAX, 1e-12 relative for double SUM);
* per-segment spot checks: the first and last segment through the HIP path equal the CPU oracle;
* counting identities: COUNT(*) without a filter is 1e9; the COUNTs of a range, of everything below it
  and of everything above it add up to 1e9; the group COUNTs add up to numDocsMatched.

Subset results are merged with the oracle's own AggregationFunction.merge restatement
(oracle_reduce.merge), not the product's.
"""
import math

import pytest

import oracle
from oracle_reduce import merge as merge_partial
from pinot_amd import datagen

pytestmark = pytest.mark.gpu

NSEG, ROWS = 100, 10_000_000
RTOL = 1e-12  # double SUM: order-dependent in both implementations (north_star tolerance)


@pytest.fixture(scope="module")
def table():
    import torch
    assert torch.cuda.is_available(), "GPU tests need a visible MI355X"
    from pinot_amd import engine as E
    segs, spot = [], {}
    for i in range(NSEG):
        b = datagen.ad_segment(f"full{i}", ROWS, seed=i)
        segs.append(E.ImmutableSegment(b))
        if i in (0, NSEG - 1):
            spot[i] = b
        del b
    return E, segs, spot


def _close(a, b):
    if isinstance(a, float):
        return math.isclose(a, b, rel_tol=RTOL, abs_tol=0.0)
    return a == b


@pytest.mark.timeout(900)
def test_full_size_combine_linearity(table):
    E, segs, _ = table
    ex = E.ServerQueryExecutor()
    q = datagen.BENCH_QUERY
    full = ex.execute(q, segs)
    assert full.kernel_info().startswith("jit")
    g_full = full.groups()
    a = ex.execute(q, segs[:37]).groups()
    b = ex.execute(q, segs[37:]).groups()
    funcs = ["COUNT", "SUM", "SUM", "SUM", "MAX"]
    merged = dict(a)
    for k, v in b.items():
        merged[k] = [merge_partial(f, x, y) for f, x, y in zip(funcs, merged[k], v)] if k in merged else v
    assert set(merged) == set(g_full) and len(g_full) == 201
    for k, v in g_full.items():
        for i, (x, y) in enumerate(zip(v, merged[k])):
            assert _close(x, y), (k, i, x, y)
    assert sum(v[0] for v in g_full.values()) == full.num_docs_matched()


@pytest.mark.timeout(900)
def test_full_size_counting_identities(table):
    E, segs, _ = table
    ex = E.ServerQueryExecutor()
    lo, hi = datagen.DAYS_BASE + 100, datagen.DAYS_BASE + 300
    (total,) = ex.execute("SELECT COUNT(*) FROM t", segs).groups()[()]
    assert total == NSEG * ROWS
    parts = [ex.execute(f"SELECT COUNT(*) FROM t WHERE {w}", segs).groups()[()][0]
             for w in (f"daysSinceEpoch BETWEEN {lo} AND {hi}", f"daysSinceEpoch < {lo}", f"daysSinceEpoch > {hi}")]
    assert sum(parts) == total
    clicks = [ex.execute(f"SELECT COUNT(*) FROM t WHERE {w}", segs).groups()[()][0]
              for w in ("clicks > 100", "clicks <= 100")]
    assert sum(clicks) == total


@pytest.mark.timeout(900)
def test_full_size_spot_segments_vs_oracle(table):
    E, segs, spot = table
    ex = E.ServerQueryExecutor()
    q = datagen.BENCH_QUERY
    for i, bufs in spot.items():
        got = ex.execute(q, [segs[i]]).groups()
        _, exp = oracle.execute(q, [bufs])
        assert set(got) == set(exp)
        for k, e in exp.items():
            for j, (x, y) in enumerate(zip(got[k], e)):
                assert _close(x, y), (i, k, j, x, y)


@pytest.mark.timeout(900)
def test_full_size_readme_query_vs_oracle(table):
    """configs[0]'s own query (README.md:95-100: an 8-day range AND an IN list, SUM(clicks), SUM(impressions)
    GROUP BY daysSinceEpoch) on the bench table: the 10M-row segments 0 and 99 equal the oracle, and the
    100-segment result equals the merge of two disjoint subsets."""
    E, segs, spot = table
    ex = E.ServerQueryExecutor()
    q = datagen.README_QUERY
    for i, bufs in spot.items():
        got = ex.execute(q, [segs[i]]).groups()
        _, exp = oracle.execute(q, [bufs])
        assert len(exp) == 8 and set(got) == set(exp), (i, sorted(got), sorted(exp))
        for k, e in exp.items():
            assert got[k] == e, (i, k, got[k], e)  # integer SUMs: exact
    full = ex.execute(q, segs)
    g = full.groups()
    a = ex.execute(q, segs[:61]).groups()
    for k, v in ex.execute(q, segs[61:]).groups().items():
        a[k] = [merge_partial(f, x, y) for f, x, y in zip(["SUM", "SUM"], a[k], v)] if k in a else v
    # SUM(impressions) passes 2^53: each subset's exact sum is rounded once, so their double merge may differ
    # from the whole table's by an ulp (the 1e-12 relative bound of north_star)
    assert set(a) == set(g) and len(g) == 8
    for k in g:
        assert all(_close(x, y) for x, y in zip(g[k], a[k])), (k, g[k], a[k])


# ------------------------------------------------------------------ configs[3] at full per-GPU size
@pytest.fixture(scope="module")
def highcard_table():
    import torch
    assert torch.cuda.is_available(), "GPU tests need a visible MI355X"
    from pinot_amd import engine as E
    segs, spot = [], {}
    for i in range(NSEG):
        b = datagen.highcard_segment(f"hc{i}", ROWS, seed=1000 + i)
        segs.append(E.ImmutableSegment(b))
        if i in (0, NSEG - 1):
            spot[i] = b
        del b
    return E, segs, spot


@pytest.mark.timeout(900)
def test_full_size_highcard_partitioned_vs_atomic_and_linearity(highcard_table, monkeypatch):
    """configs[3] per GPU: 1B rows in 100 segments, ~1M (dimA, dimB) groups. The partitioned plan
    (count / scatter / LDS-aggregate) must equal the direct HBM-atomic plan group by group (COUNT,
    integer SUM, MIN(LONG), MAX(DOUBLE) are all order-independent, so exactly), the result must be the
    merge of two disjoint segment subsets, and the first segment must equal the oracle."""
    E, segs, spots = highcard_table
    spot = spots[0]
    q = datagen.HIGHCARD_QUERY
    ex = E.ServerQueryExecutor()
    monkeypatch.setenv("PINOT_AMD_PARTITIONED", "1")
    part = ex.execute(q, segs)
    assert "partitioned" in part.kernel_info(), part.kernel_info()
    assert not part.num_groups_limit_reached()
    g_part = part.groups()
    assert len(g_part) > 900_000
    assert sum(v[0] for v in g_part.values()) == part.num_docs_matched()
    a = ex.execute(q, segs[:50]).groups()
    b = ex.execute(q, segs[50:]).groups()
    funcs = ["COUNT", "SUM", "MIN", "MAX"]
    for k, v in b.items():
        a[k] = [merge_partial(f, x, y) for f, x, y in zip(funcs, a[k], v)] if k in a else v
    assert a == g_part
    del a, b
    monkeypatch.setenv("PINOT_AMD_PARTITIONED", "0")
    atomic = ex.execute(q, segs)
    assert "partitioned" not in atomic.kernel_info()
    assert atomic.groups() == g_part
    got = ex.execute(q, [segs[0]]).groups()
    _, exp = oracle.execute(q, [spot])
    assert got == exp


@pytest.mark.timeout(900)
def test_full_size_highcard_default_limit_vs_oracle(highcard_table, monkeypatch):
    """configs[3]'s query as Pinot runs it by default (numGroupsLimit 100000 < 1M keys per segment), on the
    default plan (sequential admission over segment prefixes + partitioned aggregation of admitted docs):
    segments 0 and 99 equal the oracle's literal first-seen admission (DictionaryBasedGroupKeyGenerator
    .java:1017-1040) including numGroupsLimitReached; the 100-segment result equals the merge of two
    disjoint subsets (admission is per segment); segment 0 is the same on the first-doc admission."""
    E, segs, spots = highcard_table
    q = datagen.HIGHCARD_DEFAULT_QUERY
    ex = E.ServerQueryExecutor()
    full = ex.execute(q, segs)
    assert "+admit-seq" in full.kernel_info(), full.kernel_info()
    assert full.num_groups_limit_reached()
    g_full = full.groups()
    assert sum(v[0] for v in g_full.values()) < full.num_docs_matched()  # dropped docs were scanned
    for i, bufs in spots.items():
        r = ex.execute(q, [segs[i]])
        stats = {}
        _, exp = oracle.execute(q, [bufs], stats=stats)
        assert len(exp) == 100_000
        assert r.num_groups_limit_reached() == stats["num_groups_limit_reached"] is True
        assert r.groups() == exp, i
    funcs = ["COUNT", "SUM", "MIN", "MAX"]
    a = ex.execute(q, segs[:50]).groups()
    for k, v in ex.execute(q, segs[50:]).groups().items():
        a[k] = [merge_partial(f, x, y) for f, x, y in zip(funcs, a[k], v)] if k in a else v
    assert a == g_full
    monkeypatch.setenv("PINOT_AMD_ADMIT_SEQ", "0")
    r = ex.execute(q, [segs[0]])
    assert "+admit" in r.kernel_info() and "+admit-seq" not in r.kernel_info(), r.kernel_info()
    _, exp = oracle.execute(q, [spots[0]])
    assert r.groups() == exp


# ------------------------------------------------------------------ configs[4] at full size (SF100)
@pytest.mark.timeout(900)
def test_full_size_ssb_sf100_linearity_and_oracle_segment():
    """configs[4]: SSB SF100 denormalized lineorder, 600M rows in 60 segments (bench's generator). For
    each of the 13 queries, the 60-segment result equals the merge of two disjoint subsets (keys
    exactly, SUMs within 1e-12 relative: they are double sums of CASTs/products), and segment 0
    equals the CPU oracle."""
    import torch
    assert torch.cuda.is_available()
    from pinot_amd import engine as E
    from pinot_amd import ssb
    from pinot_amd.query import parse_sql
    segs, spot = [], None
    for i in range(60):
        b = ssb.lineorder_flat_segment(f"lo{i}", ROWS, seed=2000 + i)
        segs.append(E.ImmutableSegment(b))
        if i == 0:
            spot = b
        del b
    ex = E.ServerQueryExecutor()

    def same(g, e, what):
        assert set(g) == set(e), what
        for k in e:
            for x, y in zip(g[k], e[k]):
                assert _close(x, y), (what, k, x, y)

    for name, q in ssb.SSB_QUERIES:
        funcs = [a.func for a in parse_sql(q).aggregations]
        full = ex.execute(q, segs).groups()
        a = ex.execute(q, segs[:23]).groups()
        for k, v in ex.execute(q, segs[23:]).groups().items():
            a[k] = [merge_partial(f, x, y) for f, x, y in zip(funcs, a[k], v)] if k in a else v
        same(full, a, name)
        _, exp = oracle.execute(q, [spot])
        same(ex.execute(q, [segs[0]]).groups(), exp, name + " segment 0")


# ------------------------------------------------------------------ configs[2] at full per-GPU size
@pytest.mark.timeout(900)
def test_full_size_inverted_sweep_vs_oracle_and_linearity(monkeypatch):
    """configs[2] at bench scale: 100 segments x 10M rows (the bench's 4 distinct inverted-index segments,
    each staged 25 times), every selectivity of the sweep under the default cost model (word-level
    select + gather at 0.01-1 %, the fused forward-index scan at 10-50 %): segments 0 and 99 equal the
    CPU oracle (which expands the same RoaringBitmaps), the 100-segment result equals the merge of two
    disjoint subsets, COUNT equals numDocsMatched, and at 1 % the selection-vector and fused plans agree
    on the whole table."""
    import torch
    assert torch.cuda.is_available()
    from pinot_amd import engine as E
    distinct = [datagen.inverted_segment(f"inv{i}", ROWS, seed=i) for i in range(4)]
    segs = [E.ImmutableSegment(distinct[i % 4]) for i in range(NSEG)]
    ex = E.ServerQueryExecutor()
    funcs = ["COUNT", "SUM", "SUM"]
    for sel in datagen.INVERTED_SELECTIVITIES:
        q = datagen.inverted_query(sel)
        full = ex.execute(q, segs)
        g = full.groups()[()]
        assert g[0] == full.num_docs_matched()
        a = ex.execute(q, segs[:41]).groups()[()]
        b = ex.execute(q, segs[41:]).groups()[()]
        m = [merge_partial(f, x, y) for f, x, y in zip(funcs, a, b)]
        assert all(_close(x, y) for x, y in zip(g, m)), (sel, g, m)
        for i in (0, NSEG - 1):
            got = ex.execute(q, [segs[i]]).groups()[()]
            _, exp = oracle.execute(q, [distinct[i % 4]])
            assert all(_close(x, y) for x, y in zip(got, exp[()])), (sel, i, got, exp)
        if sel == 0.01:
            plans = {}
            for pol in ("always", "never"):
                monkeypatch.setenv("PINOT_AMD_SELECT", pol)
                r = ex.execute(q, segs)
                plans[pol] = (r.kernel_info(), r.groups()[()])
            monkeypatch.delenv("PINOT_AMD_SELECT")
            assert "select" in plans["always"][0] and "select" not in plans["never"][0], plans
            x, y = plans["always"][1], plans["never"][1]
            assert x[0] == y[0] and x[1] == y[1] and _close(x[2], y[2]), plans
