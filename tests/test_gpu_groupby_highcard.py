"""GPU parity for high-cardinality GROUP BY (BASELINE.json configs[3]): key spaces too large for an
LDS table run the partitioned plan (count -> offsets -> scatter -> per-partition LDS aggregation,
kernel_info 'jit-partitioned'). Checked against the CPU oracle (DictionaryBasedGroupKeyGenerator's
map-based holders, pinot-core/.../groupby/DictionaryBasedGroupKeyGenerator.java:304-342) and against
the direct HBM-atomic plan (PINOT_AMD_PARTITIONED=0) on the same segments: group keys, COUNT,
integer SUM, MIN/MAX bit-exact; double SUM within 1e-12 relative."""
import numpy as np
import pytest

import oracle
from helpers import random_segment
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


def _fsum(qc):
    return {i for i, a in enumerate(qc.aggregations)
            if a.func in ("SUM", "AVG") and a.column in ("r_double", "r_float", "fd")}


HC_QUERIES = [
    "SELECT d0, d1, COUNT(*), SUM(r_int), MIN(r_long), MAX(r_double) FROM t GROUP BY d0, d1",
    "SELECT d0, d1, COUNT(*), SUM(r_long), SUM(r_double), MIN(r_int), MAX(r_int) FROM t WHERE r_int < 500000 "
    "GROUP BY d0, d1",
    "SELECT d1, d0, AVG(r_double), MAX(r_long) FROM t WHERE d0 BETWEEN 100 AND 5000 OR r_long > 0 GROUP BY d1, d0",
    "SELECT d0, d1, COUNT(*) FROM t WHERE r_double > 1e9 GROUP BY d0, d1",          # no matching doc
]


@pytest.mark.parametrize("qi", range(len(HC_QUERIES)))
@pytest.mark.parametrize("n", [1, 5000, 300_007])
def test_highcard_partitioned_vs_oracle(engine, qi, n, monkeypatch):
    monkeypatch.delenv("PINOT_AMD_PARTITIONED", raising=False)
    monkeypatch.setenv("PINOT_AMD_SELECT_PARTITIONED", "0")  # the partitioned plan even where a select would win
    rng = np.random.default_rng(1000 + qi * 7 + n)
    bufs = random_segment(rng, n, bits_cards=(1000, 1000))
    seg = engine.ImmutableSegment(bufs)
    qc = parse_sql("SET numGroupsLimit = 2000000; " + HC_QUERIES[qi])
    res = engine.ServerQueryExecutor().execute(qc, [seg])
    # a 1-doc segment has 1-entry dictionaries: its key space fits the LDS table
    assert res.kernel_info() == ("jit-partitioned" if n > 1 else "jit"), res.kernel_info()
    nm, og = oracle.execute("SET numGroupsLimit = 2000000; " + HC_QUERIES[qi], [bufs])
    assert res.num_docs_matched() == nm
    assert not res.num_groups_limit_reached()
    assert_same_groups(res.groups(), og, _fsum(qc))


@pytest.mark.parametrize("stage_cap,handover", [(None, "0"), ("0", "0"), ("4", "0"), (None, "force"), (None, None)])
def test_highcard_partitioned_equals_atomic_plan(engine, monkeypatch, stage_cap, handover):
    """Same query through the partitioned plan and the direct HBM-atomic plan: identical groups.
    stage_cap: scatter records staged per partition in LDS (None: planner's choice; 0: direct
    writes; 4: tiny staging, most records take the overflow path). handover: the partitioned
    plan's device-side switch to its direct-atomic scan ("force": always, "0": never)."""
    for var, val in (("PINOT_AMD_STAGE_CAP", stage_cap), ("PINOT_AMD_ATOMIC_HANDOVER", handover)):
        if val is None:
            monkeypatch.delenv(var, raising=False)
        else:
            monkeypatch.setenv(var, val)
    rng = np.random.default_rng(77)
    bufs = [random_segment(rng, 200_000 + 999 * i, name=f"s{i}", bits_cards=(1000, 700)) for i in range(3)]
    segs = [engine.ImmutableSegment(b) for b in bufs]
    q = ("SET numGroupsLimit = 2000000; SELECT d0, d1, COUNT(*), SUM(r_int), SUM(r_long), MIN(r_double), "
         "MAX(r_long) FROM t WHERE r_long > -100000000000 GROUP BY d0, d1")
    monkeypatch.setenv("PINOT_AMD_PARTITIONED", "1")
    rp = engine.ServerQueryExecutor().execute(q, segs)
    assert rp.kernel_info() == "jit-partitioned"
    monkeypatch.setenv("PINOT_AMD_PARTITIONED", "0")
    ra = engine.ServerQueryExecutor().execute(q, segs)
    assert ra.kernel_info() == "jit"
    gp, ga = rp.groups(), ra.groups()
    assert gp == ga
    nm, og = oracle.execute(q, bufs)
    assert rp.num_docs_matched() == nm
    assert_same_groups(gp, og)
    # re-execution (the bench step) is idempotent
    rp.execute_again()
    assert rp.groups() == gp


def test_highcard_multi_segment_merged_dictionaries(engine, monkeypatch):
    """Segments with different dictionaries: keys remapped into the merged key space, then
    partitioned; dictionary-encoded FLOAT/DOUBLE metric columns feed the records."""
    rng = np.random.default_rng(5)
    bufs = []
    for i in range(4):
        n = int(rng.integers(20_000, 120_000))
        cols = {
            "a": ((rng.integers(0, 900, n) * 3 + i).astype(np.int32), S.INT, {}),
            "b": ((rng.integers(0, 400, n) * 5).astype(np.int64), S.LONG, {}),
            "f": ((rng.integers(0, 50, n) * 0.5).astype(np.float32), S.FLOAT, {}),
            "m": (rng.normal(0, 100, n), S.DOUBLE, {"dictionary": False}),
        }
        bufs.append(S.build_segment(f"m{i}", cols))
    segs = [engine.ImmutableSegment(b) for b in bufs]
    q = ("SET numGroupsLimit = 5000000; SELECT a, b, COUNT(*), SUM(f), MIN(f), MAX(m), SUM(m) FROM t "
         "WHERE f >= 1.0 GROUP BY a, b")
    res = engine.ServerQueryExecutor().execute(q, segs)
    assert res.kernel_info() == "jit-partitioned", res.kernel_info()
    nm, og = oracle.execute(q, bufs)
    assert res.num_docs_matched() == nm
    assert_same_groups(res.groups(), og, {4})  # SUM(m): double sum, order-dependent


def test_num_groups_limit_reached_flag(engine, monkeypatch):
    rng = np.random.default_rng(9)
    bufs = random_segment(rng, 50_000, bits_cards=(1000, 1000))
    seg = engine.ImmutableSegment(bufs)
    res = engine.ServerQueryExecutor().execute("SELECT d0, d1, COUNT(*) FROM t GROUP BY d0, d1", [seg])
    assert len(res.groups()) > 10_000
    assert res.num_groups_limit_reached() is False  # 50000 docs < default limit 100000 groups
    res = engine.ServerQueryExecutor().execute(
        "SELECT d0, d1, COUNT(*) FROM t GROUP BY d0, d1 OPTION(numGroupsLimit=1000)", [seg])
    assert res.num_groups_limit_reached() is True


@pytest.mark.parametrize("wide", ["1", "0"])
def test_wide_lds_table_plan(engine, monkeypatch, wide):
    """A group table between 40 KiB and the 160 KiB workgroup LDS runs in one CU-wide block per CU
    (PINOT_AMD_WIDE_LDS=0: the partitioned plan instead); both equal the oracle."""
    monkeypatch.setenv("PINOT_AMD_WIDE_LDS", wide)
    rng = np.random.default_rng(21)
    bufs = [random_segment(rng, 250_000 + 17 * i, name=f"w{i}", bits_cards=(1000, 4)) for i in range(2)]
    segs = [engine.ImmutableSegment(b) for b in bufs]
    q = ("SELECT d0, d1, COUNT(*), SUM(r_long), MAX(r_double), MIN(r_int) FROM t WHERE r_int > -500000 "
         "GROUP BY d0, d1 OPTION(numGroupsLimit=1000000)")
    res = engine.ServerQueryExecutor().execute(q, segs)
    assert res.kernel_info() == ("jit" if wide == "1" else "jit-partitioned"), res.kernel_info()
    nm, og = oracle.execute(q, bufs)
    assert res.num_docs_matched() == nm
    assert_same_groups(res.groups(), og)


@pytest.mark.parametrize("where", ["r_int < -995000", "r_int < 0", "ts = 25", "ts BETWEEN 10 AND 12 OR r_int > 999000"])
@pytest.mark.parametrize("stride", [None, "0", "7"])
def test_highcard_sampled_handover(engine, monkeypatch, where, stride):
    """Partitioned plans over >= 64 x stride tiles first count the filter's matches on every
    stride-th tile; an extrapolated count under docs/64 skips the count pass and leaves the batch to
    the direct-atomic scan. Selective (0.25%), broad (50%) and docId-clustered (sorted `ts`) filters,
    sampling off ("0") and a non-power-of-two stride: identical groups and matched-doc count."""
    monkeypatch.delenv("PINOT_AMD_PARTITIONED", raising=False)
    monkeypatch.setenv("PINOT_AMD_SELECT_PARTITIONED", "0")
    monkeypatch.delenv("PINOT_AMD_ATOMIC_HANDOVER", raising=False)
    if stride is None:
        monkeypatch.delenv("PINOT_AMD_SAMPLE_STRIDE", raising=False)
    else:
        monkeypatch.setenv("PINOT_AMD_SAMPLE_STRIDE", stride)
    rng = np.random.default_rng(31)
    bufs = [random_segment(rng, 900_000 + 4099 * i, name=f"h{i}", bits_cards=(1000, 1000), sorted_col=True)
            for i in range(3)]
    segs = [engine.ImmutableSegment(b) for b in bufs]
    q = ("SET numGroupsLimit = 2000000; SELECT d0, d1, COUNT(*), SUM(r_int), MIN(r_long), MAX(r_double) FROM t "
         f"WHERE {where} GROUP BY d0, d1")
    res = engine.ServerQueryExecutor().execute(q, segs)
    assert res.kernel_info() == "jit-partitioned"
    nm, og = oracle.execute(q, bufs)
    assert res.num_docs_matched() == nm
    assert_same_groups(res.groups(), og)
    res.execute_again()
    assert res.num_docs_matched() == nm
    assert_same_groups(res.groups(), og)


@pytest.mark.parametrize("where", ["r_int < -995000", "ts = 25", "r_double > 1e9"])
def test_highcard_select_into_hbm_table(engine, monkeypatch, where):
    """A selective filter over a key space too large for LDS: the planner prefers the selection-vector
    plan, whose gather adds the few matching docs straight into the dense HBM table (instead of the
    partitioned plan handing over to a fused direct-atomic scan of every row). Identical groups and
    matched-doc count to the oracle, also on re-execution; PINOT_AMD_SELECT_PARTITIONED=0 keeps the
    partitioned plan (the tests above)."""
    monkeypatch.delenv("PINOT_AMD_PARTITIONED", raising=False)
    monkeypatch.delenv("PINOT_AMD_SELECT", raising=False)
    monkeypatch.delenv("PINOT_AMD_SELECT_PARTITIONED", raising=False)
    rng = np.random.default_rng(41)
    bufs = [random_segment(rng, 900_000 + 4099 * i, name=f"s{i}", bits_cards=(1000, 1000), sorted_col=True)
            for i in range(3)]
    segs = [engine.ImmutableSegment(b) for b in bufs]
    q = ("SET numGroupsLimit = 2000000; SELECT d0, d1, COUNT(*), SUM(r_int), MIN(r_long), MAX(r_double) FROM t "
         f"WHERE {where} GROUP BY d0, d1")
    res = engine.ServerQueryExecutor().execute(q, segs)
    assert "select" in res.kernel_info(), res.kernel_info()
    nm, og = oracle.execute(q, bufs)
    assert res.num_docs_matched() == nm
    assert_same_groups(res.groups(), og)
    res.execute_again()
    assert res.num_docs_matched() == nm
    assert_same_groups(res.groups(), og)


@pytest.mark.parametrize("env", [{"PINOT_AMD_FLUSH_GROUP": "1"}, {"PINOT_AMD_FLUSH_GROUP": "1", "PINOT_AMD_STAGE_CAP": "6"},
                                 {"PINOT_AMD_FLUSH_GROUP": "1", "PINOT_AMD_SAMPLE_STRIDE": "8"},
                                 {"PINOT_AMD_FLUSH_GROUP": "1", "PINOT_AMD_FLUSH_EVERY": "3"},
                                 {"PINOT_AMD_FLUSH_GROUP": "0"}],
                         ids=["group", "group-cap6", "group-sampled", "group-every3", "lane-parallel"])
def test_highcard_flush_variants(engine, monkeypatch, env):
    """configs[3]'s query and data (16-byte records) through the scatter's flush variants -- four ready
    partitions per wave step in 16-lane groups (exact counts at this size, sampled allotments with the overflow
    slab at stride 8, tiny staging, a slower flush cadence) and the lane-parallel flush -- against the oracle."""
    from pinot_amd import datagen
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    bufs = [datagen.highcard_segment(f"hf{i}", 700_001 + 13 * i, seed=300 + i) for i in range(2)]
    segs = [engine.ImmutableSegment(b) for b in bufs]
    q = datagen.HIGHCARD_QUERY
    res = engine.ServerQueryExecutor().execute(q, segs)
    assert res.kernel_info() == "jit-partitioned", res.kernel_info()
    nm, og = oracle.execute(q, bufs)
    assert res.num_docs_matched() == nm
    assert_same_groups(res.groups(), og)
    res.execute_again()
    assert_same_groups(res.groups(), og)
