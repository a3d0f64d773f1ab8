"""Hash-table GROUP BY past the dense key space (DictionaryBasedGroupKeyGenerator's map-based holders,
DictionaryBasedGroupKeyGenerator.java:444-900) on the device, against the CPU oracle: the bench's wide-key
table (5 dictionary columns, two packed key words, Zipf-distributed entities) through

* the LDS-privatised first level (default), a tiny one (64 slots: most keys spill to the HBM table
  directly, the block flush merges the rest) and none (PINOT_AMD_HASH_LDS=0);
* a final table that starts far too small (PINOT_AMD_HASH_INIT_SLOTS=64): the plan grows it 4x and runs
  again until every group has a slot, and the result is unchanged.
COUNT, integer SUM and MAX(DOUBLE) are order-independent, so every case is exact."""
import pytest

import oracle
from pinot_amd import datagen

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def wide():
    import torch
    assert torch.cuda.is_available(), "GPU tests need a visible MI355X"
    from pinot_amd import engine as E
    bufs = [datagen.widekeys_segment(f"wk{i}", 300_000 + 7 * i, seed=90 + i) for i in range(2)]
    _, exp = oracle.execute(datagen.WIDEKEYS_QUERY, bufs)
    return E, bufs, [E.ImmutableSegment(b) for b in bufs], exp


@pytest.mark.parametrize("env", [{}, {"PINOT_AMD_HASH_LDS_SLOTS": "64"}, {"PINOT_AMD_HASH_LDS": "0"},
                                 {"PINOT_AMD_HASH_INIT_SLOTS": "64"},
                                 {"PINOT_AMD_HASH_INIT_SLOTS": "64", "PINOT_AMD_HASH_LDS_SLOTS": "128"},
                                 {"PINOT_AMD_HASH_LDS_ADMIT": "0"}, {"PINOT_AMD_HASH_LDS_ADMIT": "8"},
                                 {"PINOT_AMD_SPILL_BYTES": "4096"}, {"PINOT_AMD_HASH_SPILL": "0"},
                                 {"PINOT_AMD_SPILL_SORT": "0"}],
                         ids=["lds", "lds64", "nolds", "grow", "grow-lds128", "admit-all", "admit-1in256",
                              "spill-overflow", "nospill", "spill-unsorted"])
def test_widekeys_hash_plan_vs_oracle(wide, env, monkeypatch):
    E, bufs, segs, exp = wide
    monkeypatch.setenv("PINOT_AMD_HASH_CAP_CACHE", "0")  # every case sizes (and grows) its own table
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    res = E.ServerQueryExecutor().execute(datagen.WIDEKEYS_QUERY, segs)
    assert "hash" in res.kernel_info(), res.kernel_info()
    got = res.groups()
    assert len(got) == len(exp) > 10_000
    assert got == exp
    assert sum(v[0] for v in got.values()) == res.num_docs_matched()
    res.execute_again()  # a re-execution (the grown table / spill regions are kept) gives the same groups
    assert res.groups() == exp


def test_widekeys_reissued_query_starts_at_the_grown_capacity(wide, monkeypatch):
    """A query executed again through a fresh result (a new pinot_amd_execute, as a server re-issuing it) starts at
    the capacity the first execution grew to, without the overflow check's host synchronisation -- and the
    groups are the same."""
    E, bufs, segs, exp = wide
    monkeypatch.setenv("PINOT_AMD_HASH_INIT_SLOTS", "64")
    r1 = E.ServerQueryExecutor().execute(datagen.WIDEKEYS_QUERY, segs)
    t1 = r1.plan_timing()
    assert r1.groups() == exp
    r2 = E.ServerQueryExecutor().execute(datagen.WIDEKEYS_QUERY, segs)
    t2 = r2.plan_timing()
    assert t2["hash_slots_remembered"] == 1 and t2["hash_slots"] >= t1["hash_slots"] > 64, (t1, t2)
    assert r2.groups() == exp
    r2.execute_again()
    assert r2.groups() == exp


def test_widekeys_remembered_capacity_overflow_settled_at_fetch(wide, monkeypatch):
    """An execution at a remembered capacity skips the overflow check; if docs then found no slot (here: probe
    chains cut to 32 slots after the capacity was settled with 512), reading the groups grows the table and runs
    the plan again -- the groups are exact either way."""
    E, bufs, segs, exp = wide
    monkeypatch.setenv("PINOT_AMD_HASH_INIT_SLOTS", "64")
    r1 = E.ServerQueryExecutor().execute(datagen.WIDEKEYS_QUERY, segs)
    assert r1.groups() == exp
    monkeypatch.setenv("PINOT_AMD_HASH_MAX_PROBE", "32")
    r2 = E.ServerQueryExecutor().execute(datagen.WIDEKEYS_QUERY, segs)
    assert r2.plan_timing()["hash_slots_remembered"] == 1
    assert r2.groups() == exp


def test_hash_growth_lands_on_the_ceiling(monkeypatch):
    """Growth is 4x per step but stops at the plan's ceiling (2 x its group bound as a power of two): from 64 slots
    a table whose ceiling is 2^13 ends there (64 -> 256 -> 1024 -> 4096 -> 8192) instead of overshooting to 16384
    (advisor); 4000 docs over an 11100-key space hold ~3300 groups, too many for 4096 slots at 64-slot chains."""
    import numpy as np
    import torch
    assert torch.cuda.is_available()
    from helpers import random_segment
    from pinot_amd import engine as E
    monkeypatch.setenv("PINOT_AMD_HASH_CAP_CACHE", "0")
    monkeypatch.setenv("PINOT_AMD_HASH_INIT_SLOTS", "64")
    monkeypatch.setenv("PINOT_AMD_HASH_MAX_PROBE", "64")
    monkeypatch.setenv("PINOT_AMD_GROUP_PLAN", "hash")
    # every key into the LDS level as it comes (the insertion order into the HBM table this case was sized for)
    monkeypatch.setenv("PINOT_AMD_HASH_LDS_ADMIT", "0")
    rng = np.random.default_rng(3)
    bufs = [random_segment(rng, 4_000, name="hg0", bits_cards=(300, 37))]
    segs = [E.ImmutableSegment(b) for b in bufs]
    q = "SELECT d0, d1, COUNT(*), SUM(r_long) FROM t GROUP BY d0, d1"
    res = E.ServerQueryExecutor().execute(q, segs)
    _, exp = oracle.execute(q, bufs)
    got = res.groups()
    assert len(got) == len(exp) > 3000 and got == exp
    assert res.plan_timing()["hash_slots"] == 8192


def test_spill_regions_grow_after_an_overflow(wide, monkeypatch):
    """Spill regions far too small (64 records per scan block): the records past them take the HBM table, the
    groups are exact; the fetch remembers what the blocks needed, so the next execution of the same result and a
    re-issued query run with regions that hold every record -- same groups."""
    E, bufs, segs, exp = wide
    monkeypatch.setenv("PINOT_AMD_SPILL_BYTES", "4096")
    monkeypatch.setenv("PINOT_AMD_HASH_LDS_ADMIT", "8")  # most keys miss the LDS level
    r1 = E.ServerQueryExecutor().execute(datagen.WIDEKEYS_QUERY, segs)
    assert r1.groups() == exp
    r1.execute_again()
    assert r1.groups() == exp
    r2 = E.ServerQueryExecutor().execute(datagen.WIDEKEYS_QUERY, segs)
    assert r2.groups() == exp


@pytest.fixture(scope="module")
def wide_uniform():
    import torch
    assert torch.cuda.is_available(), "GPU tests need a visible MI355X"
    from pinot_amd import engine as E
    bufs = [datagen.widekeys_uniform_segment(f"wu{i}", 300_000 + 11 * i, seed=70 + i) for i in range(2)]
    _, exp = oracle.execute(datagen.WIDEKEYS_QUERY, bufs)
    return E, bufs, [E.ImmutableSegment(b) for b in bufs], exp


@pytest.mark.parametrize("env", [{}, {"PINOT_AMD_HASH_LDS": "0"}, {"PINOT_AMD_HASH_SPILL": "0"},
                                 {"PINOT_AMD_SPILL_BYTES": "4096"}],
                         ids=["default", "nolds", "nospill", "spill-overflow"])
def test_widekeys_uniform_vs_oracle(wide_uniform, env, monkeypatch):
    """Wide keys without skew (entities uniform over 1M ranks: ~450K groups in 600K docs, no key hot enough for an
    on-die first level): the hash plan the key-distribution sample picks, and the fixed alternatives."""
    E, bufs, segs, exp = wide_uniform
    monkeypatch.setenv("PINOT_AMD_HASH_CAP_CACHE", "0")
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    res = E.ServerQueryExecutor().execute(datagen.WIDEKEYS_QUERY, segs)
    assert "hash" in res.kernel_info(), res.kernel_info()
    got = res.groups()
    assert len(got) == len(exp) > 200_000
    assert got == exp
    assert sum(v[0] for v in got.values()) == res.num_docs_matched()
    res.execute_again()
    assert res.groups() == exp


def test_widekeys_uniform_drops_the_lds_level(wide_uniform, monkeypatch):
    """Most docs of a uniform key distribution miss the LDS level: after the first execution the plan drops it and
    spills every matching doc to its block's region (no LDS probe per doc). Every step exact."""
    E, bufs, segs, exp = wide_uniform
    monkeypatch.setenv("PINOT_AMD_HASH_CAP_CACHE", "0")
    monkeypatch.setenv("PINOT_AMD_HASH_DIRECT", "auto")  # (also a plan identity of its own: no prepared plan)
    res = E.ServerQueryExecutor().execute(datagen.WIDEKEYS_QUERY, segs)
    assert "+nolds" not in res.kernel_info() and "+direct" not in res.kernel_info()
    assert res.groups() == exp  # (the fetch sees most docs spilled: the LDS level goes)
    res.execute_again()
    assert "+nolds" in res.kernel_info(), res.kernel_info()
    assert res.groups() == exp
    for _ in range(2):
        res.execute_again()
        assert "+nolds" in res.kernel_info(), res.kernel_info()
        assert res.groups() == exp
        assert sum(v[0] for v in res.groups().values()) == res.num_docs_matched()


@pytest.mark.parametrize("env", [{"PINOT_AMD_HASH_DIRECT": "force"},
                                 {"PINOT_AMD_HASH_DIRECT": "force", "PINOT_AMD_HASH_INIT_SLOTS": "4096"},
                                 {"PINOT_AMD_HASH_DIRECT": "force", "PINOT_AMD_SPILL_BYTES": "65536"}],
                         ids=["force", "force-grow", "force-small-regions"])
def test_widekeys_direct_placement_forced(wide, wide_uniform, env, monkeypatch):
    """Direct placement (PINOT_AMD_HASH_DIRECT=force: no LDS level from the first execution, which counts the
    (partition, block) allotments; the later ones place each record straight into its partition, no region pass),
    over skewed and uniform keys; with a table that grows while the
    plan runs (the partition count changes: the allotments are counted again) and with spill regions too small for
    the counting execution (records past them take the HBM table; the direct one places exactly what was counted)."""
    monkeypatch.setenv("PINOT_AMD_HASH_CAP_CACHE", "0")
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    for E, bufs, segs, exp in (wide, wide_uniform):
        res = E.ServerQueryExecutor().execute(datagen.WIDEKEYS_QUERY, segs)
        assert res.groups() == exp
        for _ in range(2):
            res.execute_again()
            assert "+direct" in res.kernel_info(), res.kernel_info()
            assert res.groups() == exp



_WIDTH_QUERIES = {  # spilled record width (key word + value words; COUNT is the record itself)
    "w1": "SELECT w1, w2, w3, w4, w5, COUNT(*) FROM wide WHERE metInt < 900 GROUP BY w1, w2, w3, w4, w5",
    "w2": "SELECT w1, w2, w3, w4, w5, COUNT(*), SUM(metInt) FROM wide GROUP BY w1, w2, w3, w4, w5",
    "w5": ("SELECT w1, w2, w3, w4, w5, COUNT(*), SUM(metInt), MAX(metDouble), MIN(metDouble), MAX(metInt) "
           "FROM wide WHERE metInt < 700 GROUP BY w1, w2, w3, w4, w5"),
}


@pytest.mark.parametrize("width", sorted(_WIDTH_QUERIES))
def test_spill_record_widths_vs_oracle(wide, wide_uniform, width, monkeypatch):
    """The spill passes at other record widths than the bench's 3 words: the region pass's register prefetch of
    its next chunk and the aggregation templated on the width (kernels.hip spill_agg_kernel<W>), over skewed keys
    (LDS level + spill) and uniform keys (the LDS level dropped after the first execution: every doc spilled).
    COUNT, integer SUM and MIN / MAX are order-independent: exact."""
    q = "SET numGroupsLimit = 2000000000; " + _WIDTH_QUERIES[width]
    monkeypatch.setenv("PINOT_AMD_HASH_CAP_CACHE", "0")
    monkeypatch.setenv("PINOT_AMD_HASH_DIRECT", "auto")
    for E, bufs, segs, _ in (wide, wide_uniform):
        _, exp = oracle.execute(q, bufs)
        res = E.ServerQueryExecutor().execute(q, segs)
        assert "hash" in res.kernel_info(), res.kernel_info()
        assert res.groups() == exp
        for _ in range(2):
            res.execute_again()
            assert res.groups() == exp
            assert sum(v[0] for v in res.groups().values()) == res.num_docs_matched()
