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
                                 {"PINOT_AMD_HASH_INIT_SLOTS": "64", "PINOT_AMD_HASH_LDS_SLOTS": "128"}],
                         ids=["lds", "lds64", "nolds", "grow", "grow-lds128"])
def test_widekeys_hash_plan_vs_oracle(wide, env, monkeypatch):
    E, bufs, segs, exp = wide
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    res = E.ServerQueryExecutor().execute(datagen.WIDEKEYS_QUERY, segs)
    assert "hash" in res.kernel_info(), res.kernel_info()
    got = res.groups()
    assert len(got) == len(exp) > 10_000
    assert got == exp
    assert sum(v[0] for v in got.values()) == res.num_docs_matched()
    res.execute_again()  # a re-execution (the grown table is kept) gives the same groups
    assert res.groups() == exp
