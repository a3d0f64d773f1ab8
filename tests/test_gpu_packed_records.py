"""Partitioned GROUP BY with bit-packed records: the scatter pass stores each matching doc as the
partition-local key plus one field per aggregated value, an integer value as its offset from the
batch's value range minimum in just enough bits (dictionary ends / staged min-max; interval arithmetic
for times / minus / plus of two INT columns), FLOAT / DOUBLE as raw bits. Checked against the CPU
oracle (DictionaryBasedGroupKeyGenerator's map-based holders) for field widths from 0 (constant
column) to 64 (a LONG column spanning the whole long range), negative ranges, expressions with
negative products, dictionary-encoded value columns, and segments whose ranges differ (the batch
range covers all of them). Integer results bit-exact, double SUM within 1e-12 relative."""
import numpy as np
import pytest

import oracle
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


def _segment(rng, n, name, shift=0):
    """Two 1000-value group dimensions (1M keys: the partitioned plan) and value columns of assorted
    ranges; `shift` moves the ranges so segments of one batch differ."""
    i64 = np.iinfo(np.int64)
    full = rng.integers(i64.min, i64.max, n, dtype=np.int64, endpoint=True)
    full[:2] = [i64.min, i64.max][:min(n, 2)]
    return S.build_segment(name, {
        "a": ((rng.integers(0, 1000, n) * 3 + 1).astype(np.int32), S.INT, {}),
        "b": ((rng.integers(0, 1000, n) * 5 - 7).astype(np.int32), S.INT, {}),
        "k_const": (np.full(n, 42 + shift, np.int32), S.INT, {"dictionary": False}),
        "neg": (rng.integers(-70000 - shift, -69000, n).astype(np.int32), S.INT, {"dictionary": False}),
        "i_ext": (rng.integers(-(1 << 31), (1 << 31), n).astype(np.int32), S.INT, {"dictionary": False}),
        "l_full": (full, S.LONG, {"dictionary": False}),
        "l_nano": (rng.integers(1_700_000_000_000_000_000, 1_700_000_100_000_000_000, n).astype(np.int64), S.LONG,
                   {"dictionary": False}),
        "l_dict": ((rng.integers(0, 300, n) * 1_000_003 - 150_000_000 + shift).astype(np.int64), S.LONG, {}),
        "f": (rng.normal(0, 50, n).astype(np.float32), S.FLOAT, {"dictionary": False}),
        "dbl": (rng.normal(0, 1e6, n), S.DOUBLE, {"dictionary": False}),
        "x": (rng.integers(-30000, 30000, n).astype(np.int32), S.INT, {"dictionary": False}),
        "y": (rng.integers(-500, 9000, n).astype(np.int32), S.INT, {"dictionary": False}),
    })


QUERIES = [
    # constant (0-bit field), negative range, 32-bit INT extremes, 64-bit LONG extremes
    "SELECT a, b, COUNT(*), SUM(k_const), MIN(neg), MAX(neg), SUM(i_ext), MIN(l_full), MAX(l_full) FROM t GROUP BY a, b",
    # epoch-nanosecond LONGs (57-bit field after the offset), dictionary-encoded LONG values, FLOAT, DOUBLE
    "SELECT a, b, SUM(l_nano), MIN(l_nano), MAX(l_dict), SUM(l_dict), MAX(f), SUM(dbl) FROM t WHERE x > -20000 GROUP BY a, b",
    # expressions: times / minus / plus of two INT columns with negative operands (interval bounds)
    "SELECT a, b, SUM(x * y), MIN(y - x), MAX(x + neg), SUM(x - x) FROM t WHERE y < 8000 "
    "GROUP BY a, b",
]


@pytest.mark.parametrize("qi", range(len(QUERIES)))
def test_packed_records_vs_oracle(engine, monkeypatch, qi):
    monkeypatch.delenv("PINOT_AMD_PARTITIONED", raising=False)
    monkeypatch.setenv("PINOT_AMD_ATOMIC_HANDOVER", "0")
    rng = np.random.default_rng(77 + qi)
    bufs = [_segment(rng, n, f"pk{i}", shift=i * 1000) for i, n in enumerate([200_003, 1, 70_000])]
    segs = [engine.ImmutableSegment(b) for b in bufs]
    qc = parse_sql("SET numGroupsLimit = 2000000; " + QUERIES[qi])
    res = engine.ServerQueryExecutor().execute(qc, segs)
    assert res.kernel_info().startswith("jit-partitioned"), res.kernel_info()
    nm, og = oracle.execute("SET numGroupsLimit = 2000000; " + QUERIES[qi], bufs)
    assert res.num_docs_matched() == nm
    fs = {i for i, a in enumerate(qc.aggregations) if a.func == "SUM" and a.column in ("dbl", "f")}
    assert_same_groups(res.groups(), og, fs)
    res.execute_again()
    assert_same_groups(res.groups(), og, fs)


@pytest.mark.parametrize("scale,stage_cap,where", [
    (None, None, ""),                  # sampled capacities as planned (stride 1: the sample is exact)
    ("0.5", None, ""),                 # half the needed capacity: the rest goes to the overflow slab
    ("0", None, ""),                   # no capacity at all: every record through the slab
    ("0.7", "0", ""),                  # direct writes (no LDS staging), reservations per record
    (None, None, " WHERE x < -29500"),  # ~0.8 % match: the sample hands over to the direct-atomic scan
])
def test_sampled_capacities_vs_oracle(engine, monkeypatch, scale, stage_cap, where):
    """Sampled partitioned plans (strided histogram instead of the exact count pass; reservations per
    flushed run; records beyond a partition's capacity through the overflow slab's direct atomics):
    identical groups to the oracle whatever the capacities."""
    monkeypatch.delenv("PINOT_AMD_PARTITIONED", raising=False)
    monkeypatch.delenv("PINOT_AMD_ATOMIC_HANDOVER", raising=False)
    monkeypatch.setenv("PINOT_AMD_SELECT_PARTITIONED", "0")  # the partitioned plan's handover, not a select
    monkeypatch.setenv("PINOT_AMD_SAMPLE_STRIDE", "1")
    for var, val in (("PINOT_AMD_PART_CAP_SCALE", scale), ("PINOT_AMD_STAGE_CAP", stage_cap)):
        if val is None:
            monkeypatch.delenv(var, raising=False)
        else:
            monkeypatch.setenv(var, val)
    rng = np.random.default_rng(5)
    bufs = [_segment(rng, n, f"sc{i}", shift=i * 10) for i, n in enumerate([150_001, 90_000])]
    segs = [engine.ImmutableSegment(b) for b in bufs]
    q = ("SET numGroupsLimit = 2000000; SELECT a, b, COUNT(*), SUM(x), MIN(l_nano), MAX(dbl), SUM(dbl) FROM t"
         + where + " GROUP BY a, b")
    qc = parse_sql(q)
    res = engine.ServerQueryExecutor().execute(qc, segs)
    assert res.kernel_info().startswith("jit-partitioned"), res.kernel_info()
    nm, og = oracle.execute(q, bufs)
    assert res.num_docs_matched() == nm
    assert_same_groups(res.groups(), og, {4})
    res.execute_again()  # cursors and the slab reset per execution
    assert res.num_docs_matched() == nm
    assert_same_groups(res.groups(), og, {4})
