"""GPU parity for the hash-table GROUP BY plan, numGroupsLimit trimming and exact integer SUM.

* numGroupsLimit (DictionaryBasedGroupKeyGenerator.java:351-363 and the map holders' getGroupId(rawKey,
  numGroupsLimit), :651-659): each segment admits group keys in the order its matching docs first reach
  them, until it holds numGroupsLimit keys; later keys are dropped, and GroupByOperator.java:133 flags
  numGroupsLimitReached when a segment holds >= numGroupsLimit keys. The oracle restates the map holder
  literally (docs in docId order, a hash map of admitted keys). The device runs one of two plans:
  the dense admission plan for key spaces a dense table holds (first matching docId per (segment, key)
  over a prefix of each segment, the limit-th first docId per segment, admission bitmaps the aggregation
  reads; `+admit`), or the hash trim plan (scan tables keyed by (key, segment) with each entry's first
  matching docId, a per-segment cutoff, merge; `jit-hash-trim`). PINOT_AMD_TRIM_PLAN=hash forces the
  latter; PINOT_AMD_ADMIT_PREFIX shrinks the admission prefixes so segments are redone whole. Key
  spaces of <= 2^20 keys admit with one block per segment walking its prefix in doc order (seen keys in
  an LDS bitmap); PINOT_AMD_ADMIT_SEQ=0 forces the first-doc admission larger key spaces take.
* Exact integer SUM: INT/LONG sums accumulate in 128 bits on the device and in the oracle and are
  rounded to double once, so LONG values at epoch-nanosecond scale (~1.7e18) neither wrap nor drift.
"""
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
            if a.func in ("SUM", "AVG") and a.column in ("r_double", "r_float", "fd", "m")}


def _check(engine, q, bufs, segs, expect_trim=None):
    qc = parse_sql(q)
    res = engine.ServerQueryExecutor().execute(qc, segs)
    stats = {}
    nm, og = oracle.execute(q, bufs, stats=stats)
    if expect_trim is not None:
        info = res.kernel_info()
        assert ("trim" in info or "admit" in info) == expect_trim, info
    assert res.num_docs_matched() == nm
    assert res.num_groups_limit_reached() == stats.get("num_groups_limit_reached", False)
    assert_same_groups(res.groups(), og, _fsum(qc))
    return res, og, stats


TRIM_QUERIES = [
    "SELECT d0, d1, COUNT(*), SUM(r_int), MIN(r_long), MAX(r_double) FROM t GROUP BY d0, d1",
    "SELECT d0, COUNT(*), SUM(r_long), AVG(r_int) FROM t WHERE r_int > 0 GROUP BY d0",
    "SELECT d0, COUNT(*), SUM(r_double) FROM t WHERE d1 IN (3, 10, 66, 255) OR r_long < 0 GROUP BY d0",
]


@pytest.fixture(params=["admit", "admit-short-prefix", "admit-firstdoc", "admit-firstdoc-short-prefix", "hash"])
def trim_plan(request, monkeypatch):
    if request.param == "hash":
        monkeypatch.setenv("PINOT_AMD_TRIM_PLAN", "hash")
    if request.param.endswith("short-prefix"):  # prefixes too short: segments are redone whole
        monkeypatch.setenv("PINOT_AMD_ADMIT_PREFIX", "1024")
    if request.param.startswith("admit-firstdoc"):  # the first-doc admission (key spaces past LDS)
        monkeypatch.setenv("PINOT_AMD_ADMIT_SEQ", "0")
    return request.param


def _expect_plan(res, plan):
    info = res.kernel_info()
    assert ("hash-trim" in info) if plan == "hash" else ("+admit" in info), (plan, info)


@pytest.mark.parametrize("qi", range(len(TRIM_QUERIES)))
@pytest.mark.parametrize("limit", [1, 7, 100, 999])
def test_num_groups_limit_trimming_vs_oracle(engine, qi, limit, trim_plan):
    rng = np.random.default_rng(qi * 101 + limit)
    bufs = [random_segment(rng, 20_000 + 3_001 * i, name=f"t{i}", bits_cards=(1000, 143)) for i in range(3)]
    segs = [engine.ImmutableSegment(b) for b in bufs]
    q = f"SET numGroupsLimit = {limit}; " + TRIM_QUERIES[qi]
    res, og, stats = _check(engine, q, bufs, segs, expect_trim=True)
    _expect_plan(res, trim_plan)
    assert stats["num_groups_limit_reached"]
    # every segment admits at most `limit` keys; the combine is their union
    assert len(og) <= 3 * limit
    res.execute_again()  # the admission state resets between executions
    assert_same_groups(res.groups(), og, _fsum(parse_sql(q)))


def test_trimming_boundary_counts(engine, trim_plan):
    """A segment holding exactly numGroupsLimit keys is flagged but loses nothing; one key more and
    the last key to appear is dropped."""
    rng = np.random.default_rng(3)
    bufs = random_segment(rng, 5000, bits_cards=(40, 3))
    seg = engine.ImmutableSegment(bufs)
    q = "SELECT d0, COUNT(*), SUM(r_long) FROM t GROUP BY d0"
    full = oracle.execute(q, [bufs])[1]
    k = len(full)
    for limit, reached, ngroups in [(k + 1, False, k), (k, True, k), (k - 1, True, k - 1)]:
        res, og, stats = _check(engine, f"SET numGroupsLimit = {limit}; " + q, [bufs], [seg])
        assert res.num_groups_limit_reached() is reached
        assert len(res.groups()) == ngroups


def test_trimming_in_batches(engine, monkeypatch):
    """Hash trim plan with scan tables limited to a few MiB: segments are trimmed batch by batch and merged."""
    monkeypatch.setenv("PINOT_AMD_TRIM_PLAN", "hash")
    monkeypatch.setenv("PINOT_AMD_HASH_TABLE_BYTES", str(4 << 20))
    rng = np.random.default_rng(8)
    bufs = [random_segment(rng, 60_000 + 7 * i, name=f"b{i}", bits_cards=(1000, 1000)) for i in range(6)]
    segs = [engine.ImmutableSegment(b) for b in bufs]
    q = "SET numGroupsLimit = 20000; " + TRIM_QUERIES[0]
    res, og, _ = _check(engine, q, bufs, segs, expect_trim=True)
    res.execute_again()
    assert_same_groups(res.groups(), og, _fsum(parse_sql(q)))


def test_highcard_query_with_default_limit(engine, trim_plan):
    """BASELINE configs[3]'s query without its SET numGroupsLimit: ~1M groups per segment, the
    default limit of 100000 keys per segment applies (Pinot's default-option result)."""
    from pinot_amd import datagen
    q = datagen.HIGHCARD_QUERY.split(";", 1)[1].strip()
    bufs = [datagen.highcard_segment(f"hcd{i}", 1_500_000, seed=40 + i) for i in range(2)]
    segs = [engine.ImmutableSegment(b) for b in bufs]
    res, og, stats = _check(engine, q, bufs, segs, expect_trim=True)
    _expect_plan(res, trim_plan)
    assert stats["num_groups_limit_reached"]
    assert 100_000 <= len(og) <= 200_000


def test_admission_skewed_keys_and_untrimmed_segments(engine):
    """Dense admission where the prefix estimate is wrong: keys concentrated at the start of a segment
    and new keys only late (the prefix sees too few; the segment is redone whole), next to segments
    holding fewer keys than the limit (everything admitted) — against the oracle."""
    rng = np.random.default_rng(21)
    bufs = []
    for i, (n, cut, card_early, card_late) in enumerate([(200_000, 150_000, 30, 3000), (50_000, 25_000, 2000, 2000),
                                                         (30_000, 15_000, 20, 20)]):
        early = rng.integers(0, card_early, cut)
        late = rng.integers(0, card_late, n - cut)
        d = np.concatenate([early, late]).astype(np.int32) * 5 + 1
        bufs.append(S.build_segment(f"sk{i}", {
            "d": (d, S.INT, {}),
            "g": (rng.integers(0, 4, n).astype(np.int32), S.INT, {}),
            "v": (rng.integers(-(1 << 40), 1 << 40, n).astype(np.int64), S.LONG, {"dictionary": False}),
        }))
    segs = [engine.ImmutableSegment(b) for b in bufs]
    q = "SET numGroupsLimit = 500; SELECT d, g, COUNT(*), SUM(v), MIN(v) FROM t WHERE g < 3 GROUP BY d, g"
    res, og, stats = _check(engine, q, bufs, segs, expect_trim=True)
    assert "+admit" in res.kernel_info()
    assert stats["num_groups_limit_reached"]


def test_hash_plan_multi_word_keys_and_segments(engine, monkeypatch):
    """Five group columns over segments with different dictionaries (keys of two 64-bit words after
    packing), forced through the hash plan, against the oracle."""
    monkeypatch.setenv("PINOT_AMD_GROUP_PLAN", "hash")
    rng = np.random.default_rng(12)
    bufs = []
    for i in range(3):
        n = 40_000 + i
        cols = {
            "a": (rng.integers(0, 60000, n).astype(np.int32), S.INT, {}),
            "b": (rng.integers(0, 70000, n).astype(np.int64) * 3, S.LONG, {}),
            "c": (rng.integers(0, 50000, n).astype(np.int32), S.INT, {}),
            "d": (np.array([f"s{x}" for x in rng.integers(0, 3000, n)], dtype=object), S.STRING, {}),
            "e": (rng.integers(0, 9, n).astype(np.int32), S.INT, {}),
            "m": (rng.normal(0, 100, n), S.DOUBLE, {"dictionary": False}),
            "x": (rng.integers(-(1 << 62), 1 << 62, n, dtype=np.int64), S.LONG, {"dictionary": False}),
        }
        bufs.append(S.build_segment(f"w{i}", cols))
    segs = [engine.ImmutableSegment(b) for b in bufs]
    q = "SELECT a, b, c, d, e, COUNT(*), SUM(x), MIN(m), MAX(x) FROM t WHERE e < 7 GROUP BY a, b, c, d, e"
    res, _, _ = _check(engine, q, bufs, segs, expect_trim=False)
    assert "hash" in res.kernel_info()


# ------------------------------------------------------------------------------- exact integer SUM
def _big_long_segment(rng, n, name, sign=1):
    # epoch-nanosecond scale: every value ~1.7e18, sums pass INT64_MAX after 6 docs
    v = (np.int64(1_700_000_000_000_000_000) + rng.integers(0, 10**15, n, dtype=np.int64)) * sign
    cols = {
        "g": (rng.integers(0, 5, n).astype(np.int32), S.INT, {}),
        "ts": (v.astype(np.int64), S.LONG, {"dictionary": False}),
        "tsd": ((v // 1000).astype(np.int64), S.LONG, {}),
        "i": (rng.integers(-(1 << 31), (1 << 31) - 1, n).astype(np.int32), S.INT, {"dictionary": False}),
    }
    return S.build_segment(name, cols), v


@pytest.mark.parametrize("plan", ["auto", "hash"])
def test_int128_sums_at_epoch_nanosecond_scale(engine, monkeypatch, plan):
    if plan == "hash":
        monkeypatch.setenv("PINOT_AMD_GROUP_PLAN", "hash")
    rng = np.random.default_rng(77)
    made = [_big_long_segment(rng, 30_000, "p", 1), _big_long_segment(rng, 20_000, "n", -1),
            _big_long_segment(rng, 1_000, "q", 1)]
    bufs = [b for b, _ in made]
    segs = [engine.ImmutableSegment(b) for b in bufs]
    for q in ["SELECT g, COUNT(*), SUM(ts), SUM(tsd), AVG(ts), SUM(i) FROM t GROUP BY g",
              "SELECT COUNT(*), SUM(ts), SUM(tsd), AVG(ts), SUM(i) FROM t",
              "SELECT COUNT(*), SUM(ts) FROM t WHERE g = 3"]:
        res = engine.ServerQueryExecutor().execute(q, segs)
        _, og = oracle.execute(q, bufs)
        got = res.groups()
        assert set(got) == set(og)
        for k in og:
            assert got[k] == og[k], (q, k, got[k], og[k])  # exact sums rounded once: bit-equal doubles
    # the exact value, checked independently of the oracle
    exact = sum(int(x) for _, v in made for x in v)
    got = engine.ServerQueryExecutor().execute("SELECT SUM(ts) FROM t", segs).groups()[()][0]
    assert got == float(exact)


def test_mixed_encodings_across_segments(engine):
    """A column dictionary-encoded in some segments and raw in others, and group columns whose bit
    widths differ per segment: the batch runs as several compile-time-specialised launches into one
    table."""
    rng = np.random.default_rng(5)
    bufs = []
    for i in range(6):
        n = 30_000 + 1000 * i
        card = [3, 40, 300, 2000, 9, 70000][i]
        cols = {
            "k": ((rng.integers(0, card, n) * 11).astype(np.int32), S.INT, {}),
            "v": (rng.integers(-1000, 1000, n).astype(np.int64), S.LONG, {"dictionary": i % 2 == 0}),
            "f": (rng.normal(0, 10, n), S.DOUBLE, {"dictionary": i % 3 == 0}),
        }
        bufs.append(S.build_segment(f"mx{i}", cols))
    segs = [engine.ImmutableSegment(b) for b in bufs]
    for q in ["SELECT k, COUNT(*), SUM(v), MAX(f), SUM(f) FROM t WHERE v > -500 GROUP BY k",
              "SELECT COUNT(*), SUM(v), MIN(f) FROM t WHERE k < 2000 AND f > 0"]:
        qc = parse_sql(q)
        res = engine.ServerQueryExecutor().execute(qc, segs)
        assert " x" in res.kernel_info(), res.kernel_info()  # several launches
        nm, og = oracle.execute(q, bufs)
        assert res.num_docs_matched() == nm
        fs = {i for i, a in enumerate(qc.aggregations) if a.func == "SUM" and a.column == "f"}
        assert_same_groups(res.groups(), og, fs)


@pytest.mark.parametrize("narrow", ["1", "0"])
def test_int_sums_narrow_lds_partials(engine, monkeypatch, narrow):
    """Integer SUMs into LDS tables keep 64-bit partials when the column's value range (dictionary
    ends, or the min / max computed at staging) times the docs one block can add stays below 2^63,
    and 128-bit partials otherwise. Both ways give the exact sums: INT values at the type's extremes,
    LONG values near 2^44 (narrow) and near 2^60 (wide), in the LDS table plan and in the partitioned
    plan (whose aggregation blocks use the same rule), against the oracle."""
    monkeypatch.setenv("PINOT_AMD_NARROW_SUMS", narrow)
    rng = np.random.default_rng(31)
    bufs = []
    for i in range(3):
        n = 120_000 + 17 * i
        iv = rng.choice(np.array([-(1 << 31), (1 << 31) - 1, 0, 5], dtype=np.int64), n).astype(np.int32)
        cols = {
            "g": (rng.integers(0, 50, n).astype(np.int32), S.INT, {}),
            "a": (rng.integers(0, 700, n).astype(np.int32), S.INT, {}),
            "b": (rng.integers(0, 700, n).astype(np.int32), S.INT, {}),
            "i": (iv, S.INT, {"dictionary": False}),
            "l44": (rng.integers((1 << 44) - 1000, 1 << 44, n, dtype=np.int64), S.LONG, {"dictionary": False}),
            "l60": (rng.integers(-(1 << 60), 1 << 60, n, dtype=np.int64), S.LONG, {"dictionary": False}),
            "dl": (rng.integers(-(1 << 40), 1 << 40, n, dtype=np.int64) // 4096 * 4096, S.LONG, {}),
        }
        bufs.append(S.build_segment(f"nw{i}", cols))
    segs = [engine.ImmutableSegment(b) for b in bufs]
    for q in ["SELECT g, COUNT(*), SUM(i), SUM(l44), SUM(l60), SUM(dl), AVG(i) FROM t GROUP BY g",
              "SET numGroupsLimit = 1000000; SELECT a, b, COUNT(*), SUM(i), SUM(l44), SUM(l60) FROM t WHERE g < 40 "
              "GROUP BY a, b"]:
        res = engine.ServerQueryExecutor().execute(q, segs)
        if "GROUP BY a, b" in q:
            assert res.kernel_info().startswith("jit-partitioned"), res.kernel_info()
        _, og = oracle.execute(q, bufs)
        got = res.groups()
        miss, extra = sorted(set(og) - set(got)), sorted(set(got) - set(og))
        assert not miss and not extra, (res.kernel_info(), len(got), len(og), miss[:8], extra[:8],
                                        {k: v for k, v in res.plan_timing().items() if not isinstance(v, dict)})
        for k in og:
            assert got[k] == og[k], (q, k, got[k], og[k])
