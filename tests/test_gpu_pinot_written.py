"""Pinot-written segment bytes (tests/golden/pinot_written) staged into HBM and queried through the HIP
path: raw DOUBLE chunk files of versions 1 and 2, a V1 dictionary-encoded segment directory, and a raw
STRING (var-byte V4) column from V1 files and from a V3 columns.psf; plus random raw STRING columns of
every codec and writer version against the oracle."""
import json
import os
import sys

import numpy as np
import pytest

from pinot_amd import segment as S

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle  # noqa: E402

PW = os.path.join(ROOT, "tests", "golden", "pinot_written")
EXP = json.load(open(os.path.join(PW, "expected.json")))


@pytest.fixture(scope="module")
def engine():
    import torch
    assert torch.cuda.is_available()
    from pinot_amd import engine as E
    return E


@pytest.mark.parametrize("fname", sorted(EXP["raw_doubles"]))
def test_raw_double_files_staged(engine, fname):
    """Version-1 (SNAPPY, decoded on the device) and version-2 chunk files: staged values and a SUM / MIN /
    MAX / range-filtered COUNT over them equal value(doc i) = i + start."""
    import torch
    from pinot_amd._lib import check, lib
    e = EXP["raw_doubles"][fname]
    n = e["num_docs"]
    buf = open(os.path.join(PW, fname), "rb").read()
    seg = engine.ImmutableSegment(S.SegmentBuffers("rd", n, {"v": S.ColumnBuffers("v", S.DOUBLE, n, False, fwd=buf)}))
    out = torch.zeros(n, dtype=torch.float64, device="cuda")
    check(lib().pinot_amd_fwd_read_raw(seg.column_fwd_ptr("v"), 3, 0, n, out.data_ptr(), None))
    torch.cuda.synchronize()
    exp = np.arange(n) + e["start"]
    assert np.array_equal(out.cpu().numpy(), exp)
    ex = engine.ServerQueryExecutor()
    cnt, mn, mx = ex.execute("SELECT COUNT(*), MIN(v), MAX(v) FROM t", [seg]).groups()[()]
    assert (cnt, mn, mx) == (n, exp[0], exp[-1])
    lo = e["start"] + 100.5
    assert ex.execute(f"SELECT COUNT(*) FROM t WHERE v > {lo}", [seg]).groups()[()][0] == int((exp > lo).sum())


def test_padding_old_segment_on_device(engine):
    """The V1 dictionary-encoded segment: dictIds decoded on the device equal the loader's, and GROUP BY
    the STRING column with INT / LONG / FLOAT aggregations equals the oracle."""
    import torch
    from pinot_amd._lib import check, lib
    bufs = S.load_segment_dir(os.path.join(PW, "paddingOld"))
    seg = engine.ImmutableSegment(bufs)
    for c, cb in bufs.columns.items():
        out = torch.zeros(bufs.num_docs, dtype=torch.int32, device="cuda")
        check(lib().pinot_amd_fwd_read_dict_ids(seg.column_fwd_ptr(c), cb.bits_per_element, 0, bufs.num_docs,
                                                out.data_ptr(), None))
        torch.cuda.synchronize()
        assert out.cpu().numpy().tolist() == S.unpack_fixed_bit(cb.fwd, cb.bits_per_element, bufs.num_docs).tolist()
    for q in ["SELECT name, COUNT(*), SUM(age), MIN(outgoingName1), MAX(percent) FROM t GROUP BY name",
              "SELECT COUNT(*), SUM(outgoingName1) FROM t WHERE percent > 400 AND name != 'lynda 2.0'"]:
        got = engine.ServerQueryExecutor().execute(q, [seg]).groups()
        _, exp = oracle.execute(q, [bufs])
        assert got == exp, (q, got, exp)


@pytest.mark.parametrize("fmt", ["v1", "v3"])
def test_legacy_raw_string_on_device(engine, fmt):
    """The raw STRING column staged dictionary-encoded (ENABLE_DICTIONARY at load): the counts the
    reference's LegacyRawValueInvertedIndexMigrationIntegrationTest asserts, from V1 files and V3 psf."""
    e = EXP["legacy_raw_string"]
    c = e["column"]
    seg = engine.ImmutableSegment(S.load_segment_dir(os.path.join(PW, f"legacyRawInverted_{fmt}")))
    ex = engine.ServerQueryExecutor()

    def count(where=""):
        return ex.execute(f"SELECT COUNT(*) FROM t {where}", [seg]).groups()[()][0]
    assert count() == e["num_docs"]
    for v, cnt in e["counts"].items():
        assert count(f"WHERE {c} = '{v}'") == cnt
    assert count(f"WHERE {c} IN ('alpha', 'beta')") == e["in_alpha_beta"]
    assert count(f"WHERE {c} != 'alpha'") == e["not_eq_alpha"]
    g = ex.execute(f"SELECT {c}, COUNT(*) FROM t GROUP BY {c}", [seg]).groups()
    assert {k[0]: v[0] for k, v in g.items()} == e["counts"]


@pytest.mark.parametrize("version", [4, 6])
@pytest.mark.parametrize("comp", [S.PASS_THROUGH, S.SNAPPY, S.ZSTANDARD, S.LZ4, S.GZIP])
def test_raw_string_columns_vs_oracle(engine, version, comp):
    """Random raw STRING columns (multi-byte UTF-8, empty and huge values) over three segments with
    different value sets: EQ / IN / NOT_IN / RANGE filters and GROUP BY on the string, against the oracle."""
    rng = np.random.default_rng(version * 7 + comp)
    bufs = []
    for i in range(3):
        n = 20_000 + 333 * i
        pool = [f"k{j:03d}" for j in range(50 * (i + 1))] + ["", "ünï", "y" * 6000]
        s = np.array([pool[j] for j in rng.integers(0, len(pool), n)], dtype=object)
        bufs.append(S.build_segment(f"rs{i}", {
            "s": (s, S.STRING, {"dictionary": False, "raw_version": version, "compression": comp}),
            "m": (rng.integers(-1000, 1000, n).astype(np.int32), S.INT, {"dictionary": False})}))
    segs = [engine.ImmutableSegment(b) for b in bufs]
    ex = engine.ServerQueryExecutor()
    for q in ["SELECT s, COUNT(*), SUM(m), MAX(m) FROM t WHERE m > -500 GROUP BY s",
              "SELECT COUNT(*), SUM(m) FROM t WHERE s IN ('k001', 'ünï', '', 'k120') OR s BETWEEN 'k040' AND 'k045'",
              "SELECT COUNT(*) FROM t WHERE s NOT IN ('k002', 'k003') AND s > 'k1'"]:
        res = ex.execute(q, segs)
        nm, exp = oracle.execute(q, bufs)
        assert res.num_docs_matched() == nm, q
        assert res.groups() == exp, q


@pytest.mark.parametrize("fmt", ["v1", "v3"])
def test_legacy_embedded_bitmaps_on_device(engine, fmt, monkeypatch):
    """roaring_expand_chunks_kernel over the Pinot-written RoaringBitmaps embedded in the legacy raw-value
    inverted index (helpers.legacy_inverted_segment): EQ / IN / NOT_EQ counts the reference's
    LegacyRawValueInvertedIndexMigrationIntegrationTest asserts, and the filter's docIds equal the oracle's."""
    from helpers import legacy_inverted_segment
    monkeypatch.setenv("PINOT_AMD_INV_POLICY", "always")
    e = EXP["legacy_raw_string"]
    bufs = legacy_inverted_segment(fmt)
    seg = engine.ImmutableSegment(bufs)
    ex = engine.ServerQueryExecutor()
    c = e["column"]
    wheres = {f"{c} = '{v}'": cnt for v, cnt in e["counts"].items()}
    wheres[f"{c} IN ('alpha', 'beta')"] = e["in_alpha_beta"]
    wheres[f"{c} != 'alpha'"] = e["not_eq_alpha"]
    for w, cnt in wheres.items():
        q = f"SELECT COUNT(*) FROM t WHERE {w}"
        res = ex.execute(q, [seg])
        assert res.groups()[()][0] == cnt, w
        ids = ex.filter_doc_ids(q, [seg])[0]
        bits, _ = oracle.OracleSegment(bufs).filter_bitset(oracle.parse_sql(q), use_inverted=True)
        exp = np.flatnonzero(np.unpackbits(bits.view(np.uint8), bitorder="little")[:bufs.num_docs])
        assert np.array_equal(ids, exp), w
