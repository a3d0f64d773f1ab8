"""Segment bytes written by Pinot itself (tests/golden/pinot_written, copied from the reference's own test
resources by tests/golden/make_pinot_written.py) read through the CPU oracle and the host-side segment
loader, against the values the reference's tests assert for them."""
import json
import os
import sys

import numpy as np
import pytest

from pinot_amd import segment as S

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle  # noqa: E402

PW = os.path.join(ROOT, "tests", "golden", "pinot_written")
EXP = json.load(open(os.path.join(PW, "expected.json")))


@pytest.mark.parametrize("fname", sorted(EXP["raw_doubles"]))
def test_raw_double_forward_index_files(fname):
    """FixedByteChunkSVForwardIndexTest.testBackwardCompatibilityV1/V2: version-1 (SNAPPY, 16-byte header)
    and version-2 (SNAPPY / PASS_THROUGH) chunk files; value of doc i == i + start."""
    e = EXP["raw_doubles"][fname]
    buf = open(os.path.join(PW, fname), "rb").read()
    h = S.parse_raw_fwd_header(buf)
    assert h.size_of_entry == 8
    cb = S.ColumnBuffers("v", S.DOUBLE, e["num_docs"], False, fwd=buf)
    got = np.frombuffer(oracle.raw_values_region(cb).tobytes(), dtype=">f8", count=e["num_docs"])
    assert np.array_equal(got, np.arange(e["num_docs"]) + e["start"])


def test_padding_old_v1_segment_metadata_and_values():
    """A V1 segment directory of dictionary-encoded INT / LONG / FLOAT / STRING columns: the loader's
    buffers agree with metadata.properties (cardinality, bitsPerElement, the time column's start / end
    time = its dictionary ends) and the oracle answers queries over it consistently."""
    e = EXP["padding_old"]
    seg = S.load_segment_dir(os.path.join(PW, "paddingOld"))
    assert seg.num_docs == e["num_docs"]
    for c, card in e["cardinality"].items():
        cb = seg.columns[c]
        assert cb.cardinality == card and cb.bits_per_element == e["bits"][c] and len(cb.dict_values) == card
        ids = S.unpack_fixed_bit(cb.fwd, cb.bits_per_element, seg.num_docs)
        assert ids.max() < card
    t = seg.columns[e["time_column"]].dict_values
    assert (int(t[0]), int(t[-1])) == (e["start_time"], e["end_time"])
    # FixedByteValueReaderWriter.readUnpaddedBytes stops at the first NUL only: the old '%' padding stays
    assert list(seg.columns["name"].dict_values) == ["lynda 2.0", "lynda%%%%"]
    n, g = oracle.execute("SELECT COUNT(*), MIN(outgoingName1), MAX(outgoingName1), SUM(age) FROM t", [seg])
    assert n == 5 and g[()][:3] == [5, 246.0, 902.0]
    ages = seg.columns["age"].dict_values[S.unpack_fixed_bit(seg.columns["age"].fwd, 3, 5)]
    assert g[()][3] == float(ages.sum())


@pytest.mark.parametrize("fmt", ["v1", "v3"])
def test_legacy_raw_string_segment(fmt):
    """legacyRawInverted (VarByteChunkForwardIndexWriterV4, LZ4_LENGTH_PREFIXED raw STRING) as V1 files
    and as V3 columns.psf + index_map: the counts LegacyRawValueInvertedIndexMigrationIntegrationTest
    asserts, through the oracle (var-byte reader + ENABLE_DICTIONARY twin)."""
    e = EXP["legacy_raw_string"]
    seg = S.load_segment_dir(os.path.join(PW, f"legacyRawInverted_{fmt}"))
    c = e["column"]
    assert seg.num_docs == e["num_docs"] and not seg.columns[c].has_dictionary
    assert oracle.execute("SELECT COUNT(*) FROM t", [seg])[0] == e["num_docs"]
    for v, cnt in e["counts"].items():
        assert oracle.execute(f"SELECT COUNT(*) FROM t WHERE {c} = '{v}'", [seg])[0] == cnt
    assert oracle.execute(f"SELECT COUNT(*) FROM t WHERE {c} IN ('alpha', 'beta')", [seg])[0] == e["in_alpha_beta"]
    assert oracle.execute(f"SELECT COUNT(*) FROM t WHERE {c} != 'alpha'", [seg])[0] == e["not_eq_alpha"]
    _, g = oracle.execute(f"SELECT {c}, COUNT(*) FROM t GROUP BY {c}", [seg])
    assert {k[0]: v[0] for k, v in g.items()} == e["counts"]


def test_v1_and_v3_forward_index_bytes_identical():
    """SingleFileIndexDirectory slices (8-byte magic marker stripped) hold the V1 file's bytes."""
    v1 = S.load_segment_dir(os.path.join(PW, "legacyRawInverted_v1")).columns["category"].fwd
    v3 = S.load_segment_dir(os.path.join(PW, "legacyRawInverted_v3")).columns["category"].fwd
    assert v1 == v3 and len(v1) == 2569


@pytest.mark.parametrize("version", [4, 5, 6])
@pytest.mark.parametrize("comp", [S.PASS_THROUGH, S.SNAPPY, S.ZSTANDARD, S.LZ4, S.GZIP])
def test_var_byte_writer_reader_round_trip(version, comp):
    """Raw STRING writer (VarByteChunkForwardIndexWriterV4/V5/V6) against the oracle's reader, with
    multi-byte UTF-8, empty strings and huge values (a value alone in its chunk)."""
    rng = np.random.default_rng(version * 10 + comp)
    pool = ["alpha", "", "ünïcødé", "x" * 9000, "beta", "z" * 3]
    vals = [pool[i] for i in rng.integers(0, len(pool), 2500)]
    cb = S.build_column("c", np.array(vals, dtype=object), S.STRING, dictionary=False, raw_version=version,
                        compression=comp)
    assert oracle.var_byte_values(cb) == vals


@pytest.mark.parametrize("fmt", ["v1", "v3"])
def test_legacy_embedded_bitmaps_through_oracle(fmt):
    """The Pinot-written RoaringBitmaps embedded in the legacy raw-value inverted index
    (LegacyRawValueInvertedIndexCleanup.java:104-114) serve EQ / IN / NOT_EQ: the counts
    LegacyRawValueInvertedIndexMigrationIntegrationTest asserts, and the same docIds as the forward index."""
    from helpers import legacy_inverted_segment
    from pinot_amd.query import parse_sql
    e = EXP["legacy_raw_string"]
    seg = legacy_inverted_segment(fmt)
    c = e["column"]
    wheres = {f"{c} = '{v}'": cnt for v, cnt in e["counts"].items()}
    wheres[f"{c} IN ('alpha', 'beta')"] = e["in_alpha_beta"]
    wheres[f"{c} != 'alpha'"] = e["not_eq_alpha"]
    os_ = oracle.OracleSegment(seg)
    for w, cnt in wheres.items():
        q = f"SELECT COUNT(*) FROM t WHERE {w}"
        assert oracle.execute(q, [seg], use_inverted=True)[0] == cnt, w
        b_inv, _ = os_.filter_bitset(parse_sql(q), use_inverted=True)
        b_fwd, _ = os_.filter_bitset(parse_sql(q), use_inverted=False)
        assert np.array_equal(b_inv, b_fwd), w
