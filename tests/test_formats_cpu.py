"""CPU tests: segment byte formats vs the oracle's restated readers, the SQL front end, and the
C ABI library exporting every symbol include/pinot_amd.h declares (no device calls)."""
import ctypes as C
import os
import re
import struct

import numpy as np
import pytest

import oracle
from pinot_amd import segment as S
from pinot_amd.query import parse_sql, to_cnf

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("bits", list(range(1, 32)))
def test_fixed_bit_pack_matches_pinot_writer_and_reader(bits):
    rng = np.random.default_rng(bits)
    n = 517  # ragged
    vals = rng.integers(0, 1 << bits, n).astype(np.int32)
    packed = S.pack_fixed_bit(vals, bits)
    assert len(packed) == (n * bits + 7) // 8
    # PinotDataBitSet.writeInt restatement produces identical bytes
    buf = np.zeros(len(packed) + 8, dtype=np.uint8)
    oracle.lib().oracle_fixedbit_write(buf.ctypes.data, bits, 0, n, vals.ctypes.data)
    assert bytes(buf[:len(packed)]) == packed
    # PinotDataBitSet.readInt restatement reads every value back
    out = np.zeros(n, dtype=np.int32)
    pb = np.frombuffer(packed + b"\0" * 8, dtype=np.uint8)
    oracle.lib().oracle_fixedbit_read_range(pb.ctypes.data, bits, 0, n, out.ctypes.data)
    assert np.array_equal(out, vals)
    assert np.array_equal(S.unpack_fixed_bit(packed, bits, n), vals)


def test_fixed_bit_known_bytes():
    # 3-bit values 1,2,3,4,5 -> 001 010 011 100 101 -> 00101001 11001010 (padded)
    assert S.pack_fixed_bit(np.array([1, 2, 3, 4, 5]), 3) == bytes([0b00101001, 0b11001010])
    # getNumBitsPerValue examples from PinotDataBitSet.java:50-56
    assert [S.num_bits_per_value(v) for v in (0, 1, 2, 9, 113)] == [1, 1, 2, 4, 7]


@pytest.mark.parametrize("t", [S.INT, S.LONG, S.FLOAT, S.DOUBLE])
@pytest.mark.parametrize("version", [2, 3, 4])
def test_raw_forward_index_layout(t, version):
    rng = np.random.default_rng(1)
    v = rng.normal(0, 1e6, 3001)
    v = v.astype({S.INT: np.int32, S.LONG: np.int64, S.FLOAT: np.float32, S.DOUBLE: np.float64}[t])
    b = S.raw_fwd_bytes(v, t, version=version, docs_per_chunk=1000)
    h = S.parse_raw_fwd_header(b)
    assert (h.version, h.total_docs, h.compression, h.size_of_entry) == (version, 3001, 0, S.VALUE_SIZE[t])
    assert h.docs_per_chunk == (1024 if version >= 4 else 1000)
    raw = np.frombuffer(b, dtype=np.uint8)[h.raw_data_start:].copy()
    for i in (0, 1, 999, 1000, 3000):
        if t in (S.INT, S.LONG):
            assert oracle.lib().oracle_raw_read_i64(raw.ctypes.data, oracle.OR_TYPE[t], i) == int(v[i])
        else:
            assert oracle.lib().oracle_raw_read_f64(raw.ctypes.data, oracle.OR_TYPE[t], i) == float(v[i])


@pytest.mark.parametrize("kind", ["array", "bitmap", "run", "mixed", "empty"])
def test_roaring_roundtrip(kind):
    rng = np.random.default_rng(7)
    if kind == "array":
        docs = np.sort(rng.choice(200000, 3000, replace=False))
    elif kind == "bitmap":
        docs = np.sort(rng.choice(65536, 20000, replace=False))
    elif kind == "run":
        docs = np.r_[np.arange(10, 5000), np.arange(70000, 140000)]
    elif kind == "mixed":
        docs = np.unique(np.r_[np.arange(0, 30000), rng.choice(np.arange(65536, 131072), 9000), [200000, 262143]])
    else:
        docs = np.zeros(0, dtype=np.int64)
    ser = S.roaring_serialize(docs)
    n = 270000
    bits = np.zeros((n + 63) // 64, dtype=np.uint64)
    b = np.frombuffer(ser, dtype=np.uint8)
    assert oracle.lib().oracle_roaring_to_bitset(b.ctypes.data, len(ser), bits.ctypes.data, n) == 0
    out = np.zeros(n, dtype=np.int32)
    m = oracle.lib().oracle_bitset_to_doc_ids(bits.ctypes.data, n, out.ctypes.data)
    assert np.array_equal(out[:m], docs)


def test_roaring_known_bytes():
    # {1, 2, 65536}: two array containers, no runs -> cookie 12346, size 2, headers, offsets, payload
    ser = S.roaring_serialize(np.array([1, 2, 65536]))
    assert struct.unpack_from("<ii", ser) == (12346, 2)
    assert struct.unpack_from("<HHHH", ser, 8) == (0, 1, 1, 0)
    assert struct.unpack_from("<ii", ser, 16) == (24, 28)
    assert struct.unpack_from("<HHH", ser, 24) == (1, 2, 0)


def test_inverted_and_sorted_index_consistent():
    rng = np.random.default_rng(3)
    vals = rng.integers(0, 50, 10000)
    col = S.build_column("c", vals.astype(np.int32), S.INT, inverted=True, detect_sorted=False)
    inv = np.frombuffer(col.inverted, dtype=np.uint8)
    for d in (0, 7, 49):
        bits = np.zeros(10000 // 64 + 1, dtype=np.uint64)
        ids = np.array([d], dtype=np.int32)
        assert oracle.lib().oracle_inverted_to_bitset(inv.ctypes.data, col.cardinality, ids.ctypes.data, 1,
                                                      bits.ctypes.data, 10000) == 0
        out = np.zeros(10000, dtype=np.int32)
        m = oracle.lib().oracle_bitset_to_doc_ids(bits.ctypes.data, 10000, out.ctypes.data)
        assert np.array_equal(out[:m], np.nonzero(vals == col.dict_values[d])[0])
    s = S.build_column("s", np.sort(vals).astype(np.int32), S.INT)
    assert s.is_sorted
    sp = np.frombuffer(s.fwd, dtype=np.uint8)
    for doc in (0, 1, 5000, 9999):
        assert oracle.lib().oracle_sorted_dict_id(sp.ctypes.data, s.cardinality, doc) == \
            int(np.searchsorted(s.dict_values, np.sort(vals)[doc]))


def test_sql_front_end():
    qc = parse_sql("SELECT COUNT(*), SUM(a) AS s FROM t WHERE a > 3 AND (b IN (1, 2) OR NOT c = 'x') "
                   "AND d BETWEEN 1 AND 5 GROUP BY g1, g2 ORDER BY s DESC LIMIT 3")
    assert [a.func for a in qc.aggregations] == ["COUNT", "SUM"]
    assert qc.group_by == ["g1", "g2"] and qc.limit == 3 and qc.order_by == [("s", False)]
    cnf = qc.cnf
    assert len(cnf) == 3 and len(cnf[1]) == 2
    (p, neg), = cnf[0]
    assert p.type == "RANGE" and p.lower == 3 and not p.lower_inclusive and p.upper is None and not neg
    assert cnf[1][1][1] is True  # NOT c = 'x' -> negated leaf
    # De Morgan: NOT (a OR b) -> two clauses
    assert len(to_cnf(parse_sql("SELECT COUNT(*) FROM t WHERE NOT (a = 1 OR b = 2)").filter)) == 2
    with pytest.raises(ValueError):
        parse_sql("SELECT COUNT(*) FROM t WHERE a LIKE 'x'")


def test_capi_exports_every_declared_symbol():
    from pinot_amd import _lib
    header = open(os.path.join(ROOT, "include", "pinot_amd.h")).read()
    header = re.sub(r"/\*.*?\*/", "", header, flags=re.S)  # drop comments
    declared = set(re.findall(r"\b(pinot_amd_[a-z0-9_]+)\s*\(", header))
    assert declared, "no declarations parsed"
    assert declared == set(_lib.SIGNATURES), declared ^ set(_lib.SIGNATURES)
    L = _lib.lib()  # loads libpinot_amd.so; no device call
    for name in declared:
        assert hasattr(L, name), name
    assert L.pinot_amd_abi_version() == 1
    assert L.pinot_amd_required_padding() >= 8192


def test_jit_codegen_compiles_for_gfx950():
    """The query-specialised kernels the planner generates compile with hipRTC (no device needed)."""
    from pinot_amd import _lib
    assert _lib.lib().pinot_amd_jit_selftest(0) == 0


@pytest.mark.parametrize("comp", [S.LZ4, S.LZ4_LENGTH_PREFIXED])
@pytest.mark.parametrize("t", [S.INT, S.LONG, S.DOUBLE])
def test_lz4_chunks_roundtrip_through_oracle(comp, t):
    """Raw forward index with LZ4 chunks (Pinot's default for raw dimension columns,
    ForwardIndexType.getDefaultCompressionType) decodes to the original values."""
    rng = np.random.default_rng(comp)
    v = rng.integers(0, 40, 7001) if t != S.DOUBLE else rng.integers(0, 40, 7001) * 0.5
    v = v.astype({S.INT: np.int32, S.LONG: np.int64, S.DOUBLE: np.float64}[t])
    col = S.build_column("c", v, t, dictionary=False, compression=comp)
    h = S.parse_raw_fwd_header(col.fwd)
    assert h.compression == comp and len(col.fwd) < 7001 * S.VALUE_SIZE[t]
    raw = oracle.raw_values_region(col)
    got = np.frombuffer(raw[:v.nbytes].tobytes(), dtype=v.dtype.newbyteorder(">"))
    assert np.array_equal(got, v)


def test_lz4_known_block():
    # literal-only block and a block with an overlapping match (offset 1, run of 'a')
    assert oracle.lib().oracle_lz4_decompress(b"\x30abc", 4, (C.c_uint8 * 8)(), 8) == 3
    dst = (C.c_uint8 * 32)()
    blk = bytes([0x1F, ord("a"), 1, 0, 0x01, 0x50]) + b"bcdef"  # 'a' + match(off 1, len 4+15+1) + 'bcdef'
    n = oracle.lib().oracle_lz4_decompress(blk, len(blk), dst, 32)
    assert bytes(dst[:n]) == b"a" * 21 + b"bcdef"


ALL_CODECS = [S.SNAPPY, S.ZSTANDARD, S.LZ4, S.LZ4_LENGTH_PREFIXED, S.GZIP, S.DELTA, S.DELTADELTA]


def _codec_values(t, n, rng):
    if t in (S.INT, S.LONG):
        info = np.iinfo(np.int32 if t == S.INT else np.int64)
        v = np.cumsum(rng.integers(-3, 9, n)).astype(np.int64) + 1_600_000_000  # timestamp-like runs
        v[::97] = info.max  # wrap-around deltas
        v[1::131] = info.min
        return v.astype(np.int32 if t == S.INT else np.int64)
    return (rng.integers(0, 40, n) * 0.5).astype(np.float32 if t == S.FLOAT else np.float64)


@pytest.mark.parametrize("comp", ALL_CODECS)
@pytest.mark.parametrize("t", [S.INT, S.LONG, S.FLOAT, S.DOUBLE])
def test_chunk_codecs_roundtrip_through_oracle(comp, t):
    """Every ChunkCompressionType (ChunkCompressionType.java:22) written chunk by chunk and read back
    by the oracle's decompressors. 7001 INT values in 1024-doc chunks exercise both of DELTA's
    layouts: full chunks are a multiple of 8 bytes (LONG flag), the ragged last chunk is not."""
    if comp in (S.DELTA, S.DELTADELTA) and t not in (S.INT, S.LONG):
        pytest.skip("DELTA codecs hold INT/LONG values")
    v = _codec_values(t, 7001, np.random.default_rng(comp * 10 + len(t)))
    col = S.build_column("c", v, t, dictionary=False, compression=comp)
    h = S.parse_raw_fwd_header(col.fwd)
    assert h.compression == comp and h.num_chunks == 7
    raw = oracle.raw_values_region(col)
    got = np.frombuffer(raw[:v.nbytes].tobytes(), dtype=v.dtype.newbyteorder(">"))
    assert np.array_equal(got, v)


def test_snappy_known_block():
    # varint length 9, literal "abc", copy-1 (length 6, offset 3, overlapping) -> "abcabcabc"
    blk = bytes([9, 0x08]) + b"abc" + bytes([0x09, 0x03])
    dst = (C.c_uint8 * 16)()
    assert oracle.lib().oracle_snappy_decompress(blk, len(blk), dst, 16) == 9
    assert bytes(dst[:9]) == b"abcabcabc"
    assert oracle.lib().oracle_snappy_decompress(blk[:-1], len(blk) - 1, dst, 16) == -1  # truncated


def test_delta_known_chunk():
    # DeltaCompressor INT layout for [5, 7, 4]: flag 0, count 3, first 5, LZ4(deltas 2, -3)
    d = S.lz4_block_compress(np.array([2, -3], dtype=">i4").tobytes())
    blk = bytes([0]) + (3).to_bytes(4, "big") + (5).to_bytes(4, "big") + len(d).to_bytes(4, "big") + d
    dst = (C.c_uint8 * 12)()
    assert oracle.lib().oracle_delta_decompress(blk, len(blk), dst, 12, 0) == 12
    assert np.array_equal(np.frombuffer(bytes(dst), dtype=">i4"), [5, 7, 4])
    # the same bytes as DELTADELTA: first delta 2, then delta-of-delta -3 -> [5, 7, 6]
    assert oracle.lib().oracle_delta_decompress(blk, len(blk), dst, 12, 1) == 12
    assert np.array_equal(np.frombuffer(bytes(dst), dtype=">i4"), [5, 7, 6])


def test_vectorised_inverted_index_matches_general_builder():
    """inverted_index_bytes_fast (numpy) == one roaring_serialize per bitmap, byte for byte, and
    declines inputs that need bitmap or run containers."""
    rng = np.random.default_rng(3)
    for n, card in [(1, 1), (1000, 7), (100_000, 1000), (300_000, 50_000), (70_001, 9000)]:
        ids = rng.integers(0, card, n)
        ids[:min(card, n)] = np.arange(min(card, n))
        fast = S.inverted_index_bytes_fast(ids, card)
        assert fast is not None
        assert fast == S.inverted_index_bytes_general(ids, card)
    assert S.inverted_index_bytes_fast(rng.integers(0, 2, 70_000), 2) is None       # bitmap containers
    assert S.inverted_index_bytes_fast(np.zeros(100, np.int64), 1) is None           # one run
