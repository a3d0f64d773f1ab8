"""ctypes driver of the CPU oracle (libpinot_oracle.so). TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use this module; the
product path (pinot_amd/) never imports it, and it imports nothing of the product: SQL text is compiled by
oracle_sql.py, segment byte formats are parsed here and in pinot_oracle.c.

The predicate resolution below is an independent Python restatement of
pinot-core/.../operator/filter/predicate/PredicateEvaluatorProvider.java and the factories it
calls (RangePredicateEvaluatorFactory, InPredicateEvaluatorFactory, EqualsPredicateEvaluatorFactory,
NotEquals/NotIn): dictionary-encoded columns resolve values to dictIds, raw columns keep values
with RANGE bounds normalised to inclusive ones. The per-doc work happens in pinot_oracle.c.
"""
from __future__ import annotations

import bisect
import ctypes as C
import math
import os
import subprocess
from typing import Dict, List, Sequence

import numpy as np

import dataclasses

from oracle_sql import OAgg as Aggregation, OQuery as QueryContext, parse as _parse_sql  # the oracle's own SQL front end
from oracle_reduce import JDouble, identity_key, java_identity, merge
from oracle_reduce import rows as reduce_rows

# Segments arrive as the test fixtures' column-buffer records (name, stored_type, num_docs, has_dictionary,
# encoding, cardinality, bits_per_element, fwd / dictionary / inverted bytes, dict_values); the oracle reads
# their attributes only and parses every byte format itself (no product code in the checker).
INT, LONG, FLOAT, DOUBLE, STRING = "INT", "LONG", "FLOAT", "DOUBLE", "STRING"  # FieldSpec.DataType names
ColumnBuffers = SegmentBuffers = object  # annotations only

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "libpinot_oracle.so")

OR_TYPE = {INT: 0, LONG: 1, FLOAT: 2, DOUBLE: 3}
OR_ENC = {"FIXED_BIT": 0, "RAW": 1, "SORTED": 2}
DICT_RANGE, DICT_SET, RAW_RANGE, RAW_IN, DOC_BITSET = 0, 1, 2, 3, 4
AGG = {"COUNT": 0, "SUM": 1, "MIN": 2, "MAX": 3, "SUMLONG": 4, "RMIN": 5, "RMAX": 6}


class OColumn(C.Structure):
    _fields_ = [("encoding", C.c_int32), ("stored_type", C.c_int32), ("bits", C.c_int32), ("cardinality", C.c_int32),
                ("fwd", C.c_void_p), ("dict", C.c_void_p)]


class OLeaf(C.Structure):
    _fields_ = [("column", C.c_int32), ("kind", C.c_int32), ("negate", C.c_int32), ("clause", C.c_int32),
                ("lo_i", C.c_int64), ("hi_i", C.c_int64), ("lo_d", C.c_double), ("hi_d", C.c_double),
                ("dict_mask", C.c_void_p), ("set_i", C.c_void_p), ("set_d", C.c_void_p), ("set_n", C.c_int32),
                ("doc_bitset", C.c_void_p)]


class OAgg(C.Structure):
    _fields_ = [("func", C.c_int32), ("column", C.c_int32), ("expr", C.c_int32), ("column2", C.c_int32)]


EXPR = {"COL": 0, "MUL": 1, "SUB": 2, "ADD": 3}


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            subprocess.run(["make", "-C", HERE, "-s"], check=True)
        L = C.CDLL(LIB)
        P, I64 = C.c_void_p, C.c_int64
        L.oracle_fixedbit_read.restype = C.c_int32
        L.oracle_fixedbit_read.argtypes = [P, C.c_int32, I64]
        L.oracle_fixedbit_read_range.argtypes = [P, C.c_int32, I64, I64, P]
        L.oracle_fixedbit_write.argtypes = [P, C.c_int32, I64, I64, P]
        L.oracle_sorted_dict_id.restype = C.c_int32
        L.oracle_sorted_dict_id.argtypes = [P, C.c_int32, I64]
        L.oracle_raw_read_i64.restype = I64
        L.oracle_raw_read_i64.argtypes = [P, C.c_int32, I64]
        L.oracle_raw_read_f64.restype = C.c_double
        L.oracle_raw_read_f64.argtypes = [P, C.c_int32, I64]
        L.oracle_column_dict_ids.argtypes = [C.POINTER(OColumn), I64, I64, P]
        L.oracle_roaring_to_bitset.argtypes = [P, I64, P, I64]
        L.oracle_lz4_decompress.restype = I64
        L.oracle_lz4_decompress.argtypes = [P, I64, P, I64]
        L.oracle_snappy_decompress.restype = I64
        L.oracle_snappy_decompress.argtypes = [P, I64, P, I64]
        L.oracle_delta_decompress.restype = I64
        L.oracle_delta_decompress.argtypes = [P, I64, P, I64, C.c_int32]
        L.oracle_inverted_to_bitset.argtypes = [P, C.c_int32, P, C.c_int32, P, I64]
        L.oracle_filter.restype = I64
        L.oracle_filter.argtypes = [C.POINTER(OColumn), I64, C.POINTER(OLeaf), C.c_int32, P]
        L.oracle_bitset_to_doc_ids.restype = I64
        L.oracle_bitset_to_doc_ids.argtypes = [P, I64, P]
        L.oracle_aggregate.argtypes = [C.POINTER(OColumn), I64, P, C.POINTER(OAgg), C.c_int32, P, P, P]
        L.oracle_set_literal_int_sum.argtypes = [C.c_int32]
        L.oracle_literal_int_sum.restype = C.c_int32
        L.oracle_group_by.restype = I64
        L.oracle_group_by.argtypes = [C.POINTER(OColumn), I64, P, P, C.c_int32, C.POINTER(OAgg), C.c_int32, I64, I64,
                                      P, P, P, P, P]
        _lib = L
    return _lib


def _ptr(a: np.ndarray) -> int:
    return a.ctypes.data


# -------------------------------------------------------------------------------- predicate resolution
def _java_key(s: str) -> bytes:
    return s.encode("utf-16-be")


def _coerce(v, t):
    if t == STRING:
        return str(v)
    if t in (INT, LONG):
        return int(v)
    return float(v)


def _dict_positions(col: ColumnBuffers, values) -> List[int]:
    """Dictionary.indexOf for each value; values absent from the dictionary are dropped."""
    d = col.dict_values
    out = []
    if col.stored_type == STRING:
        keys = [_java_key(x) for x in d]
        for v in values:
            k = _java_key(_coerce(v, STRING))
            i = bisect.bisect_left(keys, k)
            if i < len(keys) and keys[i] == k:
                out.append(i)
    else:
        for v in values:
            x = _coerce(v, col.stored_type)
            i = int(np.searchsorted(d, x, side="left"))
            if i < len(d) and d[i] == x:
                out.append(i)
    return sorted(set(out))


def _dict_range(col: ColumnBuffers, p):
    """SortedDictionaryBasedRangePredicateEvaluator: [start, end) of dictIds."""
    d = col.dict_values
    if col.stored_type == STRING:
        keys = [_java_key(x) for x in d]

        def ss(v, side):
            k = _java_key(str(v))
            return bisect.bisect_left(keys, k) if side == "left" else bisect.bisect_right(keys, k)
    else:
        def ss(v, side):
            return int(np.searchsorted(d, _coerce(v, col.stored_type), side=side))
    start = 0 if p.lower is None else ss(p.lower, "left" if p.lower_inclusive else "right")
    end = len(d) if p.upper is None else ss(p.upper, "right" if p.upper_inclusive else "left")
    return start, max(end, start)


def _raw_range(col: ColumnBuffers, p):
    """*RawValueBasedRangePredicateEvaluator: inclusive bounds, unbounded = type min/max."""
    t = col.stored_type
    if t in (INT, LONG):
        info = np.iinfo(np.int32 if t == INT else np.int64)
        lo = info.min if p.lower is None else int(p.lower) + (0 if p.lower_inclusive else 1)
        hi = info.max if p.upper is None else int(p.upper) - (0 if p.upper_inclusive else 1)
        return lo, hi
    if t == FLOAT:
        f = np.float32
        lo = -math.inf if p.lower is None else float(f(p.lower) if p.lower_inclusive else np.nextafter(f(p.lower), f(np.inf)))
        hi = math.inf if p.upper is None else float(f(p.upper) if p.upper_inclusive else np.nextafter(f(p.upper), f(-np.inf)))
        return lo, hi
    lo = -math.inf if p.lower is None else (float(p.lower) if p.lower_inclusive else float(np.nextafter(float(p.lower), np.inf)))
    hi = math.inf if p.upper is None else (float(p.upper) if p.upper_inclusive else float(np.nextafter(float(p.upper), -np.inf)))
    return lo, hi


def decompress_chunk(comp: int, src: np.ndarray, dst: np.ndarray, want: int) -> int:
    """ChunkDecompressor per ChunkCompressionType (ChunkCompressorFactory.getDecompressor):
    LZ4 / SNAPPY / DELTA / DELTADELTA restated in pinot_oracle.c; ZSTANDARD (zstd-jni) through
    pyarrow's bundled libzstd and GZIP (java.util.zip.Inflater, zlib stream + BE size) through
    Python's zlib -- third-party entropy decoders used as-is by this checker."""
    if comp in (3, 4):
        return lib().oracle_lz4_decompress(src.ctypes.data, src.size, dst.ctypes.data, want)
    if comp == 1:
        return lib().oracle_snappy_decompress(src.ctypes.data, src.size, dst.ctypes.data, want)
    if comp in (6, 7):
        return lib().oracle_delta_decompress(src.ctypes.data, src.size, dst.ctypes.data, want, int(comp == 7))
    if comp == 2:
        import pyarrow as pa
        raw = pa.Codec("zstd").decompress(src.tobytes(), decompressed_size=want, asbytes=True)
    elif comp == 5:
        import zlib
        raw = zlib.decompress(src[:-4].tobytes())
    else:
        raise NotImplementedError(comp)
    dst[:len(raw)] = np.frombuffer(raw, dtype=np.uint8)
    return len(raw)


def var_byte_values(cb: ColumnBuffers) -> List[str]:
    """Every doc's value of a raw STRING forward index, as VarByteChunkForwardIndexReaderV4 / V5 / V6
    read it (segment/index/readers/forward/VarByteChunkForwardIndexReaderV4.java): BE header, LE chunk
    metadata (MSB of docIdOffset marks a huge single-value chunk), LE chunks of offsets (V6 with a codec:
    sizes) and UTF-8 bytes."""
    import struct
    b = cb.fwd
    version, target, comp, chunks_off = struct.unpack_from(">4i", b, 0)
    assert 4 <= version <= 6, version
    n = (chunks_off - 16) // 8
    meta = [struct.unpack_from("<Ii", b, 16 + 8 * k) for k in range(n)]
    out: List[str] = []
    for k, (dw, co) in enumerate(meta):
        s = chunks_off + co
        e = chunks_off + meta[k + 1][1] if k + 1 < n else len(b)
        src = np.frombuffer(b[s:e], dtype=np.uint8).copy()
        if comp == 0:
            raw = src.tobytes()
        else:
            if comp == 4:  # LZ4CompressorWithLength: LE decompressed length first
                want = int.from_bytes(src[:4].tobytes(), "little")
                src = src[4:].copy()
            elif comp == 1:  # snappy varint preamble
                want, sh, i = 0, 0, 0
                while True:
                    want |= (int(src[i]) & 127) << sh
                    sh += 7
                    i += 1
                    if not src[i - 1] & 128:
                        break
            elif comp == 5:
                want = int.from_bytes(src[-4:].tobytes(), "big")
            elif comp == 2:
                want = _zstd_content_size(src.tobytes())
            else:
                want = 2 * target + 64
            dst = np.zeros(want + 64, dtype=np.uint8)
            got = decompress_chunk(comp, src, dst, want)
            raw = dst[:got].tobytes()
        if dw & 0x80000000:
            out.append(raw.decode("utf-8"))
            continue
        nd = int.from_bytes(raw[:4], "little")
        ints = struct.unpack_from("<%di" % nd, raw, 4)
        if version == 6 and comp != 0:
            pos = 4 * (nd + 1)
            for size in ints:
                out.append(raw[pos:pos + size].decode("utf-8"))
                pos += size
        else:
            for i in range(nd):
                out.append(raw[ints[i]:ints[i + 1] if i + 1 < nd else len(raw)].decode("utf-8"))
    assert len(out) == cb.num_docs, (len(out), cb.num_docs)
    return out


def _zstd_content_size(fr: bytes) -> int:
    """Frame_Content_Size of a zstd frame header (RFC 8878 3.1.1.1)."""
    d = fr[4]
    fcs_flag, single, did = d >> 6, (d >> 5) & 1, d & 3
    pos = 5 + (0 if single else 1) + (0, 1, 2, 4)[did]
    size = (1 if single else 0, 2, 4, 8)[fcs_flag]
    v = int.from_bytes(fr[pos:pos + size], "little")
    return v + 256 if size == 2 else v


class _RawHeader:
    """BaseChunkForwardIndexReader's header fields (BaseChunkForwardIndexReader.java:60-105): version,
    chunk count, docs per chunk, entry size, then (version >= 2) total docs, ChunkCompressionType and the
    data header start; version 1 files are SNAPPY with a 16-byte header."""

    def __init__(self, buf: bytes):
        import struct
        self.version, self.num_chunks, self.docs_per_chunk, self.size_of_entry = struct.unpack_from(">4i", buf, 0)
        if self.version > 1:
            self.total_docs, self.compression, self.data_header_start = struct.unpack_from(">3i", buf, 16)
        else:
            self.total_docs, self.compression, self.data_header_start = -1, 1, 16
        self.raw_data_start = self.data_header_start + self.num_chunks * (4 if self.version <= 2 else 8)


def parse_raw_fwd_header(buf: bytes) -> _RawHeader:
    return _RawHeader(buf)


def _bits_per_value(max_value: int) -> int:
    """PinotDataBitSet.getNumBitsPerValue (PinotDataBitSet.java:61-72): at least one bit."""
    return 1 if max_value <= 1 else int(max_value).bit_length()


def _dictionary_twin(cb: ColumnBuffers) -> ColumnBuffers:
    """ForwardIndexHandler ENABLE_DICTIONARY restated for a raw STRING column: the sorted distinct values
    (SegmentDictionaryCreator; String.compareTo order = UTF-16 code units) and a fixed-bit dictId forward
    index written by the oracle's own PinotDataBitSet.writeInt restatement (oracle_fixedbit_write)."""
    vals = var_byte_values(cb)
    uniq = sorted(set(vals), key=lambda v: v.encode("utf-16-be"))
    index = {v: i for i, v in enumerate(uniq)}
    ids = np.fromiter((index[v] for v in vals), dtype=np.int32, count=len(vals))
    card = max(len(uniq), 1)
    bits = _bits_per_value(card - 1)
    packed = np.zeros((len(vals) * bits + 7) // 8 + 16, dtype=np.uint8)
    lib().oracle_fixedbit_write(_ptr(packed), bits, 0, len(vals), _ptr(ids))
    width = max([len(v.encode("utf-8")) for v in uniq] + [1])
    dict_bytes = b"".join(v.encode("utf-8").ljust(width, b"\0") for v in uniq)
    return dataclasses.replace(cb, has_dictionary=True, is_sorted=False, cardinality=card, bits_per_element=bits,
                               fwd=packed[:(len(vals) * bits + 7) // 8].tobytes(), dictionary=dict_bytes,
                               inverted=None, dict_values=np.array(uniq, dtype=object))


def raw_values_region(cb: ColumnBuffers) -> np.ndarray:
    """The contiguous big-endian values of a raw forward index: the data region of PASS_THROUGH
    chunks, or the LZ4 / LZ4_LENGTH_PREFIXED chunks decoded one by one
    (BaseChunkForwardIndexReader.decompressChunk, BaseChunkForwardIndexReader.java:150-185)."""
    h = parse_raw_fwd_header(cb.fwd)
    fb = np.frombuffer(cb.fwd, dtype=np.uint8)
    if h.compression == 0:
        return fb[h.raw_data_start:].copy()
    assert h.compression in range(1, 8), h.compression
    off_size = 4 if h.version <= 2 else 8
    offs = np.frombuffer(cb.fwd, dtype=">i4" if off_size == 4 else ">i8", count=h.num_chunks,
                         offset=h.data_header_start).astype(np.int64)
    ends = np.r_[offs[1:], len(cb.fwd)]
    total = cb.num_docs * h.size_of_entry
    out = np.zeros(total + 16, dtype=np.uint8)
    pos = 0
    for s, e in zip(offs, ends):
        src = fb[s + (4 if h.compression == 4 else 0):e].copy()
        want = min(h.docs_per_chunk * h.size_of_entry, total - pos)
        got = decompress_chunk(h.compression, src, out[pos:], want)
        assert got == want, (h.compression, got, want)
        pos += want
    return out


class OracleSegment:
    """Host view of one segment's buffers in the oracle's column layout."""

    def __init__(self, seg: SegmentBuffers):
        if any(c.stored_type == STRING and not c.has_dictionary for c in seg.columns.values()):
            seg = dataclasses.replace(seg, columns={
                n: _dictionary_twin(c) if (c.stored_type == STRING and not c.has_dictionary) else c
                for n, c in seg.columns.items()})
        self.seg = seg
        self.names = list(seg.columns)
        self.index = {n: i for i, n in enumerate(self.names)}
        self._keep = []
        cols = (OColumn * (2 * len(self.names)))()  # second half: raw columns' group ids, on demand
        self._raw_groups = {}
        for i, n in enumerate(self.names):
            cb = seg.columns[n]
            oc = cols[i]
            oc.encoding = OR_ENC[cb.encoding]
            oc.stored_type = OR_TYPE.get(cb.stored_type, 0)
            oc.bits = cb.bits_per_element
            oc.cardinality = cb.cardinality
            if cb.encoding == "RAW":
                buf = raw_values_region(cb)
            else:
                buf = np.frombuffer(cb.fwd, dtype=np.uint8).copy()
                buf = np.concatenate([buf, np.zeros(16, np.uint8)])  # reads of the last byte's neighbour
            self._keep.append(buf)
            oc.fwd = _ptr(buf)
            if cb.has_dictionary and cb.stored_type != STRING:
                dv = np.ascontiguousarray(cb.dict_values)
                self._keep.append(dv)
                oc.dict = _ptr(dv)
        self.cols = cols

    def leaves(self, qc: QueryContext, use_inverted: bool = True):
        out = []
        n = self.seg.num_docs
        for ci, clause in enumerate(qc.cnf):
            for p, neg in clause:
                cb = self.seg.columns[p.column]
                lf = OLeaf()
                lf.column = self.index[p.column]
                lf.clause = ci
                lf.negate = 1 if neg else 0
                negated_type = p.type in ("NOT_EQ", "NOT_IN")
                if negated_type:
                    lf.negate ^= 1
                if cb.has_dictionary:
                    if p.type == "RANGE":
                        s, e = _dict_range(cb, p)
                        ids = list(range(s, e))
                    else:
                        ids = _dict_positions(cb, p.values)
                    if use_inverted and cb.inverted is not None and p.type != "RANGE":
                        bits = np.zeros((n + 63) // 64 + 1, dtype=np.uint64)
                        idarr = np.array(ids, dtype=np.int32)
                        inv = np.frombuffer(cb.inverted, dtype=np.uint8)
                        rc = lib().oracle_inverted_to_bitset(_ptr(inv), cb.cardinality, _ptr(idarr), len(ids),
                                                             _ptr(bits), n)
                        assert rc == 0, rc
                        self._keep += [bits, idarr, inv]
                        lf.kind = DOC_BITSET
                        lf.doc_bitset = _ptr(bits)
                    elif p.type == "RANGE":
                        lf.kind = DICT_RANGE
                        lf.lo_i, lf.hi_i = ids[0] if ids else 0, (ids[-1] + 1) if ids else 0
                    else:
                        mask = np.zeros(cb.cardinality + 1, dtype=np.uint8)
                        mask[ids] = 1
                        self._keep.append(mask)
                        lf.kind = DICT_SET
                        lf.dict_mask = _ptr(mask)
                else:
                    if p.type == "RANGE":
                        lf.kind = RAW_RANGE
                        lo, hi = _raw_range(cb, p)
                        if cb.stored_type in (INT, LONG):
                            lf.lo_i, lf.hi_i = lo, hi
                        else:
                            lf.lo_d, lf.hi_d = lo, hi
                    else:
                        lf.kind = RAW_IN
                        if cb.stored_type in (INT, LONG):
                            arr = np.array([int(v) for v in p.values], dtype=np.int64)
                            lf.set_i = _ptr(arr)
                        else:
                            arr = np.array([float(np.float32(v)) if cb.stored_type == FLOAT else float(v)
                                            for v in p.values], dtype=np.float64)
                            lf.set_d = _ptr(arr)
                        lf.set_n = len(arr)
                        self._keep.append(arr)
                out.append(lf)
        arr = (OLeaf * max(len(out), 1))(*out)
        return arr, len(out)

    def filter_bitset(self, qc: QueryContext, use_inverted: bool = True):
        n = self.seg.num_docs
        bits = np.zeros((n + 63) // 64 + 1, dtype=np.uint64)
        leaves, nl = self.leaves(qc, use_inverted)
        cnt = lib().oracle_filter(self.cols, n, leaves, nl, _ptr(bits))
        return bits, int(cnt)

    def group_col(self, g: str) -> int:
        """Column index that yields group ids for GROUP BY g. Dictionary columns group by dictId
        (DictionaryBasedGroupKeyGenerator); raw columns by value (NoDictionarySingleColumnGroupKeyGenerator
        .java:98-143: a fastutil open hash map per stored type, whose key equality for FLOAT/DOUBLE is
        floatToIntBits/doubleToLongBits, i.e. all NaNs equal and -0.0 != 0.0). Restated as ids into the
        distinct canonical bit patterns of the column."""
        cb = self.seg.columns[g]
        if cb.encoding != "RAW":
            return self.index[g]
        if g not in self._raw_groups:
            vals = np.frombuffer(raw_values_region(cb).tobytes(), dtype=np.dtype(
                {INT: ">i4", LONG: ">i8", FLOAT: ">f4", DOUBLE: ">f8"}[cb.stored_type]),
                count=self.seg.num_docs).astype(np.dtype({INT: "i4", LONG: "i8", FLOAT: "f4", DOUBLE: "f8"}[cb.stored_type]))
            if cb.stored_type in (FLOAT, DOUBLE):
                bits = vals.view(np.uint32 if cb.stored_type == FLOAT else np.uint64).copy()
                bits[np.isnan(vals)] = 0x7FC00000 if cb.stored_type == FLOAT else 0x7FF8000000000000
                uniq, ids = np.unique(bits, return_inverse=True)
                dvals = uniq.view(vals.dtype)
            else:
                dvals, ids = np.unique(vals, return_inverse=True)
            ids = np.ascontiguousarray(ids.astype(np.int32))
            i = len(self.names) + self.index[g]
            oc = self.cols[i]
            oc.encoding = 3  # OR_ENC_IDS
            oc.stored_type = OR_TYPE[cb.stored_type]
            oc.cardinality = len(dvals)
            oc.fwd = _ptr(ids)
            self._keep.append(ids)
            self._raw_groups[g] = (i, dvals)
        return self._raw_groups[g][0]

    def values(self, col: str) -> np.ndarray:
        """Every doc's value of a column: dictionary values through the forward index's dictIds
        (FixedBitSVForwardIndexReaderV2 / SortedIndexReaderImpl + Dictionary.get), raw values decoded."""
        cb = self.seg.columns[col]
        n = self.seg.num_docs
        if cb.encoding == "RAW":
            return np.frombuffer(raw_values_region(cb).tobytes(), dtype=np.dtype(
                {INT: ">i4", LONG: ">i8", FLOAT: ">f4", DOUBLE: ">f8"}[cb.stored_type]), count=n)
        ids = np.zeros(max(n, 1), dtype=np.int32)
        lib().oracle_column_dict_ids(C.byref(self.cols[self.index[col]]), 0, n, _ptr(ids))
        dv = cb.dict_values if cb.stored_type != STRING else np.asarray(cb.dict_values, dtype=object)
        return dv[ids[:n]]

    def key_values(self, dict_ids, group_by: Sequence[str]) -> tuple:
        out = []
        for g, d in zip(group_by, dict_ids):
            cb = self.seg.columns[g]
            v = self._raw_groups[g][1][int(d)] if g in self._raw_groups else cb.dict_values[int(d)]
            out.append(v if cb.stored_type == STRING else (JDouble(v) if cb.stored_type in (FLOAT, DOUBLE) else int(v)))
        return tuple(out)


def parse_sql(query) -> QueryContext:
    """The oracle compiles SQL text itself (oracle_sql); an already compiled oracle query passes through."""
    if isinstance(query, str):
        return _parse_sql(query)
    if isinstance(query, QueryContext):
        return query
    raise TypeError("the oracle takes SQL text (it does not read the product's QueryContext)")


def execute(query, segments: Sequence[SegmentBuffers], use_inverted: bool = True, stats: dict = None,
            literal_int_sum: bool = False):
    """Run a query over segments on the CPU oracle: returns (num_docs_matched, groups) where groups
    maps key tuple -> intermediate results per aggregation (AVG as (sum, count)), combined across
    segments with AggregationFunction.merge semantics (GroupByCombineOperator's upsert by key).
    stats, when given, receives 'num_groups_limit_reached' (any segment's GroupByOperator flag).
    literal_int_sum: integer SUMs accumulate in double in doc order and merge as doubles in segment
    order, the reference's own arithmetic (SumAggregationFunction); default: exact, rounded once."""
    qc = parse_sql(query)
    if literal_int_sum:
        lib().oracle_set_literal_int_sum(1)
        try:
            return execute(qc, segments, use_inverted, stats)
        finally:
            lib().oracle_set_literal_int_sum(0)
    if any(a.func == "DISTINCTCOUNT" for a in qc.aggregations):
        return _distinct_count(qc, segments, use_inverted, stats)
    if stats is not None:
        stats["num_groups_limit_reached"] = False
    total = 0
    groups: Dict[tuple, list] = {}
    for seg in segments:
        os_ = OracleSegment(seg)
        if qc.cnf:
            bits, cnt = os_.filter_bitset(qc, use_inverted)
        else:
            bits, cnt = None, seg.num_docs
        total += cnt
        # native aggregations: AVG -> SUM + COUNT
        nat = []
        slots = []
        for a in qc.aggregations:
            if a.func == "AVG":
                nat.append(("SUM", a.column, a.expr))
                nat.append(("COUNT", "*", None))
                slots.append(("avg", len(nat) - 2, len(nat) - 1))
            elif a.func == "MINMAXRANGE":  # MinMaxRangeAggregationFunction: MinMaxRangePair(min, max)
                nat.append(("RMIN", a.column, a.expr))
                nat.append(("RMAX", a.column, a.expr))
                slots.append(("range", len(nat) - 2, len(nat) - 1))
            else:
                nat.append((a.func, a.column, a.expr))
                slots.append(("direct", len(nat) - 1))
        if not nat:
            nat.append(("COUNT", "*", None))
        def oagg(f, c, e):
            if c == "*":
                return OAgg(AGG[f], -1, 0, -1)
            if e is None or e[0] == "COL":
                return OAgg(AGG[f], os_.index[c if e is None else e[1]], 0, -1)
            return OAgg(AGG[f], os_.index[e[1]], EXPR[e[0]], os_.index[e[2]])
        aggs = (OAgg * len(nat))(*[oagg(f, c, e) for f, c, e in nat])
        int_sum = [f == "SUM" and _is_int_value(seg, c, e) and not _literal() for f, c, e in nat]
        bptr = _ptr(bits) if bits is not None else None
        if qc.group_by:
            cap = max(cnt, 1)
            keys = np.zeros(cap * len(qc.group_by), dtype=np.int32)
            vals = np.zeros(cap * len(nat), dtype=np.float64)
            vali = np.zeros(cap * len(nat), dtype=np.int64)
            valh = np.zeros(cap * len(nat), dtype=np.int64)
            gcols = np.array([os_.group_col(g) for g in qc.group_by], dtype=np.int32)
            reached = C.c_int32(0)
            ng = lib().oracle_group_by(os_.cols, seg.num_docs, bptr, _ptr(gcols), len(gcols), aggs, len(nat),
                                       qc.num_groups_limit, cap, _ptr(keys), _ptr(vals), _ptr(vali), _ptr(valh),
                                       C.byref(reached))
            assert ng >= 0, ng
            if stats is not None and reached.value:
                stats["num_groups_limit_reached"] = True
            seg_groups = {}
            for g in range(ng):
                kv = os_.key_values(keys[g * len(qc.group_by):(g + 1) * len(qc.group_by)], qc.group_by)
                sl = slice(g * len(nat), (g + 1) * len(nat))
                seg_groups[kv] = _parts(qc, slots, nat, vals[sl], vali[sl], valh[sl], int_sum)
        else:
            vals = np.zeros(len(nat), dtype=np.float64)
            vali = np.zeros(len(nat), dtype=np.int64)
            valh = np.zeros(len(nat), dtype=np.int64)
            lib().oracle_aggregate(os_.cols, seg.num_docs, bptr, aggs, len(nat), _ptr(vals), _ptr(vali), _ptr(valh))
            seg_groups = {(): _parts(qc, slots, nat, vals, vali, valh, int_sum)}
        for k, parts in seg_groups.items():
            if k in groups:
                groups[k] = [merge(a.func, x, y) for a, x, y in zip(qc.aggregations, groups[k], parts)]
            else:
                groups[k] = parts
    # integer SUM partials were carried as exact Python ints through the combine: round once
    for k, parts in groups.items():
        groups[k] = [(float(p[0]), p[1]) if a.func == "AVG" else float(p) if a.func == "SUM" else p
                     for a, p in zip(qc.aggregations, parts)]
    return total, groups


def cpu_plan(query, seg: SegmentBuffers, use_inverted: bool = True):
    """The per-doc C work of execute() for ONE segment, set up once: returns a zero-argument callable
    that re-runs the inverted-index leaves' bitmap expansion (BitmapBasedFilterOperator), the filter
    (ScanBasedFilterOperator / And / Or) and the aggregation or group-by (AggregationOperator /
    DefaultGroupByExecutor) in pinot_oracle.c and returns the matched-doc count. Predicate resolution,
    buffer setup and the Python conversion of the groups stay outside, so bench.py's cpu_baseline
    times what a Pinot server does per doc and per segment, not this module's Python."""
    qc = parse_sql(query)
    assert not any(a.func == "DISTINCTCOUNT" for a in qc.aggregations), "cpu_plan: no DISTINCTCOUNT"
    os_ = OracleSegment(seg)
    n = seg.num_docs
    L = lib()
    leaves, nl = os_.leaves(qc, use_inverted) if qc.cnf else (None, 0)
    inv_steps = []  # (inverted bytes, cardinality, dictIds, the leaf's bitset) of each inverted-index leaf
    nwords = (n + 63) // 64 + 1
    for i, (p, _neg) in enumerate(pn for clause in qc.cnf for pn in clause):
        if leaves[i].kind == DOC_BITSET:
            cb = seg.columns[p.column]
            idarr = np.array(_dict_positions(cb, p.values), dtype=np.int32)
            inv = np.frombuffer(cb.inverted, dtype=np.uint8)
            bits = np.ctypeslib.as_array(C.cast(leaves[i].doc_bitset, C.POINTER(C.c_uint64)), shape=(nwords,))
            inv_steps.append((inv, cb.cardinality, idarr, bits))
    fbits = np.zeros((n + 63) // 64 + 1, dtype=np.uint64)
    nat = []
    for a in qc.aggregations:
        if a.func == "AVG":
            nat += [("SUM", a.column, a.expr), ("COUNT", "*", None)]
        elif a.func == "MINMAXRANGE":
            nat += [("RMIN", a.column, a.expr), ("RMAX", a.column, a.expr)]
        else:
            nat.append((a.func, a.column, a.expr))
    if not nat:
        nat.append(("COUNT", "*", None))

    def oagg(f, c, e):
        if c == "*":
            return OAgg(AGG[f], -1, 0, -1)
        if e is None or e[0] == "COL":
            return OAgg(AGG[f], os_.index[c if e is None else e[1]], 0, -1)
        return OAgg(AGG[f], os_.index[e[1]], EXPR[e[0]], os_.index[e[2]])
    aggs = (OAgg * len(nat))(*[oagg(f, c, e) for f, c, e in nat])
    ng = len(qc.group_by)
    gcols = np.array([os_.group_col(g) for g in qc.group_by] or [0], dtype=np.int32)
    cap = 1
    if ng:  # groups <= min(docs, key space, numGroupsLimit)
        space = 1
        for c in gcols:
            space *= max(int(os_.cols[int(c)].cardinality), 1)
        cap = max(1, min(n, space, qc.num_groups_limit))
    keys = np.zeros(cap * max(ng, 1), dtype=np.int32)
    vals = np.zeros(cap * len(nat), dtype=np.float64)
    vali = np.zeros(cap * len(nat), dtype=np.int64)
    valh = np.zeros(cap * len(nat), dtype=np.int64)
    reached = C.c_int32(0)

    def run() -> int:
        for inv, card, idarr, bits in inv_steps:
            bits[:] = 0
            rc = L.oracle_inverted_to_bitset(_ptr(inv), card, _ptr(idarr), len(idarr), _ptr(bits), n)
            assert rc == 0, rc
        if qc.cnf:
            cnt = int(L.oracle_filter(os_.cols, n, leaves, nl, _ptr(fbits)))
            bptr = _ptr(fbits)
        else:
            cnt, bptr = n, None
        if ng:
            r = L.oracle_group_by(os_.cols, n, bptr, _ptr(gcols), ng, aggs, len(nat), qc.num_groups_limit, cap,
                                  _ptr(keys), _ptr(vals), _ptr(vali), _ptr(valh), C.byref(reached))
            assert r >= 0, r
        else:
            L.oracle_aggregate(os_.cols, n, bptr, aggs, len(nat), _ptr(vals), _ptr(vali), _ptr(valh))
        return cnt
    run.keep = (os_, leaves, inv_steps)
    return run


def _distinct_count(qc: QueryContext, segments, use_inverted: bool, stats):
    """DistinctCountAggregationFunction (aggregate / aggregateGroupBySV: add each matching doc's value
    to its group's set; merge = union; final = size), restated directly over the docs: the filter's
    matching docs, their group-by values and their DISTINCTCOUNT column values, with value identity
    as the fastutil sets have it (oracle_reduce.java_identity). The other aggregations come from the query
    without its DISTINCTCOUNTs, whose groups are the groups of the query."""
    base = dataclasses.replace(qc, aggregations=[a for a in qc.aggregations if a.func != "DISTINCTCOUNT"] or
                               [Aggregation("COUNT", "*")], order_by=[])
    total, bg = execute(base, segments, use_inverted, stats)
    dc = [i for i, a in enumerate(qc.aggregations) if a.func == "DISTINCTCOUNT"]
    sets = {i: {} for i in dc}
    for seg in segments:
        os_ = OracleSegment(seg)
        n = seg.num_docs
        if qc.cnf:
            bits, _ = os_.filter_bitset(qc, use_inverted)
            docs = np.flatnonzero(np.unpackbits(bits.view(np.uint8), bitorder="little")[:n])
        else:
            docs = np.arange(n)
        keys = [os_.values(g)[docs].tolist() for g in qc.group_by]
        for i in dc:
            vals = os_.values(qc.aggregations[i].column)[docs].tolist()
            s = sets[i]
            for d in range(len(docs)):
                k = identity_key(tuple(kc[d] for kc in keys))
                s.setdefault(k, set()).add(java_identity(vals[d]))
    rest = [j for j, a in enumerate(qc.aggregations) if a.func != "DISTINCTCOUNT"]
    out = {}
    for key, parts in bg.items():
        full = [None] * len(qc.aggregations)
        for j, p in zip(rest, parts):
            full[j] = p
        for i in dc:
            full[i] = frozenset(sets[i].get(identity_key(key), ()))
        out[key] = full
    return total, out


def _literal() -> bool:
    return bool(lib().oracle_literal_int_sum())


def _is_int_value(seg: SegmentBuffers, column, expr) -> bool:
    """agg_is_int in pinot_oracle.c: SUM over an INT/LONG column, or over times/minus/plus of two INT
    columns, is summed exactly."""
    if column == "*":
        return False
    if expr is None or expr[0] == "COL":
        c = column if expr is None else expr[1]
        return seg.columns[c].stored_type in (INT, LONG)
    return seg.columns[expr[1]].stored_type == INT and seg.columns[expr[2]].stored_type == INT


def _exact(lo, hi) -> int:
    return (int(hi) << 64) | (int(lo) & ((1 << 64) - 1))


def _parts(qc, slots, nat, vals, vali, valh, int_sum):
    def sum_of(i):
        return _exact(vali[i], valh[i]) if int_sum[i] else float(vals[i])
    out = []
    for a, s in zip(qc.aggregations, slots):
        if s[0] == "avg":
            out.append((sum_of(s[1]), int(vali[s[2]])))
        elif s[0] == "range":
            out.append((float(vals[s[1]]), float(vals[s[2]])))
        elif a.func in ("COUNT", "SUMLONG"):
            out.append(int(vali[s[1]]))
        elif a.func == "SUM":
            out.append(sum_of(s[1]))
        else:
            out.append(float(vals[s[1]]))
    return out


def rows(query, segments, use_inverted: bool = True):
    qc = parse_sql(query)
    _, groups = execute(qc, segments, use_inverted)
    return reduce_rows(qc, groups)
