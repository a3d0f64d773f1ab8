"""Immutable-segment column buffers in Pinot's on-disk byte formats (numpy, host side).

This module produces and parses the exact bytes a Pinot server mmaps as
``PinotDataBuffer``s for one immutable segment, so that the HBM stager and the
CPU oracle see the same buffers the reference's readers see:

* dictionary-encoded single-value forward index, bit packed MSB-first, big-endian
  (writer: ``FixedBitSVForwardIndexWriter`` / ``PinotDataBitSet.writeInt``,
  pinot-segment-local/.../io/util/PinotDataBitSet.java:143-170; reader:
  ``FixedBitSVForwardIndexReaderV2``, .../readers/forward/FixedBitSVForwardIndexReaderV2.java:33);
* sorted forward index: one big-endian ``(minDocId, maxDocId)`` int pair per dictId
  (.../creator/impl/fwd/SingleValueSortedForwardIndexCreator.java:53-70, read by
  ``SortedIndexReaderImpl``);
* raw fixed-byte chunk forward index, PASS_THROUGH chunks, header of 7 big-endian ints
  plus chunk offsets (.../io/writer/impl/BaseChunkForwardIndexWriter.java:131-165,
  read by ``FixedBytePower2ChunkSVForwardIndexReader`` / ``BaseChunkForwardIndexReader``
  .../readers/forward/BaseChunkForwardIndexReader.java:60-105);
* sorted dictionaries of big-endian fixed-width values, strings padded with NUL
  (``IntDictionary``/``LongDictionary``/``FloatDictionary``/``DoubleDictionary``/``StringDictionary``);
* bitmap inverted index: (cardinality+1) big-endian absolute offsets followed by
  RoaringBitmap portable serialisations
  (.../creator/impl/inv/BitmapInvertedIndexWriter.java:37-52, read by
  ``BitmapInvertedIndexReader`` .../readers/BitmapInvertedIndexReader.java:44-60).

RoaringBitmap (org.roaringbitmap:RoaringBitmap 1.6.14, pom.xml:214) is a third-party
dependency that is not vendored in the reference; its portable serialisation format
is restated here (cookie 12346 = no run containers, 12347 = with run containers).

Nothing here runs on the GPU; this is segment *creation* (test and bench input)
plus format parsing shared by the stager.
"""
from __future__ import annotations

import dataclasses
import struct
from typing import Dict, List, Optional, Sequence

import numpy as np

# FieldSpec.DataType stored types handled on the hot path
INT, LONG, FLOAT, DOUBLE, STRING = "INT", "LONG", "FLOAT", "DOUBLE", "STRING"
_NP_BE = {INT: ">i4", LONG: ">i8", FLOAT: ">f4", DOUBLE: ">f8"}
_NP_LE = {INT: "<i4", LONG: "<i8", FLOAT: "<f4", DOUBLE: "<f8"}
VALUE_SIZE = {INT: 4, LONG: 8, FLOAT: 4, DOUBLE: 8}

# ChunkCompressionType (pinot-segment-spi/.../compression/ChunkCompressionType.java:22)
PASS_THROUGH = 0
SNAPPY = 1
ZSTANDARD = 2
LZ4 = 3
LZ4_LENGTH_PREFIXED = 4
GZIP = 5
DELTA = 6
DELTADELTA = 7

# Default null values (FieldSpec.DEFAULT_*_NULL_VALUE_OF_*), used when ingesting nulls
DEFAULT_DIMENSION_NULL = {INT: np.iinfo(np.int32).min, LONG: np.iinfo(np.int64).min,
                          FLOAT: float("-inf"), DOUBLE: float("-inf"), STRING: "null"}
DEFAULT_METRIC_NULL = {INT: 0, LONG: 0, FLOAT: 0.0, DOUBLE: 0.0, STRING: "null"}


def num_bits_per_value(max_value: int) -> int:
    """PinotDataBitSet.getNumBitsPerValue (PinotDataBitSet.java:61-72): at least one bit."""
    if max_value <= 1:
        return 1
    return int(max_value).bit_length()


# --------------------------------------------------------------------------- fixed-bit
def pack_fixed_bit(values: np.ndarray, bits: int) -> bytes:
    """Bit-pack non-negative ints MSB-first into a big-endian bit stream.

    Same bytes as ``FixedBitSVForwardIndexWriter`` (value i occupies stream bits
    [i*bits, (i+1)*bits), bit 0 = MSB of byte 0; PinotDataBitSet.java:143-170).
    The buffer is sized ceil(n*bits/8) bytes like the writer's file.
    """
    v = np.ascontiguousarray(values, dtype=np.uint64)
    if v.size and (int(v.max()) >> bits) != 0:
        raise ValueError(f"value does not fit in {bits} bits")
    n = v.size
    out = np.zeros((n * bits + 7) // 8, dtype=np.uint8)
    step = 1 << 20
    for s in range(0, n, step):  # bounded temporaries
        e = min(n, s + step)
        shifts = np.arange(bits - 1, -1, -1, dtype=np.uint64)
        bitmat = ((v[s:e, None] >> shifts) & np.uint64(1)).astype(np.uint8).ravel()
        first_bit = s * bits
        # s is a multiple of 2^20, so first_bit is a multiple of 8
        packed = np.packbits(bitmat)
        out[first_bit // 8: first_bit // 8 + packed.size] |= packed
    return out.tobytes()


def unpack_fixed_bit(buf: bytes, bits: int, n: int) -> np.ndarray:
    """Vectorised inverse of :func:`pack_fixed_bit` (host helper, not the oracle)."""
    a = np.frombuffer(buf, dtype=np.uint8)
    allbits = np.unpackbits(a)[: n * bits].reshape(n, bits).astype(np.int64)
    w = (1 << np.arange(bits - 1, -1, -1, dtype=np.int64))
    return (allbits * w).sum(axis=1).astype(np.int32)


# --------------------------------------------------------------------------- sorted fwd
def sorted_fwd_bytes(dict_ids: np.ndarray, cardinality: int) -> bytes:
    """SingleValueSortedForwardIndexCreator: (minDocId, maxDocId) per dictId, big-endian ints."""
    d = np.asarray(dict_ids, dtype=np.int64)
    if d.size > 1 and np.any(np.diff(d) < 0):
        raise ValueError("column is not sorted")
    pairs = np.empty((cardinality, 2), dtype=">i4")
    pairs[:, 0] = np.iinfo(np.int32).max
    pairs[:, 1] = np.iinfo(np.int32).min
    if d.size:
        ids, first = np.unique(d, return_index=True)
        last = np.r_[first[1:], d.size] - 1
        pairs[ids, 0] = first
        pairs[ids, 1] = last
    return pairs.tobytes()


# --------------------------------------------------------------------------- raw fwd
RAW_HEADER_INTS = 7


def lz4_block_compress(data: bytes) -> bytes:
    """LZ4 block format (what lz4-java's fastCompressor emits): sequences of
    token(lit_len:4 | match_len-4:4) [lit_len ext] literals [offset u16 LE] [match_len ext];
    the last sequence is literals only and the last 5 bytes are always literals."""
    n = len(data)
    out = bytearray()
    table = {}
    anchor = 0
    i = 0
    limit = n - 12  # matches must end >= 5 bytes before the end (LZ4 end-of-block rules)

    def put_len(x):
        while x >= 255:
            out.append(255)
            x -= 255
        out.append(x)

    while i < limit:
        key = data[i:i + 4]
        cand = table.get(key)
        table[key] = i
        if cand is not None and i - cand <= 0xFFFF:
            m = 4
            while i + m < n - 5 and data[cand + m] == data[i + m]:
                m += 1
            lit = i - anchor
            tok_l = min(lit, 15)
            tok_m = min(m - 4, 15)
            out.append((tok_l << 4) | tok_m)
            if lit >= 15:
                put_len(lit - 15)
            out += data[anchor:i]
            out += struct.pack("<H", i - cand)
            if m - 4 >= 15:
                put_len(m - 4 - 15)
            i += m
            anchor = i
        else:
            i += 1
    lit = n - anchor
    out.append(min(lit, 15) << 4)
    if lit >= 15:
        put_len(lit - 15)
    out += data[anchor:]
    return bytes(out)


def raw_fwd_bytes(values: np.ndarray, stored_type: str, version: int = 4, docs_per_chunk: int = 1000,
                  compression: int = PASS_THROUGH) -> bytes:
    """FixedByteChunkForwardIndexWriter with PASS_THROUGH chunks.

    Header (BaseChunkForwardIndexWriter.java:131-165): version, numChunks,
    numDocsPerChunk, sizeOfEntry, totalDocs, compressionType, dataHeaderStart, then
    one chunk offset per chunk (int for v2, long for v3+), then the chunks. v4 rounds
    docsPerChunk up to a power of two (FixedByteChunkForwardIndexWriter.java:90-96).
    Values are big-endian (java.nio.ByteBuffer default order).
    """
    data = np.ascontiguousarray(values).astype(_NP_BE[stored_type]).tobytes()
    if compression == PASS_THROUGH:
        return raw_fwd_header(int(values.size), stored_type, version, docs_per_chunk) + data
    if compression not in (SNAPPY, ZSTANDARD, LZ4, LZ4_LENGTH_PREFIXED, GZIP, DELTA, DELTADELTA):
        raise NotImplementedError(f"compression {compression}")
    if compression in (DELTA, DELTADELTA) and stored_type not in (INT, LONG):
        raise ValueError("DELTA / DELTADELTA chunks hold INT or LONG values")
    # compressed chunks (BaseChunkForwardIndexWriter.writeChunk): offsets point at each compressed chunk
    if version >= 4 and docs_per_chunk & (docs_per_chunk - 1):
        docs_per_chunk = 1 << (docs_per_chunk - 1).bit_length()
    n = int(values.size)
    size = VALUE_SIZE[stored_type]
    chunk_bytes = docs_per_chunk * size
    chunks = []
    for c in range(0, len(data), chunk_bytes):
        raw = data[c:c + chunk_bytes]
        chunks.append(chunk_compress(raw, compression))
    num_chunks = len(chunks)
    off_size = 4 if version == 2 else 8
    header_size = RAW_HEADER_INTS * 4 + num_chunks * off_size
    hdr = struct.pack(">7i", version, num_chunks, docs_per_chunk, size, n, compression, RAW_HEADER_INTS * 4)
    offs, pos = [], header_size
    for blk in chunks:
        offs.append(pos)
        pos += len(blk)
    hdr += struct.pack(">%d%s" % (num_chunks, "i" if off_size == 4 else "q"), *offs)
    return hdr + b"".join(chunks)


def _delta_chunk(raw: bytes, dd: bool) -> bytes:
    """DeltaCompressor / DeltaDeltaCompressor.compress (io/compression/DeltaCompressor.java:45-150):
    LONG layout when the chunk is a multiple of 8 bytes (even for INT columns), else INT; flag byte,
    BE count, BE first value, BE LZ4-block size, LZ4 block of BE deltas (DELTADELTA: first delta, then
    deltas of deltas), all with Java's wrapping arithmetic."""
    w = 8 if len(raw) % 8 == 0 else 4
    v = np.frombuffer(raw, dtype=">u8" if w == 8 else ">u4").astype(np.uint64 if w == 8 else np.uint32)
    out = struct.pack(">bi", 1 if w == 8 else 0, v.size)
    if v.size == 0:
        return out
    out += raw[:w]
    if v.size == 1:
        return out
    d = np.diff(v)  # unsigned wrap-around == Java's overflowing subtraction
    if dd:
        d = np.r_[d[:1], np.diff(d)]
    blk = lz4_block_compress(d.astype(">u8" if w == 8 else ">u4").tobytes())
    return out + struct.pack(">i", len(blk)) + blk


def chunk_compress(raw: bytes, compression: int) -> bytes:
    """One chunk through ChunkCompressorFactory's compressor for `compression`
    (pinot-segment-local/.../io/compression/*Compressor.java). SNAPPY / ZSTANDARD come from pyarrow's
    bundled codecs (raw snappy block; zstd frame with content size), standing in for snappy-java /
    zstd-jni on the write side only: the readers under test decode them independently."""
    if compression in (LZ4, LZ4_LENGTH_PREFIXED):
        blk = lz4_block_compress(raw)
        if compression == LZ4_LENGTH_PREFIXED:  # LZ4CompressorWithLength: decompressed length, LE int
            blk = struct.pack("<i", len(raw)) + blk
        return blk
    if compression in (SNAPPY, ZSTANDARD):
        import pyarrow as pa
        return pa.Codec("snappy" if compression == SNAPPY else "zstd").compress(raw, asbytes=True)
    if compression == GZIP:  # java.util.zip.Deflater (zlib stream) + BE uncompressed size
        import zlib
        return zlib.compress(raw) + struct.pack(">i", len(raw))
    if compression in (DELTA, DELTADELTA):
        return _delta_chunk(raw, compression == DELTADELTA)
    raise NotImplementedError(f"compression {compression}")


def var_byte_fwd_bytes(values, version: int = 4, compression: int = PASS_THROUGH, chunk_size: int = 4096) -> bytes:
    """Raw STRING forward index as VarByteChunkForwardIndexWriterV4 / V5 / V6 write it
    (io/writer/impl/VarByteChunkForwardIndexWriterV4.java): BE header {version, target chunk size,
    compression, chunks offset}; LE metadata {docIdOffset (MSB: huge chunk), chunk offset} per chunk;
    LE chunks {numDocs, offsets (V6 with compression: sizes), UTF-8 bytes}; a value that does not fit
    a chunk is written alone as a huge chunk. LZ4 is upgraded to LZ4_LENGTH_PREFIXED like the writer."""
    comp = LZ4_LENGTH_PREFIXED if compression == LZ4 else compression
    meta, data = [], bytearray()
    cur: list = []
    state = {"pos": 4, "doc_off": 0, "next": 0}

    def write(buf: bytes, huge: bool):
        c = chunk_compress(buf, comp) if comp != PASS_THROUGH else buf
        meta.append((state["doc_off"] | (0x80000000 if huge else 0), len(data)))
        data.extend(c)
        state["doc_off"] = state["next"]

    def flush():
        if not cur:
            return
        nd = len(cur)
        offs = [4 * (nd + 1)]
        for v in cur[:-1]:
            offs.append(offs[-1] + len(v))
        ints = [len(v) for v in cur] if (version == 6 and comp != PASS_THROUGH) else offs
        write(struct.pack("<%di" % (nd + 1), nd, *ints) + b"".join(cur), False)
        cur.clear()
        state["pos"] = 4

    for s in values:
        b = s.encode("utf-8")
        need = 4 + len(b)
        if state["pos"] > chunk_size - need:
            flush()
            if need > chunk_size - 4:
                state["next"] += 1
                write(b, True)
                continue
        cur.append(b)
        state["pos"] += need
        state["next"] += 1
    flush()
    hdr = struct.pack(">4i", version, chunk_size, comp, 16 + 8 * len(meta))
    return hdr + b"".join(struct.pack("<Ii", d, o) for d, o in meta) + bytes(data)


def raw_fwd_header(n: int, stored_type: str, version: int = 4, docs_per_chunk: int = 1000) -> bytes:
    """Header + chunk-offset table of a PASS_THROUGH FixedByteChunkForwardIndexWriter file of n values."""
    if version >= 4 and docs_per_chunk & (docs_per_chunk - 1):
        docs_per_chunk = 1 << (docs_per_chunk - 1).bit_length()
    size = VALUE_SIZE[stored_type]
    num_chunks = (n + docs_per_chunk - 1) // docs_per_chunk
    off_size = 4 if version == 2 else 8
    header_size = RAW_HEADER_INTS * 4 + num_chunks * off_size
    hdr = struct.pack(">7i", version, num_chunks, docs_per_chunk, size, n, PASS_THROUGH, RAW_HEADER_INTS * 4)
    chunk_bytes = docs_per_chunk * size
    offs = np.arange(num_chunks, dtype=np.int64) * chunk_bytes + header_size
    # the last chunk is written with only its present bytes (writeChunk flips the buffer)
    return hdr + offs.astype(">i4" if off_size == 4 else ">i8").tobytes()


@dataclasses.dataclass
class RawFwdHeader:
    version: int
    num_chunks: int
    docs_per_chunk: int
    size_of_entry: int
    total_docs: int
    compression: int
    data_header_start: int
    raw_data_start: int


def parse_raw_fwd_header(buf: bytes) -> RawFwdHeader:
    """BaseChunkForwardIndexReader constructor (BaseChunkForwardIndexReader.java:60-105)."""
    version, num_chunks, dpc, size = struct.unpack_from(">4i", buf, 0)
    if version > 1:
        total, comp, dhs = struct.unpack_from(">3i", buf, 16)
    else:
        total, comp, dhs = -1, 1, 16
    off_size = 4 if version <= 2 else 8
    return RawFwdHeader(version, num_chunks, dpc, size, total, comp, dhs, dhs + num_chunks * off_size)


# --------------------------------------------------------------------------- dictionary
def dictionary_bytes(sorted_values, stored_type: str) -> bytes:
    """Fixed-width big-endian dictionary buffer (strings padded with NUL to the longest UTF-8 entry)."""
    if stored_type == STRING:
        enc = [s.encode("utf-8") for s in sorted_values]
        width = max([len(e) for e in enc] + [1])
        return b"".join(e.ljust(width, b"\0") for e in enc)
    return np.asarray(sorted_values).astype(_NP_BE[stored_type]).tobytes()


def decode_dictionary(buf: bytes, stored_type: str, cardinality: int) -> np.ndarray:
    if stored_type == STRING:
        width = len(buf) // max(cardinality, 1)
        # FixedByteValueReaderWriter.readUnpaddedBytes: a value ends at its first NUL byte
        return np.array([buf[i * width:(i + 1) * width].split(b"\0", 1)[0].decode("utf-8") for i in range(cardinality)],
                        dtype=object)
    return np.frombuffer(buf, dtype=_NP_BE[stored_type], count=cardinality).astype(_NP_LE[stored_type])


def _java_string_key(s: str):
    # String.compareTo compares UTF-16 code units
    return s.encode("utf-16-be")


def build_dictionary(values: np.ndarray, stored_type: str):
    """Sorted dictionary + dictIds (SegmentDictionaryCreator sorts the unique values)."""
    if stored_type == STRING:
        uniq = sorted(set(values.tolist()), key=_java_string_key)
        index = {v: i for i, v in enumerate(uniq)}
        ids = np.fromiter((index[v] for v in values.tolist()), dtype=np.int32, count=len(values))
        return np.array(uniq, dtype=object), ids
    uniq, ids = np.unique(np.asarray(values), return_inverse=True)
    return uniq.astype(_NP_LE[stored_type]), ids.astype(np.int32)


# --------------------------------------------------------------------------- roaring
ROARING_COOKIE_NO_RUN = 12346
ROARING_COOKIE = 12347
ROARING_NO_OFFSET_THRESHOLD = 4
ARRAY_MAX = 4096


def roaring_serialize(doc_ids: np.ndarray, run_optimize: bool = True) -> bytes:
    """RoaringBitmap.serialize (portable format) of a sorted unique set of docIds.

    Containers: array (cardinality <= 4096, sorted u16), bitmap (1024 u64 words) or,
    when ``run_optimize`` and smaller, run ((start, length-1) u16 pairs), as
    RoaringBitmap.runOptimize would choose. All little-endian.
    """
    d = np.asarray(doc_ids, dtype=np.int64)
    keys = np.unique(d >> 16) if d.size else np.zeros(0, np.int64)
    conts = []
    for k in keys.tolist():
        low = (d[(d >> 16) == k] & 0xFFFF).astype(np.int64)
        card = low.size
        starts = np.r_[True, np.diff(low) != 1]
        run_starts = low[starts]
        run_ends = np.r_[low[np.nonzero(starts)[0][1:] - 1], low[-1]]
        nruns = run_starts.size
        run_size = 2 + 4 * nruns
        std_size = 2 * card if card <= ARRAY_MAX else 8192
        if run_optimize and run_size < std_size:
            body = struct.pack("<H", nruns) + np.stack([run_starts, run_ends - run_starts], 1).astype("<u2").tobytes()
            conts.append((k, card, "run", body))
        elif card <= ARRAY_MAX:
            conts.append((k, card, "array", low.astype("<u2").tobytes()))
        else:
            words = np.zeros(1024, dtype=np.uint64)
            np.bitwise_or.at(words, low >> 6, np.uint64(1) << (low & 63).astype(np.uint64))
            conts.append((k, card, "bitmap", words.astype("<u8").tobytes()))
    size = len(conts)
    has_run = any(c[2] == "run" for c in conts)
    out = bytearray()
    if has_run:
        out += struct.pack("<i", ROARING_COOKIE | ((size - 1) << 16))
        runbits = bytearray((size + 7) // 8)
        for i, c in enumerate(conts):
            if c[2] == "run":
                runbits[i // 8] |= 1 << (i % 8)
        out += runbits
    else:
        out += struct.pack("<ii", ROARING_COOKIE_NO_RUN, size)
    for k, card, _, _ in conts:
        out += struct.pack("<HH", k, card - 1)
    if (not has_run) or size >= ROARING_NO_OFFSET_THRESHOLD:
        pos = len(out) + 4 * size
        for _, _, _, body in conts:
            out += struct.pack("<i", pos)
            pos += len(body)
    for _, _, _, body in conts:
        out += body
    return bytes(out)


def _put_le(out: np.ndarray, pos: np.ndarray, val: np.ndarray, nbytes: int) -> None:
    v = np.asarray(val, dtype=np.uint64)
    for b in range(nbytes):
        out[pos + b] = ((v >> np.uint64(8 * b)) & np.uint64(0xFF)).astype(np.uint8)


def inverted_index_bytes_fast(dict_ids: np.ndarray, cardinality: int) -> Optional[bytes]:
    """Vectorised ``inverted_index_bytes`` for the common case where every container of every
    bitmap is an array container that runOptimize would keep (no bitmap or run containers): the
    same bytes, built with numpy instead of one Python loop per container. Returns None when some
    container needs another kind (the caller then uses the general builder)."""
    d = np.asarray(dict_ids, dtype=np.int64)
    n = d.size
    card = int(cardinality)
    hdr = 4 * (card + 1)
    order = np.argsort(d, kind="stable")          # docIds ascending within each dictId
    sd = d[order]
    key = order >> 16
    newc = np.ones(n, dtype=bool)
    if n > 1:
        newc[1:] = (sd[1:] != sd[:-1]) | (key[1:] != key[:-1])
    cstart = np.nonzero(newc)[0]
    ccard = np.diff(np.r_[cstart, n])
    if n and int(ccard.max()) > ARRAY_MAX:
        return None
    brk = np.ones(n, dtype=bool)
    if n > 1:
        brk[1:] = newc[1:] | (order[1:] != order[:-1] + 1)
    nruns = np.add.reduceat(brk.astype(np.int64), cstart) if n else np.zeros(0, np.int64)
    if n and bool(((2 + 4 * nruns) < 2 * ccard).any()):   # runOptimize would pick a run container
        return None
    cdict = sd[cstart]
    ckey = key[cstart]
    nc_d = np.bincount(cdict, minlength=card).astype(np.int64)
    nd_d = np.bincount(d, minlength=card).astype(np.int64)
    size_d = 8 + 8 * nc_d + 2 * nd_d
    bstart = hdr + np.r_[0, np.cumsum(size_d)[:-1]].astype(np.int64)
    total = hdr + int(size_d.sum())
    out = np.zeros(total, dtype=np.uint8)
    out[:hdr] = np.r_[bstart, total].astype(">u4").view(np.uint8)
    _put_le(out, bstart, np.full(card, ROARING_COOKIE_NO_RUN), 4)
    _put_le(out, bstart + 4, nc_d, 4)
    cfirst = np.r_[0, np.cumsum(nc_d)[:-1]]
    dfirst = np.r_[0, np.cumsum(nd_d)[:-1]]
    cj = np.arange(cstart.size) - cfirst[cdict]
    cb = bstart[cdict]
    _put_le(out, cb + 8 + 4 * cj, ckey, 2)
    _put_le(out, cb + 10 + 4 * cj, ccard - 1, 2)
    _put_le(out, cb + 8 + 4 * nc_d[cdict] + 4 * cj, 8 + 8 * nc_d[cdict] + 2 * (cstart - dfirst[cdict]), 4)
    _put_le(out, bstart[sd] + 8 + 8 * nc_d[sd] + 2 * (np.arange(n) - dfirst[sd]), order & 0xFFFF, 2)
    return out.tobytes()


def inverted_index_bytes(dict_ids: np.ndarray, cardinality: int) -> bytes:
    """BitmapInvertedIndexWriter layout: (cardinality+1) BE absolute offsets, then bitmaps."""
    if cardinality == 0:  # an empty column: the header's one offset (the end) and no bitmaps
        return (4).to_bytes(4, "big")
    fast = inverted_index_bytes_fast(dict_ids, cardinality)
    if fast is not None:
        return fast
    return inverted_index_bytes_general(dict_ids, cardinality)


def inverted_index_bytes_general(dict_ids: np.ndarray, cardinality: int) -> bytes:
    """BitmapInvertedIndexWriter layout, any container kinds (one roaring_serialize per bitmap)."""
    d = np.asarray(dict_ids, dtype=np.int64)
    order = np.argsort(d, kind="stable")
    sd = d[order]
    bounds = np.searchsorted(sd, np.arange(cardinality + 1))
    bitmaps = [roaring_serialize(np.sort(order[bounds[i]:bounds[i + 1]])) for i in range(cardinality)]
    pos = (cardinality + 1) * 4
    offs = [pos]
    for b in bitmaps:
        pos += len(b)
        offs.append(pos)
    return struct.pack(">%dI" % (cardinality + 1), *offs) + b"".join(bitmaps)


# --------------------------------------------------------------------------- segment
@dataclasses.dataclass
class ColumnBuffers:
    """One column of an immutable segment: metadata + the PinotDataBuffers the server maps."""
    name: str
    stored_type: str
    num_docs: int
    has_dictionary: bool
    is_sorted: bool = False
    cardinality: int = 0
    bits_per_element: int = 0
    fwd: bytes = b""                     # forward index buffer (fixed-bit | sorted pairs | raw chunk file)
    dictionary: bytes = b""              # dictionary buffer (dict-encoded columns)
    inverted: Optional[bytes] = None     # bitmap inverted index buffer
    dict_values: Optional[np.ndarray] = None  # decoded dictionary (host convenience)

    @property
    def encoding(self) -> str:
        if not self.has_dictionary:
            return "RAW"
        return "SORTED" if self.is_sorted else "FIXED_BIT"


@dataclasses.dataclass
class SegmentBuffers:
    name: str
    num_docs: int
    columns: Dict[str, ColumnBuffers]

    def column(self, name: str) -> ColumnBuffers:
        return self.columns[name]


def build_column(name: str, values, stored_type: str, dictionary: bool = True, inverted: bool = False,
                 detect_sorted: bool = True, raw_version: int = 4, compression: int = PASS_THROUGH) -> ColumnBuffers:
    """Create one column's buffers the way SegmentColumnarIndexCreator would for an SV column."""
    vals = np.asarray(values, dtype=object if stored_type == STRING else _NP_LE[stored_type])
    n = int(vals.size)
    if not dictionary:
        if stored_type == STRING:
            return ColumnBuffers(name, stored_type, n, False,
                                 fwd=var_byte_fwd_bytes([str(v) for v in vals], max(raw_version, 4), compression))
        return ColumnBuffers(name, stored_type, n, False,
                             fwd=raw_fwd_bytes(vals, stored_type, raw_version, compression=compression))
    dvals, ids = build_dictionary(vals, stored_type)
    card = len(dvals)
    is_sorted = bool(detect_sorted and (n < 2 or np.all(np.diff(ids.astype(np.int64)) >= 0)))
    bits = num_bits_per_value(card - 1)
    fwd = sorted_fwd_bytes(ids, card) if is_sorted else pack_fixed_bit(ids, bits)
    inv = inverted_index_bytes(ids, card) if inverted else None
    return ColumnBuffers(name, stored_type, n, True, is_sorted, card, bits, fwd, dictionary_bytes(dvals, stored_type),
                         inv, dvals)


def build_segment(name: str, columns: Dict[str, tuple]) -> SegmentBuffers:
    """columns: name -> (values, stored_type, kwargs-dict)."""
    cols = {}
    n = None
    for cname, spec in columns.items():
        values, stype = spec[0], spec[1]
        kw = spec[2] if len(spec) > 2 else {}
        c = build_column(cname, values, stype, **kw)
        if n is None:
            n = c.num_docs
        elif c.num_docs != n:
            raise ValueError("ragged columns")
        cols[cname] = c
    return SegmentBuffers(name, n or 0, cols)


# --------------------------------------------------------------------------- segment directories
V3_MAGIC_MARKER = 0xDEADBEEFDEAFBEAD  # SingleFileIndexDirectory.java:79, written before every index


def read_properties(path: str) -> Dict[str, str]:
    """metadata.properties / index_map (java.util.Properties key = value lines; \\uXXXX escapes)."""
    out = {}
    with open(path, encoding="latin-1") as f:
        for line in f:
            line = line.strip()
            if not line or line[0] in "#!" or "=" not in line:
                continue
            k, v = line.split("=", 1)
            out[k.strip()] = v.strip().encode("latin-1").decode("unicode_escape")
    return out


_V1_FWD_SUFFIX = {"sorted": ".sv.sorted.fwd", "unsorted": ".sv.unsorted.fwd", "raw": ".sv.raw.fwd"}
_TYPE_NAMES = {"INT": INT, "LONG": LONG, "FLOAT": FLOAT, "DOUBLE": DOUBLE, "STRING": STRING}


def load_segment_dir(path: str) -> SegmentBuffers:
    """Read an immutable segment directory the way ImmutableSegmentLoader / SegmentDirectory map it
    (pinot-segment-local/.../segment/store/SegmentLocalFSDirectory.java): metadata.properties for the
    column metadata; index buffers from V1 per-index files (FilePerIndexDirectory: <col>.dict,
    <col>.sv.{sorted,unsorted,raw}.fwd, <col>.bitmap.inv) or from V3's single columns.psf sliced by
    index_map (SingleFileIndexDirectory: <col>.<index>.startOffset / .size, each index prefixed by an
    8-byte magic marker). Single-value INT / LONG / FLOAT / DOUBLE / STRING columns; a raw column's
    legacy raw-value inverted index is dropped (SegmentPreProcessor.removeLegacyRawValueInvertedIndexes)."""
    import os
    v3 = os.path.join(path, "v3")
    if os.path.isdir(v3):
        path = v3
    meta = read_properties(os.path.join(path, "metadata.properties"))
    num_docs = int(meta["segment.total.docs"])
    cols = sorted({k.split(".")[1] for k in meta if k.startswith("column.") and k.count(".") >= 2})
    psf = None
    index_map = {}
    if os.path.exists(os.path.join(path, "index_map")):
        index_map = read_properties(os.path.join(path, "index_map"))
        with open(os.path.join(path, "columns.psf"), "rb") as f:
            psf = f.read()

    def index_bytes(col: str, index: str, v1_suffix: str) -> Optional[bytes]:
        if psf is not None:
            k = f"{col}.{index}.startOffset"
            if k not in index_map:
                return None
            off, size = int(index_map[k]), int(index_map[f"{col}.{index}.size"])
            marker = int.from_bytes(psf[off:off + 8], "big")
            if marker != V3_MAGIC_MARKER:
                raise ValueError(f"{col}.{index}: bad magic marker {marker:#x}")
            return psf[off + 8:off + size]
        fn = os.path.join(path, col + v1_suffix)
        if not os.path.exists(fn):
            return None
        with open(fn, "rb") as f:
            return f.read()

    out = {}
    for c in cols:
        m = {k[len("column.") + len(c) + 1:]: v for k, v in meta.items() if k.startswith(f"column.{c}.")}
        if m.get("isSingleValues", "true") != "true":
            raise NotImplementedError(f"multi-value column {c}")
        st = _TYPE_NAMES[m["dataType"]]
        has_dict = m.get("hasDictionary", "true") == "true"
        is_sorted = m.get("isSorted", "false") == "true"
        card = int(m.get("cardinality", "0"))
        bits = int(m.get("bitsPerElement", "0"))
        if not has_dict:
            fwd = index_bytes(c, "forward_index", _V1_FWD_SUFFIX["raw"])
            out[c] = ColumnBuffers(c, st, num_docs, False, fwd=fwd)
            continue
        fwd = index_bytes(c, "forward_index", _V1_FWD_SUFFIX["sorted" if is_sorted else "unsorted"])
        dic = index_bytes(c, "dictionary", ".dict")
        inv = index_bytes(c, "inverted_index", ".bitmap.inv")
        out[c] = ColumnBuffers(c, st, num_docs, True, is_sorted, card, bits, fwd, dic, inv,
                               decode_dictionary(dic, st, card))
    return SegmentBuffers(meta.get("segment.name", os.path.basename(path)), num_docs, out)
