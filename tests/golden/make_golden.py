"""Generate the committed golden fixtures from the reference's own test data.

Run in the build container (needs /root/reference, which is read as DATA only):

    python tests/golden/make_golden.py

Outputs (committed; the GPU box has no /root/reference):
  tests/golden/test_data_sv.npz
      The 11 columns that BaseSingleValueQueriesTest selects
      (pinot-core/src/test/java/org/apache/pinot/queries/BaseSingleValueQueriesTest.java:47-80)
      from pinot-core/src/test/resources/data/test_data-sv.avro (30000 records), with
      avro nulls replaced by Pinot's default null values for the field type.
  The expected query results live in tests/golden/sv_queries_expected.json; they are
  transcribed (not computed) from the reference tests cited there.

The avro object-container reader below is a minimal restatement of the Avro 1.x
binary encoding (null codec only), enough for this file.
"""
from __future__ import annotations

import io
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF_AVRO = "/root/reference/pinot-core/src/test/resources/data/test_data-sv.avro"

# (name, pinot type, field type) — BaseSingleValueQueriesTest.java:62-74
SV_SCHEMA = [
    ("column1", "INT", "METRIC"), ("column3", "INT", "METRIC"), ("column5", "STRING", "DIMENSION"),
    ("column6", "INT", "DIMENSION"), ("column7", "INT", "DIMENSION"), ("column9", "INT", "DIMENSION"),
    ("column11", "STRING", "DIMENSION"), ("column12", "STRING", "DIMENSION"), ("column17", "INT", "METRIC"),
    ("column18", "INT", "METRIC"), ("daysSinceEpoch", "INT", "DATE_TIME"),
]


def _read_long(f) -> int:
    shift = 0
    acc = 0
    while True:
        b = f.read(1)
        if not b:
            raise EOFError
        b = b[0]
        acc |= (b & 0x7F) << shift
        shift += 7
        if not b & 0x80:
            break
    return (acc >> 1) ^ -(acc & 1)


def _read_bytes(f) -> bytes:
    n = _read_long(f)
    return f.read(n)


def _decode(f, schema):
    if isinstance(schema, list):  # union
        return _decode(f, schema[_read_long(f)])
    if isinstance(schema, dict):
        t = schema["type"]
        if t == "record":
            return {fld["name"]: _decode(f, fld["type"]) for fld in schema["fields"]}
        if t == "array":
            out = []
            while True:
                n = _read_long(f)
                if n == 0:
                    return out
                if n < 0:
                    n = -n
                    _read_long(f)
                out.extend(_decode(f, schema["items"]) for _ in range(n))
        return _decode(f, t)
    if schema == "null":
        return None
    if schema in ("int", "long"):
        return _read_long(f)
    if schema == "string":
        return _read_bytes(f).decode("utf-8")
    if schema == "bytes":
        return _read_bytes(f)
    if schema == "float":
        return float(np.frombuffer(f.read(4), "<f4")[0])
    if schema == "double":
        return float(np.frombuffer(f.read(8), "<f8")[0])
    if schema == "boolean":
        return f.read(1) != b"\0"
    raise NotImplementedError(schema)


def snappy_decompress(src: bytes) -> bytes:
    """Raw Snappy block decompression (the format's published spec: a varint uncompressed length,
    then literal / copy-1 / copy-2 / copy-4 elements), for avro's "snappy" codec."""
    pos, n, shift = 0, 0, 0
    while True:
        b = src[pos]
        pos += 1
        n |= (b & 0x7F) << shift
        shift += 7
        if not b & 0x80:
            break
    out = bytearray()
    while pos < len(src):
        tag = src[pos]
        pos += 1
        kind = tag & 3
        if kind == 0:  # literal
            ln = tag >> 2
            if ln >= 60:
                nb = ln - 59
                ln = int.from_bytes(src[pos:pos + nb], "little")
                pos += nb
            ln += 1
            out += src[pos:pos + ln]
            pos += ln
            continue
        if kind == 1:
            ln = ((tag >> 2) & 7) + 4
            off = ((tag >> 5) << 8) | src[pos]
            pos += 1
        elif kind == 2:
            ln = (tag >> 2) + 1
            off = int.from_bytes(src[pos:pos + 2], "little")
            pos += 2
        else:
            ln = (tag >> 2) + 1
            off = int.from_bytes(src[pos:pos + 4], "little")
            pos += 4
        for _ in range(ln):  # byte-serial: copies may overlap their own output
            out.append(out[-off])
    assert len(out) == n, (len(out), n)
    return bytes(out)


def read_avro(path):
    with open(path, "rb") as fh:
        f = io.BytesIO(fh.read())
    assert f.read(4) == b"Obj\x01"
    meta = {}
    while True:
        n = _read_long(f)
        if n == 0:
            break
        if n < 0:
            n = -n
            _read_long(f)
        for _ in range(n):
            k = _read_bytes(f).decode()
            meta[k] = _read_bytes(f)
    codec = meta.get("avro.codec", b"null").decode()
    assert codec in ("null", "snappy"), codec
    schema = json.loads(meta["avro.schema"])
    sync = f.read(16)
    rows = []
    while True:
        try:
            count = _read_long(f)
        except EOFError:
            break
        size = _read_long(f)  # block byte size
        block = f.read(size)
        if codec == "snappy":  # snappy block followed by a 4-byte CRC32 of the uncompressed data
            block = snappy_decompress(block[:-4])
        bf = io.BytesIO(block)
        for _ in range(count):
            rows.append(_decode(bf, schema))
        assert f.read(16) == sync
    return schema, rows


def main():
    if not os.path.exists(REF_AVRO):
        sys.exit("reference avro not present (this script only runs in the build container)")
    _, rows = read_avro(REF_AVRO)
    out = {}
    nulls = {}
    for name, ptype, ftype in SV_SCHEMA:
        vals = [r[name] for r in rows]
        nulls[name] = sum(v is None for v in vals)
        if ptype == "INT":
            # FieldSpec defaults: metric INT null -> 0, dimension/time INT null -> Integer.MIN_VALUE
            dflt = 0 if ftype == "METRIC" else -(2 ** 31)
            out[name] = np.array([dflt if v is None else v for v in vals], dtype=np.int32)
        else:
            out[name] = np.array(["null" if v is None else v for v in vals], dtype=str)
    np.savez_compressed(os.path.join(HERE, "test_data_sv.npz"), **out)
    print("rows", len(rows), "nulls", nulls)


if __name__ == "__main__":
    main()
