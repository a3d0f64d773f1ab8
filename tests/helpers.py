"""Shared test helpers: golden segment construction and random segment generators."""
import json
import os

import numpy as np

from pinot_amd.segment import build_segment, DOUBLE, FLOAT, INT, LONG, STRING

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")

# BaseSingleValueQueriesTest.java:62-80: schema + inverted index columns
SV_COLUMNS = [("column1", INT), ("column3", INT), ("column5", STRING), ("column6", INT), ("column7", INT),
              ("column9", INT), ("column11", STRING), ("column12", STRING), ("column17", INT), ("column18", INT),
              ("daysSinceEpoch", INT)]
SV_INVERTED = {"column6", "column7", "column11", "column17", "column18"}
SV_FILTER = (" WHERE column1 > 100000000 AND column3 BETWEEN 20000000 AND 1000000000 AND column5 = 'gFuH'"
             " AND (column6 < 500000000 OR column11 NOT IN ('t', 'P')) AND daysSinceEpoch = 126164076")


# Partitioned-plan self-check failures the suite injects on purpose (test_gpu_selfcheck.py adds to it; the
# conftest's session check compares the library's process-wide count with it)
EXPECTED_SELFCHECK_FAILURES = [0]


def load_expected():
    with open(os.path.join(GOLDEN, "sv_queries_expected.json")) as f:
        return json.load(f)


def sv_segment(name="testTable_126164076_167572854"):
    data = np.load(os.path.join(GOLDEN, "test_data_sv.npz"), allow_pickle=False)
    cols = {}
    for c, t in SV_COLUMNS:
        v = data[c]
        if t == STRING:
            v = v.astype(object)
        cols[c] = (v, t, {"inverted": c in SV_INVERTED})
    return build_segment(name, cols)


def random_segment(rng, n, name="seg", bits_cards=(1000, 37), raw_types=(INT, LONG, DOUBLE), inverted=(),
                   sorted_col=False, float_col=False):
    cols = {}
    for i, card in enumerate(bits_cards):
        vals = rng.integers(0, card, n) * 7 + 3  # dictionary values != dictIds
        cols[f"d{i}"] = (vals.astype(np.int32), INT, {"inverted": f"d{i}" in inverted})
    for t in raw_types:
        if t == INT:
            v = rng.integers(-1000000, 1000000, n).astype(np.int32)
        elif t == LONG:
            v = rng.integers(-(1 << 40), 1 << 40, n).astype(np.int64)
        elif t == FLOAT:
            v = rng.normal(0, 100, n).astype(np.float32)
        else:
            v = rng.normal(0, 1000, n)
        cols[f"r_{t.lower()}"] = (v, t, {"dictionary": False})
    if sorted_col:
        cols["ts"] = (np.sort(rng.integers(0, 50, n)).astype(np.int32), INT, {})
    if float_col:
        cols["fd"] = ((rng.integers(0, 20, n) * 0.25).astype(np.float64), DOUBLE, {})
    return build_segment(name, cols)


def load_ssb_expected():
    with open(os.path.join(GOLDEN, "ssb_expected.json")) as f:
        return json.load(f)


def ssb_flat_segment(name="lineorder_flat_0", split=None):
    """The reference's SSB quickstart lineorder joined with its dimensions (tests/golden/ssb_flat.npz),
    as Pinot would build it: every column dictionary-encoded except the raw INT metrics
    (pinot_amd.ssb.FLAT_COLUMNS). split=k: k segments of consecutive rows instead of one."""
    from pinot_amd.ssb import FLAT_COLUMNS
    data = np.load(os.path.join(GOLDEN, "ssb_flat.npz"), allow_pickle=False)
    n = len(data["LO_ORDERDATE"])
    bounds = [0, n] if not split else [n * i // split for i in range(split + 1)]
    segs = []
    for i in range(len(bounds) - 1):
        cols = {}
        for c, t, dict_enc in FLAT_COLUMNS:
            v = data[c][bounds[i]:bounds[i + 1]]
            if t == STRING:
                v = v.astype(object)
            cols[c] = (v, t, {"dictionary": dict_enc, "detect_sorted": False})
        segs.append(build_segment(f"{name}_{i}", cols))
    return segs


def legacy_inverted_segment(fmt="v1"):
    """legacyRawInverted with its Pinot-written bitmaps in play: the legacy raw-value inverted index file
    (RawValueBitmapInvertedIndexCreator) embeds a standard BitmapInvertedIndexWriter section after a
    44-byte header (LegacyRawValueInvertedIndexCleanup.java:104-114: version 1, cardinality, max length,
    then dict offset/length and inverted-index offset/length as big-endian longs at bytes 12/20/28/36)
    whose bitmaps are keyed by the embedded dictionary's order, the sorted distinct values. The
    category column is rebuilt dictionary-encoded (the decoded strings, sorted dictionary) and gets that
    embedded section as its inverted index, so EQ/IN predicates expand Pinot-written RoaringBitmaps.
    The V1 file holds the inverted index; the V3 fixture shares its bytes (same segment)."""
    import struct
    import oracle
    from pinot_amd import segment as S
    d = os.path.join(GOLDEN, "pinot_written", f"legacyRawInverted_{fmt}")
    seg = S.load_segment_dir(d)
    raw = open(os.path.join(GOLDEN, "pinot_written", "legacyRawInverted_v1", "category.bitmap.inv"), "rb").read()
    version, card, _ = struct.unpack(">iii", raw[:12])
    _, _, inv_off, inv_len = struct.unpack(">qqqq", raw[12:44])
    assert version == 1 and inv_off + inv_len == len(raw)
    vals = np.array(oracle.var_byte_values(seg.columns["category"]), dtype=object)
    cb = S.build_column("category", vals, S.STRING, dictionary=True)
    assert cb.cardinality == card
    cb.inverted = raw[inv_off:inv_off + inv_len]
    seg.columns["category"] = cb
    return seg
