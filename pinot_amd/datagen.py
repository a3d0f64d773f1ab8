"""Synthetic segments for the benchmark, generated on the GPU.

The bench table follows the reference README's AdAnalytics example (daysSinceEpoch, clicks,
impressions, cost) extended with the column kinds BASELINE.json config 1 names: fixed-bit
dictionary-encoded columns and raw INT / LONG / DOUBLE columns. Values are drawn on the device,
dictIds are bit-packed by ``pinot_amd_fwd_pack_dict_ids`` (FixedBitSVForwardIndexWriter) and raw
values are byte-swapped to Pinot's big-endian layout on the device; the resulting segment files
are then handed to the normal host staging path, exactly as a server would load them.
"""
from __future__ import annotations

import numpy as np

from . import segment as S
from ._lib import check, lib

DAYS_BASE = 17000          # daysSinceEpoch dictionary values DAYS_BASE .. DAYS_BASE+364
NUM_DAYS = 365
NUM_COUNTRIES = 200


def _be_bytes(t, itemsize: int) -> bytes:
    """little-endian device tensor -> big-endian host bytes."""
    return t.contiguous().view(dtype=__import__("torch").uint8).view(-1, itemsize).flip(1).contiguous().cpu().numpy().tobytes()


def _fixed_bit(ids, bits: int) -> bytes:
    import torch
    n = ids.numel()
    nbytes = (n * bits + 7) // 8
    out = torch.zeros(nbytes + 8, dtype=torch.uint8, device=ids.device)
    check(lib().pinot_amd_fwd_pack_dict_ids(ids.data_ptr(), n, bits, out.data_ptr(), None), "pack")
    torch.cuda.synchronize()
    return out[:nbytes].cpu().numpy().tobytes()


def ad_segment(name: str, num_docs: int, seed: int, device: str = "cuda") -> S.SegmentBuffers:
    """One immutable segment of the AdAnalytics-style bench table (all columns unsorted)."""
    import torch
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    n = num_docs
    cols = {}
    # fixed-bit dictionary-encoded dimensions
    for cname, card, base in (("daysSinceEpoch", NUM_DAYS, DAYS_BASE), ("country", NUM_COUNTRIES, 0)):
        ids = torch.randint(0, card, (n,), generator=g, device=device, dtype=torch.int32)
        ids[:card] = torch.arange(card, device=device, dtype=torch.int32)  # every dictionary value present
        bits = S.num_bits_per_value(card - 1)
        dvals = np.arange(base, base + card, dtype=np.int32)
        cols[cname] = S.ColumnBuffers(cname, S.INT, n, True, False, card, bits, _fixed_bit(ids, bits),
                                      S.dictionary_bytes(dvals, S.INT), None, dvals)
    # raw metrics
    clicks = torch.randint(0, 1000, (n,), generator=g, device=device, dtype=torch.int32)
    impressions = torch.randint(0, 1 << 40, (n,), generator=g, device=device, dtype=torch.int64)
    cost = torch.rand((n,), generator=g, device=device, dtype=torch.float64) * 100.0
    for cname, t, st, size in (("clicks", clicks, S.INT, 4), ("impressions", impressions, S.LONG, 8),
                               ("cost", cost, S.DOUBLE, 8)):
        cols[cname] = S.ColumnBuffers(cname, st, n, False, fwd=S.raw_fwd_header(n, st) + _be_bytes(t, size))
    torch.cuda.synchronize()
    return S.SegmentBuffers(name, n, cols)


# The benchmark query: range filter on a fixed-bit column AND on a raw INT column, group by a
# fixed-bit column, SUM/COUNT/MAX over raw INT/LONG/DOUBLE columns (README AdAnalytics shape).
BENCH_QUERY = ("SELECT daysSinceEpoch, COUNT(*), SUM(clicks), SUM(impressions), SUM(cost), MAX(cost) FROM adAnalytics "
               f"WHERE daysSinceEpoch BETWEEN {DAYS_BASE + 100} AND {DAYS_BASE + 300} AND clicks > 100 "
               "GROUP BY daysSinceEpoch")

# BASELINE.json configs[0]: the reference README's AdAnalytics example query (README.md:95-100: an 8-day
# daysSinceEpoch range AND accountId IN (...), SUM(clicks), SUM(impressions) GROUP BY daysSinceEpoch),
# with the bench table's `country` dimension in the role of accountId (Pinot's TOP n is LIMIT n)
README_QUERY = ("SELECT daysSinceEpoch, SUM(clicks), SUM(impressions) FROM AdAnalyticsTable "
                f"WHERE ((daysSinceEpoch >= {DAYS_BASE + 249} AND daysSinceEpoch <= {DAYS_BASE + 256})) "
                "AND country IN (7, 42, 123) GROUP BY daysSinceEpoch LIMIT 100")
# its column bytes per row: 9-bit daysSinceEpoch + 8-bit country + 4 B clicks + 8 B impressions
README_BYTES_PER_ROW = (S.num_bits_per_value(NUM_DAYS - 1) + S.num_bits_per_value(NUM_COUNTRIES - 1)) / 8.0 + 4 + 8

# Algorithmic HBM bytes per row of BENCH_QUERY: every referenced column is read once
# (9-bit daysSinceEpoch + 4 B clicks + 8 B impressions + 8 B cost); group accumulators stay in LDS.
BENCH_BYTES_PER_ROW = S.num_bits_per_value(NUM_DAYS - 1) / 8.0 + 4 + 8 + 8


# ---------------------------------------------------------------------------------------------
# BASELINE.json configs[3]: high-cardinality GROUP BY on 2 dimensions (~1M groups)
HC_CARD = 1000             # dimA x dimB = 1,000,000 groups


def highcard_segment(name: str, num_docs: int, seed: int, device: str = "cuda") -> S.SegmentBuffers:
    """Segment of the high-cardinality table: two fixed-bit dictionary-encoded dimensions of
    cardinality 1000 (10 bits each) and raw INT / LONG / DOUBLE metrics."""
    import torch
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    n = num_docs
    cols = {}
    for cname, base in (("dimA", 1_000_000), ("dimB", 5_000_000)):
        ids = torch.randint(0, HC_CARD, (n,), generator=g, device=device, dtype=torch.int32)
        ids[:HC_CARD] = torch.arange(HC_CARD, device=device, dtype=torch.int32)
        bits = S.num_bits_per_value(HC_CARD - 1)
        dvals = np.arange(base, base + 7 * HC_CARD, 7, dtype=np.int32)
        cols[cname] = S.ColumnBuffers(cname, S.INT, n, True, False, HC_CARD, bits, _fixed_bit(ids, bits),
                                      S.dictionary_bytes(dvals, S.INT), None, dvals)
    met_int = torch.randint(0, 1000, (n,), generator=g, device=device, dtype=torch.int32)
    met_long = torch.randint(-(1 << 40), 1 << 40, (n,), generator=g, device=device, dtype=torch.int64)
    met_double = torch.randn((n,), generator=g, device=device, dtype=torch.float64) * 1000.0
    for cname, t, st, size in (("metInt", met_int, S.INT, 4), ("metLong", met_long, S.LONG, 8),
                               ("metDouble", met_double, S.DOUBLE, 8)):
        cols[cname] = S.ColumnBuffers(cname, st, n, False, fwd=S.raw_fwd_header(n, st) + _be_bytes(t, size))
    torch.cuda.synchronize()
    return S.SegmentBuffers(name, n, cols)


# SUM / COUNT / MIN / MAX grouped by both dimensions; numGroupsLimit raised above the key space so
# Pinot keeps every group (its default, 100000, would trim)
HIGHCARD_QUERY = ("SET numGroupsLimit = 2000000; SELECT dimA, dimB, COUNT(*), SUM(metInt), MIN(metLong), "
                  "MAX(metDouble) FROM highCard WHERE metInt < 900 GROUP BY dimA, dimB")
# the same query as Pinot runs it by default (numGroupsLimit 100000 < 1M keys per segment): each segment
# admits only the first 100000 groups it sees (DictionaryBasedGroupKeyGenerator.java:351-363)
HIGHCARD_DEFAULT_QUERY = HIGHCARD_QUERY.split(";", 1)[1].strip()
HIGHCARD_BYTES_PER_ROW =2 * S.num_bits_per_value(HC_CARD - 1) / 8.0 + 4 + 8 + 8


# ---------------------------------------------------------------------------------------------
# Wide group keys (the map-based holders of DictionaryBasedGroupKeyGenerator.java:444-900): a 5-column
# GROUP BY whose key space (20000^3 x 1000 x 500 = 4e18, 64 bits: two packed key words) is far past the
# dense cap (2^28), so the hash-table plan runs. Rows belong to ~1M entities drawn Zipf(1.1) (a few
# entities hold most rows, as real dimension data does); each entity's 5 attributes are fixed functions of
# it, so the present groups number ~1M although the key space is astronomically larger.
WIDE_ENTITIES = 1 << 20
WIDE_CARDS = (20000, 20000, 20000, 1000, 500)
WIDE_COLUMNS = ("w1", "w2", "w3", "w4", "w5")
_WIDE_MUL = (2654435761, 2246822519, 3266489917, 668265263, 374761393)


def _mix32(ent, j: int):
    """A 32-bit hash of entity ids (int64 tensor, values < 2^32; murmur3's finaliser over ent * m_j + j): the
    dimension values of distinct entities are independent, so ~every entity is its own 5-column group. (Through
    round 5 the dimensions were (ent * m_j + j) mod card_j: every cardinality divides 20000, so the 5-tuple was a
    function of ent mod 20000 -- at most ~20K distinct groups, not the ~1M entities the workload describes.)"""
    m = 0xFFFFFFFF
    x = (ent * _WIDE_MUL[j] + j * 0x27D4EB2F) & m
    x = x ^ (x >> 16)
    x = (x * 0x85EBCA6B) & m
    x = x ^ (x >> 13)
    x = (x * 0xC2B2AE35) & m
    return x ^ (x >> 16)


def widekeys_segment(name: str, num_docs: int, seed: int, device: str = "cuda", uniform: bool = False) -> S.SegmentBuffers:
    """Segment of the wide-key table: entity e ~ Zipf(1.1) over WIDE_ENTITIES ranks (inverse-CDF of the
    continuous Pareto approximation) -- or, uniform=True, uniform over them (no hot keys: the unskewed case of
    the map-based holders) -- dimension j = (e * m_j + j) mod card_j as a fixed-bit dictionary column (the first
    card_j docs take every dictionary value once), raw INT / DOUBLE metrics."""
    import torch
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    n = num_docs
    u = torch.rand((n,), generator=g, device=device, dtype=torch.float64)
    if uniform:
        ent = torch.clamp((u * WIDE_ENTITIES).to(torch.int64), 0, WIDE_ENTITIES - 1)
    else:
        s_ = 1.1
        a = WIDE_ENTITIES ** (1.0 - s_)
        ent = torch.clamp(((a - 1.0) * u + 1.0) ** (1.0 / (1.0 - s_)), 1.0, float(WIDE_ENTITIES)).to(torch.int64) - 1
    cols = {}
    for j, (cname, card) in enumerate(zip(WIDE_COLUMNS, WIDE_CARDS)):
        ids = (_mix32(ent, j) % card).to(torch.int32)
        ids[:card] = torch.arange(card, device=device, dtype=torch.int32)
        bits = S.num_bits_per_value(card - 1)
        dvals = np.arange(card, dtype=np.int32)
        cols[cname] = S.ColumnBuffers(cname, S.INT, n, True, False, card, bits, _fixed_bit(ids, bits),
                                      S.dictionary_bytes(dvals, S.INT), None, dvals)
    met_int = torch.randint(0, 1000, (n,), generator=g, device=device, dtype=torch.int32)
    met_double = torch.randn((n,), generator=g, device=device, dtype=torch.float64) * 1000.0
    for cname, t, st, size in (("metInt", met_int, S.INT, 4), ("metDouble", met_double, S.DOUBLE, 8)):
        cols[cname] = S.ColumnBuffers(cname, st, n, False, fwd=S.raw_fwd_header(n, st) + _be_bytes(t, size))
    torch.cuda.synchronize()
    return S.SegmentBuffers(name, n, cols)


WIDEKEYS_QUERY = ("SET numGroupsLimit = 2000000000; SELECT w1, w2, w3, w4, w5, COUNT(*), SUM(metInt), MAX(metDouble) "
                  "FROM wide WHERE metInt < 900 GROUP BY w1, w2, w3, w4, w5")
def widekeys_uniform_segment(name: str, num_docs: int, seed: int, device: str = "cuda") -> S.SegmentBuffers:
    """The wide-key table with entities uniform over WIDE_ENTITIES (~1M groups, none hot)."""
    return widekeys_segment(name, num_docs, seed, device, uniform=True)


WIDEKEYS_BYTES_PER_ROW = sum(S.num_bits_per_value(c - 1) for c in WIDE_CARDS) / 8.0 + 4 + 8


# ---------------------------------------------------------------------------------------------
# BASELINE.json configs[2]: inverted-index EQ/IN filters combined with AND/OR across 3 columns
INV_CARD = 10000           # dictionary cardinality of invA / invB / invC (14-bit fixed-bit forward index)
INV_COLUMNS = ("invA", "invB", "invC")


def inverted_segment(name: str, num_docs: int, seed: int, device: str = "cuda") -> S.SegmentBuffers:
    """Segment with three uniformly distributed dictionary-encoded INT columns carrying bitmap
    inverted indexes (RoaringBitmap array containers, BitmapInvertedIndexWriter layout) and raw
    INT / DOUBLE metrics."""
    import torch
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    n = num_docs
    cols = {}
    bits = S.num_bits_per_value(INV_CARD - 1)
    dvals = np.arange(INV_CARD, dtype=np.int32) * 3 + 1
    for cname in INV_COLUMNS:
        ids = torch.randint(0, INV_CARD, (n,), generator=g, device=device, dtype=torch.int32)
        ids[:INV_CARD] = torch.arange(INV_CARD, device=device, dtype=torch.int32)
        inv = S.inverted_index_bytes(ids.cpu().numpy(), INV_CARD)
        cols[cname] = S.ColumnBuffers(cname, S.INT, n, True, False, INV_CARD, bits, _fixed_bit(ids, bits),
                                      S.dictionary_bytes(dvals, S.INT), inv, dvals)
    m = torch.randint(0, 1000, (n,), generator=g, device=device, dtype=torch.int32)
    cost = torch.rand((n,), generator=g, device=device, dtype=torch.float64) * 100.0
    cols["metInt"] = S.ColumnBuffers("metInt", S.INT, n, False, fwd=S.raw_fwd_header(n, S.INT) + _be_bytes(m, 4))
    cols["cost"] = S.ColumnBuffers("cost", S.DOUBLE, n, False, fwd=S.raw_fwd_header(n, S.DOUBLE) + _be_bytes(cost, 8))
    torch.cuda.synchronize()
    return S.SegmentBuffers(name, n, cols)


def inverted_fraction(selectivity: float) -> float:
    """Per-column IN fraction f with f * (1 - (1 - f)^2) = selectivity (uniform independent columns)."""
    lo, hi = 0.0, 1.0
    for _ in range(60):
        f = (lo + hi) / 2
        if f * (2 * f - f * f) < selectivity:
            lo = f
        else:
            hi = f
    return (lo + hi) / 2


def inverted_query(selectivity: float) -> str:
    """invA IN (...) AND (invB IN (...) OR invC IN (...)), each IN list a fraction f of the
    dictionary (values spread over it), for a target selectivity; COUNT + SUMs of raw metrics."""
    f = inverted_fraction(selectivity)
    k = max(1, int(round(f * INV_CARD)))
    lists = []
    for j in range(3):
        ids = (np.arange(k, dtype=np.int64) * INV_CARD // k + j * 7) % INV_CARD
        lists.append(", ".join(str(int(v) * 3 + 1) for v in np.unique(ids)))
    return (f"SELECT COUNT(*), SUM(metInt), SUM(cost) FROM invTable WHERE invA IN ({lists[0]}) AND "
            f"(invB IN ({lists[1]}) OR invC IN ({lists[2]}))")


INVERTED_SELECTIVITIES = (0.0001, 0.001, 0.01, 0.1, 0.5)
