"""Star Schema Benchmark on the denormalized lineorder table (BASELINE.json configs[4]).

The reference runs SSB through the multi-stage engine with joins
(pinot-integration-tests/src/test/resources/ssb/ssb_query_set.yaml, SSBQueryTest.java); the
config here is the denormalized ("flat") lineorder, so each query is a single-table
filter + group-by over columns named after the dimension attributes. Every query filters on
each dimension it touches, so on a lineorder left-joined with its dimensions (missing attributes
= Pinot's default null values) the flat query selects exactly the inner join's rows.

``lineorder_flat_segment`` generates SF-scaled synthetic data with dbgen's value domains
(dates 1992-01-01..1998-12-31, 5 regions / 25 nations / 250 cities, MFGR#1..5, 25 categories,
1000 brands, quantity 1..50, discount 0..10, extendedprice = quantity x part price, revenue =
extendedprice x (100 - discount) / 100, supplycost = 60 % of the part price); all attribute
columns are dictionary-encoded (fixed-bit forward indexes), the metric columns raw INT.
"""
from __future__ import annotations

import datetime

import numpy as np

from . import segment as S

_DATE_WHERE = "LO_ORDERDATE = D_DATEKEY"  # documentation only: the flat table has the D_* columns

SSB_QUERIES = [
    ("Q1.1", "select sum(CAST(LO_EXTENDEDPRICE AS DOUBLE) * LO_DISCOUNT) as revenue from lineorder_flat "
             "where D_YEAR = 1993 and LO_DISCOUNT between 1 and 3 and LO_QUANTITY < 25"),
    ("Q1.2", "select sum(CAST(LO_EXTENDEDPRICE AS DOUBLE) * LO_DISCOUNT) as revenue from lineorder_flat "
             "where D_YEARMONTHNUM = 199401 and LO_DISCOUNT between 4 and 6 and LO_QUANTITY between 26 and 35"),
    ("Q1.3", "select sum(CAST(LO_EXTENDEDPRICE AS DOUBLE) * LO_DISCOUNT) as revenue from lineorder_flat "
             "where D_WEEKNUMINYEAR = 6 and D_YEAR = 1994 and LO_DISCOUNT between 5 and 7 "
             "and LO_QUANTITY between 26 and 35"),
    ("Q2.1", "select sum(CAST(LO_REVENUE AS DOUBLE)), D_YEAR, P_BRAND1 from lineorder_flat "
             "where P_CATEGORY = 'MFGR#12' and S_REGION = 'AMERICA' group by D_YEAR, P_BRAND1 "
             "order by D_YEAR, P_BRAND1"),
    ("Q2.2", "select sum(CAST(LO_REVENUE AS DOUBLE)), D_YEAR, P_BRAND1 from lineorder_flat "
             "where P_BRAND1 between 'MFGR#2221' and 'MFGR#2228' and S_REGION = 'ASIA' group by D_YEAR, P_BRAND1 "
             "order by D_YEAR, P_BRAND1"),
    ("Q2.3", "select sum(CAST(LO_REVENUE AS DOUBLE)), D_YEAR, P_BRAND1 from lineorder_flat "
             "where P_BRAND1 = 'MFGR#2221' and S_REGION = 'EUROPE' group by D_YEAR, P_BRAND1 "
             "order by D_YEAR, P_BRAND1"),
    ("Q3.1", "select C_NATION, S_NATION, D_YEAR, sum(LO_REVENUE) as revenue from lineorder_flat "
             "where C_REGION = 'ASIA' and S_REGION = 'ASIA' and D_YEAR >= 1992 and D_YEAR <= 1997 "
             "group by C_NATION, S_NATION, D_YEAR order by D_YEAR asc, revenue desc"),
    ("Q3.2", "select C_CITY, S_CITY, D_YEAR, sum(LO_REVENUE) as revenue from lineorder_flat "
             "where C_NATION = 'UNITED STATES' and S_NATION = 'UNITED STATES' and D_YEAR >= 1992 "
             "and D_YEAR <= 1997 group by C_CITY, S_CITY, D_YEAR order by D_YEAR asc, revenue desc"),
    ("Q3.3", "select C_CITY, S_CITY, D_YEAR, sum(LO_REVENUE) as revenue from lineorder_flat "
             "where (C_CITY='UNITED KI1' or C_CITY='UNITED KI5') and (S_CITY='UNITED KI1' or S_CITY='UNITED KI5') "
             "and D_YEAR >= 1992 and D_YEAR <= 1997 group by C_CITY, S_CITY, D_YEAR "
             "order by D_YEAR asc, revenue desc"),
    ("Q3.4", "select C_CITY, S_CITY, D_YEAR, sum(LO_REVENUE) as revenue from lineorder_flat "
             "where (C_CITY='UNITED KI1' or C_CITY='UNITED KI5') and (S_CITY='UNITED KI1' or S_CITY='UNITED KI5') "
             "and D_YEARMONTH = 'Jul1995' group by C_CITY, S_CITY, D_YEAR order by D_YEAR asc, revenue desc"),
    ("Q4.1", "select D_YEAR, C_NATION, sum(LO_REVENUE - LO_SUPPLYCOST) as profit from lineorder_flat "
             "where C_REGION = 'AMERICA' and S_REGION = 'AMERICA' and (P_MFGR = 'MFGR#1' or P_MFGR = 'MFGR#2') "
             "group by D_YEAR, C_NATION order by D_YEAR, C_NATION"),
    ("Q4.2", "select D_YEAR, S_NATION, P_CATEGORY, sum(LO_REVENUE - LO_SUPPLYCOST) as profit from lineorder_flat "
             "where C_REGION = 'AMERICA' and S_REGION = 'AMERICA' and (D_YEAR = 1997 or D_YEAR = 1998) "
             "and (P_MFGR = 'MFGR#1' or P_MFGR = 'MFGR#2') group by D_YEAR, S_NATION, P_CATEGORY "
             "order by D_YEAR, S_NATION, P_CATEGORY"),
    ("Q4.3", "select D_YEAR, S_CITY, P_BRAND1, sum(LO_REVENUE - LO_SUPPLYCOST) as profit from lineorder_flat "
             "where C_REGION = 'AMERICA' and S_NATION = 'UNITED STATES' and (D_YEAR = 1997 or D_YEAR = 1998) "
             "and P_CATEGORY = 'MFGR#14' group by D_YEAR, S_CITY, P_BRAND1 order by D_YEAR, S_CITY, P_BRAND1"),
]

# flat-table columns: (name, Pinot type, dictionary-encoded)
FLAT_COLUMNS = [
    ("LO_ORDERDATE", S.INT, True), ("LO_QUANTITY", S.INT, True), ("LO_DISCOUNT", S.INT, True),
    ("LO_EXTENDEDPRICE", S.INT, False), ("LO_REVENUE", S.INT, False), ("LO_SUPPLYCOST", S.INT, False),
    ("D_YEAR", S.INT, True), ("D_YEARMONTHNUM", S.INT, True), ("D_YEARMONTH", S.STRING, True),
    ("D_WEEKNUMINYEAR", S.INT, True),
    ("P_MFGR", S.STRING, True), ("P_CATEGORY", S.STRING, True), ("P_BRAND1", S.STRING, True),
    ("S_REGION", S.STRING, True), ("S_NATION", S.STRING, True), ("S_CITY", S.STRING, True),
    ("C_REGION", S.STRING, True), ("C_NATION", S.STRING, True), ("C_CITY", S.STRING, True),
]

# dbgen nations (index = nation key) and their regions
NATIONS = ["ALGERIA", "ARGENTINA", "BRAZIL", "CANADA", "EGYPT", "ETHIOPIA", "FRANCE", "GERMANY", "INDIA",
           "INDONESIA", "IRAN", "IRAQ", "JAPAN", "JORDAN", "KENYA", "MOROCCO", "MOZAMBIQUE", "PERU", "CHINA",
           "ROMANIA", "SAUDI ARABIA", "VIETNAM", "RUSSIA", "UNITED KINGDOM", "UNITED STATES"]
NATION_REGION = [0, 1, 1, 1, 4, 0, 3, 3, 2, 2, 4, 4, 2, 4, 0, 0, 0, 1, 2, 3, 4, 2, 3, 3, 1]
REGIONS = ["AFRICA", "AMERICA", "ASIA", "EUROPE", "MIDDLE EAST"]
MONTHS = ["Jan", "Feb", "Mar", "Apr", "May", "Jun", "Jul", "Aug", "Sep", "Oct", "Nov", "Dec"]


def city_name(nation: str, i: int) -> str:
    """dbgen city: the nation name padded / cut to 9 characters + a digit."""
    return (nation + " " * 9)[:9] + str(i)


def _dates():
    d0 = datetime.date(1992, 1, 1)
    days = (datetime.date(1998, 12, 31) - d0).days + 1
    rows = []
    for k in range(days):
        d = d0 + datetime.timedelta(days=k)
        rows.append((d.year * 10000 + d.month * 100 + d.day, d.year, d.year * 100 + d.month,
                     MONTHS[d.month - 1] + str(d.year), min(53, (d.timetuple().tm_yday - 1) // 7 + 1)))
    return rows


def lineorder_flat_segment(name: str, num_docs: int, seed: int, device: str = "cuda") -> S.SegmentBuffers:
    """One segment of SF-scaled synthetic denormalized lineorder (see module docstring)."""
    import torch
    from .datagen import _be_bytes, _fixed_bit
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    n = num_docs
    ri = lambda lo, hi: torch.randint(lo, hi, (n,), generator=g, device=device, dtype=torch.int64)  # noqa: E731
    dates = _dates()
    di = ri(0, len(dates))
    nation_c, nation_s = ri(0, 25), ri(0, 25)
    city_c, city_s = nation_c * 10 + ri(0, 10), nation_s * 10 + ri(0, 10)
    mfgr = ri(0, 5)
    cat = mfgr * 5 + ri(0, 5)
    brand = cat * 40 + ri(0, 40)
    qty = ri(1, 51)
    disc = ri(0, 11)
    price = 90000 + ri(0, 111001)                  # part retail price in cents (dbgen: 900.00 .. 2010.00)
    ext = qty * price
    rev = ext * (100 - disc) // 100
    supc = price * 6 // 10
    region_of = torch.tensor(NATION_REGION, device=device)

    def dict_col(cname, ids, values, stype):
        """ids index into `values` (any order); builds the sorted dictionary + fixed-bit forward index."""
        vals = np.asarray(values, dtype=object if stype == S.STRING else np.int64)
        if stype == S.STRING:
            order = sorted(range(len(vals)), key=lambda i: S._java_string_key(vals[i]))
        else:
            order = list(np.argsort(vals, kind="stable"))
        rank = np.empty(len(vals), dtype=np.int64)
        rank[np.asarray(order, dtype=np.int64)] = np.arange(len(vals))
        present = torch.zeros(len(vals), dtype=torch.bool, device=device)
        present[ids] = True
        keep = np.asarray(order, dtype=np.int64)[present.cpu().numpy()[np.asarray(order, dtype=np.int64)]]
        # dictionary = present values in sorted order; dictIds = rank among present values
        remap = np.full(len(vals), -1, dtype=np.int64)
        remap[keep] = np.arange(len(keep))
        d_ids = torch.from_numpy(remap).to(device)[ids].to(torch.int32)
        dvals = vals[keep]
        card = len(dvals)
        bits = S.num_bits_per_value(card - 1)
        dv = dvals if stype == S.STRING else dvals.astype(np.int32)
        return S.ColumnBuffers(cname, stype, n, True, False, card, bits, _fixed_bit(d_ids, bits),
                               S.dictionary_bytes(dv, stype), None, dv)

    date_key = [r[0] for r in dates]
    cols = {
        "LO_ORDERDATE": dict_col("LO_ORDERDATE", di, date_key, S.INT),
        "LO_QUANTITY": dict_col("LO_QUANTITY", qty - 1, list(range(1, 51)), S.INT),
        "LO_DISCOUNT": dict_col("LO_DISCOUNT", disc, list(range(0, 11)), S.INT),
        "D_YEAR": dict_col("D_YEAR", (torch.tensor([r[1] for r in dates], device=device)[di] - 1992), list(range(1992, 1999)), S.INT),
        "D_YEARMONTHNUM": None, "D_YEARMONTH": None, "D_WEEKNUMINYEAR": None,
    }
    ym = torch.tensor([(r[1] - 1992) * 12 + (r[2] % 100) - 1 for r in dates], device=device)[di]
    cols["D_YEARMONTHNUM"] = dict_col("D_YEARMONTHNUM", ym, [(1992 + i // 12) * 100 + i % 12 + 1 for i in range(84)], S.INT)
    cols["D_YEARMONTH"] = dict_col("D_YEARMONTH", ym, [MONTHS[i % 12] + str(1992 + i // 12) for i in range(84)], S.STRING)
    wk = torch.tensor([r[4] for r in dates], device=device)[di] - 1
    cols["D_WEEKNUMINYEAR"] = dict_col("D_WEEKNUMINYEAR", wk, list(range(1, 54)), S.INT)
    cols["P_MFGR"] = dict_col("P_MFGR", mfgr, [f"MFGR#{i + 1}" for i in range(5)], S.STRING)
    cols["P_CATEGORY"] = dict_col("P_CATEGORY", cat, [f"MFGR#{i // 5 + 1}{i % 5 + 1}" for i in range(25)], S.STRING)
    cols["P_BRAND1"] = dict_col("P_BRAND1", brand, [f"MFGR#{i // 200 + 1}{i // 40 % 5 + 1}{i % 40 + 1}" for i in range(1000)],
                                S.STRING)
    for pre, nat, cty in (("S", nation_s, city_s), ("C", nation_c, city_c)):
        cols[f"{pre}_REGION"] = dict_col(f"{pre}_REGION", region_of[nat], REGIONS, S.STRING)
        cols[f"{pre}_NATION"] = dict_col(f"{pre}_NATION", nat, NATIONS, S.STRING)
        cols[f"{pre}_CITY"] = dict_col(f"{pre}_CITY", cty, [city_name(NATIONS[i // 10], i % 10) for i in range(250)],
                                       S.STRING)
    for cname, t in (("LO_EXTENDEDPRICE", ext), ("LO_REVENUE", rev), ("LO_SUPPLYCOST", supc)):
        cols[cname] = S.ColumnBuffers(cname, S.INT, n, False,
                                      fwd=S.raw_fwd_header(n, S.INT) + _be_bytes(t.to(torch.int32), 4))
    torch.cuda.synchronize()
    return S.SegmentBuffers(name, n, cols)
