"""SSB golden fixtures from the reference's own SSB data and query set.

Run in the build container (reads /root/reference as DATA only):

    python tests/golden/make_ssb_golden.py

Inputs: the quickstart SSB tables shipped with the reference
(pinot-tools/src/main/resources/examples/batch/ssb/{lineorder,dates,part,supplier,customer}/rawdata/*.avro,
avro snappy codec) and the 13 queries of pinot-integration-tests/src/test/resources/ssb/ssb_query_set.yaml
that SSBQueryTest.java validates against H2.

Outputs (committed; the GPU box has no /root/reference):
  tests/golden/ssb_flat.npz       lineorder (9999 rows) left-joined with its 4 dimension tables, the
                                  columns of pinot_amd.ssb.FLAT_COLUMNS; attributes of missing dimension
                                  rows are Pinot's default null values ("null", Integer.MIN_VALUE)
  tests/golden/ssb_expected.json  per query: the group-by result (every group, before ORDER BY/LIMIT)
                                  computed here by a direct restatement of each query's join + filter +
                                  group + SUM over the joined rows (inner-join semantics, exact integer
                                  sums; CAST(... AS DOUBLE) products are exact in double at these sizes)
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
from make_golden import read_avro  # noqa: E402
from pinot_amd.ssb import FLAT_COLUMNS, SSB_QUERIES  # noqa: E402

SSB = "/root/reference/pinot-tools/src/main/resources/examples/batch/ssb/"
INT_NULL = -(2 ** 31)


def load():
    t = {name: read_avro(SSB + f"{name}/rawdata/{name}.avro")[1]
         for name in ("lineorder", "dates", "part", "supplier", "customer")}
    return (t["lineorder"], {r["D_DATEKEY"]: r for r in t["dates"]}, {r["P_PARTKEY"]: r for r in t["part"]},
            {r["S_SUPPKEY"]: r for r in t["supplier"]}, {r["C_CUSTKEY"]: r for r in t["customer"]})


# each query restated: (dimensions joined, filter over the joined row, group-by columns, summed value)
def _in_years(r, lo, hi):
    return lo <= r["D_YEAR"] <= hi


UK = ("UNITED KI1", "UNITED KI5")
RESTATED = {
    "Q1.1": ("D", lambda r: r["D_YEAR"] == 1993 and 1 <= r["LO_DISCOUNT"] <= 3 and r["LO_QUANTITY"] < 25, (),
             lambda r: float(r["LO_EXTENDEDPRICE"]) * r["LO_DISCOUNT"]),
    "Q1.2": ("D", lambda r: r["D_YEARMONTHNUM"] == 199401 and 4 <= r["LO_DISCOUNT"] <= 6 and 26 <= r["LO_QUANTITY"] <= 35,
             (), lambda r: float(r["LO_EXTENDEDPRICE"]) * r["LO_DISCOUNT"]),
    "Q1.3": ("D", lambda r: r["D_WEEKNUMINYEAR"] == 6 and r["D_YEAR"] == 1994 and 5 <= r["LO_DISCOUNT"] <= 7
             and 26 <= r["LO_QUANTITY"] <= 35, (), lambda r: float(r["LO_EXTENDEDPRICE"]) * r["LO_DISCOUNT"]),
    "Q2.1": ("DPS", lambda r: r["P_CATEGORY"] == "MFGR#12" and r["S_REGION"] == "AMERICA", ("D_YEAR", "P_BRAND1"),
             lambda r: float(r["LO_REVENUE"])),
    "Q2.2": ("DPS", lambda r: "MFGR#2221" <= r["P_BRAND1"] <= "MFGR#2228" and r["S_REGION"] == "ASIA",
             ("D_YEAR", "P_BRAND1"), lambda r: float(r["LO_REVENUE"])),
    "Q2.3": ("DPS", lambda r: r["P_BRAND1"] == "MFGR#2221" and r["S_REGION"] == "EUROPE", ("D_YEAR", "P_BRAND1"),
             lambda r: float(r["LO_REVENUE"])),
    "Q3.1": ("CSD", lambda r: r["C_REGION"] == "ASIA" and r["S_REGION"] == "ASIA" and _in_years(r, 1992, 1997),
             ("C_NATION", "S_NATION", "D_YEAR"), lambda r: r["LO_REVENUE"]),
    "Q3.2": ("CSD", lambda r: r["C_NATION"] == "UNITED STATES" and r["S_NATION"] == "UNITED STATES"
             and _in_years(r, 1992, 1997), ("C_CITY", "S_CITY", "D_YEAR"), lambda r: r["LO_REVENUE"]),
    "Q3.3": ("CSD", lambda r: r["C_CITY"] in UK and r["S_CITY"] in UK and _in_years(r, 1992, 1997),
             ("C_CITY", "S_CITY", "D_YEAR"), lambda r: r["LO_REVENUE"]),
    "Q3.4": ("CSD", lambda r: r["C_CITY"] in UK and r["S_CITY"] in UK and r["D_YEARMONTH"] == "Jul1995",
             ("C_CITY", "S_CITY", "D_YEAR"), lambda r: r["LO_REVENUE"]),
    "Q4.1": ("CSPD", lambda r: r["C_REGION"] == "AMERICA" and r["S_REGION"] == "AMERICA"
             and r["P_MFGR"] in ("MFGR#1", "MFGR#2"), ("D_YEAR", "C_NATION"),
             lambda r: float(r["LO_REVENUE"] - r["LO_SUPPLYCOST"])),
    "Q4.2": ("CSPD", lambda r: r["C_REGION"] == "AMERICA" and r["S_REGION"] == "AMERICA" and r["D_YEAR"] in (1997, 1998)
             and r["P_MFGR"] in ("MFGR#1", "MFGR#2"), ("D_YEAR", "S_NATION", "P_CATEGORY"),
             lambda r: float(r["LO_REVENUE"] - r["LO_SUPPLYCOST"])),
    "Q4.3": ("CSPD", lambda r: r["C_REGION"] == "AMERICA" and r["S_NATION"] == "UNITED STATES"
             and r["D_YEAR"] in (1997, 1998) and r["P_CATEGORY"] == "MFGR#14", ("D_YEAR", "S_CITY", "P_BRAND1"),
             lambda r: float(r["LO_REVENUE"] - r["LO_SUPPLYCOST"])),
}


def main():
    if not os.path.isdir(SSB):
        sys.exit("reference SSB data not present (this script only runs in the build container)")
    lo, dates, part, supp, cust = load()
    # flat table (left join, Pinot default nulls)
    flat = {name: [] for name, _, _ in FLAT_COLUMNS}
    joined = []
    for r in lo:
        row = dict(r)
        dims = {"D": dates.get(r["LO_ORDERDATE"]), "P": part.get(r["LO_PARTKEY"]),
                "S": supp.get(r["LO_SUPPKEY"]), "C": cust.get(r["LO_CUSTKEY"])}
        for d in dims.values():
            if d:
                row.update(d)
        joined.append((row, dims))
        for name, t, _ in FLAT_COLUMNS:
            v = row.get(name)
            if v is None:
                v = "null" if t == "STRING" else INT_NULL
            flat[name].append(v)
    arrays = {name: (np.array(flat[name], dtype=str) if t == "STRING" else np.array(flat[name], dtype=np.int32))
              for name, t, _ in FLAT_COLUMNS}
    np.savez_compressed(os.path.join(HERE, "ssb_flat.npz"), **arrays)
    out = []
    for name, sql in SSB_QUERIES:
        joins, pred, gcols, val = RESTATED[name]
        groups = {}
        for row, dims in joined:
            if any(dims[j] is None for j in joins) or not pred(row):
                continue
            k = tuple(row[c] for c in gcols)
            groups[k] = groups.get(k, 0) + val(row)
        out.append({"name": name, "sql": sql, "group_by": list(gcols),
                    "groups": [list(k) + [float(v)] for k, v in sorted(groups.items())]})
        print(name, len(groups), "groups")
    with open(os.path.join(HERE, "ssb_expected.json"), "w") as f:
        json.dump({"source": "reference SSB quickstart data + ssb_query_set.yaml, restated in make_ssb_golden.py",
                   "rows": len(lo), "queries": out}, f, indent=1)


if __name__ == "__main__":
    main()
