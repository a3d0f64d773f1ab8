"""Join build/fetch_probe's known byte counts with its rocprofv3 --pmc dispatches (profiles/fetch_probe.hip).

    python3 profiles/fetch_probe.py <probe stdout> <pass dir> [<pass dir> ...] > profiles/r06/fetch_probe.json

Per probe launch: FETCH_SIZE x 1024 (bytes as reported) against the launch's known bytes at 32-, 64- and 128-byte
granularity; for a gather, the docId list's own FETCH (the probe_idx launch just before it, same list) is taken
off first. `ratio64` = reported / distinct-64-B bytes: 0.5 means the counter tallies half (double it), 1.0 means
it reads the touched sectors as they are."""
import csv
import glob
import json
import os
import sys


def dispatches(pass_dir):
    rows = {}
    for path in glob.glob(os.path.join(pass_dir, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(path)):
            k = r["Kernel_Name"].split("(")[0].strip()
            if not k.startswith("probe_") or k == "probe_flush":
                continue
            d = int(r.get("Dispatch_Id") or r.get("Correlation_Id") or 0)
            rows.setdefault((d, k), {})[r["Counter_Name"]] = rows.get((d, k), {}).get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return [(k, c) for (d, k), c in sorted(rows.items())]


def main(stdout_path, pass_dirs):
    launches = [json.loads(l) for l in open(stdout_path) if l.startswith("{")]
    counters = [{} for _ in launches]
    for pd in pass_dirs:
        ds = dispatches(pd)
        if len(ds) != len(launches):
            raise SystemExit(f"{pd}: {len(ds)} probe dispatches, {len(launches)} launches reported")
        for i, ((k, c), l) in enumerate(zip(ds, launches)):
            assert k == l["kernel"], (i, k, l["kernel"])
            counters[i].update(c)
    out = []
    prev_idx = None
    for l, c in zip(launches, counters):
        row = dict(l)
        row["counters"] = c
        if "FETCH_SIZE" in c:
            fetched = c["FETCH_SIZE"] * 1024.0
            if l["kernel"] == "probe_idx":
                prev_idx = fetched
            if l["kernel"] in ("probe_gather4", "probe_gather8") and prev_idx is not None:
                row["fetch_minus_idx"] = fetched - prev_idx
                fetched -= prev_idx
            known_extra = l.get("meta", 0)
            for g in ("b32", "b64", "b128"):
                row["ratio" + g[1:]] = round(fetched / (l[g] + known_extra), 4) if l[g] else None
        out.append(row)
    json.dump({"launches": out}, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2:])
