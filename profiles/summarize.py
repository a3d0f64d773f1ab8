"""Summarise the rocprofv3 outputs of profiles/profile_r01.sh into profiles/<round>/.

    python3 profiles/summarize.py gpurun_out/prof profiles/r01

Writes kernel_stats_*.csv (copies of rocprofv3 --stats) and pmc_summary_bench40seg.json: per counter
the mean per dispatch of the hot kernel (pinot_scan_jit), the kernel-trace mean duration, and derived
HBM bytes (MI355X_MICROARCH.md: FETCH_SIZE is in KiB and reports half the bytes of wide coalesced
streaming reads on gfx950, so read bytes = FETCH_SIZE x 1024 x 2; WRITE_SIZE x 1024 is exact)."""
import csv
import collections
import json
import os
import shutil
import sys

ROWS_PER_LAUNCH = 400_000_000        # profile_r01.sh: 40 segments x 10M rows
BYTES_PER_ROW = 9 / 8 + 4 + 8 + 8    # datagen.BENCH_BYTES_PER_ROW
HOT = "pinot_scan_jit"


def counters(path):
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Kernel_Name"].startswith(HOT):
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    return agg


def main(src, dst):
    os.makedirs(dst, exist_ok=True)
    for sub, name in (("trace", "bench40seg"), ("trace_hc", "highcard40seg"), ("trace_ssb", "ssb20seg")):
        p = os.path.join(src, sub, "run_kernel_stats.csv")
        if os.path.exists(p):
            shutil.copy(p, os.path.join(dst, f"kernel_stats_{name}.csv"))
    out = {}
    for sub in ("pmc1", "pmc2", "pmc3"):
        p = os.path.join(src, sub, "run_counter_collection.csv")
        if not os.path.exists(p):
            continue
        for k, v in counters(p).items():
            out[k] = {"dispatches": len(v), "mean_per_dispatch": sum(v) / len(v)}
    durs = []
    tp = os.path.join(src, "trace", "run_kernel_trace.csv")
    if os.path.exists(tp):
        for r in csv.DictReader(open(tp)):
            if r["Kernel_Name"].startswith(HOT):
                durs.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
    if durs:
        out[f"{HOT}_trace_ms"] = {"dispatches": len(durs), "mean": sum(durs) / len(durs), "min": min(durs),
                                  "max": max(durs)}
    if "FETCH_SIZE" in out and "WRITE_SIZE" in out:
        rd = out["FETCH_SIZE"]["mean_per_dispatch"] * 1024 * 2
        wr = out["WRITE_SIZE"]["mean_per_dispatch"] * 1024
        alg = ROWS_PER_LAUNCH * BYTES_PER_ROW
        out["derived"] = {"rows_per_launch": ROWS_PER_LAUNCH, "algorithmic_bytes": alg,
                          "hbm_read_bytes_corrected": rd, "hbm_write_bytes": wr,
                          "traffic_over_algorithmic": (rd + wr) / alg}
        if durs:
            out["derived"]["achieved_GBps_from_trace"] = alg / (sum(durs) / len(durs) / 1e3) / 1e9
    with open(os.path.join(dst, "pmc_summary_bench40seg.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out.get("derived", {}), indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
