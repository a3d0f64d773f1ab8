"""Per-kernel dispatch durations from a rocprofv3 kernel trace (run_kernel_trace.csv): for each kernel, the
number of dispatches, and the durations (us) of the last K -- the timed steps of a bench run come last.
Usage: python scripts/trace_tail.py <run_kernel_trace.csv> [K]"""
import csv
import sys
from collections import OrderedDict

path = sys.argv[1]
k = int(sys.argv[2]) if len(sys.argv) > 2 else 5
by = OrderedDict()
for r in csv.DictReader(open(path)):
    name = r.get("Kernel_Name") or r.get("Kernel Name") or "?"
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    by.setdefault(name, []).append(d)
rows = sorted(by.items(), key=lambda kv: -sum(kv[1][-k:]))
for name, ds in rows[:25]:
    tail = ds[-k:]
    print(f"{name[:70]:70s} n={len(ds):6d} last{k}_mean_us={sum(tail) / len(tail):10.1f} last=" +
          ",".join(f"{x:.0f}" for x in tail))
