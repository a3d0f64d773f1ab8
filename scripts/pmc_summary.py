"""Mean PMC counter values per kernel from rocprofv3 counter_collection CSVs (argv: csv files)."""
import csv
import sys
from collections import defaultdict

for path in sys.argv[1:]:
    acc = defaultdict(lambda: defaultdict(list))
    with open(path) as f:
        for row in csv.DictReader(f):
            k = row["Kernel_Name"][:40]
            acc[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
    print(path)
    for k, cs in acc.items():
        if not k.startswith("pinot"):
            continue
        print("  ", k, {c: "%.4g" % (sum(v) / len(v)) for c, v in sorted(cs.items())})
