# Per-dispatch PMC values of one kernel (name substring K) for one bench invocation, one pass per counter set:
#   K=pinot_scan_jit SETS="A B;C D" ARGS="--workload wide-keys --segments 40" bash scripts/pmc_dispatch.sh
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/pmcd
rm -rf $OUT; mkdir -p $OUT
IFS=';' read -ra PASSES <<< "$SETS"
i=0
for set in "${PASSES[@]}"; do
  i=$((i + 1))
  timeout -s KILL 150 rocprofv3 --pmc $set --kernel-trace --output-format csv -d $OUT/p$i -o run -- python3 bench.py $ARGS --steps 3 --warmup 1 --no-cpu-baseline > $OUT/p$i.json 2> $OUT/p$i.err || { echo "pass $i failed"; tail -5 $OUT/p$i.err; exit 1; }
done
K="$K" python3 - <<'PY'
import csv, glob, collections, os
k = os.environ["K"]
for f in sorted(glob.glob("gpurun_out/pmcd/p*/**/run_counter_collection.csv", recursive=True)):
    per = collections.OrderedDict()
    for row in csv.DictReader(open(f)):
        if k not in row["Kernel_Name"]:
            continue
        d = int(row["Dispatch_Id"])
        per.setdefault(d, collections.defaultdict(float))[row["Counter_Name"]] += float(row["Counter_Value"])
    print(f.split("/")[2])
    for d, cs in per.items():
        print("  dispatch %5d " % d + " ".join("%s=%.4g" % (c, v) for c, v in sorted(cs.items())))
for f in sorted(glob.glob("gpurun_out/pmcd/p*/**/run_kernel_trace.csv", recursive=True)):
    print(f.split("/")[2], "durations (us):", " ".join("%.0f" % ((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
          for r in csv.DictReader(open(f)) if k in r["Kernel_Name"]))
PY
find $OUT -name "run_counter_collection.csv" -o -name "run_kernel_trace.csv" | xargs rm -f
