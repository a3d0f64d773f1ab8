# Ad-hoc PMC passes for one bench invocation (one pass per counter set, each a short run of its own):
#   SETS="A B C;D E" ARGS="--workload ssb --segments 20 --query-index 11" bash scripts/pmc_custom.sh
# prints per-kernel mean of each counter (per dispatch) for the pinot_* kernels
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/pmcc
rm -rf $OUT; mkdir -p $OUT
IFS=';' read -ra PASSES <<< "$SETS"
i=0
for set in "${PASSES[@]}"; do
  i=$((i + 1))
  timeout -s KILL 150 rocprofv3 --pmc $set --output-format csv -d $OUT/p$i -o run -- python3 bench.py $ARGS --steps 3 --warmup 1 --no-cpu-baseline > $OUT/p$i.json 2> $OUT/p$i.err || { echo "pass $i failed"; tail -5 $OUT/p$i.err; exit 1; }
done
python3 - <<'PY'
import csv, glob, collections
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob("gpurun_out/pmcc/p*/**/run_counter_collection.csv", recursive=True):
    per = collections.defaultdict(float)
    for row in csv.DictReader(open(f)):
        k = row["Kernel_Name"]
        if "pinot_" not in k and "spill_" not in k:
            continue
        per[(k, row["Dispatch_Id"], row["Counter_Name"])] += float(row["Counter_Value"])
    for (k, d, c), v in per.items():
        acc[k][c].append(v)
for k, cs in sorted(acc.items()):
    print(k)
    for c, vs in sorted(cs.items()):
        print("   %-28s %14.1f  (n=%d)" % (c, sum(vs) / len(vs), len(vs)))
PY
find $OUT -name "run_counter_collection.csv" | xargs rm -f
