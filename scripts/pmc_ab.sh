# A/B PMC passes: for each case (label, env settings, bench args) one short bench run per counter set
# (rocprofv3 does not split counters over passes), then per-kernel means per dispatch for every case.
#   CASES="base||--workload highcard-default --segments 40;off|PINOT_AMD_DIAG_ADMIT_OFF=1|--workload highcard-default --segments 40" \
#   SETS="FETCH_SIZE;WRITE_SIZE;TCC_HIT_sum TCC_MISS_sum" bash scripts/pmc_ab.sh > gpurun_out/ab.txt
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/pmcab
rm -rf $OUT; mkdir -p $OUT
IFS=';' read -ra CS <<< "$CASES"
IFS=';' read -ra PASSES <<< "${SETS:-FETCH_SIZE;WRITE_SIZE}"
for c in "${CS[@]}"; do
  IFS='|' read -r label envs args <<< "$c"
  i=0
  for set in "${PASSES[@]}"; do
    i=$((i + 1))
    D=$OUT/$label/p$i
    mkdir -p $D
    # (env settings exported in a subshell: rocprofv3 must start the program itself, no env / sh hop)
    ( for kv in ${envs//,/ }; do export "$kv"; done
      timeout -s KILL 150 rocprofv3 --pmc $set --output-format csv -d $D -o run -- python3 bench.py $args --steps 3 --warmup 1 --no-cpu-baseline > $D.json 2> $D.err ) || { echo "$label pass $i failed"; tail -5 $D.err; exit 1; }
  done
  echo "$label done" >&2
done
python3 - <<'PY'
import csv, glob, collections, os
root = "gpurun_out/pmcab"
for label in sorted(os.listdir(root)):
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(f"{root}/{label}/p*/**/run_counter_collection.csv", recursive=True):
        per = collections.defaultdict(float)
        for row in csv.DictReader(open(f)):
            k = row["Kernel_Name"]
            if "pinot_" not in k and "kernel" not in k:
                continue
            per[(k, row["Dispatch_Id"], row["Counter_Name"])] += float(row["Counter_Value"])
        for (k, d, c), v in per.items():
            acc[k][c].append(v)
    print("==", label)
    for k, cs in sorted(acc.items()):
        print("  " + k[:90])
        for c, vs in sorted(cs.items()):
            print("     %-26s %16.1f  (n=%d)" % (c, sum(vs) / len(vs), len(vs)))
PY
find $OUT -name "run_counter_collection.csv" | xargs rm -f
