# One bench line per query of each workload (no CPU baseline), for before/after comparisons:
#   BENCHES="ssb scan highcard" bash scripts/gpu_benches_quick.sh
set -o pipefail
mkdir -p gpurun_out
for w in ${BENCHES:-ssb scan}; do
  timeout -k 10 300 python bench.py --workload $w --steps ${STEPS:-10} --warmup 2 --no-cpu-baseline $ARGS > gpurun_out/q_$w.json 2> gpurun_out/q_$w.err || { echo "$w failed"; tail -5 gpurun_out/q_$w.err; exit 1; }
  python - "$w" <<'PY'
import json, sys
w = sys.argv[1]
for l in open(f"gpurun_out/q_{w}.json"):
    d = json.loads(l); r = d["roofline"]
    print(w, d["config"]["scan_kernel"], "ms=%.4f" % d["ms_per_step"], "kernel_ms=%.4f" % r["kernel_ms"], "frac=%.3f" % r["frac"])
PY
done
