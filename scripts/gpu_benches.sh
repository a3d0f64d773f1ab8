set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --workload highcard --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/hc_bench.json 2> gpurun_out/hc_bench.err || { echo HC_FAILED; tail -5 gpurun_out/hc_bench.err; exit 1; }
timeout -k 10 600 python bench.py --workload inverted --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/inv_bench.json 2> gpurun_out/inv_bench.err || { echo INV_FAILED; tail -5 gpurun_out/inv_bench.err; exit 1; }
python - <<'PY'
import json
for f in ["gpurun_out/hc_bench.json", "gpurun_out/inv_bench.json"]:
    for l in open(f):
        d = json.loads(l)
        print("%-10s sel %.5f %.3e rows/s ms %.3f frac %.3f B/row %.2f %s" % (f.split('/')[1][:8], d["config"]["selectivity"], d["value"], d["roofline"]["kernel_ms"], d["roofline"]["frac"], d["roofline"]["bytes_per_row"], d["config"]["scan_kernel"]))
PY
