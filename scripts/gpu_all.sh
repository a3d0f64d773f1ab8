set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputest.log 2>&1 || { echo GPU_TEST_FAILED; tail -40 gpurun_out/gputest.log; exit 1; }
tail -2 gpurun_out/gputest.log
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bench_scan.json 2> gpurun_out/bench_scan.err || { echo BENCH_FAILED; tail -20 gpurun_out/bench_scan.err; exit 1; }
python - <<'PY'
import json
d = json.loads(open("gpurun_out/bench_scan.json").read())
print("scan: %.4g rows/s kernel %.3f ms frac %.3f" % (d["value"], d["roofline"]["kernel_ms"], d["roofline"]["frac"]))
PY
timeout -k 10 700 python bench.py --workload ssb --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/ssb_bench.json 2> gpurun_out/ssb_bench.err || { echo BENCH_FAILED; tail -20 gpurun_out/ssb_bench.err; exit 1; }
python - <<'PY'
import json
for l in open("gpurun_out/ssb_bench.json"):
    d = json.loads(l)
    print("%-50.50s sel %.5f %.3e rows/s ms %.3f frac %.3f %s" % (d["config"]["query"], d["config"]["selectivity"], d["value"], d["roofline"]["kernel_ms"], d["roofline"]["frac"], d["config"]["scan_kernel"]))
PY
