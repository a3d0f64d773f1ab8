set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_ssb.py tests/test_gpu_groupby_highcard.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ssb_test.log 2>&1 || { echo SSB_TEST_FAILED; tail -40 gpurun_out/ssb_test.log; exit 1; }
tail -2 gpurun_out/ssb_test.log
timeout -k 10 700 python bench.py --workload ssb --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/ssb_bench.json 2> gpurun_out/ssb_bench.err || { echo BENCH_FAILED; tail -20 gpurun_out/ssb_bench.err; exit 1; }
python - <<'PY'
import json
for l in open("gpurun_out/ssb_bench.json"):
    d = json.loads(l)
    print("%-60.60s sel %.5f value %.3e rows/s ms %.3f frac %.3f B/row %.2f %s" % (d["config"]["query"], d["config"]["selectivity"], d["value"], d["roofline"]["kernel_ms"], d["roofline"]["frac"], d["roofline"]["bytes_per_row"], d["config"]["scan_kernel"]))
PY
grep staged gpurun_out/ssb_bench.err | tail -1
