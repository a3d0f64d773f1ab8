set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_inverted.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/inv_test.log 2>&1 || { echo INV_TEST_FAILED; tail -40 gpurun_out/inv_test.log; exit 1; }
tail -2 gpurun_out/inv_test.log
timeout -k 10 600 python bench.py --workload inverted --segments 100 --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/inv_bench.json 2> gpurun_out/inv_bench.err || { echo BENCH_FAILED; tail -20 gpurun_out/inv_bench.err; exit 1; }
python - <<'PY'
import json
for l in open("gpurun_out/inv_bench.json"):
    d = json.loads(l)
    print("sel %.5f value %.3e rows/s kernel_ms %.3f frac %.3f %s" % (d["config"]["selectivity"], d["value"], d["roofline"]["kernel_ms"], d["roofline"]["frac"], d["config"]["scan_kernel"]))
PY
