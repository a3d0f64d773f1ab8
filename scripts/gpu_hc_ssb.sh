set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_groupby_highcard.py tests/test_gpu_ssb.py -x -q --timeout 120 --timeout-method thread > gpurun_out/gputest.log 2>&1 || { echo GPU_TEST_FAILED; tail -40 gpurun_out/gputest.log; exit 1; }
tail -2 gpurun_out/gputest.log
timeout -k 10 700 python bench.py --workload ssb --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/ssb_bench.json 2> gpurun_out/ssb_bench.err || { echo BENCH_FAILED; tail -20 gpurun_out/ssb_bench.err; exit 1; }
python - <<'PY'
import json
for l in open("gpurun_out/ssb_bench.json"):
    d = json.loads(l)
    print("%-50.50s sel %.5f %.3e rows/s ms %.3f frac %.3f %s" % (d["config"]["query"], d["config"]["selectivity"], d["value"], d["roofline"]["kernel_ms"], d["roofline"]["frac"], d["config"]["scan_kernel"]))
PY
timeout -k 10 300 python bench.py --workload highcard --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/hc_bench.json 2> gpurun_out/hc_bench.err || { echo BENCH_FAILED; tail -20 gpurun_out/hc_bench.err; exit 1; }
python -c "
import json; d=json.loads(open('gpurun_out/hc_bench.json').read()); print('highcard', d['value'], d['ms_per_step'], d['roofline'])"
