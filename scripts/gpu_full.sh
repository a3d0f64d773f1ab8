set -o pipefail
bash scripts/gpu_all.sh || exit 1
timeout -k 10 300 python bench.py --workload highcard --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/hc_bench.json 2> gpurun_out/hc_bench.err || { echo BENCH_FAILED; tail -20 gpurun_out/hc_bench.err; exit 1; }
python -c "
import json; d=json.loads(open('gpurun_out/hc_bench.json').read()); print('highcard ms %.3f frac %.3f' % (d['ms_per_step'], d['roofline']['frac']))"
timeout -k 10 400 python bench.py --workload inverted --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/inv_bench.json 2> gpurun_out/inv_bench.err || { echo BENCH_FAILED; tail -20 gpurun_out/inv_bench.err; exit 1; }
python - <<'PY'
import json
for l in open("gpurun_out/inv_bench.json"):
    d = json.loads(l)
    print("inverted sel %s ms %.3f %s" % (d["config"].get("selectivity"), d["roofline"]["kernel_ms"], d["config"].get("scan_kernel")))
PY
