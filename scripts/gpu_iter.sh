# Iteration check: the GPU tests named in $TESTS (default: the whole -m gpu suite), then the default
# bench line and the inverted-index sweep.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest ${TESTS:-tests} -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gputest.log 2>&1 || { echo GPU_TEST_FAILED; tail -60 gpurun_out/gputest.log; exit 1; }
tail -3 gpurun_out/gputest.log
timeout -k 10 400 python bench.py --no-cpu-baseline --steps 10 > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || { echo BENCH_FAILED; tail -20 gpurun_out/bench_default.err; exit 1; }
cat gpurun_out/bench_default.json
if [ -n "$INV" ]; then
timeout -k 10 400 python bench.py --no-cpu-baseline --workload inverted --steps 5 > gpurun_out/inv_bench.json 2> gpurun_out/inv_bench.err || { echo INV_FAILED; tail -20 gpurun_out/inv_bench.err; exit 1; }
python -c "
import json
for l in open('gpurun_out/inv_bench.json'):
    d=json.loads(l); r=d['roofline']; print(round(d['config']['selectivity'],5), round(d['ms_per_step'],3), r['bytes_per_row'], round(r['frac'],3), d['cold_ms'], d['cached_plan_ms'])
"
fi
