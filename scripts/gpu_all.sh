set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputest.log 2>&1 || { echo GPU_TEST_FAILED; tail -40 gpurun_out/gputest.log; exit 1; }
tail -3 gpurun_out/gputest.log
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bench_scan.json 2> gpurun_out/bench_scan.err || { echo BENCH_FAILED; tail -20 gpurun_out/bench_scan.err; exit 1; }
cat gpurun_out/bench_scan.json
timeout -k 10 300 python bench.py --workload highcard --segments 20 --steps 5 --warmup 1 --no-cpu-baseline --check > gpurun_out/hc_bench_part.json 2> gpurun_out/hc_bench_part.err || { echo BENCH_FAILED; tail -20 gpurun_out/hc_bench_part.err; exit 1; }
cat gpurun_out/hc_bench_part.json
