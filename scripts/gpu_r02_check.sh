# Round-2 first GPU check: full GPU test suite + default bench line (with CPU baseline).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputest.log 2>&1 || { echo GPU_TEST_FAILED; tail -40 gpurun_out/gputest.log; exit 1; }
tail -2 gpurun_out/gputest.log
timeout -k 10 400 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || { echo BENCH_FAILED; tail -20 gpurun_out/bench_default.err; exit 1; }
cat gpurun_out/bench_default.json
