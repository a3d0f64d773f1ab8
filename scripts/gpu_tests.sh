# GPU test suite (stops at the first failure) then the default bench line.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo SMOKE_FAILED; tail -30 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --maxfail=15 --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/gputest.log 2>&1 || { echo GPU_TEST_FAILED; tail -60 gpurun_out/gputest.log; exit 1; }
tail -3 gpurun_out/gputest.log
timeout -k 10 400 python bench.py --no-cpu-baseline > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || { echo BENCH_FAILED; tail -20 gpurun_out/bench_default.err; exit 1; }
cat gpurun_out/bench_default.json
