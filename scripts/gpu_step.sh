# Focused GPU check of the round's newest work: the trim / merge / Pinot-written tests, then bench lines
# (configs[1] with the host-time breakdown; highcard-default on the dense admission and hash trim plans).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_trim.py tests/test_gpu_server_trim.py tests/test_gpu_dist.py tests/test_gpu_pinot_written.py "tests/test_gpu_parity.py::test_group_by_raw_column" "tests/test_gpu_parity.py::test_group_by_raw_high_cardinality" "tests/test_gpu_parity.py::test_distinct_count_nan_and_signed_zero" > gpurun_out/gputest_step.log 2>&1 || { echo GPU_TEST_FAILED; tail -60 gpurun_out/gputest_step.log; exit 1; }
tail -3 gpurun_out/gputest_step.log
BENCHES="scan highcard-default" BENCH_TIMEOUT=400 STEPS=5 BENCH_ARGS=--no-cpu-baseline bash scripts/gpu_benches.sh || exit 1
cp gpurun_out/highcard-default_bench.json gpurun_out/highcard-default_admit.json
PINOT_AMD_TRIM_PLAN=hash BENCHES=highcard-default BENCH_TIMEOUT=400 STEPS=3 BENCH_ARGS=--no-cpu-baseline bash scripts/gpu_benches.sh
