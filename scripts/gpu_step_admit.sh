# Admission check: the trim tests over every admission path, then highcard-default on the sequential
# admission and on the first-doc admission, then a kernel-trace summary of the sequential one.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_trim.py > gpurun_out/gputest_admit.log 2>&1 || { echo GPU_TEST_FAILED; tail -60 gpurun_out/gputest_admit.log; exit 1; }
tail -3 gpurun_out/gputest_admit.log
BENCHES="highcard-default" BENCH_TIMEOUT=400 STEPS=5 BENCH_ARGS=--no-cpu-baseline bash scripts/gpu_benches.sh || exit 1
cp gpurun_out/highcard-default_bench.json gpurun_out/highcard-default_seq.json
PINOT_AMD_ADMIT_SEQ=0 BENCHES="highcard-default" BENCH_TIMEOUT=400 STEPS=5 BENCH_ARGS=--no-cpu-baseline bash scripts/gpu_benches.sh || exit 1
cp gpurun_out/highcard-default_bench.json gpurun_out/highcard-default_firstdoc.json
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_admit -o run -- python bench.py --workload highcard-default --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/prof_admit.log 2>&1 || { echo PROF_FAILED; tail -20 gpurun_out/prof_admit.log; exit 1; }
find gpurun_out/prof_admit -name "*kernel_stats.csv" -exec cat {} \; | cut -c1-200 | head -20
echo EXIT 0
