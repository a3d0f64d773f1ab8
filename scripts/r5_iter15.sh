# Round 5, fifteenth GPU iteration: the grouped scatter flush for 16-byte records -- parity, then configs[3]
# untrimmed and at the default limit with / without it (interleaved, 40 segments).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_groupby_highcard.py tests/test_gpu_trim.py tests/test_gpu_inverted.py tests/test_gpu_ssb.py -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/r5_gputest15.log 2>&1 || { echo GPU_TEST_FAILED; tail -60 gpurun_out/r5_gputest15.log; exit 1; }
tail -2 gpurun_out/r5_gputest15.log
SWEEP="none PINOT_AMD_FLUSH_GROUP=1 none PINOT_AMD_FLUSH_GROUP=1" ARGS="--workload highcard --segments 40" STEPS=10 timeout -k 10 600 bash scripts/gpu_sweep.sh || exit 1
cp gpurun_out/sweep.txt gpurun_out/r5_sweep_hc_flushgroup.txt
SWEEP="none PINOT_AMD_FLUSH_GROUP=1" ARGS="--workload highcard-default --segments 40" STEPS=10 timeout -k 10 600 bash scripts/gpu_sweep.sh || exit 1
cp gpurun_out/sweep.txt gpurun_out/r5_sweep_hcdef_flushgroup.txt
mkdir -p gpurun_out/r5_plan15
for w in scan ssb; do
  timeout -k 10 300 python bench.py --workload $w --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r5_plan15/$w.json 2> gpurun_out/r5_plan15/$w.err || { echo "$w FAILED"; tail -5 gpurun_out/r5_plan15/$w.err; exit 1; }
done
python scripts/plan_summary.py gpurun_out/r5_plan15/*.json | cut -c1-260
