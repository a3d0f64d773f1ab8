# LDS accept tables / select into the HBM table: the affected GPU tests, then SSB with and without the tables.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_groupby_highcard.py tests/test_gpu_packed_records.py tests/test_gpu_select.py -m gpu > gpurun_out/gputest_lut.log 2>&1 || { echo GPU_TEST_FAILED; tail -60 gpurun_out/gputest_lut.log; exit 1; }
tail -2 gpurun_out/gputest_lut.log
SWEEP="none PINOT_AMD_LEAF_LUT=0 PINOT_AMD_SELECT_PARTITIONED=0" ARGS="--workload ssb" bash scripts/gpu_sweep.sh || exit 1
cp gpurun_out/sweep.txt gpurun_out/sweep_ssb_lut.txt
