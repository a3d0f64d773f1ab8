# Round 5, sixteenth GPU iteration: the partitioned-plan mismatch of iteration 15
# (test_gpu_trim.py::test_int_sums_narrow_lds_partials[1]) -- repeated executions against the oracle under
# the scatter / pool knobs, the test alone, then the grouped-flush sweep of iteration 15.
set -o pipefail
mkdir -p gpurun_out/r5_iter16
export TMPDIR=/tmp
O=gpurun_out/r5_iter16
step() {  # name, timeout, command...: wrong results (rc 1) go on; a crash / timeout ends the call
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?
  echo "$name rc=$rc: $(grep -h SUMMARY $O/$name.log | tail -1)$(tail -1 $O/$name.log | cut -c1-160)"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP after $name"; exit 1; fi
}
step default 300 python -u scripts/repro_part_race.py 15
step flushpar0 300 python -u scripts/repro_part_race.py 15 PINOT_AMD_FLUSH_PAR=0
step batch0 300 python -u scripts/repro_part_race.py 15 PINOT_AMD_SCATTER_BATCH=0
step stage0 300 python -u scripts/repro_part_race.py 15 PINOT_AMD_STAGE_CAP=0
step pool0 300 env PINOT_AMD_POOL_BYTES=0 python -u scripts/repro_part_race.py 15
step trim_alone 400 python -u -m pytest tests/test_gpu_trim.py -m gpu -q -x --timeout 300 --timeout-method thread
step hc_trim 600 python -u -m pytest tests/test_gpu_groupby_highcard.py tests/test_gpu_trim.py -m gpu -q --timeout 300 --timeout-method thread
SWEEP="none PINOT_AMD_FLUSH_GROUP=1 none PINOT_AMD_FLUSH_GROUP=1" ARGS="--workload highcard --segments 40" STEPS=10 timeout -k 10 600 bash scripts/gpu_sweep.sh || exit 1
cp gpurun_out/sweep.txt gpurun_out/r5_sweep_hc_flushgroup.txt
SWEEP="none PINOT_AMD_FLUSH_GROUP=1" ARGS="--workload highcard-default --segments 40" STEPS=10 timeout -k 10 600 bash scripts/gpu_sweep.sh || exit 1
cp gpurun_out/sweep.txt gpurun_out/r5_sweep_hcdef_flushgroup.txt
