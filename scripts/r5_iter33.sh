# Round 5, thirty-third GPU iteration (a repeat of the twenty-eighth): the partitioned scatter's self-check (DevPartition::check) and re-execution --
# highcard + trim files three times with pytest -s (the library's "running the plan again" lines are kept).
set -o pipefail
mkdir -p gpurun_out/r5_iter33
export TMPDIR=/tmp
O=gpurun_out/r5_iter33
step() {  # name, timeout, command...: failing tests (rc 1) go on; a crash / timeout ends the call
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?
  echo "$name rc=$rc: $(grep -E '[0-9]+ (passed|failed)' $O/$name.log | tail -1 | cut -c1-160)"
  grep -h "running the plan again\|disagreed" $O/$name.log | head -3 | cut -c1-200
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP after $name"; exit 1; fi
}
PT="python -u -m pytest -s -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider"
step check_run1 500 $PT tests/test_gpu_groupby_highcard.py tests/test_gpu_trim.py
step check_run2 500 $PT tests/test_gpu_groupby_highcard.py tests/test_gpu_trim.py
