# Round 5, twenty-fifth GPU iteration: the round-4 build (commit 15fb2d6, staged under gpurun_r4/, git-ignored) through
# the same highcard + trim sequence three times -- does the partitioned-plan mismatch predate round 5?
set -o pipefail
mkdir -p gpurun_out/r5_iter25
export TMPDIR=/tmp
O=$PWD/gpurun_out/r5_iter25
step() {  # name, timeout, command...: failing tests (rc 1) go on; a crash / timeout ends the call
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?
  echo "$name rc=$rc: $(tail -1 $O/$name.log | cut -c1-160)"
  grep -h "^E  .*AssertionError\|^FAILED" $O/$name.log | head -3 | cut -c1-300
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP after $name"; exit 1; fi
}
cd gpurun_r4
PT="python -u -m pytest -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider"
step r4_run1 500 $PT tests/test_gpu_groupby_highcard.py tests/test_gpu_trim.py
step r4_run2 500 $PT tests/test_gpu_groupby_highcard.py tests/test_gpu_trim.py
step r4_run3 500 $PT tests/test_gpu_groupby_highcard.py tests/test_gpu_trim.py
