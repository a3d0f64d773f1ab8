# Round 5, twenty-third GPU iteration: device-wide cache invalidation before kernels that read host-copied bytes
# (uploads_visible / launch_cache_invalidate) against the partitioned-plan mismatch -- highcard + trim files three
# times with it (scatter diagnostic on), then once with PINOT_AMD_CACHE_INV=0 as the control.
set -o pipefail
mkdir -p gpurun_out/r5_iter23
export TMPDIR=/tmp
O=gpurun_out/r5_iter23
step() {  # name, timeout, command...: failing tests (rc 1) go on; a crash / timeout ends the call
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?
  echo "$name rc=$rc: $(tail -1 $O/$name.log | cut -c1-160)"
  grep -h "DIAG_" $O/$name.log | grep -v "unwritten 0 " | head -3 | cut -c1-400
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP after $name"; exit 1; fi
}
PT="python -u -m pytest -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider"
export PINOT_AMD_DIAG_SCATTER=1
step inv_run1 500 $PT tests/test_gpu_groupby_highcard.py tests/test_gpu_trim.py
step inv_run2 500 $PT tests/test_gpu_groupby_highcard.py tests/test_gpu_trim.py
step inv_run3 500 $PT tests/test_gpu_groupby_highcard.py tests/test_gpu_trim.py
step control_noinv 500 env PINOT_AMD_CACHE_INV=0 $PT tests/test_gpu_groupby_highcard.py tests/test_gpu_trim.py
