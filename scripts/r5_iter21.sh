# Round 5, twenty-first GPU iteration (the unwritten-record check after the aggregation pass, and the count pass re-run): the partitioned-plan mismatch with the scatter diagnostic
# (PINOT_AMD_DIAG_SCATTER=1: unwritten records reported per launch to stderr), highcard + trim files, twice.
set -o pipefail
mkdir -p gpurun_out/r5_iter21
export TMPDIR=/tmp
O=gpurun_out/r5_iter21
step() {  # name, timeout, command...: failing tests (rc 1) go on; a crash / timeout ends the call
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?
  echo "$name rc=$rc: $(tail -1 $O/$name.log | cut -c1-160)"
  grep -h "DIAG_" $O/$name.log | grep -v "unwritten 0 \|differing 0$" | head -5 | cut -c1-600
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP after $name"; exit 1; fi
}
PT="python -u -m pytest -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider"
export PINOT_AMD_DIAG_SCATTER=1
step run1 500 $PT tests/test_gpu_groupby_highcard.py tests/test_gpu_trim.py
step run2 500 $PT tests/test_gpu_groupby_highcard.py tests/test_gpu_trim.py
step run3 500 $PT tests/test_gpu_groupby_highcard.py tests/test_gpu_trim.py
