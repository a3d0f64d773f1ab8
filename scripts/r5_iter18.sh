# Round 5, eighteenth GPU iteration: test_int_sums_narrow_lds_partials after the highcard file and the trim file's
# earlier tests (iterations 15 / 16 failed that way), with the device block pool on and off, the leaf cache off.
set -o pipefail
mkdir -p gpurun_out/r5_iter18
export TMPDIR=/tmp
O=gpurun_out/r5_iter18
step() {  # name, timeout, command...: failing tests (rc 1) go on; a crash / timeout ends the call
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?
  echo "$name rc=$rc: $(tail -1 $O/$name.log | cut -c1-160)"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP after $name"; exit 1; fi
}
PT="python -u -m pytest -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider"
step hc_trim 500 $PT tests/test_gpu_groupby_highcard.py tests/test_gpu_trim.py
step hc_trim_pool0 500 env PINOT_AMD_POOL_BYTES=0 $PT tests/test_gpu_groupby_highcard.py tests/test_gpu_trim.py
step trim_trim 400 $PT tests/test_gpu_trim.py tests/test_gpu_trim.py
