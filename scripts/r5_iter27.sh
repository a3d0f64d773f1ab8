# Round 5, twenty-seventh GPU iteration: every host->device upload of <= 1 MiB (segment descriptors, leaves, remaps)
# to a never-reused address (PINOT_AMD_DIAG_FRESH_UPLOADS=1) -- does the partitioned-plan mismatch need an address
# that earlier kernels read with other contents? highcard + trim files twice, then twice with the upload arena
# (PINOT_AMD_UPLOAD_ARENA=1: small uploads from a 256 MiB ring, an address back only after the ring went round).
set -o pipefail
mkdir -p gpurun_out/r5_iter27
export TMPDIR=/tmp
O=gpurun_out/r5_iter27
step() {  # name, timeout, command...: failing tests (rc 1) go on; a crash / timeout ends the call
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?
  echo "$name rc=$rc: $(tail -1 $O/$name.log | cut -c1-160)"
  grep -h "DIAG_" $O/$name.log | grep -v "unwritten 0 " | grep "parts 240\|SEGSUM" | head -3 | cut -c1-300
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP after $name"; exit 1; fi
}
PT="python -u -m pytest -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider"
export PINOT_AMD_DIAG_SCATTER=1
step fresh_run1 500 env PINOT_AMD_DIAG_FRESH_UPLOADS=1 $PT tests/test_gpu_groupby_highcard.py tests/test_gpu_trim.py
step fresh_run2 500 env PINOT_AMD_DIAG_FRESH_UPLOADS=1 $PT tests/test_gpu_groupby_highcard.py tests/test_gpu_trim.py
step arena_run1 500 env PINOT_AMD_UPLOAD_ARENA=1 $PT tests/test_gpu_groupby_highcard.py tests/test_gpu_trim.py
step arena_run2 500 env PINOT_AMD_UPLOAD_ARENA=1 $PT tests/test_gpu_groupby_highcard.py tests/test_gpu_trim.py
