# Round 6: the self-check tests, then the round-5 failing sequence (test_gpu_groupby_highcard.py + test_gpu_trim.py)
# with the hard self-check, its forensic report (blocks' placement, the columns' bytes against their staging
# fingerprints, the count pass run again) and the session-level failure count; no JIT module is unloaded.
set -o pipefail
O=$PWD/gpurun_out/r6_verify
mkdir -p $O
export TMPDIR=/tmp
export PINOT_AMD_JIT_CACHE_DIR=$(mktemp -d /tmp/jitcache.XXXX)
step() {  # name, timeout, command...: failing tests (rc 1) go on; a crash / timeout ends the call
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?
  echo "$name rc=$rc: $(grep -E '[0-9]+ (passed|failed)' $O/$name.log | tail -1 | cut -c1-120) | $(grep -h 'self-check failures in this session' $O/$name.log | tail -1)"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP after $name"; exit 1; fi
}
PT="python -u -m pytest -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider"
step selfcheck 400 $PT tests/test_gpu_selfcheck.py
step hc_trim_1 400 $PT tests/test_gpu_groupby_highcard.py tests/test_gpu_trim.py
step hc_trim_2 400 $PT tests/test_gpu_groupby_highcard.py tests/test_gpu_trim.py
step hc_trim_3 400 $PT tests/test_gpu_groupby_highcard.py tests/test_gpu_trim.py
