# Round 5, seventeenth GPU iteration: which earlier tests make test_int_sums_narrow_lds_partials fail (iteration 16:
# it passes alone, fails after tests/test_gpu_groupby_highcard.py), and whether the device block pool is involved.
set -o pipefail
mkdir -p gpurun_out/r5_iter17
export TMPDIR=/tmp
O=gpurun_out/r5_iter17
T=tests/test_gpu_trim.py::test_int_sums_narrow_lds_partials
step() {  # name, timeout, command...: failing tests (rc 1) go on; a crash / timeout ends the call
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?
  echo "$name rc=$rc: $(grep -h SUMMARY $O/$name.log | tail -1)$(tail -1 $O/$name.log | cut -c1-160)"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP after $name"; exit 1; fi
}
PT="python -u -m pytest -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider"
step flushvar_then 400 $PT tests/test_gpu_groupby_highcard.py::test_highcard_flush_variants $T
step others_then 500 $PT tests/test_gpu_groupby_highcard.py -k "not flush_variants" $T
step pool0_all_then 500 env PINOT_AMD_POOL_BYTES=0 $PT tests/test_gpu_groupby_highcard.py $T
step repro_fresh 200 python -u scripts/repro_part_race.py 5
