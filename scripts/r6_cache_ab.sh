# Round 6: is the intermittent partitioned-plan misread tied to JIT modules loaded from the on-disk cache (the
# round-5 failures all came from the 2nd+ pytest process of a gpurun call, never from the first)? The pre-check
# build (98a21d2, worktree build/r5pre, PINOT_AMD_DIAG_SCATTER=1) over test_gpu_groupby_highcard.py +
# test_gpu_trim.py: one cold process fills a fresh cache directory, then warm processes alternate between the
# cached load as built (a probe hipModuleLoadData + hipModuleUnload, then the real load) and
# PINOT_AMD_JIT_PROBE_UNLOAD=0 (one load, nothing unloaded); AB=2: PINOT_AMD_JIT_PROBE_UNLOAD=2 (the probe module
# stays loaded: two live modules of one image, nothing unloaded) against the load as built; AB=3: kernel arguments
# in host memory (HIP_FORCE_DEV_KERNARG=0) against the load as built.
# (Recreate the worktree first: git worktree add build/r5pre 98a21d2, plus the A/B knobs of the round-6 records;
# removed at the end of round 6.)
set -o pipefail
O=$PWD/gpurun_out/r6_cache_ab
mkdir -p $O
export TMPDIR=/tmp
D=$(mktemp -d /tmp/jitcache.XXXX)
cd build/r5pre
step() {  # name, timeout, command...: failing tests (rc 1) go on; a crash / timeout ends the call
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?
  echo "$name rc=$rc: $(grep -E '[0-9]+ (passed|failed)' $O/$name.log | tail -1 | cut -c1-120) | DIAG unwritten>0 lines: $(grep -h 'DIAG_SCATTER' $O/$name.log | grep -vc 'unwritten 0 ')"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP after $name"; exit 1; fi
}
PT="python -u -m pytest -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_groupby_highcard.py tests/test_gpu_trim.py"
export PINOT_AMD_DIAG_SCATTER=1 PINOT_AMD_JIT_CACHE_DIR=$D
step p1_cold 300 $PT
ls $D | wc -l
case "${AB:-1}" in
1)  # the cached load as built vs one load
  step p2_warm_probe 300 $PT
  step p3_warm_noprobe 300 env PINOT_AMD_JIT_PROBE_UNLOAD=0 $PT
  step p4_warm_probe 300 $PT
  step p5_warm_noprobe 300 env PINOT_AMD_JIT_PROBE_UNLOAD=0 $PT ;;
2)  # the probe module loaded but never unloaded (two live modules of one image) vs the cached load as built
  step q2_warm_probe_kept 300 env PINOT_AMD_JIT_PROBE_UNLOAD=2 $PT
  step q3_warm_probe_kept 300 env PINOT_AMD_JIT_PROBE_UNLOAD=2 $PT
  step q4_warm_probe 300 $PT ;;
3)  # kernel arguments in host memory (HIP_FORCE_DEV_KERNARG=0) / dispatches serialised, with the cached load as built
  step k2_warm_probe_hostkernarg 300 env HIP_FORCE_DEV_KERNARG=0 $PT
  step k3_warm_probe_hostkernarg 300 env HIP_FORCE_DEV_KERNARG=0 $PT
  step k4_warm_probe 300 $PT ;;
esac
