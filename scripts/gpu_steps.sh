# One GPU call's worth of steps, each under its own time limit, logs in gpurun_out/$TAG/<name>.log: the recipe every
# per-round iteration script was an instance of (round 5's r5_iter*.sh, folded into this; git show 0cba8cb:scripts/
# recovers any of them). STEPS holds one step per line, "name|seconds|command" (env assignments go in the command,
# e.g. "env PINOT_AMD_SAMPLE_STRIDE=2 python -m pytest ..."). A failing test (rc 1) goes on; a crash, abort or time
# limit ends the call. PYTEST expands to the GPU test runner's usual flags. The pytest session's self-check failure
# count and the result line are echoed per step.
#   TAG=r6_verify STEPS='hc_trim|400|$PYTEST tests/test_gpu_groupby_highcard.py tests/test_gpu_trim.py' bash scripts/gpu_steps.sh
set -o pipefail
O=$PWD/gpurun_out/${TAG:-steps}
mkdir -p $O
export TMPDIR=/tmp
[ -n "$FRESH_JIT_CACHE" ] && export PINOT_AMD_JIT_CACHE_DIR=$(mktemp -d /tmp/jitcache.XXXX)
PYTEST="python -u -m pytest -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider"
while IFS='|' read -r name t cmd; do
  [ -z "$name" ] && continue
  cmd=${cmd//\$PYTEST/$PYTEST}
  timeout -k 10 "$t" bash -c "$cmd" > "$O/$name.log" 2>&1; rc=$?
  echo "$name rc=$rc: $(grep -E '[0-9]+ (passed|failed)' "$O/$name.log" | tail -1 | cut -c1-120) $(grep -h 'self-check failures in this session' "$O/$name.log" | tail -1)"
  grep -h -A4 "^pinot_amd: partitioned plan self-check" "$O/$name.log" | head -8
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP after $name"; exit 1; fi
done <<< "$STEPS"
