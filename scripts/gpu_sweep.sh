# Knob sweeps on one box (env knobs of the planner), one bench line per setting:
# (Experiment knobs outside host.cpp's knob() list are read only by a diagnostics build: PINOT_AMD_BUILD_DIAGNOSTICS=1
# python -m pinot_amd.build; the kept planner overrides work in every build.)
#   SWEEP="PINOT_AMD_PREFETCH=2 PINOT_AMD_PREFETCH=8" ARGS="--workload ssb --query-index 11" bash scripts/gpu_sweep.sh
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/sweep.txt
: > $out
for kv in ${SWEEP:-none}; do
  if [ "$kv" = none ]; then envset=""; else envset="${kv//,/ }"; fi  # A=1,B=2: several variables
  env $envset timeout -k 10 300 python bench.py $ARGS --steps ${STEPS:-10} --warmup 2 --no-cpu-baseline > gpurun_out/sweep_one.json 2> gpurun_out/sweep_one.err || { echo "$kv FAILED"; tail -5 gpurun_out/sweep_one.err; exit 1; }
  python -c "
import json
for l in open('gpurun_out/sweep_one.json'):
    d = json.loads(l); r = d['roofline']
    print('$kv', d['config']['scan_kernel'], 'ms=%.4f' % d['ms_per_step'], 'kernel_ms=%.4f' % r['kernel_ms'], 'frac=%.3f' % r['frac'])
" | tee -a $out
done
