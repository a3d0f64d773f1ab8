# Selection-vector profiles: the generated sources of SSB Q4.2 and configs[2] at 1 % (for offline ISA
# counts), then profile part 2 of the round-3 recipe (inv0 inv2 ssb10 ssb11).
set -o pipefail
mkdir -p gpurun_out/jit_q42 gpurun_out/jit_inv2
PINOT_AMD_JIT_DUMP=gpurun_out/jit_q42 timeout -k 10 200 python bench.py --workload ssb --segments 4 --query-index 11 --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/jit_q42/bench.json 2> gpurun_out/jit_q42/bench.err || { echo DUMP_FAILED; tail -20 gpurun_out/jit_q42/bench.err; exit 1; }
PINOT_AMD_JIT_DUMP=gpurun_out/jit_inv2 timeout -k 10 200 python bench.py --workload inverted --segments 4 --query-index 2 --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/jit_inv2/bench.json 2> gpurun_out/jit_inv2/bench.err || { echo DUMP_FAILED; tail -20 gpurun_out/jit_inv2/bench.err; exit 1; }
WORKLOADS="inv0 inv2 ssb10 ssb11" bash profiles/profile_r03.sh
