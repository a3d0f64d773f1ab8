set -o pipefail
mkdir -p gpurun_out/prof_ssb
export TMPDIR=/tmp
for qi in 0 7; do
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES --output-format csv -d gpurun_out/prof_ssb/pmc_q$qi -o run -- python3 bench.py --workload ssb --query-index $qi --segments 20 --steps 2 --warmup 1 --no-cpu-baseline > /dev/null 2> gpurun_out/prof_ssb/pmc_q$qi.err || exit 1
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_ssb/trace_q$qi -o run -- python3 bench.py --workload ssb --query-index $qi --segments 20 --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/prof_ssb/bench_q$qi.json 2> gpurun_out/prof_ssb/trace_q$qi.err || exit 1
done
echo done
