set -o pipefail
mkdir -p gpurun_out/prof_ssb
export TMPDIR=/tmp
W=/tmp/pmcwork
for qi in ${QIS:-0 3}; do
rm -rf $W
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SMEM SQ_BUSY_CYCLES SQ_WAVE_CYCLES --output-format csv -d $W/a -o run -- python3 bench.py --workload ssb --query-index $qi --segments 20 --steps 2 --warmup 1 --no-cpu-baseline > /dev/null 2> gpurun_out/prof_ssb/pmc_q$qi.err || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM_RD SQ_WAIT_ANY SQ_ACTIVE_INST_SCA --output-format csv -d $W/b -o run -- python3 bench.py --workload ssb --query-index $qi --segments 20 --steps 2 --warmup 1 --no-cpu-baseline > /dev/null 2> gpurun_out/prof_ssb/pmcb_q$qi.err || exit 1
for p in a b; do
  f=$(find $W/$p -name "*counter_collection.csv" | head -1)
  { head -1 "$f"; grep "pinot" "$f" || true; } > gpurun_out/prof_ssb/pmc${p}_q$qi.csv
done
done
echo done
