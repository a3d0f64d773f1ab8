# rocprofv3 recipe for the round-3 profiles (GPU box, repo root):
#   WORKLOADS="scan highcard hcdef" bash profiles/profile_r03.sh      # then: inv0 inv2 ssb10 ssb11 ssb7
# Per workload: a kernel trace with --stats, then separate PMC passes (FETCH_SIZE; WRITE_SIZE; two SQ
# sets; TCP atomics), each its own short run. One query per run (bench.py --query-index), so every
# dispatch of the run belongs to the same plan: executions per run = 2 (cold + cached plan) + warmup +
# steps. profiles/summarize_r03.py turns gpurun_out/prof3/<workload>/ into profiles/r03/.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/prof3
mkdir -p $OUT
args_for() {
  case $1 in
    scan) echo "--segments 40" ;;
    highcard) echo "--workload highcard --segments 40" ;;
    hcdef) echo "--workload highcard-default --segments 40" ;;
    inv0) echo "--workload inverted --segments 40 --query-index 0" ;;
    inv2) echo "--workload inverted --segments 40 --query-index 2" ;;
    ssb10) echo "--workload ssb --segments 20 --query-index 10" ;;
    ssb11) echo "--workload ssb --segments 20 --query-index 11" ;;
    ssb7) echo "--workload ssb --segments 20 --query-index 7" ;;
  esac
}
for w in ${WORKLOADS:-scan highcard hcdef inv0 inv2 ssb10 ssb11}; do
  A="$(args_for $w) --no-cpu-baseline"
  D=$OUT/$w
  mkdir -p $D
  timeout -s KILL 240 rocprofv3 --kernel-trace --stats --output-format csv -d $D/trace -o run -- python3 bench.py $A --steps 10 --warmup 2 > $D/trace_bench.json 2> $D/trace.err || { echo "$w trace failed"; tail -5 $D/trace.err; exit 1; }
  echo "$w trace done"
  i=0
  for set in "FETCH_SIZE" "WRITE_SIZE" \
      "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES" \
      "SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY SQ_INST_CYCLES_VMEM_WR" \
      "TCP_TCC_ATOMIC_WITH_RET_REQ_sum TCP_TCC_ATOMIC_WITHOUT_RET_REQ_sum TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum"; do
    i=$((i + 1))
    timeout -s KILL 150 rocprofv3 --pmc $set --output-format csv -d $D/pmc$i -o run -- python3 bench.py $A --steps 3 --warmup 1 > $D/pmc$i.json 2> $D/pmc$i.err || { echo "$w pmc$i failed"; tail -5 $D/pmc$i.err; exit 1; }
    echo "$w pmc$i done"
  done
done
# summarise on the box and drop the raw traces (gpurun copies back at most 64 MiB)
python3 profiles/summarize_r03.py $OUT gpurun_out/prof3_summary > /dev/null && \
  find $OUT -name "run_kernel_trace.csv" -o -name "run_counter_collection.csv" | xargs rm -f
