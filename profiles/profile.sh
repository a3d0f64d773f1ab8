# rocprofv3 recipe for the per-round profiles (GPU box, repo root):
#   ROUND=r04 COMMIT=<git rev> WORKLOADS="scan highcard hcdef" PASSES=full bash profiles/profile.sh
#   ROUND=r04 COMMIT=<git rev> WORKLOADS="inv0 inv1 inv2 inv3 inv4 ssb0 ... ssb12" PASSES=traffic bash profiles/profile.sh
# Per workload: a kernel trace with --stats, then separate PMC passes, each its own short run (rocprofv3
# does not split counters over passes): PASSES=traffic runs FETCH_SIZE and WRITE_SIZE only (the HBM
# traffic of the bench line's roofline), PASSES=full adds two SQ sets (instructions, waits, LDS bank
# conflicts) and the TCP->TCC request counters (atomics). One query per run (bench.py --query-index), so
# every dispatch of the run belongs to the same plan: executions per run = 2 (cold + cached plan) +
# warmup + steps. profiles/summarize.py turns gpurun_out/prof_<round>/<workload>/ into profiles/<round>/.
set -o pipefail
export TMPDIR=/tmp
ROUND=${ROUND:-r04}
OUT=gpurun_out/prof_$ROUND
mkdir -p $OUT
args_for() {
  case $1 in
    readme) echo "--workload readme --segments 1" ;;
    scan) echo "--segments 40" ;;
    highcard) echo "--workload highcard --segments 40" ;;
    hcdef) echo "--workload highcard-default --segments 40" ;;
    widekeys) echo "--workload wide-keys --segments 40" ;;
    wku) echo "--workload wide-keys-uniform --segments 40" ;;
    inv1[0-9]) echo "--workload inverted --segments 40 --query-index ${1#inv}" ;;
    inv[0-9]) echo "--workload inverted --segments 40 --query-index ${1#inv}" ;;
    ssb[0-9]|ssb1[0-2]) echo "--workload ssb --segments 20 --query-index ${1#ssb}" ;;
  esac
}
SETS_TRAFFIC=("FETCH_SIZE" "WRITE_SIZE")
SETS_FULL=("FETCH_SIZE" "WRITE_SIZE"
  "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES"
  "SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY SQ_INST_CYCLES_VMEM_WR"
  "TCP_TCC_ATOMIC_WITH_RET_REQ_sum TCP_TCC_ATOMIC_WITHOUT_RET_REQ_sum TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum")
for w in ${WORKLOADS:-scan highcard hcdef}; do
  A="$(args_for $w) --no-cpu-baseline"
  D=$OUT/$w
  mkdir -p $D
  timeout -s KILL 240 rocprofv3 --kernel-trace --stats --output-format csv -d $D/trace -o run -- python3 bench.py $A --steps 10 --warmup 2 > $D/trace_bench.json 2> $D/trace.err || { echo "$w trace failed"; tail -5 $D/trace.err; exit 1; }
  echo "$w trace done"
  if [ "${PASSES:-full}" = full ]; then SETS=("${SETS_FULL[@]}"); else SETS=("${SETS_TRAFFIC[@]}"); fi
  i=0
  for set in "${SETS[@]}"; do
    i=$((i + 1))
    timeout -s KILL 150 rocprofv3 --pmc $set --output-format csv -d $D/pmc$i -o run -- python3 bench.py $A --steps 3 --warmup 1 > $D/pmc$i.json 2> $D/pmc$i.err || { echo "$w pmc$i failed"; tail -5 $D/pmc$i.err; exit 1; }
    echo "$w pmc$i done"
  done
  # summarise this workload on the box and drop its raw traces (gpurun copies back at most 64 MiB)
  COMMIT=${COMMIT:-unknown} python3 profiles/summarize.py --one $OUT gpurun_out/prof_${ROUND}_summary $w > /dev/null || { echo "$w summary failed"; exit 1; }
  find $D -name "run_kernel_trace.csv" -o -name "run_counter_collection.csv" | xargs rm -f
done
