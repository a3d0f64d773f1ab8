set -o pipefail
mkdir -p gpurun_out/prof_hc
export TMPDIR=/tmp
W=/tmp/pmchc
run() {  # name counters...
  n=$1; shift
  rm -rf $W
  timeout -s KILL 150 rocprofv3 --pmc "$@" --output-format csv -d $W -o run -- python3 bench.py --workload highcard --segments 20 --steps 2 --warmup 1 --no-cpu-baseline > /dev/null 2> gpurun_out/prof_hc/$n.err || exit 1
  f=$(find $W -name "*counter_collection.csv" | head -1)
  { head -1 "$f"; grep "pinot" "$f" || true; } > gpurun_out/prof_hc/$n.csv
}
run a SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES
run b SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY SQ_INST_CYCLES_VMEM_WR
run c FETCH_SIZE
run d WRITE_SIZE
echo done
