# Round 5, twelfth GPU iteration: what bounds the wide-key scan (19.8 ms per 1B rows) -- per-dispatch counters
# of pinot_scan_jit and a knob sweep at 40 segments.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
K=pinot_scan_jit SETS="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT;SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VMEM SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU" ARGS="--workload wide-keys --segments 40" timeout -k 10 400 bash scripts/pmc_dispatch.sh > gpurun_out/r5_pmcd_wk.txt 2>&1 || { echo PMC_FAILED; tail -20 gpurun_out/r5_pmcd_wk.txt; exit 1; }
cat gpurun_out/r5_pmcd_wk.txt | cut -c1-400
SWEEP="none PINOT_AMD_HASH_LDS_SLOTS=2048 PINOT_AMD_HASH_LDS_SLOTS=1024 PINOT_AMD_PREFETCH=2 PINOT_AMD_HASH_SPILL=0" ARGS="--workload wide-keys --segments 40" STEPS=5 timeout -k 10 600 bash scripts/gpu_sweep.sh || exit 1
cp gpurun_out/sweep.txt gpurun_out/r5_sweep_wk_knobs.txt
