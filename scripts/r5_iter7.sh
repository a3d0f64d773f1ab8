# Round 5, seventh GPU iteration: counters for the wide-key hash plan's kernels (scan with the LDS first level,
# spill scatter, spill aggregation) at 40 x 10M rows, and for SSB Q4.2's select pass (waves per SIMD).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
SQ="SQ_WAVES SQ_BUSY_CU_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM"
SETS="FETCH_SIZE;WRITE_SIZE TCC_HIT_sum TCC_MISS_sum;$SQ" ARGS="--workload wide-keys --segments 40" timeout -k 10 600 bash scripts/pmc_custom.sh > gpurun_out/r5_pmc_wk.txt 2>&1 || { echo PMC_WK_FAILED; tail -20 gpurun_out/r5_pmc_wk.txt; exit 1; }
cat gpurun_out/r5_pmc_wk.txt
SETS="$SQ;SQ_INSTS_SALU SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA;FETCH_SIZE" ARGS="--workload ssb --segments 20 --query-index 11" timeout -k 10 600 bash scripts/pmc_custom.sh > gpurun_out/r5_pmc_q42.txt 2>&1 || { echo PMC_Q42_FAILED; tail -20 gpurun_out/r5_pmc_q42.txt; exit 1; }
cat gpurun_out/r5_pmc_q42.txt
SETS="$SQ;SQ_INSTS_SALU SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA" ARGS="--workload highcard --segments 40" timeout -k 10 600 bash scripts/pmc_custom.sh > gpurun_out/r5_pmc_hc.txt 2>&1 || { echo PMC_HC_FAILED; tail -20 gpurun_out/r5_pmc_hc.txt; exit 1; }
cat gpurun_out/r5_pmc_hc.txt
SETS="TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum" ARGS="--workload wide-keys --segments 40" timeout -k 10 300 bash scripts/pmc_custom.sh > gpurun_out/r5_pmc_wk_wrreq.txt 2>&1 || { echo PMC_WRREQ_FAILED; tail -5 gpurun_out/r5_pmc_wk_wrreq.txt; exit 1; }
cat gpurun_out/r5_pmc_wk_wrreq.txt
