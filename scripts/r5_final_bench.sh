# Round 5, end of round: the wide-key profile again (its spill kernels now in the plan's kernel set), then every
# workload's bench line with its CPU baseline and roofline.traffic from profiles/r05/pmc_index.json.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
ROUND=r05 COMMIT=$COMMIT WORKLOADS="widekeys" PASSES=full bash profiles/profile.sh || exit 1
cp gpurun_out/prof_r05_summary/pmc_widekeys.json gpurun_out/prof_r05_summary/kernel_stats_widekeys.csv profiles/r05/ && python3 profiles/summarize.py --index profiles/r05 > /dev/null || exit 1
BENCHES="readme scan highcard highcard-default wide-keys inverted ssb" bash scripts/gpu_benches.sh || exit 1
mkdir -p gpurun_out/final_r05
for w in readme scan highcard highcard-default wide-keys inverted ssb; do cp gpurun_out/${w}_bench.json gpurun_out/final_r05/; done
