# End of round: every workload's bench line with its CPU baseline and roofline.traffic from
# profiles/$ROUND/pmc_index.json (profile the workloads first: scripts/final_prof.sh), copied to
# gpurun_out/final_$ROUND/ for profiles/$ROUND/final/.
#   ROUND=r06 bash scripts/final_bench.sh
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=${ROUND:-r06}
W=${WORKLOADS_BENCH:-readme scan highcard highcard-default wide-keys wide-keys-uniform inverted ssb}
BENCHES="$W" bash scripts/gpu_benches.sh || exit 1
mkdir -p gpurun_out/final_$R
for w in $W; do cp gpurun_out/${w}_bench.json gpurun_out/final_$R/; done
