# Round 5, end of round: rocprofv3 kernel traces + PMC passes of every bench workload at HEAD ($COMMIT), summarised
# on the box into gpurun_out/prof_r05_summary (profiles/summarize.py), for profiles/r05/ and the bench lines'
# roofline.traffic. PART=a: the five single-query workloads, every pass; PART=b: the configs[2] and SSB queries,
# FETCH_SIZE / WRITE_SIZE only.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ "${PART:-a}" = a ]; then
  ROUND=r05 COMMIT=$COMMIT WORKLOADS="readme scan highcard hcdef widekeys" PASSES=full bash profiles/profile.sh
else
  ROUND=r05 COMMIT=$COMMIT WORKLOADS="inv0 inv1 inv2 inv3 inv4 ssb0 ssb1 ssb2 ssb3 ssb4 ssb5 ssb6 ssb7 ssb8 ssb9 ssb10 ssb11 ssb12" PASSES=traffic bash profiles/profile.sh
fi
