# End of round: rocprofv3 kernel traces + PMC passes of the bench workloads at HEAD ($COMMIT), summarised on the box
# into gpurun_out/prof_${ROUND}_summary (profiles/summarize.py), for profiles/$ROUND/ and the bench lines'
# roofline.traffic. PART=a: the single-query workloads, every pass; PART=b: the configs[2] and SSB queries,
# FETCH_SIZE / WRITE_SIZE only.
#   ROUND=r06 COMMIT=$(git rev-parse --short HEAD) PART=a bash scripts/final_prof.sh
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=${ROUND:-r06}
if [ "${PART:-a}" = a ]; then
  ROUND=$R COMMIT=$COMMIT WORKLOADS="${WORKLOADS:-readme scan highcard hcdef widekeys}" PASSES=full bash profiles/profile.sh
else
  ROUND=$R COMMIT=$COMMIT WORKLOADS="inv0 inv1 inv2 inv3 inv4 ssb0 ssb1 ssb2 ssb3 ssb4 ssb5 ssb6 ssb7 ssb8 ssb9 ssb10 ssb11 ssb12" PASSES=traffic bash profiles/profile.sh
fi
