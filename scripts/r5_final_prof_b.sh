# end of round, part b: the configs[2] and SSB queries (traffic passes)
PART=b COMMIT=2edbc5d bash scripts/r5_final_prof.sh
