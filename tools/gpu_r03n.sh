set -o pipefail
# PMC passes for cfg5's pair: DCS (dcs_round_kernel, Halley root) and MHRS (mhrs_search rounds)
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r03n; mkdir -p $O; cd $R
bash tools/prof_pmc.sh r03dcs --method DCS --n 15 --N 500000 --censor 0.3 --steps 3 || exit 1
PMC_KERNEL=dcs_round_kernel python3 tools/pmc_summary.py $R/gpurun_out/pmc_r03dcs $O/pmc_dcs.json > $O/pmc_dcs.out 2>&1 || { tail $O/pmc_dcs.out; exit 1; }
bash tools/prof_pmc.sh r03mhrs --method MHRS --n 15 --N 500000 --censor 0.3 --steps 3 || exit 1
PMC_KERNEL=mhrs_search python3 tools/pmc_summary.py $R/gpurun_out/pmc_r03mhrs $O/pmc_mhrs.json > $O/pmc_mhrs.out 2>&1 || { tail $O/pmc_mhrs.out; exit 1; }
head -12 $O/pmc_dcs.out; head -12 $O/pmc_mhrs.out
