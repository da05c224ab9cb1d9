set -o pipefail
# PMC of cfg5 ECS: the censored-range kernel (private ARMS envelope) and the exact-range kernel
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r03q; mkdir -p $O; cd $R
bash tools/prof_pmc.sh r03cens --method ECS --n 15 --N 500000 --censor 0.3 --steps 3 || exit 1
PMC_KERNEL=cens_round_kernel python3 tools/pmc_summary.py $R/gpurun_out/pmc_r03cens $O/pmc_cens.json > $O/pmc_cens.out 2>&1 || { tail $O/pmc_cens.out; exit 1; }
PMC_KERNEL=ecs_exact_kernel python3 tools/pmc_summary.py $R/gpurun_out/pmc_r03cens $O/pmc_exact15.json > $O/pmc_exact15.out 2>&1 || { tail $O/pmc_exact15.out; exit 1; }
head -12 $O/pmc_cens.out; head -12 $O/pmc_exact15.out
