set -o pipefail
# cfg5 ECS regression: n = 15 exact-only, and 30 % censored with the two ranges serialised
O=$GRAFT_REPO_ROOT/gpurun_out/r03w; mkdir -p $O; cd $GRAFT_REPO_ROOT
run() { local tag=$1; shift; timeout -k 10 400 python3 tools/ab.py --libs phasetype_amd/_variants/base.so phasetype_amd/_lib/libPhaseType.so --method ECS "$@" --rounds 4 > $O/$tag.json 2> $O/$tag.err || { tail $O/$tag.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/$tag.json'));print('$tag', {k.split('/')[-1]:(round(v['ms_per_sweep_median'],4),round(v['kernel_ms_median'],4)) for k,v in d.items()} if 'error' not in d else d)"; }
run n15_exact --n 15 --N 500000 --censor 0 --sweeps 10
PHT_CENS_SERIAL=1 run n15_cens_serial --n 15 --N 500000 --censor 0.3 --sweeps 10
run n15_cens --n 15 --N 500000 --censor 0.3 --sweeps 10
run n10_cens --n 10 --N 500000 --censor 0.3 --sweeps 10
