set -o pipefail
# censored ECS LDS envelope size at n = 15 / 20 (one process per library)
O=$GRAFT_REPO_ROOT/gpurun_out/r03aa; mkdir -p $O; cd $GRAFT_REPO_ROOT
V=phasetype_amd/_variants
ab() { local tag=$1; shift; timeout -k 10 400 python3 tools/ab.py "$@" --method ECS --rounds 5 > $O/$tag.json 2> $O/$tag.err || { tail $O/$tag.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/$tag.json'));print('$tag', {k.split('/')[-1]:(round(v['ms_per_sweep_median'],4),round(v['kernel_ms_median'],4)) for k,v in d.items()} if 'error' not in d else d)"; }
ab n15 --libs phasetype_amd/_lib/libPhaseType.so $V/k15_9.so $V/k15_5.so --n 15 --N 500000 --censor 0.3 --sweeps 10
ab n20 --libs phasetype_amd/_lib/libPhaseType.so $V/k20_9.so --n 20 --N 500000 --censor 0.3 --sweeps 10
PHT_CENS_SERIAL=1 ab n15_serial --libs phasetype_amd/_lib/libPhaseType.so $V/k15_9.so --n 15 --N 500000 --censor 0.3 --sweeps 10
