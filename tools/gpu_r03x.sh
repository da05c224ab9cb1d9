set -o pipefail
# lib load order vs the concurrent exact+censored overlap (same process: HW queue mapping)
O=$GRAFT_REPO_ROOT/gpurun_out/r03x; mkdir -p $O; cd $GRAFT_REPO_ROOT
run() { local tag=$1; shift; timeout -k 10 400 python3 tools/ab.py --method ECS "$@" --rounds 4 > $O/$tag.json 2> $O/$tag.err || { tail $O/$tag.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/$tag.json'));print('$tag', {k.split('/')[-1]:(round(v['ms_per_sweep_median'],4),round(v['kernel_ms_median'],4)) for k,v in d.items()} if 'error' not in d else d)"; }
run new_first --libs phasetype_amd/_lib/libPhaseType.so phasetype_amd/_variants/base.so --n 15 --N 500000 --censor 0.3 --sweeps 10
run new_only --libs phasetype_amd/_lib/libPhaseType.so --n 15 --N 500000 --censor 0.3 --sweeps 10
run base_only --libs phasetype_amd/_variants/base.so --n 15 --N 500000 --censor 0.3 --sweeps 10
