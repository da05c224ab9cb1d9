set -o pipefail
# timing-only ablation: approximate reciprocal division in the ARMS code (the divisions' share of the round)
O=$GRAFT_REPO_ROOT/gpurun_out/r03ac; mkdir -p $O; cd $GRAFT_REPO_ROOT
V=phasetype_amd/_variants
for cfg in "10 1000000 0 10" "10 125000 0 40"; do set -- $cfg
  timeout -k 10 400 python3 tools/ab.py --no-check --libs $V/head.so $V/fastdiv.so --method ECS --n $1 --N $2 --censor $3 --sweeps $4 --rounds 5 > $O/ab_$1_$2_$3.json 2> $O/ab_$1_$2_$3.err || { tail $O/ab_$1_$2_$3.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/ab_$1_$2_$3.json'));print('n=$1 N=$2 c=$3', {k.split('/')[-1]:(round(v['ms_per_sweep_median'],4),round(v['kernel_ms_median'],4)) for k,v in d.items()} if 'error' not in d else d)"
done
