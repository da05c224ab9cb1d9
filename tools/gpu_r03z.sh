set -o pipefail
# n = 10-only censored LDS envelope: full GPU suite, then A/B vs HEAD (one process per library)
O=$GRAFT_REPO_ROOT/gpurun_out/r03z; mkdir -p $O; cd $GRAFT_REPO_ROOT
bash tools/gpu_full.sh r03z_full || exit 1
for cfg in "10 1000000 0.3 10" "15 500000 0.3 10" "10 125000 0.3 40"; do set -- $cfg
  timeout -k 10 400 python3 tools/ab.py --libs phasetype_amd/_variants/base.so phasetype_amd/_lib/libPhaseType.so --method ECS --n $1 --N $2 --censor $3 --sweeps $4 --rounds 5 > $O/ab_$1_$2_$3.json 2> $O/ab_$1_$2_$3.err || { tail $O/ab_$1_$2_$3.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/ab_$1_$2_$3.json'));print('n=$1 N=$2 c=$3', {k.split('/')[-1]:(round(v['ms_per_sweep_median'],4),round(v['kernel_ms_median'],4)) for k,v in d.items()} if 'error' not in d else d)"
done
