set -o pipefail
O=gpurun_out/ab_ilp; mkdir -p $O
L="phasetype_amd/_variants/base.so phasetype_amd/_variants/ilp.so"
timeout -k 10 200 python3 tools/ab.py --libs $L --n 10 --N 1000000 --rounds 5 --sweeps 8 > $O/cfg4.json 2> $O/cfg4.err &&
timeout -k 10 200 python3 tools/ab.py --libs $L --n 10 --N 125000 --rounds 5 --sweeps 10 > $O/n10_125k.json 2> $O/n10_125k.err &&
timeout -k 10 200 python3 tools/ab.py --libs $L --n 20 --N 100000 --rounds 5 --sweeps 10 > $O/cfg3.json 2> $O/cfg3.err &&
timeout -k 10 200 python3 tools/ab.py --libs $L --n 5 --N 10000 --rounds 5 --sweeps 20 > $O/cfg2.json 2> $O/cfg2.err &&
timeout -k 10 200 python3 tools/ab.py --libs $L --n 15 --N 500000 --censor 0.3 --rounds 5 --sweeps 8 > $O/cfg5ecs.json 2> $O/cfg5ecs.err
