set -o pipefail
O=gpurun_out/ab_minreg; mkdir -p $O
L="phasetype_amd/_variants/base.so phasetype_amd/_variants/iterative-minreg.so"
timeout -k 10 200 python3 tools/ab.py --libs $L --n 20 --N 100000 --rounds 5 --sweeps 10 > $O/cfg3.json 2> $O/cfg3.err &&
timeout -k 10 200 python3 tools/ab.py --libs $L --n 20 --N 500000 --rounds 3 --sweeps 5 > $O/n20_500k.json 2> $O/n20_500k.err &&
timeout -k 10 200 python3 tools/ab.py --libs $L --n 20 --N 500000 --censor 0.3 --rounds 3 --sweeps 5 > $O/n20_cens.json 2> $O/n20_cens.err
