set -o pipefail
O=gpurun_out/ab_zero; mkdir -p $O
L="phasetype_amd/_variants/base.so phasetype_amd/_variants/zero_late.so"
timeout -k 10 200 python3 tools/ab.py --libs $L --n 5 --N 10000 --rounds 7 --sweeps 40 > $O/cfg2.json 2> $O/cfg2.err &&
timeout -k 10 200 python3 tools/ab.py --libs $L --n 10 --N 125000 --rounds 7 --sweeps 20 > $O/n10_125k.json 2> $O/n10_125k.err &&
timeout -k 10 200 python3 tools/ab.py --libs $L --n 3 --N 200 --rounds 7 --sweeps 100 > $O/cfg1.json 2> $O/cfg1.err
