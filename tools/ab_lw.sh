set -o pipefail
O=gpurun_out/ab_lw; mkdir -p $O
L="phasetype_amd/_variants/head.so phasetype_amd/_variants/lwcache.so"
timeout -k 10 200 python3 tools/ab.py --libs $L --n 20 --N 100000 --rounds 7 --sweeps 20 > $O/cfg3.json 2> $O/cfg3.err &&
timeout -k 10 200 python3 tools/ab.py --libs $L --n 3 --N 200 --rounds 7 --sweeps 200 > $O/cfg1.json 2> $O/cfg1.err &&
timeout -k 10 200 python3 tools/ab.py --libs $L --n 10 --N 125000 --rounds 7 --sweeps 20 > $O/n10_125k.json 2> $O/n10_125k.err
