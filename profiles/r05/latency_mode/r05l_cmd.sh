# r05 combined lease (censored rounds, MHRS record checks, latency-mode experiment, stamps)
T=tests/test_gpu_fullsize.py::test_full_size_sweep_statistics_vs_reference_algorithm
V=/root/repo/phasetype_amd/_variants
bash tools/gpu_steps.sh r05l tests=tests/test_gpu_parity.py "tests=$T[cfg5_ecs]" \
  "bench=--n 15 --N 500000 --censor 0.3 --steps 20 --no-cpu-baseline --no-alt" \
  "bench=--method MHRS --steps 100 --warmup 2 --no-cpu-baseline --no-alt" \
  "py=tools/ab.py --libs $V/head.so phasetype_amd/_lib/libPhaseType.so --method MHRS --rounds 4 --sweeps 100" \
  "shards=8" \
  "env=PHT_LIB=$V/lat.so" "tests=tests/test_gpu_parity.py -k per_observation_bitexact" "latency=--shards 8" \
  "env=PHT_ROWK=0" "env=PHT_LIB=$V/lat_st.so" "py=tools/stamps.py --top 64" "py=tools/stamps.py --N 125000" \
  "env=PHT_LIB=$V/base_st.so" "py=tools/stamps.py --top 64" "py=tools/stamps.py --N 125000" \
  "unenv=PHT_LIB" "unenv=PHT_ROWK" "env=PHT_CENS_SERIAL=1" "trace=--n 15 --N 500000 --censor 0.3 --steps 10"
