"""pht_build_params per call (us) at n = 5, 10, 15, 20 for ECS (method 2:
the eigensystem, its inverse and the spectral products) and MHRS (method 1:
no eigensystem); the per-sweep host work the pipelined loop leaves between
two sweeps.  usage (GPU box): python3 tools/bp_time.py"""
import time, numpy as np, sys, os
sys.path.insert(0, os.getcwd())
import phasetype_amd as P
from phasetype_amd.synth import bd_exit
L = P.load()
out = {}
for n in (5, 10, 15, 20):
    S, s = bd_exit(n)
    Sf = np.ascontiguousarray(S.ravel(order="F")); sc = np.ascontiguousarray(s)
    nb = L.pht_params_bytes(n); buf = np.zeros(nb, np.uint8)
    for meth in (2, 1):
        for _ in range(300): L.pht_build_params(n, Sf, sc, meth, buf.ctypes.data, nb)
        K = 3000; t = time.perf_counter()
        for _ in range(K): L.pht_build_params(n, Sf, sc, meth, buf.ctypes.data, nb)
        out[f"n{n}_m{meth}"] = round((time.perf_counter() - t) / K * 1e6, 2)
print(out)
