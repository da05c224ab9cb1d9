#!/usr/bin/env python3
"""A short resident chain for a kernel-trace profile of the update kernel
(resident_update_kernel) next to the sweep kernels.  usage: prof_resident.py
<n> <N> <method> [sweeps]; run under rocprofv3 --kernel-trace --stats."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import phasetype_amd as P  # noqa: E402
from phasetype_amd.synth import DATA_KEY, bd_exit, bd_exit_structure, simulate_ph  # noqa: E402

n, N, meth = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3]
steps = int(sys.argv[4]) if len(sys.argv) > 4 else 200
S, s = bd_exit(n)
T, theta = bd_exit_structure(n)
nu, zeta, Cm = 1 + 50 * theta, np.full(len(theta), 50.0), np.ones(T.shape)
y, cen = simulate_ph(S, s, N, seed=DATA_KEY)
mm = P.METHODS[meth]
sw = P.Sweeper(n, mm, 1)
sw.set_obs(y, cen)
P.set_seed(1)
r = sw.gibbs_resident(steps + 1, mm, nu, zeta, T, Cm, P.zexp_for(y))
print(meth, n, N, steps, "kernel ms/sweep", sw.kernel_ms_total / steps, "finite", bool(np.all(np.isfinite(r))))
sw.close()
