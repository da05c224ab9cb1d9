"""oracle/oracle.py — TEST INFRASTRUCTURE ONLY (ctypes bindings for the oracle).

The CPU oracle lives under oracle/ and is used only by tests/, bench.py's
``cpu_baseline`` leg and ``__graft_entry__.smoke()`` as the *checker*:

* ``OracleLib`` — oracle/_build/liboracle.so, our C restatement of the hot
  path (pht_oracle.c, every function citing the reference file:line it
  follows).  ``ref`` variant: R-stream RNG + libm + the reference's
  arithmetic order, i.e. the reference's algorithm draw for draw.  ``dev``
  variant: Philox + detmath + fixed-point z, bit-exact with the HIP kernels
  (the GPU specification).

PARITY UNPINNED: the reference's own tests hold no fixtures (its
tests/*.R only print) and its C needs R's headers and nmath, which this image
lacks, so it cannot be built or run here.  What checks the restatement
instead: R's published set.seed outputs for the R stream,
Random123's known answers for Philox, RNG-free analytic expectations (Van
Loan), brute-force forward simulation for censored paths, and the committed
regression vectors of tests/golden/.

Nothing in phasetype_amd/ imports this module.
"""
from __future__ import annotations

import ctypes as C
import glob
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
ORC_SO = os.path.join(HERE, "_build", "liboracle.so")

_dp = np.ctypeslib.ndpointer(dtype=np.float64, flags="C_CONTIGUOUS")
_ip = np.ctypeslib.ndpointer(dtype=np.int32, flags="C_CONTIGUOUS")
_lp = np.ctypeslib.ndpointer(dtype=np.int64, flags="C_CONTIGUOUS")


def lapack_path() -> tuple[str, str]:
    """(path, symbol prefix) of an LP64 LAPACK: scipy's bundled OpenBLAS."""
    env = os.environ.get("PHT_LAPACK_LIB")
    if env:
        return env, os.environ.get("PHT_LAPACK_PREFIX", "")
    import scipy  # noqa: F401  (only to locate the wheel's .libs dir)

    d = os.path.join(os.path.dirname(os.path.dirname(scipy.__file__)), "scipy.libs")
    cands = sorted(glob.glob(os.path.join(d, "libscipy_openblas-*.so")))
    if not cands:
        raise RuntimeError("no LP64 LAPACK found (set PHT_LAPACK_LIB)")
    return cands[0], "scipy_"


def build() -> None:
    subprocess.run(["make", "-s", "-C", HERE, "oracle"], check=True)


def gibbs_argv(it, mhit, method, n, nu, zeta, T, C_, y, censored, start, silent):
    """The 15 .C vectors of LJMA_Gibbs (src/PHT_MCMC_Aslett.c:104)."""
    m = len(nu)
    return dict(
        it=np.array([it], np.int32), mhit=np.array([mhit], np.int32),
        method=np.array([method], np.int32), n=np.array([n], np.int32),
        m=np.array([m], np.int32), nu=np.ascontiguousarray(nu, np.float64),
        zeta=np.ascontiguousarray(zeta, np.float64),
        T=np.ascontiguousarray(np.asarray(T).reshape(-1, order="F") if np.ndim(T) == 2 else T, np.int32),
        C=np.ascontiguousarray(np.asarray(C_).reshape(-1, order="F") if np.ndim(C_) == 2 else C_, np.float64),
        y=np.ascontiguousarray(y, np.float64), l=np.array([len(y)], np.int32),
        censored=np.ascontiguousarray(censored, np.int32),
        start=np.ascontiguousarray(start, np.float64), silent=np.array([silent], np.int32),
        res=np.zeros(it * m, np.float64),
    )


_u32p = np.ctypeslib.ndpointer(dtype=np.uint32, flags="C_CONTIGUOUS")


def _opt(ptype):
    """ndpointer that also accepts None (NULL)."""
    class _P(ptype):
        @classmethod
        def from_param(cls, obj):
            if obj is None:
                return None
            return ptype.from_param(obj)
    return _P


class OracleLib:
    """Our CPU restatement (oracle/_build/liboracle.so)."""

    def __init__(self, path: str = ORC_SO):
        if not os.path.exists(path):
            raise FileNotFoundError(path)
        self.lib = L = C.CDLL(path)
        L.orc_bind_lapack.argtypes = [C.c_char_p, C.c_char_p]
        p, pre = lapack_path()
        if L.orc_bind_lapack(p.encode(), pre.encode()) != 0:
            raise RuntimeError("could not bind LAPACK for the oracle")
        L.orc_set_seed.argtypes = [C.c_uint32]
        L.orc_unif_rand.restype = C.c_double
        L.orc_rgamma.restype = C.c_double
        L.orc_rgamma.argtypes = [C.c_double, C.c_double]
        L.orc_exp_rand.restype = C.c_double
        L.orc_norm_rand.restype = C.c_double
        L.orc_sp_size.restype = C.c_size_t
        self.maxn = L.orc_maxn()
        self.spsize = L.orc_sp_size()
        L.orc_sp_build.argtypes = [C.c_void_p, C.c_int, _dp, _dp, C.c_int]
        od, oi, ol, ou = _opt(_dp), _opt(_ip), _opt(_lp), _opt(_u32p)
        ostats = _opt(_lp)
        L.orc_ref_sweep.argtypes = [C.c_void_p, C.c_int, C.c_int, _dp, _ip, C.c_long, _dp, _ip, _ip,
                                    oi, oi, od, oi, oi, ou, ostats]
        L.orc_dev_sweep.argtypes = [C.c_void_p, C.c_int, C.c_int, _dp, _ip, C.c_long, C.c_long,
                                    C.c_uint32, C.c_uint32, C.c_uint32, C.c_int, _lp, _lp, _lp,
                                    oi, oi, od, ol, oi, oi, ou, ostats]
        L.orc_zexp.argtypes = [_dp, C.c_long]
        L.orc_gibbs.argtypes = [C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, _dp, _dp, _ip, _dp,
                                _dp, C.c_long, _ip, _dp, _dp]
        L.orc_gibbs_z.argtypes = [C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, _dp, _dp, _ip, _dp,
                                  _dp, C.c_long, _ip, _dp, _dp, C.c_int]
        L.orc_rgamma_ctr_v.argtypes = [C.c_uint32, C.c_uint32, C.c_double, C.c_double, C.c_long, _dp]
        L.orc_eig.argtypes = [C.c_int, _dp, _dp, _dp, _dp]
        L.orc_eig_refine.argtypes = [C.c_int, _dp, _dp, _dp, _dp, _dp, _dp]
        L.orc_eig_fallback_count.restype = C.c_long
        L.orc_set_dcs_brent.argtypes = [C.c_int]
        L.orc_set_bridge.argtypes = [C.c_int, C.c_int]

    def set_seed(self, seed: int) -> None:
        self.lib.orc_set_seed(seed & 0xFFFFFFFF)

    def sp(self, S, s, method):
        buf = C.create_string_buffer(self.spsize)
        S = np.asarray(S, np.float64)
        info = self.lib.orc_sp_build(buf, S.shape[0], np.ascontiguousarray(S.reshape(-1, order="F")),
                                     np.ascontiguousarray(s, np.float64), method)
        return buf, info

    def ref_sweep(self, method, S, s, y, censored=None, mhit=1, per_obs=True):
        n = S.shape[0]
        y = np.ascontiguousarray(y, np.float64)
        l = len(y)
        cen = np.zeros(l, np.int32) if censored is None else np.ascontiguousarray(censored, np.int32)
        sp, _ = self.sp(S, s, method)
        zt, Bt, Nt = np.zeros(n), np.zeros(n, np.int32), np.zeros(n * n, np.int32)
        if per_obs:
            B, pre, z = np.zeros(l, np.int32), np.zeros(l, np.int32), np.zeros(l * n)
            N, fl, nw = np.zeros(l * n * n, np.int32), np.zeros(l, np.int32), np.zeros(l, np.uint32)
        else:
            B = pre = z = N = fl = nw = None
        stats = np.zeros(4, np.int64)
        self.lib.orc_ref_sweep(sp, method, mhit, y, cen, l, zt, Bt, Nt, B, pre, z, N, fl, nw, stats)
        out = dict(z_tot=zt, B_tot=Bt, N_tot=Nt.reshape(n, n).T, stats=stats)
        if per_obs:
            out.update(B=B, pre=pre, z=z.reshape(l, n), N=N.reshape(l, n, n).transpose(0, 2, 1), flags=fl,
                       nword=nw)
        return out

    def dev_sweep(self, method, S, s, y, censored=None, mhit=1, key=(1, 2), sweep=1, zexp=None,
                  obs0=0, per_obs=True):
        n = S.shape[0]
        y = np.ascontiguousarray(y, np.float64)
        l = len(y)
        cen = np.zeros(l, np.int32) if censored is None else np.ascontiguousarray(censored, np.int32)
        if zexp is None:
            zexp = self.lib.orc_zexp(y, l)
        sp, _ = self.sp(S, s, method)
        zq, Bt, Nt = np.zeros(n, np.int64), np.zeros(n, np.int64), np.zeros(n * n, np.int64)
        if per_obs:
            B, pre, z = np.zeros(l, np.int32), np.zeros(l, np.int32), np.zeros(l * n)
            zqo, N = np.zeros(l * n, np.int64), np.zeros(l * n * n, np.int32)
            fl, nd = np.zeros(l, np.int32), np.zeros(l, np.uint32)
        else:
            B = pre = z = zqo = N = fl = nd = None
        stats = np.zeros(4, np.int64)
        self.lib.orc_dev_sweep(sp, method, mhit, y, cen, l, obs0, key[0], key[1], sweep, zexp, zq, Bt, Nt,
                               B, pre, z, zqo, N, fl, nd, stats)
        out = dict(zq_tot=zq, B_tot=Bt, N_tot=Nt.reshape(n, n).T, zexp=zexp, stats=stats)
        if per_obs:
            out.update(B=B, pre=pre, z=z.reshape(l, n), zq=zqo.reshape(l, n),
                       N=N.reshape(l, n, n).transpose(0, 2, 1), flags=fl, ndraw=nd)
        return out

    def gibbs_zexp(self, dev, it, mhit, method, n, nu, zeta, T, C_, y, censored, zexp, start=None):
        """gibbs() at an explicit fixed-point exponent (dev variants)."""
        if start is None:
            start = np.array([-1.0])
        a = gibbs_argv(it, mhit, method, n, nu, zeta, T, C_, y, censored, start, 1)
        self.lib.orc_gibbs_z(int(dev), it, mhit, method, n, len(nu), a["nu"], a["zeta"], a["T"], a["C"], a["y"],
                             len(y), a["censored"], a["start"], a["res"], int(zexp))
        return a["res"].reshape(len(nu), it).T.copy()

    def eig_refine(self, S, Q0, Qi0):
        """The resident chain's warm-start refinement (pht_eig_refine) of the
        eigensystem (Q0, Qi0) for S: (rc, evals, Q, Qinv), rc 2 = not
        converged (the chain then runs the full QR)."""
        S = np.asarray(S, np.float64)
        n = S.shape[0]
        f = lambda M: np.ascontiguousarray(np.asarray(M, np.float64).reshape(-1, order="F"))
        ev, Q, Qi = np.zeros(n), np.zeros(n * n), np.zeros(n * n)
        rc = self.lib.orc_eig_refine(n, f(S), f(Q0), f(Qi0), ev, Q, Qi)
        return rc, ev, Q.reshape(n, n, order="F"), Qi.reshape(n, n, order="F")

    def set_dcs_brent(self, on: bool) -> None:
        """dev variant's DCS root finder: Find02's Brent search (on) or the
        device spec's default safeguarded Halley iteration (off)."""
        self.lib.orc_set_dcs_brent(1 if on else 0)

    def halley_hist(self) -> np.ndarray:
        """evaluations per DCS jump of the dev variant's Halley root since the
        last call (bins 0..63, the last = 63 or more); clears the counts"""
        h = np.zeros(64, np.int64)
        self.lib.orc_halley_hist_take(h.ctypes.data_as(C.c_void_p))
        return h

    def set_bridge(self, mhrs: bool = False, dcs: bool = False) -> None:
        """dev variant's bridge modes (PHT_MHRS=bridge / PHT_DCS=bridge on the
        device): MHRS's / DCS's path law sampled exactly by the
        uniformisation sampler (pht_unif.h ulaw 1 / 2) instead of the
        rejection search / Hobolth's sampler."""
        self.lib.orc_set_bridge(1 if mhrs else 0, 1 if dcs else 0)

    def eig(self, S):
        """The device-resident chain's eigensystem (include/pht_eigen.h):
        (rc, evals, Q, Qinv), rc 0 = ok, 1 complex pair, 2 no convergence,
        3 singular eigenvectors."""
        S = np.asarray(S, np.float64)
        n = S.shape[0]
        ev, Q, Qi = np.zeros(n), np.zeros(n * n), np.zeros(n * n)
        rc = self.lib.orc_eig(n, np.ascontiguousarray(S.reshape(-1, order="F")), ev, Q, Qi)
        return rc, ev, Q.reshape(n, n, order="F"), Qi.reshape(n, n, order="F")

    def rgamma_ctr(self, a, scale, cnt, key=(1, 2)):
        """cnt draws of the device-resident chain's Gamma sampler (include/pht_gamma.h)."""
        out = np.zeros(cnt)
        self.lib.orc_rgamma_ctr_v(key[0], key[1], a, scale, cnt, out)
        return out

    def gibbs(self, dev, it, mhit, method, n, nu, zeta, T, C_, y, censored=None, start=None):
        """dev: 0 the reference's algorithm (R stream), 1 the GPU spec (host
        Gamma update: pht_gibbs_run), 2 the device-resident chain
        (pht_gibbs_run_resident: counter-based Gamma draws)."""
        if censored is None:
            censored = np.zeros(len(y), np.int32)
        if start is None:
            start = np.array([-1.0])
        a = gibbs_argv(it, mhit, method, n, nu, zeta, T, C_, y, censored, start, 1)
        self.lib.orc_gibbs(int(dev), it, mhit, method, n, len(nu), a["nu"], a["zeta"], a["T"], a["C"], a["y"],
                           len(y), a["censored"], a["start"], a["res"])
        return a["res"].reshape(len(nu), it).T.copy()
