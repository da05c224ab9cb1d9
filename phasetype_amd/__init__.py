"""phasetype_amd — MI355X-native PhaseType MCMC hot path.

Python mirror of the reference's R API over the C ABI of libPhaseType.so
(include/phasetype_amd.h):

* ``phtMCMC(x, states, beta, nu, zeta, n, mhit=1, ...)``   — R/phtMCMC.R:1-97
* ``phtMCMC2(x, TT, beta, nu, zeta, n, censored, C, method, mhit, ...)`` — R/phtMCMC2.R:1-86
* ``LJMA_Gibbs(...)`` — the 15-argument ``.C`` routine itself
  (src/PHT_MCMC_Aslett.c:104), as R's ``.C`` would call it.
* ``Sweeper`` — one GPU shard, one Gibbs step 1 per call (the seam of
  LJMA_MHsample_*; used by the parity tests and bench.py).

All compute runs in HIP kernels; there is no CPU fallback: without a GPU the
calls raise.  The library is loaded lazily so that importing works on a
CPU-only machine (the build check).
"""
from __future__ import annotations

import ctypes as C
import glob
import os

import numpy as np

from . import build as _build

__all__ = ["load", "LJMA_Gibbs", "phtMCMC", "phtMCMC2", "Sweeper", "gibbs_chains", "PhaseTypeError", "METHODS"]

# R/phtMCMC2.R:66-70; "UNIF" (8) is not a reference method: the opt-in
# uniformisation sampler (phasetype_amd/csrc/pht_unif.h), lowest precedence
METHODS = {"MHRS": 1, "ECS": 2, "DCS": 4, "UNIF": 8}


class PhaseTypeError(RuntimeError):
    pass


_dp = np.ctypeslib.ndpointer(dtype=np.float64, flags="C_CONTIGUOUS")
_ip = np.ctypeslib.ndpointer(dtype=np.int32, flags="C_CONTIGUOUS")
_lp = np.ctypeslib.ndpointer(dtype=np.int64, flags="C_CONTIGUOUS")
_up = np.ctypeslib.ndpointer(dtype=np.uint32, flags="C_CONTIGUOUS")
REDUCE_FN = C.CFUNCTYPE(C.c_int, C.POINTER(C.c_longlong), C.c_int, C.c_void_p)

_LIB = None

# every symbol include/phasetype_amd.h declares (tests check the exports)
EXPORTS = [
    "LJMA_Gibbs", "R_init_PhaseType", "pht_last_error", "pht_device_count", "pht_bind_lapack", "pht_set_seed",
    "pht_unif_rand", "pht_rgamma", "pht_in_R", "pht_set_verbose", "pht_zexp", "pht_params_bytes", "pht_stats_len",
    "pht_build_params", "pht_ctx_create", "pht_ctx_destroy", "pht_ctx_set_obs", "pht_ctx_sweep",
    "pht_ctx_sweep_debug", "pht_ctx_last_kernel_ms", "pht_ctx_flagged_obs", "pht_ctx_set_global_count", "pht_gibbs_run",
    "pht_gibbs_run_resident",
    "pht_gibbs_run_chains", "pht_rccl_unique_id", "pht_ctx_rccl_prepare", "pht_ctx_attach_rccl", "pht_ctx_rccl_allreduce",
]


def lib_key() -> str:
    """Identity of the loaded native library, which bench.py keys its PMC
    counters on (counters measured on another build are not reported):
    "src:<sha256 of the build inputs>" for the in-tree library (the same for
    every build of those sources: the .so bytes embed the build directory),
    "file:<sha256 of the file>" for a PHT_LIB variant."""
    import hashlib

    path = load()._pht_path
    if os.path.abspath(path) == os.path.abspath(_build.LIB) and "PHT_LIB" not in os.environ:
        return "src:" + _build.source_key()
    h = hashlib.sha256()
    with open(path, "rb") as f:
        for chunk in iter(lambda: f.read(1 << 20), b""):
            h.update(chunk)
    return "file:" + h.hexdigest()


def _lapack_path():
    env = os.environ.get("PHT_LAPACK_LIB")
    if env:
        return env, os.environ.get("PHT_LAPACK_PREFIX", "")
    import scipy

    d = os.path.join(os.path.dirname(os.path.dirname(scipy.__file__)), "scipy.libs")
    cands = sorted(glob.glob(os.path.join(d, "libscipy_openblas-*.so")))
    if not cands:
        raise PhaseTypeError("no LP64 LAPACK found for the per-sweep eigendecomposition (set PHT_LAPACK_LIB)")
    return cands[0], "scipy_"


def load(build_if_needed: bool = True) -> C.CDLL:
    """Load (building first if stale) phasetype_amd/_lib/libPhaseType.so."""
    global _LIB
    if _LIB is not None:
        return _LIB
    path = os.environ.get("PHT_LIB")  # a variant build (tools/ab.py)
    if path is None:
        if build_if_needed and _build.needs_build():
            _build.build()
        path = _build.LIB
    if not os.path.exists(path):
        raise PhaseTypeError(f"native library missing: {path} (run phasetype_amd/build.py)")
    L = C.CDLL(path, mode=C.RTLD_LOCAL)
    L._pht_path = os.path.abspath(path)
    L.pht_last_error.restype = C.c_char_p
    L.pht_bind_lapack.argtypes = [C.c_char_p, C.c_char_p]
    L.pht_set_seed.argtypes = [C.c_uint32]
    L.pht_unif_rand.restype = C.c_double
    L.pht_rgamma.restype = C.c_double
    L.pht_rgamma.argtypes = [C.c_double, C.c_double]
    L.pht_zexp.argtypes = [_dp, C.c_long]
    L.pht_build_params.argtypes = [C.c_int, _dp, _dp, C.c_int, C.c_void_p, C.c_int]
    L.pht_ctx_create.restype = C.c_void_p
    L.pht_ctx_create.argtypes = [C.c_int, C.c_int, C.c_int, C.c_int]
    L.pht_ctx_destroy.argtypes = [C.c_void_p]
    L.pht_ctx_set_obs.argtypes = [C.c_void_p, _dp, _ip, C.c_long, C.c_long]
    L.pht_ctx_sweep.argtypes = [C.c_void_p, _dp, _dp, C.c_uint32, C.c_uint32, C.c_uint32, C.c_int, _lp]
    L.pht_ctx_sweep_debug.argtypes = [C.c_void_p, _dp, _dp, C.c_uint32, C.c_uint32, C.c_uint32, C.c_int, _lp,
                                      _ip, _ip, _ip, _up, _lp, _ip]
    L.pht_ctx_last_kernel_ms.restype = C.c_float
    L.pht_ctx_last_kernel_ms.argtypes = [C.c_void_p]
    L.pht_ctx_flagged_obs.restype = C.c_longlong
    L.pht_ctx_flagged_obs.argtypes = [C.c_void_p]
    L.pht_ctx_set_global_count.argtypes = [C.c_void_p, C.c_longlong]
    L.pht_gibbs_run.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int, _dp, _dp, _ip, _dp, C.c_int, C.c_int,
                                _dp, _dp, C.c_void_p, C.c_void_p, C.POINTER(C.c_double)]
    L.pht_gibbs_run_resident.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int, _dp, _dp, _ip, _dp, C.c_int, _dp,
                                         _dp, C.POINTER(C.c_double)]
    L.pht_gibbs_run_chains.argtypes = [C.POINTER(C.c_void_p), C.c_int, _up, C.c_int, C.c_int, C.c_int, _dp, _dp,
                                       _ip, _dp, C.c_int, _dp, _dp, C.POINTER(C.c_double)]
    L.pht_rccl_unique_id.argtypes = [C.c_void_p]
    L.pht_ctx_rccl_prepare.argtypes = [C.c_void_p, C.c_int]
    L.pht_ctx_attach_rccl.argtypes = [C.c_void_p, C.c_char_p, C.c_int, C.c_int]
    L.pht_ctx_rccl_allreduce.argtypes = [C.c_void_p, _lp, C.c_int]
    L.LJMA_Gibbs.argtypes = [_ip, _ip, _ip, _ip, _ip, _dp, _dp, _ip, _dp, _dp, _ip, _ip, _dp, _ip, _dp]
    p, pre = _lapack_path()
    if L.pht_bind_lapack(p.encode(), pre.encode()) != 0:
        raise PhaseTypeError(L.pht_last_error().decode())
    _LIB = L
    return L


def _err(L) -> PhaseTypeError:
    return PhaseTypeError(L.pht_last_error().decode() or "unknown error")


def set_seed(seed: int) -> None:
    """R's set.seed() for the standalone host stream (inside R, R's own)."""
    load().pht_set_seed(int(seed) & 0xFFFFFFFF)


def device_count() -> int:
    return load().pht_device_count()


def zexp_for(y) -> int:
    y = np.ascontiguousarray(y, np.float64)
    return load().pht_zexp(y, len(y))


def stats_len(n: int) -> int:
    return 2 * n + n * n + 16


# extra-word indices (phasetype_amd/csrc/pht_layout.h): the ECS exact
# kernels' DEBUG launches count general-ARMS and private-envelope rounds there
XDBG_GENERAL, XDBG_PRIVATE = 8, 9


def split_stats(st, n):
    """int64 block -> (zq[n], B[n], N[n,n] as N[from, to], extras[16])."""
    st = np.asarray(st)
    zq = st[:n]
    B = st[n:2 * n]
    N = st[2 * n:2 * n + n * n].reshape(n, n).T  # N[i + j n] -> [i, j]
    return zq, B, N, st[2 * n + n * n:]


RCCL_ID_BYTES = 128


def rccl_unique_id() -> bytes:
    """A fresh RCCL unique id (one rank creates it and broadcasts it)."""
    L = load()
    buf = C.create_string_buffer(RCCL_ID_BYTES)
    if L.pht_rccl_unique_id(buf) != 0:
        raise _err(L)
    return buf.raw


class Sweeper:
    """One GPU shard of observations; one Gibbs step 1 per ``sweep`` call."""

    def __init__(self, n: int, method: int, mhit: int = 1, device: int = 0):
        self.L = load()
        self.n = n
        self.ctx = self.L.pht_ctx_create(device, n, method, mhit)
        if not self.ctx:
            raise _err(self.L)
        self.count = 0
        self.flagged_obs = 0  # flagged observation-sweeps of the last gibbs() (pht_ctx_flagged_obs)

    def set_obs(self, y, censored=None, obs0: int = 0):
        y = np.ascontiguousarray(y, np.float64)
        cen = np.zeros(len(y), np.int32) if censored is None else np.ascontiguousarray(censored, np.int32)
        if self.L.pht_ctx_set_obs(self.ctx, y, cen, len(y), obs0) != 0:
            raise _err(self.L)
        self.count = len(y)

    def sweep(self, S, s, key=(1, 2), sweep: int = 1, zexp: int = 40):
        out = np.zeros(stats_len(self.n), np.int64)
        Sf = np.ascontiguousarray(np.asarray(S, np.float64).reshape(-1, order="F"))
        if self.L.pht_ctx_sweep(self.ctx, Sf, np.ascontiguousarray(s, np.float64), key[0], key[1], sweep, zexp,
                                out) != 0:
            raise _err(self.L)
        return out

    def sweep_debug(self, S, s, key=(1, 2), sweep: int = 1, zexp: int = 40):
        n, l = self.n, self.count
        out = np.zeros(stats_len(n), np.int64)
        B, pre, fl = np.zeros(l, np.int32), np.zeros(l, np.int32), np.zeros(l, np.int32)
        nd = np.zeros(l, np.uint32)
        zq = np.zeros(l * n, np.int64)
        N = np.zeros(l * n * n, np.int32)
        Sf = np.ascontiguousarray(np.asarray(S, np.float64).reshape(-1, order="F"))
        if self.L.pht_ctx_sweep_debug(self.ctx, Sf, np.ascontiguousarray(s, np.float64), key[0], key[1], sweep,
                                      zexp, out, B, pre, fl, nd, zq, N) != 0:
            raise _err(self.L)
        return dict(stats=out, B=B, pre=pre, flags=fl, ndraw=nd, zq=zq.reshape(l, n),
                    N=N.reshape(l, n, n).transpose(0, 2, 1))

    def set_global_count(self, total: int) -> None:
        """Observations over all shards of a multi-process run: every sweep of
        gibbs() then checks the reduced statistics account for exactly that
        many (pht_ctx_set_global_count)."""
        if self.L.pht_ctx_set_global_count(self.ctx, int(total)) != 0:
            raise _err(self.L)

    def rccl_prepare(self, max_len: int = 256) -> None:
        """Local preconditions of attach_rccl / rccl_allreduce (RCCL loadable,
        no communicator yet, device, a staging buffer of max_len words):
        pht_ctx_rccl_prepare.  Ranks agree on it before anyone attaches."""
        if self.L.pht_ctx_rccl_prepare(self.ctx, int(max_len)) != 0:
            raise _err(self.L)

    def attach_rccl(self, uid: bytes, nranks: int, rank: int) -> None:
        """Sum every sweep's statistics block over ``nranks`` processes with
        an RCCL all-reduce on this shard's stream (pht_ctx_attach_rccl, the
        collective ncclCommInitRank); ``uid`` = rccl_unique_id() of one rank,
        the same on all, after rccl_prepare() on every rank.  gibbs() then
        needs no ``reduce``."""
        if len(uid) != RCCL_ID_BYTES:
            raise ValueError(f"RCCL unique id must be {RCCL_ID_BYTES} bytes, got {len(uid)}")
        if self.L.pht_ctx_attach_rccl(self.ctx, uid, nranks, rank) != 0:
            raise _err(self.L)

    def rccl_allreduce(self, buf: np.ndarray) -> None:
        """In-place sum of an int64 vector over the attached communicator
        (the same all-reduce a sweep runs on its statistics block)."""
        if buf.dtype != np.int64 or not buf.flags.c_contiguous:
            raise ValueError("rccl_allreduce needs a contiguous int64 array")
        if self.L.pht_ctx_rccl_allreduce(self.ctx, buf, len(buf)) != 0:
            raise _err(self.L)

    def last_kernel_ms(self) -> float:
        return self.L.pht_ctx_last_kernel_ms(self.ctx)

    def gibbs(self, it, method, nu, zeta, T, C_, zexp, start=None, reduce=None, silent=True):
        """Gibbs loop over this shard; ``reduce(stats: np.ndarray) -> None``
        sums the int64 block across shards in place (multi-process)."""
        m = len(nu)
        res = np.zeros(it * m, np.float64)
        start = np.array([-1.0]) if start is None else np.ascontiguousarray(start, np.float64)
        cb = None
        if reduce is not None:
            def _cb(ptr, ln, user):
                try:
                    arr = np.ctypeslib.as_array(ptr, shape=(ln,))
                    reduce(arr)
                    return 0
                except Exception:  # noqa: BLE001 - reported through the C status
                    return 1
            cb = REDUCE_FN(_cb)
        kms = C.c_double(0.0)
        Tf = np.ascontiguousarray(np.asarray(T).reshape(-1, order="F"), np.int32)
        Cf = np.ascontiguousarray(np.asarray(C_, np.float64).reshape(-1, order="F"))
        rc = self.L.pht_gibbs_run(self.ctx, it, method, m, np.ascontiguousarray(nu, np.float64),
                                  np.ascontiguousarray(zeta, np.float64), Tf, Cf, zexp, int(silent), start, res,
                                  C.cast(cb, C.c_void_p) if cb else None, None, C.byref(kms))
        if rc != 0:
            raise _err(self.L)
        self.kernel_ms_total = kms.value
        self.flagged_obs = int(self.L.pht_ctx_flagged_obs(self.ctx))
        return res.reshape(m, it).T.copy()

    def gibbs_resident(self, it, method, nu, zeta, T, C_, zexp, start=None):
        """The device-resident chain (pht_gibbs_run_resident; opt-in,
        non-parity: Gamma draws from the device's counter-based sampler):
        every sweep and conjugate update runs on the GPU, one host wait."""
        m = len(nu)
        res = np.zeros(it * m, np.float64)
        start = np.array([-1.0]) if start is None else np.ascontiguousarray(start, np.float64)
        kms = C.c_double(0.0)
        Tf = np.ascontiguousarray(np.asarray(T).reshape(-1, order="F"), np.int32)
        Cf = np.ascontiguousarray(np.asarray(C_, np.float64).reshape(-1, order="F"))
        if self.L.pht_gibbs_run_resident(self.ctx, it, method, m, np.ascontiguousarray(nu, np.float64),
                                         np.ascontiguousarray(zeta, np.float64), Tf, Cf, zexp, start, res,
                                         C.byref(kms)) != 0:
            raise _err(self.L)
        self.kernel_ms_total = kms.value
        self.flagged_obs = int(self.L.pht_ctx_flagged_obs(self.ctx))
        return res.reshape(m, it).T.copy()

    def close(self):
        if self.ctx:
            self.L.pht_ctx_destroy(self.ctx)
            self.ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001
            pass


def _chains_start(start, K: int, m: int) -> np.ndarray:
    """The start block pht_gibbs_run_chains reads: [-1] (draw from the prior),
    or K*m values, chain c at [c*m, (c+1)*m).  A single m-vector (what
    Sweeper.gibbs and the R API take) is broadcast to every chain; any other
    length is refused here, because the C side reads start + c*m unchecked."""
    if start is None:
        return np.array([-1.0])
    st = np.ascontiguousarray(start, np.float64).reshape(-1)
    if st.size >= 1 and st[0] < 0:
        return np.array([-1.0])
    if st.size == m:
        return np.ascontiguousarray(np.tile(st, K))
    if st.size == K * m:
        return st
    raise ValueError(f"gibbs_chains: start has {st.size} values; need {m} (one start for every chain) "
                     f"or {K}*{m} (one per chain), or a negative first value")


def gibbs_chains(seeds, y, censored, n, method, nu, zeta, T, C_, mhit: int = 1, it: int = 100, start=None,
                 device: int = 0, obs0: int = 0):
    """Independent Gibbs chains at once (pht_gibbs_run_chains):
    chain c is the single chain of ``Sweeper.gibbs`` after ``set_seed(seeds[c])``.
    Returns (draws [chains, it, m], max kernel ms)."""
    L = load()
    seeds = np.ascontiguousarray(seeds, np.uint32)
    K, m = len(seeds), len(nu)
    sws = []
    try:
        for _ in range(K):
            sw = Sweeper(n, method, mhit, device=device)
            sw.set_obs(y, censored, obs0=obs0)
            sws.append(sw)
        ctxs = (C.c_void_p * K)(*[sw.ctx for sw in sws])
        res = np.zeros(K * it * m, np.float64)
        st = _chains_start(start, K, m)
        Tf = np.ascontiguousarray(np.asarray(T).reshape(-1, order="F"), np.int32)
        Cf = np.ascontiguousarray(np.asarray(C_, np.float64).reshape(-1, order="F"))
        kms = C.c_double(0.0)
        zexp = zexp_for(y)
        if L.pht_gibbs_run_chains(ctxs, K, seeds, it, method, m, np.ascontiguousarray(nu, np.float64),
                                  np.ascontiguousarray(zeta, np.float64), Tf, Cf, zexp, st, res,
                                  C.byref(kms)) != 0:
            raise _err(L)
        return res.reshape(K, m, it).transpose(0, 2, 1).copy(), kms.value
    finally:
        for sw in sws:
            sw.close()


def LJMA_Gibbs(it, mhit, method, n, m, nu, zeta, T, C_, y, l, censored, start, silent, res):
    """The .C routine (src/PHT_MCMC_Aslett.c:104) with R's .C semantics:
    every argument is a fresh vector; returns the dict of (modified) vectors."""
    L = load()
    a = dict(it=np.array([it], np.int32), mhit=np.array([mhit], np.int32), method=np.array([method], np.int32),
             n=np.array([n], np.int32), m=np.array([m], np.int32), nu=np.array(nu, np.float64),
             zeta=np.array(zeta, np.float64), T=np.array(T, np.int32).reshape(-1, order="F"),
             C=np.array(C_, np.float64).reshape(-1, order="F"), y=np.array(y, np.float64),
             l=np.array([l], np.int32), censored=np.array(censored, np.int32), start=np.array(start, np.float64),
             silent=np.array([silent], np.int32), res=np.array(res, np.float64))
    a = {k: np.ascontiguousarray(v) for k, v in a.items()}
    L.LJMA_Gibbs(*a.values())
    msg = L.pht_last_error().decode()
    if msg:
        raise PhaseTypeError(msg)
    return a


def _r_sort(names, collation: str = "C"):
    """R's sort() of character names.  "C": byte order; "en_US": case-folded
    first (how a typical UTF-8 locale collates S12 / s1)."""
    if collation == "C":
        return sorted(names)
    return sorted(names, key=lambda s: (s.lower(), s.swapcase()))


def phtMCMC2(x, TT, beta, nu, zeta, n, censored=None, C_=None, method="ECS", mhit=1, resume=None,
             silent=False, collation="C"):
    """R/phtMCMC2.R:1-86: structured generator TT (strings, "0" = fixed zero)."""
    TT = np.asarray(TT, dtype=object).astype(str)
    nu = {k: float(nu[k]) for k in _r_sort(list(nu), collation)}
    zeta = {k: float(zeta[k]) for k in _r_sort(list(zeta), collation)}
    if int(n) < 1:
        raise ValueError(f"{n} is an invalid number of MCMC iterations.")
    if int(mhit) < 0:
        raise ValueError(f"{mhit} is an invalid number of Metropolis-Hastings iterations.")
    dimT = TT.shape[0]
    if TT.shape[0] != TT.shape[1]:
        raise ValueError("matrix of variables must be square")
    if set(np.diag(TT)) != {"0"}:
        raise ValueError("diagonal of matrix of variables must be zeros")
    if set(TT[dimT - 1, :]) != {"0"}:
        raise ValueError("last row of matrix of variables must represent absorbing state (and so be all zeros)")
    if len(beta) != dimT - 1:
        raise ValueError(f"beta should be a vector of length {dimT - 1} for the generator specified.")
    if any(b < 0 for b in beta):
        raise ValueError("beta is not a valid parameter of a Dirichlet distribution.")
    if C_ is None:
        C_ = np.ones((dimT, dimT))
    C_ = np.asarray(C_, np.float64)
    if C_.shape != (dimT, dimT):
        raise ValueError("dimension of C must match dimension of TT")
    var_names = [v for v in _r_sort(set(TT.reshape(-1)), collation) if v != "0"]
    if list(nu) != var_names:
        raise ValueError("variables specified in matrix don't match those in prior nu")
    if list(zeta) != var_names:
        raise ValueError("variables specified in matrix don't match those in prior zeta")
    start = [-1.0]
    it = int(n)
    if resume is not None:
        resume = np.asarray(resume, np.float64)
        if resume.shape[1] != len(var_names):
            raise ValueError("the variables in resume do not match the variables in generator")
        start = list(resume[-1])
        it = it + 1
    TN = np.zeros((dimT, dimT), np.int32)
    for i in range(dimT):
        for j in range(dimT):
            TN[i, j] = (["0"] + var_names).index(TT[i, j])
    meths = [method] if isinstance(method, str) else list(method)
    bad = set(meths) - set(METHODS)
    if bad:
        raise ValueError(f"Error: unknown sampling methods ({', '.join(sorted(bad))})")
    method_num = sum(METHODS[k] for k in dict.fromkeys(meths))
    x = np.asarray(x, np.float64)
    cen = np.zeros(len(x), np.int32) if censored is None else np.asarray(censored).astype(np.int32)
    out = LJMA_Gibbs(it, mhit, method_num, dimT - 1, len(var_names), list(nu.values()), list(zeta.values()), TN,
                     C_, x, len(x), cen, start, int(silent), np.zeros(it * len(var_names)))
    samples = out["res"].reshape(len(var_names), it).T
    if resume is not None:
        samples = np.vstack([resume[:-1], samples])
    return dict(samples=samples, data=x, vars=var_names, TT=TT, beta=beta, nu=nu, zeta=zeta, iterations=it,
                censored=cen, method=method, MHit=mhit)


def phtMCMC(x, states, beta, nu, zeta, n, mhit=1, resume=None, silent=False, collation="C"):
    """R/phtMCMC.R:1-97: dense generator, always MHRS."""
    if len(nu) != states * states:
        raise ValueError("nu must specify one prior Gamma shape parameter per element of the Phase-type generator")
    if len(zeta) != states:
        raise ValueError("zeta must specify one prior Gamma reciprocal scale parameter per non-absorbing row")
    TT = np.empty((states + 1, states + 1), dtype=object)
    for i in range(states):
        for j in range(states):
            TT[i, j] = f"S{i + 1}{j + 1}"
        TT[i, states] = f"s{i + 1}"
    TT[states, :] = "0"
    for i in range(states + 1):
        TT[i, i] = "0"
    names = [v for v in TT.T.T.reshape(-1) if v != "0"]  # c(t(TT)) without "0": row-major
    nu_d = dict(zip(names, [float(v) for v in nu]))
    # zeta <- as.list(rep(zeta, each=states+1)); names(zeta) <- names (R/phtMCMC.R:29-30)
    zrep = np.repeat(np.asarray(zeta, np.float64), states + 1)
    zeta_d = dict(zip(names, zrep[:len(names)]))
    return phtMCMC2(x, TT, beta, nu_d, zeta_d, n, censored=None, C_=np.ones((states + 1, states + 1)),
                    method="MHRS", mhit=mhit, resume=resume, silent=silent, collation=collation)
