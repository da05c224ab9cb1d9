"""CPU: the C-ABI library and its host-side logic (no kernel launches).

* libPhaseType.so loads and exports every function include/phasetype_amd.h
  declares; without a HIP device the GPU entry points fail loudly (no CPU
  fallback).
* The packed per-sweep parameter block (pht_build_params: P/Pfull, dgeevx
  eigensystem, Q^-1 v and the fma precomputes the kernels consume) equals
  the GPU specification in the oracle (orc_sp_build) field by field, and
  the oracle's restatement of LJMA_eigen (reference dgeevx arguments) bit
  for bit.
* Host random stream: R's set.seed/unif_rand/exp_rand/norm_rand published
  values; product and oracle streams identical (rgamma too).
* Device primitives restated on the host: Philox4x32-10 known answers,
  detmath exp/log accuracy (< 1 ulp, specials).
"""
import ctypes as C
import math
import os
import re

import numpy as np
import pytest

import phasetype_amd as P
from phasetype_amd.synth import bd_exit

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


# ------------------------------------------------------------------ the ABI
def _declared_functions():
    src = open(os.path.join(REPO, "include", "phasetype_amd.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    src = "\n".join(ln for ln in src.splitlines() if not ln.lstrip().startswith(("typedef", "#")))
    names = set(re.findall(r"^[A-Za-z_][\w \*]*?\b([A-Za-z_]\w*)\s*\(", src, flags=re.M))
    return names


def test_header_declarations_match_export_list():
    decl = _declared_functions()
    assert decl == set(P.EXPORTS), (decl ^ set(P.EXPORTS))


def test_library_exports_every_declared_symbol(lib):
    for name in _declared_functions():
        assert hasattr(lib, name), name


def test_other_headers_are_self_contained():
    """include/pht_detmath.h and pht_philox.h compile as plain C (the oracle
    includes them) — checked by building the oracle; here: they exist."""
    for h in ("pht_detmath.h", "pht_philox.h"):
        assert os.path.exists(os.path.join(REPO, "include", h))


def _no_gpu():
    try:
        return P.device_count() == 0
    except P.PhaseTypeError:
        return True


@pytest.mark.skipif(not _no_gpu(), reason="a HIP device is present")
def test_no_cpu_fallback_sweeper():
    with pytest.raises(P.PhaseTypeError):
        P.Sweeper(3, 2)


@pytest.mark.skipif(not _no_gpu(), reason="a HIP device is present")
def test_no_cpu_fallback_ljma_gibbs():
    T = np.array([[0, 1, 0], [2, 0, 3], [0, 0, 0]], np.int32)
    with pytest.raises(P.PhaseTypeError):
        P.LJMA_Gibbs(3, 1, 2, 2, 3, [2.0] * 3, [1.0] * 3, T, np.ones((3, 3)), [0.5, 1.0], 2, [0, 0], [-1.0], 1,
                     np.zeros(9))


def test_chains_start_block():
    """gibbs_chains' start: one m-vector broadcast to all K chains, K*m
    values kept, prior draw kept as [-1]; other lengths refused (the C side
    reads start + c*m without a length)."""
    K, m = 3, 4
    assert np.array_equal(P._chains_start(None, K, m), [-1.0])
    assert np.array_equal(P._chains_start([-1.0], K, m), [-1.0])
    one = np.arange(1.0, m + 1)
    assert np.array_equal(P._chains_start(one, K, m), np.tile(one, K))
    per = np.arange(1.0, K * m + 1)
    assert np.array_equal(P._chains_start(per, K, m), per)
    assert np.array_equal(P._chains_start(per.reshape(K, m), K, m), per)
    for bad in (np.ones(m - 1), np.ones(m + 1), np.ones(2 * m)):
        with pytest.raises(ValueError):
            P._chains_start(bad, K, m)


def test_stats_len(lib):
    for n in (1, 3, 10, 32):
        assert lib.pht_stats_len(n) == P.stats_len(n) == 2 * n + n * n + 16


def test_zexp_matches_oracle(lib, orc):
    rng = np.random.default_rng(3)
    for scale in (1e-12, 1e-10, 1e-3, 1.0, 50.0, 1e6):
        for N in (1, 200, 10007):
            y = rng.exponential(scale, N)
            ze = lib.pht_zexp(y, len(y))
            assert ze == orc.lib.orc_zexp(y, len(y))
            # sum(y) * 2^zexp in [2^51, 2^52): totals never overflow, and the
            # quantum 2^-zexp is ~2^-52 of sum(y) at every time scale
            assert 2.0 ** 51 <= y.sum() * 2.0 ** ze < 2.0 ** 52, (scale, N)
    y = rng.exponential(2.0, 1_000_000)
    ze = lib.pht_zexp(y, len(y))
    assert 2.0 ** 51 <= y.sum() * 2.0 ** ze < 2.0 ** 52
    # degenerate sums: a finite, valid exponent, identical in the oracle
    for y in (np.zeros(0), np.zeros(5), np.array([np.inf, 1.0]), np.array([np.nan]), np.array([1e-320])):
        ze = lib.pht_zexp(y, len(y))
        assert ze == orc.lib.orc_zexp(y, len(y)) and -1000 <= ze <= 1000


# --------------------------------------------------- packed parameter block
def _layout(n):
    """Python mirror of phasetype_amd/csrc/pht_layout.h make_layout()."""
    nn = n * n
    o, L = 0, {}
    for name, size in (("evals", n), ("s", n), ("logs", n), ("scale", n), ("logscale", n), ("piQ", n), ("pi", n),
                       ("S", nn), ("P", nn), ("QQs", nn), ("W", nn), ("Wm", 6 * n)):
        L[name] = (o, size)
        o += size
    o += o & 1  # the ECS exact path's prefix ends here (Layout::necs)
    for name, size in (("Pf", nn + n), ("QQ1", nn), ("V", nn), ("Q", nn), ("Qinv", nn)):
        L[name] = (o, size)
        o += size
    o += o & 1
    nd = o
    k, Li = 0, {}
    for name, size in (("nsuccP", n), ("succP", nn), ("nsuccPf", n), ("succPf", nn + n), ("nsuccS", n),
                       ("succS", nn)):
        Li[name] = (k, size)
        k += size
    k = (k + 3) & ~3
    return L, Li, nd * 8 + k * 4, nd


def _orc_sp_struct(M):
    d, i = C.c_double, C.c_int
    fields = [("n", i), ("S", d * (M * M)), ("s", d * M), ("pi", d * M), ("P", d * (M * M)),
              ("Pfull", d * (M * (M + 1))), ("Q", d * (M * M)), ("Qinv", d * (M * M)), ("evals", d * M),
              ("Qinv_s", d * M), ("Qinv_1", d * M), ("eig_info", i), ("QQs", d * (M * M)), ("W", d * (M * M)),
              ("QQ1", d * (M * M)), ("V", d * (M * M)), ("piQ", d * M), ("logs", d * M), ("scale", d * M),
              ("logscale", d * M), ("Wm", d * (M * 6)), ("succP", i * (M * M)), ("nsuccP", i * M), ("succPf", i * (M * (M + 1))),
              ("nsuccPf", i * M), ("succS", i * (M * M)), ("nsuccS", i * M)]
    return type("orc_sp", (C.Structure,), {"_fields_": fields})


def _spview(orc, spbuf):
    St = _orc_sp_struct(orc.maxn)
    return St.from_buffer_copy(spbuf.raw[: C.sizeof(St)])


def _perturbed(n, seed):
    S, s = bd_exit(n)
    rng = np.random.default_rng(seed)
    S = S.copy()
    mask = S > 0
    S[mask] *= rng.uniform(0.7, 1.3, mask.sum())
    s = s * rng.uniform(0.7, 1.3, n)
    s[: n // 2] *= rng.uniform(size=n // 2) < 0.5  # some zero exit rates
    np.fill_diagonal(S, 0.0)
    np.fill_diagonal(S, -(S.sum(1) + s))
    return S, s


@pytest.mark.parametrize("n,method", [(1, 2), (3, 2), (4, 4), (10, 2), (10, 1), (20, 4), (32, 2)])
def test_params_block_equals_gpu_spec(lib, orc, n, method):
    S, s = _perturbed(n, 100 + n)
    L, Li, nbytes, nd = _layout(n)
    assert lib.pht_params_bytes(n) == nbytes
    buf = np.zeros(nbytes, np.uint8)
    info = lib.pht_build_params(n, np.ascontiguousarray(S.reshape(-1, order="F")), s, method,
                                buf.ctypes.data_as(C.c_void_p), nbytes)
    assert info == 0
    dv = buf[: nd * 8].view(np.float64)
    iv = buf[nd * 8:].view(np.int32)
    spbuf, oinfo = orc.sp(S, s, method)
    assert oinfo == 0
    sp = _orc_sp_struct(orc.maxn).from_buffer_copy(spbuf.raw[: C.sizeof(_orc_sp_struct(orc.maxn))])
    assert C.sizeof(_orc_sp_struct(orc.maxn)) == orc.spsize
    eig = bool(method & 6)
    pairs = [("S", "S"), ("s", "s"), ("pi", "pi"), ("P", "P"), ("Pf", "Pfull"), ("logs", "logs"),
             ("scale", "scale"), ("logscale", "logscale")]
    if eig:
        pairs += [("evals", "evals"), ("Q", "Q"), ("Qinv", "Qinv"), ("QQs", "QQs"), ("W", "W"), ("QQ1", "QQ1"),
                  ("V", "V"), ("piQ", "piQ"), ("Wm", "Wm")]
    for mine, theirs in pairs:
        o, size = L[mine]
        want = np.ctypeslib.as_array(getattr(sp, theirs))[:size]
        got = dv[o:o + size]
        assert np.array_equal(got.view(np.uint64), want.view(np.uint64)), mine
    for mine in ("nsuccP", "nsuccPf", "nsuccS"):
        o, size = Li[mine]
        assert np.array_equal(iv[o:o + size], np.ctypeslib.as_array(getattr(sp, mine))[:size]), mine
    M = orc.maxn  # the oracle keeps its lists at row stride MAXN (MAXN + 1 for Pfull)
    for lst, cnt, width, ow in (("succP", "nsuccP", n, M), ("succPf", "nsuccPf", n + 1, M + 1),
                                ("succS", "nsuccS", n, M)):
        o = Li[lst][0]
        want = np.ctypeslib.as_array(getattr(sp, lst))
        counts = iv[Li[cnt][0]:Li[cnt][0] + n]
        for j in range(n):
            k = counts[j]
            assert np.array_equal(iv[o + j * width:o + j * width + k], want[j * ow:j * ow + k]), (lst, j)


@pytest.mark.parametrize("n", [2, 3, 5, 10, 15, 20])
def test_params_eigensystem_equals_reference(lib, orc, n):
    """evals/Q/Qinv are LJMA_eigen's (src/utility.c:87-129) output as the
    oracle restates it (dgeevx with balance 'B', both eigenvector sets and
    sense 'B', then dgetrf/dgetri), bit for bit, over 40 perturbed generators
    per n (the host skips dgeevx's condition numbers and left vectors, which do
    not feed the eigensystem)."""
    L, _, nbytes, nd = _layout(n)
    for seed in range(40):
        S, s = _perturbed(n, 7 * n + 1000 * seed)
        buf = np.zeros(nbytes, np.uint8)
        lib.pht_build_params(n, np.ascontiguousarray(S.reshape(-1, order="F")), s, 2,
                             buf.ctypes.data_as(C.c_void_p), nbytes)
        dv = buf[: nd * 8].view(np.float64)
        sp, info = orc.sp(S, s, 2)
        assert info == 0
        for name in ("evals", "Q", "Qinv"):
            o, size = L[name]
            want = np.ctypeslib.as_array(getattr(_spview(orc, sp), name))[:size]
            assert np.array_equal(dv[o:o + size], want), (name, seed)


@pytest.mark.parametrize("n", [3, 5, 10, 15, 20])
def test_w_moment_polynomial_matches_taylor_sum(lib, orc, n):
    """The ECS starting point y_t - a (device spec r03, pht_wmoments): the
    per-state polynomial sum_k Wm_k x^k equals sum_i W_i taylor5(lambda_i x)
    for |lambda| x <= 2^-8 within 8 ulp of sum_i |W_i| (both sums cancel
    alike; extended-precision reference)."""
    L, _, nbytes, nd = _layout(n)
    for seed in range(5):
        S, s = _perturbed(n, 31 * n + seed)
        buf = np.zeros(nbytes, np.uint8)
        lib.pht_build_params(n, np.ascontiguousarray(S.reshape(-1, order="F")), s, 2,
                             buf.ctypes.data_as(C.c_void_p), nbytes)
        dv = buf[: nd * 8].view(np.float64)
        ev = dv[L["evals"][0]:L["evals"][0] + n]
        W = dv[L["W"][0]:L["W"][0] + n * n].reshape(n, n, order="F")
        Wm = dv[L["Wm"][0]:L["Wm"][0] + 6 * n].reshape(n, 6, order="F")
        lam = np.abs(ev).max()
        for x in (0.0, 1e-9 / lam, 2.0 ** -12 / lam, 2.0 ** -8 / lam):
            for j in range(n):
                poly = 0.0
                for k in range(5, -1, -1):
                    poly = poly * x + Wm[j, k]
                u = np.longdouble(ev) * np.longdouble(x)
                tay = sum(u ** k / np.longdouble(math.factorial(k)) for k in range(6))
                want = float(np.sum(np.longdouble(W[j]) * tay))
                scale = np.abs(W[j]).sum()
                assert abs(poly - want) <= 8 * np.finfo(float).eps * scale + 1e-300, (n, seed, x, j)


# -------------------------------------------------------------- host stream
R_KNOWN = [  # widely published R outputs (Mersenne-Twister, Inversion)
    (1, "unif", [0.2655087, 0.3721239, 0.5728534]),
    (42, "unif", [0.9148060]),
    (123, "unif", [0.2875775]),
    (1, "exp", [0.7551818]),
    (1, "norm", [-0.6264538]),
    (123, "norm", [-0.5604756]),
]


@pytest.mark.parametrize("seed,kind,vals", R_KNOWN)
def test_r_stream_published_values(orc, seed, kind, vals):
    orc.set_seed(seed)
    f = {"unif": orc.lib.orc_unif_rand, "exp": orc.lib.orc_exp_rand, "norm": orc.lib.orc_norm_rand}[kind]
    got = [f() for _ in vals]
    assert np.allclose(got, vals, atol=5e-8, rtol=0), got


def test_product_stream_equals_oracle_stream(lib, orc):
    for seed in (1, 2024, 0xFFFFFFFF):
        lib.pht_set_seed(seed)
        orc.set_seed(seed)
        a = [lib.pht_unif_rand() for _ in range(5000)]
        b = [orc.lib.orc_unif_rand() for _ in range(5000)]
        assert a == b
        g1 = [lib.pht_rgamma(sh, 0.7) for sh in (0.3, 1.0, 2.5, 40.0, 500.0) for _ in range(50)]
        g2 = [orc.lib.orc_rgamma(sh, 0.7) for sh in (0.3, 1.0, 2.5, 40.0, 500.0) for _ in range(50)]
        assert g1 == g2


def test_not_inside_r(lib):
    assert lib.pht_in_R() == 0


# ---------------------------------------------------------- Philox, detmath
PHILOX_KAT = [  # Random123 kat_vectors, philox4x32 R=10
    ((0, 0, 0, 0), (0, 0), (0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8)),
    ((0xFFFFFFFF,) * 4, (0xFFFFFFFF, 0xFFFFFFFF), (0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD)),
    ((0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344), (0xA4093822, 0x299F31D0),
     (0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1)),
]


@pytest.mark.parametrize("ctr,key,want", PHILOX_KAT)
def test_philox_known_answers(orc, ctr, key, want):
    out = np.zeros(4, np.uint32)
    orc.lib.orc_philox(np.array(ctr, np.uint32).ctypes.data_as(C.c_void_p), C.c_uint32(key[0]), C.c_uint32(key[1]),
                       out.ctypes.data_as(C.c_void_p))
    assert tuple(int(v) for v in out) == want


def test_stream_uniforms_open_interval(orc):
    out = np.zeros(100000)
    orc.lib.orc_stream_u(C.c_uint32(1), C.c_uint32(2), C.c_uint32(3), C.c_uint32(0), C.c_uint32(4), C.c_long(len(out)),
                         out.ctypes.data_as(C.c_void_p))
    assert out.min() > 0.0 and out.max() < 1.0
    assert abs(out.mean() - 0.5) < 5 * np.sqrt(1 / 12 / len(out))
    m = np.round(out * 2.0 ** 33)  # (2w+1) 2^-33: odd multiples (one 32-bit word per uniform)
    assert np.all(m % 2 == 1)
    assert len(np.unique(out)) > 0.999 * len(out)


def _ulp_err(got, x, fn):
    xl = x.astype(np.longdouble)
    exact = fn(xl)
    ulp = np.spacing(np.abs(got)).astype(np.longdouble)
    return np.abs((got.astype(np.longdouble) - exact) / ulp)


def test_detmath_exp_accuracy(orc):
    rng = np.random.default_rng(5)
    x = np.concatenate([rng.uniform(-700, 700, 400000), rng.uniform(-1, 1, 200000), rng.uniform(-1e-8, 1e-8, 1000)])
    y = np.zeros_like(x)
    orc.lib.orc_detexp_v(x.ctypes.data_as(C.c_void_p), y.ctypes.data_as(C.c_void_p), C.c_long(len(x)))
    assert _ulp_err(y, x, np.exp).max() < 0.76
    sp = np.array([np.nan, np.inf, -np.inf, 710.0, -746.0, 0.0, -0.0, -740.0])
    out = np.zeros_like(sp)
    orc.lib.orc_detexp_v(sp.ctypes.data_as(C.c_void_p), out.ctypes.data_as(C.c_void_p), C.c_long(len(sp)))
    assert np.isnan(out[0]) and out[1] == np.inf and out[2] == 0.0 and out[3] == np.inf and out[4] == 0.0
    assert out[5] == 1.0 and out[6] == 1.0 and 0 < out[7] < 1e-300  # subnormal result


def test_detmath_exp_flush_below_lo(orc):
    """exp clamps at -1100 and relies on the final ldexp rounding to 0 below
    PHT_EXP_LO = -745.133... (include/pht_detmath.h): every argument between
    -1100 and LO's predecessor gives exactly 0, LO itself the least subnormal."""
    lo = -745.133219101941108420
    below = np.nextafter(lo, -np.inf)
    rng = np.random.default_rng(7)
    x = np.concatenate([rng.uniform(-1100.0, below, 200000),
                        below - np.arange(20000) * np.spacing(745.0), [-1100.0, -1e300, below]])
    y = np.ones_like(x)
    orc.lib.orc_detexp_v(x.ctypes.data_as(C.c_void_p), y.ctypes.data_as(C.c_void_p), C.c_long(len(x)))
    assert np.all(y == 0.0)
    one = np.array([lo])
    orc.lib.orc_detexp_v(one.ctypes.data_as(C.c_void_p), one.ctypes.data_as(C.c_void_p), C.c_long(1))
    assert one[0] == 5e-324


def test_detmath_log_accuracy(orc):
    rng = np.random.default_rng(6)
    x = np.concatenate([np.exp(rng.uniform(-700, 700, 400000)), rng.uniform(0.5, 2.0, 200000),
                        1.0 + rng.uniform(-1e-6, 1e-6, 1000), np.array([5e-324, 1e-310, 2.2250738585072014e-308])])
    y = np.zeros_like(x)
    orc.lib.orc_detlog_v(x.ctypes.data_as(C.c_void_p), y.ctypes.data_as(C.c_void_p), C.c_long(len(x)))
    ok = y != 0
    assert _ulp_err(y[ok], x[ok], np.log).max() < 0.7
    assert np.all(y[~ok] == 0) and np.all(x[~ok] == 1.0)
    sp = np.array([np.nan, -1.0, 0.0, np.inf])
    out = np.zeros_like(sp)
    orc.lib.orc_detlog_v(sp.ctypes.data_as(C.c_void_p), out.ctypes.data_as(C.c_void_p), C.c_long(len(sp)))
    assert np.isnan(out[0]) and np.isnan(out[1]) and out[2] == -np.inf and out[3] == np.inf


def test_log_pos_equals_log_on_the_draws_domain(orc):
    """pht_log_pos (the exponential draws' logarithm, dev_rexp) returns
    pht_log's value bit for bit on positive normal numbers, in particular on
    the 53-bit uniforms (2m + 1) 2^-53 it is given (pht_philox.h pht_u01)."""
    rng = np.random.default_rng(16)
    m = rng.integers(0, 2 ** 52, 500000, dtype=np.uint64)
    u = (2.0 * m.astype(np.float64) + 1.0) * 2.0 ** -53
    x = np.concatenate([u, np.array([2.0 ** -53, 1.0 - 2.0 ** -53, 0.5, 2.0 ** -1022, 1e300, 0.7071067811865476,
                                     0.7071067811865475]), np.exp(rng.uniform(-700, 700, 100000))])
    a, b = np.zeros_like(x), np.zeros_like(x)
    orc.lib.orc_detlog_v(x.ctypes.data_as(C.c_void_p), a.ctypes.data_as(C.c_void_p), C.c_long(len(x)))
    orc.lib.orc_detlogpos_v(x.ctypes.data_as(C.c_void_p), b.ctypes.data_as(C.c_void_p), C.c_long(len(x)))
    assert np.array_equal(a.view(np.uint64), b.view(np.uint64))


def test_philox_key_sources_are_launch_uniform():
    """pht_stream_block reads the key through readfirstlane
    (include/pht_philox.h), which is correct only when every lane of a wave
    uses one key.  Every device call site must take the key from its block's
    SweepArgs (a.k0, a.k1), the resident chain's ResidentArgs (r.k0, r.k1) or
    a function parameter pair (k0, k1) that is itself fed from SweepArgs."""
    import re

    csrc = os.path.join(REPO, "phasetype_amd", "csrc")
    sites = []
    for f in sorted(os.listdir(csrc)):
        if not f.endswith((".h", ".hip")):
            continue
        for m in re.finditer(r"pht_stream_init(?:_block0)?\(\s*[^,]+,\s*([^,]+),\s*([^,]+),", open(os.path.join(csrc, f)).read()):
            sites.append((f, m.group(1).strip(), m.group(2).strip()))
    assert len(sites) >= 10
    for f, k0, k1 in sites:
        assert (k0, k1) in {("a.k0", "a.k1"), ("r.k0", "r.k1"), ("k0", "k1")}, (f, k0, k1)
