"""GPU parity: the HIP kernels against the oracle's device-spec restatement
(oracle/pht_oracle_impl.h, ORC_DEV), bit for bit, per observation.

Bar: B, pre-absorption state, flags, uniforms consumed, fixed-point z and
the transition counts N are *identical* for every observation; the int64
statistics block is identical.  Sizes are those the CPU oracle finishes in
seconds.  Also: sharding invariance and full Gibbs chains bit-exact against
the oracle's device-variant LJMA_Gibbs.  Statistical agreement with the
reference's algorithm is in test_gpu_posterior.py."""
import numpy as np
import pytest

import phasetype_amd as P
from phasetype_amd.synth import bd_exit, bd_exit_structure, simulate_ph

pytestmark = pytest.mark.gpu

CASES = [
    # (n, N, censor_frac, method, mhit)
    (3, 3000, 0.0, 2, 1), (3, 3000, 0.3, 2, 1), (3, 2000, 0.3, 1, 1), (3, 2000, 0.0, 1, 4), (3, 2000, 0.0, 4, 1),
    (5, 2000, 0.3, 2, 1), (5, 1000, 0.3, 1, 2), (5, 1500, 0.3, 4, 1),
    (10, 2000, 0.3, 2, 1), (10, 1000, 0.3, 1, 1), (10, 1000, 0.0, 4, 1),
    (15, 600, 0.3, 2, 1), (15, 300, 0.3, 1, 1), (15, 300, 0.3, 4, 1),
    # n = 20 censored ECS: the censored kernel's 9-point LDS envelope and its private continuation
    (20, 600, 0.5, 2, 1),
    # the compile-time n = 20 MHRS and DCS kernels (n = 32 in test_gpu_edges.py runs the runtime-n ones)
    (20, 300, 0.3, 1, 1), (20, 300, 0.3, 4, 1),
]


def _perturbed(n, seed):
    S, s = bd_exit(n)
    rng = np.random.default_rng(seed)
    S = S.copy()
    mask = (S > 0)
    S[mask] *= rng.uniform(0.7, 1.3, mask.sum())
    s = s * rng.uniform(0.7, 1.3, n)
    np.fill_diagonal(S, 0.0)
    np.fill_diagonal(S, -(S.sum(1) + s))
    return S, s


@pytest.mark.parametrize("n,N,cf,method,mhit", CASES)
def test_per_observation_bitexact(gpu, orc, n, N, cf, method, mhit):
    S0, s0 = bd_exit(n)
    y, cen = simulate_ph(S0, s0, N, seed=1000 + n, censor_frac=cf)
    S, s = _perturbed(n, n)
    key, sweep = (0x1234567 + n, 0x89ABCDE), 7
    zexp = int(orc.lib.orc_zexp(np.ascontiguousarray(y), len(y)))
    o = orc.dev_sweep(method, S, s, y, cen, mhit=mhit, key=key, sweep=sweep, zexp=zexp)
    sw = P.Sweeper(n, method, mhit)
    sw.set_obs(y, cen)
    g = sw.sweep_debug(S, s, key=key, sweep=sweep, zexp=zexp)
    for f in ("B", "pre", "flags", "ndraw"):
        bad = np.nonzero(g[f] != o[f])[0]
        assert bad.size == 0, f"{f} differs at obs {bad[:5]}: gpu {g[f][bad[:5]]} oracle {o[f][bad[:5]]}"
    bad = np.nonzero(np.any(g["zq"] != o["zq"], axis=1))[0]
    assert bad.size == 0, f"zq differs at obs {bad[:5]}"
    bad = np.nonzero(np.any(g["N"] != o["N"], axis=(1, 2)))[0]
    assert bad.size == 0, f"N differs at obs {bad[:5]}"
    zq, B, Nt, ex = P.split_stats(g["stats"], n)
    assert np.array_equal(zq, o["zq_tot"])
    assert np.array_equal(B, o["B_tot"])
    assert np.array_equal(Nt, o["N_tot"])
    assert ex[0] == N
    # the non-debug kernel produces the same block
    st = sw.sweep(S, s, key=key, sweep=sweep, zexp=zexp)
    assert np.array_equal(st[:2 * n + n * n], g["stats"][:2 * n + n * n])


@pytest.mark.parametrize("n,N,cf", [(3, 2000, 0.0), (10, 1000, 0.3), (15, 300, 0.0), (20, 300, 0.3)])
def test_dcs_brent_root_bitexact(gpu, orc, monkeypatch, n, N, cf):
    """PHT_DCS_ROOT=brent: the jump times by Find02's Brent search (the
    reference's root finder) instead of the default Halley iteration, GPU vs
    the oracle's device spec in the same mode, bit for bit; and the default
    mode lands on the same discrete path with z equal to rounding."""
    S0, s0 = bd_exit(n)
    y, cen = simulate_ph(S0, s0, N, seed=2000 + n, censor_frac=cf)
    S, s = _perturbed(n, n + 1)
    key, sweep = (0x777 + n, 0x31), 3
    zexp = int(orc.lib.orc_zexp(np.ascontiguousarray(y), len(y)))
    monkeypatch.setenv("PHT_DCS_ROOT", "brent")
    orc.set_dcs_brent(True)
    try:
        o = orc.dev_sweep(4, S, s, y, cen, key=key, sweep=sweep, zexp=zexp)
    finally:
        orc.set_dcs_brent(False)
    sw = P.Sweeper(n, 4, 1)
    sw.set_obs(y, cen)
    g = sw.sweep_debug(S, s, key=key, sweep=sweep, zexp=zexp)
    for f in ("B", "pre", "flags", "ndraw", "zq", "N"):
        assert np.array_equal(g[f], o[f]), f
    monkeypatch.delenv("PHT_DCS_ROOT")
    h = sw.sweep_debug(S, s, key=key, sweep=sweep, zexp=zexp)
    sw.close()
    for f in ("B", "pre", "N", "ndraw"):
        assert np.array_equal(h[f], g[f]), f
    assert np.abs(h["zq"] - g["zq"]).max() <= 1e-9 * np.abs(g["zq"]).max()
    # Brent's evaluations (stats word 5) against the Halley iteration's
    assert P.split_stats(h["stats"], n)[3][5] * 2 < P.split_stats(g["stats"], n)[3][5]


@pytest.mark.parametrize("n,N,cf", [(3, 2000, 0.3), (10, 1000, 0.0), (15, 300, 0.3), (20, 300, 0.0)])
def test_dcs_end_state_prepass_bitexact(gpu, orc, monkeypatch, n, N, cf):
    """PHT_DCS_PREPASS=1: the end states from the pre-pass kernel
    (dcs_end_kernel; by default only from 100k observations per shard) give
    the same per-observation results as the oracle, bit for bit."""
    monkeypatch.setenv("PHT_DCS_PREPASS", "1")
    S0, s0 = bd_exit(n)
    y, cen = simulate_ph(S0, s0, N, seed=3000 + n, censor_frac=cf)
    S, s = _perturbed(n, n + 2)
    key, sweep = (0x999 + n, 0x17), 5
    zexp = int(orc.lib.orc_zexp(np.ascontiguousarray(y), len(y)))
    o = orc.dev_sweep(4, S, s, y, cen, key=key, sweep=sweep, zexp=zexp)
    sw = P.Sweeper(n, 4, 1)
    sw.set_obs(y, cen)
    g = sw.sweep_debug(S, s, key=key, sweep=sweep, zexp=zexp)
    st = sw.sweep(S, s, key=key, sweep=sweep, zexp=zexp)
    sw.close()
    for f in ("B", "pre", "flags", "ndraw", "zq", "N"):
        assert np.array_equal(g[f], o[f]), f
    assert np.array_equal(st[:2 * n + n * n], g["stats"][:2 * n + n * n])


@pytest.mark.parametrize("method", [1, 2, 4])
def test_shard_invariance(gpu, method):
    """Two shards (obs0 offsets) sum to the single-shard block exactly."""
    n, N = 6, 4000
    S, s = bd_exit(n)
    y, cen = simulate_ph(S, s, N, seed=77, censor_frac=0.3)
    zexp = P.zexp_for(y)
    full = P.Sweeper(n, method)
    full.set_obs(y, cen)
    a = full.sweep(S, s, key=(5, 6), sweep=3, zexp=zexp)
    parts = []
    for lo, hi in ((0, 1234), (1234, N)):
        sw = P.Sweeper(n, method)
        sw.set_obs(y[lo:hi], cen[lo:hi], obs0=lo)
        parts.append(sw.sweep(S, s, key=(5, 6), sweep=3, zexp=zexp))
    k = 2 * n + n * n
    assert np.array_equal(a[:k], parts[0][:k] + parts[1][:k])


@pytest.mark.parametrize("n", [10, 20])
def test_shard_invariance_rows(gpu, n):
    """With the row blocks active (compiled n, few observations per lane),
    three shards sum to the single-shard block exactly: each shard puts its
    own longest paths on rows."""
    S, s = bd_exit(n)
    N = 9000
    y, cen = simulate_ph(S, s, N, seed=78 + n, censor_frac=0.3)
    zexp = P.zexp_for(y)
    full = P.Sweeper(n, 2)
    full.set_obs(y, cen)
    a = full.sweep(S, s, key=(5, 7), sweep=4, zexp=zexp)
    k = 2 * n + n * n
    tot = np.zeros(k, dtype=a.dtype)
    for lo, hi in ((0, 2345), (2345, 2400), (2400, N)):
        sw = P.Sweeper(n, 2)
        sw.set_obs(y[lo:hi], cen[lo:hi], obs0=lo)
        tot += sw.sweep(S, s, key=(5, 7), sweep=4, zexp=zexp)[:k]
        sw.close()
    assert np.array_equal(a[:k], tot)


@pytest.mark.parametrize("method,n", [(2, 4), (1, 4), (4, 4), (2, 10)])
def test_gibbs_chain_bitexact(gpu, orc, method, n):
    """pht_gibbs_run (GPU step 1 + host Gamma update) == oracle device-variant
    LJMA_Gibbs, every draw of every iteration."""
    T, theta = bd_exit_structure(n)
    S, s = bd_exit(n)
    y, cen = simulate_ph(S, s, 1500, seed=5, censor_frac=0.3 if method != 4 else 0.0)
    m = len(theta)
    nu, zeta = 1 + 50 * theta, np.full(m, 50.0)
    it = 12
    Cm = np.ones_like(T, dtype=np.float64)
    orc.set_seed(2024)
    want = orc.gibbs(1, it, 1, method, n, nu, zeta, T.reshape(-1, order="F"), Cm.reshape(-1, order="F"), y, cen)
    P.set_seed(2024)
    sw = P.Sweeper(n, method, 1)
    sw.set_obs(y, cen)
    got = sw.gibbs(it, method, nu, zeta, T, Cm, P.zexp_for(y))
    assert np.array_equal(got, want), np.abs(got - want).max()
    # the .C entry point over all GPUs gives the same chain
    P.set_seed(2024)
    out = P.LJMA_Gibbs(it, 1, method, n, m, nu, zeta, T, Cm, y, len(y), cen, [-1.0], 1, np.zeros(it * m))
    assert np.array_equal(out["res"].reshape(m, it).T, want)


@pytest.mark.parametrize("occ", [1, 2])
def test_grid_occupancy_invariance(gpu, monkeypatch, occ):
    """Blocks per CU of the persistent kernel (PHT_ECS_OCC) change nothing."""
    n = 10
    S, s = bd_exit(n)
    y, cen = simulate_ph(S, s, 20000, seed=31)
    zexp = P.zexp_for(y)
    sw = P.Sweeper(n, 2)
    sw.set_obs(y, cen)
    ref = sw.sweep(S, s, key=(1, 9), sweep=2, zexp=zexp)
    monkeypatch.setenv("PHT_ECS_OCC", str(occ))
    got = sw.sweep(S, s, key=(1, 9), sweep=2, zexp=zexp)
    assert np.array_equal(ref[:2 * n + n * n], got[:2 * n + n * n])


@pytest.mark.parametrize("knob,value", [("PHT_CENS_SERIAL", "1"), ("PHT_HOT", "500"), ("PHT_NEWCAP", "0"),
                                        ("PHT_SPREAD", "1"), ("PHT_FORCE_NT0", "1"), ("PHT_ROWK", "0"),
                                        ("PHT_ROWK", "64"), ("PHT_ROWK", "100000")])
def test_launch_knobs_invariance(gpu, monkeypatch, knob, value):
    """Launch-shape knobs (serial censored range, wave priority, no new-
    observation cap, lane-major first claims, runtime-n kernels) change no
    statistic: 30 % censored ECS at n = 10.  PHT_FORCE_NT0 is read once per
    process, so it is exercised only if no earlier launch cached it."""
    n = 10
    S, s = bd_exit(n)
    y, cen = simulate_ph(S, s, 20000, seed=37, censor_frac=0.3)
    zexp = P.zexp_for(y)
    sw = P.Sweeper(n, 2)
    sw.set_obs(y, cen)
    ref = sw.sweep(S, s, key=(2, 8), sweep=3, zexp=zexp)
    monkeypatch.setenv(knob, value)
    got = sw.sweep(S, s, key=(2, 8), sweep=3, zexp=zexp)
    sw.close()
    L = 2 * n + n * n
    assert np.array_equal(ref[:L], got[:L])
    assert got[L] == len(y)  # every observation sampled


def _longest_of_million(n, k=4096):
    """The k largest of 10^6 BD-exit(n) absorption times (index order)."""
    S0, s0 = bd_exit(n)
    y, cen = simulate_ph(S0, s0, 1_000_000, seed=4242)
    idx = np.sort(np.argsort(-y)[:k])
    return S0, s0, np.ascontiguousarray(y[idx]), np.ascontiguousarray(cen[idx])


_KEYS = [((5, 6), 2), ((3, 4), 1), ((9, 1), 7), ((11, 12), 3), ((21, 8), 9), ((2, 99), 4), ((40, 41), 6),
         ((7, 77), 8), ((13, 31), 5), ((17, 71), 2), ((23, 32), 11), ((29, 92), 12)]


def _longest_paths_against_oracle(orc, n, tag):
    """(key, sweep) pairs over the 4096 longest of 10^6 paths, per
    observation against the oracle's device spec: at least three pairs, more
    (up to twelve) until the debug launches have counted three rounds whose
    envelope reached private memory.  Returns the general-ARMS and
    private-envelope round counts summed over the pairs run."""
    import json
    import os

    S0, s0, y, cen = _longest_of_million(n)
    zexp = int(orc.lib.orc_zexp(np.ascontiguousarray(y), len(y)))
    sw = P.Sweeper(n, 2, 1)
    sw.set_obs(y, cen)
    general = private = 0
    runs = 0
    for key, sweep in _KEYS:
        if runs >= 3 and private >= 3:
            break
        runs += 1
        o = orc.dev_sweep(2, S0, s0, y, cen, key=key, sweep=sweep, zexp=zexp)
        g = sw.sweep_debug(S0, s0, key=key, sweep=sweep, zexp=zexp)
        bad = np.nonzero((g["ndraw"] != o["ndraw"]) | np.any(g["zq"] != o["zq"], axis=1))[0]
        assert len(bad) == 0, (f"{len(bad)} observations differ, first {bad[:5]}: ndraw gpu "
                               f"{g['ndraw'][bad[:5]]} oracle {o['ndraw'][bad[:5]]} flags {g['flags'][bad[:5]]}")
        for f in ("B", "pre", "flags"):
            assert np.array_equal(g[f], o[f]), f
        assert np.array_equal(g["N"], o["N"])
        ex = P.split_stats(g["stats"], n)[3]
        general += int(ex[P.XDBG_GENERAL])
        private += int(ex[P.XDBG_PRIVATE])
    sw.close()
    path = os.environ.get("PHT_PARITY_REPORT")
    if path:
        with open(path, "a") as f:
            f.write(json.dumps(dict(case=f"longest4096_{tag}_n{n}", key_pairs=runs, general_rounds=general,
                                    private_rounds=private)) + "\n")
    return general, private


@pytest.mark.parametrize("n", [10, 15, 20])
def test_longest_paths_bitexact(gpu, orc, monkeypatch, n):
    """The longest latent paths (the 4096 largest of 1e6 absorption times:
    ~20-50 jumps, envelopes that outgrow the converged code) through the
    one-lane ECS kernel, per observation against the oracle's device
    specification, for three (key, sweep) pairs.  The debug launch counts
    the lane-rounds that ran the general ARMS code and those whose envelope
    reached past the LDS points (13 at n >= 15, 15 at n = 10) into private
    memory: both must occur, so the test proves it drove that continuation
    (src/arms.c:525-621 grows the envelope up to npoint = 100)."""
    monkeypatch.setenv("PHT_ROWK", "0")
    general, private = _longest_paths_against_oracle(orc, n, "lane")
    assert general > 0 and private > 0, (general, private)


@pytest.mark.parametrize("rowk,n,cf", [(10 ** 9, 10, 0.0), (300, 10, 0.3), (10 ** 9, 3, 0.3), (10 ** 9, 5, 0.0),
                                        (777, 15, 0.3), (1, 10, 0.0), (10 ** 9, 20, 0.3), (500, 20, 0.0)])
def test_row_kernel_bitexact(gpu, orc, monkeypatch, rowk, n, cf):
    """The longest exact observations on 16-lane DPP rows (pht_ecs_row.h,
    PHT_ROWK=k: positions [0, k) of the decreasing-y order, at most half
    the resident blocks' worth) give the oracle's device-spec results bit
    for bit, per observation, next to the one-lane blocks of the same
    launch; n = 20 puts two spectral indices in each lane."""
    monkeypatch.setenv("PHT_ROWK", str(rowk))
    S0, s0 = bd_exit(n)
    y, cen = simulate_ph(S0, s0, 3000, seed=3000 + n, censor_frac=cf)
    S, s = _perturbed(n, n + 2)
    zexp = int(orc.lib.orc_zexp(np.ascontiguousarray(y), len(y)))
    o = orc.dev_sweep(2, S, s, y, cen, key=(13, 17), sweep=5, zexp=zexp)
    sw = P.Sweeper(n, 2, 1)
    sw.set_obs(y, cen)
    g = sw.sweep_debug(S, s, key=(13, 17), sweep=5, zexp=zexp)
    for f in ("B", "pre", "flags", "ndraw"):
        bad = np.nonzero(g[f] != o[f])[0]
        assert bad.size == 0, f"{f} differs at obs {bad[:5]}: gpu {g[f][bad[:5]]} oracle {o[f][bad[:5]]}"
    assert np.array_equal(g["zq"], o["zq"]) and np.array_equal(g["N"], o["N"])
    st = sw.sweep(S, s, key=(13, 17), sweep=5, zexp=zexp)
    assert np.array_equal(st[:2 * n + n * n], g["stats"][:2 * n + n * n])
    _, _, _, ex = P.split_stats(st, n)
    assert ex[0] == len(y)


@pytest.mark.parametrize("n", [10, 15, 20])
def test_row_kernel_longest_paths(gpu, orc, monkeypatch, n):
    """The 4096 longest of 1e6 paths all on 16-lane rows, per observation
    against the oracle, for three (key, sweep) pairs; envelopes that outgrow
    the row's 15 points (a fourth rejection in one jump) continue in the
    general ARMS code on a private copy (counted once per row: must occur;
    more key pairs run until it has).  The debug launch takes at most half
    the resident blocks for rows, i.e. the 2048 longest here."""
    monkeypatch.setenv("PHT_ROWK", "4096")
    general, private = _longest_paths_against_oracle(orc, n, "rows")
    assert general > 0 and private == general, (general, private)


@pytest.mark.parametrize("launch", ["one", "streams"])
@pytest.mark.parametrize("method,n,cf", [(2, 5, 0.3), (2, 10, 0.0), (1, 3, 0.3), (4, 3, 0.0), (8, 6, 0.3),
                                         (1, 10, 0.3), (4, 10, 0.0),
                                         # the compile-time n = 15 / 20 chains kernels (cfg5 / cfg3 shapes)
                                         (2, 15, 0.3), (1, 15, 0.3), (4, 15, 0.3), (2, 20, 0.0)])
def test_chains_equal_single_runs(gpu, method, n, cf, launch, monkeypatch):
    """pht_gibbs_run_chains (independent chains on their own contexts,
    streams and host threads): chain c is bit-identical to
    the single chain run after set_seed(seeds[c]).  launch "one": the ECS
    chains' exact ranges go out as one ecs_chains_kernel launch per sweep
    (the default); "streams": one launch per chain on its own stream."""
    if launch == "streams":
        monkeypatch.setenv("PHT_CHAINS_LAUNCH", "streams")
    else:
        monkeypatch.delenv("PHT_CHAINS_LAUNCH", raising=False)
    S, s = bd_exit(n)
    y, cen = simulate_ph(S, s, 3000, seed=77 + n, censor_frac=cf)
    T, theta = bd_exit_structure(n)
    nu, zeta = 1 + 50 * theta, np.full(len(theta), 50.0)
    Cm = np.ones(T.shape)
    seeds = [11, 22, 33, 44]
    got, _ = P.gibbs_chains(seeds, y, cen, n, method, nu, zeta, T, Cm, it=6)
    zexp = P.zexp_for(y)
    sw = P.Sweeper(n, method, 1)
    sw.set_obs(y, cen)
    for c, sd in enumerate(seeds):
        P.set_seed(sd)
        want = sw.gibbs(6, method, nu, zeta, T, Cm, zexp)
        assert np.array_equal(got[c], want), c
    assert not np.array_equal(got[0], got[1])


@pytest.mark.parametrize("per_chain", [False, True])
def test_chains_with_start(gpu, per_chain):
    """A user start: one m-vector is broadcast to every chain, or K*m values
    give each chain its own; chain c equals Sweeper.gibbs from that start."""
    n, method = 5, 2
    S, s = bd_exit(n)
    y, cen = simulate_ph(S, s, 2000, seed=5, censor_frac=0.2)
    T, theta = bd_exit_structure(n)
    m = len(theta)
    nu, zeta = 1 + 50 * theta, np.full(m, 50.0)
    Cm = np.ones(T.shape)
    seeds = [3, 4, 5]
    starts = np.stack([theta * (1.0 + 0.1 * c) for c in range(len(seeds))])
    arg = starts.reshape(-1) if per_chain else starts[0]
    got, _ = P.gibbs_chains(seeds, y, cen, n, method, nu, zeta, T, Cm, it=5, start=arg)
    zexp = P.zexp_for(y)
    sw = P.Sweeper(n, method, 1)
    sw.set_obs(y, cen)
    for c, sd in enumerate(seeds):
        P.set_seed(sd)
        st = starts[c] if per_chain else starts[0]
        want = sw.gibbs(5, method, nu, zeta, T, Cm, zexp, start=st)
        assert np.array_equal(got[c], want), c
        assert np.array_equal(got[c][0], st)


def _run_chains_raw(ctx_list, seeds, it, method, nu, zeta, T, Cm, zexp):
    import ctypes as C

    L = P.load()
    K, m = len(seeds), len(nu)
    ctxs = (C.c_void_p * K)(*ctx_list)
    res = np.zeros(K * it * m, np.float64)
    Tf = np.ascontiguousarray(np.asarray(T).reshape(-1, order="F"), np.int32)
    Cf = np.ascontiguousarray(np.asarray(Cm, np.float64).reshape(-1, order="F"))
    kms = C.c_double(0.0)
    rc = L.pht_gibbs_run_chains(ctxs, K, np.ascontiguousarray(seeds, np.uint32), it, method, m,
                                np.ascontiguousarray(nu, np.float64), np.ascontiguousarray(zeta, np.float64),
                                Tf, Cf, zexp, np.array([-1.0]), res, C.byref(kms))
    assert rc == 0, L.pht_last_error().decode()
    return res.reshape(K, m, it).transpose(0, 2, 1)


def test_chains_one_launch_ragged(gpu, monkeypatch):
    """One launch over 12 ECS chains with different data (sizes 0 .. 20000,
    exact and censored mixes, one chain with no exact observation): each chain
    is bit-identical to its single run.  12 chains exceed the hardware queues
    a launch per stream could use at once."""
    monkeypatch.delenv("PHT_CHAINS_LAUNCH", raising=False)
    n, method, it = 5, 2, 5
    S, s = bd_exit(n)
    T, theta = bd_exit_structure(n)
    nu, zeta = 1 + 50 * theta, np.full(len(theta), 50.0)
    Cm = np.ones(T.shape)
    sizes = [20000, 1, 0, 300, 7000, 64, 65, 4096, 2500, 12000, 3, 999]
    cfs = [0.0, 0.0, 0.0, 0.3, 0.0, 1.0, 0.5, 0.0, 0.2, 0.0, 0.0, 0.1]
    data = [simulate_ph(S, s, k, seed=500 + i, censor_frac=cf) for i, (k, cf) in enumerate(zip(sizes, cfs))]
    zexp = P.zexp_for(np.concatenate([d[0] for d in data]))
    seeds = [1000 + i for i in range(len(sizes))]
    sws = []
    try:
        for y, cen in data:
            sw = P.Sweeper(n, method, 1)
            sw.set_obs(y, cen)
            sws.append(sw)
        got = _run_chains_raw([sw.ctx for sw in sws], seeds, it, method, nu, zeta, T, Cm, zexp)
        for c, sw in enumerate(sws):
            P.set_seed(seeds[c])
            want = sw.gibbs(it, method, nu, zeta, T, Cm, zexp)
            assert np.array_equal(got[c], want), (c, sizes[c])
    finally:
        for sw in sws:
            sw.close()


# ------------------------------------------- the uniformisation sampler (UNIF)
def _cyclic(n, seed=0):
    rng = np.random.default_rng(seed)
    S = np.zeros((n, n))
    for i in range(n):
        S[i, (i + 1) % n] = rng.uniform(1.5, 3.0)
        S[i, (i - 1) % n] += rng.uniform(0.0, 0.2)
    s = rng.uniform(0.1, 0.5, n)
    np.fill_diagonal(S, 0.0)
    np.fill_diagonal(S, -(S.sum(1) + s))
    return S, s


@pytest.mark.parametrize("n,N,cf,gen", [(3, 3000, 0.3, "bd"), (5, 3000, 0.0, "bd"), (10, 4000, 0.3, "bd"),
                                        (15, 2000, 0.3, "bd"), (20, 2000, 0.0, "bd"), (7, 2000, 0.3, "bd"),
                                        (32, 500, 0.3, "bd"), (6, 2000, 0.3, "cyclic"), (12, 2000, 0.0, "cyclic")])
def test_unif_per_observation_bitexact(gpu, orc, n, N, cf, gen):
    """UNIF (pht_unif.h: the per-sweep table kernel + the persistent sampler)
    against the oracle's restatement, per observation: start state, pre-
    absorption state, flags, draws, fixed-point z and N identical; complex
    spectra included (cyclic generators)."""
    S0, s0 = bd_exit(n)
    y, cen = simulate_ph(S0, s0, N, seed=4000 + n, censor_frac=cf)
    S, s = _perturbed(n, n + 3) if gen == "bd" else _cyclic(n)
    key, sweep = (0x51 + n, 0x77), 4
    zexp = int(orc.lib.orc_zexp(np.ascontiguousarray(y), len(y)))
    o = orc.dev_sweep(8, S, s, y, cen, key=key, sweep=sweep, zexp=zexp)
    sw = P.Sweeper(n, 8, 1)
    sw.set_obs(y, cen)
    g = sw.sweep_debug(S, s, key=key, sweep=sweep, zexp=zexp)
    for f in ("B", "pre", "flags", "ndraw"):
        bad = np.nonzero(g[f] != o[f])[0]
        assert bad.size == 0, f"{f} differs at obs {bad[:5]}: gpu {g[f][bad[:5]]} oracle {o[f][bad[:5]]}"
    assert np.array_equal(g["zq"], o["zq"]) and np.array_equal(g["N"], o["N"])
    st = sw.sweep(S, s, key=key, sweep=sweep, zexp=zexp)
    assert np.array_equal(st[:2 * n + n * n], g["stats"][:2 * n + n * n])
    assert P.split_stats(st, n)[3][0] == N
    assert not o["flags"].any()


def test_unif_chain_bitexact(gpu, orc):
    """pht_gibbs_run and LJMA_Gibbs with method 8 == the oracle's UNIF chain."""
    n = 6
    T, theta = bd_exit_structure(n)
    S, s = bd_exit(n)
    y, cen = simulate_ph(S, s, 3000, seed=8, censor_frac=0.3)
    m, it = len(theta), 10
    nu, zeta = 1 + 50 * theta, np.full(m, 50.0)
    Cm = np.ones_like(T, dtype=np.float64)
    orc.set_seed(99)
    want = orc.gibbs(1, it, 1, 8, n, nu, zeta, T.reshape(-1, order="F"), Cm.reshape(-1, order="F"), y, cen)
    P.set_seed(99)
    sw = P.Sweeper(n, 8, 1)
    sw.set_obs(y, cen)
    assert np.array_equal(sw.gibbs(it, 8, nu, zeta, T, Cm, P.zexp_for(y)), want)
    P.set_seed(99)
    out = P.LJMA_Gibbs(it, 1, 8, n, m, nu, zeta, T, Cm, y, len(y), cen, [-1.0], 1, np.zeros(it * m))
    assert np.array_equal(out["res"].reshape(m, it).T, want)


def test_unif_shard_invariance(gpu):
    n, N = 10, 6000
    S, s = bd_exit(n)
    y, cen = simulate_ph(S, s, N, seed=91, censor_frac=0.3)
    zexp = P.zexp_for(y)
    full = P.Sweeper(n, 8)
    full.set_obs(y, cen)
    a = full.sweep(S, s, key=(5, 6), sweep=3, zexp=zexp)
    k = 2 * n + n * n
    tot = np.zeros(k, dtype=a.dtype)
    for lo, hi in ((0, 17), (17, 2500), (2500, N)):
        sw = P.Sweeper(n, 8)
        sw.set_obs(y[lo:hi], cen[lo:hi], obs0=lo)
        tot += sw.sweep(S, s, key=(5, 6), sweep=3, zexp=zexp)[:k]
        sw.close()
    assert np.array_equal(a[:k], tot)


@pytest.mark.parametrize("method,n,mhit", [(1, 4, 2), (4, 5, 1), (8, 5, 1), (2, 5, 1)])
def test_chains_one_launch_against_oracle(gpu, orc, monkeypatch, method, n, mhit):
    """Several chains in one launch sequence (MHRS search/compaction/finish,
    DCS rounds, UNIF table + sampler, ECS exact + censored chains kernels),
    ragged shards (0 .. 6,000 observations, censored mixes), each chain
    compared with the ORACLE's chain for its seed directly (SURVEY.md §8f.4,
    VERDICT r02 item 7)."""
    monkeypatch.delenv("PHT_CHAINS_LAUNCH", raising=False)
    S, s = bd_exit(n)
    T, theta = bd_exit_structure(n)
    m, it = len(theta), 4
    nu, zeta = 1 + 50 * theta, np.full(m, 50.0)
    Cm = np.ones(T.shape)
    sizes, cfs = [6000, 0, 257, 1, 3000], [0.0, 0.0, 0.3, 0.0, 0.5]
    if method == 4:
        cfs = [0.0] * len(sizes)
    data = [simulate_ph(S, s, k, seed=700 + i, censor_frac=cf) for i, (k, cf) in enumerate(zip(sizes, cfs))]
    zexp = P.zexp_for(np.concatenate([d[0] for d in data]))
    seeds = [31 + i for i in range(len(sizes))]
    sws = []
    try:
        for y, cen in data:
            sw = P.Sweeper(n, method, mhit)
            sw.set_obs(y, cen)
            sws.append(sw)
        got = _run_chains_raw([sw.ctx for sw in sws], seeds, it, method, nu, zeta, T, Cm, zexp)
    finally:
        for sw in sws:
            sw.close()
    for c, (y, cen) in enumerate(data):
        orc.set_seed(seeds[c])
        want = _oracle_chain_zexp(orc, it, mhit, method, n, nu, zeta, T, Cm, np.ascontiguousarray(y),
                                  np.ascontiguousarray(cen, np.int32), zexp)
        assert np.array_equal(got[c], want), (c, sizes[c])


def _oracle_chain_zexp(orc, it, mhit, method, n, nu, zeta, T, Cm, y, cen, zexp):
    """orc.gibbs dev=1 at an explicit zexp: the chains share one zexp (from all
    their data); the oracle's LJMA_Gibbs would take its own from y."""
    return orc.gibbs_zexp(1, it, mhit, method, n, nu, zeta, T.reshape(-1, order="F"), Cm.reshape(-1, order="F"), y,
                          cen, zexp)
