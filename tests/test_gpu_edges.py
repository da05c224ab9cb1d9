"""GPU edge cases, per observation against the oracle's device
specification (oracle/pht_oracle_impl.h, ORC_DEV), bit for bit:
empty and ragged shards (around the 64-lane wavefront and 256-lane block),
one and two transient states, the runtime-n kernels at n = 32 (kMaxN),
zero and tiny absorption times, all-censored data, mhit 0 and 3, and the
multi-kernel MHRS search on a single observation."""
import numpy as np
import pytest

import phasetype_amd as P
from phasetype_amd.synth import bd_exit, bd_exit_structure, simulate_ph

pytestmark = pytest.mark.gpu

FIELDS = ("B", "pre", "flags", "ndraw", "zq", "N")


def _check(orc, n, method, y, cen, mhit=1, key=(3, 5), sweep=2):
    S, s = bd_exit(n)
    y = np.ascontiguousarray(y, np.float64)
    cen = np.ascontiguousarray(cen, np.int32)
    zexp = int(orc.lib.orc_zexp(y, len(y))) if len(y) else 40
    sw = P.Sweeper(n, method, mhit)
    sw.set_obs(y, cen)
    g = sw.sweep_debug(S, s, key=key, sweep=sweep, zexp=zexp)
    st = sw.sweep(S, s, key=key, sweep=sweep, zexp=zexp)
    sw.close()
    L = 2 * n + n * n
    if len(y) == 0:
        assert not np.any(st[:L])
        return
    o = orc.dev_sweep(method, S, s, y, cen, mhit=mhit, key=key, sweep=sweep, zexp=zexp)
    for f in FIELDS:
        assert np.array_equal(g[f], o[f]), (f, n, method)
    assert np.array_equal(st[:L], g["stats"][:L])


@pytest.mark.parametrize("method", [1, 2, 4])
@pytest.mark.parametrize("N", [0, 1, 63, 65, 257])
def test_empty_and_ragged_shards(gpu, orc, method, N):
    S, s = bd_exit(5)
    y, cen = simulate_ph(S, s, N, seed=900 + N, censor_frac=0.3)
    _check(orc, 5, method, y, cen)


@pytest.mark.parametrize("method", [1, 2, 4])
@pytest.mark.parametrize("n", [1, 2, 32])
def test_state_counts(gpu, orc, method, n):
    S, s = bd_exit(n)
    N = 300 if n < 32 else 120
    y, cen = simulate_ph(S, s, N, seed=1000 + n, censor_frac=0.3)
    _check(orc, n, method, y, cen)


@pytest.mark.parametrize("method", [1, 2, 4])
def test_single_state_many_per_lane(gpu, method):
    """n = 1: every path is its start state until absorption at y (no jump,
    every absorb test succeeds), so the statistics are known exactly: B = N,
    N[0,0] = N, zq = sum_i rint(y_i 2^zexp).  300,000 observations give each
    lane of the persistent ECS grid several, so every wavefront's lanes end
    their paths in the same round, round after round (r02 fix: the ECS kernel
    left a wavefront whose lanes had all hit the one-new-observation-per-round
    cap, dropping their next observations)."""
    S, s = bd_exit(1)
    rng = np.random.default_rng(12)
    N = 300_000
    y = rng.exponential(1.0, N)
    cen = np.zeros(N, np.int32)
    zexp = P.zexp_for(y)
    sw = P.Sweeper(1, method, 1)
    sw.set_obs(y, cen)
    st = sw.sweep(S, s, key=(5, 6), sweep=1, zexp=zexp)
    sw.close()
    zq, B, Nt, ex = P.split_stats(st, 1)
    assert ex[0] == N
    assert B[0] == N and Nt[0, 0] == N
    assert zq[0] == int(np.rint(y * 2.0 ** zexp).astype(np.int64).sum())


@pytest.mark.parametrize("method", [1, 2, 4])
def test_zero_and_tiny_times(gpu, orc, method):
    y = np.array([0.0, 1e-300, 1e-12, 1e-6, 0.0, 2.5, 0.0, 1e-9])
    cen = np.array([0, 0, 0, 0, 1, 0, 1, 1], np.int32)
    _check(orc, 4, method, y, cen)


@pytest.mark.parametrize("method", [1, 2, 4])
@pytest.mark.parametrize("scale", [1e-10, 1e3])
def test_time_scale(gpu, orc, method, scale):
    """Data on a sub-nanosecond (or a long) time scale: rates S/scale,
    times y*scale.  Per observation identical to the oracle, and the
    fixed-point z of each exact observation sums back to its y within
    1e-12 relative (pht_zexp follows sum(y), so the quantum scales with
    the data: ADVICE r01)."""
    n = 4
    S0, s0 = bd_exit(n)
    S, s = S0 / scale, s0 / scale
    y, cen = simulate_ph(S0, s0, 300, seed=31, censor_frac=0.3)
    y = np.ascontiguousarray(y * scale)
    zexp = int(orc.lib.orc_zexp(y, len(y)))
    assert zexp == P.zexp_for(y)
    sw = P.Sweeper(n, method, 1)
    sw.set_obs(y, cen)
    g = sw.sweep_debug(S, s, key=(9, 4), sweep=3, zexp=zexp)
    sw.close()
    o = orc.dev_sweep(method, S, s, y, cen, mhit=1, key=(9, 4), sweep=3, zexp=zexp)
    for f in FIELDS:
        assert np.array_equal(g[f], o[f]), f
    ok = (cen == 0) & (g["flags"] == 0) & (y > 0)
    tot = np.ldexp(g["zq"].sum(axis=1).astype(np.float64), -zexp)
    # each sojourn rounds to half a quantum 2^-zexp ~ 2^-52 sum(y); the old
    # fixed floor (quantum 2^-51 time units) was ~1e-6 of y at scale 1e-10
    jumps = g["N"].sum(axis=(1, 2))
    bound = (jumps + 2) * 2.0 ** -zexp + 1e-13 * y
    assert np.all(np.abs(tot[ok] - y[ok]) <= bound[ok])
    assert 2.0 ** -zexp < 1e-14 * y.sum()


@pytest.mark.parametrize("method,n", [(1, 6), (2, 6), (2, 15), (1, 15)])
def test_all_censored(gpu, orc, method, n):
    """(n = 15: the compile-time censored kernel alone, no exact range)"""
    S, s = bd_exit(n)
    y, _ = simulate_ph(S, s, 500, seed=77)
    _check(orc, n, method, y, np.ones(len(y), np.int32))


@pytest.mark.parametrize("mhit,n", [(0, 4), (3, 4), (3, 10)])
def test_mhrs_mhit(gpu, orc, mhit, n):
    S, s = bd_exit(n)
    y, cen = simulate_ph(S, s, 400, seed=31 + mhit, censor_frac=0.2)
    _check(orc, n, 1, y, cen, mhit=mhit)


def test_mhrs_single_hard_observation(gpu, orc):
    """One observation far in the tail (survival ~1e-4): its chains need
    thousands of attempts, found by the wide search rounds."""
    S, s = bd_exit(3)
    y = np.array([9.0])
    _check(orc, 3, 1, y, np.zeros(1, np.int32), mhit=2)


def test_flagged_observations_reported(gpu, capfd):
    """An exact observation no MHRS attempt can reach (survival ~e^-60) hits
    the 2^22-attempt cap in every sweep: the Gibbs run counts it
    (Sweeper.flagged_obs, pht_ctx_flagged_obs) and warns once;
    clean data reports none and prints nothing."""
    n = 3
    S, s = bd_exit(n)
    T, theta = bd_exit_structure(n)
    nu, zeta, Cm = 1 + 50 * theta, np.full(len(theta), 50.0), np.ones(T.shape)
    y, cen = simulate_ph(S, s, 300, seed=4)
    sw = P.Sweeper(n, 1, 1)
    sw.set_obs(y, cen)
    P.set_seed(2)
    sw.gibbs(3, 1, nu, zeta, T, Cm, P.zexp_for(y))
    assert sw.flagged_obs == 0
    assert "WARNING" not in capfd.readouterr().err
    y2 = y.copy()
    y2[7] = 300.0
    sw.set_obs(y2, cen)
    P.set_seed(2)
    sw.gibbs(3, 1, nu, zeta, T, Cm, P.zexp_for(y2))
    sw.close()
    assert sw.flagged_obs == 2  # one observation in each of the 2 sampled sweeps
    err = capfd.readouterr().err
    assert err.count("WARNING") == 1 and "2 observation-sweeps" in err


@pytest.mark.parametrize("n", [1, 2, 3])
def test_every_observation_processed(gpu, orc, n):
    """Short paths (many absorb at their first test, so lanes idle on the
    one-new-observation-per-round rule) over many shard sizes: the kernel's
    observation counter equals N and every observation matches the oracle."""
    S, s = bd_exit(n)
    for N in (2, 5, 17, 64, 65, 130, 300, 1000, 5000):
        y, cen = simulate_ph(S, s, N, seed=3 * N + n)
        y = y * 0.05  # short absorption times: mostly zero-jump paths
        sw = P.Sweeper(n, 2, 1)
        sw.set_obs(y, cen)
        zexp = int(orc.lib.orc_zexp(np.ascontiguousarray(y), len(y)))
        st = sw.sweep(S, s, key=(8, N), sweep=1, zexp=zexp)
        assert st[2 * n + n * n] == N, (N, st[2 * n + n * n])
        g = sw.sweep_debug(S, s, key=(8, N), sweep=1, zexp=zexp)
        o = orc.dev_sweep(2, S, s, y, cen, key=(8, N), sweep=1, zexp=zexp)
        for f in FIELDS:
            assert np.array_equal(g[f], o[f]), (N, f)
        sw.close()


# ------------------------------------------------------- drop-in hardening
def _chain_setup(n=5, N=4000, cf=0.3, seed=61):
    S, s = bd_exit(n)
    T, theta = bd_exit_structure(n)
    y, cen = simulate_ph(S, s, N, seed=seed, censor_frac=cf)
    return T, 1 + 50 * theta, np.full(len(theta), 50.0), np.ones(T.shape), y, cen


@pytest.mark.parametrize("method", [2, 1, 4])
def test_contexts_per_device_keep_the_chain(gpu, monkeypatch, method):
    """LJMA_Gibbs's multi-context loop (PHT_CTX_PER_DEVICE=k shards per
    device, each its own context and streams, all enqueued before any wait,
    statistics summed on the host): the chain is identical for k = 1, 2, 3
    (the in-process path that spreads over several GPUs, exercised on one)."""
    n = 5
    T, nu, zeta, Cm, y, cen = _chain_setup(n, cf=0.3 if method != 4 else 0.0)
    m, it = len(nu), 5
    outs = []
    for k in (1, 2, 3):
        monkeypatch.setenv("PHT_CTX_PER_DEVICE", str(k))
        P.set_seed(777)
        o = P.LJMA_Gibbs(it, 1, method, n, m, nu, zeta, T, Cm, y, len(y), cen, [-1.0], 1, np.zeros(it * m))
        outs.append(o["res"])
    assert np.array_equal(outs[0], outs[1]) and np.array_equal(outs[0], outs[2])
    assert np.all(np.isfinite(outs[0]))


def test_processed_count_guard(gpu):
    """Every sweep checks that the node-wide statistics account for exactly
    the observations: a reduce that sums the block twice (or a shard that
    dropped observations) fails the run loudly instead of biasing it."""
    n = 5
    T, nu, zeta, Cm, y, cen = _chain_setup(n)
    sw = P.Sweeper(n, 2, 1)
    sw.set_obs(y, cen)
    sw.set_global_count(len(y))
    zexp = P.zexp_for(y)
    P.set_seed(5)
    ok = sw.gibbs(3, 2, nu, zeta, T, Cm, zexp, reduce=lambda a: None)  # identity reduce: one shard
    assert np.all(np.isfinite(ok))

    def twice(a):
        a *= 2

    with pytest.raises(P.PhaseTypeError, match="sampled 8000 observations, expected 4000"):
        sw.gibbs(3, 2, nu, zeta, T, Cm, zexp, reduce=twice)
    sw.set_global_count(len(y) + 1)
    with pytest.raises(P.PhaseTypeError, match="expected 4001"):
        sw.gibbs(3, 2, nu, zeta, T, Cm, zexp, reduce=lambda a: None)
    with pytest.raises(P.PhaseTypeError):
        sw.set_global_count(len(y) - 1)
    sw.close()


@pytest.mark.parametrize("method", [2, 1])
def test_fixed_point_overflow_is_an_error(gpu, method):
    """The fixed-point z sums must not wrap.  A zexp whose
    quantum cannot hold the observed times is refused up front; censored
    paths that run ~10^4 times past tiny censoring times (pht_zexp leaves
    2^11-fold headroom over the observed total) cross 2^63 inside the sweep,
    which then fails with an error instead of using a wrapped sum."""
    n = 5
    T, nu, zeta, Cm, y, cen = _chain_setup(n)
    sw = P.Sweeper(n, method, 1)
    sw.set_obs(y, cen)
    P.set_seed(5)
    with pytest.raises(P.PhaseTypeError, match="overflows the fixed-point"):
        sw.gibbs(3, method, nu, zeta, T, Cm, 61)
    y2 = np.full(20000, 1e-4)
    sw.set_obs(y2, np.ones(len(y2), np.int32))
    P.set_seed(5)
    with pytest.raises(P.PhaseTypeError, match="overflowed int64"):
        sw.gibbs(3, method, nu, zeta, T, Cm, P.zexp_for(y2))
    sw.close()


@pytest.mark.parametrize("method", [2, 1, 4])
def test_published_statistics_equal_the_copy_path(gpu, monkeypatch, method):
    """The statistics block reaches the host through pht_stats_out_kernel
    (host-pinned words + a polled flag, gibbs_host.cpp ctx_wait) by default;
    PHT_STATS_COPY=1 (read at context creation) takes the copy + event path.
    Several sweeps of a 30 % censored shard: the same block every sweep (the
    published block is also zeroed for the next sweep by the same kernel)."""
    n = 5
    S, s = bd_exit(n)
    y, cen = simulate_ph(S, s, 3000, seed=11, censor_frac=0.3)
    zexp = P.zexp_for(y)
    out = {}
    for mode in ("pub", "copy"):
        if mode == "copy":
            monkeypatch.setenv("PHT_STATS_COPY", "1")
        else:
            monkeypatch.delenv("PHT_STATS_COPY", raising=False)
        sw = P.Sweeper(n, method, 1)
        sw.set_obs(y, cen)
        out[mode] = [sw.sweep(S, s, key=(7, 9), sweep=k, zexp=zexp).copy() for k in range(1, 5)]
        sw.close()
    for a, b in zip(out["pub"], out["copy"]):
        assert np.array_equal(a, b)
    assert not np.array_equal(out["pub"][0], out["pub"][1])  # different sweeps, different draws


@pytest.mark.parametrize("method", [2, 1, 4])
def test_pipelined_loop_equals_serial(gpu, monkeypatch, method):
    """The pipelined Gibbs loop (gibbs_host.cpp gibbs_run: sweep k + 1
    enqueued behind pht_gate_kernel while sweep k runs) against the serial
    loop (PHT_PIPELINE=0, read at context creation): the same chain, with the
    censored range's concurrent stream (ECS) and the multi-kernel MHRS sweep.
    Then a run that fails at its first sweep's check with the next sweep
    already enqueued (a reduce that double-counts) must release that sweep and
    leave the context usable: the next run equals a fresh context's chain."""
    n = 5
    T, nu, zeta, Cm, y, cen = _chain_setup(n, cf=0.3 if method != 4 else 0.0)
    zexp = P.zexp_for(y)
    res = {}
    for mode in ("serial", "pipe"):
        if mode == "serial":
            monkeypatch.setenv("PHT_PIPELINE", "0")
        else:
            monkeypatch.delenv("PHT_PIPELINE", raising=False)
        sw = P.Sweeper(n, method, 1)
        sw.set_obs(y, cen)
        sw.set_global_count(len(y))  # (checked with a reduce callback too)
        P.set_seed(31)
        res[mode] = sw.gibbs(8, method, nu, zeta, T, Cm, zexp).copy()
        if mode == "pipe":
            def twice(a):
                a *= 2

            P.set_seed(31)
            with pytest.raises(P.PhaseTypeError, match="expected"):
                sw.gibbs(8, method, nu, zeta, T, Cm, zexp, reduce=twice)
            P.set_seed(31)
            again = sw.gibbs(8, method, nu, zeta, T, Cm, zexp)
            assert np.array_equal(again, res["serial"])
        sw.close()
    assert np.array_equal(res["serial"], res["pipe"])
    assert np.all(np.isfinite(res["pipe"]))
