"""CPU: the device-resident chain's eigensystem (include/pht_eigen.h, run
serially by the oracle; the HIP update kernel runs the same loops over one
workgroup and tests/test_gpu_resident.py checks the two chains bit for bit).

Checked against LAPACK (numpy) — the reference's LJMA_eigen is dgeevx
(src/utility.c:87-129): eigenvalues to rounding, and the reconstruction
Q diag(lambda) Q^-1 = S within a small multiple of LAPACK's own error on the
same matrix (the BD-exit generators' eigenvector matrices are ill-conditioned:
cond(Q) ~ 5e5 at n = 20).  A complex spectrum is refused (rc 1), where the
reference warns and uses the real parts (src/utility.c:118-120).
"""
import numpy as np
import pytest

from phasetype_amd.synth import bd_exit


def _lapack_err(S):
    w, V = np.linalg.eig(S)
    return np.abs(V @ np.diag(w) @ np.linalg.inv(V) - S).max()


def _check(orc, S):
    rc, ev, Q, Qi = orc.eig(S)
    assert rc == 0
    w = np.linalg.eigvals(S)
    assert np.abs(w.imag).max() == 0.0
    scale = np.abs(w.real).max()
    assert np.allclose(np.sort(ev), np.sort(w.real), rtol=0, atol=64 * np.finfo(float).eps * scale)
    err = np.abs(Q @ np.diag(ev) @ Qi - S).max()
    assert err <= 8 * _lapack_err(S) + 64 * np.finfo(float).eps * scale, (err, _lapack_err(S))
    assert np.allclose(np.linalg.norm(Q, axis=0), 1.0, rtol=1e-14)


@pytest.mark.parametrize("n", [1, 2, 3, 5, 10, 15, 20, 32])
def test_eig_bd_exit(orc, n):
    S, _ = bd_exit(n)
    _check(orc, S)


@pytest.mark.parametrize("n,seed", [(4, 0), (8, 1), (12, 2), (20, 3), (20, 4)])
def test_eig_random_tridiagonal_generators(orc, n, seed):
    """Birth-death sub-generators with random rates over three decades (real
    spectrum: similar to a symmetric matrix); balancing matters here."""
    rng = np.random.default_rng(seed)
    up, dn = 10.0 ** rng.uniform(-1.5, 1.5, n - 1), 10.0 ** rng.uniform(-1.5, 1.5, n - 1)
    S = np.diag(up, 1) + np.diag(dn, -1)
    s = 10.0 ** rng.uniform(-2, 0, n)
    S[np.diag_indices(n)] = -(S.sum(1) + s)
    _check(orc, S)


@pytest.mark.parametrize("n,seed", [(5, 5), (10, 6), (16, 7)])
def test_eig_random_triangular_generators(orc, n, seed):
    """Acyclic (upper-triangular) sub-generators, e.g. Coxian: the spectrum is
    the diagonal; distinct rates."""
    rng = np.random.default_rng(seed)
    S = np.triu(rng.exponential(1.0, (n, n)) * (rng.random((n, n)) < 0.6), 1)
    s = rng.exponential(0.5, n)
    S[np.diag_indices(n)] = -(S.sum(1) + s) - np.arange(n) * 0.37
    _check(orc, S)


def test_eig_complex_spectrum_refused(orc):
    S = np.array([[-10.1, 10.0, 0.0], [0.0, -10.1, 10.0], [10.0, 0.0, -10.1]])
    rc, *_ = orc.eig(S)
    assert rc == 1


def _moved(S, s, rel, rng):
    """S with every rate scaled by exp(rel N(0,1)) (a Gibbs-like move)."""
    n = S.shape[0]
    off = S.copy()
    np.fill_diagonal(off, 0.0)
    off = off * np.exp(rel * rng.standard_normal(off.shape))
    s2 = s * np.exp(rel * rng.standard_normal(n))
    S2 = off.copy()
    np.fill_diagonal(S2, -(off.sum(1) + s2))
    return S2


@pytest.mark.parametrize("n", [2, 3, 5, 8])
def test_eig_refine_warm_start(orc, n):
    """pht_eig_refine: the previous eigensystem refined for a moved S (as the
    resident chain's next sweep does) matches LAPACK like the full QR."""
    rng = np.random.default_rng(n)
    S, s = bd_exit(n)
    rc, ev, Q, Qi = orc.eig(S)
    assert rc == 0
    for rel in (1e-3, 1e-2):
        S2 = _moved(S, s, rel, rng)
        rc2, ev2, Q2, Qi2 = orc.eig_refine(S2, Q, Qi)
        assert rc2 == 0, (n, rel)
        w = np.linalg.eigvals(S2)
        scale = np.abs(w).max()
        assert np.allclose(np.sort(ev2), np.sort(w.real), rtol=0, atol=64 * np.finfo(float).eps * scale)
        err = np.abs(Q2 @ np.diag(ev2) @ Qi2 - S2).max()
        assert err <= 8 * _lapack_err(S2) + 64 * np.finfo(float).eps * scale, err
        assert np.allclose(np.linalg.norm(Q2, axis=0), 1.0, rtol=1e-14)


def test_eig_refine_declines(orc):
    """Beyond PHT_EIG_REFINE_MAXN, or for a move that is not a small
    perturbation in the eigenbasis, the refinement returns 2 (the chain then
    runs the full QR)."""
    S, s = bd_exit(10)
    rc, ev, Q, Qi = orc.eig(S)
    assert orc.eig_refine(S, Q, Qi)[0] == 2
    S, s = bd_exit(3)
    rc, ev, Q, Qi = orc.eig(S)
    S2 = _moved(S, s, 1.5, np.random.default_rng(1))
    assert orc.eig_refine(S2, Q, Qi)[0] in (0, 2)  # converges or declines; never a wrong answer
    rc2, ev2, Q2, Qi2 = orc.eig_refine(S2, Q, Qi)
    if rc2 == 0:
        assert np.abs(Q2 @ np.diag(ev2) @ Qi2 - S2).max() < 1e-12


@pytest.mark.parametrize("n", [3, 5, 8])
def test_eig_refine_accuracy_bound(orc, n):
    """a refinement accepted at its rounding floor (no longer
    halving) must still be accurate: the accepted eigensystem diagonalises
    the moved S to <= 1e-12 of its scale (the stall is accepted only below
    that; above it the chain runs the full QR)."""
    rng = np.random.default_rng(100 + n)
    S, s = bd_exit(n)
    rc, ev, Q, Qi = orc.eig(S)
    for rel in (1e-4, 1e-3, 1e-2, 3e-2):
        S2 = _moved(S, s, rel, rng)
        rc2, ev2, Q2, Qi2 = orc.eig_refine(S2, Q, Qi)
        if rc2 != 0:
            continue
        B = Qi2 @ S2 @ Q2
        scale = np.abs(np.diag(B)).max()
        assert np.abs(B - np.diag(np.diag(B))).max() <= 2e-12 * scale, (n, rel)


@pytest.mark.parametrize("n,N", [(3, 2000), (5, 10000)])
def test_resident_chain_warm_start_rarely_falls_back(orc, n, N):
    """Along the resident chain's own trajectory (oracle gibbs dev=2) the
    warm start converges on nearly every sweep at small n."""
    from phasetype_amd.synth import bd_exit_structure, simulate_ph
    S, s = bd_exit(n)
    T, theta = bd_exit_structure(n)
    y, cen = simulate_ph(S, s, N, seed=3)
    orc.lib.orc_eig_fallback_count()
    orc.set_seed(5)
    it = 150
    ch = orc.gibbs(2, it, 1, 2, n, 1 + 50 * theta, np.full(len(theta), 50.0), T.reshape(-1, order="F"),
                   np.ones(T.size), y, cen)
    assert np.all(np.isfinite(ch))
    assert orc.lib.orc_eig_fallback_count() <= 0.1 * (it - 2)
