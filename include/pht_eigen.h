/*
 * pht_eigen.h — the eigensystem of the sub-generator S for the
 * device-resident Gibbs chain (opt-in, NON-PARITY), shared
 * by the HIP update kernel (pht_resident.hip: one workgroup, the parallel
 * loops spread over its threads) and the oracle's restatement of that chain
 * (oracle/pht_oracle.c, dev = 2: the same loops run serially), so both give
 * the same bits (every translation unit that includes this is compiled with
 * -ffp-contract=off; sqrt and division are IEEE).
 *
 * The reference calls LAPACK dgeevx (balance 'B', right eigenvectors) and
 * inverts Q by LU (src/utility.c:87-129, :50-67).  A LAPACK call cannot run
 * inside a chain that never returns to the host, so this is a restatement of
 * the same method — balancing, Householder reduction to Hessenberg form,
 * Francis double-shift QR with accumulated transformations, back-substitution
 * on the triangular Schur form (the EISPACK balanc / orthes / hqr2 sequence
 * that dgeevx also follows), then Q^-1 by LU with partial pivoting and
 * triangular solves (dgetrf + solve, where the reference calls dgetri).
 * Eigenvalues agree with LAPACK to rounding, not bit for bit; the columns of
 * Q are normalised to unit 2-norm (the spectral products the samplers use,
 * Q diag(.) Q^-1, do not depend on the scaling).
 *
 * Domain: real spectrum.  A complex pair (where the reference warns and goes
 * on with the real parts, src/utility.c:118-120) returns PHT_EIG_COMPLEX and
 * the caller stops the chain (the uniformisation sampler is the path for
 * such generators).  Iteration caps keep every loop finite.
 *
 * Threads: every thread of the workgroup calls pht_eig with the same
 * arguments; scalars are computed redundantly from shared values, the loops
 * marked PHT_EIG_FOR are split over the threads, PHT_EIG_SYNC separates
 * phases.  All arrays in ws must be visible to the whole workgroup (LDS).
 * Storage is column-major, A(i, j) = A[i + j n].
 */
#ifndef PHT_EIGEN_H
#define PHT_EIGEN_H

#include <math.h>

#include "pht_detmath.h" /* PHT_HD */

#if defined(__HIP_DEVICE_COMPILE__)
#define PHT_EIG_T0 ((int)threadIdx.x)
#define PHT_EIG_NT ((int)blockDim.x)
#define PHT_EIG_SYNC() __syncthreads()
#else
#define PHT_EIG_T0 0
#define PHT_EIG_NT 1
#define PHT_EIG_SYNC() ((void)0)
#endif
#define PHT_EIG_FOR(v, lo, hi) for (int v = (lo) + PHT_EIG_T0; v < (hi); v += PHT_EIG_NT)
#define PHT_EIG_ONE if (PHT_EIG_T0 == 0)

#define PHT_EIG_OK 0
#define PHT_EIG_COMPLEX 1  /* a complex-conjugate pair */
#define PHT_EIG_NOCONV 2   /* QR iteration cap (30 per eigenvalue, at least 300) */
#define PHT_EIG_SINGULAR 3 /* eigenvector matrix singular (defective S) */

typedef struct {
  double *H, *V, *X; /* n*n each: Hessenberg/Schur form, transformations, triangular eigenvectors */
  double *G;         /* 2 n*n: the LU factors of Q, then the row permutation */
  double *ort, *scale, *d; /* n each */
} pht_eig_ws;

#define PHT_EIG_EPS 2.220446049250313080847e-16 /* 2^-52 */

/* Balancing by powers of 2 (EISPACK balanc without the permutations):
 * D^-1 S D with row and column 1-norms (off the diagonal) made comparable. */
PHT_HD void pht_eig_balance(int n, double *H, double *scale) {
  PHT_EIG_FOR(i, 0, n) scale[i] = 1.0;
  PHT_EIG_SYNC();
  for (int sweep = 0; sweep < 64; sweep++) {
    int noconv = 0;
    for (int i = 0; i < n; i++) {
      double c = 0.0, r = 0.0;
      for (int j = 0; j < n; j++) {
        if (j == i) continue;
        c = c + fabs(H[j + i * n]);
        r = r + fabs(H[i + j * n]);
      }
      if (c == 0.0 || r == 0.0) continue;
      double g = r / 2.0, f = 1.0;
      const double s = c + r;
      for (int k = 0; k < 1100 && c < g; k++) {
        f = f * 2.0;
        c = c * 4.0;
      }
      g = r * 2.0;
      for (int k = 0; k < 1100 && c >= g; k++) {
        f = f / 2.0;
        c = c / 4.0;
      }
      if ((c + r) / f < 0.95 * s) {
        const double gi = 1.0 / f;
        noconv = 1;
        PHT_EIG_SYNC();
        PHT_EIG_ONE scale[i] = scale[i] * f;
        PHT_EIG_FOR(j, 0, n) H[i + j * n] = H[i + j * n] * gi;
        PHT_EIG_SYNC();
        PHT_EIG_FOR(j, 0, n) H[j + i * n] = H[j + i * n] * f;
        PHT_EIG_SYNC();
      }
    }
    if (!noconv) break;
  }
}

/* Householder reduction to upper Hessenberg form (orthes), the
 * transformations accumulated into V */
PHT_HD void pht_eig_hessenberg(int n, double *H, double *V, double *ort) {
  for (int m = 1; m <= n - 2; m++) {
    double sc = 0.0;
    for (int i = m; i < n; i++) sc = sc + fabs(H[i + (m - 1) * n]);
    if (sc == 0.0) continue;
    PHT_EIG_FOR(i, m, n) ort[i] = H[i + (m - 1) * n] / sc;
    PHT_EIG_SYNC();
    double h = 0.0;
    for (int i = n - 1; i >= m; i--) h = h + ort[i] * ort[i];
    double g = sqrt(h);
    if (ort[m] > 0) g = -g;
    h = h - ort[m] * g;
    const double om = ort[m] - g;
    PHT_EIG_SYNC();
    PHT_EIG_ONE ort[m] = om;
    PHT_EIG_SYNC();
    /* H = (I - u u^T / h) H (I - u u^T / h) */
    PHT_EIG_FOR(j, m, n) {
      double f = 0.0;
      for (int i = n - 1; i >= m; i--) f = f + ort[i] * H[i + j * n];
      f = f / h;
      for (int i = m; i < n; i++) H[i + j * n] = H[i + j * n] - f * ort[i];
    }
    PHT_EIG_SYNC();
    PHT_EIG_FOR(i, 0, n) {
      double f = 0.0;
      for (int j = n - 1; j >= m; j--) f = f + ort[j] * H[i + j * n];
      f = f / h;
      for (int j = m; j < n; j++) H[i + j * n] = H[i + j * n] - f * ort[j];
    }
    PHT_EIG_SYNC();
    PHT_EIG_ONE {
      ort[m] = sc * ort[m];
      H[m + (m - 1) * n] = sc * g;
    }
    PHT_EIG_SYNC();
  }
  PHT_EIG_FOR(e, 0, n * n) V[e] = (e % n == e / n) ? 1.0 : 0.0;
  PHT_EIG_SYNC();
  for (int m = n - 2; m >= 1; m--) {
    const double hm = H[m + (m - 1) * n];
    if (hm == 0.0) continue;
    PHT_EIG_FOR(i, m + 1, n) ort[i] = H[i + (m - 1) * n];
    PHT_EIG_SYNC();
    PHT_EIG_FOR(j, m, n) {
      double g = 0.0;
      for (int i = m; i < n; i++) g = g + ort[i] * V[i + j * n];
      g = (g / ort[m]) / hm; /* double division avoids underflow */
      for (int i = m; i < n; i++) V[i + j * n] = V[i + j * n] + g * ort[i];
    }
    PHT_EIG_SYNC();
  }
}

/* Francis double-shift QR on the Hessenberg H (hqr2's iteration), the
 * eigenvalues into d; on return H is upper triangular (real spectrum) */
PHT_HD int pht_eig_qr(int n, double *H, double *V, double *d) {
  double norm = 0.0;
  for (int i = 0; i < n; i++)
    for (int j = (i > 0 ? i - 1 : 0); j < n; j++) norm = norm + fabs(H[i + j * n]);
  int en = n - 1, iter = 0, total = 0;
  const int cap = 30 * (n > 10 ? n : 10);
  double exshift = 0.0, p = 0.0, q = 0.0, r = 0.0, s = 0.0, z = 0.0, w, x, y;
  while (en >= 0) {
    int l = en;
    while (l > 0) {
      s = fabs(H[(l - 1) + (l - 1) * n]) + fabs(H[l + l * n]);
      if (s == 0.0) s = norm;
      if (fabs(H[l + (l - 1) * n]) < PHT_EIG_EPS * s) break;
      l--;
    }
    if (l == en) { /* one root */
      const double v = H[en + en * n] + exshift;
      PHT_EIG_SYNC();
      PHT_EIG_ONE {
        H[en + en * n] = v;
        d[en] = v;
      }
      PHT_EIG_SYNC();
      en--;
      iter = 0;
    } else if (l == en - 1) { /* two roots */
      w = H[en + (en - 1) * n] * H[(en - 1) + en * n];
      p = (H[(en - 1) + (en - 1) * n] - H[en + en * n]) / 2.0;
      q = p * p + w;
      z = sqrt(fabs(q));
      const double hnn = H[en + en * n] + exshift, hmm = H[(en - 1) + (en - 1) * n] + exshift;
      x = hnn;
      if (q < 0.0) return PHT_EIG_COMPLEX;
      z = (p >= 0) ? p + z : p - z;
      const double d1 = x + z;
      const double d0 = (z != 0.0) ? x - w / z : d1;
      x = H[en + (en - 1) * n];
      s = fabs(x) + fabs(z);
      p = x / s;
      q = z / s;
      r = sqrt(p * p + q * q);
      p = p / r;
      q = q / r;
      PHT_EIG_SYNC();
      PHT_EIG_ONE {
        H[en + en * n] = hnn;
        H[(en - 1) + (en - 1) * n] = hmm;
        d[en - 1] = d1;
        d[en] = d0;
      }
      PHT_EIG_SYNC();
      PHT_EIG_FOR(j, en - 1, n) { /* row modification */
        const double zz = H[(en - 1) + j * n];
        H[(en - 1) + j * n] = q * zz + p * H[en + j * n];
        H[en + j * n] = q * H[en + j * n] - p * zz;
      }
      PHT_EIG_SYNC();
      PHT_EIG_FOR(i, 0, en + 1) { /* column modification */
        const double zz = H[i + (en - 1) * n];
        H[i + (en - 1) * n] = q * zz + p * H[i + en * n];
        H[i + en * n] = q * H[i + en * n] - p * zz;
      }
      PHT_EIG_FOR(i, 0, n) { /* accumulate */
        const double zz = V[i + (en - 1) * n];
        V[i + (en - 1) * n] = q * zz + p * V[i + en * n];
        V[i + en * n] = q * V[i + en * n] - p * zz;
      }
      PHT_EIG_SYNC();
      en -= 2;
      iter = 0;
    } else { /* no convergence yet */
      x = H[en + en * n];
      y = 0.0;
      w = 0.0;
      if (l < en) {
        y = H[(en - 1) + (en - 1) * n];
        w = H[en + (en - 1) * n] * H[(en - 1) + en * n];
      }
      if (iter == 10) { /* Wilkinson's exceptional shift */
        exshift = exshift + x;
        PHT_EIG_SYNC();
        PHT_EIG_FOR(i, 0, en + 1) H[i + i * n] = H[i + i * n] - x;
        PHT_EIG_SYNC();
        s = fabs(H[en + (en - 1) * n]) + fabs(H[(en - 1) + (en - 2) * n]);
        x = y = 0.75 * s;
        w = -0.4375 * s * s;
      }
      if (iter == 30) { /* MATLAB's exceptional shift */
        s = (y - x) / 2.0;
        s = s * s + w;
        if (s > 0) {
          s = sqrt(s);
          if (y < x) s = -s;
          s = x - w / ((y - x) / 2.0 + s);
          PHT_EIG_SYNC();
          PHT_EIG_FOR(i, 0, en + 1) H[i + i * n] = H[i + i * n] - s;
          PHT_EIG_SYNC();
          exshift = exshift + s;
          x = y = w = 0.964;
        }
      }
      iter++;
      if (++total > cap) return PHT_EIG_NOCONV;
      /* two consecutive small subdiagonal elements */
      int m = en - 2;
      while (m >= l) {
        z = H[m + m * n];
        r = x - z;
        s = y - z;
        p = (r * s - w) / H[(m + 1) + m * n] + H[m + (m + 1) * n];
        q = H[(m + 1) + (m + 1) * n] - z - r - s;
        r = H[(m + 2) + (m + 1) * n];
        s = fabs(p) + fabs(q) + fabs(r);
        p = p / s;
        q = q / s;
        r = r / s;
        if (m == l) break;
        if (fabs(H[m + (m - 1) * n]) * (fabs(q) + fabs(r)) <
            PHT_EIG_EPS * (fabs(p) * (fabs(H[(m - 1) + (m - 1) * n]) + fabs(z) + fabs(H[(m + 1) + (m + 1) * n]))))
          break;
        m--;
      }
      PHT_EIG_SYNC();
      PHT_EIG_FOR(i, m + 2, en + 1) {
        H[i + (i - 2) * n] = 0.0;
        if (i > m + 2) H[i + (i - 3) * n] = 0.0;
      }
      PHT_EIG_SYNC();
      /* double QR step on rows l..en, columns m..en */
      for (int k = m; k <= en - 1; k++) {
        const int notlast = (k != en - 1);
        if (k != m) {
          p = H[k + (k - 1) * n];
          q = H[(k + 1) + (k - 1) * n];
          r = notlast ? H[(k + 2) + (k - 1) * n] : 0.0;
          x = fabs(p) + fabs(q) + fabs(r);
          if (x == 0.0) continue;
          p = p / x;
          q = q / x;
          r = r / x;
        }
        s = sqrt(p * p + q * q + r * r);
        if (p < 0) s = -s;
        if (s != 0) {
          const double hk = (k != m) ? -s * x : -H[k + (k - 1) * n];
          PHT_EIG_SYNC();
          if (k != m || l != m) PHT_EIG_ONE H[k + (k - 1) * n] = hk;
          p = p + s;
          x = p / s;
          y = q / s;
          z = r / s;
          q = q / p;
          r = r / p;
          PHT_EIG_SYNC();
          PHT_EIG_FOR(j, k, n) { /* row modification */
            double pp = H[k + j * n] + q * H[(k + 1) + j * n];
            if (notlast) {
              pp = pp + r * H[(k + 2) + j * n];
              H[(k + 2) + j * n] = H[(k + 2) + j * n] - pp * z;
            }
            H[k + j * n] = H[k + j * n] - pp * x;
            H[(k + 1) + j * n] = H[(k + 1) + j * n] - pp * y;
          }
          PHT_EIG_SYNC();
          const int ih = (en < k + 3) ? en : k + 3;
          PHT_EIG_FOR(i, 0, ih + 1) { /* column modification */
            double pp = x * H[i + k * n] + y * H[i + (k + 1) * n];
            if (notlast) {
              pp = pp + z * H[i + (k + 2) * n];
              H[i + (k + 2) * n] = H[i + (k + 2) * n] - pp * r;
            }
            H[i + k * n] = H[i + k * n] - pp;
            H[i + (k + 1) * n] = H[i + (k + 1) * n] - pp * q;
          }
          PHT_EIG_FOR(i, 0, n) { /* accumulate */
            double pp = x * V[i + k * n] + y * V[i + (k + 1) * n];
            if (notlast) {
              pp = pp + z * V[i + (k + 2) * n];
              V[i + (k + 2) * n] = V[i + (k + 2) * n] - pp * r;
            }
            V[i + k * n] = V[i + k * n] - pp;
            V[i + (k + 1) * n] = V[i + (k + 1) * n] - pp * q;
          }
          PHT_EIG_SYNC();
        }
      }
    }
  }
  return norm == 0.0 ? PHT_EIG_SINGULAR : PHT_EIG_OK;
}

/*
 * evals[n], Q (n x n, right eigenvectors as columns, unit 2-norm) and
 * Qinv = Q^-1 of S.  Returns PHT_EIG_OK or an error code (uniform over the
 * workgroup).  Q and Qinv may be any memory the workgroup can write.
 */
PHT_HD int pht_eig(int n, const double *S, double *evals, double *Q, double *Qinv, pht_eig_ws *w) {
  double *H = w->H, *V = w->V, *X = w->X, *G = w->G, *d = w->d;
  PHT_EIG_FOR(e, 0, n * n) H[e] = S[e];
  PHT_EIG_SYNC();
  pht_eig_balance(n, H, w->scale);
  pht_eig_hessenberg(n, H, V, w->ort);
  int rc = pht_eig_qr(n, H, V, d);
  if (rc != PHT_EIG_OK) return rc;
  double norm = 0.0;
  for (int i = 0; i < n; i++)
    for (int j = i; j < n; j++) norm = norm + fabs(H[i + j * n]);
  /* eigenvectors of the triangular T = H, one per thread */
  PHT_EIG_FOR(en, 0, n) {
    const double lam = d[en];
    for (int i = n - 1; i > en; i--) X[i + en * n] = 0.0;
    X[en + en * n] = 1.0;
    for (int i = en - 1; i >= 0; i--) {
      const double wi = H[i + i * n] - lam;
      double r = 0.0;
      for (int j = i + 1; j <= en; j++) r = r + H[i + j * n] * X[j + en * n];
      X[i + en * n] = (wi != 0.0) ? -r / wi : -r / (PHT_EIG_EPS * norm);
      const double t = fabs(X[i + en * n]);
      if ((PHT_EIG_EPS * t) * t > 1)
        for (int j = i; j <= en; j++) X[j + en * n] = X[j + en * n] / t;
    }
  }
  PHT_EIG_SYNC();
  /* back to S's basis: Q = D V X, columns normalised */
  PHT_EIG_FOR(e, 0, n * n) {
    const int i = e % n, j = e / n;
    double zz = 0.0;
    for (int k = 0; k <= j; k++) zz = zz + V[i + k * n] * X[k + j * n];
    H[e] = w->scale[i] * zz;
  }
  PHT_EIG_SYNC();
  PHT_EIG_FOR(j, 0, n) {
    double ss = 0.0;
    for (int i = 0; i < n; i++) ss = ss + H[i + j * n] * H[i + j * n];
    const double inv = 1.0 / sqrt(ss);
    for (int i = 0; i < n; i++) {
      const double v = H[i + j * n] * inv;
      Q[i + j * n] = v;
      G[i + j * n] = v;
    }
    evals[j] = d[j];
  }
  PHT_EIG_SYNC();
  /* Q^-1: LU with partial pivoting (G = L\U in place, perm in G's second
   * half as doubles), then one forward/back substitution per column of the
   * identity, one column per thread */
  double *piv = G + n * n;
  for (int c = 0; c < n; c++) {
    int pr = c;
    double best = fabs(G[c + c * n]);
    for (int i = c + 1; i < n; i++)
      if (fabs(G[i + c * n]) > best) {
        best = fabs(G[i + c * n]);
        pr = i;
      }
    if (!(best > 0.0)) return PHT_EIG_SINGULAR;
    PHT_EIG_SYNC();
    PHT_EIG_ONE piv[c] = (double)pr;
    if (pr != c) {
      PHT_EIG_FOR(col, 0, n) {
        const double t = G[c + col * n];
        G[c + col * n] = G[pr + col * n];
        G[pr + col * n] = t;
      }
    }
    PHT_EIG_SYNC();
    const double inv = 1.0 / G[c + c * n];
    PHT_EIG_FOR(i, c + 1, n) G[i + c * n] = G[i + c * n] * inv;
    PHT_EIG_SYNC();
    PHT_EIG_FOR(col, c + 1, n) {
      const double u = G[c + col * n];
      for (int i = c + 1; i < n; i++) G[i + col * n] = G[i + col * n] - G[i + c * n] * u;
    }
    PHT_EIG_SYNC();
  }
  PHT_EIG_FOR(k, 0, n) { /* column k of Q^-1: solve L U x = P e_k */
    double *x = Qinv + k * n;
    for (int i = 0; i < n; i++) x[i] = (i == k) ? 1.0 : 0.0;
    for (int c = 0; c < n; c++) { /* the row swaps, in order */
      const int pr = (int)piv[c];
      const double t = x[c];
      x[c] = x[pr];
      x[pr] = t;
    }
    for (int i = 1; i < n; i++) {
      double acc = x[i];
      for (int j = 0; j < i; j++) acc = acc - G[i + j * n] * x[j];
      x[i] = acc;
    }
    for (int i = n - 1; i >= 0; i--) {
      double acc = x[i];
      for (int j = i + 1; j < n; j++) acc = acc - G[i + j * n] * x[j];
      x[i] = acc / G[i + i * n];
    }
  }
  PHT_EIG_SYNC();
  return PHT_EIG_OK;
}

/* ------------------------------------------------------------------
 * Warm start: the resident chain's S moves little from one sweep to the
 * next, so the previous sweep's eigenvectors Q0 (and Qi0 = Q0^-1) nearly
 * diagonalise it.  With B = Zi S Z (Z = Q0, Zi = Qi0 to start), the
 * first-order correction C_ki = B_ki / (B_ii - B_kk) (k != i) updates
 * Z <- Z (I + C), Zi <- (I - C) Zi, then one Newton-Schulz step
 * Zi <- Zi (2I - Z Zi) keeps Zi = Z^-1 to second order; the iteration
 * converges quadratically (3-5 rounds for the per-sweep moves of a Gibbs
 * chain).  Matrix products only: element-parallel, a handful of barriers per
 * round, where the QR iteration is a chain of dependent steps.  Stops when
 * max_{i != j} |B_ij| <= 64 eps max_i |B_ii|, or at its rounding floor (no
 * longer halving, below 1e-12 of the scale: the warm-started eigenvectors
 * then reproduce S to ~1e-12 relative, against ~1e-15 from the QR/LAPACK
 * path; a stall above that falls back to the QR); returns PHT_EIG_NOCONV (the
 * caller runs pht_eig) after PHT_EIG_REFINE_MAX rounds or when two diagonal
 * entries are closer than 2x the largest off-diagonal entry (the first-order
 * step needs |B_ki| well below |B_ii - B_kk|).
 * Outputs as pht_eig; Q is used as scratch until the end.
 */
#define PHT_EIG_REFINE_MAX 12
/* beyond this n the BD-type generators' eigenvector matrices are too
 * ill-conditioned (cond(Q) ~ 5e2 at n = 10) for the per-sweep move to stay
 * a small perturbation in the eigenbasis: measured fallback rates along
 * oracle chains 0-4 % at n <= 6, ~50 % at n = 8, 100 % at n >= 10 */
#define PHT_EIG_REFINE_MAXN 8

/* C = A B (n x n, column-major), element-parallel; each element's sum in
 * four interleaved partial sums (the loads of a step issue together) */
PHT_HD void pht_eig_matmul(int n, const double *A, const double *B, double *C) {
  PHT_EIG_FOR(e, 0, n * n) {
    const int i = e % n, j = e / n;
    double s0 = 0.0, s1 = 0.0, s2 = 0.0, s3 = 0.0;
    int k = 0;
    for (; k + 3 < n; k += 4) {
      s0 = fma(A[i + k * n], B[k + j * n], s0);
      s1 = fma(A[i + (k + 1) * n], B[(k + 1) + j * n], s1);
      s2 = fma(A[i + (k + 2) * n], B[(k + 2) + j * n], s2);
      s3 = fma(A[i + (k + 3) * n], B[(k + 3) + j * n], s3);
    }
    for (; k < n; k++) s0 = fma(A[i + k * n], B[k + j * n], s0);
    C[e] = (s0 + s1) + (s2 + s3);
  }
}

PHT_HD int pht_eig_refine(int n, const double *S, const double *Q0, const double *Qi0, double *evals, double *Q,
                          double *Qinv, pht_eig_ws *w) {
  if (n > PHT_EIG_REFINE_MAXN) return PHT_EIG_NOCONV;
  double *Z = w->V, *Zi = w->X, *T = w->H, *B = w->G, *U = w->G + n * n, *Y = Q;
  double *rowv = w->ort, *rowg = w->scale; /* per row: off-diagonal max, smallest diagonal gap */
  PHT_EIG_FOR(e, 0, n * n) {
    Z[e] = Q0[e];
    Zi[e] = Qi0[e];
  }
  PHT_EIG_SYNC();
  double prev = INFINITY;
  int done = 0;
  for (int it = 0; it <= PHT_EIG_REFINE_MAX; it++) {
    pht_eig_matmul(n, S, Z, T);
    PHT_EIG_SYNC();
    pht_eig_matmul(n, Zi, T, B);
    PHT_EIG_SYNC();
    PHT_EIG_FOR(i, 0, n) {
      double off = 0.0, gap = INFINITY;
      const double di = B[i + i * n];
      for (int k = 0; k < n; k++) {
        if (k == i) continue;
        off = fmax(off, fabs(B[i + k * n]));
        gap = fmin(gap, fabs(di - B[k + k * n]));
      }
      rowv[i] = off;
      rowg[i] = gap;
    }
    PHT_EIG_SYNC();
    double off = 0.0, gap = INFINITY, scale = 0.0;
    for (int i = 0; i < n; i++) {
      off = fmax(off, rowv[i]);
      gap = fmin(gap, rowg[i]);
      scale = fmax(scale, fabs(B[i + i * n]));
    }
    if (off <= 64.0 * PHT_EIG_EPS * scale || (off >= 0.5 * prev && off <= 1e-12 * scale)) {
      done = 1;
      break;
    }
    if (it == PHT_EIG_REFINE_MAX || !(gap > 2.0 * off)) return PHT_EIG_NOCONV;
    prev = off;
    PHT_EIG_SYNC();
    /* C (into T): C_ki = B_ki / (B_ii - B_kk), zero diagonal */
    PHT_EIG_FOR(e, 0, n * n) {
      const int k = e % n, i = e / n;
      T[e] = (k == i) ? 0.0 : B[e] / (B[i + i * n] - B[k + k * n]);
    }
    PHT_EIG_SYNC();
    pht_eig_matmul(n, Z, T, U); /* Z C */
    pht_eig_matmul(n, T, Zi, Y); /* C Zi */
    PHT_EIG_SYNC();
    PHT_EIG_FOR(e, 0, n * n) {
      Z[e] = Z[e] + U[e];
      Zi[e] = Zi[e] - Y[e];
    }
    PHT_EIG_SYNC();
    pht_eig_matmul(n, Z, Zi, U); /* Newton-Schulz: Zi (2I - Z Zi) */
    PHT_EIG_SYNC();
    PHT_EIG_FOR(e, 0, n * n) U[e] = ((e % n == e / n) ? 2.0 : 0.0) - U[e];
    PHT_EIG_SYNC();
    pht_eig_matmul(n, Zi, U, Y);
    PHT_EIG_SYNC();
    PHT_EIG_FOR(e, 0, n * n) Zi[e] = Y[e];
    PHT_EIG_SYNC();
  }
  if (!done) return PHT_EIG_NOCONV;
  PHT_EIG_SYNC(); /* every thread has read rowv above */
  /* unit columns of Z, rows of Zi scaled to match */
  PHT_EIG_FOR(j, 0, n) {
    double ss = 0.0;
    for (int i = 0; i < n; i++) ss = ss + Z[i + j * n] * Z[i + j * n];
    rowv[j] = sqrt(ss);
    evals[j] = B[j + j * n];
  }
  PHT_EIG_SYNC();
  PHT_EIG_FOR(e, 0, n * n) {
    const int i = e % n, j = e / n;
    Q[e] = Z[e] / rowv[j];
    Qinv[e] = Zi[e] * rowv[i];
  }
  PHT_EIG_SYNC();
  return PHT_EIG_OK;
}

#endif /* PHT_EIGEN_H */
