/*
 * oracle/pht_oracle.c — TEST INFRASTRUCTURE ONLY (never linked into the
 * product; used by tests/, bench.py's cpu_baseline and smoke()).
 *
 * CPU restatement of the PhaseType Gibbs hot path:
 *   - orc_sp_build: per-sweep embedded-chain and spectral data
 *     (src/PHT_MCMC_Aslett.c:279-297,320-333; src/utility.c:50-129)
 *   - orc_{ref,dev}_sweep: Gibbs step 1 over all observations
 *     (src/PHT_MCMC_Aslett.c:325-337 and the samplers; see pht_oracle_impl.h)
 *   - orc_{ref,dev}_gibbs: the full LJMA_Gibbs (src/PHT_MCMC_Aslett.c:104-410)
 * "ref" = R-stream/libm/reference order (bit-exact with oracle/_ref);
 * "dev" = the GPU specification (bit-exact with the HIP kernels).
 */
#include <dlfcn.h>
#include <float.h>
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "pht_detmath.h"
#include "pht_eigen.h"
#include "pht_gamma.h"
#include "pht_philox.h"
#include "../phasetype_amd/csrc/rstream.h"
#include "pht_oracle.h"

/* the host R stream of both variants (R's global RNG) */
static pht_rstream g_rs;
void orc_set_seed(uint32_t seed) { pht_rs_set_seed(&g_rs, seed); }
double orc_unif_rand(void) { return pht_rs_unif_rand(&g_rs); }
double orc_rgamma(double a, double scale) { return pht_rs_rgamma(&g_rs, a, scale); }
double orc_exp_rand(void) { return pht_rs_exp_rand(&g_rs); }
double orc_norm_rand(void) { return pht_rs_norm_rand(&g_rs); }

/* dev variant's DCS jump-time root finder: 0 = hob_halley (the device
 * spec's default), 1 = Find02 (PHT_DCS_ROOT=brent on the device) */
static int orc_dcs_brent = 0;
/* evaluations per DCS jump of the dev variant's Halley root (histogram,
 * last bin = 63 or more); read and cleared by orc_halley_hist_take */
static long orc_halley_hist[64];
void orc_halley_hist_take(long *out) {
  for (int k = 0; k < 64; k++) {
    if (out) out[k] = orc_halley_hist[k];
    orc_halley_hist[k] = 0;
  }
}
void orc_set_dcs_brent(int on) { orc_dcs_brent = on; }

/* dev variant's bridge modes (PHT_MHRS=bridge / PHT_DCS=bridge on the
 * device): MHRS's / DCS's path law sampled by the uniformisation sampler
 * (phasetype_amd/csrc/pht_unif.h, ulaw 1 / 2) */
static int orc_bridge_mhrs = 0, orc_bridge_dcs = 0;
void orc_set_bridge(int mhrs, int dcs) { orc_bridge_mhrs = mhrs; orc_bridge_dcs = dcs; }

/* ------------------------------------------------------------ variants */
#define ORC_DEV 0
#define ORC_FN(x) orcR_##x
#include "pht_oracle_impl.h"
#undef ORC_DEV
#undef ORC_FN
#undef ORC_EXP
#undef ORC_LOG
#undef ORC_EXP_NEG
#undef ORC_EXP_HI
#undef ORC_EXP_CORE
#define ORC_DEV 1
#define ORC_FN(x) orcD_##x
#include "pht_oracle_impl.h"
#undef ORC_DEV
#undef ORC_FN

/* ------------------------------------------------------------- LAPACK */
typedef void (*dgeevx_t)(const char *, const char *, const char *, const char *, const int *, double *,
                         const int *, double *, double *, double *, const int *, double *, const int *,
                         int *, int *, double *, double *, double *, double *, double *, const int *, int *,
                         int *, size_t, size_t, size_t, size_t);
typedef void (*dgetrf_t)(const int *, const int *, double *, const int *, int *, int *);
typedef void (*dgetri_t)(const int *, double *, const int *, const int *, double *, const int *, int *);
static dgeevx_t p_dgeevx;
static dgetrf_t p_dgetrf;
static dgetri_t p_dgetri;

int orc_bind_lapack(const char *path, const char *prefix) {
  void *h = dlopen(path, RTLD_NOW | RTLD_LOCAL);
  if (!h) return 1;
  char nm[64];
  snprintf(nm, sizeof nm, "%sdgeevx_", prefix); p_dgeevx = (dgeevx_t)dlsym(h, nm);
  snprintf(nm, sizeof nm, "%sdgetrf_", prefix); p_dgetrf = (dgetrf_t)dlsym(h, nm);
  snprintf(nm, sizeof nm, "%sdgetri_", prefix); p_dgetri = (dgetri_t)dlsym(h, nm);
  return (p_dgeevx && p_dgetrf && p_dgetri) ? 0 : 2;
}

/* LJMA_eigen with the LAPACK workspace sized as LJMA_Gibbs sizes it
 * (src/PHT_MCMC_Aslett.c:177-185, src/utility.c:87-129). */
static int orc_eigen(int n, const double *S, double *evals, double *Q, double *Qinv) {
  if (!p_dgeevx) { fprintf(stderr, "oracle: LAPACK not bound\n"); abort(); }
  char balanc = 'B', jobv = 'V', sense = 'B';
  int lwork = -1, info, ilo, ihi, nn = n;
  double wq, abnrm;
  double A[ORC_MAXN * ORC_MAXN], evi[ORC_MAXN], Ql[ORC_MAXN * ORC_MAXN], scl[ORC_MAXN], rce[ORC_MAXN],
      rcv[ORC_MAXN];
  int iwork[4 * ORC_MAXN], ipiv[ORC_MAXN];
  p_dgeevx(&balanc, &jobv, &jobv, &sense, &nn, A, &nn, evals, evi, Ql, &nn, Q, &nn, &ilo, &ihi, scl, &abnrm,
           rce, rcv, &wq, &lwork, NULL, &info, 1, 1, 1, 1);
  int lw = (int)wq;
  p_dgetri(&nn, NULL, &nn, NULL, &wq, &lwork, &info);
  if ((int)wq > lw) lw = (int)wq;
  double *work = (double *)malloc(sizeof(double) * (lw > 0 ? lw : 1));
  memcpy(A, S, sizeof(double) * n * n);
  p_dgeevx(&balanc, &jobv, &jobv, &sense, &nn, A, &nn, evals, evi, Ql, &nn, Q, &nn, &ilo, &ihi, scl, &abnrm,
           rce, rcv, work, &lw, iwork, &info, 1, 1, 1, 1);
  if (info != 0) { free(work); return info; }
  memcpy(Qinv, Q, sizeof(double) * n * n);
  p_dgetrf(&nn, &nn, Qinv, &nn, ipiv, &info);
  if (info == 0) p_dgetri(&nn, Qinv, &nn, ipiv, work, &lw, &info);
  free(work);
  return info;
}

/* the resident chain's eigensystem (include/pht_eigen.h, serial here; the
 * HIP update kernel runs the same loops over one workgroup) */
int orc_eig(int n, const double *S, double *evals, double *Q, double *Qinv) {
  static double H[ORC_MAXN * ORC_MAXN], V[ORC_MAXN * ORC_MAXN], X[ORC_MAXN * ORC_MAXN],
      G[2 * ORC_MAXN * ORC_MAXN], ort[ORC_MAXN], scale[ORC_MAXN], d[ORC_MAXN];
  pht_eig_ws w = {H, V, X, G, ort, scale, d};
  return pht_eig(n, S, evals, Q, Qinv, &w);
}

/* diagnostics: warm starts that fell back to the full QR (tests) */
static long orc_eig_fallbacks = 0;
long orc_eig_fallback_count(void) { long v = orc_eig_fallbacks; orc_eig_fallbacks = 0; return v; }

/* the resident chain's warm start (pht_eig_refine); Q0/Qi0 the previous
 * eigensystem (n x n, column-major) */
int orc_eig_refine(int n, const double *S, const double *Q0, const double *Qi0, double *evals, double *Q, double *Qinv) {
  static double H[ORC_MAXN * ORC_MAXN], V[ORC_MAXN * ORC_MAXN], X[ORC_MAXN * ORC_MAXN],
      G[2 * ORC_MAXN * ORC_MAXN], ort[ORC_MAXN], scale[ORC_MAXN], d[ORC_MAXN];
  pht_eig_ws w = {H, V, X, G, ort, scale, d};
  return pht_eig_refine(n, S, Q0, Qi0, evals, Q, Qinv, &w);
}

/* Per-sweep data (src/PHT_MCMC_Aslett.c:279-297, :320-332) + device-mode
 * precomputed products.  method | ORC_DEVEIG: the eigensystem by orc_eig
 * (the device-resident chain) instead of LAPACK. */
int orc_sp_build(orc_sp *sp, int n, const double *S, const double *s, int method) {
  static double Q0[ORC_MAXN * ORC_MAXN], Qi0[ORC_MAXN * ORC_MAXN];
  const int warm = (method & ORC_DEVEIG) && (method & ORC_DEVEIG_WARM);
  if (warm) {
    memcpy(Q0, sp->Q, sizeof Q0);
    memcpy(Qi0, sp->Qinv, sizeof Qi0);
  }
  memset(sp, 0, sizeof *sp);
  sp->n = n;
  memcpy(sp->S, S, sizeof(double) * n * n);
  memcpy(sp->s, s, sizeof(double) * n);
  sp->pi[0] = 1.0; /* pi = e_1 (src/PHT_MCMC_Aslett.c:190-193) */
  double *P = sp->P, *Pf = sp->Pfull;
  for (int i = 0; i < n; i++) {
    double rsum, rsumfull = 0.0;
    for (int j = 0; j < n; j++) rsumfull += Pf[i + j * n] = P[i + j * n] = -S[i + j * n] / S[i + i * n];
    rsum = rsumfull - P[i + i * n];
    rsumfull += Pf[i + n * n] = -s[i] / S[i + i * n];
    rsumfull -= Pf[i + i * n];
    Pf[i + i * n] = P[i + i * n] = 0.0;
    for (int j = 0; j < n; j++) {
      P[i + j * n] = P[i + j * n] / rsum;
      Pf[i + j * n] = Pf[i + j * n] / rsumfull;
    }
    Pf[i + n * n] = Pf[i + n * n] / rsumfull;
  }
  if (method & (ORC_ECS | ORC_DCS)) {
    if (method & ORC_DEVEIG) {
      int rc = warm ? orc_eig_refine(n, S, Q0, Qi0, sp->evals, sp->Q, sp->Qinv) : PHT_EIG_NOCONV;
      if (rc != PHT_EIG_OK) {
        if (warm && n <= PHT_EIG_REFINE_MAXN) orc_eig_fallbacks++;
        rc = orc_eig(n, S, sp->evals, sp->Q, sp->Qinv);
      }
      sp->eig_info = rc;
    } else {
      sp->eig_info = orc_eigen(n, S, sp->evals, sp->Q, sp->Qinv);
    }
    double one[ORC_MAXN];
    for (int i = 0; i < n; i++) one[i] = 1.0;
    orcR_gemv_n(n, sp->Qinv, s, sp->Qinv_s);
    orcR_gemv_n(n, sp->Qinv, one, sp->Qinv_1);
  }
  /* device-mode products */
  for (int j = 0; j < n; j++) {
    const double Sjj = S[j + j * n];
    sp->logs[j] = s[j] > 0.0 ? pht_log(s[j]) : 0.0;
    sp->scale[j] = 1.0 / -Sjj;
    sp->logscale[j] = pht_log(sp->scale[j]);
    for (int i = 0; i < n; i++) {
      double w = 0.0, v = 0.0;
      for (int k = 0; k < n; k++) {
        if (k != j) w = fma(S[j + k * n] / (-Sjj), sp->Q[k + i * n], w);
        v = fma(P[j + k * n], sp->Q[k + i * n], v);
      }
      sp->QQs[j + i * n] = sp->Q[j + i * n] * sp->Qinv_s[i];
      sp->W[j + i * n] = w * sp->Qinv_s[i];
      sp->QQ1[j + i * n] = sp->Q[j + i * n] * sp->Qinv_1[i];
      sp->V[j + i * n] = v * sp->Qinv_1[i];
    }
  }
  for (int i = 0; i < n; i++) {
    double a = 0.0;
    for (int k = 0; k < n; k++) a = fma(sp->pi[k], sp->Q[k + i * n], a);
    sp->piQ[i] = a;
  }
  for (int j = 0; j < n; j++) { /* the ECS starting point y_t - a (pht_detmath.h) */
    double m[PHT_WMOM];
    pht_wmoments(n, sp->W + j, n, sp->evals, m);
    for (int k = 0; k < PHT_WMOM; k++) sp->Wm[j + k * n] = m[k];
  }
  for (int j = 0; j < n; j++) {
    int a = 0, b = 0, c = 0;
    for (int k = 0; k < n; k++) {
      if (!(P[j + k * n] == 0.0)) sp->succP[j * ORC_MAXN + a++] = k;
      if (k != j && !(S[j + k * n] == 0.0)) sp->succS[j * ORC_MAXN + c++] = k;
    }
    for (int k = 0; k <= n; k++)
      if (!(Pf[j + k * n] == 0.0)) sp->succPf[j * (ORC_MAXN + 1) + b++] = k;
    sp->nsuccP[j] = a; sp->nsuccPf[j] = b; sp->nsuccS[j] = c;
  }
  return sp->eig_info;
}

size_t orc_sp_size(void) { return sizeof(orc_sp); }
int orc_maxn(void) { return ORC_MAXN; }

/* Copy one observation's result into flat per-observation arrays. */
static void put_obs(const orc_obs *o, int n, long i, int *B, int *pre, double *z, int64_t *zq, int *N, int *flags,
                    uint32_t *ndraw) {
  if (B) B[i] = o->B;
  if (pre) pre[i] = o->pre;
  if (flags) flags[i] = o->flags;
  if (ndraw) ndraw[i] = o->ndraw;
  for (int k = 0; k < n; k++) {
    if (z) z[i * n + k] = o->z[k];
    if (zq) zq[i * n + k] = o->zq[k];
  }
  if (N) memcpy(N + i * n * n, o->N, sizeof(int) * n * n);
}

static int dispatch(int method) {
  if (method & ORC_MHRS) return ORC_MHRS;
  if (method & ORC_DCS) return ORC_DCS;
  if (method & ORC_ECS) return ORC_ECS;
  if (method & ORC_UNIF) return ORC_UNIF;
  return 0;
}

/* ------------------------------------------------- UNIF (dev variant only)
 * The uniformisation sampler, restated from its specification in
 * phasetype_amd/csrc/pht_unif.h (no reference counterpart: an opt-in path
 * for generators whose spectrum the reference's eigen-based samplers
 * mishandle, src/utility.c:118-120).  Table layout:
 * [mu, rinv, K, 0][invk K+1][ax K+1][ac K+1][A (K+1) x n]. */
#define ORC_UNIF_MAXK 2047
#define ORC_UNIF_MAXLAM 1300.0
#define ORC_FLAG_UNIF 64

long orc_unif_tab_doubles(int n, int K) { return 4 + 3L * (K + 1) + (long)(K + 1) * n; }

/* the table length the product picks for a shard with largest time ymax */
int orc_unif_K(const orc_sp *sp, double ymax) {
  double mu = 0.0;
  for (int i = 0; i < sp->n; i++) mu = fmax(mu, -sp->S[i + i * sp->n]);
  const double lmax = mu * ymax;
  const double kd = ceil(lmax + 14.0 * sqrt(lmax) + 64.0);
  return (int)(isfinite(kd) && kd < ORC_UNIF_MAXK ? kd : ORC_UNIF_MAXK);
}

void orc_unif_table(const orc_sp *sp, int K, double *T, int ulaw) {
  const int n = sp->n;
  double mu = 0.0;
  for (int i = 0; i < n; i++) {
    const double v = -sp->S[i + i * n];
    mu = (v > mu) ? v : mu;
  }
  const double rinv = 1.0 / mu;
  T[0] = mu; T[1] = rinv; T[2] = (double)K; T[3] = 0.0;
  double *invk = T + 4, *ax = invk + (K + 1), *ac = ax + (K + 1), *A = ac + (K + 1);
  for (int k = 0; k <= K; k++) invk[k] = k ? 1.0 / (double)k : 0.0;
  for (int j = 0; j < n; j++) A[j] = sp->pi[j];
  static double Pm[2][ORC_MAXN * ORC_MAXN];
  for (int j = 0; j < n; j++)
    for (int c = 0; c < n; c++)
      Pm[0][c + j * n] = (c == j) ? fma(sp->S[c + c * n], rinv, 1.0) : sp->S[c + j * n] * rinv;
  int cur = 0;
  for (int p = 1; p <= K; p <<= 1) {
    const int rows = (K - p + 1 < p) ? K - p + 1 : p;
    for (int r = 0; r < rows; r++)
      for (int j = 0; j < n; j++) {
        double acc = 0.0;
        for (int c = 0; c < n; c++) acc = fma(A[(long)r * n + c], Pm[cur][c + j * n], acc);
        A[(long)(p + r) * n + j] = acc;
      }
    if (2 * p <= K)
      for (int j = 0; j < n; j++)
        for (int c = 0; c < n; c++) {
          double acc = 0.0;
          for (int q = 0; q < n; q++) acc = fma(Pm[cur][c + q * n], Pm[cur][q + j * n], acc);
          Pm[cur ^ 1][c + j * n] = acc;
        }
    cur ^= 1;
  }
  for (int k = 0; k <= K; k++) {
    double sx = 0.0, sc = 0.0;
    for (int j = 0; j < n; j++) {
      const double v = A[(long)k * n + j];
      /* ulaw 1 (MHRS bridge): ax = aa, the alive mass in states with exits */
      sx = (ulaw == 1) ? sx + ((sp->s[j] > 0.0) ? v : 0.0) : fma(v, sp->s[j], sx);
      sc = sc + v;
    }
    ax[k] = sx;
    ac[k] = sc;
  }
}

static inline double orc_unif_R(const orc_sp *sp, double rinv, int c, int j) {
  const int n = sp->n;
  return (c == j) ? fma(sp->S[c + c * n], rinv, 1.0) : sp->S[c + j * n] * rinv;
}

/* (k*, j*) from the Poisson weights and row k*'s end weights: e = 0 A s_j
 * (fma), 1 A (add), 2 A 1[s_j > 0] (add) -- pht_unif.h unif_pick */
static void orc_unif_pick(const orc_sp *sp, const double *A, const double *invk, const double *a, double lam,
                          double W, int kend, int e, pht_stream *r, int *ks_out, int *js_out) {
  const int n = sp->n;
  const double target = pht_next_u(r) * W;
  double w = 0x1p-1000, cum = 0.0;
  int k = 0;
  for (;;) {
    cum = fma(w, a[k], cum);
    if (cum >= target || k >= kend) break;
    k++;
    w = w * (lam * invk[k]);
  }
  const int ks = k;
  const double *Ak = A + (long)ks * n;
  const double t2 = pht_next_u(r) * a[ks];
  double c2 = 0.0;
  int js = n - 1;
  for (int j = 0; j < n; j++) {
    c2 = (e == 0) ? fma(Ak[j], sp->s[j], c2) : c2 + ((e == 1 || sp->s[j] > 0.0) ? Ak[j] : 0.0);
    if (c2 >= t2) { js = j; break; }
  }
  *ks_out = ks;
  *js_out = js;
}

static void orc_unif_obs(const orc_sp *sp, const double *T, double y, int cens, pht_stream *r, orc_obs *o,
                         double zscale, int *neval, int ulaw, int mhit) {
  const int n = sp->n;
  const int K = (int)T[2];
  const double mu = T[0], rinv = T[1];
  const double *invk = T + 4, *ax = invk + (K + 1), *ac = ax + (K + 1), *A = ac + (K + 1);
  orcD_obs_clear(o, n);
  if (ulaw == 2) cens = 0; /* DCS treats censored observations as exact */
  const double lam = y * mu;
  const double *a = cens ? ac : ax; /* ulaw 1: ax holds aa */
  int ok = (lam >= 0.0) && (lam <= ORC_UNIF_MAXLAM);
  int kend = 0;
  double W = 0.0;
  if (ok) { /* pass 1: the total weight of (k, j) */
    double w = 0x1p-1000, wmax = 0.0;
    int k = 0;
    for (;;) {
      W = fma(w, a[k], W);
      wmax = (w > wmax) ? w : wmax;
      if (k >= K) { o->flags |= ORC_FLAG_UNIF; break; }
      if ((double)k >= lam && w < wmax * 0x1p-60) break;
      k++;
      w = w * (lam * invk[k]);
    }
    kend = k;
    *neval += k + 1;
    ok = W > 0.0;
  }
  int b = 0, js = 0;
  if (ok) {
    const int e = cens ? 1 : (ulaw == 1 ? 2 : 0);
    int ks;
    orc_unif_pick(sp, A, invk, a, lam, W, kend, e, r, &ks, &js); /* pass 2: (k*, j*) */
    if (ulaw == 1 && !cens) {
      /* MHRS: mhit independence-MH steps, U < s[pre'] / s[pre]
       * (src/Simulate_AbsCTMC_eq_Bladt_MHRS.c:79-82) */
      for (int h = 0; h < mhit; h++) {
        int kp, jp;
        orc_unif_pick(sp, A, invk, a, lam, W, kend, e, r, &kp, &jp);
        const double U = pht_next_u(r);
        if (U < sp->s[jp] / sp->s[js]) { ks = kp; js = jp; }
      }
    }
    b = js;
    double lt = 0.0, tend = y;
    for (int m = ks; m >= 1; m--) { /* the bridge, backward */
      lt = fma(pht_log(pht_next_u(r)), invk[m], lt);
      const double *Am = A + (long)(m - 1) * n;
      const double tot = A[(long)m * n + b]; /* = sum_c A_{m-1}[c] R_cb */
      const double tg = pht_next_u(r) * tot;
      int cs = -1;
      if (tot > 0.0) { /* predecessors of b: R_cb > 0, increasing c */
        int last = -1;
        double cum2 = 0.0;
        for (int c = 0; c < n; c++) {
          const double v = orc_unif_R(sp, rinv, c, b);
          if (!(v > 0.0)) continue;
          cum2 = fma(Am[c], v, cum2);
          if (Am[c] > 0.0) last = c;
          if (cum2 >= tg) { cs = c; break; }
        }
        if (cs < 0) cs = last;
      }
      if (cs < 0) {
        o->flags |= ORC_FLAG_UNIF;
        cs = b;
      }
      if (cs != b) {
        const double tm = y * pht_exp_neg(lt);
        orcD_zadd(o, b, tend - tm, zscale);
        o->N[cs + b * n]++;
        tend = tm;
        b = cs;
      }
    }
    orcD_zadd(o, b, tend, zscale);
  } else {
    o->flags |= ORC_FLAG_UNIF;
    js = 0;
    b = 0;
    orcD_zadd(o, 0, y, zscale);
  }
  o->B = b;
  if (!cens) {
    o->N[js + js * n]++;
    o->pre = js;
    return;
  }
  int j = js; /* censored: on from js at y until absorption */
  for (int nj = 0;; nj++) {
    if (nj >= ORC_MAX_JUMPS) { o->flags |= 8; o->N[j + j * n]++; break; }
    orcD_zadd(o, j, orcD_rexp(r, sp->scale[j]), zscale);
    const double target = pht_next_u(r);
    const int cnt = sp->nsuccPf[j];
    double sofar = 0.0;
    int sel = -1;
    for (int q = 0; q < cnt; q++) {
      const int k = sp->succPf[j * (ORC_MAXN + 1) + q];
      sofar += sp->Pfull[j + k * n];
      if (!(sofar < target)) { sel = k; break; }
    }
    if (sel < 0) {
      o->flags |= 1;
      sel = cnt > 0 ? sp->succPf[j * (ORC_MAXN + 1) + cnt - 1] : n;
    }
    if (sel >= n) { o->N[j + j * n]++; break; }
    o->N[j + sel * n]++;
    j = sel;
  }
  o->pre = j;
}

/*
 * Reference-variant step 1: observations in order on the global R stream.
 * Totals: z_tot[n] (f64, summed per observation as the reference), B_tot[n],
 * N_tot[n*n].  Per-observation arrays may be NULL.  stats[0..3] += jumps-ish
 * counters (ARMS density evaluations, Brent evaluations).
 */
void orc_ref_sweep(const orc_sp *sp, int method, int mhit, const double *y, const int *cens, long l,
                   double *z_tot, int *B_tot, int *N_tot, int *B, int *pre, double *z, int *N, int *flags,
                   uint32_t *nword, long *stats) {
  const int n = sp->n;
  int m = dispatch(method);
  orc_obs o;
  int neval = 0, nbrent = 0;
  for (int k = 0; k < n; k++) { z_tot[k] = 0.0; B_tot[k] = 0; }
  for (int k = 0; k < n * n; k++) N_tot[k] = 0;
  if (m == ORC_UNIF) {
    fprintf(stderr, "oracle: UNIF has no reference-variant (R stream) counterpart\n");
    abort();
  }
  for (long i = 0; i < l; i++) {
    const uint64_t w0 = g_rs.nword;
    if (m == ORC_MHRS) orcR_obs_mhrs(sp, y[i], cens[i], mhit, &g_rs, &o, 0.0);
    else if (m == ORC_DCS) orcR_obs_dcs(sp, y[i], &g_rs, &o, 0.0, &nbrent);
    else if (cens[i]) orcR_obs_censored(sp, y[i], cens[i], &g_rs, &o, 0.0, &neval);
    else orcR_obs_ecs_exact(sp, y[i], &g_rs, &o, 0.0, &neval);
    B_tot[o.B]++;
    for (int k = 0; k < n; k++) z_tot[k] += o.z[k];
    for (int k = 0; k < n * n; k++) N_tot[k] += o.N[k];
    put_obs(&o, n, i, B, pre, z, NULL, N, flags, NULL);
    if (nword) nword[i] = (uint32_t)(g_rs.nword - w0); /* G4: MT words per observation */
  }
  if (stats) { stats[0] += neval; stats[1] += nbrent; }
}

/*
 * Device-variant step 1 (the GPU specification): observation i draws from
 * its own Philox stream (key k0,k1; counter obs=obs0+i, tag 0, sweep).
 * z is reduced as int64 fixed point with quantum 2^-zexp (zq_tot), counts
 * as int64.  obs0 is the global index of y[0] (sharding).
 */
void orc_dev_sweep(const orc_sp *sp, int method, int mhit, const double *y, const int *cens, long l, long obs0,
                   uint32_t k0, uint32_t k1, uint32_t sweep, int zexp, int64_t *zq_tot, int64_t *B_tot,
                   int64_t *N_tot, int *B, int *pre, double *z, int64_t *zq, int *N, int *flags, uint32_t *ndraw,
                   long *stats) {
  const int n = sp->n;
  const double zscale = ldexp(1.0, zexp);
  int m = dispatch(method);
  orc_obs o;
  int neval = 0, nbrent = 0;
  double *utab = NULL;
  /* the uniformisation kernels' path law: UNIF's own, or MHRS's / DCS's in
   * bridge mode */
  const int ulaw = (m == ORC_MHRS && orc_bridge_mhrs) ? 1 : ((m == ORC_DCS && orc_bridge_dcs) ? 2 : 0);
  if (m == ORC_UNIF || ulaw) {
    double ymax = 0.0;
    for (long i = 0; i < l; i++) ymax = fmax(ymax, y[i]);
    const int K = orc_unif_K(sp, ymax);
    utab = (double *)malloc(sizeof(double) * orc_unif_tab_doubles(n, K));
    orc_unif_table(sp, K, utab, ulaw);
  }
  for (int k = 0; k < n; k++) { zq_tot[k] = 0; B_tot[k] = 0; }
  for (int k = 0; k < n * n; k++) N_tot[k] = 0;
  for (long i = 0; i < l; i++) {
    pht_stream r;
    pht_stream_init(&r, k0, k1, (uint32_t)(obs0 + i), 0u, sweep);
    if (m == ORC_UNIF || ulaw) orc_unif_obs(sp, utab, y[i], cens[i], &r, &o, zscale, &neval, ulaw, mhit);
    else if (m == ORC_MHRS) orcD_obs_mhrs(sp, y[i], cens[i], mhit, &r, &o, zscale);
    else if (m == ORC_DCS) orcD_obs_dcs(sp, y[i], &r, &o, zscale, &nbrent);
    else if (cens[i]) orcD_obs_censored(sp, y[i], cens[i], &r, &o, zscale, &neval);
    else orcD_obs_ecs_exact(sp, y[i], &r, &o, zscale, &neval);
    if (m != ORC_MHRS || ulaw) o.ndraw = pht_stream_pos(&r);
    B_tot[o.B]++;
    for (int k = 0; k < n; k++) zq_tot[k] += o.zq[k];
    for (int k = 0; k < n * n; k++) N_tot[k] += o.N[k];
    put_obs(&o, n, i, B, pre, z, zq, N, flags, ndraw);
  }
  free(utab);
  if (stats) { stats[0] += neval; stats[1] += nbrent; }
}

/* fixed-point exponent for z: 52 - e with sum(y) < 2^e;
 * 52 for an empty, zero or non-finite sum; clamped to [-1000, 1000] */
int orc_zexp(const double *y, long l) {
  double sy = 0.0;
  for (long i = 0; i < l; i++) sy += y[i];
  if (!(sy > 0.0) || !isfinite(sy)) return 52;
  int e = 0;
  (void)frexp(sy, &e);
  int z = 52 - e;
  return z > 1000 ? 1000 : (z < -1000 ? -1000 : z);
}

/* ---------------------------------------------------------- Gibbs driver */
typedef struct { int i, j; double c; } ent;

/*
 * LJMA_Gibbs restated (src/PHT_MCMC_Aslett.c:104-410).  dev=0: the sampler
 * step is orc_ref_sweep on the global R stream (the reference's algorithm
 * draw for draw).  dev=1: the sampler step is orc_dev_sweep, keyed by two
 * uniforms drawn from the R stream at entry (k = floor(u * 2^32)), exactly
 * as the product's LJMA_Gibbs does.  dev=2: as dev=1 with the conjugate
 * draws from the counter-based Gamma sampler (include/pht_gamma.h): the
 * product's device-resident chain (pht_gibbs_run_resident).  The linked-list parameter maps are kept
 * as arrays visited in the lists' (reverse-insertion) order, which fixes the
 * floating summation order of zsum and of the diagonal refresh.
 */
/* zexp_in: the fixed-point exponent (dev variants), or ORC_ZEXP_AUTO for
 * orc_zexp(y) as the product's LJMA_Gibbs takes it */
#define ORC_ZEXP_AUTO (-100000)
void orc_gibbs_z(int dev, int it, int mhit, int method, int n, int m, const double *nu, const double *zeta,
                 const int *T, const double *C, const double *y, long l, const int *censored, const double *start,
                 double *res, int zexp_in) {
  const int n1 = n + 1;
  uint32_t k0 = 0, k1 = 0;
  int zexp = 0;
  if (dev) {
    k0 = (uint32_t)(pht_rs_unif_rand(&g_rs) * 4294967296.0);
    k1 = (uint32_t)(pht_rs_unif_rand(&g_rs) * 4294967296.0);
    zexp = zexp_in == ORC_ZEXP_AUTO ? orc_zexp(y, l) : zexp_in;
  }
  double *TT = (double *)calloc((size_t)n1 * n1, sizeof(double));
  double S[ORC_MAXN * ORC_MAXN], s[ORC_MAXN];
  /* per-parameter lists, insertion order (visited in reverse) */
  ent **Nl = (ent **)calloc(m, sizeof(ent *)), **Sl = (ent **)calloc(m, sizeof(ent *)),
      **sl = (ent **)calloc(m, sizeof(ent *)), **zl = (ent **)calloc(m, sizeof(ent *)),
      **TTl = (ent **)calloc(m, sizeof(ent *)), **Dl = (ent **)calloc(n1, sizeof(ent *));
  int *nN = calloc(m, sizeof(int)), *nS = calloc(m, sizeof(int)), *ns = calloc(m, sizeof(int)),
      *nz = calloc(m, sizeof(int)), *nTT = calloc(m, sizeof(int)), *nD = calloc(n1, sizeof(int));
  for (int k = 0; k < m; k++) {
    size_t cap = (size_t)n1 * n1;
    Nl[k] = malloc(cap * sizeof(ent)); Sl[k] = malloc(cap * sizeof(ent)); sl[k] = malloc(cap * sizeof(ent));
    zl[k] = malloc(cap * sizeof(ent)); TTl[k] = malloc(cap * sizeof(ent));
  }
  for (int i = 0; i < n1; i++) Dl[i] = malloc((size_t)n1 * sizeof(ent));

  if (start[0] < 0) {
    for (int i = 0; i < m; i++) {
      if (nu[i] > 1) {
        res[0 + (size_t)i * it] = (nu[i] - 1.0) / zeta[i];
      } else if (dev == 2) {
        pht_stream gs;
        pht_stream_init(&gs, k0, k1, PHT_GAMMA_OBS(i), PHT_GAMMA_TAG, 0u);
        res[0 + (size_t)i * it] = pht_rgamma_ctr(&gs, nu[i], 1.0 / zeta[i]);
      } else {
        res[0 + (size_t)i * it] = pht_rs_rgamma(&g_rs, nu[i], 1.0 / zeta[i]);
      }
    }
  } else {
    for (int i = 0; i < m; i++) res[0 + (size_t)i * it] = start[i];
  }
  double rsum = 0.0;
  for (int i = 0; i < n1; i++) {
    for (int j = 0; j < n1; j++) {
      int t = T[i + j * n1];
      if (t == 0) { TT[i + j * n1] = 0.0; continue; }
      int k = t - 1;
      double c = C[i + j * n1];
      rsum -= TT[i + j * n1] = res[0 + (size_t)k * it] * c;
      if (j == n) {
        Nl[k][nN[k]++] = (ent){i, i, 1.0};
        sl[k][ns[k]++] = (ent){i, 0, c};
      } else {
        Nl[k][nN[k]++] = (ent){i, j, 1.0};
        Sl[k][nS[k]++] = (ent){i, j, c};
      }
      zl[k][nz[k]++] = (ent){i, 0, c};
      TTl[k][nTT[k]++] = (ent){i, j, c};
      Dl[i][nD[i]++] = (ent){i, j, 1.0};
    }
    TT[i + i * n1] = rsum;
    rsum = 0.0;
  }
  for (int i = 0; i < n; i++)
    for (int j = 0; j < n; j++) S[i + j * n] = TT[i + j * n1];
  for (int i = 0; i < n; i++) s[i] = TT[i + n * n1];

  orc_sp *sp = (orc_sp *)malloc(sizeof(orc_sp));
  double z[ORC_MAXN];
  int Bt[ORC_MAXN], Nt[ORC_MAXN * ORC_MAXN];
  int64_t zq[ORC_MAXN], Bq[ORC_MAXN], Nq[ORC_MAXN * ORC_MAXN];
  int *Nsum = calloc(m, sizeof(int));
  double *zsum = calloc(m, sizeof(double));
  int disp = dispatch(method);
  for (int iter = 1; iter < it; iter++) {
    if (!disp) continue; /* "CRITICAL ERROR: Unknown sampling method" */
    orc_sp_build(sp, n, S, s,
                 (disp == ORC_MHRS ? ORC_MHRS : method) | (dev == 2 ? ORC_DEVEIG | (iter > 1 ? ORC_DEVEIG_WARM : 0) : 0));
    if (!dev) {
      orc_ref_sweep(sp, method, mhit, y, censored, l, z, Bt, Nt, NULL, NULL, NULL, NULL, NULL, NULL, NULL);
    } else {
      orc_dev_sweep(sp, method, mhit, y, censored, l, 0, k0, k1, (uint32_t)iter, zexp, zq, Bq, Nq, NULL, NULL,
                    NULL, NULL, NULL, NULL, NULL, NULL);
      for (int k = 0; k < n; k++) z[k] = ldexp((double)zq[k], -zexp);
      for (int k = 0; k < n * n; k++) Nt[k] = (int)Nq[k];
    }
    for (int k = 0; k < m; k++) {
      Nsum[k] = 0;
      zsum[k] = 0.0;
      for (int e = nN[k] - 1; e >= 0; e--) Nsum[k] += Nt[Nl[k][e].i + Nl[k][e].j * n];
      for (int e = nz[k] - 1; e >= 0; e--) zsum[k] += z[zl[k][e].i] / zl[k][e].c;
    }
    for (int k = 0; k < m; k++) {
      double draw;
      if (dev == 2) {
        pht_stream gs;
        pht_stream_init(&gs, k0, k1, PHT_GAMMA_OBS(k), PHT_GAMMA_TAG, (uint32_t)iter);
        draw = pht_rgamma_ctr(&gs, nu[k] + Nsum[k], 1.0 / (zeta[k] + zsum[k]));
      } else {
        draw = pht_rs_rgamma(&g_rs, nu[k] + Nsum[k], 1.0 / (zeta[k] + zsum[k]));
      }
      double tmp = res[iter + (size_t)k * it] = draw;
      for (int e = nTT[k] - 1; e >= 0; e--) TT[TTl[k][e].i + TTl[k][e].j * n1] = tmp * TTl[k][e].c;
      for (int e = nS[k] - 1; e >= 0; e--) S[Sl[k][e].i + Sl[k][e].j * n] = tmp * Sl[k][e].c;
      for (int e = ns[k] - 1; e >= 0; e--) s[sl[k][e].i] = tmp * sl[k][e].c;
    }
    for (int i = 0; i < n; i++) {
      double tmp = 0.0;
      for (int e = nD[i] - 1; e >= 0; e--) tmp -= TT[Dl[i][e].i + Dl[i][e].j * n1];
      TT[i + i * n1] = tmp;
      S[i + i * n] = tmp;
    }
  }
  free(sp); free(Nsum); free(zsum); free(TT);
  for (int k = 0; k < m; k++) { free(Nl[k]); free(Sl[k]); free(sl[k]); free(zl[k]); free(TTl[k]); }
  for (int i = 0; i < n1; i++) free(Dl[i]);
  free(Nl); free(Sl); free(sl); free(zl); free(TTl); free(Dl);
  free(nN); free(nS); free(ns); free(nz); free(nTT); free(nD);
}

void orc_gibbs(int dev, int it, int mhit, int method, int n, int m, const double *nu, const double *zeta,
               const int *T, const double *C, const double *y, long l, const int *censored, const double *start,
               double *res) {
  orc_gibbs_z(dev, it, mhit, method, n, m, nu, zeta, T, C, y, l, censored, start, res, ORC_ZEXP_AUTO);
}

/* primitive probes for tests/test_detmath.py and tests/test_philox.py */
void orc_detexp_v(const double *x, double *y, long n) { for (long i = 0; i < n; i++) y[i] = pht_exp(x[i]); }
void orc_detlog_v(const double *x, double *y, long n) { for (long i = 0; i < n; i++) y[i] = pht_log(x[i]); }
void orc_detlogpos_v(const double *x, double *y, long n) { for (long i = 0; i < n; i++) y[i] = pht_log_pos(x[i]); }
void orc_philox(const uint32_t *ctr, uint32_t k0, uint32_t k1, uint32_t *out) {
  pht_u32x4 c = {{ctr[0], ctr[1], ctr[2], ctr[3]}};
  pht_u32x4 w = pht_philox4x32_10(c, k0, k1);
  for (int i = 0; i < 4; i++) out[i] = w.v[i];
}
void orc_stream_u(uint32_t k0, uint32_t k1, uint32_t obs, uint32_t tag, uint32_t sweep, long cnt, double *out) {
  pht_stream s;
  pht_stream_init(&s, k0, k1, obs, tag, sweep);
  for (long i = 0; i < cnt; i++) out[i] = pht_next_u(&s);
}

/* probe for tests: n Gamma(a, scale) draws from the counter streams
 * (key k0,k1; parameter index i, sweep i) */
void orc_rgamma_ctr_v(uint32_t k0, uint32_t k1, double a, double scale, long cnt, double *out) {
  for (long i = 0; i < cnt; i++) {
    pht_stream s;
    pht_stream_init(&s, k0, k1, PHT_GAMMA_OBS(i & 1023), PHT_GAMMA_TAG, (uint32_t)(i >> 10));
    out[i] = pht_rgamma_ctr(&s, a, scale);
  }
}
