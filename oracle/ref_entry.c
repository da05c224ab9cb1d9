/*
 * oracle/ref_entry.c — TEST INFRASTRUCTURE ONLY.
 *
 * Thin C entry points into the reference's own compiled C (built into
 * oracle/_ref/libpht_ref.so from /root/reference/src by oracle/Makefile).
 * They let tests and fixture generators call:
 *   - LJMA_Gibbs (src/PHT_MCMC_Aslett.c:104) exactly as R's .C would, and
 *   - one Gibbs "step 1" (src/PHT_MCMC_Aslett.c:276-337) for a given S/s,
 *     observation by observation, to obtain per-observation (B, z, N).
 * The per-sweep matrices are built here by the same formulas as
 * src/PHT_MCMC_Aslett.c:280-297,320-333; eigen-decomposition, sampling and
 * all arithmetic on the path are the reference's own functions.
 */
#include <stdint.h>

#include "R.h"
#include "R_ext/BLAS.h"

/* reference symbols (prototypes restated from /root/reference/src/*.h) */
void LJMA_Gibbs(int *it, int *mhit, int *method, int *n, int *m, double *nu,
                double *zeta, int *T, double *C, double *y, int *l,
                int *censored, double *start, int *silent, double *res);
void LJMA_LAPACKspace(int *n);
void LJMA_LAPACKspaceFree(void);
int LJMA_eigen(int *n, double *S, double *evals, double *Q, double *Qinv,
               double *workD, int *workI);
void LJMA_MHsample_Bladt(double *y, int *censored, int *m, double *pi, double *S,
                         double *s, double *Pfull, int *n, int *iter,
                         double *res_z, int *res_B, int *res_N, double *workD,
                         int *workI);
void LJMA_MHsample_Aslett2(double *y, int *censored, int *m, double *pi,
                           double *S, double *s, double *Q, double *evals,
                           double *Qinv_s, double *Qinv_1, double *P,
                           double *Pfull, int *n, double *res_z, int *res_B,
                           int *res_N, double *workD, int *workI);
void LJMA_MHsample_Hobolth2(double *y, int *censored, int *m, double *pi,
                            double *S, double *s, double *Q, double *evals,
                            double *Qinv_b, double *bvec, double *Qinv, int *n,
                            int *iter, double *res_z, int *res_B, int *res_N,
                            double *workD, int *workI);
extern int LJMA_counter;
void rshim_free_all(void);

void ref_gibbs(int *it, int *mhit, int *method, int *n, int *m, double *nu,
               double *zeta, int *T, double *C, double *y, int *l, int *censored,
               double *start, int *silent, double *res) {
  LJMA_Gibbs(it, mhit, method, n, m, nu, zeta, T, C, y, l, censored, start,
             silent, res);
  rshim_free_all();
}

/* Spectral data exactly as the Gibbs loop computes it (LJMA_eigen + dgemv). */
int ref_eigen(int n, const double *S, double *evals, double *Q, double *Qinv) {
  int nn = n;
  double *workD = (double *)calloc(100000, sizeof(double));
  int *workI = (int *)calloc(100000, sizeof(int));
  LJMA_LAPACKspace(&nn);
  int info = LJMA_eigen(&nn, (double *)S, evals, Q, Qinv, workD, workI);
  LJMA_LAPACKspaceFree();
  free(workD);
  free(workI);
  return info;
}

/*
 * One step-1 sweep for fixed (S, s), method bitmask as LJMA_Gibbs.
 * per_obs != 0: outputs are per observation — z[l*n], B[l] (start state),
 * N[l*n*n], nd[l] (32-bit MT words drawn; may be NULL) — by calling the
 * sampler once per observation (the samplers keep
 * no state across observations other than the RNG stream, so the draws are
 * identical to one call over all observations).  per_obs == 0: z[n], B[n],
 * N[n*n] are the sampler's own accumulated totals.
 */
unsigned long long rshim_nword(void);
int ref_sweep(int method, int n, const double *S, const double *s, int mhit,
              const double *y, const int *censored, int l, int per_obs,
              double *z, int *B, int *N, unsigned *nd) {
  double *P = (double *)calloc((size_t)n * n, sizeof(double));
  double *Pfull = (double *)calloc((size_t)n * (n + 1), sizeof(double));
  double *Q = (double *)calloc((size_t)n * n, sizeof(double));
  double *Qinv = (double *)calloc((size_t)n * n, sizeof(double));
  double *evals = (double *)calloc(n, sizeof(double));
  double *e = (double *)calloc(n, sizeof(double));
  double *Qinv_s = (double *)calloc(n, sizeof(double));
  double *Qinv_1 = (double *)calloc(n, sizeof(double));
  double *Qinv_b = (double *)calloc(n, sizeof(double));
  double *b = (double *)calloc(n, sizeof(double));
  double *pi = (double *)calloc(n, sizeof(double));
  double *Sc = (double *)malloc(sizeof(double) * n * n);
  double *sc = (double *)malloc(sizeof(double) * n);
  double *workD = (double *)calloc(100000, sizeof(double));
  int *workI = (int *)calloc(100000, sizeof(int));
  int *rB = (int *)calloc(n, sizeof(int));
  int *rN = (int *)calloc((size_t)n * n, sizeof(int));
  double *rz = (double *)calloc(n, sizeof(double));
  memcpy(Sc, S, sizeof(double) * n * n);
  memcpy(sc, s, sizeof(double) * n);
  int nn = n, one = 1, mh = mhit;
  double oneD = 1.0, zeroD = 0.0;
  char transN = 'N';
  pi[0] = 1.0;
  for (int i = 0; i < n; i++) e[i] = 1.0;
  for (int i = 0; i < n; i++) b[i] = sc[i] > 0.0 ? 1.0 : 0.0;
  /* P / Pfull (src/PHT_MCMC_Aslett.c:280-297) */
  for (int i = 0; i < n; i++) {
    double rsum, rsumfull = 0.0;
    for (int j = 0; j < n; j++)
      rsumfull += Pfull[i + j * n] = P[i + j * n] = -Sc[i + j * n] / Sc[i + i * n];
    rsum = rsumfull - P[i + i * n];
    rsumfull += Pfull[i + n * n] = -sc[i] / Sc[i + i * n];
    rsumfull -= Pfull[i + i * n];
    Pfull[i + i * n] = P[i + i * n] = 0.0;
    for (int j = 0; j < n; j++) {
      P[i + j * n] = P[i + j * n] / rsum;
      Pfull[i + j * n] = Pfull[i + j * n] / rsumfull;
    }
    Pfull[i + n * n] = Pfull[i + n * n] / rsumfull;
  }
  int info = 0;
  if (method & 0x6) {
    LJMA_LAPACKspace(&nn);
    info = LJMA_eigen(&nn, Sc, evals, Q, Qinv, workD, workI);
    LJMA_LAPACKspaceFree();
  }
  if (method & 0x1) {
  } else if (method & 0x4) {
    dgemv_(&transN, &nn, &nn, &oneD, Qinv, &nn, b, &one, &zeroD, Qinv_b, &one, 1);
  } else if (method & 0x2) {
    dgemv_(&transN, &nn, &nn, &oneD, Qinv, &nn, sc, &one, &zeroD, Qinv_s, &one, 1);
    dgemv_(&transN, &nn, &nn, &oneD, Qinv, &nn, e, &one, &zeroD, Qinv_1, &one, 1);
  }
  int chunks = per_obs ? l : 1;
  for (int c = 0; c < chunks; c++) {
    int mm = per_obs ? 1 : l;
    double *yp = (double *)y + (per_obs ? c : 0);
    int *cp = (int *)censored + (per_obs ? c : 0);
    const unsigned long long w0 = rshim_nword();
    if (method & 0x1)
      LJMA_MHsample_Bladt(yp, cp, &mm, pi, Sc, sc, Pfull, &nn, &mh, rz, rB, rN, workD, workI);
    else if (method & 0x4)
      LJMA_MHsample_Hobolth2(yp, cp, &mm, pi, Sc, sc, Q, evals, Qinv_b, b, Qinv, &nn, &mh, rz, rB, rN, workD, workI);
    else if (method & 0x2)
      LJMA_MHsample_Aslett2(yp, cp, &mm, pi, Sc, sc, Q, evals, Qinv_s, Qinv_1, P, Pfull, &nn, rz, rB, rN, workD, workI);
    if (per_obs && nd) nd[c] = (unsigned)(rshim_nword() - w0); /* G4: MT words per observation */
    if (per_obs) {
      int bs = 0;
      for (int k = 0; k < n; k++) if (rB[k]) bs = k;
      B[c] = bs;
      memcpy(z + (size_t)c * n, rz, sizeof(double) * n);
      memcpy(N + (size_t)c * n * n, rN, sizeof(int) * n * n);
    } else {
      memcpy(B, rB, sizeof(int) * n);
      memcpy(z, rz, sizeof(double) * n);
      memcpy(N, rN, sizeof(int) * n * n);
    }
  }
  free(P); free(Pfull); free(Q); free(Qinv); free(evals); free(e); free(Qinv_s);
  free(Qinv_1); free(Qinv_b); free(b); free(pi); free(Sc); free(sc); free(workD);
  free(workI); free(rB); free(rN); free(rz);
  rshim_free_all();
  return info;
}

int ref_get_counter(void) { return LJMA_counter; }
