/*
 * oracle/rshim/rshim.c — TEST INFRASTRUCTURE ONLY.
 *
 * Supplies the R runtime pieces the reference's C sources need so that they
 * compile unmodified into oracle/_ref/libpht_ref.so (the "reference oracle"):
 *   - Rprintf/REprintf (swallowed unless verbose), R_alloc arena freed per
 *     call, GetRNGstate/PutRNGstate no-ops;
 *   - unif_rand/exp_rand/norm_rand/runif/rexp/rgamma/dexp backed by the
 *     R-compatible stream of phasetype_amd/csrc/rstream.c (one global stream
 *     seeded by rshim_set_seed, mirroring R's set.seed);
 *   - BLAS dgemv/dgemm in reference-BLAS (netlib dgemv.f/dgemm.f) loop order,
 *     no FMA contraction — the order R's bundled libRblas uses;
 *   - LAPACK dgeevx/dgetrf/dgetri forwarded to an LP64 LAPACK loaded at run
 *     time (scipy's bundled OpenBLAS: symbols scipy_dgeevx_ etc.).
 * Nothing here is linked into the product library.
 */
#include <dlfcn.h>
#include <stdarg.h>
#include <stdint.h>

#include "R.h"
#include "R_ext/BLAS.h"
#include "R_ext/Lapack.h"
#include "../../phasetype_amd/csrc/rstream.h"

/* ------------------------------------------------------------------ io */
static int g_verbose = 0;
static long g_nprint = 0;
void rshim_set_verbose(int v) { g_verbose = v; }
long rshim_print_count(void) { return g_nprint; }

void Rprintf(const char *fmt, ...) {
  g_nprint++;
  if (!g_verbose) return;
  va_list ap;
  va_start(ap, fmt);
  vprintf(fmt, ap);
  va_end(ap);
}
void REprintf(const char *fmt, ...) {
  g_nprint++;
  if (!g_verbose) return;
  va_list ap;
  va_start(ap, fmt);
  vfprintf(stderr, fmt, ap);
  va_end(ap);
}
void R_FlushConsole(void) {}
void R_CheckUserInterrupt(void) {}
void GetRNGstate(void) {}
void PutRNGstate(void) {}

/* ---------------------------------------------------------- R_alloc arena */
typedef struct blk { struct blk *next; } blk;
static blk *g_arena = NULL;
char *R_alloc(size_t n, int size) {
  size_t bytes = n * (size_t)size;
  blk *b = (blk *)calloc(1, sizeof(blk) + bytes + 16);
  if (!b) { fprintf(stderr, "rshim: R_alloc out of memory\n"); abort(); }
  b->next = g_arena;
  g_arena = b;
  return (char *)(b + 1);
}
void rshim_free_all(void) {
  while (g_arena) { blk *n = g_arena->next; free(g_arena); g_arena = n; }
}
void *rshim_calloc(size_t n, size_t size) { return calloc(n ? n : 1, size); }
void rshim_free(void *p) { free(p); }

/* ------------------------------------------------------------------ RNG */
static pht_rstream g_rs;
void rshim_set_seed(uint32_t seed) { pht_rs_set_seed(&g_rs, seed); }
/* 32-bit MT words the reference has consumed since set_seed (G4 fixtures) */
unsigned long long rshim_nword(void) { return (unsigned long long)g_rs.nword; }
void rshim_get_state(uint32_t *mt624, int *mti) {
  memcpy(mt624, g_rs.mt, sizeof(g_rs.mt));
  *mti = g_rs.mti;
}
void rshim_set_state(const uint32_t *mt624, int mti) {
  memcpy(g_rs.mt, mt624, sizeof(g_rs.mt));
  g_rs.mti = mti;
}
double unif_rand(void) { return pht_rs_unif_rand(&g_rs); }
double exp_rand(void) { return pht_rs_exp_rand(&g_rs); }
double norm_rand(void) { return pht_rs_norm_rand(&g_rs); }
double runif(double a, double b) { return pht_rs_runif(&g_rs, a, b); }
double rexp(double scale) { return pht_rs_rexp(&g_rs, scale); }
double rgamma(double a, double scale) { return pht_rs_rgamma(&g_rs, a, scale); }
double dexp(double x, double scale, int give_log) { return pht_rs_dexp(x, scale, give_log); }

/* ----------------------------------------------------- BLAS (netlib order) */
static int lsame(const char *c, char u) { return (*c == u) || (*c == (char)(u + 32)); }

void dgemv_(const char *trans, const int *m, const int *n, const double *alpha,
            const double *a, const int *lda, const double *x, const int *incx,
            const double *beta, double *y, const int *incy, size_t ltrans) {
  (void)ltrans;
  const int M = *m, N = *n, LDA = *lda;
  if (*incx != 1 || *incy != 1) { fprintf(stderr, "rshim dgemv: inc!=1\n"); abort(); }
  if (M == 0 || N == 0 || (*alpha == 0.0 && *beta == 1.0)) return;
  const int tr = !lsame(trans, 'N');
  const int leny = tr ? N : M;
  if (*beta != 1.0) {
    if (*beta == 0.0)
      for (int i = 0; i < leny; i++) y[i] = 0.0;
    else
      for (int i = 0; i < leny; i++) y[i] = *beta * y[i];
  }
  if (*alpha == 0.0) return;
  if (!tr) {
    for (int j = 0; j < N; j++) {
      double temp = *alpha * x[j];
      for (int i = 0; i < M; i++) y[i] = y[i] + temp * a[i + (size_t)j * LDA];
    }
  } else {
    for (int j = 0; j < N; j++) {
      double temp = 0.0;
      for (int i = 0; i < M; i++) temp = temp + a[i + (size_t)j * LDA] * x[i];
      y[j] = y[j] + *alpha * temp;
    }
  }
}

void dgemm_(const char *transa, const char *transb, const int *m, const int *n,
            const int *k, const double *alpha, const double *a, const int *lda,
            const double *b, const int *ldb, const double *beta, double *c,
            const int *ldc, size_t la, size_t lb) {
  (void)la; (void)lb;
  if (!lsame(transa, 'N') || !lsame(transb, 'N')) { fprintf(stderr, "rshim dgemm: only NN\n"); abort(); }
  const int M = *m, N = *n, K = *k, LDA = *lda, LDB = *ldb, LDC = *ldc;
  if (M == 0 || N == 0 || ((*alpha == 0.0 || K == 0) && *beta == 1.0)) return;
  for (int j = 0; j < N; j++) {
    if (*beta == 0.0)
      for (int i = 0; i < M; i++) c[i + (size_t)j * LDC] = 0.0;
    else if (*beta != 1.0)
      for (int i = 0; i < M; i++) c[i + (size_t)j * LDC] = *beta * c[i + (size_t)j * LDC];
    if (*alpha == 0.0) continue;
    for (int l = 0; l < K; l++) {
      double temp = *alpha * b[l + (size_t)j * LDB];
      for (int i = 0; i < M; i++) c[i + (size_t)j * LDC] = c[i + (size_t)j * LDC] + temp * a[i + (size_t)l * LDA];
    }
  }
}

/* --------------------------------------------------- LAPACK (runtime-bound) */
typedef void (*dgeevx_t)(const char *, const char *, const char *, const char *,
                         const int *, double *, const int *, double *, double *,
                         double *, const int *, double *, const int *, int *,
                         int *, double *, double *, double *, double *, double *,
                         const int *, int *, int *, size_t, size_t, size_t, size_t);
typedef void (*dgetrf_t)(const int *, const int *, double *, const int *, int *, int *);
typedef void (*dgetri_t)(const int *, double *, const int *, const int *, double *, const int *, int *);
static dgeevx_t p_dgeevx;
static dgetrf_t p_dgetrf;
static dgetri_t p_dgetri;

/* path: an LP64 LAPACK shared object; prefix: symbol prefix ("scipy_" or ""). */
int rshim_bind_lapack(const char *path, const char *prefix) {
  void *h = dlopen(path, RTLD_NOW | RTLD_LOCAL);
  if (!h) { fprintf(stderr, "rshim: dlopen(%s) failed: %s\n", path, dlerror()); return 1; }
  char nm[64];
  snprintf(nm, sizeof nm, "%sdgeevx_", prefix); p_dgeevx = (dgeevx_t)dlsym(h, nm);
  snprintf(nm, sizeof nm, "%sdgetrf_", prefix); p_dgetrf = (dgetrf_t)dlsym(h, nm);
  snprintf(nm, sizeof nm, "%sdgetri_", prefix); p_dgetri = (dgetri_t)dlsym(h, nm);
  return (p_dgeevx && p_dgetrf && p_dgetri) ? 0 : 2;
}
static void need_lapack(void) {
  if (!p_dgeevx) { fprintf(stderr, "rshim: LAPACK not bound (call rshim_bind_lapack)\n"); abort(); }
}
void dgeevx_(const char *balanc, const char *jobvl, const char *jobvr,
             const char *sense, const int *n, double *a, const int *lda,
             double *wr, double *wi, double *vl, const int *ldvl, double *vr,
             const int *ldvr, int *ilo, int *ihi, double *scale, double *abnrm,
             double *rconde, double *rcondv, double *work, const int *lwork,
             int *iwork, int *info, size_t l1, size_t l2, size_t l3, size_t l4) {
  need_lapack();
  p_dgeevx(balanc, jobvl, jobvr, sense, n, a, lda, wr, wi, vl, ldvl, vr, ldvr, ilo,
           ihi, scale, abnrm, rconde, rcondv, work, lwork, iwork, info, l1, l2, l3, l4);
}
void dgetrf_(const int *m, const int *n, double *a, const int *lda, int *ipiv, int *info) {
  need_lapack();
  p_dgetrf(m, n, a, lda, ipiv, info);
}
void dgetri_(const int *n, double *a, const int *lda, const int *ipiv, double *work,
             const int *lwork, int *info) {
  need_lapack();
  p_dgetri(n, a, lda, ipiv, work, lwork, info);
}
