/*
 * fake_r_host.c — TEST HARNESS: a process that plays R for libPhaseType.so.
 *
 * R is not installed in this image.  This host exports (with -rdynamic) the
 * R API symbols the library resolves at run time — unif_rand, rgamma,
 * GetRNGstate/PutRNGstate, Rprintf, R_FlushConsole, Rf_error,
 * R_registerRoutines, R_useDynamicSymbols, R_forceSymbols — then loads the
 * library RTLD_LOCAL as R's dyn.load does, calls R_init_PhaseType as
 * library(PhaseType) would (NAMESPACE:2 useDynLib(.registration = TRUE)),
 * and calls the registered routine the way .C(LJMA_Gibbs, ...) does
 * (R/phtMCMC2.R:73).  Prints one JSON line for tests/test_r_boundary.py.
 * Only the R API is exported (-Wl,--dynamic-list=r_api.list), so the
 * library's own symbols are never interposed by this host's.
 *
 * usage: fake_r_host <libPhaseType.so> <it> [phtMCMC2|phtMCMC] [seed]
 *   phtMCMC2: tests/phtMCMC2.R's .C vectors (ECS, 3-state repair model,
 *             set.seed(34752076)); phtMCMC: tests/phtMCMC.R's (dense
 *             3-state generator, MHRS, set.seed(576734884)); SURVEY.md §4.2.
 */
#include <dlfcn.h>
#include <math.h>
#include <setjmp.h>
#include <stdarg.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

/* ---- R's RNG: the repo's restatement of R's default generator
 * (phasetype_amd/csrc/rstream.c: Mersenne-Twister with set.seed's
 * scrambling, R's unif_rand fix-up, Ahrens-Dieter exp_rand, GD/GS rgamma),
 * compiled into this host, so the chain the library draws here is the one
 * R would give after set.seed(seed) -- and the one the oracle's device-spec
 * LJMA_Gibbs gives under the same seed (tests/test_r_boundary.py) */
#include "rstream.h"
static pht_rstream g_rs;
static long g_nunif = 0, g_ngamma = 0, g_nget = 0, g_nput = 0, g_nprint = 0;
double unif_rand(void) {
  g_nunif++;
  return pht_rs_unif_rand(&g_rs);
}
double rgamma(double a, double scale) {
  g_ngamma++;
  return pht_rs_rgamma(&g_rs, a, scale);
}
void GetRNGstate(void) { g_nget++; }
void PutRNGstate(void) { g_nput++; }
void Rprintf(const char *fmt, ...) {
  (void)fmt;
  g_nprint++;
}
void R_FlushConsole(void) {}

static jmp_buf g_jb;
static char g_err[512];
void Rf_error(const char *fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof g_err, fmt, ap);
  va_end(ap);
  longjmp(g_jb, 1);
}

/* ---- R_ext/Rdynload.h registration ABI */
typedef void *(*DL_FUNC)(void);
typedef unsigned int R_NativePrimitiveArgType;
typedef struct {
  const char *name;
  DL_FUNC fun;
  int numArgs;
  R_NativePrimitiveArgType *types;
} R_CMethodDef;

static char g_name[64];
static int g_nargs = -1, g_types[32], g_dyn = -1, g_force = -1, g_nroutines = 0;
static DL_FUNC g_fun = 0;
int R_registerRoutines(void *dll, const R_CMethodDef *c, const void *call, const void *f, const void *e) {
  (void)dll; (void)call; (void)f; (void)e;
  for (; c && c->name; c++) {
    g_nroutines++;
    snprintf(g_name, sizeof g_name, "%s", c->name);
    g_nargs = c->numArgs;
    g_fun = c->fun;
    for (int i = 0; i < c->numArgs && i < 32; i++) g_types[i] = (int)c->types[i];
  }
  return 1;
}
int R_useDynamicSymbols(void *dll, int v) { (void)dll; g_dyn = v; return 1; }
int R_forceSymbols(void *dll, int v) { (void)dll; g_force = v; return 1; }

typedef void (*gibbs_fn)(int *, int *, int *, int *, int *, double *, double *, int *, double *, double *, int *,
                         int *, double *, int *, double *);

int main(int argc, char **argv) {
  if (argc < 3) return 2;
  void *h = dlopen(argv[1], RTLD_NOW | RTLD_LOCAL);
  if (!h) {
    printf("{\"error\": \"dlopen: %s\"}\n", dlerror());
    return 3;
  }
  void (*init)(void *) = (void (*)(void *))dlsym(h, "R_init_PhaseType");
  int (*in_r)(void) = (int (*)(void))dlsym(h, "pht_in_R");
  if (!init || !in_r) return 4;
  static int fake_dll_info;
  init(&fake_dll_info);
  /* the reference's test scripts as .C vectors */
  const int dense = argc > 3 && !strcmp(argv[3], "phtMCMC");
  int it = atoi(argv[2]), mhit = 1, method = dense ? 1 : 2, n = 3, m = dense ? 9 : 2, l = 20, silent = 0;
  pht_rs_set_seed(&g_rs, argc > 4 ? (uint32_t)strtoul(argv[4], 0, 10) : (dense ? 576734884u : 34752076u));
  /* phtMCMC2: nu = list(R=180, F=24) sorted F, R (R/phtMCMC2.R:3-4);
   * phtMCMC: names sorted in the C locale S12 S13 S21 S23 S31 S32 s1 s2 s3
   * with nu = c(24,24,1,180,1,24,180,1,24) given row-major over
   * S12 S13 s1 S21 S23 s2 S31 S32 s3 (R/phtMCMC.R:17-30) */
  double nu2[2] = {24, 180}, nu9[9] = {24, 24, 180, 1, 180, 1, 1, 24, 24};
  double zeta[9] = {16, 16, 16, 16, 16, 16, 16, 16, 16}, start[1] = {-1};
  int T2[16] = {0, 2, 2, 0, 1, 0, 0, 0, 1, 0, 0, 0, 0, 1, 1, 0};
  /* T[i + 4 j] = 1-based index of the name at TT[i, j] */
  int T9[16] = {0, 3, 5, 0, 1, 0, 6, 0, 2, 4, 0, 0, 7, 8, 9, 0};
  double *nu = dense ? nu9 : nu2;
  int *T = dense ? T9 : T2;
  double C[16];
  for (int i = 0; i < 16; i++) C[i] = 1.0;
  double y[20] = {1.45353415045187, 1.85349532001349, 2.01084961814576, 0.505725921290172, 1.56252630012213,
                  3.41158665930278, 1.52674487509487, 4.3428662377235,  8.03208018151311,  2.41746547476986,
                  0.38828086509283, 2.61513815012196, 3.39148865480856, 1.82705817807965,  1.42090953713845,
                  0.851438991331866, 0.0178808867191894, 0.632198596390046, 0.959910259815998, 1.83344199966323};
  int cens[20] = {0};
  double *res = calloc((size_t)it * m, sizeof(double));
  int errored = 0;
  if (setjmp(g_jb) == 0) {
    if (g_fun) ((gibbs_fn)g_fun)(&it, &mhit, &method, &n, &m, nu, zeta, T, C, y, &l, cens, start, &silent, res);
  } else {
    errored = 1;
  }
  int finite = 1;
  for (int i = 0; i < it * m; i++) finite &= isfinite(res[i]) && res[i] > 0;
  printf("{\"routines\": %d, \"name\": \"%s\", \"nargs\": %d, \"types\": [", g_nroutines, g_name, g_nargs);
  for (int i = 0; i < g_nargs; i++) printf("%s%d", i ? ", " : "", g_types[i]);
  printf("], \"dynamic\": %d, \"force\": %d, \"in_R\": %d, \"errored\": %d, \"error\": \"%s\", "
         "\"unif\": %ld, \"gamma\": %ld, \"getrng\": %ld, \"putrng\": %ld, \"prints\": %ld, \"finite\": %d, "
         "\"m\": %d, \"res\": [",
         g_dyn, g_force, in_r(), errored, g_err, g_nunif, g_ngamma, g_nget, g_nput, g_nprint, finite, m);
  for (int i = 0; i < it * m; i++) printf("%s%.17g", i ? ", " : "", res[i]);
  printf("]}\n");
  free(res);
  return 0;
}
