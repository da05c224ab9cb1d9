/*
 * gibbs_host.cpp — host runtime of the MI355X PhaseType hot path.
 *
 *  - LJMA_Gibbs: the reference's .C entry point (src/PHT_MCMC_Aslett.c:104,
 *    registered by src/Registrations.c:6-20), re-implemented: the Gibbs
 *    bookkeeping and conjugate Gamma update stay on the host exactly as in
 *    src/PHT_MCMC_Aslett.c:187-405; step 1 (the per-observation latent-path
 *    sampling, :276-337) runs as HIP kernels on every visible GPU, each GPU
 *    owning a contiguous shard of the observations, and the integer
 *    sufficient statistics are summed on the host (exact, order-free).
 *  - R_init_PhaseType: registers LJMA_Gibbs for `.C` when loaded by R.
 *  - pht_* : the sweep-level C ABI (include/phasetype_amd.h) used by the
 *    Python mirror, the parity tests and the multi-process benchmark.
 *
 * Random numbers: inside R, R's own unif_rand/rgamma (resolved at run time);
 * standalone, the R-compatible stream of rstream.c.  Per-observation draws
 * on the device come from Philox keyed by two R-stream uniforms drawn at
 * LJMA_Gibbs entry (pht_philox.h).
 */
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <math.h>
#include <rccl/rccl.h>
#include <stdarg.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <sched.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <condition_variable>
#include <mutex>
#include <numeric>
#include <string>
#include <thread>
#include <vector>

#include "../../include/phasetype_amd.h"
#include "pht_detmath.h"
#include "pht_kernels.h"
#include "pht_layout.h"
#include "rstream.h"

using namespace pht;

/* ======================================================= error reporting */
static thread_local std::string g_err;
static void set_err(const char *fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  g_err = buf;
}
extern "C" const char *pht_last_error(void) { return g_err.c_str(); }

#define HIPCHK(x)                                                               \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      set_err("%s failed: %s (%s:%d)", #x, hipGetErrorString(e_), __FILE__, __LINE__); \
      return -1;                                                                \
    }                                                                           \
  } while (0)

/* ================================================ R runtime (when inside R) */
namespace {
typedef double (*unif_fn)(void);
typedef double (*rgamma_fn)(double, double);
typedef void (*void_fn)(void);
typedef void (*printf_fn)(const char *, ...);
typedef void (*error_fn)(const char *, ...);

struct RHost {
  bool inR = false;
  unif_fn unif = nullptr;
  rgamma_fn rgamma = nullptr;
  void_fn getrng = nullptr, putrng = nullptr, flush = nullptr;
  printf_fn rprintf = nullptr;
  error_fn rerror = nullptr;
  pht_rstream rs;
  bool seeded = false;
  RHost() {
    unif = (unif_fn)dlsym(RTLD_DEFAULT, "unif_rand");
    rgamma = (rgamma_fn)dlsym(RTLD_DEFAULT, "rgamma");
    getrng = (void_fn)dlsym(RTLD_DEFAULT, "GetRNGstate");
    putrng = (void_fn)dlsym(RTLD_DEFAULT, "PutRNGstate");
    rprintf = (printf_fn)dlsym(RTLD_DEFAULT, "Rprintf");
    rerror = (error_fn)dlsym(RTLD_DEFAULT, "Rf_error");
    flush = (void_fn)dlsym(RTLD_DEFAULT, "R_FlushConsole");
    inR = unif && rgamma && getrng && putrng && rprintf && !getenv("PHT_STANDALONE_RNG");
    pht_rs_set_seed(&rs, 1234u);
  }
  double u() { return inR ? unif() : pht_rs_unif_rand(&rs); }
  double gamma(double a, double sc) { return inR ? rgamma(a, sc) : pht_rs_rgamma(&rs, a, sc); }
  void begin() { if (inR) getrng(); }
  void end() { if (inR) putrng(); }
};
RHost &rhost() {
  static RHost h;
  return h;
}
int g_verbose = 0;
void say(const char *fmt, ...) {
  RHost &h = rhost();
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  if (h.inR) {
    h.rprintf("%s", buf);
    if (h.flush) h.flush();
  } else if (g_verbose) {
    fputs(buf, stdout);
    fflush(stdout);
  }
}
/* a warning the caller must see: Rprintf inside R, stderr otherwise */
void warn(const char *fmt, ...) {
  RHost &h = rhost();
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  if (h.inR) {
    h.rprintf("%s", buf);
    if (h.flush) h.flush();
  } else {
    fputs(buf, stderr);
    fflush(stderr);
  }
}
}  // namespace

extern "C" void pht_set_seed(uint32_t seed) { pht_rs_set_seed(&rhost().rs, seed); }
extern "C" double pht_unif_rand(void) { return rhost().u(); }
extern "C" double pht_rgamma(double a, double scale) { return rhost().gamma(a, scale); }
extern "C" void pht_set_verbose(int v) { g_verbose = v; }
extern "C" int pht_in_R(void) { return rhost().inR ? 1 : 0; }

/* ================================================================ LAPACK */
namespace {
typedef void (*dgeevx_t)(const char *, const char *, const char *, const char *, const int *, double *,
                         const int *, double *, double *, double *, const int *, double *, const int *, int *,
                         int *, double *, double *, double *, double *, double *, const int *, int *, int *,
                         size_t, size_t, size_t, size_t);
typedef void (*dgetrf_t)(const int *, const int *, double *, const int *, int *, int *);
typedef void (*dgetri_t)(const int *, double *, const int *, const int *, double *, const int *, int *);
dgeevx_t p_dgeevx = nullptr;
dgetrf_t p_dgetrf = nullptr;
dgetri_t p_dgetri = nullptr;
/* OpenBLAS's thread-count setter, when the bound LAPACK is OpenBLAS (returns
 * the previous count).  The per-sweep eigensystem is an n <= 20 problem: its
 * BLAS calls gain nothing from the thread pool and pay its hand-offs (n = 10:
 * 81 us per parameter block with the pool, 17 us on the calling thread; the
 * same bytes, tests/test_host.py) */
typedef int (*blas_threads_t)(int);
blas_threads_t p_blas_threads = nullptr;

bool lookup_lapack(void *h) {
  p_dgeevx = (dgeevx_t)dlsym(h, "dgeevx_");
  p_dgetrf = (dgetrf_t)dlsym(h, "dgetrf_");
  p_dgetri = (dgetri_t)dlsym(h, "dgetri_");
  p_blas_threads = (blas_threads_t)dlsym(h, "openblas_set_num_threads_local");
  if (p_dgeevx && p_dgetrf && p_dgetri) return true;
  p_dgeevx = nullptr;
  return false;
}

bool lapack_ready() {
  if (p_dgeevx) return true;
  /* 1. an LP64 LAPACK in the global scope (e.g. R's own libRlapack) */
  if (lookup_lapack(RTLD_DEFAULT)) return true;
  /* 2. one this library was linked against (R loads package libraries
   *    RTLD_LOCAL, so e.g. PKG_LIBS = $(LAPACK_LIBS) is only visible through
   *    our own handle, which searches our dependency tree) */
  Dl_info self{};
  if (dladdr(reinterpret_cast<void *>(&pht_bind_lapack), &self) && self.dli_fname) {
    void *h = dlopen(self.dli_fname, RTLD_LAZY | RTLD_NOLOAD);
    if (h) {
      const bool ok = lookup_lapack(h);
      dlclose(h);
      if (ok) return true;
    }
  }
  /* 3. standalone: an explicit library (pht_bind_lapack or the environment) */
  const char *path = getenv("PHT_LAPACK_LIB");
  if (path) return pht_bind_lapack(path, getenv("PHT_LAPACK_PREFIX") ? getenv("PHT_LAPACK_PREFIX") : "") == 0;
  return false;
}
}  // namespace

extern "C" int pht_bind_lapack(const char *path, const char *prefix) {
  void *h = dlopen(path, RTLD_NOW | RTLD_LOCAL);
  if (!h) {
    set_err("dlopen(%s): %s", path, dlerror());
    return 1;
  }
  std::string pre = prefix ? prefix : "";
  p_dgeevx = (dgeevx_t)dlsym(h, (pre + "dgeevx_").c_str());
  p_dgetrf = (dgetrf_t)dlsym(h, (pre + "dgetrf_").c_str());
  p_dgetri = (dgetri_t)dlsym(h, (pre + "dgetri_").c_str());
  p_blas_threads = (blas_threads_t)dlsym(h, "openblas_set_num_threads_local");
  if (!(p_dgeevx && p_dgetrf && p_dgetri)) {
    p_dgeevx = nullptr;
    set_err("LAPACK symbols %sdgeevx_/dgetrf_/dgetri_ not found in %s", pre.c_str(), path);
    return 2;
  }
  return 0;
}

/* LJMA_eigen with LJMA_Gibbs's workspace sizing (src/utility.c:87-129,
 * src/PHT_MCMC_Aslett.c:177-185). */
/* the bound OpenBLAS on one thread for the duration of a scope (the
 * outermost one sets and restores: a Gibbs run once, a lone eigen() call
 * per call) */
static thread_local int g_blas_one = 0;
struct OneBlasThread {
  int prev = 0;
  OneBlasThread() {
    if (g_blas_one++ == 0 && p_blas_threads) prev = p_blas_threads(1);
  }
  ~OneBlasThread() {
    if (--g_blas_one == 0 && p_blas_threads && prev > 1) p_blas_threads(prev);
  }
};

/* LAPACK workspace and scratch of eigen() per n, per host thread: the
 * workspace size is the reference's query result for that n (a pure function
 * of n), asked once instead of twice per sweep */
struct EigenWork {
  int n = -1, lw = 0;
  std::vector<double> A, evi, Ql, scl, rce, rcv, work;
  std::vector<int> iwork, ipiv;
};

static int eigen(int n, const double *S, double *evals, double *Q, double *Qinv) {
  OneBlasThread one;
  char balanc = 'B', jobv = 'V', sense = 'B';
  int lwork = -1, info = 0, ilo, ihi, nn = n;
  double wq = 0, abnrm;
  /* (a pointer: a thread_local object with a destructor left an undefined
   * EigenWork::~EigenWork in the shared library; one per thread, kept) */
  static thread_local EigenWork *ewp = nullptr;
  if (!ewp) ewp = new EigenWork;
  EigenWork &ew = *ewp;
  if (ew.n != n) {
    ew.A.assign(n * n, 0.0);
    ew.evi.assign(n, 0.0);
    ew.Ql.assign(n * n, 0.0);
    ew.scl.assign(n, 0.0);
    ew.rce.assign(n, 0.0);
    ew.rcv.assign(n, 0.0);
    ew.iwork.assign(2 * n + 2, 0);
    ew.ipiv.assign(n, 0);
    p_dgeevx(&balanc, &jobv, &jobv, &sense, &nn, ew.A.data(), &nn, evals, ew.evi.data(), ew.Ql.data(), &nn, Q, &nn,
             &ilo, &ihi, ew.scl.data(), &abnrm, ew.rce.data(), ew.rcv.data(), &wq, &lwork, nullptr, &info, 1, 1, 1, 1);
    int lw = (int)wq;
    p_dgetri(&nn, nullptr, &nn, nullptr, &wq, &lwork, &info);
    if ((int)wq > lw) lw = (int)wq;
    ew.lw = lw > 0 ? lw : 1;
    ew.work.assign(ew.lw, 0.0);
    ew.n = n;
  }
  int lw = ew.lw;
  double *A = ew.A.data(), *evi = ew.evi.data(), *work = ew.work.data();
  memcpy(A, S, sizeof(double) * n * n);
  /* The reference asks for condition numbers too (sense 'B'); they come
   * from dtrsna AFTER the eigenvectors and feed nothing it uses, so the
   * sweep skips them (sense 'N', same workspace as the 'B' query: the
   * Hessenberg/Schur/eigenvector arithmetic is unchanged — evals, Q and
   * Q^-1 stay bit-identical, tests/test_host.py).  That is most of the
   * per-sweep host time at n = 10. */
  char sense_n = 'N', jobvl_n = 'N';
  p_dgeevx(&balanc, &jobvl_n, &jobv, &sense_n, &nn, A, &nn, evals, evi, ew.Ql.data(), &nn, Q, &nn, &ilo,
           &ihi, ew.scl.data(), &abnrm, ew.rce.data(), ew.rcv.data(), work, &lw, ew.iwork.data(), &info, 1, 1, 1, 1);
  if (info != 0) {
    say("Error (LJMA_eigen 01): failed LAPACK call, code=%d\n", info);
    return info;
  }
  for (int i = 0; i < n; i++)
    if (evi[i] > 0) say("Error: imaginary part of eigenvalue %d found.\n", i + 1);
  memcpy(Qinv, Q, sizeof(double) * n * n);
  p_dgetrf(&nn, &nn, Qinv, &nn, ew.ipiv.data(), &info);
  if (info != 0) {
    say("Error (LJMA_inverse 01): failed LAPACK call, code=%d\n", info);
    return info;
  }
  p_dgetri(&nn, Qinv, &nn, ew.ipiv.data(), work, &lw, &info);
  if (info != 0) say("Error (LJMA_inverse 03): failed LAPACK call, code=%d\n", info);
  return info;
}

/* the device-mode spectral products of the packed block (explicit fma in
 * oracle/pht_oracle.c:orc_sp_build's order).  x86-64: a copy compiled with
 * hardware fma runs where the host has it (the baseline ISA's fma() is
 * glibc's software routine: half of build_params' time at n = 20); both are
 * correctly rounded, so the values are the same. */
static inline __attribute__((always_inline)) void spectral_products_body(int n, const double *S, const double *s,
                                                                         const double *P, const double *Q,
                                                                         const double *Qs, const double *Q1,
                                                                         double *d, const Layout &L) {
  double rj[kMaxN];
  for (int j = 0; j < n; j++) {
    const double Sjj = S[j + j * n];
    d[L.logs + j] = s[j] > 0.0 ? pht_log(s[j]) : 0.0;
    d[L.scale + j] = 1.0 / -Sjj;
    d[L.logscale + j] = pht_log(d[L.scale + j]);
    for (int k = 0; k < n; k++) rj[k] = S[j + k * n] / (-Sjj); /* hoisted: same quotients */
    for (int i = 0; i < n; i++) {
      double w = 0.0, v = 0.0;
      for (int k = 0; k < n; k++) {
        if (k != j) w = fma(rj[k], Q[k + i * n], w);
        v = fma(P[j + k * n], Q[k + i * n], v);
      }
      d[L.QQs + j + i * n] = Q[j + i * n] * Qs[i];
      d[L.W + j + i * n] = w * Qs[i];
      d[L.QQ1 + j + i * n] = Q[j + i * n] * Q1[i];
      d[L.V + j + i * n] = v * Q1[i];
    }
  }
  for (int i = 0; i < n; i++) {
    double a = 0.0;
    for (int k = 0; k < n; k++) a = fma(d[L.pi + k], Q[k + i * n], a);
    d[L.piQ + i] = a;
  }
  for (int j = 0; j < n; j++) { /* ECS starting point y_t - a (pht_detmath.h pht_wmoments) */
    double m[PHT_WMOM];
    pht_wmoments(n, d + L.W + j, n, d + L.evals, m);
    for (int k = 0; k < PHT_WMOM; k++) d[L.Wm + j + k * n] = m[k];
  }
}
#if defined(__x86_64__)
__attribute__((target("fma"))) static void spectral_products_fma(int n, const double *S, const double *s,
                                                                 const double *P, const double *Q, const double *Qs,
                                                                 const double *Q1, double *d, const Layout &L) {
  spectral_products_body(n, S, s, P, Q, Qs, Q1, d, L);
}
#endif
static void spectral_products(int n, const double *S, const double *s, const double *P, const double *Q,
                              const double *Qs, const double *Q1, double *d, const Layout &L) {
#if defined(__x86_64__)
  static const bool hw_fma = __builtin_cpu_supports("fma");
  if (hw_fma) {
    spectral_products_fma(n, S, s, P, Q, Qs, Q1, d, L);
    return;
  }
#endif
  spectral_products_body(n, S, s, P, Q, Qs, Q1, d, L);
}

/* ======================================================== sweep parameters */
/*
 * Packed per-sweep block (pht_layout.h) from (S, s): the embedded chain
 * exactly as src/PHT_MCMC_Aslett.c:279-297, the spectral data as :320-332
 * (Q⁻¹v by reference-BLAS dgemv order), and the device-mode products with
 * explicit fma in the order oracle/pht_oracle.c:orc_sp_build uses.
 */
static int build_params(int n, const double *S, const double *s, int method, std::vector<unsigned char> &out) {
  const Layout L = make_layout(n);
  out.assign(L.bytes(), 0);
  double *d = reinterpret_cast<double *>(out.data());
  int *iv = reinterpret_cast<int *>(out.data() + L.ndouble * 8);
  double *P = d + L.P, *Pf = d + L.Pf, *Q = d + L.Q, *Qinv = d + L.Qinv, *ev = d + L.evals;
  memcpy(d + L.S, S, sizeof(double) * n * n);
  memcpy(d + L.s, s, sizeof(double) * n);
  d[L.pi + 0] = 1.0;
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
  std::vector<double> Qs(n, 0.0), Q1(n, 0.0);
  int info = 0;
  if (method & (kMethodECS | kMethodDCS)) {
    if (!lapack_ready()) {
      set_err("no LAPACK bound (call pht_bind_lapack or set PHT_LAPACK_LIB)");
      return -1;
    }
    info = eigen(n, S, ev, Q, Qinv);
    /* dgemv 'N' (reference BLAS order): y = 0; y += x[c] * A[:,c] */
    for (int c = 0; c < n; c++) {
      const double ts = 1.0 * s[c], t1 = 1.0 * 1.0;
      for (int r = 0; r < n; r++) {
        Qs[r] = Qs[r] + ts * Qinv[r + c * n];
        Q1[r] = Q1[r] + t1 * Qinv[r + c * n];
      }
    }
  }
  spectral_products(n, S, s, P, Q, Qs.data(), Q1.data(), d, L);
  for (int j = 0; j < n; j++) {
    int a = 0, b = 0, c = 0;
    for (int k = 0; k < n; k++) {
      if (!(P[j + k * n] == 0.0)) iv[L.succP + j * n + a++] = k;
      if (k != j && !(S[j + k * n] == 0.0)) iv[L.succS + j * n + c++] = k;
    }
    for (int k = 0; k <= n; k++)
      if (!(Pf[j + k * n] == 0.0)) iv[L.succPf + j * (n + 1) + b++] = k;
    iv[L.nsuccP + j] = a;
    iv[L.nsuccPf + j] = b;
    iv[L.nsuccS + j] = c;
  }
  return info;
}

extern "C" int pht_build_params(int n, const double *S, const double *s, int method, unsigned char *out,
                                int out_bytes) {
  std::vector<unsigned char> v;
  int info = build_params(n, S, s, method, v);
  if (info < 0) return info;
  if ((int)v.size() > out_bytes) return -2;
  memcpy(out, v.data(), v.size());
  return info;
}
extern "C" int pht_params_bytes(int n) { return make_layout(n).bytes(); }
extern "C" int pht_stats_len(int n) { return stats_len(n); }

/* =========================================================== device shard */
/* the reference's precedence MHRS > DCS > ECS (src/PHT_MCMC_Aslett.c:325-337);
 * the opt-in uniformisation sampler (no reference counterpart) last */
static int dispatch_method(int method) {
  if (method & kMethodMHRS) return kMethodMHRS;
  if (method & kMethodDCS) return kMethodDCS;
  if (method & kMethodECS) return kMethodECS;
  if (method & kMethodUNIF) return kMethodUNIF;
  return 0;
}

struct pht_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  int n = 0, method = 0, mhit = 1;
  /* the reference method asked for (dispatch_method), and the path law of the
   * UNIF kernels when method is kMethodUNIF: 0 its own, 1 MHRS's / 2 DCS's
   * law by uniformisation (PHT_MHRS=bridge, PHT_DCS=bridge; pht_unif.h) */
  int rmethod = 0, ulaw = 0;
  long count = 0;
  long n_exact = 0;                      /* exact observations; ECS: positions [0, n_exact) (sorted first) */
  double *d_y = nullptr;
  int *d_cens = nullptr;
  uint32_t *d_gid = nullptr;
  /* MHRS attempt-search workspace (count * (1 + mhit) tasks) */
  uint32_t *d_mbest = nullptr, *d_mq0 = nullptr, *d_mq1 = nullptr;
  unsigned *d_mcnt = nullptr;
  unsigned char *d_params = nullptr;
  unsigned long long *d_stats = nullptr;
  unsigned long long *h_stats = nullptr; /* pinned */
  unsigned char *h_params = nullptr;     /* pinned */
  std::vector<long> order;               /* sorted position -> local index */
  std::vector<double> h_ysorted;         /* y in device (sorted) order */
  double ysum = 0.0;                     /* sum of the shard's y (the fixed-point range check) */
  double ymax = 0.0;                     /* largest y of the shard (UNIF table length) */
  double *d_utab = nullptr;              /* UNIF per-sweep table (pht_unif.h) */
  long utab_cap = 0;                     /* its capacity in doubles */
  int *d_dcsb = nullptr;                 /* DCS: per-position end states (dcs_end_kernel) */
  /* debug buffers */
  long long *d_zq = nullptr;
  int *d_N = nullptr, *d_B = nullptr, *d_pre = nullptr, *d_flags = nullptr;
  uint32_t *d_ndraw = nullptr;
  long dbg_cap = 0;
  float last_ms = 0.f;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  /* ECS: the censored range runs on stream2, concurrently with the exact range */
  hipStream_t stream2 = nullptr;
  hipEvent_t evf = nullptr, evj = nullptr;
  struct ChainGroup *grp = nullptr; /* pht_gibbs_run_chains: exact ECS launched with the other chains */
  int gidx = -1;
  long long flagged = 0; /* flagged observation-sweeps of the last Gibbs run (node-wide) */
  long long global_count = -1; /* observations over all shards (pht_ctx_set_global_count) */
  ncclComm_t comm = nullptr; /* pht_ctx_attach_rccl: stats summed over ranks on `stream` */
  long long *d_rccl = nullptr; /* pht_ctx_rccl_prepare: staging buffer of pht_ctx_rccl_allreduce */
  int rccl_cap = 0;
  bool stats_zero = false;   /* d_stats zeroed on `stream` after the last sweep's copy */
  hipEvent_t evd = nullptr;  /* the statistics copy to the host is done */
  /* the statistics block published by pht_stats_out_kernel: host-pinned
   * coherent words + a flag the host polls (nullptr: the copy + event path,
   * or PHT_STATS_COPY=1) */
  unsigned long long *h_out = nullptr, *d_out = nullptr;
  unsigned *h_flag = nullptr, *d_flag = nullptr;
  unsigned seq = 0;
  /* sweeps enqueued and not yet waited for (oldest first): the statistics
   * flag value each publishes and its kernel-time event pair; two in flight
   * in the pipelined Gibbs loop (gibbs_run), else one */
  struct Inflight {
    unsigned seq = 0, gate = 0;
    bool timed = false;
    int evs = 0;
  } infl[2];
  int nin = 0;
  unsigned nenq = 0;
  hipEvent_t ev0b = nullptr, ev1b = nullptr;
  /* the pipelined loop's gate (pht_gate_kernel): word 0 the released value
   * (host writes), word 16 the device's ack; the parameter block staged in
   * coherent pinned memory for the gate kernel's copy */
  unsigned *h_gate = nullptr, *d_gate = nullptr;
  unsigned long long *h_pg = nullptr, *d_pg = nullptr;
  unsigned gate_seq = 0;
};

/* lanes of the persistent ECS grid on an MI355X (256 CUs x 2 blocks x 256) */
constexpr long kSpreadLanes = 256L * 2 * 256;

/*
 * Chains whose sweeps go out together (pht_gibbs_run_chains, SURVEY.md
 * §8f.4).  Each chain's thread builds its parameters into its slot of one
 * pinned block and arrives; the last chain to arrive enqueues the whole sweep
 * of every arrived chain on the group's stream: one parameter upload, one
 * statistics reset, ONE ecs_chains_kernel launch over all exact ranges (the
 * censored-range kernels concurrently on stream2), one statistics
 * download.  The others wait for that sweep's `done` event.  A chain that
 * stops (end of run or error) leaves the group, so the others never wait
 * for it.
 */
struct ChainGroup {
  int K = 0, device = 0, n = 0, pb = 0, sl = 0, method = kMethodECS;
  std::mutex m;
  std::condition_variable cv;
  int active = 0;
  unsigned long gen = 0;
  int rc = 0;
  float ms = 0.f;
  std::vector<int> who;          /* chains arrived for the pending sweep */
  std::vector<SweepArgs> ex, ce; /* [K] exact / censored range arguments */
  unsigned char *h_params = nullptr, *d_params = nullptr;  /* [K][pb] */
  unsigned long long *h_stats = nullptr, *d_stats = nullptr; /* [K][sl] */
  SweepArgs *h_args = nullptr, *d_args = nullptr;           /* [K] packed */
  hipEvent_t ev0 = nullptr, ev1 = nullptr, done = nullptr;
  hipStream_t stream = nullptr;
  /* censored ranges run on stream2, concurrently with the exact-range launch */
  hipStream_t stream2 = nullptr;
  hipEvent_t evf = nullptr, evj = nullptr;
};

static void group_destroy(ChainGroup *g) {
  if (!g) return;
  (void)hipSetDevice(g->device);
  if (g->stream) (void)hipStreamSynchronize(g->stream);
  if (g->stream2) (void)hipStreamSynchronize(g->stream2);
  for (hipEvent_t e : {g->ev0, g->ev1, g->done, g->evf, g->evj})
    if (e) (void)hipEventDestroy(e);
  if (g->stream) (void)hipStreamDestroy(g->stream);
  if (g->stream2) (void)hipStreamDestroy(g->stream2);
  if (g->h_params) (void)hipHostFree(g->h_params);
  if (g->h_stats) (void)hipHostFree(g->h_stats);
  if (g->h_args) (void)hipHostFree(g->h_args);
  if (g->d_params) (void)hipFree(g->d_params);
  if (g->d_stats) (void)hipFree(g->d_stats);
  if (g->d_args) (void)hipFree(g->d_args);
  delete g;
}

static ChainGroup *group_create(int device, int K, int n, int method) {
  ChainGroup *g = new ChainGroup();
  g->K = K;
  g->method = method;
  g->device = device;
  g->n = n;
  g->pb = make_layout(n).bytes();
  g->sl = stats_len(n);
  g->active = K;
  g->ex.resize(K);
  g->ce.resize(K);
  const size_t P = (size_t)g->pb * K, Sb = sizeof(unsigned long long) * g->sl * K, A = sizeof(SweepArgs) * 2 * K;
  const bool ok = hipSetDevice(device) == hipSuccess &&
                  hipStreamCreateWithFlags(&g->stream, hipStreamNonBlocking) == hipSuccess &&
                  hipEventCreate(&g->ev0) == hipSuccess && hipEventCreate(&g->ev1) == hipSuccess &&
                  hipEventCreateWithFlags(&g->done, hipEventDisableTiming) == hipSuccess &&
                  hipStreamCreateWithFlags(&g->stream2, hipStreamNonBlocking) == hipSuccess &&
                  hipEventCreateWithFlags(&g->evf, hipEventDisableTiming) == hipSuccess &&
                  hipEventCreateWithFlags(&g->evj, hipEventDisableTiming) == hipSuccess &&
                  hipHostMalloc(&g->h_params, P, 0) == hipSuccess && hipMalloc(&g->d_params, P) == hipSuccess &&
                  hipHostMalloc(&g->h_stats, Sb, 0) == hipSuccess && hipMalloc(&g->d_stats, Sb) == hipSuccess &&
                  hipHostMalloc(&g->h_args, A, 0) == hipSuccess && hipMalloc(&g->d_args, A) == hipSuccess;
  if (!ok) {
    group_destroy(g);
    return nullptr;
  }
  return g;
}

/* with g->m held: enqueue the sweep of the arrived chains and release them */
static void group_fire(ChainGroup *g) {
  const int k = (int)g->who.size();
  hipError_t e = hipSetDevice(g->device);
  if (e == hipSuccess)
    e = hipMemcpyAsync(g->d_params, g->h_params, (size_t)g->pb * g->K, hipMemcpyHostToDevice, g->stream);
  if (e == hipSuccess)
    e = hipMemsetAsync(g->d_stats, 0, sizeof(unsigned long long) * g->sl * g->K, g->stream);
  if (e == hipSuccess) e = hipEventRecord(g->ev0, g->stream);
  int nx = 0, nc = 0;
  if (g->method == kMethodECS) {
    /* exact ranges [0, K), censored ranges [K, 2K) of the packed arguments */
    for (int i = 0; i < k; i++) {
      const int w = g->who[i];
      if (g->ex[w].count > 0) g->h_args[nx++] = g->ex[w];
    }
    for (int i = 0; i < k; i++) {
      const int w = g->who[i];
      if (g->ce[w].count > 0) g->h_args[g->K + nc++] = g->ce[w];
    }
  } else {
    for (int i = 0; i < k; i++)
      if (g->ex[g->who[i]].count > 0) g->h_args[nx++] = g->ex[g->who[i]];
  }
  if (e == hipSuccess)
    e = hipMemcpyAsync(g->d_args, g->h_args, sizeof(SweepArgs) * 2 * g->K, hipMemcpyHostToDevice, g->stream);
  /* ECS: every chain's censored range in one launch on stream2 while the
   * exact ranges run (as ctx_enqueue) */
  const bool fork = nc > 0 && nx > 0;
  if (e == hipSuccess && fork) e = hipEventRecord(g->evf, g->stream);
  if (e == hipSuccess && fork) e = hipStreamWaitEvent(g->stream2, g->evf, 0);
  if (e == hipSuccess && nc > 0)
    e = pht_launch_chains(g->h_args + g->K, g->d_args + g->K, nc, kMethodECS, fork ? g->stream2 : g->stream);
  if (e == hipSuccess && fork) e = hipEventRecord(g->evj, g->stream2);
  if (e == hipSuccess && nx > 0)
    e = g->method == kMethodECS ? pht_launch_ecs_chains(g->h_args, g->d_args, nx, g->stream)
                                : pht_launch_chains(g->h_args, g->d_args, nx, g->method, g->stream);
  if (e == hipSuccess && fork) e = hipStreamWaitEvent(g->stream, g->evj, 0);
  if (e == hipSuccess) e = hipEventRecord(g->ev1, g->stream);
  if (e == hipSuccess)
    e = hipMemcpyAsync(g->h_stats, g->d_stats, sizeof(unsigned long long) * g->sl * g->K, hipMemcpyDeviceToHost,
                       g->stream);
  if (e == hipSuccess) e = hipEventRecord(g->done, g->stream);
  g->rc = (e == hipSuccess) ? 0 : (int)e;
  g->who.clear();
  g->gen++;
  g->cv.notify_all();
}

static int unif_prepare(pht_ctx *c, SweepArgs &a);
static int dcs_brent();

/* chain c's sweep (parameters in c->h_params): returns when the group's sweep
 * is done, with c->h_stats and c->last_ms filled */
static int group_sweep(pht_ctx *c, uint32_t k0, uint32_t k1, uint32_t sweep, int zexp) {
  ChainGroup *g = c->grp;
  const int w = c->gidx;
  unsigned char *dp = g->d_params + (size_t)g->pb * w;
  unsigned long long *ds = g->d_stats + (size_t)g->sl * w;
  SweepArgs a;
  memset(&a, 0, sizeof a);
  a.params = dp;
  a.n = c->n;
  a.mhit = c->mhit;
  a.ulaw = c->ulaw;
  a.y = c->d_y;
  a.gid = c->d_gid;
  a.k0 = k0;
  a.k1 = k1;
  a.sweep = sweep;
  a.zscale = ldexp(1.0, zexp);
  a.dcsbrent = dcs_brent();
  a.dcsb = nullptr; /* the chains launch computes the end states in its round kernel */
  a.stats = ds;
  SweepArgs ae = a, ac = a;
  if (g->method == kMethodECS) {
    ae.begin = 0;
    ae.count = c->n_exact;
    ae.newcap = getenv("PHT_NEWCAP") ? atoi(getenv("PHT_NEWCAP")) : 1;
    ae.spread = getenv("PHT_SPREAD") ? atoi(getenv("PHT_SPREAD")) : (c->n_exact <= 2 * kSpreadLanes);
    ac.cens = c->d_cens;
    ac.begin = c->n_exact;
    ac.count = c->count - c->n_exact;
    ac.allcens = 1;
  } else {
    /* the whole shard in one argument (MHRS, DCS, UNIF) */
    ae.begin = 0;
    ae.count = c->count;
    ae.cens = c->d_cens;
    ae.mbest = c->d_mbest;
    ae.mq0 = c->d_mq0;
    ae.mq1 = c->d_mq1;
    ae.mcnt = c->d_mcnt;
    if (g->method == kMethodUNIF && unif_prepare(c, ae)) return -1;
    ac.count = 0;
  }
  std::unique_lock<std::mutex> lk(g->m);
  memcpy(g->h_params + (size_t)g->pb * w, c->h_params, g->pb);
  g->ex[w] = ae;
  g->ce[w] = ac;
  g->who.push_back(w);
  const unsigned long my = g->gen;
  if ((int)g->who.size() == g->active) group_fire(g);
  else g->cv.wait(lk, [&] { return g->gen != my; });
  const int rc = g->rc; /* the next sweep needs this chain's arrival: rc is still ours */
  lk.unlock();
  if (rc) {
    set_err("chains sweep enqueue failed (%s)", hipGetErrorString((hipError_t)rc));
    return -1;
  }
  HIPCHK(hipEventSynchronize(g->done));
  HIPCHK(hipEventElapsedTime(&c->last_ms, g->ev0, g->ev1));
  memcpy(c->h_stats, g->h_stats + (size_t)g->sl * w, sizeof(unsigned long long) * g->sl);
  return 0;
}

static void group_leave(ChainGroup *g) {
  std::lock_guard<std::mutex> lk(g->m);
  g->active--;
  if (!g->who.empty() && (int)g->who.size() == g->active) group_fire(g);
}

static void ctx_free_obs(pht_ctx *c) {
  (void)hipSetDevice(c->device);
  if (c->d_y) (void)hipFree(c->d_y);
  if (c->d_cens) (void)hipFree(c->d_cens);
  if (c->d_gid) (void)hipFree(c->d_gid);
  if (c->d_mbest) (void)hipFree(c->d_mbest);
  if (c->d_mq0) (void)hipFree(c->d_mq0);
  if (c->d_mq1) (void)hipFree(c->d_mq1);
  if (c->d_mcnt) (void)hipFree(c->d_mcnt);
  if (c->d_utab) (void)hipFree(c->d_utab);
  c->d_utab = nullptr;
  c->utab_cap = 0;
  if (c->d_dcsb) (void)hipFree(c->d_dcsb);
  c->d_dcsb = nullptr;
  c->d_y = nullptr; c->d_cens = nullptr; c->d_gid = nullptr;
  c->d_mbest = c->d_mq0 = c->d_mq1 = nullptr;
  c->d_mcnt = nullptr;
}
static void ctx_free_dbg(pht_ctx *c) {
  (void)hipSetDevice(c->device);
  if (c->d_zq) (void)hipFree(c->d_zq);
  if (c->d_N) (void)hipFree(c->d_N);
  if (c->d_B) (void)hipFree(c->d_B);
  if (c->d_pre) (void)hipFree(c->d_pre);
  if (c->d_flags) (void)hipFree(c->d_flags);
  if (c->d_ndraw) (void)hipFree(c->d_ndraw);
  c->d_zq = nullptr; c->d_N = nullptr; c->d_B = c->d_pre = c->d_flags = nullptr; c->d_ndraw = nullptr;
  c->dbg_cap = 0;
}

/*
 * RCCL bound at run time (dlopen), so the library loads where RCCL is absent
 * (inside R on a single GPU) and only multi-process runs need it.  Replaces
 * the per-sweep host callback (pht_reduce_fn) with an all-reduce on the device
 * copy of the statistics block, on the sweep's stream: no host round trip
 * between the kernels and the sum.  The reference has no distributed mode
 * (its observation loop is src/PHT_MCMC_Aslett.c:325-337).
 */
struct RcclApi {
  bool ok = false;
  ncclResult_t (*getUniqueId)(ncclUniqueId *) = nullptr;
  ncclResult_t (*commInitRank)(ncclComm_t *, int, ncclUniqueId, int) = nullptr;
  ncclResult_t (*allReduce)(const void *, void *, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t,
                            hipStream_t) = nullptr;
  ncclResult_t (*commDestroy)(ncclComm_t) = nullptr;
  const char *(*errStr)(ncclResult_t) = nullptr;
};
static RcclApi &rccl() {
  static RcclApi a;
  static std::once_flag once;
  std::call_once(once, [] {
    void *h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!h) h = dlopen("librccl.so", RTLD_NOW | RTLD_LOCAL);
    if (!h) return;
    a.getUniqueId = (decltype(a.getUniqueId))dlsym(h, "ncclGetUniqueId");
    a.commInitRank = (decltype(a.commInitRank))dlsym(h, "ncclCommInitRank");
    a.allReduce = (decltype(a.allReduce))dlsym(h, "ncclAllReduce");
    a.commDestroy = (decltype(a.commDestroy))dlsym(h, "ncclCommDestroy");
    a.errStr = (decltype(a.errStr))dlsym(h, "ncclGetErrorString");
    a.ok = a.getUniqueId && a.commInitRank && a.allReduce && a.commDestroy && a.errStr;
  });
  return a;
}
static void rccl_destroy(ncclComm_t comm) {
  if (rccl().ok) (void)rccl().commDestroy(comm);
}

extern "C" int pht_rccl_unique_id(unsigned char *id) {
  if (!id) {
    set_err("pht_rccl_unique_id: null buffer");
    return -1;
  }
  if (!rccl().ok) {
    set_err("RCCL (librccl.so.1) could not be loaded");
    return -1;
  }
  ncclUniqueId u;
  const ncclResult_t r = rccl().getUniqueId(&u);
  if (r != ncclSuccess) {
    set_err("ncclGetUniqueId failed: %s", rccl().errStr(r));
    return -1;
  }
  memcpy(id, u.internal, NCCL_UNIQUE_ID_BYTES);
  return 0;
}

/* Every local precondition of pht_ctx_attach_rccl and pht_ctx_rccl_allreduce,
 * checked BEFORE any rank enters a collective: RCCL loadable, no communicator
 * attached yet, the device selectable, and the staging buffer of the
 * all-reduce self-test (max_len int64 words) allocated.  The caller agrees on
 * the verdict across ranks first (phasetype_amd/dist.py attach_rccl), so a
 * rank that fails here cannot leave its peers waiting in ncclCommInitRank. */
extern "C" int pht_ctx_rccl_prepare(pht_ctx *c, int max_len) {
  if (!c || max_len < 1) {
    set_err("pht_ctx_rccl_prepare: need a context and max_len >= 1");
    return -1;
  }
  if (c->comm) {
    set_err("pht_ctx_rccl_prepare: a communicator is already attached");
    return -1;
  }
  if (!rccl().ok) {
    set_err("RCCL (librccl.so.1) could not be loaded");
    return -1;
  }
  if (hipSetDevice(c->device) != hipSuccess) {
    set_err("pht_ctx_rccl_prepare: device %d", c->device);
    return -1;
  }
  if (c->d_rccl && c->rccl_cap < max_len) {
    (void)hipFree(c->d_rccl);
    c->d_rccl = nullptr;
    c->rccl_cap = 0;
  }
  if (!c->d_rccl) {
    if (hipMalloc(&c->d_rccl, sizeof(long long) * (size_t)max_len) != hipSuccess) {
      c->d_rccl = nullptr;
      set_err("pht_ctx_rccl_prepare: no device memory for %d words", max_len);
      return -1;
    }
  }
  /* the agreed word count of every later pht_ctx_rccl_allreduce (ranks
   * prepare with the same max_len; a larger buffer kept from before is
   * reduced only over these words) */
  c->rccl_cap = max_len;
  return 0;
}

/* The collective step only: ncclCommInitRank with the broadcast id.  Needs
 * pht_ctx_rccl_prepare first (agreed across ranks). */
extern "C" int pht_ctx_attach_rccl(pht_ctx *c, const unsigned char *id, int nranks, int rank) {
  if (!c || !id || nranks < 1 || rank < 0 || rank >= nranks) {
    set_err("pht_ctx_attach_rccl: need a context, a unique id and 0 <= rank < nranks");
    return -1;
  }
  if (c->comm || !c->d_rccl || !rccl().ok) {
    set_err("pht_ctx_attach_rccl: call pht_ctx_rccl_prepare first (and agree on it across ranks)");
    return -1;
  }
  (void)hipSetDevice(c->device);
  ncclUniqueId u;
  memcpy(u.internal, id, NCCL_UNIQUE_ID_BYTES);
  ncclComm_t comm = nullptr;
  const ncclResult_t r = rccl().commInitRank(&comm, nranks, u, rank);
  if (r != ncclSuccess) {
    set_err("ncclCommInitRank (rank %d of %d) failed: %s", rank, nranks, rccl().errStr(r));
    return -1;
  }
  c->comm = comm;
  return 0;
}

/* in-place sum of a host int64 vector over the context's communicator, on its
 * stream (the same all-reduce a sweep runs on its statistics block): the
 * attach-time self-test of phasetype_amd/dist.py compares it with
 * torch.distributed's sum.  The staging buffer comes from
 * pht_ctx_rccl_prepare; once the communicator exists this rank always enters
 * the all-reduce, even when its upload failed (the error is reported after
 * the collective), so its peers are never left waiting. */
extern "C" int pht_ctx_rccl_allreduce(pht_ctx *c, long long *buf, int len) {
  if (!c || !c->comm) {
    set_err("pht_ctx_rccl_allreduce: need a context with an RCCL communicator");
    return -1;
  }
  /* every rank reduces exactly the prepared word count (the same on every
   * rank, pht_ctx_rccl_prepare), whatever len it was given: a bad length on
   * one rank alone then still matches its peers' collective (its words are
   * zeros), and the error is reported afterwards */
  const bool badlen = !buf || len < 1 || len > c->rccl_cap;
  const int nred = c->rccl_cap;
  (void)hipSetDevice(c->device);
  hipError_t e = hipMemsetAsync(c->d_rccl, 0, sizeof(long long) * nred, c->stream);
  if (e == hipSuccess && !badlen)
    e = hipMemcpyAsync(c->d_rccl, buf, sizeof(long long) * len, hipMemcpyHostToDevice, c->stream);
  const ncclResult_t r = rccl().allReduce(c->d_rccl, c->d_rccl, (size_t)nred, ncclUint64, ncclSum, c->comm, c->stream);
  if (e == hipSuccess && r == ncclSuccess && !badlen)
    e = hipMemcpyAsync(buf, c->d_rccl, sizeof(long long) * len, hipMemcpyDeviceToHost, c->stream);
  const hipError_t es = hipStreamSynchronize(c->stream);
  if (e == hipSuccess) e = es;
  if (badlen) {
    set_err("pht_ctx_rccl_allreduce: need 1 <= len <= the prepared size (%d), got %d", c->rccl_cap, len);
    return -1;
  }
  if (r != ncclSuccess) {
    set_err("RCCL all-reduce failed: %s", rccl().errStr(r));
    return -1;
  }
  if (e != hipSuccess) {
    set_err("pht_ctx_rccl_allreduce: %s", hipGetErrorString(e));
    return -1;
  }
  return 0;
}

extern "C" int pht_device_count(void) {
  int c = 0;
  if (hipGetDeviceCount(&c) != hipSuccess) return 0;
  return c;
}

extern "C" pht_ctx *pht_ctx_create(int device, int n, int method, int mhit) {
  if (n < 1 || n > kMaxN) {
    set_err("n=%d outside 1..%d", n, kMaxN);
    return nullptr;
  }
  int ndev = 0;
  hipError_t e = hipGetDeviceCount(&ndev);
  if (e != hipSuccess || ndev == 0) {
    set_err("no HIP device available (%s)", hipGetErrorString(e));
    return nullptr;
  }
  if (device < 0 || device >= ndev) {
    set_err("device %d out of range (%d devices)", device, ndev);
    return nullptr;
  }
  if (dispatch_method(method) == kMethodMHRS && (mhit < 0 || mhit > 1022)) {
    set_err("mhit=%d outside 0..1022 (MHRS attempt streams carry the chain index in 10 bits)", mhit);
    return nullptr;
  }
  pht_ctx *c = new pht_ctx();
  c->device = device;
  c->n = n;
  c->method = c->rmethod = dispatch_method(method);
  c->mhit = mhit;
  /* bridge mode: MHRS or DCS path laws sampled exactly by the uniformisation
   * kernels (pht_unif.h) instead of the rejection search / Hobolth's
   * endpoint-conditioned sampler; same law, no eigensystem */
  {
    const char *em = getenv("PHT_MHRS"), *ed = getenv("PHT_DCS");
    if (c->rmethod == kMethodMHRS && em && !strcmp(em, "bridge")) {
      c->method = kMethodUNIF;
      c->ulaw = 1;
    } else if (c->rmethod == kMethodDCS && ed && !strcmp(ed, "bridge")) {
      c->method = kMethodUNIF;
      c->ulaw = 2;
    }
  }
  if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess ||
      hipMalloc(&c->d_params, make_layout(n).bytes()) != hipSuccess ||
      hipMalloc(&c->d_stats, sizeof(unsigned long long) * stats_len(n)) != hipSuccess ||
      hipHostMalloc(&c->h_stats, sizeof(unsigned long long) * stats_len(n), 0) != hipSuccess ||
      hipHostMalloc(&c->h_params, make_layout(n).bytes(), 0) != hipSuccess ||
      hipEventCreate(&c->ev0) != hipSuccess || hipEventCreate(&c->ev1) != hipSuccess ||
      hipStreamCreateWithFlags(&c->stream2, hipStreamNonBlocking) != hipSuccess ||
      hipEventCreateWithFlags(&c->evf, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&c->evj, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&c->evd, hipEventDisableTiming) != hipSuccess) {
    set_err("device %d: HIP allocation failed", device);
    delete c;
    return nullptr;
  }
  /* the published statistics (optional: without them the copy + event path) */
  if (!getenv("PHT_STATS_COPY")) {
    void *ho = nullptr, *hf = nullptr, *dout = nullptr, *dflag = nullptr;
    const unsigned fl = hipHostMallocCoherent | hipHostMallocMapped;
    if (hipHostMalloc(&ho, sizeof(unsigned long long) * stats_len(n), fl) == hipSuccess &&
        hipHostMalloc(&hf, 64, fl) == hipSuccess && hipHostGetDevicePointer(&dout, ho, 0) == hipSuccess &&
        hipHostGetDevicePointer(&dflag, hf, 0) == hipSuccess) {
      c->h_out = static_cast<unsigned long long *>(ho);
      c->d_out = static_cast<unsigned long long *>(dout);
      c->h_flag = static_cast<unsigned *>(hf);
      c->d_flag = static_cast<unsigned *>(dflag);
      *c->h_flag = 0u;
    } else {
      if (ho) (void)hipHostFree(ho);
      if (hf) (void)hipHostFree(hf);
      (void)hipGetLastError();
    }
  }
  /* the pipelined loop's gate and staged parameters (optional: without them,
   * or with PHT_PIPELINE=0, the loop enqueues each sweep after the last) */
  if (c->h_out && !(getenv("PHT_PIPELINE") && !strcmp(getenv("PHT_PIPELINE"), "0"))) {
    void *hg = nullptr, *hp = nullptr, *dg = nullptr, *dp = nullptr;
    const unsigned fl = hipHostMallocCoherent | hipHostMallocMapped;
    if (hipEventCreate(&c->ev0b) == hipSuccess && hipEventCreate(&c->ev1b) == hipSuccess &&
        hipHostMalloc(&hg, 128, fl) == hipSuccess && hipHostMalloc(&hp, make_layout(n).bytes(), fl) == hipSuccess &&
        hipHostGetDevicePointer(&dg, hg, 0) == hipSuccess && hipHostGetDevicePointer(&dp, hp, 0) == hipSuccess) {
      c->h_gate = static_cast<unsigned *>(hg);
      c->d_gate = static_cast<unsigned *>(dg);
      c->h_pg = static_cast<unsigned long long *>(hp);
      c->d_pg = static_cast<unsigned long long *>(dp);
      c->h_gate[0] = 0u;
      c->h_gate[16] = 0u;
    } else {
      if (hg) (void)hipHostFree(hg);
      if (hp) (void)hipHostFree(hp);
      (void)hipGetLastError();
    }
  }
  return c;
}

extern "C" void pht_ctx_destroy(pht_ctx *c) {
  if (!c) return;
  (void)hipSetDevice(c->device);
  ctx_free_obs(c);
  ctx_free_dbg(c);
  if (c->d_params) (void)hipFree(c->d_params);
  if (c->d_stats) (void)hipFree(c->d_stats);
  if (c->h_stats) (void)hipHostFree(c->h_stats);
  if (c->h_params) (void)hipHostFree(c->h_params);
  if (c->ev0) (void)hipEventDestroy(c->ev0);
  if (c->ev1) (void)hipEventDestroy(c->ev1);
  if (c->evf) (void)hipEventDestroy(c->evf);
  if (c->evj) (void)hipEventDestroy(c->evj);
  if (c->evd) (void)hipEventDestroy(c->evd);
  if (c->h_out) (void)hipHostFree(c->h_out);
  if (c->h_flag) (void)hipHostFree(c->h_flag);
  if (c->h_gate) (void)hipHostFree(c->h_gate);
  if (c->h_pg) (void)hipHostFree(c->h_pg);
  if (c->ev0b) (void)hipEventDestroy(c->ev0b);
  if (c->ev1b) (void)hipEventDestroy(c->ev1b);
  if (c->comm) rccl_destroy(c->comm);
  if (c->d_rccl) (void)hipFree(c->d_rccl);
  if (c->stream2) (void)hipStreamDestroy(c->stream2);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  delete c;
}

/* DCS end-state pre-pass from this many observations per shard */
constexpr long kDcsPrepassMin = 100000;

/*
 * Upload this shard's observations.  obs0 = global index of y[0]; the
 * Philox counter of observation i is obs0 + i whatever the shard layout.
 * Observations are reordered on the device (exact before censored, see
 * below); results do not depend on the order.
 */
extern "C" int pht_ctx_set_obs(pht_ctx *c, const double *y, const int *cens, long count, long obs0) {
  HIPCHK(hipSetDevice(c->device));
  ctx_free_obs(c);
  ctx_free_dbg(c);
  c->count = count;
  c->n_exact = 0;
  c->ysum = 0.0;
  c->ymax = 0.0;
  c->h_ysorted.clear();
  c->order.clear();
  if (count == 0) return 0;
  std::vector<long> ord(count);
  std::iota(ord.begin(), ord.end(), 0L);
  /* by decreasing y, so the persistent kernels hand out long paths first
   * and end on short ones (a short tail).  Exact observations first, then
   * censored ones, each by decreasing y: ECS runs the two as ranges of their
   * own (two kernels, two streams), and MHRS's and UNIF's code paths differ
   * for censored observations (a wavefront of one kind does not diverge).
   * DCS treats censored observations as exact (the reference's DCS law), so
   * its one kernel takes the whole shard by decreasing y (r04: the censored
   * range's long paths started two thirds of the way through the kernel and
   * set its tail; cfg5 DCS 1.19 -> 0.89 ms).  PHT_ORDER=asc|none: A/B of
   * ECS's exact range. */
  const bool split = !(c->method == kMethodDCS || (c->method == kMethodUNIF && c->ulaw == 2));
  const char *oe = getenv("PHT_ORDER");
  const int omode = !oe ? 0 : (!strcmp(oe, "asc") ? 1 : (!strcmp(oe, "none") ? 2 : 0));
  std::stable_sort(ord.begin(), ord.end(), [&](long a, long b) {
    const int ca = cens[a] != 0, cb = cens[b] != 0;
    if (!split) return y[a] > y[b];
    if (ca != cb) return ca < cb;
    if (ca) return y[a] > y[b];
    if (omode == 2) return false;
    return omode == 1 ? (y[a] < y[b]) : (y[a] > y[b]);
  });
  std::vector<double> ys(count);
  std::vector<int> cs(count);
  std::vector<uint32_t> gs(count);
  for (long k = 0; k < count; k++) {
    ys[k] = y[ord[k]];
    cs[k] = cens[ord[k]];
    gs[k] = (uint32_t)(obs0 + ord[k]);
  }
  c->n_exact = 0;
  if (split) {
    while (c->n_exact < count && cs[c->n_exact] == 0) c->n_exact++;
  } else {
    for (long k = 0; k < count; k++) c->n_exact += (cs[k] == 0); /* (not a range here) */
  }
  c->h_ysorted = ys;
  c->ysum = 0.0;
  c->ymax = 0.0;
  for (double v : ys) {
    c->ysum += v;
    c->ymax = std::max(c->ymax, v);
  }
  c->order = std::move(ord);
  HIPCHK(hipMalloc(&c->d_y, sizeof(double) * count));
  HIPCHK(hipMalloc(&c->d_cens, sizeof(int) * count));
  HIPCHK(hipMalloc(&c->d_gid, sizeof(uint32_t) * count));
  HIPCHK(hipMemcpy(c->d_y, ys.data(), sizeof(double) * count, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(c->d_cens, cs.data(), sizeof(int) * count, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(c->d_gid, gs.data(), sizeof(uint32_t) * count, hipMemcpyHostToDevice));
  if (c->method == kMethodMHRS) {
    const size_t tasks = (size_t)count * (size_t)(1 + c->mhit);
    HIPCHK(hipMalloc(&c->d_mbest, sizeof(uint32_t) * tasks));
    HIPCHK(hipMalloc(&c->d_mq0, sizeof(uint32_t) * tasks));
    HIPCHK(hipMalloc(&c->d_mq1, sizeof(uint32_t) * tasks));
    HIPCHK(hipMalloc(&c->d_mcnt, sizeof(unsigned) * kMhrsCounters));
  }
  /* DCS: for large shards the end states come from a pre-pass kernel
   * (dcs_end_kernel; results identical).  Measured (profiles/r03/dcs_prepass/):
   * -4 % kernel time at n = 10, N = 10^6, -2 % at cfg5, flat at n = 5/20,
   * +6 % at N = 200 (one more launch).  PHT_DCS_PREPASS=1|0 forces it. */
  {
    const char *e = getenv("PHT_DCS_PREPASS");
    const bool pre = e ? atoi(e) != 0 : count >= kDcsPrepassMin;
    if (c->method == kMethodDCS && pre) HIPCHK(hipMalloc(&c->d_dcsb, sizeof(int) * count));
  }
  return 0;
}

/* blocks per CU for the persistent ECS kernel (PHT_ECS_OCC forces it) */
static int exact_occ(const pht_ctx *c) {
  if (const char *e = getenv("PHT_ECS_OCC")) return atoi(e);
  (void)c;
  return 0;
}

/* exact observations (the longest, positions [0, k) of the decreasing-y
 * order) that run one per 16-lane row (pht_ecs_row.h) instead of one per
 * lane; PHT_ROWK=k forces k (results are identical for every k) */
static long exact_rowk(const pht_ctx *c) {
  if (const char *e = getenv("PHT_ROWK")) return std::max(0L, std::min(atol(e), c->n_exact));
  /* by exact observations per one-lane slot (kSpreadLanes ~ the resident
   * lanes of one MI355X); measured (tools/rowk_sweep.sh, tools/latency.py,
   * profiles/r02/rows): the fewer per lane, the more the longest paths set
   * the sweep time and the more rows pay (the launcher caps rows at half
   * the resident blocks) */
  const long L = kSpreadLanes;
  if (c->n_exact * 10 <= 6 * L) return 4096; /* 62.5k: 0.44 ms (1,024: 0.48; none: 0.56) */
  /* the 8-GPU shards of cfg4 (125k each, r04 kernels; profiles/r04/rowk):
   * max over the 8 real shards 0.487 ms at 2,048, 0.508 at 1,024, 0.498 at
   * 4,096, 0.517 at 512 */
  if (c->n_exact * 10 <= 12 * L) return 2048;
  /* the 4-GPU shards of cfg4 (250k each; r05 kernels, profiles/r05/shards_curve/): slowest shard
   * 0.621 / 0.621 / 0.630 ms at 4,096 against 0.641 / 0.627 / 0.641 at 1,024 (r02's kernels
   * preferred 1,024: 0.57 vs 0.59 ms) */
  if (c->n_exact <= 2 * L) return c->n == 10 ? 4096 : 1024; /* measured at n = 10 only: elsewhere r04's 1,024 */
  if (c->n_exact <= 5 * L) return 128;       /* cfg5's 350k exact: +5 % */
  return 0;                                  /* cfg4's 10^6: rows cost the one-lane range more (K = 64: +1 %) */
}

/* UNIF: size (and grow) the context's table for this sweep's parameters
 * (c->h_params): the shard's largest lam = mu y with a Poisson margin
 * (pht_unif.h).  Beyond kUnifMaxK rows or lam > kUnifMaxLam an observation
 * cannot be sampled exactly: it is counted in kXUnifCap and gibbs_run fails
 * the sweep */
static int unif_prepare(pht_ctx *c, SweepArgs &a) {
  const Layout L = make_layout(c->n);
  const double *S = reinterpret_cast<const double *>(c->h_params) + L.S;
  double mu = 0.0;
  for (int i = 0; i < c->n; i++) mu = std::max(mu, -S[i + i * c->n]);
  if (!(mu > 0.0) || !std::isfinite(mu)) {
    set_err("UNIF: the generator's largest exit rate is %g (need a positive finite rate)", mu);
    return -1;
  }
  const double lmax = mu * c->ymax;
  const double kd = std::ceil(lmax + 14.0 * std::sqrt(lmax) + 64.0);
  a.uK = (int)std::min<double>(kUnifMaxK, std::isfinite(kd) ? kd : (double)kUnifMaxK);
  a.uymax = c->ymax;
  const long need = unif_tab_doubles(c->n, a.uK);
  if (need > c->utab_cap) {
    if (c->d_utab) HIPCHK(hipFree(c->d_utab));
    c->d_utab = nullptr;
    const long cap = std::max(need, unif_tab_doubles(c->n, std::min(kUnifMaxK, a.uK * 3 / 2)));
    HIPCHK(hipMalloc(&c->d_utab, sizeof(double) * cap));
    c->utab_cap = cap;
  }
  a.utab = c->d_utab;
  return 0;
}

/* DCS jump-time root finder: PHT_DCS_ROOT=brent selects the reference's
 * Find02 search (src/utility.c:233-338) over the default safeguarded Halley
 * iteration (pht_dcs_round.h hob_halley); read per sweep */
static int dcs_brent() {
  const char *e = getenv("PHT_DCS_ROOT");
  return (e && !strcmp(e, "brent")) ? 1 : 0;
}

/* the sweep kernels of one context on its stream(s): ECS exact and censored
 * ranges concurrently (stream2 joined back), the other samplers in one
 * launch; a carries the sweep's common arguments (ctx_enqueue, and the
 * resident chain per sweep) */
static int ctx_launch(pht_ctx *c, const SweepArgs &a, bool debug) {
  if (c->method == kMethodECS) {
    /* exact observations: persistent ECS kernel; censored: LJMA_samplechain path */
    SweepArgs ae = a;
    ae.begin = 0;
    ae.count = c->n_exact;
    ae.cens = nullptr;
    ae.occ = exact_occ(c);
    ae.rowk = exact_rowk(c);
    ae.rowprio = getenv("PHT_ROWPRIO") ? atoi(getenv("PHT_ROWPRIO")) : 3;
    /* lane-major first claims when the shard is within ~2 observations per
     * lane (the longest paths, one per wavefront; tools/latency.py:
     * -10 % at 31k-125k per GPU); PHT_SPREAD=0|1 forces it */
    /* one new observation per lane per round (PHT_NEWCAP=0: no limit;
     * tools/latency.py: -2 % kernel time at 1e6) */
    ae.newcap = getenv("PHT_NEWCAP") ? atoi(getenv("PHT_NEWCAP")) : 1;
    ae.spread = getenv("PHT_SPREAD") ? atoi(getenv("PHT_SPREAD")) : (c->n_exact <= 2 * kSpreadLanes);
    /* PHT_HOT=k: the remaining-time threshold is the k-th longest exact y */
    {
      const long hk = getenv("PHT_HOT") ? atol(getenv("PHT_HOT")) : 0;
      ae.hoty = (hk > 0 && hk <= c->n_exact) ? c->h_ysorted[hk - 1] : 0.0;
    }
    SweepArgs ac = a;
    ac.begin = c->n_exact;
    ac.count = c->count - c->n_exact;
    ac.allcens = 1; /* positions [n_exact, count) hold the censored observations */
    /* both ranges: the censored kernel on stream2, concurrently, so each
     * persistent kernel's tail (its longest paths) fills with the other's
     * work; cfg5 ECS 2.49 -> 1.92 ms; the launch order does not matter
     * (PHT_CENS_SERIAL=1: one stream) */
    const bool fork = ae.count > 0 && ac.count > 0 && !getenv("PHT_CENS_SERIAL");
    /* n >= 15: the exact kernel's LDS now allows two blocks per CU (compact
     * parameter prefix, r04), which pays alone (n = 15, 5e5 exact: 1.178 ->
     * 1.038 ms) but crowds out the concurrent censored kernel (cfg5: 1.224
     * -> 1.482 ms; profiles/r04/ecs_lds/): with a censored range running
     * beside it, one block per CU as before */
    if (fork && c->n >= 15 && !getenv("PHT_ECS_OCC")) ae.occ = 1;
    if (fork) {
      HIPCHK(hipEventRecord(c->evf, c->stream));
      HIPCHK(hipStreamWaitEvent(c->stream2, c->evf, 0));
      HIPCHK(pht_launch_sweep(&ac, c->method, debug ? 1 : 0, c->stream2));
      HIPCHK(hipEventRecord(c->evj, c->stream2));
      HIPCHK(pht_launch_sweep(&ae, c->method, debug ? 1 : 0, c->stream));
      HIPCHK(hipStreamWaitEvent(c->stream, c->evj, 0));
    } else {
      if (ae.count > 0) HIPCHK(pht_launch_sweep(&ae, c->method, debug ? 1 : 0, c->stream));
      if (ac.count > 0) HIPCHK(pht_launch_sweep(&ac, c->method, debug ? 1 : 0, c->stream));
    }
  } else {
    HIPCHK(pht_launch_sweep(&a, c->method, debug ? 1 : 0, c->stream));
  }
  return 0;
}

/* gate != 0: the pipelined loop's next sweep, enqueued while the current one
 * runs; its parameters come from c->h_pg once the host releases `gate`
 * (pht_gate_kernel), not from c->h_params now */
static int ctx_enqueue(pht_ctx *c, uint32_t k0, uint32_t k1, uint32_t sweep, int zexp, bool debug,
                       bool timed = true, unsigned gate = 0) {
  HIPCHK(hipSetDevice(c->device));
  if (c->nin >= 2 || (gate && (c->nin != 1 || !c->h_gate || !c->h_out))) {
    set_err("internal: sweep enqueued with %d in flight (gate %u)", c->nin, gate);
    return -1;
  }
  const int pb = make_layout(c->n).bytes();
  const int sl = stats_len(c->n);
  const int evs = (int)(c->nenq++ & 1u) && c->ev0b ? 1 : 0;
  hipEvent_t e0 = evs ? c->ev0b : c->ev0, e1 = evs ? c->ev1b : c->ev1;
  if (gate) {
    HIPCHK(pht_launch_gate(c->d_gate, gate, c->d_pg, reinterpret_cast<unsigned long long *>(c->d_params), pb / 8,
                           c->d_gate + 16, c->stream));
  } else {
    HIPCHK(hipMemcpyAsync(c->d_params, c->h_params, pb, hipMemcpyHostToDevice, c->stream));
  }
  /* the block is zeroed at the end of the previous sweep, after its copy to
   * the host (off the critical path: it runs while the host does the Gamma
   * update); only the first sweep, or one after a failed enqueue, zeroes it
   * here */
  if (!c->stats_zero) HIPCHK(hipMemsetAsync(c->d_stats, 0, sizeof(unsigned long long) * sl, c->stream));
  c->stats_zero = false;
  SweepArgs a;
  memset(&a, 0, sizeof a);
  a.params = c->d_params;
  a.n = c->n;
  a.mhit = c->mhit;
  a.ulaw = c->ulaw;
  a.count = c->count;
  a.y = c->d_y;
  a.cens = c->d_cens;
  a.gid = c->d_gid;
  a.k0 = k0;
  a.k1 = k1;
  a.sweep = sweep;
  a.zscale = ldexp(1.0, zexp);
  a.dcsbrent = dcs_brent();
  a.dcsb = c->d_dcsb;
  a.stats = c->d_stats;
  a.mbest = c->d_mbest;
  a.mq0 = c->d_mq0;
  a.mq1 = c->d_mq1;
  a.mcnt = c->d_mcnt;
  if (debug) {
    if (c->dbg_cap < c->count) {
      ctx_free_dbg(c);
      HIPCHK(hipMalloc(&c->d_zq, sizeof(long long) * c->count * c->n));
      HIPCHK(hipMalloc(&c->d_N, sizeof(int) * c->count * c->n * c->n));
      HIPCHK(hipMalloc(&c->d_B, sizeof(int) * c->count));
      HIPCHK(hipMalloc(&c->d_pre, sizeof(int) * c->count));
      HIPCHK(hipMalloc(&c->d_flags, sizeof(int) * c->count));
      HIPCHK(hipMalloc(&c->d_ndraw, sizeof(uint32_t) * c->count));
      c->dbg_cap = c->count;
    }
    HIPCHK(hipMemsetAsync(c->d_zq, 0, sizeof(long long) * c->count * c->n, c->stream));
    HIPCHK(hipMemsetAsync(c->d_N, 0, sizeof(int) * c->count * c->n * c->n, c->stream));
    HIPCHK(hipMemsetAsync(c->d_B, 0, sizeof(int) * c->count, c->stream));
    HIPCHK(hipMemsetAsync(c->d_pre, 0, sizeof(int) * c->count, c->stream));
    a.dbg_zq = c->d_zq;
    a.dbg_N = c->d_N;
    a.dbg_B = c->d_B;
    a.dbg_pre = c->d_pre;
    a.dbg_flags = c->d_flags;
    a.dbg_ndraw = c->d_ndraw;
  }
  if (c->method == kMethodUNIF && unif_prepare(c, a)) return -1;
  /* the kernel-time markers: the GPU idles while the host enqueues them
   * (~9 us per sweep at cfg4, profiles/r06/kernel_events/), so the Gibbs loop
   * records them on a sample of its sweeps only */
  if (timed) HIPCHK(hipEventRecord(e0, c->stream));
  if (ctx_launch(c, a, debug)) return -1;
  if (timed) HIPCHK(hipEventRecord(e1, c->stream));
  if (c->comm) {
    /* multi-process: the block summed over all ranks in place, on the sweep's
     * stream, before the one copy to the host (pht_ctx_attach_rccl) */
    const ncclResult_t r = rccl().allReduce(c->d_stats, c->d_stats, (size_t)sl, ncclUint64, ncclSum, c->comm, c->stream);
    if (r != ncclSuccess) {
      set_err("RCCL all-reduce of the statistics failed: %s", rccl().errStr(r));
      return -1;
    }
  }
  if (c->h_out) {
    /* one small kernel publishes the block and zeroes it; ctx_wait polls the
     * flag (kernel end -> host sees the statistics: the blit copy's dispatch,
     * its copy and the event's completion signal replaced by one dispatch and
     * a store over the link; profiles/r05/stats_out/) */
    if (++c->seq == 0u) c->seq = 1u;
    HIPCHK(pht_launch_stats_out(c->d_stats, c->d_out, c->d_flag, c->seq, sl, c->stream));
  } else {
    HIPCHK(hipMemcpyAsync(c->h_stats, c->d_stats, sizeof(unsigned long long) * sl, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipEventRecord(c->evd, c->stream)); /* ctx_wait waits for this, not for the zeroing */
    HIPCHK(hipMemsetAsync(c->d_stats, 0, sizeof(unsigned long long) * sl, c->stream));
  }
  c->stats_zero = true;
  pht_ctx::Inflight &f = c->infl[c->nin++];
  f.seq = c->seq;
  f.gate = gate;
  f.timed = timed;
  f.evs = evs;
  return 0;
}

/* sweeps left in flight by an earlier call that failed: finish them and
 * forget their records (their statistics are stale), so the next wait
 * cannot take one of them for its own sweep */
static void ctx_drain(pht_ctx *c) {
  if (c->nin) {
    (void)hipSetDevice(c->device);
    (void)hipStreamSynchronize(c->stream);
    c->nin = 0;
    c->stats_zero = false;
  }
}

/* release the pipelined sweep waiting at `gate`: its parameter block (pb
 * bytes) into the staging buffer, then the gate word (release store; the
 * gate kernel's acquire load orders its copy after it) */
static void ctx_release(pht_ctx *c, unsigned gate, const unsigned char *pb, size_t bytes) {
  if (pb) memcpy(c->h_pg, pb, bytes);
  __atomic_store_n(c->h_gate, gate, __ATOMIC_RELEASE);
}

/* the flag pht_stats_out_kernel sets for this sweep; the stream is queried
 * now and then, so a failed or finished-without-flag sweep ends the wait */
/* host threads inside wait_stats_flag right now: with more than one (several
 * chains driven from several threads, pht_gibbs_run_chains) a waiter yields
 * its core to the others' host work instead of pausing on it */
static std::atomic<int> g_stat_waiters{0};

static int wait_stats_flag_spin(pht_ctx *c, unsigned want);
static int wait_stats_flag(pht_ctx *c, unsigned want) {
  g_stat_waiters.fetch_add(1, std::memory_order_relaxed);
  const int rc = wait_stats_flag_spin(c, want);
  g_stat_waiters.fetch_sub(1, std::memory_order_relaxed);
  return rc;
}

static int wait_stats_flag_spin(pht_ctx *c, unsigned want) {
  for (unsigned long spin = 1;; spin++) {
    if (__atomic_load_n(c->h_flag, __ATOMIC_ACQUIRE) == want) return 0;
    if (g_stat_waiters.load(std::memory_order_relaxed) > 1) sched_yield();
    if ((spin & 1023ul) == 0ul) {
      const hipError_t e = hipStreamQuery(c->stream);
      if (e == hipSuccess) {
        if (__atomic_load_n(c->h_flag, __ATOMIC_ACQUIRE) == want) return 0;
        set_err("device %d: the sweep finished without publishing its statistics", c->device);
        return -1;
      }
      if (e != hipErrorNotReady) {
        set_err("device %d: %s", c->device, hipGetErrorString(e));
        return -1;
      }
    }
#if defined(__x86_64__)
    __builtin_ia32_pause();
#endif
  }
}

/* the oldest sweep in flight: its statistics into c->h_stats, its kernel
 * time into c->last_ms (-1 when it was not timed) */
static int ctx_wait(pht_ctx *c) {
  HIPCHK(hipSetDevice(c->device));
  if (c->nin < 1) {
    set_err("internal: no sweep in flight");
    return -1;
  }
  const pht_ctx::Inflight f = c->infl[0];
  c->infl[0] = c->infl[1];
  c->nin--;
  hipEvent_t e0 = f.evs ? c->ev0b : c->ev0, e1 = f.evs ? c->ev1b : c->ev1;
  if (c->h_out) {
    if (wait_stats_flag(c, f.seq)) return -1;
    memcpy(c->h_stats, c->h_out, sizeof(unsigned long long) * stats_len(c->n));
    if (f.gate && __atomic_load_n(c->h_gate + 16, __ATOMIC_ACQUIRE) != f.gate) {
      set_err("device %d: a pipelined sweep's parameters were not released in time (gate %u, ack %u)", c->device,
              f.gate, __atomic_load_n(c->h_gate + 16, __ATOMIC_ACQUIRE));
      return -1;
    }
    if (f.timed) {
      /* ev1 precedes the publishing kernel on the stream: it has completed */
      hipError_t e = hipEventElapsedTime(&c->last_ms, e0, e1);
      if (e == hipErrorNotReady) {
        HIPCHK(hipEventSynchronize(e1));
        e = hipEventElapsedTime(&c->last_ms, e0, e1);
      }
      HIPCHK(e);
    }
  } else {
    HIPCHK(hipEventSynchronize(c->evd));
    if (f.timed) HIPCHK(hipEventElapsedTime(&c->last_ms, e0, e1));
  }
  if (!f.timed) c->last_ms = -1.f; /* not measured this sweep */
  if (c->method == kMethodMHRS && c->d_mcnt && getenv("PHT_MHRS_COUNTS")) {
    /* diagnostics: tasks still unresolved after MHRS search rounds 0..4 */
    unsigned q[5];
    HIPCHK(hipMemcpy(q, c->d_mcnt, sizeof q, hipMemcpyDeviceToHost));
    fprintf(stderr, "[pht] MHRS unresolved after rounds 0-4: %u %u %u %u %u (of %ld tasks)\n", q[0], q[1], q[2],
            q[3], q[4], c->count * (1 + c->mhit));
  }
  return 0;
}

extern "C" int pht_ctx_sweep(pht_ctx *c, const double *S, const double *s, uint32_t k0, uint32_t k1,
                             uint32_t sweep, int zexp, long long *stats_out) {
  std::vector<unsigned char> pb;
  int info = build_params(c->n, S, s, c->method, pb);
  if (info < 0) return info;
  memcpy(c->h_params, pb.data(), pb.size());
  ctx_drain(c);
  if (ctx_enqueue(c, k0, k1, sweep, zexp, false) || ctx_wait(c)) return -1;
  memcpy(stats_out, c->h_stats, sizeof(long long) * stats_len(c->n));
  return 0;
}

/* Per-observation debug sweep: outputs in the caller's original observation
 * order (B, pre, flags, ndraw [count]; zq [count*n]; N [count*n*n], N[i + j n]). */
extern "C" int pht_ctx_sweep_debug(pht_ctx *c, const double *S, const double *s, uint32_t k0, uint32_t k1,
                                   uint32_t sweep, int zexp, long long *stats_out, int *B, int *pre, int *flags,
                                   uint32_t *ndraw, long long *zq, int *N) {
  std::vector<unsigned char> pb;
  int info = build_params(c->n, S, s, c->method, pb);
  if (info < 0) return info;
  memcpy(c->h_params, pb.data(), pb.size());
  ctx_drain(c);
  if (ctx_enqueue(c, k0, k1, sweep, zexp, true) || ctx_wait(c)) return -1;
  memcpy(stats_out, c->h_stats, sizeof(long long) * stats_len(c->n));
  const long cnt = c->count;
  const int n = c->n;
  std::vector<long long> hz(cnt * n);
  std::vector<int> hN(cnt * n * n), hB(cnt), hp(cnt), hf(cnt);
  std::vector<uint32_t> hd(cnt);
  HIPCHK(hipMemcpy(hz.data(), c->d_zq, sizeof(long long) * cnt * n, hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(hN.data(), c->d_N, sizeof(int) * cnt * n * n, hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(hB.data(), c->d_B, sizeof(int) * cnt, hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(hp.data(), c->d_pre, sizeof(int) * cnt, hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(hf.data(), c->d_flags, sizeof(int) * cnt, hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(hd.data(), c->d_ndraw, sizeof(uint32_t) * cnt, hipMemcpyDeviceToHost));
  for (long k = 0; k < cnt; k++) {
    const long o = c->order[k];
    B[o] = hB[k];
    pre[o] = hp[k];
    flags[o] = hf[k];
    ndraw[o] = hd[k];
    memcpy(zq + o * n, hz.data() + k * n, sizeof(long long) * n);
    memcpy(N + o * n * n, hN.data() + k * n * n, sizeof(int) * n * n);
  }
  return 0;
}

extern "C" float pht_ctx_last_kernel_ms(pht_ctx *c) { return c->last_ms; }
extern "C" long long pht_ctx_flagged_obs(pht_ctx *c) { return c->flagged; }
extern "C" int pht_ctx_set_global_count(pht_ctx *c, long long total) {
  if (!c || total < c->count) {
    set_err("pht_ctx_set_global_count: the total (%lld) must cover this shard's %ld observations", total,
            c ? c->count : 0L);
    return -1;
  }
  c->global_count = total;
  return 0;
}

/* fixed-point exponent for z: 52 - e with sum(y) < 2^e
 * (frexp), so the exact-observation total stays below 2^52 whatever the
 * time scale of the data (11 bits of int64 headroom are left for censored
 * paths running past y).  Clamped so 2^zexp is a finite normal double;
 * an empty, zero or non-finite sum gives 52. */
extern "C" int pht_zexp(const double *y, long l) {
  double sy = 0.0;
  for (long i = 0; i < l; i++) sy += y[i];
  if (!(sy > 0.0) || !std::isfinite(sy)) return 52;
  int e = 0;
  (void)frexp(sy, &e);
  return std::min(1000, std::max(-1000, 52 - e));
}

/* ============================================================ Gibbs core */
namespace {
struct Ent {
  int i, j;
  double c;
};

/* The reference's Gibbs bookkeeping (src/PHT_MCMC_Aslett.c:187-405) with
 * the linked lists kept as arrays visited in list (reverse-insertion)
 * order, so zsum and the diagonal refresh sum in the reference's order. */
struct GibbsState {
  int it, n, m, n1;
  const double *nu, *zeta;
  double *res;
  std::vector<double> TT, S, s;
  std::vector<std::vector<Ent>> Nl, Sl, sl, zl, TTl, Dl;

  template <class Rng>
  GibbsState(Rng &R, int it_, int n_, int m_, const double *nu_, const double *zeta_, const int *T, const double *C,
             const double *start, double *res_)
      : it(it_), n(n_), m(m_), n1(n_ + 1), nu(nu_), zeta(zeta_), res(res_) {
    TT.assign(n1 * n1, 0.0);
    S.assign(n * n, 0.0);
    s.assign(n, 0.0);
    Nl.resize(m); Sl.resize(m); sl.resize(m); zl.resize(m); TTl.resize(m); Dl.resize(n1);
    if (start[0] < 0) {
      for (int i = 0; i < m; i++)
        res[0 + (size_t)i * it] = (nu[i] > 1) ? (nu[i] - 1.0) / zeta[i] : R.gamma(nu[i], 1.0 / zeta[i]);
    } else {
      for (int i = 0; i < m; i++) res[0 + (size_t)i * it] = start[i];
    }
    double rsum = 0.0;
    for (int i = 0; i < n1; i++) {
      for (int j = 0; j < n1; j++) {
        const int t = T[i + j * n1];
        if (t == 0) {
          TT[i + j * n1] = 0.0;
          continue;
        }
        const int k = t - 1;
        const double c = C[i + j * n1];
        rsum -= TT[i + j * n1] = res[0 + (size_t)k * it] * c;
        if (j == n) {
          Nl[k].push_back({i, i, 1.0});
          sl[k].push_back({i, 0, c});
        } else {
          Nl[k].push_back({i, j, 1.0});
          Sl[k].push_back({i, j, c});
        }
        zl[k].push_back({i, 0, c});
        TTl[k].push_back({i, j, c});
        Dl[i].push_back({i, j, 1.0});
      }
      TT[i + i * n1] = rsum;
      rsum = 0.0;
    }
    for (int i = 0; i < n; i++)
      for (int j = 0; j < n; j++) S[i + j * n] = TT[i + j * n1];
    for (int i = 0; i < n; i++) s[i] = TT[i + n * n1];
  }

  /* steps 4-5 (:340-397): compile statistics and draw from the posteriors */
  template <class Rng>
  void update(Rng &R, int iter, const double *z, const long long *Nt) {
    std::vector<long long> Nsum(m, 0);
    std::vector<double> zsum(m, 0.0);
    for (int k = 0; k < m; k++) {
      for (int e = (int)Nl[k].size() - 1; e >= 0; e--) Nsum[k] += Nt[Nl[k][e].i + Nl[k][e].j * n];
      for (int e = (int)zl[k].size() - 1; e >= 0; e--) zsum[k] += z[zl[k][e].i] / zl[k][e].c;
    }
    for (int k = 0; k < m; k++) {
      const double tmp = res[iter + (size_t)k * it] =
          R.gamma(nu[k] + (double)(int)Nsum[k], 1.0 / (zeta[k] + zsum[k]));
      for (int e = (int)TTl[k].size() - 1; e >= 0; e--) TT[TTl[k][e].i + TTl[k][e].j * n1] = tmp * TTl[k][e].c;
      for (int e = (int)Sl[k].size() - 1; e >= 0; e--) S[Sl[k][e].i + Sl[k][e].j * n] = tmp * Sl[k][e].c;
      for (int e = (int)sl[k].size() - 1; e >= 0; e--) s[sl[k][e].i] = tmp * sl[k][e].c;
    }
    for (int i = 0; i < n; i++) {
      double tmp = 0.0;
      for (int e = (int)Dl[i].size() - 1; e >= 0; e--) tmp -= TT[Dl[i][e].i + Dl[i][e].j * n1];
      TT[i + i * n1] = tmp;
      S[i + i * n] = tmp;
    }
  }
};

/* Run the Gibbs loop over a set of device shards; reduce = optional
 * cross-process all-reduce of the int64 statistics block. */
template <class Rng>
int gibbs_run(Rng &R, int it, int mhit, int method, int n, int m, const double *nu, const double *zeta, const int *T,
              const double *C, const double *y, long l, int silent, const double *start, double *res,
              std::vector<pht_ctx *> &ctxs, uint32_t k0, uint32_t k1, int zexp, pht_reduce_fn reduce,
              void *reduce_user, double *kernel_ms_total) {
  (void)y; (void)l; (void)mhit;
  GibbsState G(R, it, n, m, nu, zeta, T, C, start, res);
  OneBlasThread one; /* the per-sweep eigensystems on this thread */
  const int disp = dispatch_method(method);
  const int sl = stats_len(n);
  std::vector<long long> tot(sl);
  std::vector<double> z(n);
  std::vector<unsigned char> pb;
  say("Starting phase-type MCMC sampler ...\n\nBegining processing ...");
  if (silent) say(" silent processing selected, there will be no further feedback until MCMC run complete");
  /* kernel time: the sweeps' events on one sweep in `every` (the last of
   * each group, so a fresh chain's first and slowest sweeps do not weigh
   * more than their share; PHT_KTIME_EVERY, default 4, 1 = every sweep; the
   * last sweep when no other was timed), the total scaled from their mean;
   * chain groups time every sweep */
  const int every = std::max(1, getenv("PHT_KTIME_EVERY") ? atoi(getenv("PHT_KTIME_EVERY")) : 4);
  auto want_time = [&](int k) { return k % every == 0 || (k == it - 1 && k - 1 < every); };
  double kms = 0.0;
  long ktimed = 0;
  long long flagged = 0;
  /* Pipelined loop (contexts not in a chains group, not UNIF, whose enqueue
   * reads the parameters): sweep k + 1 is enqueued as soon as sweep k is,
   * behind a gate kernel per context that waits for its parameters, so the
   * launch work runs while sweep k does and only the Gamma update and the
   * next parameter block stay between two sweeps (PHT_PIPELINE=0: off).  The
   * draws are the same: sweep k + 1's parameters are those the update
   * produced from sweep k's statistics. */
  for (pht_ctx *c : ctxs)
    if (!c->grp) ctx_drain(c);
  bool pipe = !ctxs.empty() && it > 2;
  for (pht_ctx *c : ctxs) pipe = pipe && !c->grp && c->h_gate && c->method != kMethodUNIF && !c->ulaw;
  bool pending = false;                        /* every context holds a gated sweep */
  std::vector<unsigned> pgate(ctxs.size(), 0u); /* its gate (0: none enqueued) */
  /* an early return with gated sweeps enqueued: release them (they run on
   * the last staged parameters) and drain the streams, so nothing waits on
   * a gate */
  auto unwind = [&]() {
    for (size_t i = 0; i < ctxs.size(); i++) {
      if (pgate[i]) {
        ctx_release(ctxs[i], pgate[i], nullptr, 0);
        (void)hipStreamSynchronize(ctxs[i]->stream);
        ctxs[i]->nin = 0;
        pgate[i] = 0u;
      }
    }
    pending = false;
  };
  int first_flagged = 0;
  /* every sweep must account for every observation of every shard: the
   * node-wide processed count (extra word kXObs, after the reduce) is checked
   * against it, so a launch-shape bug that drops observations, or a reduce
   * that sums a block twice or not at all, fails the run instead of biasing
   * the posterior.  Multi-process: the count comes from
   * pht_ctx_set_global_count (unchecked when it was not given). */
  long long expect = 0;
  {
    bool multi = reduce != nullptr;
    for (pht_ctx *c : ctxs) {
      expect += c->count;
      multi = multi || c->comm != nullptr;
    }
    if (multi) expect = ctxs.size() == 1 ? ctxs[0]->global_count : -1;
  }
  /* the observed times alone must fit the fixed point with room to spare */
  for (pht_ctx *c : ctxs) {
    if (!(ldexp(c->ysum, zexp) < 0x1p62)) {
      set_err("zexp = %d overflows the fixed-point z sums: the shard's observed times total %g (pht_zexp gives %d)",
              zexp, c->ysum, pht_zexp(c->h_ysorted.data(), (long)c->h_ysorted.size()));
      return -1;
    }
  }
  for (int iter = 1; iter < it; iter++) {
    if (!silent) say("\rProcessing iteration %d of %d (%.1lf%%)\r", iter + 1, it, (100.0 * (iter + 1)) / it);
    if (!disp) {
      say("CRITICAL ERROR: Unknown sampling method (code = %d)\n\n", method);
      continue;
    }
    /* bridge contexts run the UNIF kernels: their block needs no eigensystem */
    const int bm = ctxs[0]->ulaw ? kMethodUNIF : (disp == kMethodMHRS ? kMethodMHRS : method);
    const int info = build_params(n, G.S.data(), G.s.data(), bm, pb);
    if (info < 0) {
      unwind();
      return -1;
    }
    const bool timed = want_time(iter);
    if (pending) {
      for (size_t i = 0; i < ctxs.size(); i++) {
        memcpy(ctxs[i]->h_params, pb.data(), pb.size());
        ctx_release(ctxs[i], pgate[i], pb.data(), pb.size());
        pgate[i] = 0u;
      }
      pending = false;
    } else {
      for (pht_ctx *c : ctxs) {
        memcpy(c->h_params, pb.data(), pb.size());
        if (c->grp) {
          if (group_sweep(c, k0, k1, (uint32_t)iter, zexp)) return -1;
        } else if (ctx_enqueue(c, k0, k1, (uint32_t)iter, zexp, false, timed)) {
          return -1;
        }
      }
    }
    if (pipe && iter + 1 < it) {
      for (size_t i = 0; i < ctxs.size(); i++) {
        pht_ctx *c = ctxs[i];
        if (++c->gate_seq == 0u) c->gate_seq = 1u;
        /* (recorded first: a failed enqueue may have left the gate kernel in
         * the stream, and unwind releases it) */
        pgate[i] = c->gate_seq;
        if (ctx_enqueue(c, k0, k1, (uint32_t)(iter + 1), zexp, false, want_time(iter + 1), pgate[i])) {
          unwind();
          return -1;
        }
      }
      pending = true;
    }
    std::fill(tot.begin(), tot.end(), 0LL);
    bool wrapped = false;
    bool any_t = false;
    double ksum = 0.0;
    for (pht_ctx *c : ctxs) {
      if (!c->grp && ctx_wait(c)) {
        unwind();
        return -1;
      }
      if (c->last_ms >= 0.f) {
        ksum += c->last_ms;
        any_t = true;
      }
      for (int k = 0; k < sl; k++) wrapped |= __builtin_add_overflow(tot[k], (long long)c->h_stats[k], &tot[k]);
    }
    if (reduce && reduce(tot.data(), sl, reduce_user) != 0) {
      set_err("statistics all-reduce callback failed at sweep %d", iter);
      unwind();
      return -1;
    }
#ifndef PHT_STAMPS /* diagnostic builds carry cycle stamps in the extra words */
    const long long *xw = tot.data() + 2 * n + n * n;
    if (expect >= 0 && xw[kXObs] != expect) {
      set_err("sweep %d sampled %lld observations, expected %lld: the statistics are incomplete or summed twice",
              iter, xw[kXObs], expect);
      unwind();
      return -1;
    }
    for (int k = 0; k < n; k++) wrapped |= tot[k] < 0;
    if (wrapped || xw[kXOverflow] != 0) {
      set_err("sweep %d: the fixed-point z sums overflowed int64 (zexp = %d leaves 2^%d time units; censored paths "
              "ran far past the observed times): pass a smaller zexp",
              iter, zexp, 63 - zexp);
      unwind();
      return -1;
    }
    /* observations that hit a cap (ARMS iterations, path length, MHRS
     * attempts) or a numerical guard contribute their last attempt, where
     * the reference would keep looping (DESIGN.md §3 Caps) */
    const long long fl = xw[kXFlagged];
    if (fl > 0) {
      if (!first_flagged) first_flagged = iter;
      flagged += fl;
    }
    /* UNIF observations beyond the table or the lam cap carry a path that is
     * not a draw of the target law (pht_unif.h): an error, not a warning.
     * Only sweeps that ran the UNIF kernels: other samplers' diagnostic
     * builds (PHT_ECS_DIAG, PHT_DCS_DIAG) count their own things in word 6 */
    if (bm == kMethodUNIF && xw[kXUnifCap] > 0) {
      set_err("sweep %d: %lld UNIF observations need more than %d uniformisation steps or mu*y > %g (the largest "
              "exit rate times the largest observation); their paths would be wrong: rescale the data",
              iter, xw[kXUnifCap], kUnifMaxK, kUnifMaxLam);
      unwind();
      return -1;
    }
#endif
    if (any_t) {
      kms += ksum;
      ktimed++;
    }
    for (int k = 0; k < n; k++) z[k] = ldexp((double)tot[k], -zexp);
    G.update(R, iter, z.data(), tot.data() + 2 * n);
  }
  if (ktimed > 0) kms = kms / (double)ktimed * (double)(it - 1);
  for (pht_ctx *c : ctxs) c->flagged = flagged;
  if (flagged)
    warn("\nWARNING: %lld observation-sweeps hit a sampler cap or numerical guard (first in iteration %d); "
         "each contributed its last attempt to the sufficient statistics\n",
         flagged, first_flagged + 1);
  if (kernel_ms_total) *kernel_ms_total = kms;
  return 0;
}
}  // namespace

/*
 * Multi-process entry (one process per GPU): this process owns observations
 * [obs0, obs0 + l) of a data set of l_total observations (zexp must be the
 * same on every rank: pht_zexp over all observations); `reduce` sums the
 * statistics block across ranks (e.g. an RCCL all-reduce).  The R-stream
 * (pht_set_seed) must be seeded identically on all ranks; every rank then
 * draws identical Gamma updates and the chain is the single-process chain.
 */
extern "C" int pht_gibbs_run(pht_ctx *c, int it, int method, int m, const double *nu, const double *zeta,
                             const int *T, const double *C, int zexp, int silent, const double *start, double *res,
                             pht_reduce_fn reduce, void *reduce_user, double *kernel_ms_total) {
  if (!c) {
    set_err("pht_gibbs_run: null context");
    return -1;
  }
  if (reduce && c->comm) {
    /* the block would be summed twice: by RCCL on the stream, then here */
    set_err("pht_gibbs_run: a reduce callback was given for a context with an RCCL communicator attached");
    return -1;
  }
  RHost &R = rhost();
  R.begin();
  const uint32_t k0 = (uint32_t)(R.u() * 4294967296.0);
  const uint32_t k1 = (uint32_t)(R.u() * 4294967296.0);
  std::vector<pht_ctx *> ctxs{c};
  int rc = gibbs_run(R, it, c->mhit, method, c->n, m, nu, zeta, T, C, nullptr, c->count, silent, start, res, ctxs, k0,
                     k1, zexp, reduce, reduce_user, kernel_ms_total);
  R.end();
  return rc;
}

/*
 * Several independent chains at once: chain c runs on its
 * own context (device buffers and HIP stream) from a host thread of its own,
 * with its own R-compatible stream seeded by seeds[c] (standalone mode: the
 * Gamma draws and the Philox key come from it), so chain c is exactly the
 * single-chain pht_gibbs_run after pht_set_seed(seeds[c]).  At small N each
 * chain's kernels leave most of the GPU idle (their time is the longest
 * latent path); the chains' kernels run concurrently on their streams and the
 * host setups overlap.  res is [chain][it x m] (each block as pht_gibbs_run);
 * start is [chain][m] or start[0] < 0.  Not for use inside R (threads).
 */
namespace {
struct OwnRng {
  pht_rstream rs;
  double u() { return pht_rs_unif_rand(&rs); }
  double gamma(double a, double sc) { return pht_rs_rgamma(&rs, a, sc); }
};
}  // namespace

extern "C" int pht_gibbs_run_chains(pht_ctx **ctxs, int nchains, const uint32_t *seeds, int it, int method, int m,
                                    const double *nu, const double *zeta, const int *T, const double *C, int zexp,
                                    const double *start, double *res, double *kernel_ms_max) {
  if (nchains < 1 || !ctxs || !seeds) {
    set_err("pht_gibbs_run_chains: need nchains >= 1 contexts and seeds");
    return -1;
  }
  if (rhost().inR) {
    set_err("pht_gibbs_run_chains is not available inside R (host threads)");
    return -1;
  }
  for (int c = 0; c < nchains; c++)
    if (!ctxs[c] || ctxs[c]->comm) {
      set_err("pht_gibbs_run_chains: context %d is null or has an RCCL communicator attached", c);
      return -1;
    }
  /* all chains' sweeps in one launch sequence, when the chains share a
   * device, n and method (ECS: the exact ranges in one ecs_chains_kernel and
   * the censored ranges in one cens_chains_kernel; MHRS/DCS/UNIF: one
   * launch_chains sequence); PHT_CHAINS_LAUNCH=streams: a launch per chain */
  ChainGroup *grp = nullptr;
  {
    bool one = nchains >= 2;
    for (int c = 0; c < nchains && one; c++)
      one = ctxs[c]->method == ctxs[0]->method && ctxs[c]->ulaw == ctxs[0]->ulaw &&
            ctxs[c]->device == ctxs[0]->device && ctxs[c]->n == ctxs[0]->n && !ctxs[c]->grp;
    const char *ev = getenv("PHT_CHAINS_LAUNCH");
    if (ev && !strcmp(ev, "streams")) one = false;
    if (one) {
      grp = group_create(ctxs[0]->device, nchains, ctxs[0]->n, ctxs[0]->method);
      if (!grp) {
        set_err("pht_gibbs_run_chains: HIP allocation failed");
        return -1;
      }
      for (int c = 0; c < nchains; c++) {
        ctxs[c]->grp = grp;
        ctxs[c]->gidx = c;
      }
    }
  }
  std::vector<int> rc(nchains, 0);
  std::vector<double> kms(nchains, 0.0);
  std::vector<std::string> err(nchains);
  std::vector<std::thread> th;
  for (int c = 0; c < nchains; c++) {
    th.emplace_back([&, c]() {
      OwnRng R;
      pht_rs_set_seed(&R.rs, seeds[c]);
      const uint32_t k0 = (uint32_t)(R.u() * 4294967296.0);
      const uint32_t k1 = (uint32_t)(R.u() * 4294967296.0);
      std::vector<pht_ctx *> one{ctxs[c]};
      const double *st = (start && start[0] >= 0) ? start + (size_t)c * m : start;
      rc[c] = gibbs_run(R, it, ctxs[c]->mhit, method, ctxs[c]->n, m, nu, zeta, T, C, nullptr, ctxs[c]->count, 1,
                        st, res + (size_t)c * it * m, one, k0, k1, zexp, nullptr, nullptr, &kms[c]);
      if (rc[c]) err[c] = g_err;
      if (grp) group_leave(grp);
    });
  }
  for (auto &t : th) t.join();
  if (grp) {
    for (int c = 0; c < nchains; c++) {
      ctxs[c]->grp = nullptr;
      ctxs[c]->gidx = -1;
    }
    group_destroy(grp);
  }
  double mx = 0.0;
  for (int c = 0; c < nchains; c++) {
    if (rc[c]) {
      set_err("chain %d: %s", c, err[c].c_str());
      return -1;
    }
    mx = std::max(mx, kms[c]);
  }
  if (kernel_ms_max) *kernel_ms_max = mx;
  return 0;
}

/* ============================================ device-resident Gibbs chain */
/*
 * pht_gibbs_run_resident (opt-in, NON-PARITY): the whole
 * Gibbs loop on the device.  Per sweep the stream carries the step-1 kernels,
 * the optional RCCL all-reduce of the statistics, and resident_update_kernel
 * (pht_resident.hip: conjugate Gamma update by a counter-based sampler, the
 * next sweep's parameter block, the per-sweep checks); the host enqueues all
 * sweeps and waits once.  Every sampler: for ECS/DCS the update kernel also
 * builds the eigensystem (include/pht_eigen.h, one workgroup, in place of the
 * host's LAPACK dgeevx) and the spectral products.  The chain is a deterministic
 * function of the R stream's two key words (drawn at entry, as
 * pht_gibbs_run does) but NOT the host loop's chain (R's rgamma is replaced).
 */
namespace {
struct DevBuf {
  void *p = nullptr;
  ~DevBuf() {
    if (p) (void)hipFree(p);
  }
};
}  // namespace

extern "C" int pht_gibbs_run_resident(pht_ctx *c, int it, int method, int m, const double *nu, const double *zeta,
                                      const int *T, const double *C, int zexp, const double *start, double *res,
                                      double *kernel_ms_total) {
  if (!c || it < 1 || m < 1 || m > (kMaxN + 1) * (kMaxN + 1)) {
    set_err("pht_gibbs_run_resident: need a context, it >= 1 and 1 <= m <= (kMaxN+1)^2");
    return -1;
  }
  if (dispatch_method(method) == 0 || dispatch_method(method) != c->rmethod) {
    set_err("pht_gibbs_run_resident: method %d needs a context created for that method (context %d)", method,
            c->rmethod);
    return -1;
  }
  const int disp = c->method; /* the kernels that run (UNIF for a bridge context) */
  if (!(ldexp(c->ysum, zexp) < 0x1p62)) {
    set_err("zexp = %d overflows the fixed-point z sums (the shard's observed times total %g)", zexp, c->ysum);
    return -1;
  }
  const int n = c->n, n1 = n + 1;
  RHost &R = rhost();
  R.begin();
  const uint32_t k0 = (uint32_t)(R.u() * 4294967296.0);
  const uint32_t k1 = (uint32_t)(R.u() * 4294967296.0);
  R.end();
  /* GibbsState's parameter lists as CSR, insertion order */
  std::vector<std::vector<int>> nl(m), zi(m), tl(m), dl(n1);
  std::vector<std::vector<double>> zc(m), tc(m);
  for (int i = 0; i < n1; i++)
    for (int j = 0; j < n1; j++) {
      const int t = T[i + j * n1];
      if (t == 0) continue;
      if (t < 1 || t > m) {
        set_err("pht_gibbs_run_resident: T[%d,%d] = %d outside 0..m", i, j, t);
        return -1;
      }
      const int k = t - 1;
      const double cc = C[i + j * n1];
      nl[k].push_back(j == n ? i + i * n : i + j * n);
      zi[k].push_back(i);
      zc[k].push_back(cc);
      tl[k].push_back(i + j * n1);
      tc[k].push_back(cc);
      dl[i].push_back(i + j * n1);
    }
  std::vector<int> ints;   /* nl_off[m+1] nl_idx zl_off[m+1] zl_i tl_off[m+1] tl_ij dl_off[n+1] dl_ij */
  std::vector<double> dbl; /* nu[m] zeta[m] start[m] zl_c tl_c */
  auto csr = [&](const std::vector<std::vector<int>> &v, int rows, int &off, int &idx) {
    off = (int)ints.size();
    int acc = 0;
    for (int r = 0; r < rows; r++) {
      ints.push_back(acc);
      acc += (int)v[r].size();
    }
    ints.push_back(acc);
    idx = (int)ints.size();
    for (int r = 0; r < rows; r++) ints.insert(ints.end(), v[r].begin(), v[r].end());
  };
  int o_nl, i_nl, o_zl, i_zl, o_tl, i_tl, o_dl, i_dl;
  csr(nl, m, o_nl, i_nl);
  csr(zi, m, o_zl, i_zl);
  csr(tl, m, o_tl, i_tl);
  csr(dl, n, o_dl, i_dl);
  dbl.insert(dbl.end(), nu, nu + m);
  dbl.insert(dbl.end(), zeta, zeta + m);
  const bool has_start = start && start[0] >= 0;
  for (int k = 0; k < m; k++) dbl.push_back(has_start ? start[k] : 0.0);
  const int o_zc = (int)dbl.size();
  for (int k = 0; k < m; k++) dbl.insert(dbl.end(), zc[k].begin(), zc[k].end());
  const int o_tc = (int)dbl.size();
  for (int k = 0; k < m; k++) dbl.insert(dbl.end(), tc[k].begin(), tc[k].end());

  HIPCHK(hipSetDevice(c->device));
  DevBuf bi, bd, bres, btt, bfl, berr;
  HIPCHK(hipMalloc(&bi.p, sizeof(int) * ints.size()));
  HIPCHK(hipMalloc(&bd.p, sizeof(double) * dbl.size()));
  HIPCHK(hipMalloc(&bres.p, sizeof(double) * (size_t)it * m));
  HIPCHK(hipMalloc(&btt.p, sizeof(double) * n1 * n1));
  HIPCHK(hipMalloc(&bfl.p, sizeof(unsigned long long)));
  HIPCHK(hipMalloc(&berr.p, sizeof(int)));
  hipStream_t st = c->stream;
  HIPCHK(hipMemcpyAsync(bi.p, ints.data(), sizeof(int) * ints.size(), hipMemcpyHostToDevice, st));
  HIPCHK(hipMemcpyAsync(bd.p, dbl.data(), sizeof(double) * dbl.size(), hipMemcpyHostToDevice, st));
  HIPCHK(hipMemsetAsync(btt.p, 0, sizeof(double) * n1 * n1, st));
  HIPCHK(hipMemsetAsync(bfl.p, 0, sizeof(unsigned long long), st));
  HIPCHK(hipMemsetAsync(berr.p, 0, sizeof(int), st));
  HIPCHK(hipMemsetAsync(c->d_params, 0, make_layout(n).bytes(), st));
  HIPCHK(hipMemsetAsync(c->d_stats, 0, sizeof(unsigned long long) * stats_len(n), st));
  c->stats_zero = false;
  const int *di = static_cast<const int *>(bi.p);
  const double *dd = static_cast<const double *>(bd.p);
  ResidentArgs ra;
  memset(&ra, 0, sizeof ra);
  ra.n = n;
  ra.m = m;
  ra.it = it;
  ra.init = 1;
  ra.eig = (disp == kMethodECS || disp == kMethodDCS) ? 1 : 0;
  ra.unif = (disp == kMethodUNIF || c->ulaw) ? 1 : 0;
  ra.zs = ldexp(1.0, -zexp);
  ra.expect = c->global_count >= 0 ? c->global_count : (c->comm ? -1 : (long long)c->count);
  ra.k0 = k0;
  ra.k1 = k1;
  ra.nu = dd;
  ra.zeta = dd + m;
  ra.start = has_start ? dd + 2 * m : nullptr;
  ra.nl_off = di + o_nl;
  ra.nl_idx = di + i_nl;
  ra.zl_off = di + o_zl;
  ra.zl_i = di + i_zl;
  ra.zl_c = dd + o_zc;
  ra.tl_off = di + o_tl;
  ra.tl_ij = di + i_tl;
  ra.tl_c = dd + o_tc;
  ra.dl_off = di + o_dl;
  ra.dl_ij = di + i_dl;
  ra.stats = c->d_stats;
  ra.TT = static_cast<double *>(btt.p);
  ra.res = static_cast<double *>(bres.p);
  ra.params = c->d_params;
  ra.flagged = static_cast<unsigned long long *>(bfl.p);
  ra.err = static_cast<int *>(berr.p);
  HIPCHK(pht_launch_resident_update(&ra, 0, st));
  ra.init = 0;

  SweepArgs a;
  memset(&a, 0, sizeof a);
  a.params = c->d_params;
  a.n = n;
  a.mhit = c->mhit;
  a.ulaw = c->ulaw;
  a.count = c->count;
  a.y = c->d_y;
  a.cens = c->d_cens;
  a.gid = c->d_gid;
  a.k0 = k0;
  a.k1 = k1;
  a.zscale = ldexp(1.0, zexp);
  a.dcsbrent = dcs_brent();
  a.dcsb = c->d_dcsb;
  a.stats = c->d_stats;
  a.mbest = c->d_mbest;
  a.mq0 = c->d_mq0;
  a.mq1 = c->d_mq1;
  a.mcnt = c->d_mcnt;
  if (disp == kMethodUNIF) {
    /* table capacity: twice the prior mode's largest exit rate (the device
     * sizes each sweep's table from its own mu within it).  A chain whose mu
     * drifts past that needs rows beyond the capacity: those observations
     * are counted in kXUnifCap and the update kernel stops the run (err 16) */
    double mu0 = 0.0;
    {
      std::vector<double> rowsum(n1, 0.0);
      for (int i = 0; i < n1; i++)
        for (int j = 0; j < n1; j++) {
          const int t = T[i + j * n1];
          if (t == 0) continue;
          const int k = t - 1;
          const double th = has_start ? start[k] : (nu[k] > 1 ? (nu[k] - 1.0) / zeta[k] : nu[k] / zeta[k]);
          rowsum[i] += th * C[i + j * n1];
        }
      for (int i = 0; i < n; i++) mu0 = std::max(mu0, rowsum[i]);
    }
    const double lmax = 2.0 * mu0 * c->ymax;
    const double kd = std::ceil(lmax + 14.0 * std::sqrt(lmax) + 64.0);
    a.uK = (int)std::min<double>(kUnifMaxK, std::isfinite(kd) ? kd : (double)kUnifMaxK);
    a.uymax = c->ymax;
    const long need = unif_tab_doubles(n, a.uK);
    if (need > c->utab_cap) {
      if (c->d_utab) HIPCHK(hipFree(c->d_utab));
      c->d_utab = nullptr;
      HIPCHK(hipMalloc(&c->d_utab, sizeof(double) * need));
      c->utab_cap = need;
    }
    a.utab = c->d_utab;
  }
  HIPCHK(hipEventRecord(c->ev0, st));
  int early = 0; /* the error word, polled every kErrPoll sweeps */
  constexpr int kErrPoll = 256;
  for (int iter = 1; iter < it; iter++) {
    if (iter % kErrPoll == 0) {
      /* a failed sweep (e.g. the eigensystem) makes the update kernels
       * return at entry; stop enqueueing instead of running to `it`.  With a
       * communicator the decision is collective (the maximum of the ranks'
       * error words), so no rank leaves the loop while its peers still enter
       * the per-sweep all-reduce */
      if (c->comm && c->d_rccl) {
        HIPCHK(hipMemsetAsync(c->d_rccl, 0, sizeof(long long), st));
        HIPCHK(hipMemcpyAsync(c->d_rccl, berr.p, sizeof(int), hipMemcpyDeviceToDevice, st));
        const ncclResult_t rr = rccl().allReduce(c->d_rccl, c->d_rccl, 1, ncclUint64, ncclMax, c->comm, st);
        if (rr != ncclSuccess) {
          set_err("RCCL all-reduce of the error word failed: %s", rccl().errStr(rr));
          return -1;
        }
        long long ew = 0;
        HIPCHK(hipMemcpyAsync(&ew, c->d_rccl, sizeof ew, hipMemcpyDeviceToHost, st));
        HIPCHK(hipStreamSynchronize(st));
        early = (int)ew;
      } else {
        HIPCHK(hipMemcpyAsync(&early, berr.p, sizeof early, hipMemcpyDeviceToHost, st));
        HIPCHK(hipStreamSynchronize(st));
      }
      if (early) break;
    }
    a.sweep = (uint32_t)iter;
    if ((c->count > 0 || disp == kMethodUNIF) && ctx_launch(c, a, false)) return -1;
    if (c->comm) {
      const ncclResult_t rr =
          rccl().allReduce(c->d_stats, c->d_stats, (size_t)stats_len(n), ncclUint64, ncclSum, c->comm, st);
      if (rr != ncclSuccess) {
        set_err("RCCL all-reduce of the statistics failed: %s", rccl().errStr(rr));
        return -1;
      }
    }
    HIPCHK(pht_launch_resident_update(&ra, iter, st));
  }
  HIPCHK(hipEventRecord(c->ev1, st));
  unsigned long long fl = 0;
  int err = 0;
  HIPCHK(hipMemcpyAsync(res, bres.p, sizeof(double) * (size_t)it * m, hipMemcpyDeviceToHost, st));
  HIPCHK(hipMemcpyAsync(&fl, bfl.p, sizeof fl, hipMemcpyDeviceToHost, st));
  HIPCHK(hipMemcpyAsync(&err, berr.p, sizeof err, hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  float ms = 0.f;
  HIPCHK(hipEventElapsedTime(&ms, c->ev0, c->ev1));
  if (kernel_ms_total) *kernel_ms_total = ms;
  c->flagged = (long long)fl;
  if (err) {
    set_err("resident chain: %s%s%s%s%s", (err & 1) ? "a sweep did not sample every observation; " : "",
            (err & 2) ? "the fixed-point z sums overflowed (pass a smaller zexp); " : "",
            (err & 4) ? "a Gamma draw failed (non-finite shape/scale or the rejection cap); " : "",
            (err & 8) ? "the eigensystem failed (complex eigenvalues, no QR convergence or singular eigenvectors:"
                        " the uniformisation sampler, method 8, needs none); " : "",
            (err & 16) ? "UNIF observations needed more uniformisation steps than the table sized from the start "
                         "(twice its largest exit rate) holds, or mu*y > 1300: the chain's rates drifted far above "
                         "the start (start nearer the posterior, or use the host loop, which sizes every sweep)" : "");
    return -1;
  }
  if (fl)
    warn("\nWARNING: %llu observation-sweeps hit a sampler cap or numerical guard in the resident chain\n", fl);
  return 0;
}

/* ======================================================= .C entry point */
/*
 * Drop-in replacement of LJMA_Gibbs (src/PHT_MCMC_Aslett.c:104): same 15
 * arguments, same semantics and output (res[iter + i*it]).  Observations are
 * sharded over all visible GPUs (PHT_DEVICES=k limits the count).
 * Divergences, documented in DESIGN.md: per-observation draws come from
 * Philox (keyed by two R-stream uniforms drawn at entry) instead of R's
 * serial stream; z is reduced in exact fixed point.
 */
extern "C" void LJMA_Gibbs(int *it, int *mhit, int *method, int *n, int *m, double *nu, double *zeta, int *T,
                           double *C, double *y, int *l, int *censored, double *start, int *silent, double *res) {
  RHost &R = rhost();
  g_err.clear();
  R.begin();
  const uint32_t k0 = (uint32_t)(R.u() * 4294967296.0);
  const uint32_t k1 = (uint32_t)(R.u() * 4294967296.0);
  const int zexp = pht_zexp(y, *l);
  say("Setting up Gibbs run ...\n");
  int ndev = pht_device_count();
  if (const char *e = getenv("PHT_DEVICES")) ndev = std::min(ndev, atoi(e));
  /* PHT_CTX_PER_DEVICE=k: k shards (contexts, each with its own streams) per
   * device; the chain is the same for every k (tests/test_gpu_edges.py) */
  int per = 1;
  if (const char *e = getenv("PHT_CTX_PER_DEVICE")) per = std::max(1, std::min(16, atoi(e)));
  std::vector<pht_ctx *> ctxs;
  int rc = 0;
  if (ndev <= 0) {
    set_err("no HIP device available");
    rc = -1;
  }
  const long L = *l;
  const int nsh = ndev * per;
  for (int d = 0; d < nsh && rc == 0; d++) {
    const long lo = L * d / nsh, hi = L * (d + 1) / nsh;
    pht_ctx *c = pht_ctx_create(d / per, *n, *method, *mhit);
    if (!c) {
      rc = -1;
      break;
    }
    ctxs.push_back(c);
    if (pht_ctx_set_obs(c, y + lo, censored + lo, hi - lo, lo)) rc = -1;
  }
  if (rc == 0)
    rc = gibbs_run(R, *it, *mhit, *method, *n, *m, nu, zeta, T, C, y, L, *silent, start, res, ctxs, k0, k1, zexp,
                   nullptr, nullptr, nullptr);
  for (pht_ctx *c : ctxs) pht_ctx_destroy(c);
  if (rc == 0) say("\n\nCompleted MCMC run, returning results ...\n");
  R.end();
  if (rc != 0) {
    if (R.inR && R.rerror) R.rerror("%s", g_err.c_str());
    fprintf(stderr, "PhaseType (MI355X): %s\n", g_err.c_str());
  }
}

/* ================================================== R native registration */
/* R's registration ABI (R_ext/Rdynload.h), declared here so the library
 * also loads outside R; the R functions are resolved only when present. */
extern "C" {
typedef void *(*pht_DL_FUNC)(void);
typedef unsigned int pht_R_NativePrimitiveArgType;
typedef struct {
  const char *name;
  pht_DL_FUNC fun;
  int numArgs;
  pht_R_NativePrimitiveArgType *types;
} pht_R_CMethodDef;
}

extern "C" void R_init_PhaseType(void *dll) {
  /* INTSXP = 13, REALSXP = 14 (src/Registrations.c:6-9) */
  static pht_R_NativePrimitiveArgType types[15] = {13, 13, 13, 13, 13, 14, 14, 13, 14, 14, 13, 13, 14, 13, 14};
  static pht_R_CMethodDef cMethods[] = {{"LJMA_Gibbs", (pht_DL_FUNC)&LJMA_Gibbs, 15, types},
                                        {nullptr, nullptr, 0, nullptr}};
  typedef int (*reg_fn)(void *, const pht_R_CMethodDef *, const void *, const void *, const void *);
  typedef int (*bool_fn)(void *, int);
  reg_fn reg = (reg_fn)dlsym(RTLD_DEFAULT, "R_registerRoutines");
  bool_fn dyn = (bool_fn)dlsym(RTLD_DEFAULT, "R_useDynamicSymbols");
  bool_fn force = (bool_fn)dlsym(RTLD_DEFAULT, "R_forceSymbols");
  if (!reg || !dyn || !force) return;
  reg(dll, cMethods, nullptr, nullptr, nullptr);
  dyn(dll, 0);
  force(dll, 1);
}
