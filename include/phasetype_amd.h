/*
 * phasetype_amd.h — C ABI of the MI355X-native PhaseType hot path
 * (libPhaseType.so, built by phasetype_amd/build.py).
 *
 * 1. Drop-in boundary (what R binds).  The reference registers exactly one
 *    native routine, for `.C`:
 *      src/PHT_MCMC_Aslett.h:1-3    void LJMA_Gibbs(int*, int*, int*, int*, int*, double*, double*,
 *                                                   int*, double*, double*, int*, int*, double*, int*, double*)
 *      src/Registrations.c:6-20     R_init_PhaseType: R_registerRoutines(.C, 15 typed args),
 *                                   R_useDynamicSymbols(FALSE), R_forceSymbols(TRUE)
 *      NAMESPACE:2                  useDynLib(PhaseType, .registration = TRUE)
 *    Callers: R/phtMCMC.R:83, R/phtMCMC2.R:73.  Same names, same argument
 *    meaning, same output layout (res[iter + i*it]); see INTEGRATION.md.
 *
 * 2. Sweep-level ABI (the seam the reference's LJMA_MHsample_{Bladt,
 *    Aslett2,Hobolth2} occupy, src/PHT_MCMC_Aslett.c:325-333): one Gibbs
 *    step 1 over a shard of observations on one GPU, returning the int64
 *    sufficient-statistics block
 *      [zq n][B n][N n*n][16 counters]   (pht_stats_len(n) entries)
 *    zq = z in fixed point, z_k = zq_k * 2^-zexp; N[i + j n] = i->j
 *    transitions, diagonal = absorb-from counts (reference convention).
 *
 * Errors: functions returning int return 0 on success and non-zero on
 * failure with a message in pht_last_error().  There is no CPU fallback:
 * without a HIP device, pht_ctx_create and LJMA_Gibbs fail loudly.
 */
#ifndef PHASETYPE_AMD_H
#define PHASETYPE_AMD_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- drop-in boundary ------------------------------------------------ */
void LJMA_Gibbs(int *it, int *mhit, int *method, int *n, int *m, double *nu, double *zeta, int *T, double *C,
                double *y, int *l, int *censored, double *start, int *silent, double *res);
void R_init_PhaseType(void *dll_info);

/* ---- host services ----------------------------------------------------- */
const char *pht_last_error(void);
int pht_device_count(void);
/* Bind an LP64 LAPACK (dgeevx_/dgetrf_/dgetri_ with symbol prefix); inside R
 * the process's own LAPACK is found automatically. */
int pht_bind_lapack(const char *path, const char *prefix);
/* Standalone R-compatible random stream (ignored inside R): set.seed(seed). */
void pht_set_seed(uint32_t seed);
double pht_unif_rand(void);
double pht_rgamma(double shape, double scale);
int pht_in_R(void);
void pht_set_verbose(int v);
int pht_zexp(const double *y, long l);
int pht_params_bytes(int n);
int pht_stats_len(int n);
int pht_build_params(int n, const double *S, const double *s, int method, unsigned char *out, int out_bytes);

/* ---- sweep-level ABI ----------------------------------------------------- */
typedef struct pht_ctx pht_ctx;
pht_ctx *pht_ctx_create(int device, int n, int method, int mhit);
void pht_ctx_destroy(pht_ctx *c);
int pht_ctx_set_obs(pht_ctx *c, const double *y, const int *censored, long count, long obs0);
int pht_ctx_sweep(pht_ctx *c, const double *S, const double *s, uint32_t k0, uint32_t k1, uint32_t sweep,
                  int zexp, long long *stats_out);
int pht_ctx_sweep_debug(pht_ctx *c, const double *S, const double *s, uint32_t k0, uint32_t k1, uint32_t sweep,
                        int zexp, long long *stats_out, int *B, int *pre, int *flags, uint32_t *ndraw,
                        long long *zq, int *N);
/* Device time of the last sweep's kernels (HIP events); -1 when that sweep
 * was not timed (pht_gibbs_run times one sweep in PHT_KTIME_EVERY). */
float pht_ctx_last_kernel_ms(pht_ctx *c);
/* Observation-sweeps flagged in the last pht_gibbs_run / pht_gibbs_run_chains
 * on this context (node-wide, after the reduce): a cap (ARMS iterations, path
 * length, MHRS attempts) or a numerical guard fired, and the observation
 * contributed its last attempt.  No reference counterpart (its loops are
 * unbounded); a warning is also printed once per run. */
long long pht_ctx_flagged_obs(pht_ctx *c);
/* Observations over ALL shards of a multi-process run (this context's shard
 * included).  pht_gibbs_run checks every sweep that the node-wide statistics
 * account for exactly this many observations, and fails the run otherwise
 * (single process: the check uses the context's own count, always on).  No
 * reference counterpart (the reference has one process and no such failure
 * mode, src/PHT_MCMC_Aslett.c:325-337). */
int pht_ctx_set_global_count(pht_ctx *c, long long total);

/* Gibbs loop over one shard; reduce(stats, len, user) must sum the int64
 * block across all shards (return 0 on success), or NULL (single process, or
 * an RCCL communicator attached: passing both is an error, the block would be
 * summed twice).  Every sweep is checked: the node-wide processed count must
 * equal the observations (see pht_ctx_set_global_count), and the fixed-point
 * z sums must not overflow int64; either failure ends the run with an error.
 * kernel_ms_total: the sweeps' device time, measured by HIP events on one
 * sweep in PHT_KTIME_EVERY (default 4; the events cost the GPU ~9 us of idle
 * time per timed sweep) and scaled to all it - 1 sweeps from their mean. */
typedef int (*pht_reduce_fn)(long long *stats, int len, void *user);
int pht_gibbs_run(pht_ctx *c, int it, int method, int m, const double *nu, const double *zeta, const int *T,
                  const double *C, int zexp, int silent, const double *start, double *res, pht_reduce_fn reduce,
                  void *reduce_user, double *kernel_ms_total);

/* Multi-process runs without a host callback: every sweep's statistics
 * block on this context is summed over `nranks` processes by an RCCL
 * all-reduce (uint64, in place) on the context's stream, before its copy to
 * the host; pht_gibbs_run then takes reduce = NULL.  One rank calls
 * pht_rccl_unique_id and broadcasts the 128 bytes; every rank first calls
 * pht_ctx_rccl_prepare (all LOCAL preconditions: RCCL loadable, no
 * communicator yet, device, staging buffer of max_len words), the ranks agree
 * on its verdict, and only then every rank attaches with the same id (the
 * collective ncclCommInitRank).  RCCL is loaded at run time (librccl.so.1).
 * No reference counterpart: the reference is single-process
 * (src/PHT_MCMC_Aslett.c:325-337). */
int pht_rccl_unique_id(unsigned char *id128);
int pht_ctx_rccl_prepare(pht_ctx *c, int max_len);
int pht_ctx_attach_rccl(pht_ctx *c, const unsigned char *id128, int nranks, int rank);
/* In-place sum of buf[len] (host int64, len <= the prepared max_len) over the
 * attached communicator, on the context's stream: the all-reduce a sweep runs
 * on its statistics block, exposed so the caller can check it against its own
 * collective.  Once attached, a rank always enters the collective. */
int pht_ctx_rccl_allreduce(pht_ctx *c, long long *buf, int len);

/* Device-resident Gibbs chain (opt-in, NON-PARITY):
 * the conjugate Gamma update (src/PHT_MCMC_Aslett.c:340-397) and the next
 * sweep's parameter block (:279-297) run on the device between sweeps
 * (phasetype_amd/csrc/pht_resident.hip), so the host enqueues every sweep
 * and waits once.  Gamma draws come from a counter-based sampler
 * (include/pht_gamma.h), not R's rgamma: the chain is deterministic under
 * set.seed but not the host loop's chain.  Any method matching the context's
 * (for ECS/DCS the update also builds the eigensystem, include/pht_eigen.h,
 * instead of LAPACK: a complex spectrum stops the run with an error, where the
 * host path warns and uses the real parts as the reference does); an attached RCCL
 * communicator sums every sweep's statistics on the stream (every rank must
 * use the same R-stream seed).  Arguments and res layout as pht_gibbs_run;
 * kernel_ms_total = device time of all sweeps. */
int pht_gibbs_run_resident(pht_ctx *c, int it, int method, int m, const double *nu, const double *zeta, const int *T,
                           const double *C, int zexp, const double *start, double *res, double *kernel_ms_total);

/* Independent chains at once (no reference counterpart —
 * the reference runs one chain per LJMA_Gibbs call, src/PHT_MCMC_Aslett.c:104):
 * chain c on ctxs[c] (one context each, same n/method/mhit, observations set),
 * its own host thread and R-compatible stream seeded by seeds[c]; chain c
 * equals pht_gibbs_run after pht_set_seed(seeds[c]).  res: nchains blocks of
 * it*m (pht_gibbs_run's layout); start: exactly nchains*m values (chain c
 * reads start[c*m .. c*m+m-1]) or start[0] < 0 — the length is not checked
 * here, so a caller holding one m-vector must repeat it per chain (the
 * Python mirror phasetype_amd.gibbs_chains broadcasts and validates it).
 * Standalone builds only (fails inside R), and not on contexts with an RCCL
 * communicator attached. */
int pht_gibbs_run_chains(pht_ctx **ctxs, int nchains, const uint32_t *seeds, int it, int method, int m,
                         const double *nu, const double *zeta, const int *T, const double *C, int zexp,
                         const double *start, double *res, double *kernel_ms_max);

#ifdef __cplusplus
}
#endif
#endif
