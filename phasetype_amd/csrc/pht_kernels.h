/*
 * pht_kernels.h — host/device interface of the sweep kernels.
 */
#ifndef PHT_KERNELS_H
#define PHT_KERNELS_H

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "pht_layout.h"
#include "pht_philox.h"

namespace pht {

constexpr int kBlock = 256;
/* method bitmask values of LJMA_Gibbs (src/PHT_MCMC_Aslett.c:69-71) */
constexpr int kMethodMHRS = 0x1;
constexpr int kMethodECS = 0x2;
constexpr int kMethodDCS = 0x4;
/* not a reference method: the uniformisation sampler (pht_unif.h), opt-in */
constexpr int kMethodUNIF = 0x8;
constexpr int kMhrsCounters = 16;
/* UNIF per-sweep table in global memory (pht_unif.h):
 * [mu, rinv, K, 0][invk K+1][ax K+1][ac K+1][A (K+1) x n] */
constexpr int kUnifMaxK = 2047; /* last row index (LDS: 3 (K+1) doubles per block) */
constexpr double kUnifMaxLam = 1300.0; /* w_0 = 2^-1000 keeps every Poisson weight finite below this */
constexpr long unif_tab_doubles(int n, int K) { return 4 + 3L * (K + 1) + (long)(K + 1) * n; }

struct SweepArgs {
  const unsigned char *params; /* packed block (pht_layout.h), device */
  int n;
  int mhit;
  long begin;                  /* first position of this launch in the shard arrays */
  long count;                  /* observations in this launch */
  const double *y;             /* [count] */
  const int *cens;             /* [count]; nullptr = all exact (ECS exact kernel) */
  const uint32_t *gid;         /* [count] global observation index (Philox counter) */
  uint32_t k0, k1, sweep;
  double zscale;               /* 2^zexp */
  unsigned long long *stats;   /* [stats_len(n)] int64, accumulated */
  int occ;                     /* ECS exact: blocks per CU of the persistent grid (0 = occupancy limit) */
  int spread;                  /* ECS exact: first claims lane-major (the longest paths one per wavefront) */
  int newcap;                  /* ECS exact: observations a lane may start per round (0 = no limit) */
  double hoty;                 /* ECS exact: waves with a path whose remaining time exceeds hoty issue at high priority (0 = off) */
  int allcens;                 /* ECS: every observation of the launch is right-censored (jump-converged kernel) */
  long rowk;                   /* ECS exact: the first rowk positions (the longest paths) run one per 16-lane row;
                                  in the kernel: the rowk positions before begin */
  int rowblk;                  /* ECS exact: blocks of the launch serving those rows, before the nmain one-lane
                                  blocks (both set by the launcher) */
  int nmain;
  int rowprio;                 /* ECS exact: wave priority of the row blocks (s_setprio 0-3) */
  int dcsbrent;                /* DCS: jump times by Find02's Brent search instead of hob_halley (pht_dcs_round.h) */
  int *dcsb;                   /* DCS: per position the end state (| flag), written by dcs_end_kernel ahead of
                                  the round kernel; nullptr: computed in the round kernel */
  /* MHRS attempt search (pht_kernels.hip, MHRS section): per chain task
   * (position * (1 + mhit) + c) its first success (attempt << 8 | pre), two
   * task queues and the queue counters; allocated by the host for MHRS */
  uint32_t *mbest;             /* [count * (1 + mhit)] */
  uint32_t *mq0, *mq1;         /* [count * (1 + mhit)] */
  unsigned *mcnt;              /* [kMhrsCounters] */
  /* UNIF (pht_unif.h): the per-sweep table (written by unif_table_kernel),
   * its capacity (last row index) and the shard's largest y: the table
   * kernel sizes K from mu (known only on the device in a resident chain) */
  double *utab;
  int uK;
  double uymax;
  int ulaw;                    /* the path law the UNIF kernels sample (pht_unif.h): 0 ECS/UNIF, 1 MHRS (with
                                  mhit MH steps), 2 DCS (censored as exact) */
  /* debug per-observation outputs (DEBUG kernels only) */
  long long *dbg_zq;           /* [count*n] */
  int *dbg_N;                  /* [count*n*n] */
  int *dbg_B, *dbg_pre, *dbg_flags;
  uint32_t *dbg_ndraw;
};

/* the device-resident chain's per-sweep update (pht_resident.hip); all
 * pointers are device memory.  Parameter maps (GibbsState's lists,
 * gibbs_host.cpp) as CSR: entries of parameter k at [off[k], off[k+1]) in
 * insertion order (the update visits them in reverse, as the host does). */
struct ResidentArgs {
  int n, m, it, init;
  int eig;                      /* ECS/DCS: the eigensystem and spectral products too (include/pht_eigen.h) */
  int unif;                     /* the sweep runs the UNIF kernels (method 8 or a bridge mode): kXUnifCap applies */
  double zs;                    /* 2^-zexp */
  long long expect;             /* observations per sweep, node-wide (< 0: unchecked) */
  uint32_t k0, k1;              /* Philox key of the Gamma streams (include/pht_gamma.h) */
  const double *nu, *zeta;      /* [m] */
  const double *start;          /* [m], or nullptr: prior mode / prior draw */
  const int *nl_off, *nl_idx;   /* N counts of parameter k: stats[2n + idx] */
  const int *zl_off, *zl_i;     /* z sums: z[i] / c */
  const double *zl_c;
  const int *tl_off, *tl_ij;    /* TT cells (i + j (n+1)) = theta_k c */
  const double *tl_c;
  const int *dl_off, *dl_ij;    /* per row i: its TT cells (the diagonal) */
  unsigned long long *stats;    /* the sweep's block, read then zeroed */
  double *TT;                   /* (n+1)^2, zero outside the parameter cells */
  double *res;                  /* [it * m], res[iter + k it] */
  unsigned char *params;        /* the packed block the next sweep reads */
  unsigned long long *flagged;  /* flagged observation-sweeps, accumulated */
  int *err;                     /* bit 0: count, bit 1: z overflow, bit 2: Gamma draw, bit 3: eigensystem */
};

}  // namespace pht

extern "C" hipError_t pht_launch_resident_update(const pht::ResidentArgs *r, int iter, hipStream_t st);
extern "C" hipError_t pht_launch_sweep(const pht::SweepArgs *a, int method, int debug, hipStream_t st);
/* the statistics block -> host-pinned memory + flag = seq, and zeroed (pht_dispatch.hip) */
extern "C" hipError_t pht_launch_gate(const unsigned *gate_dev, unsigned want, const unsigned long long *src_dev,
                                      unsigned long long *dst, int nwords, unsigned *ack_dev, hipStream_t st);
extern "C" hipError_t pht_launch_stats_out(unsigned long long *d_stats, unsigned long long *h_out_dev,
                                           unsigned *flag_dev, unsigned seq, int sl, hipStream_t st);
extern "C" hipError_t pht_launch_chains(const pht::SweepArgs *h, const pht::SweepArgs *d, int K, int method,
                                        hipStream_t st);
extern "C" hipError_t pht_launch_ecs_chains(const pht::SweepArgs *h, const pht::SweepArgs *d, int K, hipStream_t st);

#endif
