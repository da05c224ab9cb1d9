/*
 * oracle/pht_oracle.h — TEST INFRASTRUCTURE ONLY.
 * Types shared by the two compilations of the CPU restatement
 * (pht_oracle_impl.h included twice by pht_oracle.c).
 */
#ifndef PHT_ORACLE_H
#define PHT_ORACLE_H
#include <stdint.h>

#define ORC_MAXN 40

/* method bitmask (src/PHT_MCMC_Aslett.c:69-71) */
#define ORC_MHRS 0x1
#define ORC_ECS 0x2
#define ORC_DCS 0x4
/* the opt-in uniformisation sampler (no reference counterpart; dev only) */
#define ORC_UNIF 0x8
/* orc_sp_build only: the eigensystem by include/pht_eigen.h (the
 * device-resident chain), not LAPACK */
#define ORC_DEVEIG 0x100
/* with ORC_DEVEIG: refine sp's current eigensystem (the previous sweep's)
 * first, as the resident chain does after its first sweep */
#define ORC_DEVEIG_WARM 0x200

/* per-sweep data handed to the samplers (src/PHT_MCMC_Aslett.c:276-333).
 * All matrices column-major A[i + j*n]; Pfull is n x (n+1). */
typedef struct {
  int n;
  double S[ORC_MAXN * ORC_MAXN], s[ORC_MAXN], pi[ORC_MAXN];
  double P[ORC_MAXN * ORC_MAXN], Pfull[ORC_MAXN * (ORC_MAXN + 1)];
  double Q[ORC_MAXN * ORC_MAXN], Qinv[ORC_MAXN * ORC_MAXN], evals[ORC_MAXN];
  double Qinv_s[ORC_MAXN], Qinv_1[ORC_MAXN];
  int eig_info;
  /* device-mode precomputes (ORC_DEV only; see pht_oracle_impl.h) */
  double QQs[ORC_MAXN * ORC_MAXN]; /* QQs[j + i n] = Q[j,i] Qinv_s[i]          */
  double W[ORC_MAXN * ORC_MAXN];   /* W[j + i n]   = (p_j^T Q)_i Qinv_s[i]     */
  double QQ1[ORC_MAXN * ORC_MAXN]; /* QQ1[j + i n] = Q[j,i] Qinv_1[i]          */
  double V[ORC_MAXN * ORC_MAXN];   /* V[j + i n]   = (P_j. Q)_i Qinv_1[i]      */
  double piQ[ORC_MAXN];            /* (pi^T Q)_i                               */
  double logs[ORC_MAXN];           /* log(s_j) (s_j > 0)                       */
  double scale[ORC_MAXN];          /* 1/-S_jj                                  */
  double logscale[ORC_MAXN];       /* log(1/-S_jj)                             */
  double Wm[ORC_MAXN * 6];         /* Wm[j + k n] = pht_wmoments(W[j,.])_k     */
  /* candidate lists (device mode scans only these, in increasing index):
   *   succP[j]  = {k : P[j,k] != 0}          (moveMass, censored jump)
   *   succPf[j] = {k in 0..n : Pfull[j,k] != 0} (MHRS, censored t >= y)
   *   succS[j]  = {i != j : S[j,i] != 0}     (DCS jump)                  */
  int succP[ORC_MAXN * ORC_MAXN], nsuccP[ORC_MAXN];
  int succPf[ORC_MAXN * (ORC_MAXN + 1)], nsuccPf[ORC_MAXN];
  int succS[ORC_MAXN * ORC_MAXN], nsuccS[ORC_MAXN];
} orc_sp;

/* per-observation result */
typedef struct {
  int B, pre;
  int flags;        /* bit0: categorical scan ran off the end (reference UB) */
  uint32_t ndraw;   /* uniforms consumed (device mode) */
  double z[ORC_MAXN];
  int64_t zq[ORC_MAXN]; /* device mode: fixed-point z, quantum 2^-zexp */
  int N[ORC_MAXN * ORC_MAXN]; /* N[i + j n]: i->j transitions; diag = absorb-from */
} orc_obs;

#endif
