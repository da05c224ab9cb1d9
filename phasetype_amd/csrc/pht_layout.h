/*
 * pht_layout.h — packed per-sweep parameter block (host builds, device
 * stages into LDS).  One contiguous f64 region followed by an int32 region;
 * offsets depend only on n.
 *
 * Contents per sweep (column-major A[i + j n]):
 *   evals  λ (real parts)                   src/utility.c:109 (dgeevx)
 *   s      exit rates                       src/PHT_MCMC_Aslett.c:244-246
 *   logs   log s_j (s_j > 0, else 0)        probAbsorb numerator (:124)
 *   scale  1/-S_jj, logscale log(1/-S_jj)   dexp in condjumpdens (:131)
 *   piQ    (π^T Q)_i                        Hobolth_endState (:20)
 *   pi     π = e_1                          src/PHT_MCMC_Aslett.c:190-193
 *   S      sub-generator
 *   P, Pf  embedded chain, Pf = [P' | absorb] src/PHT_MCMC_Aslett.c:279-297
 *   QQs    Q[j,i] (Q⁻¹s)_i                  probAbsorb den / moveMass
 *   W      (p_jᵀ Q)_i (Q⁻¹s)_i, p_j = S_j./-S_jj, p_jj = 0   ECS_dens
 *   QQ1    Q[j,i] (Q⁻¹1)_i                  phtcdf(e_j)
 *   V      (P_j.ᵀ Q)_i (Q⁻¹1)_i             phtcdf(P_j.)
 *   Q, Qinv eigenvectors and inverse        DCS
 *   Wm     Wm[j + k n], k < 6: pht_wmoments of row W[j,.]  ECS init point y_t - a
 * int region: candidate lists (increasing index) and their counts
 *   succP[j n + q]      {k : P[j,k] != 0}
 *   succPf[j (n+1) + q] {k in 0..n : Pf[j,k] != 0}
 *   succS[j n + q]      {i != j : S[j,i] != 0}
 */
#ifndef PHT_LAYOUT_H
#define PHT_LAYOUT_H

#if defined(__HIPCC__)
#define PHT_LHD __host__ __device__ constexpr
#else
#define PHT_LHD constexpr
#endif

namespace pht {

constexpr int kMaxN = 32;

struct Layout {
  int n;
  /* f64 offsets (in doubles) */
  int evals, s, logs, scale, logscale, piQ, pi, S, P, Pf, QQs, W, QQ1, V, Q, Qinv, Wm, ndouble;
  int necs; /* doubles the ECS exact path reads: a prefix of the block */
  /* int32 offsets (in ints, from the start of the int region) */
  int nsuccP, succP, nsuccPf, succPf, nsuccS, succS, nint;
  PHT_LHD int bytes() const { return ndouble * 8 + nint * 4; }
};

PHT_LHD Layout make_layout(int n) {
  Layout L{};
  int o = 0, nn = n * n;
  L.n = n;
  L.evals = o; o += n;
  L.s = o; o += n;
  L.logs = o; o += n;
  L.scale = o; o += n;
  L.logscale = o; o += n;
  L.piQ = o; o += n;
  L.pi = o; o += n;
  L.S = o; o += nn;
  L.P = o; o += nn;
  L.QQs = o; o += nn;
  L.W = o; o += nn;
  L.Wm = o; o += 6 * n;
  o += (o & 1);
  /* [0, necs): everything the ECS exact-path kernels read (r04); they stage
   * only this prefix and P's successor lists, see stage_ecs_params */
  L.necs = o;
  L.Pf = o; o += nn + n;
  L.QQ1 = o; o += nn;
  L.V = o; o += nn;
  L.Q = o; o += nn;
  L.Qinv = o; o += nn;
  o += (o & 1); /* keep the int region 16-byte aligned */
  L.ndouble = o;
  int k = 0;
  L.nsuccP = k; k += n;
  L.succP = k; k += nn;
  L.nsuccPf = k; k += n;
  L.succPf = k; k += nn + n;
  L.nsuccS = k; k += n;
  L.succS = k; k += nn;
  k = (k + 3) & ~3;
  L.nint = k;
  return L;
}

/* sufficient-statistics block written by a sweep (int64):
 *   [0, n)          zq   fixed-point z, quantum 2^-zexp
 *   [n, 2n)         B    start-state counts
 *   [2n, 2n+n^2)    N    N[i + j n] transitions i->j, diagonal = absorb-from
 *   then kStatExtra counters: obs processed, ARMS density evals, obs with
 *   flags, uniforms drawn, jumps, Brent CDF evals, UNIF cap hits, 1 spare, and 8 cycle
 *   counters filled only by diagnostic PHT_STAMPS builds */
constexpr int kStatExtra = 16; /* [8..15]: per-phase cycle stamps (PHT_STAMPS builds) */
/* extra-word indices read by the host (gibbs_host.cpp) */
constexpr int kXObs = 0;       /* observations processed: must equal the shard's count */
constexpr int kXFlagged = 2;   /* observations that hit a cap or guard */
constexpr int kXUnifCap = 6;   /* UNIF observations past the Poisson table / lam cap: the sweep is an error */
constexpr int kXOverflow = 15; /* fixed-point z accumulators crossed 2^63 (never in PHT_STAMPS builds) */
/* DEBUG (per-observation) instantiations of the ECS exact kernels only, not
 * in PHT_STAMPS builds: lane-rounds (row-rounds on 16-lane rows) that ran the
 * general ARMS code (an envelope past the converged round's points), and of
 * those the rounds whose envelope reached past the LDS / row points into
 * private memory -- the parity tests assert that they exercised that path */
constexpr int kXDbgGeneral = 8;
constexpr int kXDbgPrivate = 9;
PHT_LHD int stats_len(int n) { return 2 * n + n * n + kStatExtra; }

}  // namespace pht
#endif
