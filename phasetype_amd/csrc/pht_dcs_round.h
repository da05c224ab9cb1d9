/*
 * pht_dcs_round.h — the DCS sampler (method 4) as a persistent kernel of
 * jump-converged rounds.
 *
 * The path of an observation (LJMA_Hobolth_endState +
 * LJMA_samplechain_Hobolth + HobCDF + Find02,
 * src/Simulate_AbsCTMC_eq_AslettHobolth_DCS.c:11-51,
 * src/Simulate_AbsCTMC_gt_Hobolth_DCS.c:23-226, src/utility.c:233-338) is a
 * sequence of jumps (5.4 on average at cfg5-shaped n = 10, up to ~30), each
 * a set-up (E = e^{lambda x}, the exit test, the next state) and a Brent
 * search on HobCDF (~11 CDF evaluations).  With one lane per observation
 * running its whole path, a lane whose path is short idles until the
 * longest path of its wavefront is done.  Here a loop iteration ("round")
 * is ONE jump of every lane; a lane whose path ended takes the next
 * observation at the top of the next round (its end state and start state,
 * then its first jump in the same round), so a wavefront waits only for the
 * slowest Brent search of a jump, not for its longest path.  The round's
 * e^{lambda_i (y - t)} serve both a new observation's end state (t = 0) and
 * the jump's E.
 *
 * Every lane performs exactly the device specification's operations on
 * exactly its values, in the same order, and draws the same words: results
 * are bit-identical to the oracle's device specification
 * (oracle/pht_oracle_impl.h, orcD_dcs; the round-1 one-lane kernel that ran
 * the same path to its end was retired in r05).  Per-sweep n x n tables, computed
 * once per workgroup into LDS, take the divisions out of the CDF
 * evaluations: the near-equal-eigenvalue test |(lambda_i - S_jj) / S_jj| <
 * 1e-13 (same values), and 1 / (lambda_i - S_jj), which the device spec
 * multiplies by where the reference divides.  HobCDF's
 * factor 1/prob * S_{lastj,j} / Pab is computed once per jump.
 *
 * Measured alternative (not kept): rounds of ONE CDF evaluation per lane
 * (a lane whose Brent search ends sets up its next jump at once) remove the
 * wait for the slowest search of a jump (the wavefront's Brent loop runs
 * 1.65x the mean number of evaluations), but the set-up, end-state and
 * Brent-step code then runs divergently in every round: 10-18 % slower at
 * n = 10 and 15 (profiles/r02/dcs/).
 */
#ifndef PHT_DCS_ROUND_H
#define PHT_DCS_ROUND_H

#include "pht_device.h"

namespace pht {

/* lane phases */
enum : int { kDcsFree = 0, kDcsSetup = 1, kDcsNew = 3, kDcsDone = 4 };

/* Provenance: brent_head/brent_tail below are Brent's zeroin as in R core's
 * src/library/stats/src/zeroin.c (R_zeroin2; GPL-2), which the reference
 * carries as Find02 (src/utility.c:233-338, itself that R code).  Its
 * statement order is kept, split around the f(b) call so that a wavefront can
 * run it as a state machine, because PHT_DCS_ROOT=brent must reproduce the
 * reference's root bit for bit (the default root is hob_halley).
 *
 * Find02's state between CDF evaluations; tol = 0 and maxit = 1000 as the
 * reference calls it (src/Simulate_AbsCTMC_gt_Hobolth_DCS.c) */
struct BrentSt {
  double a, b, c, fa, fb, fc;
  int maxit;
};

/* Find02's loop head, up to the next evaluation point: returns true when
 * the search is over (root in `root`), false with b advanced (evaluate f(b)) */
__device__ __forceinline__ bool brent_head(BrentSt &s, double &root) {
  const double tol = 0.0;
  if (!(s.maxit--)) { /* while (maxit--) exhausted */
    root = s.b;
    return true;
  }
  double prev_step = s.b - s.a, tol_act, p, q, new_step;
  if (fabs(s.fc) < fabs(s.fb)) {
    s.a = s.b; s.b = s.c; s.c = s.a;
    s.fa = s.fb; s.fb = s.fc; s.fc = s.fa;
  }
  tol_act = 2 * 2.2204460492503131e-16 * fabs(s.b) + tol / 2;
  new_step = (s.c - s.b) / 2;
  if (fabs(new_step) <= tol_act || s.fb == (double)0) {
    root = s.b;
    return true;
  }
  if (fabs(prev_step) >= tol_act && fabs(s.fa) > fabs(s.fb)) {
    double t1, cb, t2;
    cb = s.c - s.b;
    if (s.a == s.c) {
      t1 = s.fb / s.fa;
      p = cb * t1;
      q = 1.0 - t1;
    } else {
      q = s.fa / s.fc; t1 = s.fb / s.fc; t2 = s.fb / s.fa;
      p = t2 * (cb * q * (q - t1) - (s.b - s.a) * (t1 - 1.0));
      q = (q - 1.0) * (t1 - 1.0) * (t2 - 1.0);
    }
    if (p > (double)0) q = -q;
    else p = -p;
    if (p < (0.75 * cb * q - fabs(tol_act * q) / 2) && p < fabs(prev_step * q / 2)) new_step = p / q;
  }
  if (fabs(new_step) < tol_act) new_step = (new_step > (double)0) ? tol_act : -tol_act;
  s.a = s.b; s.fa = s.fb;
  s.b += new_step;
  return false;
}

/* Find02's loop tail after fb = f(b) */
__device__ __forceinline__ void brent_tail(BrentSt &s, double fb) {
  s.fb = fb;
  if ((s.fb > 0 && s.fc > 0) || (s.fb < 0 && s.fc < 0)) {
    s.c = s.a;
    s.fc = s.fa;
  }
}

/*
 * The jump time: the root of HobCDF(x) = u on [0, X], X = y - t
 * (src/Simulate_AbsCTMC_gt_Hobolth_DCS.c:23-47, 184-187), by a safeguarded
 * Halley iteration — the device spec's replacement for Find02's Brent search
 * (src/utility.c:233-338; still selectable, SweepArgs::dcsbrent).  Both
 * derivatives come from the exponentials F needs: with e_i(x) =
 * e^{(X - x) lambda_i + S_jj x}, J_i = (E_i - e_i) / (lambda_i - S_jj) has
 * J_i' = e_i and J_i'' = (S_jj - lambda_i) e_i (near-equal branch: J_i =
 * x E_i, J_i' = E_i, J_i'' = 0), so with coef = S_{lastj,j} / (prob Pab)
 *   F = coef sum_i Q_ji J_i Qb_i - u,  F' = coef sum_i Q_ji e_i Qb_i,
 *   F'' = coef sum_i Q_ji e_i (S_jj - lambda_i) Qb_i.
 * Start: the truncated exponential's quantile x0 = log(1 - u (1 - e^{S_jj
 * X})) / S_jj (u X if not strictly inside (0, X)).  Each evaluation narrows
 * the sign bracket [lo, hi] (F(0) = -u < 0 < 1 - u = F(X)); the Halley point
 * x - 2 F F' / (2 F'^2 - F F'') is replaced by the bracket's midpoint when it
 * is not strictly inside.  Stops when |F| is within 16 ulps of the
 * magnitudes it is computed from, 16 eps (coef sum_i |Q_ji| |J_i| |Qb_i| +
 * u) with |J_i| taken BEFORE E_i - e_i cancels ((E_i + e_i) / |lambda_i -
 * S_jj|): below that F's own rounding decides (the Halley point is returned
 * if it is in the bracket); when a step moves x by at most 2 eps |x|
 * (Find02's tol_act at Tol = 0); or after 1000 evaluations (Find02's Maxit).
 * The root agrees with Find02's to the evaluation's rounding (~1e-10
 * relative at worst, the same as before r04's bound).  r04: the bound used
 * |J_i| after the cancellation, which is far below F's actual rounding when
 * x is small; ~3 % of jumps then bisected for 6-30 evaluations at the noise
 * floor, and a wavefront's round waits for its slowest lane (E[max of 64]
 * 9.9 -> 5.5 evaluations, mean 3.8 -> 3.5).
 */
/* a lane's e^{lambda_i (y - t)}: registers for small n, lane-interleaved
 * LDS rows from n = 10, where registers spilled
 * (n = 15 / 20 kernel -13 % / -14 %, n = 5 +4 % in LDS) */
/* where the E rows live (compile-time n >= 10: at most 20 rows; the
 * runtime-n kernel keeps E in registers, its n <= 32 rows would not fit
 * beside a 32-state parameter block) */
template <int NT>
constexpr bool dcs_e_in_lds() { return NT >= 10; }
template <int NT, bool LDS = dcs_e_in_lds<NT>()>
struct DcsE {
  double v[PHT_VEC(NT)];
  __device__ __forceinline__ double get(int i) const { return v[i]; }
  __device__ __forceinline__ void set(int i, double x) { v[i] = x; }
};
template <int NT>
struct DcsE<NT, true> {
  PHT_LDS double *p; /* this lane's column: E(i) at p[i kBlock] */
  __device__ __forceinline__ double get(int i) const { return p[i * kBlock]; }
  __device__ __forceinline__ void set(int i, double x) { p[i * kBlock] = x; }
};

/* the jump's Halley weights w_i = Q_{jn,i} Qinv_{i,b} (fixed for the whole
 * root search) in a lane-interleaved LDS column at n = 10: n conflict-free
 * reads per evaluation instead of 2n gathers of two parameter rows.  At
 * n = 15 the column (30 KB per block) would cost the second block per CU,
 * so w_i is formed in each evaluation there and at n = 20 (the same
 * product, the same value) */
template <int NT>
constexpr bool dcs_w_in_lds() { return NT == 10; }

constexpr int kDcsRootMax = 1000;
/* in the unrolled n-term loops of the n >= 10 kernels: keep the scheduler
 * from interleaving more than 4 exponentials at once (each holds ~6 double
 * temporaries; 15 in flight spilled the n = 15 kernel) */
#define PHT_DCS_CHUNK(i) \
  if (dcs_e_in_lds<NT>() && ((i) & 3) == 3) __builtin_amdgcn_sched_barrier(0)
template <int NT>
__device__ __forceinline__ double hob_halley(const Par<NT> &P, const DcsE<NT> &E, const PHT_LDS double *rv, unsigned near,
                                             double Sjj, double X, double es, double coef, double u, int jn, int b,
                                             PHT_LDS double *wl, Lane &ln) {
  const int n = P.n();
  const double eps = 2.2204460492503131e-16;
  if constexpr (dcs_w_in_lds<NT>()) {
#pragma unroll
    for (int i = 0; i < n; i++) wl[i * kBlock] = P.Q(jn, i) * P.Qinv(i, b);
  }
  double lo = 0.0, hi = X;
  const double x0 = pht_log(1.0 - u * (1.0 - es)) / Sjj;
  double xb = (x0 > lo && x0 < hi) ? x0 : u * X;
  double root = xb;
  for (int it = 0; it < kDcsRootMax; it++) {
    const double c1 = X - xb, c0 = Sjj * xb;
    double tmp = 0.0, asum = 0.0, dtmp = 0.0, d2 = 0.0;
#pragma unroll
    for (int i = 0; i < n; i++) {
      const double Ei = E.get(i), ev = P.evals(i);
      double ei, Ji, dl, Jm;
      if ((near >> i) & 1u) {
        ei = Ei;
        Ji = xb * Ei;
        dl = 0.0;
        Jm = fabs(Ji);
      } else {
        ei = pht_exp_neg(c1 * ev + c0);
        Ji = (Ei - ei) * rv[i];
        dl = Sjj - ev;
        Jm = (Ei + ei) * fabs(rv[i]); /* |J_i| before E_i - e_i cancels */
      }
      double w;
      if constexpr (dcs_w_in_lds<NT>()) w = wl[i * kBlock];
      else w = P.Q(jn, i) * P.Qinv(i, b);
      const double we = w * ei;
      tmp = fma(w, Ji, tmp);
      asum = fma(fabs(w), Jm, asum);
      dtmp = fma(w, ei, dtmp);
      d2 = fma(we, dl, d2);
      PHT_DCS_CHUNK(i);
    }
    ln.nbrent++;
    const double F = coef * tmp - u, D = coef * dtmp, D2 = coef * d2;
    if (F == 0.0) {
      root = xb;
      break;
    }
    if (F < 0.0) lo = xb;
    else hi = xb;
    double nx = xb - (2.0 * F * D) / (2.0 * D * D - F * D2);
    if (it == 0) {
      /* the first step in log-survival space: Halley on G = log(S / (1 - u)),
       * S = 1 - CDF = (1 - u) - F, G' = -F'/S, G'' = -F''/S - (F'/S)^2.  The
       * truncated-exponential start is furthest off when u is near 1, where
       * the CDF is flat and plain Halley creeps; the survival function's log
       * is close to linear there (r04: mean evaluations 3.5 -> 3.3, a
       * wavefront's slowest lane 5.5 -> 4.7; tools/dcs_halley_hist.py) */
      const double S = (1.0 - u) - F;
      if (S > 0.0) {
        const double q = D / S, G = pht_log(S / (1.0 - u));
        const double G1 = -q, G2 = -(D2 / S) - q * q;
        nx = xb - (2.0 * G * G1) / (2.0 * G1 * G1 - G * G2);
      }
    }
    if (fabs(F) <= 16.0 * eps * (coef * asum + u)) {
      root = (nx >= lo && nx <= hi) ? nx : xb;
      break;
    }
    if (!(nx > lo && nx < hi)) nx = 0.5 * (lo + hi);
    root = nx;
    if (fabs(nx - xb) <= 2.0 * eps * fabs(xb)) break;
    xb = nx;
  }
  return root;
}

/* A new observation's end state b ~ (pi e^{yS})_b s_b (LJMA_Hobolth_endState,
 * src/Simulate_AbsCTMC_eq_AslettHobolth_DCS.c:11-51) from ey_i = e^{lambda_i
 * y} and the target uniform u: shared by the round kernel and the end-state
 * pre-pass (dcs_end_kernel), so both give the same b bit for bit.  (The
 * weights are recomputed in the scan instead of kept in registers: the
 * same operations, so the same values.) */
template <int NT, class EV>
__device__ __forceinline__ int dcs_end_state(const Par<NT> &P, const EV &ey, double u, int &flags) {
  const int n = P.n();
  double av[PHT_VEC(NT)];
#pragma unroll
  for (int i = 0; i < n; i++) av[i] = P.piQ(i) * ey.get(i);
  double sum = 0.0;
#pragma unroll 1
  for (int k = 0; k < n; k++) {
    double acc = 0.0;
#pragma unroll
    for (int i = 0; i < n; i++) acc = fma(av[i], P.Qinv(i, k), acc);
    sum += acc * P.s(k);
  }
  const double tg = u * sum;
  double sofar = 0.0;
  int q = 0;
#pragma unroll 1
  for (; q < n; q++) {
    double acc = 0.0;
#pragma unroll
    for (int i = 0; i < n; i++) acc = fma(av[i], P.Qinv(i, q), acc);
    sofar += acc * P.s(q);
    if (!(sofar < tg)) break;
  }
  if (q == n) {
    flags |= kFlagScanEnd;
    q = n - 1;
  }
  return q;
}
/* the pre-pass's per-position record: b, and the scan-overrun flag */
constexpr int kDcsEndFlag = 0x100;

/* LDS layout after the sweep kernels' common part (parameter block,
 * accumulators, cursor): near masks [n] u32, then rinv [n*n] f64 */
__host__ __device__ constexpr int dcs_rinv_offset(int pbytes, int n) {
  return (pbytes + (n + kStatExtra) * 8 + (n + n * n) * 4 + 4 + 4 * n + 7) & ~7;
}
/* then each lane's e^{lambda_i (y - t)} of the current jump, lane-interleaved
 * (E(i) at [i kBlock + lane]): in registers they pushed the n = 10..20
 * kernels past 256 VGPRs (n = 15: 202 spilled, ~2.4 GB of scratch traffic
 * per cfg5 sweep) */
__host__ __device__ constexpr int dcs_e_offset(int pbytes, int n) { return dcs_rinv_offset(pbytes, n) + 8 * n * n; }
template <int NT>
constexpr int dcs_smem_bytes(int pbytes, int n) {
  return dcs_e_offset(pbytes, n) + (dcs_e_in_lds<NT>() ? 8 * n * kBlock : 0) + (dcs_w_in_lds<NT>() ? 8 * n * kBlock : 0);
}

/* per-lane path state between jumps */
struct DcsLane {
  int phase;
  double y, t;
  int j, lastj, b, njump;
  int endrec; /* the pre-pass's record of this observation (SweepArgs::dcsb) */
};

/*
 * Persistent DCS kernel body.  blk / nblk: this block's claim chunks
 * (claim_pos).  LDS: parameter block, accumulators, cursor, near masks.
 */
template <int NT, bool DEBUG>
__device__ __forceinline__ void dcs_round_body(const SweepArgs &a, unsigned blk, unsigned nblk) {
  extern __shared__ __align__(16) unsigned char smem[];
  const int n = nval<NT>(a.n);
  const Layout L = make_layout(n);
  const int pbytes = L.bytes();
  {
    const unsigned long long *src = reinterpret_cast<const unsigned long long *>(a.params);
    PHT_LDS unsigned long long *dst = (PHT_LDS unsigned long long *)smem;
    for (int k = threadIdx.x; k < pbytes / 8; k += blockDim.x) dst[k] = src[k];
  }
  PHT_LDS unsigned char *lsm = (PHT_LDS unsigned char *)smem;
  PHT_LDS unsigned long long *zq = (PHT_LDS unsigned long long *)(lsm + pbytes);
  PHT_LDS unsigned long long *xc = zq + n;
  PHT_LDS unsigned *Bc = (PHT_LDS unsigned *)(xc + kStatExtra);
  PHT_LDS unsigned *Nc = Bc + n;
  PHT_LDS int *cursor = (PHT_LDS int *)(Nc + n * n);
  PHT_LDS unsigned *nearm = (PHT_LDS unsigned *)(cursor + 1);
  /* rinv[j n + i] = 1 / (lambda_i - S_jj): J's divisor as a reciprocal
   * (device spec) */
  PHT_LDS double *rinv = (PHT_LDS double *)(lsm + dcs_rinv_offset(pbytes, n));
  DcsE<NT> e;
  if constexpr (dcs_e_in_lds<NT>()) e.p = (PHT_LDS double *)(lsm + dcs_e_offset(pbytes, n)) + threadIdx.x;
  /* the Halley weights' column (after the E rows) */
  PHT_LDS double *wl = nullptr;
  if constexpr (dcs_w_in_lds<NT>())
    wl = (PHT_LDS double *)(lsm + dcs_e_offset(pbytes, n) + 8 * n * kBlock) + threadIdx.x;
  pht_stage_math_tables();
  for (int k = threadIdx.x; k < n + kStatExtra; k += blockDim.x) zq[k] = 0ull;
  for (int k = threadIdx.x; k < n + n * n; k += blockDim.x) Bc[k] = 0u;
  if (threadIdx.x == 0) *cursor = 0;
  __syncthreads();
  Par<NT> P;
  P.d = (const PHT_LDS double *)lsm;
  P.iv = (const PHT_LDS int *)(lsm + L.ndouble * 8);
  P.Lr = L;
  /* near-equal eigenvalue predicate of HobCDF / the set-up's J
   * (src/Simulate_AbsCTMC_gt_Hobolth_DCS.c:27,139), per state */
  for (int jj = threadIdx.x; jj < n; jj += blockDim.x) {
    const double Sjj = P.S(jj, jj);
    unsigned m = 0u;
    for (int i = 0; i < n; i++)
      if (fabs((P.evals(i) - Sjj) / Sjj) < 1e-13) m |= 1u << i;
    nearm[jj] = m;
  }
  for (int k = threadIdx.x; k < n * n; k += blockDim.x) {
    const int jj = k / n, i = k % n;
    rinv[k] = 1.0 / (P.evals(i) - P.S(jj, jj));
  }
  __syncthreads();

  Sink<DEBUG> sk{zq, Bc, Nc, n, a.zscale, nullptr, nullptr, nullptr, nullptr};
  Lane ln;
  ln.flags = 0; ln.neval = 0; ln.nbrent = 0; ln.njump = 0;
  DcsLane st;
  st.phase = kDcsFree;
  long pos = 0;
  unsigned c_obs = 0, c_flag = 0, c_nd = 0, c_jump = 0, c_brent = 0;
#ifdef PHT_DCS_DIAG
  /* diagnostic builds: wavefront-level Brent iterations and rounds (the
   * statistics block's spare words 6 and 7), against the lanes' evaluations
   * (word 5) and jumps (word 4): the lane utilisation of each loop */
  unsigned c_witer = 0, c_wround = 0;
  auto __lane_id_first = [&]() { return __lane_id() == (unsigned)__builtin_ctzll(__ballot(1)); };
#endif

  /* observation complete: counters, debug rows; the lane is free again */
  auto finish_obs = [&]() {
    const uint32_t nd = pht_stream_pos(&ln.r);
    if (DEBUG) {
      a.dbg_flags[pos] = ln.flags;
      a.dbg_ndraw[pos] = nd;
    }
    c_obs++;
    c_flag += ln.flags ? 1u : 0u;
    c_nd += nd;
    c_jump += (unsigned)ln.njump;
    c_brent += (unsigned)ln.nbrent;
    st.phase = kDcsFree;
  };
  /* the head of the path's jump loop (while (t < y) { if (njump++ >= cap) ...),
   * src/Simulate_AbsCTMC_gt_Hobolth_DCS.c */
  auto jump_head = [&]() {
    if (!(st.t < st.y)) { /* the loop condition (t < y always holds after a jump) */
      finish_obs();
      return;
    }
    if (st.njump++ >= kMaxJumps) {
      ln.flags |= kFlagJumpCap;
      finish_obs();
      return;
    }
    st.lastj = st.j;
    st.phase = kDcsSetup;
  };

  /* a new observation's end state ~ (pi e^{yS})_b s_b (endState,
   * src/Simulate_AbsCTMC_eq_AslettHobolth_DCS.c:11-51) from its
   * e^{lambda_i y}, start state, and the jump loop's head */
  auto new_obs = [&](const DcsE<NT> &ey) {
    if (a.dcsb) { /* computed by dcs_end_kernel from the same word */
      const int v = st.endrec;
      (void)pht_next_w(&ln.r);
      if (v & kDcsEndFlag) ln.flags |= kFlagScanEnd;
      st.b = v & (kDcsEndFlag - 1);
    } else {
      st.b = dcs_end_state(P, ey, dev_u(ln.r), ln.flags);
    }
    const double target = dev_u(ln.r);
    const int B = pistart(P, target, ln.flags);
    sk.start(B);
    st.t = 0.0;
    st.j = B;
    st.njump = 0;
    jump_head(); /* t = 0 < y unless y <= 0 */
  };
  /* the end of a jump: Find02's root through the reference's halving guard, the
   * statistics, the next loop head */
  auto end_jump = [&](double root) {
    double jtime = root;
    while (st.t + jtime >= st.y) jtime = jtime / 2;
    sk.N(st.lastj, st.j);
    sk.z(st.lastj, jtime);
    st.t += jtime;
    ln.njump++;
    jump_head();
  };
  {
  for (;;) {
    /* ---- free lanes take the next observation */
    if (st.phase == kDcsFree) {
      const long tk = __hip_atomic_fetch_add(cursor, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      const long p = claim_pos(tk, blk, nblk);
      if (p >= a.count) {
        st.phase = kDcsDone;
      } else {
        pos = a.begin + p;
        pht_stream_init(&ln.r, a.k0, a.k1, a.gid[pos], 0u, a.sweep);
        ln.flags = 0; ln.neval = 0; ln.nbrent = 0; ln.njump = 0;
        if (DEBUG) {
          sk.dz = a.dbg_zq + pos * n;
          sk.dN = a.dbg_N + pos * n * n;
          sk.dB = a.dbg_B + pos;
          sk.dpre = a.dbg_pre + pos;
        }
        st.y = a.y[pos];
        if (a.dcsb) st.endrec = a.dcsb[pos];
        st.t = 0.0;
        st.phase = kDcsNew;
      }
    }
    const bool act = (st.phase != kDcsDone);
    if (!__any(act)) break;
#ifdef PHT_DCS_DIAG
    if (__lane_id_first()) c_wround++;
#endif
    /* one converged Philox block per round (a jump draws at most 3 words,
     * a new observation 2 more) */
    if (act) pht_stream_topup(&ln.r);

    /* ---- e^{lambda_i (y - t)} for every lane (converged): this jump's E,
     * and for a new observation (t = 0) also its end-state vector */
    if (act) {
      const double x = st.y - st.t;
#pragma unroll
      for (int i = 0; i < n; i++) {
        e.set(i, pht_exp_neg(P.evals(i) * x));
        PHT_DCS_CHUNK(i);
      }
    }

    /* ---- a new observation: end state ~ (pi e^{yS})_b s_b (endState,
     * src/Simulate_AbsCTMC_eq_AslettHobolth_DCS.c:11-51), start state,
     * the jump loop's head */
    if (st.phase == kDcsNew) new_obs(e);

    /* ---- one jump of every active lane (the jump loop's body) */
    if (st.phase == kDcsSetup) {
      const int j = st.j;
      const double x = st.y - st.t;
      const double Sjj = P.S(j, j);
      const unsigned near = nearm[j];
      const DcsE<NT> &E = e; /* this jump's e^{lambda_i x} */
      double Pab = 0.0;
#pragma unroll
      for (int i = 0; i < n; i++) Pab = fma(P.Q(j, i) * E.get(i), P.Qinv(i, st.b), Pab);
      bool done = false;
      if (j == st.b) {
        if (dev_runif(ln.r, 0.0, 1.0) < pht_exp_neg(Sjj * (st.y - st.t)) / Pab) {
          sk.z(j, (st.y - st.t));
          sk.N(j, j);
          sk.pre(j);
          finish_obs();
          done = true;
        }
      }
      if (!done) {
        double J[PHT_VEC(NT)];
        const double es = pht_exp_neg(Sjj * x);
#pragma unroll
        for (int i = 0; i < n; i++) {
          if ((near >> i) & 1u) J[i] = x * E.get(i);
          else J[i] = (E.get(i) - es) * rinv[j * n + i];
        }
        const int cnt = P.nsuccS(j);
        /* successor weights S_ji / Pab * (Q J Qb)_i: summed here, then
         * recomputed (same operations, same values) in the scan below, so no
         * per-lane array indexed by the runtime successor count lands in
         * scratch */
        auto weight = [&](int q) {
          const int i = P.succS(j, q);
          double tmp = 0.0;
#pragma unroll
          for (int k = 0; k < n; k++) tmp = fma(P.Q(i, k) * J[k], P.Qinv(k, st.b), tmp);
          return P.S(j, i) / Pab * tmp;
        };
        double p_sum = 0.0;
        for (int q = 0; q < cnt; q++) p_sum += weight(q);
        const double target = dev_runif(ln.r, 0.0, p_sum);
        if (!(target > 0.0)) {
          ln.flags |= kFlagDcsZero;
          sk.pre(j);
          finish_obs();
          done = true;
        } else {
          double sofar = 0.0, prob = 0.0;
          int q = 0;
          for (; q < cnt; q++) {
            prob = weight(q);
            sofar += prob;
            if (!(sofar < target)) break;
          }
          if (q == cnt) { /* prob is the last successor's weight */
            ln.flags |= kFlagScanEnd;
            q = cnt - 1;
          }
          st.j = P.succS(j, q);
          /* HobCDF (src/Simulate_AbsCTMC_gt_Hobolth_DCS.c:23-47):
           * 1/prob * S_{lastj,j} / Pab * sum_i Q_ji J_i(x) Qb_i - u, its
           * factor hoisted out of the evaluations (same operations) */
          const double coef = 1 / prob * P.S(st.lastj, st.j) / Pab;
          const double u = dev_runif(ln.r, 0.0, 1.0);
          const int jn = st.j;
          double root;
          if (!a.dcsbrent) {
            root = hob_halley<NT>(P, E, rinv + j * n, near, Sjj, x, es, coef, u, jn, st.b, wl, ln);
          } else {
          /* Find02(0, y - t, -u, 1 - u, HobCDF, Tol = 0, Maxit = 1000) */
          BrentSt bs;
          bs.a = 0.0;
          bs.b = st.y - st.t;
          bs.fa = -u;
          bs.fb = 1.0 - u;
          bs.c = bs.a;
          bs.fc = bs.fa;
          bs.maxit = 1000 + 1;
          if (bs.fa == 0.0) {
            root = bs.a;
          } else if (bs.fb == 0.0) {
            root = bs.b;
          } else {
            while (!brent_head(bs, root)) {
#ifdef PHT_DCS_DIAG
              if (__lane_id_first()) c_witer++;
#endif
              const double xb = bs.b;
              const double c1 = st.y - st.t - xb, c0 = Sjj * xb;
              double tmp = 0.0;
#pragma unroll
              for (int i = 0; i < n; i++) {
                const double ev = P.evals(i), Ei = E.get(i);
                double Ji;
                if ((near >> i) & 1u) Ji = xb * Ei;
                else Ji = (Ei - pht_exp_neg(c1 * ev + c0)) * rinv[j * n + i];
                tmp = fma(P.Q(jn, i) * Ji, P.Qinv(i, st.b), tmp);
                PHT_DCS_CHUNK(i);
              }
              ln.nbrent++;
              brent_tail(bs, coef * tmp - u);
            }
          }
          }
          end_jump(root);
        }
      }
    }
  }
  }
  lds_add(&xc[0], (unsigned long long)c_obs);
  lds_add(&xc[2], (unsigned long long)c_flag);
  lds_add(&xc[3], (unsigned long long)c_nd);
  lds_add(&xc[4], (unsigned long long)c_jump);
  lds_add(&xc[5], (unsigned long long)c_brent);
#ifdef PHT_DCS_DIAG
  lds_add(&xc[6], (unsigned long long)c_witer);
  lds_add(&xc[7], (unsigned long long)c_wround);
#endif
  __syncthreads();
  flush_stats(a.stats, zq, Bc, Nc, xc, n);
}

}  // namespace pht
#endif
