/*
 * pht_unif.h — the uniformisation sampler ("UNIF", method bit 8): an
 * opt-in, non-parity path sampler that needs no eigendecomposition, so it
 * serves generators whose spectrum is complex or defective, where the
 * reference's ECS/DCS keep only the real parts of the eigenvalues
 * (src/utility.c:118-120) and are wrong.  It is BASELINE.json cfg3's
 * "LDS-tiled uniformisation exp{yS}" and north_star's "exp{y_i S} by
 * uniformisation".  It samples the same conditional path law as ECS (exact
 * observation: absorbed at y; censored: absorbed after y) exactly, up to a
 * Poisson tail below 2^-60 of its peak term.  Specification (the oracle's
 * orc_unif_* in oracle/pht_oracle.c follows it operation for operation):
 *
 * Per sweep (unif_table_kernel, one workgroup): mu = max_i -S_ii (i
 * increasing), rinv = 1 / mu, the uniformised chain R = I + S / mu
 * (R_cj = S_cj * rinv, R_cc = fma(S_cc, rinv, 1)), its squarings
 * P_0 = R, P_i = P_{i-1} P_{i-1}, and for k = 0..K the forward vectors
 * A_k = pi R^k by doubling: A_0 = pi, A_k = A_r P_i with k = 2^i + r,
 * 0 <= r < 2^i (depth log2 K instead of K); every product sums with fma in
 * increasing inner index.  ax_k = sum_j A_k[j] s_j (fma, increasing j:
 * absorption at a virtual step after k steps), ac_k = sum_j A_k[j] (alive),
 * invk_k = 1 / k.  K covers the shard's largest lam = mu y (host:
 * mu y_max + 14 sqrt(mu y_max) + 64, at most kUnifMaxK).
 *
 * Per observation (unif_obs), lam = y mu, a = ax (exact) or ac (censored):
 *  1. (k*, j*) ~ Pois(k; lam) A_k[j] (s_j | 1): unnormalised Poisson weights
 *     w_0 = 2^-1000, w_k = w_{k-1} (lam invk_k); W = sum fma(w_k, a_k, .)
 *     for k = 0.. until k >= lam and w_k < 2^-60 max w (or k = K: flag);
 *     k* = first k whose running sum reaches U W (same sums), j* = first j
 *     whose running sum of A_k*[j] (s_j) reaches U a_k*.  lam > 1300 (where
 *     the unnormalised weights would overflow) or W = 0: flagged fallback.
 *  2. The path on [0, y] given X_{k*} = j* is bridged BACKWARD with the
 *     forward vectors: X_{m-1} ~ A_{m-1}[c] R_{c,X_m} (m = k*, ..., 1), so
 *     no power table is needed; X_0 ~ pi comes out last (the start state B).
 *     The normaliser is the table's A_m[X_m] (= sum_c A_{m-1}[c] R_{c,X_m});
 *     the scan runs over X_m's predecessors only — the c with R_{c,X_m} > 0,
 *     increasing c — with fma running sums; first c whose sum reaches U A_m;
 *     if rounding leaves the sum short, the last predecessor with
 *     A_{m-1}[c] > 0; if A_m[X_m] <= 0 or no such c: flagged, X_{m-1} = X_m.
 *     The k* virtual event times are uniform order statistics on (0, y),
 *     drawn in decreasing order with the bridge in log form:
 *     l_m = fma(log(U), invk_m, l_{m+1}), l_{k*+1} = 0, t_m = y exp(l_m),
 *     evaluated only where the path really moves.  Self-loops are virtual;
 *     a real transition c -> b at t_m closes b's sojourn (z_b += end - t_m)
 *     and counts N[c,b].  Draws per step: U (time), U (state).
 *  3. Exact: absorbed from j* at y (N[j*,j*]++, the reference's diagonal
 *     convention).  Censored: from j* at y the chain runs forward
 *     (memoryless): sojourn Exp(-S_jj) (pht_next_uexp: one word, rarely two), Pfull categorical over
 *     succPf (one word; an overrun takes the last candidate, flag 1), until
 *     absorption.
 * Draw order: U1 (k*), U2 (j*), [U time, U state] x k*, then the censored
 * continuation.
 *
 * The same machinery samples the path laws of the reference's other two
 * samplers exactly ("bridge" mode, SweepArgs::ulaw; PHT_MHRS=bridge,
 * PHT_DCS=bridge):
 *  - ulaw 1, MHRS (LJMA_MHsample_Bladt, src/Simulate_AbsCTMC_eq_Bladt_MHRS.c:
 *    63-114): an attempt of LJMA_samplechain_Bladt is a forward path; the
 *    first success is a draw of that path conditioned on success — exact:
 *    alive at y in a state j with s_j > 0 (the re-draw loop :65-68), i.e.
 *    (k*, j*) ~ Pois(k; lam) A_k[j] 1[s_j > 0] (the table's ax column then
 *    holds aa_k = sum_j 1[s_j > 0] A_k[j], plain adds in increasing j, and
 *    the j* scan adds 1[s_j > 0] A_k*[j]); censored: absorbed after y, i.e.
 *    alive at y then forward, which is ulaw 0's censored law.  The reference
 *    then runs mhit independence-MH steps (:70-101): proposal (k', j') the
 *    same draw, accepted when U < s_j' / s_j*.  Here the current and every
 *    proposal draw only (k*, j*) (two words each, plus the acceptance
 *    uniform), the Poisson total W once; the accepted chain's path is then
 *    bridged.  Draw order (exact): U1 U2 (current), [U1 U2 U] x mhit, the
 *    bridge.  Same law as the rejection search, none of its attempts.
 *  - ulaw 2, DCS (LJMA_MHsample_Hobolth2, src/Simulate_AbsCTMC_eq_
 *    AslettHobolth_DCS.c:92-147): end state b ~ (pi e^{yS})_b s_b, then the
 *    endpoint-conditioned path — ulaw 0's exact law; DCS treats censored
 *    observations as exact (:132-133), so every observation runs ulaw 0's
 *    exact mode.  Flags: kFlagUnifCap (table end, lam cap, zero weights): the
 * observation's path is then NOT a draw of the target law (a truncated
 * Poisson sum, or a placeholder path z(0) = y absorbed from state 0), so a
 * sweep with any such observation is an error (statistics word kXUnifCap;
 * gibbs_host.cpp fails the run, the resident update sets err bit 16).
 */
#ifndef PHT_UNIF_H
#define PHT_UNIF_H

#include "pht_device.h"
#include "pht_kernels.h"

namespace pht {

constexpr int kFlagUnifCap = 64;      /* UNIF: Poisson table end, lam cap or zero weights (an error) */
/* kUnifMaxK, kUnifMaxLam and unif_tab_doubles: pht_kernels.h (the host sizes
 * the table and reports the cap) */

template <class APtr>
struct UnifTab {
  const PHT_LDS double *invk, *ax, *ac; /* staged in LDS */
  APtr A;                               /* row k at A + k n (the global table, L2-resident) */
  const PHT_LDS double *pv;             /* predecessors of b in R: values R_{c,b} at pv[b n + q], */
  const PHT_LDS int *pc, *np;           /* c at pc[b n + q], q < np[b] (unif_preds) */
  int K;
  double mu, rinv;
};

template <int NT>
__device__ __forceinline__ double unif_R(const Par<NT> &P, double rinv, int c, int j) {
  return (c == j) ? fma(P.S(c, c), rinv, 1.0) : P.S(c, j) * rinv;
}

/* b's predecessor list (threads b < n of a block; LDS) */
template <int NT>
__device__ __forceinline__ void unif_preds(const Par<NT> &P, double rinv, PHT_LDS double *pv, PHT_LDS int *pc,
                                           PHT_LDS int *np) {
  const int n = P.n(), b = threadIdx.x;
  if (b >= n) return;
  int q = 0;
  for (int c = 0; c < n; c++) {
    const double v = unif_R(P, rinv, c, b);
    if (v > 0.0) {
      pv[b * n + q] = v;
      pc[b * n + q] = c;
      q++;
    }
  }
  np[b] = q;
}

/* (k*, j*) from the Poisson weights w_k a_k (total W, the last row kend of
 * pass 1) and row k*'s end weights: e = 0 A s_j (fma), 1 A (censored: add),
 * 2 A 1[s_j > 0] (add) */
template <int NT, class APtr>
__device__ __forceinline__ void unif_pick(const Par<NT> &P, const UnifTab<APtr> &T, const PHT_LDS double *a,
                                          double lam, double W, int kend, int e, Lane &ln, int &ks, int &js) {
  const int n = P.n();
  const double target = dev_u(ln.r) * W;
  double w = 0x1p-1000, cum = 0.0;
  int k = 0;
  for (;;) {
    cum = fma(w, a[k], cum);
    if (cum >= target || k >= kend) break;
    k++;
    w = w * (lam * T.invk[k]);
  }
  ks = k;
  const APtr Ak = T.A + (long)ks * n;
  const double t2 = dev_u(ln.r) * a[ks];
  double c2 = 0.0;
  js = n - 1;
  for (int j = 0; j < n; j++) {
    c2 = (e == 0) ? fma(Ak[j], P.s(j), c2) : c2 + ((e == 1 || P.s(j) > 0.0) ? Ak[j] : 0.0);
    if (c2 >= t2) {
      js = j;
      break;
    }
  }
}

template <int NT, class Sink, class APtr>
__device__ __forceinline__ void unif_obs(const Par<NT> &P, const UnifTab<APtr> &T, double y, int cens, Lane &ln,
                                         Sink &sk, int ulaw = 0, int mhit = 0) {
  const int n = P.n();
  if (ulaw == 2) cens = 0; /* DCS: censored observations are treated as exact */
  const double lam = y * T.mu;
  const PHT_LDS double *a = cens ? T.ac : T.ax; /* ulaw 1: ax holds aa */
  bool ok = (lam >= 0.0) && (lam <= kUnifMaxLam);
  int kend = 0;
  double W = 0.0;
  if (ok) {
    double w = 0x1p-1000, wmax = 0.0;
    int k = 0;
    for (;;) {
      W = fma(w, a[k], W);
      wmax = (w > wmax) ? w : wmax;
      if (k >= T.K) {
        ln.flags |= kFlagUnifCap;
        break;
      }
      if ((double)k >= lam && w < wmax * 0x1p-60) break;
      k++;
      w = w * (lam * T.invk[k]);
    }
    kend = k;
    ln.neval += k + 1;
    ok = W > 0.0;
  }
  int b = 0, js = 0;
  if (ok) {
    const int e = cens ? 1 : (ulaw == 1 ? 2 : 0);
    int ks;
    unif_pick(P, T, a, lam, W, kend, e, ln, ks, js);
    if (ulaw == 1 && !cens) {
      /* MHRS: mhit independence-MH steps between draws of the same law,
       * accepted when U < s[pre'] / s[pre] (src/Simulate_AbsCTMC_eq_Bladt_
       * MHRS.c:79-82); only (k, j) of each draw is needed */
      for (int h = 0; h < mhit; h++) {
        int kp, jp;
        unif_pick(P, T, a, lam, W, kend, e, ln, kp, jp);
        const double U = dev_u(ln.r);
        if (U < P.s(jp) / P.s(js)) {
          ks = kp;
          js = jp;
        }
      }
    }
    /* backward bridge */
    b = js;
    double lt = 0.0, tend = y;
    for (int m = ks; m >= 1; m--) {
      lt = fma(pht_log(dev_u(ln.r)), T.invk[m], lt);
      const APtr Am = T.A + (long)(m - 1) * n;
      const double tot = T.A[(long)m * n + b];
      const double tg = dev_u(ln.r) * tot;
      int cs = -1;
      if (tot > 0.0) {
        const int np = T.np[b];
        int last = -1;
        double cum2 = 0.0;
        for (int q = 0; q < np; q++) {
          const int c = T.pc[b * n + q];
          const double av = Am[c];
          cum2 = fma(av, T.pv[b * n + q], cum2);
          last = (av > 0.0) ? c : last;
          if (cum2 >= tg) {
            cs = c;
            break;
          }
        }
        if (cs < 0) cs = last;
      }
      if (cs < 0) {
        ln.flags |= kFlagUnifCap;
        cs = b;
      }
      if (cs != b) {
        const double tm = y * pht_exp_neg(lt);
        sk.z(b, tend - tm);
        sk.N(cs, b);
        ln.njump++;
        tend = tm;
        b = cs;
      }
    }
    sk.z(b, tend);
  } else {
    ln.flags |= kFlagUnifCap;
    js = 0;
    b = 0;
    sk.z(0, y);
  }
  sk.start(b);
  if (!cens) {
    sk.N(js, js);
    sk.pre(js);
    return;
  }
  /* censored: the chain runs on from js at y until absorption */
  int j = js;
  for (int nj = 0;; nj++) {
    if (nj >= kMaxJumps) {
      ln.flags |= kFlagJumpCap;
      sk.N(j, j);
      break;
    }
    sk.z(j, dev_rexp(ln.r, P.scale(j)));
    const double target = dev_u(ln.r);
    const int cnt = P.nsuccPf(j);
    double sofar = 0.0;
    int sel = -1;
    for (int q = 0; q < cnt; q++) {
      const int k = P.succPf(j, q);
      sofar += P.Pf(j, k);
      if (!(sofar < target)) {
        sel = k;
        break;
      }
    }
    if (sel < 0) {
      ln.flags |= kFlagScanEnd;
      sel = cnt > 0 ? P.succPf(j, cnt - 1) : n;
    }
    if (sel >= n) {
      sk.N(j, j);
      break;
    }
    sk.N(j, sel);
    ln.njump++;
    j = sel;
  }
  sk.pre(j);
}

}  // namespace pht
#endif
