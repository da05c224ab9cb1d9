/*
 * pht_cens_round.h — the ECS sampler's right-censored observations
 * (LJMA_samplechain + LJMA_condjump_r_ars, src/Simulate_AbsCTMC_gt_Aslett_DCS.c:
 * 184-260, 299-418) as a persistent kernel of jump-converged rounds.
 *
 * One lane running censored() to the end of its path idles, once its path
 * is done, until the longest path of its wavefront is (a censored path
 * runs past y until absorption, so path lengths vary widely).  Here a loop
 * iteration ("round") is ONE jump of every lane (censored_jump in
 * pht_device.h: the sojourn by the stay test / ARMS / exponential, then
 * the next state); a lane whose path ended takes the next observation at
 * the top of the next round and makes its first jump in that round.
 * Every lane performs exactly censored()'s operations and draws: results
 * are bit-identical to the one-lane kernel and to the oracle's device
 * specification (orcD_censored).  The launch must hold censored
 * observations only (SweepArgs::allcens; ctx_enqueue's censored range).
 */
#ifndef PHT_CENS_ROUND_H
#define PHT_CENS_ROUND_H

#include "pht_device.h"
#include "pht_ecs_round.h"
#include "pht_env.h"

#include <type_traits>

namespace pht {

/* the ARMS envelope's x and y of the first K points in LDS (lane-
 * interleaved, as the exact kernel's; cum and later points private).  The
 * fully private envelope moves ~2.9 KB of scratch per censored observation
 * (cfg5: 435 MB per sweep).  One process per library, 30 % censored
 * (profiles/r03/cens_env_ab2/): n = 10 at 1e6, K = 15: 1.97 -> 1.68 ms;
 * n = 20 at 5e5, K = 9: 2.35 -> 2.30 ms (262 -> 223 VGPRs, two waves);
 * n = 15 (cfg5) K = 15: 1.49 -> 1.87 ms (the ~61 KB per block crowds out
 * the concurrent exact-range kernel), K = 5 or 9: no gain, so private;
 * n = 5: unchanged. */
#ifndef PHT_CENS_K15
#define PHT_CENS_K15 0
#endif
#ifndef PHT_CENS_K20
#define PHT_CENS_K20 9
#endif
/* LDS points per lane (0: the private envelope) */
template <int NT>
constexpr int cens_env_k() { return NT == 10 ? PHT_SLOW_K : NT == 15 ? PHT_CENS_K15 : NT == 20 ? PHT_CENS_K20 : 0; }
template <int NT>
constexpr bool cens_env_lds() { return cens_env_k<NT>() > 0; }
template <int NT>
constexpr int cens_env_bytes() { return cens_env_lds<NT>() ? 2 * cens_env_k<NT>() * 8 * kBlock : 0; }

/*
 * One converged ARMS round of the censored sojourns (r05): `start` lanes
 * begin the ARMS call of their jump (initial envelope, the density at
 * xprev = 0, the first iteration), `pend` lanes end their rejected
 * iteration (the update) and run the next one; both through the exact
 * path's converged blocks (pht_ecs_round.h: meets, cumulate, invert over the
 * widest envelope of the wavefront), so a wavefront no longer waits for its
 * longest rejection chain inside a round.  Same draws, evaluations and
 * arithmetic per lane as arms() (the general ARMS code beyond kRoundCap
 * points).  On return fin tells that the sojourn is drawn (xsamp, ainfo).
 */
template <int NT, class Env>
__device__ __forceinline__ void cens_arms_round(CjDens<NT> &f, Lane &ln, Env &env, bool start, bool &pend, ArmsPend &pd,
                                                double &xsamp, int &ainfo, bool &fin) {
  fin = false;
  ainfo = 0;
  xsamp = 0.0;
  bool big = false;
  if (start) {
    const double x = f.xr;
    double xinit[4];
    xinit[0] = (x) / 1e6;
    xinit[1] = (x) / 3.0;
    xinit[2] = xinit[1] * 2.0;
    xinit[3] = x - xinit[0];
    if ((xinit[0] <= 0.0) || (xinit[3] >= x)) {
      ainfo = 1003;
      fin = true;
    } else if (xinit[1] <= xinit[0] || xinit[2] <= xinit[1] || xinit[3] <= xinit[2]) {
      ainfo = 1004;
      fin = true;
    } else {
      double yv[4];
      f.init4(xinit, yv);
      env.cnt = 9;
      env.sX(0, 0.0);
#pragma unroll
      for (int k = 0; k < 4; k++) {
        env.sX(2 * k + 1, xinit[k]);
        env.sY(2 * k + 1, yv[k]);
      }
      ln.neval += 4;
      env.sX(8, x);
    }
  }
  if (pend) big = (env.cnt + 2 > kRoundCap);
  if (__any(pend && !big && env.cnt > 9)) {
    if (pend && !big) round_insert<13>(env, pd, f, ln);
  } else {
    if (pend && !big) round_insert<11>(env, pd, f, ln);
  }
  const bool arm = (start && !fin) || (pend && !big);
  const int cap = __any(arm && env.cnt > 11) ? 13 : (__any(arm && env.cnt > 9) ? 11 : 9);
  double cs[kRoundCap];
  if (arm) {
    if (cap == 9) round_meets<9>(env, env.cnt - 1);
    else if (cap == 11) round_meets<11>(env, env.cnt - 1);
    else round_meets<13>(env, env.cnt - 1);
  }
  if (arm) {
    if (cap == 9) round_cumulate<9>(env, cs);
    else if (cap == 11) round_cumulate<11>(env, cs);
    else round_cumulate<13>(env, cs);
  }
  if (start && !fin) {
    pd.yprev = f(0.0); /* xprev = 0 */
    ln.neval++;
    pd.it = 0;
  }
  if (pend && !big && pd.it >= kArmsMaxIt) {
    ainfo = 4;
    fin = true;
  }
  const bool itr = arm && !fin;
  WPt q;
  double yv = 0.0, ynew = 0.0;
  if (itr) {
    const double pu = dev_u(ln.r);
    if (cap == 9) round_invert<9>(env, cs, pu, q);
    else if (cap == 11) round_invert<11>(env, cs, pu, q);
    else round_invert<13>(env, cs, pu, q);
    const double u = dev_u(ln.r) * q.ey;
    yv = logshift(u, env.ymax);
  }
  double s0x = 0.0, s0y = 0.0, s1x = 0.0, s1y = 0.0;
  if (itr) {
    s0x = env.X(0); s0y = env.Y(0); s1x = env.X(1); s1y = env.Y(1);
    ynew = f(q.x);
    ln.neval++;
  }
  if (itr) {
    if (yv >= ynew) {
      pd.px = q.x; pd.py = ynew; pd.pey = expshift(ynew, env.ymax); pd.pr = q.pr;
      pd.it++;
      pend = true;
    } else {
      xsamp = round_metropolis(env, q, ynew, 0.0, pd.yprev, s0x, s0y, s1x, s1y, ln);
      fin = true;
      pend = false;
    }
  }
  if (big) {
    const int rc = arms_step(env, f, pd, 0.0, xsamp, ln);
    if (rc != 1) {
      ainfo = rc;
      fin = true;
      pend = false;
    }
  }
  if (fin) pend = false;
}

template <int NT, bool DEBUG>
__device__ __forceinline__ void cens_round_body(const SweepArgs &a, unsigned blk, unsigned nblk) {
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
  PHT_LDS double *envl = (PHT_LDS double *)(lsm + ((pbytes + (n + kStatExtra) * 8 + (n + n * n) * 4 + 4 + 15) & ~15));
  pht_stage_math_tables();
  for (int k = threadIdx.x; k < n + kStatExtra; k += blockDim.x) zq[k] = 0ull;
  for (int k = threadIdx.x; k < n + n * n; k += blockDim.x) Bc[k] = 0u;
  if (threadIdx.x == 0) *cursor = 0;
  __syncthreads();
  Par<NT> P;
  P.d = (const PHT_LDS double *)lsm;
  P.iv = (const PHT_LDS int *)(lsm + L.ndouble * 8);
  P.Lr = L;

  Sink<DEBUG> sk{zq, Bc, Nc, n, a.zscale, nullptr, nullptr, nullptr, nullptr, xc};
  Lane ln;
  ln.flags = 0; ln.neval = 0; ln.nbrent = 0; ln.njump = 0;
  CensLane<NT> cl;
  cl.xr = 0.0; cl.j = 0;
  using EnvL = EnvLdsXY<(cens_env_lds<NT>() ? cens_env_k<NT>() : 1), kBlock>;
  typename std::conditional<cens_env_lds<NT>(), EnvL, EnvPrivate>::type env;
  double spill[2 * EnvL::kSpill];
  double cumv[100];
  if constexpr (cens_env_lds<NT>()) env.bind(envl, threadIdx.x, (PHT_PRIV double *)spill, (PHT_PRIV double *)cumv);
  env.cnt = 0;
  const double lam = lam_max(P);
  ArmsPend pd;
  bool pend = false;
  bool have = false, done = false;
  long pos = 0;
  unsigned c_obs = 0, c_neval = 0, c_flag = 0, c_nd = 0, c_jump = 0;
  auto complete = [&]() {
    const uint32_t nd = pht_stream_pos(&ln.r);
    if (DEBUG) {
      a.dbg_flags[pos] = ln.flags;
      a.dbg_ndraw[pos] = nd;
    }
    c_obs++;
    c_neval += (unsigned)ln.neval;
    c_flag += ln.flags ? 1u : 0u;
    c_nd += nd;
    c_jump += (unsigned)ln.njump;
    have = false;
  };
  for (;;) {
    bool start = false;
    if (!pend) {
      /* ---- a free lane takes the next observation and starts its path */
      if (!have && !done) {
        const long tk = __hip_atomic_fetch_add(cursor, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        const long p = claim_pos(tk, blk, nblk);
        if (p >= a.count) {
          done = true;
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
          censored_begin(P, a.y[pos], ln, sk, cl);
          have = true;
        }
      }
    }
    if (!__any(have)) break;
    /* one converged Philox block per round for the jump's first part (the
     * stay test and the sojourn draw 1-3 words) */
    if (have && !pend) pht_stream_topup(&ln.r);
    /* ---- a jump without ARMS (t >= y, or the stay-past-y branch) ends in
     * this round; an ARMS sojourn starts in the converged block below */
    if (have && !pend) {
      double d = 0.0;
      const int st = censored_step(P, ln, sk, cl, d);
      if (st == 2) complete();
      else if (st == 0) {
        if (censored_finish(P, ln, sk, cl, d, (const CjDens<NT> *)nullptr)) complete();
      } else {
        start = true;
      }
    }
    /* ---- converged ARMS: one iteration of every lane in a sojourn */
    if (__any(start || pend)) {
      /* the iteration draws up to 4 words (invert, test, Metropolis, the next
       * state): a second converged top-up */
      if (start || pend) pht_stream_topup(&ln.r);
      CjDens<NT> f = censored_dens(P, cl, lam);
      double xsamp = 0.0;
      int ainfo = 0;
      bool fin = false;
      cens_arms_round(f, ln, env, start, pend, pd, xsamp, ainfo, fin);
      if (fin) {
        if (ainfo) ln.flags |= (ainfo == 4) ? kFlagArmsCap : kFlagArmsErr;
        if (censored_finish(P, ln, sk, cl, xsamp, &f)) complete();
      }
    }
  }
  lds_add(&xc[0], (unsigned long long)c_obs);
  lds_add(&xc[1], (unsigned long long)c_neval);
  lds_add(&xc[2], (unsigned long long)c_flag);
  lds_add(&xc[3], (unsigned long long)c_nd);
  lds_add(&xc[4], (unsigned long long)c_jump);
  __syncthreads();
  flush_stats(a.stats, zq, Bc, Nc, xc, n);
}

}  // namespace pht
#endif
