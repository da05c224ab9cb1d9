/*
 * pht_ecs_group.h — the ECS-exact path with G lanes per observation.
 *
 * When a GPU holds few observations per lane (the strong-scaling regime: the
 * benchmark's N = 1e6 spread over 8 GPUs), the kernel time is set by the
 * longest paths, one jump per round, and a round's latency is what counts.
 * Here a group of G lanes (G | 64, aligned in the wavefront) carries one
 * observation:
 *   - the spectral vectors are split by residue: lane l holds the slots
 *     r = l + G q (q < 16/G) of the 16-slot layout of pht_dot16, so a density
 *     evaluation is 16/G exponentials per lane plus the pht_dot16 tree (local
 *     levels, then __shfl_xor levels) — the same sum, same order, as one lane;
 *   - the envelope (<= kGrpCap points) lives once per group in LDS; meets and
 *     cumulate's exponentials/areas are spread over the lanes, the prefix sum
 *     and the serial parts (invert, tests, categorical draws) are replicated;
 *   - the per-observation control state and random stream are replicated, so
 *     control flow is uniform within a group; the group leader (l = 0) alone
 *     updates the statistics.
 * Every observation gets exactly the draws, evaluations and arithmetic of
 * the one-lane kernel (pht_ecs_round.h), so results are bit-identical.
 */
#ifndef PHT_ECS_GROUP_H
#define PHT_ECS_GROUP_H

#include "pht_device.h"
#include "pht_ecs_round.h"
#include "pht_env.h"

namespace pht {

constexpr int kGrpCap = 15; /* envelope points held in LDS per group */
constexpr int kGrpArr = 16; /* doubles per envelope array */

/* order LDS accesses of different lanes of one wavefront */
__device__ __forceinline__ void grp_sync() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

/* slots per lane: Q for i < 16 (+ Q for 16 <= i < 32) */
template <int NT, int G>
struct GSlice {
  static constexpr int Q = 16 / G;
  static constexpr int H = (PHT_VEC(NT) > 16) ? 2 : 1;
  static constexpr int S = Q * H;
};

/* E[h Q + q] = e^{lambda_i x}, i = gl + G q + 16 h (0 for i >= n) */
template <int NT, int G>
__device__ __forceinline__ void gexp(const Par<NT> &P, double x, double *E, int gl, int n) {
  using SL = GSlice<NT, G>;
#pragma unroll
  for (int h = 0; h < SL::H; h++) {
#pragma unroll
    for (int q = 0; q < SL::Q; q++) {
      const int i = gl + G * q + 16 * h;
      E[h * SL::Q + q] = (i < n) ? pht_exp_neg(P.evals(i) * x) : 0.0;
    }
  }
}

/* pht_dot16 over a group: every lane returns the full sum */
template <int NT, int G, class Cf>
__device__ __forceinline__ double gdot16(const Cf &cf, const double *E, int gl, int n) {
  using SL = GSlice<NT, G>;
  constexpr int Q = SL::Q;
  double p[Q];
#pragma unroll
  for (int q = 0; q < Q; q++) {
    const int r = gl + G * q;
    p[q] = (r < n) ? cf(r) * E[q] : 0.0;
    if constexpr (SL::H > 1) {
      if (r + 16 < n) p[q] = fma(cf(r + 16), E[Q + q], p[q]);
    }
  }
#pragma unroll
  for (int s = 8; s >= G; s >>= 1) {
#pragma unroll
    for (int q = 0; q < s / G; q++) {
      const int r = gl + G * q;
      if (r + s < n) p[q] = p[q] + p[q + s / G];
    }
  }
  double v = p[0];
#pragma unroll
  for (int s = G / 2; s >= 1; s >>= 1) {
    const double o = __shfl_xor(v, s, G);
    const bool low = !(gl & s);
    const bool has = ((gl & (s - 1)) + s) < n;
    v = has ? (low ? v + o : o + v) : (low ? v : o);
  }
  return v;
}

/* group density of the ECS sojourn (EcsDens, distributed) */
template <int NT, int G>
struct GDens {
  using SL = GSlice<NT, G>;
  const Par<NT> &P;
  int j, gl;
  double y_t, Sjj;
  const double *E0; /* slice: e^{lambda y_t} */
  double lastd;
  double El[SL::S]; /* slice of the most recent evaluation */
  __device__ __forceinline__ double eval_acc(double d) {
    const int n = P.n();
    if (d == 0.0) {
#pragma unroll
      for (int s = 0; s < SL::S; s++) El[s] = E0[s];
    } else {
      gexp<NT, G>(P, y_t - d, El, gl, n);
    }
    lastd = d;
    const int jj = j;
    return gdot16<NT, G>([&](int i) { return P.W(jj, i); }, El, gl, n);
  }
  __device__ __forceinline__ double operator()(double d) { return pht_log(eval_acc(d)) + Sjj * d; }
  /* EcsDens::init4 on slices: the four sums (every lane gets all four) */
  __device__ __forceinline__ void init4_acc(const double xinit[4], double acc[4]) {
    const int n = P.n();
    const int jj = j;
    auto Wj = [&](int i) { return P.W(jj, i); };
    double lammax = 0.0;
    for (int i = 0; i < n; i++) lammax = fmax(lammax, fabs(P.evals(i)));
    const double x3 = y_t - xinit[3];
    if (pht_ecs_init_ok(lammax, xinit[0], x3)) {
      double F[SL::S], T[SL::S];
      gexp<NT, G>(P, y_t - xinit[2], F, gl, n);
      acc[2] = gdot16<NT, G>(Wj, F, gl, n);
#pragma unroll
      for (int s = 0; s < SL::S; s++) T[s] = F[s] * F[s];
      acc[1] = gdot16<NT, G>(Wj, T, gl, n);
#pragma unroll
      for (int h = 0; h < SL::H; h++)
#pragma unroll
        for (int q = 0; q < SL::Q; q++) {
          const int i = gl + G * q + 16 * h;
          const double lam = (i < n) ? P.evals(i) : 0.0;
          T[h * SL::Q + q] = E0[h * SL::Q + q] * pht_exp_taylor(-lam * xinit[0]);
          El[h * SL::Q + q] = pht_exp_taylor(lam * x3);
        }
      acc[0] = gdot16<NT, G>(Wj, T, gl, n);
      acc[3] = gdot16<NT, G>(Wj, El, gl, n);
    } else {
#pragma unroll
      for (int k = 0; k < 4; k++) {
        gexp<NT, G>(P, y_t - xinit[k], El, gl, n);
        acc[k] = gdot16<NT, G>(Wj, El, gl, n);
      }
    }
    lastd = xinit[3];
  }
};

/* per-group envelope in LDS */
struct GEnv {
  PHT_LDS double *x, *y, *ey, *ar, *cum; /* [kGrpArr] each */
  int cnt;
  double ymax;
};

/* arms_meet at a (lane-dependent) position k */
__device__ __forceinline__ void gmeet(GEnv &e, int k, int last) {
  const bool active = (k <= last);
  const bool il = (k >= 3), ir = (k + 3 <= last), irl = (k >= 1 && k + 1 <= last);
  const int km1 = k >= 1 ? k - 1 : 0, km3 = k >= 3 ? k - 3 : 0;
  const int kp1 = k + 1 < kGrpArr ? k + 1 : kGrpArr - 1, kp3 = k + 3 < kGrpArr ? k + 3 : kGrpArr - 1;
  const double xk = e.x[k], yk = e.y[k];
  const double xm1 = (k >= 1) ? e.x[km1] : 0.0, ym1 = (k >= 1) ? e.y[km1] : 0.0;
  const double xm3 = e.x[km3], ym3 = e.y[km3];
  const double xp1 = e.x[kp1], yp1 = e.y[kp1], xp3 = e.x[kp3], yp3 = e.y[kp3];
  double gl = 0.0, gr = 0.0, grl = 0.0, dl = 0.0, dr = 0.0;
  gl = il ? PHT_DIV((ym1 - ym3), (xm1 - xm3)) : 0.0;
  gr = ir ? PHT_DIV((yp1 - yp3), (xp1 - xp3)) : 0.0;
  grl = irl ? PHT_DIV((yp1 - ym1), (xp1 - xm1)) : 0.0;
  if (irl && il && (gl < grl)) gl = gl + (1.0 + 1.0) * (grl - gl);
  if (irl && ir && (gr > grl)) gr = gr + (1.0 + 1.0) * (grl - gr);
  if (il && irl) {
    dr = (gl - grl) * (xp1 - xm1);
    dr = (dr < kYEps) ? kYEps : dr;
  }
  if (ir && irl) {
    dl = (grl - gr) * (xp1 - xm1);
    dl = (dl < kYEps) ? kYEps : dl;
  }
  double nx = xk, ny = yk;
  if (il && ir && irl) {
    nx = PHT_DIV((dl * xp1 + dr * xm1), (dl + dr));
    ny = PHT_DIV((dl * yp1 + dr * ym1 + dl * dr), (dl + dr));
  } else if (il && irl) {
    nx = xp1;
    ny = yp1 + dr;
  } else if (ir && irl) {
    nx = xm1;
    ny = ym1 + dl;
  } else if (il) {
    ny = ym1 + gl * (xk - xm1);
  } else if (ir) {
    ny = yp1 - gr * (xp1 - xk);
  }
  if (active) {
    e.x[k] = nx;
    e.y[k] = ny;
  }
}

/* all intersection points of the group's envelope (cnt <= kGrpCap) */
template <int G>
__device__ __forceinline__ void gmeets(GEnv &e, int gl) {
  const int last = e.cnt - 1;
#pragma unroll
  for (int t = 0; t < (8 + G - 1) / G; t++) {
    const int m = gl + G * t;
    if (m < 8) gmeet(e, 2 * m, last);
  }
  grp_sync();
}

/* arms_cumulate over the group: ey and areas spread over the lanes, the
 * prefix sum replicated in sequence (cum_k = cum_{k-1} + a_k) */
template <int G>
__device__ __forceinline__ void gcumulate(GEnv &e, int gl) {
  const int cnt = e.cnt;
  double ymax = e.y[0];
#pragma unroll
  for (int k = 1; k < kGrpCap; k++) {
    const double yk = e.y[k];
    ymax = (k < cnt && yk > ymax) ? yk : ymax;
  }
  e.ymax = ymax;
#pragma unroll
  for (int t = 0; t < (kGrpCap + G - 1) / G; t++) {
    const int k = gl + G * t;
    if (k < cnt) e.ey[k] = expshift(e.y[k], ymax);
  }
  grp_sync();
#pragma unroll
  for (int t = 0; t < (kGrpCap + G - 1) / G; t++) {
    const int k = gl + G * t;
    if (k >= 1 && k < cnt) {
      const double xp = e.x[k - 1], xk = e.x[k], yp = e.y[k - 1], yk = e.y[k];
      const double eyp = e.ey[k - 1], eyk = e.ey[k];
      const double lin = 0.5 * (eyk + eyp) * (xk - xp);
      const double ex = (PHT_DIV((eyk - eyp), (yk - yp))) * (xk - xp);
      e.ar[k] = (xp == xk) ? 0. : ((fabs(yk - yp) < kYEps) ? lin : ex);
    }
  }
  grp_sync();
  double cum = 0.;
  if (gl == 0) e.cum[0] = cum;
#pragma unroll
  for (int k = 1; k < kGrpCap; k++) {
    if (k < cnt) {
      cum = cum + e.ar[k];
      if ((k % G) == gl) e.cum[k] = cum;
    }
  }
  grp_sync();
}

/* arms_invert on the group envelope (replicated; reads LDS) */
__device__ __forceinline__ void ginvert(GEnv &e, double prob, WPt &p) {
  const int last = e.cnt - 1;
  const double u = prob * e.cum[last];
  int q = last;
  bool go = true;
#pragma unroll
  for (int k = kGrpCap - 2; k >= 1; k--) {
    if (k <= last - 1) {
      go = go && (e.cum[k] > u);
      q = go ? k : q;
    }
  }
  p.pr = q;
  const double cr = e.cum[q], cl = e.cum[q - 1];
  const double prop = PHT_DIV((u - cl), (cr - cl));
  const double xl = e.x[q - 1], xr = e.x[q];
  const double yr = e.y[q], yl = e.y[q - 1];
  const double eyr = expshift(yr, e.ymax);
  if (xl == xr) {
    p.x = xr; p.y = yr; p.ey = eyr;
    return;
  }
  const double eyl = expshift(yl, e.ymax);
  if (fabs(yr - yl) < kYEps) {
    if (fabs(eyr - eyl) > kEYEps * fabs(eyr + eyl))
      p.x = xl + (PHT_DIV((xr - xl), (eyr - eyl))) * (-eyl + sqrt((1. - prop) * eyl * eyl + prop * eyr * eyr));
    else
      p.x = xl + (xr - xl) * prop;
    p.ey = (PHT_DIV((p.x - xl), (xr - xl))) * (eyr - eyl) + eyl;
    p.y = logshift(p.ey, e.ymax);
  } else {
    p.x = xl + (PHT_DIV((xr - xl), (yr - yl))) * (-yl + logshift(((1. - prop) * eyl + prop * eyr), e.ymax));
    p.y = (PHT_DIV((p.x - xl), (xr - xl))) * (yr - yl) + yl;
    p.ey = expshift(p.y, e.ymax);
  }
}

/* shift + insert + XEPS adjustment of arms_update (cnt + 2 <= kGrpCap) */
template <int NT, int G>
__device__ __forceinline__ void ginsert(GEnv &e, const ArmsPend &pd, GDens<NT, G> &f, Lane &ln, int gl) {
  const int pr = pd.pr, last = e.cnt - 1;
  double xs[(kGrpCap + G - 1) / G], ys[(kGrpCap + G - 1) / G];
#pragma unroll
  for (int t = 0; t < (kGrpCap + G - 1) / G; t++) {
    const int k = gl + G * t;
    const int kk = k < kGrpArr ? k : kGrpArr - 1;
    xs[t] = e.x[kk];
    ys[t] = e.y[kk];
  }
  grp_sync();
#pragma unroll
  for (int t = 0; t < (kGrpCap + G - 1) / G; t++) {
    const int k = gl + G * t;
    if (k >= pr && k <= last) {
      e.x[k + 2] = xs[t];
      e.y[k + 2] = ys[t];
    }
  }
  grp_sync();
  e.cnt += 2;
  const int qi = ((pr - 1) & 1) ? pr + 1 : pr;
  if (gl == 0) {
    e.x[qi] = pd.px;
    e.y[qi] = pd.py;
  }
  grp_sync();
  const int ql = (qi >= 2) ? qi - 2 : qi - 1;
  const int qr = (qi + 2 <= e.cnt - 1) ? qi + 2 : qi + 1;
  const double xl = e.x[ql], xr = e.x[qr];
  bool adj = false;
  double xn = 0.0;
  if (pd.px < (1. - kXEps) * xl + kXEps * xr) {
    xn = (1. - kXEps) * xl + kXEps * xr;
    adj = true;
  } else if (pd.px > kXEps * xl + (1. - kXEps) * xr) {
    xn = kXEps * xl + (1. - kXEps) * xr;
    adj = true;
  }
  if (adj) { /* group-uniform */
    const double yn = f(xn);
    ln.neval++;
    grp_sync();
    if (gl == 0) {
      e.x[qi] = xn;
      e.y[qi] = yn;
    }
  }
  grp_sync();
}

/* per-observation state of a group (replicated, E0 sliced) */
template <int NT, int G>
struct GState {
  double yt;
  int j, njump;
  bool haveE0;
  double E0[GSlice<NT, G>::S];
};

/* absorb test (ecs_try_absorb); true = path complete */
template <int NT, int G, class Sink>
__device__ __forceinline__ bool g_try_absorb(const Par<NT> &P, Lane &ln, Sink &sk, GState<NT, G> &st, int gl) {
  const int n = P.n();
  const int j = st.j;
  bool fin = false;
  if (st.njump >= kMaxJumps) {
    ln.flags |= kFlagJumpCap;
    fin = true;
  } else if (P.s(j) > 0.0) {
    const double y_t = st.yt;
    const double U = dev_u(ln.r);
    if (!st.haveE0) {
      gexp<NT, G>(P, y_t, st.E0, gl, n);
      st.haveE0 = true;
    }
    const double den = gdot16<NT, G>([&](int i) { return P.QQs(j, i); }, st.E0, gl, n);
    const double pab = pht_exp(fma(P.S(j, j), y_t, P.logs(j)) - pht_log(den));
    fin = (U < pab);
  }
  if (fin && gl == 0) {
    sk.N(j, j);
    sk.z(j, st.yt);
    sk.pre(j);
  }
  return fin;
}

/* moveMass + categorical + statistics (ecs_jump_finish, distributed dots) */
template <int NT, int G, class Sink>
__device__ __forceinline__ void g_jump_finish(const Par<NT> &P, Lane &ln, Sink &sk, GState<NT, G> &st,
                                              const GDens<NT, G> &f, double xsamp, int ainfo, int gl) {
  using SL = GSlice<NT, G>;
  const int n = P.n();
  const int j = st.j;
  const double y_t = st.yt;
  if (ainfo) ln.flags |= (ainfo == 4) ? kFlagArmsCap : kFlagArmsErr;
  const double d = xsamp;
  const double x = y_t - d;
  double *E = st.E0;
  if (d == f.lastd) {
#pragma unroll
    for (int s = 0; s < SL::S; s++) E[s] = f.El[s];
  } else if (d == 0.0) {
  } else {
    gexp<NT, G>(P, x, E, gl, n);
  }
  st.yt = x;
  st.haveE0 = true;
  const int cnt = P.nsuccP(j);
  double w[PHT_VEC(NT)];
  double sum = 0.0;
#pragma unroll
  for (int q = 0; q < PHT_VEC(NT); q++) {
    if (q < cnt) {
      const int k = P.succP(j, q);
      const double acc = gdot16<NT, G>([&](int i) { return P.QQs(k, i); }, E, gl, n);
      w[q] = P.P(j, k) * acc;
      sum += w[q];
    }
  }
  const double target = dev_u(ln.r) * sum;
  int nj;
  {
    double sofar = 0.0;
    int sel = -1;
#pragma unroll
    for (int q = 0; q < PHT_VEC(NT); q++) {
      if (q < cnt && sel < 0) {
        sofar += w[q];
        if (!(sofar < target)) sel = q;
      }
    }
    if (sel < 0) {
      ln.flags |= kFlagScanEnd;
      sel = cnt - 1;
    }
    nj = (cnt > 0) ? P.succP(j, sel) : 0;
  }
  if (gl == 0) {
    sk.z(j, d);
    sk.N(j, nj);
  }
  ln.njump++;
  st.njump++;
  st.j = nj;
}

/*
 * One ARMS round of a group (ecs_round, distributed).  `start`: begin a jump
 * at st.j; `pend`: continue one.  `bigenv`/`big`: envelopes beyond kGrpCap
 * continue in the general one-lane code on a private copy.
 */
template <int NT, int G, class Sink>
__device__ __forceinline__ void g_round(const Par<NT> &P, Lane &ln, GEnv &env, EnvPrivate &benv, Sink &sk,
                                        GState<NT, G> &st, bool start, bool &pend, bool &big, ArmsPend &pd,
                                        int gl) {
  using SL = GSlice<NT, G>;
  const int n = P.n();
  const double y_t = st.yt;
  if (start || pend) pht_stream_topup(&ln.r);
  if (start && !st.haveE0) {
    gexp<NT, G>(P, y_t, st.E0, gl, n);
    st.haveE0 = true;
  }
  GDens<NT, G> f{P, st.j, gl, y_t, P.S(st.j, st.j), st.E0, -1.0, {}};
  double xsamp = 0.0;
  int ainfo = 0;
  bool fin = false;
  /* ---- starting groups: initial envelope (4 evaluations, logs spread) */
  if (start) {
    double xinit[4];
    xinit[0] = (y_t) / 1e6;
    xinit[1] = (y_t) / 3.0;
    xinit[2] = xinit[1] * 2.0;
    xinit[3] = y_t - xinit[0];
    if ((xinit[0] <= 0.0) || (xinit[3] >= y_t)) {
      ainfo = 1003;
      fin = true;
    } else if (xinit[1] <= xinit[0] || xinit[2] <= xinit[1] || xinit[3] <= xinit[2]) {
      ainfo = 1004;
      fin = true;
    } else {
      double acc[4];
      f.init4_acc(xinit, acc);
      ln.neval += 4;
      env.cnt = 9;
#pragma unroll
      for (int t = 0; t < (4 + G - 1) / G; t++) {
        const int k = gl + G * t;
        if (k < 4) {
          const double a = (k == 0) ? acc[0] : (k == 1) ? acc[1] : (k == 2) ? acc[2] : acc[3];
          const double xk = (k == 0) ? xinit[0] : (k == 1) ? xinit[1] : (k == 2) ? xinit[2] : xinit[3];
          env.x[2 * k + 1] = xk;
          env.y[2 * k + 1] = pht_log(a) + f.Sjj * xk;
        }
      }
      if (gl == 0) {
        env.x[0] = 0.0;
        env.x[8] = y_t;
      }
      grp_sync();
    }
  }
  /* ---- pending groups: the update ending the rejected iteration */
  if (pend && !big) {
    if (env.cnt + 2 > kGrpCap) {
      /* hand the envelope to the general code (private copy per lane) */
      benv.cnt = env.cnt;
      benv.ymax = env.ymax;
      for (int k = 0; k < env.cnt; k++) {
        benv.sX(k, env.x[k]);
        benv.sY(k, env.y[k]);
        benv.sCUM(k, env.cum[k]);
      }
      big = true;
    } else {
      ginsert<NT, G>(env, pd, f, ln, gl);
    }
  }
  const bool arm = (start && !fin) || (pend && !big);
  if (arm) {
    gmeets<G>(env, gl);
    gcumulate<G>(env, gl);
  }
  if (start && !fin) {
    pd.yprev = f(0.0);
    ln.neval++;
    pd.it = 0;
  }
  if (pend && !big && pd.it >= kArmsMaxIt) {
    ainfo = 4;
    fin = true;
  }
  bool acc = false;
  WPt q;
  double ynew = 0.0, yv = 0.0;
  const bool start0 = start, big0 = big;
  if (arm && !fin) {
    ginvert(env, dev_u(ln.r), q);
    const double u = dev_u(ln.r) * q.ey;
    yv = logshift(u, env.ymax);
    ynew = f(q.x);
    ln.neval++;
    if (yv >= ynew) {
      pd.px = q.x; pd.py = ynew; pd.pey = expshift(ynew, env.ymax); pd.pr = q.pr;
      pd.it++;
      pend = true;
    } else {
      /* Metropolis (xprev = 0 -> first segment) */
      int ql = 0;
      while (env.x[ql + 1] < 0.0) ql++;
      const int qr = ql + 1;
      const double xql = env.x[ql], yql = env.y[ql];
      double w = PHT_DIV((0.0 - xql), (env.x[qr] - xql));
      double zold = yql + w * (env.y[qr] - yql);
      double znew = q.y;
      if (pd.yprev < zold) zold = pd.yprev;
      if (ynew < znew) znew = ynew;
      w = ynew - znew - pd.yprev + zold;
      if (w > 0.0) w = 0.0;
      w = (w > -kYCeil) ? pht_exp_core(w) : 0.0;
      const double um = dev_u(ln.r);
      xsamp = (um > w) ? 0.0 : q.x;
      acc = true;
    }
  }
  /* ---- rare: envelopes beyond kGrpCap, one-lane code on the private copy */
  if (big) {
    double E0f[PHT_VEC(NT)];
#pragma unroll
    for (int i = 0; i < PHT_VEC(NT); i++) {
      const int r = i & 15, h = i >> 4;
      E0f[i] = __shfl(st.E0[h * SL::Q + r / G], r % G, G);
    }
    EcsDens<NT> f1{P, st.j, st.yt, P.S(st.j, st.j), E0f, true, -1.0, {}, 0.0, {}};
    f1.load(lam_max(P)); /* W[j, .] into registers (the density's weights) */
    const int rc = arms_step(benv, f1, pd, 0.0, xsamp, ln);
    if (rc != 1) {
      ainfo = rc;
      acc = true;
      big = false;
      /* hand the last evaluation back as slices */
      f.lastd = f1.lastd;
#pragma unroll
      for (int h = 0; h < SL::H; h++)
#pragma unroll
        for (int q = 0; q < SL::Q; q++) {
          const int i = gl + G * q + 16 * h;
          double v = 0.0;
#pragma unroll
          for (int ii = 0; ii < PHT_VEC(NT); ii++) v = (ii == i) ? f1.Elast[ii] : v;
          f.El[h * SL::Q + q] = v;
        }
    }
  }
#ifdef PHT_TRACE_GID
  if (ln.r.obs == PHT_TRACE_GID && gl == 0 && (start0 || pend || big0 || acc || fin))
    printf("T%d j=%d yt=%.17g st=%d pend=%d big=%d cnt=%d qx=%.17g ynew=%.17g yv=%.17g acc=%d xs=%.17g ai=%d\n", G,
           st.j, y_t, (int)start0, (int)pend, (int)big0, big0 ? benv.cnt : env.cnt, q.x, ynew, yv, (int)acc, xsamp,
           ainfo);
#endif
  if (acc || fin) {
    pend = false;
    g_jump_finish<NT, G>(P, ln, sk, st, f, xsamp, ainfo, gl);
  }
}

}  // namespace pht
#endif
