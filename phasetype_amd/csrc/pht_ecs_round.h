/*
 * pht_ecs_round.h — the ARMS part of one round of the persistent ECS-exact
 * kernel, converged across lanes.
 *
 * In a round every lane that needs a sojourn is either
 *   starting  a jump: fresh 9-point envelope (4 density evaluations), or
 *   pending : its previous proposal was rejected; the envelope update that
 *             ends that iteration (src/arms.c:525-621) is due, then the
 *             next iteration.
 * Both kinds then run the SAME code: meets, cumulate, invert, one density
 * evaluation, the acceptance test, Metropolis and moveMass.  The envelope
 * lives in EnvLds with compile-time positions 0..kRoundCap-1 (predicated by
 * the lane's cnt), so these blocks execute once per round for all jumping
 * lanes instead of once per lane kind and rejection chain.  Lanes whose
 * envelope would outgrow kRoundCap use the general code (arms_step).
 *
 * Same draws, same evaluations, same arithmetic per lane as arms() /
 * arms_loop(): meet() is a pure function of its neighbours (and of cnt
 * through the boundary flags), so recomputing every intersection point
 * after an update reproduces the reference's targeted recomputation of the
 * ones next to the new point (src/arms.c:600-615) value for value.
 */
#ifndef PHT_ECS_ROUND_H
#define PHT_ECS_ROUND_H

#include "pht_device.h"

namespace pht {

constexpr int kRoundCap = 13; /* envelope points handled by the converged code */
template <class Env>
constexpr bool round_env_ok() { return Env::kLds == 0 || Env::kLds >= kRoundCap; }
/* run-time envelope positions of the converged round (invert's segment, the
 * insert's neighbours and new point) read through the LDS-only accessors
 * (no private-memory branch: ~900 instructions less per kernel; cfg5 ECS
 * -2.0 %, the 125k shard -1.6 %, cfg4 -0.1 %); not at n = 20, where the
 * allocator then spills 74 VGPRs instead of 43 in the one-lane body (cfg3
 * +1.2 %; profiles/r05/env_lds_only/) */
template <int NT>
constexpr bool round_lds_only() { return NT > 0 && NT < 20; }

/*
 * All intersection points (even positions) of an envelope of at most CAP
 * points (cnt = last + 1), branch-free, with arms_meet's expressions
 * (src/arms.c:700-763).  The slopes arms_meet divides for are those of the
 * segments between consecutive odd (evaluated) points, and each one serves
 * up to three intersection points: gl at K = gr at K - 4 = grl at K - 2.
 * They are divided once here (5 divisions at CAP = 13 instead of 3 per
 * point), and the two divisions of an interior point run only at the
 * positions that can be interior (K = 4, 6, 8: K >= 3 and K + 3 <= last).
 * Every value equals arms_meet's bit for bit: gl and grl are the same
 * quotients; gr is arms_meet's (y_{K+1} - y_{K+3}) / (x_{K+1} - x_{K+3}),
 * the same quotient with both operands negated, which is exact except for
 * the sign of a zero slope, restored explicitly.
 */
template <int CAP, class Env>
__device__ __forceinline__ void round_meets(Env &e, int last) {
  static_assert(CAP % 2 == 1 && CAP >= 5 && CAP <= 13, "converged meets: odd CAP <= 13");
  constexpr int NO = (CAP - 1) / 2; /* odd positions 1, 3, ..., CAP - 2 */
  /* sf[m]: slope of odd points m -> m + 1 (positions 2m+1 -> 2m+3), forward
   * orientation; sb[m]: the same segment in arms_meet's "gr" orientation */
  double sf[NO - 1], sb[NO - 1];
  {
    double xa = e.X(1), ya = e.Y(1);
#pragma unroll
    for (int m = 0; m + 1 < NO; m++) {
      const double xb = e.X(2 * m + 3), yb = e.Y(2 * m + 3);
      const double q = PHT_DIV((yb - ya), (xb - xa));
      sf[m] = q;
      /* (ya - yb) / (xa - xb): = q, but a zero numerator (ya == yb) gives
       * a zero with the sign of (xa - xb) */
      sb[m] = (ya == yb && q == 0.0) ? ((xa - xb < 0.0) ? -0.0 : 0.0) : q;
      xa = xb;
      ya = yb;
    }
  }
#pragma unroll
  for (int K = 0; K < CAP; K += 2) {
    const int mo = K / 2; /* odd index of position K + 1 */
    const bool active = (K <= last);
    const bool il = (K >= 3), ir = (K + 3 <= last), irl = (K >= 1 && K + 1 <= last);
    double xm1 = 0.0, ym1 = 0.0, xp1 = 0.0, yp1 = 0.0;
    if (K >= 1) { xm1 = e.X(K - 1); ym1 = e.Y(K - 1); }
    if (K + 1 < CAP) { xp1 = e.X(K + 1); yp1 = e.Y(K + 1); }
    const double xk = e.X(K), yk = e.Y(K);
    double gl = 0.0, gr = 0.0, grl = 0.0, dl = 0.0, dr = 0.0;
    if (K >= 3) gl = sf[mo - 2];
    if (K + 3 < CAP) gr = ir ? sb[mo] : 0.0;
    if (K >= 1 && K + 1 < CAP) grl = irl ? sf[mo - 1] : 0.0;
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
    bool done = false;
    if (K >= 3 && K + 3 <= CAP - 1) { /* interior: possible only here */
      if (il && ir && irl) {
        nx = PHT_DIV((dl * xp1 + dr * xm1), (dl + dr));
        ny = PHT_DIV((dl * yp1 + dr * ym1 + dl * dr), (dl + dr));
        done = true;
      }
    }
    if (!done) {
      if (il && irl) {
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
    }
    if (active) {
      e.sX(K, nx);
      e.sY(K, ny);
    }
  }
}

/* arms_cumulate over the first CAP positions (cnt <= CAP); the cumulative
 * areas go to cs[] (registers), not to the envelope */
template <int CAP, class Env>
__device__ __forceinline__ void round_cumulate(Env &e, double *cs) {
  const int cnt = e.cnt;
  double xs[CAP], ys[CAP];
#pragma unroll
  for (int k = 0; k < CAP; k++) {
    xs[k] = e.X(k);
    ys[k] = e.Y(k);
  }
  double ymax = ys[0];
#pragma unroll
  for (int k = 1; k < CAP; k++) ymax = (k < cnt && ys[k] > ymax) ? ys[k] : ymax;
  e.ymax = ymax;
  /* (positions < cnt lie at or below ymax; those beyond are never read) */
  double eyp = expshift_le(ys[0], ymax);
  double cum = 0.;
  cs[0] = cum;
#pragma unroll
  for (int k = 1; k < CAP; k++) {
    const double xp = xs[k - 1], xk = xs[k], yp = ys[k - 1], yk = ys[k];
    const double eyk = expshift_le(yk, ymax);
    const double lin = 0.5 * (eyk + eyp) * (xk - xp);
    const double ex = (PHT_DIV((eyk - eyp), (yk - yp))) * (xk - xp);
    const double a = (xp == xk) ? 0. : ((fabs(yk - yp) < kYEps) ? lin : ex);
    cum = cum + a;
    cs[k] = cum;
    eyp = eyk;
  }
}

/* arms_invert with the unrolled scan over cs[] (registers); the segment's
 * ends are tracked along the scan; ey of the two ends recomputed */
template <int CAP, bool LD, class Env>
__device__ __forceinline__ void round_invert(Env &e, const double *cs, double prob, WPt &p) {
  const int last = e.cnt - 1;
  /* cum at last and last - 1 (the segment's ends before the scan moves) */
  double clast = cs[0], cprev = cs[0];
#pragma unroll
  for (int k = 1; k < CAP; k++) {
    clast = (k == last) ? cs[k] : clast;
    cprev = (k == last) ? cs[k - 1] : cprev;
  }
  const double u = prob * clast;
  /* q moves down from last while cum[q-1] > u; the segment's ends follow */
  int q = last;
  double cr = clast, cl = cprev;
  bool go = true;
#pragma unroll
  for (int k = CAP - 2; k >= 1; k--) {
    if (k <= last - 1) {
      go = go && (cs[k] > u);
      q = go ? k : q;
      cr = go ? cs[k] : cr;
      cl = go ? cs[k - 1] : cl;
    }
  }
  p.pr = q;
  const double prop = PHT_DIV((u - cl), (cr - cl));
  /* (1 <= q <= last < CAP <= the LDS points) */
  const double xl = LD ? e.XL(q - 1) : e.X(q - 1), xr = LD ? e.XL(q) : e.X(q);
  const double yr = LD ? e.YL(q) : e.Y(q), yl = LD ? e.YL(q - 1) : e.Y(q - 1);
  const double eyr = expshift_le(yr, e.ymax);
  /* the point is built in scalars and stored once: assigning p's fields in
   * both branches let the compiler merge them into one store through a
   * selected field address, which put p (and its reloads) in scratch every
   * round (r03: ~167 scratch stores per wave per sweep at cfg4) */
  double px, py, pey;
  if (xl == xr) {
    px = xr; py = yr; pey = eyr;
  } else {
    const double eyl = expshift_le(yl, e.ymax);
    if (fabs(yr - yl) < kYEps) {
      if (fabs(eyr - eyl) > kEYEps * fabs(eyr + eyl))
        px = xl + (PHT_DIV((xr - xl), (eyr - eyl))) * (-eyl + sqrt((1. - prop) * eyl * eyl + prop * eyr * eyr));
      else
        px = xl + (xr - xl) * prop;
      pey = (PHT_DIV((px - xl), (xr - xl))) * (eyr - eyl) + eyl;
      py = logshift(pey, e.ymax);
    } else {
      px = xl + (PHT_DIV((xr - xl), (yr - yl))) * (-yl + logshift(((1. - prop) * eyl + prop * eyr), e.ymax));
      py = (PHT_DIV((px - xl), (xr - xl))) * (yr - yl) + yl;
      pey = expshift_le(py, e.ymax);
    }
  }
  p.x = px;
  p.y = py;
  p.ey = pey;
}

/* the first half of arms_update (shift + insert + XEPS adjustment), for an
 * envelope that stays within kRoundCap points; meets and cumulate follow
 * in the converged block */
template <int CAP, bool LD, class Env, class F>
__device__ __forceinline__ void round_insert(Env &e, const ArmsPend &pd, F &f, Lane &ln) {
  /* cnt + 2 <= CAP */
  const int pr = pd.pr;
  const int last = e.cnt - 1;
  const int qi = ((pr - 1) & 1) ? pr + 1 : pr;
  const int ql = (qi >= 2) ? qi - 2 : qi - 1;
  const int qr = (qi + 2 <= last + 2) ? qi + 2 : qi + 1;
  /* the new point's neighbours, read from the old envelope before the shift
   * (new position m holds old m - 2 where the shift moves it, else old m;
   * ql < qi < qr, so neither is the new point): no store -> load wait */
  auto src = [&](int m) { return (m >= 2 && m - 2 >= pr && m - 2 <= last) ? m - 2 : m; };
  /* (every position here is < CAP <= the LDS points) */
  const double xl = LD ? e.XL(src(ql)) : e.X(src(ql)), xr = LD ? e.XL(src(qr)) : e.X(src(qr));
  double xs[CAP], ys[CAP];
#pragma unroll
  for (int k = 0; k + 2 < CAP; k++) {
    xs[k] = e.X(k);
    ys[k] = e.Y(k);
  }
  /* positions k + 2 with k in [pr, last] take old k; the others keep their
   * value (stores only where it moves) */
#pragma unroll
  for (int k = 0; k + 2 < CAP; k++) {
    if (k >= pr && k <= last) {
      e.sX(k + 2, xs[k]);
      e.sY(k + 2, ys[k]);
    }
  }
  e.cnt += 2;
  auto put = [&](double x, double y) {
    if constexpr (LD) {
      e.sXL(qi, x);
      e.sYL(qi, y);
    } else {
      e.sX(qi, x);
      e.sY(qi, y);
    }
  };
  put(pd.px, pd.py);
  if (pd.px < (1. - kXEps) * xl + kXEps * xr) {
    PHT_ISA_SUB("rare");
    const double xn = (1. - kXEps) * xl + kXEps * xr;
    put(xn, f(xn));
    ln.neval++;
    PHT_ISA_SUB("end");
  } else if (pd.px > kXEps * xl + (1. - kXEps) * xr) {
    PHT_ISA_SUB("rare");
    const double xn = kXEps * xl + (1. - kXEps) * xr;
    put(xn, f(xn));
    ln.neval++;
    PHT_ISA_SUB("end");
  }
}

/* Metropolis step with the scan unrolled over the converged envelope; s0/s1
 * = the envelope's points 0 and 1 (read by the caller ahead of the proposal's
 * evaluation, so the LDS round trip is off this step's chain): the segment
 * when X(1) >= xprev, as always for ECS's xprev = 0 */
template <class Env>
__device__ __forceinline__ double round_metropolis(const Env &e, const WPt &p, double ynew, double xprev, double yprev,
                                                   double s0x, double s0y, double s1x, double s1y, Lane &ln) {
  double xql = s0x, yql = s0y, xqr = s1x, yqr = s1y;
  if (s1x < xprev) { /* (not for ECS) */
    int ql = 1;
    while (e.X(ql + 1) < xprev) ql++;
    xql = e.X(ql); yql = e.Y(ql); xqr = e.X(ql + 1); yqr = e.Y(ql + 1);
  }
  double w = PHT_DIV((xprev - xql), (xqr - xql));
  double zold = yql + w * (yqr - yql);
  double znew = p.y;
  if (yprev < zold) zold = yprev;
  if (ynew < znew) znew = ynew;
  w = ynew - znew - yprev + zold;
  if (w > 0.0) w = 0.0;
  w = (w > -kYCeil) ? pht_exp_core(w) : 0.0;
  const double um = dev_u(ln.r);
  return (um > w) ? xprev : p.x;
}

/*
 * One converged ARMS round for the lanes with `start` (begin a jump at
 * st.j) or `pend` (continue one).  On return pend tells whether the lane's
 * jump is still pending; completed jumps have been recorded (moveMass,
 * statistics) exactly as ecs_jump_finish does.
 */
template <int NT, class Env, class Sink>
__device__ __forceinline__ void ecs_round(const Par<NT> &P, Lane &ln, Env &env, Sink &sk, EcsLane<NT> &st, bool start,
                                          bool &pend, ArmsPend &pd, double lam, bool &obsdone) {
  static_assert(round_env_ok<Env>(), "the converged round's positions must lie in the LDS part");
  const int n = P.n();
  const double y_t = st.yt;
  const int j = st.j;
  /* (the caller has generated the next Philox block for this round's
   * draws: invert, test, Metropolis, moveMass, at most 4 words; a new
   * observation's first absorb test takes one more) */
  /* a starting lane without E0 is at its observation's first sojourn: the
   * initial envelope produces E0 from its own vector (ecs_first_E0's rule) */
  const bool mk = start && !st.haveE0;
  EcsDens<NT> f = ecs_dens(P, st, lam);
  PHT_STAMP(ln, 1);
  double xsamp = 0.0;
  int ainfo = 0;
  bool fin = false;  /* the jump ends this round without an iteration */
  bool big = false;  /* envelope outgrows kRoundCap: general code */
  obsdone = false;

  /* ---- starting lanes: initial envelope (arms(), src/arms.c:226-333) */
  if (start) {
    double xinit[4];
    xinit[0] = (y_t) / 1e6;
    xinit[1] = (y_t) / 3.0;
    xinit[2] = xinit[1] * 2.0;
    xinit[3] = y_t - xinit[0];
    double yv[4];
    if ((xinit[0] <= 0.0) || (xinit[3] >= y_t)) {
      ainfo = 1003;
      fin = true;
    } else if (xinit[1] <= xinit[0] || xinit[2] <= xinit[1] || xinit[3] <= xinit[2]) {
      ainfo = 1004;
      fin = true;
    } else {
      f.init4(xinit, yv, mk, st.E0);
    }
    if (mk && fin) { /* rare: no envelope computed it */
      PHT_ISA_SUB("rare");
      ecs_first_E0(P, y_t, lam, st.E0);
      PHT_ISA_SUB("end");
    }
    st.haveE0 = true;
    /* a new observation's first absorb test (ecs_try_absorb: the same draw
     * and arithmetic, after its E0 above) */
    if (st.fold) {
      st.fold = false;
      if (P.s(j) > 0.0) {
        const double U = dev_u(ln.r);
        const double den = dev_dot16([&](int i) { return P.QQs(j, i); }, st.E0, n);
        if (ecs_absorbs(U, P.S(j, j), y_t, P.logs(j), den)) {
          sk.N(j, j);
          sk.z(j, y_t);
          sk.pre(j);
          obsdone = true;
          fin = false;
          ainfo = 0;
        }
      }
    }
    if (!fin && !obsdone) {
      env.cnt = 9;
      env.sX(0, 0.0);
#pragma unroll
      for (int k = 0; k < 4; k++) {
        env.sX(2 * k + 1, xinit[k]);
        env.sY(2 * k + 1, yv[k]);
      }
      ln.neval += 4;
      env.sX(8, y_t);
    }
  }
  start = start && !obsdone;
  PHT_STAMP(ln, 2);
  /* ---- pending lanes: the update that ends the rejected iteration */
  if (pend) big = (env.cnt + 2 > kRoundCap);
  if (__any(pend && !big && env.cnt > 9)) {
    PHT_ISA_SUB("c13");
    if (pend && !big) round_insert<13, round_lds_only<NT>()>(env, pd, f, ln);
    PHT_ISA_SUB("end");
  } else {
    PHT_ISA_SUB("c11");
    if (pend && !big) round_insert<11, round_lds_only<NT>()>(env, pd, f, ln);
    PHT_ISA_SUB("end");
  }
  PHT_STAMP(ln, 3);
  /* ---- converged: intersections and areas over the widest envelope in
   * the wavefront (9, 11 or 13 points) */
  const bool arm = (start && !fin) || (pend && !big);
  const int cap = __any(arm && env.cnt > 11) ? 13 : (__any(arm && env.cnt > 9) ? 11 : 9);
  double cs[kRoundCap]; /* cumulative areas, cumulate -> invert */
  if (arm) {
    if (cap == 9) { PHT_ISA_SUB("c9"); round_meets<9>(env, env.cnt - 1); PHT_ISA_SUB("end"); }
    else if (cap == 11) { PHT_ISA_SUB("c11"); round_meets<11>(env, env.cnt - 1); PHT_ISA_SUB("end"); }
    else { PHT_ISA_SUB("c13"); round_meets<13>(env, env.cnt - 1); PHT_ISA_SUB("end"); }
  }
  PHT_STAMP(ln, 4);
  if (arm) {
    if (cap == 9) { PHT_ISA_SUB("c9"); round_cumulate<9>(env, cs); PHT_ISA_SUB("end"); }
    else if (cap == 11) { PHT_ISA_SUB("c11"); round_cumulate<11>(env, cs); PHT_ISA_SUB("end"); }
    else { PHT_ISA_SUB("c13"); round_cumulate<13>(env, cs); PHT_ISA_SUB("end"); }
  }
  PHT_STAMP(ln, 5);
  if (start && !fin) {
    pd.yprev = f(0.0); /* xprev = 0 lies in [xl, xr] = [0, y_t] */
    ln.neval++;
    pd.it = 0;
  }
  /* the iteration cap is checked after the update (arms_loop) */
  if (pend && !big && pd.it >= kArmsMaxIt) {
    ainfo = 4;
    fin = true;
  }
  PHT_STAMP(ln, 6);
  /* ---- converged: one iteration (sample, evaluate, test) */
  bool acc = false;
  const bool itr = arm && !fin;
  WPt q;
  double yv = 0.0, ynew = 0.0;
  if (itr) {
    const double pu = dev_u(ln.r);
    constexpr bool LD = round_lds_only<NT>();
    if (cap == 9) { PHT_ISA_SUB("c9"); round_invert<9, LD>(env, cs, pu, q); PHT_ISA_SUB("end"); }
    else if (cap == 11) { PHT_ISA_SUB("c11"); round_invert<11, LD>(env, cs, pu, q); PHT_ISA_SUB("end"); }
    else { PHT_ISA_SUB("c13"); round_invert<13, LD>(env, cs, pu, q); PHT_ISA_SUB("end"); }
    const double u = dev_u(ln.r) * q.ey;
    yv = logshift(u, env.ymax);
  }
  PHT_STAMP(ln, 7);
  double s0x = 0.0, s0y = 0.0, s1x = 0.0, s1y = 0.0; /* Metropolis' segment, loaded ahead */
  if (itr) {
    s0x = env.X(0); s0y = env.Y(0); s1x = env.X(1); s1y = env.Y(1);
    ynew = f(q.x);
    ln.neval++;
  }
  PHT_STAMP(ln, 8);
  if (itr) {
    if (yv >= ynew) {
      pd.px = q.x; pd.py = ynew; pd.pey = expshift(ynew, env.ymax); pd.pr = q.pr;
      pd.it++;
      pend = true;
    } else {
      xsamp = round_metropolis(env, q, ynew, 0.0, pd.yprev, s0x, s0y, s1x, s1y, ln);
      acc = true;
    }
  }
  PHT_STAMP(ln, 9);
  /* ---- rare: envelopes beyond kRoundCap continue in the general code */
  if (big) {
    const int rc = arms_step(env, f, pd, 0.0, xsamp, ln);
    if (rc != 1) {
      ainfo = rc;
      acc = true;
    }
    sk.arms_diag(true, env.cnt > Env::kLds);
  }
  PHT_STAMP(ln, 10);
#ifdef PHT_TRACE_GID
  if (ln.r.obs == PHT_TRACE_GID && (start || pend || big || acc || fin))
    printf("T1 j=%d yt=%.17g st=%d pend=%d big=%d cnt=%d qx=%.17g ynew=%.17g yv=%.17g acc=%d xs=%.17g ai=%d\n", st.j,
           y_t, (int)start, (int)pend, (int)big, env.cnt, q.x, ynew, yv, (int)acc, xsamp, ainfo);
#endif
  if (acc || fin) {
    pend = false;
    ecs_jump_finish(P, ln, sk, st, f, xsamp, ainfo);
  }
  PHT_STAMP(ln, 11);
}

}  // namespace pht
#endif
