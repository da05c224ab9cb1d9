/*
 * pht_device.h — per-observation latent-path samplers for one GPU lane.
 *
 * Each function follows the device specification restated on the CPU in
 * oracle/pht_oracle_impl.h (ORC_DEV == 1) operation for operation, so a
 * lane and the oracle produce bit-identical (B, z, N) for the same
 * observation, Philox key, sweep and parameters.  Reference provenance:
 *   ecs_exact      LJMA_samplechain_Aslett2  src/Simulate_AbsCTMC_eq_Aslett_ECS.c:205-373
 *                  (+ LJMA_probAbsorb :120-136, LJMA_ECS_dens :150-171, LJMA_moveMass :21-41)
 *   censored       LJMA_samplechain / LJMA_condjump_r_ars / LJMA_condjumpdens
 *                  src/Simulate_AbsCTMC_gt_Aslett_DCS.c:111-418
 *   mhrs_attempt   one attempt of LJMA_samplechain_Bladt (the search over
 *                  attempts and LJMA_MHsample_Bladt's MH step: pht_mhrs.h)
 *                  src/Simulate_AbsCTMC_eq_Bladt_MHRS.c:37-117, src/Simulate_AbsCTMC_gt_Bladt_MHRS.c:34-160
 *   dcs            LJMA_Hobolth_endState + LJMA_samplechain_Hobolth + HobCDF + Find02
 *                  src/Simulate_AbsCTMC_eq_AslettHobolth_DCS.c:11-51, src/Simulate_AbsCTMC_gt_Hobolth_DCS.c:23-226,
 *                  src/utility.c:233-338
 *   arms           src/arms.c:115-812 (metropolis on, ninit 4, npoint 100)
 *
 * Template parameter NT: compile-time number of transient states (NT > 0:
 * fully unrolled loops, small vectors in registers) or 0 (runtime n).
 * Env: ARMS envelope storage policy (pht_env.h).
 */
#ifndef PHT_DEVICE_H
#define PHT_DEVICE_H

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "pht_detmath.h"
#include "pht_layout.h"
#include "pht_philox.h"

/* LDS (address space 3) qualifier: pointers into the workgroup's LDS must
 * carry it, or hipcc emits generic FLAT loads/stores instead of ds_* */
#define PHT_LDS __attribute__((address_space(3)))

namespace pht {

/* flag bits (per observation) */
constexpr int kFlagScanEnd = 1;    /* categorical scan ran past the last candidate */
constexpr int kFlagDcsZero = 2;    /* DCS jump weights summed to 0 / NaN */
constexpr int kFlagArmsCap = 4;    /* ARMS iteration cap */
constexpr int kFlagJumpCap = 8;    /* path length cap */
constexpr int kFlagMhrsCap = 16;   /* MHRS rejection-attempt cap */
constexpr int kFlagArmsErr = 32;   /* ARMS initial-point error (1003/1004/1007) */

constexpr int kArmsNPoint = 100;
constexpr int kArmsMaxIt = 10000;
constexpr int kMaxJumps = 1 << 20;
constexpr int kMhrsMaxAtt = 1 << 22;
constexpr double kXEps = 0.00001, kYEps = 0.1, kEYEps = 0.001, kYCeil = 50.;

/* parameter block accessor (pointers into LDS or global memory) */
template <int NT>
struct Par {
  const PHT_LDS double *d;
  const PHT_LDS int *iv;
  Layout Lr; /* runtime layout (NT == 0) */
  /* offsets: compile-time constants when NT > 0 */
  __device__ __forceinline__ Layout lay() const {
    if constexpr (NT > 0) {
      constexpr Layout c = make_layout(NT);
      return c;
    } else {
      return Lr;
    }
  }
  __device__ __forceinline__ int n() const { return NT > 0 ? NT : Lr.n; }
  __device__ __forceinline__ double evals(int i) const { return d[lay().evals + i]; }
  __device__ __forceinline__ double s(int i) const { return d[lay().s + i]; }
  __device__ __forceinline__ double logs(int i) const { return d[lay().logs + i]; }
  __device__ __forceinline__ double scale(int i) const { return d[lay().scale + i]; }
  __device__ __forceinline__ double logscale(int i) const { return d[lay().logscale + i]; }
  __device__ __forceinline__ double piQ(int i) const { return d[lay().piQ + i]; }
  __device__ __forceinline__ double pi(int i) const { return d[lay().pi + i]; }
  __device__ __forceinline__ double S(int i, int j) const { return d[lay().S + i + j * n()]; }
  __device__ __forceinline__ double P(int i, int j) const { return d[lay().P + i + j * n()]; }
  __device__ __forceinline__ double Pf(int i, int j) const { return d[lay().Pf + i + j * n()]; }
  __device__ __forceinline__ double QQs(int i, int j) const { return d[lay().QQs + i + j * n()]; }
  __device__ __forceinline__ double W(int i, int j) const { return d[lay().W + i + j * n()]; }
  __device__ __forceinline__ double QQ1(int i, int j) const { return d[lay().QQ1 + i + j * n()]; }
  __device__ __forceinline__ double V(int i, int j) const { return d[lay().V + i + j * n()]; }
  __device__ __forceinline__ double Q(int i, int j) const { return d[lay().Q + i + j * n()]; }
  __device__ __forceinline__ double Qinv(int i, int j) const { return d[lay().Qinv + i + j * n()]; }
  __device__ __forceinline__ const PHT_LDS double *Wm(int j) const { return d + lay().Wm + j; } /* stride n() */
  __device__ __forceinline__ int nsuccP(int j) const { return iv[lay().nsuccP + j]; }
  __device__ __forceinline__ int succP(int j, int q) const { return iv[lay().succP + j * n() + q]; }
  __device__ __forceinline__ int nsuccPf(int j) const { return iv[lay().nsuccPf + j]; }
  __device__ __forceinline__ int succPf(int j, int q) const { return iv[lay().succPf + j * (n() + 1) + q]; }
  __device__ __forceinline__ int nsuccS(int j) const { return iv[lay().nsuccS + j]; }
  __device__ __forceinline__ int succS(int j, int q) const { return iv[lay().succS + j * n() + q]; }
};

#define PHT_VEC(NT) ((NT) > 0 ? (NT) : kMaxN)

/* pht_dot16 (include/pht_detmath.h) with coefficients read through an
 * accessor cf(i): the ECS path's spectral dot products in spec order */
template <class Cf>
__device__ __forceinline__ double dev_dot16(const Cf &cf, const double *E, int n) {
  double p[16];
#pragma unroll
  for (int r = 0; r < 16; r++) {
    p[r] = (r < n) ? cf(r) * E[r] : 0.0;
    if (r + 16 < n) p[r] = fma(cf(r + 16), E[r + 16], p[r]);
  }
#pragma unroll
  for (int s = 8; s >= 1; s >>= 1) {
#pragma unroll
    for (int r = 0; r < s; r++)
      if (r + s < n) p[r] = p[r] + p[r + s];
  }
  return p[0];
}

/* division in the ARMS envelope code; PHT_FASTDIV_ABLATION is a timing-only
 * diagnostic build (approximate reciprocal: results differ) */
#ifdef PHT_FASTDIV_ABLATION
#define PHT_DIV(a, b) ((a) * __builtin_amdgcn_rcp(b))
#else
#define PHT_DIV(a, b) ((a) / (b))
#endif

/* per-lane random stream helpers (oracle: orcD_u / orcD_runif / orcD_rexp) */
__device__ __forceinline__ double dev_u(pht_stream &r) { return pht_next_u(&r); }
__device__ __forceinline__ double dev_runif(pht_stream &r, double a, double b) {
  if (!isfinite(a) || !isfinite(b) || b < a) return __builtin_nan("");
  if (a == b) return a;
  return a + (b - a) * pht_next_u(&r);
}
__device__ __forceinline__ double dev_rexp(pht_stream &r, double scale) {
  if (!isfinite(scale) || scale <= 0.0) return scale == 0.0 ? 0.0 : __builtin_nan("");
  return scale * -pht_log_pos(pht_next_uexp(&r)); /* the uniform is in [2^-53, 1): pht_log's value */
}

/* Lane context: random stream, flags and counters of the current observation. */
struct Lane {
  pht_stream r;
  int flags;
  int neval;
  int nbrent;
  int njump;
#ifdef PHT_STAMPS
  unsigned long long st_last, st_acc[15], st_rounds;
#endif
};

/* diagnostic per-phase cycle stamps (wave-uniform s_memtime) */
#ifdef PHT_STAMPS
#define PHT_STAMP(ln, k)                                              \
  do {                                                                \
    const unsigned long long t_ = __builtin_amdgcn_s_memtime();       \
    (ln).st_acc[k] += t_ - (ln).st_last;                              \
    (ln).st_last = t_;                                                \
  } while (0)
#elif defined(PHT_ISA_MARKS)
/* static-analysis builds only (tools/isa_phases.py, never run): an assembly
 * comment at each stamp site splits the kernel's ISA into the stamped phases */
#define PHT_STAMP(ln, k) asm volatile("; @phase " #k)
/* a wave-uniform variant inside a phase (e.g. the converged blocks' width),
 * closed by PHT_ISA_SUB("end") */
#define PHT_ISA_SUB(tag) asm volatile("; @sub " tag)
#else
#define PHT_STAMP(ln, k) do { } while (0)
#endif
#ifndef PHT_ISA_SUB
#define PHT_ISA_SUB(tag) do { } while (0)
#endif

/* ===================================================================== ARMS */
/* Envelope policies (pht_env.h) expose X/Y/CUM getters and sX/sY/sCUM
 * setters; ey = expshift(y, ymax) is recomputed where needed instead of
 * stored (the reference stores it, src/arms.c:19; recomputation from the
 * same y and ymax is bit-identical). */
__device__ __forceinline__ double expshift(double y, double y0) {
  return (y - y0 > -2.0 * kYCeil) ? pht_exp_hi(y - y0 + kYCeil) : 0.0;
}
/* expshift where y - y0 <= 659 is known (envelope points and hull points
 * against their own ymax: y <= ymax up to rounding): pht_exp_hi's overflow
 * clamp cannot act there, so the same value without it */
__device__ __forceinline__ double expshift_le(double y, double y0) {
  return (y - y0 > -2.0 * kYCeil) ? pht_exp_core(y - y0 + kYCeil) : 0.0;
}
__device__ __forceinline__ double logshift(double y, double y0) { return pht_log(y) + y0 - kYCeil; }

template <class Env>
__device__ __forceinline__ void arms_meet(Env &e, int k) {
  double gl = 0.0, gr = 0.0, grl = 0.0, dl = 0.0, dr = 0.0;
  const int last = e.cnt - 1;
  const bool il = (k >= 3), ir = (k + 3 <= last), irl = (k >= 1 && k + 1 <= last);
  double xm1 = 0.0, ym1 = 0.0, xp1 = 0.0, yp1 = 0.0;
  if (k >= 1) { xm1 = e.X(k - 1); ym1 = e.Y(k - 1); }
  if (k + 1 <= last) { xp1 = e.X(k + 1); yp1 = e.Y(k + 1); }
  if (il) gl = PHT_DIV((ym1 - e.Y(k - 3)), (xm1 - e.X(k - 3)));
  if (ir) gr = PHT_DIV((yp1 - e.Y(k + 3)), (xp1 - e.X(k + 3)));
  if (irl) grl = PHT_DIV((yp1 - ym1), (xp1 - xm1));
  if (irl && il && (gl < grl)) gl = gl + (1.0 + 1.0) * (grl - gl);
  if (irl && ir && (gr > grl)) gr = gr + (1.0 + 1.0) * (grl - gr);
  if (il && irl) {
    dr = (gl - grl) * (xp1 - xm1);
    if (dr < kYEps) dr = kYEps;
  }
  if (ir && irl) {
    dl = (grl - gr) * (xp1 - xm1);
    if (dl < kYEps) dl = kYEps;
  }
  if (il && ir && irl) {
    e.sX(k, PHT_DIV((dl * xp1 + dr * xm1), (dl + dr)));
    e.sY(k, PHT_DIV((dl * yp1 + dr * ym1 + dl * dr), (dl + dr)));
  } else if (il && irl) {
    e.sX(k, xp1);
    e.sY(k, yp1 + dr);
  } else if (ir && irl) {
    e.sX(k, xm1);
    e.sY(k, ym1 + dl);
  } else if (il) {
    e.sY(k, ym1 + gl * (e.X(k) - xm1));
  } else if (ir) {
    e.sY(k, yp1 - gr * (xp1 - e.X(k)));
  }
}

/* Envelopes of up to kArmsU points (the initial 9 plus two updates) use
 * fixed-trip unrolled loops: every access has a compile-time position, so
 * the loads issue together instead of one dependent load per iteration.
 * Positions >= cnt hold stale values that are read and then discarded by
 * selects, or written where no live point is; results are those of the
 * rolled loops. */
constexpr int kArmsU = 13;

template <class Env>
__device__ __forceinline__ void arms_cumulate_u(Env &e) {
  const int cnt = e.cnt;
  double xs[kArmsU], ys[kArmsU];
#pragma unroll
  for (int k = 0; k < kArmsU; k++) {
    xs[k] = e.X(k);
    ys[k] = e.Y(k);
  }
  double ymax = ys[0];
#pragma unroll
  for (int k = 1; k < kArmsU; k++) ymax = (k < cnt && ys[k] > ymax) ? ys[k] : ymax;
  e.ymax = ymax;
  double eyp = expshift_le(ys[0], ymax);
  double cum = 0.;
  e.sCUM(0, cum);
#pragma unroll
  for (int k = 1; k < kArmsU; k++) {
    const double xp = xs[k - 1], xk = xs[k], yp = ys[k - 1], yk = ys[k];
    const double eyk = expshift_le(yk, ymax);
    const double lin = 0.5 * (eyk + eyp) * (xk - xp);
    const double ex = (PHT_DIV((eyk - eyp), (yk - yp))) * (xk - xp);
    const double a = (xp == xk) ? 0. : ((fabs(yk - yp) < kYEps) ? lin : ex);
    cum = cum + a;
    e.sCUM(k, cum);
    eyp = eyk;
  }
}

template <class Env>
__device__ __forceinline__ void arms_cumulate(Env &e) {
  if (Env::kUnroll && e.cnt <= kArmsU) {
    arms_cumulate_u(e);
    return;
  }
  double ymax = e.Y(0);
  for (int k = 1; k < e.cnt; k++) {
    const double yk = e.Y(k);
    if (yk > ymax) ymax = yk;
  }
  e.ymax = ymax;
  double xp = e.X(0), yp = e.Y(0);
  double eyp = expshift_le(yp, ymax);
  double cum = 0.;
  e.sCUM(0, cum);
  for (int k = 1; k < e.cnt; k++) {
    const double xk = e.X(k), yk = e.Y(k);
    const double eyk = expshift_le(yk, ymax);
    double a;
#ifdef PHT_AREA_SELECT
    /* branch-free: both cheap forms, then select (same values) */
    {
      const double lin = 0.5 * (eyk + eyp) * (xk - xp);
      const double ex = (PHT_DIV((eyk - eyp), (yk - yp))) * (xk - xp);
      a = (xp == xk) ? 0. : ((fabs(yk - yp) < kYEps) ? lin : ex);
    }
#else
    if (xp == xk) a = 0.;
    else if (fabs(yk - yp) < kYEps) a = 0.5 * (eyk + eyp) * (xk - xp);
    else a = (PHT_DIV((eyk - eyp), (yk - yp))) * (xk - xp);
#endif
    cum = cum + a;
    e.sCUM(k, cum);
    xp = xk; yp = yk; eyp = eyk;
  }
}

struct WPt {
  double x, y, ey;
  int pr;
};

template <class Env>
__device__ __forceinline__ void arms_invert(Env &e, double prob, WPt &p) {
  int q = e.cnt - 1;
  const double u = prob * e.CUM(q);
  double cl, cr;
  if (Env::kUnroll && e.cnt <= kArmsU) {
    /* q moves down from last while cum[q-1] > u (scan unrolled) */
    const int last = e.cnt - 1;
    double cs[kArmsU];
#pragma unroll
    for (int k = 0; k < kArmsU; k++) cs[k] = e.CUM(k);
    bool go = true;
#pragma unroll
    for (int k = kArmsU - 2; k >= 1; k--) {
      if (k <= last - 1) {
        go = go && (cs[k] > u);
        q = go ? k : q;
      }
    }
    cr = e.CUM(q);
    cl = e.CUM(q - 1);
  } else {
    const double cr0 = e.CUM(q);
    cl = e.CUM(q - 1);
    cr = cr0;
    while (cl > u) {
      q--;
      cr = cl;
      cl = e.CUM(q - 1);
    }
  }
  p.pr = q;
  const double prop = PHT_DIV((u - cl), (cr - cl));
  const double xl = e.X(q - 1), xr = e.X(q);
  const double yr = e.Y(q);
  if (xl == xr) {
    p.x = xr; p.y = yr; p.ey = expshift_le(yr, e.ymax);
    return;
  }
  const double yl = e.Y(q - 1), eyl = expshift_le(yl, e.ymax), eyr = expshift_le(yr, e.ymax);
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
    p.ey = expshift_le(p.y, e.ymax);
  }
}

template <class Env, class F>
__device__ __forceinline__ void arms_update(Env &e, const WPt &p, F &f, Lane &ln) {
  if (e.cnt > kArmsNPoint - 2) return;
  const int pr = p.pr;
  const int last = e.cnt - 1;
  const int qi = ((pr - 1) & 1) ? pr + 1 : pr;
  const int ql = (qi >= 2) ? qi - 2 : qi - 1;
  const int qr = (qi + 2 <= last + 2) ? qi + 2 : qi + 1;
  /* the new point's neighbours from the old envelope, before the shift's
   * stores (new position m holds old m - 2 where the shift moves it, else
   * old m; ql < qi < qr): no store -> load wait (pht_ecs_round.h) */
  const int sl = (ql >= 2 && ql - 2 >= pr && ql - 2 <= last) ? ql - 2 : ql;
  const int sr = (qr >= 2 && qr - 2 >= pr && qr - 2 <= last) ? qr - 2 : qr;
  const double xl = e.X(sl), xr = e.X(sr);
  if (Env::kUnroll && e.cnt <= kArmsU) {
    /* positions pr..cnt-1 move up by 2 (stores only where a point moves) */
    double xs[kArmsU], ys[kArmsU];
#pragma unroll
    for (int k = 0; k < kArmsU; k++) {
      xs[k] = e.X(k);
      ys[k] = e.Y(k);
    }
#pragma unroll
    for (int k = 0; k < kArmsU; k++) {
      if (k >= pr && k <= last) {
        e.sX(k + 2, xs[k]);
        e.sY(k + 2, ys[k]);
      }
    }
  } else {
    for (int k = e.cnt - 1; k >= pr; k--) {
      e.sX(k + 2, e.X(k));
      e.sY(k + 2, e.Y(k));
    }
  }
  e.cnt += 2;
  e.sX(qi, p.x);
  e.sY(qi, p.y);
  if (p.x < (1. - kXEps) * xl + kXEps * xr) {
    const double xn = (1. - kXEps) * xl + kXEps * xr;
    e.sX(qi, xn);
    e.sY(qi, f(xn));
    ln.neval++;
  } else if (p.x > kXEps * xl + (1. - kXEps) * xr) {
    const double xn = kXEps * xl + (1. - kXEps) * xr;
    e.sX(qi, xn);
    e.sY(qi, f(xn));
    ln.neval++;
  }
  arms_meet(e, qi - 1);
  arms_meet(e, qi + 1);
  if (qi >= 2) arms_meet(e, qi - 3);
  if (qi + 2 <= e.cnt - 1) arms_meet(e, qi + 3);
  arms_cumulate(e);
}

/* The sampling loop of arms() from iteration it0 on (src/arms.c:180-215:
 * sample, test, update or Metropolis). */
template <class Env, class F>
__device__ __forceinline__ int arms_loop(Env &e, F &f, double xprev, double yprev, double &xsamp, Lane &ln, int it0) {
  for (int it = it0;; it++) {
    if (it >= kArmsMaxIt) {
      xsamp = xprev;
      return 4;
    }
    WPt p;
    arms_invert(e, dev_u(ln.r), p);
    const double u = dev_u(ln.r) * p.ey;
    const double y = logshift(u, e.ymax);
    const double ynew = f(p.x);
    ln.neval++;
    if (y >= ynew) {
      p.y = ynew;
      p.ey = expshift(p.y, e.ymax);
      arms_update(e, p, f, ln);
      continue;
    }
    int ql = 0;
    while (e.X(ql + 1) < xprev) ql++;
    const int qr = ql + 1;
    const double xql = e.X(ql), yql = e.Y(ql);
    double w = PHT_DIV((xprev - xql), (e.X(qr) - xql));
    double zold = yql + w * (e.Y(qr) - yql);
    double znew = p.y;
    if (yprev < zold) zold = yprev;
    if (ynew < znew) znew = ynew;
    w = ynew - znew - yprev + zold;
    if (w > 0.0) w = 0.0;
    w = (w > -kYCeil) ? pht_exp_core(w) : 0.0;
    const double um = dev_u(ln.r);
    xsamp = (um > w) ? xprev : p.x;
    return 0;
  }
}

/* Metropolis step that ends an accepted iteration (src/arms.c:190-213) */
template <class Env>
__device__ __forceinline__ double arms_metropolis(const Env &e, const WPt &p, double ynew, double xprev, double yprev,
                                                  Lane &ln) {
  int ql = 0;
  while (e.X(ql + 1) < xprev) ql++;
  const int qr = ql + 1;
  const double xql = e.X(ql), yql = e.Y(ql);
  double w = PHT_DIV((xprev - xql), (e.X(qr) - xql));
  double zold = yql + w * (e.Y(qr) - yql);
  double znew = p.y;
  if (yprev < zold) zold = yprev;
  if (ynew < znew) znew = ynew;
  w = ynew - znew - yprev + zold;
  if (w > 0.0) w = 0.0;
  w = (w > -kYCeil) ? pht_exp_core(w) : 0.0;
  const double um = dev_u(ln.r);
  return (um > w) ? xprev : p.x;
}

/* Step-wise arms_loop for persistent kernels: a lane whose proposal was
 * rejected keeps the rejected point pending and performs ONE step per call
 * (the envelope update that ends the rejected iteration, then the next
 * iteration), so a wavefront never waits for its longest rejection chain.
 * Draws, evaluations and results are those of arms_loop. */
struct ArmsPend {
  double px, py, pey, yprev;
  int pr, it; /* it: index of the next iteration */
};

/* returns 0 (xsamp set), 1 (still pending) or 4 (iteration cap) */
template <class Env, class F>
__device__ __forceinline__ int arms_step(Env &e, F &f, ArmsPend &pd, double xprev, double &xsamp, Lane &ln) {
  WPt p;
  p.x = pd.px; p.y = pd.py; p.ey = pd.pey; p.pr = pd.pr;
  arms_update(e, p, f, ln);
  if (pd.it >= kArmsMaxIt) {
    xsamp = xprev;
    return 4;
  }
  WPt q;
  arms_invert(e, dev_u(ln.r), q);
  const double u = dev_u(ln.r) * q.ey;
  const double y = logshift(u, e.ymax);
  const double ynew = f(q.x);
  ln.neval++;
  if (y >= ynew) {
    pd.px = q.x; pd.py = ynew; pd.pey = expshift(ynew, e.ymax); pd.pr = q.pr;
    pd.it++;
    return 1;
  }
  xsamp = arms_metropolis(e, q, ynew, xprev, pd.yprev, ln);
  return 0;
}

/* arms() as used by the reference (xprev 0, one sample).  Returns 0, an
 * initial-point error code, or 4 on the iteration cap. */
template <class Env, class F>
__device__ __forceinline__ int arms(Env &e, const double xinit[4], double xl, double xr, F &f, double xprev, double &xsamp,
                    Lane &ln) {
  if ((xinit[0] <= xl) || (xinit[3] >= xr)) return 1003;
  if (xinit[1] <= xinit[0] || xinit[2] <= xinit[1] || xinit[3] <= xinit[2]) return 1004;
  e.cnt = 9;
  e.sX(0, xl);
  if constexpr (F::kInit4) {
    double yv[4];
    f.init4(xinit, yv);
#pragma unroll
    for (int k = 0; k < 4; k++) {
      e.sX(2 * k + 1, xinit[k]);
      e.sY(2 * k + 1, yv[k]);
    }
  } else {
#pragma unroll
    for (int k = 0; k < 4; k++) {
      e.sX(2 * k + 1, xinit[k]);
      e.sY(2 * k + 1, f(xinit[k]));
    }
  }
  ln.neval += 4;
  e.sX(8, xr);
#pragma unroll
  for (int k = 0; k < 9; k += 2) arms_meet(e, k);
  arms_cumulate(e);
  if ((xprev < xl) || (xprev > xr)) return 1007;
  const double yprev = f(xprev);
  ln.neval++;
  PHT_STAMP(ln, 1);
  return arms_loop(e, f, xprev, yprev, xsamp, ln, 0);
}

/* ====================================================== categorical scans */
/* start state ~ pi (oracle: orcD_pistart) */
template <int NT>
__device__ __forceinline__ int pistart(const Par<NT> &P, double target, int &flags) {
  const int n = P.n();
  double sofar = 0.0;
  int B = 0;
  while (sofar < target) {
    if (B >= n) {
      flags |= kFlagScanEnd;
      return n - 1;
    }
    sofar += P.pi(B++);
  }
  return B - 1;
}

/* ======================================================= ECS exact path */
template <int NT>
struct EcsDens { /* log(sum_i W[j,i] e^{λ_i (y_t - d)}) + S_jj d */
  const Par<NT> &P;
  int j;
  double y_t, Sjj;
  /* exponentials of the absorb test at this state, e^{λ_i y_t} (= the
   * density's at d = 0), and of the most recent evaluation: reused, not
   * recomputed (same expression, same operands: bit-identical) */
  const double *E0;
  bool haveE0;
  double lastd;
  double Elast[PHT_VEC(NT)];
  double lammax;            /* max_i |lambda_i| (init4) */
  /* W[j, .] in registers, except at n >= 15, where it is read from the LDS
   * parameter block (the registers go to a second wave instead) */
  static constexpr bool kWrReg = !(NT >= 15);
  double Wr[kWrReg ? PHT_VEC(NT) : 1];
  __device__ __forceinline__ double w(int i) const {
    if constexpr (kWrReg) return Wr[i];
    else return P.W(j, i);
  }
  __device__ __forceinline__ void load(double lam) {
    const int n = P.n();
    if constexpr (kWrReg) {
#pragma unroll
      for (int i = 0; i < n; i++) Wr[i] = P.W(j, i);
    }
    lammax = lam;
  }
  /* Elast holds the vector of the most recent evaluation at lastd != 0;
   * at d = 0 the sum reads E0 itself (no copy: ecs_jump_finish takes E0 for
   * d = 0 first), so Elast is live only from an evaluation to its use */
  __device__ __forceinline__ double operator()(double d) {
    const int n = P.n();
    const double x = y_t - d;
    double acc;
    if (haveE0 && d == 0.0) {
      PHT_ISA_SUB("d0");
      acc = dev_dot16([&](int i) { return w(i); }, E0, n);
      PHT_ISA_SUB("end");
    } else {
      PHT_ISA_SUB("dx");
#pragma unroll
      for (int i = 0; i < n; i++) Elast[i] = pht_exp_neg(P.evals(i) * x);
      acc = dev_dot16([&](int i) { return w(i); }, Elast, n);
      lastd = d;
      PHT_ISA_SUB("end");
    }
    return pht_log(acc) + Sjj * d;
  }
  /* the four ARMS starting points at once (device spec: pht_ecs_init_ok in
   * include/pht_detmath.h; oracle orcD_ecs_init4) */
  static constexpr bool kInit4 = true;
  /* mk: the observation's first sojourn, E0w (= E0) is produced here
   * (ecs_first_E0's rule, sharing F) */
  __device__ __forceinline__ void init4(const double xinit[4], double yv[4], bool mk = false,
                                        double *E0w = nullptr) {
    const int n = P.n();
    auto Wj = [&](int i) { return w(i); };
    const double x3 = y_t - xinit[3];
    double acc[4];
    if (pht_ecs_init_ok(lammax, xinit[0], x3)) {
      double F[PHT_VEC(NT)], T[PHT_VEC(NT)];
#pragma unroll
      for (int i = 0; i < n; i++) F[i] = pht_exp_neg(P.evals(i) * (y_t - xinit[2]));
      acc[2] = dev_dot16(Wj, F, n);
      /* (E0 in the same loop: F dies here, no extra vector live) */
#pragma unroll
      for (int i = 0; i < n; i++) {
        T[i] = F[i] * F[i];
        if (E0w) E0w[i] = mk ? T[i] * F[i] : E0w[i];
      }
      acc[1] = dev_dot16(Wj, T, n);
#pragma unroll
      for (int i = 0; i < n; i++) T[i] = E0[i] * pht_exp_taylor(-P.evals(i) * xinit[0]);
      acc[0] = dev_dot16(Wj, T, n);
      /* point y_t - a: sum_i W_i taylor5(lambda_i x3) as the state's W-moment
       * polynomial (pht_wmoments; no vector) */
      {
        const PHT_LDS double *m = P.Wm(j);
        const int st = n;
        double q = m[5 * st];
        q = fma(q, x3, m[4 * st]);
        q = fma(q, x3, m[3 * st]);
        q = fma(q, x3, m[2 * st]);
        q = fma(q, x3, m[1 * st]);
        acc[3] = fma(q, x3, m[0]);
      }
    } else {
      PHT_ISA_SUB("rare");
      if (E0w && mk) {
#pragma unroll
        for (int i = 0; i < n; i++) E0w[i] = pht_exp_neg(P.evals(i) * y_t);
      }
#pragma unroll
      for (int k = 0; k < 4; k++) {
        double T[PHT_VEC(NT)];
#pragma unroll
        for (int i = 0; i < n; i++) T[i] = pht_exp_neg(P.evals(i) * (y_t - xinit[k]));
        acc[k] = dev_dot16(Wj, T, n);
      }
      PHT_ISA_SUB("end");
    }
#pragma unroll
    for (int k = 0; k < 4; k++) yv[k] = pht_log(acc[k]) + Sjj * xinit[k];
  }
};

/* The exact-observation path split into phases so a persistent kernel can
 * refill lanes between jumps (pht_kernels.hip); ecs_exact() composes them
 * into the reference's loop (src/Simulate_AbsCTMC_eq_Aslett_ECS.c:231-369). */
template <int NT>
struct EcsLane {
  double yt;                 /* remaining time y - t, carried as yt <- yt - d (device spec) */
  int j, njump;
  bool haveE0;               /* E0 valid for the current remaining time */
  bool haveDen;              /* den valid for (j, E0) */
  double den;                /* pht_dot16(QQs[j,.], E0): moveMass computed it for the chosen state */
  bool fold;                 /* the observation's first absorb test is due inside the next round
                              * (persistent kernel: it shares that round's initial-envelope vector) */
  double E0[PHT_VEC(NT)];    /* e^{λ_i yt}: absorb test / previous moveMass */
};

/* max_i |lambda_i| of the sweep (uniform) */
template <int NT>
__device__ __forceinline__ double lam_max(const Par<NT> &P) {
  double m = 0.0;
#pragma unroll
  for (int i = 0; i < P.n(); i++) m = fmax(m, fabs(P.evals(i)));
  return m;
}

/* E0 = e^{λ_i y_t} at an observation's first sojourn (device spec,
 * pht_ecs_e0_cube): (F F) F from the vector F = e^{λ_i (y_t - 2b)} of that
 * sojourn's ARMS starting points when pht_ecs_init_ok holds, else directly */
template <int NT>
__device__ __forceinline__ void ecs_first_E0(const Par<NT> &P, double y_t, double lammax, double *E0) {
  const int n = P.n();
  const double a = (y_t) / 1e6, b2 = ((y_t) / 3.0) * 2.0;
  if (pht_ecs_init_ok(lammax, a, y_t - (y_t - a))) {
#pragma unroll
    for (int i = 0; i < n; i++) E0[i] = pht_ecs_e0_cube(pht_exp_neg(P.evals(i) * (y_t - b2)));
  } else {
#pragma unroll
    for (int i = 0; i < n; i++) E0[i] = pht_exp_neg(P.evals(i) * y_t);
  }
}

template <int NT, class Sink>
__device__ __forceinline__ void ecs_begin(const Par<NT> &P, double y, Lane &ln, Sink &sk, EcsLane<NT> &st) {
  const double target = dev_u(ln.r);
  const int B = pistart(P, target, ln.flags);
  sk.start(B);
  st.yt = y;
  st.j = B;
  st.njump = 0;
  st.haveE0 = false;
  st.haveDen = false;
  st.fold = false;
}

/* LJMA_probAbsorb's test U < exp(S_jj y_t + log s_j - log den) (:120-136,
 * :251-255) in the device spec's form U den < exp(S_jj y_t + log s_j): the
 * same decision up to rounding, one logarithm less per test (den = 0
 * absorbs, den < 0 does not, as the log form) */
__device__ __forceinline__ bool ecs_absorbs(double U, double Sjj, double y_t, double logs, double den) {
  return (den > 0.0) ? (U * den < pht_exp(fma(Sjj, y_t, logs))) : (den == 0.0);
}

/* absorb test at the current state (LJMA_probAbsorb + runif, :251-255);
 * true = the path is complete and its last sojourn has been recorded */
template <int NT, class Sink>
__device__ __forceinline__ bool ecs_try_absorb(const Par<NT> &P, Lane &ln, Sink &sk, EcsLane<NT> &st) {
  const int n = P.n();
  const int j = st.j;
  bool fin = false;
  if (st.njump >= kMaxJumps) {
    ln.flags |= kFlagJumpCap;
    fin = true;
  } else if (P.s(j) > 0.0) {
    const double y_t = st.yt;
    const double U = dev_u(ln.r);
    if (!st.haveE0) { /* the observation's first sojourn */
      ecs_first_E0(P, y_t, lam_max(P), st.E0);
      st.haveE0 = true;
      st.haveDen = false;
    }
    const double den = st.haveDen ? st.den : dev_dot16([&](int i) { return P.QQs(j, i); }, st.E0, n);
    fin = ecs_absorbs(U, P.S(j, j), y_t, P.logs(j), den);
  }
  if (fin) {
    sk.N(j, j);
    sk.z(j, st.yt);
    sk.pre(j);
  }
  return fin;
}

/* end of a non-absorbing jump once the sojourn d is drawn: moveMass +
 * categorical (:350-358), statistics (:362-363) */
template <int NT, class Sink>
__device__ __forceinline__ void ecs_jump_finish(const Par<NT> &P, Lane &ln, Sink &sk, EcsLane<NT> &st,
                                                const EcsDens<NT> &f, double xsamp, int ainfo) {
  const int n = P.n();
  const int j = st.j;
  const double y_t = st.yt;
  if (ainfo) ln.flags |= (ainfo == 4) ? kFlagArmsCap : kFlagArmsErr;
  const double d = xsamp;
  const double x = y_t - d;
  /* e^{λ_i (y_t - d)}: the accepted proposal's density evaluation already
   * computed them (d = lastd), or d = 0 = the absorb test's; they become
   * the next absorb test's (yt <- x) */
  double *E = st.E0;
  if (d == 0.0) {
    /* E0 already holds e^{λ_i y_t} = e^{λ_i x} */
  } else if (d == f.lastd) {
#pragma unroll
    for (int i = 0; i < n; i++) E[i] = f.Elast[i];
  } else {
    PHT_ISA_SUB("rare");
#pragma unroll
    for (int i = 0; i < n; i++) E[i] = pht_exp_neg(P.evals(i) * x);
    PHT_ISA_SUB("end");
  }
  st.yt = x;
  st.haveE0 = true;
  const int cnt = P.nsuccP(j);
  int nj;
  /* weights w_q = P[j,k_q] (QQs[k_q,.] . E) over the successors, their sum,
   * then the categorical scan (:352-358).  The first two successors' values
   * are kept (every state of a birth-death chain has at most two); any
   * further one is recomputed in the scan, the same expressions in the same
   * order, so the result does not depend on how many are kept.  (Register
   * arrays over all n possible successors cost ~100 moves per round at
   * n = 10, their zero-fill and shuffles, and pushed n = 20 further into
   * spills: cfg3 kernel -6.7 %, cfg5 -3.0 %, cfg4 -0.75 %) */
  double w0 = 0.0, w1 = 0.0, a0 = 0.0, a1 = 0.0;
  double sum = 0.0;
  for (int q = 0; q < cnt; q++) {
    const int k = P.succP(j, q);
    const double acc = dev_dot16([&](int i) { return P.QQs(k, i); }, E, n);
    const double wq = P.P(j, k) * acc;
    if (q == 0) {
      a0 = acc;
      w0 = wq;
    } else if (q == 1) {
      a1 = acc;
      w1 = wq;
    }
    sum += wq;
  }
  const double target = dev_u(ln.r) * sum;
  {
    double sofar = 0.0, dsel = 0.0;
    int sel = -1;
    for (int q = 0; q < cnt; q++) {
      double wq, aq;
      if (q == 0) {
        wq = w0;
        aq = a0;
      } else if (q == 1) {
        wq = w1;
        aq = a1;
      } else {
        const int k = P.succP(j, q);
        aq = dev_dot16([&](int i) { return P.QQs(k, i); }, E, n);
        wq = P.P(j, k) * aq;
      }
      sofar += wq;
      dsel = aq; /* the selected one, or the last (scan end) */
      if (!(sofar < target)) {
        sel = q;
        break;
      }
    }
    if (sel < 0) {
      ln.flags |= kFlagScanEnd;
      sel = cnt - 1;
    }
    nj = (cnt > 0) ? P.succP(j, sel) : 0;
    /* the next absorb test's denominator: same dot product, same E */
    st.den = dsel;
    st.haveDen = (cnt > 0);
  }
  sk.z(j, d);
  sk.N(j, nj);
  ln.njump++;
  st.njump++;
  st.j = nj;
}

template <int NT>
__device__ __forceinline__ EcsDens<NT> ecs_dens(const Par<NT> &P, EcsLane<NT> &st, double lam) {
  EcsDens<NT> f{P, st.j, st.yt, P.S(st.j, st.j), st.E0, true, -1.0, {}, 0.0, {}};
  f.load(lam);
  return f;
}
template <int NT>
__device__ __forceinline__ EcsDens<NT> ecs_dens(const Par<NT> &P, EcsLane<NT> &st) {
  return ecs_dens(P, st, lam_max(P));
}

/* ===================================================== censored path */
/*
 * Device specification of the censored path (r05, "v2"; the oracle's dev
 * variant orcD_obs_censored follows it operation for operation):
 *  - the remaining time to y is carried, xr <- xr - d (the reference
 *    recomputes y - t); every "t < y" decision reads xr > 0 and the sojourn
 *    density's argument is xr - d (the exact path's y_t carry, r01);
 *  - the four ARMS starting points share one exponential vector under
 *    pht_ecs_init_ok, as the exact path's (pht_detmath.h): F at 2b directly,
 *    F F at b, e^{lambda xr} taylor(-lambda a) at a, taylor(lambda x3) at
 *    xr - a; outside that condition the four vectors directly.
 * With the carry, the exponentials e^{lambda_i xr} of a jump's stay test
 * (denominator), of ARMS's xprev = 0 and of the previous jump's categorical
 * are the same values, and so are those of the accepted proposal and the
 * next categorical: the GPU computes each vector once (bit-identical to
 * recomputing it).  The statistics keep the absolute times (z += t - lastt).
 */
template <int NT>
struct CjDens { /* log F_{P_j}(xr - d) + log dexp(d; 1/-S_jj) */
  static constexpr bool kInit4 = true;
  const Par<NT> &P;
  int j;
  double xr, scale, logscale;
  const double *Ex; /* e^{lambda_i xr}: the density at d = 0 */
  double lammax;
  double lastd;
  double Elast[PHT_VEC(NT)]; /* the vector of the most recent evaluation at lastd != 0 */
  __device__ __forceinline__ double operator()(double d) {
    const int n = P.n();
    const double x1 = xr - d;
    double r1;
    if (x1 > 0) {
      double acc = 0.0;
      if (d == 0.0) {
#pragma unroll
        for (int i = 0; i < n; i++) acc = fma(P.V(j, i), Ex[i], acc);
      } else {
#pragma unroll
        for (int i = 0; i < n; i++) Elast[i] = pht_exp_neg(P.evals(i) * x1);
#pragma unroll
        for (int i = 0; i < n; i++) acc = fma(P.V(j, i), Elast[i], acc);
        lastd = d;
      }
      r1 = acc;
    } else {
      r1 = 1;
    }
    return pht_log(r1) + ((-d / scale) - logscale);
  }
  /* the four starting points at once (xinit = {a, b, 2b, xr - a}; the
   * caller has checked 0 < a < b < 2b < xr - a < xr, so every x1 > 0) */
  __device__ __forceinline__ void init4(const double xinit[4], double yv[4]) {
    const int n = P.n();
    const double x3 = xr - xinit[3];
    double acc[4] = {0.0, 0.0, 0.0, 0.0};
    if (pht_ecs_init_ok(lammax, xinit[0], x3)) {
#pragma unroll
      for (int i = 0; i < n; i++) {
        const double F = pht_exp_neg(P.evals(i) * (xr - xinit[2]));
        const double v = P.V(j, i);
        acc[2] = fma(v, F, acc[2]);
        acc[1] = fma(v, F * F, acc[1]);
        acc[0] = fma(v, Ex[i] * pht_exp_taylor(-P.evals(i) * xinit[0]), acc[0]);
        acc[3] = fma(v, pht_exp_taylor(P.evals(i) * x3), acc[3]);
      }
    } else {
#pragma unroll
      for (int k = 0; k < 4; k++) {
        const double x1 = xr - xinit[k];
#pragma unroll
        for (int i = 0; i < n; i++) acc[k] = fma(P.V(j, i), pht_exp_neg(P.evals(i) * x1), acc[k]);
      }
    }
#pragma unroll
    for (int k = 0; k < 4; k++) yv[k] = pht_log(acc[k]) + ((-xinit[k] / scale) - logscale);
  }
};

/* path state of a censored observation between jumps */
template <int NT>
struct CensLane {
  double y, t, lastt;
  double xr;                /* remaining time to y, carried xr <- xr - d (device spec v2) */
  int j, lastj, njump;
  bool haveEx;              /* Ex = e^{lambda_i xr} (from the previous jump's categorical) */
  double Ex[PHT_VEC(NT)];
};

/* start state (LJMA_samplechain, src/Simulate_AbsCTMC_gt_Aslett_DCS.c:315) */
template <int NT, class Sink>
__device__ __forceinline__ void censored_begin(const Par<NT> &P, double y, Lane &ln, Sink &sk, CensLane<NT> &c) {
  const double target = dev_u(ln.r);
  const int B = pistart(P, target, ln.flags);
  sk.start(B);
  c.y = y;
  c.t = 0.0;
  c.lastt = 0.0;
  c.xr = y;
  c.j = B;
  c.lastj = 0;
  c.njump = 0;
  c.haveEx = false;
}

/* one jump of the censored path (the loop body of LJMA_samplechain,
 * src/Simulate_AbsCTMC_gt_Aslett_DCS.c:320-388, with LJMA_condjump_r_ars
 * :184-260); true = the path is complete and recorded */
template <int NT, class Env, class Sink>
__device__ __forceinline__ bool censored_jump(const Par<NT> &P, Lane &ln, Env &env, Sink &sk, CensLane<NT> &c) {
  const int n = P.n();
  bool done = false;
  if (c.njump++ >= kMaxJumps) {
    ln.flags |= kFlagJumpCap;
    done = true;
  } else {
    const double t = c.t;
    const int j = c.j;
    c.lastt = t;
    c.lastj = j;
    const double Sjj = P.S(j, j);
    const double x = c.xr;
    double d;
    CjDens<NT> f{P, j, x, P.scale(j), P.logscale(j), c.Ex, 0.0, -1.0, {}};
    bool armsd = false; /* d from ARMS: its vectors may serve the categorical */
    /* LJMA_condjump_r_ars */
    if (!(x > 0)) { /* t >= y */
      d = dev_rexp(ln.r, 1.0 / -Sjj);
    } else {
      if (!c.haveEx) {
#pragma unroll
        for (int i = 0; i < n; i++) c.Ex[i] = pht_exp_neg(P.evals(i) * x);
      }
      double denom = 0.0;
#pragma unroll
      for (int i = 0; i < n; i++) denom = fma(P.QQ1(j, i), c.Ex[i], denom);
      if (dev_runif(ln.r, 0.0, 1.0) < pht_exp_neg(Sjj * x) / denom) {
        d = x + dev_rexp(ln.r, 1.0 / -Sjj);
      } else {
        f.lammax = lam_max(P);
        double xinit[4];
        xinit[0] = (x) / 1e6;
        xinit[1] = (x) / 3.0;
        xinit[2] = xinit[1] * 2.0;
        xinit[3] = x - xinit[0];
        double xsamp = 0.0;
        const int ainfo = arms(env, xinit, 0.0, x, f, 0.0, xsamp, ln);
        if (ainfo) ln.flags |= (ainfo == 4) ? kFlagArmsCap : kFlagArmsErr;
        d = xsamp;
        armsd = true;
      }
    }
    const int lastj = j;
    const double tn = t + d;
    c.t = tn;
    const double x1 = x - d;
    c.xr = x1;
    c.haveEx = false;
    const double target = dev_u(ln.r);
    int nj;
    if (x1 > 0) { /* tn < y: x1 > 0 needs x > 0 and d < x, i.e. the ARMS branch */
      /* e^{lambda_i x1}: the accepted proposal's (d == lastd) or, for d = 0,
       * the stay test's vector; they become the next jump's Ex */
      if (armsd && d == f.lastd) {
#pragma unroll
        for (int i = 0; i < n; i++) c.Ex[i] = f.Elast[i];
      } else if (!(d == 0.0)) {
#pragma unroll
        for (int i = 0; i < n; i++) c.Ex[i] = pht_exp_neg(P.evals(i) * x1);
      }
      c.haveEx = true;
      double r2 = 0.0;
#pragma unroll
      for (int i = 0; i < n; i++) r2 = fma(P.V(lastj, i), c.Ex[i], r2);
      const int cnt = P.nsuccP(lastj);
      const double tg = target * r2;
      double sofar = 0.0;
      int q = 0, sel = -1;
      for (; q < cnt; q++) {
        const int k = P.succP(lastj, q);
        double r1 = 0.0;
#pragma unroll
        for (int i = 0; i < n; i++) r1 = fma(P.QQ1(k, i), c.Ex[i], r1);
        sofar += r1 * P.P(lastj, k);
        if (!(sofar < tg)) {
          sel = k;
          break;
        }
      }
      if (sel < 0) {
        ln.flags |= kFlagScanEnd;
        sel = (cnt > 0) ? P.succP(lastj, cnt - 1) : 0;
      }
      nj = sel;
    } else {
      const int cnt = P.nsuccPf(lastj);
      double sofar = 0.0;
      int sel = -1;
      for (int q = 0; q < cnt; q++) {
        const int k = P.succPf(lastj, q);
        sofar += P.Pf(lastj, k);
        if (!(sofar < target)) {
          sel = k;
          break;
        }
      }
      if (sel < 0) {
        ln.flags |= kFlagScanEnd;
        sel = (cnt > 0) ? P.succPf(lastj, cnt - 1) : 0;
      }
      nj = sel;
    }
    c.j = nj;
    if (nj == n) {
      done = true;
    } else {
      sk.z(lastj, tn - c.lastt);
      sk.N(lastj, nj);
      ln.njump++;
    }
  }
  if (done) {
    sk.z(c.lastj, c.t - c.lastt);
    sk.pre(c.lastj);
    sk.N(c.lastj, c.lastj);
  }
  return done;
}

/* ================================================================ MHRS */
/*
 * Device specification of LJMA_MHsample_Bladt / LJMA_samplechain_Bladt
 * (src/Simulate_AbsCTMC_eq_Bladt_MHRS.c:63-114,
 * src/Simulate_AbsCTMC_gt_Bladt_MHRS.c:49-121).  The reference's rejection
 * loop is a search for the FIRST successful attempt of each chain (c = 0:
 * the current path, c = 1..mhit: the proposals).  Attempt a of chain c
 * draws from its own Philox stream, tag ((c + 1) << 22) | a, so attempts
 * are independent: any lanes may try them in any order (pht_mhrs.h) and the
 * first success is the same.  An attempt succeeds when the reference
 * accepts it (alive at y for an exact observation, absorbed after y for a
 * censored one) and s[pre] > 0 (the caller's re-draw loop, :65-76).  The
 * observation's own stream (tag 0) gives the mhit acceptance uniforms; the
 * accepted chain's first successful attempt is replayed for the statistics.
 */
constexpr int kMhrsTagShift = 22; /* attempts per chain < 2^22 = kMhrsMaxAtt */
__device__ __forceinline__ uint32_t mhrs_tag(int c, uint32_t att) {
  return ((uint32_t)(c + 1) << kMhrsTagShift) | att;
}
constexpr uint32_t kMhrsUnresolved = 0xffffffffu;
/* first-success record of a chain: (attempt << 8) | pre; min = first */
__device__ __forceinline__ uint32_t mhrs_pack(uint32_t att, int pre) { return (att << 8) | (uint32_t)pre; }

struct NoSink {
  __device__ __forceinline__ void start(int) {}
  __device__ __forceinline__ void z(int, double) {}
  __device__ __forceinline__ void N(int, int) {}
  __device__ __forceinline__ void pre(int) {}
};

/* One attempt of LJMA_samplechain_Bladt's loop (:54-121) on stream r;
 * REC: also record the path's statistics (the accepted attempt). */
template <int NT, bool REC, class Sink>
__device__ __forceinline__ bool mhrs_attempt(const Par<NT> &P, double y, int cens, pht_stream &r, int &pre,
                                             int &flags, int &njump, Sink &sk) {
  const int n = P.n();
  double t = 0.0, lastt = 0.0, sofar = 0.0;
  double target = pht_next_u(&r);
  int B2 = 0;
  while (sofar < target && B2 <= n) sofar += (B2 < n ? P.pi(B2) : 0.0), B2++;
  B2--;
  int j = B2, lastj = j, nj = 0;
  if (REC) sk.start(B2);
  while ((t < y && j < n) || (cens && j < n)) {
    if (nj++ >= kMaxJumps) {
      flags |= kFlagJumpCap;
      t = y;
      break;
    }
    t = t + dev_rexp(r, P.scale(j)) /* = 1.0 / -S_jj, per sweep (pht_layout.h) */;
    target = pht_next_u(&r);
    const int cnt = P.nsuccPf(j);
    sofar = 0.0;
    int sel = n + 1;
    for (int q = 0; q < cnt; q++) {
      const int k = P.succPf(j, q);
      sofar += P.Pf(j, k);
      if (!(sofar < target)) {
        sel = k;
        break;
      }
    }
    j = sel;
    if ((t < y && j < n) || (cens && j < n)) {
      if (REC) {
        sk.z(lastj, t - lastt);
        sk.N(lastj, j);
        njump++;
      }
      lastj = j;
      lastt = t;
    }
  }
  if (REC) {
    sk.z(lastj, cens ? t - lastt : y - lastt);
    sk.N(lastj, lastj);
  }
  pre = lastj;
  return !(t < y) && lastj < n && P.s(lastj) > 0.0;
}

/* attempt (c, att) of observation gid, no recording */
template <int NT>
__device__ __forceinline__ bool mhrs_try(const Par<NT> &P, double y, int cens, uint32_t k0, uint32_t k1,
                                         uint32_t gid, uint32_t sweep, int c, uint32_t att, int &pre) {
  pht_stream r;
  pht_stream_init(&r, k0, k1, gid, mhrs_tag(c, att), sweep);
  int fl = 0, nj = 0;
  NoSink ns;
  return mhrs_attempt<NT, false>(P, y, cens, r, pre, fl, nj, ns);
}

}  // namespace pht
#endif
