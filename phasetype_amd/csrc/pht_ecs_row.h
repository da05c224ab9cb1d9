/*
 * pht_ecs_row.h — the ECS-exact path of ONE observation on a 16-lane DPP row.
 *
 * Why: with few observations per lane (the benchmark's N = 1e6 over 8 GPUs is
 * 125k per GPU, about one per lane) the sweep time is the latency of the
 * longest latent paths: ~50 jumps in sequence, each a serial ARMS chain.  One
 * lane runs that chain at ~12 cycles per VALU instruction (rocprofv3 of a lone
 * wavefront).  Here a row of 16 lanes carries one observation
 * and spreads every step that has parallelism over its lanes:
 *   - spectral index i lives in lane gray^-1(i) (slot = rl ^ (rl >> 1)): a
 *     density evaluation is ONE exponential per lane, and pht_dot16's pairwise
 *     tree is a DPP butterfly (row_mirror, row_half_mirror, quad mirror,
 *     quad xor 1 pair exactly the slots s, s ^ 8, s ^ 4, s ^ 2, s ^ 1 that
 *     pht_dot16 adds), so every lane ends with pht_dot16's value;
 *   - envelope point k lives in lane k (up to kRowCap points): the meets and
 *     the areas of cumulate run one per lane (neighbours by DPP row shifts);
 *     the prefix sum of the areas keeps its sequential order (one DPP step
 *     per point); invert finds its segment with one ballot;
 *   - the four ARMS starting points' sums and logs run side by side.
 * Per-observation control state and the random stream are replicated in the
 * row's 16 lanes, so control flow is uniform within a row; lane 0 alone
 * records the statistics.  Every observation gets exactly the draws,
 * evaluations and arithmetic of the one-lane kernel (pht_ecs_round.h), so
 * results are bit-identical; envelopes beyond kRowCap points continue in the
 * general one-lane ARMS code (arms_step) on a private copy, as there.
 *
 * The host hands the K longest exact observations of a sweep (positions
 * [0, K) of the decreasing-y order) to the row blocks of the ECS launch
 * (ecs_exact_kernel, pht_kernels_impl.h); the rest run one per lane.
 * Reference: LJMA_samplechain_Aslett2 src/Simulate_AbsCTMC_eq_Aslett_ECS.c:205-373,
 * arms src/arms.c:115-846 (via the one-lane restatement in pht_device.h).
 */
#ifndef PHT_ECS_ROW_H
#define PHT_ECS_ROW_H

#include "pht_device.h"
#include "pht_env.h"

namespace pht {

constexpr int kRowW = 16;   /* lanes per observation */
constexpr int kRowCap = 15; /* envelope points held by the row (point k in lane k) */
template <int NT>
constexpr bool row_ok() {
  return NT > 0 && NT <= 2 * kRowW;
}

/* DPP controls (gfx9 family): quad_perm, row shifts, mirrors */
constexpr int kDppQuadRev = 0x1B;  /* quad_perm [3,2,1,0] */
constexpr int kDppQuadX1 = 0xB1;   /* quad_perm [1,0,3,2] */
constexpr int kDppMirror = 0x140;  /* lane l <- lane 15 - l (in the row) */
constexpr int kDppHalfMirror = 0x141; /* lane l <- lane 7 - l (in each half row) */
constexpr int dpp_shl(int s) { return 0x100 + s; } /* lane l <- lane l + s */
constexpr int dpp_shr(int s) { return 0x110 + s; } /* lane l <- lane l - s */

/* A cross-lane read must run where the whole row is active: DPP and
 * ds_bpermute read a source lane's register whether or not that lane took
 * part, so a read the compiler sank into a lane-divergent branch would see
 * stale values (it did: a select turned into a branch around the row
 * scan's shifts).  pin() materialises a value at its program point (an
 * empty volatile asm: not sunk, not reordered past other volatile asm);
 * dpp_pd pins the shifts whose values are used only under lane-divergent
 * conditions (the reductions and row_get feed unconditional arithmetic or
 * row-uniform branches, and stay unpinned so their chains interleave). */
template <class T>
__device__ __forceinline__ T pin(T v) {
  asm volatile("" : "+v"(v));
  return v;
}

/* out-of-row sources read 0 (bound_ctrl off, old = 0); every caller selects
 * such lanes away */
template <int CTRL>
__device__ __forceinline__ int dpp_i(int v) {
  return __builtin_amdgcn_update_dpp(0, v, CTRL, 0xF, 0xF, false);
}
template <int CTRL>
__device__ __forceinline__ double dpp_d(double v) {
  const unsigned long long u = (unsigned long long)__double_as_longlong(v);
  const unsigned lo = (unsigned)dpp_i<CTRL>((int)(unsigned)u);
  const unsigned hi = (unsigned)dpp_i<CTRL>((int)(unsigned)(u >> 32));
  return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}
/* a row shift whose value is used only under lane-divergent conditions */
template <int CTRL>
__device__ __forceinline__ double dpp_pd(double v) {
  return pin(dpp_d<CTRL>(v));
}

/* value of lane k of the row (k row-uniform) */
__device__ __forceinline__ double row_get(double v, int k) { return __shfl(v, k, kRowW); }
/* the row's 16 bits of a wavefront ballot */
__device__ __forceinline__ unsigned row_ballot(bool p) {
  const unsigned long long m = __ballot(p);
  return (unsigned)(m >> (threadIdx.x & 48u)) & 0xFFFFu;
}

/* one level of pht_dot16's tree: slots r and r + s (r < s) are added when
 * r + s < n; both lanes of the pair compute the same value */
__device__ __forceinline__ double row_level(double v, double o, int slot, int s, int n) {
  const bool low = (slot & s) == 0;
  const bool has = (slot & (s - 1)) + s < n;
  return has ? v + o : (low ? v : o);
}
/* pht_dot16 over the row (n <= 16): v = this lane's slot product (0 beyond
 * n); every lane returns the sum */
__device__ __forceinline__ double row_sum16(double v, int slot, int n) {
  v = row_level(v, dpp_d<kDppMirror>(v), slot, 8, n);
  v = row_level(v, dpp_d<kDppHalfMirror>(v), slot, 4, n);
  v = row_level(v, dpp_d<kDppQuadRev>(v), slot, 2, n);
  v = row_level(v, dpp_d<kDppQuadX1>(v), slot, 1, n);
  return v;
}

/* a lane's spectral values: index slot, and slot + 16 when n > 16
 * (pht_dot16's slot r holds c_r e_r + c_{r+16} e_{r+16}) */
template <int NT>
struct RowV {
  static constexpr int H = (NT > kRowW) ? 2 : 1;
  double v[H];
};

/* lane-constant row data */
template <int NT>
struct RowId {
  static constexpr int H = RowV<NT>::H;
  int rl;        /* lane in the row = envelope position */
  int slot;      /* pht_dot16 slot of this lane (gray code of rl) */
  int ix[H];     /* spectral index slot + 16 h, or 0 beyond n (parameter-block index) */
  bool sv[H];    /* slot + 16 h < n */
  bool lead;     /* rl == 0: records the statistics */
  double lam[H]; /* evals(slot + 16 h) (0 beyond n) */
  double lammax;
};
template <int NT, class Par>
__device__ __forceinline__ RowId<NT> row_id(const Par &P, int rl) {
  RowId<NT> id;
  id.rl = rl;
  id.slot = rl ^ (rl >> 1);
  id.lead = (rl == 0);
#pragma unroll
  for (int h = 0; h < RowId<NT>::H; h++) {
    const int i = id.slot + kRowW * h;
    id.sv[h] = i < NT;
    id.ix[h] = id.sv[h] ? i : 0;
    id.lam[h] = id.sv[h] ? P.evals(id.ix[h]) : 0.0;
  }
  id.lammax = lam_max(P);
  return id;
}

/* the lane's slots of e^{lambda_i x} */
template <int NT>
__device__ __forceinline__ RowV<NT> rv_exp(const RowId<NT> &id, double x) {
  RowV<NT> r;
#pragma unroll
  for (int h = 0; h < RowV<NT>::H; h++) r.v[h] = id.sv[h] ? pht_exp_neg(id.lam[h] * x) : 0.0;
  return r;
}
/* the lane's slots of E0 at an observation's first sojourn (ecs_first_E0's
 * rule: (F F) F from the starting points' vector F, or directly) */
template <int NT>
__device__ __forceinline__ RowV<NT> rv_first_E0(const RowId<NT> &id, double y_t) {
  const double a = (y_t) / 1e6, b2 = ((y_t) / 3.0) * 2.0;
  if (pht_ecs_init_ok(id.lammax, a, y_t - (y_t - a))) {
    RowV<NT> r = rv_exp(id, y_t - b2);
#pragma unroll
    for (int h = 0; h < RowV<NT>::H; h++) r.v[h] = pht_ecs_e0_cube(r.v[h]);
    return r;
  }
  return rv_exp(id, y_t);
}
/* the lane's slots of a coefficient row c(i) */
template <int NT, class Cf>
__device__ __forceinline__ RowV<NT> rv_coef(const RowId<NT> &id, const Cf &cf) {
  RowV<NT> r;
#pragma unroll
  for (int h = 0; h < RowV<NT>::H; h++) r.v[h] = id.sv[h] ? cf(id.ix[h]) : 0.0;
  return r;
}
/* pht_dot16(c, e) over the row: every lane returns it */
template <int NT>
__device__ __forceinline__ double rv_dot(const RowId<NT> &id, const RowV<NT> &c, const RowV<NT> &e) {
  double p = id.sv[0] ? c.v[0] * e.v[0] : 0.0;
  if constexpr (RowV<NT>::H > 1) p = id.sv[1] ? fma(c.v[1], e.v[1], p) : p;
  return row_sum16(p, id.slot, NT);
}

/* per-observation state (replicated; E0 holds this lane's slots) */
template <int NT>
struct RowObs {
  double yt;
  int j, njump;
  bool haveE0, haveDen;
  bool fold; /* the absorb test after a jump runs at the start of the next round (row_round) */
  double den;
  RowV<NT> E0; /* e^{lambda_i yt} */
};

/* the row's envelope: point rl (x, y), count and ymax (replicated) */
struct RowEnv {
  double x, y;
  int cnt;
  double ymax;
};

/* EcsDens on a row: log(sum_i W[j,i] e^{lambda_i (y_t - d)}) + S_jj d */
template <int NT>
struct RowDens {
  static constexpr int H = RowV<NT>::H;
  const RowId<NT> &id;
  int j;
  double y_t, Sjj;
  RowV<NT> w;  /* W[j, i] */
  RowV<NT> E0; /* e^{lambda_i y_t} */
  RowV<NT> El; /* the most recent evaluation */
  double lastd;
  const PHT_LDS double *Wm; /* the state's W moments (stride NT) */
  __device__ __forceinline__ double sum(const RowV<NT> &e) const { return rv_dot(id, w, e); }
  __device__ __forceinline__ double operator()(double d) {
    const double x = y_t - d;
    if (d == 0.0) El = E0;
    else El = rv_exp(id, x);
    const double acc = sum(El);
    lastd = d;
    return pht_log(acc) + Sjj * d;
  }
  /* EcsDens::init4: the four sums (every lane gets all four) */
  __device__ __forceinline__ void init4(const double xinit[4], double acc[4]) {
    const double x3 = y_t - xinit[3];
    if (pht_ecs_init_ok(id.lammax, xinit[0], x3)) {
      const RowV<NT> F = rv_exp(id, y_t - xinit[2]);
      RowV<NT> T1, T0;
#pragma unroll
      for (int h = 0; h < H; h++) {
        T1.v[h] = F.v[h] * F.v[h];
        T0.v[h] = E0.v[h] * pht_exp_taylor(-id.lam[h] * xinit[0]);
      }
      acc[2] = sum(F);
      acc[1] = sum(T1);
      acc[0] = sum(T0);
      /* point y_t - a: the state's W-moment polynomial (pht_wmoments) */
      {
        const PHT_LDS double *m = Wm;
        double q = m[5 * NT];
        q = fma(q, x3, m[4 * NT]);
        q = fma(q, x3, m[3 * NT]);
        q = fma(q, x3, m[2 * NT]);
        q = fma(q, x3, m[1 * NT]);
        acc[3] = fma(q, x3, m[0]);
      }
    } else {
#pragma unroll
      for (int k = 0; k < 4; k++) {
        El = rv_exp(id, y_t - xinit[k]);
        acc[k] = sum(El);
      }
      lastd = xinit[3];
    }
  }
};

/* round_meets on the row: every intersection point (even positions) at once */
__device__ __forceinline__ void row_meets(RowEnv &e, int rl) {
  const int last = e.cnt - 1;
  const int K = rl;
  /* slope of the segment from this (odd) point to the next odd point */
  const double xb = dpp_pd<dpp_shl(2)>(e.x), yb = dpp_pd<dpp_shl(2)>(e.y);
  const double q = PHT_DIV((yb - e.y), (xb - e.x));
  const double sb = (e.y == yb && q == 0.0) ? ((e.x - xb < 0.0) ? -0.0 : 0.0) : q;
  const double glv = dpp_pd<dpp_shr(3)>(q), grlv = dpp_pd<dpp_shr(1)>(q), grv = dpp_pd<dpp_shl(1)>(sb);
  const double xm1 = dpp_pd<dpp_shr(1)>(e.x), ym1 = dpp_pd<dpp_shr(1)>(e.y);
  const double xp1 = dpp_pd<dpp_shl(1)>(e.x), yp1 = dpp_pd<dpp_shl(1)>(e.y);
  const bool il = (K >= 3), ir = (K + 3 <= last), irl = (K >= 1 && K + 1 <= last);
  const double xk = e.x, yk = e.y;
  double gl = il ? glv : 0.0, gr = ir ? grv : 0.0, grl = irl ? grlv : 0.0, dl = 0.0, dr = 0.0;
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
  const bool active = ((K & 1) == 0) && (K <= last);
  e.x = active ? nx : e.x;
  e.y = active ? ny : e.y;
}

/* arms_cumulate's ymax: a scan from position 0 with a strict > keeps the
 * first maximum, skips NaN at positions >= 1 and sticks to a NaN at 0.  As a
 * total order on (class, value, position) it reduces in any pairing. */
struct RowMax {
  double v;
  int k;  /* position, or >= 64 for points beyond cnt */
};
__device__ __forceinline__ int rowmax_cls(const RowMax &a) {
  if (a.k >= 64) return 0;
  if (a.v != a.v) return a.k == 0 ? 3 : 1;
  return 2;
}
__device__ __forceinline__ bool rowmax_better(const RowMax &a, const RowMax &b) {
  const int ca = rowmax_cls(a), cb = rowmax_cls(b);
  if (ca != cb) return ca > cb;
  if (ca == 2 && a.v != b.v) return a.v > b.v;
  return a.k < b.k;
}
template <int CTRL>
__device__ __forceinline__ RowMax rowmax_step(RowMax m) {
  RowMax o;
  o.v = dpp_d<CTRL>(m.v);
  o.k = dpp_i<CTRL>(m.k);
  return rowmax_better(o, m) ? o : m;
}

/* round_cumulate on the row: ymax, then this lane's area (segment rl-1 ->
 * rl) and the prefix sum in position order; returns cum at position rl
 * (and ey = expshift(y, ymax) there, which invert reuses) */
__device__ __forceinline__ double row_cumulate(RowEnv &e, int rl, double &ey) {
  /* fmax reduction (NaN ignored, as the scan ignores NaN at positions >=
   * 1); it can differ from the scan only for a NaN at position 0 or a zero
   * maximum (+0 against -0): those rows take the exact order reduction */
  double mx = (rl < e.cnt) ? e.y : -INFINITY;
  mx = fmax(mx, dpp_d<kDppMirror>(mx));
  mx = fmax(mx, dpp_d<kDppHalfMirror>(mx));
  mx = fmax(mx, dpp_d<kDppQuadRev>(mx));
  mx = fmax(mx, dpp_d<kDppQuadX1>(mx));
  const bool nan0 = row_ballot(rl == 0 && e.y != e.y) != 0u;
  if (nan0 || mx == 0.0) {
    RowMax m;
    m.v = e.y;
    m.k = (rl < e.cnt) ? rl : 64 + rl;
    m = rowmax_step<kDppMirror>(m);
    m = rowmax_step<kDppHalfMirror>(m);
    m = rowmax_step<kDppQuadRev>(m);
    m = rowmax_step<kDppQuadX1>(m);
    mx = m.v;
  }
  const double ymax = mx;
  e.ymax = ymax;
  const double eyk = expshift_le(e.y, ymax); /* (lanes beyond cnt: never read) */
  ey = eyk;
  const double xp = dpp_pd<dpp_shr(1)>(e.x), yp = dpp_pd<dpp_shr(1)>(e.y), eyp = dpp_pd<dpp_shr(1)>(eyk);
  const double xk = e.x, yk = e.y;
  const double lin = 0.5 * (eyk + eyp) * (xk - xp);
  const double ex = (PHT_DIV((eyk - eyp), (yk - yp))) * (xk - xp);
  const double a = (xp == xk) ? 0. : ((fabs(yk - yp) < kYEps) ? lin : ex);
  /* cum_k = (((0 + a_1) + a_2) + ...) + a_k in this order: lane k takes
   * a_{k-s} by one row shift per s (independent moves, issued together) and
   * adds them from s = k - 1 down to 0; the dependent chain is the adds */
  double cum = 0.;
#ifdef PHT_ROW_OLDSCAN
#pragma unroll
  for (int t = 1; t < kRowCap; t++) {
    if (!__any(t < e.cnt)) break;
    const double v = dpp_d<dpp_shr(1)>(cum);
    cum = (rl == t) ? v + a : cum;
  }
  return cum;
#endif
  /* (an invalid step adds +0 to cum = +0: cum is never -0, so the sum is
   * the select's value) */
#define PHT_ROW_CUM(S)                           \
  {                                              \
    const double t_ = dpp_pd<dpp_shr(S)>(a);     \
    cum = cum + ((rl - (S) >= 1) ? t_ : 0.0);    \
  }
  PHT_ROW_CUM(14); PHT_ROW_CUM(13); PHT_ROW_CUM(12); PHT_ROW_CUM(11); PHT_ROW_CUM(10);
  PHT_ROW_CUM(9); PHT_ROW_CUM(8); PHT_ROW_CUM(7); PHT_ROW_CUM(6); PHT_ROW_CUM(5);
  PHT_ROW_CUM(4); PHT_ROW_CUM(3); PHT_ROW_CUM(2); PHT_ROW_CUM(1);
#undef PHT_ROW_CUM
  cum = (rl >= 1) ? cum + a : cum;
  return cum;
}

/* round_invert on the row (cum, ey: this lane's cumulative area and
 * expshift(y, ymax) from row_cumulate; the same values round_invert
 * recomputes) */
__device__ __forceinline__ void row_invert(const RowEnv &e, double cum, double ey, int rl, double prob, WPt &p) {
  const int last = e.cnt - 1;
  const double clast = row_get(cum, last);
  const double u = prob * clast;
  /* q moves down from last while cum[q-1] > u */
  const unsigned stop = row_ballot(rl >= 1 && rl <= last - 1 && !(cum > u));
  const int q = stop ? (31 - __builtin_clz(stop)) + 1 : 1;
  p.pr = q;
  const double cr = row_get(cum, q), cl = row_get(cum, q - 1);
  const double xl = row_get(e.x, q - 1), xr = row_get(e.x, q);
  const double yr = row_get(e.y, q), yl = row_get(e.y, q - 1);
  const double eyr = row_get(ey, q), eyl = row_get(ey, q - 1);
  const double prop = PHT_DIV((u - cl), (cr - cl));
  if (xl == xr) {
    p.x = xr; p.y = yr; p.ey = eyr;
    return;
  }
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

/* round_insert on the row (cnt + 2 <= kRowCap) */
template <int NT>
__device__ __forceinline__ void row_insert(RowEnv &e, const ArmsPend &pd, RowDens<NT> &f, Lane &ln, int rl) {
  const int pr = pd.pr, last = e.cnt - 1;
  const double xs = dpp_pd<dpp_shr(2)>(e.x), ys = dpp_pd<dpp_shr(2)>(e.y);
  const bool mv = (rl >= 2) && (rl - 2 >= pr) && (rl - 2 <= last);
  e.x = mv ? xs : e.x;
  e.y = mv ? ys : e.y;
  e.cnt += 2;
  const int qi = ((pr - 1) & 1) ? pr + 1 : pr;
  e.x = (rl == qi) ? pd.px : e.x;
  e.y = (rl == qi) ? pd.py : e.y;
  const int ql = (qi >= 2) ? qi - 2 : qi - 1;
  const int qr = (qi + 2 <= e.cnt - 1) ? qi + 2 : qi + 1;
  const double xl = row_get(e.x, ql), xr = row_get(e.x, qr);
  bool adj = false;
  double xn = 0.0;
  if (pd.px < (1. - kXEps) * xl + kXEps * xr) {
    xn = (1. - kXEps) * xl + kXEps * xr;
    adj = true;
  } else if (pd.px > kXEps * xl + (1. - kXEps) * xr) {
    xn = kXEps * xl + (1. - kXEps) * xr;
    adj = true;
  }
  if (adj) {
    const double yn = f(xn);
    ln.neval++;
    e.x = (rl == qi) ? xn : e.x;
    e.y = (rl == qi) ? yn : e.y;
  }
}

/* the envelope segment round_metropolis reads (xprev's): ql with
 * X(ql) <= xprev < X(ql + 1) scanning from 0, and its two points; read as
 * soon as the round's envelope is final (after the meets) */
struct RowMetroSeg {
  double xql, yql, xqr, yqr;
};
__device__ __forceinline__ RowMetroSeg row_metro_seg(const RowEnv &e, int rl, double xprev) {
  /* ql: while (X(ql + 1) < xprev) ql++ */
  const unsigned stop = row_ballot(rl >= 1 && !(e.x < xprev));
  const int ql = stop ? __builtin_ctz(stop) - 1 : kRowW - 2;
  const int qr = ql + 1;
  RowMetroSeg m;
  m.xql = row_get(e.x, ql);
  m.yql = row_get(e.y, ql);
  m.xqr = row_get(e.x, qr);
  m.yqr = row_get(e.y, qr);
  return m;
}

/* round_metropolis on the row */
__device__ __forceinline__ double row_metropolis(const RowMetroSeg &m, const WPt &p, double ynew, double xprev,
                                                 double yprev, Lane &ln) {
  double w = PHT_DIV((xprev - m.xql), (m.xqr - m.xql));
  double zold = m.yql + w * (m.yqr - m.yql);
  double znew = p.y;
  if (yprev < zold) zold = yprev;
  if (ynew < znew) znew = ynew;
  w = ynew - znew - yprev + zold;
  if (w > 0.0) w = 0.0;
  w = (w > -kYCeil) ? pht_exp_core(w) : 0.0;
  const double um = dev_u(ln.r);
  return (um > w) ? xprev : p.x;
}

/* absorb test (ecs_try_absorb); true = path complete and recorded */
template <int NT, class Sink>
__device__ __forceinline__ bool row_try_absorb(const Par<NT> &P, const RowId<NT> &id, Lane &ln, Sink &sk,
                                               RowObs<NT> &st) {
  const int j = st.j;
  bool fin = false;
  if (st.njump >= kMaxJumps) {
    ln.flags |= kFlagJumpCap;
    fin = true;
  } else if (P.s(j) > 0.0) {
    const double y_t = st.yt;
    const double U = dev_u(ln.r);
    if (!st.haveE0) { /* the observation's first sojourn */
      st.E0 = rv_first_E0(id, y_t);
      st.haveE0 = true;
      st.haveDen = false;
    }
    const double den =
        st.haveDen ? st.den : rv_dot(id, rv_coef(id, [&](int i) { return P.QQs(j, i); }), st.E0);
    fin = ecs_absorbs(U, P.S(j, j), y_t, P.logs(j), den);
  }
  if (fin && id.lead) {
    sk.N(j, j);
    sk.z(j, st.yt);
    sk.pre(j);
  }
  return fin;
}

/* the first kRowSuccPre successors of state j (moveMass' candidates), read
 * at the start of the round so the loads are off the finish's chain */
constexpr int kRowSuccPre = 2;
template <int NT>
struct RowSucc {
  int cnt;
  int k[kRowSuccPre];
  double p[kRowSuccPre];      /* P[j,k] */
  RowV<NT> qq[kRowSuccPre];   /* QQs[k, i] */
};
template <int NT>
__device__ __forceinline__ RowSucc<NT> row_succ(const Par<NT> &P, const RowId<NT> &id, int j) {
  RowSucc<NT> r;
  r.cnt = P.nsuccP(j);
#pragma unroll
  for (int q = 0; q < kRowSuccPre; q++) {
    const int k = P.succP(j, (q < NT) ? q : 0);
    r.k[q] = k;
    const int kc = (q < r.cnt) ? k : 0; /* entries beyond cnt are not read */
    r.p[q] = P.P(j, kc);
    r.qq[q] = rv_coef(id, [&](int i) { return P.QQs(kc, i); });
  }
  return r;
}

/* ecs_jump_finish: moveMass + categorical + statistics */
template <int NT, class Sink>
__device__ __forceinline__ void row_jump_finish(const Par<NT> &P, const RowId<NT> &id, Lane &ln, Sink &sk,
                                                RowObs<NT> &st, const RowDens<NT> &f, double xsamp, int ainfo,
                                                const RowSucc<NT> &su) {
  const int j = st.j;
  const double y_t = st.yt;
  if (ainfo) ln.flags |= (ainfo == 4) ? kFlagArmsCap : kFlagArmsErr;
  const double d = xsamp;
  const double x = y_t - d;
  if (d == f.lastd) {
    st.E0 = f.El;
  } else if (d == 0.0) {
    /* E0 already holds e^{lambda y_t} */
  } else {
    st.E0 = rv_exp(id, x);
  }
  st.yt = x;
  st.haveE0 = true;
  const int cnt = su.cnt;
  double w[NT], accs[NT];
  double sum = 0.0;
#pragma unroll
  for (int q = 0; q < NT; q++) {
    if (q < cnt) {
      const int k = (q < kRowSuccPre) ? su.k[q] : P.succP(j, q);
      RowV<NT> qq;
      if (q < kRowSuccPre) qq = su.qq[q];
      else qq = rv_coef(id, [&](int i) { return P.QQs(k, i); });
      const double pjk = (q < kRowSuccPre) ? su.p[q] : P.P(j, k);
      accs[q] = rv_dot(id, qq, st.E0);
      w[q] = pjk * accs[q];
      sum += w[q];
    }
  }
  const double target = dev_u(ln.r) * sum;
  int nj;
  {
    double sofar = 0.0;
    int sel = -1;
#pragma unroll
    for (int q = 0; q < NT; q++) {
      if (q < cnt && sel < 0) {
        sofar += w[q];
        if (!(sofar < target)) sel = q;
      }
    }
    if (sel < 0) {
      ln.flags |= kFlagScanEnd;
      sel = cnt - 1;
    }
    nj = (cnt > 0) ? ((sel < kRowSuccPre) ? su.k[sel < kRowSuccPre ? sel : 0] : P.succP(j, sel)) : 0;
    double dsel = 0.0;
#pragma unroll
    for (int q = 0; q < NT; q++) dsel = (q == sel) ? accs[q] : dsel;
    st.den = dsel;
    st.haveDen = (cnt > 0);
    st.fold = st.haveDen;
  }
  if (id.lead) {
    sk.z(j, d);
    sk.N(j, nj);
  }
  ln.njump++;
  st.njump++;
  st.j = nj;
}

/*
 * One ARMS round of a row (ecs_round).  start: begin a jump at st.j; pend:
 * continue one.  bigm: the jump's envelope outgrew kRowCap and continues in
 * the general one-lane code on the private copy benv (every lane of the row
 * runs it, replicated).
 */
template <int NT, class Sink>
__device__ __forceinline__ bool row_round(const Par<NT> &P, const RowId<NT> &id, Lane &ln, RowEnv &ev,
                                          EnvPrivateBig &benv, Sink &sk, RowObs<NT> &st, bool start, bool &pend,
                                          bool &bigm, ArmsPend &pd) {
  const int rl = id.rl;
  const double y_t = st.yt;
  if (start && !st.haveE0) { /* s_j = 0 at the first sojourn */
    st.E0 = rv_first_E0(id, y_t);
    st.haveE0 = true;
    st.haveDen = false;
  }
  const int j = st.j;
  const RowSucc<NT> su = row_succ<NT>(P, id, j);
  RowDens<NT> f{id, j, y_t, P.S(j, j), rv_coef(id, [&](int i) { return P.W(j, i); }), st.E0, {}, -1.0, P.Wm(j)};
  PHT_STAMP(ln, 1);
  double xsamp = 0.0;
  int ainfo = 0;
  bool fin = false;
  /* ---- starting rows: initial envelope (4 evaluations side by side).
   * A path that has just jumped (st.fold) first takes its absorb test
   * (ecs_try_absorb: same draw, same arithmetic); it is computed alongside
   * the envelope, which is dropped when the path ends here. */
  if (start) {
    const bool test = st.fold;
    st.fold = false;
    const bool capj = test && st.njump >= kMaxJumps;
    const bool draw = test && !capj && P.s(j) > 0.0;
    double U = 1.0;
    if (draw) U = dev_u(ln.r);
    const bool absorbs = ecs_absorbs(U, P.S(j, j), y_t, P.logs(j), st.den);
    double xinit[4];
    xinit[0] = (y_t) / 1e6;
    xinit[1] = (y_t) / 3.0;
    xinit[2] = xinit[1] * 2.0;
    xinit[3] = y_t - xinit[0];
    const bool e1003 = (xinit[0] <= 0.0) || (xinit[3] >= y_t);
    const bool e1004 = !e1003 && (xinit[1] <= xinit[0] || xinit[2] <= xinit[1] || xinit[3] <= xinit[2]);
    double acc[4];
    f.init4(xinit, acc);
    /* lanes 1, 3, 5, 7: the starting points; 0 and 8: the interval ends */
    const int k = (rl >> 1) & 3;
    const double xk = (k == 0) ? xinit[0] : (k == 1) ? xinit[1] : (k == 2) ? xinit[2] : xinit[3];
    const double ak = (k == 0) ? acc[0] : (k == 1) ? acc[1] : (k == 2) ? acc[2] : acc[3];
    const double yk = pht_log(ak) + f.Sjj * xk;
    if (capj || (draw && absorbs)) { /* the path is complete */
      if (capj) ln.flags |= kFlagJumpCap;
      if (id.lead) {
        sk.N(j, j);
        sk.z(j, y_t);
        sk.pre(j);
      }
      return true;
    }
    if (e1003) {
      ainfo = 1003;
      fin = true;
    } else if (e1004) {
      ainfo = 1004;
      fin = true;
    } else {
      ln.neval += 4;
      ev.cnt = 9;
      const bool odd = (rl & 1) && rl < 8;
      ev.x = (rl == 0) ? 0.0 : (odd ? xk : ((rl == 8) ? y_t : ev.x));
      ev.y = odd ? yk : ev.y;
    }
  }
  PHT_STAMP(ln, 2);
  /* ---- pending rows: the update ending the rejected iteration */
  if (pend && !bigm && ev.cnt + 2 > kRowCap) {
    /* hand the envelope to the general code (private copy in every lane) */
    benv.cnt = ev.cnt;
    benv.ymax = ev.ymax;
    for (int k = 0; k < ev.cnt; k++) {
      benv.sX(k, row_get(ev.x, k));
      benv.sY(k, row_get(ev.y, k));
    }
    bigm = true;
  }
  const bool big = pend && bigm;
  if (pend && !big) row_insert<NT>(ev, pd, f, ln, rl);
  PHT_STAMP(ln, 3);
  const bool arm = (start && !fin) || (pend && !big);
  double cum = 0.0, eyv = 0.0;
  RowMetroSeg mseg{0.0, 0.0, 0.0, 0.0};
  if (arm) {
    row_meets(ev, rl);
#ifndef PHT_ROW_OLDMETRO
    mseg = row_metro_seg(ev, rl, 0.0);
#endif
  }
  PHT_STAMP(ln, 4);
  if (arm) cum = row_cumulate(ev, rl, eyv);
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
  bool acc = false;
  const bool itr = arm && !fin;
  WPt q;
  double yv = 0.0, ynew = 0.0;
  if (itr) {
    const double pu = dev_u(ln.r);
    row_invert(ev, cum, eyv, rl, pu, q);
    const double u = dev_u(ln.r) * q.ey;
    yv = logshift(u, ev.ymax);
  }
  PHT_STAMP(ln, 7);
  if (itr) {
    ynew = f(q.x);
    ln.neval++;
  }
  PHT_STAMP(ln, 8);
  if (itr) {
    if (yv >= ynew) {
      pd.px = q.x; pd.py = ynew; pd.pey = expshift(ynew, ev.ymax); pd.pr = q.pr;
      pd.it++;
      pend = true;
    } else {
#ifdef PHT_ROW_OLDMETRO
      mseg = row_metro_seg(ev, rl, 0.0);
#endif
      xsamp = row_metropolis(mseg, q, ynew, 0.0, pd.yprev, ln);
      acc = true;
    }
  }
  PHT_STAMP(ln, 9);
  /* ---- rare: envelopes beyond kRowCap, one-lane code on the private copy */
  if (big) {
    /* every spectral index from the lane holding it: index i is slot i % 16
     * of lane gray^-1(i % 16), half i / 16 */
    double E0f[NT];
#pragma unroll
    for (int i = 0; i < NT; i++) {
      const int r = i % kRowW;
      E0f[i] = row_get(st.E0.v[i / kRowW], r ^ (r >> 1) ^ (r >> 2) ^ (r >> 3));
    }
    EcsDens<NT> f1{P, j, y_t, P.S(j, j), E0f, true, -1.0, {}, 0.0, {}};
    f1.load(id.lammax);
    const int rc = arms_step(benv, f1, pd, 0.0, xsamp, ln);
    sk.arms_diag(id.lead, id.lead); /* the private copy, once per row */
    if (rc != 1) {
      ainfo = rc;
      acc = true;
      bigm = false;
      f.lastd = f1.lastd;
#pragma unroll
      for (int h = 0; h < RowV<NT>::H; h++) {
        double v = 0.0;
#pragma unroll
        for (int i = 0; i < NT; i++) v = (i == id.slot + kRowW * h) ? f1.Elast[i] : v;
        f.El.v[h] = v;
      }
    }
  }
  PHT_STAMP(ln, 10);
  if (acc || fin) {
    pend = false;
    row_jump_finish<NT>(P, id, ln, sk, st, f, xsamp, ainfo, su);
  }
  PHT_STAMP(ln, 11);
  return false;
}

}  // namespace pht
#endif
