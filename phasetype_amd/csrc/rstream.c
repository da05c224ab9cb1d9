/*
 * rstream.c — restatement of R's default random stream for standalone runs.
 * See rstream.h for scope and the self-check values.  Algorithms follow the
 * published sources of R's nmath (RNG.c MT19937 + RNG_Init scrambling,
 * sexp.c, snorm.c INVERSION, qnorm.c AS241, rgamma.c GD/GS, runif.c,
 * rexp.c, dexp.c); R itself is not under /root/reference.
 */
#include "rstream.h"

#include <math.h>

#define MT_N 624
#define MT_M 397
#define MATRIX_A 0x9908b0dfU
#define UPPER_MASK 0x80000000U
#define LOWER_MASK 0x7fffffffU

static const double i2_32m1 = 2.328306437080797e-10; /* 1/(2^32 - 1) */

void pht_rs_set_seed(pht_rstream *rs, uint32_t seed) {
  /* RNG_Init: 50 LCG scrambles, then fill .Random.seed[0..624]; [0] is mti
   * and is immediately reset to 624 by FixupSeeds(initial=1). */
  for (int j = 0; j < 50; j++) seed = 69069U * seed + 1U;
  seed = 69069U * seed + 1U; /* .Random.seed[0] (dummy[0]) */
  for (int j = 0; j < MT_N; j++) {
    seed = 69069U * seed + 1U;
    rs->mt[j] = seed;
  }
  rs->mti = MT_N;
  rs->nword = 0;
}

static double mt_genrand(pht_rstream *rs) {
  static const uint32_t mag01[2] = {0x0U, MATRIX_A};
  uint32_t *mt = rs->mt;
  uint32_t y;
  if (rs->mti >= MT_N) {
    int kk;
    for (kk = 0; kk < MT_N - MT_M; kk++) {
      y = (mt[kk] & UPPER_MASK) | (mt[kk + 1] & LOWER_MASK);
      mt[kk] = mt[kk + MT_M] ^ (y >> 1) ^ mag01[y & 0x1U];
    }
    for (; kk < MT_N - 1; kk++) {
      y = (mt[kk] & UPPER_MASK) | (mt[kk + 1] & LOWER_MASK);
      mt[kk] = mt[kk + (MT_M - MT_N)] ^ (y >> 1) ^ mag01[y & 0x1U];
    }
    y = (mt[MT_N - 1] & UPPER_MASK) | (mt[0] & LOWER_MASK);
    mt[MT_N - 1] = mt[MT_M - 1] ^ (y >> 1) ^ mag01[y & 0x1U];
    rs->mti = 0;
  }
  y = mt[rs->mti++];
  rs->nword++;
  y ^= (y >> 11);
  y ^= (y << 7) & 0x9d2c5680U;
  y ^= (y << 15) & 0xefc60000U;
  y ^= (y >> 18);
  return (double)y * 2.3283064365386963e-10;
}

double pht_rs_unif_rand(pht_rstream *rs) {
  double x = mt_genrand(rs);
  if (x <= 0.0) return 0.5 * i2_32m1;
  if ((1.0 - x) <= 0.0) return 1.0 - 0.5 * i2_32m1;
  return x;
}

double pht_rs_exp_rand(pht_rstream *rs) {
  /* q[k-1] = sum_{i=1..k} ln(2)^i / i!  (literal table as in sexp.c) */
  static const double q[] = {
      0.6931471805599453, 0.9333736875190459, 0.9888777961838675,
      0.9984959252914960040, 0.9998292811061389, 0.9999833164100727,
      0.9999985691438767, 0.9999998906925558, 0.9999999924734159,
      0.9999999995283275, 0.9999999999728814, 0.9999999999985598,
      0.9999999999999289, 0.9999999999999968, 0.9999999999999999,
      1.0000000000000000};
  double a = 0.;
  double u = pht_rs_unif_rand(rs);
  while (u <= 0. || u >= 1.) u = pht_rs_unif_rand(rs);
  for (;;) {
    u += u;
    if (u > 1.) break;
    a += q[0];
  }
  u -= 1.;
  if (u <= q[0]) return a + u;
  int i = 0;
  double ustar = pht_rs_unif_rand(rs), umin = ustar;
  do {
    ustar = pht_rs_unif_rand(rs);
    if (umin > ustar) umin = ustar;
    i++;
  } while (u > q[i]);
  return a + umin * q[0];
}

double pht_rs_qnorm(double p) {
  /* qnorm5(p, 0, 1, lower_tail=TRUE, log_p=FALSE), Wichura AS241 */
  if (isnan(p)) return p;
  if (p <= 0.0) return p == 0.0 ? -INFINITY : NAN;
  if (p >= 1.0) return p == 1.0 ? INFINITY : NAN;
  double q = p - 0.5, r, val;
  if (fabs(q) <= .425) {
    r = .180625 - q * q;
    val = q * (((((((r * 2509.0809287301226727 + 33430.575583588128105) * r +
                    67265.770927008700853) * r + 45921.953931549871457) * r +
                  13731.693765509461125) * r + 1971.5909503065514427) * r +
                133.14166789178437745) * r + 3.387132872796366608) /
          (((((((r * 5226.495278852545925 + 28729.085735721942674) * r +
                39307.89580009271061) * r + 21213.794301586595867) * r +
              5394.1960214247511077) * r + 687.1870074920579083) * r +
            42.313330701600911252) * r + 1.);
    return val;
  }
  double lp = log((q > 0) ? (0.5 - p + 0.5) : p);
  r = sqrt(-lp);
  if (r <= 5.) {
    r += -1.6;
    val = (((((((r * 7.7454501427834140764e-4 + .0227238449892691845833) * r +
                .24178072517745061177) * r + 1.27045825245236838258) * r +
              3.64784832476320460504) * r + 5.7694972214606914055) * r +
            4.6303378461565452959) * r + 1.42343711074968357734) /
          (((((((r * 1.05075007164441684324e-9 + 5.475938084995344946e-4) * r +
                .0151986665636164571966) * r + .14810397642748007459) * r +
              .68976733498510000455) * r + 1.6763848301838038494) * r +
            2.05319162663775882187) * r + 1.);
  } else {
    r += -5.;
    val = (((((((r * 2.01033439929228813265e-7 + 2.71155556874348757815e-5) * r +
                .0012426609473880784386) * r + .026532189526576123093) * r +
              .29656057182850489123) * r + 1.7848265399172913358) * r +
            5.4637849111641143699) * r + 6.6579046435011037772) /
          (((((((r * 2.04426310338993978564e-15 + 1.4215117583164458887e-7) * r +
                1.8463183175100546818e-5) * r + 7.868691311456132591e-4) * r +
              .0148753612908506148525) * r + .13692988092273580531) * r +
            .59983220655588793769) * r + 1.);
  }
  if (q < 0.0) val = -val;
  return val;
}

double pht_rs_norm_rand(pht_rstream *rs) {
  /* INVERSION: unif_rand() alone is not of high enough precision */
  const double BIG = 134217728; /* 2^27 */
  double u = pht_rs_unif_rand(rs);
  u = (int)(BIG * u) + pht_rs_unif_rand(rs);
  return pht_rs_qnorm(u / BIG);
}

double pht_rs_runif(pht_rstream *rs, double a, double b) {
  if (!isfinite(a) || !isfinite(b) || b < a) return NAN;
  if (a == b) return a;
  double u;
  do {
    u = pht_rs_unif_rand(rs);
  } while (u <= 0 || u >= 1);
  return a + (b - a) * u;
}

double pht_rs_rexp(pht_rstream *rs, double scale) {
  if (!isfinite(scale) || scale <= 0.0) {
    if (scale == 0.) return 0.;
    return NAN;
  }
  return scale * pht_rs_exp_rand(rs);
}

double pht_rs_dexp(double x, double scale, int give_log) {
  if (isnan(x) || isnan(scale)) return x + scale;
  if (scale <= 0.0) return NAN;
  if (x < 0.) return give_log ? -INFINITY : 0.;
  return give_log ? (-x / scale) - log(scale) : exp(-x / scale) / scale;
}

double pht_rs_rgamma(pht_rstream *rs, double a, double scale) {
  const double sqrt32 = 5.656854;
  const double exp_m1 = 0.36787944117144233; /* exp(-1) = 1/e */
  const double q1 = 0.04166669, q2 = 0.02083148, q3 = 0.00801191,
               q4 = 0.00144121, q5 = -7.388e-5, q6 = 2.4511e-4, q7 = 2.424e-4;
  const double a1 = 0.3333333, a2 = -0.250003, a3 = 0.2000062,
               a4 = -0.1662921, a5 = 0.1423657, a6 = -0.1367177,
               a7 = 0.1233795;
  double s, s2, d, q0, b, si, c;
  double e, p, q, r, t, u, v, w, x, ret_val;

  if (isnan(a) || isnan(scale)) return NAN;
  if (a <= 0.0 || scale <= 0.0) {
    if (scale == 0. || a == 0.) return 0.;
    return NAN;
  }
  if (!isfinite(a) || !isfinite(scale)) return INFINITY;

  if (a < 1.) { /* GS algorithm for parameters a < 1 */
    e = 1.0 + exp_m1 * a;
    for (;;) {
      p = e * pht_rs_unif_rand(rs);
      if (p >= 1.0) {
        x = -log((e - p) / a);
        if (pht_rs_exp_rand(rs) >= (1.0 - a) * log(x)) break;
      } else {
        x = exp(log(p) / a);
        if (pht_rs_exp_rand(rs) >= x) break;
      }
    }
    return scale * x;
  }

  /* GD algorithm, a >= 1 (the constants R caches per `a` are recomputed) */
  s2 = a - 0.5;
  s = sqrt(s2);
  d = sqrt32 - s * 12.;

  t = pht_rs_norm_rand(rs);
  x = s + 0.5 * t;
  ret_val = x * x;
  if (t >= 0.) return scale * ret_val;

  u = pht_rs_unif_rand(rs);
  if (d * u <= t * t * t) return scale * ret_val;

  r = 1. / a;
  q0 = ((((((q7 * r + q6) * r + q5) * r + q4) * r + q3) * r + q2) * r + q1) * r;
  if (a <= 3.686) {
    b = 0.463 + s + 0.178 * s2;
    si = 1.235;
    c = 0.195 / s - 0.079 + 0.16 * s;
  } else if (a <= 13.022) {
    b = 1.654 + 0.0076 * s2;
    si = 1.68 / s + 0.275;
    c = 0.062 / s + 0.024;
  } else {
    b = 1.77;
    si = 0.75;
    c = 0.1515 / s;
  }

  if (x > 0.) {
    v = t / (s + s);
    if (fabs(v) <= 0.25)
      q = q0 + 0.5 * t * t *
                   ((((((a7 * v + a6) * v + a5) * v + a4) * v + a3) * v + a2) * v + a1) * v;
    else
      q = q0 - s * t + 0.25 * t * t + (s2 + s2) * log(1.0 + v);
    if (log(1.0 - u) <= q) return scale * ret_val;
  }

  for (;;) {
    e = pht_rs_exp_rand(rs);
    u = pht_rs_unif_rand(rs);
    u = u + u - 1.0;
    if (u < 0.0)
      t = b - si * e;
    else
      t = b + si * e;
    if (t >= -0.71874483771719) {
      v = t / (s + s);
      if (fabs(v) <= 0.25)
        q = q0 + 0.5 * t * t *
                     ((((((a7 * v + a6) * v + a5) * v + a4) * v + a3) * v + a2) * v + a1) * v;
      else
        q = q0 - s * t + 0.25 * t * t + (s2 + s2) * log(1.0 + v);
      if (q > 0.0) {
        w = expm1(q);
        if (c * fabs(u) <= w * exp(e - 0.5 * t * t)) break;
      }
    }
  }
  x = s + 0.5 * t;
  return scale * x * x;
}
