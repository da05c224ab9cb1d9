/*
 * pht_detmath.h — deterministic FP64 exp/log shared by the HIP kernels and
 * the oracle's device-mode restatement (oracle/pht_oracle.c, ORC_DEV).
 *
 * Why: the reference evaluates exp/log through glibc (src/arms.c:792-812,
 * src/Simulate_AbsCTMC_eq_Aslett_ECS.c:25,124-134,163,170, ...).  glibc and
 * the GPU's ocml differ in the last ulp on some inputs, and ARMS / the
 * categorical jumps turn last-ulp differences into different discrete
 * decisions.  Defining exp/log here from IEEE-754 basic operations and
 * explicit fma() only (no contraction: every translation unit that includes
 * this is compiled with -ffp-contract=off) makes a GPU lane and the CPU
 * restatement produce bit-identical results for the same inputs.
 *
 * Accuracy: < 1 ulp over the full double range (checked against mpmath in
 * tests/test_detmath.py).  Not correctly rounded; deterministic.
 *   exp: Cody–Waite reduction x = k ln2 + r (|r| <= ln2/2, k by the 1.5·2^52
 *        shifter), degree-13 Taylor for e^r by fma Horner, scale by 2^k.
 *   log: x = 2^k m, m in [sqrt(1/2), sqrt(2)), f = m-1, s = f/(2+f),
 *        log(1+f) = f - (hfsq - s(hfsq + R(s^2))) with the classic fdlibm
 *        e_log.c minimax coefficients Lg1..Lg7.
 */
#ifndef PHT_DETMATH_H
#define PHT_DETMATH_H

#include <math.h>
#include <stdint.h>
#include <string.h>

#if defined(__HIPCC__)
#define PHT_HD __host__ __device__ __forceinline__
#else
#define PHT_HD static inline
#endif

PHT_HD uint64_t pht_d2u(double x) { uint64_t u; memcpy(&u, &x, 8); return u; }
PHT_HD double pht_u2d(uint64_t u) { double x; memcpy(&x, &u, 8); return x; }

PHT_HD double pht_exp(double x) {
  const double INV_LN2 = 1.4426950408889634074;      /* 1/ln2 */
  const double LN2_HI = 6.93147180559945286227e-01;   /* ln2 rounded */
  const double LN2_LO = 2.31904681384629955842e-17;   /* ln2 - LN2_HI */
  const double SHIFT = 6755399441055744.0;            /* 1.5 * 2^52 */
  if (x != x) return x;
  if (x > 709.782712893383973096) return INFINITY;
  if (x < -745.133219101941108420) return 0.0;
  double kd = fma(x, INV_LN2, SHIFT) - SHIFT; /* round-to-nearest-even integer */
  double r = fma(-kd, LN2_HI, x);
  r = fma(-kd, LN2_LO, r);
  double p = 1.6059043836821614599e-10;               /* 1/13! */
  p = fma(p, r, 2.0876756987868098979e-09);           /* 1/12! */
  p = fma(p, r, 2.5052108385441718775e-08);           /* 1/11! */
  p = fma(p, r, 2.7557319223985890653e-07);           /* 1/10! */
  p = fma(p, r, 2.7557319223985892511e-06);           /* 1/9!  */
  p = fma(p, r, 2.4801587301587301566e-05);           /* 1/8!  */
  p = fma(p, r, 1.9841269841269841253e-04);           /* 1/7!  */
  p = fma(p, r, 1.3888888888888889419e-03);           /* 1/6!  */
  p = fma(p, r, 8.3333333333333332177e-03);           /* 1/5!  */
  p = fma(p, r, 4.1666666666666664354e-02);           /* 1/4!  */
  p = fma(p, r, 1.6666666666666665741e-01);           /* 1/3!  */
  p = fma(p, r, 0.5);
  p = fma(p, r, 1.0);
  p = fma(p, r, 1.0);
  int k = (int)kd;
  if (k > 1023) return p * 2.0 * pht_u2d((uint64_t)(k - 1 + 1023) << 52);
  if (k < -1022) return (p * pht_u2d((uint64_t)(k + 54 + 1023) << 52)) * 5.5511151231257827021e-17; /* 2^-54 */
  return p * pht_u2d((uint64_t)(k + 1023) << 52);
}

PHT_HD double pht_log(double x) {
  const double LN2_HI = 6.93147180369123816490e-01; /* 0x3fe62e42fee00000 */
  const double LN2_LO = 1.90821492927058770002e-10; /* 0x3dea39ef35793c76 */
  const double Lg1 = 6.666666666666735130e-01, Lg2 = 3.999999999940941908e-01,
               Lg3 = 2.857142874366239149e-01, Lg4 = 2.222219843214978396e-01,
               Lg5 = 1.818357216161805012e-01, Lg6 = 1.531383769920937332e-01,
               Lg7 = 1.479819860511658591e-01;
  if (x != x) return x;
  if (x < 0.0) return NAN;
  if (x == 0.0) return -INFINITY;
  if (x == INFINITY) return x;
  uint64_t u = pht_d2u(x);
  int k = 0;
  if (u < 0x0010000000000000ULL) { /* subnormal */
    x *= 18014398509481984.0;      /* 2^54 */
    u = pht_d2u(x);
    k = -54;
  }
  k += (int)(u >> 52) - 1023;
  uint64_t mant = u & 0x000fffffffffffffULL;
  /* m in [1,2); if m >= sqrt(2) use m/2 and k+1 */
  if (mant >= 0x6a09e667f3bcdULL) { /* sqrt(2) mantissa */
    u = mant | 0x3fe0000000000000ULL;
    k += 1;
  } else {
    u = mant | 0x3ff0000000000000ULL;
  }
  double f = pht_u2d(u) - 1.0;
  double hfsq = 0.5 * f * f;
  double s = f / (2.0 + f);
  double z = s * s;
  double w = z * z;
  double t1 = w * fma(w, fma(w, Lg6, Lg4), Lg2);
  double t2 = z * fma(w, fma(w, fma(w, Lg7, Lg5), Lg3), Lg1);
  double R = t2 + t1;
  double dk = (double)k;
  return dk * LN2_HI - ((hfsq - (s * (hfsq + R) + dk * LN2_LO)) - f);
}

#endif /* PHT_DETMATH_H */
