/*
 * pht_gamma.h — counter-based Gamma draws for the device-resident Gibbs
 * chain (pht_gibbs_run_resident), shared by the HIP update kernel and the
 * oracle's restatement of that chain, so both produce the same draws bit
 * for bit (every translation unit that includes this is compiled with
 * -ffp-contract=off; exp/log are pht_detmath.h's, sqrt is IEEE).
 *
 * The reference draws the conjugate update with R's rgamma on R's serial
 * stream (src/PHT_MCMC_Aslett.c:366); the host loop of this library
 * reproduces that exactly (rstream.c).  A chain that never returns to the
 * host needs its own sampler: NON-PARITY, validated in distribution
 * (tests: shape/scale moments and the posterior harness).
 *
 * Stream: parameter k at Gibbs iteration it draws from the Philox word
 * stream (obs = 0xFFFFFFFF - k, tag = 0x7FFFFFFF, sweep = it) under the
 * chain's key; no observation has such an id (ids < 2^31).
 *
 * Normal: Marsaglia's polar method (the second variate is discarded, so a
 * draw needs no state).  Gamma(a, scale): Marsaglia & Tsang (2000) for
 * a >= 1; for a < 1, Gamma(a + 1) * U^(1/a) with U drawn after the loop.
 * Loops are capped (PHT_GAMMA_MAXIT) so a wave always terminates; a capped
 * draw returns NaN, which the caller counts as an error.
 */
#ifndef PHT_GAMMA_H
#define PHT_GAMMA_H

#include "pht_detmath.h"
#include "pht_philox.h"

#define PHT_GAMMA_MAXIT 1000
#define PHT_GAMMA_OBS(k) (0xFFFFFFFFu - (uint32_t)(k))
#define PHT_GAMMA_TAG 0x7FFFFFFFu

PHT_HD double pht_rnorm(pht_stream *s) {
  for (int it = 0; it < PHT_GAMMA_MAXIT; it++) {
    const double u = 2.0 * pht_next_u(s) - 1.0;
    const double v = 2.0 * pht_next_u(s) - 1.0;
    const double q = u * u + v * v;
    if (q > 0.0 && q < 1.0) return u * sqrt(-2.0 * pht_log(q) / q);
  }
  return NAN;
}

PHT_HD double pht_rgamma_ctr(pht_stream *s, double a, double scale) {
  if (!(a > 0.0) || !(scale > 0.0) || !isfinite(a) || !isfinite(scale)) return NAN;
  const double a1 = (a < 1.0) ? a + 1.0 : a;
  const double d = a1 - 1.0 / 3.0;
  const double c = 1.0 / sqrt(9.0 * d);
  double g = NAN;
  for (int it = 0; it < PHT_GAMMA_MAXIT; it++) {
    const double x = pht_rnorm(s);
    double v = 1.0 + c * x;
    if (!(v > 0.0)) continue;
    v = v * v * v;
    const double u = pht_next_u(s);
    const double x2 = x * x;
    if (u < 1.0 - 0.0331 * (x2 * x2)) {
      g = d * v;
      break;
    }
    if (pht_log(u) < 0.5 * x2 + d * (1.0 - v + pht_log(v))) {
      g = d * v;
      break;
    }
  }
  if (a < 1.0) g = g * pht_exp(pht_log(pht_next_u(s)) / a);
  return g * scale;
}

#endif /* PHT_GAMMA_H */
