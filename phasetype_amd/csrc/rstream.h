/*
 * rstream.h — R-compatible host random stream (standalone builds only).
 *
 * The reference draws every random number through R's nmath/RNG
 * (`unif_rand`, `exp_rand`, `norm_rand`, `rgamma`, `runif`, `rexp`, `dexp`;
 * call sites: src/PHT_MCMC_Aslett.c:200,366, src/arms.c:838-846,
 * src/Simulate_AbsCTMC_*.c).  Inside an R process the product library calls
 * R's own functions (resolved at load time, see gibbs_host.cpp); outside R
 * (pytest, bench.py, the GPU box) it uses this restatement of R's default
 * generator: Mersenne-Twister with R's `set.seed` scrambling, Ahrens-Dieter
 * (1972) `exp_rand`, inversion `norm_rand` (Wichura AS241) and
 * Ahrens-Dieter GD/GS `rgamma`.
 *
 * Self-check values (R documentation / widely published outputs):
 *   set.seed(1); runif(3)  -> 0.2655087 0.3721239 0.5728534
 *   set.seed(1); rexp(1)   -> 0.7551818
 *   set.seed(1); rnorm(5)  -> -0.6264538 0.1836433 -0.8356286 1.5952808 0.3295078
 * (tests/test_rstream.py).  rgamma has no such published vector available
 * offline: it is "parity unpinned" beyond the shared exp_rand/norm_rand/
 * unif_rand primitives it is built from.
 */
#ifndef PHT_RSTREAM_H
#define PHT_RSTREAM_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* R's .Random.seed for Mersenne-Twister: mti followed by mt[624]. */
typedef struct pht_rstream {
  uint32_t mt[624];
  int mti;
  uint64_t nword; /* 32-bit MT outputs consumed since set_seed (draw-order checks) */
} pht_rstream;

void   pht_rs_set_seed(pht_rstream *rs, uint32_t seed);      /* set.seed(seed) */
double pht_rs_unif_rand(pht_rstream *rs);                     /* unif_rand()   */
double pht_rs_exp_rand(pht_rstream *rs);                      /* exp_rand()    */
double pht_rs_norm_rand(pht_rstream *rs);                     /* norm_rand(), INVERSION */
double pht_rs_runif(pht_rstream *rs, double a, double b);     /* runif(a,b)    */
double pht_rs_rexp(pht_rstream *rs, double scale);            /* rexp(scale)   */
double pht_rs_rgamma(pht_rstream *rs, double a, double scale);/* rgamma(a,scale) */
double pht_rs_dexp(double x, double scale, int give_log);     /* dexp(x,scale,log) */
double pht_rs_qnorm(double p);                                /* qnorm5(p,0,1,TRUE,FALSE) */

#ifdef __cplusplus
}
#endif
#endif
