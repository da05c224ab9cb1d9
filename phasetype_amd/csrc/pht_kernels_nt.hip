/*
 * pht_kernels_nt.hip — one compile-time n of the sweep kernels
 * (pht_kernels_impl.h).  Compiled once per PHT_NT in {3, 5, 10, 15, 20, 0}
 * (0 = runtime n) into separate objects; pht_dispatch.hip picks by n.
 */
#include "pht_kernels_impl.h"

#ifndef PHT_NT
#error "compile with -DPHT_NT=<n> (0 = runtime n)"
#endif

#define PHT_CAT2(a, b) a##b
#define PHT_CAT(a, b) PHT_CAT2(a, b)

extern "C" hipError_t PHT_CAT(pht_launch_nt_, PHT_NT)(const pht::SweepArgs *a, int method, int debug,
                                                     hipStream_t st) {
  return pht::launch_nt<PHT_NT>(*a, method, debug != 0, st);
}

extern "C" hipError_t PHT_CAT(pht_launch_chains_nt_, PHT_NT)(const pht::SweepArgs *h, const pht::SweepArgs *d, int K,
                                                            hipStream_t st) {
  return pht::launch_ecs_chains<PHT_NT>(h, d, K, st);
}

extern "C" hipError_t PHT_CAT(pht_launch_mchains_nt_, PHT_NT)(const pht::SweepArgs *h, const pht::SweepArgs *d, int K,
                                                             int method, hipStream_t st) {
  return pht::launch_chains<PHT_NT>(h, d, K, method, st);
}
