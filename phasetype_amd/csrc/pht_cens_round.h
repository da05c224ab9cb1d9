/*
 * pht_cens_round.h — the ECS sampler's right-censored observations
 * (LJMA_samplechain + LJMA_condjump_r_ars, src/Simulate_AbsCTMC_gt_Aslett_DCS.c:
 * 184-260, 299-418) as a persistent kernel of jump-converged rounds.
 *
 * One lane running a censored path to its end idles, once its path
 * is done, until the longest path of its wavefront is (a censored path
 * runs past y until absorption, so path lengths vary widely).  Here a loop
 * iteration ("round") is ONE jump of every lane (censored_jump in
 * pht_device.h: the sojourn by the stay test / ARMS / exponential, then
 * the next state); a lane whose path ended takes the next observation at
 * the top of the next round and makes its first jump in that round.
 * Every lane performs exactly the device specification's operations and
 * draws (censored_begin + censored_jump until done): results are
 * bit-identical to the oracle's device specification (orcD_censored).  The launch must hold censored
 * observations only (SweepArgs::allcens; ctx_enqueue's censored range).
 */
#ifndef PHT_CENS_ROUND_H
#define PHT_CENS_ROUND_H

#include "pht_device.h"
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

  Sink<DEBUG> sk{zq, Bc, Nc, n, a.zscale, nullptr, nullptr, nullptr, nullptr};
  Lane ln;
  ln.flags = 0; ln.neval = 0; ln.nbrent = 0; ln.njump = 0;
  CensLane<NT> cl;
  using EnvL = EnvLdsXY<(cens_env_lds<NT>() ? cens_env_k<NT>() : 1), kBlock>;
  typename std::conditional<cens_env_lds<NT>(), EnvL, EnvPrivate>::type env;
  double spill[2 * EnvL::kSpill];
  double cumv[100];
  if constexpr (cens_env_lds<NT>()) env.bind(envl, threadIdx.x, (PHT_PRIV double *)spill, (PHT_PRIV double *)cumv);
  bool have = false, done = false;
  long pos = 0;
  unsigned c_obs = 0, c_neval = 0, c_flag = 0, c_nd = 0, c_jump = 0;
  for (;;) {
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
    if (!__any(have)) break;
    /* one converged Philox block per round (the stay test, the sojourn
     * and the next state draw 2-4 words outside ARMS) */
#ifdef PHT_CENS_PHILOX_UNROLL
    if (have) pht_stream_topup_unrolled(&ln.r);
#else
    if (have) pht_stream_topup(&ln.r);
#endif
    /* ---- one jump of every lane with a path */
    if (have && censored_jump(P, ln, env, sk, cl)) {
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
