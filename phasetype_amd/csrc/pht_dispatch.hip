/*
 * pht_dispatch.hip — pht_launch_sweep: validates the launch and picks the
 * kernels compiled for this n (pht_kernels_nt.hip; fully unrolled spectral
 * sums for n in {3, 5, 10, 15, 20}, runtime-n loops otherwise).
 */
#include <hip/hip_runtime.h>
#include <stdlib.h>

#include "pht_kernels.h"
#include "pht_layout.h"

#define PHT_DECL(K) \
  extern "C" hipError_t pht_launch_nt_##K(const pht::SweepArgs *a, int method, int debug, hipStream_t st); \
  extern "C" hipError_t pht_launch_chains_nt_##K(const pht::SweepArgs *h, const pht::SweepArgs *d, int nch, \
                                                 hipStream_t st);                                            \
  extern "C" hipError_t pht_launch_mchains_nt_##K(const pht::SweepArgs *h, const pht::SweepArgs *d, int nch,  \
                                                  int method, hipStream_t st);
PHT_DECL(0)
PHT_DECL(3)
PHT_DECL(5)
PHT_DECL(10)
PHT_DECL(15)
PHT_DECL(20)
#undef PHT_DECL

/* The sweep's statistics block to the host without a copy engine round trip
 * (ctx_enqueue, gibbs_host.cpp): one workgroup reads the block, stores it
 * into host-pinned coherent memory and zeroes it for the next sweep; after
 * a system-scope fence of every thread, thread 0 publishes seq in the
 * host-visible flag with a release store.  The host polls that flag instead
 * of waiting on an event behind a blit copy and a fill. */
__global__ void __launch_bounds__(256) pht_stats_out_kernel(unsigned long long *d, unsigned long long *h,
                                                            unsigned *flag, unsigned seq, int sl) {
  for (int k = threadIdx.x; k < sl; k += blockDim.x) {
    h[k] = d[k];
    d[k] = 0ull;
  }
  __threadfence_system();
  __syncthreads();
  if (threadIdx.x == 0) __hip_atomic_store(flag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

extern "C" hipError_t pht_launch_stats_out(unsigned long long *d_stats, unsigned long long *h_out_dev,
                                           unsigned *flag_dev, unsigned seq, int sl, hipStream_t st) {
  if (sl < 1 || !d_stats || !h_out_dev || !flag_dev) return hipErrorInvalidValue;
  hipLaunchKernelGGL(pht_stats_out_kernel, dim3(1), dim3(256), 0, st, d_stats, h_out_dev, flag_dev, seq, sl);
  return hipGetLastError();
}

/* The pipelined Gibbs loop's gate (gibbs_host.cpp, gibbs_run): the next
 * sweep is enqueued while the current one runs, behind this one-workgroup
 * kernel, which waits until the host has written that sweep's parameter
 * block (host-pinned coherent memory) and released `want` in the gate word,
 * then copies the block to the device.  Thread 0 polls the gate with
 * system-scope acquire loads (vector loads: nothing here goes through the
 * scalar cache); a gate not released within ~20 s ends the wait anyway and
 * the ack word says so (the host then fails the run: the sweep ran on stale
 * parameters), so no wave waits without bound.  ack = want after a good
 * copy. */
__global__ void __launch_bounds__(256) pht_gate_kernel(const unsigned *gate, unsigned want,
                                                       const unsigned long long *src, unsigned long long *dst,
                                                       int nwords, unsigned *ack) {
  __shared__ int ok;
  if (threadIdx.x == 0) {
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime(); /* 100 MHz */
    int good = 0;
    for (;;) {
      if (__hip_atomic_load(gate, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) == want) {
        good = 1;
        break;
      }
      if (__builtin_amdgcn_s_memrealtime() - t0 > 2000000000ull) break;
      __builtin_amdgcn_s_sleep(2);
    }
    ok = good;
  }
  __syncthreads();
  if (ok) {
    /* eight loads in flight per thread (one link round trip per 2,048 words,
     * the whole block at n <= 16) */
    for (int base = 0; base < nwords; base += 8 * 256) {
      unsigned long long v[8];
#pragma unroll
      for (int q = 0; q < 8; q++) {
        const int k = base + q * 256 + (int)threadIdx.x;
        v[q] = k < nwords ? __hip_atomic_load(&src[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) : 0ull;
      }
#pragma unroll
      for (int q = 0; q < 8; q++) {
        const int k = base + q * 256 + (int)threadIdx.x;
        if (k < nwords) dst[k] = v[q];
      }
    }
  }
  __threadfence_system();
  __syncthreads();
  if (threadIdx.x == 0) __hip_atomic_store(ack, ok ? want : ~want, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

extern "C" hipError_t pht_launch_gate(const unsigned *gate_dev, unsigned want, const unsigned long long *src_dev,
                                      unsigned long long *dst, int nwords, unsigned *ack_dev, hipStream_t st) {
  if (!gate_dev || !src_dev || !dst || !ack_dev || nwords < 1) return hipErrorInvalidValue;
  hipLaunchKernelGGL(pht_gate_kernel, dim3(1), dim3(256), 0, st, gate_dev, want, src_dev, dst, nwords, ack_dev);
  return hipGetLastError();
}

extern "C" hipError_t pht_launch_sweep(const pht::SweepArgs *a, int method, int debug, hipStream_t st) {
  using namespace pht;
  if (a->n < 1 || a->n > kMaxN) return hipErrorInvalidValue;
  if ((make_layout(a->n).bytes() & 15) != 0) return hipErrorInvalidValue;
  static const bool generic = getenv("PHT_FORCE_NT0") != nullptr; /* A/B: runtime-n kernels only */
  if (generic) return pht_launch_nt_0(a, method, debug, st);
  switch (a->n) {
    case 3: return pht_launch_nt_3(a, method, debug, st);
    case 5: return pht_launch_nt_5(a, method, debug, st);
    case 10: return pht_launch_nt_10(a, method, debug, st);
    case 15: return pht_launch_nt_15(a, method, debug, st);
    case 20: return pht_launch_nt_20(a, method, debug, st);
    default: return pht_launch_nt_0(a, method, debug, st);
  }
}

/* K chains' exact ECS ranges in one launch (h on the host, the same K
 * SweepArgs already copied to d on the device, in stream order before the
 * launch); the chains must share n.  See ecs_chains_kernel. */
extern "C" hipError_t pht_launch_ecs_chains(const pht::SweepArgs *h, const pht::SweepArgs *d, int K, hipStream_t st) {
  using namespace pht;
  if (K < 1) return hipErrorInvalidValue;
  const int n = h[0].n;
  if (n < 1 || n > kMaxN || (make_layout(n).bytes() & 15) != 0) return hipErrorInvalidValue;
  for (int c = 0; c < K; c++)
    if (h[c].n != n || h[c].cens != nullptr || h[c].dbg_zq != nullptr) return hipErrorInvalidValue;
  switch (n) {
    case 3: return pht_launch_chains_nt_3(h, d, K, st);
    case 5: return pht_launch_chains_nt_5(h, d, K, st);
    case 10: return pht_launch_chains_nt_10(h, d, K, st);
    case 15: return pht_launch_chains_nt_15(h, d, K, st);
    case 20: return pht_launch_chains_nt_20(h, d, K, st);
    default: return pht_launch_chains_nt_0(h, d, K, st);
  }
}

/* K chains' sweeps in one launch sequence for MHRS, DCS, UNIF (whole
 * shards) or ECS's censored ranges; see launch_chains */
extern "C" hipError_t pht_launch_chains(const pht::SweepArgs *h, const pht::SweepArgs *d, int K, int method,
                                        hipStream_t st) {
  using namespace pht;
  if (K < 1) return hipErrorInvalidValue;
  const int n = h[0].n;
  if (n < 1 || n > kMaxN || (make_layout(n).bytes() & 15) != 0) return hipErrorInvalidValue;
  for (int c = 0; c < K; c++)
    if (h[c].n != n || h[c].dbg_zq != nullptr) return hipErrorInvalidValue;
  static const bool generic = getenv("PHT_FORCE_NT0") != nullptr;
  if (generic) return pht_launch_mchains_nt_0(h, d, K, method, st);
  switch (n) {
    case 3: return pht_launch_mchains_nt_3(h, d, K, method, st);
    case 5: return pht_launch_mchains_nt_5(h, d, K, method, st);
    case 10: return pht_launch_mchains_nt_10(h, d, K, method, st);
    case 15: return pht_launch_mchains_nt_15(h, d, K, method, st);
    case 20: return pht_launch_mchains_nt_20(h, d, K, method, st);
    default: return pht_launch_mchains_nt_0(h, d, K, method, st);
  }
}
