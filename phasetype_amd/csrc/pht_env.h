/*
 * pht_env.h — storage policies for the ARMS envelope of one lane.
 *
 * The reference keeps up to 100 POINTs {x, y, ey, cum, f, pl, pr} in a
 * stack array linked by pointers (src/arms.c:17-32).  The device keeps the
 * same points as position-ordered arrays (f = parity of the position, see
 * oracle/pht_oracle_impl.h) and stores only x, y and cum: ey is recomputed
 * from (y, ymax) where used (bit-identical).
 *
 * EnvPrivate  all 100 points in lane-private memory (scratch).
 * EnvLdsXY<K> x and y of the first K points in LDS, lane-interleaved (point
 *             k of lane t at base[k * stride + t]: a wavefront touching
 *             the same k reads 512 contiguous bytes, conflict-free
 *             ds_read_b64); cum and points K..99 in private memory.  Same
 *             results as EnvPrivate for any K.
 */
#ifndef PHT_ENV_H
#define PHT_ENV_H

#include <hip/hip_runtime.h>

#ifndef PHT_LDS
#define PHT_LDS __attribute__((address_space(3)))
#endif

namespace pht {

struct EnvPrivate {
  static constexpr bool kUnroll = true; /* arms_*: unrolled code for envelopes of <= kArmsU points */
  static constexpr int kLds = 0;        /* points held outside private memory */
  double x[100], y[100], cum[100];
  int cnt;
  double ymax;
  __device__ __forceinline__ double X(int k) const { return x[k]; }
  __device__ __forceinline__ double Y(int k) const { return y[k]; }
  __device__ __forceinline__ double CUM(int k) const { return cum[k]; }
  __device__ __forceinline__ void sX(int k, double v) { x[k] = v; }
  __device__ __forceinline__ void sY(int k, double v) { y[k] = v; }
  __device__ __forceinline__ void sCUM(int k, double v) { cum[k] = v; }
  /* positions known to lie below kLds (EnvLdsXY): the same storage here */
  __device__ __forceinline__ double XL(int k) const { return x[k]; }
  __device__ __forceinline__ double YL(int k) const { return y[k]; }
  __device__ __forceinline__ void sXL(int k, double v) { x[k] = v; }
  __device__ __forceinline__ void sYL(int k, double v) { y[k] = v; }
};

/* EnvPrivate for envelopes known to exceed kArmsU points (the ECS row
 * kernel's general-code continuation): the rolled loops only, which keeps
 * the unrolled code's register arrays out of the caller (same values) */
struct EnvPrivateBig : EnvPrivate {
  static constexpr bool kUnroll = false;
};

#ifndef PHT_PRIV
#define PHT_PRIV __attribute__((address_space(5)))
#endif

/* x and y of the first K points per lane in LDS (lane-interleaved), the
 * rest and all of cum in private memory.  The converged ECS round keeps cum
 * in registers between cumulate and invert and never touches the private
 * part for envelopes of up to K points; the general ARMS code (rare, long
 * rejection chains) uses the full accessors. */
template <int K, int STRIDE>
struct EnvLdsXY {
  static constexpr bool kUnroll = true;
  static constexpr int kLds = K;
  static constexpr int kSpill = 100 - K;
  PHT_LDS double *l;   /* lane's element 0 */
  PHT_PRIV double *ov; /* [2][kSpill] x, y beyond K */
  PHT_PRIV double *cm; /* [100] cum */
  int cnt;
  double ymax;
  __device__ __forceinline__ void bind(PHT_LDS double *lds, int tid, PHT_PRIV double *spill, PHT_PRIV double *cum) {
    l = lds + tid;
    ov = spill;
    cm = cum;
  }
  static constexpr int lds_doubles_per_lane() { return 2 * K; }
  __device__ __forceinline__ double X(int k) const { if (k < K) return l[k * STRIDE]; return ov[k - K]; }
  __device__ __forceinline__ double Y(int k) const { if (k < K) return l[(K + k) * STRIDE]; return ov[kSpill + k - K]; }
  __device__ __forceinline__ double CUM(int k) const { return cm[k]; }
  __device__ __forceinline__ void sX(int k, double v) { if (k < K) l[k * STRIDE] = v; else ov[k - K] = v; }
  __device__ __forceinline__ void sY(int k, double v) {
    if (k < K) l[(K + k) * STRIDE] = v; else ov[kSpill + k - K] = v;
  }
  __device__ __forceinline__ void sCUM(int k, double v) { cm[k] = v; }
  /* run-time positions the caller knows to be < K (the converged round's
   * envelope, pht_ecs_round.h): LDS only, no private-memory branch */
  __device__ __forceinline__ double XL(int k) const { return l[k * STRIDE]; }
  __device__ __forceinline__ double YL(int k) const { return l[(K + k) * STRIDE]; }
  __device__ __forceinline__ void sXL(int k, double v) { l[k * STRIDE] = v; }
  __device__ __forceinline__ void sYL(int k, double v) { l[(K + k) * STRIDE] = v; }
};

}  // namespace pht
#endif
