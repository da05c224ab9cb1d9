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
 * EnvLds<K>   the first K points in LDS, lane-interleaved (point k of lane t
 *             at base[k * stride + t], so a wavefront touching the same k
 *             reads 512 contiguous bytes: conflict-free ds_read_b64), points
 *             K..99 in private memory.  An ARMS call holds 9 points plus 2
 *             per rejection; K = 11 keeps one rejection in LDS, rarer calls
 *             spill.  Same results as EnvPrivate for any K.
 */
#ifndef PHT_ENV_H
#define PHT_ENV_H

#include <hip/hip_runtime.h>

namespace pht {

struct EnvPrivate {
  double x[100], y[100], cum[100];
  int cnt;
  double ymax;
  __device__ __forceinline__ double X(int k) const { return x[k]; }
  __device__ __forceinline__ double Y(int k) const { return y[k]; }
  __device__ __forceinline__ double CUM(int k) const { return cum[k]; }
  __device__ __forceinline__ void sX(int k, double v) { x[k] = v; }
  __device__ __forceinline__ void sY(int k, double v) { y[k] = v; }
  __device__ __forceinline__ void sCUM(int k, double v) { cum[k] = v; }
};

template <int K>
struct EnvLds {
  double *lx, *ly, *lc; /* LDS: lane's element 0; element k at +k*stride */
  int stride;
  double ox[100 - K], oy[100 - K], oc[100 - K];
  int cnt;
  double ymax;
  __device__ __forceinline__ void bind(double *lds, int nthreads, int tid) {
    stride = nthreads;
    lx = lds + tid;
    ly = lds + K * nthreads + tid;
    lc = lds + 2 * K * nthreads + tid;
  }
  static constexpr int lds_doubles_per_lane() { return 3 * K; }
  __device__ __forceinline__ double X(int k) const { if (k < K) return lx[k * stride]; return ox[k - K]; }
  __device__ __forceinline__ double Y(int k) const { if (k < K) return ly[k * stride]; return oy[k - K]; }
  __device__ __forceinline__ double CUM(int k) const { if (k < K) return lc[k * stride]; return oc[k - K]; }
  __device__ __forceinline__ void sX(int k, double v) { if (k < K) lx[k * stride] = v; else ox[k - K] = v; }
  __device__ __forceinline__ void sY(int k, double v) { if (k < K) ly[k * stride] = v; else oy[k - K] = v; }
  __device__ __forceinline__ void sCUM(int k, double v) { if (k < K) lc[k * stride] = v; else oc[k - K] = v; }
};

}  // namespace pht
#endif
