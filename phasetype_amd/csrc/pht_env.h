/*
 * pht_env.h — storage policies for the ARMS envelope of one lane.
 *
 * The reference keeps up to 100 POINTs {x, y, ey, cum, f, pl, pr} in a
 * stack array linked by pointers (src/arms.c:17-32).  The device keeps the
 * same points as position-ordered arrays (f = parity of the position; see
 * oracle/pht_oracle_impl.h), so only x, y, ey, cum are stored.
 *
 * EnvPrivate: all 100 points in lane-private memory (scratch); the
 * capacity-exact baseline policy.
 */
#ifndef PHT_ENV_H
#define PHT_ENV_H

#include <hip/hip_runtime.h>

namespace pht {

struct EnvPrivate {
  double x[100], y[100], ey[100], cum[100];
  int cnt;
  double ymax;
  __device__ __forceinline__ void bind(int) {}
  __device__ __forceinline__ double &X(int k) { return x[k]; }
  __device__ __forceinline__ double &Y(int k) { return y[k]; }
  __device__ __forceinline__ double &EY(int k) { return ey[k]; }
  __device__ __forceinline__ double &CUM(int k) { return cum[k]; }
};

}  // namespace pht
#endif
