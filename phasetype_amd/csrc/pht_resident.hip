/*
 * pht_resident.hip — the device-resident Gibbs chain's per-sweep update
 * (opt-in, NON-PARITY): everything LJMA_Gibbs does on the
 * host between two step-1 sweeps, as one workgroup, so sweeps chain on the
 * stream with no host round trip:
 *
 *   step 4-5 (src/PHT_MCMC_Aslett.c:340-397): Nsum/zsum per parameter from
 *     the (reduced) statistics block in the reference's list order, the
 *     conjugate draw Gamma(nu + Nsum, 1 / (zeta + zsum)) — counter-based
 *     (include/pht_gamma.h) instead of R's rgamma — the TT/S/s refresh and
 *     the diagonal in reverse list order;
 *   step 1's setup (src/PHT_MCMC_Aslett.c:279-297, :320-332): the packed
 *     parameter block of the next sweep (P, Pfull, exit data, candidate
 *     lists) with build_params's arithmetic; for ECS/DCS also the
 *     eigensystem (include/pht_eigen.h, in place of LAPACK dgeevx) and the
 *     spectral products;
 *   the checks of the host loop (processed count, z overflow), into an
 *     error word; flagged observations accumulated.
 * init = 1: iteration 0 (GibbsState's constructor: the start row, or the
 * prior mode / prior draw, and the forward-order diagonal).
 */
#include <hip/hip_runtime.h>

#include "pht_detmath.h"
#include "pht_eigen.h"
#include "pht_gamma.h"
#include "pht_kernels.h"
#include "pht_layout.h"

namespace pht {

/* one wavefront: the eigensolver's phases are separated by barriers, which
 * cost least within a single wave */
constexpr int kResThreads = 64;
constexpr int kResMaxM = (kMaxN + 1) * (kMaxN + 1);

/*
 * ECS/DCS: the spectral part of build_params (gibbs_host.cpp; the
 * reference's src/PHT_MCMC_Aslett.c:320-332) from this sweep's S, s, P in
 * the parameter block: the eigensystem (include/pht_eigen.h: refined from
 * the previous sweep's, the full QR at init or when that fails) in place of
 * LAPACK, then Q^-1 s and Q^-1 1 in the reference BLAS dgemv order
 * and the products QQs, W, QQ1, V, piQ with build_params's fma order.  A
 * failed eigensystem sets err bit 3 and leaves the previous sweep's spectral
 * data in place (finite values; the host reports the error after the run);
 * at init it writes diag(S) and identity vectors instead.
 */
/* the ECS starting point's W moments from the block's W and evals (as
 * build_params; W and evals complete before the call) */
__device__ __forceinline__ void wmoments(int n, const Layout &L, double *dv) {
  for (int j = threadIdx.x; j < n; j += blockDim.x) {
    double m[PHT_WMOM];
    pht_wmoments(n, dv + L.W + j, n, dv + L.evals, m);
    for (int k = 0; k < PHT_WMOM; k++) dv[L.Wm + j + k * n] = m[k];
  }
}

__device__ __forceinline__ void spectral(const ResidentArgs &r, int n, const Layout &L, double *dv) {
  __shared__ double eH[kMaxN * kMaxN], eV[kMaxN * kMaxN], eX[kMaxN * kMaxN], eG[2 * kMaxN * kMaxN];
  __shared__ double eQ[kMaxN * kMaxN], eort[kMaxN], escale[kMaxN], ed[kMaxN], eev[kMaxN], eQs[kMaxN], eQ1[kMaxN];
  const int tid = threadIdx.x, nt = blockDim.x;
  pht_eig_ws w;
  w.H = eH; w.V = eV; w.X = eX; w.G = eG; w.ort = eort; w.scale = escale; w.d = ed;
  /* Q^-1 lands in eX (free once the eigenvectors are back-transformed).
   * After the first sweep: refined from the previous sweep's eigensystem
   * (the block still holds it), the full QR only if that does not converge */
  int rc = r.init ? PHT_EIG_NOCONV : pht_eig_refine(n, dv + L.S, dv + L.Q, dv + L.Qinv, eev, eQ, eX, &w);
  if (rc != PHT_EIG_OK) rc = pht_eig(n, dv + L.S, eev, eQ, eX, &w);
  __syncthreads();
  if (rc != PHT_EIG_OK) {
    if (tid == 0) atomicOr(r.err, 8);
    if (r.init) {
      for (int e = tid; e < n * n; e += nt) {
        const double id = (e % n == e / n) ? 1.0 : 0.0;
        dv[L.Q + e] = id; dv[L.Qinv + e] = id;
        dv[L.QQs + e] = id; dv[L.W + e] = id; dv[L.QQ1 + e] = id; dv[L.V + e] = id;
      }
      for (int i = tid; i < n; i += nt) {
        dv[L.evals + i] = dv[L.S + i + i * n];
        dv[L.piQ + i] = (i == 0) ? 1.0 : 0.0;
      }
      __syncthreads();
      wmoments(n, L, dv);
    }
    return;
  }
  const double *Qi = eX, *s = dv + L.s, *S = dv + L.S, *P = dv + L.P;
  for (int e = tid; e < n * n; e += nt) {
    dv[L.Q + e] = eQ[e];
    dv[L.Qinv + e] = Qi[e];
  }
  for (int rr = tid; rr < n; rr += nt) { /* dgemv 'N' order: y = 0; y += x[c] A[:, c] */
    double qs = 0.0, q1 = 0.0;
    for (int c = 0; c < n; c++) {
      const double ts = 1.0 * s[c], t1 = 1.0 * 1.0;
      qs = qs + ts * Qi[rr + c * n];
      q1 = q1 + t1 * Qi[rr + c * n];
    }
    eQs[rr] = qs;
    eQ1[rr] = q1;
    dv[L.evals + rr] = eev[rr];
  }
  __syncthreads();
  for (int e = tid; e < n * n; e += nt) {
    const int j = e % n, i = e / n;
    const double Sjj = S[j + j * n];
    double wv = 0.0, v = 0.0;
    for (int k = 0; k < n; k++) {
      if (k != j) wv = fma(S[j + k * n] / (-Sjj), eQ[k + i * n], wv);
      v = fma(P[j + k * n], eQ[k + i * n], v);
    }
    dv[L.QQs + j + i * n] = eQ[j + i * n] * eQs[i];
    dv[L.W + j + i * n] = wv * eQs[i];
    dv[L.QQ1 + j + i * n] = eQ[j + i * n] * eQ1[i];
    dv[L.V + j + i * n] = v * eQ1[i];
  }
  for (int i = tid; i < n; i += nt) {
    double a = 0.0;
    for (int k = 0; k < n; k++) a = fma(dv[L.pi + k], eQ[k + i * n], a);
    dv[L.piQ + i] = a;
  }
  __syncthreads(); /* W and evals complete */
  wmoments(n, L, dv);
}

__global__ void __launch_bounds__(kResThreads) resident_update_kernel(ResidentArgs r, int iter) {
  __shared__ double theta[kResMaxM];
  pht_stage_math_tables();
  const int n = r.n, n1 = n + 1, m = r.m, tid = threadIdx.x;
  const int sl = stats_len(n);
  const unsigned long long *st = r.stats;
  /* a failed earlier sweep: stop updating (the host polls the error word and
   * stops enqueueing; the remaining sweeps are wasted, never reported) */
  if (!r.init && __hip_atomic_load(r.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) return;
  __syncthreads();
  if (!r.init) {
    if (tid == 0) {
      const unsigned long long *xw = st + 2 * n + n * n;
      if (r.expect >= 0 && (long long)xw[kXObs] != r.expect) atomicOr(r.err, 1);
      if (xw[kXOverflow] != 0ull) atomicOr(r.err, 2);
      if (xw[kXFlagged] != 0ull) atomicAdd(r.flagged, xw[kXFlagged]);
      if (r.unif && xw[kXUnifCap] != 0ull) atomicOr(r.err, 16); /* (word 6 is a DIAG counter in other samplers' diagnostic builds) */
    }
    for (int k = tid; k < m; k += blockDim.x) {
      long long nsum = 0;
      for (int e = r.nl_off[k + 1] - 1; e >= r.nl_off[k]; e--) nsum += (long long)st[2 * n + r.nl_idx[e]];
      double zsum = 0.0;
      for (int e = r.zl_off[k + 1] - 1; e >= r.zl_off[k]; e--) {
        const long long q = (long long)st[r.zl_i[e]];
        if (q < 0) atomicOr(r.err, 2);
        zsum += ((double)q * r.zs) / r.zl_c[e];
      }
      pht_stream s;
      pht_stream_init(&s, r.k0, r.k1, PHT_GAMMA_OBS(k), PHT_GAMMA_TAG, (uint32_t)iter);
      const double th = pht_rgamma_ctr(&s, r.nu[k] + (double)(int)nsum, 1.0 / (r.zeta[k] + zsum));
      if (!(th > 0.0) || !isfinite(th)) atomicOr(r.err, 4);
      r.res[iter + (long)k * r.it] = th;
      theta[k] = th;
    }
  } else {
    for (int k = tid; k < m; k += blockDim.x) {
      double th;
      if (r.start) {
        th = r.start[k];
      } else if (r.nu[k] > 1) {
        th = (r.nu[k] - 1.0) / r.zeta[k];
      } else {
        pht_stream s;
        pht_stream_init(&s, r.k0, r.k1, PHT_GAMMA_OBS(k), PHT_GAMMA_TAG, 0u);
        th = pht_rgamma_ctr(&s, r.nu[k], 1.0 / r.zeta[k]);
      }
      r.res[(long)k * r.it] = th;
      theta[k] = th;
    }
  }
  __syncthreads();
  /* TT cells of every parameter (each cell belongs to one parameter) */
  for (int k = tid; k < m; k += blockDim.x)
    for (int e = r.tl_off[k]; e < r.tl_off[k + 1]; e++) r.TT[r.tl_ij[e]] = theta[k] * r.tl_c[e];
  __syncthreads();
  /* the diagonal: the constructor sums a row forward, the update in reverse
   * list order (GibbsState, gibbs_host.cpp) */
  if (tid < n) {
    const int i = tid;
    double d = 0.0;
    if (r.init) {
      for (int e = r.dl_off[i]; e < r.dl_off[i + 1]; e++) d -= r.TT[r.dl_ij[e]];
    } else {
      for (int e = r.dl_off[i + 1] - 1; e >= r.dl_off[i]; e--) d -= r.TT[r.dl_ij[e]];
    }
    r.TT[i + i * n1] = d;
  }
  __syncthreads();
  /* the next sweep's parameter block (build_params without the eigensystem) */
  const Layout L = make_layout(n);
  double *dv = reinterpret_cast<double *>(r.params);
  int *iv = reinterpret_cast<int *>(r.params + L.ndouble * 8);
  if (tid < n) {
    const int i = tid;
    const double *TT = r.TT;
    double *P = dv + L.P, *Pf = dv + L.Pf;
    for (int j = 0; j < n; j++) dv[L.S + i + j * n] = TT[i + j * n1];
    const double si = TT[i + n * n1];
    dv[L.s + i] = si;
    dv[L.pi + i] = (i == 0) ? 1.0 : 0.0;
    const double Sii = TT[i + i * n1];
    double rsum, rsumfull = 0.0;
    for (int j = 0; j < n; j++) {
      const double v = -TT[i + j * n1] / Sii;
      P[i + j * n] = v;
      Pf[i + j * n] = v;
      rsumfull += v;
    }
    rsum = rsumfull - P[i + i * n];
    {
      const double v = -si / Sii;
      Pf[i + n * n] = v;
      rsumfull += v;
    }
    rsumfull -= Pf[i + i * n];
    Pf[i + i * n] = 0.0;
    P[i + i * n] = 0.0;
    for (int j = 0; j < n; j++) {
      P[i + j * n] = P[i + j * n] / rsum;
      Pf[i + j * n] = Pf[i + j * n] / rsumfull;
    }
    Pf[i + n * n] = Pf[i + n * n] / rsumfull;
    dv[L.logs + i] = si > 0.0 ? pht_log(si) : 0.0;
    const double sc = 1.0 / -Sii;
    dv[L.scale + i] = sc;
    dv[L.logscale + i] = pht_log(sc);
  }
  __syncthreads();
  if (tid < n) {
    const int j = tid;
    const double *P = dv + L.P, *Pf = dv + L.Pf, *S = dv + L.S;
    int a = 0, b = 0, c = 0;
    for (int k = 0; k < n; k++) {
      if (!(P[j + k * n] == 0.0)) iv[L.succP + j * n + a++] = k;
      if (k != j && !(S[j + k * n] == 0.0)) iv[L.succS + j * n + c++] = k;
    }
    for (int k = 0; k <= n; k++)
      if (!(Pf[j + k * n] == 0.0)) iv[L.succPf + j * (n + 1) + b++] = k;
    iv[L.nsuccP + j] = a;
    iv[L.nsuccPf + j] = b;
    iv[L.nsuccS + j] = c;
  }
  if (r.eig) {
    __syncthreads();
    spectral(r, n, L, dv);
  }
  /* the next sweep accumulates into a zeroed block */
  for (int k = tid; k < sl; k += blockDim.x) r.stats[k] = 0ull;
}

}  // namespace pht

extern "C" hipError_t pht_launch_resident_update(const pht::ResidentArgs *r, int iter, hipStream_t st) {
  using namespace pht;
  if (r->n < 1 || r->n > kMaxN || r->m < 1 || r->m > kResMaxM) return hipErrorInvalidValue;
  hipLaunchKernelGGL(resident_update_kernel, dim3(1), dim3(kResThreads), 0, st, *r, iter);
  return hipGetLastError();
}
