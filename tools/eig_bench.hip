/*
 * tools/eig_bench.hip — where the device eigensystem's time goes (the
 * resident chain's update kernel, include/pht_eigen.h), per phase, one
 * 64-thread workgroup as in pht_resident.hip.  Diagnostic only.
 *
 * build: hipcc -x hip --offload-arch=gfx950 -O3 -ffp-contract=off -std=c++17
 *        -Iinclude tools/eig_bench.hip -o tools/eig_bench
 * run (GPU box): tools/eig_bench  -> one JSON line per n
 */
#include <hip/hip_runtime.h>
#include <stdio.h>

#include "pht_eigen.h"

constexpr int kMaxN = 32;

__global__ void __launch_bounds__(64) eig_phases(int n, const double *S, long long *t, int reps) {
  __shared__ double eH[kMaxN * kMaxN], eV[kMaxN * kMaxN], eX[kMaxN * kMaxN], eG[2 * kMaxN * kMaxN];
  __shared__ double eQ[kMaxN * kMaxN], eort[kMaxN], escale[kMaxN], ed[kMaxN], eev[kMaxN];
  pht_eig_ws w;
  w.H = eH; w.V = eV; w.X = eX; w.G = eG; w.ort = eort; w.scale = escale; w.d = ed;
  long long acc[5] = {0, 0, 0, 0, 0};
  for (int r = 0; r < reps; r++) {
    __syncthreads();
    long long c0 = wall_clock64();
    for (int e = threadIdx.x; e < n * n; e += blockDim.x) eH[e] = S[e];
    __syncthreads();
    pht_eig_balance(n, eH, escale);
    __syncthreads();
    long long c1 = wall_clock64();
    pht_eig_hessenberg(n, eH, eV, eort);
    __syncthreads();
    long long c2 = wall_clock64();
    int rc = pht_eig_qr(n, eH, eV, ed);
    __syncthreads();
    long long c3 = wall_clock64();
    rc |= pht_eig(n, S, eev, eQ, eX, &w);
    __syncthreads();
    long long c4 = wall_clock64();
    acc[0] += c1 - c0;
    acc[1] += c2 - c1;
    acc[2] += c3 - c2;
    acc[3] += c4 - c3;
    acc[4] += rc;
  }
  if (threadIdx.x == 0)
    for (int k = 0; k < 5; k++) t[k] = acc[k];
}

static void bd_exit(int n, double *S) { /* column-major, as phasetype_amd/synth.py */
  for (int e = 0; e < n * n; e++) S[e] = 0.0;
  for (int i = 0; i < n; i++) {
    double row = (i == n - 1) ? 2.0 : 0.3;
    if (i + 1 < n) { S[i + (i + 1) * n] = 2.0; row += 2.0; }
    if (i > 0) { S[i + (i - 1) * n] = 0.5; row += 0.5; }
    S[i + i * n] = -row;
  }
}

int main() {
  int rate = 0;
  hipDeviceGetAttribute(&rate, hipDeviceAttributeWallClockRate, 0); /* kHz */
  const int ns[] = {3, 5, 10, 15, 20};
  for (int n : ns) {
    double hS[kMaxN * kMaxN];
    bd_exit(n, hS);
    double *dS;
    long long *dt, ht[5];
    hipMalloc(&dS, sizeof(double) * n * n);
    hipMalloc(&dt, sizeof ht);
    hipMemcpy(dS, hS, sizeof(double) * n * n, hipMemcpyHostToDevice);
    const int reps = 20;
    hipLaunchKernelGGL(eig_phases, dim3(1), dim3(64), 0, 0, n, dS, dt, 2); /* warm-up */
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0, 0);
    hipLaunchKernelGGL(eig_phases, dim3(1), dim3(64), 0, 0, n, dS, dt, reps);
    hipEventRecord(e1, 0);
    hipEventSynchronize(e1);
    float ms = 0.f;
    hipEventElapsedTime(&ms, e0, e1);
    hipMemcpy(ht, dt, sizeof ht, hipMemcpyDeviceToHost);
    const double us = 1e3 / rate / reps; /* wall-clock ticks -> us per rep */
    printf("{\"n\": %d, \"balance_us\": %.2f, \"hessenberg_us\": %.2f, \"qr_us\": %.2f, \"full_pht_eig_us\": %.2f, "
           "\"rc\": %lld, \"kernel_us_per_rep\": %.2f}\n",
           n, ht[0] * us, ht[1] * us, ht[2] * us, ht[3] * us, ht[4], ms * 1e3 / reps);
    hipFree(dS);
    hipFree(dt);
  }
  return 0;
}
