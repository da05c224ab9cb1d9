/*
 * pht_kernels_impl.h — the Gibbs "step 1" sweep kernels for gfx950
 * (templates; instantiated per compile-time n by pht_kernels_nt.hip, one
 * translation unit per n so that they compile in parallel).
 *
 * One lane = one observation (SURVEY.md §8e sharding).  A workgroup stages
 * the packed per-sweep parameter block (pht_layout.h) into LDS once, each
 * lane runs its observation's latent-path sampler (pht_device.h) and adds
 * its sufficient statistics into workgroup-level integer accumulators in
 * LDS (z as int64 fixed point, counts as u32), which are flushed to the
 * global int64 statistics block with integer atomics.  Integer sums are
 * order-independent, so the result is bit-identical for any grid, any
 * workgroup schedule and any number of GPUs.
 *
 * Replaces, per sweep: LJMA_MHsample_Bladt / LJMA_MHsample_Aslett2 /
 * LJMA_MHsample_Hobolth2 (src/PHT_MCMC_Aslett.c:325-333).
 */
#ifndef PHT_KERNELS_IMPL_H
#define PHT_KERNELS_IMPL_H
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <type_traits>
#include <mutex>

#include "pht_device.h"
#include "pht_ecs_round.h"
#include "pht_ecs_row.h"
#include "pht_env.h"
#include "pht_kernels.h"
#include "pht_unif.h"

namespace pht {

/* Statistics sink: workgroup accumulators in LDS (+ per-observation debug
 * rows in global memory when DEBUG). */
template <class T>
__device__ __forceinline__ void lds_add(PHT_LDS T *p, T v) {
  __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

/* A workgroup's accumulators into the global int64 block [zq n][B n][N n*n]
 * [extra] (after a __syncthreads).  z quanta are non-negative, so the sums
 * only grow: a block or global z total reaching 2^63 (which the host reads as
 * int64) counts in extra word kXOverflow, and the host fails the sweep rather
 * than use a wrapped sum (a data set whose censored paths run far past its
 * observed times can exceed pht_zexp's 2^11-fold headroom). */
__device__ __forceinline__ void flush_stats(unsigned long long *g, const PHT_LDS unsigned long long *zq,
                                            const PHT_LDS unsigned *Bc, const PHT_LDS unsigned *Nc,
                                            const PHT_LDS unsigned long long *xc, int n) {
  for (int k = threadIdx.x; k < n; k += blockDim.x) {
    const unsigned long long v = zq[k];
    if (v) {
      const unsigned long long old = atomicAdd(&g[k], v);
      if ((v >> 63) | ((old + v) >> 63) | (unsigned long long)(old + v < old))
        atomicAdd(&g[2 * n + n * n + kXOverflow], 1ull);
    }
    if (Bc[k]) atomicAdd(&g[n + k], (unsigned long long)Bc[k]);
  }
  for (int k = threadIdx.x; k < n * n; k += blockDim.x)
    if (Nc[k]) atomicAdd(&g[2 * n + k], (unsigned long long)Nc[k]);
  for (int k = threadIdx.x; k < kStatExtra; k += blockDim.x)
    if (xc[k]) atomicAdd(&g[2 * n + n * n + k], xc[k]);
}

template <bool DEBUG>
struct Sink {
  PHT_LDS unsigned long long *zq; /* LDS [n] */
  PHT_LDS unsigned *Bc;           /* LDS [n] */
  PHT_LDS unsigned *Nc;           /* LDS [n*n] */
  int n;
  double zscale;
  long long *dz;          /* debug row [n] */
  int *dN;                /* debug row [n*n] */
  int *dB, *dpre;
  PHT_LDS unsigned long long *xc = nullptr; /* LDS extra words (arms_diag) */
  __device__ __forceinline__ void z(int k, double d) {
    const long long q = (long long)rint(d * zscale);
    lds_add(&zq[k], (unsigned long long)q);
    if (DEBUG) dz[k] += q;
  }
  __device__ __forceinline__ void N(int i, int j) {
    lds_add(&Nc[i + j * n], 1u);
    if (DEBUG) dN[i + j * n] += 1;
  }
  __device__ __forceinline__ void start(int b) {
    lds_add(&Bc[b], 1u);
    if (DEBUG) *dB = b;
  }
  __device__ __forceinline__ void pre(int j) {
    if (DEBUG) *dpre = j;
  }
  /* DEBUG instantiations: a round in the general ARMS code, and whether its
   * envelope reached private memory (kXDbgGeneral, kXDbgPrivate).  Not in
   * PHT_STAMPS or PHT_ECS_DIAG builds, whose extra words 8 / 9 carry their
   * own counters (stamps; wave-rounds and active lane-rounds) */
  __device__ __forceinline__ void arms_diag(bool general, bool priv) {
#if !defined(PHT_STAMPS) && !defined(PHT_ECS_DIAG)
    if constexpr (DEBUG) {
      if (general) lds_add(&xc[kXDbgGeneral], 1ull);
      if (priv) lds_add(&xc[kXDbgPrivate], 1ull);
    }
#else
    (void)general; (void)priv;
#endif
  }
};

template <int NT>
__device__ __forceinline__ int nval(int n) { return NT > 0 ? NT : n; }

/* Position of a block's t-th claim in the persistent kernels: chunks of
 * kClaimChunk consecutive positions, block b taking chunks b, b + grid, ...
 * (the sorted order is walked by all blocks together; a wavefront's claims
 * are contiguous, so its y/gid loads coalesce).  Increasing in t. */
constexpr int kClaimChunk = 64;
__device__ __forceinline__ long claim_pos(long t, unsigned blk, unsigned nblk) {
  return ((t / kClaimChunk) * (long)nblk + blk) * kClaimChunk + (t % kClaimChunk);
}
__device__ __forceinline__ long claim_pos(long t) { return claim_pos(t, blockIdx.x, gridDim.x); }

/* ================================================================ MHRS */
/*
 * The attempt search (device spec: pht_device.h, mhrs_attempt).  Every
 * chain of every observation is a task, task = position * (1 + mhit) + c
 * (c = 0 the current path, 1..mhit the proposals; censored observations
 * have only c = 0).  The first successful attempt index of a task is found
 * in rounds of growing width, because an observation whose survival
 * probability is p needs ~1/p attempts and p is ~uniform over the data
 * (a few tasks per sweep need ~1e5-1e6 attempts, the reference's whole
 * run time; one lane per observation would serialise them):
 *   round 0  one lane per task, attempts [0, 16)
 *   round r  W = 16, 128, 2048, 32768, 131072 lanes per unresolved task,
 *            K = 8 (32) attempts each: attempt A0 + l + W k for lane l
 * (mhrs_search: jump-converged, the tasks' records lowered by atomicMin;
 * mhrs_compact collects the unresolved tasks between rounds).
 * Attempt streams are per (task, attempt), so the first success does not
 * depend on which lane tried what.  mhrs_finish then makes the MH decisions
 * (tag-0 stream) and replays the accepted attempt for the statistics.
 */
#ifndef PHT_MHRS_SCHED
#define PHT_MHRS_SCHED 0
#endif
#if PHT_MHRS_SCHED == 4
constexpr int kMhrsK0 = 8;
#elif PHT_MHRS_SCHED == 5
constexpr int kMhrsK0 = 32;
#elif PHT_MHRS_SCHED == 6
constexpr int kMhrsK0 = 24;
#else
constexpr int kMhrsK0 = 16;
#endif
struct MhrsRound {
  int W, K;
  uint32_t A0;
};
/* rounds 1-4 with K = 8 attempts per item (r04; r03 had K = 16 and half the
 * lanes per task): shorter items leave shorter round tails.  Interleaved A/B
 * (profiles/r04/mhrs_ab/sched_*.json): cfg4 -1 %, cfg5 -19 %; K = 4 or
 * round 0 at 8 attempts gained at cfg5 but lost 8-15 % at cfg4, K = 32 lost
 * 26 %.  (PHT_MHRS_SCHED selects the alternatives in variant builds.) */
constexpr MhrsRound kMhrsRounds[5] = {
#if PHT_MHRS_SCHED == 0
    {16, 8, 16}, {128, 8, 144}, {2048, 8, 1168}, {32768, 8, 17552}, {131072, 32, 279696}};
#elif PHT_MHRS_SCHED == 1 /* r03's schedule */
    {8, 16, 16}, {64, 16, 144}, {1024, 16, 1168}, {16384, 16, 17552}, {131072, 32, 279696}};
#elif PHT_MHRS_SCHED == 3 /* A/B: K = 4 */
    {32, 4, 16}, {256, 4, 144}, {4096, 4, 1168}, {65536, 4, 17552}, {131072, 32, 279696}};
#elif PHT_MHRS_SCHED == 4 /* A/B: round 0 K0 = 8, then K = 8 */
    {16, 8, 8}, {128, 8, 136}, {2048, 8, 1160}, {32768, 8, 17544}, {131072, 32, 279688}};
#elif PHT_MHRS_SCHED == 5 /* A/B: round 0 K0 = 32 */
    {16, 8, 32}, {128, 8, 160}, {2048, 8, 1184}, {32768, 8, 17568}, {131072, 32, 279712}};
#elif PHT_MHRS_SCHED == 6 /* A/B: round 0 K0 = 24 */
    {16, 8, 24}, {128, 8, 152}, {2048, 8, 1176}, {32768, 8, 17560}, {131072, 32, 279704}};
#else /* 2, A/B: longer items (K = 32), half the lanes per task */
    {4, 32, 16}, {32, 32, 144}, {512, 32, 1168}, {8192, 32, 17552}, {131072, 32, 279696}};
#endif

/* the MHRS search's per-row running sums of Pfull over the successor list
 * (mhrs_search_body), after the parameter block and the claim cursor; only
 * where they cost no occupancy (n <= 15: at n = 20 the block's LDS would
 * drop the search from 4 to 3 blocks per CU) */
__host__ __device__ inline int mhrs_cum_bytes(int n) { return n <= 15 ? n * (n + 1) * 8 : 0; }

template <int NT>
__device__ __forceinline__ Par<NT> stage_params(const SweepArgs &a, PHT_LDS unsigned char *lsm) {
  const int n = nval<NT>(a.n);
  const Layout L = make_layout(n);
  const unsigned long long *src = reinterpret_cast<const unsigned long long *>(a.params);
  PHT_LDS unsigned long long *dst = (PHT_LDS unsigned long long *)lsm;
  for (int k = threadIdx.x; k < L.bytes() / 8; k += blockDim.x) dst[k] = src[k];
  Par<NT> P;
  P.d = (const PHT_LDS double *)lsm;
  P.iv = (const PHT_LDS int *)(lsm + L.ndouble * 8);
  P.Lr = L;
  return P;
}

/*
 * Jump-converged search round: each lane works through items (task, l) of
 * the round, i.e. attempts A0 + l + W k (k < K) of the task, one JUMP per
 * loop iteration; a lane whose attempt ends starts its next attempt (or
 * item) in the next iteration, so a wavefront never waits for its longest
 * attempt.  A success lowers the task's record with atomicMin; a lane skips
 * attempts above the record (it tries its own attempts in increasing order,
 * so every attempt below the final record is tried: first success exact).
 * qin == nullptr: all tasks (round 0; the censored observations' proposal
 * tasks are marked resolved).  Unresolved tasks are collected afterwards by
 * mhrs_compact.
 */
template <int NT, int W, int K>
__device__ __forceinline__ void mhrs_search_body(const SweepArgs &a, uint32_t A0, const uint32_t *qin,
                                                 const unsigned *cin, unsigned blk, unsigned nblk) {
  extern __shared__ __align__(16) unsigned char smem[];
  const int T1 = 1 + a.mhit;
  const long total = (qin ? (long)(*cin) : a.count * T1) * W;
  /* round 0 zeroes the queue counters the later rounds' compactions add to
   * (they run after it on the stream; no separate fill per sweep) */
  if (qin == nullptr && blk == 0 && threadIdx.x < kMhrsCounters) a.mcnt[threadIdx.x] = 0u;
  /* block b owns claim chunks b, b + grid, ...: none when b * 64 >= total
   * (small shards, empty rounds): leave before staging anything */
  if ((long)blk * kClaimChunk >= total) return;
  const Par<NT> P = stage_params<NT>(a, (PHT_LDS unsigned char *)smem);
  /* items are claimed one at a time through an LDS cursor (claim_pos: the
   * block's 64-item chunks), so a lane whose item ends takes the next one
   * and the wavefront stays full until the round's items run out */
  PHT_LDS int *cursor = (PHT_LDS int *)((PHT_LDS unsigned char *)smem + make_layout(a.n).bytes());
  if (threadIdx.x == 0) *cursor = 0;
  pht_stage_math_tables();
  __syncthreads();
  const int n = P.n();
  /* the jump's categorical scan adds Pfull[j, k] over j's successor list in
   * order and stops at the first running sum >= its uniform: the running
   * sums, the same additions in the same order, are formed once per block
   * (row j: cum[j (n + 1) + q]), so the scan reads a sum and a successor
   * with no dependent load and no addition (the same state every time) */
  /* (round 0 only: in the later rounds the sums' loads cost 4 VGPRs, 7 -> 6
   * waves per SIMD at n = 10, and the rounds ran slower, cfg4 MHRS +3.4 %
   * against -3.0 % with round 0 alone; held to 7 waves +1.4 %, the
   * successor read only on a hit: neutral; profiles/r06/mhrs_cum/) */
  const bool usecum = mhrs_cum_bytes(n) > 0 && W == 1;
  PHT_LDS double *cum = (PHT_LDS double *)((PHT_LDS unsigned char *)cursor + 16);
  if (usecum) {
    if ((int)threadIdx.x < n) {
      const int jr = threadIdx.x, cnt = P.nsuccPf(jr);
      double sofar = 0.0;
      for (int q = 0; q < cnt; q++) {
        sofar += P.Pf(jr, P.succPf(jr, q));
        cum[jr * (n + 1) + q] = sofar;
      }
    }
    __syncthreads();
  }
  /* the start-state scan's result when it does not depend on the draw: pi's
   * first nonzero entry is >= 1 (pi = e_1 in every LJMA_Gibbs sweep,
   * src/PHT_MCMC_Aslett.c:190-193): the scan stops there for every uniform
   * in (0, 1), so an attempt takes that state (its uniform still drawn) */
  int pifix = -1;
  for (int i = 0; i < n; i++) {
    const double pv = P.pi(i);
    if (!(pv == 0.0)) {
      pifix = (pv >= 1.0) ? i : -1;
      break;
    }
  }
  pifix = __builtin_amdgcn_readfirstlane(pifix); /* (the same in every lane: a scalar) */
  long item = 0;
  /* item state */
  bool have = false;
  uint32_t task = 0, gid = 0;
  int c = 0, cens = 0, l = 0, k = 0;
  double y = 0.0;
  /* attempt state */
  bool inatt = false, fresh = false;
  uint32_t lrec = 0xffffffffu; /* the current task's record as last read */
  pht_stream r;
  double t = 0.0;
  int j = 0, lastj = 0, nj = 0;
  uint32_t att = 0;
#ifdef PHT_MHRS_DIAG
  /* diagnostic builds: wave iterations, lane iterations with an attempt, and
   * wave iterations with at most 8 such lanes (the round's tail), all rounds
   * (extra words 8, 9, 10) and rounds 0 / 1 (11, 12 / 13, 14) */
  unsigned long long d_wit = 0, d_lit = 0, d_tail = 0;
#endif
#ifdef PHT_MHRS_STAMPS
  /* diagnostic builds: wave cycles in the refill code (claim, item loads,
   * stream init) and in the rest of the iteration, wave iterations, and the
   * refill cycles and count of iterations in which a lane claimed an item
   * (extra words 8..12; 13, 14: refill and all cycles of round 0) */
  unsigned long long s_ref = 0, s_rest = 0, s_it = 0, s_cref = 0, s_cit = 0;
  unsigned long long s_last = __builtin_amdgcn_s_memtime();
  bool s_claimed = false;
#endif
  for (;;) {
#ifdef PHT_MHRS_STAMPS
    s_claimed = false;
#endif
    while (!inatt) { /* next attempt of this item, or the next item */
      if (!have) {
        if (item >= total) break;
        item = claim_pos(__hip_atomic_fetch_add(cursor, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP), blk, nblk);
        if (item >= total) break;
#ifdef PHT_MHRS_STAMPS
        s_claimed = true;
#endif
        const long q = item / W;
        l = (int)(item % W);
        task = qin ? qin[q] : (uint32_t)q;
        const long pos = task / T1;
        c = (int)(task % T1);
        /* the item's three loads issued together (one memory latency per
         * claim, not two) */
        cens = a.cens[pos];
        y = a.y[pos];
        gid = a.gid[pos];
        if (c > 0 && cens) { /* censored observations have no proposals */
          if (l == 0) a.mbest[task] = 0u;
          continue;
        }
        k = 0;
        have = true;
        lrec = 0xffffffffu;
      }
      if (k >= K) {
        /* round 0 (one lane per task, every task): no success in its K
         * attempts -- this lane writes the task's record, so round 0 leaves
         * every record defined and the sweep needs no fill of mbest */
        if constexpr (W == 1) a.mbest[task] = kMhrsUnresolved;
        have = false;
        continue;
      }
      att = A0 + (uint32_t)l + (uint32_t)W * (uint32_t)k;
      k++;
      /* a record below att means another lane of the task found an earlier
       * success; with one lane per task (round 0) only this lane writes the
       * record, and it stops at its own success: no load needed */
      bool stop = att >= (uint32_t)kMhrsMaxAtt;
      /* the task's record as this lane last read it (below, once per
       * iteration): no global load on the refill path (r06: MHRS cfg4
       * -1.7 %, cfg5 -1.5 %, profiles/r06/mhrs_lrec/); a record that moved
       * since drops the attempt after its first jump instead */
      if constexpr (W > 1) stop = stop || (lrec >> 8) < att;
      if (stop) {
        have = false;
        continue;
      }
      /* the stream's blocks come from the converged top-up below */
      pht_stream_init(&r, a.k0, a.k1, gid, mhrs_tag(c, att), a.sweep);
      fresh = true;
      inatt = true;
    }
    if (!__any(inatt)) break;
#ifdef PHT_MHRS_STAMPS
    unsigned long long s_t1;
    {
      /* (y, gid, cens of a claimed item are consumed in the refill code or
       * by the stream's first block: make the stamp wait for them) */
      __builtin_amdgcn_s_waitcnt(0);
      s_t1 = __builtin_amdgcn_s_memtime();
      s_ref += s_t1 - s_last;
      s_it++;
      if (__any(s_claimed)) { s_cref += s_t1 - s_last; s_cit++; }
    }
#endif
#ifdef PHT_MHRS_DIAG
    {
      const unsigned act = (unsigned)__popcll(__ballot(inatt));
      d_wit++;
      d_lit += act;
      d_tail += (act <= 8u) ? 1ull : 0ull;
    }
#endif
    /* converged Philox: every lane with an attempt generates its next block
     * here, once per iteration, instead of inside the draws (where only the
     * lanes whose buffer ran dry would, one draw site at a time); a step
     * uses at most 4 words (start draw + a jump's 3), and the buffer then
     * holds >= 4 (same word sequence either way) */
#ifdef PHT_MHRS_PHILOX_UNROLL
    if (inatt) pht_stream_topup_unrolled(&r);
#else
    if (inatt) pht_stream_topup(&r);
#endif
    /* several lanes per task (rounds 1-5): an attempt above the task's
     * record can no longer be the first success; the record is read here and
     * tested after the jump (the load's latency hidden by the jump), and such
     * an attempt is dropped mid-way with the lane's remaining ones (all
     * larger).  The first success is unchanged: every attempt below the
     * final record still runs to its end */
    uint32_t rec = 0xffffffffu;
    if constexpr (W > 1) {
      if (inatt && !fresh) rec = __hip_atomic_load(&a.mbest[task], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (inatt && !fresh) lrec = rec;
    }
    if (inatt && fresh) { /* start state of the attempt */
      const double target = pht_next_u(&r);
      int B2 = pifix + 1;
      if (pifix < 0) {
        double sofar = 0.0;
        B2 = 0;
        while (sofar < target && B2 <= n) sofar += (B2 < n ? P.pi(B2) : 0.0), B2++;
      }
      j = lastj = B2 - 1;
      t = 0.0;
      nj = 0;
      fresh = false;
    }
    if (inatt) {
      /* one jump of mhrs_attempt (pht_device.h) */
      if ((t < y && j < n) || (cens && j < n)) {
        if (nj++ >= kMaxJumps) {
          t = y;
          j = n; /* ends the attempt; t >= y: accepted as in mhrs_attempt */
        } else {
          t = t + dev_rexp(r, P.scale(j)) /* = 1.0 / -S_jj, per sweep (pht_layout.h) */;
          const double target = pht_next_u(&r);
          const int cnt = P.nsuccPf(j);
          int sel = n + 1;
          if (usecum) {
            for (int q = 0; q < cnt; q++) {
              const double cq = cum[j * (n + 1) + q];
              const int kk = P.succPf(j, q);
              if (!(cq < target)) {
                sel = kk;
                break;
              }
            }
          } else {
            double sofar = 0.0;
            for (int q = 0; q < cnt; q++) {
              const int kk = P.succPf(j, q);
              sofar += P.Pf(j, kk);
              if (!(sofar < target)) {
                sel = kk;
                break;
              }
            }
          }
          j = sel;
          if ((t < y && j < n) || (cens && j < n)) lastj = j;
        }
      }
      if (!((t < y && j < n) || (cens && j < n))) {
        inatt = false;
        if (!(t < y) && lastj < n && P.s(lastj) > 0.0) {
          /* one lane per task (round 0): the task's only writer, stopping at
           * its first success, so a plain store is the atomicMin's result
           * (device-scope atomics go to memory: 48 MB of writes per round-0
           * launch at cfg4, profiles/r05/mhrs/pmc_cfg4_mhrs_per_kernel.json) */
          if constexpr (W == 1) a.mbest[task] = mhrs_pack(att, lastj);
          else atomicMin(&a.mbest[task], mhrs_pack(att, lastj));
          have = false; /* this lane's further attempts are larger */
        }
      }
      if constexpr (W > 1) {
        if (inatt && (rec >> 8) < att) {
          inatt = false;
          have = false;
        }
      }
    }
#ifdef PHT_MHRS_STAMPS
    {
      __builtin_amdgcn_s_waitcnt(0);
      const unsigned long long t2 = __builtin_amdgcn_s_memtime();
      s_rest += t2 - s_t1;
      s_last = t2;
    }
#endif
  }
#ifdef PHT_MHRS_STAMPS
  if ((threadIdx.x & 63u) == 0u) {
    unsigned long long *x = a.stats + 2 * a.n + a.n * a.n;
    atomicAdd(&x[8], s_ref);
    atomicAdd(&x[9], s_rest);
    atomicAdd(&x[10], s_it);
    atomicAdd(&x[11], s_cref);
    atomicAdd(&x[12], s_cit);
    if (A0 == 0u) { atomicAdd(&x[13], s_ref); atomicAdd(&x[14], s_ref + s_rest); }
  }
#endif
#ifdef PHT_MHRS_DIAG
  if ((threadIdx.x & 63u) == 0u) {
    unsigned long long *x = a.stats + 2 * a.n + a.n * a.n;
    atomicAdd(&x[8], d_wit);
    atomicAdd(&x[9], d_lit);
    atomicAdd(&x[10], d_tail);
    if (A0 == 0u) { atomicAdd(&x[11], d_wit); atomicAdd(&x[12], d_lit); }
    if (A0 == kMhrsRounds[0].A0) { atomicAdd(&x[13], d_wit); atomicAdd(&x[14], d_lit); }
  }
#endif
}

template <int NT, int W, int K>
__global__ void __launch_bounds__(kBlock) mhrs_search(SweepArgs a, uint32_t A0, const uint32_t *qin,
                                                      const unsigned *cin) {
  mhrs_search_body<NT, W, K>(a, A0, qin, cin, blockIdx.x, gridDim.x);
}

/* tasks of qin still unresolved -> qout */
__device__ __forceinline__ void mhrs_compact_body(const SweepArgs &a, const uint32_t *qin, const unsigned *cin,
                                                  uint32_t *qout, unsigned *cout, unsigned blk, unsigned nblk) {
  /* ONE counter atomic per block: block b owns a contiguous range of the
   * queue, counts its unresolved tasks, reserves that many slots, then
   * writes them (wavefront ballots, LDS offsets).  A counter atomic per task
   * or per wavefront (device scope, one address) made the first compaction
   * ~0.1 ms at cfg4 (profiles/r04/mhrs_ab/).  The queue's order does not
   * matter: attempt streams are per (task, attempt). */
  __shared__ unsigned wsum[kBlock / 64], sbase;
  const long cnt = qin ? (long)(*cin) : a.count * (1 + a.mhit);
  const long per = ((cnt + nblk - 1) / nblk + kBlock - 1) / kBlock * kBlock;
  const long lo = (long)blk * per, hi = (lo + per < cnt) ? lo + per : cnt;
  if (lo >= hi) return; /* (uniform per block) */
  const unsigned lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
  auto unres = [&](long q, uint32_t &task) {
    task = qin ? qin[q] : (uint32_t)q;
    return a.mbest[task] == kMhrsUnresolved;
  };
  unsigned mine = 0;
  for (long q = lo + threadIdx.x; q < hi; q += kBlock) {
    uint32_t task;
    mine += unres(q, task) ? 1u : 0u;
  }
  for (int o = 32; o > 0; o >>= 1) mine += __shfl_xor(mine, o);
  if (lane == 0) wsum[wv] = mine;
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned tot = 0;
    for (int w = 0; w < kBlock / 64; w++) tot += wsum[w];
    sbase = tot ? atomicAdd(cout, tot) : 0u;
  }
  __syncthreads();
  unsigned base = sbase;
  for (long q0 = lo; q0 < hi; q0 += kBlock) {
    const long q = q0 + threadIdx.x;
    uint32_t task = 0;
    const bool un = (q < hi) && unres(q, task);
    const unsigned long long m = __ballot(un);
    __syncthreads(); /* (the previous step's wsum reads are done) */
    if (lane == 0) wsum[wv] = (unsigned)__popcll(m);
    __syncthreads();
    unsigned off = base;
    for (unsigned w = 0; w < wv; w++) off += wsum[w];
    if (un) qout[off + (unsigned)__popcll(m & ((1ull << lane) - 1ull))] = task;
    for (int w = 0; w < kBlock / 64; w++) base += wsum[w];
  }
}
/* (templated only to keep one copy per pht_kernels_nt.hip unit) */
template <int NT>
__global__ void __launch_bounds__(kBlock) mhrs_compact(SweepArgs a, const uint32_t *qin, const unsigned *cin,
                                                       uint32_t *qout, unsigned *cout) {
  mhrs_compact_body(a, qin, cin, qout, cout, blockIdx.x, gridDim.x);
}

/* LJMA_MHsample_Bladt's MH step over the chains' first successes, then the
 * accepted attempt replayed with recording.  ln.neval <- attempts made. */
template <int NT, class Sink>
__device__ __forceinline__ void mhrs_finish(const Par<NT> &P, const SweepArgs &a, long i, double y, int cens,
                                            Lane &ln, Sink &sk) {
  const int T1 = 1 + a.mhit;
  const uint32_t gid = a.gid[i];
  auto first = [&](int c, int &pre) -> uint32_t {
    const uint32_t b = a.mbest[i * T1 + c];
    if (b != kMhrsUnresolved) {
      pre = (int)(b & 0xffu);
      return b >> 8;
    }
    /* no success within the cap: the last attempt, flagged */
    ln.flags |= kFlagMhrsCap;
    const uint32_t att = (uint32_t)kMhrsMaxAtt - 1u;
    (void)mhrs_try<NT>(P, y, cens, a.k0, a.k1, gid, a.sweep, c, att, pre);
    return att;
  };
  int cpre = 0;
  uint32_t catt = first(0, cpre);
  uint32_t natt = catt + 1u;
  int cc = 0;
  if (cens == 0) {
    for (int k = 1; k <= a.mhit; k++) {
      int ppre = 0;
      const uint32_t patt = first(k, ppre);
      natt += patt + 1u;
      const double U = dev_u(ln.r);
      if (U < P.s(ppre) / P.s(cpre)) {
        cpre = ppre;
        catt = patt;
        cc = k;
      }
    }
  }
  pht_stream r;
  pht_stream_init(&r, a.k0, a.k1, gid, mhrs_tag(cc, catt), a.sweep);
  int pre2 = 0;
  (void)mhrs_attempt<NT, true>(P, y, cens, r, pre2, ln.flags, ln.njump, sk);
  sk.pre(cpre);
  ln.neval = (int)natt;
}

/* MHRS's MH decisions and the accepted attempt's replay, one observation per
 * lane on a persistent grid: a lane claims the next 64-position chunk slot
 * through an LDS cursor as soon as its observation is done. */
template <int NT, bool DEBUG>
__device__ __forceinline__ void mhrs_finish_body(const SweepArgs &a, unsigned blk, unsigned nblk) {
  extern __shared__ __align__(16) unsigned char smem[];
  const int n = nval<NT>(a.n);
  const Layout L = make_layout(n);
  const int pbytes = L.bytes();
  /* stage the parameter block */
  {
    const unsigned long long *src = reinterpret_cast<const unsigned long long *>(a.params);
    PHT_LDS unsigned long long *dst = (PHT_LDS unsigned long long *)smem;
    for (int k = threadIdx.x; k < pbytes / 8; k += blockDim.x) dst[k] = src[k];
  }
  PHT_LDS unsigned char *lsm = (PHT_LDS unsigned char *)smem;
  PHT_LDS unsigned long long *zq = (PHT_LDS unsigned long long *)(lsm + pbytes);
  PHT_LDS unsigned long long *xc = zq + n; /* kStatExtra counters */
  PHT_LDS unsigned *Bc = (PHT_LDS unsigned *)(xc + kStatExtra);
  PHT_LDS unsigned *Nc = Bc + n;
  PHT_LDS int *cursor = (PHT_LDS int *)(Nc + n * n);
  pht_stage_math_tables();
  for (int k = threadIdx.x; k < n + kStatExtra; k += blockDim.x) zq[k] = 0ull;
  for (int k = threadIdx.x; k < n + n * n; k += blockDim.x) Bc[k] = 0u;
  if (threadIdx.x == 0) *cursor = 0;
  __syncthreads();

  Par<NT> P;
  P.d = (const PHT_LDS double *)lsm;
  P.iv = (const PHT_LDS int *)(lsm + L.ndouble * 8);
  P.Lr = L;

  for (;;) {
    const long t = __hip_atomic_fetch_add(cursor, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    const long p = claim_pos(t, blk, nblk);
    if (p >= a.count) break;
    const long i = a.begin + p;
    Lane ln;
    pht_stream_init(&ln.r, a.k0, a.k1, a.gid[i], 0u, a.sweep);
    ln.flags = 0; ln.neval = 0; ln.nbrent = 0; ln.njump = 0;
    Sink<DEBUG> sk{zq, Bc, Nc, n, a.zscale, nullptr, nullptr, nullptr, nullptr};
    if (DEBUG) {
      sk.dz = a.dbg_zq + i * n;
      sk.dN = a.dbg_N + i * n * n;
      sk.dB = a.dbg_B + i;
      sk.dpre = a.dbg_pre + i;
    }
    mhrs_finish<NT>(P, a, i, a.y[i], a.cens[i], ln, sk);
    /* draws: stream words + attempts (ln.neval, see mhrs_finish) */
    const uint32_t nd = pht_stream_pos(&ln.r) + (uint32_t)ln.neval;
    if (DEBUG) {
      a.dbg_flags[i] = ln.flags;
      a.dbg_ndraw[i] = nd;
    }
    lds_add(&xc[0], 1ull);
    lds_add(&xc[1], (unsigned long long)ln.neval);
    if (ln.flags) lds_add(&xc[2], 1ull);
    lds_add(&xc[3], (unsigned long long)nd);
    lds_add(&xc[4], (unsigned long long)ln.njump);
    lds_add(&xc[5], (unsigned long long)ln.nbrent);
  }
  __syncthreads();
  /* flush: [zq n][B n][N n*n][extra] */
  flush_stats(a.stats, zq, Bc, Nc, xc, n);
}

/* MHRS's finish (MH decisions + the accepted attempt replayed) on a
 * persistent grid: one block per observation chunk of 256 meant ~3,900
 * blocks at 10^6 observations, each adding its n + n^2 + extra statistics
 * words into the same global block (~500k same-address atomics per sweep) */
template <int NT, bool DEBUG>
__global__ void __launch_bounds__(kBlock) mhrs_finish_kernel(SweepArgs a) {
  mhrs_finish_body<NT, DEBUG>(a, blockIdx.x, gridDim.x);
}

/* waves per SIMD the persistent kernel is compiled for: the DCS kernel at
 * n = 10 needs 410 VGPRs (one wave); held to two waves it spills 251 VGPRs
 * outside its Brent loop and runs 11 % faster (cfg5-shaped n = 10: 3.09 ->
 * 2.75 ms).  At n = 15 two waves are 19 % slower (5.65 -> 6.74 ms), so only
 * n = 10 is held (tools/ab.py; PHT_PERSIST_WAVES=k forces every kernel). */
#ifndef PHT_PERSIST_WAVES
#define PHT_PERSIST_WAVES 0
#endif
template <int NT, int METHOD>
constexpr int persist_waves() {
  return PHT_PERSIST_WAVES > 0 ? PHT_PERSIST_WAVES : ((NT == 10 && METHOD == kMethodDCS) ? 2 : 1);
}
/* LDS bytes a workgroup needs: parameter block + accumulators (+ cursor) */
static int smem_bytes(int n) {
  const Layout L = make_layout(n);
  return L.bytes() + (n + kStatExtra) * 8 + (n + n * n) * 4 + 4;
}

/*
 * Per-kernel launch configuration, shared by every host thread that
 * launches the kernel (pht_gibbs_run_chains runs chains from several
 * threads), kept per device: LJMA_Gibbs drives every visible GPU from one
 * process, and both the dynamic-LDS limit (hipFuncSetAttribute) and the
 * device properties are per device.  The limit is raised whenever a larger
 * footprint is launched on that device (the runtime-n kernels see several n
 * per process) and the occupancy is queried again after it; a mutex orders
 * all of it.
 */
constexpr int kMaxDevices = 64;
struct LaunchCfg {
  struct Dev {
    int occ = -1, cus = 0, lds = 0, occ_sm = -1;
  };
  std::mutex m;
  Dev d[kMaxDevices];
};

static hipError_t launch_config(LaunchCfg &cfg, const void *kernel, int sm, int *occ, int *cus) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDevices) return hipErrorInvalidDevice;
  std::lock_guard<std::mutex> lock(cfg.m);
  LaunchCfg::Dev &c = cfg.d[dev];
  if (sm > c.lds) {
    if (hipFuncSetAttribute(kernel, hipFuncAttributeMaxDynamicSharedMemorySize, sm) != hipSuccess)
      return hipErrorUnknown;
    c.lds = sm;
  }
  if (c.occ < 0 || sm != c.occ_sm) {
    c.occ_sm = sm;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, dev) != hipSuccess) return hipErrorUnknown;
    int b = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, kernel, kBlock, sm) != hipSuccess || b < 1) b = 1;
    c.cus = prop.multiProcessorCount;
    c.occ = b;
  }
  *occ = c.occ;
  *cus = c.cus;
  return hipSuccess;
}

/*
 * ECS exact observations, persistent lanes.  Block b owns chunks of 64
 * positions (claim_pos) of the launch range and hands them to its lanes
 * through an LDS cursor: a lane that finishes a path takes the
 * next observation at once, so the expensive ARMS phase runs with (almost)
 * all lanes of a wavefront active instead of waiting for the longest path.
 * The ARMS envelope's x/y live in LDS (EnvLdsXY), lane-interleaved.
 */
#ifndef PHT_SLOW_K
#define PHT_SLOW_K 15
#endif
/* envelope points kept in LDS (lane-interleaved x and y; beyond them the
 * general ARMS code's rare long envelopes go to private memory).  At
 * n >= 15 only the converged round's 13 (with the compact parameter prefix
 * below, two blocks per CU then fit at n = 15 and 20) */
template <int NT>
constexpr int ecs_env_k() { return NT >= 15 ? 13 : PHT_SLOW_K; }

/* The ECS exact-path kernels (one-lane, rows, chains, hand-off) stage into
 * LDS only what they read: the parameter block's double prefix [0, necs)
 * (the n-vectors, S, P, QQs, W, the W moments) and P's successor lists,
 * which follow it in LDS (P.iv).  The full block (22 KB at n = 15) plus the
 * envelope region and the math tables exceeded half of the CU's 160 KB, so
 * the n = 15 and 20 kernels ran one block, i.e. one wave per SIMD (r04). */
__host__ __device__ inline int ecs_param_bytes(const Layout &L) {
  return L.necs * 8 + (((L.n + L.n * L.n) * 4 + 15) & ~15);
}
__device__ __forceinline__ void stage_ecs_params(const SweepArgs &a, PHT_LDS unsigned char *lsm, const Layout &L) {
  const unsigned long long *g = reinterpret_cast<const unsigned long long *>(a.params);
  PHT_LDS unsigned long long *d = (PHT_LDS unsigned long long *)lsm;
  for (int k = threadIdx.x; k < L.necs; k += blockDim.x) d[k] = g[k];
  const int *gi = reinterpret_cast<const int *>(reinterpret_cast<const unsigned char *>(a.params) + L.ndouble * 8);
  PHT_LDS int *di = (PHT_LDS int *)(lsm + L.necs * 8);
  const int ni = L.n + L.n * L.n; /* nsuccP, succP: the int region's prefix */
  for (int k = threadIdx.x; k < ni; k += blockDim.x) di[k] = gi[k];
}

#ifndef PHT_ECS_WAVES
#define PHT_ECS_WAVES 0
#endif
/* blk / nblk: the block's index and the block count of its chain's grid
 * (blockIdx.x / gridDim.x, except in ecs_chains_kernel) */
template <int NT, bool DEBUG>
__device__ __forceinline__ void ecs_exact_body(const SweepArgs &a, unsigned blk, unsigned nblk) {
  extern __shared__ __align__(16) unsigned char smem[];
  const int n = nval<NT>(a.n);
  const Layout L = make_layout(n);
  const int pbytes = ecs_param_bytes(L);
  stage_ecs_params(a, (PHT_LDS unsigned char *)smem, L);
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
  P.iv = (const PHT_LDS int *)(lsm + L.necs * 8);
  P.Lr = L;
  /* the envelope's x and y in LDS (lane-interleaved) up to PHT_SLOW_K
   * points; cum lives in registers within a round (pht_ecs_round.h) and in
   * private memory for the general ARMS code */
  EnvLdsXY<ecs_env_k<NT>(), kBlock> env;
  double spill[2 * EnvLdsXY<ecs_env_k<NT>(), kBlock>::kSpill];
  double cumv[100];
  env.bind(envl, threadIdx.x, (PHT_PRIV double *)spill, (PHT_PRIV double *)cumv);
  Sink<DEBUG> sk{zq, Bc, Nc, n, a.zscale, nullptr, nullptr, nullptr, nullptr, xc};
  Lane ln;
#ifdef PHT_STAMPS
  ln.st_last = __builtin_amdgcn_s_memtime();
  for (int q = 0; q < 15; q++) ln.st_acc[q] = 0ull;
  ln.st_rounds = 0ull;
#endif
  EcsLane<NT> st;
  /* a lane without an observation still runs the converged round code
   * (its results unused): keep its state index in range */
  st.j = 0;
  st.yt = 0.0;
  long pos = 0;
  bool have = false, done = false;
  /* the lane's next observation is claimed and its (y, gid) loaded one
   * observation ahead, so a refill never waits on global memory */
  auto claim = [&]() -> long {
    const long t = __hip_atomic_fetch_add(cursor, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    /* spread: a lane's first claim is lane-major over the grid's
     * wavefronts, so the longest paths (the first positions) go one per
     * wavefront instead of 64 to wavefront 0 */
    if (a.spread && t < kBlock)
      return (long)(t & 63) * ((long)nblk * (kBlock / 64)) + (long)(t >> 6) * nblk + blk;
    return claim_pos(t, blk, nblk);
  };
  long nextp = claim();
  double ny = 0.0;
  uint32_t ngid = 0;
  if (nextp < a.count) {
    ny = a.y[a.begin + nextp];
    ngid = a.gid[a.begin + nextp];
  }
  /* a lane whose sojourn proposal was rejected finishes that jump one ARMS
   * step per round (ecs_jump_resume) while the other lanes go on */
  ArmsPend pd;
  bool pend = false;
  const double lam = lam_max(P);
  /* Philox blocks generated ahead at converged points, one per lane per
   * point: the current stream's next block, or else block 0 of the next
   * observation (so a new observation never runs Philox divergently) */
  pht_u32x4 nxw;
  bool nxReady = false;
  auto topup = [&](bool act) {
    const bool cur = act && have && !ln.r.nb;
    const bool nxt = act && !cur && !nxReady && nextp < a.count;
    if (cur || nxt) {
      pht_u32x4 c;
      c.v[0] = cur ? ln.r.obs : ngid;
      c.v[1] = cur ? ln.r.tag : 0u;
      c.v[2] = a.sweep;
      c.v[3] = cur ? ln.r.blk : 0u;
#ifdef PHT_ECS_PHILOX_UNROLL
      const pht_u32x4 w = pht_philox4x32_10_unrolled(c, a.k0, a.k1);
#else
      const pht_u32x4 w = pht_philox4x32_10(c, a.k0, a.k1);
#endif
      if (cur) {
        ln.r.b0 = w.v[0]; ln.r.b1 = w.v[1]; ln.r.b2 = w.v[2]; ln.r.b3 = w.v[3];
        ln.r.nb = 1;
        ln.r.blk++;
      } else {
        nxw = w;
        nxReady = true;
      }
    }
  };
  /* per-lane observation counters, flushed once at the end */
  unsigned c_obs = 0, c_neval = 0, c_flag = 0, c_nd = 0, c_jump = 0;
#ifdef PHT_ECS_DIAG
  unsigned c_big = 0, c_wbig = 0, c_wround = 0, c_act = 0;
  unsigned c_start = 0, c_pend = 0, c_new = 0, c_wnew = 0, c_wpend = 0, c_w13 = 0;
#endif
  for (;;) {
    bool need = false;
    topup(!pend);
    int nnew = 0; /* observations started by this lane in this round */
    while (!done && !pend) {
      if (!have) {
        if (nextp >= a.count) {
          done = true;
          break;
        }
        /* newcap: a lane starts at most that many observations per round
         * (a path that ends at its first absorb test leaves the lane idle
         * until the next round instead of running phase A again) */
        if (a.newcap > 0 && nnew >= a.newcap) break;
        nnew++;
        pos = a.begin + nextp;
        const double yobs = ny;
        const uint32_t gobs = ngid;
        nextp = claim();
        if (nextp < a.count) {
          ny = a.y[a.begin + nextp];
          ngid = a.gid[a.begin + nextp];
        }
        if (nxReady) pht_stream_init_block0(&ln.r, a.k0, a.k1, gobs, 0u, a.sweep, nxw);
        else pht_stream_init(&ln.r, a.k0, a.k1, gobs, 0u, a.sweep);
        nxReady = false;
        ln.flags = 0; ln.neval = 0; ln.nbrent = 0; ln.njump = 0;
        if (DEBUG) {
          sk.dz = a.dbg_zq + pos * n;
          sk.dN = a.dbg_N + pos * n * n;
          sk.dB = a.dbg_B + pos;
          sk.dpre = a.dbg_pre + pos;
        }
        ecs_begin(P, yobs, ln, sk, st);
        have = true;
        /* its first absorb test runs inside the round, after the initial
         * envelope whose vector gives its E0 (pht_ecs_round.h) */
        st.fold = true;
        need = true;
        break;
      }
      if (ecs_try_absorb(P, ln, sk, st)) {
        const uint32_t nd = pht_stream_pos(&ln.r);
        if (DEBUG) {
          a.dbg_flags[pos] = ln.flags;
          a.dbg_ndraw[pos] = nd;
        }
        c_obs++;
        c_neval += ln.neval;
        c_flag += ln.flags ? 1u : 0u;
        c_nd += nd;
        c_jump += ln.njump;
        have = false;
        continue;
      }
      need = true;
      break;
    }
    PHT_STAMP(ln, 0);
    /* leave only when every lane is done: a lane that hit the newcap of
     * this round (its new observation ended at its first absorb test) has
     * its next observation claimed and starts it in the next round, even
     * when no lane of the wavefront has a sojourn to sample now (r02 fix:
     * such wavefronts used to leave, dropping those observations).  Such a
     * round runs ecs_round with no lane active (a rare case), which keeps
     * the loop's single back-edge: a `continue` here changed the register
     * allocation (n = 10: 285 VGPRs, one wave per SIMD) */
    if (!__any(need) && !__any(pend) && !__any(!done)) break;
    /* the waves carrying the longest remaining paths issue first, so the
     * sweep's critical path is not slowed by the others */
    if (a.hoty > 0.0) {
      if (__any(have && st.yt > a.hoty)) __builtin_amdgcn_s_setprio(3);
      else __builtin_amdgcn_s_setprio(0);
    }
#ifdef PHT_STAMPS
    ln.st_rounds++;
#endif
#ifdef PHT_ECS_DIAG
    /* diagnostic builds: lane-rounds in the general ARMS code (envelope
     * beyond kRoundCap), wave-rounds with at least one such lane, wave-rounds,
     * lane-rounds with a sojourn to sample (extra words 6, 7, 8, 9) */
    {
      const bool bigl = pend && env.cnt + 2 > kRoundCap;
      c_big += bigl ? 1u : 0u;
      c_act += (need || pend) ? 1u : 0u;
      c_start += need ? 1u : 0u;
      c_pend += pend ? 1u : 0u;
      c_new += (nnew > 0) ? 1u : 0u;
      const bool wnew = __any(nnew > 0), wpend = __any(pend);
      /* the converged blocks run at 13 points this round (a pending lane
       * with 11 points before its insert) */
      const bool w13 = __any(pend && !bigl && env.cnt + 2 > 11);
      if ((threadIdx.x & 63) == 0) {
        c_w13 += w13 ? 1u : 0u;
        c_wbig += __any(bigl) ? 1u : 0u;
        c_wround++;
        c_wnew += wnew ? 1u : 0u;
        c_wpend += wpend ? 1u : 0u;
      }
    }
#endif
    topup(need || pend);
    PHT_STAMP(ln, 12);
    bool obsdone;
    ecs_round(P, ln, env, sk, st, need, pend, pd, lam, obsdone);
    if (obsdone) { /* absorbed at its first test (folded into the round) */
      const uint32_t nd = pht_stream_pos(&ln.r);
      if (DEBUG) {
        a.dbg_flags[pos] = ln.flags;
        a.dbg_ndraw[pos] = nd;
      }
      c_obs++;
      c_neval += ln.neval;
      c_flag += ln.flags ? 1u : 0u;
      c_nd += nd;
      c_jump += ln.njump;
      have = false;
    }
  }
#ifdef PHT_STAMPS
  /* diagnostic builds: the extra words carry [rounds, 15 stamp slots] */
  (void)c_obs; (void)c_neval; (void)c_flag; (void)c_nd; (void)c_jump;
  if ((threadIdx.x & 63) == 0) {
    lds_add(&xc[0], ln.st_rounds);
    for (int q = 0; q < 15; q++) lds_add(&xc[1 + q], ln.st_acc[q]);
  }
#else
  lds_add(&xc[0], (unsigned long long)c_obs);
  lds_add(&xc[1], (unsigned long long)c_neval);
  lds_add(&xc[2], (unsigned long long)c_flag);
  lds_add(&xc[3], (unsigned long long)c_nd);
  lds_add(&xc[4], (unsigned long long)c_jump);
#endif
#ifdef PHT_ECS_DIAG
  lds_add(&xc[6], (unsigned long long)c_big);
  lds_add(&xc[7], (unsigned long long)c_wbig);
  lds_add(&xc[8], (unsigned long long)c_wround);
  lds_add(&xc[9], (unsigned long long)c_act);
  lds_add(&xc[10], (unsigned long long)c_start);
  lds_add(&xc[11], (unsigned long long)c_pend);
  lds_add(&xc[12], (unsigned long long)c_new);
  lds_add(&xc[13], (unsigned long long)c_wnew);
  lds_add(&xc[14], (unsigned long long)c_wpend);
  lds_add(&xc[5], (unsigned long long)c_w13);
#endif
  __syncthreads();
  flush_stats(a.stats, zq, Bc, Nc, xc, n);
}

/*
 * The longest exact observations, one per 16-lane row (pht_ecs_row.h):
 * the a.rowk positions before the one-lane range (decreasing y), block b of the
 * nblk row blocks taking positions b, b + nblk, ... through its LDS cursor.
 * The row waves issue at raised priority: they carry the sweep's critical
 * path while one-lane blocks share their CUs.
 */
template <int NT, bool DEBUG>
__device__ __forceinline__ void ecs_row_body(const SweepArgs &a, unsigned blk, unsigned nblk) {
  extern __shared__ __align__(16) unsigned char smem[];
  constexpr int n = NT;
  const Layout L = make_layout(n);
  const int pbytes = ecs_param_bytes(L);
  stage_ecs_params(a, (PHT_LDS unsigned char *)smem, L);
  PHT_LDS unsigned char *lsm = (PHT_LDS unsigned char *)smem;
  PHT_LDS unsigned long long *zq = (PHT_LDS unsigned long long *)(lsm + pbytes);
  PHT_LDS unsigned long long *xc = zq + n;
  PHT_LDS unsigned *Bc = (PHT_LDS unsigned *)(xc + kStatExtra);
  PHT_LDS unsigned *Nc = Bc + n;
  PHT_LDS int *cursor = (PHT_LDS int *)(Nc + n * n);
  pht_stage_math_tables();
  for (int k = threadIdx.x; k < n + kStatExtra; k += blockDim.x) zq[k] = 0ull;
  for (int k = threadIdx.x; k < n + n * n; k += blockDim.x) Bc[k] = 0u;
  if (threadIdx.x == 0) *cursor = 0;
  __syncthreads();
  switch (a.rowprio) { /* s_setprio takes an immediate */
    case 0: break;
    case 1: __builtin_amdgcn_s_setprio(1); break;
    case 2: __builtin_amdgcn_s_setprio(2); break;
    default: __builtin_amdgcn_s_setprio(3); break;
  }

  Par<NT> P;
  P.d = (const PHT_LDS double *)lsm;
  P.iv = (const PHT_LDS int *)(lsm + L.necs * 8);
  P.Lr = L;
  const RowId<NT> id = row_id<NT>(P, (int)(threadIdx.x & (kRowW - 1)));
  Sink<DEBUG> sk{zq, Bc, Nc, n, a.zscale, nullptr, nullptr, nullptr, nullptr, xc};
  Lane ln;
  RowObs<NT> st;
  st.yt = 0.0; st.j = 0; st.njump = 0; st.haveE0 = false; st.haveDen = false; st.fold = false; st.den = 0.0;
  for (int h = 0; h < RowV<NT>::H; h++) st.E0.v[h] = 0.0;
  RowEnv ev;
  ev.x = 0.0; ev.y = 0.0; ev.cnt = 0; ev.ymax = 0.0;
  EnvPrivateBig benv;
  ArmsPend pd;
  bool pend = false, bigm = false;
  long pos = 0;
  bool have = false, done = false;
  unsigned c_obs = 0, c_neval = 0, c_flag = 0, c_nd = 0, c_jump = 0;
  /* the path of the row is complete (its statistics recorded) */
  auto complete = [&]() {
    const uint32_t nd = pht_stream_pos(&ln.r);
    if (id.lead) {
      if (DEBUG) {
        a.dbg_flags[pos] = ln.flags;
        a.dbg_ndraw[pos] = nd;
      }
      c_obs++;
      c_neval += ln.neval;
      c_flag += ln.flags ? 1u : 0u;
      c_nd += nd;
      c_jump += ln.njump;
    }
    have = false;
  };
#ifdef PHT_STAMPS
  ln.st_last = __builtin_amdgcn_s_memtime();
  for (int q = 0; q < 15; q++) ln.st_acc[q] = 0ull;
  ln.st_rounds = 0ull;
#endif
  for (;;) {
    bool need = false;
    if (have && !pend) pht_stream_topup(&ln.r);
    while (!done && !pend) {
      if (!have) {
        int t = 0;
        if (id.lead) t = __hip_atomic_fetch_add(cursor, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        t = __shfl(t, 0, kRowW);
        const long p = (long)t * nblk + blk;
        if (p >= a.rowk) {
          done = true;
          break;
        }
        pos = a.begin - a.rowk + p; /* the rows' positions precede the launch range */
        pht_stream_init(&ln.r, a.k0, a.k1, a.gid[pos], 0u, a.sweep);
        ln.flags = 0; ln.neval = 0; ln.nbrent = 0; ln.njump = 0;
        if (DEBUG) {
          sk.dz = a.dbg_zq + pos * n;
          sk.dN = a.dbg_N + pos * n * n;
          sk.dB = a.dbg_B + pos;
          sk.dpre = a.dbg_pre + pos;
        }
        /* ecs_begin */
        const double target = dev_u(ln.r);
        const int B = pistart(P, target, ln.flags);
        if (id.lead) sk.start(B);
        st.yt = a.y[pos];
        st.j = B;
        st.njump = 0;
        st.haveE0 = false;
        st.haveDen = false;
        st.fold = false;
        have = true;
      }
      /* after a jump the absorb test runs inside the round (row_round) */
      if (!st.fold && row_try_absorb<NT>(P, id, ln, sk, st)) {
        complete();
        continue;
      }
      need = true;
      break;
    }
    PHT_STAMP(ln, 0);
    if (!__any(need) && !__any(pend) && !__any(!done)) break;
#ifdef PHT_STAMPS
    ln.st_rounds++;
#endif
    if (need || pend) pht_stream_topup(&ln.r);
    PHT_STAMP(ln, 12);
    if (row_round<NT>(P, id, ln, ev, benv, sk, st, need, pend, bigm, pd)) complete();
  }
#ifdef PHT_STAMPS
  (void)c_obs; (void)c_neval; (void)c_flag; (void)c_nd; (void)c_jump;
  if ((threadIdx.x & 63) == 0) {
    lds_add(&xc[0], ln.st_rounds);
    for (int q = 0; q < 15; q++) lds_add(&xc[1 + q], ln.st_acc[q]);
  }
#else
  lds_add(&xc[0], (unsigned long long)c_obs);
  lds_add(&xc[1], (unsigned long long)c_neval);
  lds_add(&xc[2], (unsigned long long)c_flag);
  lds_add(&xc[3], (unsigned long long)c_nd);
  lds_add(&xc[4], (unsigned long long)c_jump);
#endif
  __syncthreads();
  flush_stats(a.stats, zq, Bc, Nc, xc, n);
}

/* waves per SIMD the ECS kernel is compiled for (its DEBUG instantiation,
 * per-observation outputs for the parity tests, is left unconstrained): two
 * at n = 10 with row blocks (the row code would otherwise take it to one)
 * and at n = 15, where the
 * W row read from LDS (EcsDens) lets it fit (255 VGPRs, no spills, per the
 * built library's metadata: tools/kernel_regs.py); at n = 20 two as well
 * since the compact parameter prefix lets two blocks share a CU (r04: 43
 * spilled VGPRs in the one-lane body, cfg3 kernel 0.858 -> 0.824 ms in an
 * interleaved A/B); otherwise what the registers allow (PHT_ECS_WAVES=k
 * forces every n).  The DEBUG=true
 * instantiations (per-observation outputs for the parity tests) may spill a
 * few VGPRs: they are never timed. */
template <int NT, bool ROWS = false>
constexpr int ecs_waves() {
  return PHT_ECS_WAVES > 0 ? PHT_ECS_WAVES : ((NT == 15 || NT == 20 || (ROWS && NT == 10)) ? 2 : 1);
}
template <int NT, bool DEBUG, bool ROWS>
__global__ void __launch_bounds__(kBlock)
__attribute__((amdgpu_waves_per_eu(DEBUG ? 1 : ecs_waves<NT, ROWS>())))
ecs_exact_kernel(SweepArgs a) {
  if constexpr (ROWS) {
    /* blocks [0, rowblk): the a.rowk longest observations, one per row
     * (positions [begin - rowk, begin)), dispatched first so that a kernel
     * running concurrently (the censored range) cannot take their slots;
     * then the nmain one-lane blocks over the launch range (set by the
     * launcher).  A separate instantiation: without rows the kernel is the
     * one-lane body alone (its register and SGPR allocation untouched by the
     * row code) */
    if (__builtin_expect(blockIdx.x < (unsigned)a.rowblk, 0)) {
      ecs_row_body<NT, DEBUG>(a, blockIdx.x, (unsigned)a.rowblk);
      return;
    }
    ecs_exact_body<NT, DEBUG>(a, blockIdx.x - (unsigned)a.rowblk, (unsigned)a.nmain);
  } else {
    ecs_exact_body<NT, DEBUG>(a, blockIdx.x, gridDim.x);
  }
}

/*
 * K independent chains' exact ECS observations in ONE launch (SURVEY.md
 * §8f.4): block b serves chain b % K as its block b / K of nblk, staging that
 * chain's parameters and adding into that chain's statistics.  An
 * observation's result depends only on (its id, the chain's key, sweep and
 * parameters), so every chain equals its own single launch bit for bit.
 */
template <int NT>
__global__ void __launch_bounds__(kBlock)
__attribute__((amdgpu_waves_per_eu(ecs_waves<NT>())))
ecs_chains_kernel(const SweepArgs *args, int K, unsigned nblk) {
  const SweepArgs a = args[blockIdx.x % (unsigned)K];
  ecs_exact_body<NT, false>(a, blockIdx.x / (unsigned)K, nblk);
}

template <int NT>
static int smem_bytes_ecs(int n) {
  const Layout L = make_layout(n);
  return ((ecs_param_bytes(L) + (n + kStatExtra) * 8 + (n + n * n) * 4 + 4 + 4 + 15) & ~15) +
         2 * ecs_env_k<NT>() * 8 * kBlock;
}

template <int NT, bool DEBUG>
static hipError_t launch_ecs_exact(const SweepArgs &a, hipStream_t st) {
  static LaunchCfg cfg, cfgr;
  const int sm = smem_bytes_ecs<NT>(a.n);
  const bool rows = row_ok<NT>() && a.rowk > 0;
  const void *kfn = rows ? (const void *)ecs_exact_kernel<NT, DEBUG, row_ok<NT>()>
                         : (const void *)ecs_exact_kernel<NT, DEBUG, false>;
  int occ = 0, cus = 0;
  if (hipError_t e = launch_config(rows ? cfgr : cfg, kfn, sm, &occ, &cus); e != hipSuccess)
    return e;
  /* the rowk longest observations on 16-lane rows (kBlock / kRowW per
   * block), ahead of the one-lane blocks in the same launch */
  /* blocks per CU: the occupancy limit, or fewer (a.occ) when the shard is
   * small and the longest paths, not throughput, set the time */
  const int bpc = (a.occ > 0 && a.occ < occ) ? a.occ : occ;
  const long slots = (long)cus * bpc;
  SweepArgs b = a;
  /* rows take at most half the resident blocks, or more when every
   * one-lane block the rest of the range wants (one lane per observation)
   * still fits beside them: the one-lane blocks must be resident too (a
   * persistent block that started late would still own its claim chunks) */
  constexpr long kRows = kBlock / kRowW;
  const long half = (slots / 2) * kRows;
  long rk = row_ok<NT>() ? std::max(0L, std::min(a.rowk, a.count)) : 0;
  while (rk > half && rk >= kRows && (rk + kRows - 1) / kRows + (a.count - rk + kBlock - 1) / kBlock > slots)
    rk -= kRows;
  b.rowk = std::max(0L, rk);
  b.rowblk = (int)((b.rowk + (kBlock / kRowW) - 1) / (kBlock / kRowW));
  b.begin = a.begin + b.rowk;
  b.count = a.count - b.rowk;
  const long want = (b.count + kBlock - 1) / kBlock;
  long grid = slots - b.rowblk;
  if (grid > want) grid = want;
  if (grid < 0) grid = 0;
  b.nmain = (int)grid;
  if (grid + b.rowblk < 1) return hipSuccess;
  if (rows)
    hipLaunchKernelGGL((ecs_exact_kernel<NT, DEBUG, row_ok<NT>()>), dim3((unsigned)(grid + b.rowblk)), dim3(kBlock), sm,
                       st, b);
  else
    hipLaunchKernelGGL((ecs_exact_kernel<NT, DEBUG, false>), dim3((unsigned)grid), dim3(kBlock), sm, st, b);
  return hipGetLastError();
}

/* h: the chains' arguments on the host (sizing), d: the same on the device */
template <int NT>
static hipError_t launch_ecs_chains(const SweepArgs *h, const SweepArgs *d, int K, hipStream_t st) {
  static LaunchCfg cfg;
  const int sm = smem_bytes_ecs<NT>(h[0].n);
  int occ = 0, cus = 0;
  if (hipError_t e = launch_config(cfg, (const void *)ecs_chains_kernel<NT>, sm, &occ, &cus); e != hipSuccess)
    return e;
  long want = 0;
  for (int c = 0; c < K; c++) want = std::max(want, (h[c].count + kBlock - 1) / kBlock);
  /* every chain gets the same share of the resident grid (at least one block) */
  long nblk = std::max(1L, (long)cus * occ / K);
  if (nblk > want) nblk = want;
  if (nblk < 1) return hipSuccess;
  hipLaunchKernelGGL((ecs_chains_kernel<NT>), dim3((unsigned)(nblk * K)), dim3(kBlock), sm, st, d, K, (unsigned)nblk);
  return hipGetLastError();
}

/* the MHRS attempt search: round 0, rounds 1-5 (compaction after the
 * multi-wavefront rounds); queue counts stay on the device (no host sync) */
template <int NT>
static hipError_t launch_mhrs_search(const SweepArgs &a, hipStream_t st) {
  if (a.mbest == nullptr || a.mq0 == nullptr || a.mq1 == nullptr || a.mcnt == nullptr || a.begin != 0)
    return hipErrorInvalidValue;
  const int sm = make_layout(a.n).bytes();
  const long tasks = a.count * (1 + a.mhit);
  /* (the queue counters are zeroed by round 0's block 0, every task's record
   * is written by round 0: no fills per sweep) */
  {
    const int smc = sm + 16 + mhrs_cum_bytes(a.n); /* + the claim cursor, the running sums */
    /* persistent grid: exactly the resident blocks (a block that started
     * late would still own its share of the claim chunks); the rounds'
     * instantiations share one resource footprint */
    static LaunchCfg cfg;
    int occc = 0, cus = 0;
    if (hipError_t e = launch_config(cfg, (const void *)mhrs_search<NT, 1, kMhrsK0>, smc, &occc, &cus);
        e != hipSuccess)
      return e;
    /* compaction grids: after round 0 every task is scanned (~4096 per
     * block); the later queues are short */
    const dim3 g((unsigned)(cus * occc)), gc(256),
        gc0((unsigned)std::min(std::max((tasks + 4095) / 4096, 1L), 1024L));
    unsigned *c = a.mcnt;
    hipLaunchKernelGGL((mhrs_search<NT, 1, kMhrsK0>), g, dim3(kBlock), smc, st, a, 0u, nullptr, nullptr);
    hipLaunchKernelGGL((mhrs_compact<NT>), gc0, dim3(kBlock), 0, st, a, nullptr, nullptr, a.mq0, c + 0);
    constexpr MhrsRound R1 = kMhrsRounds[0], R2 = kMhrsRounds[1], R3 = kMhrsRounds[2], R4 = kMhrsRounds[3],
                        R5 = kMhrsRounds[4];
    hipLaunchKernelGGL((mhrs_search<NT, R1.W, R1.K>), g, dim3(kBlock), smc, st, a, R1.A0, a.mq0, c + 0);
    hipLaunchKernelGGL((mhrs_compact<NT>), gc, dim3(kBlock), 0, st, a, a.mq0, c + 0, a.mq1, c + 1);
    hipLaunchKernelGGL((mhrs_search<NT, R2.W, R2.K>), g, dim3(kBlock), smc, st, a, R2.A0, a.mq1, c + 1);
    hipLaunchKernelGGL((mhrs_compact<NT>), gc, dim3(kBlock), 0, st, a, a.mq1, c + 1, a.mq0, c + 2);
    hipLaunchKernelGGL((mhrs_search<NT, R3.W, R3.K>), g, dim3(kBlock), smc, st, a, R3.A0, a.mq0, c + 2);
    hipLaunchKernelGGL((mhrs_compact<NT>), gc, dim3(kBlock), 0, st, a, a.mq0, c + 2, a.mq1, c + 3);
    hipLaunchKernelGGL((mhrs_search<NT, R4.W, R4.K>), g, dim3(kBlock), smc, st, a, R4.A0, a.mq1, c + 3);
    hipLaunchKernelGGL((mhrs_compact<NT>), gc, dim3(kBlock), 0, st, a, a.mq1, c + 3, a.mq0, c + 4);
    hipLaunchKernelGGL((mhrs_search<NT, R5.W, R5.K>), g, dim3(kBlock), smc, st, a, R5.A0, a.mq0, c + 4);
  }
  return hipGetLastError();
}

}  // namespace pht
/* needs Sink, SweepArgs, claim_pos and lds_add from above */
#include "pht_dcs_round.h"
#include "pht_cens_round.h"
namespace pht {

/* DCS: converged rounds (pht_dcs_round.h), persistent grid */
#ifndef PHT_DCS_WAVES
#define PHT_DCS_WAVES 0
#endif
/* n = 20: the block's LDS (parameters, reciprocals and the E rows, 82 KB)
 * allows one block per CU, so the kernel is compiled for one wave per SIMD
 * (it spilled 141 VGPRs holding to two it could never get) */
template <int NT>
constexpr int dcs_waves() {
  return PHT_DCS_WAVES > 0 ? PHT_DCS_WAVES : (NT == 20 ? 1 : 2);
}
template <int NT, bool DEBUG>
__global__ void __launch_bounds__(kBlock)
__attribute__((amdgpu_waves_per_eu(dcs_waves<NT>())))
dcs_round_kernel(SweepArgs a) {
  dcs_round_body<NT, DEBUG>(a, blockIdx.x, gridDim.x);
}
/* DCS end-state pre-pass: for every position of the launch, the end state
 * the round kernel would draw (dcs_end_state on e^{lambda_i y} and the
 * observation stream's first word), into a.dcsb */
template <int NT>
__global__ void __launch_bounds__(kBlock) dcs_end_kernel(SweepArgs a) {
  extern __shared__ __align__(16) unsigned char smem[];
  const Par<NT> P = stage_params<NT>(a, (PHT_LDS unsigned char *)smem);
  pht_stage_math_tables();
  __syncthreads();
  const int n = P.n();
  for (long p = (long)blockIdx.x * kBlock + threadIdx.x; p < a.count; p += (long)gridDim.x * kBlock) {
    const long pos = a.begin + p;
    const double x = a.y[pos] - 0.0; /* the round kernel's y - t at t = 0 */
    DcsE<NT, false> ey;
#pragma unroll
    for (int i = 0; i < n; i++) ey.set(i, pht_exp_neg(P.evals(i) * x));
    pht_stream r;
    pht_stream_init(&r, a.k0, a.k1, a.gid[pos], 0u, a.sweep);
    int flags = 0;
    const int b = dcs_end_state(P, ey, dev_u(r), flags);
    a.dcsb[pos] = b | (flags ? kDcsEndFlag : 0);
  }
}

template <int NT, bool DEBUG>
static hipError_t launch_dcs_round(const SweepArgs &a, hipStream_t st) {
  /* every observation's end state first, one thread per position (the round
   * kernel would run that n^2 scan in almost every round: some lane of the
   * wavefront starts an observation) */
  if (a.dcsb && a.count > 0) {
    static LaunchCfg cfge;
    const int sme = make_layout(a.n).bytes();
    int occe = 0, cuse = 0;
    if (hipError_t e = launch_config(cfge, (const void *)dcs_end_kernel<NT>, sme, &occe, &cuse); e != hipSuccess)
      return e;
    const long ge = std::min<long>((a.count + kBlock - 1) / kBlock, (long)cuse * occe);
    hipLaunchKernelGGL((dcs_end_kernel<NT>), dim3((unsigned)ge), dim3(kBlock), sme, st, a);
  }
  static LaunchCfg cfg;
  const int sm = dcs_smem_bytes<NT>(make_layout(a.n).bytes(), a.n); /* + near masks, reciprocals */
  int occ = 0, cus = 0;
  if (hipError_t e = launch_config(cfg, (const void *)dcs_round_kernel<NT, DEBUG>, sm, &occ, &cus);
      e != hipSuccess)
    return e;
  long grid = (long)cus * occ;
  const long want = (a.count + kClaimChunk - 1) / kClaimChunk;
  if (grid > want) grid = want;
  if (grid < 1) return hipSuccess;
  hipLaunchKernelGGL((dcs_round_kernel<NT, DEBUG>), dim3((unsigned)grid), dim3(kBlock), sm, st, a);
  return hipGetLastError();
}
/* ECS censored range: jump-converged rounds (pht_cens_round.h) */
template <int NT, bool DEBUG>
__global__ void __launch_bounds__(kBlock)
__attribute__((amdgpu_waves_per_eu(persist_waves<NT, kMethodECS>())))
cens_round_kernel(SweepArgs a) {
  cens_round_body<NT, DEBUG>(a, blockIdx.x, gridDim.x);
}
template <int NT, bool DEBUG>
static hipError_t launch_cens_round(const SweepArgs &a, hipStream_t st) {
  static LaunchCfg cfg;
  const int sm = ((smem_bytes(a.n) + 4 + 15) & ~15) + cens_env_bytes<NT>();
  int occ = 0, cus = 0;
  if (hipError_t e = launch_config(cfg, (const void *)cens_round_kernel<NT, DEBUG>, sm, &occ, &cus); e != hipSuccess)
    return e;
  long grid = (long)cus * occ;
  const long want = (a.count + kClaimChunk - 1) / kClaimChunk;
  if (grid > want) grid = want;
  if (grid < 1) return hipSuccess;
  hipLaunchKernelGGL((cens_round_kernel<NT, DEBUG>), dim3((unsigned)grid), dim3(kBlock), sm, st, a);
  return hipGetLastError();
}
/* ================================================================ UNIF */
/* The per-sweep uniformisation table (pht_unif.h spec), one workgroup:
 * mu, R and its squarings in LDS, the forward vectors A_k by doubling
 * (rows [2^i, 2^(i+1)) from rows [0, 2^i) and P_i), then ax, ac, invk. */
constexpr int kUnifTabThreads = 1024;
/* the forward vectors in LDS while they are built (one dependent LDS
 * round trip per doubling step instead of an L2 one), when (K+1) n doubles
 * fit this budget; else in the global table directly */
constexpr int kUnifTabLds = 128 * 1024;
template <class APtr>
__device__ __forceinline__ void unif_doubling(APtr A, double (*Pm)[kMaxN * kMaxN], int n, int K) {
  const int tid = threadIdx.x, nt = blockDim.x;
  int cur = 0;
  for (int p = 1; p <= K; p <<= 1) {
    /* rows p + r, r < p, from rows r and P = Pm[cur] (= R^p) */
    const int rows = (K - p + 1 < p) ? K - p + 1 : p;
    for (int e = tid; e < rows * n; e += nt) {
      const int r = e / n, j = e % n;
      double acc = 0.0;
      for (int c = 0; c < n; c++) acc = fma(A[(long)r * n + c], Pm[cur][c + j * n], acc);
      A[(long)(p + r) * n + j] = acc;
    }
    if (2 * p <= K) { /* P_{i+1} = P_i P_i */
      for (int e = tid; e < n * n; e += nt) {
        const int c = e % n, j = e / n;
        double acc = 0.0;
        for (int q = 0; q < n; q++) acc = fma(Pm[cur][c + q * n], Pm[cur][q + j * n], acc);
        Pm[cur ^ 1][e] = acc;
      }
    }
    __syncthreads();
    cur ^= 1;
  }
}
template <int NT, bool LDSA>
__device__ __forceinline__ void unif_table_body(const SweepArgs &a) {
  __shared__ double Pm[2][kMaxN * kMaxN];
  __shared__ double hdr[2];
  extern __shared__ __align__(16) unsigned char smem[];
  const int n = nval<NT>(a.n);
  const Layout L = make_layout(n);
  const double *d = reinterpret_cast<const double *>(a.params);
  __shared__ int Ksh;
  double *T = a.utab;
  const int tid = threadIdx.x, nt = blockDim.x;
  if (tid == 0) {
    double mu = 0.0;
    for (int i = 0; i < n; i++) {
      const double v = -d[L.S + i + i * n];
      mu = (v > mu) ? v : mu;
    }
    hdr[0] = mu;
    hdr[1] = 1.0 / mu;
    /* rows: the shard's largest lam with a Poisson margin, within the
     * capacity a.uK (the host's sizing).  An observation that needs rows
     * beyond it (or lam > kUnifMaxLam) is sampled from a truncated Poisson
     * sum or a placeholder path, i.e. WRONG: it sets kFlagUnifCap, counted
     * in the statistics' kXUnifCap word, and the host loop / resident
     * update turn any such count into an error */
    const double lmax = mu * a.uymax;
    const double kd = ceil(lmax + 14.0 * sqrt(lmax) + 64.0);
    Ksh = (kd < (double)a.uK) ? (int)kd : a.uK;
    T[0] = mu;
    T[1] = hdr[1];
    T[2] = (double)Ksh;
    T[3] = 0.0;
  }
  __syncthreads();
  const int K = Ksh;
  double *invk = T + 4, *ax = invk + (K + 1), *ac = ax + (K + 1), *A = ac + (K + 1);
  PHT_LDS double *Al = (PHT_LDS double *)smem;
  for (int k = tid; k <= K; k += nt) invk[k] = k ? 1.0 / (double)k : 0.0;
  if (tid < n) {
    if (LDSA) Al[tid] = d[L.pi + tid];
    else A[tid] = d[L.pi + tid];
  }
  const double rinv = hdr[1];
  for (int e = tid; e < n * n; e += nt) { /* Pm[0][c + j n] = R_cj */
    const int c = e % n, j = e / n;
    Pm[0][e] = (c == j) ? fma(d[L.S + c + c * n], rinv, 1.0) : d[L.S + c + j * n] * rinv;
  }
  __syncthreads();
  if (LDSA) unif_doubling(Al, Pm, n, K);
  else unif_doubling(A, Pm, n, K);
  if (LDSA)
    for (long e = tid; e < (long)(K + 1) * n; e += nt) A[e] = Al[e];
  for (int k = tid; k <= K; k += nt) {
    double sx = 0.0, sc = 0.0;
    for (int j = 0; j < n; j++) {
      const double v = LDSA ? Al[(long)k * n + j] : A[(long)k * n + j];
      /* ulaw 1 (MHRS bridge): ax = aa, the alive mass in states with exits */
      sx = (a.ulaw == 1) ? sx + ((d[L.s + j] > 0.0) ? v : 0.0) : fma(v, d[L.s + j], sx);
      sc = sc + v;
    }
    ax[k] = sx;
    ac[k] = sc;
  }
}

template <int NT, bool LDSA>
__global__ void __launch_bounds__(kUnifTabThreads) unif_table_kernel(SweepArgs a) {
  unif_table_body<NT, LDSA>(a);
}
/* the table launch: LDS working rows when they fit (capacity a.uK) */
template <int NT>
static hipError_t launch_unif_table(const SweepArgs &a, hipStream_t st) {
  const long bytes = (long)(a.uK + 1) * a.n * 8;
  if (bytes <= kUnifTabLds) {
    static LaunchCfg cfg;
    int occ = 0, cus = 0;
    if (hipError_t e = launch_config(cfg, (const void *)unif_table_kernel<NT, true>, (int)bytes, &occ, &cus);
        e != hipSuccess)
      return e;
    hipLaunchKernelGGL((unif_table_kernel<NT, true>), dim3(1), dim3(kUnifTabThreads), (int)bytes, st, a);
  } else {
    hipLaunchKernelGGL((unif_table_kernel<NT, false>), dim3(1), dim3(kUnifTabThreads), 0, st, a);
  }
  return hipGetLastError();
}

/* UNIF sweep: persistent lanes, one observation per lane to its end
 * (claims as the other persistent kernels: 64-position chunks through an
 * LDS cursor), exact and censored observations in one launch */
static int smem_bytes_unif(int n, int K) {
  return ((smem_bytes(n) + 15) & ~15) + 3 * (K + 1) * 8 + n * n * 12 + n * 4; /* + predecessor lists */
}

template <int NT, bool DEBUG>
__device__ __forceinline__ void unif_body(const SweepArgs &a, unsigned blk, unsigned nblk) {
  extern __shared__ __align__(16) unsigned char smem[];
  const int n = nval<NT>(a.n);
  const Layout L = make_layout(n);
  const int pbytes = L.bytes();
  if ((long)blk * kClaimChunk >= a.count) return;
  const Par<NT> P = stage_params<NT>(a, (PHT_LDS unsigned char *)smem);
  PHT_LDS unsigned char *lsm = (PHT_LDS unsigned char *)smem;
  PHT_LDS unsigned long long *zq = (PHT_LDS unsigned long long *)(lsm + pbytes);
  PHT_LDS unsigned long long *xc = zq + n;
  PHT_LDS unsigned *Bc = (PHT_LDS unsigned *)(xc + kStatExtra);
  PHT_LDS unsigned *Nc = Bc + n;
  PHT_LDS int *cursor = (PHT_LDS int *)(Nc + n * n);
  PHT_LDS double *tl = (PHT_LDS double *)(lsm + ((pbytes + (n + kStatExtra) * 8 + (n + n * n) * 4 + 4 + 15) & ~15));
  const double *T = a.utab;
  const int K = (int)T[2]; /* rows of this sweep's table (<= a.uK, the LDS sizing) */
  /* invk, ax, ac staged into LDS */
  const long nstage = 3L * (K + 1);
  for (long k = threadIdx.x; k < nstage; k += blockDim.x) tl[k] = T[4 + k];
  for (int k = threadIdx.x; k < n + kStatExtra; k += blockDim.x) zq[k] = 0ull;
  for (int k = threadIdx.x; k < n + n * n; k += blockDim.x) Bc[k] = 0u;
  if (threadIdx.x == 0) *cursor = 0;
  pht_stage_math_tables();
  __syncthreads();
  PHT_LDS double *pv = tl + nstage;
  PHT_LDS int *pc = (PHT_LDS int *)(pv + n * n), *np = pc + n * n;
  unif_preds<NT>(P, T[1], pv, pc, np);
  __syncthreads();
  UnifTab<const double *> U;
  U.invk = tl;
  U.ax = tl + (K + 1);
  U.ac = tl + 2 * (K + 1);
  U.A = T + 4 + 3 * (K + 1);
  U.pv = pv;
  U.pc = pc;
  U.np = np;
  U.K = K;
  U.mu = T[0];
  U.rinv = T[1];
  Sink<DEBUG> sk{zq, Bc, Nc, n, a.zscale, nullptr, nullptr, nullptr, nullptr};
  unsigned c_obs = 0, c_neval = 0, c_flag = 0, c_nd = 0, c_jump = 0, c_ucap = 0;
  for (;;) {
    const long p = claim_pos(__hip_atomic_fetch_add(cursor, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP), blk, nblk);
    if (p >= a.count) break;
    const long i = a.begin + p;
    Lane ln;
    pht_stream_init(&ln.r, a.k0, a.k1, a.gid[i], 0u, a.sweep);
    ln.flags = 0; ln.neval = 0; ln.nbrent = 0; ln.njump = 0;
    if (DEBUG) {
      sk.dz = a.dbg_zq + i * n;
      sk.dN = a.dbg_N + i * n * n;
      sk.dB = a.dbg_B + i;
      sk.dpre = a.dbg_pre + i;
    }
    unif_obs<NT>(P, U, a.y[i], a.cens ? a.cens[i] : 0, ln, sk, a.ulaw, a.mhit);
    const uint32_t nd = pht_stream_pos(&ln.r);
    if (DEBUG) {
      a.dbg_flags[i] = ln.flags;
      a.dbg_ndraw[i] = nd;
    }
    c_obs++;
    c_neval += ln.neval;
    c_flag += ln.flags ? 1u : 0u;
    c_ucap += (ln.flags & kFlagUnifCap) ? 1u : 0u;
    c_nd += nd;
    c_jump += ln.njump;
  }
  lds_add(&xc[0], (unsigned long long)c_obs);
  lds_add(&xc[1], (unsigned long long)c_neval);
  lds_add(&xc[2], (unsigned long long)c_flag);
  lds_add(&xc[3], (unsigned long long)c_nd);
  lds_add(&xc[4], (unsigned long long)c_jump);
  if (c_ucap) lds_add(&xc[kXUnifCap], (unsigned long long)c_ucap);
  __syncthreads();
  flush_stats(a.stats, zq, Bc, Nc, xc, n);
}

template <int NT, bool DEBUG>
__global__ void __launch_bounds__(kBlock) unif_kernel(SweepArgs a) {
  unif_body<NT, DEBUG>(a, blockIdx.x, gridDim.x);
}

template <int NT, bool DEBUG>
static hipError_t launch_unif(const SweepArgs &a, hipStream_t st) {
  if (a.utab == nullptr || a.uK < 1 || a.uK > kUnifMaxK || a.begin != 0) return hipErrorInvalidValue;
  if (hipError_t e = launch_unif_table<NT>(a, st); e != hipSuccess) return e;
  if (a.count < 1) return hipGetLastError();
  /* the forward vectors stay in the global table (L2): staging them in LDS
   * as well measured no faster at n = 10..20 (r03) */
  static LaunchCfg cfg;
  const int sm = smem_bytes_unif(a.n, a.uK);
  int occ = 0, cus = 0;
  if (hipError_t e = launch_config(cfg, (const void *)unif_kernel<NT, DEBUG>, sm, &occ, &cus); e != hipSuccess)
    return e;
  long grid = (long)cus * occ;
  const long want = (a.count + kClaimChunk - 1) / kClaimChunk;
  if (grid > want) grid = want;
  hipLaunchKernelGGL((unif_kernel<NT, DEBUG>), dim3((unsigned)grid), dim3(kBlock), sm, st, a);
  return hipGetLastError();
}

/* ====================================== several chains in one launch (§8f.4)
 * Block b of a chains launch serves chain b % K as its block b / K of nblk
 * (the bodies take their block index and count), staging that chain's
 * parameters and adding into that chain's statistics.  An observation's
 * result depends only on (its id, the chain's key, sweep and parameters), so
 * every chain equals its own single launch bit for bit. */
template <int NT>
__global__ void __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(dcs_waves<NT>())))
dcs_chains_kernel(const SweepArgs *args, int K, unsigned nblk) {
  dcs_round_body<NT, false>(args[blockIdx.x % (unsigned)K], blockIdx.x / (unsigned)K, nblk);
}
template <int NT>
__global__ void __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(persist_waves<NT, kMethodECS>())))
cens_chains_kernel(const SweepArgs *args, int K, unsigned nblk) {
  cens_round_body<NT, false>(args[blockIdx.x % (unsigned)K], blockIdx.x / (unsigned)K, nblk);
}
template <int NT>
__global__ void __launch_bounds__(kUnifTabThreads) unif_table_chains_kernel(const SweepArgs *args) {
  unif_table_body<NT, false>(args[blockIdx.x]);
}
template <int NT>
__global__ void __launch_bounds__(kBlock) unif_chains_kernel(const SweepArgs *args, int K, unsigned nblk) {
  unif_body<NT, false>(args[blockIdx.x % (unsigned)K], blockIdx.x / (unsigned)K, nblk);
}
/* MHRS: per chain, the first-success records to "unresolved" and the queue
 * counters to zero (grid-stride over each chain's tasks) */
template <int NT> /* (templated only to keep one copy per pht_kernels_nt.hip unit) */
__global__ void __launch_bounds__(kBlock) mhrs_init_chains(const SweepArgs *args, int K, unsigned nblk) {
  const SweepArgs &a = args[blockIdx.x % (unsigned)K];
  const unsigned blk = blockIdx.x / (unsigned)K;
  const long tasks = a.count * (1 + a.mhit);
  for (long q = (long)blk * kBlock + threadIdx.x; q < tasks; q += (long)nblk * kBlock) a.mbest[q] = kMhrsUnresolved;
  if (blk == 0 && threadIdx.x < kMhrsCounters) a.mcnt[threadIdx.x] = 0u;
}
/* search round r (0..5) of every chain: round r >= 1 reads the queue the
 * compaction after round r - 1 wrote (launch_mhrs_search's sequence) */
template <int NT, int W, int KA>
__global__ void __launch_bounds__(kBlock) mhrs_search_chains(const SweepArgs *args, int K, unsigned nblk, int r,
                                                             uint32_t A0) {
  const SweepArgs &a = args[blockIdx.x % (unsigned)K];
  const uint32_t *qin = r == 0 ? nullptr : ((r & 1) ? a.mq0 : a.mq1);
  const unsigned *cin = r == 0 ? nullptr : a.mcnt + (r - 1);
  mhrs_search_body<NT, W, KA>(a, A0, qin, cin, blockIdx.x / (unsigned)K, nblk);
}
template <int NT>
__global__ void __launch_bounds__(kBlock) mhrs_compact_chains(const SweepArgs *args, int K, unsigned nblk, int r) {
  const SweepArgs &a = args[blockIdx.x % (unsigned)K];
  const uint32_t *qin = r == 0 ? nullptr : ((r & 1) ? a.mq0 : a.mq1);
  const unsigned *cin = r == 0 ? nullptr : a.mcnt + (r - 1);
  mhrs_compact_body(a, qin, cin, (r & 1) ? a.mq1 : a.mq0, a.mcnt + r, blockIdx.x / (unsigned)K, nblk);
}
template <int NT>
__global__ void __launch_bounds__(kBlock) mhrs_finish_chains(const SweepArgs *args, int K, unsigned nblk) {
  const SweepArgs &a = args[blockIdx.x % (unsigned)K];
  const unsigned blk = blockIdx.x / (unsigned)K;
  if ((long)blk * kClaimChunk >= a.count) return; /* the whole block: its chain has fewer observations */
  mhrs_finish_body<NT, false>(a, blk, nblk); /* persistent (mhrs_finish_kernel) */
}

/* h: the chains' arguments on the host (sizing), d: the same K SweepArgs on
 * the device.  ECS: the censored ranges (allcens); the exact ranges use
 * launch_ecs_chains.  MHRS, DCS, UNIF: whole shards (begin = 0). */
template <int NT>
static hipError_t launch_chains(const SweepArgs *h, const SweepArgs *d, int K, int method, hipStream_t st) {
  long maxc = 0;
  for (int c = 0; c < K; c++) maxc = std::max(maxc, h[c].count);
  auto share = [&](int occ, int cus, long want) -> long { /* blocks per chain */
    long nb = std::max(1L, (long)cus * occ / K);
    return std::min(nb, std::max(1L, want));
  };
  if (method == kMethodECS) {
    static LaunchCfg cfg;
    const int sm = ((smem_bytes(h[0].n) + 4 + 15) & ~15) + cens_env_bytes<NT>();
    int occ = 0, cus = 0;
    if (hipError_t e = launch_config(cfg, (const void *)cens_chains_kernel<NT>, sm, &occ, &cus); e != hipSuccess)
      return e;
    const long nb = share(occ, cus, (maxc + kClaimChunk - 1) / kClaimChunk);
    hipLaunchKernelGGL((cens_chains_kernel<NT>), dim3((unsigned)(nb * K)), dim3(kBlock), sm, st, d, K, (unsigned)nb);
    return hipGetLastError();
  }
  if (method == kMethodDCS) {
    static LaunchCfg cfg;
    const int sm = dcs_smem_bytes<NT>(make_layout(h[0].n).bytes(), h[0].n);
    int occ = 0, cus = 0;
    if (hipError_t e = launch_config(cfg, (const void *)dcs_chains_kernel<NT>, sm, &occ, &cus); e != hipSuccess)
      return e;
    const long nb = share(occ, cus, (maxc + kClaimChunk - 1) / kClaimChunk);
    hipLaunchKernelGGL((dcs_chains_kernel<NT>), dim3((unsigned)(nb * K)), dim3(kBlock), sm, st, d, K, (unsigned)nb);
    return hipGetLastError();
  }
  if (method == kMethodUNIF) {
    int uK = 0;
    for (int c = 0; c < K; c++) {
      if (h[c].utab == nullptr || h[c].uK < 1 || h[c].uK > kUnifMaxK) return hipErrorInvalidValue;
      uK = std::max(uK, h[c].uK);
    }
    hipLaunchKernelGGL((unif_table_chains_kernel<NT>), dim3((unsigned)K), dim3(kUnifTabThreads), 0, st, d);
    if (maxc < 1) return hipGetLastError();
    static LaunchCfg cfg;
    const int sm = smem_bytes_unif(h[0].n, uK);
    int occ = 0, cus = 0;
    if (hipError_t e = launch_config(cfg, (const void *)unif_chains_kernel<NT>, sm, &occ, &cus); e != hipSuccess)
      return e;
    const long nb = share(occ, cus, (maxc + kClaimChunk - 1) / kClaimChunk);
    hipLaunchKernelGGL((unif_chains_kernel<NT>), dim3((unsigned)(nb * K)), dim3(kBlock), sm, st, d, K, (unsigned)nb);
    return hipGetLastError();
  }
  if (method == kMethodMHRS) {
    long maxt = 0;
    for (int c = 0; c < K; c++) {
      if (h[c].mbest == nullptr || h[c].mq0 == nullptr || h[c].mq1 == nullptr || h[c].mcnt == nullptr || h[c].begin)
        return hipErrorInvalidValue;
      maxt = std::max(maxt, h[c].count * (1 + h[c].mhit));
    }
    if (maxc < 1) return hipSuccess;
    const int smc = make_layout(h[0].n).bytes() + 16 + mhrs_cum_bytes(h[0].n);
    static LaunchCfg cfg;
    int occ = 0, cus = 0;
    if (hipError_t e = launch_config(cfg, (const void *)mhrs_search_chains<NT, 1, kMhrsK0>, smc, &occ, &cus);
        e != hipSuccess)
      return e;
    const long nbi = std::max(1L, std::min(1024L / K + 1, (maxt + kBlock - 1) / kBlock));
    hipLaunchKernelGGL((mhrs_init_chains<NT>), dim3((unsigned)(nbi * K)), dim3(kBlock), 0, st, d, K, (unsigned)nbi);
    const long nb = std::max(1L, (long)cus * occ / K); /* persistent: the resident blocks, shared */
    const dim3 g((unsigned)(nb * K));
    const long nbc = std::max(1L, 256L / K);
    const dim3 gc((unsigned)(nbc * K));
    /* the first compaction scans every task (launch_mhrs_search) */
    const long nbc0 = std::max(1L, std::min(std::max(1024L / K, 1L), (maxt + 4095) / 4096));
    const dim3 gc0((unsigned)(nbc0 * K));
    constexpr MhrsRound R1 = kMhrsRounds[0], R2 = kMhrsRounds[1], R3 = kMhrsRounds[2], R4 = kMhrsRounds[3],
                        R5 = kMhrsRounds[4];
    hipLaunchKernelGGL((mhrs_search_chains<NT, 1, kMhrsK0>), g, dim3(kBlock), smc, st, d, K, (unsigned)nb, 0, 0u);
    hipLaunchKernelGGL((mhrs_compact_chains<NT>), gc0, dim3(kBlock), 0, st, d, K, (unsigned)nbc0, 0);
    hipLaunchKernelGGL((mhrs_search_chains<NT, R1.W, R1.K>), g, dim3(kBlock), smc, st, d, K, (unsigned)nb, 1, R1.A0);
    hipLaunchKernelGGL((mhrs_compact_chains<NT>), gc, dim3(kBlock), 0, st, d, K, (unsigned)nbc, 1);
    hipLaunchKernelGGL((mhrs_search_chains<NT, R2.W, R2.K>), g, dim3(kBlock), smc, st, d, K, (unsigned)nb, 2, R2.A0);
    hipLaunchKernelGGL((mhrs_compact_chains<NT>), gc, dim3(kBlock), 0, st, d, K, (unsigned)nbc, 2);
    hipLaunchKernelGGL((mhrs_search_chains<NT, R3.W, R3.K>), g, dim3(kBlock), smc, st, d, K, (unsigned)nb, 3, R3.A0);
    hipLaunchKernelGGL((mhrs_compact_chains<NT>), gc, dim3(kBlock), 0, st, d, K, (unsigned)nbc, 3);
    hipLaunchKernelGGL((mhrs_search_chains<NT, R4.W, R4.K>), g, dim3(kBlock), smc, st, d, K, (unsigned)nb, 4, R4.A0);
    hipLaunchKernelGGL((mhrs_compact_chains<NT>), gc, dim3(kBlock), 0, st, d, K, (unsigned)nbc, 4);
    hipLaunchKernelGGL((mhrs_search_chains<NT, R5.W, R5.K>), g, dim3(kBlock), smc, st, d, K, (unsigned)nb, 5, R5.A0);
    static LaunchCfg cfgf;
    int occf = 0, cusf = 0;
    if (hipError_t e = launch_config(cfgf, (const void *)mhrs_finish_chains<NT>, smem_bytes(h[0].n), &occf, &cusf);
        e != hipSuccess)
      return e;
    const long nbf = std::max(1L, std::min((maxc + kBlock - 1) / kBlock, (long)cusf * occf / K));
    hipLaunchKernelGGL((mhrs_finish_chains<NT>), dim3((unsigned)(nbf * K)), dim3(kBlock), smem_bytes(h[0].n), st, d,
                       K, (unsigned)nbf);
    return hipGetLastError();
  }
  return hipErrorInvalidValue;
}

template <int NT, bool DEBUG>
static hipError_t launch_mhrs_finish(const SweepArgs &a, hipStream_t st) {
  static LaunchCfg cfg;
  const int sm = smem_bytes(a.n);
  int occ = 0, cus = 0;
  if (hipError_t e = launch_config(cfg, (const void *)mhrs_finish_kernel<NT, DEBUG>, sm, &occ, &cus); e != hipSuccess)
    return e;
  long grid = (long)cus * occ;
  const long want = (a.count + kBlock - 1) / kBlock;
  if (grid > want) grid = want;
  if (grid < 1) return hipSuccess;
  hipLaunchKernelGGL((mhrs_finish_kernel<NT, DEBUG>), dim3((unsigned)grid), dim3(kBlock), sm, st, a);
  return hipGetLastError();
}

template <int NT>
static hipError_t launch_nt(const SweepArgs &a, int method, bool debug, hipStream_t st) {
  if (method == kMethodECS && a.cens == nullptr) /* exact-only range */
    return debug ? launch_ecs_exact<NT, true>(a, st) : launch_ecs_exact<NT, false>(a, st);
  if (method == kMethodUNIF) return debug ? launch_unif<NT, true>(a, st) : launch_unif<NT, false>(a, st);
  if (a.count <= 0) return hipSuccess;
  if (method == kMethodMHRS) {
    if (hipError_t e = launch_mhrs_search<NT>(a, st); e != hipSuccess) return e;
    return debug ? launch_mhrs_finish<NT, true>(a, st) : launch_mhrs_finish<NT, false>(a, st);
  } else if (method == kMethodDCS) {
    return debug ? launch_dcs_round<NT, true>(a, st) : launch_dcs_round<NT, false>(a, st);
  } else {
    /* ECS censored observations: the host always launches them as their own
     * range (allcens), concurrently with the exact range */
    if (!a.allcens) return hipErrorInvalidValue;
    return debug ? launch_cens_round<NT, true>(a, st) : launch_cens_round<NT, false>(a, st);
  }
  return hipGetLastError();
}

}  // namespace pht
#endif
