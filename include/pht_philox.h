/*
 * pht_philox.h — the counter-based random stream of the GPU path.
 *
 * The reference consumes R's serial Mersenne-Twister stream in a
 * data-dependent order, which no parallel device can
 * replay.  The device path therefore draws every uniform from
 * Philox4x32-10 (Salmon et al., SC'11; Random123 constants), addressed by
 *   key     = (k0, k1)                  — two words from R's stream at
 *                                         LJMA_Gibbs entry (gibbs_host.cpp)
 *   counter = (obs, stream, sweep, blk) — obs index, stream tag (0 = main),
 *                                         Gibbs sweep, block index
 * An observation's stream is the word sequence block 0 words 0..3, block 1
 * words 0..3, ...; word number i comes from block i/4, so any lane can
 * replay any observation from any word index (used by the MHRS kernel).
 *
 * uniform  (one word w):    u = (2w+1) * 2^-33, exact, 0 < u < 1 — the
 *                           resolution of R's unif_rand (2^-32);
 * uniform53 (two words a,b): m = (a << 20) | (b >> 12) (52 bits),
 *                           u = (2m+1) * 2^-53;
 * exponential uniform:      one word a >= 2^24 -> uniform53(a, 2^31) (the
 *                           centre of a's 2^-32 cell), else uniform53(a, b)
 *                           with a second word: -log(u) keeps its tail
 *                           (exponential sojourns, pht_next_uexp).
 */
#ifndef PHT_PHILOX_H
#define PHT_PHILOX_H

#include <stdint.h>

#if defined(__HIPCC__)
#define PHT_HD2 __host__ __device__ __forceinline__
#else
#define PHT_HD2 static inline
#endif

typedef struct { uint32_t v[4]; } pht_u32x4;

PHT_HD2 uint32_t pht_mulhilo(uint32_t a, uint32_t b, uint32_t *hi) {
  uint64_t p = (uint64_t)a * (uint64_t)b;
  *hi = (uint32_t)(p >> 32);
  return (uint32_t)p;
}

PHT_HD2 pht_u32x4 pht_philox_round(pht_u32x4 c, uint32_t k0, uint32_t k1) {
  uint32_t hi0, hi1;
  const uint32_t lo0 = pht_mulhilo(0xD2511F53U, c.v[0], &hi0);
  const uint32_t lo1 = pht_mulhilo(0xCD9E8D57U, c.v[2], &hi1);
  pht_u32x4 o;
  o.v[0] = hi1 ^ c.v[1] ^ k0;
  o.v[1] = lo1;
  o.v[2] = hi0 ^ c.v[3] ^ k1;
  o.v[3] = lo0;
  return o;
}

/* (device: the compiler keeps the ten rounds as a loop of two; compilation
 * units built with PHT_PHILOX_UNROLL unroll them, see phasetype_amd/build.py) */
PHT_HD2 pht_u32x4 pht_philox4x32_10(pht_u32x4 c, uint32_t k0, uint32_t k1) {
#if defined(__HIP_DEVICE_COMPILE__) && defined(PHT_PHILOX_UNROLL)
#pragma unroll
#endif
  for (int r = 0; r < 10; r++) {
    uint32_t hi0, hi1;
    uint32_t lo0 = pht_mulhilo(0xD2511F53U, c.v[0], &hi0);
    uint32_t lo1 = pht_mulhilo(0xCD9E8D57U, c.v[2], &hi1);
    pht_u32x4 o;
    o.v[0] = hi1 ^ c.v[1] ^ k0;
    o.v[1] = lo1;
    o.v[2] = hi0 ^ c.v[3] ^ k1;
    o.v[3] = lo0;
    c = o;
    k0 += 0x9E3779B9U;
    k1 += 0xBB67AE85U;
  }
  return c;
}

PHT_HD2 double pht_u01(uint32_t whi, uint32_t wlo) {
  uint64_t m = ((uint64_t)whi << 20) | (uint64_t)(wlo >> 12);
  return (double)(2 * m + 1) * 1.1102230246251565404e-16; /* 2^-53 */
}

/* Per-observation word stream.  The current block is a shift register
 * (a0 is the next word, na words left); a second block (b0..b3, valid when
 * nb) can be generated ahead at a convenient point (pht_stream_topup): on a
 * GPU, at a point where a whole wavefront executes it once, instead of at
 * whichever draw finds the buffer empty.  The word sequence is the same
 * whenever blocks are generated. */
typedef struct {
  uint32_t k0, k1;     /* key */
  uint32_t obs, tag;   /* counter words 0,1 */
  uint32_t sweep;      /* counter word 2 */
  uint32_t blk;        /* counter word 3: next block to generate */
  uint32_t a0, a1, a2, a3;
  uint32_t b0, b1, b2, b3;
  int na, nb;
} pht_stream;

PHT_HD2 void pht_stream_init(pht_stream *s, uint32_t k0, uint32_t k1, uint32_t obs,
                             uint32_t tag, uint32_t sweep) {
  s->k0 = k0; s->k1 = k1; s->obs = obs; s->tag = tag; s->sweep = sweep;
  s->blk = 0; s->na = 0; s->nb = 0;
  /* (na = nb = 0: no buffered word is read before a block fills it; the
   * device skips the eight register clears, ~0.5 % of an MHRS sweep at cfg4,
   * profiles/r06/mhrs_hoist/) */
#if !defined(__HIP_DEVICE_COMPILE__)
  s->a0 = s->a1 = s->a2 = s->a3 = 0u;
  s->b0 = s->b1 = s->b2 = s->b3 = 0u;
#endif
}

/* as pht_stream_init, with block 0 already generated (w = its four words) */
PHT_HD2 void pht_stream_init_block0(pht_stream *s, uint32_t k0, uint32_t k1, uint32_t obs, uint32_t tag,
                                    uint32_t sweep, pht_u32x4 w) {
  pht_stream_init(s, k0, k1, obs, tag, sweep);
  s->a0 = w.v[0]; s->a1 = w.v[1]; s->a2 = w.v[2]; s->a3 = w.v[3];
  s->na = 4;
  s->blk = 1;
}

PHT_HD2 pht_u32x4 pht_stream_block(pht_stream *s) {
  pht_u32x4 c; c.v[0] = s->obs; c.v[1] = s->tag; c.v[2] = s->sweep; c.v[3] = s->blk++;
#if defined(__HIP_DEVICE_COMPILE__)
  /* every stream a wavefront holds carries its launch's key (SweepArgs k0/k1,
   * one per workgroup): read it as a wave-uniform value, so that the key
   * schedule runs on the scalar unit and the rounds' xors take it from SGPRs.
   * INVARIANT (every pht_stream_init call site in phasetype_amd/csrc passes
   * a.k0 / a.k1 of the block's own SweepArgs; ecs_chains_kernel and the
   * *_chains kernels select one SweepArgs per block): all lanes of a wave
   * use ONE key.  A kernel that mixed keys within a wave would get other
   * lanes' streams here; tests/test_gpu_parity.py's chains tests (a
   * different key per chain, chains interleaved block by block) are the
   * guard, and tests/test_host.py checks that no call site takes its key
   * from anything but SweepArgs. */
  return pht_philox4x32_10(c, __builtin_amdgcn_readfirstlane(s->k0), __builtin_amdgcn_readfirstlane(s->k1));
#else
  return pht_philox4x32_10(c, s->k0, s->k1);
#endif
}

/* generate the next block ahead (no effect on the word sequence) */
PHT_HD2 void pht_stream_topup(pht_stream *s) {
  if (!s->nb) {
    pht_u32x4 w = pht_stream_block(s);
    s->b0 = w.v[0]; s->b1 = w.v[1]; s->b2 = w.v[2]; s->b3 = w.v[3];
    s->nb = 1;
  }
}

#if defined(__HIPCC__)
/* the block with its ten rounds unrolled (the same words), and
 * pht_stream_topup on it: for one kernel of a unit that keeps the loop
 * elsewhere (PHT_MHRS_PHILOX_UNROLL etc., phasetype_amd/build.py) */
__device__ __forceinline__ pht_u32x4 pht_philox4x32_10_unrolled(pht_u32x4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; r++) {
    c = pht_philox_round(c, k0, k1);
    k0 += 0x9E3779B9U;
    k1 += 0xBB67AE85U;
  }
  return c;
}
__device__ __forceinline__ void pht_stream_topup_unrolled(pht_stream *s) {
  if (!s->nb) {
    pht_u32x4 c;
    c.v[0] = s->obs; c.v[1] = s->tag; c.v[2] = s->sweep; c.v[3] = s->blk++;
#if defined(__HIP_DEVICE_COMPILE__)
    c = pht_philox4x32_10_unrolled(c, __builtin_amdgcn_readfirstlane(s->k0), __builtin_amdgcn_readfirstlane(s->k1));
#else
    c = pht_philox4x32_10_unrolled(c, s->k0, s->k1);
#endif
    s->b0 = c.v[0]; s->b1 = c.v[1]; s->b2 = c.v[2]; s->b3 = c.v[3];
    s->nb = 1;
  }
}
#endif

PHT_HD2 uint32_t pht_next_w(pht_stream *s) {
  if (s->na == 0) {
    if (s->nb) {
      s->a0 = s->b0; s->a1 = s->b1; s->a2 = s->b2; s->a3 = s->b3;
      s->nb = 0;
    } else {
      pht_u32x4 w = pht_stream_block(s);
      s->a0 = w.v[0]; s->a1 = w.v[1]; s->a2 = w.v[2]; s->a3 = w.v[3];
    }
    s->na = 4;
  }
  const uint32_t w = s->a0;
  s->a0 = s->a1; s->a1 = s->a2; s->a2 = s->a3;
  s->na--;
  return w;
}

/* number of words drawn so far */
PHT_HD2 uint32_t pht_stream_pos(const pht_stream *s) {
  return 4u * s->blk - (uint32_t)s->na - 4u * (uint32_t)s->nb;
}

PHT_HD2 double pht_next_u(pht_stream *s) {
  return (double)(2.0 * (double)pht_next_w(s) + 1.0) * 1.16415321826934814453125e-10; /* 2^-33 */
}

PHT_HD2 double pht_next_u53(pht_stream *s) {
  const uint32_t a = pht_next_w(s);
  const uint32_t b = pht_next_w(s);
  return pht_u01(a, b);
}

/* the uniform of an exponential draw E = -log(U) (device spec, r06): one
 * word when that word is >= 2^24 (U >= 2^-8, probability 1 - 2^-8), U = the
 * centre of the word's 2^-32 cell; below, a second word places U on
 * pht_u01's 2^-52 grid, so the tail of -log U (E > 5.5) keeps the
 * resolution of the two-word uniform.  Words per exponential 2 -> 1.004
 * (the MHRS attempt search draws one per jump; until r05 every exponential
 * took pht_next_u53's two words) */
PHT_HD2 double pht_next_uexp(pht_stream *s) {
  const uint32_t a = pht_next_w(s);
  if (a >= (1u << 24)) return pht_u01(a, 1u << 31);
  return pht_u01(a, pht_next_w(s));
}

/* reposition to word index pos (replay) */
PHT_HD2 void pht_stream_seek(pht_stream *s, uint32_t pos) {
  s->blk = pos >> 2; s->na = 0; s->nb = 0;
  for (uint32_t i = 0; i < (pos & 3u); i++) (void)pht_next_w(s);
}

#endif /* PHT_PHILOX_H */
