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
 *                                         Gibbs sweep, 64-bit-pair block
 * One Philox block yields two uniforms (words 0,1 then 2,3).  Uniform draw
 * number i of an observation comes from block i/2, half i%2, so any lane can
 * replay any observation from any draw index (used by the MHRS kernel).
 *
 * uniform: m = (w_hi << 20) | (w_lo >> 12) (52 bits), u = (2m+1) * 2^-53,
 * so u is exact and 0 < u < 1.
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

PHT_HD2 pht_u32x4 pht_philox4x32_10(pht_u32x4 c, uint32_t k0, uint32_t k1) {
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

/* Per-observation uniform stream with a one-uniform buffer. */
typedef struct {
  uint32_t k0, k1;     /* key */
  uint32_t obs, tag;   /* counter words 0,1 */
  uint32_t sweep;      /* counter word 2 */
  uint32_t blk;        /* counter word 3: next Philox block */
  double buf;          /* second uniform of the last block */
  int have;            /* buf valid */
} pht_stream;

PHT_HD2 void pht_stream_init(pht_stream *s, uint32_t k0, uint32_t k1, uint32_t obs,
                             uint32_t tag, uint32_t sweep) {
  s->k0 = k0; s->k1 = k1; s->obs = obs; s->tag = tag; s->sweep = sweep;
  s->blk = 0; s->buf = 0.0; s->have = 0;
}

/* number of uniforms drawn so far */
PHT_HD2 uint32_t pht_stream_pos(const pht_stream *s) { return 2 * s->blk - (uint32_t)s->have; }

PHT_HD2 double pht_next_u(pht_stream *s) {
  if (s->have) { s->have = 0; return s->buf; }
  pht_u32x4 c; c.v[0] = s->obs; c.v[1] = s->tag; c.v[2] = s->sweep; c.v[3] = s->blk++;
  pht_u32x4 w = pht_philox4x32_10(c, s->k0, s->k1);
  s->buf = pht_u01(w.v[2], w.v[3]);
  s->have = 1;
  return pht_u01(w.v[0], w.v[1]);
}

/* reposition to uniform index pos (replay) */
PHT_HD2 void pht_stream_seek(pht_stream *s, uint32_t pos) {
  s->blk = pos >> 1; s->have = 0;
  if (pos & 1u) (void)pht_next_u(s);
}

#endif /* PHT_PHILOX_H */
