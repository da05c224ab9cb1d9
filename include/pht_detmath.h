/*
 * pht_detmath.h — deterministic FP64 exp/log shared by the HIP kernels and
 * the oracle's device-mode restatement (oracle/pht_oracle.c, ORC_DEV).
 *
 * Why: the reference evaluates exp/log through glibc (src/arms.c:792-812,
 * src/Simulate_AbsCTMC_eq_Aslett_ECS.c:25,124-134,163,170, ...).  glibc and
 * the GPU's ocml differ in the last ulp on some inputs, and ARMS / the
 * categorical jumps turn last-ulp differences into different discrete
 * decisions.  Defining exp/log here from IEEE-754 basic operations and
 * explicit fma() only (no contraction: every translation unit that includes
 * this is compiled with -ffp-contract=off) makes a GPU lane and the CPU
 * restatement produce bit-identical results for the same inputs.
 *
 * Accuracy: < 1 ulp over the full double range (checked against mpmath in
 * tests/test_detmath.py).  Not correctly rounded; deterministic.
 *   exp: x = (64 k + j) ln2/64 + r (|r| <= ln2/128; two-part ln2/64, the
 *        1.5·2^52 shifter for the integer), e^x = 2^k · 2^(j/64) · e^r with
 *        2^(j/64) from a 64-entry (hi, lo) table and e^r - 1 a degree-6
 *        Taylor polynomial by fma Horner.
 *   log: x = 2^k z, z in [sqrt(1/2), sqrt(2)); z's bin (7 mantissa bits)
 *        gives c with invc = RN(1/c) and logc = -log(invc) (double-double);
 *        r = fma(z, invc, -1) (|r| < 2^-7), log x = k ln2 + logc + log1p(r)
 *        with a degree-8 Taylor log1p; no division.
 */
#ifndef PHT_DETMATH_H
#define PHT_DETMATH_H

#include <math.h>
#include <stdint.h>
#include <string.h>

#if defined(__HIPCC__)
#define PHT_HD __host__ __device__ __forceinline__
#else
#define PHT_HD static inline
#endif

PHT_HD uint64_t pht_d2u(double x) { uint64_t u; memcpy(&u, &x, 8); return u; }
PHT_HD double pht_u2d(uint64_t u) { double x; memcpy(&x, &u, 8); return x; }

/* 2^(j/64), j = 0..63, as (hi, lo) pairs: hi = RN(2^(j/64)), lo = RN(2^(j/64) - hi) */
#if defined(__HIP_DEVICE_COMPILE__)
static __constant__ const double pht_exp_tab[128] = {
#else
static const double pht_exp_tab[128] = {
#endif
    0x1.0000000000000p+0, 0x0.0p+0,
    0x1.02c9a3e778061p+0, -0x1.19083535b085dp-56,
    0x1.059b0d3158574p+0, 0x1.d73e2a475b465p-55,
    0x1.0874518759bc8p+0, 0x1.186be4bb284ffp-57,
    0x1.0b5586cf9890fp+0, 0x1.8a62e4adc610bp-54,
    0x1.0e3ec32d3d1a2p+0, 0x1.03a1727c57b53p-59,
    0x1.11301d0125b51p+0, -0x1.6c51039449b3ap-54,
    0x1.1429aaea92de0p+0, -0x1.32fbf9af1369ep-54,
    0x1.172b83c7d517bp+0, -0x1.19041b9d78a76p-55,
    0x1.1a35beb6fcb75p+0, 0x1.e5b4c7b4968e4p-55,
    0x1.1d4873168b9aap+0, 0x1.e016e00a2643cp-54,
    0x1.2063b88628cd6p+0, 0x1.dc775814a8495p-55,
    0x1.2387a6e756238p+0, 0x1.9b07eb6c70573p-54,
    0x1.26b4565e27cddp+0, 0x1.2bd339940e9d9p-55,
    0x1.29e9df51fdee1p+0, 0x1.612e8afad1255p-55,
    0x1.2d285a6e4030bp+0, 0x1.0024754db41d5p-54,
    0x1.306fe0a31b715p+0, 0x1.6f46ad23182e4p-55,
    0x1.33c08b26416ffp+0, 0x1.32721843659a6p-54,
    0x1.371a7373aa9cbp+0, -0x1.63aeabf42eae2p-54,
    0x1.3a7db34e59ff7p+0, -0x1.5e436d661f5e3p-56,
    0x1.3dea64c123422p+0, 0x1.ada0911f09ebcp-55,
    0x1.4160a21f72e2ap+0, -0x1.ef3691c309278p-58,
    0x1.44e086061892dp+0, 0x1.89b7a04ef80d0p-59,
    0x1.486a2b5c13cd0p+0, 0x1.3c1a3b69062f0p-56,
    0x1.4bfdad5362a27p+0, 0x1.d4397afec42e2p-56,
    0x1.4f9b2769d2ca7p+0, -0x1.4b309d25957e3p-54,
    0x1.5342b569d4f82p+0, -0x1.07abe1db13cadp-55,
    0x1.56f4736b527dap+0, 0x1.9bb2c011d93adp-54,
    0x1.5ab07dd485429p+0, 0x1.6324c054647adp-54,
    0x1.5e76f15ad2148p+0, 0x1.ba6f93080e65ep-54,
    0x1.6247eb03a5585p+0, -0x1.383c17e40b497p-54,
    0x1.6623882552225p+0, -0x1.bb60987591c34p-54,
    0x1.6a09e667f3bcdp+0, -0x1.bdd3413b26456p-54,
    0x1.6dfb23c651a2fp+0, -0x1.bbe3a683c88abp-57,
    0x1.71f75e8ec5f74p+0, -0x1.16e4786887a99p-55,
    0x1.75feb564267c9p+0, -0x1.0245957316dd3p-54,
    0x1.7a11473eb0187p+0, -0x1.41577ee04992fp-55,
    0x1.7e2f336cf4e62p+0, 0x1.05d02ba15797ep-56,
    0x1.82589994cce13p+0, -0x1.d4c1dd41532d8p-54,
    0x1.868d99b4492edp+0, -0x1.fc6f89bd4f6bap-54,
    0x1.8ace5422aa0dbp+0, 0x1.6e9f156864b27p-54,
    0x1.8f1ae99157736p+0, 0x1.5cc13a2e3976cp-55,
    0x1.93737b0cdc5e5p+0, -0x1.75fc781b57ebcp-57,
    0x1.97d829fde4e50p+0, -0x1.d185b7c1b85d1p-54,
    0x1.9c49182a3f090p+0, 0x1.c7c46b071f2bep-56,
    0x1.a0c667b5de565p+0, -0x1.359495d1cd533p-54,
    0x1.a5503b23e255dp+0, -0x1.d2f6edb8d41e1p-54,
    0x1.a9e6b5579fdbfp+0, 0x1.0fac90ef7fd31p-54,
    0x1.ae89f995ad3adp+0, 0x1.7a1cd345dcc81p-54,
    0x1.b33a2b84f15fbp+0, -0x1.2805e3084d708p-57,
    0x1.b7f76f2fb5e47p+0, -0x1.5584f7e54ac3bp-56,
    0x1.bcc1e904bc1d2p+0, 0x1.23dd07a2d9e84p-55,
    0x1.c199bdd85529cp+0, 0x1.11065895048ddp-55,
    0x1.c67f12e57d14bp+0, 0x1.2884dff483cadp-54,
    0x1.cb720dcef9069p+0, 0x1.503cbd1e949dbp-56,
    0x1.d072d4a07897cp+0, -0x1.cbc3743797a9cp-54,
    0x1.d5818dcfba487p+0, 0x1.2ed02d75b3707p-55,
    0x1.da9e603db3285p+0, 0x1.c2300696db532p-54,
    0x1.dfc97337b9b5fp+0, -0x1.1a5cd4f184b5cp-54,
    0x1.e502ee78b3ff6p+0, 0x1.39e8980a9cc8fp-55,
    0x1.ea4afa2a490dap+0, -0x1.e9c23179c2893p-54,
    0x1.efa1bee615a27p+0, 0x1.dc7f486a4b6b0p-54,
    0x1.f50765b6e4540p+0, 0x1.9d3e12dd8a18bp-54,
    0x1.fa7c1819e90d8p+0, 0x1.74853f3a5931ep-55,
};

/* Where the device reads the tables: by default the __constant__ copies
 * (vector-memory loads through the L1); with PHT_DETMATH_LDS, workgroup LDS
 * copies that every kernel stages first (pht_stage_math_tables). */
#if defined(__HIP_DEVICE_COMPILE__) && defined(PHT_DETMATH_LDS)
__shared__ double pht_lds_exp_tab[128];
__shared__ double pht_lds_log_tab[768];
#define PHT_EXP_TAB pht_lds_exp_tab
#define PHT_LOG_TAB pht_lds_log_tab
#else
#define PHT_EXP_TAB pht_exp_tab
#define PHT_LOG_TAB pht_log_tab
#endif

#ifndef PHT_EXP_ASMC
#define PHT_EXP_ASMC(c) "v"(c)
#endif
#ifndef PHT_EXP_LOWK
#define PHT_EXP_LOWK 1
#endif

/* Core of every exp below: e^x for -1100 <= x <= 709.78 with no
 * special-case handling (callers clamp to that domain or select around it).
 * Below PHT_EXP_LO (-745.13) the result is 0 from the final ldexp's
 * rounding (checked for the 2e7 doubles below PHT_EXP_LO and on a 1e-4 grid
 * down to -1100), so the callers clamp there instead of selecting 0. */
PHT_HD double pht_exp_core(double x) {
  const double INV_LN2_N = 0x1.71547652b82fep+6; /* 64/ln2 */
  const double LN2_HI_N = 0x1.62e42fefa39efp-7;  /* ln2/64 rounded */
  const double LN2_LO_N = 0x1.abc9e3b39803fp-62; /* ln2/64 - LN2_HI_N */
  const double SHIFT = 6755399441055744.0;       /* 1.5 * 2^52 */
  const double ts = fma(x, INV_LN2_N, SHIFT); /* SHIFT + round-to-nearest-even integer */
  const double kd = ts - SHIFT;
  double r = fma(-kd, LN2_HI_N, x);
  r = fma(-kd, LN2_LO_N, r); /* |r| <= ln2/128 */
#if PHT_EXP_LOWK
  /* the integer is the low word of ts (its mantissa is 2^51 + ki) */
  uint64_t tsb;
  memcpy(&tsb, &ts, sizeof tsb);
  const int ki = (int)(uint32_t)tsb;
#else
  const int ki = (int)kd;
#endif
  const int idx = ki & 63;
  const int k = ki >> 6; /* floor(ki / 64) */
  const double sc = PHT_EXP_TAB[2 * idx], tail = PHT_EXP_TAB[2 * idx + 1];
#if defined(__HIP_DEVICE_COMPILE__) && defined(PHT_EXP_ASMFMA)
  /* the same fmas as three-address v_fma_f64 (no v_fmac with a copied
   * constant accumulator under register pressure) */
  double q;
  const double c6 = 1.3888888888888889419e-03, c5 = 8.3333333333333332177e-03, c4 = 4.1666666666666664354e-02,
               c3 = 1.6666666666666665741e-01;
  asm("v_fma_f64 %0, %1, %2, %3" : "=v"(q) : PHT_EXP_ASMC(c6), "v"(r), PHT_EXP_ASMC(c5));
  asm("v_fma_f64 %0, %1, %2, %3" : "=v"(q) : "v"(q), "v"(r), PHT_EXP_ASMC(c4));
  asm("v_fma_f64 %0, %1, %2, %3" : "=v"(q) : "v"(q), "v"(r), PHT_EXP_ASMC(c3));
  q = fma(q, r, 0.5);
#else
  double q = 1.3888888888888889419e-03;   /* 1/6! */
  q = fma(q, r, 8.3333333333333332177e-03); /* 1/5! */
  q = fma(q, r, 4.1666666666666664354e-02); /* 1/4! */
  q = fma(q, r, 1.6666666666666665741e-01); /* 1/3! */
  q = fma(q, r, 0.5);
#endif
  const double p = fma(r * r, q, r); /* e^r - 1 */
  /* res * 2^k with one rounding (subnormal results) */
  return ldexp(sc + fma(sc, p, tail), k);
}

#define PHT_EXP_HI 709.782712893383973096
#define PHT_EXP_LO (-745.133219101941108420)
#define PHT_EXP_FLUSH (-1100.0) /* pht_exp_core(x) = 0 for x <= PHT_EXP_LO's predecessor */

/* e^x for every x: straight-line (selects, no branches on the GPU). */
PHT_HD double pht_exp(double x) {
  const double xc = fmin(fmax(x, PHT_EXP_FLUSH), PHT_EXP_HI); /* NaN -> FLUSH */
  const double res = pht_exp_core(xc);
  const double out = (x > PHT_EXP_HI) ? INFINITY : res;
  return (x != x) ? x : out;
}

/* e^x for x >= LO (no underflow or NaN handling): pht_exp(x) there. */
PHT_HD double pht_exp_hi(double x) {
  const double res = pht_exp_core(fmin(x, PHT_EXP_HI));
  return (x > PHT_EXP_HI) ? INFINITY : res;
}

/* e^x for x <= 709.78 (no overflow or NaN handling): pht_exp(x) there. */
PHT_HD double pht_exp_neg(double x) { return pht_exp_core(fmax(x, PHT_EXP_FLUSH)); }

/* log table, index i + 128 h (i = top 7 mantissa bits of m in [1,2), h = 1
 * when m >= sqrt2 and z = m/2 is used): (invc, logc_hi, logc_lo) with
 * c = the bin centre (c = 1 for the two bins touching 1), invc = RN(1/c),
 * logc = -log(invc) to double-double precision. */
#if defined(__HIP_DEVICE_COMPILE__)
static __constant__ const double pht_log_tab[768] = {
#else
static const double pht_log_tab[768] = {
#endif
    0x1.0000000000000p+0, 0x0.0p+0, 0x0.0p+0,
    0x1.fa11caa01fa12p-1, 0x1.7dc475f810a69p-7, 0x1.74944bc161072p-61,
    0x1.f6310aca0dbb5p-1, 0x1.3cea44346a584p-6, -0x1.865ad48159d00p-61,
    0x1.f25f644230ab5p-1, 0x1.b9fc027af919ap-6, -0x1.90ae69229dc86p-60,
    0x1.ee9c7f8458e02p-1, 0x1.1b0d98923d97fp-5, -0x1.74d7444dd6241p-59,
    0x1.eae807aba01ebp-1, 0x1.58a5bafc8e4d3p-5, -0x1.cab8569c56e40p-64,
    0x1.e741aa59750e4p-1, 0x1.95c830ec8e3f2p-5, 0x1.eb41d00a417e9p-60,
    0x1.e3a9179dc1a73p-1, 0x1.d276b8adb0b56p-5, 0x1.078f14c95ff53p-59,
    0x1.e01e01e01e01ep-1, 0x1.075983598e471p-4, 0x1.006d2999e22dcp-58,
    0x1.dca01dca01dcap-1, 0x1.253f62f0a1417p-4, 0x1.1f6d34e01d981p-61,
    0x1.d92f2231e7f8ap-1, 0x1.42edcbea646eep-4, -0x1.511583653349bp-58,
    0x1.d5cac807572b2p-1, 0x1.60658a93750c4p-4, -0x1.f108b1d8436d3p-59,
    0x1.d272ca3fc5b1ap-1, 0x1.7da766d7b12d0p-4, 0x1.a2240644d7da2p-59,
    0x1.cf26e5c44bfc6p-1, 0x1.9ab42462033aep-4, -0x1.a099e1c184e8ep-59,
    0x1.cbe6d9601cbe7p-1, 0x1.b78c82bb0eda0p-4, -0x1.3ef0e61f9b03cp-58,
    0x1.c8b265afb8a42p-1, 0x1.d4313d66cb35dp-4, 0x1.b90dd951d90fap-58,
    0x1.c5894d10d4986p-1, 0x1.f0a30c01162a4p-4, 0x1.8be64b8b7759bp-59,
    0x1.c26b5392ea01cp-1, 0x1.0671512ca596fp-3, -0x1.2f39b81479b67p-58,
    0x1.bf583ee868d8bp-1, 0x1.14785846742acp-3, 0x1.94409f1d3f83ap-60,
    0x1.bc4fd65883e7bp-1, 0x1.2266f190a5acdp-3, -0x1.dab840e7f6177p-57,
    0x1.b951e2b18ff23p-1, 0x1.303d718e47fd5p-3, -0x1.b5ae71f658247p-57,
    0x1.b65e2e3beee05p-1, 0x1.3dfc2b0ecc62ap-3, 0x1.ba62b8c13f7f4p-57,
    0x1.b37484ad806cep-1, 0x1.4ba36f39a55e5p-3, -0x1.f767e433c98aap-57,
    0x1.b094b31d922a4p-1, 0x1.59338d9982085p-3, 0x1.8d16eaaba9419p-57,
    0x1.adbe87f94905ep-1, 0x1.66acd4272ad51p-3, -0x1.9201c9c3d5165p-59,
    0x1.aaf1d2f87ebfdp-1, 0x1.740f8f54037a3p-3, 0x1.6d9bf9d57b326p-58,
    0x1.a82e65130e159p-1, 0x1.815c0a14357e9p-3, 0x1.141b7f8c5fa9ep-58,
    0x1.a574107688a4ap-1, 0x1.8e928de886d41p-3, 0x1.2589eb96a6240p-59,
    0x1.a2c2a87c51ca0p-1, 0x1.9bb362e7dfb85p-3, -0x1.51439c1ff83e7p-58,
    0x1.a01a01a01a01ap-1, 0x1.a8becfc882f19p-3, -0x1.a8c37918c39ebp-58,
    0x1.9d79f176b682dp-1, 0x1.b5b519e8fb5a6p-3, -0x1.d5d8023e61e5fp-57,
    0x1.9ae24ea5510dap-1, 0x1.c2968558c18c2p-3, 0x1.6108e3ae024acp-60,
    0x1.9852f0d8ec0ffp-1, 0x1.cf6354e09c5ddp-3, 0x1.339a07d55b696p-57,
    0x1.95cbb0be377aep-1, 0x1.dc1bca0abec7bp-3, 0x1.c698a33316dfbp-58,
    0x1.934c67f9b2ce6p-1, 0x1.e8c0252aa5a60p-3, -0x1.dc074737f9135p-60,
    0x1.90d4f120190d5p-1, 0x1.f550a564b7b37p-3, -0x1.13a09202fe73dp-57,
    0x1.8e6527af1373fp-1, 0x1.00e6c45ad501dp-2, -0x1.3b9568ff6feadp-57,
    0x1.8bfce8062ff3ap-1, 0x1.071b85fcd590dp-2, 0x1.08b83fcbdef40p-57,
    0x1.899c0f601899cp-1, 0x1.0d46b579ab74bp-2, 0x1.21f640e1e5ec9p-56,
    0x1.87427bcc092b9p-1, 0x1.136870293a8b0p-2, 0x1.86cc531dba494p-57,
    0x1.84f00c2780614p-1, 0x1.1980d2dd4236fp-2, -0x1.02c2e4f1b2eb9p-56,
    0x1.82a4a0182a4a0p-1, 0x1.1f8ff9e48a2f3p-2, -0x1.93fbf3418960dp-57,
    0x1.8060180601806p-1, 0x1.2596010df763ap-2, -0x1.9eed8ae0ebd3cp-59,
    0x1.7e225515a4f1dp-1, 0x1.2b9303ab89d25p-2, -0x1.85ad7f614ab51p-58,
    0x1.7beb3922e017cp-1, 0x1.31871c9544185p-2, -0x1.ea3598981366fp-57,
    0x1.79baa6bb6398bp-1, 0x1.3772662bfd85cp-2, 0x1.02a7589fba088p-57,
    0x1.77908119ac60dp-1, 0x1.3d54fa5c1f710p-2, 0x1.53668e578d9cdp-58,
    0x1.756cac201756dp-1, 0x1.432ef2a04e813p-2, -0x1.83262e2b59206p-57,
    0x1.734f0c541fe8dp-1, 0x1.49006804009d0p-2, -0x1.bff0d07c5df6dp-59,
    0x1.713786d9c7c09p-1, 0x1.4ec9732600269p-2, -0x1.1aa87d977dc5ep-56,
    0x1.6f26016f26017p-1, 0x1.548a2c3add263p-2, -0x1.58ce7bf1846eep-56,
    0x1.6d1a62681c861p-1, 0x1.5a42ab0f4cfe2p-2, -0x1.c6bcb7dee9a3dp-56,
    0x1.6b1490aa31a3dp-1, 0x1.5ff3070a793d4p-2, -0x1.063077d7e37b7p-56,
    0x1.691473a88d0c0p-1, 0x1.659b57303e1f2p-2, 0x1.db0af8efb83c7p-62,
    0x1.6719f3601671ap-1, 0x1.6b3bb2235943dp-2, 0x1.957a93326784dp-56,
    0x1.6524f853b4aa3p-1, 0x1.70d42e2789236p-2, 0x1.ee99bf7143954p-56,
    0x1.63356b88ac0dep-1, 0x1.7664e1239dbcfp-2, -0x1.d6d5d64f5daf8p-57,
    0x1.614b36831ae94p-1, 0x1.7bede0a37afbfp-2, -0x1.6783cb9801a5bp-56,
    0x1.5f66434292dfcp-1, 0x1.816f41da0d495p-2, 0x1.76dc35fb48fe4p-56,
    0x1.5d867c3ece2a5p-1, 0x1.86e919a330ba1p-2, -0x1.700c9d2029045p-56,
    0x1.5babcc647fa91p-1, 0x1.8c5b7c858b48bp-2, 0x1.d754b0205fa6cp-56,
    0x1.59d61f123ccaap-1, 0x1.91c67eb45a83ep-2, 0x1.5e3ea3b96a3dfp-57,
    0x1.5805601580560p-1, 0x1.972a341135159p-2, -0x1.5a3f62db48f27p-56,
    0x1.56397ba7c52e2p-1, 0x1.9c86b02dc0862p-2, 0x1.7e81149622bdfp-56,
    0x1.54725e6bb82fep-1, 0x1.a1dc064d5b995p-2, 0x1.a0128698ba0b8p-56,
    0x1.52aff56a8054bp-1, 0x1.a72a4966bd9e9p-2, 0x1.529dac69f61f1p-56,
    0x1.50f22e111c4c5p-1, 0x1.ac718c258b0e5p-2, 0x1.682c7ade8dee3p-56,
    0x1.4f38f62dd4c9bp-1, 0x1.b1b1e0ebdfc5ap-2, -0x1.0ee1a7dd74ea6p-58,
    0x1.4d843bedc2c4cp-1, 0x1.b6eb59d3cf35cp-2, 0x1.1524332cd95c4p-56,
    0x1.4bd3edda68fe1p-1, 0x1.bc1e08b0dad0ap-2, -0x1.385e3e3ea99a8p-58,
    0x1.4a27fad76014ap-1, 0x1.c149ff115f027p-2, 0x1.46868de7f39f6p-57,
    0x1.4880522014880p-1, 0x1.c66f4e3ff6ff9p-2, -0x1.82947258b6889p-58,
    0x1.46dce34596066p-1, 0x1.cb8e0744d7acap-2, 0x1.c5bbc32ef5aebp-56,
    0x1.453d9e2c776cap-1, 0x1.d0a63ae721e64p-2, 0x1.4acce112c40f2p-57,
    0x1.43a2730abee4dp-1, 0x1.d5b7f9ae2c684p-2, 0x1.4841807b53f96p-57,
    0x1.420b5265e5951p-1, 0x1.dac353e2c5955p-2, -0x1.abc65a3f2f204p-56,
    0x1.40782d10e6566p-1, 0x1.dfc859906d5b5p-2, 0x1.51e1399f96398p-56,
    0x1.3ee8f42a5af07p-1, 0x1.e4c71a8687704p-2, -0x1.34c36e0f052b9p-56,
    0x1.3d5d991aa75c6p-1, 0x1.e9bfa659861f5p-2, -0x1.de45038241ecfp-56,
    0x1.3bd60d9232955p-1, 0x1.eeb20c640ddf3p-2, -0x1.81e47141b8404p-56,
    0x1.3a524387ac822p-1, 0x1.f39e5bc811e5dp-2, 0x1.200e221139873p-59,
    0x1.38d22d366088ep-1, 0x1.f884a36fe9ec1p-2, 0x1.618ae4f008400p-56,
    0x1.3755bd1c945eep-1, 0x1.fd64f20f61571p-2, -0x1.b615859d5a349p-62,
    0x1.35dce5f9f2af8p-1, 0x1.011fab125ff8ap-1, 0x1.4043750211778p-55,
    0x1.34679ace01346p-1, 0x1.0389eefce633cp-1, 0x1.8aae29a41ba4ap-59,
    0x1.32f5ced6a1dfap-1, 0x1.05f14bd26459cp-1, 0x1.935b8ee4f9efep-58,
    0x1.3187758e9ebb6p-1, 0x1.0855c884b450ep-1, 0x1.785826e49f318p-55,
    0x1.301c82ac40260p-1, 0x1.0ab76bece14d2p-1, 0x1.02936cabac09ap-56,
    0x1.2eb4ea1fed14bp-1, 0x1.0d163ccb9d6b8p-1, 0x1.6119595d0f3c3p-59,
    0x1.2d50a012d50a0p-1, 0x1.0f7241c9b497dp-1, 0x1.ba8443b9db19dp-55,
    0x1.2bef98e5a3711p-1, 0x1.11cb81787ccf8p-1, 0x1.dc70f563f9920p-56,
    0x1.2a91c92f3c105p-1, 0x1.1422025243d45p-1, 0x1.7e5e3b6a496ecp-55,
    0x1.293725bb804a5p-1, 0x1.1675cababa60ep-1, -0x1.cb19c15477c8ep-56,
    0x1.27dfa38a1ce4dp-1, 0x1.18c6e0ff5cf07p-1, -0x1.9a6baf4f4e637p-56,
    0x1.268b37cd60127p-1, 0x1.1b154b57da29ep-1, 0x1.2770a5c124ab5p-56,
    0x1.2539d7e9177b2p-1, 0x1.1d610fe677003p-1, 0x1.d27563647963dp-56,
    0x1.23eb79717605bp-1, 0x1.1faa34b87094cp-1, 0x1.c42f71ef43276p-55,
    0x1.22a0122a0122ap-1, 0x1.21f0bfc65beecp-1, -0x1.c24f0c9187c92p-57,
    0x1.21579804855e6p-1, 0x1.2434b6f483934p-1, -0x1.bebb8cf0f6d11p-57,
    0x1.2012012012012p-1, 0x1.26762013430e0p-1, -0x1.86a95781c6727p-56,
    0x1.1ecf43c7fb84cp-1, 0x1.28b500df60783p-1, 0x1.813f3f4aaa9a3p-60,
    0x1.1d8f5672e4abdp-1, 0x1.2af15f02640acp-1, 0x1.ed8322925675ap-56,
    0x1.1c522fc1ce059p-1, 0x1.2d2b4012edc9dp-1, 0x1.9ae9d3664e355p-55,
    0x1.1b17c67f2bae3p-1, 0x1.2f62a99509546p-1, -0x1.7dcbcc6300133p-55,
    0x1.19e0119e0119ep-1, 0x1.3197a0fa7fe6ap-1, 0x1.f6348fb97128fp-57,
    0x1.18ab083902bdbp-1, 0x1.33ca2ba328994p-1, 0x1.1c6ba66fd0910p-55,
    0x1.1778a191bd684p-1, 0x1.35fa4edd36ea0p-1, 0x1.727d468096436p-56,
    0x1.1648d50fc3201p-1, 0x1.38280fe58797fp-1, -0x1.756f4d8a9b974p-57,
    0x1.151b9a3fdd5c9p-1, 0x1.3a5373e7ebdf9p-1, 0x1.5ce11148e1124p-56,
    0x1.13f0e8d344724p-1, 0x1.3c7c7fff73206p-1, -0x1.e80db7025bed1p-60,
    0x1.12c8b89edc0acp-1, 0x1.3ea33936b2f5bp-1, 0x1.f66e975ec9f52p-59,
    0x1.11a3019a74826p-1, 0x1.40c7a4880dceap-1, 0x1.13c8b79ff2789p-58,
    0x1.107fbbe011080p-1, 0x1.42e9c6ddf80bfp-1, -0x1.4d411c2cd7cf1p-55,
    0x1.0f5edfab325a2p-1, 0x1.4509a5133bb0ap-1, -0x1.5701d7ad284a5p-55,
    0x1.0e40655826011p-1, 0x1.472743f33aaadp-1, -0x1.a930fed5d6b7ep-60,
    0x1.0d24456359e3ap-1, 0x1.4942a83a2fc07p-1, 0x1.2a18a88ca56b5p-56,
    0x1.0c0a7868b4171p-1, 0x1.4b5bd6956e273p-1, -0x1.2c7a06beea772p-55,
    0x1.0af2f722eecb5p-1, 0x1.4d72d3a39fd01p-1, 0x1.01a9a829c011bp-56,
    0x1.09ddba6af8360p-1, 0x1.4f87a3f5026e9p-1, -0x1.68ca8b1bcea9dp-55,
    0x1.08cabb37565e2p-1, 0x1.519a4c0ba3446p-1, 0x1.a332128e4a77fp-55,
    0x1.07b9f29b8eae2p-1, 0x1.53aad05b99b7cp-1, -0x1.7722c14b894e2p-57,
    0x1.06ab59c7912fbp-1, 0x1.55b9354b40bcep-1, -0x1.1f342e541a63dp-59,
    0x1.059eea0727586p-1, 0x1.57c57f336f191p-1, 0x1.1eac5c4377e6ep-55,
    0x1.04949cc1664c5p-1, 0x1.59cfb25fae87fp-1, -0x1.bb94822ace357p-57,
    0x1.038c6b78247fcp-1, 0x1.5bd7d30e71c73p-1, -0x1.c9649352e8e44p-67,
    0x1.02864fc7729e9p-1, 0x1.5ddde57149923p-1, 0x1.0fa37d75ef285p-59,
    0x1.0182436517a37p-1, 0x1.5fe1edad18919p-1, 0x1.92e93de3ce483p-56,
    0x1.0080402010080p-1, 0x1.61e3efda46467p-1, 0x1.7923604841473p-57,
    0x1.fe01fe01fe020p+0, -0x1.60e52f45788e4p-1, 0x1.ab432fd38e6b4p-55,
    0x1.fa11caa01fa12p+0, -0x1.5ced1e17c35c6p-1, 0x1.bfed5f5539822p-55,
    0x1.f6310aca0dbb5p+0, -0x1.58fcddce004c3p-1, -0x1.6ff974af45a4ep-57,
    0x1.f25f644230ab5p+0, -0x1.55144fdbcbd62p-1, -0x1.a26a6522e0f04p-55,
    0x1.ee9c7f8458e02p+0, -0x1.513356667fc57p-1, -0x1.2d32661ea9644p-55,
    0x1.eae807aba01ebp+0, -0x1.4d59d43fdaba2p-1, -0x1.6ca4e051a2d6bp-59,
    0x1.e741aa59750e4p+0, -0x1.4987ace0dabb0p-1, -0x1.1a2b8d65e7d81p-57,
    0x1.e3a9179dc1a73p+0, -0x1.45bcc464c893ap-1, 0x1.7527fee593fabp-56,
    0x1.e01e01e01e01ep+0, -0x1.41f8ff8471d61p-1, -0x1.aeba65347de21p-58,
    0x1.dca01dca01dcap+0, -0x1.3e3c43918f76cp-1, -0x1.51673d064b8bap-55,
    0x1.d92f2231e7f8ap+0, -0x1.3a86767257112p-1, 0x1.fff85db98d94dp-55,
    0x1.d5cac807572b2p+0, -0x1.36d77e9d34fd7p-1, 0x1.0b0a8308afc73p-55,
    0x1.d272ca3fc5b1ap+0, -0x1.332f4314ad795p-1, -0x1.778562eafd08bp-56,
    0x1.cf26e5c44bfc6p+0, -0x1.2f8dab6363379p-1, -0x1.efee8ff5e4508p-55,
    0x1.cbe6d9601cbe7p+0, -0x1.2bf29f9841c3bp-1, -0x1.fb861d3b7ec4ep-56,
    0x1.c8b265afb8a42p+0, -0x1.285e0842ca384p-1, 0x1.e13cc9506f200p-55,
    0x1.c5894d10d4986p+0, -0x1.24cfce6f80d9bp-1, 0x1.42d972deeb73ap-55,
    0x1.c26b5392ea01cp+0, -0x1.2147dba47a393p-1, -0x1.fbcc28dc5b38cp-55,
    0x1.bf583ee868d8bp+0, -0x1.1dc619de06944p-1, -0x1.9285d9c1c40bcp-56,
    0x1.bc4fd65883e7bp+0, -0x1.1a4a738b7a33cp-1, -0x1.324c084f261f6p-57,
    0x1.b951e2b18ff23p+0, -0x1.16d4d38c119fap-1, -0x1.0d42395d882c6p-57,
    0x1.b65e2e3beee05p+0, -0x1.1365252bf0865p-1, 0x1.98b3bc5683ddep-55,
    0x1.b37484ad806cep+0, -0x1.0ffb54213a476p-1, -0x1.4efbab9af9928p-57,
    0x1.b094b31d922a4p+0, -0x1.0c974c89431cep-1, 0x1.1ac191a23c9cdp-56,
    0x1.adbe87f94905ep+0, -0x1.0938fae5d8e9bp-1, 0x1.0faf189f6aca2p-59,
    0x1.aaf1d2f87ebfdp+0, -0x1.05e04c1aa2c06p-1, -0x1.a831729f1c9bbp-55,
    0x1.a82e65130e159p+0, -0x1.028d2d6a963f5p-1, 0x1.3279f85effcd1p-57,
    0x1.a574107688a4ap+0, -0x1.fe7f18eb03d3ep-2, 0x1.e39d66fcf3023p-58,
    0x1.a2c2a87c51ca0p+0, -0x1.f7eeae6b5761cp-2, -0x1.acabb96138d4ep-68,
    0x1.a01a01a01a01ap+0, -0x1.f168f7fb05c52p-2, -0x1.5fac1f9c8eb9fp-60,
    0x1.9d79f176b682dp+0, -0x1.eaedd2eac990cp-2, 0x1.694a1b2d37091p-56,
    0x1.9ae24ea5510dap+0, -0x1.e47d1d32e677dp-2, -0x1.95b95578b7df4p-56,
    0x1.9852f0d8ec0ffp+0, -0x1.de16b56ef90f0p-2, 0x1.dc06406e2b617p-57,
    0x1.95cbb0be377aep+0, -0x1.d7ba7ad9e7da1p-2, 0x1.8bb88a325b67fp-57,
    0x1.934c67f9b2ce6p+0, -0x1.d1684d49f46aep-2, -0x1.c98a582717953p-56,
    0x1.90d4f120190d5p+0, -0x1.cb200d2ceb643p-2, -0x1.acd165a8b9eecp-59,
    0x1.8e6527af1373fp+0, -0x1.c4e19b84723c2p-2, 0x1.b66b67ccb006ap-56,
    0x1.8bfce8062ff3ap+0, -0x1.beacd9e271ad1p-2, -0x1.276dc3cda889fp-56,
    0x1.899c0f601899cp+0, -0x1.b881aa659bc93p-2, -0x1.13a745a3642ecp-57,
    0x1.87427bcc092b9p+0, -0x1.b25fefb60cb2ep-2, -0x1.d0c7744975beap-57,
    0x1.84f00c2780614p+0, -0x1.ac478d0205070p-2, 0x1.5173375ab5108p-56,
    0x1.82a4a0182a4a0p+0, -0x1.a63865fabd0ecp-2, 0x1.8a3822aba34bap-56,
    0x1.8060180601806p+0, -0x1.a0325ed14fda4p-2, -0x1.dfa7950fb57e7p-56,
    0x1.7e225515a4f1dp+0, -0x1.9a355c33bd6bap-2, 0x1.f2cabc74154edp-56,
    0x1.7beb3922e017cp+0, -0x1.9441434a0325ap-2, 0x1.5f1b50005e489p-56,
    0x1.79baa6bb6398bp+0, -0x1.8e55f9b349b82p-2, -0x1.2a763763baffbp-56,
    0x1.77908119ac60dp+0, -0x1.8873658327ccep-2, -0x1.56f0401db49ccp-56,
    0x1.756cac201756dp+0, -0x1.82996d3ef8bccp-2, 0x1.92a30536bb6bep-56,
    0x1.734f0c541fe8dp+0, -0x1.7cc7f7db46a0ep-2, -0x1.e3c7fdc323c2dp-56,
    0x1.713786d9c7c09p+0, -0x1.76feecb947176p-2, 0x1.398d9eb4ea363p-56,
    0x1.6f26016f26017p+0, -0x1.713e33a46a17cp-2, 0x1.f6cf40b5c71a6p-57,
    0x1.6d1a62681c861p+0, -0x1.6b85b4cffa3fdp-2, 0x1.1af2c8dafcb08p-57,
    0x1.6b1490aa31a3dp+0, -0x1.65d558d4ce00bp-2, 0x1.4e05a4748480ap-56,
    0x1.691473a88d0c0p+0, -0x1.602d08af091ecp-2, -0x1.a45db7cfd9230p-56,
    0x1.6719f3601671ap+0, -0x1.5a8cadbbedfa1p-2, -0x1.64f5081307f22p-60,
    0x1.6524f853b4aa3p+0, -0x1.54f431b7be1a8p-2, 0x1.0b3f6ef6ae452p-58,
    0x1.63356b88ac0dep+0, -0x1.4f637ebba9810p-2, 0x1.68cb3124b9245p-56,
    0x1.614b36831ae94p+0, -0x1.49da7f3bcc420p-2, 0x1.d964a168ccacbp-57,
    0x1.5f66434292dfcp+0, -0x1.44591e0539f49p-2, -0x1.a76d6dc2782dap-59,
    0x1.5d867c3ece2a5p+0, -0x1.3edf463c1683ep-2, 0x1.c852fe587def8p-57,
    0x1.5babcc647fa91p+0, -0x1.396ce359bbf53p-2, 0x1.5c5663663d163p-59,
    0x1.59d61f123ccaap+0, -0x1.3401e12aecba0p-2, -0x1.f95523adc5c9fp-57,
    0x1.5805601580560p+0, -0x1.2e9e2bce12286p-2, 0x1.f3ed72e23e134p-57,
    0x1.56397ba7c52e2p+0, -0x1.2941afb186b7cp-2, -0x1.6a4678ebaa300p-59,
    0x1.54725e6bb82fep+0, -0x1.23ec5991eba49p-2, -0x1.76eba35bbf0dfp-61,
    0x1.52aff56a8054bp+0, -0x1.1e9e1678899f5p-2, -0x1.64b0dd2687939p-58,
    0x1.50f22e111c4c5p+0, -0x1.1956d3b9bc2f9p-2, -0x1.0e75a3542856fp-58,
    0x1.4f38f62dd4c9bp+0, -0x1.14167ef367784p-2, -0x1.ef824daaf53e9p-56,
    0x1.4d843bedc2c4cp+0, -0x1.0edd060b78082p-2, -0x1.2d4b610d7d4f5p-57,
    0x1.4bd3edda68fe1p+0, -0x1.09aa572e6c6d4p-2, -0x1.f9e17343426a9p-56,
    0x1.4a27fad76014ap+0, -0x1.047e60cde83b7p-2, -0x1.08869cbf9e344p-56,
    0x1.4880522014880p+0, -0x1.feb2233ea07cbp-3, -0x1.8de00938b4c30p-61,
    0x1.46dce34596066p+0, -0x1.f474b134df228p-3, 0x1.9f1df7b5daab7p-60,
    0x1.453d9e2c776cap+0, -0x1.ea4449f04aaf5p-3, 0x1.f33919ab94074p-57,
    0x1.43a2730abee4dp+0, -0x1.e020cc6235ab5p-3, 0x1.f0adb91423f18p-57,
    0x1.420b5265e5951p+0, -0x1.d60a17f903514p-3, 0x1.50df841a71b7ap-57,
    0x1.40782d10e6566p+0, -0x1.cc000c9db3c52p-3, -0x1.67a2a8500729ep-58,
    0x1.3ee8f42a5af07p+0, -0x1.c2028ab17f9b5p-3, -0x1.c11aa3853a5f0p-57,
    0x1.3d5d991aa75c6p+0, -0x1.b811730b823d4p-3, 0x1.d7c46328983c6p-58,
    0x1.3bd60d9232955p+0, -0x1.ae2ca6f672bd8p-3, 0x1.a4a356155f779p-57,
    0x1.3a524387ac822p+0, -0x1.a454082e6ab03p-3, 0x1.e0df823a3cb3dp-58,
    0x1.38d22d366088ep+0, -0x1.9a8778debaa3ap-3, -0x1.28fbfb0e3f0fcp-58,
    0x1.3755bd1c945eep+0, -0x1.90c6db9fcbcdbp-3, 0x1.357718d7ca4cfp-58,
    0x1.35dce5f9f2af8p+0, -0x1.871213750e994p-3, 0x1.a97a0ca115d60p-57,
    0x1.34679ace01346p+0, -0x1.7d6903caf5acdp-3, 0x1.0b17c301d6e14p-57,
    0x1.32f5ced6a1dfap+0, -0x1.73cb9074fd14dp-3, 0x1.721a000b4cf01p-57,
    0x1.3187758e9ebb6p+0, -0x1.6a399dabbd383p-3, -0x1.76332bd4b341fp-57,
    0x1.301c82ac40260p+0, -0x1.60b3100b09474p-3, -0x1.526cee0fd7f4ap-57,
    0x1.2eb4ea1fed14bp+0, -0x1.5737cc9018cddp-3, 0x1.00b28ef013c72p-57,
    0x1.2d50a012d50a0p+0, -0x1.4dc7b897bc1c7p-3, -0x1.b60ae1ff0e82ep-59,
    0x1.2bef98e5a3711p+0, -0x1.4462b9dc9b3dcp-3, 0x1.85388d830c709p-59,
    0x1.2a91c92f3c105p+0, -0x1.3b08b6757f2a7p-3, -0x1.5e1ad9be0a4cdp-57,
    0x1.293725bb804a5p+0, -0x1.31b994d3a4f86p-3, 0x1.1238b5efe0665p-57,
    0x1.27dfa38a1ce4dp+0, -0x1.28753bc11aba2p-3, 0x1.7394d9fa33313p-57,
    0x1.268b37cd60127p+0, -0x1.1f3b925f25d44p-3, -0x1.08b27be4e6b15p-57,
    0x1.2539d7e9177b2p+0, -0x1.160c8024b27b0p-3, 0x1.355bfd870afebp-59,
    0x1.23eb79717605bp+0, -0x1.0ce7ecdccc28bp-3, -0x1.1b57fea88da98p-59,
    0x1.22a0122a0122ap+0, -0x1.03cdc0a51ec0dp-3, -0x1.19e2d3f8b7d10p-57,
    0x1.21579804855e6p+0, -0x1.f57bc7d9005dbp-4, 0x1.d361574fb24e2p-58,
    0x1.2012012012012p+0, -0x1.e3707ee30487bp-4, -0x1.9399d9aaf3b33p-59,
    0x1.1ecf43c7fb84cp+0, -0x1.d179788219362p-4, 0x1.b12841044a96cp-58,
    0x1.1d8f5672e4abdp+0, -0x1.bf968769fca18p-4, 0x1.06e4fb7af9c69p-58,
    0x1.1c522fc1ce059p+0, -0x1.adc77ee5aea8ep-4, -0x1.d7d8f39bee658p-58,
    0x1.1b17c67f2bae3p+0, -0x1.9c0c32d4d254dp-4, 0x1.627a0e199f569p-58,
    0x1.19e0119e0119ep+0, -0x1.8a6477a91dc29p-4, 0x1.3d4190a482421p-58,
    0x1.18ab083902bdbp+0, -0x1.78d02263d82d7p-4, -0x1.cbca5b4fdb87ep-58,
    0x1.1778a191bd684p+0, -0x1.674f089365a78p-4, -0x1.ca64e9980e048p-59,
    0x1.1648d50fc3201p+0, -0x1.55e10050e0382p-4, -0x1.9a0629e3973e4p-58,
    0x1.151b9a3fdd5c9p+0, -0x1.4485e03dbdfb0p-4, -0x1.3ba349aadbc6dp-58,
    0x1.13f0e8d344724p+0, -0x1.333d7f8183f4ap-4, 0x1.adaa06e211e9ep-59,
    0x1.12c8b89edc0acp+0, -0x1.2207b5c7854a1p-4, -0x1.b3f0431efb154p-58,
    0x1.11a3019a74826p+0, -0x1.10e45b3cae829p-4, -0x1.9b5ed72e6d974p-58,
    0x1.107fbbe011080p+0, -0x1.ffa6911ab9309p-5, 0x1.cd9f1f95c2ef1p-59,
    0x1.0f5edfab325a2p+0, -0x1.dda8adc67ee59p-5, 0x1.31936790bb3b2p-59,
    0x1.0e40655826011p+0, -0x1.bbcebfc68f424p-5, 0x1.cd1862f854848p-59,
    0x1.0d24456359e3ap+0, -0x1.9a187b573de81p-5, -0x1.b13b26f298a6ap-64,
    0x1.0c0a7868b4171p+0, -0x1.788595a3577c8p-5, -0x1.2f7c4c5b3c8bdp-62,
    0x1.0af2f722eecb5p+0, -0x1.5715c4c03cee1p-5, -0x1.5101dc4ebf91fp-59,
    0x1.09ddba6af8360p+0, -0x1.35c8bfaa13069p-5, 0x1.50830a65543a8p-63,
    0x1.08cabb37565e2p+0, -0x1.149e3e4005a8dp-5, 0x1.a9a4168fcebebp-60,
    0x1.07b9f29b8eae2p+0, -0x1.e72bf2813ce6ap-6, 0x1.8a4bba6a354fap-60,
    0x1.06ab59c7912fbp+0, -0x1.a55f548c5c427p-6, -0x1.f60d2fc36a0d9p-61,
    0x1.059eea0727586p+0, -0x1.63d6178690bbep-6, 0x1.18ed4d357c9dcp-60,
    0x1.04949cc1664c5p+0, -0x1.228fb1fea2e0ap-6, -0x1.3284991fe3d5cp-61,
    0x1.038c6b78247fcp+0, -0x1.c317384c75f0dp-7, -0x1.806208c04c21fp-61,
    0x1.02864fc7729e9p+0, -0x1.41929f968330cp-7, -0x1.3aae809b43dd0p-61,
    0x1.0182436517a37p+0, -0x1.8121214586b02p-8, 0x1.c7d68c0d910f2p-62,
    0x1.0000000000000p+0, 0x0.0p+0, 0x0.0p+0,
};

PHT_HD double pht_log(double x) {
  /* straight-line (no branches: on the GPU every special case is a select) */
  const double LN2_HI = 0x1.62e42fee00000p-1; /* 21 trailing zero bits: k*LN2_HI exact */
  const double LN2_LO = 0x1.a39ef35793c76p-33;
  const int sub = (x < 0x1p-1022);                 /* subnormal (or <= 0) */
  const double xs = sub ? x * 18014398509481984.0 : x; /* 2^54 */
  const uint64_t u = pht_d2u(xs);
  const int k0 = (int)((u >> 52) & 0x7ff) - 1023 - (sub ? 54 : 0);
  const uint64_t mant = u & 0x000fffffffffffffULL;
  const int half = (mant >= 0x6a09e667f3bcdULL); /* m >= sqrt(2): z = m/2 */
  const uint64_t zb = mant | (half ? 0x3fe0000000000000ULL : 0x3ff0000000000000ULL);
  const int k = k0 + half;
  const int idx = (int)(mant >> 45) + (half ? 128 : 0); /* top 7 bits */
  const double z = pht_u2d(zb);
  const double invc = PHT_LOG_TAB[3 * idx], logc = PHT_LOG_TAB[3 * idx + 1], logclo = PHT_LOG_TAB[3 * idx + 2];
  const double r = fma(z, invc, -1.0); /* |r| < 2^-7 */
  const double kd = (double)k;
  const double a = kd * LN2_HI;            /* exact */
  const double w = a + logc;
  const double werr = (a - w) + logc;      /* Fast2Sum: |a| >= |logc| or a = 0 */
  const double hi = w + r;
  const double lo = (w - hi) + r;          /* Fast2Sum: |w| >= |r| by construction of the bins */
  /* log1p(r) - r = r^2 q(r), degree-8 Taylor */
  double q = -0x1.0000000000000p-3;  /* -1/8 */
  q = fma(q, r, 0x1.2492492492492p-3);  /*  1/7 */
  q = fma(q, r, -0x1.5555555555555p-3); /* -1/6 */
  q = fma(q, r, 0x1.999999999999ap-3);  /*  1/5 */
  q = fma(q, r, -0x1.0000000000000p-2); /* -1/4 */
  q = fma(q, r, 0x1.5555555555555p-2);  /*  1/3 */
  q = fma(q, r, -0x1.0000000000000p-1); /* -1/2 */
  const double tail = fma(r * r, q, (lo + werr) + fma(kd, LN2_LO, logclo));
  const double res = hi + tail;
  /* specials: NaN -> NaN, x < 0 -> NaN, 0 -> -inf, +inf -> +inf */
  const double spec = (x == 0.0) ? -INFINITY : ((x < 0.0) ? NAN : x);
  return (x != x || x <= 0.0 || x == INFINITY) ? spec : res;
}

/* pht_log for a positive normal finite x (2^-1022 <= x < inf): the same
 * value without the subnormal scaling and the special-case selects (the
 * sampled uniforms of the exponential draws, [2^-53, 1 - 2^-53]) */
PHT_HD double pht_log_pos(double x) {
  const double LN2_HI = 0x1.62e42fee00000p-1;
  const double LN2_LO = 0x1.a39ef35793c76p-33;
  const uint64_t u = pht_d2u(x);
  const int k0 = (int)((u >> 52) & 0x7ff) - 1023;
  const uint64_t mant = u & 0x000fffffffffffffULL;
  const int half = (mant >= 0x6a09e667f3bcdULL);
  const uint64_t zb = mant | (half ? 0x3fe0000000000000ULL : 0x3ff0000000000000ULL);
  const int k = k0 + half;
  const int idx = (int)(mant >> 45) + (half ? 128 : 0);
  const double z = pht_u2d(zb);
  const double invc = PHT_LOG_TAB[3 * idx], logc = PHT_LOG_TAB[3 * idx + 1], logclo = PHT_LOG_TAB[3 * idx + 2];
  const double r = fma(z, invc, -1.0);
  const double kd = (double)k;
  const double a = kd * LN2_HI;
  const double w = a + logc;
  const double werr = (a - w) + logc;
  const double hi = w + r;
  const double lo = (w - hi) + r;
  double q = -0x1.0000000000000p-3;
  q = fma(q, r, 0x1.2492492492492p-3);
  q = fma(q, r, -0x1.5555555555555p-3);
  q = fma(q, r, 0x1.999999999999ap-3);
  q = fma(q, r, -0x1.0000000000000p-2);
  q = fma(q, r, 0x1.5555555555555p-2);
  q = fma(q, r, -0x1.0000000000000p-1);
  const double tail = fma(r * r, q, (lo + werr) + fma(kd, LN2_LO, logclo));
  return hi + tail;
}

/* e^u for |u| <= 2^-8 (degree-5 Taylor, truncation < 2^-60 relative) */
PHT_HD double pht_exp_taylor(double u) {
  double q = 8.3333333333333332177e-03;      /* 1/5! */
  q = fma(q, u, 4.1666666666666664354e-02);  /* 1/4! */
  q = fma(q, u, 1.6666666666666665741e-01);  /* 1/3! */
  q = fma(q, u, 0.5);
  q = fma(q, u, 1.0);
  return fma(q, u, 1.0);
}

/* Exponential vectors of the four ARMS starting points of an ECS sojourn
 * (xinit = {a, b, 2b, y_t - a}, a = y_t/1e6, b = y_t/3; the density at d
 * needs e^{lambda_i (y_t - d)}):
 *   point 2b : e^{lambda (y_t - 2b)} directly          (F)
 *   point b  : F^2                                       (y_t - b ~ 2 (y_t - 2b))
 *   point a  : e^{lambda y_t} * taylor(-lambda a)        (E0 is known)
 *   point y_t - a : taylor(lambda (y_t - (y_t - a)))
 * used when max|lambda| * max(a, y_t - (y_t - a)) <= 2^-8, else direct
 * exponentials for all four.  Returns whether the identities were used. */
PHT_HD int pht_ecs_init_ok(double lammax, double a, double x3) {
  return lammax * (a > x3 ? a : x3) <= 0x1p-8;
}

/* E0 = e^{lambda_i y_t} at an observation's FIRST sojourn (device spec, r03):
 * (F F) F from the point-2b vector F of that sojourn's starting points when
 * pht_ecs_init_ok holds (the GPU computes F there anyway, so the first absorb
 * test needs no exponential of its own), else e^{lambda_i y_t} directly.
 * Later sojourns carry E0 from the previous jump's evaluation, as before.
 * Error: ~3 ulp plus |lambda y_t| 2^-52 from y_t ~ 3 (y_t - 2b). */
PHT_HD double pht_ecs_e0_cube(double F) { return (F * F) * F; }

/* W moments (device spec, r03): Wm_k = c_k sum_i W_i lambda_i^k, k = 0..5,
 * with c_k pht_exp_taylor's coefficients (1, 1, 1/2, 1/3!, 1/4!, 1/5!), so
 * that sum_i W_i taylor5(lambda_i x) = pht_wmom_eval(Wm, x): the ECS density
 * at the starting point y_t - a (x = a's image, |lambda| x <= 2^-8) becomes
 * one degree-5 polynomial per state instead of n Taylor factors and a dot
 * product per sojourn.  Per-sweep constants (host, resident kernel, oracle
 * all call this with the same operation order). */
#define PHT_WMOM 6
PHT_HD void pht_wmoments(int n, const double *W, long wstride, const double *evals, double *out) {
  const double c[PHT_WMOM] = {1.0, 1.0, 0.5, 1.6666666666666665741e-01, 4.1666666666666664354e-02,
                              8.3333333333333332177e-03};
  for (int k = 0; k < PHT_WMOM; k++) {
    double acc = 0.0;
    for (int i = 0; i < n; i++) {
      double lp = 1.0;
      for (int m = 0; m < k; m++) lp = lp * evals[i];
      acc = fma(W[i * wstride], lp, acc);
    }
    out[k] = acc * c[k];
  }
}
/* the moments' polynomial at x (Wm_k at Wm[k * stride]) */
PHT_HD double pht_wmom_eval(const double *Wm, long stride, double x) {
  double q = Wm[5 * stride];
  q = fma(q, x, Wm[4 * stride]);
  q = fma(q, x, Wm[3 * stride]);
  q = fma(q, x, Wm[2 * stride]);
  q = fma(q, x, Wm[1 * stride]);
  return fma(q, x, Wm[0]);
}

/* Spectral dot product sum_i c_i e_i of the ECS path, in the order every
 * implementation (one lane per observation, or G lanes sharing one) can
 * reproduce: 16 residue slots p_r = c_r e_r (fma with c_{r+16} e_{r+16}
 * for n > 16), then a pairwise tree p_r += p_{r+s} for s = 8, 4, 2, 1,
 * adding only slots that exist (r + s < n). */
PHT_HD double pht_dot16(const double *c, long cstride, const double *e, int n) {
  double p[16];
  for (int r = 0; r < 16; r++) {
    p[r] = (r < n) ? c[r * cstride] * e[r] : 0.0;
    if (r + 16 < n) p[r] = fma(c[(r + 16) * cstride], e[r + 16], p[r]);
  }
  for (int s = 8; s >= 1; s >>= 1)
    for (int r = 0; r < s; r++)
      if (r + s < n) p[r] = p[r] + p[r + s];
  return p[0];
}

#if defined(__HIPCC__)
/* copy the math tables into LDS (PHT_DETMATH_LDS); call at kernel entry,
 * before the first __syncthreads() */
__device__ __forceinline__ void pht_stage_math_tables() {
#if defined(__HIP_DEVICE_COMPILE__) && defined(PHT_DETMATH_LDS)
  for (int k = threadIdx.x; k < 128; k += blockDim.x) pht_lds_exp_tab[k] = pht_exp_tab[k];
  for (int k = threadIdx.x; k < 768; k += blockDim.x) pht_lds_log_tab[k] = pht_log_tab[k];
#endif
}
#endif

#endif /* PHT_DETMATH_H */
