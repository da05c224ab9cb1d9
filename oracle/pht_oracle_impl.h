/*
 * oracle/pht_oracle_impl.h — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the PhaseType MCMC hot path (SURVEY.md §8a rows
 * a3–a15), included twice by pht_oracle.c:
 *
 *   ORC_DEV == 0  "ref" variant: R's random stream, glibc exp/log and the
 *                 reference's own expression/loop order (natural-order
 *                 BLAS): the reference's algorithm draw for draw.  PARITY
 *                 UNPINNED: the reference needs R's headers and nmath,
 *                 absent here, so nothing compiles it; the rounds-1/2
 *                 stand-in build is retired.  The committed regression
 *                 vectors tests/golden/g1-g3 (first written by that build,
 *                 regenerated bit for bit by tools/make_golden.py --check)
 *                 are the only remaining link to the reference's C
 *                 (DESIGN.md §2).
 *   ORC_DEV == 1  "dev" variant: the GPU specification — Philox stream per
 *                 observation (include/pht_philox.h), detmath exp/log
 *                 (include/pht_detmath.h), per-sweep precomputed products
 *                 (orc_sp W/QQs/QQ1/V) evaluated with explicit fma, and z
 *                 reduced in exact fixed point.  The HIP kernels reproduce
 *                 it bit for bit (tests/test_gpu_parity.py).
 *
 * Both variants share the control flow below, which restates:
 *   LJMA_samplechain_Bladt         src/Simulate_AbsCTMC_gt_Bladt_MHRS.c:34-160
 *   LJMA_MHsample_Bladt (per obs)  src/Simulate_AbsCTMC_eq_Bladt_MHRS.c:37-117
 *   LJMA_probAbsorb / ECS_dens /
 *   moveMass / samplechain_Aslett2 src/Simulate_AbsCTMC_eq_Aslett_ECS.c:21-41,120-171,205-373
 *   phtcdf / condjumpdens /
 *   condjump_r_ars / samplechain   src/Simulate_AbsCTMC_gt_Aslett_DCS.c:26-418
 *   Hobolth_endState / MHsample_Hobolth2
 *                                  src/Simulate_AbsCTMC_eq_AslettHobolth_DCS.c:11-147
 *   HobCDF / samplechain_Hobolth   src/Simulate_AbsCTMC_gt_Hobolth_DCS.c:23-226
 *   Find02 (Brent zeroin)          src/utility.c:233-338
 *   arms/initial/sample/invert/test/update/cumulate/meet/area/
 *   expshift/logshift              src/arms.c:115-812
 *
 * ARMS is restated with the envelope held as a position-ordered array
 * instead of a pointer-linked list: the reference's list always alternates
 * evaluated points (f=1) with intersection/bound points (f=0) starting and
 * ending with a bound, so "f" is the parity of the position and pl/pr are
 * position -1/+1.  Every arithmetic step is unchanged.
 */

/* ---------------------------------------------------------------- RNG */
#if ORC_DEV
typedef pht_stream ORC_FN(rng);
static inline double ORC_FN(u)(ORC_FN(rng) *r) { return pht_next_u(r); }
static inline double ORC_FN(runif)(ORC_FN(rng) *r, double a, double b) {
  if (!isfinite(a) || !isfinite(b) || b < a) return NAN;
  if (a == b) return a;
  return a + (b - a) * pht_next_u(r);
}
static inline double ORC_FN(rexp)(ORC_FN(rng) *r, double scale) {
  if (!isfinite(scale) || scale <= 0.0) return scale == 0.0 ? 0.0 : NAN;
  return scale * -pht_log(pht_next_uexp(r));
}
#define ORC_EXP pht_exp
#define ORC_EXP_NEG pht_exp_neg   /* arguments <= 0: spectral sums, stay-past-y */
#define ORC_EXP_HI pht_exp_hi     /* arguments >= -50: expshift */
#define ORC_EXP_CORE pht_exp_core /* arguments in (-50, 0]: Metropolis */
#define ORC_LOG pht_log
#else
typedef pht_rstream ORC_FN(rng);
static inline double ORC_FN(u)(ORC_FN(rng) *r) { return pht_rs_unif_rand(r); }
static inline double ORC_FN(runif)(ORC_FN(rng) *r, double a, double b) { return pht_rs_runif(r, a, b); }
static inline double ORC_FN(rexp)(ORC_FN(rng) *r, double scale) { return pht_rs_rexp(r, scale); }
#define ORC_EXP exp
#define ORC_EXP_NEG exp
#define ORC_EXP_HI exp
#define ORC_EXP_CORE exp
#define ORC_LOG log
#endif

/* ------------------------------------------------------- accumulation */
static inline void ORC_FN(zadd)(orc_obs *o, int k, double d, double zscale) {
  o->z[k] += d;
#if ORC_DEV
  o->zq[k] += (int64_t)rint(d * zscale);
#else
  (void)zscale;
#endif
}
static void ORC_FN(obs_clear)(orc_obs *o, int n) {
  o->B = 0; o->pre = 0; o->flags = 0; o->ndraw = 0;
  for (int i = 0; i < n; i++) { o->z[i] = 0.0; o->zq[i] = 0; }
  for (int i = 0; i < n * n; i++) o->N[i] = 0;
}

/* Device-mode termination caps: where the reference would loop forever or
 * for an unbounded time (an ARMS envelope that rejects every proposal, a
 * rejection sampler with vanishing acceptance), the device variant stops,
 * sets a flag bit and carries on; the GPU must not hang a wave. */
#define ORC_ARMS_MAXIT 10000      /* flag 4  */
#define ORC_MAX_JUMPS (1 << 20)   /* flag 8  */
#define ORC_MHRS_MAXATT (1 << 22) /* flag 16 */

/* ------------------------------------------------------------- ARMS */
#define ARMS_XEPS 0.00001
#define ARMS_YEPS 0.1
#define ARMS_EYEPS 0.001
#define ARMS_YCEIL 50.
#define ARMS_NPOINT 100

typedef double (*orc_dens)(double x, void *ctx);

typedef struct {
  double x[ARMS_NPOINT], y[ARMS_NPOINT], ey[ARMS_NPOINT], cum[ARMS_NPOINT];
  int cnt;       /* points in the envelope (odd) */
  double ymax;
  int neval;
  double convex;
  /* metropolis */
  double xprev, yprev;
} ORC_FN(env);

static inline double ORC_FN(expshift)(double y, double y0) {
  return (y - y0 > -2.0 * ARMS_YCEIL) ? ORC_EXP_HI(y - y0 + ARMS_YCEIL) : 0.0;
}
static inline double ORC_FN(logshift)(double y, double y0) { return ORC_LOG(y) + y0 - ARMS_YCEIL; }

/* meet(): intersection point at (even) position k (src/arms.c:659-764) */
static void ORC_FN(meet)(ORC_FN(env) *e, int k) {
  double gl = 0.0, gr = 0.0, grl = 0.0, dl = 0.0, dr = 0.0;
  const int last = e->cnt - 1;
  int il = (k >= 3), ir = (k + 3 <= last), irl = (k >= 1 && k + 1 <= last);
  if (il) gl = (e->y[k - 1] - e->y[k - 3]) / (e->x[k - 1] - e->x[k - 3]);
  if (ir) gr = (e->y[k + 1] - e->y[k + 3]) / (e->x[k + 1] - e->x[k + 3]);
  if (irl) grl = (e->y[k + 1] - e->y[k - 1]) / (e->x[k + 1] - e->x[k - 1]);
  /* metropolis is always on here: convexity violations adjust, never fail */
  if (irl && il && (gl < grl)) gl = gl + (1.0 + e->convex) * (grl - gl);
  if (irl && ir && (gr > grl)) gr = gr + (1.0 + e->convex) * (grl - gr);
  if (il && irl) {
    dr = (gl - grl) * (e->x[k + 1] - e->x[k - 1]);
    if (dr < ARMS_YEPS) dr = ARMS_YEPS;
  }
  if (ir && irl) {
    dl = (grl - gr) * (e->x[k + 1] - e->x[k - 1]);
    if (dl < ARMS_YEPS) dl = ARMS_YEPS;
  }
  if (il && ir && irl) {
    e->x[k] = (dl * e->x[k + 1] + dr * e->x[k - 1]) / (dl + dr);
    e->y[k] = (dl * e->y[k + 1] + dr * e->y[k - 1] + dl * dr) / (dl + dr);
  } else if (il && irl) {
    e->x[k] = e->x[k + 1];
    e->y[k] = e->y[k + 1] + dr;
  } else if (ir && irl) {
    e->x[k] = e->x[k - 1];
    e->y[k] = e->y[k - 1] + dl;
  } else if (il) {
    e->y[k] = e->y[k - 1] + gl * (e->x[k] - e->x[k - 1]);
  } else if (ir) {
    e->y[k] = e->y[k + 1] - gr * (e->x[k + 1] - e->x[k]);
  }
}

/* area of the piece to the left of position k (src/arms.c:768-790) */
static inline double ORC_FN(area)(const ORC_FN(env) *e, int k) {
  if (e->x[k - 1] == e->x[k]) return 0.;
  if (fabs(e->y[k] - e->y[k - 1]) < ARMS_YEPS)
    return 0.5 * (e->ey[k] + e->ey[k - 1]) * (e->x[k] - e->x[k - 1]);
  return ((e->ey[k] - e->ey[k - 1]) / (e->y[k] - e->y[k - 1])) * (e->x[k] - e->x[k - 1]);
}

/* cumulate(): exponentiate and integrate the envelope (src/arms.c:625-655) */
static void ORC_FN(cumulate)(ORC_FN(env) *e) {
  double ymax = e->y[0];
  for (int k = 1; k < e->cnt; k++)
    if (e->y[k] > ymax) ymax = e->y[k];
  e->ymax = ymax;
  for (int k = 0; k < e->cnt; k++) e->ey[k] = ORC_FN(expshift)(e->y[k], ymax);
  e->cum[0] = 0.;
  for (int k = 1; k < e->cnt; k++) e->cum[k] = e->cum[k - 1] + ORC_FN(area)(e, k);
}

typedef struct { double x, y, ey; int pr; } ORC_FN(wpt); /* sampled point; piece = (pr-1, pr) */

/* invert(): point at cumulative probability prob (src/arms.c:356-420) */
static void ORC_FN(invert)(const ORC_FN(env) *e, double prob, ORC_FN(wpt) *p) {
  int q = e->cnt - 1;
  double u = prob * e->cum[q];
  while (e->cum[q - 1] > u) q--;
  p->pr = q;
  double prop = (u - e->cum[q - 1]) / (e->cum[q] - e->cum[q - 1]);
  if (e->x[q - 1] == e->x[q]) {
    p->x = e->x[q]; p->y = e->y[q]; p->ey = e->ey[q];
    return;
  }
  double xl = e->x[q - 1], xr = e->x[q], yl = e->y[q - 1], yr = e->y[q];
  double eyl = e->ey[q - 1], eyr = e->ey[q];
  if (fabs(yr - yl) < ARMS_YEPS) {
    if (fabs(eyr - eyl) > ARMS_EYEPS * fabs(eyr + eyl))
      p->x = xl + ((xr - xl) / (eyr - eyl)) * (-eyl + sqrt((1. - prop) * eyl * eyl + prop * eyr * eyr));
    else
      p->x = xl + (xr - xl) * prop;
    p->ey = ((p->x - xl) / (xr - xl)) * (eyr - eyl) + eyl;
    p->y = ORC_FN(logshift)(p->ey, e->ymax);
  } else {
    p->x = xl + ((xr - xl) / (yr - yl)) * (-yl + ORC_FN(logshift)(((1. - prop) * eyl + prop * eyr), e->ymax));
    p->y = ((p->x - xl) / (xr - xl)) * (yr - yl) + yl;
    p->ey = ORC_FN(expshift)(p->y, e->ymax);
  }
}

/* update(): add evaluated point p to the envelope (src/arms.c:525-621) */
static void ORC_FN(update)(ORC_FN(env) *e, const ORC_FN(wpt) *p, orc_dens f, void *ctx) {
  if (e->cnt > ARMS_NPOINT - 2) return;
  int pr = p->pr, qi;
  /* shift [pr, cnt) right by two; new evaluated point q and intersection m */
  for (int k = e->cnt - 1; k >= pr; k--) {
    e->x[k + 2] = e->x[k]; e->y[k + 2] = e->y[k];
  }
  e->cnt += 2;
  if ((pr - 1) & 1) { /* left end on the density: ..., pl, m, q, pr, ... */
    qi = pr + 1;
  } else {            /* right end on the density: ..., pl, q, m, pr, ... */
    qi = pr;
  }
  e->x[qi] = p->x;
  e->y[qi] = p->y;
  int ql = (qi >= 2) ? qi - 2 : qi - 1;
  int qr = (qi + 2 <= e->cnt - 1) ? qi + 2 : qi + 1;
  if (e->x[qi] < (1. - ARMS_XEPS) * e->x[ql] + ARMS_XEPS * e->x[qr]) {
    e->x[qi] = (1. - ARMS_XEPS) * e->x[ql] + ARMS_XEPS * e->x[qr];
    e->y[qi] = f(e->x[qi], ctx); e->neval++;
  } else if (e->x[qi] > ARMS_XEPS * e->x[ql] + (1. - ARMS_XEPS) * e->x[qr]) {
    e->x[qi] = ARMS_XEPS * e->x[ql] + (1. - ARMS_XEPS) * e->x[qr];
    e->y[qi] = f(e->x[qi], ctx); e->neval++;
  }
  ORC_FN(meet)(e, qi - 1);
  ORC_FN(meet)(e, qi + 1);
  if (qi >= 2) ORC_FN(meet)(e, qi - 3);
  if (qi + 2 <= e->cnt - 1) ORC_FN(meet)(e, qi + 3);
  ORC_FN(cumulate)(e);
}

/*
 * arms() with ninit=4, npoint=100, convex=1, dometrop=1, nsamp=1, ncent=0
 * (the only configuration the reference uses: src/Simulate_AbsCTMC_eq_Aslett_ECS.c:315-338,
 * src/Simulate_AbsCTMC_gt_Aslett_DCS.c:227-250).  Returns the error code
 * and writes the sample (left at 0 on error, as the callers' xsamp=0).
 */
/* optional evaluator of the four starting points at once (device spec of
 * the ECS sojourn density, pht_detmath.h pht_ecs_init_ok); NULL: f each */
typedef void (*orc_dens_init)(const double xinit[4], double y[4], void *ctx);

static int ORC_FN(arms)(const double xinit[4], double xl, double xr, orc_dens f, void *ctx,
                        double xprev, double *xsamp, ORC_FN(rng) *rng, int *neval_out, orc_dens_init finit) {
  ORC_FN(env) e;
  e.convex = 1.0;
  e.neval = 0;
  if ((xinit[0] <= xl) || (xinit[3] >= xr)) return 1003;
  for (int i = 1; i < 4; i++)
    if (xinit[i] <= xinit[i - 1]) return 1004;
  e.cnt = 9;
  e.x[0] = xl;
  double yi[4];
  if (finit) finit(xinit, yi, ctx);
  for (int k = 0; k < 4; k++) {
    e.x[2 * k + 1] = xinit[k];
    e.y[2 * k + 1] = finit ? yi[k] : f(xinit[k], ctx);
    e.neval++;
  }
  e.x[8] = xr;
  for (int k = 0; k < 9; k += 2) ORC_FN(meet)(&e, k);
  ORC_FN(cumulate)(&e);
  if ((xprev < xl) || (xprev > xr)) return 1007;
  e.xprev = xprev;
  e.yprev = f(xprev, ctx);
  e.neval++;
#if ORC_DEV
  for (int it = 0;; it++) {
    if (it >= ORC_ARMS_MAXIT) { *xsamp = e.xprev; if (neval_out) *neval_out += e.neval; return 4; }
#else
  for (;;) {
#endif
    ORC_FN(wpt) p;
    ORC_FN(invert)(&e, ORC_FN(u)(rng), &p);
    /* test() (src/arms.c:424-521), metropolis on: no squeezing */
    double u = ORC_FN(u)(rng) * p.ey;
    double y = ORC_FN(logshift)(u, e.ymax);
    double ynew = f(p.x, ctx);
    e.neval++;
    if (y >= ynew) {
      p.y = ynew;
      p.ey = ORC_FN(expshift)(p.y, e.ymax);
      ORC_FN(update)(&e, &p, f, ctx);
      continue; /* rejected */
    }
    /* metropolis step */
    double yold = e.yprev;
    int ql = 0;
    while (e.x[ql + 1] < e.xprev) ql++;
    int qr = ql + 1;
    double w = (e.xprev - e.x[ql]) / (e.x[qr] - e.x[ql]);
    double zold = e.y[ql] + w * (e.y[qr] - e.y[ql]);
    double znew = p.y;
    if (yold < zold) zold = yold;
    if (ynew < znew) znew = ynew;
    w = ynew - znew - yold + zold;
    if (w > 0.0) w = 0.0;
    w = (w > -ARMS_YCEIL) ? ORC_EXP_CORE(w) : 0.0;
    double um = ORC_FN(u)(rng);
    *xsamp = (um > w) ? e.xprev : p.x;
    if (neval_out) *neval_out += e.neval;
    return 0;
  }
}

/* ----------------------------------------------- linear-algebra helpers */
#if !ORC_DEV
/* netlib dgemv 'T' with beta=0, alpha=1: out[c] = 0 + 1*sum_r A[r,c] x[r] */
static inline void ORC_FN(gemv_t)(int n, const double *A, const double *x, double *out) {
  for (int c = 0; c < n; c++) {
    double t = 0.0;
    for (int r = 0; r < n; r++) t = t + A[r + c * n] * x[r];
    out[c] = 0.0 + 1.0 * t;
  }
}
/* netlib dgemv 'N' with beta=0, alpha=1 */
static inline void ORC_FN(gemv_n)(int n, const double *A, const double *x, double *out) {
  for (int r = 0; r < n; r++) out[r] = 0.0;
  for (int c = 0; c < n; c++) {
    double t = 1.0 * x[c];
    for (int r = 0; r < n; r++) out[r] = out[r] + t * A[r + c * n];
  }
}
#endif

/* categorical scan "while(sofar < target) sofar += p[j++]; j--" over w[0..len),
 * with sofar compared against target (already scaled by the total for the
 * device variant).  Running off the end is reference UB: clamp + flag. */
static inline int ORC_FN(catscan_s)(const double *w, int stride, int len, double target, int *flags) {
  double sofar = 0.0;
  int j = 0;
  while (sofar < target) {
    if (j >= len) { *flags |= 1; return len - 1; }
    sofar += w[(size_t)(j++) * stride];
  }
  return j - 1;
}
static inline int ORC_FN(catscan)(const double *w, int len, double target, int *flags) {
  return ORC_FN(catscan_s)(w, 1, len, target, flags);
}
/* device mode: scan weights w[0..cnt) of candidates idx[0..cnt); running off
 * the end (reference UB) selects the last candidate and flags it. */
static inline int ORC_FN(catlist)(const double *w, const int *idx, int cnt, double target, int *flags) {
  double sofar = 0.0;
  for (int q = 0; q < cnt; q++) {
    sofar += w[q];
    if (!(sofar < target)) return idx[q];
  }
  *flags |= 1;
  return cnt > 0 ? idx[cnt - 1] : 0;
}
/* start state ~ pi: "while(sofar < target) sofar += pi[B++]; B--" */
static inline int ORC_FN(pistart)(const orc_sp *sp, double target, int *flags) {
  double sofar = 0.0;
  int B = 0;
#if ORC_DEV
  while (sofar < target) {
    if (B >= sp->n) { *flags |= 1; return sp->n - 1; }
    sofar += sp->pi[B++];
  }
#else
  (void)flags;
  while (sofar < target) sofar += sp->pi[B++];
#endif
  return B - 1;
}

/* ============================================================== MHRS */
/*
 * One call of LJMA_samplechain_Bladt: rejection loop to an accepted path.
 * Returns pre (state at absorption); *start_pos receives the stream position
 * where the accepted attempt began (device variant: the GPU replays from it).
 */
static int ORC_FN(bladt_chain)(const orc_sp *sp, double y, int cens, ORC_FN(rng) *rng,
                               orc_obs *o, double zscale, int record, uint32_t *start_pos) {
  const int n = sp->n;
  double t = 0.0, lastt = 0.0;
  int B2 = 0, lastj = 0, j, natt = 0;
  double z2[ORC_MAXN];
  int N2[ORC_MAXN * ORC_MAXN];
  while (t < y) {
#if ORC_DEV
    if (natt++ >= ORC_MHRS_MAXATT) { o->flags |= 16; break; }
#endif
#if ORC_DEV
    if (start_pos) *start_pos = pht_stream_pos(rng);
#endif
    t = 0;
    for (int i = 0; i < n * n; i++) N2[i] = 0;
    for (int i = 0; i < n; i++) z2[i] = 0.0;
    double target = ORC_FN(u)(rng), sofar = 0.0;
    B2 = 0;
    while (sofar < target && B2 <= n) sofar += sp->pi[B2++];
    B2--;
    j = B2;
    lastt = t;
    lastj = j;
    int njump = 0;
    while ((t < y && j < n) || (cens && j < n)) {
#if ORC_DEV
      if (njump++ >= ORC_MAX_JUMPS) { o->flags |= 8; t = y; break; }
#endif
      t = t + ORC_FN(rexp)(rng, 1.0 / -sp->S[j + j * n]);
      target = ORC_FN(u)(rng);
#if ORC_DEV
      {
        const int *L = sp->succPf + j * (ORC_MAXN + 1);
        int cnt = sp->nsuccPf[j], q = 0;
        sofar = 0.0;
        for (; q < cnt; q++) {
          sofar += sp->Pfull[j + L[q] * n];
          if (!(sofar < target)) break;
        }
        j = (q < cnt) ? L[q] : n + 1;
      }
#else
      int jj = 0;
      sofar = 0.0;
      while (sofar < target && jj <= n) sofar += sp->Pfull[j + jj * n], jj++;
      j = (sofar < target) ? n + 1 : jj - 1; /* scan past Pfull reads workspace: j=n+1 either way */
#endif
      if ((t < y && j < n) || (cens && j < n)) {
        z2[lastj] += t - lastt;
        N2[lastj + j * n]++;
        lastj = j;
        lastt = t;
      }
    }
  }
  if (cens == 0) z2[lastj] += y - lastt;
  else z2[lastj] += t - lastt;
  N2[lastj + lastj * n]++;
  if (record) {
    /* copy the accepted path's statistics (res_* of samplechain_Bladt) */
    o->B = B2;
    for (int i = 0; i < n * n; i++) o->N[i] = N2[i];
    for (int i = 0; i < n; i++) o->z[i] = z2[i];
  }
  (void)zscale;
  return lastj;
}

#if ORC_DEV
/* Device spec (phasetype_amd/csrc/pht_device.h, mhrs_attempt): attempt
 * `att` of chain c runs on its own stream, tag ((c + 1) << 22) | att; it
 * succeeds when the reference would accept it (alive at y / absorbed after
 * y, src/Simulate_AbsCTMC_gt_Bladt_MHRS.c:49-121) and s[pre] > 0 (the
 * re-draw loop of src/Simulate_AbsCTMC_eq_Bladt_MHRS.c:65-76).  With
 * o != NULL the attempt's path is recorded (fixed-point z per sojourn). */
static int ORC_FN(mhrs_attempt)(const orc_sp *sp, double y, int cens, const ORC_FN(rng) *base, int c,
                                uint32_t att, int *pre, orc_obs *o, double zscale) {
  const int n = sp->n;
  ORC_FN(rng) r;
  pht_stream_init(&r, base->k0, base->k1, base->obs, ((uint32_t)(c + 1) << 22) | att, base->sweep);
  double t = 0.0, lastt = 0.0, sofar = 0.0;
  double target = ORC_FN(u)(&r);
  int B2 = 0;
  while (sofar < target && B2 <= n) sofar += (B2 < n ? sp->pi[B2] : 0.0), B2++;
  B2--;
  int j = B2, lastj = j, njump = 0;
  if (o) o->B = B2;
  while ((t < y && j < n) || (cens && j < n)) {
    if (njump++ >= ORC_MAX_JUMPS) { if (o) o->flags |= 8; t = y; break; }
    t = t + ORC_FN(rexp)(&r, 1.0 / -sp->S[j + j * n]);
    target = ORC_FN(u)(&r);
    {
      const int *L = sp->succPf + j * (ORC_MAXN + 1);
      int cnt = sp->nsuccPf[j], q = 0;
      sofar = 0.0;
      for (; q < cnt; q++) {
        sofar += sp->Pfull[j + L[q] * n];
        if (!(sofar < target)) break;
      }
      j = (q < cnt) ? L[q] : n + 1;
    }
    if ((t < y && j < n) || (cens && j < n)) {
      if (o) {
        ORC_FN(zadd)(o, lastj, t - lastt, zscale);
        o->N[lastj + j * n]++;
      }
      lastj = j;
      lastt = t;
    }
  }
  if (o) {
    ORC_FN(zadd)(o, lastj, cens ? t - lastt : y - lastt, zscale);
    o->N[lastj + lastj * n]++;
  }
  *pre = lastj;
  return !(t < y) && lastj < n && sp->s[lastj] > 0;
}

/* first successful attempt of chain c (the reference's rejection loop);
 * none within the cap: the last attempt, flag 16 */
static uint32_t ORC_FN(mhrs_first)(const orc_sp *sp, double y, int cens, const ORC_FN(rng) *base, int c,
                                   int *pre, orc_obs *o) {
  for (uint32_t att = 0; att < (uint32_t)ORC_MHRS_MAXATT; att++)
    if (ORC_FN(mhrs_attempt)(sp, y, cens, base, c, att, pre, NULL, 0.0)) return att;
  o->flags |= 16;
  return (uint32_t)ORC_MHRS_MAXATT - 1u;
}
#endif

/* LJMA_MHsample_Bladt, one observation (src/Simulate_AbsCTMC_eq_Bladt_MHRS.c:63-114) */
static void ORC_FN(obs_mhrs)(const orc_sp *sp, double y, int cens, int mhit, ORC_FN(rng) *rng,
                             orc_obs *o, double zscale) {
  const int n = sp->n;
  ORC_FN(obs_clear)(o, n);
#if ORC_DEV
  /* device variant: first successes of the chains (attempt streams), MH
   * decisions on the observation's stream, the accepted attempt replayed;
   * ndraw = attempts + acceptance words */
  int cpre = 0, cc = 0;
  uint32_t catt = ORC_FN(mhrs_first)(sp, y, cens, rng, 0, &cpre, o);
  uint32_t natt = catt + 1u;
  if (cens == 0) {
    for (int k = 1; k <= mhit; k++) {
      int ppre = 0;
      const uint32_t patt = ORC_FN(mhrs_first)(sp, y, cens, rng, k, &ppre, o);
      natt += patt + 1u;
      double U = ORC_FN(u)(rng);
      if (U < sp->s[ppre] / sp->s[cpre]) { cpre = ppre; catt = patt; cc = k; }
    }
  }
  {
    const int fl = o->flags;
    ORC_FN(obs_clear)(o, n);
    o->flags = fl;
  }
  int pre2 = 0;
  (void)ORC_FN(mhrs_attempt)(sp, y, cens, rng, cc, catt, &pre2, o, zscale);
  o->ndraw = pht_stream_pos(rng) + natt;
  o->pre = cpre;
#else
  orc_obs prop;
  int cpre = ORC_FN(bladt_chain)(sp, y, cens, rng, o, zscale, 1, NULL);
  while (sp->s[cpre] == 0) cpre = ORC_FN(bladt_chain)(sp, y, cens, rng, o, zscale, 1, NULL);
  if (cens == 0) {
    for (int k = 0; k < mhit; k++) {
      int ppre = ORC_FN(bladt_chain)(sp, y, cens, rng, &prop, zscale, 1, NULL);
      while (sp->s[ppre] == 0) ppre = ORC_FN(bladt_chain)(sp, y, cens, rng, &prop, zscale, 1, NULL);
      double U = ORC_FN(runif)(rng, 0.0, 1.0);
      if (U < sp->s[ppre] / sp->s[cpre]) {
        o->B = prop.B;
        for (int i = 0; i < n; i++) o->z[i] = prop.z[i];
        for (int i = 0; i < n * n; i++) o->N[i] = prop.N[i];
        cpre = ppre;
      }
    }
  }
  o->pre = cpre;
#endif
}

/* ====================================================== ECS (exact) */
typedef struct {
  const orc_sp *sp;
  int j;
  double y_t;
  const double *p; /* ref: rate row p_j (p_jj = 0) */
#if ORC_DEV
  const double *E0; /* dev: e^{lambda_i y_t} as the GPU carries it (density at d = 0, init4's point a) */
#endif
} ORC_FN(ecs_ctx);

#if ORC_DEV
/* the four starting points of an ECS sojourn (device spec, pht_detmath.h) */
static void ORC_FN(ecs_init4)(const double xinit[4], double yv[4], void *vctx);
#endif
/* LJMA_ECS_dens (src/Simulate_AbsCTMC_eq_Aslett_ECS.c:150-171) */
static double ORC_FN(ecs_dens)(double d, void *vctx) {
  ORC_FN(ecs_ctx) *c = (ORC_FN(ecs_ctx) *)vctx;
  const orc_sp *sp = c->sp;
  const int n = sp->n, j = c->j;
#if ORC_DEV
  /* log(sum_i W[j,i] e^{lambda_i (y_t - d)}) + S_jj d; at d = 0 the GPU
   * reuses E0 (pht_device.h EcsDens) */
  double x = c->y_t - d, E[ORC_MAXN];
  for (int i = 0; i < n; i++) E[i] = (d == 0.0) ? c->E0[i] : ORC_EXP_NEG(sp->evals[i] * x);
  const double acc = pht_dot16(sp->W + j, n, E, n);
  return ORC_LOG(acc) + sp->S[j + j * n] * d;
#else
  double pq[ORC_MAXN];
  ORC_FN(gemv_t)(n, sp->Q, c->p, pq);
  for (int i = 0; i < n; i++) pq[i] *= ORC_EXP_NEG(sp->evals[i] * (c->y_t - d));
  double term1 = 0.0;
  for (int i = 0; i < n; i++) term1 += pq[i] * sp->Qinv_s[i];
  return ORC_LOG(term1) + sp->S[j + j * n] * d;
#endif
}

#if ORC_DEV
static void ORC_FN(ecs_init4)(const double xinit[4], double yv[4], void *vctx) {
  ORC_FN(ecs_ctx) *c = (ORC_FN(ecs_ctx) *)vctx;
  const orc_sp *sp = c->sp;
  const int n = sp->n, j = c->j;
  const double y_t = c->y_t;
  double lammax = 0.0;
  for (int i = 0; i < n; i++) lammax = fmax(lammax, fabs(sp->evals[i]));
  const double x3 = y_t - xinit[3];
  double E[4][ORC_MAXN];
  if (pht_ecs_init_ok(lammax, xinit[0], x3)) {
    for (int i = 0; i < n; i++) {
      const double F = ORC_EXP_NEG(sp->evals[i] * (y_t - xinit[2]));
      E[2][i] = F;
      E[1][i] = F * F;
      E[0][i] = c->E0[i] * pht_exp_taylor(-sp->evals[i] * xinit[0]);
    }
    /* point y_t - a: the state's W-moment polynomial (pht_wmoments) */
    yv[3] = ORC_LOG(pht_wmom_eval(sp->Wm + j, n, x3)) + sp->S[j + j * n] * xinit[3];
    for (int k = 0; k < 3; k++)
      yv[k] = ORC_LOG(pht_dot16(sp->W + j, n, E[k], n)) + sp->S[j + j * n] * xinit[k];
    return;
  } else {
    for (int k = 0; k < 4; k++)
      for (int i = 0; i < n; i++) E[k][i] = ORC_EXP_NEG(sp->evals[i] * (y_t - xinit[k]));
  }
  for (int k = 0; k < 4; k++)
    yv[k] = ORC_LOG(pht_dot16(sp->W + j, n, E[k], n)) + sp->S[j + j * n] * xinit[k];
}
#endif

/* LJMA_samplechain_Aslett2 (src/Simulate_AbsCTMC_eq_Aslett_ECS.c:205-373) */
static void ORC_FN(obs_ecs_exact)(const orc_sp *sp, double y, ORC_FN(rng) *rng, orc_obs *o,
                                  double zscale, int *neval) {
  const int n = sp->n;
  ORC_FN(obs_clear)(o, n);
  double target = ORC_FN(u)(rng);
  int B = ORC_FN(pistart)(sp, target, &o->flags);
  o->B = B;
  double t = 0.0, d;
  int j = B, lastj;
  double p[ORC_MAXN + 1];
#if ORC_DEV
  /* device spec: the remaining time is carried as y_t <- y_t - d (the
   * reference recomputes y - t); the exponentials of moveMass are then
   * exactly those of the next absorb test, which the GPU reuses.  E0 =
   * e^{lambda_i y_t} is carried the same way: at the first sojourn it is
   * pht_ecs_e0_cube of the starting points' vector F (or direct, outside
   * pht_ecs_init_ok), after a jump by d the direct e^{lambda_i (y_t - d)},
   * unchanged after d = 0 */
  double yt = y;
  double E0[ORC_MAXN];
  {
    double lammax = 0.0;
    for (int i = 0; i < n; i++) lammax = fmax(lammax, fabs(sp->evals[i]));
    const double a = (y) / 1e6, b2 = ((y) / 3.0) * 2.0;
    const int ok = pht_ecs_init_ok(lammax, a, y - (y - a));
    for (int i = 0; i < n; i++)
      E0[i] = ok ? pht_ecs_e0_cube(ORC_EXP_NEG(sp->evals[i] * (y - b2))) : ORC_EXP_NEG(sp->evals[i] * y);
  }
#endif
  for (int njump = 0;; njump++) {
#if ORC_DEV
    if (njump >= ORC_MAX_JUMPS) { o->flags |= 8; break; }
    double y_t = yt;
#else
    double y_t = y - t;
#endif
    if (sp->s[j] > 0.0) {
      double U = ORC_FN(u)(rng), pab;
#if ORC_DEV
      const double den = pht_dot16(sp->QQs + j, n, E0, n);
      /* device spec (pht_device.h ecs_absorbs): U den < exp(S_jj y_t + log s_j) */
      const int absorbs = (den > 0.0) ? (U * den < ORC_EXP(fma(sp->S[j + j * n], y_t, sp->logs[j]))) : (den == 0.0);
      pab = absorbs ? 2.0 : 0.0; /* U < pab <=> absorbs (U < 1) */
#else
      /* LJMA_probAbsorb (:120-136) */
      double num = (sp->S[j + j * n] * (y_t)) + log(sp->s[j]);
      double den = 0.0;
      for (int i = 0; i < n; i++) den += sp->Q[j + i * n] * ORC_EXP_NEG(sp->evals[i] * (y_t)) * sp->Qinv_s[i];
      pab = exp(num - log(den));
#endif
      if (U < pab) break;
    }
    lastj = j;
    for (int i = 0; i < n; i++) p[i] = sp->S[j + i * n] / (-sp->S[j + j * n]);
    p[j] = 0.0;
#if ORC_DEV
    ORC_FN(ecs_ctx) ctx = {sp, j, y_t, p, E0};
#else
    ORC_FN(ecs_ctx) ctx = {sp, j, y_t, p};
#endif
    double xinit[4];
    xinit[0] = (y_t) / 1e6;
    xinit[1] = (y_t) / 3.0;
    xinit[2] = xinit[1] * 2.0;
    xinit[3] = y_t - xinit[0];
    double xsamp = 0.0;
    #if ORC_DEV
    int ainfo = ORC_FN(arms)(xinit, 0.0, y_t, ORC_FN(ecs_dens), &ctx, 0.0, &xsamp, rng, neval, ORC_FN(ecs_init4));
#else
    int ainfo = ORC_FN(arms)(xinit, 0.0, y_t, ORC_FN(ecs_dens), &ctx, 0.0, &xsamp, rng, neval, NULL);
#endif
    if (ainfo) o->flags |= (ainfo == 4) ? 4 : 32;
    t += d = xsamp;
    /* LJMA_moveMass (:21-41) then the categorical draw (:352-358) */
    double x = y_t - d;
#if ORC_DEV
    yt = x;
#endif
#if ORC_DEV
    double E[ORC_MAXN], w[ORC_MAXN], sum = 0.0;
    const int *L = sp->succP + j * ORC_MAXN;
    const int cnt = sp->nsuccP[j];
    for (int i = 0; i < n; i++) E[i] = (d == 0.0) ? E0[i] : ORC_EXP_NEG(sp->evals[i] * x);
    for (int i = 0; i < n; i++) E0[i] = E[i];
    for (int q = 0; q < cnt; q++) {
      const int k = L[q];
      const double acc = pht_dot16(sp->QQs + k, n, E, n);
      w[q] = sp->P[j + k * n] * acc;
      sum += w[q];
    }
    target = ORC_FN(u)(rng) * sum;
    j = ORC_FN(catlist)(w, L, cnt, target, &o->flags);
#else
    double tmp[ORC_MAXN], pp[ORC_MAXN], sum = 0.0;
    for (int i = 0; i < n; i++) tmp[i] = ORC_EXP_NEG(sp->evals[i] * x) * sp->Qinv_s[i];
    ORC_FN(gemv_n)(n, sp->Q, tmp, pp);
    for (int i = 0; i < n; i++) sum += pp[i] = pp[i] * sp->P[j + i * n];
    for (int i = 0; i < n; i++) pp[i] = pp[i] / sum;
    target = ORC_FN(runif)(rng, 0.0, 1.0);
    j = ORC_FN(catscan)(pp, n, target, &o->flags);
#endif
    ORC_FN(zadd)(o, lastj, d, zscale);
    o->N[lastj + j * n]++;
  }
  o->N[j + j * n]++;
#if ORC_DEV
  ORC_FN(zadd)(o, j, yt, zscale);
#else
  ORC_FN(zadd)(o, j, y - t, zscale);
#endif
  o->pre = j;
}

/* ============================================ censored ("gt") sampler */
typedef struct {
  const orc_sp *sp;
  int j;
  double tnow, y;
#if ORC_DEV
  double xr; /* dev (r05): the remaining time y - t as the GPU carries it (xr <- xr - d) */
#endif
} ORC_FN(cj_ctx);

#if !ORC_DEV
/* LJMA_phtcdf (src/Simulate_AbsCTMC_gt_Aslett_DCS.c:26-81) */
static double ORC_FN(phtcdf)(const orc_sp *sp, double x, const double *pi) {
  if (!(x > 0)) return 1.0;
  const int n = sp->n;
  double piQ[ORC_MAXN];
  ORC_FN(gemv_t)(n, sp->Q, pi, piQ);
  double r = 0.0;
  for (int i = 0; i < n; i++) r += piQ[i] * ORC_EXP_NEG(x * sp->evals[i]) * sp->Qinv_1[i];
  return r;
}
#endif

/* LJMA_condjumpdens (:111-132): log F_{P_j}(y - t - d) + log dexp(d) */
static double ORC_FN(cj_dens)(double d, void *vctx) {
  ORC_FN(cj_ctx) *c = (ORC_FN(cj_ctx) *)vctx;
  const orc_sp *sp = c->sp;
  const int n = sp->n, j = c->j;
#if ORC_DEV
  double x1 = c->xr - d, r1; /* device spec v2 (pht_device.h CjDens) */
  if (x1 > 0) {
    double acc = 0.0;
    for (int i = 0; i < n; i++) acc = fma(sp->V[j + i * n], ORC_EXP_NEG(sp->evals[i] * x1), acc);
    r1 = acc;
  } else {
    r1 = 1;
  }
  return ORC_LOG(r1) + ((-d / sp->scale[j]) - sp->logscale[j]);
#else
  double x1 = c->y - c->tnow - d, r1;
  double pi1[ORC_MAXN];
  for (int i = 0; i < n; i++) pi1[i] = sp->P[j + i * n];
  if (x1 > 0) r1 = ORC_FN(phtcdf)(sp, x1, pi1); else r1 = 1;
  return log(r1) + pht_rs_dexp(d, -1.0 / sp->S[j + j * n], 1);
#endif
}

#if ORC_DEV
/* the four starting points of a censored sojourn at once (device spec v2,
 * pht_device.h CjDens::init4): under pht_ecs_init_ok one vector F at 2b,
 * F F at b, e^{lambda xr} taylor(-lambda a) at a, taylor(lambda x3) at
 * xr - a; each sum a sequential fma chain over i */
static void ORC_FN(cj_init4)(const double xinit[4], double yv[4], void *vctx) {
  ORC_FN(cj_ctx) *c = (ORC_FN(cj_ctx) *)vctx;
  const orc_sp *sp = c->sp;
  const int n = sp->n, j = c->j;
  const double xr = c->xr, x3 = xr - xinit[3];
  double lammax = 0.0;
  for (int i = 0; i < n; i++) lammax = fmax(lammax, fabs(sp->evals[i]));
  double acc[4] = {0.0, 0.0, 0.0, 0.0};
  if (pht_ecs_init_ok(lammax, xinit[0], x3)) {
    for (int i = 0; i < n; i++) {
      const double F = ORC_EXP_NEG(sp->evals[i] * (xr - xinit[2]));
      const double v = sp->V[j + i * n];
      const double Ex = ORC_EXP_NEG(sp->evals[i] * xr);
      acc[2] = fma(v, F, acc[2]);
      acc[1] = fma(v, F * F, acc[1]);
      acc[0] = fma(v, Ex * pht_exp_taylor(-sp->evals[i] * xinit[0]), acc[0]);
      acc[3] = fma(v, pht_exp_taylor(sp->evals[i] * x3), acc[3]);
    }
  } else {
    for (int k = 0; k < 4; k++) {
      const double x1 = xr - xinit[k];
      for (int i = 0; i < n; i++) acc[k] = fma(sp->V[j + i * n], ORC_EXP_NEG(sp->evals[i] * x1), acc[k]);
    }
  }
  for (int k = 0; k < 4; k++) yv[k] = ORC_LOG(acc[k]) + ((-xinit[k] / sp->scale[j]) - sp->logscale[j]);
}
#endif

/* LJMA_condjump_r_ars (:184-260); dev: xr = the carried remaining time
 * (device spec v2), the reference's y - tnow otherwise */
static double ORC_FN(condjump)(const orc_sp *sp, double tnow, int jnow, double y, double xr, ORC_FN(rng) *rng,
                               int *neval, int *flags) {
  const int n = sp->n;
#if ORC_DEV
  if (!(xr > 0)) return ORC_FN(rexp)(rng, 1.0 / -sp->S[jnow + jnow * n]);
  const double x = xr;
  double denom;
  double acc = 0.0;
  for (int i = 0; i < n; i++) acc = fma(sp->QQ1[jnow + i * n], ORC_EXP_NEG(sp->evals[i] * x), acc);
  denom = acc;
  if (ORC_FN(runif)(rng, 0.0, 1.0) < ORC_EXP_NEG(sp->S[jnow + jnow * n] * x) / denom)
    return x + ORC_FN(rexp)(rng, 1.0 / -sp->S[jnow + jnow * n]);
  ORC_FN(cj_ctx) ctx = {sp, jnow, tnow, y, x};
  double xinit[4];
  xinit[0] = (x) / 1e6;
  xinit[1] = (x) / 3.0;
  xinit[2] = xinit[1] * 2.0;
  xinit[3] = x - xinit[0];
  double xsamp = 0.0;
  int ainfo = ORC_FN(arms)(xinit, 0.0, x, ORC_FN(cj_dens), &ctx, 0.0, &xsamp, rng, neval, ORC_FN(cj_init4));
  if (ainfo) *flags |= (ainfo == 4) ? 4 : 32;
  return xsamp;
#else
  (void)xr;
  if (tnow >= y) return ORC_FN(rexp)(rng, 1.0 / -sp->S[jnow + jnow * n]);
  double x = y - tnow, denom;
  double pi[ORC_MAXN];
  for (int i = 0; i < n; i++) pi[i] = 0.0;
  pi[jnow] = 1.0;
  denom = ORC_FN(phtcdf)(sp, x, pi);
  if (tnow < y && ORC_FN(runif)(rng, 0.0, 1.0) < ORC_EXP_NEG(sp->S[jnow + jnow * n] * (y - tnow)) / denom)
    return y - tnow + ORC_FN(rexp)(rng, 1.0 / -sp->S[jnow + jnow * n]);
  ORC_FN(cj_ctx) ctx = {sp, jnow, tnow, y};
  double xinit[4];
  xinit[0] = (y - tnow) / 1e6;
  xinit[1] = (y - tnow) / 3.0;
  xinit[2] = xinit[1] * 2.0;
  xinit[3] = y - tnow - xinit[0];
  double xsamp = 0.0;
  int ainfo = ORC_FN(arms)(xinit, 0.0, y - tnow, ORC_FN(cj_dens), &ctx, 0.0, &xsamp, rng, neval, NULL);
  if (ainfo) *flags |= (ainfo == 4) ? 4 : 32;
  return xsamp;
#endif
}

/* LJMA_samplechain, reverse=0 (:299-418) */
static void ORC_FN(obs_censored)(const orc_sp *sp, double y, int cens, ORC_FN(rng) *rng, orc_obs *o,
                                 double zscale, int *neval) {
  const int n = sp->n;
  ORC_FN(obs_clear)(o, n);
  double target = ORC_FN(u)(rng), sofar = 0.0;
  int B = ORC_FN(pistart)(sp, target, &o->flags);
  o->B = B;
  double t = 0.0, lastt = 0.0;
  int j = B, lastj = 0, njump = 0;
#if ORC_DEV
  /* device spec v2 (pht_device.h censored_jump): the remaining time carried,
   * xr <- xr - d; "t < y" decisions read xr > 0 */
  double xr = y;
#define ORC_CENS_BEFORE_Y (xr > 0)
#else
  double xr = 0.0;
#define ORC_CENS_BEFORE_Y (t < y)
#endif
  while (ORC_CENS_BEFORE_Y || cens) {
#if ORC_DEV
    if (njump++ >= ORC_MAX_JUMPS) { o->flags |= 8; break; }
#endif
    lastt = t;
    lastj = j;
    double d = ORC_FN(condjump)(sp, t, j, y, xr, rng, neval, &o->flags);
    t += d;
#if ORC_DEV
    xr = xr - d;
#endif
    target = ORC_FN(u)(rng);
    if (ORC_CENS_BEFORE_Y) {
#if ORC_DEV
      double x1 = xr;
#else
      double x1 = y - t;
#endif
#if ORC_DEV
      double E[ORC_MAXN], w[ORC_MAXN], r2 = 0.0;
      (void)sofar;
      const int *L = sp->succP + lastj * ORC_MAXN;
      const int cnt = sp->nsuccP[lastj];
      for (int i = 0; i < n; i++) E[i] = ORC_EXP_NEG(sp->evals[i] * x1);
      for (int i = 0; i < n; i++) r2 = fma(sp->V[lastj + i * n], E[i], r2);
      for (int q = 0; q < cnt; q++) {
        const int k = L[q];
        double r1 = 0.0;
        for (int i = 0; i < n; i++) r1 = fma(sp->QQ1[k + i * n], E[i], r1);
        w[q] = r1 * sp->P[lastj + k * n];
      }
      j = ORC_FN(catlist)(w, L, cnt, target * r2, &o->flags);
#else
      double pi2[ORC_MAXN], pi1[ORC_MAXN];
      for (int i = 0; i < n; i++) pi2[i] = sp->P[lastj + i * n];
      double r2 = ORC_FN(phtcdf)(sp, x1, pi2);
      sofar = 0.0;
      j = 0;
      while (sofar < target) {
        if (j >= n) { o->flags |= 1; j = n; break; }
        if (sp->P[lastj + j * n] == 0.0) { j++; continue; }
        for (int i = 0; i < n; i++) pi1[i] = 0.0;
        pi1[j] = 1.0;
        double r1 = ORC_FN(phtcdf)(sp, x1, pi1);
        sofar += r1 * sp->P[lastj + (j++) * n] / r2;
      }
      j--;
#endif
    } else {
#if ORC_DEV
      {
        const int *L = sp->succPf + lastj * (ORC_MAXN + 1);
        const int cnt = sp->nsuccPf[lastj];
        double w[ORC_MAXN + 1];
        for (int q = 0; q < cnt; q++) w[q] = sp->Pfull[lastj + L[q] * n];
        j = ORC_FN(catlist)(w, L, cnt, target, &o->flags);
      }
#else
      j = ORC_FN(catscan_s)(sp->Pfull + lastj, n, n + 1, target, &o->flags);
#endif
    }
    if (j == n) break;
    if (ORC_CENS_BEFORE_Y || cens) {
      ORC_FN(zadd)(o, lastj, t - lastt, zscale);
      o->N[lastj + j * n]++;
    }
  }
#undef ORC_CENS_BEFORE_Y
  if (cens == 0) ORC_FN(zadd)(o, lastj, y - lastt, zscale);
  else ORC_FN(zadd)(o, lastj, t - lastt, zscale);
  o->pre = lastj;
  o->N[lastj + lastj * n]++;
}

/* ================================================================ DCS */
typedef struct {
  const orc_sp *sp;
  int lastj, j;
  double prob, Pab, y, t, u;
  const double *Qb; /* Qinv e_b */
  double *J;
  const double *E;  /* device mode: e^{lambda_i (y - t)} of this jump */
} ORC_FN(hob_ctx);

/* HobCDF (src/Simulate_AbsCTMC_gt_Hobolth_DCS.c:23-40) */
static double ORC_FN(hobcdf)(double x, void *vctx) {
  ORC_FN(hob_ctx) *c = (ORC_FN(hob_ctx) *)vctx;
  const orc_sp *sp = c->sp;
  const int n = sp->n;
  const double Sll = sp->S[c->lastj + c->lastj * n];
  for (int i = 0; i < n; i++) {
#if ORC_DEV
    const double Ei = c->E[i];
#else
    const double Ei = ORC_EXP_NEG(sp->evals[i] * (c->y - c->t));
#endif
    if (fabs((sp->evals[i] - Sll) / Sll) < 1e-13)
      c->J[i] = x * Ei;
    else
#if ORC_DEV /* device spec: times the reciprocal 1 / (lambda_i - S_ll) */
      c->J[i] = (Ei - ORC_EXP_NEG((c->y - c->t - x) * sp->evals[i] + Sll * x)) * (1.0 / (sp->evals[i] - Sll));
#else
      c->J[i] = (Ei - ORC_EXP_NEG((c->y - c->t - x) * sp->evals[i] + Sll * x)) / (sp->evals[i] - Sll);
#endif
  }
  double tmp = 0.0;
#if ORC_DEV
  for (int i = 0; i < n; i++) tmp = fma(sp->Q[c->j + i * n] * c->J[i], c->Qb[i], tmp);
#else
  for (int i = 0; i < n; i++) tmp += sp->Q[c->j + i * n] * c->J[i] * c->Qb[i];
#endif
  return 1 / c->prob * sp->S[c->lastj + c->j * n] / c->Pab * tmp - c->u;
}

/* Find02 (src/utility.c:233-338), Brent's zeroin with Dalgaard's maxit */
static double ORC_FN(find02)(double ax, double bx, double fa, double fb, orc_dens f, void *info,
                             double *Tol, int *Maxit) {
  double a, b, c, fc, tol;
  int maxit;
  a = ax; b = bx;
  c = a; fc = fa;
  maxit = *Maxit + 1; tol = *Tol;
  if (fa == 0.0) { *Tol = 0.0; *Maxit = 0; return a; }
  if (fb == 0.0) { *Tol = 0.0; *Maxit = 0; return b; }
  while (maxit--) {
    double prev_step = b - a, tol_act, p, q, new_step;
    if (fabs(fc) < fabs(fb)) {
      a = b; b = c; c = a;
      fa = fb; fb = fc; fc = fa;
    }
    tol_act = 2 * DBL_EPSILON * fabs(b) + tol / 2;
    new_step = (c - b) / 2;
    if (fabs(new_step) <= tol_act || fb == (double)0) {
      *Maxit -= maxit;
      *Tol = fabs(c - b);
      return b;
    }
    if (fabs(prev_step) >= tol_act && fabs(fa) > fabs(fb)) {
      double t1, cb, t2;
      cb = c - b;
      if (a == c) {
        t1 = fb / fa;
        p = cb * t1;
        q = 1.0 - t1;
      } else {
        q = fa / fc; t1 = fb / fc; t2 = fb / fa;
        p = t2 * (cb * q * (q - t1) - (b - a) * (t1 - 1.0));
        q = (q - 1.0) * (t1 - 1.0) * (t2 - 1.0);
      }
      if (p > (double)0) q = -q;
      else p = -p;
      if (p < (0.75 * cb * q - fabs(tol_act * q) / 2) && p < fabs(prev_step * q / 2)) new_step = p / q;
    }
    if (fabs(new_step) < tol_act) new_step = (new_step > (double)0) ? tol_act : -tol_act;
    a = b; fa = fb;
    b += new_step; fb = (*f)(b, info);
    if ((fb > 0 && fc > 0) || (fb < 0 && fc < 0)) { c = a; fc = fa; }
  }
  *Tol = fabs(c - b);
  *Maxit = -1;
  return b;
}

#if ORC_DEV
/* the device spec's jump-time root (pht_dcs_round.h hob_halley): safeguarded
 * Halley on HobCDF, F' and F'' from the same exponentials, stop at the
 * evaluation's rounding level; E, Qb, coef as the kernel hoists them.
 * Evaluations counted into *nev. */
static double ORC_FN(hob_halley)(const ORC_FN(hob_ctx) *c, double es, int *nev) {
  const orc_sp *sp = c->sp;
  const int n = sp->n;
  const double eps = 2.2204460492503131e-16;
  const double Sll = sp->S[c->lastj + c->lastj * n];
  const double X = c->y - c->t;
  const double coef = 1 / c->prob * sp->S[c->lastj + c->j * n] / c->Pab;
  double lo = 0.0, hi = X;
  const double x0 = ORC_LOG(1.0 - c->u * (1.0 - es)) / Sll;
  double xb = (x0 > lo && x0 < hi) ? x0 : c->u * X;
  double root = xb;
  for (int it = 0; it < 1000; it++) {
    const double c1 = X - xb, c0 = Sll * xb;
    double tmp = 0.0, asum = 0.0, dtmp = 0.0, d2 = 0.0;
    for (int i = 0; i < n; i++) {
      const double Ei = c->E[i], ev = sp->evals[i];
      double ei, Ji, dl, Jm;
      if (fabs((ev - Sll) / Sll) < 1e-13) {
        ei = Ei;
        Ji = xb * Ei;
        dl = 0.0;
        Jm = fabs(Ji);
      } else {
        ei = ORC_EXP_NEG(c1 * ev + c0);
        Ji = (Ei - ei) * (1.0 / (ev - Sll));
        dl = Sll - ev;
        Jm = (Ei + ei) * fabs(1.0 / (ev - Sll)); /* |J_i| before E_i - e_i cancels */
      }
      const double w = sp->Q[c->j + i * n] * c->Qb[i]; /* the jump's weight Q_ji Qb_i */
      const double we = w * ei;
      tmp = fma(w, Ji, tmp);
      asum = fma(fabs(w), Jm, asum);
      dtmp = fma(w, ei, dtmp);
      d2 = fma(we, dl, d2);
    }
    (*nev)++;
    const double F = coef * tmp - c->u, D = coef * dtmp, D2 = coef * d2;
    if (F == 0.0) { root = xb; break; }
    if (F < 0.0) lo = xb;
    else hi = xb;
    double nx = xb - (2.0 * F * D) / (2.0 * D * D - F * D2);
    if (it == 0) { /* the first step in log-survival space (pht_dcs_round.h) */
      const double S = (1.0 - c->u) - F;
      if (S > 0.0) {
        const double q = D / S, G = ORC_LOG(S / (1.0 - c->u));
        const double G1 = -q, G2 = -(D2 / S) - q * q;
        nx = xb - (2.0 * G * G1) / (2.0 * G1 * G1 - G * G2);
      }
    }
    if (fabs(F) <= 16.0 * eps * (coef * asum + c->u)) {
      root = (nx >= lo && nx <= hi) ? nx : xb;
      break;
    }
    if (!(nx > lo && nx < hi)) nx = 0.5 * (lo + hi);
    root = nx;
    if (fabs(nx - xb) <= 2.0 * eps * fabs(xb)) break;
    xb = nx;
  }
  return root;
}
#endif

/* LJMA_Hobolth_endState + LJMA_samplechain_Hobolth, one observation
 * (censoring ignored, as the reference: :132). */
static void ORC_FN(obs_dcs)(const orc_sp *sp, double y, ORC_FN(rng) *rng, orc_obs *o, double zscale,
                            int *nbrent) {
  const int n = sp->n;
  ORC_FN(obs_clear)(o, n);
  /* end state b ~ (pi e^{yS})_b s_b */
  double pend[ORC_MAXN], sum = 0.0;
#if ORC_DEV
  double a[ORC_MAXN];
  for (int i = 0; i < n; i++) a[i] = sp->piQ[i] * ORC_EXP_NEG(sp->evals[i] * y);
  for (int k = 0; k < n; k++) {
    double acc = 0.0;
    for (int i = 0; i < n; i++) acc = fma(a[i], sp->Qinv[i + k * n], acc);
    pend[k] = acc * sp->s[k];
    sum += pend[k];
  }
  int allidx[ORC_MAXN];
  for (int k = 0; k < n; k++) allidx[k] = k;
  int b = ORC_FN(catlist)(pend, allidx, n, ORC_FN(u)(rng) * sum, &o->flags);
#else
  double pq[ORC_MAXN], tmp[ORC_MAXN];
  ORC_FN(gemv_t)(n, sp->Q, sp->pi, pq);
  for (int i = 0; i < n; i++) pq[i] *= ORC_EXP_NEG(sp->evals[i] * y);
  ORC_FN(gemv_t)(n, sp->Qinv, pq, tmp);
  for (int i = 0; i < n; i++) sum += pend[i] = tmp[i] * sp->s[i];
  for (int i = 0; i < n; i++) pend[i] = pend[i] / sum;
  int b = ORC_FN(catscan)(pend, n, ORC_FN(runif)(rng, 0.0, 1.0), &o->flags);
#endif
  double bvec[ORC_MAXN], Qb[ORC_MAXN];
  for (int i = 0; i < n; i++) bvec[i] = (i == b) ? 1.0 : 0.0;
#if ORC_DEV
  for (int i = 0; i < n; i++) Qb[i] = sp->Qinv[i + b * n];
#else
  ORC_FN(gemv_n)(n, sp->Qinv, bvec, Qb);
#endif
  /* LJMA_samplechain_Hobolth */
  double target = ORC_FN(u)(rng);
  int B = ORC_FN(pistart)(sp, target, &o->flags);
  o->B = B;
  double t = 0.0, jtime = 0.0, J[ORC_MAXN], p[ORC_MAXN];
  (void)p;
  int j = B, lastj, njump = 0;
  while (t < y) {
#if ORC_DEV
    if (njump++ >= ORC_MAX_JUMPS) { o->flags |= 8; break; }
#endif
    lastj = j;
    double Pab = 0.0, x = y - t;
    (void)x;
    const double Sjj = sp->S[j + j * n];
#if ORC_DEV
    double E[ORC_MAXN];
    for (int i = 0; i < n; i++) E[i] = ORC_EXP_NEG(sp->evals[i] * x);
    for (int i = 0; i < n; i++) Pab = fma(sp->Q[j + i * n] * E[i], Qb[i], Pab);
#else
    for (int i = 0; i < n; i++) Pab += sp->Q[j + i * n] * ORC_EXP_NEG(sp->evals[i] * (y - t)) * Qb[i];
#endif
    if (bvec[j] > 0.0) {
      if (ORC_FN(runif)(rng, 0.0, 1.0) < ORC_EXP_NEG(Sjj * (y - t)) / Pab) {
        ORC_FN(zadd)(o, j, (y - t), zscale);
        o->N[j + j * n] = 1;
        o->pre = j;
        return;
      }
    }
    for (int i = 0; i < n; i++) {
#if ORC_DEV
      if (fabs((sp->evals[i] - Sjj) / Sjj) < 1e-13) J[i] = x * E[i];
      else J[i] = (E[i] - ORC_EXP_NEG(Sjj * x)) * (1.0 / (sp->evals[i] - Sjj));
#else
      if (fabs((sp->evals[i] - Sjj) / Sjj) < 1e-13) J[i] = (y - t) * ORC_EXP_NEG(sp->evals[i] * (y - t));
      else J[i] = (ORC_EXP_NEG(sp->evals[i] * (y - t)) - ORC_EXP_NEG(Sjj * (y - t))) / (sp->evals[i] - Sjj);
#endif
    }
    double p_sum = 0.0, prob;
#if ORC_DEV
    const int *L = sp->succS + j * ORC_MAXN;
    const int cnt = sp->nsuccS[j];
    double pw[ORC_MAXN];
    for (int q = 0; q < cnt; q++) {
      const int i = L[q];
      double tmp = 0.0;
      for (int k = 0; k < n; k++) tmp = fma(sp->Q[i + k * n] * J[k], Qb[k], tmp);
      p_sum += pw[q] = sp->S[j + i * n] / Pab * tmp;
    }
    target = ORC_FN(runif)(rng, 0.0, p_sum);
    if (!(target > 0.0)) { o->flags |= 2; o->pre = j; return; } /* reference reads p[-1]: UB */
    {
      double sofar = 0.0;
      int q = 0;
      for (; q < cnt; q++) { sofar += pw[q]; if (!(sofar < target)) break; }
      if (q == cnt) { o->flags |= 1; q = cnt - 1; }
      j = L[q];
      prob = pw[q];
    }
#else
    for (int i = 0; i < n; i++) {
      if (i == j) continue;
      double tmp = 0.0;
      for (int k = 0; k < n; k++) tmp += sp->Q[i + k * n] * J[k] * Qb[k];
      p_sum += p[i] = sp->S[j + i * n] / Pab * tmp;
    }
    p[j] = 0.0;
    target = ORC_FN(runif)(rng, 0.0, p_sum);
    if (!(target > 0.0)) { o->flags |= 2; o->pre = j; return; } /* reference reads p[-1]: UB */
    j = ORC_FN(catscan)(p, n, target, &o->flags);
    prob = p[j];
#endif
    ORC_FN(hob_ctx) hc = {sp, lastj, j, prob, Pab, y, t, 0.0, Qb, J, NULL};
#if ORC_DEV
    hc.E = E;
#endif
    hc.u = ORC_FN(runif)(rng, 0.0, 1.0);
#if ORC_DEV
    if (!orc_dcs_brent) {
      int nev = 0;
      jtime = ORC_FN(hob_halley)(&hc, ORC_EXP_NEG(Sjj * x), &nev);
      if (nbrent) *nbrent += nev;
      orc_halley_hist[nev < 63 ? nev : 63]++; /* diagnostics: tools/dcs_halley_hist.py */
    } else
#endif
    {
      double Tol = 0.0;
      int Maxit = 1000;
      jtime = ORC_FN(find02)(0.0, y - t, -hc.u, 1.0 - hc.u, ORC_FN(hobcdf), &hc, &Tol, &Maxit);
      if (nbrent) *nbrent += (Maxit < 0) ? 1000 : Maxit;
    }
    while (t + jtime >= y) jtime = jtime / 2;
    o->N[lastj + j * n]++;
    ORC_FN(zadd)(o, lastj, jtime, zscale);
    t += jtime;
  }
}
