/*
 * gm_oracle.c — CPU ORACLE (test infrastructure only; see gm_oracle.h).
 *
 * Part 1: the random-number / special-function spec (restated from the
 * engine's documentation in DESIGN.md "RNG spec": Philox4x32-10, 24/53-bit
 * uniforms, Box-Muller cosine branch, FreeBSD-msun log/exp polynomials).
 * Part 2 (gm_oracle_t.inc, instantiated for double and float): targets, HMC,
 * MH, NUTS, each citing the reference lines it restates.
 * Part 3: split-R-hat / ESS / autocovariance / MultiChainTracker (stats.rs).
 *
 * Build: oracle/Makefile (gcc -O2 -ffp-contract=off; no -ffast-math).
 */
#include "gm_oracle.h"

#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

enum {
  TAG_INIT = 1, TAG_MOM = 2, TAG_ACC = 3, TAG_MH_PROP = 4, TAG_MH_ACC = 5, TAG_NUTS_MOM = 6,
  TAG_NUTS_EXP = 7, TAG_NUTS_DIR = 8, TAG_NUTS_TOP = 9, TAG_NUTS_MRG = 10, TAG_NUTS_INIT = 11,
  TAG_NUTS_PROBE = 12 /* probe momentum after a mass-matrix update (generic_nuts.rs:905-909) */
};

/* ===================== Part 1: RNG spec ===================== */
void or_philox(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]) {
  uint32_t c0 = ctr[0], c1 = ctr[1], c2 = ctr[2], c3 = ctr[3];
  uint32_t k0 = key[0], k1 = key[1];
  for (int r = 0; r < 10; ++r) {
    uint64_t p0 = (uint64_t)0xD2511F53u * c0;
    uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
    uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
    uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
    uint32_t n0 = hi1 ^ c1 ^ k0, n1 = lo1, n2 = hi0 ^ c3 ^ k1, n3 = lo0;
    c0 = n0; c1 = n1; c2 = n2; c3 = n3;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

static uint64_t bits_d(double x) { uint64_t u; memcpy(&u, &x, 8); return u; }
static double from_bits_d(uint64_t u) { double x; memcpy(&x, &u, 8); return x; }
static uint32_t bits_f(float x) { uint32_t u; memcpy(&u, &x, 4); return u; }
static float from_bits_f(uint32_t u) { float x; memcpy(&x, &u, 4); return x; }

static double unif_co_d(uint32_t a, uint32_t b) {
  uint64_t k = ((uint64_t)(a >> 5) << 26) | (uint64_t)(b >> 6);
  return (double)k * 1.1102230246251565e-16;
}
static double unif_oc_d(uint32_t a, uint32_t b) {
  uint64_t k = ((uint64_t)(a >> 5) << 26) | (uint64_t)(b >> 6);
  return (double)(k + 1u) * 1.1102230246251565e-16;
}
static float unif_co_f(uint32_t a) { return (float)(a >> 8) * 5.9604644775390625e-08f; }
static float unif_oc_f(uint32_t a) { return (float)((a >> 8) + 1u) * 5.9604644775390625e-08f; }

/* natural log: FreeBSD msun e_log.c */
double or_log_d(double x) {
  const double ln2_hi = 6.93147180369123816490e-01, ln2_lo = 1.90821492927058770002e-10;
  const double Lg1 = 6.666666666666735130e-01, Lg2 = 3.999999999940941908e-01,
               Lg3 = 2.857142874366239149e-01, Lg4 = 2.222219843214978396e-01,
               Lg5 = 1.818357216161805012e-01, Lg6 = 1.531383769920937332e-01,
               Lg7 = 1.479819860511658591e-01;
  if (x != x) return x;
  if (x < 0.0) return from_bits_d(0x7ff8000000000000ull);
  if (x == 0.0) return -from_bits_d(0x7ff0000000000000ull);
  uint64_t u = bits_d(x);
  if ((u >> 52) >= 0x7ff) return x;
  int k = 0;
  if ((u >> 52) == 0) { x = x * 18014398509481984.0; u = bits_d(x); k = -54; }
  k += (int)(u >> 52) - 1023;
  double m = from_bits_d((u & 0x000fffffffffffffull) | 0x3ff0000000000000ull);
  if (m > 1.4142135623730951) { m = m * 0.5; k += 1; }
  double f = m - 1.0;
  double s = f / (2.0 + f);
  double z = s * s, w = z * z;
  double t1 = w * (Lg2 + w * (Lg4 + w * Lg6));
  double t2 = z * (Lg1 + w * (Lg3 + w * (Lg5 + w * Lg7)));
  double R = t2 + t1;
  double hfsq = 0.5 * f * f;
  double dk = (double)k;
  return dk * ln2_hi - ((hfsq - (s * (hfsq + R) + dk * ln2_lo)) - f);
}

/* FreeBSD msun e_logf.c */
float or_log_f(float x) {
  const float ln2_hi = 6.9313812256e-01f, ln2_lo = 9.0580006145e-06f;
  const float Lg1 = 0.66666662693f, Lg2 = 0.40000972152f, Lg3 = 0.28498786688f, Lg4 = 0.24279078841f;
  if (x != x) return x;
  if (x < 0.0f) return from_bits_f(0x7fc00000u);
  if (x == 0.0f) return -from_bits_f(0x7f800000u);
  uint32_t u = bits_f(x);
  if ((u >> 23) >= 0xff) return x;
  int k = 0;
  if ((u >> 23) == 0) { x = x * 33554432.0f; u = bits_f(x); k = -25; }
  k += (int)(u >> 23) - 127;
  float m = from_bits_f((u & 0x007fffffu) | 0x3f800000u);
  if (m > 1.41421353816986083984f) { m = m * 0.5f; k += 1; }
  float f = m - 1.0f;
  float s = f / (2.0f + f);
  float z = s * s, w = z * z;
  float t1 = w * (Lg2 + w * Lg4);
  float t2 = z * (Lg1 + w * Lg3);
  float R = t2 + t1;
  float hfsq = 0.5f * f * f;
  float dk = (float)k;
  return dk * ln2_hi - ((hfsq - (s * (hfsq + R) + dk * ln2_lo)) - f);
}

/* exp: FreeBSD msun e_exp.c, with k = (int)(x/ln2 +- 1/2) for every x */
static double scale2_d(double y, int k) {
  if (k > 1023) return y * from_bits_d(0x7fe0000000000000ull) * from_bits_d((uint64_t)(k) << 52);
  if (k < -1021)
    return y * from_bits_d((uint64_t)(k + 1000 + 1023) << 52) * from_bits_d((uint64_t)(23) << 52);
  return y * from_bits_d((uint64_t)(k + 1023) << 52);
}
double or_exp_d(double x) {
  const double o_th = 7.09782712893383973096e+02, u_th = -7.45133219101941108420e+02;
  const double ln2HI = 6.93147180369123816490e-01, ln2LO = 1.90821492927058770002e-10;
  const double invln2 = 1.44269504088896338700e+00;
  const double P1 = 1.66666666666666019037e-01, P2 = -2.77777777770155933842e-03,
               P3 = 6.61375632143793436117e-05, P4 = -1.65339022054652515390e-06,
               P5 = 4.13813679705723846039e-08;
  if (x != x) return x;
  if (x > o_th) return from_bits_d(0x7ff0000000000000ull);
  if (x < u_th) return 0.0;
  int k = (int)(invln2 * x + (x < 0.0 ? -0.5 : 0.5));
  double dk = (double)k;
  double hi = x - dk * ln2HI, lo = dk * ln2LO;
  double r = hi - lo;
  double t = r * r;
  double c = r - t * (P1 + t * (P2 + t * (P3 + t * (P4 + t * P5))));
  double y = 1.0 - ((lo - (r * c) / (2.0 - c)) - hi);
  return scale2_d(y, k);
}
/* The NUTS leaf's acceptance statistic in f64, min(1, exp(x)) (generic_nuts.rs
 * :1212; NaN gives 1), the kernels' division-free form (gm_rng.h
 * leaf_alpha_tab): exp(max(min(x, 0), -746)) with k = rint(64 x / ln2),
 * r = x - k ln2/64 by two fmas, exp(r) - 1 to degree 6, and 2^(j/64) from the
 * table GM_EXP64_INIT (gm_bm_tables.h). fmin/fmax return the non-NaN
 * operand, as the device's min/max do. */
#include "gm_bm_tables.h"
static const double exp64_tab[64] = {GM_EXP64_INIT};
double or_leaf_alpha_d(double x) {
  const double xs = fmax(fmin(x, 0.0), -746.0);
  const double dk = rint(xs * 0x1.71547652b82fep+6);
  const int k = (int)dk;
  double r = fma(-dk, 0x1.62e42fee00000p-7, xs);
  r = fma(-dk, 0x1.a39ef35793c76p-39, r);
  double a = fma(r, 0x1.6c16c16c16c17p-10, 0x1.1111111111111p-7);
  a = fma(r, a, 0x1.5555555555555p-5);
  a = fma(r, a, 0x1.5555555555555p-3);
  a = fma(r, a, 0.5);
  const double p = fma(r * r, a, r);
  const double tv = exp64_tab[k & 63];
  return ldexp(fma(tv, p, tv), k >> 6);
}
static float scale2_f(float y, int k) {
  if (k > 127) return y * from_bits_f(0x7f000000u) * from_bits_f((uint32_t)(k) << 23);
  if (k < -125) return y * from_bits_f((uint32_t)(k + 100 + 127) << 23) * from_bits_f((uint32_t)(27) << 23);
  return y * from_bits_f((uint32_t)(k + 127) << 23);
}
float or_exp_f(float x) {
  const float o_th = 8.8721679688e+01f, u_th = -1.0397208405e+02f;
  const float ln2HI = 6.9314575195e-01f, ln2LO = 1.4286067653e-06f, invln2 = 1.4426950216e+00f;
  const float P1 = 1.6666625440e-1f, P2 = -2.7667332906e-3f;
  if (x != x) return x;
  if (x > o_th) return from_bits_f(0x7f800000u);
  if (x < u_th) return 0.0f;
  int k = (int)(invln2 * x + (x < 0.0f ? -0.5f : 0.5f));
  float dk = (float)k;
  float hi = x - dk * ln2HI, lo = dk * ln2LO;
  float r = hi - lo;
  float t = r * r;
  float c = r - t * (P1 + t * P2);
  float y = 1.0f - ((lo - (r * c) / (2.0f - c)) - hi);
  return scale2_f(y, k);
}

/* cos(2 pi u) for u in [0,1): symmetric reduction in u, fdlibm kernels (f64),
 * Taylor kernels (f32). */
static double ksin_d(double x) {
  const double S1 = -1.66666666666666324348e-01, S2 = 8.33333333332248946124e-03,
               S3 = -1.98412698298579493134e-04, S4 = 2.75573137070700676789e-06,
               S5 = -2.50507602534068634195e-08, S6 = 1.58969099521155010221e-10;
  double z = x * x, v = z * x;
  double r = S2 + z * (S3 + z * (S4 + z * (S5 + z * S6)));
  return x + v * (S1 + z * r);
}
static double kcos_d(double x) {
  const double C1 = 4.16666666666666019037e-02, C2 = -1.38888888888741095749e-03,
               C3 = 2.48015872894767294178e-05, C4 = -2.75573143513906633035e-07,
               C5 = 2.08757232129817482790e-09, C6 = -1.13596475577881948265e-11;
  double z = x * x, w = z * z;
  double r = z * (C1 + z * (C2 + z * C3)) + w * w * (C4 + z * (C5 + z * C6));
  double hz = 0.5 * z;
  double ww = 1.0 - hz;
  return ww + (((1.0 - ww) - hz) + z * r);
}
static float ksin_f(float x) {
  float z = x * x;
  return x + x * z * (-1.6666667163e-01f + z * (8.3333337680e-03f + z * (-1.9841270114e-04f + z * 2.7557314297e-06f)));
}
static float kcos_f(float x) {
  float z = x * x;
  return 1.0f - 0.5f * z + z * z * (4.1666667908e-02f + z * (-1.3888889225e-03f + z * (2.4801587642e-05f + z * -2.7557314297e-07f)));
}
/* sin and cos of 2 pi u for u in [0,1): quadrant q = floor(4u), r = u - q/4
 * (exact); first octant direct kernels, second octant complements; rotate. */
static void sincos2pi_d(double u, double* c, double* s) {
  const double twopi = 6.283185307179586476925286766559;
  const int q = (int)(u * 4.0);
  const double r = u - (double)q * 0.25;
  double c0, s0;
  if (r <= 0.125) { c0 = kcos_d(r * twopi); s0 = ksin_d(r * twopi); }
  else { double x = (0.25 - r) * twopi; c0 = ksin_d(x); s0 = kcos_d(x); }
  if (q == 0) { *c = c0; *s = s0; }
  else if (q == 1) { *c = -s0; *s = c0; }
  else if (q == 2) { *c = -c0; *s = -s0; }
  else { *c = s0; *s = -c0; }
}
static void sincos2pi_f(float u, float* c, float* s) {
  const float twopi = (float)6.283185307179586476925286766559;
  const int q = (int)(u * 4.0f);
  const float r = u - (float)q * 0.25f;
  float c0, s0;
  if (r <= 0.125f) { c0 = kcos_f(r * twopi); s0 = ksin_f(r * twopi); }
  else { float x = (0.25f - r) * twopi; c0 = ksin_f(x); s0 = kcos_f(x); }
  if (q == 0) { *c = c0; *s = s0; }
  else if (q == 1) { *c = -s0; *s = c0; }
  else if (q == 2) { *c = -c0; *s = -s0; }
  else { *c = s0; *s = -c0; }
}
double or_cos2pi_d(double u) { double c, s; sincos2pi_d(u, &c, &s); return c; }
float or_cos2pi_f(float u) { float c, s; sincos2pi_f(u, &c, &s); return c; }

/* Stream spec v2: a block x = philox({idx, chain, blk, tag | blk_hi << 8}, seed),
 * blk = step / S (S = 4 for f32 draws, 2 for f64 draws), serves S steps. */
static void block(uint64_t seed, uint32_t chain, uint64_t blk, uint32_t tag, uint32_t idx,
                  uint32_t out[4]) {
  uint32_t ctr[4] = {idx, chain, (uint32_t)blk, tag | ((uint32_t)(blk >> 32) << 8)};
  uint32_t key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
  or_philox(ctr, key, out);
}
double or_normal_d(uint64_t seed, uint32_t chain, uint64_t step, uint32_t tag, uint32_t idx) {
  uint32_t x[4];
  block(seed, chain, step / 2, tag, idx, x);
  double r = sqrt(-2.0 * or_log_d(unif_oc_d(x[0], x[1])));
  double c, s;
  sincos2pi_d(unif_co_d(x[2], x[3]), &c, &s);
  return (step % 2 == 0) ? r * c : r * s;
}
/* Spec v5, the f64 MH proposal normals: the same Box-Muller pairs with ln and
 * sin/cos from tables (gm_bm_tables.h, tools/make_bm_tables.py):
 * ln u1 = e ln2 + ln c_j + ln(1 + r), r = fma(m, 1/c_j, -1); 2 pi u2 =
 * 2 pi j/256 + th, angle addition with degree-7 sin th and degree-6 cos th - 1. */
#include "gm_bm_tables.h"
static const double bm_log[256] = {GM_BM_LOG_INIT};
static const double bm_sincos[512] = {GM_BM_SINCOS_INIT};
/* The pair (z0, z1) of one block's words x. -2 ln u1 is clamped at +0: for
 * u1 = 1 (probability 2^-53) the table form's ln rounds to +1.6e-17, and the
 * clamp keeps that r = 0 instead of sqrt of a negative (NaN). */
void or_tab_normal_pair(const uint32_t x[4], double z[2]) {
  const double u1 = unif_oc_d(x[0], x[1]);
  const uint64_t b = bits_d(u1);
  const int e = (int)(b >> 52) - 1023;
  const uint64_t mb = b & 0x000fffffffffffffull;
  const double m = from_bits_d(mb | 0x3ff0000000000000ull);
  const int jl = (int)(mb >> 45);
  const double invc = bm_log[2 * jl], logc = bm_log[2 * jl + 1];
  const double r = fma(m, invc, -1.0);
  double p = fma(r, -0x1.5555555555555p-3, 0x1.999999999999ap-3);
  p = fma(r, p, -0.25);
  p = fma(r, p, 0x1.5555555555555p-2);
  p = fma(r, p, -0.5);
  const double l1 = fma(r * r, p, r);
  const double de = (double)e;
  const double lnu = fma(de, 0x1.62e42fefa39efp-1, fma(de, 0x1.abc9e3b39803fp-56, logc + l1));
  const double m2l = -2.0 * lnu;
  const double rad = sqrt(m2l > 0.0 ? m2l : 0.0);
  const double u2 = unif_co_d(x[2], x[3]);
  const int j = (int)(u2 * 256.0);
  const double th = (u2 - (double)j * 0.00390625) * 0x1.921fb54442d18p+2;
  const double zz = th * th;
  const double sth = fma(th * zz, fma(zz, fma(zz, -0x1.a01a01a01a01ap-13, 0x1.1111111111111p-7), -0x1.5555555555555p-3), th);
  const double cm = zz * fma(zz, fma(zz, -0x1.6c16c16c16c17p-10, 0x1.5555555555555p-5), -0.5);
  const double S = bm_sincos[2 * j], Cc = bm_sincos[2 * j + 1];
  const double sv = fma(Cc, sth, fma(S, cm, S));
  const double cv = fma(-S, sth, fma(Cc, cm, Cc));
  z[0] = rad * cv;
  z[1] = rad * sv;
}
double or_tab_normal_d(uint64_t seed, uint32_t chain, uint64_t step, uint32_t tag, uint32_t idx) {
  uint32_t x[4];
  double z[2];
  block(seed, chain, step / 2, tag, idx, x);
  or_tab_normal_pair(x, z);
  return z[step % 2];
}
/* Spec v5 for the f32 HMC momenta (gm_rng.h normal_pair_tab32): the pair of
 * words (w1, w2) as or_normal_f's Box-Muller pair, ln and sin/cos from the f32
 * tables (1/c_j rounded to f32 and ln of its reciprocal; sin/cos rounded):
 * ln(1 + r) to degree 3, sin th to degree 3, cos th - 1 to degree 4. */
static const float bm32_log[256] = {GM_BM32_LOG_INIT};
static const float bm32_sincos[512] = {GM_BM32_SINCOS_INIT};
void or_tab_normal_pair_f(uint32_t w1, uint32_t w2, float z[2]) {
  const float u1 = unif_oc_f(w1);
  uint32_t b;
  memcpy(&b, &u1, 4);
  const int e = (int)(b >> 23) - 127;
  const uint32_t mb = b & 0x007fffffu, mbits = mb | 0x3f800000u;
  float m;
  memcpy(&m, &mbits, 4);
  const int jl = (int)(mb >> 16);
  const float invc = bm32_log[2 * jl], logc = bm32_log[2 * jl + 1];
  const float r = fmaf(m, invc, -1.0f);
  const float l1 = fmaf(r * r, fmaf(r, 0x1.555556p-2f, -0.5f), r);
  const float de = (float)e;
  const float lnu = fmaf(de, 6.9313812256e-01f, fmaf(de, 9.0580006145e-06f, logc + l1));
  const float m2l = -2.0f * lnu;
  const float rad = sqrtf(m2l > 0.0f ? m2l : 0.0f);
  const float u2 = unif_co_f(w2);
  const int j = (int)(u2 * 256.0f);
  const float th = (u2 - (float)j * 0.00390625f) * 0x1.921fb6p+2f;
  const float zz = th * th;
  const float sth = fmaf(th * zz, -0x1.555556p-3f, th);
  const float cm = zz * fmaf(zz, 0x1.555556p-5f, -0.5f);
  const float S = bm32_sincos[2 * j], Cc = bm32_sincos[2 * j + 1];
  const float sv = fmaf(Cc, sth, fmaf(S, cm, S));
  const float cv = fmaf(-S, sth, fmaf(Cc, cm, Cc));
  z[0] = rad * cv;
  z[1] = rad * sv;
}
/* the HMC momentum draw for `step` (TAG_MOM streams): f32 the table pairs of
 * the block's 4 words, f64 msun's pair (spec v2) */
float or_mom_normal_f(uint64_t seed, uint32_t chain, uint64_t step, uint32_t tag, uint32_t idx) {
  uint32_t x[4];
  float z[2];
  block(seed, chain, step / 4, tag, idx, x);
  const int k = (int)(step % 4), pair = k / 2;
  or_tab_normal_pair_f(x[2 * pair], x[2 * pair + 1], z);
  return z[k % 2];
}
double or_mom_normal_d(uint64_t seed, uint32_t chain, uint64_t step, uint32_t tag, uint32_t idx) {
  return or_normal_d(seed, chain, step, tag, idx);
}
float or_normal_f(uint64_t seed, uint32_t chain, uint64_t step, uint32_t tag, uint32_t idx);
static float or_mh_normal_f(uint64_t seed, uint32_t chain, uint64_t step, uint32_t tag, uint32_t idx) {
  return or_normal_f(seed, chain, step, tag, idx);
}
float or_normal_f(uint64_t seed, uint32_t chain, uint64_t step, uint32_t tag, uint32_t idx) {
  uint32_t x[4];
  block(seed, chain, step / 4, tag, idx, x);
  const int k = (int)(step % 4), pair = k / 2;
  float r = sqrtf(-2.0f * or_log_f(unif_oc_f(x[2 * pair])));
  float c, s;
  sincos2pi_f(unif_co_f(x[2 * pair + 1]), &c, &s);
  return (k % 2 == 0) ? r * c : r * s;
}
double or_uniform_co_d(uint64_t seed, uint32_t chain, uint64_t step, uint32_t tag, uint32_t idx) {
  uint32_t x[4];
  block(seed, chain, step / 2, tag, idx, x);
  const int k = (int)(step % 2);
  return unif_co_d(x[2 * k], x[2 * k + 1]);
}
float or_uniform_co_f(uint64_t seed, uint32_t chain, uint64_t step, uint32_t tag, uint32_t idx) {
  uint32_t x[4];
  block(seed, chain, step / 4, tag, idx, x);
  return unif_co_f(x[step % 4]);
}
static double uniform_oc_d(uint64_t seed, uint32_t chain, uint64_t step, uint32_t tag, uint32_t idx) {
  uint32_t x[4];
  block(seed, chain, step / 2, tag, idx, x);
  const int k = (int)(step % 2);
  return unif_oc_d(x[2 * k], x[2 * k + 1]);
}
static float uniform_oc_f(uint64_t seed, uint32_t chain, uint64_t step, uint32_t tag, uint32_t idx) {
  uint32_t x[4];
  block(seed, chain, step / 4, tag, idx, x);
  return unif_oc_f(x[step % 4]);
}

/* NUTS per-transition draws (stream spec v3). One Philox
 * block per (chain, transition st):
 *   x = philox({0, chain, st_lo, TAG_NUTS_EXP | st_hi << 8}, seed)
 * words 0,1: the transition's 64-bit stream key K (x0 | x1 << 32);
 * words 2,3: the slice variable's Exp1 = -ln u, u in (0,1] (f64 from (x2, x3),
 * f32 from x2). Every other scalar draw of the transition is
 *   h(K, idx) = mix64(K + (idx + 1) * 0x9E3779B97F4A7C15)
 * (the SplitMix64 finalizer over a Weyl sequence): doubling j's direction
 * uniform idx 2j, its top-level accept uniform idx 2j + 1, merge m (recursion
 * post-order) idx 64 + m; uniforms in [0,1): f64 (h >> 11) 2^-53, f32 (h >> 40)
 * 2^-24. One Philox per transition instead of one per draw. */
uint64_t or_mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
uint64_t or_nuts_key(uint64_t seed, uint32_t chain, uint64_t st, uint32_t w[4]) {
  block(seed, chain, st, TAG_NUTS_EXP, 0u, w);
  return (uint64_t)w[0] | ((uint64_t)w[1] << 32);
}
double or_nuts_u_d(uint64_t key, uint32_t idx) {
  const uint64_t h = or_mix64(key + (uint64_t)(idx + 1u) * 0x9E3779B97F4A7C15ull);
  return (double)(h >> 11) * 1.1102230246251565e-16;
}
float or_nuts_u_f(uint64_t key, uint32_t idx) {
  const uint64_t h = or_mix64(key + (uint64_t)(idx + 1u) * 0x9E3779B97F4A7C15ull);
  return (float)(uint32_t)(h >> 40) * 5.9604644775390625e-08f;
}
static double nuts_exp1_d(const uint32_t w[4]) { return -or_log_d(unif_oc_d(w[2], w[3])); }
static float nuts_exp1_f(const uint32_t w[4]) { return -or_log_f(unif_oc_f(w[2])); }

/* ===================== threading helper ===================== */
typedef struct {
  void (*fn)(void* ctx, int64_t c0, int64_t c1);
  void* ctx;
  int64_t c0, c1;
} or_job;
static void* or_job_main(void* p) {
  or_job* j = (or_job*)p;
  j->fn(j->ctx, j->c0, j->c1);
  return NULL;
}
static void parallel_chains(int64_t C, int threads, void (*fn)(void*, int64_t, int64_t), void* ctx) {
  if (threads <= 1 || C < 2) {
    fn(ctx, 0, C);
    return;
  }
  if (threads > C) threads = (int)C;
  pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * threads);
  or_job* jobs = (or_job*)malloc(sizeof(or_job) * threads);
  for (int i = 0; i < threads; ++i) {
    jobs[i].fn = fn;
    jobs[i].ctx = ctx;
    jobs[i].c0 = C * i / threads;
    jobs[i].c1 = C * (i + 1) / threads;
    pthread_create(&th[i], NULL, or_job_main, &jobs[i]);
  }
  for (int i = 0; i < threads; ++i) pthread_join(th[i], NULL);
  free(th);
  free(jobs);
}

/* ===================== Part 2: templated samplers ===================== */
#define CAT_(a, b) a##b
#define CAT(a, b) CAT_(a, b)

#define T double
#define SFX _d
#define LOG or_log_d
#define EXP or_exp_d
#define SQRT sqrt
#define FMA fma
#define NORMAL or_normal_d
#define MOM_NORMAL or_mom_normal_d
#define MH_NORMAL or_tab_normal_d
#define UNIF_CO or_uniform_co_d
#define UNIF_OC uniform_oc_d
#define NUTS_U or_nuts_u_d
#define NUTS_EXP1 nuts_exp1_d
#define MACH_EPS 2.220446049250313e-16
/* form 1's elementary functions: the C library's, which the reference's
 * f64::exp / ln / powf call on Linux (LLVM lowers them to libm) */
#define REXP exp
#define RLOG log
#define RPOW pow
#include "gm_oracle_t.inc"
#undef T
#undef SFX
#undef LOG
#undef EXP
#undef SQRT
#undef FMA
#undef NORMAL
#undef MOM_NORMAL
#undef MH_NORMAL
#undef UNIF_CO
#undef UNIF_OC
#undef NUTS_U
#undef NUTS_EXP1
#undef MACH_EPS
#undef REXP
#undef RLOG
#undef RPOW

#define T float
#define SFX _f
#define LOG or_log_f
#define EXP or_exp_f
#define SQRT sqrtf
#define FMA fmaf
#define NORMAL or_normal_f
#define MOM_NORMAL or_mom_normal_f
#define MH_NORMAL or_mh_normal_f
#define UNIF_CO or_uniform_co_f
#define UNIF_OC uniform_oc_f
#define NUTS_U or_nuts_u_f
#define NUTS_EXP1 nuts_exp1_f
#define MACH_EPS 1.1920928955078125e-07f
#define REXP expf
#define RLOG logf
#define RPOW powf
#include "gm_oracle_t.inc"
#undef T
#undef SFX

/* ---- mass-matrix warm-up: state init and the reference's unit tests ---- */
void or_mass_state_init(const or_mass_cfg* cfg, int64_t C, int D, int dtype_is_f64, or_mass_state* st) {
  (void)D;
  (void)dtype_is_f64;
  const int64_t sb = cfg->start_buffer > 1 ? cfg->start_buffer : 1;   /* MassMatrixWarmup::new */
  const int64_t wl = cfg->initial_window > 10 ? cfg->initial_window : 10;
  st->sched[0] = sb + wl;
  st->sched[1] = wl;
  for (int64_t c = 0; c < C; ++c) st->kind[c] = 0;  /* MassMatrix::identity */
}

int or_mass_diag_kat(const double* var, int D, double jitter, const double* p, double* ke,
                     double* inv_mul_out) {
  double inv[64], sq[64];
  if (D > 64) return 1;
  diag_from_var_d(var, D, jitter, inv, sq);
  double q = 0.0;  /* MassMatrix::kinetic, diagonal (generic_nuts.rs:239-245) */
  for (int i = 0; i < D; ++i) q = q + p[i] * p[i] * inv[i];
  *ke = 0.5 * q;
  mass_d M = {1, inv, sq, NULL};
  inv_mul_d(&M, p, inv_mul_out, D, 1);  /* the reference's two roundings */
  return 0;
}

int or_mass_dense_kat(const double* cov, int D, double jitter, const double* p, double* inv_mul_out) {
  double inv[64 * 64], chol[64 * 64];
  if (D > 64) return 1;
  if (!dense_from_cov_d(cov, D, jitter, inv, chol)) return 2;
  mass_d M = {2, inv, NULL, chol};
  inv_mul_d(&M, p, inv_mul_out, D, 1);  /* the reference's two roundings */
  return 0;
}

int or_mass_warmup_diag_kat(const double* xs, int n, int D, double reg, double jitter, double* inv,
                            double* sqrt_out) {
  double mean[64], m2d[64], delta[64];
  if (D > 64) return 1;
  running_d r = {0, mean, m2d, NULL, delta};
  running_reset_d(&r, D, 0);
  for (int k = 0; k < n; ++k) running_update_d(&r, xs + (size_t)k * D, D, 0);
  or_mass_cfg cfg = {1, 1, 1, 4, reg, jitter};
  mass_d M = {0, inv, sqrt_out, NULL};
  return maybe_update_d(&cfg, &r, D, &M, inv, sqrt_out) ? 0 : 2;
}

/* ===================== Part 3: diagnostics (stats.rs, f32) ===================== */

/* ndarray-style contiguous f32 sum: eight interleaved accumulators, folded. */
static float sum_f32(const float* v, int64_t n, int64_t stride) {
  float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  int64_t i = 0;
  for (; i + 8 <= n; i += 8)
    for (int k = 0; k < 8; ++k) acc[k] += v[(i + k) * stride];
  float tail = 0.0f;
  for (; i < n; ++i) tail += v[i * stride];
  return ((acc[0] + acc[4]) + (acc[1] + acc[5])) + ((acc[2] + acc[6]) + (acc[3] + acc[7])) + tail;
}

/* autocov_bf (stats.rs:659-681): x is [n][d] row-major */
void or_autocov_bf(const float* x, int64_t n, int64_t d, float* out) {
  float* col = (float*)malloc(sizeof(float) * (n > 0 ? n : 1));
  for (int64_t c = 0; c < d; ++c) {
    for (int64_t t = 0; t < n; ++t) col[t] = x[t * d + c];
    float mean = sum_f32(col, n, 1) / (float)n;
    for (int64_t t = 0; t < n; ++t) col[t] = col[t] - mean;
    for (int64_t lag = 0; lag < n; ++lag) {
      float s = 0.0f;
      for (int64_t t = 0; t < n - lag; ++t) s += col[t] * col[t + lag];
      out[lag * d + c] = s / (float)n;
    }
  }
  free(col);
}

/* autocov_fft (stats.rs:603-647): zero-pad to a power of two >= 2n-1, FFT,
 * |X|^2, inverse FFT, scale by 1/n_padded/n. Iterative radix-2 in f32. */
static void fft_f32(float* re, float* im, int64_t n, int inverse) {
  for (int64_t i = 1, j = 0; i < n; ++i) {
    int64_t bit = n >> 1;
    for (; j & bit; bit >>= 1) j ^= bit;
    j ^= bit;
    if (i < j) {
      float t = re[i]; re[i] = re[j]; re[j] = t;
      t = im[i]; im[i] = im[j]; im[j] = t;
    }
  }
  for (int64_t len = 2; len <= n; len <<= 1) {
    double ang = 2.0 * 3.14159265358979323846 / (double)len * (inverse ? 1.0 : -1.0);
    for (int64_t i = 0; i < n; i += len)
      for (int64_t k = 0; k < len / 2; ++k) {
        float wr = (float)cos(ang * (double)k), wi = (float)sin(ang * (double)k);
        float ur = re[i + k], ui = im[i + k];
        float vr = re[i + k + len / 2] * wr - im[i + k + len / 2] * wi;
        float vi = re[i + k + len / 2] * wi + im[i + k + len / 2] * wr;
        re[i + k] = ur + vr; im[i + k] = ui + vi;
        re[i + k + len / 2] = ur - vr; im[i + k + len / 2] = ui - vi;
      }
  }
}
void or_autocov_fft(const float* x, int64_t n, int64_t d, float* out) {
  int64_t np = 1;
  while (np < 2 * n - 1) np <<= 1;
  float* re = (float*)malloc(sizeof(float) * np);
  float* im = (float*)malloc(sizeof(float) * np);
  for (int64_t c = 0; c < d; ++c) {
    float s = 0.0f;
    for (int64_t t = 0; t < n; ++t) s += x[t * d + c];
    float mean = s / (float)n;
    for (int64_t t = 0; t < np; ++t) {
      re[t] = t < n ? x[t * d + c] - mean : 0.0f;
      im[t] = 0.0f;
    }
    fft_f32(re, im, np, 0);
    for (int64_t t = 0; t < np; ++t) {
      re[t] = re[t] * re[t] + im[t] * im[t];
      im[t] = 0.0f;
    }
    fft_f32(re, im, np, 1);
    for (int64_t t = 0; t < n; ++t) out[t * d + c] = re[t] / (float)np / (float)n;
  }
  free(re);
  free(im);
}

/* split_rhat_mean_ess (stats.rs:439-573) on parameters [p0, p0 + P) of an
 * f32 [C][N][Ptot] sample; rhat/ess receive P values. Parameters are
 * independent in every step of the reference (withinvar and ess map over
 * them, stats.rs:463-466, 545-548; the chain-axis mean of ess is
 * elementwise, :535), so a parameter range computes the same bits as the
 * whole sample does for those parameters. */
static void split_rhat_ess_range(const float* x, int64_t C, int64_t N, int64_t Ptot, int64_t p0,
                                 int64_t P, float* rhat, float* ess) {
  const int64_t h = N / 2, K = 2 * C;
  /* splitcat: [2C][h][P] */
  float* y = (float*)malloc(sizeof(float) * (size_t)(K * h * P > 0 ? K * h * P : 1));
  for (int64_t c = 0; c < C; ++c)
    for (int64_t t = 0; t < h; ++t)
      for (int64_t p = 0; p < P; ++p) {
        y[(c * h + t) * P + p] = x[(c * N + t) * Ptot + p0 + p];
        y[((C + c) * h + t) * P + p] = x[(c * N + (N - h) + t) * Ptot + p0 + p];
      }
  float* within = (float*)malloc(sizeof(float) * P);
  float* var = (float*)malloc(sizeof(float) * P);
  float* cms = (float*)malloc(sizeof(float) * K);
  float* sq = (float*)malloc(sizeof(float) * K);
  for (int64_t p = 0; p < P; ++p) { /* withinvar (stats.rs:456-504) */
    for (int64_t k = 0; k < K; ++k) cms[k] = sum_f32(&y[(k * h) * P + p], h, P) / (float)h;
    float overall = sum_f32(cms, K, 1) / (float)K;
    for (int64_t k = 0; k < K; ++k) { float d = cms[k] - overall; sq[k] = d * d; }
    float b = sum_f32(sq, K, 1) * ((float)h / (float)(K - 1));
    for (int64_t k = 0; k < K; ++k) {
      float s = 0.0f;
      for (int64_t t = 0; t < h; ++t) {
        float v = y[(k * h + t) * P + p];
        s += (v - cms[k]) * (v - cms[k]);
      }
      sq[k] = s / (float)h;
    }
    float w = sum_f32(sq, K, 1) / (float)K;
    within[p] = w;
    var[p] = (((float)h - 1.0f) / (float)h) * w + b / (float)h;
    rhat[p] = sqrtf(w / var[p]); /* rhat (stats.rs:452-454) */
  }
  /* ess (stats.rs:523-573): mean over chains of autocov, rho, Geyer */
  float* avg = (float*)calloc((size_t)(h * P > 0 ? h * P : 1), sizeof(float));
  float* ac = (float*)malloc(sizeof(float) * (size_t)(h * P > 0 ? h * P : 1));
  for (int64_t k = 0; k < K; ++k) {
    if (h <= 100) or_autocov_bf(&y[k * h * P], h, P, ac);
    else or_autocov_fft(&y[k * h * P], h, P, ac);
    for (int64_t i = 0; i < h * P; ++i) avg[i] += ac[i];
  }
  for (int64_t i = 0; i < h * P; ++i) avg[i] = avg[i] / (float)K;
  for (int64_t p = 0; p < P; ++p) {
    float mn = (h >= 2) ? (1.0f - (within[p] - avg[0 * P + p]) / var[p]) +
                              (1.0f - (within[p] - avg[1 * P + p]) / var[p])
                        : 0.0f;
    float out = 0.0f;
    for (int64_t i = 0; 2 * i + 1 < h; ++i) {
      float r0 = 1.0f - (within[p] - avg[(2 * i) * P + p]) / var[p];
      float r1 = 1.0f - (within[p] - avg[(2 * i + 1) * P + p]) / var[p];
      float pt = r0 + r1;
      if (pt <= 0.0f) break;
      if (pt > mn) pt = mn;
      mn = pt;
      out += pt;
    }
    float tau = -1.0f + 2.0f * out;
    ess[p] = (1.0f / tau) * (float)K * (float)h;
  }
  free(y); free(within); free(var); free(cms); free(sq); free(avg); free(ac);
}

void or_split_rhat_ess(const float* x, int64_t C, int64_t N, int64_t P, float* rhat, float* ess) {
  split_rhat_ess_range(x, C, N, P, 0, P, rhat, ess);
}

/* The same on `nthreads` threads, each owning a contiguous parameter range
 * (the reference's rayon map over parameters, stats.rs:464, 546); results
 * are bitwise those of or_split_rhat_ess. Lets the config-size parity tests
 * (65,536-262,144 split chains) finish in seconds. */
typedef struct {
  const float* x;
  int64_t C, N, P, p0, np;
  float *rhat, *ess;
} srange_job;
static void* srange_worker(void* arg) {
  srange_job* j = (srange_job*)arg;
  if (j->np > 0) split_rhat_ess_range(j->x, j->C, j->N, j->P, j->p0, j->np, j->rhat + j->p0, j->ess + j->p0);
  return NULL;
}
void or_split_rhat_ess_mt(const float* x, int64_t C, int64_t N, int64_t P, float* rhat, float* ess,
                          int nthreads) {
  if (nthreads < 1) nthreads = 1;
  if (nthreads > P) nthreads = (int)P;
  pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * (size_t)nthreads);
  srange_job* jobs = (srange_job*)malloc(sizeof(srange_job) * (size_t)nthreads);
  for (int i = 0; i < nthreads; ++i) {
    const int64_t a = P * i / nthreads, b = P * (i + 1) / nthreads;
    srange_job j = {x, C, N, P, a, b - a, rhat, ess};
    jobs[i] = j;
    pthread_create(&th[i], NULL, srange_worker, &jobs[i]);
  }
  for (int i = 0; i < nthreads; ++i) pthread_join(th[i], NULL);
  free(th);
  free(jobs);
}

/* MultiChainTracker (stats.rs:199-339): step() updates, then rhat(). */
void or_mct_rhat(const float* steps, int64_t nsteps, int64_t C, int64_t P, float* rhat) {
  float* mean = (float*)calloc((size_t)(C * P), sizeof(float));
  float* mean_sq = (float*)calloc((size_t)(C * P), sizeof(float));
  for (int64_t s = 0; s < nsteps; ++s) {
    float n = (float)(s + 1);
    for (int64_t i = 0; i < C * P; ++i) {
      float x = steps[s * C * P + i];
      mean[i] = (mean[i] * (n - 1.0f) + x) / n;
      if (s == 0) mean_sq[i] = x * x;
      else mean_sq[i] = (mean_sq[i] * (n - 1.0f) + x * x) / n;
    }
  }
  float n = (float)nsteps, nc = (float)C;
  float fac = n / (nc - 1.0f);
  for (int64_t p = 0; p < P; ++p) {
    float mc = 0.0f;
    for (int64_t c = 0; c < C; ++c) mc += mean[c * P + p];
    mc /= nc;
    float between = 0.0f, within = 0.0f;
    for (int64_t c = 0; c < C; ++c) {
      float d = mean[c * P + p] - mc;
      between += d * d;
    }
    between *= fac;
    for (int64_t c = 0; c < C; ++c) {
      float m = mean[c * P + p];
      within += (mean_sq[c * P + p] - m * m) * n / (n - 1.0f);
    }
    within /= nc;
    float v = within * ((n - 1.0f) / n) + between * (1.0f / n);
    rhat[p] = sqrtf(v / within);
  }
  free(mean);
  free(mean_sq);
}

/* MultiChainTracker acceptance EMA (stats.rs:256-265): p starts at 0, and
 * each step folds over the chains in order, accepted = row differs from the
 * previous step's row (the first step compares against zeros). */
float or_mct_p_accept(const float* steps, int64_t nsteps, int64_t C, int64_t P) {
  const float alpha = 0.01f;
  float p = 0.0f;
  for (int64_t s = 0; s < nsteps; ++s)
    for (int64_t c = 0; c < C; ++c) {
      int diff = 0;
      for (int64_t j = 0; j < P; ++j) {
        const float prev = s ? steps[((s - 1) * C + c) * P + j] : 0.0f;
        diff |= steps[(s * C + c) * P + j] != prev;
      }
      p = (1.0f - alpha) * p + alpha * (float)diff;
    }
  return p;
}

/* A batch of C ChainTrackers (stats.rs:24-131). or_ct_init = new(): n = 0,
 * p_accept = -1, last_state = initial state, mean = mean_sq = 0.
 * or_ct_step = step() with n the count after the increment. */
void or_ct_init(int64_t C, int64_t P, const float* x0, float* p_accept, float* last, float* mean,
                float* msq) {
  for (int64_t c = 0; c < C; ++c) p_accept[c] = -1.0f;
  for (int64_t i = 0; i < C * P; ++i) {
    last[i] = x0[i];
    mean[i] = 0.0f;
    msq[i] = 0.0f;
  }
}
void or_ct_step(int64_t C, int64_t P, uint64_t n_after, const float* x, float* p_accept, float* last,
                float* mean, float* msq) {
  const float alpha = 0.01f;
  const float n = (float)n_after;
  for (int64_t c = 0; c < C; ++c) {
    const float* xc = x + c * P;
    float* m = mean + c * P;
    float* q = msq + c * P;
    float* l = last + c * P;
    for (int64_t j = 0; j < P; ++j) {
      m[j] = (m[j] * (n - 1.0f) + xc[j]) / n;
      q[j] = (n_after == 1) ? xc[j] * xc[j] : (q[j] * (n - 1.0f) + xc[j] * xc[j]) / n;
    }
    const float p_start = p_accept[c] >= 0.0f ? p_accept[c] : (float)(xc[0] != l[0]);
    int diff = 0;
    for (int64_t j = 0; j < P; ++j) diff |= xc[j] != l[j];
    p_accept[c] = (1.0f - alpha) * p_start + alpha * (float)diff;
    for (int64_t j = 0; j < P; ++j) l[j] = xc[j];
  }
}
/* ChainTracker::stats (stats.rs:122-131) of every chain, then collect_rhat
 * over them (stats.rs:139-193): between divides by (C*P - 1), the element
 * count of the [C, P] difference array (diffs.len()). */
void or_collect_rhat(int64_t C, int64_t P, uint64_t n_steps, const float* mean, const float* msq,
                     float* rhat) {
  const float n = (float)n_steps, nc = (float)C;
  float nsum = 0.0f;
  for (int64_t c = 0; c < C; ++c) nsum += n;
  const float navg = nsum / nc;
  for (int64_t p = 0; p < P; ++p) {
    float within = 0.0f, gm = 0.0f, between = 0.0f;
    for (int64_t c = 0; c < C; ++c) {
      const float m = mean[c * P + p];
      within += (msq[c * P + p] - m * m) * n / (n - 1.0f);
    }
    within /= nc;
    for (int64_t c = 0; c < C; ++c) gm += mean[c * P + p];
    gm /= nc;
    for (int64_t c = 0; c < C; ++c) {
      const float d = mean[c * P + p] - gm;
      between += d * d;
    }
    between /= (float)(C * P - 1);
    const float var = between + within * ((navg - 1.0f) / navg);
    rhat[p] = sqrtf(var / within);
  }
}

/* ===================== KAT entry points (double) ===================== */
double or_find_reasonable_epsilon_d(const or_target* t, int lanes, int elems, const double* q,
                                    const double* p) {
  nctx_d cx;
  memset(&cx, 0, sizeof(cx));
  cx.t = t; cx.lanes = lanes; cx.elems = elems; cx.D = t->dim;
  cx.tmpv = (double*)malloc(sizeof(double) * t->dim);
  cx.tmpv2 = (double*)malloc(sizeof(double) * t->dim);
  double e = find_eps_d(&cx, q, p);
  free(cx.tmpv);
  free(cx.tmpv2);
  return e;
}

void or_build_tree_d(const or_target* t, int lanes, int elems, const double* q, const double* p,
                     const double* g, double logu, int v, int j, double eps, double joint0,
                     uint64_t seed, uint32_t chain, uint64_t step, double* out_vecs,
                     double* out_scalars) {
  const int D = t->dim;
  nctx_d cx;
  memset(&cx, 0, sizeof(cx));
  cx.t = t; cx.lanes = lanes; cx.elems = elems; cx.D = D;
  cx.seed = seed; cx.cid = chain; cx.step = step;
  uint32_t kw[4];
  cx.key = or_nuts_key(seed, chain, step, kw);
  for (int k = 0; k < 32; ++k) tree_alloc_d(&cx.ws[k], D);
  cx.tmpv = (double*)malloc(sizeof(double) * D);
  cx.tmpv2 = (double*)malloc(sizeof(double) * D);
  tree_d out;
  tree_alloc_d(&out, D);
  build_tree_d(&cx, q, p, g, NULL, NULL, logu, v, j, eps, joint0, &out);  /* identity mass */
  const double* vs[8] = {out.qm, out.pm, out.gm, out.qp, out.pp, out.gp, out.qprime, out.gprime};
  for (int k = 0; k < 8; ++k) memcpy(out_vecs + k * D, vs[k], sizeof(double) * D);
  out_scalars[0] = out.logp_prime;
  out_scalars[1] = (double)out.n;
  out_scalars[2] = (double)out.s;
  out_scalars[3] = out.alpha;
  out_scalars[4] = (double)out.n_alpha;
  for (int k = 0; k < 32; ++k) free(cx.ws[k].qm);
  free(out.qm);
  free(cx.tmpv);
  free(cx.tmpv2);
}
