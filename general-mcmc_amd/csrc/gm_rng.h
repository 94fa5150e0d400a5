// gm_rng.h — counter-based randomness and the transcendental functions the
// samplers need, written so that the host build (g++) and the gfx950 device
// build (hipcc) produce bit-identical results.
//
// Why this exists: the reference draws from rand 0.9 SmallRng + rand_distr
// (generic_hmc.rs:177,197; generic_nuts.rs:283,767,783,865,1305;
// metropolis_hastings.rs:313) and from burn's backend-global RNG
// (euclidean.rs:484-509). Neither stream can be reproduced here (no crate
// sources), and a serial stream cannot be split across 10^5 chains anyway.
// Every random number in this engine is instead a pure function of
//     (seed, chain, step, tag, idx)
// so a chain's draws do not depend on how chains are placed on lanes, waves or
// GPUs (bitwise-identical samples at 1/2/4/8 GPUs).
//
// Stream spec (v2). One Philox4x32-10 block
//     x = philox(counter = {idx, chain, blk, tag | blk_hi << 8}, key = seed),
//     blk = step / S,  S = 4 for f32 draws, 2 for f64 draws,
// serves S consecutive steps: f32 uniforms use one word each (u_k from x_k,
// k = step % 4); f64 uniforms use two words (u_k from x_{2k}, x_{2k+1},
// k = step % 2). Normals come in Box-Muller pairs that use both branches:
// f32 (z0,z1) from (u0,u1), (z2,z3) from (u2,u3); f64 (z0,z1) from (u0,u1),
// with z_{2j} = r cos(2 pi u_{2j+1}), z_{2j+1} = r sin(2 pi u_{2j+1}),
// r = sqrt(-2 ln u_{2j}) (u_{2j} from the (0,1] form); the draw for `step` is
// z_{step % S}. A kernel that runs consecutive steps computes each block once.
// Spec v5 keeps these pairs but evaluates ln and sin/cos from tables, with
// explicit fused multiply-adds (normals_tab: the f64 MH proposals;
// normals_tab32: the f32 HMC momenta); the oracle evaluates the same.
//
// Bit-exactness rules (both sides): only IEEE +,-,*,/ and sqrt (correctly
// rounded on gfx950 and x86), no FMA contraction (-ffp-contract=off), and our
// own log/exp/cos built from those. The CPU oracle (oracle/gm_oracle.c)
// restates the same spec independently.
#pragma once
#include <stdint.h>

#if defined(__HIPCC_RTC__)
#define GM_HD __host__ __device__ __forceinline__
#elif defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define GM_HD __host__ __device__ __forceinline__
#else
#include <math.h>
#include <string.h>
#define GM_HD static inline
#endif

namespace gm {

// Stream tags (counter word 3, low 8 bits).
enum : uint32_t {
  TAG_INIT = 1,      // initial positions (core.rs:444-475 init_det analogue)
  TAG_MOM = 2,       // HMC momentum (batched_hmc.rs:131)
  TAG_ACC = 3,       // HMC accept uniform (batched_hmc.rs:157)
  TAG_MH_PROP = 4,   // MH proposal noise (distributions.rs:368-376)
  TAG_MH_ACC = 5,    // MH accept uniform (metropolis_hastings.rs:313)
  TAG_NUTS_MOM = 6,  // NUTS momentum (generic_nuts.rs:760)
  TAG_NUTS_EXP = 7,  // NUTS slice Exp1 (generic_nuts.rs:767)
  TAG_NUTS_DIR = 8,  // NUTS direction uniform (generic_nuts.rs:783)
  TAG_NUTS_TOP = 9,  // NUTS top-level accept uniform (generic_nuts.rs:865)
  TAG_NUTS_MRG = 10, // NUTS subtree-merge f64 uniform (generic_nuts.rs:1305)
  TAG_NUTS_INIT = 11, // NUTS init momentum for find_reasonable_epsilon (:739)
  TAG_NUTS_PROBE = 12 // NUTS probe momentum after a mass-matrix update (:905-909)
};

struct u32x4 { uint32_t x, y, z, w; };

GM_HD uint32_t mulhi32(uint32_t a, uint32_t b) {
  return (uint32_t)(((uint64_t)a * (uint64_t)b) >> 32);
}

// Philox4x32-10 (Salmon et al., SC'11), the Random123 reference constants.
GM_HD u32x4 philox(u32x4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    // one 32x32->64 product per multiplier (a single v_mad_u64_u32 on gfx950)
    const uint64_t p0 = (uint64_t)0xD2511F53u * c.x, p1 = (uint64_t)0xCD9E8D57u * c.z;
    const uint32_t lo0 = (uint32_t)p0, hi0 = (uint32_t)(p0 >> 32);
    const uint32_t lo1 = (uint32_t)p1, hi1 = (uint32_t)(p1 >> 32);
    c = u32x4{hi1 ^ c.y ^ k0, lo1, hi0 ^ c.w ^ k1, lo0};
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return c;
}


// ---- bit casts -------------------------------------------------------------
GM_HD uint32_t f2u(float f) {
#if defined(__HIPCC__)
  return __builtin_bit_cast(uint32_t, f);
#else
  uint32_t u; memcpy(&u, &f, 4); return u;
#endif
}
GM_HD float u2f(uint32_t u) {
#if defined(__HIPCC__)
  return __builtin_bit_cast(float, u);
#else
  float f; memcpy(&f, &u, 4); return f;
#endif
}
GM_HD uint64_t d2u(double f) {
#if defined(__HIPCC__)
  return __builtin_bit_cast(uint64_t, f);
#else
  uint64_t u; memcpy(&u, &f, 8); return u;
#endif
}
GM_HD double u2d(uint64_t u) {
#if defined(__HIPCC__)
  return __builtin_bit_cast(double, u);
#else
  double f; memcpy(&f, &u, 8); return f;
#endif
}

GM_HD float gsqrt(float x) {
#if defined(__HIPCC__)
  return __builtin_sqrtf(x);
#else
  return sqrtf(x);
#endif
}
GM_HD double gsqrt(double x) {
#if defined(__HIPCC__)
  return __builtin_sqrt(x);
#else
  return sqrt(x);
#endif
}

// ---- uniforms ----------------------------------------------------------------
// [0,1):  f32 = (w>>8)*2^-24 ; f64 = ((a>>5)*2^26 + (b>>6)) * 2^-53
// (0,1]:  the same integer plus one.
template <class T> struct Unif;
template <> struct Unif<float> {
  GM_HD static float co(uint32_t a, uint32_t) { return (float)(a >> 8) * 5.9604644775390625e-08f; }
  GM_HD static float oc(uint32_t a, uint32_t) { return (float)((a >> 8) + 1u) * 5.9604644775390625e-08f; }
};
template <> struct Unif<double> {
  GM_HD static double co(uint32_t a, uint32_t b) {
    const uint64_t k = ((uint64_t)(a >> 5) << 26) | (uint64_t)(b >> 6);
    return (double)k * 1.1102230246251565e-16;
  }
  GM_HD static double oc(uint32_t a, uint32_t b) {
    const uint64_t k = ((uint64_t)(a >> 5) << 26) | (uint64_t)(b >> 6);
    return (double)(k + 1u) * 1.1102230246251565e-16;
  }
};

// ---- log (FreeBSD msun e_log.c / e_logf.c polynomials) ----------------------
GM_HD double glog(double x) {
  const double ln2_hi = 6.93147180369123816490e-01, ln2_lo = 1.90821492927058770002e-10;
  const double Lg1 = 6.666666666666735130e-01, Lg2 = 3.999999999940941908e-01,
               Lg3 = 2.857142874366239149e-01, Lg4 = 2.222219843214978396e-01,
               Lg5 = 1.818357216161805012e-01, Lg6 = 1.531383769920937332e-01,
               Lg7 = 1.479819860511658591e-01;
  uint64_t u = d2u(x);
  if (x != x) return x;                      // NaN
  if (x < 0.0) return u2d(0x7ff8000000000000ull);
  if (x == 0.0) return -u2d(0x7ff0000000000000ull);
  if ((u >> 52) >= 0x7ff) return x;          // +inf
  int k = 0;
  if ((u >> 52) == 0) { x = x * 18014398509481984.0; u = d2u(x); k = -54; }  // subnormal: *2^54
  k += (int)(u >> 52) - 1023;
  double m = u2d((u & 0x000fffffffffffffull) | 0x3ff0000000000000ull);  // [1,2)
  if (m > 1.4142135623730951) { m = m * 0.5; k += 1; }
  const double f = m - 1.0;
  const double s = f / (2.0 + f);
  const double z = s * s, w = z * z;
  const double t1 = w * (Lg2 + w * (Lg4 + w * Lg6));
  const double t2 = z * (Lg1 + w * (Lg3 + w * (Lg5 + w * Lg7)));
  const double R = t2 + t1;
  const double hfsq = 0.5 * f * f;
  const double dk = (double)k;
  return dk * ln2_hi - ((hfsq - (s * (hfsq + R) + dk * ln2_lo)) - f);
}

GM_HD float glog(float x) {
  const float ln2_hi = 6.9313812256e-01f, ln2_lo = 9.0580006145e-06f;
  const float Lg1 = 0.66666662693f, Lg2 = 0.40000972152f, Lg3 = 0.28498786688f, Lg4 = 0.24279078841f;
  uint32_t u = f2u(x);
  if (x != x) return x;
  if (x < 0.0f) return u2f(0x7fc00000u);
  if (x == 0.0f) return -u2f(0x7f800000u);
  if ((u >> 23) >= 0xff) return x;
  int k = 0;
  if ((u >> 23) == 0) { x = x * 33554432.0f; u = f2u(x); k = -25; }  // subnormal: *2^25
  k += (int)(u >> 23) - 127;
  float m = u2f((u & 0x007fffffu) | 0x3f800000u);
  if (m > 1.41421353816986083984f) { m = m * 0.5f; k += 1; }
  const float f = m - 1.0f;
  const float s = f / (2.0f + f);
  const float z = s * s, w = z * z;
  const float t1 = w * (Lg2 + w * Lg4);
  const float t2 = z * (Lg1 + w * Lg3);
  const float R = t2 + t1;
  const float hfsq = 0.5f * f * f;
  const float dk = (float)k;
  return dk * ln2_hi - ((hfsq - (s * (hfsq + R) + dk * ln2_lo)) - f);
}

// The same polynomials restricted to a positive normal finite x (no special
// cases: the uniforms fed to it are >= 2^-24 for f32 and >= 2^-53 for f64),
// identical bits to glog on that domain; branch-free.
GM_HD double glog_pos(double x) {
  const double ln2_hi = 6.93147180369123816490e-01, ln2_lo = 1.90821492927058770002e-10;
  const double Lg1 = 6.666666666666735130e-01, Lg2 = 3.999999999940941908e-01,
               Lg3 = 2.857142874366239149e-01, Lg4 = 2.222219843214978396e-01,
               Lg5 = 1.818357216161805012e-01, Lg6 = 1.531383769920937332e-01,
               Lg7 = 1.479819860511658591e-01;
  const uint64_t u = d2u(x);
  int k = (int)(u >> 52) - 1023;
  double m = u2d((u & 0x000fffffffffffffull) | 0x3ff0000000000000ull);
  const bool big = m > 1.4142135623730951;
  m = big ? m * 0.5 : m;
  k += big ? 1 : 0;
  const double f = m - 1.0;
  const double s = f / (2.0 + f);
  const double z = s * s, w = z * z;
  const double t1 = w * (Lg2 + w * (Lg4 + w * Lg6));
  const double t2 = z * (Lg1 + w * (Lg3 + w * (Lg5 + w * Lg7)));
  const double R = t2 + t1;
  const double hfsq = 0.5 * f * f;
  const double dk = (double)k;
  return dk * ln2_hi - ((hfsq - (s * (hfsq + R) + dk * ln2_lo)) - f);
}
GM_HD float glog_pos(float x) {
  const float ln2_hi = 6.9313812256e-01f, ln2_lo = 9.0580006145e-06f;
  const float Lg1 = 0.66666662693f, Lg2 = 0.40000972152f, Lg3 = 0.28498786688f, Lg4 = 0.24279078841f;
  const uint32_t u = f2u(x);
  int k = (int)(u >> 23) - 127;
  float m = u2f((u & 0x007fffffu) | 0x3f800000u);
  const bool big = m > 1.41421353816986083984f;
  m = big ? m * 0.5f : m;
  k += big ? 1 : 0;
  const float f = m - 1.0f;
  const float s = f / (2.0f + f);
  const float z = s * s, w = z * z;
  const float t1 = w * (Lg2 + w * Lg4);
  const float t2 = z * (Lg1 + w * Lg3);
  const float R = t2 + t1;
  const float hfsq = 0.5f * f * f;
  const float dk = (float)k;
  return dk * ln2_hi - ((hfsq - (s * (hfsq + R) + dk * ln2_lo)) - f);
}
// log of a [0,1) uniform: glog_pos, or -inf at 0 (the only special input).
template <class T> GM_HD T glog_unif(T u) {
  const T l = glog_pos(u);
  return (u == (T)0) ? (T)(-u2d(0x7ff0000000000000ull)) : l;
}

// ---- exp (FreeBSD msun e_exp.c / e_expf.c) -----------------------------------
GM_HD double scale2(double y, int k) {  // y * 2^k, y in [0.5, 2]
  if (k > 1023) return y * u2d(0x7fe0000000000000ull) * u2d((uint64_t)(k - 1023 + 1023) << 52);
  if (k < -1021) return y * u2d((uint64_t)(k + 1000 + 1023) << 52) * u2d((uint64_t)(-1000 + 1023) << 52);
  return y * u2d((uint64_t)(k + 1023) << 52);
}
// The constants of gexp(double); ExpConsts::pinned() holds them in VGPRs for a
// hot loop (a VALU operation with an SGPR operand issues at about half rate,
// and the compiler otherwise rebuilds each 64-bit constant with two scalar
// moves at every use). Same values either way.
struct ExpConsts {
  double o_th = 7.09782712893383973096e+02, u_th = -7.45133219101941108420e+02;
  double ln2HI = 6.93147180369123816490e-01, ln2LO = 1.90821492927058770002e-10;
  double invln2 = 1.44269504088896338700e+00;
  double P1 = 1.66666666666666019037e-01, P2 = -2.77777777770155933842e-03,
         P3 = 6.61375632143793436117e-05, P4 = -1.65339022054652515390e-06,
         P5 = 4.13813679705723846039e-08;
#if defined(__HIPCC__) || defined(__HIPCC_RTC__)
  __device__ static ExpConsts pinned() {
    ExpConsts K;
    asm volatile("" : "+v"(K.o_th), "+v"(K.u_th), "+v"(K.ln2HI), "+v"(K.ln2LO), "+v"(K.invln2));
    asm volatile("" : "+v"(K.P1), "+v"(K.P2), "+v"(K.P3), "+v"(K.P4), "+v"(K.P5));
    return K;
  }
#endif
};
GM_HD double gexp(double x, const ExpConsts& K) {
  const double o_th = K.o_th, u_th = K.u_th, ln2HI = K.ln2HI, ln2LO = K.ln2LO, invln2 = K.invln2;
  const double P1 = K.P1, P2 = K.P2, P3 = K.P3, P4 = K.P4, P5 = K.P5;
  // Branch-free (the NUTS leaf evaluates it for every chain of a wave): the
  // main path runs on a safe input and the special cases are selected at
  // the end; scale2's three forms are selected by their exponent fields.
  // Same values as the branching form.
  const bool nan = x != x, over = x > o_th, under = x < u_th;
  const double xs = (nan || over || under) ? 0.0 : x;
  const int k = (int)(invln2 * xs + (xs < 0.0 ? -0.5 : 0.5));
  const double dk = (double)k;
  const double hi = xs - dk * ln2HI, lo = dk * ln2LO;
  const double r = hi - lo;
  const double t = r * r;
  const double c = r - t * (P1 + t * (P2 + t * (P3 + t * (P4 + t * P5))));
  const double y = 1.0 - ((lo - (r * c) / (2.0 - c)) - hi);
  // scale2(y, k): (y * 2^1023) * 2^(k-1023) | (y * 2^(k+1000)) * 2^-1000 | (y * 2^k) * 1
  const bool big = k > 1023, small = k < -1021;
  const int e1 = big ? 2046 : small ? k + 2023 : k + 1023;
  const int e2 = big ? k : small ? 23 : 1023;
  const double res = (y * u2d((uint64_t)(uint32_t)e1 << 52)) * u2d((uint64_t)(uint32_t)e2 << 52);
  return nan ? x : over ? u2d(0x7ff0000000000000ull) : under ? 0.0 : res;
}
GM_HD double gexp(double x) { return gexp(x, ExpConsts{}); }
GM_HD float scale2f(float y, int k) {
  if (k > 127) return y * u2f(0x7f000000u) * u2f((uint32_t)(k - 127 + 127) << 23);
  if (k < -125) return y * u2f((uint32_t)(k + 100 + 127) << 23) * u2f((uint32_t)(-100 + 127) << 23);
  return y * u2f((uint32_t)(k + 127) << 23);
}
GM_HD float gexp(float x) {
  const float o_th = 8.8721679688e+01f, u_th = -1.0397208405e+02f;
  const float ln2HI = 6.9314575195e-01f, ln2LO = 1.4286067653e-06f, invln2 = 1.4426950216e+00f;
  const float P1 = 1.6666625440e-1f, P2 = -2.7667332906e-3f;
  if (x != x) return x;
  if (x > o_th) return u2f(0x7f800000u);
  if (x < u_th) return 0.0f;
  const int k = (int)(invln2 * x + (x < 0.0f ? -0.5f : 0.5f));
  const float dk = (float)k;
  const float hi = x - dk * ln2HI, lo = dk * ln2LO;
  const float r = hi - lo;
  const float t = r * r;
  const float c = r - t * (P1 + t * P2);
  const float y = 1.0f - ((lo - (r * c) / (2.0f - c)) - hi);
  return scale2f(y, k);
}
GM_HD float gexp(float x, const ExpConsts&) { return gexp(x); }

// ---- cos / sin of 2*pi*u, u in [0,1) ---------------------------------------
// Quadrant q = floor(4u), r = u - q/4 in [0, 1/4) (both exact); the first
// octant uses the sine/cosine kernels directly, the second their complements.
GM_HD double ksin(double x) {
  const double S1 = -1.66666666666666324348e-01, S2 = 8.33333333332248946124e-03,
               S3 = -1.98412698298579493134e-04, S4 = 2.75573137070700676789e-06,
               S5 = -2.50507602534068634195e-08, S6 = 1.58969099521155010221e-10;
  const double z = x * x, v = z * x;
  const double r = S2 + z * (S3 + z * (S4 + z * (S5 + z * S6)));
  return x + v * (S1 + z * r);
}
GM_HD double kcos(double x) {
  const double C1 = 4.16666666666666019037e-02, C2 = -1.38888888888741095749e-03,
               C3 = 2.48015872894767294178e-05, C4 = -2.75573143513906633035e-07,
               C5 = 2.08757232129817482790e-09, C6 = -1.13596475577881948265e-11;
  const double z = x * x, w = z * z;
  const double r = z * (C1 + z * (C2 + z * C3)) + w * w * (C4 + z * (C5 + z * C6));
  const double hz = 0.5 * z;
  const double ww = 1.0 - hz;
  return ww + (((1.0 - ww) - hz) + z * r);
}
GM_HD float ksin(float x) {
  const float z = x * x;
  return x + x * z * (-1.6666667163e-01f + z * (8.3333337680e-03f + z * (-1.9841270114e-04f + z * 2.7557314297e-06f)));
}
GM_HD float kcos(float x) {
  const float z = x * x;
  return 1.0f - 0.5f * z + z * z * (4.1666667908e-02f + z * (-1.3888889225e-03f + z * (2.4801587642e-05f + z * -2.7557314297e-07f)));
}
template <class T> GM_HD void sincos2pi(T u, T* c, T* s) {
  const T twopi = (T)6.283185307179586476925286766559;
  const T f4 = u * (T)4;
  const int q = (int)f4;          // u in [0,1): q in 0..3
  const T r = u - (T)q * (T)0.25;  // exact
  // branch-free: the same kernels on the same argument, then selects
  const bool lo = r <= (T)0.125;
  const T x = lo ? r * twopi : ((T)0.25 - r) * twopi;  // exact difference
  const T kc = kcos(x), ks = ksin(x);
  const T c0 = lo ? kc : ks, s0 = lo ? ks : kc;
  // rotate by q quarter turns: q=1 (-s0, c0), q=2 (-c0, -s0), q=3 (s0, -c0)
  const bool odd = (q & 1) != 0;
  const T cc = odd ? s0 : c0, ss = odd ? c0 : s0;
  *c = (q == 1 || q == 2) ? -cc : cc;
  *s = (q >= 2) ? -ss : ss;
}

// ---- blocked draws ---------------------------------------------------------
template <class T> struct Blk;  // draws per Philox block
template <> struct Blk<float> { static constexpr int S = 4; };
template <> struct Blk<double> { static constexpr int S = 2; };

GM_HD u32x4 draw_block(uint64_t seed, uint32_t chain, uint64_t blk, uint32_t tag, uint32_t idx) {
  u32x4 c{idx, chain, (uint32_t)blk, tag | ((uint32_t)(blk >> 32) << 8)};
  return philox(c, (uint32_t)seed, (uint32_t)(seed >> 32));
}

#if defined(__HIPCC__) || defined(__HIPCC_RTC__)
// Philox round keys held in VGPRs (device only): a VALU operation with an
// SGPR source issues at about half rate on gfx950 at 4 waves per SIMD
// (tools/probes/bank_probe.hip), and the vector Philox of the HMC draw block
// XORs a key into every round. Same values as philox(c, k0, k1).
struct PhiloxKeys {
  uint32_t k0[10], k1[10];
};
__device__ __forceinline__ PhiloxKeys philox_keys(uint64_t seed) {
  PhiloxKeys K;
  uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    uint32_t a = k0, b = k1;
    asm volatile("" : "+v"(a), "+v"(b));
    K.k0[r] = a;
    K.k1[r] = b;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return K;
}
__device__ __forceinline__ u32x4 draw_block(const PhiloxKeys& K, uint32_t chain, uint64_t blk, uint32_t tag,
                                            uint32_t idx) {
  u32x4 c{idx, chain, (uint32_t)blk, tag | ((uint32_t)(blk >> 32) << 8)};
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint64_t p0 = (uint64_t)0xD2511F53u * c.x, p1 = (uint64_t)0xCD9E8D57u * c.z;
    const uint32_t lo0 = (uint32_t)p0, hi0 = (uint32_t)(p0 >> 32);
    const uint32_t lo1 = (uint32_t)p1, hi1 = (uint32_t)(p1 >> 32);
    c = u32x4{hi1 ^ c.y ^ K.k0[r], lo1, hi0 ^ c.w ^ K.k1[r], lo0};
  }
  return c;
}
// The same block with the round keys re-derived by scalar adds inside the
// call: the seed is made opaque first, so the compiler cannot hoist the 20
// loop-invariant round keys out of a sampler's loop. In the register-heavy
// NUTS kernel those hoisted keys were spilled to VGPR lanes and restored by a
// v_readlane (plus its wait state) at every use; two SGPRs and ten s_add
// pairs replace them.
__device__ __forceinline__ u32x4 draw_block_s(uint64_t seed, uint32_t chain, uint64_t blk, uint32_t tag,
                                              uint32_t idx) {
  uint32_t k0 = __builtin_amdgcn_readfirstlane((uint32_t)seed);  // (uniform: a no-op where it is in SGPRs)
  uint32_t k1 = __builtin_amdgcn_readfirstlane((uint32_t)(seed >> 32));
  asm volatile("" : "+s"(k0), "+s"(k1));
  u32x4 c{idx, chain, (uint32_t)blk, tag | ((uint32_t)(blk >> 32) << 8)};
  return philox(c, k0, k1);
}
// The same block for a lane-varying counter: each round's two key mixings
// c.y ^ hi1 ^ k0 and c.w ^ hi0 ^ k1 as one v_bitop3_b32 each (truth table
// 0x96, a three-input XOR) instead of two v_xor_b32: the MH proposal
// normals, 20 of a block's ~55 integer instructions. (Only where the words
// are divergent: bitop3 is a vector instruction, and a wave-uniform block,
// e.g. an HMC chain's accept uniforms, would lose its scalar-unit form.)
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}
__device__ __forceinline__ u32x4 draw_block_v(uint64_t seed, uint32_t chain, uint64_t blk, uint32_t tag,
                                              uint32_t idx) {
  u32x4 c{idx, chain, (uint32_t)blk, tag | ((uint32_t)(blk >> 32) << 8)};
  uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint64_t p0 = (uint64_t)0xD2511F53u * c.x, p1 = (uint64_t)0xCD9E8D57u * c.z;
    const uint32_t lo0 = (uint32_t)p0, hi0 = (uint32_t)(p0 >> 32);
    const uint32_t lo1 = (uint32_t)p1, hi1 = (uint32_t)(p1 >> 32);
    c = u32x4{xor3(hi1, c.y, k0), lo1, xor3(hi0, c.w, k1), lo0};
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return c;
}
// N blocks of consecutive idx0 + n (the same chain, block and tag), rounds
// outermost: the N independent round chains are issued side by side, so each
// multiply's latency is covered by the other blocks' (the MH proposal draws
// of a lane's E coordinates). Each block equals draw_block_v's.
template <int N>
__device__ __forceinline__ void draw_blocks_v(u32x4 (&c)[N], uint64_t seed, uint32_t chain, uint64_t blk,
                                              uint32_t tag, uint32_t idx0) {
#pragma unroll
  for (int n = 0; n < N; ++n) c[n] = u32x4{idx0 + (uint32_t)n, chain, (uint32_t)blk, tag | ((uint32_t)(blk >> 32) << 8)};
  uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
#pragma unroll
  for (int r = 0; r < 10; ++r) {
#pragma unroll
    for (int n = 0; n < N; ++n) {
      const uint64_t p0 = (uint64_t)0xD2511F53u * c[n].x, p1 = (uint64_t)0xCD9E8D57u * c[n].z;
      const uint32_t lo0 = (uint32_t)p0, hi0 = (uint32_t)(p0 >> 32);
      const uint32_t lo1 = (uint32_t)p1, hi1 = (uint32_t)(p1 >> 32);
      c[n] = u32x4{xor3(hi1, c[n].y, k0), lo1, xor3(hi0, c[n].w, k1), lo0};
    }
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
}
#endif

// ---- NUTS per-transition draws (stream spec v3) ----------------------------
// One Philox block per (chain, transition st), TAG_NUTS_EXP: words x, y are
// the transition's 64-bit stream key K, words z, w the slice variable's Exp1
// uniform ((0,1] form). Every other scalar draw of the transition is
//   h(K, idx) = mix64(K + (idx + 1) * 0x9E3779B97F4A7C15)
// (SplitMix64's finalizer over a Weyl sequence): doubling j's direction idx
// 2j, its top-level accept idx 2j + 1, merge m (recursion post-order) idx
// 64 + m. One Philox per transition instead of one per draw.
GM_HD uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
GM_HD uint64_t nuts_key(u32x4 w) { return (uint64_t)w.x | ((uint64_t)w.y << 32); }
template <class T> GM_HD T nuts_u(uint64_t key, uint32_t idx);
template <> GM_HD double nuts_u<double>(uint64_t key, uint32_t idx) {
  const uint64_t h = mix64(key + (uint64_t)(idx + 1u) * 0x9E3779B97F4A7C15ull);
  return (double)(h >> 11) * 1.1102230246251565e-16;
}
template <> GM_HD float nuts_u<float>(uint64_t key, uint32_t idx) {
  const uint64_t h = mix64(key + (uint64_t)(idx + 1u) * 0x9E3779B97F4A7C15ull);
  return (float)(uint32_t)(h >> 40) * 5.9604644775390625e-08f;
}

// the S normals of a block
GM_HD void normals_of(u32x4 x, float (&z)[4]) {
  float c, s;
  const float r0 = gsqrt(-2.0f * glog_pos(Unif<float>::oc(x.x, 0)));
  sincos2pi<float>(Unif<float>::co(x.y, 0), &c, &s);
  z[0] = r0 * c;
  z[1] = r0 * s;
  const float r1 = gsqrt(-2.0f * glog_pos(Unif<float>::oc(x.z, 0)));
  sincos2pi<float>(Unif<float>::co(x.w, 0), &c, &s);
  z[2] = r1 * c;
  z[3] = r1 * s;
}
GM_HD void normals_of(u32x4 x, double (&z)[2]) {
  double c, s;
  const double r0 = gsqrt(-2.0 * glog_pos(Unif<double>::oc(x.x, x.y)));
  sincos2pi<double>(Unif<double>::co(x.z, x.w), &c, &s);
  z[0] = r0 * c;
  z[1] = r0 * s;
}
// the S uniforms of a block, [0,1) form
GM_HD void uniforms_of(u32x4 x, float (&u)[4]) {
  u[0] = Unif<float>::co(x.x, 0);
  u[1] = Unif<float>::co(x.y, 0);
  u[2] = Unif<float>::co(x.z, 0);
  u[3] = Unif<float>::co(x.w, 0);
}
GM_HD void uniforms_of(u32x4 x, double (&u)[2]) {
  u[0] = Unif<double>::co(x.x, x.y);
  u[1] = Unif<double>::co(x.z, x.w);
}
GM_HD float uniform_oc_k(u32x4 x, int k, float) {
  const uint32_t w = k == 0 ? x.x : k == 1 ? x.y : k == 2 ? x.z : x.w;
  return Unif<float>::oc(w, 0);
}
GM_HD double uniform_oc_k(u32x4 x, int k, double) {
  return k == 0 ? Unif<double>::oc(x.x, x.y) : Unif<double>::oc(x.z, x.w);
}

template <class T, int N> GM_HD T pick(const T (&v)[N], int k) {
  T r = v[0];
#pragma unroll
  for (int i = 1; i < N; ++i) r = (k == i) ? v[i] : r;
  return r;
}

// single draws (no caching)
template <class T> GM_HD T normal(uint64_t seed, uint32_t chain, uint64_t step, uint32_t tag, uint32_t idx) {
  T z[Blk<T>::S];
  normals_of(draw_block(seed, chain, step / Blk<T>::S, tag, idx), z);
  return pick(z, (int)(step % Blk<T>::S));
}
template <class T> GM_HD T uniform_co(uint64_t seed, uint32_t chain, uint64_t step, uint32_t tag, uint32_t idx) {
  T u[Blk<T>::S];
  uniforms_of(draw_block(seed, chain, step / Blk<T>::S, tag, idx), u);
  return pick(u, (int)(step % Blk<T>::S));
}
template <class T> GM_HD T uniform_oc(uint64_t seed, uint32_t chain, uint64_t step, uint32_t tag, uint32_t idx) {
  return uniform_oc_k(draw_block(seed, chain, step / Blk<T>::S, tag, idx), (int)(step % Blk<T>::S), (T)0);
}
template <class T> GM_HD T exp1(uint64_t seed, uint32_t chain, uint64_t step, uint32_t tag, uint32_t idx) {
  return -glog_pos(uniform_oc<T>(seed, chain, step, tag, idx));
}

// ---- table-driven f64 Box-Muller (spec v5: the f64 MH proposal normals) ---
// The same pairs as normals_of (z0 = r cos 2 pi u2, z1 = r sin 2 pi u2,
// r = sqrt(-2 ln u1), u1 in (0,1], u2 in [0,1) from the block's two word
// pairs), with ln and sin/cos from tables (gm_bm_tables.h,
// tools/make_bm_tables.py) instead of msun's polynomials and division:
//   ln u1 = e ln2 + ln c_j + ln(1 + r),  r = fma(m, 1/c_j, -1), |r| < 2^-8,
//     m in [1,2) the significand, j its top 7 bits, ln(1 + r) to degree 6;
//   2 pi u2 = 2 pi j/256 + th, th in [0, 2 pi/256): sin/cos(2 pi j/256) from
//     the table, sin th to degree 7, cos th - 1 to degree 6, angle addition.
#include "gm_bm_tables.h"
#if defined(__HIPCC__) || defined(__HIPCC_RTC__)
static __constant__ double gm_bm_log[256] = {GM_BM_LOG_INIT};
static __constant__ double gm_bm_sincos[512] = {GM_BM_SINCOS_INIT};
typedef double gm_bm_d2 __attribute__((ext_vector_type(2)));
struct BmLds {  // the tables as 16-byte pairs in LDS
  gm_bm_d2 lg[128], sc[256];
};
__device__ __forceinline__ void bm_lds_fill(BmLds& t) {
  for (int k = threadIdx.x; k < 256; k += blockDim.x) {
    if (k < 128) t.lg[k] = gm_bm_d2{gm_bm_log[2 * k], gm_bm_log[2 * k + 1]};
    t.sc[k] = gm_bm_d2{gm_bm_sincos[2 * k], gm_bm_sincos[2 * k + 1]};
  }
}
// ---- the NUTS leaf's acceptance statistic, f64 (leaf_alpha_tab) -----------
// min(1, exp(x)) (generic_nuts.rs:1212; Rust's f64::min gives 1 for a NaN) as
// exp(max(min(x, 0), -746)): a NaN or positive x yields exp(+-0) = 1 exactly,
// and below -746 the power underflows to +0 as exp's does. The exp is
// table-driven and division-free (msun's gexp ends in a quotient whose
// reciprocal and corrections sat on every leaf's critical path):
//   k = rint(64 x / ln2), r = x - k ln2/64 by two fmas (msun's split of ln2,
//   scaled by 1/64: k times the high part is exact), |r| <= ln2/128;
//   exp(r) - 1 = r + r^2 (1/2 + r/6 + ... + r^4/720) (truncation < 3e-20);
//   exp(x) = ldexp(fma(t, p, t), k >> 6), t = 2^((k & 63)/64) from the table
//   (gm_bm_tables.h GM_EXP64_INIT, staged in LDS).
// Within about 1 ulp of exp; oracle/gm_oracle.c or_leaf_alpha_d restates it
// operation for operation.
static __constant__ double gm_exp64[64] = {GM_EXP64_INIT};
__device__ __forceinline__ void exp64_lds_fill(double* t) {
  for (int k = threadIdx.x; k < 64; k += blockDim.x) t[k] = gm_exp64[k];
}
// Its 8 constants live in VGPRs from before the sampler's loop (make()): as
// SGPR pairs the compiler rebuilt them per use beside the kernel's spilled
// scalars. Measured against the msun form (profiles/r06/ab_nuts_leaf_exp.log,
// alternating processes): cfg3 3.59e9 -> 3.77e9 (constants left to the
// compiler) -> 3.87e9 leapfrogs/s (pinned), dense metric 1.14e9 -> 1.21e9 ->
// 1.24e9; bitwise against the oracle (434 GPU tests).
#ifndef GM_LEAF_EXP_PIN
#define GM_LEAF_EXP_PIN 1
#endif
struct LeafExpK {
  double c[8] = {-746.0, 0x1.71547652b82fep+6, 0x1.62e42fee00000p-7, 0x1.a39ef35793c76p-39,
                 0x1.6c16c16c16c17p-10, 0x1.1111111111111p-7, 0x1.5555555555555p-5, 0x1.5555555555555p-3};
  __device__ static LeafExpK make() {
    LeafExpK K;
    if (GM_LEAF_EXP_PIN) {
#pragma unroll
      for (int i = 0; i < 8; ++i) asm volatile("" : "+v"(K.c[i]));
    }
    return K;
  }
};
__device__ __forceinline__ double leaf_alpha_tab(double x, const double* t, const LeafExpK& K) {
  const double (&c)[8] = K.c;
  const double xs = __builtin_fmax(__builtin_fmin(x, 0.0), c[0]);
  const double dk = __builtin_rint(xs * c[1]);
  const int k = (int)dk;
  double r = __builtin_fma(-dk, c[2], xs);
  r = __builtin_fma(-dk, c[3], r);
  double a = __builtin_fma(r, c[4], c[5]);
  a = __builtin_fma(r, a, c[6]);
  a = __builtin_fma(r, a, c[7]);
  a = __builtin_fma(r, a, 0.5);
  const double p = __builtin_fma(r * r, a, r);
  const double tv = t[k & 63];
  return __builtin_ldexp(__builtin_fma(tv, p, tv), k >> 6);
}
// sqrt(x) for x = 0 or 2^-767 <= x < inf: LLVM's gfx950 f64 sequence (rsq, a
// Goldschmidt step, two Newton corrections) without its small-input scaling,
// which is the identity on that range; the same bits as gsqrt there.
__device__ __forceinline__ double sqrt_unscaled(double x) {
  const double y = __builtin_amdgcn_rsq(x);
  double g = x * y, h = y * 0.5;
  const double r = __builtin_fma(-h, g, 0.5);
  g = __builtin_fma(g, r, g);
  h = __builtin_fma(h, r, h);
  double d = __builtin_fma(-g, g, x);
  g = __builtin_fma(d, h, g);
  d = __builtin_fma(-g, g, x);
  g = __builtin_fma(d, h, g);
  return x == 0.0 ? x : g;
}
// N pairs side by side, statement by statement (the same operations per
// pair as normals_tab below, so the same bits): the pairs' dependent f64
// chains are independent of one another, and issuing them interleaved lets
// each cover the others' latency.
template <int N>
__device__ __forceinline__ void normals_tab_n(const u32x4 (&x)[N], double (&z0)[N], double (&z1)[N], const BmLds& t) {
  double u1[N], r[N], p[N], lnu[N], rad[N], th[N], zz[N], sth[N], cm[N];
  gm_bm_d2 lc[N], sc[N];
  int e[N];
#pragma unroll
  for (int n = 0; n < N; ++n) {
    const double D1 = u2d(((uint64_t)(0x43300000u | (x[n].x >> 12)) << 32) |
                          (((x[n].x << 20) & 0xFE000000u) | (x[n].y >> 7)));
    u1[n] = __builtin_fma(D1, 0x1p-52, u2d((x[n].y & 64u) ? 0xBFEFFFFFFFFFFFFEull : 0xBFEFFFFFFFFFFFFFull));
  }
#pragma unroll
  for (int n = 0; n < N; ++n) {
    const uint64_t b = d2u(u1[n]);
    e[n] = (int)(b >> 52) - 1023;
    const uint64_t mb = b & 0x000fffffffffffffull;
    lc[n] = t.lg[(int)(mb >> 45)];
    sc[n] = t.sc[(int)(x[n].z >> 24)];
  }
#pragma unroll
  for (int n = 0; n < N; ++n) {
    const uint64_t mb = d2u(u1[n]) & 0x000fffffffffffffull;
    const double m = u2d(mb | 0x3ff0000000000000ull);
    r[n] = __builtin_fma(m, lc[n].x, -1.0);
    const double D2 = u2d(((uint64_t)(0x43300000u | ((x[n].z >> 11) & 0x1FFFu)) << 32) |
                          (((x[n].z << 21) & 0xFC000000u) | (x[n].w >> 6)));
    th[n] = __builtin_fma(D2, 0x1.921fb54442d18p-51, -0x1.921fb54442d18p+1);
  }
#pragma unroll
  for (int n = 0; n < N; ++n) p[n] = __builtin_fma(r[n], -0x1.5555555555555p-3, 0x1.999999999999ap-3);
#pragma unroll
  for (int n = 0; n < N; ++n) zz[n] = th[n] * th[n];
#pragma unroll
  for (int n = 0; n < N; ++n) p[n] = __builtin_fma(r[n], p[n], -0.25);
#pragma unroll
  for (int n = 0; n < N; ++n) {
    sth[n] = __builtin_fma(th[n] * zz[n], __builtin_fma(zz[n], __builtin_fma(zz[n], -0x1.a01a01a01a01ap-13, 0x1.1111111111111p-7),
                                                        -0x1.5555555555555p-3), th[n]);
    cm[n] = zz[n] * __builtin_fma(zz[n], __builtin_fma(zz[n], -0x1.6c16c16c16c17p-10, 0x1.5555555555555p-5), -0.5);
  }
#pragma unroll
  for (int n = 0; n < N; ++n) p[n] = __builtin_fma(r[n], p[n], 0x1.5555555555555p-2);
#pragma unroll
  for (int n = 0; n < N; ++n) p[n] = __builtin_fma(r[n], p[n], -0.5);
#pragma unroll
  for (int n = 0; n < N; ++n) {
    const double l1 = __builtin_fma(r[n] * r[n], p[n], r[n]);
    const double de = (double)e[n];
    lnu[n] = __builtin_fma(de, 0x1.62e42fefa39efp-1, __builtin_fma(de, 0x1.abc9e3b39803fp-56, lc[n].y + l1));
  }
#pragma unroll
  for (int n = 0; n < N; ++n) {
    const double m2l = -2.0 * lnu[n];
    rad[n] = sqrt_unscaled(m2l > 0.0 ? m2l : 0.0);
  }
#pragma unroll
  for (int n = 0; n < N; ++n) {
    const double sv = __builtin_fma(sc[n].y, sth[n], __builtin_fma(sc[n].x, cm[n], sc[n].x));
    const double cv = __builtin_fma(-sc[n].x, sth[n], __builtin_fma(sc[n].y, cm[n], sc[n].y));
    z0[n] = rad[n] * cv;
    z1[n] = rad[n] * sv;
  }
}
__device__ __forceinline__ void normals_tab(u32x4 x, double (&z)[2], const BmLds& t) {
  // ln u1
  // u1 = (k + 1) 2^-53, k = (x >> 5) 2^26 + (y >> 6) (Unif<double>::oc) without
  // integer-to-double conversions: D = 2^52 + (k >> 1) assembled from its bits,
  // then u1 = fma(D, 2^-52, c), c = -1 + (1 + (k & 1)) 2^-53; the product and
  // the sum are exact and so is the result (a multiple of 2^-53 in (0, 1]).
  const double D1 = u2d(((uint64_t)(0x43300000u | (x.x >> 12)) << 32) |
                        (((x.x << 20) & 0xFE000000u) | (x.y >> 7)));
  const double u1 = __builtin_fma(D1, 0x1p-52, u2d((x.y & 64u) ? 0xBFEFFFFFFFFFFFFEull : 0xBFEFFFFFFFFFFFFFull));
  const uint64_t b = d2u(u1);
  const int e = (int)(b >> 52) - 1023;
  const uint64_t mb = b & 0x000fffffffffffffull;
  const double m = u2d(mb | 0x3ff0000000000000ull);
  const gm_bm_d2 lc = t.lg[(int)(mb >> 45)];
  const double r = __builtin_fma(m, lc.x, -1.0);
  double p = __builtin_fma(r, -0x1.5555555555555p-3, 0x1.999999999999ap-3);
  p = __builtin_fma(r, p, -0.25);
  p = __builtin_fma(r, p, 0x1.5555555555555p-2);
  p = __builtin_fma(r, p, -0.5);
  const double l1 = __builtin_fma(r * r, p, r);
  const double de = (double)e;
  const double lnu = __builtin_fma(de, 0x1.62e42fefa39efp-1, __builtin_fma(de, 0x1.abc9e3b39803fp-56, lc.y + l1));
  // clamped at +0: for u1 = 1 (probability 2^-53) ln u1 rounds to +1.6e-17
  const double m2l = -2.0 * lnu;
  // -2 ln u1 is 0 (clamped) or >= 2^-52 (u1 <= 1 - 2^-53)
  const double rad = sqrt_unscaled(m2l > 0.0 ? m2l : 0.0);
  // sin / cos of 2 pi u2, u2 = k2 2^-53 (Unif<double>::co): j = floor(256 u2)
  // is the top 8 bits of z, and th = RN((u2 - j/256) 2 pi) = RN(n 2^-53 2 pi)
  // with n = k2 mod 2^45: one fma on D = 2^52 + n from its bits, exact up to
  // the final rounding (D c - 2^52 c = n c for c = 2 pi 2^-53).
  const int j = (int)(x.z >> 24);
  const double D2 = u2d(((uint64_t)(0x43300000u | ((x.z >> 11) & 0x1FFFu)) << 32) |
                        (((x.z << 21) & 0xFC000000u) | (x.w >> 6)));
  const double th = __builtin_fma(D2, 0x1.921fb54442d18p-51, -0x1.921fb54442d18p+1);
  const double zz = th * th;
  const double sth = __builtin_fma(th * zz, __builtin_fma(zz, __builtin_fma(zz, -0x1.a01a01a01a01ap-13, 0x1.1111111111111p-7),
                                                          -0x1.5555555555555p-3), th);
  const double cm = zz * __builtin_fma(zz, __builtin_fma(zz, -0x1.6c16c16c16c17p-10, 0x1.5555555555555p-5), -0.5);
  const gm_bm_d2 sc = t.sc[j];
  const double sv = __builtin_fma(sc.y, sth, __builtin_fma(sc.x, cm, sc.x));
  const double cv = __builtin_fma(-sc.x, sth, __builtin_fma(sc.y, cm, sc.y));
  z[0] = rad * cv;
  z[1] = rad * sv;
}

// The f32 form (spec v5 for the f32 HMC momenta): the 4 normals of a block,
// pairs (x.x, x.y) and (x.z, x.w) as normals_of(float), with f32 tables
// (1/c_j rounded to f32 and ln of its reciprocal, sin/cos rounded):
//   ln u1 = e ln2 + ln c_j + ln(1 + r), r = fma(m, 1/c_j, -1), |r| < 2^-8,
//     ln(1 + r) to degree 3 (the next term < 2^-34);
//   sin th to degree 3 and cos th - 1 to degree 4, th < 2 pi/256.
// No division and no branch: 2 LDS reads and ~25 VALU per pair instead of
// msun's logf (a division) and sinf/cosf polynomials.
static __constant__ float gm_bm32_log[256] = {GM_BM32_LOG_INIT};
static __constant__ float gm_bm32_sincos[512] = {GM_BM32_SINCOS_INIT};
typedef float gm_bm_f2 __attribute__((ext_vector_type(2)));
struct BmLds32 {  // the f32 tables as 8-byte pairs in LDS (3 KiB)
  gm_bm_f2 lg[128], sc[256];
};
__device__ __forceinline__ void bm_lds_fill32(BmLds32& t) {
  for (int k = threadIdx.x; k < 256; k += blockDim.x) {
    if (k < 128) t.lg[k] = gm_bm_f2{gm_bm32_log[2 * k], gm_bm32_log[2 * k + 1]};
    t.sc[k] = gm_bm_f2{gm_bm32_sincos[2 * k], gm_bm32_sincos[2 * k + 1]};
  }
}
__device__ __forceinline__ void normal_pair_tab32(uint32_t w1, uint32_t w2, float& z0, float& z1,
                                                  const BmLds32& t) {
  const float u1 = Unif<float>::oc(w1, 0);
  const uint32_t b = f2u(u1);
  const int e = (int)(b >> 23) - 127;
  const uint32_t mb = b & 0x007fffffu;
  const float m = u2f(mb | 0x3f800000u);
  const gm_bm_f2 lc = t.lg[mb >> 16];
  const float r = __builtin_fmaf(m, lc.x, -1.0f);
  const float l1 = __builtin_fmaf(r * r, __builtin_fmaf(r, 0x1.555556p-2f, -0.5f), r);
  const float de = (float)e;
  // e ln2 as msun's logf split (ln2_hi has 17 significant bits: de * ln2_hi is exact)
  const float lnu = __builtin_fmaf(de, 6.9313812256e-01f, __builtin_fmaf(de, 9.0580006145e-06f, lc.y + l1));
  const float m2l = -2.0f * lnu;
  const float rad = gsqrt(m2l > 0.0f ? m2l : 0.0f);
  const float u2 = Unif<float>::co(w2, 0);
  const int j = (int)(u2 * 256.0f);
  const float th = (u2 - (float)j * 0.00390625f) * 0x1.921fb6p+2f;
  const float zz = th * th;
  const float sth = __builtin_fmaf(th * zz, -0x1.555556p-3f, th);
  const float cm = zz * __builtin_fmaf(zz, 0x1.555556p-5f, -0.5f);
  const gm_bm_f2 sc = t.sc[j];
  const float sv = __builtin_fmaf(sc.y, sth, __builtin_fmaf(sc.x, cm, sc.x));
  const float cv = __builtin_fmaf(-sc.x, sth, __builtin_fmaf(sc.y, cm, sc.y));
  z0 = rad * cv;
  z1 = rad * sv;
}
__device__ __forceinline__ void normals_tab32(u32x4 x, float (&z)[4], const BmLds32& t) {
  normal_pair_tab32(x.x, x.y, z[0], z[1], t);
  normal_pair_tab32(x.z, x.w, z[2], z[3], t);
}
// the HMC momenta of a block: the f32 table form, msun's f64 pairs
__device__ __forceinline__ void momenta_of(u32x4 x, float (&z)[4], const BmLds32& t) { normals_tab32(x, z, t); }
__device__ __forceinline__ void momenta_of(u32x4 x, double (&z)[2], const BmLds32&) { normals_of(x, z); }
#endif

// A per-lane cache of one block of draws for consecutive steps.
template <class T> struct NormalCache {
  T z[Blk<T>::S];
  uint64_t blk = ~0ull;
  GM_HD T get(uint64_t seed, uint32_t chain, uint64_t step, uint32_t tag, uint32_t idx) {
    const uint64_t b = step / Blk<T>::S;
    if (b != blk) {
      normals_of(draw_block(seed, chain, b, tag, idx), z);
      blk = b;
    }
    return pick(z, (int)(step % Blk<T>::S));
  }
#if defined(__HIPCC__) || defined(__HIPCC_RTC__)
  // get() with draw_block_s (scalar round keys; the NUTS momenta)
  __device__ T get_s(uint64_t seed, uint32_t chain, uint64_t step, uint32_t tag, uint32_t idx) {
    const uint64_t b = step / Blk<T>::S;
    if (b != blk) {
      normals_of(draw_block_s(seed, chain, b, tag, idx), z);
      blk = b;
    }
    return pick(z, (int)(step % Blk<T>::S));
  }
#endif
};
template <class T> struct UniformCache {
  T u[Blk<T>::S];
  uint64_t blk = ~0ull;
  GM_HD T get(uint64_t seed, uint32_t chain, uint64_t step, uint32_t tag, uint32_t idx) {
    const uint64_t b = step / Blk<T>::S;
    if (b != blk) {
      uniforms_of(draw_block(seed, chain, b, tag, idx), u);
      blk = b;
    }
    return pick(u, (int)(step % Blk<T>::S));
  }
};

// Register-resident draws for a kernel that walks consecutive steps: the
// block for step st is generated once (at the first step and at each block
// boundary), then consumed front to back by shifting, so no array is ever
// indexed by a runtime value (which the compiler would spill to LDS).
template <class T, int S> GM_HD void shift_front(T (&v)[S]) {
#pragma unroll
  for (int i = 0; i + 1 < S; ++i) v[i] = v[i + 1];
}
// drop the first k slots (k = st % S when a walk starts mid-block)
template <class T, int S> GM_HD void skip_front(T (&v)[S], int k) {
  for (int j = 0; j < k; ++j) shift_front(v);
}

}  // namespace gm
