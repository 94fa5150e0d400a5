// gm_device.h — lane-group primitives and built-in targets for the gfx950
// sampling kernels.
//
// Layout: a chain is owned by a group of LPC consecutive lanes of one
// wavefront (LPC in {1,2,...,64}); lane l of the group holds coordinates
// [l*E, (l+1)*E) of the chain in registers. Coordinates >= D are padding and
// stay exactly 0.
//
// Reduction order (the engine's defined summation order, mirrored by the CPU
// oracle): each lane sums its E terms left to right, then pairwise stages over
// the group's lanes, stage k combining lane l with lane partner_k(l):
//   l^1, l^2 (DPP quad_perm), l^7 (DPP row_half_mirror), l^15 (DPP row_mirror),
//   l^16, l^32 (ds_swizzle / bpermute),
// as many stages as log2(LPC). Each partner map is an involution and IEEE
// addition is commutative, so every lane of the group ends with the same total.
#pragma once
#include "gm_rng.h"

namespace gm {

// DPP move of a 32/64-bit value: lane l receives the value of the lane that
// the DPP control selects (sources out of range read 0).
template <int CTRL> __device__ __forceinline__ float dpp(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL,
                                                               0xf, 0xf, true));
}
template <int CTRL> __device__ __forceinline__ int dpp(int v) {
  return __builtin_amdgcn_update_dpp(0, v, CTRL, 0xf, 0xf, true);
}
template <int CTRL> __device__ __forceinline__ double dpp(double v) {
  const unsigned long long u = __builtin_bit_cast(unsigned long long, v);
  const int lo = __builtin_amdgcn_update_dpp(0, (int)(unsigned)u, CTRL, 0xf, 0xf, true);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(unsigned)(u >> 32), CTRL, 0xf, 0xf, true);
  return __builtin_bit_cast(double, ((unsigned long long)(unsigned)hi << 32) | (unsigned)lo);
}
enum : int {
  DPP_QUAD_XOR1 = 0xB1,   // quad_perm [1,0,3,2]
  DPP_QUAD_XOR2 = 0x4E,   // quad_perm [2,3,0,1]
  DPP_ROW_HALF_MIRROR = 0x141,
  DPP_ROW_MIRROR = 0x140,
  DPP_WAVE_SHL1 = 0x130,  // lane l <- lane l+1 (measured on gfx950, tools/probes/dpp_probe.hip)
  DPP_WAVE_SHR1 = 0x138   // lane l <- lane l-1
};

// Row broadcasts with a row mask: rows outside ROWMASK receive 0.
template <int CTRL, int ROWMASK> __device__ __forceinline__ float dpp_rows(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL,
                                                               ROWMASK, 0xf, false));
}
template <int CTRL, int ROWMASK> __device__ __forceinline__ double dpp_rows(double v) {
  const unsigned long long u = __builtin_bit_cast(unsigned long long, v);
  const int lo = __builtin_amdgcn_update_dpp(0, (int)(unsigned)u, CTRL, ROWMASK, 0xf, false);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(unsigned)(u >> 32), CTRL, ROWMASK, 0xf, false);
  return __builtin_bit_cast(double, ((unsigned long long)(unsigned)hi << 32) | (unsigned)lo);
}
template <int CTRL, int ROWMASK> __device__ __forceinline__ int dpp_rows(int v) {
  return __builtin_amdgcn_update_dpp(0, v, CTRL, ROWMASK, 0xf, false);
}
enum : int { DPP_ROW_BCAST15 = 0x142, DPP_ROW_BCAST31 = 0x143 };

__device__ __forceinline__ float lane63(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 63));
}
__device__ __forceinline__ int lane63(int v) { return __builtin_amdgcn_readlane(v, 63); }
__device__ __forceinline__ double lane63(double v) {
  const unsigned long long u = __builtin_bit_cast(unsigned long long, v);
  const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)u, 63);
  const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(u >> 32), 63);
  return __builtin_bit_cast(double, ((unsigned long long)hi << 32) | lo);
}

// value of lane k (wave-uniform result)
__device__ __forceinline__ float lane_k(float v, int k) {
  return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), k));
}
__device__ __forceinline__ double lane_k(double v, int k) {
  const unsigned long long u = __builtin_bit_cast(unsigned long long, v);
  const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)u, k);
  const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(u >> 32), k);
  return __builtin_bit_cast(double, ((unsigned long long)hi << 32) | lo);
}

// A chain of LPC > 64 lanes is the whole workgroup (the wide NUTS layouts,
// one chain per block of LPC/64 waves): its sum is each wave's 64-lane total
// (the group_sum<64> order) added over the waves left to right, through LDS
// (the oracle's order for lanes > 64, as block_sum). Every wave of the block
// reaches it together: the chain's control flow is uniform over the block.
template <int LPC, int N, class T> __device__ __forceinline__ void block_totals(T (&v)[N]) {
  constexpr int W = LPC / 64;
  __shared__ T red[N][W];
  const int w = (int)(threadIdx.x >> 6);
  if ((threadIdx.x & 63) == 0) {
#pragma unroll
    for (int k = 0; k < N; ++k) red[k][w] = v[k];
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < N; ++k) {
    T s = red[k][0];
#pragma unroll
    for (int u = 1; u < W; ++u) s = s + red[k][u];
    v[k] = s;
  }
  __syncthreads();  // red is reused by the next sum
}

// v + (the value of lane l ^ 16): rows r and r ^ 1 exchanged by one
// v_permlane16_swap per 32-bit half (a VALU op) instead of __shfl_xor's LDS
// round trip (ds_bpermute); the pair sum is the same in both rows (IEEE
// addition commutes), as with the shuffle.
__device__ __forceinline__ float xor16_sum(float v) {
  const unsigned u = __builtin_bit_cast(unsigned, v);
  const auto r = __builtin_amdgcn_permlane16_swap(u, u, false, false);
  return __builtin_bit_cast(float, (unsigned)r[0]) + __builtin_bit_cast(float, (unsigned)r[1]);
}
__device__ __forceinline__ double xor16_sum(double v) {
  const unsigned long long u = __builtin_bit_cast(unsigned long long, v);
  const auto lo = __builtin_amdgcn_permlane16_swap((unsigned)u, (unsigned)u, false, false);
  const auto hi = __builtin_amdgcn_permlane16_swap((unsigned)(u >> 32), (unsigned)(u >> 32), false, false);
  const double a = __builtin_bit_cast(double, ((unsigned long long)(unsigned)hi[0] << 32) | (unsigned)lo[0]);
  const double b = __builtin_bit_cast(double, ((unsigned long long)(unsigned)hi[1] << 32) | (unsigned)lo[1]);
  return a + b;
}
__device__ __forceinline__ int xor16_sum(int v) {
  const auto r = __builtin_amdgcn_permlane16_swap((unsigned)v, (unsigned)v, false, false);
  return (int)r[0] + (int)r[1];
}

template <int LPC, class T> __device__ __forceinline__ T group_sum(T v) {
  if constexpr (LPC > 64) {
    T t[1] = {group_sum<64>(v)};
    block_totals<LPC, 1>(t);
    return t[0];
  }
  if constexpr (LPC >= 2) v = v + dpp<DPP_QUAD_XOR1>(v);
  if constexpr (LPC >= 4) v = v + dpp<DPP_QUAD_XOR2>(v);
  if constexpr (LPC >= 8) v = v + dpp<DPP_ROW_HALF_MIRROR>(v);
  if constexpr (LPC >= 16) v = v + dpp<DPP_ROW_MIRROR>(v);
  if constexpr (LPC == 32) v = xor16_sum(v);
  if constexpr (LPC >= 64) {
    // Every lane of row r now holds the row total r_r. Rows 1 and 3 add the
    // broadcast of rows 0 and 2 (r1+r0, r3+r2), then row 3 adds row 1's value:
    // lane 63 = (r3+r2) + (r1+r0), bitwise the l^16, l^32 stage result
    // (r0+r1)+(r2+r3) since IEEE addition commutes. The total comes back
    // wave-uniform (one chain per wave).
    v = v + dpp_rows<DPP_ROW_BCAST15, 0xa>(v);
    v = v + dpp_rows<DPP_ROW_BCAST31, 0x8>(v);
    v = lane63(v);
  }
  return v;
}
// N independent group sums, stage-major: the same stages (and bits) as N
// calls of group_sum, issued interleaved so that each DPP stage's latency is
// covered by the other sums' stages instead of wait states.
// X without const (no <type_traits> under the runtime compiler)
template <class X> struct Bare { using type = X; };
template <class X> struct Bare<const X> { using type = X; };

template <int LPC, int N, class T> __device__ __forceinline__ void group_sum_n(T (&v)[N]) {
  // sched_barrier(0) between stages keeps the machine scheduler from
  // regrouping the stages per sum (it does, without them)
#define GM_STAGE(COND, EXPR)                                  \
  if constexpr (COND) {                                       \
    __builtin_amdgcn_sched_barrier(0);                        \
    _Pragma("unroll") for (int k = 0; k < N; ++k) v[k] = EXPR; \
  }
  GM_STAGE(LPC >= 2, v[k] + dpp<DPP_QUAD_XOR1>(v[k]))
  GM_STAGE(LPC >= 4, v[k] + dpp<DPP_QUAD_XOR2>(v[k]))
  GM_STAGE(LPC >= 8, v[k] + dpp<DPP_ROW_HALF_MIRROR>(v[k]))
  GM_STAGE(LPC >= 16, v[k] + dpp<DPP_ROW_MIRROR>(v[k]))
  GM_STAGE(LPC == 32, xor16_sum(v[k]))
  GM_STAGE(LPC >= 64, v[k] + (dpp_rows<DPP_ROW_BCAST15, 0xa>(v[k])))
  GM_STAGE(LPC >= 64, v[k] + (dpp_rows<DPP_ROW_BCAST31, 0x8>(v[k])))
  GM_STAGE(LPC >= 64, lane63(v[k]))
#undef GM_STAGE
  __builtin_amdgcn_sched_barrier(0);
  if constexpr (LPC > 64) block_totals<LPC, N>(v);
}
// lane l receives lane l+1's value. Wave-wide DPP shift: at a group's last
// lane the value comes from the next group (or 0); callers mask it, since a
// group's last coordinate never has a successor inside the chain.
template <int LPC, class T> __device__ __forceinline__ T from_next(T v) {
  if constexpr (LPC == 1) return v;
  else return dpp<DPP_WAVE_SHL1>(v);
}
// lane l receives lane l-1's value (group's first lane: masked by callers)
template <int LPC, class T> __device__ __forceinline__ T from_prev(T v) {
  if constexpr (LPC == 1) return v;
  else return dpp<DPP_WAVE_SHR1>(v);
}

// A chain spread over the W waves of one workgroup (hmc_wide_kernel, for
// dim > 1024): thread t of the block holds coordinates [t*E, (t+1)*E). Per-
// chain sums are each wave's 64-lane total (the group_sum<64> order) added
// over the waves left to right; Rosenbrock's neighbour values cross wave
// boundaries through LDS (double-buffered, one barrier per evaluation).
constexpr int GM_WIDE_MAX_WAVES = 16;
// threads per chain the wide kernels allow for E elements of esz bytes: up
// to 32 bytes per lane in 1024 threads (128 VGPRs), more in 512 (256 VGPRs)
__host__ __device__ constexpr int gm_wide_max_threads(int esz, int E) { return esz * E <= 32 ? 1024 : 512; }
template <class T> struct WideCtx {
  int w, W, lane;  // wave in the block, waves per chain, lane in the wave
  T* xfirst;       // LDS [2][16]: x[0] of each wave's lane 0
  T* xxlast;       // LDS [2][16]: x[E-1]^2 of each wave's lane 63
  T* red;          // LDS [16]: wave totals
  int par;         // buffer parity of the next evaluation
};
template <class T> __device__ __forceinline__ T block_sum(T v, const WideCtx<T>& c) {
  v = group_sum<64>(v);  // wave total, wave-uniform
  if (c.lane == 0) c.red[c.w] = v;
  __syncthreads();
  T s = c.red[0];
  for (int k = 1; k < c.W; ++k) s = s + c.red[k];
  __syncthreads();  // red is reused by the next sum
  return s;
}

// Branch-free "c ? v : +0" with a per-lane mask the compiler cannot see
// through (an empty asm), so it stays one v_and per use instead of being
// turned back into a select and then into a divergent branch around the
// guarded arithmetic.
template <class T> struct MaskOf;
template <> struct MaskOf<float> { using type = uint32_t; };
template <> struct MaskOf<double> { using type = uint64_t; };
template <class T> __device__ __forceinline__ typename MaskOf<T>::type lane_mask(bool c) {
  using M = typename MaskOf<T>::type;
  M m = c ? ~(M)0 : (M)0;
  asm("" : "+v"(m));
  return m;
}
template <class T> __device__ __forceinline__ T keep(T v, typename MaskOf<T>::type m) {
  using M = typename MaskOf<T>::type;
  return __builtin_bit_cast(T, __builtin_bit_cast(M, v) & m);
}

// ---------------------------------------------------------------------------
// Rosenbrock: logp = -sum_{i<=D-2} [ b*(x_{i+1}-x_i^2)^2 + (a-x_i)^2 ]
// RosenbrockND (distributions.rs:544-554) is a=1, b=100; Rosenbrock2D
// (distributions.rs:502-515) is D=2 with free a,b. Gradient (analytic form of
// what autodiff computes, hmc.rs:42-61), evaluated branch-free as
//   g_i = A_i - B_i,  A_i = [i<=D-2] ( (4b x_i) t_i + 2 (a - x_i) ),
//                     B_i = [1<=i<=D-1] (2b t_{i-1}),   t_i = x_{i+1} - x_i^2
// ([.] selects +0 when false).
// explicit fused multiply-add (one rounding; C fma/fmaf in the oracle)
__device__ __forceinline__ float gfma(float a, float b, float c) { return __builtin_fmaf(a, b, c); }
__device__ __forceinline__ double gfma(double a, double b, double c) { return __builtin_fma(a, b, c); }

// a / b for a divisor b fixed over a kernel, with y = RN(1/b) precomputed:
// the IEEE quotient RN(a/b) in one multiply and four fused multiply-adds
// instead of the ~10-instruction division sequence. q0 = RN(a y) is within
// 1.5 ulp of a/b; one Newton-Markstein correction q1 = RN(q0 + RN(a - b q0) y)
// is faithful; a second one, q2, is then the correctly rounded quotient
// (Markstein's theorem: y within half an ulp of 1/b and a faithful q). The
// theorem needs each remainder a - b q exact, which holds while the dividend
// is at least 2^(emin + p) (f64 2^-969, f32 2^-102; below that the remainder
// can fall into the subnormal range and round), and excludes under/overflow
// and non-finite a. So q2 is returned with `bad` set when |q2| is outside the
// exponent range [lo, hi] where both hold: hi = 2^1000 (f32 2^98), and lo the
// larger of 2^-1000 (f32 2^-99) and the quotient of the smallest safe
// dividend, 2^-968 (f32 2^-100), by b -- one per divisor (DivConst), so the
// test stays one exponent compare per quotient. The caller tests one flag for
// several quotients and takes the IEEE division in its rare branch (zero,
// subnormal, inf and NaN quotients are all outside; a = 0 then keeps its sign).
template <class T> struct DivConst {
  T b, y;             // the divisor and RN(1 / b)
  uint32_t lo, span;  // q2's biased exponent must lie in [lo, lo + span]
  __host__ __device__ static DivConst make(T b) {
    DivConst d;
    d.b = b;
    d.y = (T)1 / b;
    // eb = floor(log2 b) for a normal b > 0 (else the bound below is moot:
    // y or q0 is then non-finite and q2 falls out of range by itself)
    if constexpr (sizeof(T) == 8) {
      const int eb = (int)((__builtin_bit_cast(uint64_t, b) >> 52) & 0x7FF) - 1023;
      const int lo = 57 - eb > 23 ? 57 - eb : 23;  // |q2| >= 2^(lo-1023) => |a| >= 2^-968
      d.lo = lo > 2022 ? 2022u : (uint32_t)lo;
      d.span = 2022u - d.lo;
    } else {
      const int eb = (int)((__builtin_bit_cast(uint32_t, b) >> 23) & 0xFF) - 127;
      const int lo = 28 - eb > 28 ? 28 - eb : 28;   // |q2| >= 2^(lo-127) => |a| >= 2^-100
      d.lo = lo > 225 ? 225u : (uint32_t)lo;
      d.span = 225u - d.lo;
    }
    return d;
  }
};
template <class T> __device__ __forceinline__ T div_by_const_q(T a, const DivConst<T>& dc, bool& bad) {
  const T b = dc.b, y = dc.y;
  const T q0 = a * y;
  const T q1 = gfma(gfma(-b, q0, a), y, q0);
  const T q2 = gfma(gfma(-b, q1, a), y, q1);
  if constexpr (sizeof(T) == 8) {
    const uint32_t ex = (uint32_t)(__builtin_bit_cast(uint64_t, q2) >> 52) & 0x7FFu;
    bad |= ex - dc.lo > dc.span;
  } else {
    const uint32_t ex = (__builtin_bit_cast(uint32_t, q2) >> 23) & 0xFFu;
    bad |= ex - dc.lo > dc.span;
  }
  return q2;
}

template <class T, int E> struct RosenbrockLane;
template <class T> struct RosenbrockT {
  T a, b, b2, b4;  // b2 = 2b, b4 = 4b (rounded once, host side)
  int D;
  // per-lane view with the coordinate masks computed once per kernel
  template <int LPC, int E> __host__ __device__ size_t lds_bytes() const { return 0; }
  template <int LPC, int E> __device__ __forceinline__ RosenbrockLane<T, E> bind(int lane) const {
    RosenbrockLane<T, E> r;
    r.a = a; r.b = b; r.b2 = b2; r.b4 = b4; r.Dc = D;
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const int i = lane * E + e;
      r.ms[e] = lane_mask<T>(i <= D - 2);
      r.mp[e] = lane_mask<T>((i >= 1) & (i <= D - 1));
      r.b4m[e] = (i <= D - 2) ? b4 : (T)0;
      r.nc2m[e] = (i <= D - 2) ? (T)-2 : (T)0;
      r.cam[e] = (i <= D - 2) ? (T)2 * a : (T)0;
      r.nb2m[e] = ((i >= 1) & (i <= D - 1)) ? -b2 : (T)0;
    }
    return r;
  }
};
template <class T, int E> struct RosenbrockLane {
  T a, b, b2, b4;
  int Dc;
  typename MaskOf<T>::type ms[E], mp[E];  // [i <= D-2], [1 <= i <= D-1]
  T b4m[E], nc2m[E], cam[E], nb2m[E];     // 4b, -2, 2a, -2b where those masks hold, else 0
  template <int LPC, int E_, bool LOGP>
  __device__ __forceinline__ T eval(const T (&x)[E], T (&g)[E], int) const {
    static_assert(E_ == E, "layout mismatch");
    if constexpr (LPC >= 64) {
      const T part = LPC == 64 ? eval64<LOGP>(x, g) : eval_cross<LPC, LOGP>(x, g);
      if (LOGP) return -group_sum<LPC>(part);
      return (T)0;
    }
    T t[E];
    // Both lane shifts read x only: t_{i-1} for a group's first slot is
    // recomputed from x_{i-1} (the operands lane i-1 uses, so the same bits)
    // instead of being shifted out of t, which keeps one DPP off the chain.
    const T nx = from_next<LPC>(x[0]);
    const T px = from_prev<LPC>(x[E - 1]);
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const T xn = (e + 1 < E) ? x[(e + 1 < E) ? e + 1 : e] : nx;
      t[e] = xn - x[e] * x[e];
    }
    const T tp = x[0] - px * px;
    T part = (T)0;
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const T tprev = (e > 0) ? t[(e > 0) ? e - 1 : 0] : tp;
      const T am = a - x[e];
      const T A = keep((b4 * x[e]) * t[e] + (T)2 * am, ms[e]);
      const T B = keep(b2 * tprev, mp[e]);
      g[e] = A - B;
      if (LOGP) {
        const T s = keep(b * (t[e] * t[e]) + am * am, ms[e]);
        part = (e == 0) ? s : part + s;
      }
    }
    if (LOGP) return -group_sum<LPC>(part);
    return (T)0;
  }
  // The evaluation split for callers that reduce the log-density together
  // with another per-chain sum (hmc_kernel's last leapfrog, every NUTS leaf):
  // eval_part returns this lane's unreduced term (the operations of eval),
  // logp = finish(group_sum(part)).
  template <int LPC> static constexpr bool has_part = true;
  template <int LPC, int E_>
  __device__ __forceinline__ T eval_part(const T (&x)[E], T (&g)[E], int) const {
    static_assert(E_ == E, "layout mismatch");
    if constexpr (LPC == 64) {
      return eval64<true>(x, g);
    } else if constexpr (LPC > 64) {
      return eval_cross<LPC, true>(x, g);
    } else {
      T t[E];
      const T nx = from_next<LPC>(x[0]);
      const T px = from_prev<LPC>(x[E - 1]);
#pragma unroll
      for (int e = 0; e < E; ++e) {
        const T xn = (e + 1 < E) ? x[(e + 1 < E) ? e + 1 : e] : nx;
        t[e] = xn - x[e] * x[e];
      }
      const T tp = x[0] - px * px;
      T part = (T)0;
#pragma unroll
      for (int e = 0; e < E; ++e) {
        const T tprev = (e > 0) ? t[(e > 0) ? e - 1 : 0] : tp;
        const T am = a - x[e];
        const T A = keep((b4 * x[e]) * t[e] + (T)2 * am, ms[e]);
        const T B = keep(b2 * tprev, mp[e]);
        g[e] = A - B;
        const T s = keep(b * (t[e] * t[e]) + am * am, ms[e]);
        part = (e == 0) ? s : part + s;
      }
      return part;
    }
  }
  __device__ __forceinline__ T finish(T total) const { return -total; }
  // The 64-lane form for a chain of LPC > 64 lanes, i.e. the whole
  // workgroup (the wide NUTS layouts): the wave-boundary neighbours x_{i+1}
  // and (x_{i-1})^2 come from LDS instead of reading 0, so the operands, and
  // the bits, are those of a single group holding the whole chain. Every
  // wave of the block evaluates together (the chain's control flow).
  template <int LPC, bool LOGP>
  __device__ __forceinline__ T eval_cross(const T (&x)[E], T (&g)[E]) const {
    constexpr int W = LPC / 64;
    __shared__ T xb[2][W];  // each wave's lane-0 x[0] and lane-63 x[E-1]^2
    const int w = (int)(threadIdx.x >> 6), ln = (int)(threadIdx.x & 63);
    T xx[E];
#pragma unroll
    for (int e = 0; e < E; ++e) xx[e] = x[e] * x[e];
    if (ln == 0) xb[0][w] = x[0];
    if (ln == 63) xb[1][w] = xx[E - 1];
    __syncthreads();
    const T bnx = (w + 1 < W) ? xb[0][w + 1 < W ? w + 1 : w] : (T)0;  // wave-uniform reads
    const T bpxx = (w > 0) ? xb[1][w > 0 ? w - 1 : 0] : (T)0;
    __syncthreads();  // xb is rewritten by the next evaluation
    T nx = from_next<64>(x[0]);
    T pxx = from_prev<64>(xx[E - 1]);
    nx = (ln == 63) ? bnx : nx;
    pxx = (ln == 0) ? bpxx : pxx;
    return eval64_core<LOGP>(x, g, xx, nx, pxx);
  }
  template <bool LOGP>
  __device__ __forceinline__ T eval64(const T (&x)[E], T (&g)[E]) const {
    constexpr int LPC = 64;
    T xx[E];
#pragma unroll
    for (int e = 0; e < E; ++e) xx[e] = x[e] * x[e];
    const T nx = from_next<LPC>(x[0]);
    const T pxx = from_prev<LPC>(xx[E - 1]);
    return eval64_core<LOGP>(x, g, xx, nx, pxx);
  }
  template <bool LOGP>
  __device__ __forceinline__ T eval64_core(const T (&x)[E], T (&g)[E], const T (&xx)[E], T nx, T pxx) const {
    {
      // One chain per wave: the lane shifts read 0 beyond the wave and the
      // padding coordinates are 0, so a boundary lane can only see finite
      // values of its own chain. The [.] factors are then applied by
      // multiplying with per-lane constants that are 0 where the term is
      // absent (the engine's canonical form for 64-lane groups; the oracle
      // mirrors it), and (x_{i-1})^2 is shifted in from the lane that
      // computed it, so t_{i-1} is one DPP-fed subtract.
      T t[E];
#pragma unroll
      for (int e = 0; e < E; ++e) {
        const T xn = (e + 1 < E) ? x[(e + 1 < E) ? e + 1 : e] : nx;
        t[e] = xn - xx[e];
      }
      const T tp = x[0] - pxx;
      T part = (T)0;
#pragma unroll
      for (int e = 0; e < E; ++e) {
        const T tprev = (e > 0) ? t[(e > 0) ? e - 1 : 0] : tp;
        // g = x (4b t - 2) + (2a - 2b t_prev) as three fused multiply-adds,
        // the t_prev term beside the t chain (two dependent fmas after t)
        g[e] = gfma(x[e], gfma(b4m[e], t[e], nc2m[e]), gfma(nb2m[e], tprev, cam[e]));
        if (LOGP) {
          const T am = a - x[e];
          const T s = keep(b * (t[e] * t[e]) + am * am, ms[e]);
          part = (e == 0) ? s : part + s;
        }
      }
      return part;
    }
  }
  // The 64-lane form (eval64) for a chain spread over a workgroup: the wave-
  // boundary neighbours come from LDS instead of reading 0 (same operands,
  // same bits as a single group holding the whole chain). The [.] factors
  // are the constants themselves in waves without a chain-end coordinate
  // (wave-uniform branch) and are derived from the index in the two others,
  // instead of 5*E per-lane registers.
  template <int E_, bool LOGP>
  __device__ __forceinline__ T eval_wide(const T (&x)[E], T (&g)[E], WideCtx<T>& c) const {
    static_assert(E_ == E, "layout mismatch");
    const int bb = c.par * GM_WIDE_MAX_WAVES;
    c.par ^= 1;
    const T xxl = x[E - 1] * x[E - 1];
    if (c.lane == 0) c.xfirst[bb + c.w] = x[0];
    if (c.lane == 63) c.xxlast[bb + c.w] = xxl;
    __syncthreads();
    const T bnx = (c.w + 1 < c.W) ? c.xfirst[bb + c.w + 1] : (T)0;  // wave-uniform reads
    const T bpxx = (c.w > 0) ? c.xxlast[bb + c.w - 1] : (T)0;
    T nx = from_next<64>(x[0]);
    T pxx = from_prev<64>(xxl);
    nx = (c.lane == 63) ? bnx : nx;
    pxx = (c.lane == 0) ? bpxx : pxx;
    const int D = Dc;
    const int i0 = (c.w * 64 + c.lane) * E;
    const bool interior = c.w * 64 * E >= 1 && (c.w * 64 + 63) * E + E - 1 <= D - 2;
    T part = (T)0;
    // streamed over e (t_e computed when first needed, carried as t_{e-1})
    T tprev = x[0] - pxx;
    if (interior) {
#pragma unroll
      for (int e = 0; e < E; ++e) {
        const T xn = (e + 1 < E) ? x[(e + 1 < E) ? e + 1 : e] : nx;
        const T te = xn - x[e] * x[e];
        g[e] = gfma(x[e], gfma(b4, te, (T)-2), gfma(-b2, tprev, (T)2 * a));
        if (LOGP) {
          const T am = a - x[e];
          const T s = b * (te * te) + am * am;
          part = (e == 0) ? s : part + s;
        }
        tprev = te;
      }
    } else {
      // an opaque copy of D keeps the per-element factors from being hoisted
      // out of the leapfrog loop into 3*E loop-invariant registers
      int Dv = D;
      asm volatile("" : "+s"(Dv));
#pragma unroll
      for (int e = 0; e < E; ++e) {
        const int i = i0 + e;
        const bool hs = i <= Dv - 2, hp = (i >= 1) & (i <= Dv - 1);
        const T xn = (e + 1 < E) ? x[(e + 1 < E) ? e + 1 : e] : nx;
        const T te = xn - x[e] * x[e];
        g[e] = gfma(x[e], gfma(hs ? b4 : (T)0, te, hs ? (T)-2 : (T)0), gfma(hp ? -b2 : (T)0, tprev, hs ? (T)2 * a : (T)0));
        if (LOGP) {
          const T am = a - x[e];
          const T s = hs ? b * (te * te) + am * am : (T)0;
          part = (e == 0) ? s : part + s;
        }
        tprev = te;
      }
    }
    if (LOGP) return -block_sum(part, c);
    return (T)0;
  }
};

// IsotropicGaussian as a target (distributions.rs:398-406):
//   logp = (-0.5 * sum x^2) / (std*std),  g = (-x) / (std*std)
// The quotients are the IEEE ones, taken by div_by_const_q with the
// reciprocal computed once per kernel (bind), the division itself only in
// the branch for the fast form's excluded range.
template <class T> struct IsoGaussLane;
template <class T> struct IsoGaussT {
  T var;  // std*std
  int D;
  template <int LPC, int E> __host__ __device__ size_t lds_bytes() const { return 0; }
  template <int LPC, int E> __device__ __forceinline__ IsoGaussLane<T> bind(int) const;
};
template <class T> struct IsoGaussLane {
  T var;
  DivConst<T> dv;  // std*std, its reciprocal and the fast quotient's range
  int D;
  // g = (-x) / var for the coordinates i0 + e < D, +0 past D
  template <int E> __device__ __forceinline__ void grad(const T (&x)[E], T (&g)[E], int i0) const {
    bool bad = false;
#pragma unroll
    for (int e = 0; e < E; ++e) g[e] = (i0 + e < D) ? div_by_const_q(-x[e], dv, bad) : (T)0;
    if (__builtin_expect(bad, 0)) {
#pragma unroll
      for (int e = 0; e < E; ++e)
        if (i0 + e < D) g[e] = (-x[e]) / var;
    }
  }
  // this lane's sum of x^2 over its E slots. No mask for the padded slots:
  // every sampler keeps a padded coordinate at +0 (loaded as +0, its momentum
  // and gradient +0), and +0 * +0 = +0 added to a sum of squares (never -0)
  // changes no bit, so the sum is the masked one's.
  template <int E> __device__ __forceinline__ T sq_part(const T (&x)[E]) const {
    T part = x[0] * x[0];
#pragma unroll
    for (int e = 1; e < E; ++e) part = part + x[e] * x[e];
    return part;
  }
  __device__ __forceinline__ T quot(T a) const {
    bool bad = false;
    T q = div_by_const_q(a, dv, bad);
    if (__builtin_expect(bad, 0)) q = a / var;
    return q;
  }
  // unreduced term sum x^2 of this lane; logp = finish(group_sum(part))
  template <int LPC> static constexpr bool has_part = true;
  template <int LPC, int E>
  __device__ __forceinline__ T eval_part(const T (&x)[E], T (&g)[E], int lane) const {
    grad<E>(x, g, lane * E);
    return sq_part<E>(x);
  }
  __device__ __forceinline__ T finish(T total) const { return quot((T)-0.5 * total); }
  template <int LPC, int E, bool LOGP>
  __device__ __forceinline__ T eval(const T (&x)[E], T (&g)[E], int lane) const {
    grad<E>(x, g, lane * E);
    if (!LOGP) return (T)0;
    return quot((T)-0.5 * group_sum<LPC>(sq_part<E>(x)));
  }
  template <int E, bool LOGP>
  __device__ __forceinline__ T eval_wide(const T (&x)[E], T (&g)[E], WideCtx<T>& c) const {
    const int t0 = (c.w * 64 + c.lane) * E;
    grad<E>(x, g, t0);
    if (!LOGP) return (T)0;
    return quot((T)-0.5 * block_sum(sq_part<E>(x), c));
  }
};
template <class T>
template <int LPC, int E>
__device__ __forceinline__ IsoGaussLane<T> IsoGaussT<T>::bind(int) const {
  IsoGaussLane<T> r;
  r.var = var;
  r.dv = DivConst<T>::make(var);
  r.D = D;
  return r;
}

// Dense Gaussian (DiffableGaussian2D generalised, distributions.rs:257-292):
//   d = x - mu; w_k = sum_j P_kj d_j; logp = nc - 0.5*sum_k w_k d_k;
//   g = -w   (= -0.5 (P + P^T) d for symmetric P, the autodiff result)
// The product is an fma chain in ascending j, w = fma(P_kj, d_j, w) from
// w = 0 (the reference's matmul goes through ndarray/matrixmultiply, whose
// order and FMA use are its own; the oracle defines this one).
//
// The precision matrix is stored transposed (prec[j*D + i] = P_ij) so that
// lane i's column-j reads are consecutive across the chain's lanes. When it
// fits (use_lds, decided per layout by the launcher) bind() stages it once per
// block into LDS with a row stride of S = LPC*E (zero columns for i >= D, so
// no lane needs a bounds test), and each evaluation publishes d in a per-group
// LDS slot from which coordinate j is read as a broadcast: per column one LDS
// read of P and one broadcast read of d_j, no shuffles, no global loads.
//
// Matrix-core form (f64, 16 lanes x 2 coordinates per chain, D <= 32: NUTS
// cfg3's layout). A wave holds 4 chains; w = P [d_0 .. d_3] is a 32x32 by
// 32x4 product, 16 v_mfma_f64_4x4x4_4b_f64 (two output halves g x eight
// 4-column steps s). Measured on gfx950 (tools/probes/mfma_f64_probe.hip,
// profiles/r02/mfma/): the instruction's result is bit for bit the
// k-ascending fma chain from C, so accumulating s ascending from C = +0 is
// exactly the oracle's j-ascending chain (a product's two factors commute);
// lane l = 16r + 4b + q holds A[m=q][k=r], B[k=r][n=q] and C/D[m=r][n=q] of
// block b. The chains are the rows of the product: A = the 4 chains' d
// (A[m][k] = d_m[4s + k]) and B = P^T (B[k][n] of block b = P[8b + 2n + g]
// [4s + k]), so C/D[m][n] of block b lands on lane 16m + 4b + n, i.e. on
// chain m's own lane 4b + n as its coordinate 2(4b + n) + g = w[e = g]: the
// result needs no routing. A lane's A values are the d of chain l&3 at
// 4s + (l>>4), s = 0..7, read from a per-chain LDS slot where d is published
// transposed (slot [r][s] = d_{4s+r}: 64 contiguous bytes per lane). bind()
// stages B once per block in fragment order (lane l's 16 values as 8 16-byte
// pairs). All 64 lanes take part, so the form runs only with the whole wave
// active (a partial last wave, or a chain-divergent call such as the step
// size search, takes the global-memory VALU product: the same chain, so the
// same bits).
extern __shared__ __attribute__((aligned(16))) unsigned char gm_dyn_lds[];

// fused multiply-add, one rounding (the oracle's FMA)

#ifndef GM_GEMV_UNROLL
#define GM_GEMV_UNROLL 4  // columns of the LDS GEMV loop in flight per iteration
#endif
// matrix-core form: a chain's d slot in LDS, 16E doubles padded by 2 so that
// the 4 chains of a wave fall in different banks (16-byte aligned)
template <int E> __host__ __device__ constexpr int gm_mf_slot() { return 16 * E + 2; }
template <class T, int LPC, int E> struct GaussLane;
template <class T> struct GaussT {
  const T* mu;    // [D] device
  const T* prec;  // [D*D] device, transposed: prec[j*D + i] = P_ij
  T nc;
  int D;
  int use_lds = 0;
  // the matrix-core form applies to layout (LPC, E) (at D <= 16 E): f64, a
  // chain on one 16-lane row with 2 (D <= 32) or 4 (D <= 64) coordinates per lane
  template <int LPC, int E> __host__ __device__ static constexpr bool mfma_form() {
    return sizeof(T) == 8 && LPC == 16 && (E == 2 || E == 4);
  }
  // P's fragments: 4E K-steps x 64 lanes x E output groups (1024 doubles at E = 2)
  template <int E> __host__ __device__ static constexpr int mf_frag() { return 64 * 4 * E * E; }
  // dynamic LDS bytes a 256-thread block needs for layout (LPC, E)
  template <int LPC, int E> __host__ __device__ static size_t lds_need(int D) {
    if (mfma_form<LPC, E>() && D <= 16 * E)
      return ((size_t)mf_frag<E>() + (size_t)(256 / LPC) * gm_mf_slot<E>()) * sizeof(T);
    return ((size_t)D * LPC * E + (size_t)256 * E) * sizeof(T);
  }
  template <int LPC, int E> __host__ __device__ size_t lds_bytes() const {
    return use_lds ? lds_need<LPC, E>(D) : 0;
  }
  template <int LPC, int E> __device__ __forceinline__ GaussLane<T, LPC, E> bind(int lane) const {
    GaussLane<T, LPC, E> r;
    r.mu = mu;
#pragma unroll
    for (int e = 0; e < E; ++e) r.mur[e] = (lane * E + e < D) ? mu[lane * E + e] : (T)0;
    r.prec = prec;
    r.nc = nc;
    r.D = D;
    r.sprec = nullptr;
    r.sd = nullptr;
    r.mf = false;
    if constexpr (mfma_form<LPC, E>()) {
      if (use_lds && D <= 16 * E) {  // fragment order: k = (s * 64 + lane) * E + g
        T* sp = (T*)gm_dyn_lds;
        for (int k = threadIdx.x; k < mf_frag<E>(); k += blockDim.x) {
          const int l = (k / E) & 63, g = k % E, st = k / (64 * E);
          const int row = 4 * E * ((l >> 2) & 3) + E * (l & 3) + g, col = 4 * st + (l >> 4);
          sp[k] = (row < D && col < D) ? prec[(long long)col * D + row] : (T)0;
        }
        __syncthreads();
        r.sprec = sp;
        r.sd = sp + mf_frag<E>() + (threadIdx.x >> 4) * gm_mf_slot<E>();
        r.mf = true;
        return r;
      }
    }
    if (use_lds) {  // every thread of the block reaches bind() (kernels return after it)
      constexpr int S = LPC * E;
      T* sp = (T*)gm_dyn_lds;
      const int n = D * S;
      for (int k = threadIdx.x; k < n; k += blockDim.x) {
        const int j = k / S, i = k - j * S;
        sp[k] = (i < D) ? prec[(long long)j * D + i] : (T)0;
      }
      __syncthreads();
      r.sprec = sp;
      r.sd = sp + n + (threadIdx.x / LPC) * S;
    }
    return r;
  }
};
template <class T, int LPC, int E> struct GaussLane {
  const T* mu;
  T mur[E];  // this lane's mean coordinates (0 past D)
  const T* prec;
  T nc;
  int D;
  const T* sprec;  // LDS [D][S], or the matrix-core fragments (mf), or null
  T* sd;           // LDS slot of this lane group's d [S] (mf: transposed [4][8])
  bool mf;         // matrix-core form (see above)
#ifdef GM_NUTS_PROF
  mutable unsigned long long prof_prod = 0;  // measurement build: cycles in mfma_product
#endif
  // unreduced log-density term for callers that reduce it together with
  // another per-chain sum: logp = finish(group_sum(eval_part(...)))
  template <int LPC_> static constexpr bool has_part = true;
  template <int LPC_, int E_>
  __device__ __forceinline__ T eval_part(const T (&x)[E], T (&g)[E], int lane) const {
    return eval_impl<LPC_, E_, true>(x, g, lane);
  }
  __device__ __forceinline__ T finish(T total) const { return nc - total * (T)0.5; }
  template <int LPC_, int E_, bool LOGP>
  __device__ __forceinline__ T eval(const T (&x)[E], T (&g)[E], int lane) const {
    const T part = eval_impl<LPC_, E_, LOGP>(x, g, lane);
    if (LOGP) return finish(group_sum<LPC>(part));
    return (T)0;
  }
  // w = P d of the wave's 4 chains on the matrix cores (the form above)
  __device__ __forceinline__ void mfma_product(const T (&d)[E], T (&w)[E]) const {
    if constexpr (GaussT<T>::template mfma_form<LPC, E>()) {
      typedef double v2 __attribute__((ext_vector_type(2)));
      constexpr int KS = 4 * E;  // K-steps of 4 coordinates: D <= 16 E
      constexpr int SL = gm_mf_slot<E>();
#ifdef GM_NUTS_PROF
      const unsigned long long pt0 = __builtin_amdgcn_s_memtime();
#endif
      const int l = threadIdx.x & 63;
      const int wb = (threadIdx.x >> 6) * 4;  // the wave's first chain slot in the block
      // the previous evaluation's reads of the slots are done before they are replaced
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
#pragma unroll
      for (int e = 0; e < E; ++e) {
        const int j = (l & 15) * E + e;
        sd[(j & 3) * KS + (j >> 2)] = d[e];
      }
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      // A: chain l&3's d_{4s + (l>>4)}, s = 0..KS-1
      const T* at = sprec + GaussT<T>::template mf_frag<E>() + (wb + (l & 3)) * SL + (l >> 4) * KS;
      v2 dv[KS / 2];
#pragma unroll
      for (int t = 0; t < KS / 2; ++t) dv[t] = *(const v2*)(at + 2 * t);
      // D[m = l>>4][n = l&3] of block (l>>2)&3: chain l>>4's w at E(l&15) + g, this lane's w[g];
      // the E accumulations are independent chains, each in ascending s from +0
      double acc[E];
#pragma unroll
      for (int g = 0; g < E; ++g) acc[g] = 0.0;
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        const double a = dv[s >> 1][s & 1];
        const T* pb = sprec + (s * 64 + l) * E;
#pragma unroll
        for (int g = 0; g < E; g += 2) {
          const v2 pv = *(const v2*)(pb + g);
          acc[g] = __builtin_amdgcn_mfma_f64_4x4x4f64(a, pv[0], acc[g], 0, 0, 0);
          acc[g + 1] = __builtin_amdgcn_mfma_f64_4x4x4f64(a, pv[1], acc[g + 1], 0, 0, 0);
        }
      }
#pragma unroll
      for (int g = 0; g < E; ++g) w[g] = acc[g];
#ifdef GM_NUTS_PROF
      __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): the product's last read has landed
      prof_prod += __builtin_amdgcn_s_memtime() - pt0;
#endif
    }
  }
  template <int LPC_, int E_, bool LOGP>
  __device__ __forceinline__ T eval_impl(const T (&x)[E], T (&g)[E], int lane) const {
    // (a mask-free copy for chains that fill their lanes, chosen by a
    // wave-uniform branch, measured -15 % at cfg3: the duplicated evaluation,
    // profiles/r04/ab_nuts_maskfree_gauss_eval.log; not kept)
    static_assert(LPC_ == LPC && E_ == E, "layout mismatch");
    T d[E], w[E];
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const int i = lane * E + e;
      d[e] = (i < D) ? x[e] - mur[e] : (T)0;
    }
    bool done = false;
    if constexpr (GaussT<T>::template mfma_form<LPC, E>()) {
      if (mf && __builtin_amdgcn_read_exec() == ~0ull) {
        mfma_product(d, w);
        done = true;
      }
    }
    if (done) {
    } else if (sprec && !mf) {
      constexpr int S = LPC * E;
      // the previous evaluation's broadcast reads are done before d is replaced
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
#pragma unroll
      for (int e = 0; e < E; ++e) sd[lane * E + e] = d[e];
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      const T* pr = sprec + lane * E;
      // a lane's E entries of row j are contiguous and (E*sizeof(T))-aligned:
      // read them as 16-byte vectors where E allows (ds_read_b128, 4 LDS
      // cycles, instead of ds_read2_b64 pairs at 8)
      auto row = [&](int j, T (&pj)[E]) __attribute__((always_inline)) {
        if constexpr (E * sizeof(T) % 16 == 0) {
          typedef T v16 __attribute__((ext_vector_type(16 / sizeof(T))));
          constexpr int V = 16 / sizeof(T);
#pragma unroll
          for (int k = 0; k < E / V; ++k) {
            const v16 t = *(const v16*)(pr + j * S + k * V);
#pragma unroll
            for (int u = 0; u < V; ++u) pj[k * V + u] = t[u];
          }
        } else {
#pragma unroll
          for (int e = 0; e < E; ++e) pj[e] = pr[j * S + e];
        }
      };
#pragma unroll
      for (int e = 0; e < E; ++e) w[e] = (T)0;  // fma(p, d_0, +0): the chain's first term
      int j = 0;
      if constexpr (S % 2 == 0 && sizeof(T) == 8) {
        // column pairs: d_j, d_{j+1} in one 16-byte broadcast read
        typedef T v2 __attribute__((ext_vector_type(2)));
#pragma unroll GM_GEMV_UNROLL
        for (; j + 1 < D; j += 2) {
          const v2 dd = *(const v2*)(sd + j);
          T pj[E];
          row(j, pj);
#pragma unroll
          for (int e = 0; e < E; ++e) w[e] = gfma(pj[e], dd[0], w[e]);
          row(j + 1, pj);
#pragma unroll
          for (int e = 0; e < E; ++e) w[e] = gfma(pj[e], dd[1], w[e]);
        }
      }
#pragma unroll GM_GEMV_UNROLL
      for (; j < D; ++j) {
        const T dj = sd[j];
        T pj[E];
        row(j, pj);
#pragma unroll
        for (int e = 0; e < E; ++e) w[e] = gfma(pj[e], dj, w[e]);
      }
    } else {
      // Columns in batches of GU: the batch's global loads and lane
      // broadcasts are issued together; the accumulation stays in ascending j.
      constexpr int GU = 8;
      for (int j0 = 0; j0 < D; j0 += GU) {
        T pj[GU][E], dj[GU];
#pragma unroll
        for (int u = 0; u < GU; ++u) {
          const int j = (j0 + u < D) ? j0 + u : D - 1;
          // coordinate j lives in lane j/E, slot j%E of this chain's group
          const int src = j / E, slot = j % E;
          T mine = d[0];
#pragma unroll
          for (int e = 1; e < E; ++e) mine = (slot == e) ? d[e] : mine;
          if constexpr (LPC == 1) dj[u] = mine;
          else dj[u] = __shfl(mine, src, LPC);
#pragma unroll
          for (int e = 0; e < E; ++e) {
            const int i = lane * E + e;
            pj[u][e] = (i < D) ? prec[(long long)j * D + i] : (T)0;
          }
        }
#pragma unroll
        for (int u = 0; u < GU; ++u) {
          if (j0 + u < D) {
#pragma unroll
            for (int e = 0; e < E; ++e) w[e] = gfma(pj[u][e], dj[u], (j0 + u == 0) ? (T)0 : w[e]);
          }
        }
      }
    }
    T part = (T)0;
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const int i = lane * E + e;
      g[e] = (i < D) ? -w[e] : (T)0;
      if (LOGP) {
        const T s = (i < D) ? w[e] * d[e] : (T)0;
        part = (e == 0) ? s : part + s;
      }
    }
    return part;
  }
};

}  // namespace gm
