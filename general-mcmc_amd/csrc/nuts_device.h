// nuts_device.h — the NUTS transition kernel and its tree / metric helpers
// (device code only; compiled ahead of time by nuts_kernels.hip and at run
// time for user targets by gm_jit.cpp). See nuts_kernels.hip for the notes.
#pragma once
#include "gm_device.h"
#include "gm_launch.h"
#include "gm_track.h"

namespace gm {


// coordinate j of a chain's vector: lane j/E of the group, slot j%E
template <int LPC, int E, class T>
__device__ __forceinline__ T coord(const T (&x)[E], int j) {
  const int src = j / E, slot = j % E;
  T mine = x[0];
#pragma unroll
  for (int e = 1; e < E; ++e) mine = (slot == e) ? x[e] : mine;
  if constexpr (LPC == 1) return mine;
  else return __shfl(mine, src, LPC);
}

// MassMatrix (generic_nuts.rs:175-304) of one chain, this lane's view. K is
// the most general metric the kernel supports, known at compile time: 0 the
// identity only (a sampler without mass-matrix adaptation: no metric branch
// is emitted), 1 identity or diagonal (diagonal adaptation: no dense code),
// 2 any (dense adaptation), 3 every chain dense and the metric frozen for the
// launch (dense adaptation past its last warm-up window: no identity or
// diagonal branch, no Welford state; nuts_run picks it).
template <class T, int E, int K = 2> struct MassDev {
  static constexpr bool DENSE = K >= 2;
  int kind_ = 0;            // 0 identity, 1 diagonal, 2 dense
  T inv[E], sq[E];          // diagonal
  const T* minvT = nullptr;  // dense M^-1, transposed: minvT[j][i] = M^-1_ij (nuts_run)
  int minv_lds = 0;          // M^-1 resident in LDS: 1 packed (minv_packed_lds), 2 full; the chain's slot at lds_off
  unsigned lds_off = 0;
  const T* cholT = nullptr;  // its Cholesky factor L, transposed: cholT[j][i] = L_ij
  const T* cholR = nullptr;  // L row-major (cholR[i][j] = L_ij; the 16 x 2 start's rows)
  int chol_lds = 0;          // L resident in LDS, rows packed: the chain's slot at chol_off
  unsigned chol_off = 0;
  int D = 0;
  __device__ __forceinline__ int kind() const {
    if constexpr (K >= 3) return 2;
    else if constexpr (K > 0) return kind_;
    else return 0;
  }
};

// Dense M^-1 resident in LDS (layout 16 x 2, the matrix-core layout of cfg3).
// M^-1 is exactly symmetric (invert_spd_from_cholesky writes inv[i][j] and
// inv[j][i] from one sum), so a chain keeps only its lower triangle, rows
// packed: M^-1_ij at tri(max(i,j)) + min(i,j), tri(i) = i(i+1)/2, over the
// DP = LPC*E padded rows (zeros past D): 528 doubles = 4,224 B per chain at
// D = 32, so the 16 chains of a block take 67,584 B and two blocks per CU
// (2 waves per SIMD) still fit the 160 KiB next to the target's staging (the
// full matrices, 128 KiB per block, allowed one block per CU only and ran
// slower than re-reading them from L2/MALL). A lane's row r reads, for
// column j, tri(r) + j while j <= r and tri(j) + r after: one address select
// per element, its immediate offset 8j common to both forms. p_j reaches the
// chain's lanes by a DPP row broadcast (row_newbcast: a chain is one 16-lane
// DPP row), no LDS traffic. The sums are the global form's (j ascending from
// +0, separate multiply and add), so the bits are the oracle's.
__host__ __device__ constexpr int tri_n(int i) { return i * (i + 1) / 2; }
template <int LPC, int E, class T> __host__ __device__ constexpr size_t minv_packed_bytes() {
  return (size_t)tri_n(LPC * E) * sizeof(T);
}
// lane K of the 16-lane row: one v_mov_b64_dpp (row_newbcast is the one DPP
// control gfx950's 64-bit DPP moves take; every lane has a source, so the
// old value is never read)
template <int K> __device__ __forceinline__ double row_bcast(double v) {
  return __builtin_amdgcn_mov_dpp(v, 0x150 + K, 0xf, 0xf, false);
}
template <int K> __device__ __forceinline__ float row_bcast(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x150 + K, 0xf, 0xf,
                                                               false));
}
// coordinates J+K .. J+NB-1 of a 16-lane chain's vector (E per lane) into
// pj[K ..], each broadcast to the chain's lanes
template <int E, class T, int J, int K, int NB>
__device__ __forceinline__ void row_bcasts(const T (&p)[E], T (&pj)[NB]) {
  if constexpr (K < NB) {
    pj[K] = row_bcast<(J + K) / E>(p[(J + K) % E]);
    row_bcasts<E, T, J, K + 1, NB>(p, pj);
  }
}
// Columns [J, J + NB) of v = M^-1 p from the packed triangle: the batch's
// LDS reads and row broadcasts are issued first (a straight-line stretch the
// scheduler cannot reorder past the sched_barrier), then its sums in
// ascending j. No test j < D: the padded coordinates of p and the padded
// rows/columns of the triangle are exactly +0, and adding +0 leaves an
// accumulator that starts at +0 unchanged (it can never become -0: x + y
// rounds to -0 only when both are -0), so the padded columns change no bit.
// (PB columns per batch: 8 at one wave per SIMD, 4 in the frozen-dense
// kernel at two, where 8 cost 12 more spilled registers: measured 9.19e8 vs
// 9.58e8 leapfrogs/s at cfg3_dense, profiles/r05/ab_dense_batches.log; re-measured
// after the round-6 start pre-pass: 8 still -2 %, ab_nuts_dense_l1reg_pb8.log)
#ifndef GM_PACKED_BATCH
#define GM_PACKED_BATCH 8
#endif
#ifndef GM_FROZEN_PACKED_BATCH
#define GM_FROZEN_PACKED_BATCH 4
#endif
template <int LPC, int E, class T, int J, bool CHOL, int PB = GM_PACKED_BATCH>
__device__ __forceinline__ void packed_cols(const unsigned (&aA)[E], const unsigned (&aB)[E], const int (&r)[E],
                                            const T (&p)[E], T (&acc)[E]) {
  constexpr int NB = PB < LPC * E - J ? PB : LPC * E - J;
  if constexpr (NB > 0) {
    T m[NB][E], pj[NB];
#pragma unroll
    for (int u = 0; u < NB; ++u) {
      const int j = J + u;
#pragma unroll
      for (int e = 0; e < E; ++e) {
        unsigned ad;
        if constexpr (CHOL)  // L: row r's entries j <= r are contiguous; j > r is +-0 (below)
          ad = aA[e] + (unsigned)(((j <= r[e]) ? j : 0) * (int)sizeof(T));
        else  // M^-1: tri(r) + j while j <= r, tri(j) + r after
          ad = (j <= r[e]) ? aA[e] + (unsigned)(j * (int)sizeof(T))
                           : aB[e] + (unsigned)(tri_n(j) * (int)sizeof(T));
        m[u][e] = *(const T*)(gm_dyn_lds + ad);
      }
    }
    row_bcasts<E, T, J, 0, NB>(p, pj);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int u = 0; u < NB; ++u) {
#pragma unroll
      for (int e = 0; e < E; ++e) {
        // p = L z skips the terms j > r (L_rj = 0); adding 0 * z_j = +-0 to
        // the +0-started sum changes no bit either
        const T mm = (CHOL && J + u > r[e]) ? (T)0 : m[u][e];
        if constexpr (CHOL) acc[e] = acc[e] + mm * pj[u];
        else acc[e] = gfma(mm, pj[u], acc[e]);  // M^-1 p: the engine's fma chain (oracle inv_mul)
      }
    }
    packed_cols<LPC, E, T, J + NB, CHOL, PB>(aA, aB, r, p, acc);
  }
}

// Columns [J, J + NB) of v = M^-1 p from the full matrix in LDS (minv_lds
// == 2, the one-block-per-CU budget: 8 KiB per chain at D = 32), stored
// [j][i] so that a lane's two entries of column j are one 16-byte read at an
// immediate offset: no address arithmetic. Same sums and +0 padding as above.
template <int LPC, int E, class T, int J>
__device__ __forceinline__ void full_cols(unsigned base, const T (&p)[E], T (&acc)[E]) {
  constexpr int DP = LPC * E;
  constexpr int NB = GM_PACKED_BATCH < DP - J ? GM_PACKED_BATCH : DP - J;
  if constexpr (NB > 0) {
    typedef T vE __attribute__((ext_vector_type(E)));
    vE m[NB];
    T pj[NB];
#pragma unroll
    for (int u = 0; u < NB; ++u) m[u] = *(const vE*)(gm_dyn_lds + base + (J + u) * DP * sizeof(T));
    row_bcasts<E, T, J, 0, NB>(p, pj);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int u = 0; u < NB; ++u) {
#pragma unroll
      for (int e = 0; e < E; ++e) acc[e] = gfma(m[u][e], pj[u], acc[e]);
    }
    full_cols<LPC, E, T, J + NB>(base, p, acc);
  }
}

// Columns [J, J + NB) of p = L z from the global factor when it is not
// resident in LDS: each lane reads its own rows of the row-major L (pb[e] =
// row r, clamped to a valid row; column j at the immediate offset 8j, so no
// address arithmetic and no hoisted column offsets -- the transposed form's
// j*D offsets were kept in spilled scalars; the buffer has D elements of
// slack past the last row for the padded columns j >= D of a D < 32 chain).
// The batch's loads and row broadcasts first, then the sums in ascending j.
// Terms with j > i (L_ij = 0 there, and every padded column), padded rows
// (i >= D) and padded coordinates (z_j = +0) add +-0 to the +0-started sum:
// no bit changes, as in packed_cols.
#ifndef GM_CHOL_BATCH
#define GM_CHOL_BATCH 8
#endif
template <int LPC, int E, class T, int J>
__device__ __forceinline__ void chol_global_cols(const T* const (&pb)[E], int D, const int (&r)[E],
                                                 const T (&z)[E], T (&acc)[E]) {
  constexpr int DP = LPC * E;
  constexpr int NB = GM_CHOL_BATCH < DP - J ? GM_CHOL_BATCH : DP - J;
  if constexpr (NB > 0) {
    T m[NB][E], zj[NB];
#pragma unroll
    for (int u = 0; u < NB; ++u) {
#pragma unroll
      for (int e = 0; e < E; ++e) m[u][e] = pb[e][J + u];
    }
    row_bcasts<E, T, J, 0, NB>(z, zj);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int u = 0; u < NB; ++u) {
#pragma unroll
      for (int e = 0; e < E; ++e) {
        const T mm = (J + u > r[e] || r[e] >= D) ? (T)0 : m[u][e];
        acc[e] = acc[e] + mm * zj[u];
      }
    }
    chol_global_cols<LPC, E, T, J + NB>(pb, D, r, z, acc);
  }
}

// columns per batch of the dense products (their loads / broadcasts issued
// together; the sums stay in ascending j). 4 keeps the dense-metric kernel
// within 256 registers (2 waves per SIMD; 8 took it to 276 and 1 wave).
#ifndef GM_DENSE_BATCH
#define GM_DENSE_BATCH 4
#endif

// inv_mul (:255-273): v = M^-1 p
template <int LPC, int E, class T, int K>
__device__ __forceinline__ void inv_mul(const MassDev<T, E, K>& M, const T (&p)[E], T (&v)[E], int lane) {
  if (M.kind() == 1) {
#pragma unroll
    for (int e = 0; e < E; ++e) v[e] = M.inv[e] * p[e];
  } else if (MassDev<T, E, K>::DENSE && M.kind() == 2) {
    T acc[E];
#pragma unroll
    for (int e = 0; e < E; ++e) acc[e] = (T)0;
    if constexpr (LPC == 16 && E == 2) {
      // (the frozen-dense kernel's plan is the packed triangle or global
      // memory: its 2 blocks per CU leave no room for the full form)
      if (K != 3 && M.minv_lds == 2) {
        // (software-pipelining the batches, batch J+1's reads and broadcasts
        // issued before batch J's sums, measured -1 % / -5 % at 4 / 8
        // columns per batch, profiles/r04/ab_dense_pipe.log: not kept)
        full_cols<LPC, E, T, 0>(M.lds_off + (unsigned)(lane * E * (int)sizeof(T)), p, acc);
#pragma unroll
        for (int e = 0; e < E; ++e) v[e] = acc[e];
        return;
      }
      if (M.minv_lds) {
        unsigned aA[E], aB[E];
        int r[E];
#pragma unroll
        for (int e = 0; e < E; ++e) {
          r[e] = lane * E + e;
          aA[e] = M.lds_off + (unsigned)(tri_n(r[e]) * (int)sizeof(T));
          aB[e] = M.lds_off + (unsigned)(r[e] * (int)sizeof(T));
          // opaque bases: otherwise the compiler hoists the 2 x 32 column
          // addresses of every inlined product out of the main loop and, at
          // 256 registers, spills them (215 scratch reloads per iteration)
          __asm__ volatile("" : "+v"(aA[e]), "+v"(aB[e]), "+v"(r[e]));
        }
        packed_cols<LPC, E, T, 0, false, K == 3 ? GM_FROZEN_PACKED_BATCH : GM_PACKED_BATCH>(aA, aB, r, p, acc);
#pragma unroll
        for (int e = 0; e < E; ++e) v[e] = acc[e];
        return;
      }
    }
    // columns in batches of 8: a batch's loads and broadcasts are issued
    // together (a runtime-trip loop around the shuffles is not unrolled by the
    // compiler); the sums stay in ascending j
    constexpr int GB = GM_DENSE_BATCH;
    for (int j0 = 0; j0 < M.D; j0 += GB) {
      T mv[GB][E], pv[GB];
#pragma unroll
      for (int u = 0; u < GB; ++u) {
        const int j = (j0 + u < M.D) ? j0 + u : M.D - 1;
        pv[u] = coord<LPC, E>(p, j);
#pragma unroll
        for (int e = 0; e < E; ++e) {
          const int i = lane * E + e;
          mv[u][e] = (i < M.D) ? M.minvT[(long long)j * M.D + i] : (T)0;
        }
      }
#pragma unroll
      for (int u = 0; u < GB; ++u) {
        if (j0 + u < M.D) {
#pragma unroll
          for (int e = 0; e < E; ++e)
            if (lane * E + e < M.D) acc[e] = gfma(mv[u][e], pv[u], acc[e]);
        }
      }
    }
#pragma unroll
    for (int e = 0; e < E; ++e) v[e] = acc[e];
  } else {
#pragma unroll
    for (int e = 0; e < E; ++e) v[e] = p[e];
  }
}

// sample_momentum (:275-303) applied to standard normals z
template <int LPC, int E, class T, int K>
__device__ __forceinline__ void momentum_from(const MassDev<T, E, K>& M, const T (&z)[E], T (&p)[E], int lane) {
  if (M.kind() == 1) {
#pragma unroll
    for (int e = 0; e < E; ++e) p[e] = z[e] * M.sq[e];
  } else if (MassDev<T, E, K>::DENSE && M.kind() == 2) {
    T acc[E];
#pragma unroll
    for (int e = 0; e < E; ++e) acc[e] = (T)0;
    if constexpr (LPC == 16 && E == 2) {
      if (K != 3 && M.chol_lds) {  // (never in the frozen-dense plan)
        unsigned aA[E];
        int r[E];
#pragma unroll
        for (int e = 0; e < E; ++e) {
          r[e] = lane * E + e;
          aA[e] = M.chol_off + (unsigned)(tri_n(r[e]) * (int)sizeof(T));
          __asm__ volatile("" : "+v"(aA[e]), "+v"(r[e]));  // (as in inv_mul: not hoisted)
        }
        packed_cols<LPC, E, T, 0, true>(aA, aA, r, z, acc);
#pragma unroll
        for (int e = 0; e < E; ++e) p[e] = acc[e];
        return;
      }
#ifndef GM_CHOL_LOOP
      {
        int r[E];
        const T* pb[E];  // row r's entries (clamped to a valid row); opaque, so
                         // the column addresses are not hoisted out of the loop
#pragma unroll
        for (int e = 0; e < E; ++e) {
          r[e] = lane * E + e;
          pb[e] = M.cholR + (long long)(r[e] < M.D ? r[e] : M.D - 1) * M.D;
          // opaque: else the 2 x 32 masks (j > r) are hoisted and spilled
          __asm__ volatile("" : "+v"(pb[e]), "+v"(r[e]));
        }
        chol_global_cols<LPC, E, T, 0>(pb, M.D, r, z, acc);
#pragma unroll
        for (int e = 0; e < E; ++e) p[e] = acc[e];
        return;
      }
#endif
    }
    constexpr int GB = GM_DENSE_BATCH;
    for (int j0 = 0; j0 < M.D; j0 += GB) {  // batches of GB columns, as inv_mul
      T mv[GB][E], zv[GB];
#pragma unroll
      for (int u = 0; u < GB; ++u) {
        const int j = (j0 + u < M.D) ? j0 + u : M.D - 1;
        zv[u] = coord<LPC, E>(z, j);
#pragma unroll
        for (int e = 0; e < E; ++e) {
          const int i = lane * E + e;
          mv[u][e] = (i < M.D) ? M.cholT[(long long)j * M.D + i] : (T)0;
        }
      }
#pragma unroll
      for (int u = 0; u < GB; ++u) {
        const int j = j0 + u;
        if (j < M.D) {
#pragma unroll
          for (int e = 0; e < E; ++e) {
            const int i = lane * E + e;
            if (i < M.D && j <= i) acc[e] = acc[e] + mv[u][e] * zv[u];
          }
        }
      }
    }
#pragma unroll
    for (int e = 0; e < E; ++e) p[e] = acc[e];
  } else {
#pragma unroll
    for (int e = 0; e < E; ++e) p[e] = z[e];
  }
}

template <int LPC, int E, class T>
__device__ __forceinline__ T dot_group(const T (&a)[E], const T (&b)[E]) {
  T part = a[0] * b[0];
#pragma unroll
  for (int e = 1; e < E; ++e) part = part + a[e] * b[e];
  return group_sum<LPC>(part);
}

// MassMatrix::kinetic, identity (generic_nuts.rs:230-238): 0.5 * sum p^2
template <int LPC, int E, class T>
__device__ __forceinline__ T kinetic(const T (&p)[E]) {
  return (T)0.5 * dot_group<LPC, E>(p, p);
}

// leapfrog_with_mass, identity (generic_nuts.rs:1396-1418)
template <int LPC, int E, class T, class TG>
__device__ __forceinline__ T leapfrog(const TG& tg, T (&q)[E], T (&p)[E], T (&g)[E], T epsv, int lane) {
  const T h = epsv * (T)0.5;
#pragma unroll
  for (int e = 0; e < E; ++e) p[e] = p[e] + g[e] * h;
#pragma unroll
  for (int e = 0; e < E; ++e) q[e] = q[e] + p[e] * epsv;
  const T lp = tg.template eval<LPC, E, true>(q, g, lane);
#pragma unroll
  for (int e = 0; e < E; ++e) p[e] = p[e] + g[e] * h;
  return lp;
}

// stop_criterion (generic_nuts.rs:1354-1378), identity mass:
// (q+ - q-) . p- >= 0  and  (q+ - q-) . p+ >= 0
template <int LPC, int E, class T>
__device__ __forceinline__ bool no_uturn(const T (&qm)[E], const T (&qp)[E], const T (&pm)[E],
                                         const T (&pp)[E]) {
  T d[E];
#pragma unroll
  for (int e = 0; e < E; ++e) d[e] = qp[e] - qm[e];
  // dot_group(d, pm), dot_group(d, pp), their reductions interleaved
  T dd[2];
  dd[0] = d[0] * pm[0];
  dd[1] = d[0] * pp[0];
#pragma unroll
  for (int e = 1; e < E; ++e) {
    dd[0] = dd[0] + d[e] * pm[e];
    dd[1] = dd[1] + d[e] * pp[e];
  }
  group_sum_n<LPC>(dd);
  return dd[0] >= (T)0 && dd[1] >= (T)0;
}

// MassMatrix::kinetic (:226-253), canonical-order sum of the per-coordinate
// terms p*p*inv (diagonal) or p_i (M^-1 p)_i (dense)
template <int LPC, int E, class T, int K>
__device__ __forceinline__ T kinetic_m(const MassDev<T, E, K>& M, const T (&p)[E], int lane) {
  if (M.kind() == 0) return kinetic<LPC, E>(p);
  T t[E];
  if (M.kind() == 1) {
#pragma unroll
    for (int e = 0; e < E; ++e) t[e] = p[e] * p[e] * M.inv[e];
  } else {
    inv_mul<LPC, E>(M, p, t, lane);
#pragma unroll
    for (int e = 0; e < E; ++e) t[e] = p[e] * t[e];
  }
  T part = t[0];
#pragma unroll
  for (int e = 1; e < E; ++e) part = part + t[e];
  return (T)0.5 * group_sum<LPC>(part);
}

// leapfrog_with_mass (:1396-1418): drift by M^-1 p
template <int LPC, int E, class T, class TG, int K>
__device__ __forceinline__ T leapfrog_m(const TG& tg, const MassDev<T, E, K>& M, T (&q)[E], T (&p)[E],
                                        T (&g)[E], T epsv, int lane) {
  if (M.kind() == 0) return leapfrog<LPC, E>(tg, q, p, g, epsv, lane);
  const T h = epsv * (T)0.5;
#pragma unroll
  for (int e = 0; e < E; ++e) p[e] = p[e] + g[e] * h;
  T v[E];
  inv_mul<LPC, E>(M, p, v, lane);
#pragma unroll
  for (int e = 0; e < E; ++e) q[e] = q[e] + v[e] * epsv;
  const T lp = tg.template eval<LPC, E, true>(q, g, lane);
#pragma unroll
  for (int e = 0; e < E; ++e) p[e] = p[e] + g[e] * h;
  return lp;
}

// Unreduced per-lane term of MassMatrix::kinetic (:226-253) without the
// 0.5: sum_e p_e^2 (identity), p_e^2 inv_e (diagonal), p_e (M^-1 p)_e
// (dense); kinetic = 0.5 * group_sum(part), the operations of kinetic_m.
template <int LPC, int E, class T, int K>
__device__ __forceinline__ T kin_part_m(const MassDev<T, E, K>& M, const T (&p)[E], int lane) {
  T t[E];
  if (M.kind() == 0) {
#pragma unroll
    for (int e = 0; e < E; ++e) t[e] = p[e] * p[e];
  } else if (M.kind() == 1) {
#pragma unroll
    for (int e = 0; e < E; ++e) t[e] = p[e] * p[e] * M.inv[e];
  } else {
    inv_mul<LPC, E>(M, p, t, lane);
#pragma unroll
    for (int e = 0; e < E; ++e) t[e] = p[e] * t[e];
  }
  T part = t[0];
#pragma unroll
  for (int e = 1; e < E; ++e) part = part + t[e];
  return part;
}

// stop_criterion_with_mass (:1354-1378), the top-level U-turn
template <int LPC, int E, class T, int K>
__device__ __forceinline__ bool no_uturn_m(const MassDev<T, E, K>& M, const T (&qm)[E], const T (&qp)[E],
                                           const T (&pm)[E], const T (&pp)[E], int lane) {
  if (M.kind() == 0) return no_uturn<LPC, E>(qm, qp, pm, pp);
  T d[E], vm[E], vp[E];
#pragma unroll
  for (int e = 0; e < E; ++e) d[e] = qp[e] - qm[e];
  // (the two products fused, one LDS read of each column for both: -2 %,
  // profiles/r04/ab_dense_uturn_pair.log, not kept)
  inv_mul<LPC, E>(M, pm, vm, lane);
  inv_mul<LPC, E>(M, pp, vp, lane);
  const T dm = dot_group<LPC, E>(d, vm);
  const T dp = dot_group<LPC, E>(d, vp);
  return dm >= (T)0 && dp >= (T)0;
}

// The same two criteria from the trajectory's ends without ordering them: x
// the end on side v (being integrated) and o the other one. The minus-to-plus
// difference is q+ - q- = v (x_q - o_q), exactly (IEEE subtraction is
// antisymmetric up to the sign of a zero), so each per-lane product and every
// stage of the group sum is the negation of the ordered form's when v < 0:
// the sums differ at most in the sign of a zero, which `>= 0` does not see,
// and NaN fails either way. The two tests ((q+ - q-).p- and .p+) are the
// pair {S_o, S_x} in some order, and both must hold. So the decision is the
// ordered form's bit for bit, without the 4E selects that ordered the ends.
template <int LPC, int E, class T>
__device__ __forceinline__ bool no_uturn_ends(const T (&xq)[E], const T (&oq)[E], const T (&xp)[E],
                                              const T (&op)[E], int v) {
  T d[E];
#pragma unroll
  for (int e = 0; e < E; ++e) d[e] = xq[e] - oq[e];
  T dd[2];
  dd[0] = d[0] * op[0];
  dd[1] = d[0] * xp[0];
#pragma unroll
  for (int e = 1; e < E; ++e) {
    dd[0] = dd[0] + d[e] * op[e];
    dd[1] = dd[1] + d[e] * xp[e];
  }
  group_sum_n<LPC>(dd);
  const T sv = (T)v;
  return sv * dd[0] >= (T)0 && sv * dd[1] >= (T)0;
}
template <int LPC, int E, class T, int K>
__device__ __forceinline__ bool no_uturn_ends_m(const MassDev<T, E, K>& M, const T (&xq)[E], const T (&oq)[E],
                                                const T (&xp)[E], const T (&op)[E], int v, int lane) {
  if (M.kind() == 0) return no_uturn_ends<LPC, E>(xq, oq, xp, op, v);
  T d[E], vo[E], vx[E];
#pragma unroll
  for (int e = 0; e < E; ++e) d[e] = xq[e] - oq[e];
  inv_mul<LPC, E>(M, op, vo, lane);
  inv_mul<LPC, E>(M, xp, vx, lane);
  const T so = dot_group<LPC, E>(d, vo);
  const T sx = dot_group<LPC, E>(d, vx);
  const T sv = (T)v;
  return sv * so >= (T)0 && sv * sx >= (T)0;
}

template <int LPC, class T>
__device__ __forceinline__ bool all_finite(const T (&x)[1]) { return true; }

template <int LPC, int E, class T>
__device__ __forceinline__ bool group_all_finite(const T (&x)[E], int lane, int D) {
  int bad = 0;
#pragma unroll
  for (int e = 0; e < E; ++e) {
    const int i = lane * E + e;
    const T v = x[e];
    if (i < D && !(v - v == (T)0)) bad = 1;  // inf - inf and NaN - NaN are NaN
  }
  return group_sum<LPC>(bad) == 0;
}

template <class T> __device__ __forceinline__ T rust_min1(T x) {  // T::one().min(x): NaN -> 1
  return (x != x) ? (T)1 : (x < (T)1 ? x : (T)1);
}

// u < RN(a / b) for exact non-negative integers a <= b (b >= 1) held in T
// and a draw u = k 2^-P (k < 2^P; P = 53 for double, 24 for float: nuts_u),
// without the IEEE division on the common path. w = RN(u b) is within
// 2^-P u b of the exact product, so when d = w - a is farther than a 2^-(P-4)
// from 0 its sign is that of u b - a, i.e. of u - a/b; and then u and a/b lie
// on the same side of RN(a/b) too (|RN(a/b) - a/b| <= 2^-P a/b), so
// u < RN(a/b) exactly when d < 0. Inside that band (u within ~2^-(P-5)
// relative of a/b, or a = 0 with u b tiny) the quotient itself decides, in a
// branch that a wave takes about once per 2^15 merges. Bitwise the
// decision u < (T)a / (T)b (generic_nuts.rs:1305-1306, 860-861).
template <class T> __device__ __forceinline__ bool draw_below_ratio(T u, T a, T b) {
  constexpr T rel = sizeof(T) == 8 ? (T)0x1p-49 : (T)0x1p-20f;
  const T d = u * b - a;
  const T m = a * rel;
  if (__builtin_expect(d < -m, 1)) return true;
  if (__builtin_expect(d > m, 1)) return false;
  return u < a / b;
}

template <class T> struct MachEps;
template <> struct MachEps<float> { static constexpr float v = 1.1920928955078125e-07f; };
template <> struct MachEps<double> { static constexpr double v = 2.220446049250313e-16; };

// find_reasonable_epsilon_with_mass (generic_nuts.rs:1025-1102), identity mass.
// (not inlined: called once per launch at most, it would otherwise put its
// leapfrog loops and their registers into the hot tree loop's code). One
// copy per kernel instantiation (TAG = the kernel's MASS): an out-of-line
// function shared by kernels of different launch bounds is compiled once,
// and its registers then count against the most demanding caller's budget.
template <int LPC, int E, class T, class TG, int TAG = 0>
__device__ __attribute__((noinline)) T find_reasonable_epsilon(const TG& tg, const T (&q0)[E], const T (&p0)[E], int lane, int D) {
  const T half = (T)0.5;
  T eps = (T)1;
  T g0[E];
  const T ulogp = tg.template eval<LPC, E, true>(q0, g0, lane);
  T q[E], p[E], g[E];
#pragma unroll
  for (int e = 0; e < E; ++e) { q[e] = q0[e]; p[e] = p0[e]; g[e] = g0[e]; }
  T ulogp1 = leapfrog<LPC, E>(tg, q, p, g, eps, lane);
  T k = (T)1;
  for (int it = 0; it < 1100; ++it) {  // bounded: k underflows to 0 long before
    const bool fin = (ulogp1 - ulogp1 == (T)0) && group_all_finite<LPC, E>(g, lane, D);
    if (fin) break;
    k = k * half;
#pragma unroll
    for (int e = 0; e < E; ++e) { q[e] = q0[e]; p[e] = p0[e]; g[e] = g0[e]; }
    ulogp1 = leapfrog<LPC, E>(tg, q, p, g, eps * k, lane);
  }
  eps = half * k * eps;
  const T k0 = kinetic<LPC, E>(p0);
  T la = ulogp1 - ulogp - (kinetic<LPC, E>(p) - k0);
  const T a = (la > glog(half)) ? (T)1 : (T)-1;
  const T ln2 = glog((T)2);
  for (int it = 0; it < 2200; ++it) {  // bounded (the reference is not)
    if (!(a * la > -a * ln2)) break;
    eps = eps * (a > (T)0 ? (T)2 : (T)0.5);  // 2^a, a = +-1
#pragma unroll
    for (int e = 0; e < E; ++e) { q[e] = q0[e]; p[e] = p0[e]; g[e] = g0[e]; }
    ulogp1 = leapfrog<LPC, E>(tg, q, p, g, eps, lane);
    la = ulogp1 - ulogp - (kinetic<LPC, E>(p) - k0);
  }
  return eps;
}


// ---------------------------------------------------------------------------
// nuts_kernel: every chain's NUTS transitions, lockstep by leaf.
//
// Each iteration of the main loop performs ONE target evaluation for every
// chain of the wave: the next leaf's leapfrog for a chain inside its tree, or
// the evaluation at q that starts a transition (generic_nuts.rs:758-768) for
// a chain that finished its previous one. Chains therefore do not wait for
// the deepest tree of their wave at every transition: a wave runs until its
// chains have each done n_steps transitions, and only the per-leaf merge
// climb, the end of a doubling and the end of a transition diverge.
//
// The tree (build_tree_with_mass, generic_nuts.rs:1153-1341) is evaluated
// iteratively: leaves in trajectory order; a leaf then climbs the levels of
// its doubling, merging with the stored left sibling of every level where it
// completes a right child (the recursion's post-order, so the merge draws are
// the recursion's) and storing itself where it is a left child. A truncated
// subtree (s' = false) climbs without storing (its parent builds no right
// half) and ends the doubling. The trajectory ends live in registers as the
// edge (the end being integrated, side v) and the far end; a direction change
// swaps them.
#ifdef GM_NUTS_PROF
// Measurement build only (tools/ab_variants.sh nprof "-DGM_NUTS_PROF"): per
// wave, the shader cycles of each lockstep iteration binned by what the
// wave's chains did in it (bit 0 a transition start, 1 a subtree merge,
// 2 a doubling end, 3 a transition end) plus the evaluation's share;
// read back by gm_nuts_prof_read (nuts_kernels.hip).
// slots 35..42: cycles of the iteration's segments (see GM_PSEG below)
constexpr int NPROF_SLOTS = 16 * 2 + 3 + 8;
constexpr int NPROF_WAVES = 8192;
__device__ unsigned long long gm_nuts_prof_buf[NPROF_WAVES * NPROF_SLOTS];
#endif

// Launch bound: 2 blocks (2 waves per SIMD) per CU, 256 registers per lane,
// for up to 8 f32 or 2 f64 coordinates per lane (cfg3's 16x2 measured
// fastest there, profiles/r03/ab/nuts_layouts.jsonl); 1 (512 registers) for
// the dense-metric instantiation (at 256 it spilled ~500 B per lane to
// scratch inside the loop, measured 2.1e8 leapfrogs/s at cfg3) and for
// wider lanes, whose dozen per-lane state arrays of E values each spill at
// 256 (tools/kernel_resources.py over the build's resource remarks,
// profiles/r04/nuts_resources.txt). Measured at 2048 chains, IsotropicGaussian
// (tools/probe_nuts_highdim.py, profiles/r04/nuts_highdim.jsonl): 1 wave per
// SIMD f64 64x4 +4 %, 64x8 +78 %, 64x16 +150 %, f32 64x16 +55 %, but f32
// 64x4 -6 % and 64x8 -4 %, which therefore keep 2.
//
// Wide chains (LPC > 64; D > 256, identity or diagonal metric, targets with
// a cross-wave evaluation): one chain per workgroup of LPC/64 waves, every
// per-chain sum a block reduction (group_sum), so that the chain's state
// fits the registers without spills (64 x 8 / 64 x 16 f64 spilled 77-1268
// registers, profiles/r04/nuts_resources.txt); nuts_wide_waves (gm_launch.h)
// waves per SIMD for them.
template <class T, int LPC, int E, class TG, int MASS>
__global__ __launch_bounds__(LPC > 256 ? LPC : 256,
                             MASS == 2 ? GM_DENSE_WAVES : MASS == 3 ? GM_FROZEN_WAVES
                             : LPC > 64 ? nuts_wide_waves((int)sizeof(T), E)
                             : (E * (int)sizeof(T) > 32 || (sizeof(T) == 8 && E > 2)) ? 1 : 2)
void nuts_kernel(NutsLaunch a, TG tg_) {
  const long long gtid = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long c = gtid / LPC;
  const int lane = (int)(gtid % LPC);
  // f64: the leaf's exp table (leaf_alpha_tab), 512 B of static LDS inside
  // the 1 KiB per block that nuts_size_lds leaves beside the dynamic plan;
  // filled by the whole block before any thread returns
  __shared__ double exp_lds[sizeof(T) == 8 ? 64 : 1];
  if constexpr (sizeof(T) == 8) {
    exp64_lds_fill(exp_lds);
    __syncthreads();
  }
  const auto tg = tg_.template bind<LPC, E>(lane);  // per-lane target view
  if (c >= a.C) return;
  const int D = a.D;
  const long long C = a.C;
  const uint32_t cid = a.chain_offset + (uint32_t)c;
  T* __restrict__ qs = (T*)a.q;
  // Subtree stack. Level k < KL: LDS, vectors [k][field][thread*E + e] of
  // this block, scalars [k][chain in block] (every lane of a chain writes the
  // same value); a lane reads back only what it or its group wrote, so no
  // synchronisation. Deeper levels: HBM, one entry of a.stk_es bytes per
  // (chain, level), the chain's entries contiguous: vectors [field][coord],
  // then alpha, n, n_alpha: a merge's reads are one stretch of cache lines
  // (the scalars in three [level][chain] arrays cost three more lines per
  // merge: the frozen-dense kernel, whose levels >= 1 are all in HBM, +5 %,
  // profiles/r06/ab_nuts_stack_slab.log).
  char* __restrict__ sbase = (char*)a.stk_vec + c * (long long)a.max_depth * a.stk_es;
  // threads per block (nuts_part.inc): 256, or one chain's LPC > 64
  constexpr int NT = LPC > 64 ? LPC : 256;
  constexpr int CPB = NT / LPC;
  const int KL = a.lds_levels;
  T* __restrict__ lvec = (T*)(gm_dyn_lds + a.lds_stack_off);
  T* __restrict__ lalpha = lvec + (long long)KL * 3 * NT * E;
  int* __restrict__ lnn = (int*)(lalpha + KL * CPB);
  int* __restrict__ lnna = lnn + KL * CPB;
  const int tix = threadIdx.x;
  const int cib = tix / LPC;  // chain in block
  // Level 0 of the stack in registers (GM_L0REG): level 0 is half of all
  // stack traffic -- an even leaf stores itself there and the next leaf
  // merges with it one iteration later -- and an LDS (or, in the frozen-dense
  // kernel, whose packed M^-1 fills the LDS, an HBM) round trip on the
  // merge's critical path. A level-0 entry is a single leaf: its proposal is
  // its first q, so q and p are kept (8 registers at 16 x 2 f64) and field 2
  // reads field 0. Measured: cfg3 3.12e9 -> 3.31e9, cfg3_dense 9.75e8 ->
  // 1.04e9 leapfrogs/s (profiles/r05/ab_*_l0_registers.log).
#ifndef GM_L0REG
#define GM_L0REG 1
#endif
  // (not on the wide layouts: 512 x 2 Rosenbrock would spill 16 registers,
  // and their one-chain blocks keep level 0 in LDS)
  constexpr bool L0REG = GM_L0REG && LPC <= 64;
  T l0q[E], l0p[E], l0a = (T)0;
  int l0n = 0, l0na = 0;
#pragma unroll
  for (int e = 0; e < E; ++e) l0q[e] = l0p[e] = (T)0;
  // Level 1 in registers as well in the frozen-dense kernel (12 more, three
  // vectors and the scalars): its stack levels are otherwise all in global
  // memory, and level 1 is half of their traffic. With the start's products
  // in the pre-pass the kernel spills 64 registers instead of 28 and runs
  // 0.3-1.8 % faster (3 of 3 alternating rounds, 1.321e9 -> 1.334e9 median,
  // profiles/r06/ab_nuts_dense_l1reg_pb8.log; before the pre-pass it spilled
  // 60 and ran 5 % slower, profiles/r05/ab_dense_l1_registers.log). Level 2
  // in registers too: 63 spills, -7 % (1.332e9 -> 1.236e9 median of 4,
  // profiles/r06/ab_nuts_dense_l2reg.log).
#ifndef GM_L1REG_FROZEN
#define GM_L1REG_FROZEN 1
#endif
  constexpr bool L1R = GM_L1REG_FROZEN && MASS == 3 && L0REG;
  T l1q[E], l1p[E], l1r[E], l1a = (T)0;
  int l1n = 0, l1na = 0;
#pragma unroll
  for (int e = 0; e < E; ++e) l1q[e] = l1p[e] = l1r[e] = (T)0;
  // (level 1 in registers in cfg3's identity kernel: it reached 256 and ran
  // 13 % slower, profiles/r05/ab_cfg3_l1_registers.log)
  auto stack_store = [&](int k, const T (&f0)[E], const T (&f1)[E], const T (&f2)[E], T al, int nn,
                         int nna) __attribute__((always_inline)) {
    if (L0REG && k == 0) {
#pragma unroll
      for (int e = 0; e < E; ++e) {
        l0q[e] = f0[e];
        l0p[e] = f1[e];
      }
      l0a = al;
      l0n = nn;
      l0na = nna;
    } else if (L1R && k == 1) {
#pragma unroll
      for (int e = 0; e < E; ++e) {
        l1q[e] = f0[e];
        l1p[e] = f1[e];
        l1r[e] = f2[e];
      }
      l1a = al;
      l1n = nn;
      l1na = nna;
    } else if (k < KL) {
      T* v = lvec + (long long)k * 3 * NT * E + tix * E;
#pragma unroll
      for (int e = 0; e < E; ++e) {
        v[e] = f0[e];
        v[NT * E + e] = f1[e];
        v[2 * NT * E + e] = f2[e];
      }
      lalpha[k * CPB + cib] = al;
      lnn[k * CPB + cib] = nn;
      lnna[k * CPB + cib] = nna;
    } else {
      T* sv = (T*)(sbase + k * a.stk_es);
#pragma unroll
      for (int e = 0; e < E; ++e) {
        const int i = lane * E + e;
        if (i < D) {
          sv[i] = f0[e];
          sv[D + i] = f1[e];
          sv[2 * D + i] = f2[e];
        }
      }
      sv[3 * D] = al;
      int* sn = (int*)(sv + 3 * D + 1);
      sn[0] = nn;
      sn[1] = nna;
    }
  };
  // field f (0 first q, 1 first p, 2 proposal) of level k
  auto stack_vec = [&](int k, int f, T (&out)[E]) __attribute__((always_inline)) {
    if (L0REG && k == 0) {
#pragma unroll
      for (int e = 0; e < E; ++e) out[e] = f == 1 ? l0p[e] : l0q[e];
    } else if (L1R && k == 1) {
#pragma unroll
      for (int e = 0; e < E; ++e) out[e] = f == 0 ? l1q[e] : f == 1 ? l1p[e] : l1r[e];
    } else if (k < KL) {
      const T* v = lvec + ((long long)k * 3 + f) * NT * E + tix * E;
#pragma unroll
      for (int e = 0; e < E; ++e) out[e] = v[e];
    } else {
      const T* sv = (const T*)(sbase + k * a.stk_es) + f * D;
#pragma unroll
      for (int e = 0; e < E; ++e) {
        const int i = lane * E + e;
        out[e] = (i < D) ? sv[i] : (T)0;
      }
    }
  };
  // the same read for a wave-uniform level k where only some chains use it:
  // registers and LDS are read by every lane (in bounds, and an LDS read costs
  // no more for the lanes that discard it), HBM only by the lanes of pred
  auto stack_vec_if = [&](int k, int f, T (&out)[E], bool pred) __attribute__((always_inline)) {
    if ((L0REG && k == 0) || (L1R && k == 1) || k < KL) {
      stack_vec(k, f, out);
    } else {
      const T* sv = (const T*)(sbase + k * a.stk_es) + f * D;
#pragma unroll
      for (int e = 0; e < E; ++e) {
        const int i = lane * E + e;
        out[e] = (pred && i < D) ? sv[i] : (T)0;
      }
    }
  };
  auto stack_scalars = [&](int k, T& al, int& nn, int& nna) __attribute__((always_inline)) {
    if (L0REG && k == 0) {
      al = l0a;
      nn = l0n;
      nna = l0na;
    } else if (L1R && k == 1) {
      al = l1a;
      nn = l1n;
      nna = l1na;
    } else if (k < KL) {
      al = lalpha[k * CPB + cib];
      nn = lnn[k * CPB + cib];
      nna = lnna[k * CPB + cib];
    } else {
      const T* sv = (const T*)(sbase + k * a.stk_es) + 3 * D;
      al = sv[0];
      const int* sn = (const int*)(sv + 1);
      nn = sn[0];
      nna = sn[1];
    }
  };

  T q[E];
#pragma unroll
  for (int e = 0; e < E; ++e) {
    const int i = lane * E + e;
    q[e] = (i < D) ? qs[c * D + i] : (T)0;
  }
  T eps = ((T*)a.eps)[c], eps_bar = ((T*)a.eps_bar)[c], h_bar = ((T*)a.h_bar)[c], mu = ((T*)a.mu)[c];
  const T gamma = (T)0.05, kappa = (T)0.75, delta = (T)a.target_accept;
  const long long t0c = 10;

  // the chain's metric and warm-up statistics (generic_nuts.rs:33-359)
  MassDev<T, E, MASS> M;
  M.D = D;
  int rn = 0;
  T rmean[E], rm2d[E];
  if (MASS == 3) {  // every chain dense (the host checked a.mkind)
    M.minvT = (const T*)a.minv + (long long)c * D * D;
    M.cholT = (const T*)a.mchol + (long long)c * D * D;
    M.cholR = (const T*)a.mchol_rm + (long long)c * D * D;
  }
  if (MASS && MASS != 3 && a.mass_mode) {
    M.kind_ = a.mkind[c];
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const int i = lane * E + e;
      M.inv[e] = (i < D) ? ((const T*)a.dinv)[c * D + i] : (T)0;
      M.sq[e] = (i < D) ? ((const T*)a.dsq)[c * D + i] : (T)0;
      rmean[e] = (i < D) ? ((const T*)a.rmean)[c * D + i] : (T)0;
      rm2d[e] = (i < D) ? ((const T*)a.rm2d)[c * D + i] : (T)0;
    }
    if (MASS == 2 && a.mass_mode == 2) {
      M.minvT = (const T*)a.minv + (long long)c * D * D;
      M.cholT = (const T*)a.mchol + (long long)c * D * D;
      M.cholR = (const T*)a.mchol_rm + (long long)c * D * D;
    }
    rn = a.rn[c];
  }
  if (MASS >= 2 && a.mass_mode == 2) {
    {
      if constexpr (LPC == 16 && E == 2) {
        if (a.minv_lds == 2) {
          // the chain's M^-1 into its LDS slot, full and transposed ([j][i]):
          // each lane copies exactly the entries it reads (no barrier)
          constexpr int DP = LPC * E;
          M.lds_off = a.minv_lds_off + (unsigned)(cib * DP * DP * sizeof(T));
          T* ml = (T*)(gm_dyn_lds + M.lds_off);
          for (int jj = 0; jj < DP; ++jj) {
#pragma unroll
            for (int e = 0; e < E; ++e) {
              const int r = lane * E + e;
              ml[jj * DP + r] = (r < D && jj < D) ? M.minvT[(long long)jj * D + r] : (T)0;
            }
          }
          M.minv_lds = 2;
        } else if (a.minv_lds) {
          // the chain's M^-1 into its LDS slot, lower triangle packed
          // (minv_packed_lds): each lane writes its own rows; the chain's
          // lanes (one wave) read each other's rows after the wave barrier
          M.lds_off = a.minv_lds_off + (unsigned)(cib * minv_packed_bytes<LPC, E, T>());
          T* ml = (T*)(gm_dyn_lds + M.lds_off);
#pragma unroll
          for (int e = 0; e < E; ++e) {
            const int r = lane * E + e;
            for (int jj = 0; jj <= r; ++jj) ml[tri_n(r) + jj] = (r < D) ? M.minvT[(long long)jj * D + r] : (T)0;
          }
          M.minv_lds = 1;
          if (a.chol_lds) {  // and its Cholesky factor's rows, packed the same way
            M.chol_off = a.chol_lds_off + (unsigned)(cib * minv_packed_bytes<LPC, E, T>());
            T* cl = (T*)(gm_dyn_lds + M.chol_off);
#pragma unroll
            for (int e = 0; e < E; ++e) {
              const int r = lane * E + e;
              for (int jj = 0; jj <= r; ++jj) cl[tri_n(r) + jj] = (r < D) ? M.cholT[(long long)jj * D + r] : (T)0;
            }
            M.chol_lds = 1;
          }
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
          __builtin_amdgcn_wave_barrier();
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        }
      }
    }
  }

  if (a.do_init) {  // init_chain_state (generic_nuts.rs:731-753)
    T z[E], p0[E];
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const int i = lane * E + e;
      z[e] = (i < D) ? normal<T>(a.seed, cid, a.init_step, TAG_NUTS_INIT, (uint32_t)i) : (T)0;
    }
    momentum_from<LPC, E>(M, z, p0, lane);
    const T ae = eps + (T)1;
    // copies: the out-of-line search takes its arrays by address, which would
    // otherwise keep the loop's q and momentum in scratch memory
    T qc[E], pc[E];
#pragma unroll
    for (int e = 0; e < E; ++e) { qc[e] = q[e]; pc[e] = p0[e]; }
    if ((ae < (T)0 ? -ae : ae) <= MachEps<T>::v) eps = find_reasonable_epsilon<LPC, E, T, decltype(tg), MASS>(tg, qc, pc, lane, D);
    mu = glog((T)10 * eps);
  }
  if (MASS != 3 && a.do_refind && a.updated[c]) {  // after a metric update (generic_nuts.rs:905-918)
    T z[E], probe[E];
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const int i = lane * E + e;
      z[e] = (i < D) ? normal<T>(a.seed, cid, a.refind_step, TAG_NUTS_PROBE, (uint32_t)i) : (T)0;
    }
    momentum_from<LPC, E>(M, z, probe, lane);
    T qc[E];
#pragma unroll
    for (int e = 0; e < E; ++e) qc[e] = q[e];
    eps = find_reasonable_epsilon<LPC, E, T, decltype(tg), MASS>(tg, qc, probe, lane, D);  // identity-mass leapfrog (:1009-1023)
    mu = glog((T)10 * eps);
    eps_bar = eps;
    h_bar = (T)0;
  }
  auto record = [&](long long t) {
    const long long row = t - a.row_shift;
    if (row >= 0 && row < a.n_rows && a.samples != nullptr) {
      T* __restrict__ out = (T*)a.samples + (row * C + c) * D;
#pragma unroll
      for (int e = 0; e < E; ++e) {
        const int i = lane * E + e;
        if (i < D) out[i] = q[e];
      }
    }
  };
  if (a.t0 == 0) record(0);

  long long acc = 0, nlf = 0;
  NormalCache<T> ncache[E];  // (one joint refill of the lane's E coordinates
                             // measured -6 %, profiles/r04/ab_nuts_joint_momentum_refill.log)
  const bool track = a.trk.mean != nullptr;  // run_progress (generic_nuts.rs:688-704)
  ChainTrack<LPC, E> tr;
  // (the frozen-dense kernel keeps the tracker's vectors in memory between
  // transitions: its registers are short)
  if (track) {
    if constexpr (MASS == 3) tr.p = a.trk.p[c];
    else tr.load(a.trk, c, lane, D);
  }

  // per-chain loop state
  int s = 0;             // transitions completed in this launch
  bool starting = true;  // the next evaluation starts transition s
  T p0o[E];              // the transition's momentum (starting chains)
  T qe[E], pe[E], ge[E];  // edge: the trajectory end on side v (being integrated)
  T qf[E], pf[E], gf[E];  // the far end
  // dense metric: M^-1 p and M^-1 g of both ends, carried by linearity
  // (carried_velocity below); the start's M^-1 p0
  T ve[E], we[E], vf[E], wf[E], v0o[E];
  int v = 1, j = 0;
  // tree counts fit 32 bits: the depth cap (<= NUTS_MAX_DEPTH_LIMIT = 30) bounds n by 2^30
  int l = 0, n = 1;
  T joint0 = (T)0, logu = (T)0;
  uint64_t key = 0;
  uint32_t dirb = 0;  // the transition's direction bits (pre-pass record)
// The frozen-dense kernel keeps its in-kernel start draws: with the records
// its spills grew (61 -> 73 VGPRs) and cfg3_dense ran 1.7 % slower, against
// +2.6 % for cfg3 (profiles/r06/ab_nuts_start_records.log).
#ifndef GM_SREC_DENSE
#define GM_SREC_DENSE 0
#endif
  uint32_t merge_ctr = 0;
  T fq[E], fp[E], pr[E];  // current subtree: first q, first p, proposal
  int tn = 0, tna = 0;
  bool ts = true;
  T ta = (T)0;
#pragma unroll
  for (int e = 0; e < E; ++e) {
    qe[e] = pe[e] = ge[e] = qf[e] = pf[e] = gf[e] = fq[e] = fp[e] = pr[e] = p0o[e] = (T)0;
    ve[e] = we[e] = vf[e] = wf[e] = v0o[e] = (T)0;
  }

#ifdef GM_NUTS_PROF
  // segments: 0 top -> after momentum draw, 1 -> after kick/drift, 2 -> after
  // the target's eval_part, 3 -> after the second kick and kinetic part,
  // 4 -> after the reduction, 5 -> after the leaf rules (joint, exp),
  // 6 -> after the merge climb, 7 -> end of iteration (doubling / transition end)
  unsigned long long pseg[8] = {}, pst = 0;
#define GM_PSEG(i)                                                        \
  do {                                                                    \
    __builtin_amdgcn_s_waitcnt(0);                                        \
    const unsigned long long _n = __builtin_amdgcn_s_memtime();           \
    pseg[i] += _n - pst;                                                  \
    pst = _n;                                                             \
  } while (0)
  unsigned long long pcnt[16] = {}, pcyc[16] = {}, peval = 0, piter = 0;
  unsigned long long ptop = __builtin_amdgcn_s_memtime();
  bool f_start = false, f_merge = false, f_dbl = false, f_trans = false;
#endif
  // Every load issued before the loop (state, step sizes, tracker) is
  // complete here. On gfx9 stores count in vmcnt too: with a load still
  // pending at the loop entry, the wait the compiler puts at the loop head
  // would also wait out the previous transition's sample stores.
  __builtin_amdgcn_s_waitcnt(0);
  const LeafExpK lek = LeafExpK::make();  // the leaf exp's constants (f64)
  // the launch's start records from the momentum pre-pass (a.zrec)
  const bool srec = (GM_SREC_DENSE || MASS != 3) && a.zmom != nullptr;
  // the frozen-dense kernel's momenta with the metric applied (a.pv0)
  // (non-temporal loads of p0 / M^-1 p0 and stores of the samples measured
  // -1.5 %, HBM 31.6 -> 29.0 GB: not kept, profiles/r06/ab_nuts_dense_prep2.log)
  // (known at compile time in the default build: no in-kernel draw, L
  // product or start-time M^-1 product is emitted there)
  const bool prepd = MASS == 3 && (GM_DENSE_PREP || a.pv0 != nullptr);
  while (true) {
    const bool live = s < a.n_steps;
#ifdef GM_NUTS_PROF
    {
      const unsigned long long now = __builtin_amdgcn_s_memtime();
      const int bin = (__builtin_amdgcn_ballot_w64(f_start) != 0 ? 1 : 0) |
                      (__builtin_amdgcn_ballot_w64(f_merge) != 0 ? 2 : 0) |
                      (__builtin_amdgcn_ballot_w64(f_dbl) != 0 ? 4 : 0) |
                      (__builtin_amdgcn_ballot_w64(f_trans) != 0 ? 8 : 0);
      if (piter > 0) {
#pragma unroll
        for (int b = 0; b < 16; ++b)
          if (b == bin) { pcnt[b] += 1; pcyc[b] += now - ptop; }
      }
      ++piter;
      ptop = now;
      if (piter > 1) pseg[7] += now - pst;
      pst = now;
      f_start = f_merge = f_dbl = f_trans = false;
    }
#endif
    if (__builtin_amdgcn_ballot_w64(live) == 0) break;  // every chain of the wave is done
    const uint64_t st = a.step0 + (uint64_t)s;
    const T epsv = (T)v * eps;
    const T h = epsv * (T)0.5;
    // --- the evaluation point: q (a starting transition) or the next leaf
    T x[E], gx[E];
    // The start's momentum p0 and M^-1 p0 are used in the iteration that
    // draws them only. The frozen-dense kernel keeps them iteration-local
    // (zero elsewhere: 8 registers it cannot spare); the others keep the
    // loop-carried arrays of their measured schedule.
    T p0l[E], v0l[E];
#pragma unroll
    for (int e = 0; e < E; ++e) p0l[e] = v0l[e] = (T)0;
    T (&p0)[E] = [&]() -> T (&)[E] {
      if constexpr (MASS == 3) return p0l;
      else return p0o;
    }();
    T (&v0)[E] = [&]() -> T (&)[E] {
      if constexpr (MASS == 3) return v0l;
      else return v0o;
    }();
    // the transition's standard normals (generic_nuts.rs:758-762): from the
    // launch's pre-drawn block (their loads in flight under the evaluation
    // below), else drawn here; the metric's product after the evaluation
    T zs[E];
    // with the pre-pass: the transition's start record as well (its key, the
    // slice variable's log and the direction bits), loaded with the momenta.
    // (Left unset otherwise, like zs: zeroing them would make the loop head
    // wait for the previous iteration's loads into the same registers, and on
    // gfx9 that vmcnt wait includes every outstanding store.)
    uint64_t skey;
    T slnu;
    uint32_t sdir;
    if (live && starting) {
      if (srec) {
        const NutsStartRec<T>* __restrict__ r = (const NutsStartRec<T>*)a.zrec + ((long long)s * C + c);
        skey = r->key;
        slnu = r->lnu;
        sdir = r->dir;
      }
      if (prepd) {  // p0 and M^-1 p0 from the pre-pass (a.pv0)
        const long long o = ((long long)s * C + c) * D;
        const T* __restrict__ pm = (const T*)a.zmom + o;
        const T* __restrict__ vm = (const T*)a.pv0 + o;
#pragma unroll
        for (int e = 0; e < E; ++e) {
          const int i = lane * E + e;
          p0l[e] = (i < D) ? pm[i] : (T)0;
          v0l[e] = (i < D) ? vm[i] : (T)0;
        }
      } else if (a.zmom != nullptr) {
        const T* __restrict__ zm = (const T*)a.zmom + ((long long)s * C + c) * D;
#pragma unroll
        for (int e = 0; e < E; ++e) {
          const int i = lane * E + e;
          zs[e] = (i < D) ? zm[i] : (T)0;
        }
      } else {
#pragma unroll
        for (int e = 0; e < E; ++e) {
          const int i = lane * E + e;
          zs[e] = (i < D) ? ncache[e].get_s(a.seed, cid, st, TAG_NUTS_MOM, (uint32_t)i) : (T)0;
        }
      }
    }
#ifdef GM_NUTS_PROF
    GM_PSEG(0);
#endif
    if constexpr (MASS == 0) {  // leapfrog (:1396-1418): kick, drift
      // unconditionally: a starting chain overwrites its edge with the
      // transition's start below, and a finished chain's edge is never read
      // again, so neither needs the old values kept (no selects)
#pragma unroll
      for (int e = 0; e < E; ++e) {
        pe[e] = pe[e] + ge[e] * h;
        qe[e] = qe[e] + pe[e] * epsv;
      }
    }
    // the drift's M^-1 p (the kicked momentum); with a dense metric carried
    // from the edge: M^-1 (p + g h) = M^-1 p + (M^-1 g) h
    T vv[E];
    if constexpr (MASS != 0) {
      if (live && !starting) {  // leapfrog_with_mass (:1396-1418): kick, drift by M^-1 p
#pragma unroll
        for (int e = 0; e < E; ++e) pe[e] = pe[e] + ge[e] * h;
        if (MASS >= 2 && M.kind() == 2) {
#pragma unroll
          for (int e = 0; e < E; ++e) vv[e] = ve[e] + we[e] * h;
        } else {
          inv_mul<LPC, E>(M, pe, vv, lane);
        }
#pragma unroll
        for (int e = 0; e < E; ++e) qe[e] = qe[e] + vv[e] * epsv;
      }
    }
#pragma unroll
    for (int e = 0; e < E; ++e) x[e] = starting ? q[e] : qe[e];
    T sums[2];
#ifdef GM_NUTS_PROF
    GM_PSEG(1);
#endif
    sums[0] = tg.template eval_part<LPC, E>(x, gx, lane);
#ifdef GM_NUTS_PROF
    GM_PSEG(2);
#endif
#pragma unroll
    for (int e = 0; e < E; ++e) pe[e] = pe[e] + gx[e] * h;  // (unconditionally, as above)
    if (live && starting && !prepd) momentum_from<LPC, E>(M, zs, p0, lane);  // sample_momentum (:275-303)
    T wx[E];  // dense metric: M^-1 g at the evaluation point
    {
      T pk[E];
#pragma unroll
      for (int e = 0; e < E; ++e) pk[e] = starting ? p0[e] : pe[e];
      if constexpr (MASS >= 2) {
        // carried_velocity: one product per evaluation (M^-1 g) instead of
        // two (the drift's M^-1 p and the kinetic energy's); a starting
        // chain's M^-1 p0 only in iterations where some chain of the wave
        // starts a transition
        inv_mul<LPC, E>(M, gx, wx, lane);
        if (!prepd && __builtin_amdgcn_ballot_w64(live && starting && M.kind() == 2) != 0)
          inv_mul<LPC, E>(M, p0, v0, lane);
        if (M.kind() == 2) {
          T t[E];
#pragma unroll
          for (int e = 0; e < E; ++e) {
            vv[e] = starting ? v0[e] : vv[e] + wx[e] * h;  // M^-1 p at the evaluation point
            t[e] = pk[e] * vv[e];
          }
          T part = t[0];
#pragma unroll
          for (int e = 1; e < E; ++e) part = part + t[e];
          sums[1] = part;
        } else {
          sums[1] = kin_part_m<LPC, E>(M, pk, lane);
        }
      } else {
        sums[1] = kin_part_m<LPC, E>(M, pk, lane);
      }
    }
#ifdef GM_NUTS_PROF
    GM_PSEG(3);
#endif
    group_sum_n<LPC>(sums);  // log-density and kinetic energy, reduced together
#ifdef GM_NUTS_PROF
    GM_PSEG(4);
#endif
#ifdef GM_NUTS_PROF
    peval += __builtin_amdgcn_s_memtime() - ptop;
#endif
    const T lp = tg.finish(sums[0]);
    const T kin = (T)0.5 * sums[1];
    if (!live) continue;

    if (starting) {
#ifdef GM_NUTS_PROF
      f_start = true;
#endif
      // --- transition start: slice variable, trajectory ends (:764-781)
      joint0 = lp - kin;
      if (srec) {  // the pre-pass's record (nuts_starts_kernel): the same values
        key = skey;
        logu = joint0 + slnu;
        dirb = sdir;
      } else {
        const u32x4 kw = draw_block_s(a.seed, cid, st, TAG_NUTS_EXP, 0u);
        key = nuts_key(kw);
        // (the table-driven Box-Muller of spec v5 for these momenta and this
        // Exp1 draw measured -4 % at cfg3, profiles/r04/ab_nuts_tab_momenta.log:
        // its 6 KiB of LDS tables and ~10 registers cost more than its
        // instructions save)
        logu = joint0 + glog_pos(Unif<T>::oc(kw.z, kw.w));  // joint - Exp1
      }
#pragma unroll
      for (int e = 0; e < E; ++e) {
        qe[e] = q[e]; pe[e] = p0[e]; ge[e] = gx[e];
        qf[e] = q[e]; pf[e] = p0[e]; gf[e] = gx[e];
      }
      if constexpr (MASS >= 2) {
#pragma unroll
        for (int e = 0; e < E; ++e) {
          ve[e] = v0[e]; we[e] = wx[e];
          vf[e] = v0[e]; wf[e] = wx[e];
        }
      }
      n = 1;
      j = 0;
      l = 0;
      merge_ctr = 0;
      v = (srec ? (dirb & 1u) != 0 : nuts_u<T>(key, 0u) < (T)0.5) ? 1 : -1;  // doubling 0's direction (:783-784)
      starting = false;
      continue;
    }

    // --- a leaf (build_tree_with_mass base case, :1187-1212)
    ++nlf;
#pragma unroll
    for (int e = 0; e < E; ++e) ge[e] = gx[e];
    if constexpr (MASS >= 2) {
#pragma unroll
      for (int e = 0; e < E; ++e) { ve[e] = vv[e]; we[e] = wx[e]; }
    }
    const T joint = lp - kin;
    tn = (logu < joint) ? 1 : 0;
    ts = (logu - (T)1000) < joint;
    // min(1, exp(joint - joint0)): f64 by the division-free table form
    if constexpr (sizeof(T) == 8) ta = leaf_alpha_tab(joint - joint0, exp_lds, lek);
    else ta = rust_min1(gexp(joint - joint0));
    tna = 1;
#pragma unroll
    for (int e = 0; e < E; ++e) { fq[e] = qe[e]; fp[e] = pe[e]; pr[e] = qe[e]; }
#ifdef GM_NUTS_PROF
    GM_PSEG(5);
#endif
    // climb: merge with the stored left siblings this leaf completes
    bool done = false;
    // Wave-uniform climb: the level k is one counter for the wave (a scalar),
    // and each chain's part of trip k is decided by selects. A chain at level
    // k < j either completes a right child (bit k of its leaf index l is 1:
    // merge with the stored left sibling and go on up), or is a left child:
    // stored there if its subtree goes on (ts), else passed up unchanged (a
    // truncated left subtree's parent builds no right half). At k == j the
    // doubling is complete. The trips are the wave's longest climb, as in the
    // per-chain loop, without its exec-mask bookkeeping; the merges and their
    // draws are each chain's own, in the recursion's post-order.
    {
      bool act = true;
      for (int k = 0;; ++k) {
        const bool top = act && k == j;
        done = done || top;
        act = act && !top;
        const bool rbit = ((l >> k) & 1) != 0;
        const bool mrg = act && rbit;
        const bool sto = act && !rbit && ts;
        act = act && !sto;
        if (__builtin_amdgcn_ballot_w64(mrg) != 0) {
#ifdef GM_NUTS_PROF
          f_merge = true;
#endif
          T lq[E], lpv[E], lpr[E];
          stack_vec_if(k, 0, lq, mrg);
          stack_vec_if(k, 1, lpv, mrg);
          stack_vec_if(k, 2, lpr, mrg);
          // (values, not places: without this the compiler selects between
          // the arrays' addresses and keeps both in scratch)
#pragma unroll
          for (int e = 0; e < E; ++e) asm volatile("" : "+v"(lq[e]), "+v"(lpv[e]), "+v"(lpr[e]));
          // the U-turn over the merged subtree's ends: the edge (qe, pe) and
          // the left sibling's first point (lq, lpv), unordered (no_uturn_ends)
          const bool nu = no_uturn_ends<LPC, E>(qe, lq, pe, lpv, v);
#pragma unroll
          for (int e = 0; e < E; ++e) {
            fq[e] = mrg ? lq[e] : fq[e];
            fp[e] = mrg ? lpv[e] : fp[e];
          }
          int ln_, lna;
          T lal;
          stack_scalars(k, lal, ln_, lna);
          const double u = nuts_u<double>(key, 64u + merge_ctr);
          merge_ctr += mrg ? 1u : 0u;
          const int den = (ln_ + tn) > 1 ? (ln_ + tn) : 1;
          const bool below = draw_below_ratio(u, (double)tn, (double)den);
          const bool keep_left = mrg & !below;
#pragma unroll
          for (int e = 0; e < E; ++e) pr[e] = keep_left ? lpr[e] : pr[e];
          tn = mrg ? ln_ + tn : tn;
          ts = mrg ? (ts && nu) : ts;
          ta = mrg ? lal + ta : ta;
          tna = mrg ? lna + tna : tna;
        }
        if (__builtin_amdgcn_ballot_w64(sto) != 0) {
          if (sto) stack_store(k, fq, fp, pr, ta, tn, tna);
        }
        if (__builtin_amdgcn_ballot_w64(act) == 0) break;
      }
    }
#ifdef GM_NUTS_PROF
    GM_PSEG(6);
#endif
    if (!done) {
      ++l;
      continue;
    }

    // --- the doubling is complete (or truncated): top level (:785-880).
    // The new end on side v is the edge; alpha / n_alpha are this subtree's.
    const T alpha = ta;
    const int n_alpha = tna;
#ifdef GM_NUTS_PROF
    f_dbl = true;
#endif
    {
      // u2 < min(1, tn / n) (:860-861): always when tn >= n (u2 < 1)
      const T u2 = nuts_u<T>(key, 2u * (uint32_t)j + 1u);
      const bool move = ts && (tn >= n || draw_below_ratio(u2, (T)tn, (T)n));
#pragma unroll
      for (int e = 0; e < E; ++e) q[e] = move ? pr[e] : q[e];
      acc += move ? 1 : 0;
      n += tn;
      bool s_ok = ts;
      {
        // the trajectory's ends: the edge (qe, pe) on side v and the far end
        // (qf, pf), unordered (no_uturn_ends)
        if constexpr (MASS >= 2) {  // dense: the ends' carried M^-1 p (no product)
          if (s_ok) {
            if (M.kind() == 2) s_ok = no_uturn_ends<LPC, E>(qe, qf, ve, vf, v);
            else s_ok = no_uturn_ends_m<LPC, E>(M, qe, qf, pe, pf, v, lane);
          }
        } else {
          const bool nu = no_uturn_ends_m<LPC, E>(M, qe, qf, pe, pf, v, lane);
          s_ok = s_ok && nu;
        }
      }
      ++j;
      if (s_ok && j < a.max_depth) {  // next doubling
        const bool up = srec ? ((dirb >> j) & 1u) != 0 : nuts_u<T>(key, 2u * (uint32_t)j) < (T)0.5;
        const int v2 = up ? 1 : -1;
        const bool sw = v2 != v;  // integrate from the other end
#pragma unroll
        for (int e = 0; e < E; ++e) {
          const T a0 = qe[e], a1 = pe[e], a2 = ge[e];
          qe[e] = sw ? qf[e] : qe[e];
          pe[e] = sw ? pf[e] : pe[e];
          ge[e] = sw ? gf[e] : ge[e];
          qf[e] = sw ? a0 : qf[e];
          pf[e] = sw ? a1 : pf[e];
          gf[e] = sw ? a2 : gf[e];
        }
        if constexpr (MASS >= 2) {
#pragma unroll
          for (int e = 0; e < E; ++e) {
            const T b0 = ve[e], b1 = we[e];
            ve[e] = sw ? vf[e] : ve[e];
            we[e] = sw ? wf[e] : we[e];
            vf[e] = sw ? b0 : vf[e];
            wf[e] = sw ? b1 : wf[e];
          }
        }
        v = v2;
        l = 0;
        continue;
      }
    }

    // --- the transition is complete: dual averaging (generic_nuts.rs:882-924)
#ifdef GM_NUTS_PROF
    f_trans = true;
#endif
    const long long m = a.m0 + s + 1;
    T eta = (T)1 / (T)(m + t0c);
    h_bar = ((T)1 - eta) * h_bar + eta * (delta - alpha / (T)n_alpha);
    if (m <= a.n_discard) {
      const T mf = (T)m;
      eps = gexp(mu - gsqrt(mf) / gamma * h_bar);
      eta = gexp(-kappa * glog(mf));  // m^(-kappa)
      eps_bar = gexp(((T)1 - eta) * glog(eps_bar) + eta * glog(eps));
      // RunningCov::update inside the collection window (:897-903, 108-129)
      const long long lim = a.n_discard > a.eb ? a.n_discard - a.eb : 0;
      if (MASS && MASS != 3 && a.mass_mode && m > a.sb && m < lim) {
        rn += 1;
        const T ns = (T)rn;
        T d1[E], d2[E];
#pragma unroll
        for (int e = 0; e < E; ++e) {
          d1[e] = q[e] - rmean[e];
          rmean[e] = rmean[e] + d1[e] / ns;
          d2[e] = q[e] - rmean[e];
          rm2d[e] = rm2d[e] + d1[e] * d2[e];
        }
        if (MASS == 2 && a.mass_mode == 2) {
          T* m2 = (T*)a.rm2 + (long long)c * D * D;
          for (int jj = 0; jj < D; ++jj) {
            const T dj = coord<LPC, E>(d2, jj);
#pragma unroll
            for (int e = 0; e < E; ++e) {
              const int i = lane * E + e;
              if (i < D && jj >= i) m2[(long long)i * D + jj] = m2[(long long)i * D + jj] + d1[e] * dj;
            }
          }
        }
      }
    } else {
      eps = eps_bar;
    }
    if (track) {
      if constexpr (MASS == 3) tr.load_vec(a.trk, c, lane, D);
      tr.step(q, a.trk.n0 + (unsigned long long)s + 1ull, lane, D);
      if constexpr (MASS == 3) tr.store_vec(a.trk, c, lane, D);
    }
    record(a.t0 + s + 1);
    ++s;
    starting = true;
  }
#ifdef GM_NUTS_PROF
  {
    const long long wv = ((long long)blockIdx.x * blockDim.x + threadIdx.x) / 64;
    if ((threadIdx.x & 63) == 0 && wv < NPROF_WAVES) {
      unsigned long long* o = gm_nuts_prof_buf + wv * NPROF_SLOTS;
      for (int b = 0; b < 16; ++b) { o[2 * b] = pcnt[b]; o[2 * b + 1] = pcyc[b]; }
      o[32] = peval;
      o[33] = piter;
      unsigned long long pprod = 0;  // cycles inside the target's matrix-core product, if it has one
      if constexpr (requires { tg.prof_prod; }) pprod = tg.prof_prod;
      o[34] = pprod;
      for (int b = 0; b < 8; ++b) o[35 + b] = pseg[b];
    }
  }
#endif
  if (track) {
    if constexpr (MASS == 3) {
      if (lane == 0) a.trk.p[c] = tr.p;
    } else {
      tr.store(a.trk, c, lane, D);
    }
  }
  if (MASS && MASS != 3 && a.mass_mode) {
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const int i = lane * E + e;
      if (i < D) {
        ((T*)a.rmean)[c * D + i] = rmean[e];
        ((T*)a.rm2d)[c * D + i] = rm2d[e];
      }
    }
    if (lane == 0) a.rn[c] = rn;
  }
#pragma unroll
  for (int e = 0; e < E; ++e) {
    const int i = lane * E + e;
    if (i < D) qs[c * D + i] = q[e];
  }
  if (lane == 0) {
    ((T*)a.eps)[c] = eps;
    ((T*)a.eps_bar)[c] = eps_bar;
    ((T*)a.h_bar)[c] = h_bar;
    ((T*)a.mu)[c] = mu;
    a.accepts[c] += acc;
    a.n_leapfrog[c] += nlf;
  }
}

}  // namespace gm
