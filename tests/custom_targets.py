"""HIP sources of user targets for the CustomTarget tests: the built-in
targets restated as user code in the oracle's one-chain-per-lane arithmetic
(lanes 1, elems = dim: plain left-to-right sums), so that samples from the
runtime-compiled kernels can be compared bit for bit with the oracle."""

# RosenbrockND in the select form of oracle/gm_oracle_t.inc (params: a, b)
ROSENBROCK = r"""
template <class T>
__device__ T gm_logp_grad(const T* x, T* g, const T* p) {
  const T a = p[0], b = p[1], b2 = (T)2 * b, b4 = (T)4 * b;
  T part = (T)0;
#pragma unroll
  for (int i = 0; i < GM_DIM; ++i) {
    const bool hs = i <= GM_DIM - 2, hp = i >= 1;
    const T am = a - x[i];
    const T ti = hs ? x[hs ? i + 1 : i] - x[i] * x[i] : (T)0;
    const T A = hs ? (b4 * x[i]) * ti + (T)2 * am : (T)0;
    const T B = hp ? b2 * (x[i] - x[hp ? i - 1 : i] * x[hp ? i - 1 : i]) : (T)0;
    g[i] = A - B;
    const T s = hs ? b * (ti * ti) + am * am : (T)0;
    part = (i == 0) ? s : part + s;
  }
  return -part;
}
"""

# IsotropicGaussian as a target (params: var = std*std in the sampler dtype)
ISO_GAUSS = r"""
template <class T>
__device__ T gm_logp_grad(const T* x, T* g, const T* p) {
  const T var = p[0];
  T part = (T)0;
#pragma unroll
  for (int i = 0; i < GM_DIM; ++i) {
    g[i] = (-x[i]) / var;
    const T s = x[i] * x[i];
    part = (i == 0) ? s : part + s;
  }
  return ((T)-0.5 * part) / var;
}
"""

BROKEN = r"""
template <class T>
__device__ T gm_logp_grad(const T* x, T* g, const T* p) { return undefined_symbol(x); }
"""
