/*
 * gm_oracle.h — CPU ORACLE (test infrastructure only; never linked into the
 * product). A plain-C restatement of the reference algorithms of
 * SauersML/general-mcmc for the HMC / NUTS / MH / split-R-hat path, driven by
 * the engine's documented random-number spec so that the GPU kernels can be
 * checked bit-for-bit on the same inputs.
 *
 * Parity pins: the reference's RNG-free known-answer tests (tests/golden/
 * reference_kat.json, see tests/test_oracle_kat.py): build_tree
 * (nuts.rs:521-586), find_reasonable_epsilon (nuts.rs:508-519), chain_1
 * (nuts.rs:588-601), MultiChainTracker R-hat (stats.rs:734-783), autocov BF
 * and FFT (stats.rs:808-839), IsotropicGaussian / Gaussian2D densities
 * (distributions.rs:580-614, 820-839) and the mass-matrix algebra
 * (generic_nuts.rs:1427-1489). The reference's random streams (rand 0.9
 * SmallRng, rand_distr, burn backend RNG) cannot be reproduced offline; sample
 * streams are therefore pinned to the engine's Philox spec, not to the
 * reference's bits.
 *
 * Summation order: per-chain sums (kinetic energy, log-density, U-turn dots)
 * are taken in the engine's declared order, parameterised by the lane layout
 * (lanes x elems): each lane sums its elems left to right, then an xor
 * butterfly over lanes (offsets 1, 2, 4, ...). Layouts wider than one wave
 * (lanes = 64*W, HMC for dim > 1024) add the W wave totals left to right.
 */
#ifndef GM_ORACLE_H
#define GM_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* largest dimension of the wide (one chain per workgroup) HMC path */
#define GM_MAX_DIM 16384

typedef struct or_target {
  int32_t kind; /* 1 rosenbrock, 2 iso gauss, 3 gauss */
  int32_t dim;
  double a, b, std;
  const double* mean; /* [dim] */
  const double* prec; /* [dim*dim] */
  double norm_const;
} or_target;

/* ---- RNG spec ---- */
void or_philox(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]);
double or_log_d(double x);
float or_log_f(float x);
double or_exp_d(double x);
double or_leaf_alpha_d(double x); /* the NUTS leaf's f64 min(1, exp(x)), the kernels' table form */
float or_exp_f(float x);
double or_cos2pi_d(double u);
float or_cos2pi_f(float u);
double or_normal_d(uint64_t seed, uint32_t chain, uint64_t step, uint32_t tag, uint32_t idx);
/* spec v5 f32 (the HMC momenta): one table-driven Box-Muller pair of the
 * words (w1, w2); the HMC momentum draws (f32 table form, f64 = or_normal_d) */
void or_tab_normal_pair_f(uint32_t w1, uint32_t w2, float z[2]);
float or_mom_normal_f(uint64_t seed, uint32_t chain, uint64_t step, uint32_t tag, uint32_t idx);
double or_mom_normal_d(uint64_t seed, uint32_t chain, uint64_t step, uint32_t tag, uint32_t idx);
float or_normal_f(uint64_t seed, uint32_t chain, uint64_t step, uint32_t tag, uint32_t idx);
/* the f64 MH proposal normal (spec v5: table-driven Box-Muller) */
void or_tab_normal_pair(const uint32_t x[4], double z[2]);
double or_tab_normal_d(uint64_t seed, uint32_t chain, uint64_t step, uint32_t tag, uint32_t idx);
double or_uniform_co_d(uint64_t seed, uint32_t chain, uint64_t step, uint32_t tag, uint32_t idx);
float or_uniform_co_f(uint64_t seed, uint32_t chain, uint64_t step, uint32_t tag, uint32_t idx);

/* NUTS per-transition stream (spec v3): key block and the hashed draws */
uint64_t or_mix64(uint64_t z);
uint64_t or_nuts_key(uint64_t seed, uint32_t chain, uint64_t st, uint32_t w[4]);
double or_nuts_u_d(uint64_t key, uint32_t idx);
float or_nuts_u_f(uint64_t key, uint32_t idx);

/* ---- targets ---- */
double or_logp_grad_d(const or_target* t, int lanes, int elems, const double* x, double* g);
float or_logp_grad_f(const or_target* t, int lanes, int elems, const float* x, float* g);

/* ---- HMC: batched_hmc.rs:129-190 per chain; form 0 the engine's fused
 * multiply-add kicks and drift (the kernels), 1 the reference's op structure
 * (two roundings each: the composed tier-2 ops) ---- */
int or_hmc_run_d(const or_target* t, int lanes, int elems, int64_t C, int D, double* q, double eps,
                 int L, uint64_t seed, uint64_t step0, uint32_t chain_offset, int64_t n_steps,
                 int64_t collect_from, double* samples, int64_t* accepts, int threads, int form);
int or_hmc_run_f(const or_target* t, int lanes, int elems, int64_t C, int D, float* q, double eps,
                 int L, uint64_t seed, uint64_t step0, uint32_t chain_offset, int64_t n_steps,
                 int64_t collect_from, float* samples, int64_t* accepts, int threads, int form);

/* ---- MH: metropolis_hastings.rs:306-318 per chain ---- */
/* form 0: the kernels' arithmetic (canonical-order sums, the forward and
 * backward proposal densities one value, the carried log-density); form 1:
 * the reference's op structure (IsotropicGaussian's proposal and target sums
 * left to right, distributions.rs:378-406; log q forward and backward
 * separately and the current log-density recomputed, :306-318) */
int or_mh_run_d(const or_target* t, int lanes, int elems, int64_t C, int D, double* q,
                double prop_std, uint64_t seed, uint64_t step0, uint32_t chain_offset,
                int64_t n_steps, int64_t collect_from, double* samples, int64_t* accepts,
                int threads, int form);
int or_mh_run_f(const or_target* t, int lanes, int elems, int64_t C, int D, float* q,
                double prop_std, uint64_t seed, uint64_t step0, uint32_t chain_offset,
                int64_t n_steps, int64_t collect_from, float* samples, int64_t* accepts,
                int threads, int form);
/* one step's terms from states x [C][D] at counter st, in either form: the
 * log acceptance ratio la, the proposal's log-density lp1, the accept
 * log-uniform lnu (each [C]); the states are not moved */
int or_mh_terms_d(const or_target* t, int lanes, int elems, int64_t C, int D, const double* x,
                  double prop_std, uint64_t seed, uint64_t st, uint32_t chain_offset, int form,
                  double* la, double* lp1, double* lnu, int threads);
int or_mh_terms_f(const or_target* t, int lanes, int elems, int64_t C, int D, const float* x,
                  double prop_std, uint64_t seed, uint64_t st, uint32_t chain_offset, int form,
                  float* la, float* lp1, float* lnu, int threads);

/* ---- NUTS: generic_nuts.rs:731-1418 per chain (identity mass; the
 * engine's arithmetic -- or_nuts_mass_run with mode 0 and form 1 is the
 * reference's op structure: left-to-right kinetic sum and U-turn dots) ----
 * state arrays eps/eps_bar/h_bar/mu are [C]; progress selects run_progress
 * semantics; samples [n_collect][C][D]. init_step is the counter value of the
 * init draw; transitions use init_step + 0 .. total-1. */
int or_nuts_run_d(const or_target* t, int lanes, int elems, int64_t C, int D, double* q,
                  double* eps, double* eps_bar, double* h_bar, double* mu, double target_accept,
                  int max_depth, uint64_t seed, uint64_t init_step, uint32_t chain_offset,
                  int64_t n_collect, int64_t n_discard, int progress, double* samples,
                  int64_t* accepts, int64_t* n_leapfrog, int threads);
int or_nuts_run_f(const or_target* t, int lanes, int elems, int64_t C, int D, float* q,
                  float* eps, float* eps_bar, float* h_bar, float* mu, double target_accept,
                  int max_depth, uint64_t seed, uint64_t init_step, uint32_t chain_offset,
                  int64_t n_collect, int64_t n_discard, int progress, float* samples,
                  int64_t* accepts, int64_t* n_leapfrog, int threads);
/* NUTS::step (nuts.rs:431-433 -> generic_nuts.rs:755-925): n_steps
 * transitions without init_chain_state, adaptation counter from m0 against
 * n_discard, transition s drawing at counter step0 + s; nothing collected. */
int or_nuts_step_d(const or_target* t, int lanes, int elems, int64_t C, int D, double* q,
                   double* eps, double* eps_bar, double* h_bar, double* mu, double target_accept,
                   int max_depth, uint64_t seed, uint64_t step0, uint32_t chain_offset,
                   int64_t n_steps, int64_t m0, int64_t n_discard, int64_t* accepts,
                   int64_t* n_leapfrog, int threads);
int or_nuts_step_f(const or_target* t, int lanes, int elems, int64_t C, int D, float* q,
                   float* eps, float* eps_bar, float* h_bar, float* mu, double target_accept,
                   int max_depth, uint64_t seed, uint64_t step0, uint32_t chain_offset,
                   int64_t n_steps, int64_t m0, int64_t n_discard, int64_t* accepts,
                   int64_t* n_leapfrog, int threads);
/* ---- NUTS mass-matrix warmup (generic_nuts.rs:33-359, 897-921) ----
 * GenericNUTS::new_with_mass_matrix: Welford windows during warm-up, the
 * diagonal or dense metric, the probe + find_reasonable_epsilon re-start
 * after each update. The state persists across runs. */
typedef struct or_mass_cfg {
  int mode; /* 0 none, 1 diagonal, 2 dense (dense_max_dim already applied) */
  int64_t start_buffer, end_buffer, initial_window;
  double regularize, jitter;
  int form; /* NUTS arithmetic: 0 the engine's (the kernels, bitwise), 1 the reference's op
             * structure (generic_nuts.rs:227-276, 1343-1418: fresh M^-1 products with two
             * roundings, left-to-right kinetic sums and U-turn dots; with mode 0 the
             * identity metric's) */
} or_mass_cfg;
typedef struct or_mass_state {
  int32_t* kind;     /* [C]: 0 identity, 1 diagonal, 2 dense */
  void* dinv;        /* [C][D] T: diagonal inverse */
  void* dsqrt;       /* [C][D] T: diagonal sqrt */
  void* minv;        /* [C][D][D] T: dense inverse (mode 2) */
  void* mchol;       /* [C][D][D] T: dense Cholesky factor (mode 2) */
  int64_t sched[2];  /* next_window_end, window_len (MassMatrixWarmup::new, :141-151) */
} or_mass_state;
/* MassMatrixWarmup::new's schedule and identity for every chain */
void or_mass_state_init(const or_mass_cfg* cfg, int64_t C, int D, int dtype_is_f64, or_mass_state* st);
int or_nuts_mass_run_d(const or_target* t, int lanes, int elems, int64_t C, int D, double* q,
                       double* eps, double* eps_bar, double* h_bar, double* mu, double target_accept,
                       int max_depth, uint64_t seed, uint64_t init_step, uint32_t chain_offset,
                       int64_t n_collect, int64_t n_discard, int progress, double* samples,
                       int64_t* accepts, int64_t* n_leapfrog, const or_mass_cfg* cfg,
                       or_mass_state* ms, int threads);
int or_nuts_mass_run_f(const or_target* t, int lanes, int elems, int64_t C, int D, float* q,
                       float* eps, float* eps_bar, float* h_bar, float* mu, double target_accept,
                       int max_depth, uint64_t seed, uint64_t init_step, uint32_t chain_offset,
                       int64_t n_collect, int64_t n_discard, int progress, float* samples,
                       int64_t* accepts, int64_t* n_leapfrog, const or_mass_cfg* cfg,
                       or_mass_state* ms, int threads);
/* A trajectory of n_leap leapfrogs under a dense metric M^-1 = inv [D][D]
 * from (q, p), in either form: 0 the engine's (M^-1 p and M^-1 g carried by
 * linearity, fma-chain products, canonical-order kinetic sum), 1 the
 * reference's leapfrog_with_mass / kinetic (generic_nuts.rs:1396-1418,
 * 227-276). q, p are updated in place; vel = M^-1 p at the end (form 0 the
 * carried value, form 1 a fresh product); out[0] = logp, out[1] = kinetic.
 * Returns 0 on success. */
int or_dense_traj_d(const or_target* t, int lanes, int elems, int D, const double* inv, double* q,
                    double* p, double eps, int n_leap, int form, double* vel, double* out);
int or_dense_traj_f(const or_target* t, int lanes, int elems, int D, const float* inv, float* q,
                    float* p, double eps, int n_leap, int form, float* vel, float* out);
/* the reference's MassMatrix unit tests (generic_nuts.rs:1427-1489):
 * diagonal_from_var -> kinetic / inv_mul; dense_from_cov -> inv_mul;
 * RunningCov + maybe_update_mass_matrix (diagonal). Return 0 on success. */
int or_mass_diag_kat(const double* var, int D, double jitter, const double* p, double* ke,
                     double* inv_mul_out);
int or_mass_dense_kat(const double* cov, int D, double jitter, const double* p, double* inv_mul_out);
int or_mass_warmup_diag_kat(const double* xs, int n, int D, double reg, double jitter, double* inv,
                            double* sqrt_out);
double or_find_reasonable_epsilon_d(const or_target* t, int lanes, int elems, const double* q,
                                    const double* p);
/* build_tree (generic_nuts.rs:1105-1341), identity mass; out vectors [dim]:
 * qm pm gm qp pp gp qprime gprime; scalars logp_prime, n, s, alpha, n_alpha.
 * merge uniforms come from (seed, chain, step, MRG, counter). */
void or_build_tree_d(const or_target* t, int lanes, int elems, const double* q, const double* p,
                     const double* g, double logu, int v, int j, double eps, double joint0,
                     uint64_t seed, uint32_t chain, uint64_t step, double* out_vecs,
                     double* out_scalars);

/* ---- diagnostics: stats.rs (f32, the reference's arithmetic) ---- */
void or_split_rhat_ess(const float* x, int64_t C, int64_t N, int64_t P, float* rhat, float* ess);
void or_split_rhat_ess_mt(const float* x, int64_t C, int64_t N, int64_t P, float* rhat, float* ess,
                          int nthreads);
void or_autocov_bf(const float* x, int64_t n, int64_t d, float* out);
void or_autocov_fft(const float* x, int64_t n, int64_t d, float* out);
/* MultiChainTracker: steps [nsteps][C][P] -> rhat [P] (stats.rs:199-339) */
void or_mct_rhat(const float* steps, int64_t nsteps, int64_t C, int64_t P, float* rhat);
float or_mct_p_accept(const float* steps, int64_t nsteps, int64_t C, int64_t P);
void or_ct_init(int64_t C, int64_t P, const float* x0, float* p_accept, float* last, float* mean,
                float* msq);
void or_ct_step(int64_t C, int64_t P, uint64_t n_after, const float* x, float* p_accept, float* last,
                float* mean, float* msq);
void or_collect_rhat(int64_t C, int64_t P, uint64_t n_steps, const float* mean, const float* msq,
                     float* rhat);

#ifdef __cplusplus
}
#endif
#endif
