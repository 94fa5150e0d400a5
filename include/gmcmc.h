/*
 * gmcmc.h — C ABI of the MI355X many-chain HMC / NUTS / Metropolis-Hastings
 * engine (libgmcmc.so, HIP kernels for gfx950).
 *
 * This is the drop-in boundary for the hot path of SauersML/general-mcmc
 * (reference snapshot under /root/reference). Each entry point names the
 * reference interface it replaces. Plain pointers and sizes only; no torch
 * types. All functions return GM_OK (0) or an error code; the message of the
 * last error on the calling thread is available from gm_last_error(). No
 * function aborts the process: the reference's panics (shape asserts,
 * euclidean.rs:116-120/432-437, distributions.rs:267) become GM_EINVAL.
 *
 * Data layout conventions
 *   - host initial positions / host outputs are row-major, reference layout:
 *     init [n_chains][dim]           (hmc.rs:119-124, Vec<Vec<T>> flattened)
 *     samples [n_chains][n_collect][dim] (hmc.rs:179-180 stack+permute)
 *   - device-resident samples (gm_*_run_device) are [n_collect][n_chains][dim]
 *     (one contiguous [C,D] slab per collected step, as BatchedGenericHMC::
 *     run_positions returns one Tensor<B,2> per step, batched_hmc.rs:115-123).
 *   - element type is given by gm_dtype (f32 or f64) everywhere.
 *
 * Threading: one sampler must not be used from two threads at once
 * (&mut self in the reference, hmc.rs:164). Distinct samplers may run
 * concurrently; each owns a HIP stream on the device that was current
 * (gm_set_device) when it was created.
 */
#ifndef GMCMC_H
#define GMCMC_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- status codes ---------------------------------------------------- */
#define GM_OK 0
#define GM_EINVAL 1 /* bad argument / shape (reference: assert_eq!/expect panics) */
#define GM_EHIP 2   /* HIP runtime error */
#define GM_ENOMEM 3 /* device allocation failed */
#define GM_ERCCL 4  /* RCCL error */
#define GM_ESTATE 5 /* call not valid in the sampler's current state */

/* GM_DTYPE_INT_: not a dtype; it widens the enum's value range to int, so a
 * caller passing any other integer gets GM_EINVAL instead of undefined
 * behaviour in the C++ implementation (found by the UBSan host build). */
typedef enum gm_dtype { GM_F32 = 0, GM_F64 = 1, GM_DTYPE_INT_ = 0x7fffffff } gm_dtype;

/* ---- targets (replaces the user-implemented traits) ---------------------
 * BatchedGradientTarget::unnorm_logp_batch   distributions.rs:67-78
 * GradientTarget::unnorm_logp(+_and_grad)     distributions.rs:80-90
 * Target::unnorm_logp                         distributions.rs:107-110
 * Built-in targets get analytic gradients instead of burn autodiff
 * (hmc.rs:42-61).                                                          */
typedef enum gm_target_kind {
  GM_TARGET_ROSENBROCK = 1, /* RosenbrockND (a=1,b=100) distributions.rs:535-555;
                               Rosenbrock2D{a,b} distributions.rs:495-530    */
  GM_TARGET_ISO_GAUSS = 2,  /* IsotropicGaussian as Target, distributions.rs:398-406 */
  GM_TARGET_GAUSS = 3,      /* DiffableGaussian2D distributions.rs:215-320 generalised
                               to D dims: logp = norm_const - 0.5 (x-mu)^T P (x-mu),
                               P = Sigma^-1 supplied row-major; also Gaussian2D as a
                               Target (distributions.rs:193-207) with norm_const = 0 */
  GM_TARGET_CUSTOM = 4      /* user code (the reference's Target / GradientTarget
                               traits, distributions.rs:67-110): HIP source defining
                                 template <class T> __device__
                                 T gm_logp_grad(const T* x, T* g, const T* params);
                               for one chain (x, g of length GM_DIM, a macro = dim),
                               compiled at run time (hiprtc) into the sampler kernels;
                               one chain per lane, dim <= 256 */
} gm_target_kind;

typedef struct gm_target {
  int32_t kind;          /* gm_target_kind */
  int32_t reserved;
  int64_t dim;           /* must equal the sampler's dim */
  double a, b;           /* ROSENBROCK: logp = -sum_i [ b (x_{i+1}-x_i^2)^2 + (a-x_i)^2 ] */
  double std;            /* ISO_GAUSS: logp = -0.5 * sum x^2 / std^2 */
  const double* mean;    /* GAUSS: [dim] */
  const double* prec;    /* GAUSS: [dim*dim] row-major inverse covariance */
  double norm_const;     /* GAUSS: additive constant */
  const char* source;    /* CUSTOM: HIP source of gm_logp_grad (copied) */
  const double* params;  /* CUSTOM: [n_params] copied to the device in the sampler dtype */
  int64_t n_params;      /* CUSTOM: passed to gm_logp_grad as `params` */
} gm_target;

/* Compile a CUSTOM target's source for the sampler kernels without running it
 * (kind: 1 HMC, 2 MH, 3 NUTS, 0 log-density/gradient); GM_EINVAL with the
 * compiler log in gm_last_error() when it does not compile. */
int gm_custom_target_check(const char* source, gm_dtype dtype, int64_t dim, int32_t kind);

/* DiffableGaussian2D::new (distributions.rs:229-253) generalised: from a mean
 * and covariance compute the precision matrix and norm_const =
 * -(dim ln(2 pi) + ln|Sigma|)/2. For dim == 2 the closed-form 2x2 inverse of
 * the reference is used bit-for-bit; otherwise a Cholesky factorisation. */
int gm_gauss_from_cov(int64_t dim, const double* cov, double* prec_out, double* norm_const_out);

/* Evaluate a target on host-provided points (device compute): logp [n],
 * grad [n][dim] (grad may be NULL). Replaces logp_and_grad
 * (batched_hmc.rs:18-22, hmc.rs:42-61). */
int gm_target_logp_grad(const gm_target* target, gm_dtype dtype, int64_t n, const void* x,
                        void* logp_out, void* grad_out);

/* Initial positions: n x dim iid N(0,1) from the engine's counter-based
 * stream keyed by `seed` (core.rs:434-475 init / init_det / init_with_seed
 * analogue: same distribution and row-by-row meaning, not the same numbers,
 * see gm_rng.h). Host-side; out is [n][dim] of dtype. */
int gm_init_positions(uint64_t seed, int64_t n, int64_t dim, gm_dtype dtype, void* out);
/* Rows [row0, row0 + n) of the same stream (a shard's block of a global
 * start: rank r of a sharded run takes rows [offset_r, offset_r + n_r)). */
int gm_init_positions_rows(uint64_t seed, int64_t row0, int64_t n, int64_t dim, gm_dtype dtype, void* out);

/* ---- device / errors ------------------------------------------------ */
const char* gm_last_error(void);

/* "src:<digest>": the digest of the sources this library was built from
 * (tools/source_digest.py over csrc/, this header and the Makefile); the
 * Python layer refuses a library whose digest differs from its tree's. */
const char* gm_build_info(void);
int gm_device_count(int* count);
/* Select the calling thread's device. Called before the device is first used,
 * it also makes the thread's host waits spin (hipDeviceScheduleSpin): run
 * completion is then seen microseconds sooner. */
int gm_set_device(int device);
int gm_device_synchronize(void);

/* ---- samplers ----------------------------------------------------------- */
typedef struct gm_sampler gm_sampler;

/* HMC::new (hmc.rs:113-134) / BatchedGenericHMC::new (batched_hmc.rs:62-84).
 * init: host [n_chains][dim] of dtype. chain_offset: global id of chain 0
 * (used to key the per-chain random streams; 0 unless chains are sharded
 * across processes/GPUs). */
int gm_hmc_create(const gm_target* target, gm_dtype dtype, int64_t n_chains, int64_t dim,
                  const void* init, double step_size, int64_t n_leapfrog,
                  int64_t chain_offset, gm_sampler** out);

/* MetropolisHastings::new (metropolis_hastings.rs:151-161) with an
 * IsotropicGaussian proposal of standard deviation proposal_std
 * (distributions.rs:349-390), driven like ChainRunner::run (core.rs:219-229). */
int gm_mh_create(const gm_target* target, gm_dtype dtype, int64_t n_chains, int64_t dim,
                 const void* init, double proposal_std, int64_t chain_offset,
                 gm_sampler** out);

/* NUTS::new (nuts.rs:156-180) -> GenericNUTS::new (generic_nuts.rs:370-377):
 * identity mass matrix, dual-averaging step size (gamma .05, t0 10, kappa .75).
 * max_depth bounds the doubling loop (the reference has no bound,
 * generic_nuts.rs:782); pass 0 for the engine default (10). */
int gm_nuts_create(const gm_target* target, gm_dtype dtype, int64_t n_chains, int64_t dim,
                   const void* init, double target_accept_p, int32_t max_depth,
                   int64_t chain_offset, gm_sampler** out);

/* set_seed: hmc.rs:143-148, generic_nuts.rs:550-556, metropolis_hastings.rs:189-197.
 * Resets the sampler's transition counter so a re-seeded sampler replays. */
int gm_set_seed(gm_sampler* s, uint64_t seed);

/* One transition of every chain (HMC::step hmc.rs:316-318 /
 * BatchedGenericHMC::step batched_hmc.rs:129-163 / MHMarkovChain::step
 * metropolis_hastings.rs:306-318 / GenericNUTSChain::step generic_nuts.rs:755-925). */
int gm_step(gm_sampler* s);

/* run(n_collect, n_discard): hmc.rs:164-181, core.rs:219-229, nuts.rs:214-259.
 * out: host [n_chains][n_collect][dim] (may be NULL to skip the copy).
 * Step-count semantics follow the reference per sampler kind:
 *   HMC, MH: n_discard + n_collect transitions, every post-burn-in state kept;
 *   NUTS:    n_discard + n_collect - 1 transitions, row r = state after
 *            n_discard + r transitions (row 0 = start when n_discard == 0). */
int gm_run(gm_sampler* s, int64_t n_collect, int64_t n_discard, void* out);

/* run_positions (batched_hmc.rs:115-123): same transitions, samples stay on
 * the device as [n_collect][n_chains][dim]; *dev_samples is owned by the
 * sampler and valid until the next run/destroy. */
int gm_run_device(gm_sampler* s, int64_t n_collect, int64_t n_discard, const void** dev_samples);

/* NUTS::run_progress semantics (generic_nuts.rs:675-717): n_discard + n_collect
 * transitions, row r = state after n_discard + r + 1 transitions. Other
 * sampler kinds: identical to gm_run_device. */
int gm_run_device_progress(gm_sampler* s, int64_t n_collect, int64_t n_discard,
                           const void** dev_samples);

/* run_progress (hmc.rs:245-306, generic_nuts.rs:414-548, core.rs:251-403)
 * without the terminal UI: the transitions of gm_run_device_progress, samples
 * copied to host [n_chains][n_collect][dim] (out may be NULL), and the
 * device-side split R-hat / ESS of the collected draws (RunStats::from,
 * stats.rs:383-394) in rhat_out/ess_out [dim] (may be NULL; needs n_collect >= 2). */
int gm_run_progress(gm_sampler* s, int64_t n_collect, int64_t n_discard, void* out,
                    float* rhat_out, float* ess_out);

/* Copy the samples of the last run (device [n_collect][n_chains][dim]) to host
 * in the reference layout [n_chains][n_collect][dim]. n_rows must equal that
 * run's n_collect (the size of `out` in rows): GM_EINVAL otherwise, so a
 * buffer sized for an earlier, smaller run is never overrun. */
int gm_copy_samples(gm_sampler* s, int64_t n_rows, void* out);

/* A block of the last run's device samples, rows [row0, row0+n_rows) x
 * chains [chain0, chain0+n_chains), copied to the host as
 * [n_rows][n_chains][dim] (one strided copy): the streaming egress used by
 * the CSV / Arrow / Parquet writers (io/csv.rs, io/arrow.rs, io/parquet.rs) so that a sample larger than
 * host memory never has to exist there whole. */
int gm_copy_sample_block(gm_sampler* s, int64_t row0, int64_t n_rows, int64_t chain0, int64_t n_chains,
                         void* out);
/* positions() (hmc.rs:326-328): host [n_chains][dim]. */
int gm_get_positions(gm_sampler* s, void* out);
int gm_set_positions(gm_sampler* s, const void* in);

/* Per-chain count of accepted transitions since creation / set_seed
 * (the quantity behind MultiChainTracker::p_accept, stats.rs:238-269). */
int gm_get_accept_counts(gm_sampler* s, int64_t* out);

/* Per-chain count of leapfrog steps integrated since creation (HMC:
 * n_leapfrog per transition; NUTS: the tree sizes actually built; MH: 0). */
int gm_get_leapfrog_counts(gm_sampler* s, int64_t* out);

/* NUTS per-chain adaptation state: step size epsilon and epsilon_bar
 * (generic_nuts.rs:573-582). Pass NULL to skip either. */
int gm_nuts_get_step_size(gm_sampler* s, double* eps, double* eps_bar);

/* Mass-matrix warm-up, GenericNUTS::new_with_mass_matrix (generic_nuts.rs:
 * 33-65, 379-398): mode 0 none (NUTS::new), 1 diagonal, 2 dense (falls back
 * to diagonal when dim > dense_max_dim). During warm-up (m <= n_discard) the
 * positions inside the window (start_buffer < m < n_discard - end_buffer)
 * feed a Welford covariance; at each window end (initial_window, doubling
 * up to 400) the metric becomes (1-regularize)*cov + regularize (diagonal
 * floored at jitter), the step size is re-found from a probe momentum and
 * dual averaging restarts (:897-921, 948-997). Resets the metric to identity
 * and the window schedule to its start; call before the first run. A dense
 * metric runs on a one-wave layout: once the mode is accepted, a wide layout
 * (lanes > 64) is replaced by the default one, and restored when a later call
 * selects mode 0 or 1; on an error the layout is unchanged. */
int gm_nuts_set_mass_adaptation(gm_sampler* s, int32_t mode, int64_t start_buffer, int64_t end_buffer,
                                int64_t initial_window, double regularize, double jitter,
                                int64_t dense_max_dim);
/* The current metric: mode, per-chain kind [C] (0 identity, 1 diagonal,
 * 2 dense), diagonal inverse and sqrt [C][dim], dense inverse and Cholesky
 * factor [C][dim][dim] (mode 2). Any output may be NULL. */
/* Where a NUTS sampler keeps the levels of its subtree stack (the stored
 * left siblings of build_tree's recursion): the first `levels` in LDS, deeper
 * ones in HBM; -1 (the default) puts as many in LDS as fit next to the
 * target's staging area. Results are identical for every value. */
int gm_nuts_set_lds_levels(gm_sampler* s, int32_t levels);

/* Where a dense-metric NUTS sampler (layout 16 x 2, dim <= 32) keeps each
 * chain's M^-1 and Cholesky factor: minv_lds 1 (the default, also -1) the
 * packed lower triangles in LDS, which leaves room for 6 subtree-stack
 * levels on chip; 2 the full matrices when they fit next to the target's
 * staging (else packed: one stack level, ~10x the HBM traffic, ~2 % faster);
 * 0 global memory. chol_lds 1 also packs the Cholesky factor into LDS when
 * the packed M^-1 leaves room (default, also -1: 0). Every form gives
 * identical results (no reference counterpart: a placement choice of this
 * engine). */
int gm_nuts_set_dense_forms(gm_sampler* s, int32_t minv_lds, int32_t chol_lds);

/* The last NUTS launch's on-chip plan: plan[0] subtree-stack levels in LDS,
 * plan[1] M^-1 form (0 global, 1 packed, 2 full), plan[2] its LDS offset,
 * plan[3] Cholesky factor in LDS (0/1), plan[4] its offset, plan[5] 1 when
 * the launch ran the frozen-dense kernel (every chain's metric dense, no
 * warm-up window, the momentum pass on: GM_FROZEN_WAVES waves per SIMD).
 * The first min(cap, 6)
 * values are written to plan (cap >= 1); returns GM_OK. */
int gm_nuts_get_plan(gm_sampler* s, int32_t* plan, int32_t cap);

/* Where the NUTS transition momenta are drawn: on (default) in one parallel
 * pass per launch ahead of the tree kernel, into a [steps][C][D] buffer that
 * the sampler keeps for its later launches (at most 4 GiB and a quarter of
 * the device memory free when it grows; a launch it does not fit draws in the
 * kernel), off in the tree kernel at each transition start (switching it off
 * releases the buffer). With a dense metric the pass also applies it (the
 * momenta L z and their M^-1 L z, in a second [steps][C][D] buffer) for the
 * frozen-dense kernel, which needs it: with the pass off those launches run
 * the adaptive dense kernel. The same Philox/Box-Muller values and the same
 * sums either way (identical results); no reference counterpart. */
int gm_nuts_set_momentum_pass(gm_sampler* s, int32_t on);

int gm_nuts_get_mass(gm_sampler* s, int32_t* mode, int32_t* kind, void* dinv, void* dsqrt, void* minv,
                     void* mchol);

/* Lane layout the kernels use for this sampler: `lanes` lanes cooperate on
 * one chain, each holding `elems` consecutive coordinates. Per-chain sums
 * (kinetic energy, log-density) are reduced lane-sequentially then by an xor
 * butterfly over the lanes, which fixes the floating-point summation order. */
int gm_sampler_layout(gm_sampler* s, int32_t* lanes, int32_t* elems);
int gm_sampler_set_layout(gm_sampler* s, int32_t lanes, int32_t elems);

/* Device time (ms) of the sampling kernels launched by the last run, and the
 * number of launches (HIP events on the sampler's stream). */
int gm_sampler_last_run_stats(gm_sampler* s, double* kernel_ms, int64_t* launches);

/* Asynchronous runs (HMC and MH samplers; NUTS runs stay synchronous):
 * with on != 0, gm_run_device / gm_step return once the sampler's kernels
 * are enqueued on its stream instead of waiting for them. The caller then
 * waits with gm_sampler_synchronize or gm_device_synchronize before reading
 * the samples from another stream (the diagnostics, gm_memcpy_*); the
 * sampler's own calls (copies, positions, state) are ordered after the run
 * on its stream. A benchmark that brackets a run with device synchronizes
 * uses it to wait once instead of twice. */
int gm_sampler_set_async(gm_sampler* s, int32_t on);
int gm_sampler_synchronize(gm_sampler* s);

/* Transitions per kernel launch (state stays in registers inside a launch). */
int gm_sampler_set_steps_per_launch(gm_sampler* s, int64_t steps);

/* HMC leapfrog-loop unroll of the fused kernel: 0 (default) chosen by the
 * launch's waves per SIMD, or forced to 1, 2 or 4 (tests and measurements;
 * identical results in every form). No reference counterpart. */
int gm_sampler_set_unroll(gm_sampler* s, int32_t n);

/* Pre-size the device sample buffer for runs collecting up to n_collect
 * transitions, so that a later gm_run / gm_run_device does no device
 * allocation (the buffer only grows; hmc.rs:164-181 allocates its output on
 * every run). */
int gm_sampler_reserve(gm_sampler* s, int64_t n_collect);

/* Checkpoint / resume. The reference keeps a sampler's state only in the
 * object between run calls (batched_hmc.rs:40; generic_nuts.rs:573-582, 744)
 * and leaves checkpointing as a TODO (core.rs:177). gm_state_save writes that
 * state (positions, accept / leapfrog counts, seed and stream position; NUTS
 * step-size adaptation, metric and warm-up schedule) to a caller-owned host
 * buffer of gm_state_size bytes; gm_state_load restores it into a sampler
 * created with the same kind, dtype, n_chains, dim and chain_offset, which
 * then continues the same random streams bit for bit. */
int gm_state_size(gm_sampler* s, uint64_t* bytes);
int gm_state_save(gm_sampler* s, void* out, uint64_t bytes);
int gm_state_load(gm_sampler* s, const void* in, uint64_t bytes);

int gm_destroy(gm_sampler* s);

/* ---- diagnostics (stats.rs) ---------------------------------------------
 * split_rhat_mean_ess (stats.rs:439-450, Appendix B of SURVEY.md): returns
 * split R-hat = sqrt(W/V) (the reference's orientation, stats.rs:452-454) and
 * ESS per parameter, as f32, like the reference.
 * Host variant: sample is host [n_chains][n_draws][n_params] (reference
 * layout). Device variant: sample is a device pointer with explicit element
 * strides (chain, draw, param). */
int gm_split_rhat_ess(const void* sample, gm_dtype dtype, int64_t n_chains, int64_t n_draws,
                      int64_t n_params, float* rhat_out, float* ess_out);
int gm_split_rhat_ess_device(const void* dev_sample, gm_dtype dtype, int64_t n_chains,
                             int64_t n_draws, int64_t n_params, int64_t stride_chain,
                             int64_t stride_draw, int64_t stride_param, float* rhat_out,
                             float* ess_out);

/* ---- multi-GPU (one process per GPU, RCCL over xGMI) -------------------
 * Chains are sharded in contiguous blocks; sampling needs no communication.
 * The only exchange is an RCCL all-gather of per-split-chain summaries for
 * split-R-hat/ESS. */
typedef struct gm_comm gm_comm;
#define GM_UNIQUE_ID_BYTES 128
int gm_comm_get_unique_id(void* id_out /* GM_UNIQUE_ID_BYTES */);
int gm_comm_init(const void* id, int32_t nranks, int32_t rank, gm_comm** out);
int gm_comm_destroy(gm_comm* comm);
/* What RCCL itself reports for the communicator (ncclCommCount,
 * ncclCommUserRank, ncclCommCuDevice): the ranks the exchange really spans.
 * Any pointer may be NULL. */
int gm_comm_info(gm_comm* comm, int32_t* nranks, int32_t* rank, int32_t* device);
/* Same result on every rank: diagnostics of the union of all ranks' chains
 * (rank r holds global chains [offset_r, offset_r + n_chains_local)).
 * Every rank must pass the same (n_chains_local, n_draws, n_params, dtype).
 * The first call with a given shape on a communicator checks that with one
 * small all-gather (a mismatch is GM_EINVAL on every rank); later calls with
 * that shape go straight to the one grouped all-gather of the summaries. */
int gm_split_rhat_ess_dist(gm_comm* comm, const void* dev_sample, gm_dtype dtype,
                           int64_t n_chains_local, int64_t n_draws, int64_t n_params,
                           int64_t stride_chain, int64_t stride_draw, int64_t stride_param,
                           float* rhat_out, float* ess_out);
/* The same exchange with all R shards on the calling thread's device
 * (equal chain counts, same strides): shard r's summaries land where the
 * all-gather puts rank r's, and one final kernel reads them. Equals
 * split_rhat_mean_ess (stats.rs:439-450) of the concatenated chains, up to
 * summation order; one process driving several shards uses it, and it
 * checks the multi-rank assembly on a single GPU. */
int gm_split_rhat_ess_shards(const void* const* dev_shards, int32_t n_shards, gm_dtype dtype,
                             int64_t n_chains_per_shard, int64_t n_draws, int64_t n_params,
                             int64_t stride_chain, int64_t stride_draw, int64_t stride_param,
                             float* rhat_out, float* ess_out);

/* ---- run_progress with live statistics -------------------------------
 * The reference's run_progress draws progress bars fed by chain trackers:
 * HMC steps a MultiChainTracker with the current positions at most every
 * 500 ms and at the last step (hmc.rs:245-306); ChainRunner (MH) and NUTS
 * step a ChainTracker per chain after EVERY transition, burn-in included,
 * and report collect_rhat over the chains every second (core.rs:132-176,
 * 251-387; generic_nuts.rs:675-716). Here the trackers live on the device
 * (MH / NUTS: fused into the sampling kernels) and `cb`, when not NULL, is
 * called between launches at most every `interval_s` seconds and after the
 * last transition. The returned samples and R-hat/ESS are those of
 * gm_run_progress. */
typedef struct gm_progress {
  int64_t done;   /* transitions done (HMC: of the n_collect phase; MH/NUTS: of all) */
  int64_t total;  /* HMC: n_collect; MH/NUTS: n_discard + n_collect */
  float p_accept; /* HMC: MultiChainTracker::p_accept; MH/NUTS: mean over chains of
                     the ChainTracker acceptance EMA */
  float max_rhat; /* max over parameters of the tracker R-hat, NaN skipped
                     (stats.rs:139-161, 298-317) */
} gm_progress;
typedef void (*gm_progress_fn)(void* user, const gm_progress* info);
int gm_run_progress_cb(gm_sampler* s, int64_t n_collect, int64_t n_discard, void* out,
                       float* rhat_out, float* ess_out, gm_progress_fn cb, void* user,
                       double interval_s);
/* ChainTracker::stats of every chain after an MH / NUTS run_progress
 * (stats.rs:122-131): steps taken, p_accept [C], mean [C][dim], sm2 [C][dim]
 * (any output may be NULL). */
int gm_sampler_chain_stats(gm_sampler* s, uint64_t* n, float* p_accept, float* mean, float* sm2);

/* MultiChainTracker (stats.rs:199-339) over [n_chains][n_params] device
 * positions of either dtype. */
typedef struct gm_mct gm_mct;
int gm_mct_create(int64_t n_chains, int64_t n_params, gm_mct** out);
int gm_mct_step(gm_mct* t, const void* dev_positions, gm_dtype dtype);
/* p_accept, rhat [n_params] and max_rhat (any may be NULL) */
int gm_mct_stats(gm_mct* t, float* p_accept, float* rhat, float* max_rhat);
int gm_mct_destroy(gm_mct* t);

/* ---- granular BatchVector ops (tier 2 of the boundary) ----------------
 * The reference's plug-in seam is the BatchVector trait implemented for
 * Tensor<B,2> [n_chains, dim] (euclidean.rs:145-195, 358-534) plus
 * BatchedHamiltonianTarget::logp_and_grad (batched_hmc.rs:18-22). These
 * entry points are those operations on caller-held DEVICE buffers, so a
 * BatchVector implementation (or BatchedGenericHMC::step itself,
 * batched_hmc.rs:129-190) can be driven op by op. A step composed of them
 * equals the fused gm_step bit for bit: same Philox streams (momentum:
 * tag 2, accept: tag 3, keyed by global chain id and step), same rounding,
 * and per-chain sums in the canonical order of the default layout of `dim`.
 * Matrices are [n_chains][dim] row-major, energies [n_chains], masks
 * uint8 [n_chains]. Ops are enqueued in order on the device's null stream;
 * gm_device_synchronize waits for them. */
int gm_malloc(void** dev_ptr, size_t bytes);
int gm_free(void* dev_ptr);
int gm_memcpy_htod(void* dev_dst, const void* host_src, size_t bytes);
int gm_memcpy_dtoh(void* host_dst, const void* dev_src, size_t bytes);
/* assign (euclidean.rs:380-382): dev_dst = dev_src */
int gm_memcpy_dtod(void* dev_dst, const void* dev_src, size_t bytes);

/* kinetic_energy (euclidean.rs:464-472): ke[c] = (sum_j p[c,j]^2) * 0.5 */
int gm_bv_kinetic_energy(gm_dtype dtype, int64_t n_chains, int64_t dim, const void* p, void* ke);
/* masked_assign (euclidean.rs:474-482): x[c,:] = other[c,:] where mask[c] != 0 */
int gm_bv_masked_assign(gm_dtype dtype, int64_t n_chains, int64_t dim, void* x, const void* other,
                        const uint8_t* mask);
/* add_scaled_assign (euclidean.rs:392-394): x = x + other * alpha, two
 * roundings, alpha rounded to dtype first; n = number of elements */
int gm_bv_add_scaled_assign(gm_dtype dtype, int64_t n, void* x, const void* other, double alpha);
/* fill_random_normal (euclidean.rs:484-496): out[c,j] = momentum draw of
 * chain chain_offset+c, coordinate j, transition `step` under `seed` */
int gm_bv_fill_random_normal(gm_dtype dtype, int64_t n_chains, int64_t dim, void* out, uint64_t seed,
                             uint32_t chain_offset, uint64_t step);
/* sample_uniform (euclidean.rs:498-509): out[c] in [0,1), the accept draw */
int gm_bv_sample_uniform(gm_dtype dtype, int64_t n_chains, void* out, uint64_t seed,
                         uint32_t chain_offset, uint64_t step);
/* energy_sub / energy_add / energy_neg / energy_ln (euclidean.rs:511-525) */
int gm_bv_energy_sub(gm_dtype dtype, int64_t n, const void* a, const void* b, void* out);
int gm_bv_energy_add(gm_dtype dtype, int64_t n, const void* a, const void* b, void* out);
int gm_bv_energy_neg(gm_dtype dtype, int64_t n, const void* a, void* out);
int gm_bv_energy_ln(gm_dtype dtype, int64_t n, const void* a, void* out);
/* accept_mask (euclidean.rs:527-533): mask[c] = log_accept[c] >= ln_u[c]
 * (NaN -> 0) */
int gm_bv_accept_mask(gm_dtype dtype, int64_t n, const void* log_accept, const void* ln_u,
                      uint8_t* mask);
/* EuclideanVector's remaining in-place ops on a [n] device vector
 * (euclidean.rs:11-60): scale_assign x = x * alpha (:396-398); fill
 * (fill_zero / zeros_like with value 0); dot = sum of a*b over all elements
 * (:400-403) into a host double (T partials, fixed order). */
int gm_bv_scale_assign(gm_dtype dtype, int64_t n, void* x, double alpha);
int gm_bv_fill(gm_dtype dtype, int64_t n, void* x, double value);
int gm_bv_dot(gm_dtype dtype, int64_t n, const void* a, const void* b, double* out);

/* A built-in target resident on the device, for logp_and_grad on device
 * buffers (BatchedHamiltonianTarget, batched_hmc.rs:18-22; hmc.rs:42-61). */
typedef struct gm_bv_target gm_bv_target;
int gm_bv_target_create(const gm_target* target, gm_dtype dtype, gm_bv_target** out);
/* grad[c,:] = d logp / d x at x[c,:]; returns logp[c] (either output may be NULL) */
int gm_bv_logp_and_grad(gm_bv_target* t, int64_t n_chains, const void* x, void* grad, void* logp);
int gm_bv_target_destroy(gm_bv_target* t);
/* One leapfrog of n_chains chains with q, p, g ([C][D]) and logp ([C],
 * nullable) in device memory, updated in place: the loop body of
 * BatchedGenericHMC::leapfrog (batched_hmc.rs:166-190) -- add_scaled_assign
 * (euclidean.rs:392-394) of the half kick, the drift, logp_and_grad
 * (hmc.rs:42-61), the second half kick -- as one kernel. Bitwise the composed
 * ops. Built-in targets, dim <= 1024. */
int gm_bv_leapfrog(gm_bv_target* t, int64_t n_chains, void* q, void* p, void* g, void* logp,
                   double step_size);

#ifdef __cplusplus
}
#endif
#endif /* GMCMC_H */
