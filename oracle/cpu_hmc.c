/*
 * cpu_hmc.c — CPU BASELINE (benchmark infrastructure only; never linked into
 * the product, only bench.py's cpu_baseline leg loads it).
 *
 * The reference's batched HMC step on the CPU, with the reference's
 * operation structure: BatchedGenericHMC::step (batched_hmc.rs:129-163) and
 * its leapfrog (batched_hmc.rs:166-190) as one pass per BatchVector op over a
 * [chains x dim] block (euclidean.rs:392-394 add_scaled_assign, 464-472
 * kinetic_energy, 474-482 masked_assign, 527-533 accept_mask), with the L + 2
 * target evaluations per transition the reference makes (batched_hmc.rs:138,
 * 169, 182), per-chain sums left to right (ndarray sum_dim), the RosenbrockND
 * log-density and its gradient (distributions.rs:544-554; the gradient in
 * closed form, what burn autodiff computes). Threads own contiguous chain
 * blocks, like rayon's par_iter over chains (core.rs:221-225).
 *
 * Built with gcc -O3 -march=native (oracle/Makefile): the fastest faithful
 * CPU restatement here, not a bit-matching one -- its momenta and accept
 * uniforms come from its own xoshiro256++ streams (the reference's SmallRng
 * family) through Box-Muller with libm, not the engine's Philox spec.
 */
#include <math.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef struct {
  uint64_t s[4];
} xo256;

static inline uint64_t rotl(uint64_t x, int k) { return (x << k) | (x >> (64 - k)); }
static inline uint64_t xo_next(xo256* r) {  /* xoshiro256++ (rand 0.9 SmallRng on 64-bit) */
  const uint64_t result = rotl(r->s[0] + r->s[3], 23) + r->s[0];
  const uint64_t t = r->s[1] << 17;
  r->s[2] ^= r->s[0];
  r->s[3] ^= r->s[1];
  r->s[1] ^= r->s[2];
  r->s[0] ^= r->s[3];
  r->s[2] ^= t;
  r->s[3] = rotl(r->s[3], 45);
  return result;
}
static void xo_seed(xo256* r, uint64_t seed) {  /* splitmix64 expansion */
  for (int i = 0; i < 4; ++i) {
    uint64_t z = (seed += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    r->s[i] = z ^ (z >> 31);
  }
}
static inline float xo_unif(xo256* r) { return (float)(xo_next(r) >> 40) * 5.9604644775390625e-08f; }

typedef struct {
  float* q;
  int64_t c0, c1;
  int D, L;
  float eps;
  int64_t n_steps;
  uint64_t seed;
  int64_t* accepts;
} job;

/* logp_and_grad over a block: RosenbrockND a = 1, b = 100 */
static void rosen_block(const float* x, float* g, float* lp, int64_t nb, int D) {
  const float a = 1.0f, b = 100.0f;
  for (int64_t c = 0; c < nb; ++c) {
    const float* xc = x + c * D;
    float* gc = g + c * D;
    float s = 0.0f;
    for (int i = 0; i < D; ++i) gc[i] = 0.0f;
    for (int i = 0; i + 1 < D; ++i) {
      const float t = xc[i + 1] - xc[i] * xc[i];
      const float am = a - xc[i];
      s += b * t * t + am * am;
      gc[i] += 4.0f * b * xc[i] * t + 2.0f * am;
      gc[i + 1] -= 2.0f * b * t;
    }
    lp[c] = -s;
  }
}

static void add_scaled(float* x, const float* y, float alpha, int64_t n) {
  for (int64_t i = 0; i < n; ++i) x[i] = x[i] + y[i] * alpha;
}

static void kinetic(const float* p, float* ke, int64_t nb, int D) {
  for (int64_t c = 0; c < nb; ++c) {
    float s = 0.0f;
    for (int i = 0; i < D; ++i) s += p[c * D + i] * p[c * D + i];
    ke[c] = s * 0.5f;
  }
}

static void* run_block(void* arg) {
  job* j = (job*)arg;
  const int D = j->D;
  const int64_t nb = j->c1 - j->c0, n = nb * D;
  float* q = j->q + j->c0 * D;
  float *p = malloc(4 * n), *q1 = malloc(4 * n), *p1 = malloc(4 * n), *g = malloc(4 * n);
  float *lp0 = malloc(4 * nb), *lp1 = malloc(4 * nb), *ke0 = malloc(4 * nb), *ke1 = malloc(4 * nb);
  xo256 r;
  xo_seed(&r, j->seed ^ ((uint64_t)j->c0 * 0xD1342543DE82EF95ull));
  const float half = 0.5f * j->eps;
  for (int64_t st = 0; st < j->n_steps; ++st) {
    /* 1. momentum (fill_random_normal), Box-Muller pairs */
    for (int64_t i = 0; i < n; i += 2) {
      const float u1 = 1.0f - xo_unif(&r), u2 = xo_unif(&r);
      const float rr = sqrtf(-2.0f * logf(u1));
      p[i] = rr * cosf(6.2831853f * u2);
      if (i + 1 < n) p[i + 1] = rr * sinf(6.2831853f * u2);
    }
    kinetic(p, ke0, nb, D);             /* 2 */
    rosen_block(q, g, lp0, nb, D);      /* 3 */
    memcpy(q1, q, 4 * n);               /* 4 */
    memcpy(p1, p, 4 * n);
    rosen_block(q1, g, lp1, nb, D);     /* 5: leapfrog */
    for (int l = 0; l < j->L; ++l) {
      add_scaled(p1, g, half, n);
      add_scaled(q1, p1, j->eps, n);
      rosen_block(q1, g, lp1, nb, D);
      add_scaled(p1, g, half, n);
    }
    kinetic(p1, ke1, nb, D);            /* 6 */
    for (int64_t c = 0; c < nb; ++c) {  /* 7-9 */
      const float la = (lp1[c] - lp0[c]) + (ke0[c] - ke1[c]);
      const float lu = logf(xo_unif(&r));
      if (la >= lu) {
        memcpy(q + c * D, q1 + c * D, 4 * D);
        if (j->accepts) j->accepts[j->c0 + c] += 1;
      }
    }
  }
  free(p); free(q1); free(p1); free(g); free(lp0); free(lp1); free(ke0); free(ke1);
  return NULL;
}

/* n_steps transitions of C chains x D (RosenbrockND f32), q [C][D] in place */
int cpu_hmc_rosenbrock_f32(float* q, int64_t C, int D, double eps, int L, int64_t n_steps, uint64_t seed,
                           int threads, int64_t* accepts) {
  if (C < 1 || D < 2 || L < 0 || threads < 1) return 1;
  if (threads > C) threads = (int)C;
  pthread_t* th = malloc(sizeof(pthread_t) * threads);
  job* jobs = malloc(sizeof(job) * threads);
  for (int t = 0; t < threads; ++t) {
    jobs[t] = (job){q, C * t / threads, C * (t + 1) / threads, D, L, (float)eps, n_steps, seed, accepts};
    pthread_create(&th[t], NULL, run_block, &jobs[t]);
  }
  for (int t = 0; t < threads; ++t) pthread_join(th[t], NULL);
  free(th);
  free(jobs);
  return 0;
}
