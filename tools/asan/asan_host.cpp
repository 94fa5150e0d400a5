// asan_host.cpp — AddressSanitizer driver for libgmcmc's host code (SURVEY.md
// section 5: ASan/UBSan builds of the C++ host). Runs without a GPU: every
// call below either validates its arguments or parses host memory before it
// would touch the device, and must do so without an out-of-bounds access,
// returning GM_EINVAL (or GM_EHIP where a GPU would be needed).
//
// Built by tools/asan/Makefile against libgmcmc_asan.so (the host sources
// compiled with -Xarch_host -fsanitize=address,undefined and GM_HOST_TEST).
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#include "../../include/gmcmc.h"

extern "C" {
gm_sampler* gm_test_sampler(int kind, int dtype, long long C, int D, int mass_mode);
void gm_test_sampler_free(gm_sampler* s);
uint64_t gm_test_state_header(gm_sampler* s, void* out);
}

static int fails = 0;
#define EXPECT(cond, what)                                   \
  do {                                                       \
    if (!(cond)) {                                           \
      std::printf("FAIL %s (line %d)\n", what, __LINE__);    \
      ++fails;                                               \
    }                                                        \
  } while (0)

static void state_blobs() {
  std::mt19937_64 rng(7);
  // kinds: 1 HMC, 2 MH, 3 NUTS (mass 0, 1, 2)
  const int cases[][3] = {{1, 0, 0}, {2, 1, 0}, {3, 1, 0}, {3, 0, 1}, {3, 1, 2}};
  for (auto& k : cases) {
    gm_sampler* s = gm_test_sampler(k[0], k[1], 7, 5, k[2]);
    uint64_t need = 0;
    EXPECT(gm_state_size(s, &need) == GM_OK && need > 64, "state size");
    std::vector<unsigned char> blob(need);
    const uint64_t hb = gm_test_state_header(s, blob.data());
    for (uint64_t i = hb; i < need; ++i) blob[i] = (unsigned char)rng();
    // every truncation is rejected before any state is touched
    for (uint64_t len = 0; len < need; len += 1 + len / 7) {
      std::vector<unsigned char> t(blob.begin(), blob.begin() + (long)len);  // exact-size heap copy
      EXPECT(gm_state_load(s, t.empty() ? (const void*)"" : t.data(), len) == GM_EINVAL, "truncated blob");
    }
    // corrupt headers: random bit flips anywhere in the header
    for (int r = 0; r < 2000; ++r) {
      std::vector<unsigned char> t(blob);
      const int nflip = 1 + (int)(rng() % 4);
      for (int f = 0; f < nflip; ++f) t[rng() % hb] ^= (unsigned char)(1u << (rng() % 8));
      const int rc = gm_state_load(s, t.data(), t.size());
      EXPECT(rc == GM_EINVAL || rc == GM_EHIP || rc == GM_OK, "corrupt header status");
    }
    // random garbage of every small length
    for (int len = 0; len < 512; ++len) {
      std::vector<unsigned char> t((size_t)len + 1);
      for (auto& c : t) c = (unsigned char)rng();
      EXPECT(gm_state_load(s, t.data(), (uint64_t)len) == GM_EINVAL, "garbage blob");
    }
    gm_test_sampler_free(s);
  }
}

static void gauss_from_cov() {
  std::mt19937_64 rng(3);
  std::normal_distribution<double> nd;
  for (int dim = 1; dim <= 9; ++dim) {
    std::vector<double> a((size_t)dim * dim), cov((size_t)dim * dim), prec((size_t)dim * dim);
    for (auto& v : a) v = nd(rng);
    for (int i = 0; i < dim; ++i)
      for (int j = 0; j < dim; ++j) {
        double s = i == j ? 1.0 : 0.0;
        for (int k = 0; k < dim; ++k) s += a[(size_t)i * dim + k] * a[(size_t)j * dim + k];
        cov[(size_t)i * dim + j] = s;
      }
    double nc = 0;
    EXPECT(gm_gauss_from_cov(dim, cov.data(), prec.data(), &nc) == GM_OK, "spd covariance");
    cov[0] = -1.0;  // not positive definite
    EXPECT(gm_gauss_from_cov(dim, cov.data(), prec.data(), &nc) == GM_EINVAL, "non-pd covariance");
    cov[0] = 0.0 / 0.0;
    EXPECT(gm_gauss_from_cov(dim, cov.data(), prec.data(), &nc) == GM_EINVAL, "nan covariance");
  }
  double nc;
  EXPECT(gm_gauss_from_cov(0, nullptr, nullptr, &nc) == GM_EINVAL, "dim 0");
  EXPECT(gm_gauss_from_cov(3, nullptr, nullptr, &nc) == GM_EINVAL, "null cov");
}

static void argument_checks() {
  gm_target t;
  std::memset(&t, 0, sizeof(t));
  t.kind = GM_TARGET_ROSENBROCK;
  t.dim = 4;
  t.a = 1;
  t.b = 100;
  std::vector<float> x(16, 0.5f);
  gm_sampler* s = nullptr;
  EXPECT(gm_hmc_create(&t, GM_F32, 0, 4, x.data(), 0.01, 5, 0, &s) == GM_EINVAL, "zero chains");
  EXPECT(gm_hmc_create(&t, GM_F32, 4, 4, nullptr, 0.01, 5, 0, &s) == GM_EINVAL, "null init");
  EXPECT(gm_hmc_create(&t, (gm_dtype)9, 4, 4, x.data(), 0.01, 5, 0, &s) == GM_EINVAL, "bad dtype");
  EXPECT(gm_hmc_create(&t, GM_F32, 4, 5, x.data(), 0.01, 5, 0, &s) == GM_EINVAL, "dim mismatch");
  EXPECT(gm_hmc_create(&t, GM_F32, 4, 4, x.data(), 0.01, -1, 0, &s) == GM_EINVAL, "negative L");
  EXPECT(gm_nuts_create(&t, GM_F32, 4, 4, x.data(), 0.8, 99, 0, &s) == GM_EINVAL, "max_depth");
  EXPECT(gm_mh_create(&t, GM_F32, 4, 4, x.data(), -1.0, 0, &s) == GM_EINVAL, "proposal std");
  EXPECT(gm_hmc_create(&t, GM_F32, 4, 4, x.data(), 0.01, 5, (1LL << 32), &s) == GM_EINVAL, "chain offset");
  float r[4], e[4];
  EXPECT(gm_split_rhat_ess(x.data(), GM_F32, 4, 1, 4, r, e) == GM_EINVAL, "one draw");
  EXPECT(gm_split_rhat_ess(nullptr, GM_F32, 4, 4, 1, r, e) == GM_EINVAL, "null sample");
  EXPECT(gm_copy_samples(nullptr, 0, nullptr) == GM_EINVAL, "null sampler");
  EXPECT(gm_step(nullptr) == GM_EINVAL, "null step");
  EXPECT(gm_bv_add_scaled_assign(GM_F32, -1, nullptr, nullptr, 1.0) == GM_EINVAL, "bv negative n");
  EXPECT(gm_bv_dot(GM_F32, 3, nullptr, nullptr, nullptr) == GM_EINVAL, "bv dot null");
  // host-only: initial positions into an exactly sized buffer
  for (int n = 0; n < 5; ++n)
    for (int d = 0; d < 7; ++d) {
      std::vector<double> out((size_t)n * d + 0);
      EXPECT(gm_init_positions(42, n, d, GM_F64, out.empty() ? nullptr : out.data()) == GM_OK, "init");
    }
}

int main() {
  state_blobs();
  gauss_from_cov();
  argument_checks();
  std::printf("%s\n", fails ? "ASAN HOST CHECKS FAILED" : "asan host checks ok");
  return fails ? 1 : 0;
}
