// Host-side sanitizer harness for the native runtime ("AddressSanitizer-enabled
// host builds").  Compiles csrc/cpu/{cpu_adam,loader}.cpp WITHOUT their pybind11 module and
// drives them from main() so the binary can be built with -fsanitize=address,undefined or
// -fsanitize=thread (GPU sanitizers are not available on the pool; the HIP kernels are
// covered by the GPU numerics tests).  Exit code 0 = every check passed and the sanitizer
// reported nothing (sanitizer reports abort with a non-zero code).
#define LIPA_SANITIZER_HARNESS 1
#include "../../llm_in_practise_amd/csrc/cpu/cpu_adam.cpp"
#include "../../llm_in_practise_amd/csrc/cpu/loader.cpp"

#include <cstdio>
#include <set>

#define CHECK(c)                                                 \
  do {                                                           \
    if (!(c)) {                                                  \
      std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
      return 1;                                                  \
    }                                                            \
  } while (0)

static int test_adamw() {
  const int64_t n = 10007;  // odd size: exercises the vector-loop remainder
  auto p = torch::randn({n}), g = torch::randn({n}), m = torch::zeros({n}), v = torch::zeros({n});
  auto pb = torch::empty({n}, torch::kBFloat16);
  auto p_ref = p.clone(), m_ref = m.clone(), v_ref = v.clone();
  for (int64_t step = 1; step <= 3; ++step) {
    adamw_step(p, g, m, v, 1e-2, 0.9, 0.999, 1e-8, 0.01, step, 0.5, pb);
    auto gs = g * 0.5;
    m_ref = 0.9 * m_ref + 0.1 * gs;
    v_ref = 0.999 * v_ref + 0.001 * gs * gs;
    const double bc1 = 1 - std::pow(0.9, step), bc2 = 1 - std::pow(0.999, step);
    p_ref = p_ref * (1 - 1e-2 * 0.01) - (1e-2 / bc1) * m_ref / ((v_ref / bc2).sqrt() + 1e-8);
  }
  CHECK(torch::allclose(p, p_ref, 1e-5, 1e-6));
  CHECK(torch::allclose(pb.to(torch::kFloat), p, 1e-2, 1e-2));
  const double ss = sum_squares(g), ss_ref = (g.to(torch::kDouble) * g.to(torch::kDouble)).sum().item<double>();
  CHECK(std::abs(ss - ss_ref) <= 1e-6 * ss_ref);
  return 0;
}

static int test_loader() {
  const int64_t block = 16, batch = 3, world = 2;
  auto toks = torch::arange(0, 17 * 40, torch::kLong);  // 40 blocks of block+1 tokens
  std::set<int64_t> seen;
  for (int64_t r = 0; r < world; ++r) {
    TokenBlockLoader ld(toks, block, batch, r, world, 7, true, 2, false);
    CHECK(ld.steps_per_epoch() == 40 / world / batch);
    for (int64_t s = 0; s < ld.steps_per_epoch(); ++s) {
      auto xy = ld.next();
      CHECK(xy[0].size(0) == batch && xy[0].size(1) == block);
      CHECK(torch::equal(xy[0].narrow(1, 1, block - 1), xy[1].narrow(1, 0, block - 1)));
      for (int64_t b = 0; b < batch; ++b) {
        const int64_t first = xy[0][b][0].item<int64_t>();
        CHECK(first % 17 == 0);
        CHECK(seen.insert(first / 17).second);  // ranks never share a block within an epoch
      }
    }
    CHECK(ld.position().first == 1 && ld.position().second == 0);
  }
  // resume determinism: a loader restarted at (epoch 1, cursor 2) reproduces the same batch
  TokenBlockLoader a(toks, block, batch, 0, 1, 3, true, 4, false);
  std::vector<torch::Tensor> want;
  for (int64_t s = 0; s < a.steps_per_epoch() + 3; ++s) want = a.next();
  TokenBlockLoader b(toks, block, batch, 0, 1, 3, true, 4, false);
  b.start_epoch(1, 2);
  CHECK(torch::equal(b.next()[0], want[0]));
  // destruction while the producer is blocked on a full prefetch ring, repeatedly
  for (int i = 0; i < 20; ++i) {
    TokenBlockLoader c(toks, block, batch, 0, 1, i, true, 1, false);
    if (i % 2) c.next();
  }
  return 0;
}

int main() {
  torch::manual_seed(0);
  if (int rc = test_adamw()) return rc;
  if (int rc = test_loader()) return rc;
  std::printf("sanitize_host: all checks passed\n");
  return 0;
}
