// gemm4w plain NT 256x256 over a set of shapes (argv: M N K splits ...) — per-K-tile cost and per-round fixed cost
// of the main loop, with the shipped epilogue or (-DLIPA_G4W_NOSTORE) no stores.  Min of 5 x 10 launches.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "gemm4w_kernel.h"

__global__ void fill_k(lipa::bf16* p, size_t n, uint32_t seed) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    uint32_t x = (uint32_t)i * 2654435761u ^ seed;
    x ^= x >> 13; x *= 0x5bd1e995u; x ^= x >> 15;
    p[i] = (lipa::bf16)((x & 0xFFFF) / 32768.f - 1.f);
  }
}

int main(int argc, char** argv) {
#if defined(LIPA_G4W_NOSTORE)
  const char* tag = "nostore";
#else
  const char* tag = "shipped";
#endif
  const size_t maxe = (size_t)8192 * 16384;
  lipa::bf16 *a, *b, *c;
  float* ws;
  hipMalloc(&a, maxe * 2);
  hipMalloc(&b, maxe * 2);
  hipMalloc(&c, maxe * 2);
  hipMalloc(&ws, (size_t)4 * 2048 * 8192 * 4);
  fill_k<<<2048, 256>>>(a, maxe, 1u);
  fill_k<<<2048, 256>>>(b, maxe, 2u);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int i = 1; i + 3 < argc + 0 && i + 3 <= argc; i += 4) {
    const int M = atoi(argv[i]), N = atoi(argv[i + 1]), K = atoi(argv[i + 2]), sp = atoi(argv[i + 3]);
    if ((size_t)M * K > maxe || (size_t)N * K > maxe || (size_t)M * N > maxe) { printf("too big\n"); return 1; }
    const int grid = tiles_of(M, N, 256, 256) * sp;
    auto run = [&] {
      if (sp > 1)
        gemm4w_k<256, 256, false, true, 0, 0><<<grid, NT>>>(a, K, b, K, nullptr, c, M, N, K, sp, nullptr, nullptr, 0, ws,
                                                             nullptr, nullptr, LoraEpi{}, LoraDx{});
      else
        gemm4w_k<256, 256, false, false, 0, 0><<<grid, NT>>>(a, K, b, K, nullptr, c, M, N, K, 1, nullptr, nullptr, 0,
                                                              nullptr, nullptr, nullptr, LoraEpi{}, LoraDx{});
    };
    float best = 1e9f;
    for (int r = 0; r < 5; ++r) {
      for (int j = 0; j < 3; ++j) run();
      hipEventRecord(e0);
      for (int j = 0; j < 10; ++j) run();
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      best = fminf(best, ms * 100.f);
    }
    const int rounds = (grid + 255) / 256, kt = K / 64 / sp;
    printf("%-8s M=%5d N=%6d K=%6d s%d  grid %5d rounds %d ktiles/wg %4d  %8.1f us  %6.0f TF/s  %.3f us/ktile/round\n", tag,
           M, N, K, sp, grid, rounds, kt, best, 2.0 * M * N * K / best / 1e6, best / rounds / kt);
  }
  return 0;
}
