// Epilogue-cost probe for gemm4w: times the step's multi-round GEMM roles with the shipped epilogue and
// (-DLIPA_G4W_NOSTORE) every output value computed but not stored — how much of each kernel is the
// serialized store traffic at the end of each round of tiles (the fixed cost per round of
// profiles/r5/gemm4w_round_fixed_cost.txt).  One process, uniform operands, min of 5 x 10 launches.
#include <cmath>
#include <cstdio>
#include <vector>

#include "gemm4w_kernel.h"

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

__global__ void fill_k(lipa::bf16* p, size_t n, uint32_t seed) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    uint32_t x = (uint32_t)i * 2654435761u ^ seed;
    x ^= x >> 13; x *= 0x5bd1e995u; x ^= x >> 15;
    p[i] = (lipa::bf16)((x & 0xFFFF) / 32768.f - 1.f);
  }
}

__global__ void hash_k(const uint32_t* p, size_t n, unsigned long long* out) {
  unsigned long long h = 0;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    h += (unsigned long long)(p[i] * 2654435761u) ^ (i * 0x9E3779B97F4A7C15ull);
  atomicAdd(out, h);
}

int main() {
#if defined(LIPA_G4W_NOSTORE)
  const char* tag = "nostore";

#else
  const char* tag = "shipped";
#endif
  const int M = 2048, F = 12288, Dm = 4096;
  lipa::bf16 *x, *w, *gu, *h, *dy, *dgu, *y;
  float* ws;
  CK(hipMalloc(&x, (size_t)M * 24576 * 2));
  CK(hipMalloc(&w, (size_t)24576 * 4096 * 2));
  CK(hipMalloc(&gu, (size_t)M * 2 * F * 2));
  CK(hipMalloc(&h, (size_t)M * F * 2));
  CK(hipMalloc(&dy, (size_t)M * 4096 * 2));
  CK(hipMalloc(&dgu, (size_t)M * 2 * F * 2));
  CK(hipMalloc(&y, (size_t)M * 24576 * 2));
  CK(hipMalloc(&ws, (size_t)2 * M * 4096 * 4));
  fill_k<<<2048, 256>>>(x, (size_t)M * 24576, 1u);
  fill_k<<<2048, 256>>>(w, (size_t)24576 * 4096, 2u);
  fill_k<<<2048, 256>>>(gu, (size_t)M * 2 * F, 3u);
  fill_k<<<2048, 256>>>(dy, (size_t)M * 4096, 4u);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto timeit = [&](auto&& fn) {
    float best = 1e9f;
    for (int r = 0; r < 5; ++r) {
      for (int i = 0; i < 3; ++i) fn();
      hipEventRecord(e0);
      for (int i = 0; i < 10; ++i) fn();
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      best = fminf(best, ms * 100.f);
    }
    return best;
  };
  struct R { const char* name; float us; double gf; };
  std::vector<R> rs;
  // gate|up forward + SwiGLU: x [M, 4096] · W_gu [2F, 4096]ᵀ, 256x256 tiles, 3 rounds
  rs.push_back({"swiglu_fwd 256x256", timeit([&] {
    gemm4w_k<256, 256, false, false, 1, 0><<<tiles_of(M, 2 * F, 256, 256), NT>>>(x, Dm, w, Dm, nullptr, gu, M, 2 * F, Dm, 1,
        nullptr, h, F, nullptr, nullptr, nullptr, LoraEpi{}, LoraDx{}); }), 2.0 * M * 2 * F * Dm});
  // plain NT, the same grid (y [M, 24576])
  rs.push_back({"plain_nt 256x256", timeit([&] {
    gemm4w_k<256, 256, false, false, 0, 0><<<tiles_of(M, 2 * F, 256, 256), NT>>>(x, Dm, w, Dm, nullptr, y, M, 2 * F, Dm, 1,
        nullptr, nullptr, 0, nullptr, nullptr, nullptr, LoraEpi{}, LoraDx{}); }), 2.0 * M * 2 * F * Dm});
  // down dX + dSwiGLU: dy [M, 4096] · W_down [4096, F], transposed-B 256x192, 2 rounds
  rs.push_back({"dswiglu 256x192bt", timeit([&] {
    gemm4w_k<256, 192, true, false, 2, 0><<<tiles_of(M, F, 256, 192), NT>>>(dy, Dm, w, F, nullptr, dgu, M, F, Dm, 1,
        gu, nullptr, F, nullptr, nullptr, nullptr, LoraEpi{}, LoraDx{}); }), 2.0 * M * F * Dm});
  // down forward: h [M, F] · W_down [4096, F]ᵀ split-K 2 (fp32 slabs), 2 rounds (the slab reduce not included)
  rs.push_back({"down_fwd_split2 256x256", timeit([&] {
    gemm4w_k<256, 256, false, true, 0, 0><<<2 * tiles_of(M, Dm, 256, 256), NT>>>(h, F, w, F, nullptr, y, M, Dm, F, 2,
        nullptr, nullptr, 0, ws, nullptr, nullptr, LoraEpi{}, LoraDx{}); }), 2.0 * M * Dm * F});
  // down forward, no split, residual in the epilogue (fp32 staging in the LDS build)
  rs.push_back({"down_fwd_res 256x256", timeit([&] {
    gemm4w_k<256, 256, false, false, 0, 0><<<tiles_of(M, Dm, 256, 256), NT>>>(h, F, w, F, dy, y, M, Dm, F, 1,
        nullptr, nullptr, 0, nullptr, nullptr, nullptr, LoraEpi{}, LoraDx{}); }), 2.0 * M * Dm * F});
  CK(hipDeviceSynchronize());
  // output hashes (must agree between the register and the LDS-staged epilogue builds)
  unsigned long long* hd;
  CK(hipMalloc(&hd, 8));
  auto hsh = [&](const void* p, size_t bytes) {
    hipMemset(hd, 0, 8);
    hash_k<<<1024, 256>>>((const uint32_t*)p, bytes / 4, hd);
    unsigned long long v;
    hipMemcpy(&v, hd, 8, hipMemcpyDeviceToHost);
    return v;
  };
  hipMemset(gu, 0, (size_t)M * 2 * F * 2); hipMemset(h, 0, (size_t)M * F * 2);
  gemm4w_k<256, 256, false, false, 1, 0><<<tiles_of(M, 2 * F, 256, 256), NT>>>(x, Dm, w, Dm, nullptr, gu, M, 2 * F, Dm, 1,
      nullptr, h, F, nullptr, nullptr, nullptr, LoraEpi{}, LoraDx{});
  const unsigned long long h1 = hsh(gu, (size_t)M * 2 * F * 2), h2 = hsh(h, (size_t)M * F * 2);
  hipMemset(y, 0, (size_t)M * 2 * F * 2);
  gemm4w_k<256, 256, false, false, 0, 0><<<tiles_of(M, 2 * F, 256, 256), NT>>>(x, Dm, w, Dm, nullptr, y, M, 2 * F, Dm, 1,
      nullptr, nullptr, 0, nullptr, nullptr, nullptr, LoraEpi{}, LoraDx{});
  const unsigned long long h3 = hsh(y, (size_t)M * 2 * F * 2);
  hipMemset(dgu, 0, (size_t)M * 2 * F * 2);
  gemm4w_k<256, 192, true, false, 2, 0><<<tiles_of(M, F, 256, 192), NT>>>(dy, Dm, w, F, nullptr, dgu, M, F, Dm, 1,
      gu, nullptr, F, nullptr, nullptr, nullptr, LoraEpi{}, LoraDx{});
  const unsigned long long h4 = hsh(dgu, (size_t)M * 2 * F * 2);
  hipMemset(ws, 0, (size_t)2 * M * 4096 * 4);
  gemm4w_k<256, 256, false, true, 0, 0><<<2 * tiles_of(M, Dm, 256, 256), NT>>>(h, F, w, F, nullptr, y, M, Dm, F, 2,
      nullptr, nullptr, 0, ws, nullptr, nullptr, LoraEpi{}, LoraDx{});
  const unsigned long long h5 = hsh(ws, (size_t)2 * M * 4096 * 4);
  hipMemset(y, 0, (size_t)M * 4096 * 2);
  gemm4w_k<256, 256, false, false, 0, 0><<<tiles_of(M, Dm, 256, 256), NT>>>(h, F, w, F, dy, y, M, Dm, F, 1,
      nullptr, nullptr, 0, nullptr, nullptr, nullptr, LoraEpi{}, LoraDx{});
  const unsigned long long h6 = hsh(y, (size_t)M * 4096 * 2);
  CK(hipDeviceSynchronize());
  printf("%-8s hashes swiglu %016llx %016llx plain %016llx dswiglu %016llx split %016llx res %016llx\n", tag, h1, h2,
         h3, h4, h5, h6);
  for (auto& r : rs) printf("%-8s %-26s %8.1f us %6.0f TF/s\n", tag, r.name, r.us, r.gf / r.us / 1e6);
  return 0;
}
