// Dropout with a counter-based RNG (K13): the keep-mask is a pure function of
// (seed, offset, element index), so the forward writes only the scaled activations and the
// backward REGENERATES the mask instead of reading a stored one (no mask tensor, no extra
// HBM traffic).  Used for the LoRA input dropout (PEFT ``lora_dropout``).
//
// RNG: a 64-bit mix (splitmix64 finaliser) of (seed ^ offset-key, index/4) yields four
// 16-bit uniforms per hash — one per element — so keep-probability resolution is 2^-16.
#include "common.h"

using namespace lipa;

namespace {

__device__ __forceinline__ uint32_t keep8(uint64_t key, size_t v, uint32_t thr16) {
  return dropout_keep8(key, v, thr16);
}

__global__ __launch_bounds__(256) void dropout_fwd_k(const bf16* __restrict__ x, bf16* __restrict__ y, size_t n,
                                                     uint64_t key, uint32_t thr16, float scale) {
  const size_t nv = n / 8;
  for (size_t v = (size_t)blockIdx.x * 256 + threadIdx.x; v < nv; v += (size_t)gridDim.x * 256) {
    const uint32_t m = keep8(key, v, thr16);
    float f[8];
    load8(x + v * 8, f);
#pragma unroll
    for (int i = 0; i < 8; ++i) f[i] = ((m >> i) & 1) ? f[i] * scale : 0.f;
    store8(y + v * 8, f);
  }
}

// dx += mask ⊙ t · scale
__global__ __launch_bounds__(256) void dropout_bwd_add_k(bf16* __restrict__ dx, const bf16* __restrict__ t, size_t n,
                                                         uint64_t key, uint32_t thr16, float scale) {
  const size_t nv = n / 8;
  for (size_t v = (size_t)blockIdx.x * 256 + threadIdx.x; v < nv; v += (size_t)gridDim.x * 256) {
    const uint32_t m = keep8(key, v, thr16);
    float a[8], b[8];
    load8(dx + v * 8, a);
    load8(t + v * 8, b);
#pragma unroll
    for (int i = 0; i < 8; ++i) a[i] += ((m >> i) & 1) ? b[i] * scale : 0.f;
    store8(dx + v * 8, a);
  }
}

inline int grid_for(size_t nv) {
  size_t g = (nv + 255) / 256;
  return (int)(g < 4096 ? (g ? g : 1) : 4096);
}

}  // namespace

void launch_dropout_fwd(const void* x, void* y, size_t n, uint64_t key, float p, hipStream_t st) {
  const uint32_t thr = (uint32_t)(p * 65536.0f + 0.5f);
  dropout_fwd_k<<<grid_for(n / 8), 256, 0, st>>>((const bf16*)x, (bf16*)y, n, key, thr, 1.f / (1.f - p));
  LIPA_CHECK_LAUNCH();
}

void launch_dropout_bwd_add(void* dx, const void* t, size_t n, uint64_t key, float p, hipStream_t st) {
  const uint32_t thr = (uint32_t)(p * 65536.0f + 0.5f);
  dropout_bwd_add_k<<<grid_for(n / 8), 256, 0, st>>>((bf16*)dx, (const bf16*)t, n, key, thr, 1.f / (1.f - p));
  LIPA_CHECK_LAUNCH();
}
