// Shared device helpers for the gfx950 (CDNA4, MI355X) kernels.
// Wave = 64 lanes everywhere; bf16 loads are always vectorised (8-16 B per lane).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace lipa {

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

constexpr int WAVE = 64;

__device__ __forceinline__ float bf2f(bf16 v) { return (float)v; }
__device__ __forceinline__ bf16 f2bf(float f) { return (bf16)f; }  // v_cvt_pk_bf16_f32 (RNE, NaN-safe)

template <typename T> __device__ __forceinline__ float to_f(T v) { return (float)v; }
template <typename T> __device__ __forceinline__ T from_f(float v) { return (T)v; }

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Block-wide sum for blockDim = NW*64; `scratch` >= NW floats of LDS. Result in every lane.
template <int NW>
__device__ __forceinline__ float block_sum(float v, float* scratch) {
  v = wave_sum(v);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  if (NW == 1) return v;
  __syncthreads();
  if (l == 0) scratch[w] = v;
  __syncthreads();
  float t = 0.f;
#pragma unroll
  for (int i = 0; i < NW; ++i) t += scratch[i];
  return t;
}
template <int NW>
__device__ __forceinline__ float block_max(float v, float* scratch) {
  v = wave_max(v);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  if (NW == 1) return v;
  __syncthreads();
  if (l == 0) scratch[w] = v;
  __syncthreads();
  float t = -INFINITY;
#pragma unroll
  for (int i = 0; i < NW; ++i) t = fmaxf(t, scratch[i]);
  return t;
}

// Vector load/store of 8 bf16 as 16 B.
__device__ __forceinline__ void load8(const bf16* p, float (&f)[8]) {
  bf16x8 v = *reinterpret_cast<const bf16x8*>(p);
#pragma unroll
  for (int i = 0; i < 8; ++i) f[i] = (float)v[i];
}
__device__ __forceinline__ void store8(bf16* p, const float (&f)[8]) {
  bf16x8 v;
#pragma unroll
  for (int i = 0; i < 8; ++i) v[i] = (bf16)f[i];
  *reinterpret_cast<bf16x8*>(p) = v;
}
__device__ __forceinline__ void load8(const float* p, float (&f)[8]) {
  f32x4 a = *reinterpret_cast<const f32x4*>(p), b = *reinterpret_cast<const f32x4*>(p + 4);
  f[0] = a[0]; f[1] = a[1]; f[2] = a[2]; f[3] = a[3]; f[4] = b[0]; f[5] = b[1]; f[6] = b[2]; f[7] = b[3];
}
__device__ __forceinline__ void store8(float* p, const float (&f)[8]) {
  *reinterpret_cast<f32x4*>(p) = f32x4{f[0], f[1], f[2], f[3]};
  *reinterpret_cast<f32x4*>(p + 4) = f32x4{f[4], f[5], f[6], f[7]};
}

// Bijective XCD-aware block remap (8 XCDs, blocks dealt round-robin): consecutive logical
// tiles land on the same XCD so neighbouring tiles share that XCD's L2.
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int q = nwg / 8, r = nwg % 8, x = bid % 8;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + bid / 8;
}

// Counter-based dropout mask shared by every kernel that applies or regenerates the LoRA input
// dropout (dropout.hip, lora.hip): 8 keep flags for elements [8v, 8v+8) of the row-major tensor,
// a pure function of (key, v) — masks are never stored.
__device__ __forceinline__ uint64_t splitmix_fin(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
__device__ __forceinline__ uint32_t dropout_keep8(uint64_t key, size_t v, uint32_t thr16) {
  const uint64_t h0 = splitmix_fin(key + 2 * v), h1 = splitmix_fin(key + 2 * v + 1);
  uint32_t m = 0;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    m |= (uint32_t)(((h0 >> (16 * i)) & 0xFFFF) >= thr16) << i;
    m |= (uint32_t)(((h1 >> (16 * i)) & 0xFFFF) >= thr16) << (i + 4);
  }
  return m;
}

}  // namespace lipa

#define LIPA_CHECK_LAUNCH()                                                              \
  do {                                                                                   \
    hipError_t e__ = hipGetLastError();                                                  \
    if (e__ != hipSuccess) {                                                             \
      fprintf(stderr, "HIP launch error %s at %s:%d\n", hipGetErrorString(e__), __FILE__, \
              __LINE__);                                                                 \
    }                                                                                    \
  } while (0)
