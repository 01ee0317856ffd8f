// Elementwise kernels (K5): SwiGLU over the fused [gate | up] projection, exact GELU.
// 16-byte vector loads per lane (8 bf16), grid-stride, memory-bound by design.
#include "common.h"

using namespace lipa;

namespace {

__device__ __forceinline__ float silu(float g) { return g / (1.f + __expf(-g)); }

// gu [M, 2F] -> y [M, F];  F % 8 == 0
// One 8-element vector per thread on a (row, column-chunk) grid: no index division (the grid-stride
// form spent most of its VALU on a 64-bit e / F, e % F per vector) and every load in flight at once.
__global__ __launch_bounds__(256) void swiglu_fwd_k(const bf16* __restrict__ gu, bf16* __restrict__ y, int M, int F) {
  const int f = (blockIdx.y * 256 + threadIdx.x) * 8;
  if (f >= F) return;
  const size_t m = blockIdx.x;
  float g[8], u[8], o[8];
  load8(gu + m * 2 * F + f, g);
  load8(gu + m * 2 * F + F + f, u);
#pragma unroll
  for (int i = 0; i < 8; ++i) o[i] = silu(g[i]) * u[i];
  store8(y + m * F + f, o);
}

// dgu = [dy*u*silu'(g) | dy*silu(g)]
__global__ __launch_bounds__(256) void swiglu_bwd_k(const bf16* __restrict__ dy, const bf16* __restrict__ gu,
                                                    bf16* __restrict__ dgu, int M, int F) {
  const int f = (blockIdx.y * 256 + threadIdx.x) * 8;
  if (f >= F) return;
  const size_t m = blockIdx.x;
  float g[8], u[8], d[8], dg[8], du[8];
  load8(gu + m * 2 * F + f, g);
  load8(gu + m * 2 * F + F + f, u);
  load8(dy + m * F + f, d);
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const float sg = 1.f / (1.f + __expf(-g[i]));
    const float s = g[i] * sg;
    du[i] = d[i] * s;
    dg[i] = d[i] * u[i] * (sg * (1.f + g[i] * (1.f - sg)));
  }
  store8(dgu + m * 2 * F + f, dg);
  store8(dgu + m * 2 * F + F + f, du);
}

template <typename T>
__global__ __launch_bounds__(256) void gelu_fwd_k(const T* __restrict__ x, T* __restrict__ y, size_t n) {
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
    const float v = (float)x[i];
    y[i] = (T)(0.5f * v * (1.f + erff(v * 0.70710678118654752f)));
  }
}

template <typename T>
__global__ __launch_bounds__(256) void gelu_bwd_k(const T* __restrict__ dy, const T* __restrict__ x, T* __restrict__ dx,
                                                  size_t n) {
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
    const float v = (float)x[i];
    const float cdf = 0.5f * (1.f + erff(v * 0.70710678118654752f));
    const float pdf = 0.3989422804014327f * __expf(-0.5f * v * v);
    dx[i] = (T)((float)dy[i] * (cdf + v * pdf));
  }
}

// y[n] = Σ_s x[s·stride + ·] (fp32 sum of S bf16 slices: the split-K partials of a batched GEMM)
template <int S>
__global__ __launch_bounds__(256) void sum_slices_k(const bf16* __restrict__ x, bf16* __restrict__ y, size_t n8,
                                                    size_t stride) {
  for (size_t v = (size_t)blockIdx.x * 256 + threadIdx.x; v < n8; v += (size_t)gridDim.x * 256) {
    float a[S][8], o[8];
#pragma unroll
    for (int s = 0; s < S; ++s) load8(x + s * stride + v * 8, a[s]);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      o[i] = a[0][i];
#pragma unroll
      for (int s = 1; s < S; ++s) o[i] += a[s][i];
    }
    store8(y + v * 8, o);
  }
}

inline int grid_for(size_t work) {
  size_t g = (work + 255) / 256;
  return (int)(g < 2048 ? (g ? g : 1) : 2048);
}

}  // namespace

void launch_swiglu_fwd(const void* gu, void* y, int M, int F, hipStream_t st) {
  if (M <= 0) return;
  const dim3 g(M, (F / 8 + 255) / 256);
  swiglu_fwd_k<<<g, 256, 0, st>>>((const bf16*)gu, (bf16*)y, M, F);
  LIPA_CHECK_LAUNCH();
}
void launch_swiglu_bwd(const void* dy, const void* gu, void* dgu, int M, int F, hipStream_t st) {
  if (M <= 0) return;
  const dim3 g(M, (F / 8 + 255) / 256);
  swiglu_bwd_k<<<g, 256, 0, st>>>((const bf16*)dy, (const bf16*)gu, (bf16*)dgu, M, F);
  LIPA_CHECK_LAUNCH();
}
void launch_gelu_fwd(int dtype, const void* x, void* y, size_t n, hipStream_t st) {
  if (dtype == 1) gelu_fwd_k<bf16><<<grid_for(n), 256, 0, st>>>((const bf16*)x, (bf16*)y, n);
  else gelu_fwd_k<float><<<grid_for(n), 256, 0, st>>>((const float*)x, (float*)y, n);
  LIPA_CHECK_LAUNCH();
}
void launch_gelu_bwd(int dtype, const void* dy, const void* x, void* dx, size_t n, hipStream_t st) {
  if (dtype == 1) gelu_bwd_k<bf16><<<grid_for(n), 256, 0, st>>>((const bf16*)dy, (const bf16*)x, (bf16*)dx, n);
  else gelu_bwd_k<float><<<grid_for(n), 256, 0, st>>>((const float*)dy, (const float*)x, (float*)dx, n);
  LIPA_CHECK_LAUNCH();
}
void launch_sum_slices(const void* x, void* y, int S, size_t n, size_t stride, hipStream_t st) {
  const size_t n8 = n / 8;
  const int g = grid_for(n8);
  switch (S) {
    case 2: sum_slices_k<2><<<g, 256, 0, st>>>((const bf16*)x, (bf16*)y, n8, stride); break;
    case 3: sum_slices_k<3><<<g, 256, 0, st>>>((const bf16*)x, (bf16*)y, n8, stride); break;
    case 4: sum_slices_k<4><<<g, 256, 0, st>>>((const bf16*)x, (bf16*)y, n8, stride); break;
    default: sum_slices_k<8><<<g, 256, 0, st>>>((const bf16*)x, (bf16*)y, n8, stride); break;
  }
  LIPA_CHECK_LAUNCH();
}
