// Fused optimizer kernels (K10, K11, K12).
//
// Parameters, gradients and states live in flat fp32 buffers (the optimizer flattens the
// trainable set once; param.grad are views into the flat grad buffer, which is also the
// single DDP / ZeRO communication buffer).  Everything is sync-free: the global grad norm,
// the clip coefficient and the fp16 overflow flag stay on the device and are consumed by
// the update kernels through pointers, so an optimizer step is a handful of launches and
// never a host round trip.
//   * adamw:      torch.optim.AdamW semantics (decoupled weight decay, bias correction)
//   * adamw_8bit: blockwise (256) dynamic-map 8-bit m / v states (bnb "paged_adamw_8bit"
//                 state format [ext]); m signed map, v unsigned map, per-block absmax
//   * l2norm:     two-stage sum of squares -> {norm, clip_coef}
//   * unscale:    fp16 dynamic loss scaling: g *= 1/scale, found_inf flag
#include "common.h"

using namespace lipa;

namespace {

constexpr int NT = 256;

template <typename G>
__global__ __launch_bounds__(NT) void sumsq_partial_k(const G* __restrict__ g, size_t n, float* __restrict__ part) {
  __shared__ float red[NT / 64];
  float s = 0.f;
  for (size_t i = (size_t)blockIdx.x * NT + threadIdx.x; i < n; i += (size_t)gridDim.x * NT) {
    const float v = (float)g[i];
    s += v * v;
  }
  s = block_sum<NT / 64>(s, red);
  if (threadIdx.x == 0) part[blockIdx.x] = s;
}

// out[0] = ||g||, out[1] = clip coefficient min(1, max_norm / (norm + 1e-6)) (1 if max_norm <= 0)
__global__ __launch_bounds__(NT) void norm_finalize_k(const float* __restrict__ part, int P, float max_norm,
                                                      float* __restrict__ out, int accumulate) {
  __shared__ float red[NT / 64];
  float s = 0.f;
  for (int i = threadIdx.x; i < P; i += NT) s += part[i];
  s = block_sum<NT / 64>(s, red);
  if (threadIdx.x == 0) {
    if (accumulate) s += out[2];          // add an already-reduced sum of squares (ZeRO / multi-group)
    const float nrm = sqrtf(s);
    out[0] = nrm;
    out[1] = (max_norm > 0.f) ? fminf(1.f, max_norm / (nrm + 1e-6f)) : 1.f;
    out[2] = s;
  }
}

template <typename G>
__global__ __launch_bounds__(NT) void adamw_k(float* __restrict__ p, const G* __restrict__ g, float* __restrict__ m,
                                              float* __restrict__ v, bf16* __restrict__ p16, size_t n, float lr,
                                              float b1, float b2, float eps, float wd, float bc1, float bc2,
                                              const float* __restrict__ gscale, const float* __restrict__ skip) {
  if (skip && *skip != 0.f) return;                    // fp16 overflow: skip the step
  const float cs = gscale ? gscale[1] : 1.f;           // clip coefficient
  const float step_size = lr / bc1;
  const float bc2s = rsqrtf(bc2);
  for (size_t i = (size_t)blockIdx.x * NT + threadIdx.x; i < n; i += (size_t)gridDim.x * NT) {
    const float gi = (float)g[i] * cs;
    float pi = p[i] * (1.f - lr * wd);
    const float mi = b1 * m[i] + (1.f - b1) * gi;
    const float vi = b2 * v[i] + (1.f - b2) * gi * gi;
    m[i] = mi;
    v[i] = vi;
    pi -= step_size * mi / (sqrtf(vi) * bc2s + eps);
    p[i] = pi;
    if (p16) p16[i] = (bf16)pi;
  }
}

// ---------------------------------------------------------------- 8-bit blockwise states
__device__ __forceinline__ int nearest_code(const float* __restrict__ code, float x) {
  // code sorted ascending (256 entries): binary search then pick the closer neighbour
  int lo = 0, hi = 255;
#pragma unroll
  for (int it = 0; it < 8; ++it) {
    const int mid = (lo + hi + 1) >> 1;
    if (code[mid] <= x) lo = mid;
    else hi = mid - 1;
  }
  int best = lo;
  if (lo < 255 && fabsf(code[lo + 1] - x) < fabsf(code[lo] - x)) best = lo + 1;
  return best;
}

// one 256-thread block per 256-element state block
template <typename G>
__global__ __launch_bounds__(NT) void adamw8bit_k(float* __restrict__ p, const G* __restrict__ g,
                                                  uint8_t* __restrict__ qm, uint8_t* __restrict__ qv,
                                                  float* __restrict__ am, float* __restrict__ av,
                                                  const float* __restrict__ code_s, const float* __restrict__ code_u,
                                                  bf16* __restrict__ p16, size_t n, float lr, float b1, float b2,
                                                  float eps, float wd, float bc1, float bc2,
                                                  const float* __restrict__ gscale, const float* __restrict__ skip) {
  __shared__ float cs_l[256], cu_l[256], red[NT / 64];
  if (skip && *skip != 0.f) return;
  cs_l[threadIdx.x] = code_s[threadIdx.x];
  cu_l[threadIdx.x] = code_u[threadIdx.x];
  __syncthreads();
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  const bool ok = i < n;
  const float clip = gscale ? gscale[1] : 1.f;
  float mi = 0.f, vi = 0.f, pi = 0.f;
  if (ok) {
    const float gi = (float)g[i] * clip;
    mi = b1 * cs_l[qm[i]] * am[blockIdx.x] + (1.f - b1) * gi;
    vi = b2 * cu_l[qv[i]] * av[blockIdx.x] + (1.f - b2) * gi * gi;
    pi = p[i] * (1.f - lr * wd);
    pi -= (lr / bc1) * mi / (sqrtf(vi / bc2) + eps);
    p[i] = pi;
    if (p16) p16[i] = (bf16)pi;
  }
  const float mmax = block_max<NT / 64>(ok ? fabsf(mi) : 0.f, red);
  __syncthreads();
  const float vmax = block_max<NT / 64>(ok ? vi : 0.f, red);
  if (ok) {
    qm[i] = (uint8_t)nearest_code(cs_l, mmax > 0.f ? mi / mmax : 0.f);
    qv[i] = (uint8_t)nearest_code(cu_l, vmax > 0.f ? vi / vmax : 0.f);
  }
  if (threadIdx.x == 0) {
    am[blockIdx.x] = mmax;
    av[blockIdx.x] = vmax;
  }
}

template <typename G>
__global__ __launch_bounds__(NT) void unscale_k(G* __restrict__ g, size_t n, const float* __restrict__ inv_scale,
                                                float* __restrict__ found_inf) {
  const float s = *inv_scale;
  for (size_t i = (size_t)blockIdx.x * NT + threadIdx.x; i < n; i += (size_t)gridDim.x * NT) {
    const float v = (float)g[i] * s;
    if (!isfinite(v)) *found_inf = 1.f;
    g[i] = (G)v;
  }
}

inline int grid_for(size_t n) {
  size_t b = (n + NT - 1) / NT;
  return (int)(b < 4096 ? (b ? b : 1) : 4096);
}

}  // namespace

constexpr int kNormParts = 1024;

// dtype of g: 0 fp32, 1 bf16. partial: scratch[kNormParts]; out[3] fp32 (norm, coef, sumsq)
void launch_grad_norm(int dtype, const void* g, size_t n, float* partial, float* out, float max_norm, int accumulate,
                      hipStream_t st) {
  int P = grid_for(n);
  if (P > kNormParts) P = kNormParts;
  if (dtype == 1) sumsq_partial_k<bf16><<<P, NT, 0, st>>>((const bf16*)g, n, partial);
  else sumsq_partial_k<float><<<P, NT, 0, st>>>((const float*)g, n, partial);
  norm_finalize_k<<<1, NT, 0, st>>>(partial, P, max_norm, out, accumulate);
  LIPA_CHECK_LAUNCH();
}

void launch_adamw(int gdtype, float* p, const void* g, float* m, float* v, void* p16, size_t n, float lr, float b1,
                  float b2, float eps, float wd, float bc1, float bc2, const float* gscale, const float* skip,
                  hipStream_t st) {
  if (gdtype == 1)
    adamw_k<bf16><<<grid_for(n), NT, 0, st>>>(p, (const bf16*)g, m, v, (bf16*)p16, n, lr, b1, b2, eps, wd, bc1, bc2,
                                              gscale, skip);
  else
    adamw_k<float><<<grid_for(n), NT, 0, st>>>(p, (const float*)g, m, v, (bf16*)p16, n, lr, b1, b2, eps, wd, bc1,
                                               bc2, gscale, skip);
  LIPA_CHECK_LAUNCH();
}

void launch_adamw8bit(int gdtype, float* p, const void* g, uint8_t* qm, uint8_t* qv, float* am, float* av,
                      const float* code_s, const float* code_u, void* p16, size_t n, float lr, float b1, float b2,
                      float eps, float wd, float bc1, float bc2, const float* gscale, const float* skip,
                      hipStream_t st) {
  const int blocks = (int)((n + 255) / 256);
  if (gdtype == 1)
    adamw8bit_k<bf16><<<blocks, NT, 0, st>>>(p, (const bf16*)g, qm, qv, am, av, code_s, code_u, (bf16*)p16, n, lr,
                                             b1, b2, eps, wd, bc1, bc2, gscale, skip);
  else
    adamw8bit_k<float><<<blocks, NT, 0, st>>>(p, (const float*)g, qm, qv, am, av, code_s, code_u, (bf16*)p16, n,
                                              lr, b1, b2, eps, wd, bc1, bc2, gscale, skip);
  LIPA_CHECK_LAUNCH();
}

void launch_unscale(int dtype, void* g, size_t n, const float* inv_scale, float* found_inf, hipStream_t st) {
  if (dtype == 1) unscale_k<bf16><<<grid_for(n), NT, 0, st>>>((bf16*)g, n, inv_scale, found_inf);
  else unscale_k<float><<<grid_for(n), NT, 0, st>>>((float*)g, n, inv_scale, found_inf);
  LIPA_CHECK_LAUNCH();
}
