// RoPE (K3) and the fused Qwen3 per-head q/k RMSNorm + rotate-half RoPE, fwd + bwd.
//
// Layout: token-major fused projection output qkv[T, (hq+2hkv)*D].  A head-row of D
// elements is owned by P = D/8 lanes; lane j holds elements [4j, 4j+4) of the first half
// and [D/2+4j, D/2+4j+4) of the second half, so each rotate-half pair (i, i+D/2) lives in
// one lane and every access is an 8-byte vector.  The per-head RMS reduction is a
// shuffle-xor over the P-lane group.  cos/sin are per token [T, D/2] fp32.
#include "common.h"

using namespace lipa;

namespace {

__device__ __forceinline__ void ld4(const bf16* p, float (&f)[4]) {
  bf16x4 v = *reinterpret_cast<const bf16x4*>(p);
  f[0] = (float)v[0]; f[1] = (float)v[1]; f[2] = (float)v[2]; f[3] = (float)v[3];
}
__device__ __forceinline__ void st4(bf16* p, const float (&f)[4]) {
  bf16x4 v;
  v[0] = (bf16)f[0]; v[1] = (bf16)f[1]; v[2] = (bf16)f[2]; v[3] = (bf16)f[3];
  *reinterpret_cast<bf16x4*>(p) = v;
}
__device__ __forceinline__ void ld4f(const float* p, float (&f)[4]) {
  f32x4 v = *reinterpret_cast<const f32x4*>(p);
  f[0] = v[0]; f[1] = v[1]; f[2] = v[2]; f[3] = v[3];
}

template <int P>
__device__ __forceinline__ float group_sum(float v) {
#pragma unroll
  for (int o = P / 2; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// rows: 0..T*hq-1 are q heads, T*hq.. are k heads
template <int D>
__global__ __launch_bounds__(256) void qk_norm_rope_fwd_k(const bf16* __restrict__ qkv, const bf16* __restrict__ qw,
                                                          const bf16* __restrict__ kw, const float* __restrict__ cosb,
                                                          const float* __restrict__ sinb, bf16* __restrict__ q,
                                                          bf16* __restrict__ k, float* __restrict__ rq,
                                                          float* __restrict__ rk, int T, int hq, int hkv, float eps) {
  constexpr int P = D / 8, H = D / 2;
  const int gid = blockIdx.x * 256 + threadIdx.x;
  const int row = gid / P, j = gid % P;
  const int nq = T * hq, nrows = nq + T * hkv;
  if (row >= nrows) return;  // whole P-groups exit together
  const bool isq = row < nq;
  const int t = isq ? row / hq : (row - nq) / hkv;
  const int h = isq ? row % hq : (row - nq) % hkv;
  const int ld = (hq + 2 * hkv) * D;
  const bf16* src = qkv + (size_t)t * ld + (isq ? h * D : (hq + h) * D);
  float a[4], b[4];
  ld4(src + 4 * j, a);
  ld4(src + H + 4 * j, b);
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < 4; ++i) ss += a[i] * a[i] + b[i] * b[i];
  ss = group_sum<P>(ss);
  const float r = rsqrtf(ss / D + eps);
  const bf16* w = isq ? qw : kw;
  float wa[4], wb[4];
  if (w) {
    ld4(w + 4 * j, wa);
    ld4(w + H + 4 * j, wb);
  } else {
#pragma unroll
    for (int i = 0; i < 4; ++i) wa[i] = wb[i] = 1.f;
  }
  float c[4], s[4];
  ld4f(cosb + (size_t)t * H + 4 * j, c);
  ld4f(sinb + (size_t)t * H + 4 * j, s);
  float oa[4], ob[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    // Qwen3 rounds the normed value to the model dtype before RoPE
    const float x1 = (float)(bf16)(a[i] * r * wa[i]);
    const float x2 = (float)(bf16)(b[i] * r * wb[i]);
    oa[i] = x1 * c[i] - x2 * s[i];
    ob[i] = x2 * c[i] + x1 * s[i];
  }
  bf16* dst = isq ? q + (size_t)t * hq * D + h * D : k + (size_t)t * hkv * D + h * D;
  st4(dst + 4 * j, oa);
  st4(dst + H + 4 * j, ob);
  if (j == 0) {
    if (isq) rq[row] = r;
    else rk[row - nq] = r;
  }
}

template <int D>
__global__ __launch_bounds__(256) void qk_norm_rope_bwd_k(const bf16* __restrict__ dq, const bf16* __restrict__ dk,
                                                          const bf16* __restrict__ dv, const bf16* __restrict__ qkv, const bf16* __restrict__ qw,
                                                          const bf16* __restrict__ kw, const float* __restrict__ cosb,
                                                          const float* __restrict__ sinb, const float* __restrict__ rq,
                                                          const float* __restrict__ rk, bf16* __restrict__ dqkv, int T,
                                                          int hq, int hkv) {
  constexpr int P = D / 8, H = D / 2;
  const int gid = blockIdx.x * 256 + threadIdx.x;
  const int row = gid / P, j = gid % P;
  const int nq = T * hq, nrows = nq + T * hkv;
  if (row >= nrows) {
    // rows past q and k: the v head rows of dqkv (dv passes through, or zeros without a dv)
    const int vr = row - nrows;
    if (vr >= T * hkv) return;
    const int t = vr / hkv, h = vr % hkv;
    bf16* o = dqkv + (size_t)t * (hq + 2 * hkv) * D + (hq + hkv + h) * D;
    float va[4] = {0.f, 0.f, 0.f, 0.f}, vb[4] = {0.f, 0.f, 0.f, 0.f};
    if (dv) {
      ld4(dv + (size_t)vr * D + 4 * j, va);
      ld4(dv + (size_t)vr * D + H + 4 * j, vb);
    }
    st4(o + 4 * j, va);
    st4(o + H + 4 * j, vb);
    return;
  }
  const bool isq = row < nq;
  const int t = isq ? row / hq : (row - nq) / hkv;
  const int h = isq ? row % hq : (row - nq) % hkv;
  const int ld = (hq + 2 * hkv) * D;
  const size_t off = (size_t)t * ld + (isq ? h * D : (hq + h) * D);
  const bf16* g = isq ? dq + (size_t)t * hq * D + h * D : dk + (size_t)t * hkv * D + h * D;
  float ga[4], gb[4], c[4], s[4], a[4], b[4], wa[4], wb[4];
  ld4(g + 4 * j, ga);
  ld4(g + H + 4 * j, gb);
  ld4f(cosb + (size_t)t * H + 4 * j, c);
  ld4f(sinb + (size_t)t * H + 4 * j, s);
  ld4(qkv + off + 4 * j, a);
  ld4(qkv + off + H + 4 * j, b);
  const bf16* w = isq ? qw : kw;
  if (w) {
    ld4(w + 4 * j, wa);
    ld4(w + H + 4 * j, wb);
  } else {
#pragma unroll
    for (int i = 0; i < 4; ++i) wa[i] = wb[i] = 1.f;
  }
  const float r = isq ? rq[row] : rk[row - nq];
  float dot = 0.f;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    // inverse rotation of the gradient
    const float g1 = ga[i] * c[i] + gb[i] * s[i];
    const float g2 = gb[i] * c[i] - ga[i] * s[i];
    ga[i] = g1 * wa[i];  // grad wrt xhat (times weight)
    gb[i] = g2 * wb[i];
    a[i] *= r;
    b[i] *= r;
    dot += a[i] * ga[i] + b[i] * gb[i];
  }
  dot = group_sum<P>(dot) / D;
  float oa[4], ob[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    oa[i] = r * (ga[i] - a[i] * dot);
    ob[i] = r * (gb[i] - b[i] * dot);
  }
  st4(dqkv + off + 4 * j, oa);
  st4(dqkv + off + H + 4 * j, ob);
}

// generic rope on x[T, H, D]; interleaved (pairs 2i,2i+1) or rotate-half; inverse = rotate by -theta
template <typename T>
__global__ __launch_bounds__(256) void rope_k(const T* __restrict__ x, const float* __restrict__ cosb,
                                              const float* __restrict__ sinb, T* __restrict__ y, int Tn, int H, int D,
                                              int interleaved, int inverse) {
  const size_t idx = (size_t)blockIdx.x * 256 + threadIdx.x;
  const int half = D / 2;
  const size_t total = (size_t)Tn * H * half;
  if (idx >= total) return;
  const int i = idx % half;
  const size_t th = idx / half;
  const int t = th / H;
  const T* xr = x + th * D;
  T* yr = y + th * D;
  const float c = cosb[(size_t)t * half + i];
  const float s = inverse ? -sinb[(size_t)t * half + i] : sinb[(size_t)t * half + i];
  const int i1 = interleaved ? 2 * i : i, i2 = interleaved ? 2 * i + 1 : i + half;
  const float x1 = (float)xr[i1], x2 = (float)xr[i2];
  yr[i1] = (T)(x1 * c - x2 * s);
  yr[i2] = (T)(x2 * c + x1 * s);
}

}  // namespace

void launch_qk_norm_rope_fwd(const void* qkv, const void* qw, const void* kw, const float* cosb, const float* sinb,
                             void* q, void* k, float* rq, float* rk, int T, int hq, int hkv, int D, float eps,
                             hipStream_t st) {
  const long rows = (long)T * (hq + hkv);
  const long threads = rows * (D / 8);
  dim3 g((threads + 255) / 256), b(256);
#define F(DD)                                                                                                \
  qk_norm_rope_fwd_k<DD><<<g, b, 0, st>>>((const bf16*)qkv, (const bf16*)qw, (const bf16*)kw, cosb, sinb, \
                                          (bf16*)q, (bf16*)k, rq, rk, T, hq, hkv, eps)
  switch (D) {
    case 32: F(32); break;
    case 64: F(64); break;
    case 128: F(128); break;
    case 256: F(256); break;
    default: fprintf(stderr, "qk_norm_rope: unsupported head_dim %d\n", D);
  }
#undef F
  LIPA_CHECK_LAUNCH();
}

void launch_qk_norm_rope_bwd(const void* dq, const void* dk, const void* dv, const void* qkv, const void* qw,
                             const void* kw, const float* cosb, const float* sinb, const float* rq, const float* rk,
                             void* dqkv, int T, int hq, int hkv, int D, hipStream_t st) {
  const long rows = (long)T * (hq + 2 * hkv);
  const long threads = rows * (D / 8);
  dim3 g((threads + 255) / 256), b(256);
#define F(DD)                                                                                                  \
  qk_norm_rope_bwd_k<DD><<<g, b, 0, st>>>((const bf16*)dq, (const bf16*)dk, (const bf16*)dv, (const bf16*)qkv, (const bf16*)qw, \
                                          (const bf16*)kw, cosb, sinb, rq, rk, (bf16*)dqkv, T, hq, hkv)
  switch (D) {
    case 32: F(32); break;
    case 64: F(64); break;
    case 128: F(128); break;
    case 256: F(256); break;
    default: fprintf(stderr, "qk_norm_rope: unsupported head_dim %d\n", D);
  }
#undef F
  LIPA_CHECK_LAUNCH();
}

void launch_rope(int dtype, const void* x, const float* cosb, const float* sinb, void* y, int T, int H, int D,
                 int interleaved, int inverse, hipStream_t st) {
  const size_t total = (size_t)T * H * (D / 2);
  dim3 g((total + 255) / 256), b(256);
  if (dtype == 1)
    rope_k<bf16><<<g, b, 0, st>>>((const bf16*)x, cosb, sinb, (bf16*)y, T, H, D, interleaved, inverse);
  else
    rope_k<float><<<g, b, 0, st>>>((const float*)x, cosb, sinb, (float*)y, T, H, D, interleaved, inverse);
  LIPA_CHECK_LAUNCH();
}
