// RMSNorm / LayerNorm forward + backward for gfx950.
//
// One wave (64 lanes) per row; each lane owns CH chunks of 8 contiguous elements loaded as
// 16-byte vectors (bf16) so a row of 4096 bf16 is 8 independent 16-B loads per lane in
// flight.  The row stays in registers between the reduction and the normalisation (single
// HBM pass).  4 rows per 256-thread workgroup.  Backward optionally accumulates dW/db with
// per-workgroup fp32 partial rows + a second reduction kernel (no float atomics).
#include "common.h"

using namespace lipa;

namespace {

constexpr int ROWS = 4;  // waves (rows) per workgroup

template <typename T, typename TW, int CH>
__global__ __launch_bounds__(256) void rmsnorm_fwd_k(const T* __restrict__ x, const TW* __restrict__ w,
                                                     T* __restrict__ y, float* __restrict__ rstd_out, int M,
                                                     int N, float eps) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * ROWS + (threadIdx.x >> 6);
  if (row >= M) return;
  const T* xr = x + (size_t)row * N;
  float v[CH][8];
  bf16x8 wb[CH];  // the weight row is loaded with x, before the reduction (no second round trip)
  float ss = 0.f;
#pragma unroll
  for (int c = 0; c < CH; ++c) {
    const int col = (c * 64 + lane) * 8;
    if (col < N) {
      load8(xr + col, v[c]);
      if constexpr (sizeof(TW) == 2) {
        if (w) wb[c] = *reinterpret_cast<const bf16x8*>(w + col);
      }
#pragma unroll
      for (int i = 0; i < 8; ++i) ss += v[c][i] * v[c][i];
    }
  }
  ss = wave_sum(ss);
  const float r = rsqrtf(ss / N + eps);
  if (lane == 0) rstd_out[row] = r;
  T* yr = y + (size_t)row * N;
#pragma unroll
  for (int c = 0; c < CH; ++c) {
    const int col = (c * 64 + lane) * 8;
    if (col < N) {
      float wv[8];
      if (w) {
        if constexpr (sizeof(TW) == 2) {
#pragma unroll
          for (int i = 0; i < 8; ++i) wv[i] = (float)wb[c][i];
        } else {
          load8(w + col, wv);
        }
      }
      float o[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) o[i] = v[c][i] * r * (w ? wv[i] : 1.f);
      store8(yr + col, o);
    }
  }
}

// dx = r * (w*dy - xhat * mean(xhat * w * dy)) ; dw_part[blk] += dy * xhat
template <typename T, typename TW, int CH>
__global__ __launch_bounds__(256) void rmsnorm_bwd_k(const T* __restrict__ dy, const T* __restrict__ x,
                                                     const TW* __restrict__ w, const float* __restrict__ rstd,
                                                     T* __restrict__ dx, float* __restrict__ dw_part, int M,
                                                     int N, const T* __restrict__ dres) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int row = blockIdx.x * ROWS + wid;
  const bool valid = row < M;
  float xv[CH][8], gv[CH][8];
  T rb[CH][8];  // residual-branch gradient, fetched with x / dy (one round trip per row)
  float dot = 0.f;
  const float r = valid ? rstd[row] : 0.f;
#pragma unroll
  for (int c = 0; c < CH; ++c) {
    const int col = (c * 64 + lane) * 8;
    if (valid && col < N) {
      load8(x + (size_t)row * N + col, xv[c]);
      load8(dy + (size_t)row * N + col, gv[c]);
      if (dres) {
        if constexpr (sizeof(T) == 2)
          *reinterpret_cast<bf16x8*>(rb[c]) = *reinterpret_cast<const bf16x8*>(dres + (size_t)row * N + col);
        else
#pragma unroll
          for (int i = 0; i < 8; ++i) rb[c][i] = dres[(size_t)row * N + col + i];
      }
      float wv[8];
      if (w) load8(w + col, wv);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        xv[c][i] *= r;                                  // xhat
        const float wg = gv[c][i] * (w ? wv[i] : 1.f);
        dot += xv[c][i] * wg;
      }
    } else {
#pragma unroll
      for (int i = 0; i < 8; ++i) xv[c][i] = gv[c][i] = 0.f;
    }
  }
  dot = wave_sum(dot) / N;
#pragma unroll
  for (int c = 0; c < CH; ++c) {
    const int col = (c * 64 + lane) * 8;
    if (valid && col < N) {
      float wv[8];
      if (w) load8(w + col, wv);
      float o[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) o[i] = r * (gv[c][i] * (w ? wv[i] : 1.f) - xv[c][i] * dot);
      if (dres) {  // the residual branch's gradient (x feeds both the norm and the skip connection)
#pragma unroll
        for (int i = 0; i < 8; ++i) o[i] += (float)rb[c][i];
      }
      store8(dx + (size_t)row * N + col, o);
    }
  }
  if (dw_part) {
    // reduce dy*xhat over the block's rows through LDS, one partial row per block
    __shared__ float red[ROWS][8 * 64 + 4];
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      const int col = (c * 64 + lane) * 8;
#pragma unroll
      for (int i = 0; i < 8; ++i) red[wid][lane * 8 + i] = gv[c][i] * xv[c][i];
      __syncthreads();
      for (int t = threadIdx.x; t < 512; t += 256) {
        const int cc = c * 512 + t;
        if (cc < N) {
          float s = 0.f;
#pragma unroll
          for (int q = 0; q < ROWS; ++q) s += red[q][t];
          dw_part[(size_t)blockIdx.x * N + cc] = s;
        }
      }
      __syncthreads();
      (void)col;
    }
  }
}

template <typename T, typename TW, int CH>
__global__ __launch_bounds__(256) void layernorm_fwd_k(const T* __restrict__ x, const TW* __restrict__ w,
                                                       const TW* __restrict__ b, T* __restrict__ y,
                                                       float* __restrict__ mean_out, float* __restrict__ rstd_out,
                                                       int M, int N, float eps) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * ROWS + (threadIdx.x >> 6);
  if (row >= M) return;
  const T* xr = x + (size_t)row * N;
  float v[CH][8];
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < CH; ++c) {
    const int col = (c * 64 + lane) * 8;
    if (col < N) {
      load8(xr + col, v[c]);
#pragma unroll
      for (int i = 0; i < 8; ++i) s += v[c][i];
    }
  }
  const float mu = wave_sum(s) / N;
  float ss = 0.f;
#pragma unroll
  for (int c = 0; c < CH; ++c) {
    const int col = (c * 64 + lane) * 8;
    if (col < N) {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const float d = v[c][i] - mu;
        ss += d * d;
      }
    }
  }
  const float r = rsqrtf(wave_sum(ss) / N + eps);
  if (lane == 0) {
    mean_out[row] = mu;
    rstd_out[row] = r;
  }
  T* yr = y + (size_t)row * N;
#pragma unroll
  for (int c = 0; c < CH; ++c) {
    const int col = (c * 64 + lane) * 8;
    if (col < N) {
      float wv[8], bv[8], o[8];
      if (w) load8(w + col, wv);
      if (b) load8(b + col, bv);
#pragma unroll
      for (int i = 0; i < 8; ++i) o[i] = (v[c][i] - mu) * r * (w ? wv[i] : 1.f) + (b ? bv[i] : 0.f);
      store8(yr + col, o);
    }
  }
}

template <typename T, typename TW, int CH>
__global__ __launch_bounds__(256) void layernorm_bwd_k(const T* __restrict__ dy, const T* __restrict__ x,
                                                       const TW* __restrict__ w, const float* __restrict__ mean,
                                                       const float* __restrict__ rstd, T* __restrict__ dx,
                                                       float* __restrict__ dw_part, float* __restrict__ db_part,
                                                       int M, int N) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int row = blockIdx.x * ROWS + wid;
  const bool valid = row < M;
  float xv[CH][8], gv[CH][8];
  float s1 = 0.f, s2 = 0.f;
  const float mu = valid ? mean[row] : 0.f, r = valid ? rstd[row] : 0.f;
#pragma unroll
  for (int c = 0; c < CH; ++c) {
    const int col = (c * 64 + lane) * 8;
    if (valid && col < N) {
      load8(x + (size_t)row * N + col, xv[c]);
      load8(dy + (size_t)row * N + col, gv[c]);
      float wv[8];
      if (w) load8(w + col, wv);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        xv[c][i] = (xv[c][i] - mu) * r;
        const float wg = gv[c][i] * (w ? wv[i] : 1.f);
        s1 += wg;
        s2 += wg * xv[c][i];
      }
    } else {
#pragma unroll
      for (int i = 0; i < 8; ++i) xv[c][i] = gv[c][i] = 0.f;
    }
  }
  s1 = wave_sum(s1) / N;
  s2 = wave_sum(s2) / N;
#pragma unroll
  for (int c = 0; c < CH; ++c) {
    const int col = (c * 64 + lane) * 8;
    if (valid && col < N) {
      float wv[8], o[8];
      if (w) load8(w + col, wv);
#pragma unroll
      for (int i = 0; i < 8; ++i) o[i] = r * (gv[c][i] * (w ? wv[i] : 1.f) - s1 - xv[c][i] * s2);
      store8(dx + (size_t)row * N + col, o);
    }
  }
  if (dw_part) {
    __shared__ float red[2][ROWS][8 * 64 + 4];
#pragma unroll
    for (int c = 0; c < CH; ++c) {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        red[0][wid][lane * 8 + i] = gv[c][i] * xv[c][i];
        red[1][wid][lane * 8 + i] = gv[c][i];
      }
      __syncthreads();
      for (int t = threadIdx.x; t < 512; t += 256) {
        const int cc = c * 512 + t;
        if (cc < N) {
          float a = 0.f, bb = 0.f;
#pragma unroll
          for (int q = 0; q < ROWS; ++q) {
            a += red[0][q][t];
            bb += red[1][q][t];
          }
          dw_part[(size_t)blockIdx.x * N + cc] = a;
          db_part[(size_t)blockIdx.x * N + cc] = bb;
        }
      }
      __syncthreads();
    }
  }
}

// sum partial rows [P, N] -> out [N] (fp32)
__global__ __launch_bounds__(256) void colsum_k(const float* __restrict__ part, float* __restrict__ out, int P, int N) {
  const int col = blockIdx.x * 256 + threadIdx.x;
  if (col >= N) return;
  float s = 0.f;
  for (int p = 0; p < P; ++p) s += part[(size_t)p * N + col];
  out[col] = s;
}

template <int CH>
struct ChTag {};

#define LIPA_CH_DISPATCH(N, FN)                                    \
  do {                                                             \
    const int ch__ = ((N) + 511) / 512;                            \
    if (ch__ <= 1) { FN(1); }                                      \
    else if (ch__ <= 2) { FN(2); }                                 \
    else if (ch__ <= 4) { FN(4); }                                 \
    else if (ch__ <= 8) { FN(8); }                                 \
    else if (ch__ <= 10) { FN(10); }                               \
    else if (ch__ <= 12) { FN(12); }                               \
    else if (ch__ <= 16) { FN(16); }                               \
    else { fprintf(stderr, "norm: N=%d too large\n", (int)(N)); }  \
  } while (0)


// ---- split rows (bf16, no weight gradient): WPR waves share one row, so a 2048-row activation is
// 4096 waves (4 per SIMD) with half the registers each — the single-wave-per-row form leaves the
// memory latency of its one round trip exposed at 2 waves per SIMD.  Partial sums meet in LDS.
template <int CH, int WPR>
__global__ __launch_bounds__(256) void rmsnorm_fwd_split_k(const bf16* __restrict__ x, const bf16* __restrict__ w,
                                                           bf16* __restrict__ y, float* __restrict__ rstd_out, int M,
                                                           int N, float eps) {
  constexpr int RPB = 4 / WPR;  // rows per workgroup
  __shared__ float part[4];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int row = blockIdx.x * RPB + wid / WPR, pw = wid % WPR;
  const bool valid = row < M;
  const bf16* xr = x + (size_t)(valid ? row : 0) * N;
  float v[CH][8];
  bf16x8 wb[CH];
  float ss = 0.f;
#pragma unroll
  for (int c = 0; c < CH; ++c) {
    const int col = ((c * WPR + pw) * 64 + lane) * 8;
    load8(xr + col, v[c]);
    if (w) wb[c] = *reinterpret_cast<const bf16x8*>(w + col);
#pragma unroll
    for (int i = 0; i < 8; ++i) ss += v[c][i] * v[c][i];
  }
  ss = wave_sum(ss);
  if (lane == 0) part[wid] = ss;
  __syncthreads();
  float tot = 0.f;
#pragma unroll
  for (int p = 0; p < WPR; ++p) tot += part[(wid / WPR) * WPR + p];
  if (!valid) return;
  const float r = rsqrtf(tot / N + eps);
  if (lane == 0 && pw == 0) rstd_out[row] = r;
  bf16* yr = y + (size_t)row * N;
#pragma unroll
  for (int c = 0; c < CH; ++c) {
    const int col = ((c * WPR + pw) * 64 + lane) * 8;
    float o[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) o[i] = v[c][i] * r * (w ? (float)wb[c][i] : 1.f);
    store8(yr + col, o);
  }
}

template <int CH, int WPR>
__global__ __launch_bounds__(256) void rmsnorm_bwd_split_k(const bf16* __restrict__ dy, const bf16* __restrict__ x,
                                                           const bf16* __restrict__ w, const float* __restrict__ rstd,
                                                           bf16* __restrict__ dx, int M, int N,
                                                           const bf16* __restrict__ dres) {
  constexpr int RPB = 4 / WPR;
  __shared__ float part[4];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int row = blockIdx.x * RPB + wid / WPR, pw = wid % WPR;
  const bool valid = row < M;
  const size_t ro = (size_t)(valid ? row : 0) * N;
  const float r = rstd[valid ? row : 0];
  float xv[CH][8], gv[CH][8];
  bf16x8 rb[CH], wb[CH];
  float dot = 0.f;
#pragma unroll
  for (int c = 0; c < CH; ++c) {
    const int col = ((c * WPR + pw) * 64 + lane) * 8;
    load8(x + ro + col, xv[c]);
    load8(dy + ro + col, gv[c]);
    if (dres) rb[c] = *reinterpret_cast<const bf16x8*>(dres + ro + col);
    if (w) wb[c] = *reinterpret_cast<const bf16x8*>(w + col);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      xv[c][i] *= r;
      dot += xv[c][i] * gv[c][i] * (w ? (float)wb[c][i] : 1.f);
    }
  }
  dot = wave_sum(dot);
  if (lane == 0) part[wid] = dot;
  __syncthreads();
  float tot = 0.f;
#pragma unroll
  for (int p = 0; p < WPR; ++p) tot += part[(wid / WPR) * WPR + p];
  if (!valid) return;
  tot /= N;
#pragma unroll
  for (int c = 0; c < CH; ++c) {
    const int col = ((c * WPR + pw) * 64 + lane) * 8;
    float o[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      o[i] = r * (gv[c][i] * (w ? (float)wb[c][i] : 1.f) - xv[c][i] * tot);
      if (dres) o[i] += (float)rb[c][i];
    }
    store8(dx + ro + col, o);
  }
}

// waves per row: 2 (4 measured no faster at the Qwen3 widths); the template's CH is N / (512·WPR)
static int norm_wpr(int) { return 2; }

// split-row form for bf16 rows of N = 1024·{1, 2, 4, 8}
static int norm_split_ch(int dtype, int N) {
  if (dtype != 1 || N % 1024) return 0;
  const int ch = N / 1024;
  return (ch == 1 || ch == 2 || ch == 4 || ch == 8) ? ch : 0;
}

}  // namespace

// ------------------------------------------------------------------------------ launchers
// dtype: 0 = fp32, 1 = bf16 (activations and weight share the dtype)
void launch_rmsnorm_fwd(int dtype, const void* x, const void* w, void* y, float* rstd, int M, int N, float eps,
                        hipStream_t st) {
  if (const int ch = norm_split_ch(dtype, N)) {
    const int wpr = norm_wpr(ch);
    dim3 g2((M * wpr + 3) / 4), b2(256);
#define S(CH_, W_)                                                                                                \
  rmsnorm_fwd_split_k<CH_, W_><<<g2, b2, 0, st>>>((const bf16*)x, (const bf16*)w, (bf16*)y, rstd, M, N, eps)
    if (wpr == 4) {
      if (ch == 2) S(1, 4); else if (ch == 4) S(2, 4); else S(4, 4);
    } else {
      if (ch == 1) S(1, 2); else if (ch == 2) S(2, 2); else if (ch == 4) S(4, 2); else S(8, 2);
    }
#undef S
    LIPA_CHECK_LAUNCH();
    return;
  }
  dim3 g((M + ROWS - 1) / ROWS), b(256);
#define F(CH)                                                                                                  \
  if (dtype == 1)                                                                                              \
    rmsnorm_fwd_k<bf16, bf16, CH><<<g, b, 0, st>>>((const bf16*)x, (const bf16*)w, (bf16*)y, rstd, M, N, eps); \
  else                                                                                                         \
    rmsnorm_fwd_k<float, float, CH><<<g, b, 0, st>>>((const float*)x, (const float*)w, (float*)y, rstd, M, N, eps);
  LIPA_CH_DISPATCH(N, F);
#undef F
  LIPA_CHECK_LAUNCH();
}

void launch_rmsnorm_bwd(int dtype, const void* dy, const void* x, const void* w, const float* rstd, void* dx,
                        float* dw_part, float* dw, int M, int N, const void* dres, hipStream_t st) {
  if (const int ch = dw_part ? 0 : norm_split_ch(dtype, N)) {
    const int wpr = norm_wpr(ch);
    dim3 g2((M * wpr + 3) / 4), b2(256);
#define S(CH_, W_)                                                                                          \
  rmsnorm_bwd_split_k<CH_, W_><<<g2, b2, 0, st>>>((const bf16*)dy, (const bf16*)x, (const bf16*)w, rstd, \
                                                 (bf16*)dx, M, N, (const bf16*)dres)
    if (wpr == 4) {
      if (ch == 2) S(1, 4); else if (ch == 4) S(2, 4); else S(4, 4);
    } else {
      if (ch == 1) S(1, 2); else if (ch == 2) S(2, 2); else if (ch == 4) S(4, 2); else S(8, 2);
    }
#undef S
    LIPA_CHECK_LAUNCH();
    return;
  }
  dim3 g((M + ROWS - 1) / ROWS), b(256);
#define F(CH)                                                                                               \
  if (dtype == 1)                                                                                           \
    rmsnorm_bwd_k<bf16, bf16, CH><<<g, b, 0, st>>>((const bf16*)dy, (const bf16*)x, (const bf16*)w, rstd,   \
                                                   (bf16*)dx, dw_part, M, N, (const bf16*)dres);          \
  else                                                                                                      \
    rmsnorm_bwd_k<float, float, CH><<<g, b, 0, st>>>((const float*)dy, (const float*)x, (const float*)w,    \
                                                     rstd, (float*)dx, dw_part, M, N, (const float*)dres);
  LIPA_CH_DISPATCH(N, F);
#undef F
  if (dw_part) colsum_k<<<(N + 255) / 256, 256, 0, st>>>(dw_part, dw, g.x, N);
  LIPA_CHECK_LAUNCH();
}

void launch_layernorm_fwd(int dtype, const void* x, const void* w, const void* bias, void* y, float* mean,
                          float* rstd, int M, int N, float eps, hipStream_t st) {
  dim3 g((M + ROWS - 1) / ROWS), b(256);
#define F(CH)                                                                                            \
  if (dtype == 1)                                                                                        \
    layernorm_fwd_k<bf16, bf16, CH><<<g, b, 0, st>>>((const bf16*)x, (const bf16*)w, (const bf16*)bias, \
                                                     (bf16*)y, mean, rstd, M, N, eps);                   \
  else                                                                                                   \
    layernorm_fwd_k<float, float, CH><<<g, b, 0, st>>>((const float*)x, (const float*)w,                \
                                                       (const float*)bias, (float*)y, mean, rstd, M, N, eps);
  LIPA_CH_DISPATCH(N, F);
#undef F
  LIPA_CHECK_LAUNCH();
}

void launch_layernorm_bwd(int dtype, const void* dy, const void* x, const void* w, const float* mean,
                          const float* rstd, void* dx, float* part, float* dw, float* db, int M, int N,
                          hipStream_t st) {
  dim3 g((M + ROWS - 1) / ROWS), b(256);
  float* dwp = part;
  float* dbp = part ? part + (size_t)g.x * N : nullptr;
#define F(CH)                                                                                              \
  if (dtype == 1)                                                                                          \
    layernorm_bwd_k<bf16, bf16, CH><<<g, b, 0, st>>>((const bf16*)dy, (const bf16*)x, (const bf16*)w, mean, \
                                                     rstd, (bf16*)dx, dwp, dbp, M, N);                     \
  else                                                                                                     \
    layernorm_bwd_k<float, float, CH><<<g, b, 0, st>>>((const float*)dy, (const float*)x,                  \
                                                       (const float*)w, mean, rstd, (float*)dx, dwp, dbp, M, N);
  LIPA_CH_DISPATCH(N, F);
#undef F
  if (part) {
    colsum_k<<<(N + 255) / 256, 256, 0, st>>>(dwp, dw, g.x, N);
    colsum_k<<<(N + 255) / 256, 256, 0, st>>>(dbp, db, g.x, N);
  }
  LIPA_CHECK_LAUNCH();
}

int norm_partial_rows(int M) { return (M + ROWS - 1) / ROWS; }
