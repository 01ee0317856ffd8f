// Decode-time weight GEMV for 4-bit weights (SURVEY.md K9/K15 small-M variant): Y[M,N] =
// X[M,K]·deq(W)ᵀ for M <= 8 tokens (one decode step of a small batch).
//
// At M <= 8 an MFMA tile wastes >= 94 % of its rows and the kernel is bound by the weight
// stream (N·K/2 bytes), so this path never touches the matrix cores or LDS staging:
//  * weights are read in their storage layout (codes [N][K/2] bytes, high nibble = even k;
//    block scales [N][K/blk] fp32), 16 B (32 weights) per lane per load, each wave owns
//    COLS columns and keeps COLS loads in flight;
//  * the block scale is applied once per 32-weight chunk: Σ x·(lut[q]·s) = s·Σ x·lut[q], and for
//    affine int4 Σ x·(q·s + b) = s·Σ x·q + b·Σ x — one FMA per weight;
//  * activations come straight from L2 (16 B loads), partial dots are wave-reduced by xor
//    shuffles, lane 0 writes bf16 (+ optional residual).
// MODE 0 = NF4 (blocksize 64), MODE 2 = affine int4 (group size g, bias = −z·s).
#include "common.h"

using namespace lipa;

namespace {

__constant__ float kNF4g[16] = {
    -1.0f, -0.6961928009986877f, -0.5250730514526367f, -0.39491748809814453f,
    -0.28444138169288635f, -0.18477343022823334f, -0.09105003625154495f, 0.0f,
    0.07958029955625534f, 0.16093020141124725f, 0.24611230194568634f, 0.33791524171829224f,
    0.44070982933044434f, 0.5626170039176941f, 0.7229568362236023f, 1.0f};

constexpr int GV_THR = 256;
constexpr int COLS = 4;  // columns per wave

template <int MODE, int MR>
__global__ __launch_bounds__(GV_THR) void gemv_w4_k(const bf16* __restrict__ x, int ldx, const uint8_t* __restrict__ codes,
                                                    const float* __restrict__ sc, const float* __restrict__ bi,
                                                    int blk, const bf16* __restrict__ residual,
                                                    bf16* __restrict__ out, int M, int N, int K) {
  __shared__ float lut[16];
  if (threadIdx.x < 16) lut[threadIdx.x] = MODE == 0 ? kNF4g[threadIdx.x] : (float)threadIdx.x;
  __syncthreads();
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int n0 = (blockIdx.x * (GV_THR / 64) + w) * COLS;
  if (n0 >= N) return;
  const int nb = K / blk;
  float acc[COLS][MR];
#pragma unroll
  for (int c = 0; c < COLS; ++c)
#pragma unroll
    for (int m = 0; m < MR; ++m) acc[c][m] = 0.f;

  for (int k0 = lane * 32; k0 < K; k0 += 64 * 32) {
    // all COLS weight chunks + scales first (COLS 16-B loads in flight), then 4 sub-chunks of 8
    u32x4 q[COLS];
    float s[COLS], b[COLS];
#pragma unroll
    for (int c = 0; c < COLS; ++c) {
      const int n = min(n0 + c, N - 1);
      q[c] = *reinterpret_cast<const u32x4*>(codes + (size_t)n * (K / 2) + k0 / 2);
      s[c] = sc[(size_t)n * nb + k0 / blk];
      b[c] = MODE == 2 ? bi[(size_t)n * nb + k0 / blk] : 0.f;
    }
    float d[COLS][MR];
    float xs[MR];
#pragma unroll
    for (int m = 0; m < MR; ++m) {
      xs[m] = 0.f;
#pragma unroll
      for (int c = 0; c < COLS; ++c) d[c][m] = 0.f;
    }
#pragma unroll
    for (int dw = 0; dw < 4; ++dw) {
      float xv[MR][8];
#pragma unroll
      for (int m = 0; m < MR; ++m) {
        const int mm = m < M ? m : 0;
        const bf16x8 t = *reinterpret_cast<const bf16x8*>(x + (size_t)mm * ldx + k0 + dw * 8);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          xv[m][j] = m < M ? (float)t[j] : 0.f;
          xs[m] += xv[m][j];
        }
      }
#pragma unroll
      for (int c = 0; c < COLS; ++c) {
        const uint32_t word = q[c][dw];
#pragma unroll
        for (int by = 0; by < 4; ++by) {
          const uint32_t byte = (word >> (8 * by)) & 0xFF;
          const float vhi = lut[byte >> 4], vlo = lut[byte & 15];   // high nibble = even k
#pragma unroll
          for (int m = 0; m < MR; ++m) d[c][m] += xv[m][2 * by] * vhi + xv[m][2 * by + 1] * vlo;
        }
      }
    }
#pragma unroll
    for (int c = 0; c < COLS; ++c)
#pragma unroll
      for (int m = 0; m < MR; ++m) acc[c][m] += d[c][m] * s[c] + (MODE == 2 ? b[c] * xs[m] : 0.f);
  }
#pragma unroll
  for (int c = 0; c < COLS; ++c)
#pragma unroll
    for (int m = 0; m < MR; ++m) acc[c][m] = wave_sum(acc[c][m]);
  if (lane == 0) {
#pragma unroll
    for (int c = 0; c < COLS; ++c) {
      const int n = n0 + c;
      if (n >= N) break;
#pragma unroll
      for (int m = 0; m < MR; ++m) {
        if (m >= M) break;
        float v = acc[c][m];
        if (residual) v += (float)residual[(size_t)m * N + n];
        out[(size_t)m * N + n] = (bf16)v;
      }
    }
  }
}

}  // namespace

// codes: bnb byte layout [N][K/2]; sc: [N][K/blk] fp32 (NF4: decoded absmax, blk 64; int4: scale);
// bi: [N][K/blk] fp32 (int4 bias = −zero·scale) or null.  Requires K % 32 == 0 and blk % 32 == 0.
void launch_gemv_w4(int mode, const void* x, int ldx, const uint8_t* codes, const float* sc, const float* bi, int blk,
                    const void* residual, void* out, int M, int N, int K, hipStream_t st) {
  const int per_block = (GV_THR / 64) * COLS;
  const int grid = (N + per_block - 1) / per_block;
#define G(MODE_, MR_)                                                                                        \
  gemv_w4_k<MODE_, MR_><<<grid, GV_THR, 0, st>>>((const bf16*)x, ldx, codes, sc, bi, blk,                   \
                                                 (const bf16*)residual, (bf16*)out, M, N, K)
  if (mode == 0) {
    if (M <= 1) G(0, 1); else if (M <= 2) G(0, 2); else if (M <= 4) G(0, 4); else G(0, 8);
  } else {
    if (M <= 1) G(2, 1); else if (M <= 2) G(2, 2); else if (M <= 4) G(2, 4); else G(2, 8);
  }
#undef G
  LIPA_CHECK_LAUNCH();
}
