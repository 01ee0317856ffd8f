// Decode-time weight GEMV for 4-bit weights (SURVEY.md K9/K15 small-M variant): Y[M,N] =
// X[M,K]·deq(W)ᵀ for M <= 8 tokens (one decode step of a small batch; int4 dispatches it at M <= 2).
//
// At M <= 8 an MFMA tile wastes >= 94 % of its rows and the kernel is bound by the weight
// stream (N·K/2 bytes), so this path never touches the matrix cores or LDS staging:
//  * weights are read in their storage layout (codes [N][K/2] bytes, high nibble = even k;
//    block scales [N][K/blk] fp32), 16 B (32 weights) per lane per load, each wave owns
//    COLS columns; the next iteration's codes (and x, M <= 2) load while the current one computes;
//  * the block scale is applied once per 32-weight chunk: Σ x·(lut[q]·s) = s·Σ x·lut[q] (NF4, codebook
//    in LDS), and for affine int4 Σ x·(q·s + b) = s·Σ x·(128+q) + (b − 128s)·Σ x with bf16(128+q)
//    made by a byte permute and summed by v_dot2_f32_bf16 (no table, no conversion);
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

__device__ __forceinline__ uint32_t vperm(uint32_t hi, uint32_t lo, uint32_t sel) {
  return __builtin_amdgcn_perm(hi, lo, sel);
}

// v_dot2_f32_bf16: acc + a.lo·b.lo + a.hi·b.hi on two packed bf16 pairs.  The builtin is declared on
// short2 — the operands must be BIT-cast to it (a bf16x2 argument would be value-converted to int16)
typedef short s16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ float dot2bf(uint32_t a, uint32_t b, float acc) {
  return __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(s16x2, a), __builtin_bit_cast(s16x2, b), acc, false);
}

// One 16-B chunk per column: 32 weights of k = k0 .. k0+31 (byte i of a dword = q[2i] << 4 | q[2i+1]).
template <int MR>
struct GvSet {
  u32x4 q[COLS];
  float s[COLS], b[COLS];
  u32x4 x[MR][4];   // x[m][k0 + 8dw .. +8] (MR <= 2: prefetched with the codes; else loaded at use)
};

template <int MODE, int MR>
__global__ __launch_bounds__(GV_THR) void gemv_w4_k(const bf16* __restrict__ x, int ldx, const uint8_t* __restrict__ codes,
                                                    const float* __restrict__ sc, const float* __restrict__ bi,
                                                    int blk, const bf16* __restrict__ residual,
                                                    bf16* __restrict__ out, int M, int N, int K) {
  constexpr bool PX = MR <= 2 && MODE == 2;
  __shared__ float lut[16];
  if (MODE == 0) {
    if (threadIdx.x < 16) lut[threadIdx.x] = kNF4g[threadIdx.x];
    __syncthreads();
  }
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int n0 = (blockIdx.x * (GV_THR / 64) + w) * COLS;
  if (n0 >= N) return;
  const int nb = K / blk;
  float acc[COLS][MR];
#pragma unroll
  for (int c = 0; c < COLS; ++c)
#pragma unroll
    for (int m = 0; m < MR; ++m) acc[c][m] = 0.f;

  auto load = [&](GvSet<MR>& st, int k0) {
#pragma unroll
    for (int c = 0; c < COLS; ++c) {
      const int n = min(n0 + c, N - 1);
      st.q[c] = *reinterpret_cast<const u32x4*>(codes + (size_t)n * (K / 2) + k0 / 2);
      st.s[c] = sc[(size_t)n * nb + k0 / blk];
      st.b[c] = MODE == 2 ? bi[(size_t)n * nb + k0 / blk] : 0.f;
    }
    if constexpr (PX) {
#pragma unroll
      for (int m = 0; m < MR; ++m)
#pragma unroll
        for (int dw = 0; dw < 4; ++dw)
          st.x[m][dw] = *reinterpret_cast<const u32x4*>(x + (size_t)(m < M ? m : 0) * ldx + k0 + dw * 8);
    }
  };
  auto compute = [&](GvSet<MR>& st, int k0) {
    if constexpr (!PX) {
#pragma unroll
      for (int m = 0; m < MR; ++m)
#pragma unroll
        for (int dw = 0; dw < 4; ++dw)
          st.x[m][dw] = *reinterpret_cast<const u32x4*>(x + (size_t)(m < M ? m : 0) * ldx + k0 + dw * 8);
    }
    if constexpr (MODE == 2) {
      // affine int4: a nibble q becomes bf16(128 + q) by one byte permute (0x43 = the exponent of 128);
      // Σ x·(128+q) by v_dot2_f32_bf16 with x in the same permuted pair order, then per chunk
      // s·G + (b − 128·s)·Σx.  No LDS, one permute + one dot per weight pair.
      constexpr uint32_t C43 = 0x43434343u, ONES = 0x3F803F80u;
      u32x4 xp[MR][4];
      float xs[MR];
#pragma unroll
      for (int m = 0; m < MR; ++m) {
        xs[m] = 0.f;
#pragma unroll
        for (int dw = 0; dw < 4; ++dw) {
          const u32x4 d = st.x[m][dw];
          xp[m][dw][0] = vperm(d[1], d[0], 0x07060302u);   // (x1, x3)
          xp[m][dw][1] = vperm(d[3], d[2], 0x07060302u);   // (x5, x7)
          xp[m][dw][2] = vperm(d[1], d[0], 0x05040100u);   // (x0, x2)
          xp[m][dw][3] = vperm(d[3], d[2], 0x05040100u);   // (x4, x6)
#pragma unroll
          for (int p = 0; p < 4; ++p)
            xs[m] = dot2bf(xp[m][dw][p], ONES, xs[m]);
        }
      }
#pragma unroll
      for (int c = 0; c < COLS; ++c) {
        float g[MR];
#pragma unroll
        for (int m = 0; m < MR; ++m) g[m] = 0.f;
#pragma unroll
        for (int dw = 0; dw < 4; ++dw) {
          const uint32_t wd = st.q[c][dw];
          const uint32_t lo = wd & 0x0F0F0F0Fu, hi = (wd >> 4) & 0x0F0F0F0Fu;
          const uint32_t wp[4] = {vperm(C43, lo, 0x04010400u), vperm(C43, lo, 0x04030402u),
                                  vperm(C43, hi, 0x04010400u), vperm(C43, hi, 0x04030402u)};
#pragma unroll
          for (int p = 0; p < 4; ++p)
#pragma unroll
            for (int m = 0; m < MR; ++m)
              g[m] = dot2bf(wp[p], xp[m][dw][p], g[m]);
        }
        const float s = st.s[c], cc = st.b[c] - 128.f * s;
#pragma unroll
        for (int m = 0; m < MR; ++m) acc[c][m] += s * g[m] + cc * xs[m];
      }
    } else {
      // NF4: codebook from LDS, Σ x·cb[q] per chunk, × absmax (x converted once per 8 values, shared by
      // the COLS columns)
      float d[COLS][MR];
#pragma unroll
      for (int c = 0; c < COLS; ++c)
#pragma unroll
        for (int m = 0; m < MR; ++m) d[c][m] = 0.f;
#pragma unroll
      for (int dw = 0; dw < 4; ++dw) {
        float xv[MR][8];
#pragma unroll
        for (int m = 0; m < MR; ++m) {
          const bf16x8 t = __builtin_bit_cast(bf16x8, st.x[m][dw]);
#pragma unroll
          for (int j = 0; j < 8; ++j) xv[m][j] = m < M ? (float)t[j] : 0.f;
        }
#pragma unroll
        for (int c = 0; c < COLS; ++c) {
          const uint32_t word = st.q[c][dw];
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
        for (int m = 0; m < MR; ++m) acc[c][m] += d[c][m] * st.s[c];
    }
  };

  // the codes (and, MR <= 2, the x chunk) of iteration it + 1 are in flight while iteration it computes
  const int nit = K > lane * 32 ? (K - lane * 32 + 2047) / 2048 : 0;
  GvSet<MR> sa, sb;
  if constexpr (MODE == 0) {   // NF4: the LDS codebook reads already hold ~100 VGPRs; a second code set
    for (int it = 0; it < nit; ++it) {   // would halve the occupancy (4 → 2 waves/SIMD) for nothing
      load(sa, lane * 32 + it * 2048);
      compute(sa, lane * 32 + it * 2048);
    }
  } else {
  if (nit > 0) load(sa, lane * 32);
  for (int it = 0; it < nit; it += 2) {
    if (it + 1 < nit) load(sb, lane * 32 + (it + 1) * 2048);
    compute(sa, lane * 32 + it * 2048);
    if (it + 1 < nit) {
      if (it + 2 < nit) load(sa, lane * 32 + (it + 2) * 2048);
      compute(sb, lane * 32 + (it + 1) * 2048);
    }
  }
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
