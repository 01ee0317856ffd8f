// Fused LoRA low-rank kernels (SURVEY.md K8 + K13): every skinny product of a LoRA branch in one
// pass over the activations, with the input dropout mask regenerated in-kernel (never stored).
//
// A rank-r branch (r <= 16) of y += s·D(x)·Aᵀ·Bᵀ needs, per training step:
//   fwd  xa_s = s·D(x)·Aᵀ                 [M, r]   (feeds the base GEMM's extra K-slice)
//   bwd  g    = s·dy_i·B                  [M, r]
//        dA   = gᵀ·D(x)                   [r, K]
//        dB   = dy_iᵀ·xa_s                [n, r]
//        dx  += D'(g·A)                   [M, K]   (dropout branches; others fold into the base GEMM)
// The previous composition (dropout kernel → hipBLASLt skinny GEMMs → scale / cast / add
// kernels → materialised g·A) cost ≈125 µs per branch per step on Qwen3-8B shapes (rocprofv3,
// profiles/bench_qwen3_8b_qlora_kernels_v2.txt) for ≈20 µs of compulsory HBM traffic.
//
// lora_proj_k  (MFMA): out[m, j] = scale·Σ_k D(X)[m,k]·W[j,k] — a workgroup = 16 rows × 1024 of K
//              (grid M/16 × K/1024 for enough memory parallelism), its 4 waves each own 256 of K with
//              all 8 fragment loads in flight, v_mfma_f32_16x16x32_bf16 with X rows as the A operand
//              (dropout applied to the fragment) and W rows as the B operand; LDS reduction of the 4
//              partials, one fp32 atomic add per output element per workgroup.
// lora_acc_k   (VALU): part[c][j][k] = Σ_{m∈chunk c} G[m,j]·D(X)[m,k]  and optionally
//              DX[m,k] += D(Σ_j G[m,j]·W[j,k]) — each thread owns 8 consecutive k of one row stream,
//              reads X and DX once; the per-chunk (64-row) partials are summed by the caller.
#include "common.h"

using namespace lipa;

namespace {

// One workgroup = 16 rows × ALL of K: its NW waves each own K/NW (all fragment loads of a wave in
// flight at once), partials meet in LDS and the result is written once (fp32 and/or bf16) — no
// atomics, no zero-initialised output, no follow-up cast kernel.
template <int NW>
__global__ __launch_bounds__(NW * 64) void lora_proj_k(const bf16* __restrict__ X, int ldx, const bf16* __restrict__ W,
                                                      int r, int K, float* __restrict__ outf, int ldof,
                                                      bf16* __restrict__ outb, int ldob, int M, uint64_t key,
                                                      uint32_t thr16, float dscale, float scale, size_t mask_ld) {
  __shared__ f32x4 red[NW][64];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int m0 = blockIdx.x * 16;
  const int row = min(m0 + (lane & 15), M - 1);
  const int kw = K / NW;
  const int kbeg = w * kw;
  const bf16* xr = X + (size_t)row * ldx;
  const int n = lane & 15;
  const bf16* wr = W + (size_t)(n < r ? n : 0) * K;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  for (int k0 = kbeg; k0 < kbeg + kw; k0 += 8 * 32) {
    bf16x8 av[8], bv[8];
    const int ns = min(8, (kbeg + kw - k0) / 32);
#pragma unroll
    for (int s = 0; s < 8; ++s)
      if (s < ns) {
        const int k = k0 + s * 32 + 8 * (lane >> 4);
        av[s] = *reinterpret_cast<const bf16x8*>(xr + k);
        bv[s] = *reinterpret_cast<const bf16x8*>(wr + k);
      }
#pragma unroll
    for (int s = 0; s < 8; ++s)
      if (s < ns) {
        bf16x8 a = av[s];
        if (thr16) {
          const int k = k0 + s * 32 + 8 * (lane >> 4);
          const uint32_t keep = dropout_keep8(key, ((size_t)row * mask_ld + k) >> 3, thr16);
#pragma unroll
          for (int i = 0; i < 8; ++i) a[i] = ((keep >> i) & 1) ? (bf16)((float)a[i] * dscale) : (bf16)0.f;
        }
        const bf16x8 b = n < r ? bv[s] : bf16x8{};
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc, 0, 0, 0);
      }
  }
  red[w][lane] = acc;
  __syncthreads();
  if (w != 0) return;
  f32x4 t = red[0][lane];
#pragma unroll
  for (int i = 1; i < NW; ++i) t += red[i][lane];
  // D layout: col = lane & 15 (output j), rows 4*(lane>>4)+i (token)
  const int j = lane & 15;
  if (j >= r) return;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int m = m0 + 4 * (lane >> 4) + i;
    if (m >= M) continue;
    const float v = t[i] * scale;
    if (outf) outf[(size_t)m * ldof + j] = v;
    if (outb) outb[(size_t)m * ldob + j] = (bf16)v;
  }
}

template <int R, bool DXU>
__global__ __launch_bounds__(256) void lora_acc_k(const float* __restrict__ G, int ldg, int r,
                                                 const bf16* __restrict__ X, int ldx, bf16* __restrict__ DX, int lddx,
                                                 const bf16* __restrict__ W, int K, float* __restrict__ out,
                                                 int64_t sj, int64_t sk, float* __restrict__ part, int M,
                                                 int rows_per_chunk, uint64_t key, uint32_t thr16, float dscale,
                                                 size_t mask_ld) {
  __shared__ float red[64][R * 8 + 1];
  const int tid = threadIdx.x;
  const int kv = blockIdx.x * 64 + (tid & 63), rl = tid >> 6;
  const int k0 = kv * 8;
  const bool kin = k0 < K;
  const int c = blockIdx.y;
  const int mb = c * rows_per_chunk, me = min(mb + rows_per_chunk, M);
  float acc[R][8];
#pragma unroll
  for (int j = 0; j < R; ++j)
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[j][i] = 0.f;
  bf16x8 wv[DXU ? R : 1];
  if constexpr (DXU) {
#pragma unroll
    for (int j = 0; j < R; ++j) wv[j] = (kin && j < r) ? *reinterpret_cast<const bf16x8*>(W + (size_t)j * K + k0) : bf16x8{};
  }
  // rows m = mb + rl + 4i; RB rows are loaded together (x, dx, g) so RB × 16-32 B per thread are in
  // flight — one dependent HBM round trip per RB rows instead of per row
  constexpr int RB = 4;
  const float ds = thr16 ? dscale : 1.f;
  for (int m0 = mb + rl; kin && m0 < me; m0 += 4 * RB) {
    float xv[RB][8], dv[DXU ? RB : 1][8], g[RB][R];
    uint32_t keep[RB];
#pragma unroll
    for (int q = 0; q < RB; ++q) {
      const int m = min(m0 + 4 * q, M - 1);
      load8(X + (size_t)m * ldx + k0, xv[q]);
      if constexpr (DXU) load8(DX + (size_t)m * lddx + k0, dv[q]);
#pragma unroll
      for (int j = 0; j < R; ++j) g[q][j] = (j < r && m0 + 4 * q < me) ? G[(size_t)m * ldg + j] : 0.f;
      keep[q] = thr16 ? dropout_keep8(key, ((size_t)m * mask_ld + k0) >> 3, thr16) : 0xFFu;
    }
#pragma unroll
    for (int q = 0; q < RB; ++q) {
#pragma unroll
      for (int i = 0; i < 8; ++i) xv[q][i] = ((keep[q] >> i) & 1) ? xv[q][i] * ds : 0.f;
#pragma unroll
      for (int j = 0; j < R; ++j)
#pragma unroll
        for (int i = 0; i < 8; ++i) acc[j][i] += g[q][j] * xv[q][i];
      if constexpr (DXU) {
        if (m0 + 4 * q < me) {
          float t[8];
#pragma unroll
          for (int i = 0; i < 8; ++i) t[i] = 0.f;
#pragma unroll
          for (int j = 0; j < R; ++j)
#pragma unroll
            for (int i = 0; i < 8; ++i) t[i] += g[q][j] * (float)wv[j][i];
#pragma unroll
          for (int i = 0; i < 8; ++i) dv[q][i] += ((keep[q] >> i) & 1) ? t[i] * ds : 0.f;
          store8(DX + (size_t)(m0 + 4 * q) * lddx + k0, dv[q]);
        }
      }
    }
  }
  // reduce the 4 row-lanes through LDS (one wave at a time), then write this chunk's partial
  for (int s = 0; s < 4; ++s) {
    if (rl == s) {
#pragma unroll
      for (int j = 0; j < R; ++j)
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          float& dst = red[tid & 63][j * 8 + i];
          dst = (s == 0 ? 0.f : dst) + acc[j][i];
        }
    }
    __syncthreads();
  }
  // this workgroup's 512-wide k block: 256 threads add j-rows with consecutive k per lane (full-rate
  // 256-B atomic wave instructions when sk == 1), straight into the fp32 destination (the grad)
  const int kb = blockIdx.x * 512;
  const bool jfast = sj == 1;        // order lanes along the destination's unit stride (full-rate atomics)
  for (int idx = tid; idx < r * 512; idx += 256) {
    const int j = jfast ? idx % r : idx / 512, kk = jfast ? idx / r : idx % 512;
    if (kb + kk >= K) continue;
    const float v = red[kk / 8][j * 8 + (kk & 7)];
    if (part)   // deterministic mode: per-chunk partial, summed in a fixed order by the caller
      part[((size_t)blockIdx.y * r + j) * K + kb + kk] = v;
    else
      atomicAdd(out + j * sj + (int64_t)(kb + kk) * sk, v);
  }
}

}  // namespace

// X row stride ldx (elements), W [r, K] bf16 contiguous; K % 32 == 0; outf/outb may each be null.
void launch_lora_proj(const void* X, int ldx, const void* W, int r, int K, float* outf, int ldof, void* outb, int ldob,
                      int M, uint64_t key, float p, float scale, size_t mask_ld, hipStream_t st) {
  const uint32_t thr = p > 0.f ? (uint32_t)(p * 65536.0f + 0.5f) : 0u;
  const float ds = p > 0.f ? 1.f / (1.f - p) : 1.f;
  const int grid = (M + 15) / 16;
  if (K % (16 * 32) == 0)
    lora_proj_k<16><<<grid, 1024, 0, st>>>((const bf16*)X, ldx, (const bf16*)W, r, K, outf, ldof, (bf16*)outb, ldob,
                                           M, key, thr, ds, scale, mask_ld);
  else
    lora_proj_k<1><<<grid, 64, 0, st>>>((const bf16*)X, ldx, (const bf16*)W, r, K, outf, ldof, (bf16*)outb, ldob, M,
                                        key, thr, ds, scale, mask_ld);
  LIPA_CHECK_LAUNCH();
}

// out[j*sj + k*sk] += Σ_m G[m,j]·D(X)[m,k] (fp32 atomics: accumulate straight into a gradient), or
// with part != null the per-64-row-chunk partials [chunks, r, K] (deterministic mode);
// with DX: DX[m,k] += D(Σ_j G[m,j]·W[j,k]).
int lora_acc_chunks(int M) { return (M + 63) / 64; }

void launch_lora_acc(const float* G, int ldg, int r, const void* X, int ldx, void* DX, int lddx, const void* W, int K,
                     float* out, int64_t sj, int64_t sk, float* part, int M, uint64_t key, float p, size_t mask_ld,
                     hipStream_t st) {
  const uint32_t thr = p > 0.f ? (uint32_t)(p * 65536.0f + 0.5f) : 0u;
  const float ds = p > 0.f ? 1.f / (1.f - p) : 1.f;
  const int rows = 64;
  dim3 grid((K / 8 + 63) / 64, (M + rows - 1) / rows);
#define A(R_, D_)                                                                                             \
  lora_acc_k<R_, D_><<<grid, 256, 0, st>>>(G, ldg, r, (const bf16*)X, ldx, (bf16*)DX, lddx, (const bf16*)W, K, \
                                           out, sj, sk, part, M, rows, key, thr, ds, mask_ld)
  if (r <= 8) {
    if (DX) A(8, true); else A(8, false);
  } else {
    if (DX) A(16, true); else A(16, false);
  }
#undef A
  LIPA_CHECK_LAUNCH();
}
