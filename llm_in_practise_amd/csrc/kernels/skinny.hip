// Decode-shaped bf16 GEMM (SURVEY.md K8 at serving sizes): y[M, N] = x[M, K] · W[N, K]ᵀ (+ residual)
// for M <= 64 — the weight-streaming regime, where the whole cost is reading W once from HBM.
//
// hipBLASLt reaches 2-4.7 TB/s on these shapes (profiles/decode_skinny_gemm.txt: 128-column
// tiles give N/128 workgroups, too few loads in flight).  Here:
//  * grid (N/128, S): a workgroup owns 128 rows of W (4 waves x 32) and 1/S of K (split-K, S chosen
//    on the host so that >= ~512 workgroups stream W); XCD-aware remap so the S splits of one
//    N-block share an L2;
//  * a wave's two 16-row W fragments are the MFMA A operands, loaded straight from HBM (16 B per
//    lane, eight k-steps in flight); x (tiny, L2-resident) supplies the B operands of up to four
//    16-column m-tiles, so every W byte feeds MT MFMAs (v_mfma_f32_16x16x32_bf16);
//  * split-K partials go to an fp32 [S, M, N] buffer; a second kernel sums the S slices, adds the
//    residual and writes bf16 (deterministic — no atomics).
#include <cstdlib>

#include "common.h"

using namespace lipa;

namespace {

constexpr int SK_NB = 128;      // W rows per workgroup
constexpr int SK_KS = 8;        // k-steps (of 32) per load batch

template <int MT>
__global__ __launch_bounds__(256) void gemm_skinny_k(const bf16* __restrict__ X, int ldx, const bf16* __restrict__ W,
                                                     float* __restrict__ part, int M, int N, int K, int kc) {
  const int nblk = gridDim.x, S = gridDim.y;
  const int id = xcd_remap(blockIdx.x * S + blockIdx.y, nblk * S);
  const int bn = id / S, sp = id % S;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, li = lane & 15, g = lane >> 4;
  const int n0 = bn * SK_NB + 32 * w;
  const int k0 = sp * kc, k1 = min(K, k0 + kc);
  const bf16* wr0 = W + (size_t)min(n0 + li, N - 1) * K + 8 * g;
  const bf16* wr1 = W + (size_t)min(n0 + 16 + li, N - 1) * K + 8 * g;
  const bf16* xr[MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) xr[mt] = X + (size_t)min(16 * mt + li, M - 1) * ldx + 8 * g;
  f32x4 acc[2][MT];
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) acc[t][mt] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int kb = k0; kb < k1; kb += 32 * SK_KS) {
    const int ns = min(SK_KS, (k1 - kb) / 32);
    bf16x8 a0[SK_KS], a1[SK_KS];
#pragma unroll
    for (int s = 0; s < SK_KS; ++s)
      if (s < ns) {
        a0[s] = *reinterpret_cast<const bf16x8*>(wr0 + kb + 32 * s);
        a1[s] = *reinterpret_cast<const bf16x8*>(wr1 + kb + 32 * s);
      }
#pragma unroll
    for (int s = 0; s < SK_KS; ++s)
      if (s < ns) {
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) {
          const bf16x8 b = *reinterpret_cast<const bf16x8*>(xr[mt] + kb + 32 * s);
          acc[0][mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0[s], b, acc[0][mt], 0, 0, 0);
          acc[1][mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1[s], b, acc[1][mt], 0, 0, 0);
        }
      }
  }
  // lane holds C[n = n0 + 16t + 4g + i][m = 16mt + li]
  float* pp = part + (size_t)sp * M * N;
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
    const int m = 16 * mt + li;
    if (m >= M) continue;
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int n = n0 + 16 * t + 4 * g;
      if (n < N) *reinterpret_cast<f32x4*>(pp + (size_t)m * N + n) = acc[t][mt];
    }
  }
}


// ---- W4A16 variant (SURVEY.md K15 at decode batch sizes): the same split-K weight-streaming
// structure, W read as 4-bit codes (uint8 [N, K/2], high nibble = even k) with one fp32 scale and
// bias (= −zero·scale) per (row, group).  A lane's A fragment for k-step s of a 128-deep block is
// the 8 weights k = kb + 32g + 8s + [0, 8): the four k-steps of one 128-block come from ONE 16-byte
// code load per lane (x is read with the same k permutation, so the MFMA sum is unchanged).
// Dequant: nibbles split into bytes (2 ANDs + 1 shift per 8 weights), byte → f32 conversion, one
// FMA with (scale, bias), packed to bf16 pairs that are already in k order.
__device__ __forceinline__ bf16x8 dequant8(uint32_t w, float sc, float bi) {
  const uint32_t hi = (w >> 4) & 0x0F0F0F0Fu, lo = w & 0x0F0F0F0Fu;
  bf16x8 r;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    r[2 * j] = (bf16)fmaf((float)((hi >> (8 * j)) & 0xFFu), sc, bi);
    r[2 * j + 1] = (bf16)fmaf((float)((lo >> (8 * j)) & 0xFFu), sc, bi);
  }
  return r;
}

template <int MT, bool PAD>
__global__ __launch_bounds__(256) void gemm_w4_skinny_k(const bf16* __restrict__ X, int ldx,
                                                        const uint8_t* __restrict__ codes,
                                                        const float* __restrict__ scales,
                                                        const float* __restrict__ biases, int gs,
                                                        float* __restrict__ part, int M, int N, int K, int kc) {
  const int nblk = gridDim.x, S = gridDim.y;
  const int id = xcd_remap(blockIdx.x * S + blockIdx.y, nblk * S);
  const int bn = id / S, sp = id % S;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, li = lane & 15, g = lane >> 4;
  const int n0 = bn * SK_NB + 32 * w;
  const int k0 = sp * kc, k1 = min(K, k0 + kc);
  const int ng = K / gs;
  const int r0 = min(n0 + li, N - 1), r1 = min(n0 + 16 + li, N - 1);
  const uint8_t* c0 = codes + (size_t)r0 * (K / 2) + 16 * g;
  const uint8_t* c1 = codes + (size_t)r1 * (K / 2) + 16 * g;
  const float* s0p = scales + (size_t)r0 * ng;
  const float* s1p = scales + (size_t)r1 * ng;
  const float* b0p = biases + (size_t)r0 * ng;
  const float* b1p = biases + (size_t)r1 * ng;
  const bf16* xr[MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) xr[mt] = X + (size_t)min(16 * mt + li, M - 1) * ldx + 32 * g;
  f32x4 acc[2][MT];
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) acc[t][mt] = f32x4{0.f, 0.f, 0.f, 0.f};
  constexpr int KB = 2;                 // 128-deep blocks per load batch
  for (int kb = k0; kb < k1; kb += 128 * KB) {
    const int nb = min(KB, (k1 - kb) / 128);
    u32x4 q0[KB], q1[KB];
    float sc0[KB], sc1[KB], bi0[KB], bi1[KB];
#pragma unroll
    for (int b = 0; b < KB; ++b)
      if (b < nb) {
        const int kk = kb + 128 * b;
        q0[b] = *reinterpret_cast<const u32x4*>(c0 + kk / 2);
        q1[b] = *reinterpret_cast<const u32x4*>(c1 + kk / 2);
        const int gi = kk / gs;
        sc0[b] = s0p[gi]; bi0[b] = b0p[gi];
        sc1[b] = s1p[gi]; bi1[b] = b1p[gi];
      }
#pragma unroll
    for (int b = 0; b < KB; ++b)
      if (b < nb) {
        const int kk = kb + 128 * b;
        // x fragments of the whole block into their own registers first (their loads overlap the
        // dequant), then the 8 dequantised A fragments, then the MFMAs; no register the MFMA
        // phase reads is rewritten before the closing pad (see the launcher's note)
        bf16x8 xb[4][MT];
#pragma unroll
        for (int s = 0; s < 4; ++s)
#pragma unroll
          for (int mt = 0; mt < MT; ++mt) xb[s][mt] = *reinterpret_cast<const bf16x8*>(xr[mt] + kk + 8 * s);
        bf16x8 a0[4], a1[4];
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          a0[s] = dequant8(q0[b][s], sc0[b], bi0[b]);
          a1[s] = dequant8(q1[b][s], sc1[b], bi1[b]);
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int s = 0; s < 4; ++s)
#pragma unroll
          for (int mt = 0; mt < MT; ++mt) {
            acc[0][mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0[s], xb[s][mt], acc[0][mt], 0, 0, 0);
            acc[1][mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1[s], xb[s][mt], acc[1][mt], 0, 0, 0);
          }
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (PAD) asm volatile("s_nop 7\n\ts_nop 7" ::: "memory");
      }
  }
  float* pp = part + (size_t)sp * M * N;
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
    const int m = 16 * mt + li;
    if (m >= M) continue;
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int n = n0 + 16 * t + 4 * g;
      if (n < N) *reinterpret_cast<f32x4*>(pp + (size_t)m * N + n) = acc[t][mt];
    }
  }
}

// out[m, n] = Σ_s part[s, m, n] (+ residual) → bf16; 8 outputs per thread
__global__ __launch_bounds__(256) void skinny_reduce_k(const float* __restrict__ part, const bf16* __restrict__ res,
                                                       bf16* __restrict__ out, int S, size_t MN) {
  const size_t i = ((size_t)blockIdx.x * 256 + threadIdx.x) * 8;
  if (i >= MN) return;
  float v[8];
  {
    const f32x4 a = *reinterpret_cast<const f32x4*>(part + i), b = *reinterpret_cast<const f32x4*>(part + i + 4);
    v[0] = a[0]; v[1] = a[1]; v[2] = a[2]; v[3] = a[3]; v[4] = b[0]; v[5] = b[1]; v[6] = b[2]; v[7] = b[3];
  }
  for (int s = 1; s < S; ++s) {
    const float* p = part + (size_t)s * MN + i;
    const f32x4 a = *reinterpret_cast<const f32x4*>(p), b = *reinterpret_cast<const f32x4*>(p + 4);
    v[0] += a[0]; v[1] += a[1]; v[2] += a[2]; v[3] += a[3]; v[4] += b[0]; v[5] += b[1]; v[6] += b[2]; v[7] += b[3];
  }
  if (res) {
    const bf16x8 r = *reinterpret_cast<const bf16x8*>(res + i);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] += (float)r[j];
  }
  bf16x8 o;
#pragma unroll
  for (int j = 0; j < 8; ++j) o[j] = (bf16)v[j];
  *reinterpret_cast<bf16x8*>(out + i) = o;
}

}  // namespace

// Split count: >= ~512 workgroups, K-slice a multiple of 32·SK_KS where possible.
int skinny_splits(int N, int K) {
  const int nblk = (N + SK_NB - 1) / SK_NB;
  int s = 1;
  while (nblk * s < 512 && K % (64 * s) == 0 && K / (2 * s) >= 256) s *= 2;
  return s;
}

void launch_gemm_skinny(const void* X, int ldx, const void* W, const void* res, void* out, float* part, int M, int N,
                        int K, int S, hipStream_t st) {
  const int kc = K / S;
  dim3 grid((N + SK_NB - 1) / SK_NB, S);
#define L(MT) gemm_skinny_k<MT><<<grid, 256, 0, st>>>((const bf16*)X, ldx, (const bf16*)W, part, M, N, K, kc)
  if (M <= 16) L(1);
  else if (M <= 32) L(2);
  else L(4);
#undef L
  const size_t MN = (size_t)M * N;
  skinny_reduce_k<<<(MN / 8 + 255) / 256, 256, 0, st>>>(part, (const bf16*)res, (bf16*)out, S, MN);
  LIPA_CHECK_LAUNCH();
}

// W4A16 split count: K-slices in whole 128-deep blocks, >= ~512 workgroups
int w4_skinny_splits(int N, int K) {
  const int nblk = (N + SK_NB - 1) / SK_NB;
  int s = 1;
  while (nblk * s < 512 && K % (256 * s) == 0 && K / (2 * s) >= 512) s *= 2;
  return s;
}

void launch_gemm_w4_skinny(const void* X, int ldx, const uint8_t* codes, const float* scales, const float* biases,
                           int gs, const void* res, void* out, float* part, int M, int N, int K, int S,
                           hipStream_t st) {
  const int kc = K / S;
  dim3 grid((N + SK_NB - 1) / SK_NB, S);
  // MT >= 2 runs one workgroup per CU (a 96 KB dynamic-LDS reservation; the kernel uses no LDS):
  // measured on MI355X (ROCm 7.2), two co-resident workgroups of the MT >= 2 code returned
  // nondeterministically wrong fragments (scripts/experiments/dbg_w4.py); one per CU is exact.
  // LIPA_W4_SKINNY_MODE (diagnosis): bit 0 drops the reservation, bit 1 drops the post-MFMA pad.
  static const int mode = [] {
    const char* e = getenv("LIPA_W4_SKINNY_MODE");
    return e ? atoi(e) : 0;
  }();
  const bool reserve = !(mode & 1), pad = !(mode & 2);
#define L(MT)                                                                                                     \
  do {                                                                                                            \
    const size_t lds = (MT) >= 2 && reserve ? 98304 : 0;                                                          \
    if (pad)                                                                                                      \
      gemm_w4_skinny_k<MT, true><<<grid, 256, lds, st>>>((const bf16*)X, ldx, codes, scales, biases, gs, part, M, \
                                                         N, K, kc);                                               \
    else                                                                                                          \
      gemm_w4_skinny_k<MT, false><<<grid, 256, lds, st>>>((const bf16*)X, ldx, codes, scales, biases, gs, part,   \
                                                          M, N, K, kc);                                           \
  } while (0)
  if (M <= 16) L(1);
  else if (M <= 32) L(2);
  else L(4);
#undef L
  const size_t MN = (size_t)M * N;
  skinny_reduce_k<<<(MN / 8 + 255) / 256, 256, 0, st>>>(part, (const bf16*)res, (bf16*)out, S, MN);
  LIPA_CHECK_LAUNCH();
}
