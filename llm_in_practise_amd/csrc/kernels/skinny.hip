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
