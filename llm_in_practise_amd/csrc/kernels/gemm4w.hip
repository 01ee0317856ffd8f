// One-wave-per-SIMD 256×256 MFMA GEMM for gfx950: C = A·Bᵀ (+ residual)
//
//   A [M, K] bf16, row stride lda (activations, K contiguous)
//   B [N, K] bf16, row stride ldb (a frozen weight, K contiguous)
//
// Why this shape (profiles/gemm8_pmc_vs_hipblaslt.txt): the 8-wave ping-pong kernel (gemm8.hip)
// re-reads every fragment from LDS for a 128×64 wave tile (192 KB of ds_read per K-tile per CU —
// the LDS port is saturated) and parks one wave group per phase.  Here:
//  * 256 threads = 4 waves as 2 (M) × 2 (N); each wave owns a 128×128 output block: 8×8
//    v_mfma_f32_16x16x32_bf16 accumulators = 256 fp32 per lane, held in AGPRs (the unified
//    512-entry register file at one wave per SIMD), so LDS read traffic is 128 KB per K-tile.
//  * in-wave software pipeline over the two 32-deep halves of a 64-deep K-tile: the fragments of
//    the next half are read from LDS while the 64 MFMAs of the current half run; ONE barrier per
//    K-tile, in the middle, after which the next-next K-tile's LDS-DMA is issued, so a tile's DMA
//    has two MFMA halves (≈2k cycles) to land before its `vmcnt(0)`.
//  * all global→LDS traffic is LDS-DMA (buffer_load … lds, 1 KB per wave-instruction, whole 128-B
//    lines); LDS image = 1 KB subtiles of 8 rows × 64 k with the chunk permutation of gemm8.hip
//    (slot 8r + (c ^ (r & 6)), measured conflict-free), swizzle applied on the SOURCE address.
//  * XCD-aware tile order: consecutive m-tiles of one weight panel share an XCD's L2.
//  * split-K (tile grids smaller than the chip): fp32 slabs + one reduce kernel (+ residual).
#include "common.h"

using namespace lipa;

namespace {

typedef __attribute__((address_space(3))) void* lds_ptr_t;
typedef __amdgpu_buffer_rsrc_t rsrc_t;

constexpr int BM = 256, BN = 256, BK = 64;
constexpr int NT = 256;
constexpr int IMG = 32768;          // one 256 × 64 bf16 operand image: 32 subtiles of 8 rows × 128 B
constexpr int LDS_BYTES = 5 * IMG;  // a ring of five operand images: 160 KB

__device__ __forceinline__ rsrc_t make_rsrc(const void* base, uint64_t bytes) {
  const uint64_t p = reinterpret_cast<uint64_t>(base);
  const uint32_t lo = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(p));
  const uint32_t hi = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(p >> 32));
  const uint32_t n = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(bytes > 0xFFFFFFFFull ? 0xFFFFFFFFull : bytes));
  void* b = reinterpret_cast<void*>((static_cast<uint64_t>(hi) << 32) | lo);
  return __builtin_amdgcn_make_buffer_rsrc(b, 0, n, 0x00020000);
}

__device__ __forceinline__ int slot_of(int r8, int c) { return 8 * r8 + (c ^ (r8 & 6)); }

struct Loader {
  rsrc_t rs;
  uint32_t voff[8];   // per-lane source byte offsets of this wave's 8 subtiles (row clamp + chunk swizzle)
};

struct Frags {
  bf16x8 a[8];   // m fragments (rows wr*128 + 16i)
  bf16x8 b[8];   // n fragments (rows wc*128 + 16j)
};

__device__ __forceinline__ bf16x8 lds_frag(const char* p) { return *reinterpret_cast<const bf16x8*>(p); }

template <bool SPLIT>
__global__ __launch_bounds__(NT, 1) void gemm4w_nt_k(const bf16* __restrict__ A, int lda, const bf16* __restrict__ B,
                                                     int ldb, const bf16* __restrict__ residual, void* __restrict__ out,
                                                     int M, int N, int K, int splits) {
  __shared__ __attribute__((aligned(16))) char lds[LDS_BYTES];

  const int tiles_m = (M + BM - 1) / BM, tiles_n = (N + BN - 1) / BN;
  const int nwg = tiles_m * tiles_n * splits;
  const int id = xcd_remap(blockIdx.x, nwg);
  const int sp = id % splits;
  const int tid = id / splits;
  const int tm = tid % tiles_m, tn = tid / tiles_m;
  const int m0 = tm * BM, n0 = tn * BN;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const int wr = w >> 1, wc = w & 1;

  const int nk_all = K / BK;
  const int per = (nk_all + splits - 1) / splits;
  const int kt0 = sp * per;
  const int nk = max(0, min(nk_all, kt0 + per) - kt0);

  Loader la, lb;
  la.rs = make_rsrc(A, (uint64_t)((size_t)(M - 1) * lda + K) * 2);
  lb.rs = make_rsrc(B, (uint64_t)((size_t)(N - 1) * ldb + K) * 2);
  {
    const int r8 = lane >> 3, c = (lane & 7) ^ (r8 & 6);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      int ra = m0 + w * 64 + i * 8 + r8;
      ra = ra < M ? ra : M - 1;
      int rb = n0 + w * 64 + i * 8 + r8;
      rb = rb < N ? rb : N - 1;
      la.voff[i] = ((uint32_t)ra * (uint32_t)lda + (uint32_t)(kt0 * BK + c * 8)) * 2u;
      lb.voff[i] = ((uint32_t)rb * (uint32_t)ldb + (uint32_t)(kt0 * BK + c * 8)) * 2u;
    }
  }

  // fragment read offsets: 16-row fragment = subtiles 2f, 2f+1; lane reads row lane & 15 of it
  // (subtile (lane >> 3) & 1, row lane & 7) at chunk 4s + (lane >> 4) for K-half s
  int lo[2];
#pragma unroll
  for (int s = 0; s < 2; ++s) lo[s] = ((lane >> 3) & 1) * 1024 + 16 * slot_of(lane & 7, 4 * s + (lane >> 4));
  const int a_off = wr * 8 * 2048;
  const int b_off = wc * 8 * 2048;

  f32x4 acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // Operand images live in a ring of 5 slots of 32 KB: image i (A_t = 2t, B_t = 2t + 1) in slot
  // i mod 5.  A_{t+2} reuses B_{t-1}'s slot (free since the barrier of iteration t-1) and is
  // DMA'd during the first half of iteration t; B_{t+2} reuses A_t's slot (free after iteration
  // t's barrier) and is DMA'd during the second half.  So every MFMA group of either half issues
  // ONE LDS-DMA per wave (TA and LDS-write load spread evenly), and each image has ≥ one half
  // (≈1k cycles) to land before the barrier that publishes it.
  auto img = [&](int i) -> char* { return lds + (i % 5) * IMG; };
  Frags f0, f1;
  auto read_q = [&](Frags& f, const char* ia, const char* ib, int s, int q) {
    f.a[q] = lds_frag(ia + a_off + q * 2048 + lo[s]);
    f.b[q] = lds_frag(ib + b_off + q * 2048 + lo[s]);
  };
  auto mma_row = [&](const Frags& f, int i) {
#pragma unroll
    for (int j = 0; j < 8; ++j)
      acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f.b[j], f.a[i], acc[i][j], 0, 0, 0);
  };
  // one LDS-DMA: subtile 8w + q of K-tile t's A (or B) image
  auto dma = [&](const Loader& L, char* im, int t, int q) {
    __builtin_amdgcn_raw_ptr_buffer_load_lds(L.rs, (lds_ptr_t)(im + w * 8192 + q * 1024), 16, L.voff[q],
                                             (uint32_t)t * (BK * 2), 0, 0);
  };

  if (nk > 0) {
    const int t1 = nk > 1 ? 1 : 0;
#pragma unroll
    for (int q = 0; q < 8; ++q) dma(la, img(0), 0, q);
#pragma unroll
    for (int q = 0; q < 8; ++q) dma(lb, img(1), 0, q);
#pragma unroll
    for (int q = 0; q < 8; ++q) dma(la, img(2), t1, q);
#pragma unroll
    for (int q = 0; q < 8; ++q) dma(lb, img(3), t1, q);
    asm volatile("s_waitcnt vmcnt(16)" ::: "memory");   // tile 0 landed (tile 1's 16 DMAs may fly)
    __builtin_amdgcn_s_barrier();
#pragma unroll
    for (int q = 0; q < 8; ++q) read_q(f0, img(0), img(1), 0, q);
  }
  // Per K-tile t (F0 = its first K-half in registers):
  //   [64 MFMAs on F0 ∥ read F1 (second half) ∥ DMA A_{t+2}] → vmcnt(8) lgkmcnt(0) barrier →
  //   [64 MFMAs on F1 ∥ read F0 of tile t+1 ∥ DMA B_{t+2}]
  // Branch-free: past the last K-tile the DMAs re-stage tile nk-1 into slots nobody reads again and
  // the last F0 reads are discarded.  Waits are compiler-visible s_waitcnt builtins
  // (0xC07F = lgkmcnt(0), 0x0F78 = vmcnt(8)) so the waitcnt pass adds none of its own.
  for (int t = 0; t < nk; ++t) {
    const int t2 = t + 2 < nk ? t + 2 : nk - 1;
    char* const ia = img(2 * t);
    char* const ib = img(2 * t + 1);
    char* const na = img(2 * t + 2);
    char* const nb = img(2 * t + 3);
    char* const da = img(2 * t + 4);
    char* const db = img(2 * t + 5);
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      mma_row(f0, q);
      __builtin_amdgcn_sched_barrier(0);
      read_q(f1, ia, ib, 1, q);
      dma(la, da, t2, q);
      __builtin_amdgcn_sched_barrier(0);
    }
    __builtin_amdgcn_s_waitcnt(0x0F78);   // all but this half's 8 DMAs landed: tile t+1 is complete
    __builtin_amdgcn_s_waitcnt(0xC07F);   // this wave's reads of tile t are done
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      read_q(f0, na, nb, 0, q);
      dma(lb, db, t2, q);
      __builtin_amdgcn_sched_barrier(0);
      mma_row(f1, q);
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");

  // ---- epilogue: lane holds C[m = col][n = 4·(lane>>4) + r … +3] of each 16×16 block
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int m = m0 + wr * 128 + i * 16 + (lane & 15);
    if (m >= M) continue;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int n = n0 + wc * 128 + j * 16 + 4 * (lane >> 4);
      if (n >= N) continue;
      f32x4 v = acc[i][j];
      if constexpr (SPLIT) {
        float* ws = reinterpret_cast<float*>(out) + ((size_t)sp * M + m) * N + n;
        *reinterpret_cast<f32x4*>(ws) = v;
      } else {
        if (residual) {
          const bf16x4 rr = *reinterpret_cast<const bf16x4*>(residual + (size_t)m * N + n);
          v[0] += (float)rr[0]; v[1] += (float)rr[1]; v[2] += (float)rr[2]; v[3] += (float)rr[3];
        }
        bf16x4 o;
        o[0] = (bf16)v[0]; o[1] = (bf16)v[1]; o[2] = (bf16)v[2]; o[3] = (bf16)v[3];
        *reinterpret_cast<bf16x4*>(reinterpret_cast<bf16*>(out) + (size_t)m * N + n) = o;
      }
    }
  }
}

__global__ __launch_bounds__(256) void splitk_sum_k(const float* __restrict__ ws, const bf16* __restrict__ residual,
                                                    bf16* __restrict__ out, size_t MN, int splits) {
  for (size_t i = ((size_t)blockIdx.x * 256 + threadIdx.x) * 8; i < MN; i += (size_t)gridDim.x * 256 * 8) {
    float v[8];
    load8(ws + i, v);
    for (int s = 1; s < splits; ++s) {
      float u[8];
      load8(ws + (size_t)s * MN + i, u);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] += u[j];
    }
    if (residual) {
      float r[8];
      load8(residual + i, r);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] += r[j];
    }
    store8(out + i, v);
  }
}

}  // namespace

bool gemm4w_supported(int M, int N, int K, int lda, int ldb) {
  return M > 0 && K % BK == 0 && K >= BK && N % 8 == 0 && lda % 8 == 0 && ldb % 8 == 0 &&
         (uint64_t)M * lda * 2 < 0xFFFFFFFFull && (uint64_t)N * ldb * 2 < 0xFFFFFFFFull;
}

// K-splits for a tile grid smaller than the chip (M = 2048 × N = 4096 is 128 tiles for 256 CUs)
int gemm4w_splits(int M, int N, int K) {
  static const int forced = [] {
    const char* e = getenv("LIPA_GEMM4W_SPLITS");
    return e ? atoi(e) : 0;
  }();
  if (forced > 0) return forced;
  const int tiles = ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
  const int nk = K / BK;
  int s = 1;
  while (tiles * s < 200 && nk / (2 * s) >= 16) s *= 2;
  return s;
}

void launch_gemm4w(const void* A, int lda, const void* B, int ldb, const void* residual, void* out, float* ws, int M,
                   int N, int K, int splits, hipStream_t st) {
  const int tiles = ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
  if (splits <= 1) {
    gemm4w_nt_k<false><<<tiles, NT, 0, st>>>((const bf16*)A, lda, (const bf16*)B, ldb, (const bf16*)residual, out, M,
                                             N, K, 1);
  } else {
    gemm4w_nt_k<true><<<tiles * splits, NT, 0, st>>>((const bf16*)A, lda, (const bf16*)B, ldb, nullptr, ws, M, N, K,
                                                     splits);
    const size_t MN = (size_t)M * N;
    const int blocks = (int)std::min<size_t>((MN / 8 + 255) / 256, 2048);
    splitk_sum_k<<<blocks, 256, 0, st>>>(ws, (const bf16*)residual, (bf16*)out, MN, splits);
  }
  LIPA_CHECK_LAUNCH();
}
