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
//    The MFMAs are one-instruction asm statements with the accumulator a tied "+a" operand: with
//    the builtin, hipcc split the accumulator phis between the two K-halves and shuffled ~48
//    v_accvgpr_mov/read/write per K-tile through the MFMA results (each a dependent stall).
//    Hazards the asm hides from hipcc: none in the loop (a fragment register is rewritten ≥ 8
//    MFMAs after its last reader); the epilogue's AGPR reads sit behind 16 wait states.
//  * in-wave software pipeline over the two 32-deep halves of a 64-deep K-tile: the fragments of
//    the next half are read from LDS while the 64 MFMAs of the current half run; ONE barrier per
//    K-tile, in the middle, after which the next-next K-tile's LDS-DMA is issued, so a tile's DMA
//    has two MFMA halves (≈2k cycles) to land before its `vmcnt(0)`.
//  * all global→LDS traffic is LDS-DMA (buffer_load … lds, 1 KB per wave-instruction, whole 128-B
//    lines); LDS image = 1 KB subtiles of 8 rows × 64 k with the chunk permutation of gemm8.hip
//    (slot 8r + (c ^ (r & 6)), measured conflict-free), swizzle applied on the SOURCE address.
//  * XCD-aware tile order: consecutive m-tiles of one weight panel share an XCD's L2.
//  * split-K (tile grids smaller than the chip): fp32 slabs + one reduce kernel (+ residual).
#include <type_traits>

#include "common.h"

using namespace lipa;

namespace {

typedef __attribute__((address_space(3))) void* lds_ptr_t;
typedef __amdgpu_buffer_rsrc_t rsrc_t;

constexpr int BM = 256, BN = 256, BK = 64;
constexpr int NT = 256;
constexpr int IMG = 32768;
constexpr int LDS_BYTES = 5 * IMG;

__device__ __forceinline__ rsrc_t make_rsrc(const void* base, uint64_t bytes) {
  const uint64_t p = reinterpret_cast<uint64_t>(base);
  const uint32_t lo = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(p));
  const uint32_t hi = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(p >> 32));
  const uint32_t n = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(bytes > 0xFFFFFFFFull ? 0xFFFFFFFFull : bytes));
  void* b = reinterpret_cast<void*>((static_cast<uint64_t>(hi) << 32) | lo);
  return __builtin_amdgcn_make_buffer_rsrc(b, 0, n, 0x00020000);
}

__device__ __forceinline__ int slot_of(int r8, int c) { return 8 * r8 + (c ^ (r8 & 6)); }

struct Frags {
  bf16x8 a[8];
  bf16x8 b[8];
};

// compile-time unrolled k-loop: f(std::integral_constant<int, k>) for k in [K, N)
template <int K, int N>
struct Unroll {
  template <typename F>
  __device__ __forceinline__ static void run(F&& f) {
    f(std::integral_constant<int, K>{});
    Unroll<K + 1, N>::run(f);
  }
};
template <int N>
struct Unroll<N, N> {
  template <typename F>
  __device__ __forceinline__ static void run(F&&) {}
};

// MFMA order of a 64-MFMA K-half: shells of max(i, j) — shell s is (s, 0..s) then (0..s-1, s), so
// it needs only fragments a[0..s], b[0..s]
struct ShellOrder {
  int i[64], j[64];
};
constexpr ShellOrder make_shell_order() {
  ShellOrder o{};
  int k = 0;
  for (int s = 0; s < 8; ++s) {
    for (int j = 0; j <= s; ++j) { o.i[k] = s; o.j[k] = j; ++k; }
    for (int i = 0; i < s; ++i) { o.i[k] = i; o.j[k] = s; ++k; }
  }
  return o;
}
constexpr ShellOrder kShell = make_shell_order();

__device__ __forceinline__ bf16x8 lds_frag(const char* p) { return *reinterpret_cast<const bf16x8*>(p); }

// accumulator pinned to AGPRs, D == C (tied): no allocator copies between the two K-halves
__device__ __forceinline__ void mfma_acc(f32x4& acc, const bf16x8& a, const bf16x8& b) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(a), "v"(b));
}
__device__ __forceinline__ void mfma_zero(f32x4& acc, const bf16x8& a, const bf16x8& b) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, 0" : "=a"(acc) : "v"(a), "v"(b));
}

// VAR: diagnostic ablations (scripts/experiments/gemm4w_var.py; wrong results by design):
//   1 = no LDS-DMA in the K-loop, 2 = no fragment reads in the K-loop, 4 = no mid-tile wait + barrier
template <bool SPLIT, int VAR = 0>
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

  const rsrc_t rsa = make_rsrc(A, (uint64_t)((size_t)(M - 1) * lda + K) * 2);
  const rsrc_t rsb = make_rsrc(B, (uint64_t)((size_t)(N - 1) * ldb + K) * 2);
  uint32_t va[8], vb[8];
  {
    const int r8 = lane >> 3, c = (lane & 7) ^ (r8 & 6);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      int ra = m0 + w * 64 + i * 8 + r8;
      ra = ra < M ? ra : M - 1;
      int rb = n0 + w * 64 + i * 8 + r8;
      rb = rb < N ? rb : N - 1;
      va[i] = ((uint32_t)ra * (uint32_t)lda + (uint32_t)(kt0 * BK + c * 8)) * 2u;
      vb[i] = ((uint32_t)rb * (uint32_t)ldb + (uint32_t)(kt0 * BK + c * 8)) * 2u;
    }
  }

  int lo[2];
#pragma unroll
  for (int s = 0; s < 2; ++s) lo[s] = ((lane >> 3) & 1) * 1024 + 16 * slot_of(lane & 7, 4 * s + (lane >> 4));
  const int a_off = wr * 8 * 2048;
  const int b_off = wc * 8 * 2048;

  f32x4 acc[8][8];
  Frags f0, f1;

  // producer order inside a half: group g (0..7) reads a[2g], a[2g+1] (g < 4) or b[2g-8], b[2g-7];
  // consumer order: column j of 8 MFMAs needs b[j] and every a[i] — the a's land first
  auto read_g = [&](Frags& f, const char* ia, const char* ib, int s, int g) {
    if (g < 4) {
      f.a[2 * g] = lds_frag(ia + a_off + (2 * g) * 2048 + lo[s]);
      f.a[2 * g + 1] = lds_frag(ia + a_off + (2 * g + 1) * 2048 + lo[s]);
    } else {
      const int j = 2 * (g - 4);
      f.b[j] = lds_frag(ib + b_off + j * 2048 + lo[s]);
      f.b[j + 1] = lds_frag(ib + b_off + (j + 1) * 2048 + lo[s]);
    }
  };
  auto mma_col = [&](const Frags& f, int j) {
#pragma unroll
    for (int i = 0; i < 8; ++i) mfma_acc(acc[i][j], f.b[j], f.a[i]);
  };
  auto mma_col0 = [&](const Frags& f, int j) {
#pragma unroll
    for (int i = 0; i < 8; ++i) mfma_zero(acc[i][j], f.b[j], f.a[i]);
  };
  auto dma = [&](const rsrc_t& rs, const uint32_t* voff, char* im, int t, int q) {
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_ptr_t)(im + w * 8192 + q * 1024), 16, voff[q],
                                             (uint32_t)t * (BK * 2), 0, 0);
  };

  if (nk <= 0) {
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  } else if constexpr (VAR == 8) {
    // Double-buffered form: two 64 KB stages (A image + B image each).  Per K-tile t, one
    // 128-MFMA stream: MFMAs 0-63 on the first K-half (fA), 64-127 on the second (fB);
    //   MFMA  0-15: + one fragment read each of tile t's second half (into fB)
    //   after 25  : lgkmcnt(0) + barrier 1 — nobody reads stage t&1 any more
    //   MFMA 26-101, every 5th: one LDS-DMA of tile t+2 into stage t&1 (8 A, then 8 B)
    //   after 111 : vmcnt(16) (tile t+1 landed; t+2's 16 in flight) + barrier 2
    //   MFMA 112-127: + one fragment read each of tile t+1's first half (into fA)
    // The first half's MFMAs walk (i, j) in shells of max(i, j): shell s needs reads 2s, 2s+1 only.
    const int t1 = nk > 1 ? 1 : 0;
#pragma unroll
    for (int q = 0; q < 8; ++q) dma(rsa, va, lds + 0 * IMG, 0, q);
#pragma unroll
    for (int q = 0; q < 8; ++q) dma(rsb, vb, lds + 1 * IMG, 0, q);
#pragma unroll
    for (int q = 0; q < 8; ++q) dma(rsa, va, lds + 2 * IMG, t1, q);
#pragma unroll
    for (int q = 0; q < 8; ++q) dma(rsb, vb, lds + 3 * IMG, t1, q);
    asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    auto read_r = [&](Frags& f, const char* ia, const char* ib, int s, int r) {
      if ((r & 1) == 0) f.a[r >> 1] = lds_frag(ia + a_off + (r >> 1) * 2048 + lo[s]);
      else f.b[r >> 1] = lds_frag(ib + b_off + (r >> 1) * 2048 + lo[s]);
    };
#pragma unroll
    for (int r = 0; r < 16; ++r) read_r(f0, lds, lds + IMG, 0, r);
    int cur = 0;
    auto body = [&](auto first, int t) {
      const int t2 = t + 2 < nk ? t + 2 : nk - 1;
      char* const ca = lds + cur;
      char* const cb = ca + IMG;
      char* const na = lds + (cur ^ (2 * IMG));
      char* const nb = na + IMG;
      Unroll<0, 128>::run([&](auto kc) {
        constexpr int k = decltype(kc)::value;
        constexpr int i = kShell.i[k & 63], j = kShell.j[k & 63];
        if constexpr (k < 64) {
          if constexpr (decltype(first)::value) mfma_zero(acc[i][j], f0.b[j], f0.a[i]);
          else mfma_acc(acc[i][j], f0.b[j], f0.a[i]);
        } else {
          mfma_acc(acc[i][j], f1.b[j], f1.a[i]);
        }
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (k < 16) read_r(f1, ca, cb, 1, k);
        if constexpr (k == 25) {
          __builtin_amdgcn_s_waitcnt(0xC07F);   // lgkmcnt(0)
          __builtin_amdgcn_s_barrier();
        }
        if constexpr (k >= 26 && k <= 101 && (k - 26) % 5 == 0) {
          constexpr int d = (k - 26) / 5;
          if constexpr (d < 8) dma(rsa, va, ca, t2, d);
          else dma(rsb, vb, cb, t2, d - 8);
        }
        if constexpr (k == 111) {
          __builtin_amdgcn_s_waitcnt(0x4F70);   // vmcnt(16)
          __builtin_amdgcn_s_barrier();
        }
        if constexpr (k >= 112) read_r(f0, na, nb, 0, k - 112);
        __builtin_amdgcn_sched_barrier(0);
      });
      cur ^= 2 * IMG;
    };
    body(std::integral_constant<bool, true>{}, 0);
    for (int t = 1; t < nk; ++t) body(std::integral_constant<bool, false>{}, t);
    asm volatile("s_waitcnt vmcnt(0)\n\ts_nop 7\n\ts_nop 7" ::: "memory");
  } else {
    const int t1 = nk > 1 ? 1 : 0;
#pragma unroll
    for (int q = 0; q < 8; ++q) dma(rsa, va, lds + 0 * IMG, 0, q);
#pragma unroll
    for (int q = 0; q < 8; ++q) dma(rsb, vb, lds + 1 * IMG, 0, q);
#pragma unroll
    for (int q = 0; q < 8; ++q) dma(rsa, va, lds + 2 * IMG, t1, q);
#pragma unroll
    for (int q = 0; q < 8; ++q) dma(rsb, vb, lds + 3 * IMG, t1, q);
    asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
    __builtin_amdgcn_s_barrier();
#pragma unroll
    for (int g = 0; g < 8; ++g) read_g(f0, lds, lds + IMG, 0, g);
    if constexpr ((VAR & 2) != 0) f1 = f0;

    // ring slots of the images A_t = 2t, B_t = 2t + 1 (mod 5), advanced incrementally
    int s_ia = 0;   // slot of A_t
    for (int t = 0; t < nk; ++t) {
      const int t2 = t + 2 < nk ? t + 2 : nk - 1;
      const int s_ib = s_ia + 1 >= 5 ? s_ia - 4 : s_ia + 1;
      const int s_na = s_ib + 1 >= 5 ? s_ib - 4 : s_ib + 1;
      const int s_nb = s_na + 1 >= 5 ? s_na - 4 : s_na + 1;
      const int s_da = s_nb + 1 >= 5 ? s_nb - 4 : s_nb + 1;   // == slot of B_{t-1}
      const int s_db = s_ia;                                   // A_t's slot, free after the mid barrier
      char* const ia = lds + s_ia * IMG;
      char* const ib = lds + s_ib * IMG;
      char* const na = lds + s_na * IMG;
      char* const nb = lds + s_nb * IMG;
      char* const da = lds + s_da * IMG;
      char* const db = lds + s_db * IMG;
      if (t == 0) {
#pragma unroll
        for (int g = 0; g < 8; ++g) {
          mma_col0(f0, g);
          __builtin_amdgcn_sched_barrier(0);
          if constexpr ((VAR & 2) == 0) read_g(f1, ia, ib, 1, g);
          if constexpr ((VAR & 1) == 0) dma(rsa, va, da, t2, g);
          __builtin_amdgcn_sched_barrier(0);
        }
      } else {
#pragma unroll
        for (int g = 0; g < 8; ++g) {
          mma_col(f0, g);
          __builtin_amdgcn_sched_barrier(0);
          if constexpr ((VAR & 2) == 0) read_g(f1, ia, ib, 1, g);
          if constexpr ((VAR & 1) == 0) dma(rsa, va, da, t2, g);
          __builtin_amdgcn_sched_barrier(0);
        }
      }
      if constexpr ((VAR & 4) == 0) {
        __builtin_amdgcn_s_waitcnt(0x0F78);   // vmcnt(8): tile t+1 complete
        __builtin_amdgcn_s_waitcnt(0xC07F);   // lgkmcnt(0)
        __builtin_amdgcn_s_barrier();
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int g = 0; g < 8; ++g) {
        if constexpr ((VAR & 2) == 0) read_g(f0, na, nb, 0, g);
        if constexpr ((VAR & 1) == 0) dma(rsb, vb, db, t2, g);
        __builtin_amdgcn_sched_barrier(0);
        mma_col(f1, g);
        __builtin_amdgcn_sched_barrier(0);
      }
      s_ia = s_na;
    }
    asm volatile("s_waitcnt vmcnt(0)\n\ts_nop 7\n\ts_nop 7" ::: "memory");
  }

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
  static const int var = [] {
    const char* e = getenv("LIPA_GEMM4W_VAR");
    return e ? atoi(e) : 0;
  }();
  if (splits <= 1) {
#define G4W_VAR(V)                                                                                                 \
  case V:                                                                                                          \
    gemm4w_nt_k<false, V><<<tiles, NT, 0, st>>>((const bf16*)A, lda, (const bf16*)B, ldb, (const bf16*)residual, out, \
                                                M, N, K, 1);                                                        \
    break;
    switch (var) {
      G4W_VAR(1) G4W_VAR(2) G4W_VAR(3) G4W_VAR(4) G4W_VAR(5) G4W_VAR(7) G4W_VAR(8)
      default:
        gemm4w_nt_k<false><<<tiles, NT, 0, st>>>((const bf16*)A, lda, (const bf16*)B, ldb, (const bf16*)residual, out,
                                                 M, N, K, 1);
    }
#undef G4W_VAR
  } else {
    gemm4w_nt_k<true><<<tiles * splits, NT, 0, st>>>((const bf16*)A, lda, (const bf16*)B, ldb, nullptr, ws, M, N, K,
                                                     splits);
    const size_t MN = (size_t)M * N;
    const int blocks = (int)std::min<size_t>((MN / 8 + 255) / 256, 2048);
    splitk_sum_k<<<blocks, 256, 0, st>>>(ws, (const bf16*)residual, (bf16*)out, MN, splits);
  }
  LIPA_CHECK_LAUNCH();
}
