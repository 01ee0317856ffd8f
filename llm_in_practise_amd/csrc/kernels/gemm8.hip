// 256×256 eight-phase MFMA GEMM for gfx950: C = A·Bᵀ (+ LoRA K-slice) (+ residual)
//
//   A [M, K] bf16, row stride lda (activations, K contiguous)
//   B [N, K] bf16, row stride ldb (a frozen nn.Linear weight, K contiguous)
//
// Structure (cdna_hip_programming.md §5 "256² 8-phase template", built from its description):
//  * 512 threads = 8 waves as 2 (M) × 4 (N); each wave owns a 128×64 output block split into four
//    64×32 quadrants, one quadrant (16 × v_mfma_f32_16x16x32_bf16 over K = 64) per phase.
//  * The 256×64 A and B K-tiles are each stored as two 128-row "half-tiles" (16 KB), and a wave's
//    rows / columns are interleaved over the halves (64 of its rows in each A half, 32 of its columns
//    in each B half), so each half-tile's last ds_read happens in a known phase:
//        P1 reads A-h0 + B-h0, P2 reads B-h1, P3 reads A-h1, P4 reads nothing (B0 is still in VGPRs).
//  * Every global load is an LDS-DMA (buffer_load … lds, 1 KB per wave-instruction, swizzle on the
//    per-lane SOURCE address); each phase issues one half-tile (2 per wave) of a later K-tile into a
//    half whose reads are finished, and a counted `s_waitcnt vmcnt(6)` (never 0 in the loop) at
//    phases 4 and 8 keeps three half-tiles in flight across the raw `s_barrier`s.
//  * LDS image: 1 KB subtiles of 8 rows × 64 k, so one LDS-DMA wave-instruction fetches whole
//    128-B lines (fragment-shaped 16 × 64-B pieces double the TA work); inside a subtile the 16-B
//    chunk c of row r sits at slot 8r + (c ^ (r & 6)): each 16-lane group of a ds_read_b128 of a
//    16x16x32 fragment (rows r and r+8 share banks, chunks 4s+q) hits 16 distinct bank quads.
//  * One __shared__ array (a second one can make hipcc drain vmcnt before ds_reads).
//  * XCD-aware tile order: the 8 m-tiles of one weight panel run on one XCD (shared L2 for B).
//  * Split-K (low tile counts: M = 2048 tokens × N = 4096 is only 128 tiles for 256 CUs): each
//    split writes an fp32 slab, a reduce kernel sums the slabs (+ residual) into bf16.
#include "common.h"

using namespace lipa;

namespace {

typedef __attribute__((address_space(3))) void* lds_ptr_t;
typedef __amdgpu_buffer_rsrc_t rsrc_t;

constexpr int BM = 256, BN = 256, BK = 64;
constexpr int NT = 512;
constexpr int HALF = 16384;        // bytes of one 128 × 64 bf16 half-tile
constexpr int BUF = 4 * HALF;      // A-h0 A-h1 B-h0 B-h1
constexpr int LDS_BYTES = 2 * BUF; // 128 KB

__device__ __forceinline__ rsrc_t make_rsrc(const void* base, uint64_t bytes) {
  const uint64_t p = reinterpret_cast<uint64_t>(base);
  const uint32_t lo = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(p));
  const uint32_t hi = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(p >> 32));
  const uint32_t n = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(bytes > 0xFFFFFFFFull ? 0xFFFFFFFFull : bytes));
  void* b = reinterpret_cast<void*>((static_cast<uint64_t>(hi) << 32) | lo);
  return __builtin_amdgcn_make_buffer_rsrc(b, 0, n, 0x00020000);
}

// chunk permutation inside an 8-row × 64-k subtile (8 chunks of 16 B per row)
__device__ __forceinline__ int slot_of(int r8, int c) { return 8 * r8 + (c ^ (r8 & 6)); }

__device__ __forceinline__ void barrier() { __builtin_amdgcn_s_barrier(); }
__device__ __forceinline__ void lgkm0() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }
__device__ __forceinline__ void vm6() { asm volatile("s_waitcnt vmcnt(6)" ::: "memory"); }
__device__ __forceinline__ void vm0() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

struct Stager {
  rsrc_t rs;
  uint32_t voff[2][2];   // [half][sub] per-lane source byte offset (row clamp + chunk swizzle)
};

// one half-tile = 16 subtiles of 8 rows; this wave DMAs subtiles 2w, 2w+1 (its 16 rows)
__device__ __forceinline__ void stage_half(const Stager& s, int half, uint32_t k_byte, char* dst_half, int w) {
  char* d = dst_half + w * 2048;
  __builtin_amdgcn_raw_ptr_buffer_load_lds(s.rs, (lds_ptr_t)d, 16, s.voff[half][0], k_byte, 0, 0);
  __builtin_amdgcn_raw_ptr_buffer_load_lds(s.rs, (lds_ptr_t)(d + 1024), 16, s.voff[half][1], k_byte, 0, 0);
}

__device__ __forceinline__ bf16x8 lds_frag(const char* p) { return *reinterpret_cast<const bf16x8*>(p); }

template <bool SPLIT>
__global__ __launch_bounds__(NT, 1) void gemm8_nt_k(const bf16* __restrict__ A, int lda, const bf16* __restrict__ B,
                                                    int ldb, const bf16* __restrict__ ext_a,
                                                    const bf16* __restrict__ ext_b, int R_ext,
                                                    const bf16* __restrict__ residual, void* __restrict__ out,
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
  const int wr = w >> 2, wc = w & 3;

  const int nk_all = K / BK;
  const int per = (nk_all + splits - 1) / splits;
  const int kt0 = sp * per;
  const int nk = max(0, min(nk_all, kt0 + per) - kt0);

  // ---- staging descriptors: lane L of a 1-KB DMA writes slot L of a subtile
  Stager sa, sb;
  sa.rs = make_rsrc(A, (uint64_t)((size_t)(M - 1) * lda + K) * 2);
  sb.rs = make_rsrc(B, (uint64_t)((size_t)(N - 1) * ldb + K) * 2);
  {
    const int r8 = lane >> 3, c = (lane & 7) ^ (r8 & 6);
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int sub = 0; sub < 2; ++sub) {
        int ra = m0 + h * 128 + w * 16 + sub * 8 + r8;
        ra = ra < M ? ra : M - 1;
        int rb = n0 + h * 128 + w * 16 + sub * 8 + r8;
        rb = rb < N ? rb : N - 1;
        sa.voff[h][sub] = ((uint32_t)ra * (uint32_t)lda + (uint32_t)(kt0 * BK + c * 8)) * 2u;
        sb.voff[h][sub] = ((uint32_t)rb * (uint32_t)ldb + (uint32_t)(kt0 * BK + c * 8)) * 2u;
      }
  }
  auto kbyte = [&](int t) -> uint32_t { return (uint32_t)(t < nk ? t : nk - 1) * (BK * 2); };
  char* const buf0 = lds;
  char* const buf1 = lds + BUF;
  // half index inside a buffer: 0 A-h0, 1 A-h1, 2 B-h0, 3 B-h1
  auto stageA = [&](char* buf, int h, int t) { stage_half(sa, h, kbyte(t), buf + h * HALF, w); };
  auto stageB = [&](char* buf, int h, int t) { stage_half(sb, h, kbyte(t), buf + (2 + h) * HALF, w); };

  // ---- fragment read offsets: A rows h*128 + wr*64 + 16i, B rows h*128 + wc*32 + 16j; lane reads
  //      row (lane & 15) of the 16-row fragment = subtile +((lane>>3)&1), row lane&7, chunk 4s + lane>>4
  int lo[2];
#pragma unroll
  for (int s = 0; s < 2; ++s) lo[s] = ((lane >> 3) & 1) * 1024 + 16 * slot_of(lane & 7, 4 * s + (lane >> 4));
  const int a_base = (wr * 8) * 1024;     // 16-row block i = subtiles 2i, 2i+1
  const int b_base = (wc * 4) * 1024;

  f32x4 acc[2][4][2][2];   // [A part][m frag][B part][n frag]  (Cᵀ orientation: lane col = m)
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[a][i][b][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  bf16x8 fa[4][2], fb0[2][2], fb1[2][2];

  auto readA = [&](const char* buf, int h) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int s = 0; s < 2; ++s) fa[i][s] = lds_frag(buf + h * HALF + a_base + i * 2048 + lo[s]);
  };
  auto readB = [&](const char* buf, int h, bf16x8 (&fb)[2][2]) {
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int s = 0; s < 2; ++s) fb[j][s] = lds_frag(buf + (2 + h) * HALF + b_base + j * 2048 + lo[s]);
  };
  auto quad = [&](int ap, int bp, const bf16x8 (&fb)[2][2]) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[ap][i][bp][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[j][s], fa[i][s], acc[ap][i][bp][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };

  // ---- prologue: K-tile 0 whole + K-tile 1 minus its A-h1 (staged in the first phase)
  if (nk > 0) {
    stageA(buf0, 0, 0); stageA(buf0, 1, 0); stageB(buf0, 0, 0); stageB(buf0, 1, 0);
    stageA(buf1, 0, 1); stageB(buf1, 0, 1); stageB(buf1, 1, 1);
    vm6();
    barrier();
  }

  // Ping-pong: waves 4-7 (wr = 1) run one barrier behind waves 0-3, so on every SIMD one wave's
  // MFMA segment overlaps its partner's ds_read / LDS-DMA segment.  Every read segment retires its
  // own ds_reads (lgkmcnt(0)) BEFORE its closing barrier, so a buffer restaged one phase after its
  // last read is safe even though the other group read it one interval later.
  if (nk > 0 && wr == 1) barrier();
  const int iters = (nk + 1) / 2;
  for (int it = 0; it < iters; ++it) {
    const int te = 2 * it, to = 2 * it + 1;
    const bool odd_live = to < nk;
    // P1: B-h0 + A-h0 of the even tile; stage odd A-h1
    readB(buf0, 0, fb0);
    __builtin_amdgcn_sched_barrier(0);
    readA(buf0, 0);
    stageA(buf1, 1, to);
    lgkm0(); barrier();
    quad(0, 0, fb0);
    barrier();
    // P2: B-h1; stage even A-h0 (tile te+2)
    readB(buf0, 1, fb1);
    stageA(buf0, 0, te + 2);
    lgkm0(); barrier();
    quad(0, 1, fb1);
    barrier();
    // P3: A-h1; stage even B-h0
    readA(buf0, 1);
    stageB(buf0, 0, te + 2);
    lgkm0(); barrier();
    quad(1, 1, fb1);
    barrier();
    // P4: (registers only); stage even B-h1; retire the odd tile
    stageB(buf0, 1, te + 2);
    vm6();
    barrier();
    quad(1, 0, fb0);
    barrier();
    // P5: odd tile B-h0 + A-h0; stage even A-h1 (tile te+2)
    readB(buf1, 0, fb0);
    __builtin_amdgcn_sched_barrier(0);
    readA(buf1, 0);
    stageA(buf0, 1, te + 2);
    lgkm0(); barrier();
    if (odd_live) quad(0, 0, fb0);
    barrier();
    // P6
    readB(buf1, 1, fb1);
    stageA(buf1, 0, to + 2);
    lgkm0(); barrier();
    if (odd_live) quad(0, 1, fb1);
    barrier();
    // P7
    readA(buf1, 1);
    stageB(buf1, 0, to + 2);
    lgkm0(); barrier();
    if (odd_live) quad(1, 1, fb1);
    barrier();
    // P8: retire the even tile te+2
    stageB(buf1, 1, to + 2);
    vm6();
    barrier();
    if (odd_live) quad(1, 0, fb0);
    barrier();
  }
  if (nk > 0 && wr == 0) barrier();   // re-align the two groups' barrier counts
  vm0();          // no LDS-DMA may still be landing when the workgroup exits

  // ---- LoRA K-slice: C += ext_a · ext_bᵀ (split 0 only), operands straight from global
  if (ext_a != nullptr && sp == 0) {
    for (int e0 = 0; e0 < R_ext; e0 += 32) {
      const int ke = e0 + 8 * (lane >> 4);
#pragma unroll
      for (int ap = 0; ap < 2; ++ap) {
        bf16x8 xa[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          int m = m0 + ap * 128 + wr * 64 + i * 16 + (lane & 15);
          m = m < M ? m : M - 1;
          xa[i] = *reinterpret_cast<const bf16x8*>(ext_a + (size_t)m * R_ext + ke);
        }
#pragma unroll
        for (int bp = 0; bp < 2; ++bp)
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            int n = n0 + bp * 128 + wc * 32 + j * 16 + (lane & 15);
            n = n < N ? n : N - 1;
            const bf16x8 xb = *reinterpret_cast<const bf16x8*>(ext_b + (size_t)n * R_ext + ke);
#pragma unroll
            for (int i = 0; i < 4; ++i)
              acc[ap][i][bp][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xb, xa[i], acc[ap][i][bp][j], 0, 0, 0);
          }
      }
    }
  }

  // ---- epilogue: lane holds C[m = col][n = 4·(lane>>4) + r .. +3]
#pragma unroll
  for (int ap = 0; ap < 2; ++ap)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int m = m0 + ap * 128 + wr * 64 + i * 16 + (lane & 15);
      if (m >= M) continue;
#pragma unroll
      for (int bp = 0; bp < 2; ++bp)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const int n = n0 + bp * 128 + wc * 32 + j * 16 + 4 * (lane >> 4);
          if (n >= N) continue;
          f32x4 v = acc[ap][i][bp][j];
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

// sum the split-K slabs (+ residual) → bf16; 8 outputs per thread
__global__ __launch_bounds__(256) void splitk_reduce_k(const float* __restrict__ ws, const bf16* __restrict__ residual,
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

bool gemm8_supported(int M, int N, int K, int lda, int ldb) {
  return K % BK == 0 && K >= BK && N % 8 == 0 && lda % 8 == 0 && ldb % 8 == 0 &&
         (uint64_t)M * lda * 2 < 0xFFFFFFFFull && (uint64_t)N * ldb * 2 < 0xFFFFFFFFull;
}

// splits for a tile grid smaller than the chip: fill ≥ ~256 workgroups without K-tiles < 8 per split
int gemm8_splits(int M, int N, int K) {
  static const int forced = [] {
    const char* e = getenv("LIPA_GEMM8_SPLITS");
    return e ? atoi(e) : 0;
  }();
  if (forced > 0) return forced;
  const int tiles = ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
  const int nk = K / BK;
  int s = 1;
  while (tiles * s < 200 && nk / (2 * s) >= 16) s *= 2;
  return s;
}

void launch_gemm8(const void* A, int lda, const void* B, int ldb, const void* ext_a, const void* ext_b, int R_ext,
                  const void* residual, void* out, float* ws, int M, int N, int K, int splits, hipStream_t st) {
  const int tiles = ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
  if (splits <= 1) {
    gemm8_nt_k<false><<<tiles, NT, 0, st>>>((const bf16*)A, lda, (const bf16*)B, ldb, (const bf16*)ext_a,
                                            (const bf16*)ext_b, R_ext, (const bf16*)residual, out, M, N, K, 1);
  } else {
    gemm8_nt_k<true><<<tiles * splits, NT, 0, st>>>((const bf16*)A, lda, (const bf16*)B, ldb, (const bf16*)ext_a,
                                                    (const bf16*)ext_b, R_ext, nullptr, ws, M, N, K, splits);
    const size_t MN = (size_t)M * N;
    const int blocks = (int)std::min<size_t>((MN / 8 + 255) / 256, 2048);
    splitk_reduce_k<<<blocks, 256, 0, st>>>(ws, (const bf16*)residual, (bf16*)out, MN, splits);
  }
  LIPA_CHECK_LAUNCH();
}
