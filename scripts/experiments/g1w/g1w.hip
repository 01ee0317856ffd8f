// Experiment: 256x{256,128}x64 bf16 NT GEMM, 4 waves = ONE wave per SIMD, accumulators in AGPRs,
// in-wave software pipeline (ds_read of the next k-substep under the current substep's MFMAs),
// LDS-DMA staging into two buffers, one barrier per K-tile.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void* lds_ptr_t;
typedef __amdgpu_buffer_rsrc_t rsrc_t;

namespace {

constexpr int BM = 256, BK = 64, NT = 256;

__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int q = nwg / 8, r = nwg % 8, x = bid % 8;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + bid / 8;
}

__device__ __forceinline__ rsrc_t make_rsrc(const void* base, uint64_t bytes) {
  const uint64_t p = reinterpret_cast<uint64_t>(base);
  const uint32_t lo = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(p));
  const uint32_t hi = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(p >> 32));
  const uint32_t n = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(bytes > 0xFFFFFFFFull ? 0xFFFFFFFFull : bytes));
  void* b = reinterpret_cast<void*>((static_cast<uint64_t>(hi) << 32) | lo);
  return __builtin_amdgcn_make_buffer_rsrc(b, 0, n, 0x00020000);
}

__device__ __forceinline__ int slot_of(int r8, int c) { return 8 * r8 + (c ^ (r8 & 6)); }
__device__ __forceinline__ void barrier() { __builtin_amdgcn_s_barrier(); }
__device__ __forceinline__ void lgkm0() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }
__device__ __forceinline__ void vm0() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
// MFMA with the accumulator tied to an AGPR quad (the builtin lets the allocator untie dst and srcC,
// which at 256 accumulators turns into hundreds of v_accvgpr moves per K-tile)
// Everything in the K-loop is volatile asm so it issues in program order (the machine scheduler
// otherwise sinks each fragment read to just before its MFMA); the waits are explicit.
__device__ __forceinline__ void mfma16(f32x4& acc, const bf16x8& a, const bf16x8& b) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(a), "v"(b));
}
__device__ __forceinline__ void ds_read128(bf16x8& d, uint32_t addr, int off) {
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(d) : "v"(addr), "i"(off));
}

// ABL (ablation bits): 1 = no DMA in the loop, 2 = no vmcnt/barrier in the loop, 4 = no ds_read in the loop,
//                     8 = persistent (grid = CUs, tiles strided; next tile's prologue DMAs issued before the epilogue)
template <int BN, bool SPLIT, int ABL = 0>
__global__ __launch_bounds__(NT, 1) __attribute__((amdgpu_waves_per_eu(1, 1))) void g1w_nt_k(const bf16* __restrict__ A, int lda, const bf16* __restrict__ B,
                                                  int ldb, const bf16* __restrict__ residual, void* __restrict__ out,
                                                  int ldc, int M, int N, int K, int splits) {
  constexpr int ABYTES = BM * BK * 2;          // 32 KB
  constexpr int BBYTES = BN * BK * 2;          // 32 / 16 KB
  constexpr int BUF = ABYTES + BBYTES;
  constexpr int NJ = BN / 32;                  // n fragments per wave (wave covers BN/2 columns)
  constexpr int ASUB = BM / 8 / 4;             // A subtiles DMA'd per wave per K-tile (8)
  constexpr int BSUB = BN / 8 / 4;             // B subtiles per wave (8 / 4)
  __shared__ __attribute__((aligned(16))) char lds[2 * BUF];

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

  const rsrc_t ra = make_rsrc(A, (uint64_t)M * lda * 2);
  const rsrc_t rb = make_rsrc(B, (uint64_t)N * ldb * 2);
  // lane L of a 1-KB DMA writes slot L of an 8-row x 64-k subtile: row L>>3, chunk (L&7)^(row&6)
  const int r8 = lane >> 3, ch = (lane & 7) ^ (r8 & 6);
  const uint32_t va = ((uint32_t)(m0 + w * ASUB * 8 + r8) * lda + ch * 8) * 2u;
  const uint32_t vb = ((uint32_t)(n0 + w * BSUB * 8 + r8) * ldb + ch * 8) * 2u;



  // LDS byte addresses of this lane's fragment rows, per buffer and k-substep (wave row/col folded in)
  const uint32_t lds0 = (uint32_t)(uintptr_t)(lds_ptr_t)lds;
  uint32_t pa[2][2], pb[2][2];
#pragma unroll
  for (int b = 0; b < 2; ++b)
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const uint32_t lo = ((lane >> 3) & 1) * 1024 + 16 * slot_of(lane & 7, 4 * s + (lane >> 4));
      pa[b][s] = lds0 + b * BUF + wr * 16 * 1024 + lo;
      pb[b][s] = lds0 + b * BUF + ABYTES + wc * (BN / 16) * 1024 + lo;
    }

  f32x4 acc[8][NJ];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  bf16x8 fa0[8], fb0[NJ], fa1[8], fb1[NJ];
  // fragment r of a k-substep (0..7: A m-frag r, 8..: B n-frag r-8)
  auto rd = [&](int b, int s, int r, bf16x8 (&fa)[8], bf16x8 (&fb)[NJ]) {
    if (r < 8) ds_read128(fa[r], pa[b][s], r * 2048);
    else ds_read128(fb[r - 8], pb[b][s], (r - 8) * 2048);
  };
  char* const buf0 = lds;
  char* const buf1 = lds + BUF;
  auto dma = [&](int t, char* buf, int q) {     // DMA q (0..ASUB+BSUB-1) of K-tile t into buf
    const uint32_t kb = (uint32_t)(kt0 + t) * (BK * 2);
    if (q < ASUB)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(ra, (lds_ptr_t)(buf + (w * ASUB + q) * 1024), 16, va,
                                               kb + (uint32_t)(q * 8 * lda * 2), 0, 0);
    else
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rb, (lds_ptr_t)(buf + ABYTES + (w * BSUB + q - ASUB) * 1024), 16, vb,
                                               kb + (uint32_t)((q - ASUB) * 8 * ldb * 2), 0, 0);
  };
  constexpr int NR = 8 + NJ;             // fragment reads per k-substep
  constexpr int NQ = ASUB + BSUB;        // DMAs per K-tile per wave
  constexpr int NM = 8 * NJ;             // MFMAs per k-substep

  // nk is even (host check); tiles past the end are clamped re-loads into a buffer nobody reads again
  auto clampt = [&](int t) { return t < nk ? t : nk - 1; };
  auto step = [&](int t, int bc, char* cur) {
    // H1: MFMA k-substep 0 (F0) under the reads of k-substep 1 (F1) from `cur`
#pragma unroll
    for (int q = 0; q < NM; ++q) {
      mfma16(acc[q / NJ][q % NJ], fb0[q % NJ], fa0[q / NJ]);
      if (!(ABL & 4) && q % (NM / NR) == 0 && q / (NM / NR) < NR) rd(bc, 1, q / (NM / NR), fa1, fb1);
    }
    lgkm0();
    if (!(ABL & 2)) {
      vm0();          // K-tile t+1 (DMA'd during the previous H2) has landed
      barrier();      // every wave is done reading `cur`; t+1 is visible to all
    }
    // H2: MFMA k-substep 1 (F1); restage `cur` with K-tile t+2; read k-substep 0 of t+1 (F0)
    const int t2 = clampt(t + 2);
#pragma unroll
    for (int q = 0; q < NM; ++q) {
      mfma16(acc[q / NJ][q % NJ], fb1[q % NJ], fa1[q / NJ]);
      if (!(ABL & 1) && q % (NM / NQ) == 0 && q / (NM / NQ) < NQ) dma(t2, cur, q / (NM / NQ));
      if (!(ABL & 4) && q % (NM / NR) == (NM / NR) / 2 && q / (NM / NR) < NR) rd(bc ^ 1, 0, q / (NM / NR), fa0, fb0);
    }
    lgkm0();
  };
  if (nk > 0) {
    for (int q = 0; q < NQ; ++q) dma(0, buf0, q);
    for (int q = 0; q < NQ; ++q) dma(clampt(1), buf1, q);
    asm volatile("s_waitcnt vmcnt(%0)" :: "n"(NQ) : "memory");
    barrier();
    for (int r = 0; r < NR; ++r) rd(0, 0, r, fa0, fb0);
    lgkm0();
    for (int t = 0; t < nk; t += 2) {
      step(t, 0, buf0);
      step(t + 1, 1, buf1);
    }
  }
  vm0();
  asm volatile("s_nop 15\n s_nop 15" ::: "memory");   // MFMA results -> accvgpr reads (asm MFMAs are invisible to the hazard pass)

  // epilogue: lane holds C[m = lane&15 row of m-frag i][n = 4*(lane>>4) .. +3 of n-frag j]
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int m = m0 + wr * 128 + i * 16 + (lane & 15);
    if (m >= M) continue;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int n = n0 + wc * (BN / 2) + j * 16 + 4 * (lane >> 4);
      if (n >= N) continue;
      f32x4 v = acc[i][j];
      if constexpr (SPLIT) {
        float* ws = reinterpret_cast<float*>(out) + ((size_t)sp * M + m) * ldc + n;
        *reinterpret_cast<f32x4*>(ws) = v;
      } else {
        if (residual) {
          const bf16x4 rr = *reinterpret_cast<const bf16x4*>(residual + (size_t)m * ldc + n);
          v[0] += (float)rr[0]; v[1] += (float)rr[1]; v[2] += (float)rr[2]; v[3] += (float)rr[3];
        }
        bf16x4 o;
        o[0] = (bf16)v[0]; o[1] = (bf16)v[1]; o[2] = (bf16)v[2]; o[3] = (bf16)v[3];
        *reinterpret_cast<bf16x4*>(reinterpret_cast<bf16*>(out) + (size_t)m * ldc + n) = o;
      }
    }
  }
}


// ---- v2: BK = 32, NBUF = 4 LDS stages (32 KB each), DMA of K-tile t+4 issued in step t (3 tiles in flight)
//      64-B LDS rows, 1 KB = 16 rows per DMA; chunk c of row r at physical chunk c ^ ((-(r >> 2)) & 3)
//      (conflict-free for the 16x16x32 fragment read: lane l reads row l & 15, chunk l >> 4)
template <int BN, bool SPLIT>
__global__ __launch_bounds__(NT, 1) __attribute__((amdgpu_waves_per_eu(1, 1))) void g1w32_nt_k(
    const bf16* __restrict__ A, int lda, const bf16* __restrict__ B, int ldb, const bf16* __restrict__ residual,
    void* __restrict__ out, int ldc, int M, int N, int K, int splits) {
  constexpr int BK2 = 32, NBUF = 4;
  constexpr int ABYTES = BM * BK2 * 2;         // 16 KB
  constexpr int BBYTES = BN * BK2 * 2;
  constexpr int BUF = ABYTES + BBYTES;
  constexpr int NJ = BN / 32;
  constexpr int QA = BM / 16 / 4;              // A DMAs (16-row blocks) per wave per K-tile
  constexpr int QB = BN / 16 / 4;
  constexpr int NQ = QA + QB;
  constexpr int NR = 8 + NJ;
  constexpr int NM = 8 * NJ;
  __shared__ __attribute__((aligned(16))) char lds[NBUF * BUF];

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

  const int nk_all = K / BK2;
  const int per = (nk_all + splits - 1) / splits;
  const int kt0 = sp * per;
  const int nk = max(0, min(nk_all, kt0 + per) - kt0);

  const rsrc_t ra = make_rsrc(A, (uint64_t)M * lda * 2);
  const rsrc_t rb = make_rsrc(B, (uint64_t)N * ldb * 2);
  const int r16 = lane >> 2, pc = lane & 3, lc = pc ^ ((-(r16 >> 2)) & 3);
  const uint32_t va = ((uint32_t)(m0 + w * QA * 16 + r16) * lda + lc * 8) * 2u;
  const uint32_t vb = ((uint32_t)(n0 + w * QB * 16 + r16) * ldb + lc * 8) * 2u;

  const uint32_t lds0 = (uint32_t)(uintptr_t)(lds_ptr_t)lds;
  const int fr = lane & 15, fcc = lane >> 4;
  const uint32_t flo = fr * 64 + 16 * (fcc ^ ((-(fr >> 2)) & 3));
  uint32_t pa[NBUF], pb[NBUF];
#pragma unroll
  for (int b = 0; b < NBUF; ++b) {
    pa[b] = lds0 + b * BUF + wr * 8 * 1024 + flo;
    pb[b] = lds0 + b * BUF + ABYTES + wc * (BN / 32) * 1024 + flo;
  }

  f32x4 acc[8][NJ];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  bf16x8 fa[2][8], fb[2][NJ];
  auto rd = [&](int b, int p, int r) {
    if (r < 8) ds_read128(fa[p][r], pa[b], r * 1024);
    else ds_read128(fb[p][r - 8], pb[b], (r - 8) * 1024);
  };
  auto dma = [&](int t, int b, int q) {
    const uint32_t kb = (uint32_t)(kt0 + (t < nk ? t : nk - 1)) * (BK2 * 2);
    char* buf = lds + b * BUF;
    if (q < QA)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(ra, (lds_ptr_t)(buf + (w * QA + q) * 1024), 16, va,
                                               kb + (uint32_t)(q * 16 * lda * 2), 0, 0);
    else
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rb, (lds_ptr_t)(buf + ABYTES + (w * QB + q - QA) * 1024), 16, vb,
                                               kb + (uint32_t)((q - QA) * 16 * ldb * 2), 0, 0);
  };
  constexpr int PRE = 4;   // MFMAs issued before the step's barrier
  auto step = [&](int t, int b, int p) {
#pragma unroll
    for (int q = 0; q < PRE; ++q) mfma16(acc[q / NJ][q % NJ], fb[p][q % NJ], fa[p][q / NJ]);
    asm volatile("s_waitcnt vmcnt(%0)" :: "n"(2 * NQ) : "memory");   // K-tile t+1 landed (t+2, t+3 in flight)
    barrier();                                                      // ... for every wave; buffer b is free
#pragma unroll
    for (int q = PRE; q < NM; ++q) {
      mfma16(acc[q / NJ][q % NJ], fb[p][q % NJ], fa[p][q / NJ]);
      const int u = q - PRE;
      if (u % 2 == 0 && u / 2 < NR) rd((b + 1) % NBUF, p ^ 1, u / 2);
      if (u % 3 == 1 && u / 3 < NQ) dma(t + NBUF, b, u / 3);
    }
    lgkm0();
  };
  if (nk > 0) {
    for (int b = 0; b < NBUF; ++b)
      for (int q = 0; q < NQ; ++q) dma(b, b, q);
    asm volatile("s_waitcnt vmcnt(%0)" :: "n"((NBUF - 1) * NQ) : "memory");
    barrier();
    for (int r = 0; r < NR; ++r) rd(0, 0, r);
    lgkm0();
    for (int t = 0; t < nk; t += 4) {
      step(t, 0, 0);
      step(t + 1, 1, 1);
      step(t + 2, 2, 0);
      step(t + 3, 3, 1);
    }
  }
  vm0();
  asm volatile("s_nop 15\n s_nop 15" ::: "memory");

#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int m = m0 + wr * 128 + i * 16 + (lane & 15);
    if (m >= M) continue;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int n = n0 + wc * (BN / 2) + j * 16 + 4 * (lane >> 4);
      if (n >= N) continue;
      f32x4 v = acc[i][j];
      if constexpr (SPLIT) {
        float* ws = reinterpret_cast<float*>(out) + ((size_t)sp * M + m) * ldc + n;
        *reinterpret_cast<f32x4*>(ws) = v;
      } else {
        bf16x4 o;
        o[0] = (bf16)v[0]; o[1] = (bf16)v[1]; o[2] = (bf16)v[2]; o[3] = (bf16)v[3];
        *reinterpret_cast<bf16x4*>(reinterpret_cast<bf16*>(out) + (size_t)m * ldc + n) = o;
      }
    }
  }
}


// ---- v3: v1's K-step (BK = 64, full 128-B line DMAs) with the A operand in 3 LDS slots and B in 2
//      (160 KB): A(t+2) is DMA'd during H1 into the slot of A(t-1), B(t+2) during H2 into the slot of
//      B(t), so the TA sees 8 DMAs per wave in each half instead of 16 in H2 only.
__device__ unsigned long long* g_dbg = nullptr;
template <bool SPLIT, bool PERSIST, int ABL = 0>
__global__ __launch_bounds__(NT, 1) __attribute__((amdgpu_waves_per_eu(1, 1))) void g1w3_nt_k(
    const bf16* __restrict__ A, int lda, const bf16* __restrict__ B, int ldb, const bf16* __restrict__ residual,
    void* __restrict__ out, int ldc, int M, int N, int K, int splits) {
  const unsigned long long c0 = __builtin_readcyclecounter(), r0 = __builtin_amdgcn_s_memrealtime();
  constexpr int BN = 256;
  constexpr int SLOT = BM * BK * 2;            // 32 KB
  constexpr int NJ = 8, NR = 16, NM = 64;
  constexpr int QA = 8, QB = 8;                // DMAs per wave per operand per K-tile
  __shared__ __attribute__((aligned(16))) char lds[5 * SLOT];
  // slots: A0 A1 A2 B0 B1
  const int tiles_m = (M + BM - 1) / BM, tiles_n = (N + BN - 1) / BN;
  const int ntiles = tiles_m * tiles_n * splits;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const int wr = w >> 1, wc = w & 1;
  const int nk_all = K / BK;
  const int per = (nk_all + splits - 1) / splits;

  const rsrc_t ra = make_rsrc(A, (uint64_t)M * lda * 2);
  const rsrc_t rb = make_rsrc(B, (uint64_t)N * ldb * 2);
  const int r8 = lane >> 3, ch = (lane & 7) ^ (r8 & 6);
  const uint32_t lds0 = (uint32_t)(uintptr_t)(lds_ptr_t)lds;
  uint32_t lo[2];
#pragma unroll
  for (int s = 0; s < 2; ++s) lo[s] = ((lane >> 3) & 1) * 1024 + 16 * slot_of(lane & 7, 4 * s + (lane >> 4));

  for (int item = blockIdx.x; item < ntiles; item += (PERSIST ? gridDim.x : ntiles)) {
    const int id = PERSIST ? item : xcd_remap(item, ntiles);
    const int sp = id % splits;
    const int tid = id / splits;
    const int tm = tid % tiles_m, tn = tid / tiles_m;
    const int m0 = tm * BM, n0 = tn * BN;
    const int kt0 = sp * per;
    const int nk = max(0, min(nk_all, kt0 + per) - kt0);
    const uint32_t va = ((uint32_t)(m0 + w * QA * 8 + r8) * lda + ch * 8) * 2u;
    const uint32_t vb = ((uint32_t)(n0 + w * QB * 8 + r8) * ldb + ch * 8) * 2u;

    f32x4 acc[8][NJ];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    bf16x8 fa[2][8], fb[2][NJ];

    auto dmaA = [&](int t, int slot, int q) {
      const uint32_t kb = (uint32_t)(kt0 + (t < nk ? t : nk - 1)) * (BK * 2);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(ra, (lds_ptr_t)(lds + slot * SLOT + (w * QA + q) * 1024), 16, va,
                                               kb + (uint32_t)(q * 8 * lda * 2), 0, 0);
    };
    auto dmaB = [&](int t, int slot, int q) {
      const uint32_t kb = (uint32_t)(kt0 + (t < nk ? t : nk - 1)) * (BK * 2);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rb, (lds_ptr_t)(lds + (3 + slot) * SLOT + (w * QB + q) * 1024), 16, vb,
                                               kb + (uint32_t)(q * 8 * ldb * 2), 0, 0);
    };
    // fragment r (0..7 A, 8..15 B) of k-substep s of the tile in A-slot sa / B-slot sb
    auto rd = [&](int sa, int sb, int s, int p, int r) {
      if (r < 8) ds_read128(fa[p][r], lds0 + sa * SLOT + wr * 16 * 1024 + lo[s], r * 2048);
      else ds_read128(fb[p][r - 8], lds0 + (3 + sb) * SLOT + wc * 16 * 1024 + lo[s], (r - 8) * 2048);
    };
    // step t: A(t) in slot t % 3, B(t) in slot t % 2; F0 = fa/fb[0] holds k-substep 0 of tile t
    auto step = [&](int t, int sa, int sb) {
      const int sa1 = sa == 2 ? 0 : sa + 1, sa2 = sa1 == 2 ? 0 : sa1 + 1;   // slots of t+1, t+2 (= t-1)
      // H1: MFMA ks0; read ks1 of tile t; DMA A(t+2) into the slot of A(t-1)
#pragma unroll
      for (int q = 0; q < NM; ++q) {
        mfma16(acc[q / NJ][q % NJ], fb[0][q % NJ], fa[0][q / NJ]);
        if (!(ABL & 4) && q % 4 == 0) rd(sa, sb, 1, 1, q / 4);
        if (!(ABL & 1) && q % 8 == 2) dmaA(t + 2, sa2, q / 8);
      }
      lgkm0();
      if (!(ABL & 2)) {
        asm volatile("s_waitcnt vmcnt(%0)" :: "n"(QA) : "memory");   // A(t+1), B(t+1) landed; A(t+2) may fly
        barrier();
      }
      // H2: MFMA ks1; read ks0 of tile t+1; DMA B(t+2) into the slot of B(t)
#pragma unroll
      for (int q = 0; q < NM; ++q) {
        mfma16(acc[q / NJ][q % NJ], fb[1][q % NJ], fa[1][q / NJ]);
        if (!(ABL & 4) && q % 4 == 2) rd(sa1, sb ^ 1, 0, 0, q / 4);
        if (!(ABL & 1) && q % 8 == 4) dmaB(t + 2, sb, q / 8);
      }
      lgkm0();
    };
    if (nk > 0) {
      for (int q = 0; q < QA; ++q) dmaA(0, 0, q);
      for (int q = 0; q < QB; ++q) dmaB(0, 0, q);
      for (int q = 0; q < QA; ++q) dmaA(1, 1, q);
      for (int q = 0; q < QB; ++q) dmaB(1, 1, q);
      asm volatile("s_waitcnt vmcnt(%0)" :: "n"(QA + QB) : "memory");
      barrier();
      for (int r = 0; r < NR; ++r) rd(0, 0, 0, 0, r);
      lgkm0();
      int sa = 0;
      for (int t = 0; t < nk; t += 2) {
        step(t, sa, 0);
        sa = sa == 2 ? 0 : sa + 1;
        step(t + 1, sa, 1);
        sa = sa == 2 ? 0 : sa + 1;
      }
    }
    vm0();
    asm volatile("s_nop 15\n s_nop 15" ::: "memory");
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int m = m0 + wr * 128 + i * 16 + (lane & 15);
      if (m >= M) continue;
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int n = n0 + wc * (BN / 2) + j * 16 + 4 * (lane >> 4);
        if (n >= N) continue;
        f32x4 v = acc[i][j];
        if constexpr (SPLIT) {
          float* ws = reinterpret_cast<float*>(out) + ((size_t)sp * M + m) * ldc + n;
          *reinterpret_cast<f32x4*>(ws) = v;
        } else {
          bf16x4 o;
          o[0] = (bf16)v[0]; o[1] = (bf16)v[1]; o[2] = (bf16)v[2]; o[3] = (bf16)v[3];
          *reinterpret_cast<bf16x4*>(reinterpret_cast<bf16*>(out) + (size_t)m * ldc + n) = o;
        }
      }
    }
    if constexpr (PERSIST) barrier();   // LDS reuse by the next tile
  }
  if (g_dbg && threadIdx.x == 0) {
    const unsigned long long c1 = __builtin_readcyclecounter(), r1 = __builtin_amdgcn_s_memrealtime();
    unsigned xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    g_dbg[blockIdx.x * 4 + 0] = c1 - c0;
    g_dbg[blockIdx.x * 4 + 1] = r1 - r0;
    g_dbg[blockIdx.x * 4 + 2] = r0;
    g_dbg[blockIdx.x * 4 + 3] = xcc;
  }
}

__global__ __launch_bounds__(256) void splitk_reduce_k(const float* __restrict__ ws, bf16* __restrict__ out, size_t MN,
                                                       int splits) {
  for (size_t i = ((size_t)blockIdx.x * 256 + threadIdx.x) * 4; i < MN; i += (size_t)gridDim.x * 256 * 4) {
    f32x4 v = *reinterpret_cast<const f32x4*>(ws + i);
    for (int s = 1; s < splits; ++s) v += *reinterpret_cast<const f32x4*>(ws + (size_t)s * MN + i);
    bf16x4 o;
    o[0] = (bf16)v[0]; o[1] = (bf16)v[1]; o[2] = (bf16)v[2]; o[3] = (bf16)v[3];
    *reinterpret_cast<bf16x4*>(out + i) = o;
  }
}

}  // namespace

extern "C" int g1w_set_dbg(void* p) { return hipMemcpyToSymbol(HIP_SYMBOL(g_dbg), &p, sizeof(p)) == hipSuccess ? 0 : 1; }

extern "C" int g1w_launch(const void* A, const void* B, void* out, float* ws, int M, int N, int K, int bn, int splits,
                          hipStream_t st) {
  const bool v3 = bn > 1000;
  if (v3) {   // bn = 1256: v3, 2256: v3 persistent
    if (splits < 1) splits = 1;
    if (K % 128 || N % 256 || M % 16 || (K / BK) % (2 * splits)) return 1;
    const int tiles = ((M + BM - 1) / BM) * (N / 256) * splits;
    void* o = splits > 1 ? (void*)ws : out;
    const bool pers = bn > 2000;
    const int g = pers ? (tiles < 256 ? tiles : 256) : tiles;
    if (splits > 1) {
      if (pers) g1w3_nt_k<true, true><<<g, NT, 0, st>>>((const bf16*)A, K, (const bf16*)B, K, nullptr, o, N, M, N, K, splits);
      else g1w3_nt_k<true, false><<<g, NT, 0, st>>>((const bf16*)A, K, (const bf16*)B, K, nullptr, o, N, M, N, K, splits);
      splitk_reduce_k<<<2048, 256, 0, st>>>(ws, (bf16*)out, (size_t)M * N, splits);
    } else {
      static const int abl = getenv("G1W_ABL") ? atoi(getenv("G1W_ABL")) : 0;
#define L3(AB) g1w3_nt_k<false, false, AB><<<g, NT, 0, st>>>((const bf16*)A, K, (const bf16*)B, K, nullptr, o, N, M, N, K, splits)
      if (pers) g1w3_nt_k<false, true><<<g, NT, 0, st>>>((const bf16*)A, K, (const bf16*)B, K, nullptr, o, N, M, N, K, splits);
      else if (abl == 1) L3(1);
      else if (abl == 2) L3(2);
      else if (abl == 3) L3(3);
      else if (abl == 4) L3(4);
      else if (abl == 7) L3(7);
      else L3(0);
    }
    return hipGetLastError() == hipSuccess ? 0 : 2;
  }
  const bool v2 = bn < 0;
  if (v2) bn = -bn;
  if (splits < 1) splits = 1;
  const int kq = v2 ? 32 * 4 : BK * 2;
  if (K % kq || N % bn || M % 16 || (K / kq) % splits) return 1;
  const int tiles = ((M + BM - 1) / BM) * ((N + bn - 1) / bn);
  const int g = tiles * splits;
  void* o = splits > 1 ? (void*)ws : out;
#define L1(BN_, S_) g1w_nt_k<BN_, S_><<<g, NT, 0, st>>>((const bf16*)A, K, (const bf16*)B, K, nullptr, o, N, M, N, K, splits)
#define L2(BN_, S_) g1w32_nt_k<BN_, S_><<<g, NT, 0, st>>>((const bf16*)A, K, (const bf16*)B, K, nullptr, o, N, M, N, K, splits)
  static const int abl = getenv("G1W_ABL") ? atoi(getenv("G1W_ABL")) : 0;
  if (!v2 && bn == 256 && splits == 1 && abl) {
    if (abl == 1) g1w_nt_k<256, false, 1><<<g, NT, 0, st>>>((const bf16*)A, K, (const bf16*)B, K, nullptr, o, N, M, N, K, splits);
    if (abl == 2) g1w_nt_k<256, false, 2><<<g, NT, 0, st>>>((const bf16*)A, K, (const bf16*)B, K, nullptr, o, N, M, N, K, splits);
    if (abl == 3) g1w_nt_k<256, false, 3><<<g, NT, 0, st>>>((const bf16*)A, K, (const bf16*)B, K, nullptr, o, N, M, N, K, splits);
    if (abl == 7) g1w_nt_k<256, false, 7><<<g, NT, 0, st>>>((const bf16*)A, K, (const bf16*)B, K, nullptr, o, N, M, N, K, splits);
  } else if (!v2) {
    if (bn == 256) { if (splits > 1) L1(256, true); else L1(256, false); }
    else { if (splits > 1) L1(128, true); else L1(128, false); }
  } else {
    if (bn == 256) { if (splits > 1) L2(256, true); else L2(256, false); }
    else { if (splits > 1) L2(128, true); else L2(128, false); }
  }
  if (splits > 1) {
    const size_t MN = (size_t)M * N;
    splitk_reduce_k<<<2048, 256, 0, st>>>(ws, (bf16*)out, MN, splits);
  }
  return hipGetLastError() == hipSuccess ? 0 : 2;
}
