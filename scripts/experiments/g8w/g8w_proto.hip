// Prototype: 8-wave (2 waves per SIMD) ping-pong 256x256x64 bf16 GEMM, NT: y = A·Bᵀ (+ residual).
// Standalone harness: times it against gemm4w (one-wave-per-SIMD, the shipped kernel) in ONE process on
// uniform [-1, 1) operands and checks it against gemm4w's output.
//
// Schedule (per wave, per K-tile: 4 phases of 16 MFMAs = one C-quadrant x K 64):
//   wave w: wr = w >> 2 (128-row half), wc = w & 3 (64-column quarter); waves w and w + 4 share a SIMD.
//   group 1 (wr = 1) runs one s_barrier behind group 0, so each SIMD alternates the two waves' 16-MFMA
//   clusters and each wave's LDS reads + LDS-DMA issue sit beside its partner's MFMAs.
//   LDS: 2 buffers (tile parity) x 4 quarters of 16 KB: QALO / QAHI = A rows the waves read in their
//   a-lo / a-hi quadrants, QBLO / QBHI = B rows of the b-lo / b-hi quadrants.  Quarter issue order
//   (tile T phase k): Qb_hi(T+1), Qb_lo(T+1), Qa_hi(T+1), Qa_lo(T+2); vmcnt(6) in phase 1, vmcnt(4) in phase 3
//   (vmcnt(0) / vmcnt(2) at the last tiles, where fewer DMAs follow).
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include <type_traits>
#include "common.h"
// gemm4w (the shipped kernel) is linked in from its prebuilt object
int gemm4w_plan(int M, int N, int K, bool bt, int bn, int splits, int* bn_out, int bm, int* bm_out, bool w4);
void launch_gemm4w(const void* A, int lda, const void* B, int ldb, const void* residual, void* out, float* ws,
                   const float* bscale, const float* bzero, int M, int N, int K, int splits, bool bt, int bn, int bm,
                   hipStream_t st);

namespace g8 {
using namespace lipa;
typedef __amdgpu_buffer_rsrc_t rsrc_t;

constexpr int NTH = 512, QB = 16384, BUF = 65536;
constexpr int QALO = 0, QAHI = 1, QBLO = 2, QBHI = 3;
constexpr int WAIT_LGKM0 = 0 | (7 << 4) | (0 << 8) | (3 << 14);

__device__ __forceinline__ rsrc_t make_rsrc(const void* base, uint64_t bytes) {
  const uint64_t p = reinterpret_cast<uint64_t>(base);
  const uint32_t lo = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(p));
  const uint32_t hi = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(p >> 32));
  const uint32_t n = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(bytes > 0xFFFFFFFFull ? 0xFFFFFFFFull : bytes));
  void* b = reinterpret_cast<void*>((static_cast<uint64_t>(hi) << 32) | lo);
  return __builtin_amdgcn_make_buffer_rsrc(b, 0, n, 0x00020000);
}
__device__ __forceinline__ void dma_lds(const rsrc_t& rs, uint32_t dst, uint32_t voff, uint32_t soff) {
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %1\n\t"
      "s_nop 0\n\t"
      "buffer_load_dwordx4 %2, %3, %4 offen lds\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "s"(dst), "v"(voff), "s"(rs), "s"(soff)
      : "memory");
}
template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
__device__ __forceinline__ void mfma_acc(f32x4& acc, const bf16x8& a, const bf16x8& b) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(a), "v"(b));
}
__device__ __forceinline__ bf16x8 lds_frag(const char* p) { return *reinterpret_cast<const bf16x8*>(p); }

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

// local row rl (0..127) of quarter q -> row of the 256-row A or B tile
__device__ __forceinline__ int quarter_row(int q, int rl) {
  if (q == QALO) return 128 * (rl >> 6) + (rl & 63);
  if (q == QAHI) return 128 * (rl >> 6) + 64 + (rl & 63);
  if (q == QBLO) return 64 * (rl >> 5) + (rl & 31);
  return 64 * (rl >> 5) + 32 + (rl & 31);
}

template <int PRIO>
__global__ __launch_bounds__(NTH, 1) void g8w_k(const bf16* __restrict__ A, int lda, const bf16* __restrict__ B, int ldb,
                                                const bf16* __restrict__ residual, bf16* __restrict__ out, int M, int N,
                                                int K) {
  __shared__ __attribute__((aligned(16))) char lds[2 * BUF];
  const int tiles_m = (M + 255) / 256, tiles_n = (N + 255) / 256;
  const int id = xcd_remap(blockIdx.x, tiles_m * tiles_n);
  const int tm = id % tiles_m, tn = id / tiles_m;
  const int m0 = tm * 256, n0 = tn * 256;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const int wr = w >> 2, wc = w & 3;
  const int nk = K / 64;

  const rsrc_t rsa = make_rsrc(A, (uint64_t)((size_t)(M - 1) * lda + K) * 2);
  const rsrc_t rsb = make_rsrc(B, (uint64_t)((size_t)(N - 1) * ldb + K) * 2);
  // per-lane DMA source offsets: quarter q, piece p = 2w + i (local rows 8p .. 8p + 7)
  uint32_t vo[4][2];
  {
    const int r8 = lane >> 3, c = (lane & 7) ^ (r8 & 6);
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int rl = 8 * (2 * w + i) + r8;
        const int tr = quarter_row(q, rl);
        if (q < 2) {
          const int ra = min(m0 + tr, M - 1);
          vo[q][i] = ((uint32_t)ra * (uint32_t)lda + (uint32_t)(c * 8)) * 2u;
        } else {
          const int rb = min(n0 + tr, N - 1);
          vo[q][i] = ((uint32_t)rb * (uint32_t)ldb + (uint32_t)(c * 8)) * 2u;
        }
      }
  }
  const uint32_t lds_base = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(__attribute__((address_space(3))) void*)lds);
  auto dma_q = [&](int q, int t) {   // this wave's 2 pieces of quarter q of K-tile t into buffer t & 1
    if (t >= nk) return;
    const uint32_t dst = lds_base + (uint32_t)((t & 1) * BUF + q * QB + (2 * w) * 1024);
    const rsrc_t& rs = q < 2 ? rsa : rsb;
    dma_lds(rs, dst, vo[q][0], (uint32_t)t * 128u);
    dma_lds(rs, dst + 1024, vo[q][1], (uint32_t)t * 128u);
  };

  // fragment read offsets within a 2 KB (16-row) fragment
  int lo[2];
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    const int r8 = lane & 7, c = 4 * s + (lane >> 4);
    lo[s] = ((lane >> 3) & 1) * 1024 + 16 * (8 * r8 + (c ^ (r8 & 6)));
  }
  const int a_off = wr * 4 * 2048;   // the wave's 4 fragments inside an A quarter
  const int b_off = wc * 2 * 2048;   // the wave's 2 fragments inside a B quarter

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  bf16x8 fa[4][2], fb[2][2];

  // prologue: Qa_lo(0), Qb_lo(0), Qb_hi(0), Qa_hi(0), Qa_lo(1)
  dma_q(QALO, 0);
  dma_q(QBLO, 0);
  dma_q(QBHI, 0);
  dma_q(QAHI, 0);
  dma_q(QALO, 1);
  if (nk > 1) wait_vmcnt<4>();   // QAHI(0), QALO(1) may stay in flight
  else wait_vmcnt<2>();
  __builtin_amdgcn_s_barrier();
  if (wr == 1) __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);

  for (int t = 0; t < nk; ++t) {
    const char* cur = lds + (t & 1) * BUF;
    Unroll<0, 4>::run([&](auto kc) {
      constexpr int k = decltype(kc)::value;
      // ---- load part: this quadrant's fragments, two LDS-DMA pieces of a later tile
      if constexpr (k == 0 || k == 2) {
        const char* qa = cur + (k == 0 ? QALO : QAHI) * QB + a_off;
#pragma unroll
        for (int f = 0; f < 4; ++f)
#pragma unroll
          for (int s = 0; s < 2; ++s) fa[f][s] = lds_frag(qa + f * 2048 + lo[s]);
      }
      if constexpr (k != 2) {
        const char* qb = cur + (k == 1 ? QBHI : QBLO) * QB + b_off;
#pragma unroll
        for (int f = 0; f < 2; ++f)
#pragma unroll
          for (int s = 0; s < 2; ++s) fb[f][s] = lds_frag(qb + f * 2048 + lo[s]);
      }
      if constexpr (k == 0) dma_q(QBHI, t + 1);
      // counted waits, exact at the tail too (the round-5 build used vmcnt(6) / vmcnt(4) on every tile: at the last
      // two tiles the skipped DMAs made those counts let QBLO / QAHI of the current tile through unlanded)
      //   phase 1: QAHI(t) landed; issued after it: QALO(t+1), QBHI(t+1), QBLO(t+1) — 6 if t+1 < nk, else 0
      //   phase 3: QALO/QBHI/QBLO(t+1) landed; issued after: QAHI(t+1), QALO(t+2) — 4 if t+2 < nk, 2 if t+1 < nk
      if constexpr (k == 1) {
        dma_q(QBLO, t + 1);
        if (t + 1 < nk) wait_vmcnt<6>();
        else wait_vmcnt<0>();
      }
      if constexpr (k == 2) dma_q(QAHI, t + 1);
      if constexpr (k == 3) {
        dma_q(QALO, t + 2);
        if (t + 2 < nk) wait_vmcnt<4>();
        else wait_vmcnt<2>();
      }
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_s_waitcnt(WAIT_LGKM0);
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (PRIO) __builtin_amdgcn_s_setprio(1);
      constexpr int i0 = (k == 0 || k == 1) ? 0 : 4;
      constexpr int j0 = (k == 0 || k == 3) ? 0 : 2;
#pragma unroll
      for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j) mfma_acc(acc[i0 + i][j0 + j], fb[j][s], fa[i][s]);
      if constexpr (PRIO) __builtin_amdgcn_s_setprio(0);
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
    });
  }
  if (wr == 0) __builtin_amdgcn_s_barrier();
  asm volatile("s_waitcnt vmcnt(0)\n\ts_nop 7\n\ts_nop 7" ::: "memory");

  // epilogue: lane holds C[m = 16 i + (lane & 15)][n = 16 j + 4 (lane >> 4) + e] of the wave's 128 x 64
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int m = m0 + 128 * wr + 16 * i + (lane & 15);
    if (m >= M) continue;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int n = n0 + 64 * wc + 16 * j + 4 * (lane >> 4);
      if (n >= N) continue;
      bf16x4 o;
      if (residual) {
        const bf16x4 r = *reinterpret_cast<const bf16x4*>(residual + (size_t)m * N + n);
#pragma unroll
        for (int e = 0; e < 4; ++e) o[e] = (bf16)(acc[i][j][e] + (float)r[e]);
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) o[e] = (bf16)acc[i][j][e];
      }
      *reinterpret_cast<bf16x4*>(out + (size_t)m * N + n) = o;
    }
  }
}
}  // namespace g8

#define CK(x)                                                                         \
  do {                                                                                \
    hipError_t e = (x);                                                               \
    if (e != hipSuccess) {                                                            \
      fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); \
      exit(1);                                                                        \
    }                                                                                 \
  } while (0)

__global__ void fill_k(lipa::bf16* p, size_t n, uint32_t seed) {
  size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  for (; i < n; i += (size_t)gridDim.x * 256) {
    uint32_t h = (uint32_t)i * 2654435761u ^ seed;
    h ^= h >> 13; h *= 0x5bd1e995u; h ^= h >> 15;
    p[i] = (lipa::bf16)((float)(h & 0xFFFFFF) / 8388608.f - 1.f);
  }
}
__global__ void diff_k(const lipa::bf16* a, const lipa::bf16* b, size_t n, float* out) {
  __shared__ float s[2][256];
  float d = 0.f, r = 0.f;
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
    float x = (float)a[i], y = (float)b[i];
    d += (x - y) * (x - y);
    r += y * y;
  }
  s[0][threadIdx.x] = d;
  s[1][threadIdx.x] = r;
  __syncthreads();
  if (threadIdx.x == 0) {
    float dd = 0.f, rr = 0.f;
    for (int i = 0; i < 256; ++i) { dd += s[0][i]; rr += s[1][i]; }
    atomicAdd(out, dd);
    atomicAdd(out + 1, rr);
  }
}

int main(int argc, char** argv) {
  struct Shape { const char* name; int M, N, K; };
  std::vector<Shape> shapes = {{"gate_up", 2048, 24576, 4096}, {"o", 2048, 4096, 4096},   {"qkv", 2048, 6144, 4096},
                               {"down", 2048, 4096, 12288},    {"sq4k", 4096, 4096, 4096}, {"sq8k", 8192, 8192, 8192},
                               {"dX_down_nt", 2048, 12288, 4096}};
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  float* dd;
  CK(hipMalloc(&dd, 8));
  for (const auto& s : shapes) {
    const size_t na = (size_t)s.M * s.K, nb = (size_t)s.N * s.K, nc = (size_t)s.M * s.N;
    lipa::bf16 *a, *b, *c1, *c2;
    float* ws;
    CK(hipMalloc(&a, na * 2));
    CK(hipMalloc(&b, nb * 2));
    CK(hipMalloc(&c1, nc * 2));
    CK(hipMalloc(&c2, nc * 2));
    CK(hipMalloc(&ws, nc * 4 * 4));
    fill_k<<<2048, 256>>>(a, na, 1234u);
    fill_k<<<2048, 256>>>(b, nb, 987u);
    int bn = 0, bm = 0;
    const int sp = gemm4w_plan(s.M, s.N, s.K, false, 0, 0, &bn, 0, &bm, false);
    auto run4 = [&]() { launch_gemm4w(a, s.K, b, s.K, nullptr, c1, ws, nullptr, nullptr, s.M, s.N, s.K, sp, false, bn, bm, 0); };
    // gemm4w forced onto g8w's own tiling (256 x 256, whole K): the same-work comparison
    int bnf = 0, bmf = 0;
    const int spf = gemm4w_plan(s.M, s.N, s.K, false, 256, 1, &bnf, 256, &bmf, false);
    auto run4f = [&]() { launch_gemm4w(a, s.K, b, s.K, nullptr, c1, ws, nullptr, nullptr, s.M, s.N, s.K, spf, false, bnf, bmf, 0); };
    const int grid8 = ((s.M + 255) / 256) * ((s.N + 255) / 256);
    auto run8 = [&](int prio) {
      if (prio) g8::g8w_k<1><<<grid8, 512, 0, 0>>>(a, s.K, b, s.K, nullptr, c2, s.M, s.N, s.K);
      else g8::g8w_k<0><<<grid8, 512, 0, 0>>>(a, s.K, b, s.K, nullptr, c2, s.M, s.N, s.K);
    };
    run4f();   // the bit-exactness reference: gemm4w on the same tiling (whole K, K-tiles summed in the same order)
    run8(1);
    CK(hipDeviceSynchronize());
    CK(hipMemset(dd, 0, 8));
    diff_k<<<1024, 256>>>(c2, c1, nc, dd);
    float h[2];
    CK(hipMemcpy(h, dd, 8, hipMemcpyDeviceToHost));
    const double fl = 2.0 * s.M * s.N * s.K;
    auto timeit = [&](auto&& fn) {
      for (int i = 0; i < 3; ++i) fn();
      CK(hipEventRecord(e0));
      const int it = 10;
      for (int i = 0; i < it; ++i) fn();
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      return ms * 1000.f / it;
    };
    float b4 = 1e9, b4f = 1e9, b8 = 1e9, b8n = 1e9;
    for (int r = 0; r < 5; ++r) {
      b4 = fminf(b4, timeit(run4));
      b4f = fminf(b4f, timeit(run4f));
      b8 = fminf(b8, timeit([&] { run8(1); }));
      b8n = fminf(b8n, timeit([&] { run8(0); }));
    }
    printf("%-10s M=%5d N=%6d K=%6d  gemm4w(%dx%d s%d) %7.1f us %5.0f TF/s | gemm4w(256x256 s%d) %7.1f us %5.0f TF/s | "
           "g8w %7.1f us %5.0f TF/s | g8w-noprio %7.1f us %5.0f TF/s | g8w vs gemm4w 256x256 s1: %s (relerr %.2e)\n",
           s.name, s.M, s.N, s.K, bm, bn, sp, b4, fl / b4 / 1e6, spf, b4f, fl / b4f / 1e6, b8, fl / b8 / 1e6, b8n,
           fl / b8n / 1e6, h[0] == 0.f ? "bit-exact" : "DIFFERENT", std::sqrt(h[0] / h[1]));
    fflush(stdout);
    CK(hipFree(a));
    CK(hipFree(b));
    CK(hipFree(c1));
    CK(hipFree(c2));
    CK(hipFree(ws));
  }
  return 0;
}
