// One-wave-per-SIMD MFMA GEMM for gfx950 — the frozen-base GEMMs of the QLoRA step:
//
//   forward   y  = x·Wᵀ (+ residual)      A = x [M, K],  B = W  [N, K]   (NT)
//   backward  dX = dY·W (+ C)             A = dY [M, K], B = W  [K, N]   (BT: W used as stored)
//
// Design (profiles/gemm4w_*.txt):
//  * 256 threads = 4 waves as 2 (M) × 2 (N), one wave per SIMD; a wave owns a 128 × BN/2 output block
//    of v_mfma_f32_16x16x32_bf16 accumulators (256 or 128 fp32 per lane) held in AGPRs.  The MFMAs
//    are one-instruction asm statements with the accumulator a tied "+a" operand: with the builtin,
//    hipcc split the accumulator phis between the two K-halves and shuffled ~48 v_accvgpr_mov/read/
//    write per K-tile through the MFMA results.  Hazards the asm hides from hipcc: none in the loop
//    (a fragment register is rewritten ≥ 16 MFMAs after its last reader; a single wave per SIMD, so
//    no partner's MFMAs sit between); the epilogue's AGPR reads sit behind 16 wait states.
//  * BN = 256 (grids of ≥ 256 tiles: gate|up forward, the LM head) or BN = 128 (the M = 2048 × 4096
//    shapes — o / down forward and every dX to d_model: 256 tiles fill the chip without split-K).
//  * global → LDS only by LDS-DMA (buffer_load … lds, 1 KB per wave-instruction, whole 128-B lines),
//    STAGES K-tile stages (2 for BN = 256: 128 KB; 3 for BN = 128: 144 KB).  Per K-tile one
//    compile-time-unrolled stream of 16·BN/32 MFMAs (first K-half on fA, second on fB):
//      - the first R MFMAs each carry one fragment read of this tile's second half (into fB);
//      - barrier 1 (lgkmcnt(0)): nobody reads stage t % STAGES any more → its LDS-DMA refill with
//        tile t + STAGES is spread over the middle MFMAs;
//      - barrier 2 (vmcnt((STAGES − 1)·D)): tile t + 1 has landed;
//      - the last R MFMAs each carry one fragment read of tile t + 1's first half (into fA).
//    The first half walks (i, j) in shells of max(i, j), so MFMA k waits only on reads issued ≥ 14
//    MFMAs earlier.
//  * NT images: 1 KB subtiles of 8 rows × 64 k, 16-B chunk c of row r at slot 8r + (c ^ (r & 6))
//    (conflict-free ds_read_b128).  BT image: 64 k-rows × 2·BN bytes with the 32-B column pairs XOR-
//    permuted by h(k) = (k & 3) | ((k >> 1) & 4), read as the B operand by two ds_read_b64_tr_b16 per
//    fragment (a 32-lane half reads rows {0-3, 8-11} (+4) of a 16-row group: 8 distinct h → conflict-
//    free).  Every swizzle is applied on the DMA SOURCE address (the LDS side is lane-linear).
//  * XCD-aware tile order: the m-tiles of one weight panel are consecutive ids and share an XCD's L2.
//  * split-K (grids still smaller than the chip): fp32 slabs + one reduce launch (+ residual); the
//    in-launch form (the tile's last-arriving split sums the slabs after an agent release / ticket /
//    acquire) is kept behind LIPA_GEMM4W_INLAUNCH_REDUCE=1 — measured 1.1 ms/step slower.
#include <type_traits>

#include "common.h"

using namespace lipa;

namespace {

typedef __attribute__((address_space(3))) void* lds_ptr_t;
typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4;
typedef __amdgpu_buffer_rsrc_t rsrc_t;

constexpr int BK = 64, NT = 256;

__device__ __forceinline__ rsrc_t make_rsrc(const void* base, uint64_t bytes) {
  const uint64_t p = reinterpret_cast<uint64_t>(base);
  const uint32_t lo = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(p));
  const uint32_t hi = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(p >> 32));
  const uint32_t n = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(bytes > 0xFFFFFFFFull ? 0xFFFFFFFFull : bytes));
  void* b = reinterpret_cast<void*>((static_cast<uint64_t>(hi) << 32) | lo);
  return __builtin_amdgcn_make_buffer_rsrc(b, 0, n, 0x00020000);
}

__device__ __forceinline__ int slot_of(int r8, int c) { return 8 * r8 + (c ^ (r8 & 6)); }

__device__ __forceinline__ bf16x8 lds_frag(const char* p) { return *reinterpret_cast<const bf16x8*>(p); }

__device__ __forceinline__ void mfma_acc(f32x4& acc, const bf16x8& a, const bf16x8& b) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(a), "v"(b));
}
__device__ __forceinline__ void mfma_zero(f32x4& acc, const bf16x8& a, const bf16x8& b) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, 0" : "=a"(acc) : "v"(a), "v"(b));
}

// s_waitcnt immediate for lgkmcnt(0) (gfx9 encoding: vmcnt[3:0] | expcnt[6:4] | lgkmcnt[11:8] | vmcnt[5:4] << 14)
constexpr int WAIT_LGKM0 = 0 | (7 << 4) | (0 << 8) | (3 << 14);

// vmcnt wait as an asm statement (the DMAs it counts are asm too, invisible to hipcc's counters)
template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// one wave-instruction of LDS-DMA: 64 lanes × 16 B from rs + voff + soff into LDS [dst, dst + 1 KB);
// M0 (the LDS base, compiler-reserved) is written and restored inside the statement.  dst and soff
// are SALU values (never fresh from v_readfirstlane, so no VALU→SGPR→VMEM wait states are needed)
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

// compile-time unrolled loop: f(std::integral_constant<int, k>) for k in [K, N)
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

// Per-tile schedule tables (NA a-fragments × NB b-fragments per wave and K-half): MFMA order of a
// K-half (shells of max(i, j), then the remaining rows / columns) and the fragment-read order
// (a0 b0 a1 b1 …, then the remaining a's or b's) — MFMA k waits only on reads issued well before it.
template <int NA, int NB>
struct Sched {
  int i[NA * NB], j[NA * NB];
  int rd_a[NA + NB], rd_i[NA + NB];   // read item r: a fragment? index
};
template <int NA, int NB>
constexpr Sched<NA, NB> make_sched() {
  Sched<NA, NB> o{};
  constexpr int S = NA < NB ? NA : NB;
  int k = 0;
  for (int s = 0; s < S; ++s) {
    for (int j = 0; j <= s; ++j) { o.i[k] = s; o.j[k] = j; ++k; }
    for (int i = 0; i < s; ++i) { o.i[k] = i; o.j[k] = s; ++k; }
  }
  for (int i = S; i < NA; ++i)
    for (int j = 0; j < NB; ++j) { o.i[k] = i; o.j[k] = j; ++k; }
  for (int j = S; j < NB; ++j)
    for (int i = 0; i < S; ++i) { o.i[k] = i; o.j[k] = j; ++k; }
  int r = 0;
  for (int s = 0; s < S; ++s) {
    o.rd_a[r] = 1; o.rd_i[r] = s; ++r;
    o.rd_a[r] = 0; o.rd_i[r] = s; ++r;
  }
  for (int i = S; i < NA; ++i) { o.rd_a[r] = 1; o.rd_i[r] = i; ++r; }
  for (int j = S; j < NB; ++j) { o.rd_a[r] = 0; o.rd_i[r] = j; ++r; }
  return o;
}
constexpr Sched<8, 8> kSched88 = make_sched<8, 8>();
constexpr Sched<8, 4> kSched84 = make_sched<8, 4>();
constexpr Sched<8, 6> kSched86 = make_sched<8, 6>();
constexpr Sched<4, 8> kSched48 = make_sched<4, 8>();
constexpr Sched<4, 4> kSched44 = make_sched<4, 4>();
constexpr Sched<4, 6> kSched46 = make_sched<4, 6>();
template <int NA, int NB>
__host__ __device__ constexpr const Sched<NA, NB>& sched_of();
#define G4W_SCHED(A_, B_) \
  template <>             \
  __host__ __device__ constexpr const Sched<A_, B_>& sched_of<A_, B_>() { return kSched##A_##B_; }
G4W_SCHED(8, 8)
G4W_SCHED(8, 4)
G4W_SCHED(8, 6)
G4W_SCHED(4, 8)
G4W_SCHED(4, 4)
G4W_SCHED(4, 6)
#undef G4W_SCHED

__device__ __forceinline__ float silu_f(float g) { return g / (1.f + __expf(-g)); }

// EPI (fused MLP epilogues; SURVEY.md K5 "activation in the GEMM epilogue"):
//   1  SwiGLU forward on the gate|up projection (NT, no split).  B = W_gu [2F, K] as stored ([gate | up]
//      rows); the tile's B rows are gathered so that fragment pair (2c, 2c+1) of a wave is gate rows
//      16c'…+15 and the matching up rows — every lane then holds g and u of the same (m, col).  Writes
//      gu [M, 2F] in the [gate | up] layout (saved for backward) and h = silu(g)·u [M, F] to aux_out.
//      N = 2F (virtual columns).
//   2  SwiGLU backward fused into the down projection's dX (BT, no split): the GEMM tile is dh [M, F];
//      the epilogue reads g, u from aux = gu [M, 2F] and writes dgu = [dh·u·silu'(g) | dh·silu(g)].
//      N = F.
// Both round the GEMM result to bf16 first, exactly where the unfused path stores it.
template <int BMT, int BN, bool BT, bool SPLIT, int EPI = 0>
__global__ __launch_bounds__(NT, 1) void gemm4w_k(const bf16* __restrict__ A, int lda, const bf16* __restrict__ B,
                                                  int ldb, const bf16* __restrict__ residual, void* __restrict__ out,
                                                  int M, int N, int K, int splits, const bf16* __restrict__ aux,
                                                  bf16* __restrict__ aux_out, int F, float* __restrict__ ws,
                                                  int* __restrict__ cnt) {
  static_assert(EPI == 0 || !SPLIT, "fused epilogues run on whole-K tiles");
  static_assert(EPI != 1 || !BT, "SwiGLU forward epilogue: NT only");
  static_assert(EPI != 2 || BT, "SwiGLU backward epilogue: the transposed-B dX only");
  static_assert(BMT == 256 || BMT == 128, "tile heights: 256, 128");
  constexpr int NA = BMT / 32;                 // a fragments per wave per K-half
  constexpr int NB = BN / 32;                  // b fragments per wave per K-half
  constexpr int IMG_AT = BMT * BK * 2;
  constexpr int IMG_B = BN * BK * 2;
  constexpr int STAGE = IMG_AT + IMG_B;
  constexpr int STAGES = 3 * STAGE <= 160 * 1024 ? 3 : 2;
  static_assert(BN == 128 || BN == 256 || (BN == 192 && !BT), "tile widths: 128, 256 (NT / BT), 192 (NT)");
  constexpr int KT = 2 * NA * NB;              // MFMAs per K-tile per wave
  constexpr int H = KT / 2;
  constexpr int R = NA + NB;                   // fragment-read items per K-half
  constexpr int DA = BMT / 32;                 // A DMAs per wave per K-tile
  constexpr int DB = BN / 32;                  // B DMAs per wave per K-tile
  constexpr int D = DA + DB;                   // all DMAs per wave per K-tile
  constexpr bool BIG = NA == 8;
  constexpr int K1 = R + (BIG ? 9 : 1);        // barrier 1 after this MFMA
  constexpr int K2 = KT - R - 1;               // barrier 2 after this MFMA
  constexpr int DSP = (K2 - (BIG ? 10 : 2) - (K1 + 1)) / D;   // DMA spacing
  static_assert(DSP >= 1, "schedule");
  __shared__ __attribute__((aligned(16))) char lds[STAGES * STAGE];

  const int tiles_m = (M + BMT - 1) / BMT, tiles_n = (N + BN - 1) / BN;
  const int nwg = tiles_m * tiles_n * splits;
  const int id = xcd_remap(blockIdx.x, nwg);
  const int sp = id % splits;
  const int tid = id / splits;
  const int tm = tid % tiles_m, tn = tid / tiles_m;
  const int m0 = tm * BMT, n0 = tn * BN;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const int wr = w >> 1, wc = w & 1;

  const int nk_all = K / BK;
  const int per = (nk_all + splits - 1) / splits;
  const int kt0 = sp * per;
  const int nk = max(0, min(nk_all, kt0 + per) - kt0);

  // ---- DMA sources (per-lane byte offsets; the K-tile step goes in the scalar offset)
  const rsrc_t rsa = make_rsrc(A, (uint64_t)((size_t)(M - 1) * lda + K) * 2);
  const rsrc_t rsb = BT ? make_rsrc(B, (uint64_t)((size_t)(K - 1) * ldb + N) * 2)
                        : make_rsrc(B, (uint64_t)((size_t)(N - 1) * ldb + K) * 2);
  uint32_t va[8], vb[8];   // (fixed sizes: a lambda capturing a template-sized local array drops the
                          // kernel's host-side instantiation — hipcc / clang, ROCm 7.2)
  {
    const int r8 = lane >> 3, c = (lane & 7) ^ (r8 & 6);
#pragma unroll
    for (int i = 0; i < DA; ++i) {   // A: wave w, DMA i → rows (BMT/4)·w + 8i + r8
      const int ra = min(m0 + w * (BMT / 4) + i * 8 + r8, M - 1);
      va[i] = ((uint32_t)ra * (uint32_t)lda + (uint32_t)(kt0 * BK + c * 8)) * 2u;
    }
    if constexpr (!BT) {
#pragma unroll
      for (int i = 0; i < DB; ++i) {   // B rows (BN/4)·w + 8i + r8
        int rb;
        if constexpr (EPI == 1) {   // tile row rt → gate row or up row of h-column block 16·(rt / 32)
          const int rt = w * (BN / 4) + i * 8 + r8;
          const int hr = min(tn * (BN / 2) + 16 * (rt >> 5) + (rt & 15), F - 1);
          rb = (rt & 16) ? F + hr : hr;
        } else {
          rb = min(n0 + w * (BN / 4) + i * 8 + r8, N - 1);
        }
        vb[i] = ((uint32_t)rb * (uint32_t)ldb + (uint32_t)(kt0 * BK + c * 8)) * 2u;
      }
    } else {
      constexpr int CPR = BN / 8;             // 16-B chunks per k-row (32 or 16)
      constexpr int RPD = 64 / CPR;            // k-rows per DMA (2 or 4)
#pragma unroll
      for (int i = 0; i < DB; ++i) {   // k-rows (16)·w + RPD·i + lane / CPR
        const int kr = 16 * w + RPD * i + lane / CPR;
        const int hk = (kr & 3) | ((kr >> 1) & 4);
        const int cc = (lane % CPR) ^ (2 * hk);
        vb[i] = ((uint32_t)(kt0 * BK + kr) * (uint32_t)ldb + (uint32_t)(n0 + 8 * cc)) * 2u;
      }
    }
  }
  const uint32_t b_step = BT ? (uint32_t)BK * (uint32_t)ldb * 2u : (uint32_t)(BK * 2);

  // ---- fragment read offsets
  int lo[2];
#pragma unroll
  for (int s = 0; s < 2; ++s) lo[s] = ((lane >> 3) & 1) * 1024 + 16 * slot_of(lane & 7, 4 * s + (lane >> 4));
  const int a_off = wr * NA * 2048;
  const int b_off = wc * NB * 2048;
  int boff_t[8];
  if constexpr (BT) {
    const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
    const int hk = q | ((g & 1) << 2);
#pragma unroll
    for (int j = 0; j < NB; ++j)
      boff_t[j] = (8 * g + q) * (2 * BN) + 32 * ((wc * NB + j) ^ hk) + 16 * (p >> 1) + 8 * (p & 1);
  }

  f32x4 acc[8][8];   // [NA..7][NB..7] unused for the smaller tiles
  bf16x8 fa0[8], fb0[8], fa1[8], fb1[8];

  // LDS-DMA as asm statements: hipcc then tracks no LDS-DMA and does not drain the whole queue
  // (vmcnt(0)) in front of the first ds_read_b64_tr_b16 of the next tile, which it cannot prove
  // disjoint from the in-flight stages (measured: the dX kernel waited 33 % of its cycles there).
  // Every ordering of DMA'd data is by the explicit vmcnt + barrier pairs below.
  const uint32_t lds_base = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(lds_ptr_t)lds);
  const uint32_t wa = lds_base + (uint32_t)w * (IMG_AT / 4), wb = lds_base + IMG_AT + (uint32_t)w * (IMG_B / 4);
  auto dma_a = [&](uint32_t st, int t, int q) {
    dma_lds(rsa, wa + st + q * 1024, va[q], (uint32_t)t * (BK * 2));
  };
  auto dma_b = [&](uint32_t st, int t, int q) {
    dma_lds(rsb, wb + st + q * 1024, vb[q], (uint32_t)t * b_step);
  };
  auto dma_tile = [&](uint32_t st, int t) {
#pragma unroll
    for (int q = 0; q < DA; ++q) dma_a(st, t, q);
#pragma unroll
    for (int q = 0; q < DB; ++q) dma_b(st, t, q);
  };
  // read item r of K-half s of the stage at st into (fa, fb)
  auto read_item = [&](bf16x8* fa, bf16x8* fb, const char* st, int s, int r) {
    if (sched_of<NA, NB>().rd_a[r]) {
      fa[sched_of<NA, NB>().rd_i[r]] = lds_frag(st + a_off + sched_of<NA, NB>().rd_i[r] * 2048 + lo[s]);
    } else if constexpr (BT) {
      const char* pb = st + IMG_AT + s * (32 * 2 * BN) + boff_t[sched_of<NA, NB>().rd_i[r]];
      const bf16x4 x0 = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)pb);
      const bf16x4 x1 = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(pb + 4 * 2 * BN));
      fb[sched_of<NA, NB>().rd_i[r]] = bf16x8{x0[0], x0[1], x0[2], x0[3], x1[0], x1[1], x1[2], x1[3]};
    } else {
      fb[sched_of<NA, NB>().rd_i[r]] = lds_frag(st + IMG_AT + b_off + sched_of<NA, NB>().rd_i[r] * 2048 + lo[s]);
    }
  };

  if (nk <= 0) {
#pragma unroll
    for (int i = 0; i < NA; ++i)
#pragma unroll
      for (int j = 0; j < NB; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  } else {
    // prologue: tiles 0 .. STAGES-1 (clamped: past the last tile the DMAs re-stage tile nk-1 into
    // stages nobody reads again), wait for tile 0, read its first half
#pragma unroll
    for (int s = 0; s < STAGES; ++s) dma_tile(s * STAGE, min(s, nk - 1));
    wait_vmcnt<(STAGES - 1) * D>();
    __builtin_amdgcn_s_barrier();
#pragma unroll
    for (int r = 0; r < R; ++r) read_item(fa0, fb0, lds, 0, r);

    int cur = 0;   // stage of tile t (byte offset)
    auto body = [&](auto first, int t) {
      const int tn_ = t + STAGES < nk ? t + STAGES : nk - 1;
      char* const cs = lds + cur;
      char* const ns = lds + (cur + STAGE == STAGES * STAGE ? 0 : cur + STAGE);
      Unroll<0, KT>::run([&](auto kc) {
        constexpr int k = decltype(kc)::value;
        constexpr int i = sched_of<NA, NB>().i[k % H], j = sched_of<NA, NB>().j[k % H];
        if constexpr (k < H) {
          if constexpr (decltype(first)::value) mfma_zero(acc[i][j], fb0[j], fa0[i]);
          else mfma_acc(acc[i][j], fb0[j], fa0[i]);
        } else {
          mfma_acc(acc[i][j], fb1[j], fa1[i]);
        }
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (k < R) read_item(fa1, fb1, cs, 1, k);
        if constexpr (k == K1) {
          __builtin_amdgcn_s_waitcnt(WAIT_LGKM0);
          __builtin_amdgcn_s_barrier();
        }
        if constexpr (k > K1 && (k - K1 - 1) % DSP == 0 && (k - K1 - 1) / DSP < D) {
          constexpr int d = (k - K1 - 1) / DSP;
          if constexpr (d < DA) dma_a(cur, tn_, d);
          else dma_b(cur, tn_, d - DA);
        }
        if constexpr (k == K2) {
          wait_vmcnt<(STAGES - 1) * D>();
          __builtin_amdgcn_s_barrier();
        }
        if constexpr (k > K2) read_item(fa0, fb0, ns, 0, k - K2 - 1);
        __builtin_amdgcn_sched_barrier(0);
      });
      cur = cur + STAGE == STAGES * STAGE ? 0 : cur + STAGE;
    };
    body(std::integral_constant<bool, true>{}, 0);
    for (int t = 1; t < nk; ++t) body(std::integral_constant<bool, false>{}, t);
    asm volatile("s_waitcnt vmcnt(0)\n\ts_nop 7\n\ts_nop 7" ::: "memory");
  }

  // ---- epilogue: lane holds C[m = col][n = 4·(lane>>4) + r … +3] of each 16×16 block
  if constexpr (EPI == 1) {
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      const int m = m0 + wr * (BMT / 2) + i * 16 + (lane & 15);
      if (m >= M) continue;
#pragma unroll
      for (int j = 0; j < NB; j += 2) {
        const int hc = tn * (BN / 2) + 16 * (wc * (NB / 2) + j / 2) + 4 * (lane >> 4);
        if (hc >= F) continue;
        bf16x4 g, u, h;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          g[e] = (bf16)acc[i][j][e];
          u[e] = (bf16)acc[i][j + 1][e];
          h[e] = (bf16)(silu_f((float)g[e]) * (float)u[e]);
        }
        bf16* gu = reinterpret_cast<bf16*>(out) + (size_t)m * 2 * F + hc;
        *reinterpret_cast<bf16x4*>(gu) = g;
        *reinterpret_cast<bf16x4*>(gu + F) = u;
        *reinterpret_cast<bf16x4*>(aux_out + (size_t)m * F + hc) = h;
      }
    }
    return;
  }
  if constexpr (SPLIT) {
    // Split-K, reduced in this launch by the LAST arriving split of the tile
    // (cdna_hip_programming.md §5 "Projection GEMM" item 2): every split stores its fp32 slab, drains
    // it (vmcnt(0) in every wave, barrier), and one lane releases at agent scope and takes a ticket;
    // the split that draws splits-1 acquires at agent scope, adds the other slabs to its registers and
    // runs the normal bf16 epilogue (residual included).  Correct for any placement of a tile's
    // splits over XCDs; the ticket is reset by the last arriver (zeroed once at allocation).
    float* wsf = ws;
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      const int m = m0 + wr * (BMT / 2) + i * 16 + (lane & 15);
      if (m >= M) continue;
#pragma unroll
      for (int j = 0; j < NB; ++j) {
        const int n = n0 + wc * (BN / 2) + j * 16 + 4 * (lane >> 4);
        if (n < N) *reinterpret_cast<f32x4*>(wsf + ((size_t)sp * M + m) * N + n) = acc[i][j];
      }
    }
    if (cnt == nullptr) return;                // slabs only: splitk_sum_k reduces them
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    int* flag = reinterpret_cast<int*>(lds);   // the one LDS array (free: every DMA has landed)
    if (threadIdx.x == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      const int old = __hip_atomic_fetch_add(cnt + tid, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const int last = old == splits - 1;
      if (last) {
        __hip_atomic_store(cnt + tid, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      *flag = last;
    }
    __syncthreads();
    if (*reinterpret_cast<volatile int*>(flag) == 0) return;
  }
  // Epilogues that read global memory (residual; EPI 2's g / u) issue every load of four accumulator
  // rows before the first use, from clamped (always valid) addresses — one latency per four rows, not
  // one per 16×16 block (a load behind a per-block bounds branch waits vmcnt(0) each time)
  const bool has_res = EPI == 0 && residual != nullptr;
  // rows per chunk: 4 (2 when a 256-wide tile also sums split-K slabs: register budget)
  constexpr int RC = (SPLIT && NB >= 6) ? 2 : 4;   // (NA is 4 or 8: a multiple)
  auto rows = [&](auto hh_c, auto res_c) {
    constexpr int i0 = RC * decltype(hh_c)::value;
    constexpr bool RES = decltype(res_c)::value;
    bf16x4 la[RC][8], lb[RC][8];
    f32x4 tot[RC][8];
#pragma unroll
    for (int ii = 0; ii < RC; ++ii)
#pragma unroll
      for (int j = 0; j < NB; ++j) tot[ii][j] = acc[i0 + ii][j];
#pragma unroll
    for (int ii = 0; ii < RC; ++ii) {
      const int m = min(m0 + wr * (BMT / 2) + (i0 + ii) * 16 + (lane & 15), M - 1);
#pragma unroll
      for (int j = 0; j < NB; ++j) {
        const int n = min(n0 + wc * (BN / 2) + j * 16 + 4 * (lane >> 4), N - 4);
        if constexpr (EPI == 2) {
          const bf16* gp = aux + (size_t)m * 2 * F + n;
          la[ii][j] = *reinterpret_cast<const bf16x4*>(gp);
          lb[ii][j] = *reinterpret_cast<const bf16x4*>(gp + F);
        } else if constexpr (RES) {
          la[ii][j] = *reinterpret_cast<const bf16x4*>(residual + (size_t)m * N + n);
        }
      }
    }
    if constexpr (SPLIT) {   // the last arriver adds the other splits' slabs
      for (int s2 = 0; s2 < splits; ++s2) {
        if (s2 == sp) continue;
        f32x4 pv[RC][8];
#pragma unroll
        for (int ii = 0; ii < RC; ++ii) {
          const int m = min(m0 + wr * (BMT / 2) + (i0 + ii) * 16 + (lane & 15), M - 1);
#pragma unroll
          for (int j = 0; j < NB; ++j) {
            const int n = min(n0 + wc * (BN / 2) + j * 16 + 4 * (lane >> 4), N - 4);
            pv[ii][j] = *reinterpret_cast<const f32x4*>(ws + ((size_t)s2 * M + m) * N + n);
          }
        }
#pragma unroll
        for (int ii = 0; ii < RC; ++ii)
#pragma unroll
          for (int j = 0; j < NB; ++j) tot[ii][j] += pv[ii][j];
      }
    }
#pragma unroll
    for (int ii = 0; ii < RC; ++ii) {
      const int m = m0 + wr * (BMT / 2) + (i0 + ii) * 16 + (lane & 15);
      if (m >= M) continue;
#pragma unroll
      for (int j = 0; j < NB; ++j) {
        const int n = n0 + wc * (BN / 2) + j * 16 + 4 * (lane >> 4);
        if (n >= N) continue;
        const f32x4 v = tot[ii][j];
        if constexpr (EPI == 2) {
          bf16x4 dg, du;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float d = (float)(bf16)v[e], g = (float)la[ii][j][e], uu = (float)lb[ii][j][e];
            const float sg = 1.f / (1.f + __expf(-g));
            du[e] = (bf16)(d * (g * sg));
            dg[e] = (bf16)(d * uu * (sg * (1.f + g * (1.f - sg))));
          }
          bf16* dp = reinterpret_cast<bf16*>(out) + (size_t)m * 2 * F + n;
          *reinterpret_cast<bf16x4*>(dp) = dg;
          *reinterpret_cast<bf16x4*>(dp + F) = du;
        } else {
          bf16x4 o;
#pragma unroll
          for (int e = 0; e < 4; ++e) o[e] = (bf16)(RES ? v[e] + (float)la[ii][j][e] : v[e]);
          *reinterpret_cast<bf16x4*>(reinterpret_cast<bf16*>(out) + (size_t)m * N + n) = o;
        }
      }
    }
  };
  if (has_res) {
    Unroll<0, NA / RC>::run([&](auto hc) { rows(hc, std::true_type{}); });
  } else {
    Unroll<0, NA / RC>::run([&](auto hc) { rows(hc, std::false_type{}); });
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


int tiles_of(int M, int N, int bm, int bn) { return ((M + bm - 1) / bm) * ((N + bn - 1) / bn); }

}  // namespace

// bt: B given as [K, N] (row stride ldb) instead of [N, K]
bool gemm4w_supported(int M, int N, int K, int lda, int ldb, bool bt) {
  return M > 0 && K % BK == 0 && K >= BK && N % 8 == 0 && lda % 8 == 0 && ldb % 8 == 0 &&
         (uint64_t)M * lda * 2 < 0xFFFFFFFFull &&
         (bt ? (uint64_t)K * ldb * 2 < 0xFFFFFFFFull : (uint64_t)N * ldb * 2 < 0xFFFFFFFFull);
}

// Tile (height × width) and K-splits from one cost model: (rounds of 256 workgroups) × (K-tiles per
// workgroup) × the measured in-step time of one K-tile of that tile (256 × 256: 1.5 µs,
// transposed-B 1.52, 256 × 192: 1.22, 256 × 128: 0.92; the 128-high tiles ≈ 0.56 × those) + the split-K
// reduce launch (its fp32 slabs: M·N·(8s + 2) bytes at ≈12 TB/s effective + a launch).  At M = 2048
// this picks: q|k|v fwd 256 × 192 (256 tiles); gate|up fwd / LM head 256 × 256; o fwd, the dX GEMMs to
// d_model and down dX 128 × 256; down fwd and gate|up dX 256 × 256 with 2 splits.  At M = 1024 (the
// sequential-GA micro-batches of the reference-faithful step) the 128-high tiles fill the chip without
// split-K for q|k|v, o and their dX (profiles/r3/step_timeline_faithful_bm128.txt: splitk_sum_k launches 650 → 290 per step).
// LIPA_GEMM4W_BN / LIPA_GEMM4W_BM / LIPA_GEMM4W_SPLITS force a choice.
struct G4wCfg {
  int bm, bn, splits;
};
static int env_int(const char* name) {
  const char* e = getenv(name);
  return e ? atoi(e) : 0;
}
G4wCfg gemm4w_cfg(int M, int N, int K, bool bt, int bn_req, int sp_req, int bm_req) {
  static const int forced_bn = env_int("LIPA_GEMM4W_BN"), forced_sp = env_int("LIPA_GEMM4W_SPLITS"),
                   forced_bm = env_int("LIPA_GEMM4W_BM");
  if (bn_req == 0) bn_req = forced_bn;
  if (sp_req <= 0) sp_req = forced_sp;
  if (bm_req == 0) bm_req = forced_bm;
  const int nk = K / BK;
  G4wCfg best{256, 128, 1};
  double best_t = 1e30;
  for (int bm : {256, 128}) {
    if (bm_req && bm != bm_req) continue;
    for (int bn : {256, 192, 128}) {
      if (bn == 192 && bt) continue;
      if (bn_req && bn != bn_req) continue;
      const int tiles = tiles_of(M, N, bm, bn);
      double kt_us = bn == 256 ? (bt ? 1.52 : 1.5) : bn == 192 ? 1.22 : 0.92;
      if (bm == 128) kt_us *= 0.56;
      for (int s = 1; s <= 8; s *= 2) {
        if (sp_req > 0 && s != sp_req) continue;
        if (s > 1 && sp_req <= 0 && nk / s < 8) break;
        double t = (double)((tiles * s + 255) / 256) * ((nk + s - 1) / s) * kt_us;
        if (s > 1) t += (double)M * N * (8.0 * s + 2.0) / 12e6 + 2.0;
        if (t < best_t - 1e-9) {
          best_t = t;
          best = G4wCfg{bm, bn, s};
        }
      }
    }
  }
  if (sp_req > 0) best.splits = sp_req;
  return best;
}

// bn / splits / bm: 0 = chosen by gemm4w_cfg.  Returns the split count used (the caller's fp32
// workspace must hold splits·M·N floats when it is > 1) and the tile through bn_out / bm_out.
int gemm4w_plan(int M, int N, int K, bool bt, int bn, int splits, int* bn_out, int bm, int* bm_out) {
  const G4wCfg c = gemm4w_cfg(M, N, K, bt, bn, splits, bm);
  if (bn_out) *bn_out = c.bn;
  if (bm_out) *bm_out = c.bm;
  return c.splits;
}

int gemm4w_tiles(int M, int N, int bm, int bn) { return tiles_of(M, N, bm, bn); }

// ws: splits·M·N fp32 slabs, cnt: one zero-initialised int per tile (both only when splits > 1);
// cnt == nullptr: the slabs are summed by a separate splitk_sum_k launch instead of the last arriver.
// Callers pass the (bm, bn, splits) that gemm4w_plan returned.
void launch_gemm4w(const void* A, int lda, const void* B, int ldb, const void* residual, void* out, float* ws,
                   int* cnt, int M, int N, int K, int splits, bool bt, int bn, int bm, hipStream_t st) {
  const int tiles = tiles_of(M, N, bm, bn);
  const bool split = splits > 1;
  const bf16* a = (const bf16*)A;
  const bf16* b = (const bf16*)B;
  const bf16* r = (const bf16*)residual;
  void* o = out;
  const int grid = tiles * (split ? splits : 1), sp = split ? splits : 1;
#define G4W(BM_, BN_, BT_, SP_) \
  gemm4w_k<BM_, BN_, BT_, SP_><<<grid, NT, 0, st>>>(a, lda, b, ldb, r, o, M, N, K, sp, nullptr, nullptr, 0, ws, cnt)
#define G4W_BN(BM_)                                                                \
  if (bn == 256) {                                                                 \
    if (bt) { if (split) G4W(BM_, 256, true, true); else G4W(BM_, 256, true, false); }   \
    else { if (split) G4W(BM_, 256, false, true); else G4W(BM_, 256, false, false); }    \
  } else if (bn == 192) {                                                          \
    if (split) G4W(BM_, 192, false, true); else G4W(BM_, 192, false, false);       \
  } else {                                                                         \
    if (bt) { if (split) G4W(BM_, 128, true, true); else G4W(BM_, 128, true, false); }   \
    else { if (split) G4W(BM_, 128, false, true); else G4W(BM_, 128, false, false); }    \
  }
  if (bm == 256) {
    G4W_BN(256)
  } else {
    G4W_BN(128)
  }
#undef G4W_BN
#undef G4W
  if (split && cnt == nullptr) {
    const size_t MN = (size_t)M * N;
    const int blocks = (int)std::min<size_t>((MN / 8 + 255) / 256, 2048);
    splitk_sum_k<<<blocks, 256, 0, st>>>(ws, (const bf16*)residual, (bf16*)out, MN, splits);
  }
  LIPA_CHECK_LAUNCH();
}

// gu [M, 2F] and h = silu(gate)·up [M, F] from x [M, K] and W_gu [2F, K] ([gate | up] rows), one launch
void launch_gemm4w_swiglu(const void* X, int ldx, const void* W, void* gu, void* h, int M, int F, int K, int bn,
                          int bm, hipStream_t st) {
  const int N = 2 * F;
  const int tiles = tiles_of(M, N, bm, bn);
  const bf16* a = (const bf16*)X;
  const bf16* b = (const bf16*)W;
#define G4S(BM_, BN_)                                                                                          \
  gemm4w_k<BM_, BN_, false, false, 1><<<tiles, NT, 0, st>>>(a, ldx, b, K, nullptr, gu, M, N, K, 1, nullptr,    \
                                                            (bf16*)h, F, nullptr, nullptr)
  if (bm == 256) {
    if (bn == 256) G4S(256, 256); else if (bn == 192) G4S(256, 192); else G4S(256, 128);
  } else {
    if (bn == 256) G4S(128, 256); else if (bn == 192) G4S(128, 192); else G4S(128, 128);
  }
#undef G4S
  LIPA_CHECK_LAUNCH();
}

// dgu [M, 2F] = SwiGLU-backward(dh = dY·W_down, gu) with W_down [N_w, F] used as stored, one launch
void launch_gemm4w_dswiglu(const void* DY, int lddy, const void* W, const void* gu, void* dgu, int M, int F, int Nw,
                           int bn, int bm, hipStream_t st) {
  const int tiles = tiles_of(M, F, bm, bn);
  const bf16* a = (const bf16*)DY;
  const bf16* b = (const bf16*)W;
#define G4D(BM_, BN_)                                                                                        \
  gemm4w_k<BM_, BN_, true, false, 2><<<tiles, NT, 0, st>>>(a, lddy, b, F, nullptr, dgu, M, F, Nw, 1,         \
                                                           (const bf16*)gu, nullptr, F, nullptr, nullptr)
  if (bm == 256) {
    if (bn == 256) G4D(256, 256); else G4D(256, 128);
  } else {
    if (bn == 256) G4D(128, 256); else G4D(128, 128);
  }
#undef G4D
  LIPA_CHECK_LAUNCH();
}
