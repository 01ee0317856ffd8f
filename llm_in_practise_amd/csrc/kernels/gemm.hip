// Weight-only GEMMs on gfx950 MFMA: the NF4 dequant-GEMM used by QLoRA
// (forward Y = X·deq(W)ᵀ and backward dX = dY·deq(W)) and the bf16 frozen-base GEMM, both
// with the LoRA low-rank product fused as an extra K-slice and the residual add fused into
// the epilogue.
//
// Design (MI355X-first, not a CUDA tiling):
//  * Output tile 128 (or 256) tokens × 128 weight-columns per 256-thread workgroup; the 4
//    waves split the 128 columns (32 each) and every wave covers ALL tile rows, so each
//    weight element is dequantised exactly once per workgroup (no dequant redundancy).
//  * Weights never touch LDS: NF4 codes are stored in a fragment-native layout (one 16-B
//    load per lane per 64-deep K-step gives the lane its four MFMA A-fragments), are
//    dequantised in registers (16-entry code table in LDS, ×absmax, v_cvt_pk_bf16_f32) and
//    fed to v_mfma_f32_16x16x32_bf16 directly.  The backward uses a second fragment-native
//    packing of the SAME codes (nibbles grouped along the output-row axis) so dX needs no
//    transpose: both layouts are permutations of the bitsandbytes codes.
//  * Activations (X / dY) are the MFMA B operand: staged HBM→LDS with global_load_lds
//    (16 B per lane, LDS-DMA, no VGPR round trip) into a double-buffered tile whose 16-B
//    chunks are XOR-swizzled through the per-lane SOURCE address (chunk ^= (row>>1)&7), which
//    makes every ds_read_b128 fragment read bank-conflict free.
//  * Operand roles are swapped (W is the A operand) so each lane's accumulator holds 4
//    consecutive output columns of one token row → 8-byte epilogue stores / residual loads.
//  * XCD-aware bijective block remap: the workgroups that share one weight column-tile run
//    on one XCD, so its L2 serves the codes to all of them.
#include "common.h"

using namespace lipa;

namespace {

constexpr int BN = 128;     // weight columns per workgroup
constexpr int BK = 64;      // reduction depth per K-step (= NF4 block size)
constexpr int NTHR = 256;

__constant__ float kNF4[16] = {
    -1.0f, -0.6961928009986877f, -0.5250730514526367f, -0.39491748809814453f,
    -0.28444138169288635f, -0.18477343022823334f, -0.09105003625154495f, 0.0f,
    0.07958029955625534f, 0.16093020141124725f, 0.24611230194568634f, 0.33791524171829224f,
    0.44070982933044434f, 0.5626170039176941f, 0.7229568362236023f, 1.0f};

typedef __attribute__((address_space(3))) void* lds_ptr_t;
typedef const __attribute__((address_space(1))) void* gbl_ptr_t;

__device__ __forceinline__ void glds16(const void* g, char* lds_wave_base) {
  __builtin_amdgcn_global_load_lds((gbl_ptr_t)g, (lds_ptr_t)lds_wave_base, 16, 0, 0);
}

__device__ __forceinline__ bf16x8 lds_read16(const char* p) { return *reinterpret_cast<const bf16x8*>(p); }

// Stage a BM×64 bf16 tile of A (row-major, leading dim lda) into an LDS image with
// XOR-swizzled 16-B chunks.  Rows >= M are clamped (their outputs are never stored).
template <int BM>
__device__ __forceinline__ void stage_a(const bf16* __restrict__ A, int lda, int m0, int M, int r0, char* buf) {
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  constexpr int PER_WAVE = BM / 32;  // 1-KB DMA instructions per wave
#pragma unroll
  for (int i = 0; i < PER_WAVE; ++i) {
    const int slot = (w * PER_WAVE + i) * 64 + lane;
    const int row = slot >> 3, q = slot & 7;
    const int c = q ^ ((row >> 1) & 7);
    int gr = m0 + row;
    gr = gr < M ? gr : M - 1;
    glds16(A + (size_t)gr * lda + r0 + c * 8, buf + (w * PER_WAVE + i) * 1024);
  }
}

__device__ __forceinline__ const char* a_frag_addr(const char* buf, int mt, int s, int lane) {
  const int r = 16 * mt + (lane & 15);
  const int c = 4 * s + (lane >> 4);
  return buf + r * 128 + ((c ^ ((r >> 1) & 7)) << 4);
}

// LUT lookup by byte offset (nibble*4) into the 16-entry fp32 code table in LDS
__device__ __forceinline__ float lut_at(const float* lut, uint32_t byte_off) {
  return *reinterpret_cast<const float*>(reinterpret_cast<const char*>(lut) + byte_off);
}
// 8 nibbles (nibble j at bits 4j) → 8 byte offsets: lo4 holds nibbles 0,2,4,6 ×4, hi4 nibbles 1,3,5,7 ×4
__device__ __forceinline__ void nib_offsets(uint32_t x, uint32_t& lo4, uint32_t& hi4) {
  lo4 = (x << 2) & 0x3C3C3C3Cu;
  hi4 = (x >> 2) & 0x3C3C3C3Cu;
}
typedef float f32x2 __attribute__((ext_vector_type(2)));
// one v_bfe_u32 (hipcc otherwise expands ubfe into shift+and: 2 VALU per nibble)
template <int OFF>
__device__ __forceinline__ uint32_t bfe8_c(uint32_t x) {
  if constexpr (OFF == 0) return x & 0xFFu;
  else if constexpr (OFF == 24) return x >> 24;
  else {
    uint32_t r;
    asm("v_bfe_u32 %0, %1, %2, 8" : "=v"(r) : "v"(x), "i"(OFF));
    return r;
  }
}
__device__ __forceinline__ uint32_t bfe8(uint32_t x, int off) {
  switch (off) {
    case 0: return bfe8_c<0>(x);
    case 8: return bfe8_c<8>(x);
    case 16: return bfe8_c<16>(x);
    default: return bfe8_c<24>(x);
  }
}
// two fp32 → packed bf16x2 in one v_cvt_pk_bf16_f32
__device__ __forceinline__ uint32_t pk2(float a, float b) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(f32x2{a, b}, bf16x2));
}
// 8 LUT values for the 8 nibbles of x: one v_bfe_u32 per element on the pre-scaled (×4)
// nibble images, then ds_read_b32 from the LDS code table
__device__ __forceinline__ void lut8(uint32_t x, const float* lut, float (&v)[8]) {
  uint32_t lo4, hi4;
  nib_offsets(x, lo4, hi4);
#pragma unroll
  for (int b = 0; b < 4; ++b) {
    v[2 * b] = lut_at(lut, bfe8(lo4, 8 * b));
    v[2 * b + 1] = lut_at(lut, bfe8(hi4, 8 * b));
  }
}
// fwd: one absmax for all 8 elements
__device__ __forceinline__ bf16x8 dequant8(uint32_t x, float sc, const float* lut) {
  float v[8];
  lut8(x, lut, v);
  u32x4 r{pk2(v[0] * sc, v[1] * sc), pk2(v[2] * sc, v[3] * sc), pk2(v[4] * sc, v[5] * sc),
          pk2(v[6] * sc, v[7] * sc)};
  return __builtin_bit_cast(bf16x8, r);
}
// bwd: nibble j has its own absmax
__device__ __forceinline__ bf16x8 dequant8v(uint32_t x, f32x4 s0, f32x4 s1, const float* lut) {
  float v[8];
  lut8(x, lut, v);
  u32x4 r{pk2(v[0] * s0[0], v[1] * s0[1]), pk2(v[2] * s0[2], v[3] * s0[3]), pk2(v[4] * s1[0], v[5] * s1[1]),
          pk2(v[6] * s1[2], v[7] * s1[3])};
  return __builtin_bit_cast(bf16x8, r);
}

// One K-step worth of a wave's packed weights: 4 code dwords + absmax (fwd: 2 scalars for
// the lane's two columns; bwd: 8 per 32-row half for the lane's 8 reduction rows).
template <bool BWD>
struct StepW;
template <>
struct StepW<false> {
  u32x4 c;
  float a0, a1;
};
template <>
struct StepW<true> {
  u32x4 c;
  f32x4 a[4];
};

template <bool BWD>
__device__ __forceinline__ void load_step(StepW<BWD>& q, const u32x4* cptr, const float* aptr, int t, int C) {
  q.c = cptr[(size_t)t * 64];
  if constexpr (!BWD) {
    q.a0 = aptr[(size_t)t * C];
    q.a1 = aptr[(size_t)t * C + 16];
  } else {
    const float* p = aptr + t * BK;
    q.a[0] = *reinterpret_cast<const f32x4*>(p);
    q.a[1] = *reinterpret_cast<const f32x4*>(p + 4);
    q.a[2] = *reinterpret_cast<const f32x4*>(p + 32);
    q.a[3] = *reinterpret_cast<const f32x4*>(p + 36);
  }
}

// half h = column half st (fwd) — both reduction substeps of one 16-column fragment pair
template <bool BWD>
__device__ __forceinline__ void dequant_half(const StepW<BWD>& q, const float* lut, bf16x8 (&wf)[2][2], int h) {
  if constexpr (!BWD) {
    const float a = h ? q.a1 : q.a0;
    wf[h][0] = dequant8(q.c[2 * h], a, lut);
    wf[h][1] = dequant8(q.c[2 * h + 1], a, lut);
  } else {
    wf[h][0] = dequant8v(q.c[2 * h], q.a[0], q.a[1], lut);
    wf[h][1] = dequant8v(q.c[2 * h + 1], q.a[2], q.a[3], lut);
  }
}

template <bool BWD>
__device__ __forceinline__ void dequant_step(const StepW<BWD>& q, const float* lut, bf16x8 (&wf)[2][2]) {
  if constexpr (!BWD) {
    wf[0][0] = dequant8(q.c[0], q.a0, lut);
    wf[0][1] = dequant8(q.c[1], q.a0, lut);
    wf[1][0] = dequant8(q.c[2], q.a1, lut);
    wf[1][1] = dequant8(q.c[3], q.a1, lut);
  } else {
    // dword (st, s): rows 32s + 8(lane>>4) + j share the lane's absmax run for half s
    wf[0][0] = dequant8v(q.c[0], q.a[0], q.a[1], lut);
    wf[0][1] = dequant8v(q.c[1], q.a[2], q.a[3], lut);
    wf[1][0] = dequant8v(q.c[2], q.a[0], q.a[1], lut);
    wf[1][1] = dequant8v(q.c[3], q.a[2], q.a[3], lut);
  }
}

// OUT[m][c] = Σ_r A[m][r] · Wop(c, r)  (+ Σ_e ext_a[m][e]·ext_b[c][e])  (+ residual[m][c])
//   fwd (BWD=false): Wop(c, r) = W[c][r], C = N, R = K ; absmax_t[(r/64)*C + c]
//   bwd (BWD=true) : Wop(c, r) = W[r][c], C = K, R = N ; absmax_t[(c/64)*R + r]
// codes: packed [C/32][R/64][64 lanes][4 dwords], dword d = st*2 + s,
//   nibble j of dword (st, s) of lane l ↔ (c = 32T + 16st + (l&15), r = 64tk + 32s + 8(l>>4) + j)
template <int MT, bool BWD>
__global__ __launch_bounds__(NTHR) void gemm_w4_k(const bf16* __restrict__ A, int lda, const uint32_t* __restrict__ codes,
                                                  const float* __restrict__ absmax_t, const bf16* __restrict__ ext_a,
                                                  const bf16* __restrict__ ext_b, int R_ext,
                                                  const bf16* __restrict__ residual, bf16* __restrict__ out, int M,
                                                  int C, int R) {
  constexpr int BM = MT * 16;
  constexpr int ABUF = BM * BK * 2;
  __shared__ __attribute__((aligned(16))) char smem[2 * ABUF + 64];
  float* lut = reinterpret_cast<float*>(smem + 2 * ABUF);
  if (threadIdx.x < 16) lut[threadIdx.x] = kNF4[threadIdx.x];

  const int tiles_m = (M + BM - 1) / BM, tiles_c = (C + BN - 1) / BN;
  const int nwg = tiles_m * tiles_c;
  const int id = xcd_remap(blockIdx.x, nwg);
  const int tm = id % tiles_m, tc = id / tiles_m;
  const int m0 = tm * BM;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int cw = tc * BN + 32 * w;  // this wave's first output column
  const bool active = cw < C;
  const int T = cw >> 5;
  const int nk = R / BK;

  f32x4 acc[2][MT];
#pragma unroll
  for (int st = 0; st < 2; ++st)
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) acc[st][mt] = f32x4{0.f, 0.f, 0.f, 0.f};

  // Software pipeline (per wave, registers): codes + absmax are loaded TWO K-steps ahead and
  // dequantised ONE step ahead, so the dequant VALU/LUT work of step t+1 overlaps the MFMAs
  // of step t and no register load is ever consumed in the iteration that issued it (the
  // end-of-iteration barrier drains the LDS-DMA and the register loads together).
  const u32x4* cptr = reinterpret_cast<const u32x4*>(codes) + ((size_t)(active ? T : 0) * nk) * 64 + lane;
  const float* aptr = BWD ? absmax_t + (size_t)((active ? cw : 0) >> 6) * R + 8 * (lane >> 4)
                          : absmax_t + (active ? cw : 0) + (lane & 15);
  StepW<BWD> q1, q2;
  if (active) {
    load_step<BWD>(q1, cptr, aptr, 0, C);
    if (nk > 1) load_step<BWD>(q2, cptr, aptr, 1, C);
  }
  stage_a<BM>(A, lda, m0, M, 0, smem);
  __syncthreads();
  bf16x8 wf[2][2];
  if (active) dequant_step<BWD>(q1, lut, wf);
  q1 = q2;

  for (int t = 0; t < nk; ++t) {
    const char* cur = smem + (t & 1) * ABUF;
    // branch-free prefetch: past the end, re-load the last step (into a buffer / registers
    // nobody reads again) so the loop body is one basic block the scheduler can interleave
    stage_a<BM>(A, lda, m0, M, min(t + 1, nk - 1) * BK, smem + ((t + 1) & 1) * ABUF);
    if (active) load_step<BWD>(q2, cptr, aptr, min(t + 2, nk - 1), C);
    if (active) {
      // MFMA over the staged activation tile (weights of step t in wf) with the dequant of
      // step t+1 interleaved: substep s=0 overlaps the column-half-0 fragments, s=1 the
      // column-half-1 fragments; activation fragments are read one substep ahead.
      bf16x8 wn[2][2];
      // activation fragments f = s*MT + mt stream through a register ring of depth RD
      constexpr int RD = MT < 8 ? MT : 8;
      bf16x8 xr[RD];
#pragma unroll
      for (int f = 0; f < RD; ++f) xr[f] = lds_read16(a_frag_addr(cur, f % MT, f / MT, lane));
#pragma unroll
      for (int f = 0; f < 2 * MT; ++f) {
        const int s = f / MT, mt = f % MT;
        if (f == 0) dequant_half<BWD>(q1, lut, wn, 0);
        if (f == MT) dequant_half<BWD>(q1, lut, wn, 1);
        const bf16x8 xf = xr[f % RD];
        if (f + RD < 2 * MT) xr[f % RD] = lds_read16(a_frag_addr(cur, (f + RD) % MT, (f + RD) / MT, lane));
        acc[0][mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[0][s], xf, acc[0][mt], 0, 0, 0);
        acc[1][mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[1][s], xf, acc[1][mt], 0, 0, 0);
      }
#pragma unroll
      for (int i = 0; i < 4 * MT; ++i) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // 1 MFMA
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // 1 DS read (LUT / next fragment)
        __builtin_amdgcn_sched_group_barrier(0x002, 2, 0);  // 2 VALU (dequant)
      }
      wf[0][0] = wn[0][0]; wf[0][1] = wn[0][1]; wf[1][0] = wn[1][0]; wf[1][1] = wn[1][1];
      q1 = q2;
    }
    __syncthreads();
  }

  if (!active) return;
  // ---- LoRA extension K-slice: ext_b[c][e] (A operand) × ext_a[m][e] (B operand)
  for (int e0 = 0; ext_a && e0 < R_ext; e0 += 32) {
    bf16x8 eb[2];
#pragma unroll
    for (int st = 0; st < 2; ++st) {
      const int c = cw + 16 * st + (lane & 15);
      eb[st] = *reinterpret_cast<const bf16x8*>(ext_b + (size_t)c * R_ext + e0 + 8 * (lane >> 4));
    }
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      int m = m0 + 16 * mt + (lane & 15);
      m = m < M ? m : M - 1;
      const bf16x8 ea = *reinterpret_cast<const bf16x8*>(ext_a + (size_t)m * R_ext + e0 + 8 * (lane >> 4));
      acc[0][mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(eb[0], ea, acc[0][mt], 0, 0, 0);
      acc[1][mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(eb[1], ea, acc[1][mt], 0, 0, 0);
    }
  }
  // ---- epilogue: lane holds out[m][c..c+3], c = cw + 16st + 4(lane>>4), m = m0 + 16mt + (lane&15)
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
    const int m = m0 + 16 * mt + (lane & 15);
    if (m >= M) continue;
#pragma unroll
    for (int st = 0; st < 2; ++st) {
      const int c = cw + 16 * st + 4 * (lane >> 4);
      f32x4 v = acc[st][mt];
      if (residual) {
        const bf16x4 rr = *reinterpret_cast<const bf16x4*>(residual + (size_t)m * C + c);
        v[0] += (float)rr[0]; v[1] += (float)rr[1]; v[2] += (float)rr[2]; v[3] += (float)rr[3];
      }
      bf16x4 o;
      o[0] = (bf16)v[0]; o[1] = (bf16)v[1]; o[2] = (bf16)v[2]; o[3] = (bf16)v[3];
      *reinterpret_cast<bf16x4*>(out + (size_t)m * C + c) = o;
    }
  }
}

// bf16 frozen base W [C, R] row-major (forward only): weight fragments straight from
// global (16 B per lane, no LDS), activations staged as above.
template <int MT>
__global__ __launch_bounds__(NTHR) void gemm_bf16w_k(const bf16* __restrict__ A, int lda, const bf16* __restrict__ W,
                                                     const bf16* __restrict__ ext_a, const bf16* __restrict__ ext_b,
                                                     int R_ext, const bf16* __restrict__ residual,
                                                     bf16* __restrict__ out, int M, int C, int R) {
  constexpr int BM = MT * 16;
  constexpr int ABUF = BM * BK * 2;
  __shared__ __attribute__((aligned(16))) char smem[2 * ABUF];
  const int tiles_m = (M + BM - 1) / BM, tiles_c = (C + BN - 1) / BN;
  const int id = xcd_remap(blockIdx.x, tiles_m * tiles_c);
  const int tm = id % tiles_m, tc = id / tiles_m;
  const int m0 = tm * BM;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int cw = tc * BN + 32 * w;
  const bool active = cw < C;
  const int nk = R / BK;
  f32x4 acc[2][MT];
#pragma unroll
  for (int st = 0; st < 2; ++st)
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) acc[st][mt] = f32x4{0.f, 0.f, 0.f, 0.f};
  const bf16* wrow0 = W + (size_t)(active ? cw + (lane & 15) : 0) * R + 8 * (lane >> 4);
  const bf16* wrow1 = wrow0 + (size_t)16 * R;
  stage_a<BM>(A, lda, m0, M, 0, smem);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int t = 0; t < nk; ++t) {
    char* cur = smem + (t & 1) * ABUF;
    if (t + 1 < nk) stage_a<BM>(A, lda, m0, M, (t + 1) * BK, smem + ((t + 1) & 1) * ABUF);
    if (active) {
      bf16x8 wf[2][2];
      wf[0][0] = *reinterpret_cast<const bf16x8*>(wrow0 + t * BK);
      wf[0][1] = *reinterpret_cast<const bf16x8*>(wrow0 + t * BK + 32);
      wf[1][0] = *reinterpret_cast<const bf16x8*>(wrow1 + t * BK);
      wf[1][1] = *reinterpret_cast<const bf16x8*>(wrow1 + t * BK + 32);
#pragma unroll
      for (int s = 0; s < 2; ++s) {
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) {
          const bf16x8 xf = lds_read16(a_frag_addr(cur, mt, s, lane));
          acc[0][mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[0][s], xf, acc[0][mt], 0, 0, 0);
          acc[1][mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[1][s], xf, acc[1][mt], 0, 0, 0);
        }
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  if (!active) return;
  for (int e0 = 0; ext_a && e0 < R_ext; e0 += 32) {
    bf16x8 eb[2];
#pragma unroll
    for (int st = 0; st < 2; ++st) {
      const int c = cw + 16 * st + (lane & 15);
      eb[st] = *reinterpret_cast<const bf16x8*>(ext_b + (size_t)c * R_ext + e0 + 8 * (lane >> 4));
    }
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      int m = m0 + 16 * mt + (lane & 15);
      m = m < M ? m : M - 1;
      const bf16x8 ea = *reinterpret_cast<const bf16x8*>(ext_a + (size_t)m * R_ext + e0 + 8 * (lane >> 4));
      acc[0][mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(eb[0], ea, acc[0][mt], 0, 0, 0);
      acc[1][mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(eb[1], ea, acc[1][mt], 0, 0, 0);
    }
  }
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
    const int m = m0 + 16 * mt + (lane & 15);
    if (m >= M) continue;
#pragma unroll
    for (int st = 0; st < 2; ++st) {
      const int c = cw + 16 * st + 4 * (lane >> 4);
      f32x4 v = acc[st][mt];
      if (residual) {
        const bf16x4 rr = *reinterpret_cast<const bf16x4*>(residual + (size_t)m * C + c);
        v[0] += (float)rr[0]; v[1] += (float)rr[1]; v[2] += (float)rr[2]; v[3] += (float)rr[3];
      }
      bf16x4 o;
      o[0] = (bf16)v[0]; o[1] = (bf16)v[1]; o[2] = (bf16)v[2]; o[3] = (bf16)v[3];
      *reinterpret_cast<bf16x4*>(out + (size_t)m * C + c) = o;
    }
  }
}

// ------------------------------------------------------------------ packing / (de)quantisation
// bnb-layout codes [N][K/2] (high nibble = even k) → fragment-native packed dwords
__global__ __launch_bounds__(256) void pack_nf4_k(const uint8_t* __restrict__ src, uint32_t* __restrict__ dst, int N,
                                                  int K, int bwd) {
  const size_t total = (size_t)N * K / 8;
  const size_t idx = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (idx >= total) return;
  const int C = bwd ? K : N, R = bwd ? N : K;
  const int d = idx & 3;
  const int lane = (idx >> 2) & 63;
  const size_t rest = idx >> 8;
  const int nk = R / 64;
  const int tk = rest % nk;
  const int T = rest / nk;
  const int st = d >> 1, s = d & 1;
  const int c = 32 * T + 16 * st + (lane & 15);
  const int rb = 64 * tk + 32 * s + 8 * (lane >> 4);
  uint32_t v = 0;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int r = rb + j;
    const int n = bwd ? r : c, k = bwd ? c : r;
    const uint8_t byte = src[(size_t)n * (K / 2) + (k >> 1)];
    const uint32_t nib = (k & 1) ? (byte & 15) : (byte >> 4);
    v |= nib << (4 * j);
  }
  dst[idx] = v;
}

// per-block absmax (row-major [N][K/64], fp32 or double-quant) → absmax_t [K/64][N] fp32
__global__ __launch_bounds__(256) void absmax_t_k(const float* __restrict__ absmax, const uint8_t* __restrict__ qabs,
                                                  const float* __restrict__ absmax2, const float* __restrict__ offset,
                                                  const float* __restrict__ dcode, float* __restrict__ out, int N,
                                                  int KB) {
  const size_t idx = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (idx >= (size_t)N * KB) return;
  const int n = idx / KB, kb = idx % KB;
  float v;
  if (absmax) v = absmax[idx];
  else {
    const size_t g = idx / 256;
    v = dcode[qabs[idx]] * absmax2[g] + offset[g];
  }
  out[(size_t)kb * N + n] = v;
}

// w [N][K] bf16 → codes [N][K/2] (bnb layout), absmax [N*K/64]; one lane per 8 elements
__global__ __launch_bounds__(256) void nf4_quantize_k(const bf16* __restrict__ w, uint8_t* __restrict__ codes,
                                                      float* __restrict__ absmax, size_t nelem) {
  const size_t v = (size_t)blockIdx.x * 256 + threadIdx.x;  // vector of 8 elements
  const bool ok = v * 8 < nelem;
  float f[8];
  if (ok) load8(w + v * 8, f);
  else
    for (int i = 0; i < 8; ++i) f[i] = 0.f;
  float m = 0.f;
#pragma unroll
  for (int i = 0; i < 8; ++i) m = fmaxf(m, fabsf(f[i]));
  // 8 lanes share a 64-element block
  m = fmaxf(m, __shfl_xor(m, 1, 64));
  m = fmaxf(m, __shfl_xor(m, 2, 64));
  m = fmaxf(m, __shfl_xor(m, 4, 64));
  m = fmaxf(m, 1e-12f);
  if (!ok) return;
  if ((threadIdx.x & 7) == 0) absmax[v / 8] = m;
  uint32_t packed = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const float x = f[i] / m;
    int q = 0;
#pragma unroll
    for (int c = 0; c < 15; ++c) q += x > 0.5f * (kNF4[c] + kNF4[c + 1]) ? 1 : 0;
    // byte layout: element 2b -> high nibble, 2b+1 -> low nibble
    packed |= (uint32_t)q << ((i & 1) ? (8 * (i >> 1)) : (8 * (i >> 1) + 4));
  }
  *reinterpret_cast<uint32_t*>(codes + v * 4) = packed;
}


// bnb-layout codes + decoded fp32 block absmax → bf16 [N][K] at HBM speed (the per-step
// dequant of the "dequant" NF4 mode, ops/linear.py): one lane per 32 elements — one 16-B code
// load, one absmax, a 256-entry LDS table of (hi, lo) nibble-value pairs, four 16-B stores
// (a wave writes 4 KB contiguous).
__global__ __launch_bounds__(256) void nf4_dequant2_k(const uint4* __restrict__ codes, const float* __restrict__ absmax,
                                                      bf16* __restrict__ w, size_t n32) {
  __shared__ float2 tab[256];
  tab[threadIdx.x] = make_float2(kNF4[threadIdx.x >> 4], kNF4[threadIdx.x & 15]);
  __syncthreads();
  const size_t g = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (g >= n32) return;
  const uint4 c = codes[g];
  const float a = absmax[g >> 1];
  const uint32_t words[4] = {c.x, c.y, c.z, c.w};
  bf16x8* dst = reinterpret_cast<bf16x8*>(w + g * 32);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    bf16x8 o;
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      const float2 t = tab[(words[j] >> (8 * b)) & 0xff];
      o[2 * b] = (bf16)(t.x * a);
      o[2 * b + 1] = (bf16)(t.y * a);
    }
    dst[j] = o;
  }
}


// variant 3: one lane per 8 elements, 4 items per lane strided by the block (every load / store
// instruction of a wave covers one contiguous range: 256 B of codes, 1 KB of bf16)
__global__ __launch_bounds__(256) void nf4_dequant3_k(const uint32_t* __restrict__ codes,
                                                      const float* __restrict__ absmax, bf16* __restrict__ w,
                                                      size_t n8) {
  __shared__ float2 tab[256];
  tab[threadIdx.x] = make_float2(kNF4[threadIdx.x >> 4], kNF4[threadIdx.x & 15]);
  __syncthreads();
  const size_t base = (size_t)blockIdx.x * 1024 + threadIdx.x;
  uint32_t c[4];
  float a[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const size_t i = base + 256 * j;
    c[j] = i < n8 ? codes[i] : 0u;
    a[j] = i < n8 ? absmax[i >> 3] : 0.f;
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const size_t i = base + 256 * j;
    if (i >= n8) break;
    bf16x8 o;
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      const float2 t = tab[(c[j] >> (8 * b)) & 0xff];
      o[2 * b] = (bf16)(t.x * a[j]);
      o[2 * b + 1] = (bf16)(t.y * a[j]);
    }
    *reinterpret_cast<bf16x8*>(w + i * 8) = o;
  }
}

// bnb-layout codes → bf16 (reference / merge path)
__global__ __launch_bounds__(256) void nf4_dequant_k(const uint8_t* __restrict__ codes, const float* __restrict__ absmax,
                                                     const uint8_t* __restrict__ qabs, const float* __restrict__ absmax2,
                                                     const float* __restrict__ offset, const float* __restrict__ dcode,
                                                     bf16* __restrict__ w, size_t nelem) {
  const size_t v = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (v * 8 >= nelem) return;
  const size_t blk = v / 8;
  const float a = absmax ? absmax[blk] : dcode[qabs[blk]] * absmax2[blk / 256] + offset[blk / 256];
  const uint32_t x = *reinterpret_cast<const uint32_t*>(codes + v * 4);
  float f[8];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const uint32_t byte = (x >> (8 * i)) & 0xff;
    f[2 * i] = kNF4[byte >> 4] * a;
    f[2 * i + 1] = kNF4[byte & 15] * a;
  }
  store8(w + v * 8, f);
}

}  // namespace

// ------------------------------------------------------------------ launchers
static inline int pick_mt(int M, int C) {
  static const int forced = [] {
    const char* e = getenv("LIPA_GEMM_MT");  // A/B experiments: 8 or 16
    return e ? atoi(e) : 0;
  }();
  if (forced == 8 || forced == 16) return forced;
  // Measured (scripts/bench_gemm.py, MI355X): the 128-row tile at 2 waves/SIMD beats the
  // 256-row tile (1 wave/SIMD at 338 registers) at every Qwen3 shape for M = 1024-2048;
  // 256-row tiles only win once there are >= 4 of them per CU.
  const long tiles256 = (long)((M + 255) / 256) * ((C + BN - 1) / BN);
  return tiles256 >= 1024 ? 16 : 8;
}

bool gemm_w4v2_supported(int M, int C, int R, int lda);
void launch_gemm_w4v2(int bwd, const void* A, int lda, const uint32_t* codes, const float* absmax_t,
                      const void* ext_a, const void* ext_b, int R_ext, const void* residual, void* out, int M, int C,
                      int R, hipStream_t st);

bool gemm_w4v3_supported(int M, int C, int R, int lda);
void launch_gemm_w4v3(int bwd, const void* A, int lda, const uint32_t* codes, const float* absmax_t,
                      const void* ext_a, const void* ext_b, int R_ext, const void* residual, void* out, int M, int C,
                      int R, hipStream_t st);

extern int g_gemm3_tab;
static int g_gemm_impl_override = 0;
// 1 = generation 1, 2 = buffer-SRD staging (default), 3 = gen 3 pair table, 4 = gen 3 with the 16-entry
// table.  Gen 3 is 7 % faster in the isolated-GEMM microbenchmark but 2-4 % SLOWER in the full
// training step on the same box (profiles/gemm_gen3_ab.txt), so generation 2 stays the default.
void set_gemm_impl(int impl) { g_gemm_impl_override = impl; }  // A/B benches in one process
static inline int gemm_impl() {
  static const int impl = [] {
    const char* e = getenv("LIPA_GEMM_IMPL");
    return e ? atoi(e) : 2;
  }();
  const int r = g_gemm_impl_override ? g_gemm_impl_override : impl;
  g_gemm3_tab = r == 4 ? 0 : 1;
  return r == 4 ? 3 : r;
}

void launch_gemm_w4(int bwd, const void* A, int lda, const uint32_t* codes, const float* absmax_t, const void* ext_a,
                    const void* ext_b, int R_ext, const void* residual, void* out, int M, int C, int R,
                    hipStream_t st) {
  if (gemm_impl() == 3 && gemm_w4v3_supported(M, C, R, lda)) {
    launch_gemm_w4v3(bwd, A, lda, codes, absmax_t, ext_a, ext_b, R_ext, residual, out, M, C, R, st);
    return;
  }
  if (gemm_impl() >= 2 && gemm_w4v2_supported(M, C, R, lda)) {
    launch_gemm_w4v2(bwd, A, lda, codes, absmax_t, ext_a, ext_b, R_ext, residual, out, M, C, R, st);
    return;
  }
  const int mt = pick_mt(M, C);
  const int BM = mt * 16;
  const int nwg = ((M + BM - 1) / BM) * ((C + BN - 1) / BN);
#define L(MT, B)                                                                                                 \
  gemm_w4_k<MT, B><<<nwg, NTHR, 0, st>>>((const bf16*)A, lda, codes, absmax_t, (const bf16*)ext_a,              \
                                         (const bf16*)ext_b, R_ext, (const bf16*)residual, (bf16*)out, M, C, R)
  if (bwd) {
    if (mt == 16) L(16, true);
    else L(8, true);
  } else {
    if (mt == 16) L(16, false);
    else L(8, false);
  }
#undef L
  LIPA_CHECK_LAUNCH();
}

void launch_gemm_int4(const void* A, int lda, const uint32_t* codes, const float* scale_t, const float* bias_t,
                      const void* ext_a, const void* ext_b, int R_ext, const void* residual, void* out, int M, int N,
                      int K, hipStream_t st);
void launch_gemm_int4_v3(const void* A, int lda, const uint32_t* codes, const float* scale_t, const float* bias_t,
                         const void* ext_a, const void* ext_b, int R_ext, const void* residual, void* out, int M, int N,
                         int K, hipStream_t st);
void launch_gemm_int4_any(const void* A, int lda, const uint32_t* codes, const float* scale_t, const float* bias_t,
                          const void* ext_a, const void* ext_b, int R_ext, const void* residual, void* out, int M, int N,
                          int K, hipStream_t st) {
  if (gemm_impl() == 3)
    launch_gemm_int4_v3(A, lda, codes, scale_t, bias_t, ext_a, ext_b, R_ext, residual, out, M, N, K, st);
  else
    launch_gemm_int4(A, lda, codes, scale_t, bias_t, ext_a, ext_b, R_ext, residual, out, M, N, K, st);
}

void launch_gemm_bf16w(const void* A, int lda, const void* W, const void* ext_a, const void* ext_b, int R_ext,
                       const void* residual, void* out, int M, int C, int R, hipStream_t st) {
  const int mt = pick_mt(M, C);
  const int BM = mt * 16;
  const int nwg = ((M + BM - 1) / BM) * ((C + BN - 1) / BN);
  if (mt == 16)
    gemm_bf16w_k<16><<<nwg, NTHR, 0, st>>>((const bf16*)A, lda, (const bf16*)W, (const bf16*)ext_a,
                                           (const bf16*)ext_b, R_ext, (const bf16*)residual, (bf16*)out, M, C, R);
  else
    gemm_bf16w_k<8><<<nwg, NTHR, 0, st>>>((const bf16*)A, lda, (const bf16*)W, (const bf16*)ext_a,
                                          (const bf16*)ext_b, R_ext, (const bf16*)residual, (bf16*)out, M, C, R);
  LIPA_CHECK_LAUNCH();
}

void launch_pack_nf4(const uint8_t* src, uint32_t* dst, int N, int K, int bwd, hipStream_t st) {
  const size_t total = (size_t)N * K / 8;
  pack_nf4_k<<<(total + 255) / 256, 256, 0, st>>>(src, dst, N, K, bwd);
  LIPA_CHECK_LAUNCH();
}

void launch_absmax_t(const float* absmax, const uint8_t* qabs, const float* absmax2, const float* offset,
                     const float* dcode, float* out, int N, int K, hipStream_t st) {
  const size_t total = (size_t)N * (K / 64);
  absmax_t_k<<<(total + 255) / 256, 256, 0, st>>>(absmax, qabs, absmax2, offset, dcode, out, N, K / 64);
  LIPA_CHECK_LAUNCH();
}

void launch_nf4_quantize(const void* w, uint8_t* codes, float* absmax, size_t nelem, hipStream_t st) {
  const size_t vecs = nelem / 8;
  nf4_quantize_k<<<(vecs + 255) / 256, 256, 0, st>>>((const bf16*)w, codes, absmax, nelem);
  LIPA_CHECK_LAUNCH();
}

static int g_dequant_variant = 3;
void set_dequant_variant(int v) { g_dequant_variant = v; }
void launch_nf4_dequant2(const uint8_t* codes, const float* absmax, void* w, size_t nelem, hipStream_t st) {
  if (g_dequant_variant == 2) {
    const size_t n32 = nelem / 32;
    nf4_dequant2_k<<<(n32 + 255) / 256, 256, 0, st>>>((const uint4*)codes, absmax, (bf16*)w, n32);
  } else {
    const size_t n8 = nelem / 8;
    nf4_dequant3_k<<<(n8 + 1023) / 1024, 256, 0, st>>>((const uint32_t*)codes, absmax, (bf16*)w, n8);
  }
  LIPA_CHECK_LAUNCH();
}

void launch_nf4_dequant(const uint8_t* codes, const float* absmax, const uint8_t* qabs, const float* absmax2,
                        const float* offset, const float* dcode, void* w, size_t nelem, hipStream_t st) {
  const size_t vecs = nelem / 8;
  nf4_dequant_k<<<(vecs + 255) / 256, 256, 0, st>>>(codes, absmax, qabs, absmax2, offset, dcode, (bf16*)w, nelem);
  LIPA_CHECK_LAUNCH();
}
