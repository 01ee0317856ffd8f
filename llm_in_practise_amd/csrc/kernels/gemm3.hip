// NF4 / int4 weight GEMM, generation 3.  Same packed layouts, tiling and
// buffer-SRD staging as generation 2 (gemm2.hip); the dequantisation was rebuilt after the
// gen-2 PMC counters (profiles/): waves spent 37-45 % of their cycles parked at s_waitcnt,
// most of it on the code-table ds_read_b32 whose result the next v_mul consumed at once.
//  * pair table: 256 float2 entries indexed by a whole code BYTE (two nibbles) — one
//    ds_read_b64 per two weights instead of one ds_read_b32 per weight;
//  * byte offsets by SDWA: v_lshlrev_b32_sdwa …, 3, x src1_sel:BYTE_b extracts and scales a
//    byte in ONE VALU (gen 2: 1.5 VALU per weight for nibble extraction);
//  * the table reads for step t+1 are issued at the top of step t (16 ds_read_b64 in flight)
//    and consumed (×absmax, v_cvt_pk_bf16_f32) in the second half of step t's MFMAs, so LDS
//    latency sits under the matrix work instead of in front of a dependent v_mul.
#include "common.h"

using namespace lipa;

namespace {

constexpr int BN = 128;
constexpr int BK = 64;
constexpr int NTHR = 256;

__constant__ float kNF4v3[16] = {
    -1.0f, -0.6961928009986877f, -0.5250730514526367f, -0.39491748809814453f,
    -0.28444138169288635f, -0.18477343022823334f, -0.09105003625154495f, 0.0f,
    0.07958029955625534f, 0.16093020141124725f, 0.24611230194568634f, 0.33791524171829224f,
    0.44070982933044434f, 0.5626170039176941f, 0.7229568362236023f, 1.0f};

typedef __attribute__((address_space(3))) void* lds_ptr_t;
typedef __amdgpu_buffer_rsrc_t rsrc_t;
typedef float f32x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ rsrc_t make_rsrc(const void* base, uint64_t bytes) {
  const uint64_t p = reinterpret_cast<uint64_t>(base);
  const uint32_t lo = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(p));
  const uint32_t hi = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(p >> 32));
  const uint32_t n = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(bytes > 0xFFFFFFFFull ? 0xFFFFFFFFull : bytes));
  void* b = reinterpret_cast<void*>((static_cast<uint64_t>(hi) << 32) | lo);
  return __builtin_amdgcn_make_buffer_rsrc(b, 0, n, 0x00020000);
}

__device__ __forceinline__ float fmul(float a, float b) {
  float r;
  asm("v_mul_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
__device__ __forceinline__ uint32_t pk2(float a, float b) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(f32x2{a, b}, bf16x2));
}
// byte B of x, times 8 (a float2 table offset), in one SDWA VALU
template <int B>
__device__ __forceinline__ uint32_t boff(uint32_t x) {
  uint32_t r;
  if constexpr (B == 0)
    asm("v_lshlrev_b32_sdwa %0, 3, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_0" : "=v"(r) : "v"(x));
  else if constexpr (B == 1)
    asm("v_lshlrev_b32_sdwa %0, 3, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_1" : "=v"(r) : "v"(x));
  else if constexpr (B == 2)
    asm("v_lshlrev_b32_sdwa %0, 3, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_2" : "=v"(r) : "v"(x));
  else
    asm("v_lshlrev_b32_sdwa %0, 3, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_3" : "=v"(r) : "v"(x));
  return r;
}
// 8 nibbles (nibble j at bits 4j) → 4 table pairs {val(2b), val(2b+1)}
__device__ __forceinline__ void lut_issue(uint32_t x, const char* lut2, f32x2 (&p)[4]) {
  p[0] = *reinterpret_cast<const f32x2*>(lut2 + boff<0>(x));
  p[1] = *reinterpret_cast<const f32x2*>(lut2 + boff<1>(x));
  p[2] = *reinterpret_cast<const f32x2*>(lut2 + boff<2>(x));
  p[3] = *reinterpret_cast<const f32x2*>(lut2 + boff<3>(x));
}
// 16-entry f32 table variant (generation-2 extraction: nibble×4 via lo4/hi4 masks + bfe)
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
__device__ __forceinline__ float lut_at(const char* lut, uint32_t byte_off) {
  return *reinterpret_cast<const float*>(lut + byte_off);
}
__device__ __forceinline__ void lut_issue16(uint32_t x, const char* lut, f32x2 (&p)[4]) {
  const uint32_t lo4 = (x << 2) & 0x3C3C3C3Cu, hi4 = (x >> 2) & 0x3C3C3C3Cu;
  p[0] = f32x2{lut_at(lut, bfe8_c<0>(lo4)), lut_at(lut, bfe8_c<0>(hi4))};
  p[1] = f32x2{lut_at(lut, bfe8_c<8>(lo4)), lut_at(lut, bfe8_c<8>(hi4))};
  p[2] = f32x2{lut_at(lut, bfe8_c<16>(lo4)), lut_at(lut, bfe8_c<16>(hi4))};
  p[3] = f32x2{lut_at(lut, bfe8_c<24>(lo4)), lut_at(lut, bfe8_c<24>(hi4))};
}
__device__ __forceinline__ bf16x8 cvt8(const f32x2 (&v)[4], float sc) {
  u32x4 r{pk2(fmul(v[0][0], sc), fmul(v[0][1], sc)), pk2(fmul(v[1][0], sc), fmul(v[1][1], sc)),
          pk2(fmul(v[2][0], sc), fmul(v[2][1], sc)), pk2(fmul(v[3][0], sc), fmul(v[3][1], sc))};
  return __builtin_bit_cast(bf16x8, r);
}
__device__ __forceinline__ bf16x8 cvt8v(const f32x2 (&v)[4], f32x4 s0, f32x4 s1) {
  u32x4 r{pk2(fmul(v[0][0], s0[0]), fmul(v[0][1], s0[1])), pk2(fmul(v[1][0], s0[2]), fmul(v[1][1], s0[3])),
          pk2(fmul(v[2][0], s1[0]), fmul(v[2][1], s1[1])), pk2(fmul(v[3][0], s1[2]), fmul(v[3][1], s1[3]))};
  return __builtin_bit_cast(bf16x8, r);
}

// MODE 0: NF4 forward  (Y = X·deq(W)ᵀ, one absmax per lane column per K-step)
// MODE 1: NF4 backward (dX = dY·deq(W), one absmax per reduction row)
// MODE 2: affine int4 forward (W4A16 GPTQ/AWQ, K15): w = q·s + b with b = −z·s per (group, column)
template <int MODE>
struct StepW {
  u32x4 c;
  float a0, a1;
};
template <>
struct StepW<1> {
  u32x4 c;
  f32x4 a[4];
};
template <>
struct StepW<2> {
  u32x4 c;
  float a0, a1, b0, b1;
};

__device__ __forceinline__ float ffma(float a, float b, float c) {
  float r;
  asm("v_fma_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}
__device__ __forceinline__ bf16x8 cvt8a(const f32x2 (&v)[4], float sc, float bi) {
  u32x4 r{pk2(ffma(v[0][0], sc, bi), ffma(v[0][1], sc, bi)), pk2(ffma(v[1][0], sc, bi), ffma(v[1][1], sc, bi)),
          pk2(ffma(v[2][0], sc, bi), ffma(v[2][1], sc, bi)), pk2(ffma(v[3][0], sc, bi), ffma(v[3][1], sc, bi))};
  return __builtin_bit_cast(bf16x8, r);
}

// codes: wave's [nk][64 lanes][16 B] run; absmax/scale: fwd [K/64][C] fp32, bwd [C/64][R] fp32
template <int MODE>
__device__ __forceinline__ void load_step(StepW<MODE>& q, rsrc_t cr, uint32_t coff, rsrc_t ar, rsrc_t br,
                                          uint32_t aoff, int t, int C) {
  q.c = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(cr, coff, t * 1024, 0));
  if constexpr (MODE != 1) {
    const uint32_t so = (uint32_t)t * (uint32_t)C * 4u;
    q.a0 = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(ar, aoff, so, 0));
    q.a1 = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(ar, aoff + 64, so, 0));
    if constexpr (MODE == 2) {
      q.b0 = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(br, aoff, so, 0));
      q.b1 = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(br, aoff + 64, so, 0));
    }
  } else {
    const uint32_t so = (uint32_t)t * BK * 4u;
    q.a[0] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(ar, aoff, so, 0));
    q.a[1] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(ar, aoff + 16, so, 0));
    q.a[2] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(ar, aoff + 128, so, 0));
    q.a[3] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(ar, aoff + 144, so, 0));
  }
}

// table values of one K-step (codes in q) → bf16 fragments, scaled per MODE
template <int MODE>
__device__ __forceinline__ void convert_half(const StepW<MODE>& q, const f32x2 (&lv)[2][2][4], bf16x8 (&wf)[2][2],
                                             int h) {
  if constexpr (MODE == 0) {
    const float a = h ? q.a1 : q.a0;
    wf[h][0] = cvt8(lv[h][0], a);
    wf[h][1] = cvt8(lv[h][1], a);
  } else if constexpr (MODE == 2) {
    const float a = h ? q.a1 : q.a0, b = h ? q.b1 : q.b0;
    wf[h][0] = cvt8a(lv[h][0], a, b);
    wf[h][1] = cvt8a(lv[h][1], a, b);
  } else {
    wf[h][0] = cvt8v(lv[h][0], q.a[0], q.a[1]);
    wf[h][1] = cvt8v(lv[h][1], q.a[2], q.a[3]);
  }
}
template <int MODE, int TAB>
__device__ __forceinline__ void lut_step(const StepW<MODE>& q, const char* lut2, f32x2 (&lv)[2][2][4]) {
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      if constexpr (TAB) lut_issue(q.c[2 * h + s], lut2, lv[h][s]);
      else lut_issue16(q.c[2 * h + s], lut2, lv[h][s]);
    }
}

__device__ __forceinline__ const char* a_frag_addr(const char* buf, int mt, int s, int lane) {
  const int r = 16 * mt + (lane & 15);
  const int c = 4 * s + (lane >> 4);
  return buf + r * 128 + ((c ^ ((r >> 1) & 7)) << 4);
}

// Stage the 256×64 activation tile: 32 LDS-DMA instructions (1 KB each) per workgroup, 8 per
// wave.  voff[i] is the lane's precomputed source byte offset (row clamp + chunk swizzle), the
// K-step advance is the scalar soffset.
// (not a template: hipcc rejects __amdgpu_buffer_rsrc_t in a deduced template signature; pw is
// a literal at every call site, so the loop still unrolls after inlining)
__device__ __forceinline__ void stage_a(rsrc_t ar, const uint32_t* voff, int pw, uint32_t soff, char* wave_dst) {
#pragma unroll
  for (int i = 0; i < pw; ++i)
    __builtin_amdgcn_raw_ptr_buffer_load_lds(ar, (lds_ptr_t)(wave_dst + i * 1024), 16, voff[i], soff, 0, 0);
}

template <int MT, int MODE, int TAB>
__global__ __launch_bounds__(NTHR, 2) void gemm_w4v3_k(const bf16* __restrict__ A, int lda,
                                                      const uint32_t* __restrict__ codes,
                                                      const float* __restrict__ absmax_t,
                                                      const float* __restrict__ bias_t,
                                                      const bf16* __restrict__ ext_a, const bf16* __restrict__ ext_b,
                                                      int R_ext, const bf16* __restrict__ residual,
                                                      bf16* __restrict__ out, int M, int C, int R) {
  // one LDS array (a second __shared__ object can make hipcc drain vmcnt before ds_reads):
  // [0, 64) NF4 code table — at offset 0 so every LUT ds_read is "base-free" (immediate
  // offsets are 16-bit), then the two 32 KB activation buffers
  constexpr int BM = MT * 16;
  constexpr int ABUF = BM * BK * 2;  // 32 KB (MT 16) / 16 KB (MT 8)
  constexpr int PW = BM / 32;        // 1-KB LDS-DMA instructions per wave per K-step
  __shared__ __attribute__((aligned(16))) char lds[2048 + 2 * ABUF];
  const char* lut2 = lds;  // 256 × float2 pair table at LDS offset 0
  char* smem = lds + 2048;
  constexpr bool BWD = MODE == 1;
  if constexpr (TAB) {
    const uint32_t v = threadIdx.x;  // NTHR == 256: one entry per thread
    const float lo = MODE == 2 ? (float)(v & 15) : kNF4v3[v & 15];
    const float hi = MODE == 2 ? (float)(v >> 4) : kNF4v3[v >> 4];
    reinterpret_cast<f32x2*>(lds)[v] = f32x2{lo, hi};
  } else if (threadIdx.x < 16) {
    reinterpret_cast<float*>(lds)[threadIdx.x] = MODE == 2 ? (float)threadIdx.x : kNF4v3[threadIdx.x];
  }

  const int tiles_m = (M + BM - 1) / BM, tiles_c = (C + BN - 1) / BN;
  const int nwg = tiles_m * tiles_c;
  const int id = xcd_remap(blockIdx.x, nwg);
  const int tm = id % tiles_m, tc = id / tiles_m;
  const int m0 = tm * BM;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int wu = __builtin_amdgcn_readfirstlane(w);
  const int cw = tc * BN + 32 * wu;
  const bool active = cw < C;
  const int T = cw >> 5;
  const int nk = R / BK;

  // ---- descriptors (wave-uniform) and per-lane offsets (computed once)
  const rsrc_t a_rs = make_rsrc(A, (uint64_t)M * lda * 2);
  const rsrc_t c_rs = make_rsrc(codes, (uint64_t)C * R / 2);
  const rsrc_t s_rs = make_rsrc(absmax_t, (uint64_t)C * R / 64 * 4);
  const rsrc_t b_rs = make_rsrc(MODE == 2 ? bias_t : absmax_t, (uint64_t)C * R / 64 * 4);
  uint32_t voff[PW];
#pragma unroll
  for (int i = 0; i < PW; ++i) {
    const int slot = (wu * PW + i) * 64 + lane;
    const int row = slot >> 3, q = slot & 7;
    const int c = q ^ ((row >> 1) & 7);
    int gr = m0 + row;
    gr = gr < M ? gr : M - 1;
    voff[i] = (uint32_t)gr * (uint32_t)lda * 2u + (uint32_t)c * 16u;
  }
  char* wave_dst0 = smem + wu * PW * 1024;
  const int Ts = active ? T : 0;
  const uint32_t coff = ((uint32_t)Ts * (uint32_t)nk * 64u + lane) * 16u;
  const int cws = active ? cw : 0;
  const uint32_t aoff = BWD ? ((uint32_t)(cws >> 6) * (uint32_t)R + 8u * (lane >> 4)) * 4u
                            : (uint32_t)(cws + (lane & 15)) * 4u;

  f32x4 acc[2][MT];
#pragma unroll
  for (int st = 0; st < 2; ++st)
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) acc[st][mt] = f32x4{0.f, 0.f, 0.f, 0.f};

  StepW<MODE> q1, q2;
  load_step<MODE>(q1, c_rs, coff, s_rs, b_rs, aoff, 0, C);
  load_step<MODE>(q2, c_rs, coff, s_rs, b_rs, aoff, nk > 1 ? 1 : 0, C);
  stage_a(a_rs, voff, PW, 0, wave_dst0);
  __syncthreads();
  bf16x8 wf[2][2];
  f32x2 lv[2][2][4];
  lut_step<MODE, TAB>(q1, lut2, lv);
  convert_half<MODE>(q1, lv, wf, 0);
  convert_half<MODE>(q1, lv, wf, 1);
  q1 = q2;

  constexpr int RD = BWD ? 4 : (MT < 8 ? MT : 6);  // fragment read-ahead ring (the table values take 32 VGPRs)
  for (int t = 0; t < nk; ++t) {
    const char* cur = smem + (t & 1) * ABUF;
    const int tn = t + 1 < nk ? t + 1 : nk - 1;
    stage_a(a_rs, voff, PW, (uint32_t)tn * BK * 2u, wave_dst0 + ((t + 1) & 1) * ABUF);
    lut_step<MODE, TAB>(q1, lut2, lv);  // table reads for step t+1, consumed in the second half
    load_step<MODE>(q2, c_rs, coff, s_rs, b_rs, aoff, t + 2 < nk ? t + 2 : nk - 1, C);
    bf16x8 wn[2][2];
    bf16x8 xr[RD];
#pragma unroll
    for (int f = 0; f < RD; ++f) xr[f] = *reinterpret_cast<const bf16x8*>(a_frag_addr(cur, f % MT, f / MT, lane));
#pragma unroll
    for (int f = 0; f < 2 * MT; ++f) {
      const int s = f / MT, mt = f % MT;
      if (f == MT) {
        convert_half<MODE>(q1, lv, wn, 0);
        convert_half<MODE>(q1, lv, wn, 1);
      }
      const bf16x8 xf = xr[f % RD];
      if (f + RD < 2 * MT)
        xr[f % RD] = *reinterpret_cast<const bf16x8*>(a_frag_addr(cur, (f + RD) % MT, (f + RD) / MT, lane));
      acc[0][mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[0][s], xf, acc[0][mt], 0, 0, 0);
      acc[1][mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[1][s], xf, acc[1][mt], 0, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < 2 * MT; ++i) {  // first half: MFMAs beside the table / fragment reads
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // 1 MFMA
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // 1 DS read
      __builtin_amdgcn_sched_group_barrier(0x002, 1, 0);  // 1 VALU
    }
#pragma unroll
    for (int i = 0; i < 2 * MT; ++i) {  // second half: MFMAs beside the ×absmax / cvt VALU
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x002, 2, 0);
    }
    wf[0][0] = wn[0][0]; wf[0][1] = wn[0][1]; wf[1][0] = wn[1][0]; wf[1][1] = wn[1][1];
    q1 = q2;
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

}  // namespace

bool gemm_w4v3_supported(int M, int C, int R, int lda) {
  // 32-bit buffer offsets; every K-step a whole NF4 block
  return (uint64_t)M * lda * 2 < 0xFFFFFFFFull && (uint64_t)C * R / 2 < 0xFFFFFFFFull && R % BK == 0 && C % 32 == 0;
}

// 256-row tiles need >= 2 workgroups per CU (their occupancy) to pay; otherwise 128-row tiles
// (twice the workgroups, 1 dequantised value per MFMA).  LIPA_GEMM_MT=8|16 forces one.
static int pick_mt_v3(int M, int C) {
  static const int forced = [] {
    const char* e = getenv("LIPA_GEMM_MT");
    return e ? atoi(e) : 0;
  }();
  if (forced == 8 || forced == 16) return forced;
  const long tiles256 = (long)((M + 255) / 256) * ((C + BN - 1) / BN);
  return tiles256 >= 512 ? 16 : 8;
}

int g_gemm3_tab = 1;  // 1: 256-entry pair table, 0: 16-entry table (A/B knob)

void launch_gemm_w4v3(int bwd, const void* A, int lda, const uint32_t* codes, const float* absmax_t,
                      const void* ext_a, const void* ext_b, int R_ext, const void* residual, void* out, int M, int C,
                      int R, hipStream_t st) {
  const int mt = pick_mt_v3(M, C);
  const int BM = mt * 16;
  const int nwg = ((M + BM - 1) / BM) * ((C + BN - 1) / BN);
#define L(MT_, MODE_, TAB_)                                                                                    \
  gemm_w4v3_k<MT_, MODE_, TAB_><<<nwg, NTHR, 0, st>>>((const bf16*)A, lda, codes, absmax_t, nullptr,          \
                                                      (const bf16*)ext_a, (const bf16*)ext_b, R_ext,          \
                                                      (const bf16*)residual, (bf16*)out, M, C, R)
#define L2(MT_, MODE_)      \
  if (g_gemm3_tab)          \
    L(MT_, MODE_, 1);       \
  else                      \
    L(MT_, MODE_, 0)
  if (bwd) {
    if (mt == 16) { L2(16, 1); }
    else { L2(8, 1); }
  } else {
    if (mt == 16) { L2(16, 0); }
    else { L2(8, 0); }
  }
#undef L2
#undef L
  LIPA_CHECK_LAUNCH();
}

// W4A16 affine int4 forward (GPTQ / AWQ / compressed-tensors weights repacked at load time):
// codes in the NF4 fragment-native forward packing, scale_t/bias_t fp32 [K/64][N] (group 128 →
// each value repeated for the group's two 64-deep K-steps), w = q·scale + bias.
void launch_gemm_int4_v3(const void* A, int lda, const uint32_t* codes, const float* scale_t, const float* bias_t,
                      const void* ext_a, const void* ext_b, int R_ext, const void* residual, void* out, int M, int N,
                      int K, hipStream_t st) {
  const int mt = pick_mt_v3(M, N);
  const int BM = mt * 16;
  const int nwg = ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
  if (mt == 16)
    gemm_w4v3_k<16, 2, 1><<<nwg, NTHR, 0, st>>>((const bf16*)A, lda, codes, scale_t, bias_t, (const bf16*)ext_a,
                                             (const bf16*)ext_b, R_ext, (const bf16*)residual, (bf16*)out, M, N, K);
  else
    gemm_w4v3_k<8, 2, 1><<<nwg, NTHR, 0, st>>>((const bf16*)A, lda, codes, scale_t, bias_t, (const bf16*)ext_a,
                                            (const bf16*)ext_b, R_ext, (const bf16*)residual, (bf16*)out, M, N, K);
  LIPA_CHECK_LAUNCH();
}
