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
bool gemm_w4v2_supported(int M, int C, int R, int lda);
void launch_gemm_w4v2(int bwd, const void* A, int lda, const uint32_t* codes, const float* absmax_t,
                      const void* ext_a, const void* ext_b, int R_ext, const void* residual, void* out, int M, int C,
                      int R, hipStream_t st);

// NF4 register-dequant MFMA GEMM (gemm2.hip; the gen-1 kernel of round 1 and the gen-3 256-entry
// pair-table variant, slower end-to-end — profiles/gemm_gen3_ab.txt — are retired)
bool gemm_w4_supported(int M, int C, int R, int lda) { return gemm_w4v2_supported(M, C, R, lda); }
void launch_gemm_w4(int bwd, const void* A, int lda, const uint32_t* codes, const float* absmax_t, const void* ext_a,
                    const void* ext_b, int R_ext, const void* residual, void* out, int M, int C, int R,
                    hipStream_t st) {
  launch_gemm_w4v2(bwd, A, lda, codes, absmax_t, ext_a, ext_b, R_ext, residual, out, M, C, R, st);
}

void launch_gemm_int4(const void* A, int lda, const uint32_t* codes, const float* scale_t, const float* bias_t,
                      const void* ext_a, const void* ext_b, int R_ext, const void* residual, void* out, int M, int N,
                      int K, hipStream_t st);
void launch_gemm_int4_any(const void* A, int lda, const uint32_t* codes, const float* scale_t, const float* bias_t,
                          const void* ext_a, const void* ext_b, int R_ext, const void* residual, void* out, int M, int N,
                          int K, hipStream_t st) {
  launch_gemm_int4(A, lda, codes, scale_t, bias_t, ext_a, ext_b, R_ext, residual, out, M, N, K, st);
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
