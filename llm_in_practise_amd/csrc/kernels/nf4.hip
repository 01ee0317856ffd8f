// NF4 (bitsandbytes layout) quantisation and bf16 expansion on gfx950: the
// QLoRA load-time quantiser (bf16 → 4-bit codes + fp32 block absmax, 64-element blocks) and the
// HBM-speed expansion kernels behind the "expand" NF4 form (ops/linear.py ``_nf4_expand``: one bf16
// copy that the forward and the dX GEMM share).  The dequant-GEMM itself — NF4 codes fed straight
// into the MFMA GEMM — is csrc/kernels/gemm4w.hip (W4 = 1).
#include "common.h"

using namespace lipa;

namespace {

__constant__ float kNF4[16] = {
    -1.0f, -0.6961928009986877f, -0.5250730514526367f, -0.39491748809814453f,
    -0.28444138169288635f, -0.18477343022823334f, -0.09105003625154495f, 0.0f,
    0.07958029955625534f, 0.16093020141124725f, 0.24611230194568634f, 0.33791524171829224f,
    0.44070982933044434f, 0.5626170039176941f, 0.7229568362236023f, 1.0f};

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


// Affine int4 (GPTQ / AWQ, ``quant/int4.py``) → bf16 at HBM speed, the nf4_dequant3_k pattern: codes
// [N, K/2] (per byte: element 2i = high nibble, 2i + 1 = low), w = q·s + b per group (b = −z·s), fp32
// tables [N, K/g]; one lane per 8 elements, 4 items per lane strided by the block.  The W4A16 prefill
// path (quant/int4.py: M >= 2048) expands each weight into a transient copy for the bf16 gemm4w.
__global__ __launch_bounds__(256) void int4_dequant_k(const uint32_t* __restrict__ codes, const float* __restrict__ sc,
                                                      const float* __restrict__ bi, bf16* __restrict__ w, size_t n8,
                                                      int g8) {
  const size_t base = (size_t)blockIdx.x * 1024 + threadIdx.x;
  uint32_t c[4];
  float s[4], b[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const size_t i = base + 256 * j;
    const size_t t = i < n8 ? i / g8 : 0;
    c[j] = i < n8 ? codes[i] : 0u;
    s[j] = sc[t];
    b[j] = bi[t];
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const size_t i = base + 256 * j;
    if (i >= n8) break;
    bf16x8 o;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const uint32_t byte = (c[j] >> (8 * e)) & 0xffu;
      o[2 * e] = (bf16)fmaf((float)(byte >> 4), s[j], b[j]);
      o[2 * e + 1] = (bf16)fmaf((float)(byte & 15u), s[j], b[j]);
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


void launch_int4_dequant(const uint8_t* codes, const float* sc, const float* bi, void* w, size_t nelem, int group,
                         hipStream_t st) {
  const size_t n8 = nelem / 8;
  int4_dequant_k<<<(n8 + 1023) / 1024, 256, 0, st>>>((const uint32_t*)codes, sc, bi, (bf16*)w, n8, group / 8);
  LIPA_CHECK_LAUNCH();
}

void launch_nf4_dequant(const uint8_t* codes, const float* absmax, const uint8_t* qabs, const float* absmax2,
                        const float* offset, const float* dcode, void* w, size_t nelem, hipStream_t st) {
  const size_t vecs = nelem / 8;
  nf4_dequant_k<<<(vecs + 255) / 256, 256, 0, st>>>(codes, absmax, qabs, absmax2, offset, dcode, (bf16*)w, nelem);
  LIPA_CHECK_LAUNCH();
}
