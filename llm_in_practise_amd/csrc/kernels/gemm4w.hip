// gemm4w launchers: the plain / residual / split-K forms, the tile cost model, the NF4 g4w packing.
// The kernel (design notes) is csrc/kernels/gemm4w_kernel.h; the LoRA-epilogue launchers are in
// gemm4w_lora.hip and the fused-MLP ones in gemm4w_mlp.hip (separate translation units: parallel builds).
#include "gemm4w_kernel.h"

using namespace lipa;

namespace {

// out = Σ_s ws[s] (+ residual), 16 elements per thread with every load issued before the first add
// (10 16-B loads in flight per lane at 2 splits; default cache policy: the slabs were just written and
// mostly hit the MALL — non-temporal loads measured 20.8 vs 15 µs per call).
// SP: the split count (2 or 4), or 0 = any count up to 8 (runtime).  A tail of 8 (M·N % 16 == 8) runs
// the 8-wide path.
template <int SP>
__global__ __launch_bounds__(256) void splitk_sum_k(const float* __restrict__ ws, const bf16* __restrict__ residual,
                                                    bf16* __restrict__ out, size_t MN, int splits) {
  const size_t i = ((size_t)blockIdx.x * 256 + threadIdx.x) * 16;
  if (i >= MN) return;
  const int ns = SP ? SP : splits;
  if (i + 16 > MN) {   // the 8-element tail
    float v[8];
    load8(ws + i, v);
    for (int s = 1; s < ns; ++s) {
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
    return;
  }
  constexpr int MAXS = SP ? SP : 8;
  f32x4 v[MAXS][4];
#pragma unroll
  for (int s = 0; s < MAXS; ++s) {
    if (s >= ns) break;
#pragma unroll
    for (int q = 0; q < 4; ++q) v[s][q] = reinterpret_cast<const f32x4*>(ws + (size_t)s * MN + i)[q];
  }
  bf16x8 r0, r1;
  if (residual) {
    r0 = *reinterpret_cast<const bf16x8*>(residual + i);
    r1 = *reinterpret_cast<const bf16x8*>(residual + i + 8);
  }
  bf16x8 o0, o1;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    f32x4 t = v[0][q];
#pragma unroll
    for (int s = 1; s < MAXS; ++s)
      if (s < ns) t += v[s][q];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int j = 4 * q + e;
      float x = t[e];
      if (residual) x += (float)(j < 8 ? r0[j] : r1[j - 8]);
      if (j < 8) o0[j] = (bf16)x;
      else o1[j - 8] = (bf16)x;
    }
  }
  *reinterpret_cast<bf16x8*>(out + i) = o0;
  *reinterpret_cast<bf16x8*>(out + i + 8) = o1;
}

// bnb-layout NF4 codes [R][C/2] (element 2j in the high nibble of byte j) → the g4w layout
// [R/64][C/64][2][64][16 B]: 16 B = elements 32h … 32h+31 of one row's block; in each dword (8 elements
// 8c … 8c+7) byte j holds element j in its low nibble and element j + 4 in its high nibble
__global__ __launch_bounds__(256) void pack_g4w_k(const uint8_t* __restrict__ src, uint32_t* __restrict__ dst, int R,
                                                  int C) {
  const size_t idx = (size_t)blockIdx.x * 256 + threadIdx.x;   // one output dword
  if (idx >= (size_t)R * C / 8) return;
  const int d = idx & 3;
  const int r = (idx >> 2) & 63;
  const int h = (idx >> 8) & 1;
  const size_t blk = idx >> 9;
  const int CB = C / 64;
  const int kb = blk % CB, g = blk / CB;
  const int row = g * 64 + r, c0 = kb * 64 + 32 * h + 8 * d;
  const uint8_t* s = src + (size_t)row * (C / 2) + c0 / 2;
  uint32_t v = 0;
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const uint32_t nib = (e & 1) ? (s[e >> 1] & 15u) : (s[e >> 1] >> 4);
    v |= nib << (8 * (e & 3) + 4 * (e >> 2));
  }
  dst[idx] = v;
}

}  // namespace


// bt: B given as [K, N] (row stride ldb) instead of [N, K]; w4: B = g4w-packed NF4 codes (the shape
// of a bf16 W with ldb = its row length; rows and columns multiples of 64)
bool gemm4w_supported(int M, int N, int K, int lda, int ldb, bool bt, bool w4) {
  if (!(M > 0 && K % BK == 0 && K >= BK && N % 8 == 0 && lda % 8 == 0 && (uint64_t)M * lda * 2 < 0xFFFFFFFFull))
    return false;
  if (w4) return N % 64 == 0 && (uint64_t)N * K / 2 < 0xFFFFFFFFull;
  return ldb % 8 == 0 && (bt ? (uint64_t)K * ldb * 2 < 0xFFFFFFFFull : (uint64_t)N * ldb * 2 < 0xFFFFFFFFull);
}

// Tile (height × width) and K-splits from one cost model: (rounds of 256 workgroups) × (K-tiles per
// workgroup) × the measured in-step time of one K-tile of that tile (256 × 256: 1.5 µs,
// transposed-B 1.52, 256 × 192: 1.22, 256 × 128: 0.92; the 128-high tiles ≈ 0.56 × those; W4 tiles
// ×W4_COST, and 128-high W4 tiles — twice the expansion work per MFMA — ×W4_COST128) + the split-K
// reduce launch (its fp32 slabs: M·N·(8s + 2) bytes at ≈12 TB/s effective + a launch).  At M = 2048
// (bf16) this picks: q|k|v fwd 256 × 192 (256 tiles); gate|up fwd / LM head 256 × 256; o fwd, the dX
// GEMMs to d_model and down dX 128 × 256; down fwd and gate|up dX 256 × 256 with 2 splits.
// Callers may force bn / bm / splits through the binding arguments (the A/B scripts do); bn_req = -1 excludes
// the 192 tile (the LoRA dX kernel has no 192-wide instance).
struct G4wCfg {
  int bm, bn, splits;
};
G4wCfg gemm4w_cfg(int M, int N, int K, bool bt, int bn_req, int sp_req, int bm_req, bool w4) {
  // W4 (NF4 codes expanded in-kernel): the measured cost of a K-tile relative to bf16 per tile height
  // (profiles/r4/gemm4w_nf4_ab.txt)
  constexpr double w4_cost = 1.0, w4_cost128 = 1.35;
  const int nk = K / BK;
  G4wCfg best{256, 128, 1};
  double best_t = 1e30;
  for (int bm : {256, 128}) {
    if (bm_req && bm != bm_req) continue;
    for (int bn : {256, 192, 128}) {
      if (bn == 192 && (w4 || (bt && bm != 256))) continue;   // (instantiated: NT any height, BT 256-high)
      if (bn_req > 0 && bn != bn_req) continue;
      if (bn_req < 0 && bn == 192) continue;                    // -1: any width the caller instantiates but 192
      const int tiles = tiles_of(M, N, bm, bn);
      double kt_us = bn == 256 ? (bt ? 1.52 : 1.5) : bn == 192 ? (bt ? 1.24 : 1.22) : 0.92;
      if (bm == 128) kt_us *= 0.56;
      if (w4) kt_us *= bm == 128 ? w4_cost128 : w4_cost;
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
  if (sp_req > 0) best.splits = std::min(sp_req, 8);
  return best;
}

// bn / splits / bm: 0 = chosen by gemm4w_cfg.  Returns the split count used (the caller's fp32
// workspace must hold splits·M·N floats when it is > 1) and the tile through bn_out / bm_out.
int gemm4w_plan(int M, int N, int K, bool bt, int bn, int splits, int* bn_out, int bm, int* bm_out, bool w4) {
  const G4wCfg c = gemm4w_cfg(M, N, K, bt, bn, splits, bm, w4);
  if (bn_out) *bn_out = c.bn;
  if (bm_out) *bm_out = c.bm;
  return c.splits;
}

int gemm4w_tiles(int M, int N, int bm, int bn) { return tiles_of(M, N, bm, bn); }

// ws: splits·M·N fp32 slabs (splits > 1).  Callers pass the (bm, bn, splits) that gemm4w_plan
// returned.  bscale != nullptr: B is g4w-packed NF4 codes, bscale the transposed fp32 block absmax.
void launch_gemm4w(const void* A, int lda, const void* B, int ldb, const void* residual, void* out, float* ws,
                   const float* bscale, const float* bzero, int M, int N, int K, int splits, bool bt, int bn, int bm,
                   hipStream_t st) {
  const int tiles = tiles_of(M, N, bm, bn);
  const bool split = splits > 1;
  const bf16* a = (const bf16*)A;
  const bf16* r = (const bf16*)residual;
  void* o = out;
  const int grid = tiles * (split ? splits : 1), sp = split ? splits : 1;
#define G4W(BM_, BN_, BT_, SP_, W4_)                                                                            \
  gemm4w_k<BM_, BN_, BT_, SP_, 0, W4_><<<grid, NT, 0, st>>>(a, lda, B, ldb, r, o, M, N, K, sp, nullptr, nullptr, \
                                                             0, ws, bscale, bzero, LoraEpi{}, LoraDx{})
#define G4W_SP(BM_, BN_, BT_, W4_) \
  if (split) G4W(BM_, BN_, BT_, true, W4_); else G4W(BM_, BN_, BT_, false, W4_);
#define G4W_BN(BM_)                                                                           \
  if (bzero) {                                                                                \
    if (bn == 256) { G4W_SP(BM_, 256, false, 2) } else { G4W_SP(BM_, 128, false, 2) }         \
  } else if (bscale) {                                                                        \
    if (bn == 256) { if (bt) { G4W_SP(BM_, 256, true, 1) } else { G4W_SP(BM_, 256, false, 1) } } \
    else { if (bt) { G4W_SP(BM_, 128, true, 1) } else { G4W_SP(BM_, 128, false, 1) } }           \
  } else if (bn == 256) {                                                                     \
    if (bt) { G4W_SP(BM_, 256, true, 0) } else { G4W_SP(BM_, 256, false, 0) }                 \
  } else if (bn == 192) {                                                                     \
    if (bt) { G4W_SP(256, 192, true, 0) } else { G4W_SP(BM_, 192, false, 0) }                  \
  } else {                                                                                    \
    if (bt) { G4W_SP(BM_, 128, true, 0) } else { G4W_SP(BM_, 128, false, 0) }                 \
  }
  if (bm == 256) {
    G4W_BN(256)
  } else {
    G4W_BN(128)
  }
#undef G4W_BN
#undef G4W_SP
#undef G4W
  if (split) {
    const size_t MN = (size_t)M * N;
    const unsigned blocks = (unsigned)(((MN + 15) / 16 + 255) / 256);
    const bf16* res = (const bf16*)residual;
    if (splits == 2) splitk_sum_k<2><<<blocks, 256, 0, st>>>(ws, res, (bf16*)out, MN, 2);
    else if (splits == 4) splitk_sum_k<4><<<blocks, 256, 0, st>>>(ws, res, (bf16*)out, MN, 4);
    else splitk_sum_k<0><<<blocks, 256, 0, st>>>(ws, res, (bf16*)out, MN, splits);
  }
  LIPA_CHECK_LAUNCH();
}

void launch_pack_g4w(const uint8_t* codes, void* out, int R, int C, hipStream_t st) {
  const size_t n = (size_t)R * C / 8;
  pack_g4w_k<<<(unsigned)((n + 255) / 256), 256, 0, st>>>(codes, (uint32_t*)out, R, C);
  LIPA_CHECK_LAUNCH();
}
