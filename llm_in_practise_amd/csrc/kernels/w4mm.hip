// W4A16 GEMM for decode batches and short prefills (the AWQ / GPTQ / RTN int4 serving
// artifact of Quantization/LoRA-AWQ and Deployment/litellm-proxy/docker-compose-router-lb.yaml:85):
//     y[M, N] = x[M, K] · deq(W)ᵀ (+ residual),   M <= 64,   deq(W)[n, k] = q·s[n, g] + b[n, g]
// with W as 4-bit codes (uint8 [N, K/2], high nibble = even k) and one fp32 (scale, bias = −zero·scale)
// per (row, 128·j-deep group).
//
// At these M the cost is streaming W once (N·K/2 bytes), so the design is about bytes in flight and
// a cheap dequant, with the matrix cores doing the arithmetic:
//  * grid = (N/128 column spans) × (KS K-slices); a 256-thread workgroup owns 128 columns × 128·NKB
//    of K, each wave 32 columns (two 16-column MFMA tiles); every code (16 B per lane per tile and
//    128-deep block) and scale of the wave's whole slice is loaded up front — 4-16 KB per wave in
//    flight, the whole matrix in flight across the chip;
//  * dequant in 7 VALU per 8 weights and no conversion: a nibble q becomes the bf16 bit pattern
//    0x4300|q = 128+q by a byte permute (v_perm with a 0x43 byte plane), so the MFMA accumulates
//    G = Σ x·(128+q) per group; X = Σ x per (row, group) is reduced once while x is staged, and the
//    group folds as y += s·G + (b − 128·s)·X — scale and zero point never touch the weights;
//  * the permute yields the lane's 8 weights in k order (1,3,5,7,0,2,4,6); x is staged once per
//    workgroup into LDS (M × 128·NKB, 16-B padded rows: conflict-free ds_read_b128) in the same
//    order, so every A/B k-slot pair matches (the MFMA sum is order-free);
//  * v_mfma_f32_16x16x32_bf16 with x as A (rows = tokens, 16 per tile, RT tiles) and the codes as B;
//    the lane's B column is its load column, so its output column needs just its own (s, c) pair;
//  * KS > 1: fp32 partials [KS, M, N] + one reduce launch (the residual folds there); KS = 1 writes
//    bf16 directly.  XCD-aware block order: the column spans of one K-slice (same x slice) share an
//    L2.
#include "common.h"

using namespace lipa;

namespace {

constexpr int W4_CT = 2;                      // 16-column MFMA tiles per wave
constexpr int W4_COLS = 4 * 16 * W4_CT;       // columns per workgroup

__device__ __forceinline__ uint32_t vperm(uint32_t hi, uint32_t lo, uint32_t sel) {
  return __builtin_amdgcn_perm(hi, lo, sel);
}

// one code dword (k = 0..7; byte i = q[2i] << 4 | q[2i+1]) → four bf16 pairs of 128+q in k order
// (1,3) (5,7) (0,2) (4,6)
__device__ __forceinline__ bf16x8 i4_bf16(uint32_t w) {
  constexpr uint32_t C = 0x43434343u;
  const uint32_t lo = w & 0x0F0F0F0Fu, hi = (w >> 4) & 0x0F0F0F0Fu;
  u32x4 o;
  o[0] = vperm(C, lo, 0x04010400u);
  o[1] = vperm(C, lo, 0x04030402u);
  o[2] = vperm(C, hi, 0x04010400u);
  o[3] = vperm(C, hi, 0x04030402u);
  return __builtin_bit_cast(bf16x8, o);
}

// 8 bf16 of x in k order → the same (1,3,5,7,0,2,4,6) order
__device__ __forceinline__ u32x4 x_perm(u32x4 d) {
  u32x4 o;
  o[0] = vperm(d[1], d[0], 0x07060302u);
  o[1] = vperm(d[3], d[2], 0x07060302u);
  o[2] = vperm(d[1], d[0], 0x05040100u);
  o[3] = vperm(d[3], d[2], 0x05040100u);
  return o;
}

template <int RT, int NKB>
__global__ __launch_bounds__(256) void w4mm_k(const bf16* __restrict__ X, int ldx, const uint8_t* __restrict__ codes,
                                              const float2* __restrict__ sc, int gs, const bf16* __restrict__ residual,
                                              bf16* __restrict__ out, float* __restrict__ part, int M, int N, int K,
                                              int ncs) {
  constexpr int KR = 128 * NKB;           // K per workgroup
  constexpr int LDXS = KR + 8;            // LDS row stride (bf16): 16-B pad
  extern __shared__ __attribute__((aligned(16))) char lds_raw[];
  bf16* xs = reinterpret_cast<bf16*>(lds_raw);
  const int KS = gridDim.x / ncs;
  const int id = xcd_remap(blockIdx.x, gridDim.x);
  const int cs = id % ncs, ks = id / ncs;
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63, li = lane & 15, q = lane >> 4;
  const int k0 = ks * KR;
  const int G = K / gs;

  // 1) the wave's codes and (scale, c) pairs for the whole K slice, all in flight at once
  u32x4 cq[NKB][W4_CT];
  float2 s2[NKB][W4_CT];
  int ncol[W4_CT];
#pragma unroll
  for (int ct = 0; ct < W4_CT; ++ct) ncol[ct] = min(cs * W4_COLS + 32 * w + 16 * ct + li, N - 1);
#pragma unroll
  for (int kb = 0; kb < NKB; ++kb)
#pragma unroll
    for (int ct = 0; ct < W4_CT; ++ct) {
      const int kk = k0 + 128 * kb;
      cq[kb][ct] = *reinterpret_cast<const u32x4*>(codes + (size_t)ncol[ct] * (K / 2) + (kk + 32 * q) / 2);
      s2[kb][ct] = sc[(size_t)ncol[ct] * G + kk / gs];
    }

  // 2) x slice → LDS, permuted to the dequant's k order; rows >= M are zero.  The 16 lanes that hold one
  //    128-deep group of a row also reduce its sum Σx (xsum[kb][row], fp32) for the group fold
  constexpr int CH = KR / 8;              // 16-B chunks per row (a multiple of 16)
  constexpr int RWS = RT * 16;
  float* xsum = reinterpret_cast<float*>(lds_raw + (size_t)RWS * LDXS * 2);
  for (int c = tid; c < RWS * CH; c += 256) {
    const int r = c / CH, kc = c - r * CH;
    u32x4 v = {0u, 0u, 0u, 0u};
    if (r < M) v = *reinterpret_cast<const u32x4*>(X + (size_t)r * ldx + k0 + 8 * kc);
    const bf16x8 xb = __builtin_bit_cast(bf16x8, v);
    float t = 0.f;
#pragma unroll
    for (int e = 0; e < 8; ++e) t += (float)xb[e];
    t += __shfl_xor(t, 1, 64);
    t += __shfl_xor(t, 2, 64);
    t += __shfl_xor(t, 4, 64);
    t += __shfl_xor(t, 8, 64);
    if ((kc & 15) == 0) xsum[(kc >> 4) * RWS + r] = t;
    *reinterpret_cast<u32x4*>(xs + r * LDXS + 8 * kc) = x_perm(v);
  }
  __syncthreads();

  f32x4 acc[W4_CT][RT];
#pragma unroll
  for (int ct = 0; ct < W4_CT; ++ct)
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) acc[ct][rt] = f32x4{0.f, 0.f, 0.f, 0.f};
  const f32x4 zero = {0.f, 0.f, 0.f, 0.f};

#pragma unroll
  for (int kb = 0; kb < NKB; ++kb) {
    bf16x8 bq[W4_CT][4];
#pragma unroll
    for (int ct = 0; ct < W4_CT; ++ct)
#pragma unroll
      for (int j = 0; j < 4; ++j) bq[ct][j] = i4_bf16(cq[kb][ct][j]);
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) {
      bf16x8 xa[4];
#pragma unroll
      for (int j = 0; j < 4; ++j)
        xa[j] = *reinterpret_cast<const bf16x8*>(xs + (16 * rt + li) * LDXS + 128 * kb + 32 * q + 8 * j);
      const f32x4 ax = *reinterpret_cast<const f32x4*>(xsum + kb * RWS + 16 * rt + 4 * q);   // Σx of rows 4q..4q+3
#pragma unroll
      for (int ct = 0; ct < W4_CT; ++ct) {
        f32x4 g = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xa[0], bq[ct][0], zero, 0, 0, 0);
#pragma unroll
        for (int j = 1; j < 4; ++j) g = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xa[j], bq[ct][j], g, 0, 0, 0);
        const float s = s2[kb][ct].x, cc = s2[kb][ct].y;
#pragma unroll
        for (int i = 0; i < 4; ++i) acc[ct][rt][i] = fmaf(s, g[i], fmaf(cc, ax[i], acc[ct][rt][i]));
      }
    }
  }

  // 3) lane holds y[m = 16·rt + 4q + i][n = its load column]
#pragma unroll
  for (int ct = 0; ct < W4_CT; ++ct) {
    const int n = cs * W4_COLS + 32 * w + 16 * ct + li;
    if (n >= N) continue;
#pragma unroll
    for (int rt = 0; rt < RT; ++rt)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int m = 16 * rt + 4 * q + i;
        if (m >= M) continue;
        if (KS == 1) {
          float v = acc[ct][rt][i];
          if (residual) v += (float)residual[(size_t)m * N + n];
          out[(size_t)m * N + n] = (bf16)v;
        } else {
          part[((size_t)ks * M + m) * N + n] = acc[ct][rt][i];
        }
      }
  }
}

// out[m, n] = Σ_s part[s, m, n] (+ residual) → bf16; 2 outputs per thread and every slice's load issued
// before the adds (the grid is small at decode sizes — M·N/512 workgroups — so each thread's slice loads
// must overlap, not run as KS dependent round trips)
template <int SU>
__global__ __launch_bounds__(256) void w4mm_reduce_k(const float* __restrict__ part, const bf16* __restrict__ res,
                                                     bf16* __restrict__ out, int S, size_t MN) {
  const size_t i = ((size_t)blockIdx.x * 256 + threadIdx.x) * 2;
  if (i >= MN) return;
  float2 v = {0.f, 0.f};
  for (int s0 = 0; s0 < S; s0 += SU) {
    float2 t[SU];
#pragma unroll
    for (int u = 0; u < SU; ++u)
      t[u] = s0 + u < S ? *reinterpret_cast<const float2*>(part + (size_t)(s0 + u) * MN + i) : float2{0.f, 0.f};
#pragma unroll
    for (int u = 0; u < SU; ++u) {
      v.x += t[u].x;
      v.y += t[u].y;
    }
  }
  if (res) {
    v.x += (float)res[i];
    v.y += (float)res[i + 1];
  }
  bf16x2 o = {(bf16)v.x, (bf16)v.y};
  *reinterpret_cast<bf16x2*>(out + i) = o;
}

// ============================================================================ w4g: 32 < M <= 64
// The same dequant and group fold, tiled for decode batches: a workgroup owns BM = 16·RT rows × BN = 64·CT
// columns (4 waves × 16·CT, each wave every row) over a K slice of nkb 128-deep blocks.  x is streamed per
// block through a double-buffered LDS tile (permuted to the dequant's k order), x, the codes and (scale, c)
// pairs PD blocks ahead in a register ring — so x crosses L2→LDS once per column span (not once per K-slice × span
// as in w4mm), each code dword feeds RT MFMAs, and PD·CT·16 B per lane of codes stay in flight.  Σx per (row,
// block) for the zero-point fold is one more MFMA chain against a ones operand (no cross-lane reduction).
// Split-K (KS > 1) writes fp32 partials for w4mm_reduce_k.  Measured (profiles/r5/w4g_decode.txt): ahead of
// w4mm and gemm4w W4=2 on the Qwen3-8B projections at M = 33..64; at M = 128 / 256 gemm4w W4=2 wins (the
// per-block fold and x restaging scale with the rows), and prefetching 3 blocks instead of 2 loses.
template <int RT, int CT, int PD>
__global__ __launch_bounds__(256, 2) void w4g_k(const bf16* __restrict__ X, int ldx, const uint8_t* __restrict__ codes,
                                                const float2* __restrict__ sc, int gs, const bf16* __restrict__ residual,
                                                bf16* __restrict__ out, float* __restrict__ part, int M, int N, int K,
                                                int ncs, int nrb, int nkb) {
  constexpr int BM = 16 * RT, LDXS = 128 + 8;   // 272-B rows: the 16 rows of a ds_read_b128 group hit distinct banks
  constexpr int NR = PD + 1;                    // code ring depth
  __shared__ __attribute__((aligned(16))) bf16 xs[2][BM * LDXS];
  const int id = xcd_remap(blockIdx.x, gridDim.x);
  const int cs = id % ncs, rb = (id / ncs) % nrb, ks = id / (ncs * nrb);
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63, li = lane & 15, q = lane >> 4;
  const int m0 = rb * BM, kb0 = ks * nkb;
  const int G = K / gs;
  const uint8_t* cp[CT];
  const float2* sp[CT];
#pragma unroll
  for (int ct = 0; ct < CT; ++ct) {
    const int n = cs * (64 * CT) + 16 * CT * w + 16 * ct + li;
    cp[ct] = codes + (size_t)n * (K / 2) + 16 * q;
    sp[ct] = sc + (size_t)n * G;
  }

  u32x4 cq[NR][CT];
  float2 s2[NR][CT];
  auto load_codes = [&](int set, int kb) {
#pragma unroll
    for (int ct = 0; ct < CT; ++ct) {
      cq[set][ct] = *reinterpret_cast<const u32x4*>(cp[ct] + (size_t)kb * 64);
      s2[set][ct] = sp[ct][kb * 128 / gs];
    }
  };
  // x block: BM rows × 16 chunks of 16 B, RT chunks per thread, in the same ring as the codes
  u32x4 xr[NR][RT];
  auto load_x = [&](int set, int kb) {
#pragma unroll
    for (int p = 0; p < RT; ++p) {
      const int r = 16 * p + (tid >> 4), kc = tid & 15;
      u32x4 v = {0u, 0u, 0u, 0u};
      if (m0 + r < M) v = *reinterpret_cast<const u32x4*>(X + (size_t)(m0 + r) * ldx + kb * 128 + 8 * kc);
      xr[set][p] = v;
    }
  };
  auto store_x = [&](int set, int buf) {
#pragma unroll
    for (int p = 0; p < RT; ++p) {
      const int r = 16 * p + (tid >> 4), kc = tid & 15;
      *reinterpret_cast<u32x4*>(xs[buf] + r * LDXS + 8 * kc) = x_perm(xr[set][p]);
    }
  };

  f32x4 acc[CT][RT];
#pragma unroll
  for (int ct = 0; ct < CT; ++ct)
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) acc[ct][rt] = f32x4{0.f, 0.f, 0.f, 0.f};
  const f32x4 zero = {0.f, 0.f, 0.f, 0.f};
  bf16x8 ones;
#pragma unroll
  for (int e = 0; e < 8; ++e) ones[e] = (bf16)1.f;

  // blocks 0..PD-1 in flight; block 0's x staged
#pragma unroll
  for (int d = 0; d < PD; ++d)
    if (d < nkb) {
      load_codes(d, kb0 + d);
      load_x(d, kb0 + d);
    }
  store_x(0, 0);
  __syncthreads();
  for (int i0 = 0; i0 < nkb; i0 += NR) {
#pragma unroll
    for (int u = 0; u < NR; ++u) {   // static ring slot u = block i % NR
      const int i = i0 + u;
      if (i >= nkb) break;
      if (i + PD < nkb) {
        load_codes((u + PD) % NR, kb0 + i + PD);
        load_x((u + PD) % NR, kb0 + i + PD);
      }
      const int buf = i & 1;
      bf16x8 bq[CT][4];
#pragma unroll
      for (int ct = 0; ct < CT; ++ct)
#pragma unroll
        for (int j = 0; j < 4; ++j) bq[ct][j] = i4_bf16(cq[u][ct][j]);
#pragma unroll
      for (int rt = 0; rt < RT; ++rt) {
        bf16x8 xa[4];
#pragma unroll
        for (int j = 0; j < 4; ++j)
          xa[j] = *reinterpret_cast<const bf16x8*>(xs[buf] + (16 * rt + li) * LDXS + 32 * q + 8 * j);
        f32x4 ax = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xa[0], ones, zero, 0, 0, 0);   // Σx, rows 4q..4q+3
#pragma unroll
        for (int j = 1; j < 4; ++j) ax = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xa[j], ones, ax, 0, 0, 0);
#pragma unroll
        for (int ct = 0; ct < CT; ++ct) {
          f32x4 g = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xa[0], bq[ct][0], zero, 0, 0, 0);
#pragma unroll
          for (int j = 1; j < 4; ++j) g = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xa[j], bq[ct][j], g, 0, 0, 0);
          const float sv = s2[u][ct].x, c = s2[u][ct].y;
#pragma unroll
          for (int e = 0; e < 4; ++e) acc[ct][rt][e] = fmaf(sv, g[e], fmaf(c, ax[e], acc[ct][rt][e]));
        }
      }
      if (i + 1 < nkb) store_x((u + 1) % NR, buf ^ 1);   // block i+1 (loaded PD-1 blocks ago) into the buffer block i-1 used
      __syncthreads();
    }
  }
  // lane holds y[m = m0 + 16·rt + 4q + e][n]
#pragma unroll
  for (int ct = 0; ct < CT; ++ct)
#pragma unroll
    for (int rt = 0; rt < RT; ++rt)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int m = m0 + 16 * rt + 4 * q + e, n = cs * (64 * CT) + 16 * CT * w + 16 * ct + li;
        if (m >= M) continue;
        if (!part) {
          float v = acc[ct][rt][e];
          if (residual) v += (float)residual[(size_t)m * N + n];
          out[(size_t)m * N + n] = (bf16)v;
        } else {
          part[((size_t)ks * M + m) * N + n] = acc[ct][rt][e];
        }
      }
}

}  // namespace

bool w4g_supported(int M, int N, int K, int gs) {
  return M >= 1 && M <= 64 && N % 128 == 0 && K % 128 == 0 && gs % 128 == 0 && K % gs == 0;
}

// K slices: the fewest (halving the 128-deep blocks per workgroup, at least 2 left) that put >= 256 workgroups
// on the 256 CUs (BN = 128: 32 columns per wave; 64 per wave halves the x re-reads of wide N but spills)
int w4g_splits(int M, int N, int K) {
  const int ncs = N / 128, kb = K / 128;
  int ks = 1;
  while (ncs * ks < 256 && kb % (2 * ks) == 0 && kb / (2 * ks) >= 2) ks *= 2;
  return ks;
}

void launch_w4g(const void* X, int ldx, const uint8_t* codes, const float* sc2, int gs, const void* res, void* out,
                float* part, int M, int N, int K, int ks, hipStream_t st) {
  const int ncs = N / 128, nkb = K / 128 / ks, grid = ncs * ks;
  w4g_k<4, 2, 2><<<grid, 256, 0, st>>>((const bf16*)X, ldx, codes, (const float2*)sc2, gs,
                                       ks > 1 ? nullptr : (const bf16*)res, (bf16*)out, ks > 1 ? part : nullptr, M, N,
                                       K, ncs, 1, nkb);
  if (ks > 1) {
    const size_t MN = (size_t)M * N;
    w4mm_reduce_k<8><<<(MN / 2 + 255) / 256, 256, 0, st>>>(part, (const bf16*)res, (bf16*)out, ks, MN);
  }
  LIPA_CHECK_LAUNCH();
}

bool w4mm_supported(int M, int N, int K, int gs) {
  return M >= 1 && M <= 64 && N % W4_COLS == 0 && K % 128 == 0 && gs % 128 == 0 && K % gs == 0;
}

// 128-deep blocks per workgroup (measured per shape at M = 1..64 with the unrolled reduce,
// profiles/r4/w4a16_w4mm_reduce.txt): 4, or 2 for M <= 8 when 4 would leave fewer than 512 workgroups
// (q|k|v, o: more, shorter weight streams win there); 2 / 1 when K allows nothing larger
int w4mm_nkb(int M, int N, int K) {
  const int ncs = N / W4_COLS, kb = K / 128;
  if (kb % 4 == 0 && !(M <= 8 && ncs * (kb / 4) < 512)) return 4;
  return kb % 2 == 0 ? 2 : 1;
}

void launch_w4mm(const void* X, int ldx, const uint8_t* codes, const float* sc2, int gs, const void* res, void* out,
                 float* part, int M, int N, int K, int nkb, hipStream_t st) {
  const int ncs = N / W4_COLS, KS = K / (128 * nkb);
  const int RT = M <= 16 ? 1 : M <= 32 ? 2 : 4;
  const size_t lds = (size_t)RT * 16 * (128 * nkb + 8) * 2 + (size_t)nkb * RT * 16 * 4;
#define L(RT_, NKB_)                                                                                            \
  w4mm_k<RT_, NKB_><<<ncs * KS, 256, lds, st>>>((const bf16*)X, ldx, codes, (const float2*)sc2, gs,             \
                                                (const bf16*)res, (bf16*)out, part, M, N, K, ncs)
#define LN(RT_)                                                                                                 \
  do {                                                                                                          \
    if (nkb == 8) L(RT_, 8); else if (nkb == 4) L(RT_, 4); else if (nkb == 2) L(RT_, 2); else L(RT_, 1);       \
  } while (0)
  if (RT == 1) LN(1); else if (RT == 2) LN(2); else LN(4);
#undef LN
#undef L
  if (KS > 1) {
    const size_t MN = (size_t)M * N;
    w4mm_reduce_k<8><<<(MN / 2 + 255) / 256, 256, 0, st>>>(part, (const bf16*)res, (bf16*)out, KS, MN);
  }
  LIPA_CHECK_LAUNCH();
}
