// Flash attention forward / backward for gfx950: causal, GQA by head
// broadcast (K/V never repeated), right-padding via per-batch kv length, query offsets (chunked /
// prefix-cache prefill), attention dropout, bf16 I/O, fp32 online softmax.  Token-major layout:
// q [T, Hq*D], k/v [T, Hkv*D] with arbitrary row stride (k/v may be strided views into the fused
// qkv projection output).  One kernel per (head dim class, pass):
//
//  * D = 128 (every Qwen / Llama shape): v_mfma_f32_32x32x16_bf16 kernels whose K / V (forward, dQ)
//    and Q / dO (dK/dV) tiles arrive by LDS-DMA (buffer_load … lds, the swizzle applied on the global
//    side) into double-buffered XOR-addressed LDS images, one barrier per tile:
//      attn_fwd128_k     Sᵀ = K·Qᵀ (each lane owns one query: lane-local softmax), Oᵀ += Vᵀ·Pᵀ;
//      attn_bwd_dq128_k  dQ, and delta = rowsum(dO∘O) for the dK/dV kernel;
//      attn_bwd_dkv128_k 8 waves, K / V images resident, dKᵀ / dVᵀ accumulated in registers over
//                        the query sweep (no atomics); key blocks split over two workgroups when the
//                        causal grid is too small for the chip (attn_dkv_nsplit + attn_dkv_fin_k).
//    Row strides must be multiples of 128 elements (256-B DMA rows; the binding checks).
//  * D = 32 / 64 / 96: the 16x16x32 kernels attn_fwd_k / attn_bwd_dq_k / attn_bwd_dkv_k (register-staged
//    tiles; GQA partial dK/dV per q-head summed in a deterministic finalize pass).

#include "common.h"

using namespace lipa;

namespace {

typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4;

__device__ __forceinline__ bf16x4 tr_read(const bf16* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(p));
}
__device__ __forceinline__ bf16x8 cat8(bf16x4 a, bf16x4 b) {
  return bf16x8{a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
}
__device__ __forceinline__ bf16x8 f2b8(f32x4 a, f32x4 b) {
  return bf16x8{(bf16)a[0], (bf16)a[1], (bf16)a[2], (bf16)a[3], (bf16)b[0], (bf16)b[1], (bf16)b[2], (bf16)b[3]};
}

constexpr float LOG2E = 1.4426950408889634f;

// raw v_exp_f32 (no denormal range reduction: the arguments here are <= 0 and a flushed tiny
// probability is harmless)
__device__ __forceinline__ float fexp2(float x) { return __builtin_amdgcn_exp2f(x); }

// Attention-probability dropout (the teaching models' nn.MultiheadAttention(dropout=p)): a
// counter-based keep bit per (batch·head, query, key), regenerated identically by the forward and
// both backward kernels, never stored.  keep ⇔ hash ≥ thresh (thresh = p·2³²); kept P is scaled by
// rinv = 1/(1-p).  The row normaliser l and the backward's delta = rowsum(dO∘O) use the
// un-dropped P, as in FlashAttention-2.
__device__ __forceinline__ uint32_t drop_hash(uint32_t s0, uint32_t s1, uint32_t bh, uint32_t q, uint32_t k) {
  uint32_t x = s0 ^ (bh * 0x9E3779B9u);
  x ^= q * 0x85EBCA6Bu + s1;
  x ^= k * 0xC2B2AE35u;
  x ^= x >> 16;
  x *= 0x7FEB352Du;
  x ^= x >> 15;
  x *= 0x846CA68Bu;
  x ^= x >> 16;
  return x;
}

struct DropParams {
  uint32_t s0, s1, thresh;  // thresh == 0: no dropout
  float rinv;
};

// Grid (n0, n1, n2) → logical block (i0, i1, i2) with consecutive logical blocks (i0 fastest)
// on the same XCD, so the blocks that re-read one (batch, kv-head)'s K/V (or Q/dO) share its L2.
__device__ __forceinline__ void xcd_grid3(int& i0, int& i1, int& i2) {
  const int n0 = gridDim.x, n1 = gridDim.y;
  const int nwg = n0 * n1 * gridDim.z;
  const int id = xcd_remap(blockIdx.x + n0 * (blockIdx.y + n1 * blockIdx.z), nwg);
  i0 = id % n0;
  i1 = (id / n0) % n1;
  i2 = id / (n0 * n1);
}

// Causal grids (i0 = query block, work grows with it): the same XCD grouping, but inside each run of
// n0·G consecutive logical blocks (G (head, batch) pairs — one XCD's share at the training shapes)
// the block index varies SLOWEST, so every XCD dispatches all its heavy blocks before any light one
// (longest-first: the light blocks then fill the slots the heavy ones leave).  lpt = 0: the
// plain xcd_grid3 order.
__device__ __forceinline__ void xcd_grid3_lpt(int& i0, int& i1, int& i2, int lpt) {
  if (!lpt) {
    xcd_grid3(i0, i1, i2);
    return;
  }
  const int n0 = gridDim.x, n1 = gridDim.y;
  const int npair = n1 * gridDim.z;
  const int nwg = n0 * npair;
  const int id = xcd_remap(blockIdx.x + n0 * (blockIdx.y + n1 * blockIdx.z), nwg);
  // pairs per run = one XCD's share of the grid (xcd_remap gives XCD x the contiguous logical range
  // [x·nwg/8, (x+1)·nwg/8)), so every XCD holds the whole heavy-to-light range of its pairs: a run
  // spanning two XCDs hands one of them only heavy blocks (the 128-query forward at [4, 512, 32, 8]:
  // 448 vs 192 tile-sweeps per XCD)
  const int G = max(1, min(npair, (nwg / 8) / n0));
  const int run = id / (n0 * G), t = id % (n0 * G);
  const int g = min(G, npair - run * G);       // the last run may hold fewer pairs
  i0 = t / g;
  if (lpt == 1 && nwg <= 8 * 64) {
    // the whole grid is resident at once (2 workgroups per CU): the first 32 of an XCD's blocks take
    // one slot of each CU, the next 32 the other, so a snake order (heavy half descending, light half
    // ascending) gives every CU one heavy + one light block instead of two of the heaviest
    const int m = (n0 + 1) / 2;
    i0 = i0 < m ? i0 : n0 - 1 - (i0 - m);
  }
  const int pr = run * G + t % g;
  i1 = pr % n1;
  i2 = pr / n1;
}

// 1: longest-first (+ snake when the grid is resident) — measured best against the plain XCD-grouped
// order (0) and longest-first only (2), profiles/r4/attention_knobs_ab.txt
static int attn_lpt() { return 1; }


// ============================================================================ forward
// Sq queries per batch row attend to Skv keys (K/V rows of batch b start at b·kv_rows: a KV cache
// may be allocated longer than it is filled).  Query i of batch b sits at absolute position
// q_offs[b] + i (0 without q_offs): chunked / prefix-cache suffix prefill is the same kernel with
// the causal limit key ≤ q_off + i.  kv_lens[b] (optional) masks keys ≥ kv_lens[b] (right padding,
// BERT key-padding masks, the filled part of a cache).
template <int D, int PF, int QT>
__global__ __launch_bounds__(256, 2) void attn_fwd_k(const bf16* __restrict__ Q, const bf16* __restrict__ K,
                                                  const bf16* __restrict__ V, int ldq, int ldk, int ldv,
                                                  const int* __restrict__ kv_lens, const int* __restrict__ q_offs,
                                                  bf16* __restrict__ O, float* __restrict__ lse, int Sq, int Skv,
                                                  int kv_rows, int hq, int hkv, int causal, float scale_log2,
                                                  DropParams dp) {
  // padded LDS row (elements): a 288-B row stride (D = 128; D + 16 for every D) makes both fragment reads
  // bank-conflict free — ds_read_b128 of rows 16t + li at column 32s + 8g, and ds_read_b64_tr_b16 of rows
  // 4g + li/4 (+16) at column 16dt + 4(li%4) (the D + 8 stride was 2-way on both: 41 % of the LDS cycles
  // of the backward were conflict cycles, profiles/r4/pmc_step_kernels.txt)
  constexpr int LDR = D + 16;
  constexpr int CH = D / 8;         // 16-B chunks per row
  constexpr int TILE = 64 * LDR;    // elements per K or V tile
  constexpr int NS = D / 32;        // k-steps over head dim
  constexpr int ND = D / 16;        // d-subtiles of O
  constexpr int LOADS = 64 * CH / 256;
  __shared__ __attribute__((aligned(16))) bf16 smem[4 * TILE];  // K0 V0 K1 V1

  constexpr int QB = 64 * QT;       // queries per workgroup (QT 16-query subtiles per wave)
  const int nqb = (Sq + QB - 1) / QB;
  int i0, h, b;
  xcd_grid3_lpt(i0, h, b, causal >> 1);   // causal bit 1: longest-first order
  const int qb = nqb - 1 - i0;  // heavy (late, causal) blocks first
  const int hk = h / (hq / hkv);
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, g = lane >> 4, li = lane & 15;
  const int q0 = qb * QB + 16 * QT * w;
  const int qoff = q_offs ? q_offs[b] : 0;
  const int kvlen = min(kv_lens ? kv_lens[b] : Skv, Skv);
  const size_t tok0 = (size_t)b * Sq;          // query / output rows
  const size_t ktok0 = (size_t)b * kv_rows;     // key / value rows

  // Q fragments (B operand of Sᵀ = K·Qᵀ): Q[q0 + 16qt + li][32s + 8g + j]
  bf16x8 qf[QT][NS];
#pragma unroll
  for (int qt = 0; qt < QT; ++qt) {
    int q = q0 + 16 * qt + li;
    q = q < Sq ? q : Sq - 1;
#pragma unroll
    for (int s = 0; s < NS; ++s)
      qf[qt][s] = *reinterpret_cast<const bf16x8*>(Q + (tok0 + q) * ldq + h * D + 32 * s + 8 * g);
  }

  int kend = causal ? min(Skv, qoff + qb * QB + QB) : Skv;
  kend = min(kend, kvlen);
  const int nt = (kend + 63) / 64;

  f32x4 acc[ND][QT];
  float m_run[QT], l_run[QT];
#pragma unroll
  for (int qt = 0; qt < QT; ++qt) {
#pragma unroll
    for (int dt = 0; dt < ND; ++dt) acc[dt][qt] = f32x4{0.f, 0.f, 0.f, 0.f};
    m_run[qt] = -INFINITY;
    l_run[qt] = 0.f;
  }

  // K/V tiles are register-staged PF tiles ahead (PF register sets, the loop unrolled by 2 so
  // each set is static): with PF = 2 a tile's global loads get two tile-computations of latency
  // budget before their LDS store.
  bf16x8 kr[PF][LOADS], vr[PF][LOADS];
  auto load_tile = [&](int set, int t) {
#pragma unroll
    for (int p = 0; p < LOADS; ++p) {
      const int ci = p * 256 + threadIdx.x;
      const int row = ci / CH, ch = ci % CH;
      int key = t * 64 + row;
      key = key < Skv ? key : Skv - 1;
      kr[set][p] = *reinterpret_cast<const bf16x8*>(K + (ktok0 + key) * ldk + hk * D + ch * 8);
      vr[set][p] = *reinterpret_cast<const bf16x8*>(V + (ktok0 + key) * ldv + hk * D + ch * 8);
    }
  };
  auto store_tile = [&](int set, int buf) {
    bf16* Kl = smem + buf * 2 * TILE;
    bf16* Vl = Kl + TILE;
#pragma unroll
    for (int p = 0; p < LOADS; ++p) {
      const int ci = p * 256 + threadIdx.x;
      const int row = ci / CH, ch = ci % CH;
      *reinterpret_cast<bf16x8*>(Kl + row * LDR + ch * 8) = kr[set][p];
      *reinterpret_cast<bf16x8*>(Vl + row * LDR + ch * 8) = vr[set][p];
    }
  };

  if (nt > 0) load_tile(0, 0);
  if (PF == 2 && nt > 1) load_tile(PF - 1, 1);
  for (int t2 = 0; t2 < nt; t2 += 2) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
    const int t = t2 + u;
    if (t >= nt) break;
    const int set = PF == 2 ? u : 0;
    store_tile(set, u);
    __syncthreads();
    if (t + PF < nt) load_tile(set, t + PF);
    const bf16* Kl = smem + u * 2 * TILE;
    const bf16* Vl = Kl + TILE;
    const int k0 = t * 64;
    // ---- Sᵀ[key][q] for 4 key-subtiles × 2 query-subtiles
    f32x4 sc[4][QT];
#pragma unroll
    for (int kt = 0; kt < 4; ++kt) {
#pragma unroll
      for (int qt = 0; qt < QT; ++qt) sc[kt][qt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < NS; ++s) {
        const bf16x8 kf = *reinterpret_cast<const bf16x8*>(Kl + (16 * kt + li) * LDR + 32 * s + 8 * g);
#pragma unroll
        for (int qt = 0; qt < QT; ++qt)
          sc[kt][qt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf, qf[qt][s], sc[kt][qt], 0, 0, 0);
      }
    }
    // ---- masks + online softmax (lane owns query q0 + 16qt + li; keys k0 + 16kt + 4g + r)
    const bool need_mask = (causal && k0 + 63 > qoff + q0) || (k0 + 64 > kvlen);
    bf16x8 pf[QT][2];
#pragma unroll
    for (int qt = 0; qt < QT; ++qt) {
      const int qa = q0 + 16 * qt + li;
      const int klim = min(causal ? qoff + qa : Skv, kvlen - 1);  // last key this query may see
      // raw scores: the log2(e)/√D scale is folded into the exponent's FMA below
      if (need_mask) {
#pragma unroll
        for (int kt = 0; kt < 4; ++kt)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            sc[kt][qt][r] = (k0 + 16 * kt + 4 * g + r <= klim) ? sc[kt][qt][r] : -INFINITY;
      }
      float mx = -INFINITY;
#pragma unroll
      for (int kt = 0; kt < 4; ++kt)
#pragma unroll
        for (int r = 0; r < 4; ++r) mx = fmaxf(mx, sc[kt][qt][r]);
      mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
      mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
      const float mn = fmaxf(m_run[qt], mx);
      const bool dead = mn == -INFINITY;   // every key so far masked for this query
      const float alpha = dead ? 1.f : fexp2((m_run[qt] - mn) * scale_log2);
      const float mc = dead ? 0.f : mn * scale_log2;
      float rs = 0.f;
#pragma unroll
      for (int kt = 0; kt < 4; ++kt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float p = dead ? 0.f : fexp2(fmaf(sc[kt][qt][r], scale_log2, -mc));
          sc[kt][qt][r] = p;
          rs += p;
        }
      rs += __shfl_xor(rs, 16, 64);
      rs += __shfl_xor(rs, 32, 64);
      l_run[qt] = l_run[qt] * alpha + rs;
      m_run[qt] = mn;
      if (__any(alpha != 1.f)) {   // the running max moved for some query of the wave: rescale O
#pragma unroll
        for (int dt = 0; dt < ND; ++dt) acc[dt][qt] *= alpha;
      }
      if (dp.thresh) {
        const uint32_t bh = (uint32_t)(b * hq + h);
#pragma unroll
        for (int kt = 0; kt < 4; ++kt)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            sc[kt][qt][r] = drop_hash(dp.s0, dp.s1, bh, qa, k0 + 16 * kt + 4 * g + r) >= dp.thresh
                                ? sc[kt][qt][r] * dp.rinv : 0.f;
      }
      // P as B operand, permuted key order j ↔ 32kb + 16(j>>2) + 4g + (j&3)
      pf[qt][0] = f2b8(sc[0][qt], sc[1][qt]);
      pf[qt][1] = f2b8(sc[2][qt], sc[3][qt]);
    }
    // ---- Oᵀ[d][q] += Vᵀ[d][key] · Pᵀ[key][q]
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
#pragma unroll
      for (int dt = 0; dt < ND; ++dt) {
        // lane 4q'+p' of each 16-group addresses row r0+q', cols 16dt+4p'..+3
        const bf16* p0 = Vl + (32 * kb + 4 * g + (li >> 2)) * LDR + 16 * dt + 4 * (li & 3);
        const bf16x8 vf = cat8(tr_read(p0), tr_read(p0 + 16 * LDR));
#pragma unroll
        for (int qt = 0; qt < QT; ++qt)
          acc[dt][qt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vf, pf[qt][kb], acc[dt][qt], 0, 0, 0);
      }
    }
    }
  }
  // ---- epilogue: O[q][16dt + 4g + r] = acc / l ; lse = (m + log2 l) * ln2
#pragma unroll
  for (int qt = 0; qt < QT; ++qt) {
    const int q = q0 + 16 * qt + li;
    if (q >= Sq) continue;
    const float inv = l_run[qt] > 0.f ? 1.f / l_run[qt] : 0.f;
#pragma unroll
    for (int dt = 0; dt < ND; ++dt) {
      bf16x4 o;
#pragma unroll
      for (int r = 0; r < 4; ++r) o[r] = (bf16)(acc[dt][qt][r] * inv);
      *reinterpret_cast<bf16x4*>(O + (tok0 + q) * (size_t)(hq * D) + h * D + 16 * dt + 4 * g) = o;
    }
    if (g == 0)
      lse[((size_t)b * hq + h) * Sq + q] =
          l_run[qt] > 0.f ? (m_run[qt] * scale_log2 + log2f(l_run[qt])) * 0.6931471805599453f : INFINITY;
  }
}

// ============================================================================ forward, D = 128
// The 32x32x16 form.  Same contract as attn_fwd_k (128 queries per workgroup, 4 waves × 32, 64-key K/V
// tiles register-staged one tile ahead), but:
//  * Sᵀ = K·Qᵀ with v_mfma_f32_32x32x16_bf16: a lane owns ONE query (column lane&31) and 32 of the tile's 64
//    keys; the row max is lane-local + one v_permlane32_swap with the other half (no ds_bpermute), the row
//    sum stays a per-lane partial until the epilogue;
//  * P feeds Oᵀ += Vᵀ·Pᵀ as the B operand with no lane movement: the k-slot order of each 16-key step is the
//    accumulator's row order (keys +{0-3, 8-11} in the low half, +{4-7, 12-15} in the high half) and the
//    transposed V reads (ds_read_b64_tr_b16) fetch exactly those rows;
//  * K and V tiles are one XOR-swizzled image each (256-B rows, chunk ^ ((row&3)<<2 | (row>>2)&3)): the
//    row-wise ds_read_b128 of K and the transposed reads of V are both conflict-free;
//  * deferred rescale: the running max moves only when a tile's max exceeds it by more than 2^8 in the
//    exponent (P ≤ 256 in bf16, l and O in fp32 see the same factor), so O is rarely rescaled;
//  * a wave skips the MFMAs of tiles wholly above its causal diagonal;
//  * the output rows are stored 16 B per lane after a permlane32 exchange of the accumulator halves.
__device__ __forceinline__ int swz128(int row) { return ((row & 3) << 2) | ((row >> 2) & 3); }
// byte offset of 16-B chunk `ch` of row `row` in a [64][128 × bf16] tile image
__device__ __forceinline__ int toff(int row, int ch) { return 256 * row + 16 * (ch ^ swz128(row)); }

// lanes 32-63 of `a` trade places with lanes 0-31 of `b` (v_permlane32_swap): afterwards the low half holds
// (a_lo, a_hi→b) and the high half (b_lo→a, b_hi) — see the callers for the element bookkeeping
__device__ __forceinline__ void swap32(float& a, float& b) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(a), __float_as_uint(b), false, false);
  a = __uint_as_float(r[0]);
  b = __uint_as_float(r[1]);
}

// LDS-DMA and raw-buffer helpers (attn_fwd128_k<0>, attn_bwd_dkv128_k).  A raw buffer descriptor (stride 0) range-checks the
// per-lane offset against num_records: rows past the end read as zero and never touch memory.
typedef __amdgpu_buffer_rsrc_t rsrc_t;
typedef __attribute__((address_space(3))) void* lds_ptr_t;
__device__ __forceinline__ rsrc_t attn_rsrc(const void* base, size_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0,
                                           (int)(bytes > 0x7fffffffull ? 0x7fffffffull : bytes), 0x00020000);
}
// one wave-instruction of LDS-DMA: lane l's 16 B from rs + voff land at LDS m0v + 16·l (M0 saved / restored)
__device__ __forceinline__ void attn_dma16(const rsrc_t& rs, uint32_t m0v, uint32_t voff) {
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %1\n\t"
      "s_nop 0\n\t"
      "buffer_load_dwordx4 %2, %3, 0 offen lds\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "s"(m0v), "v"(voff), "s"(rs)
      : "memory");
}

template <bool DROP>
__global__ __launch_bounds__(256, 2) void attn_fwd128_k(const bf16* __restrict__ Q, const bf16* __restrict__ K,
                                                     const bf16* __restrict__ V, int ldq, int ldk, int ldv,
                                                     const int* __restrict__ kv_lens, const int* __restrict__ q_offs,
                                                     bf16* __restrict__ O, float* __restrict__ lse, int Sq, int Skv,
                                                     int kv_rows, int hq, int hkv, int causal, float scale_log2,
                                                     DropParams dp) {
  constexpr int D = 128, TB = 64 * 256;   // bytes per K or V tile image
  __shared__ __attribute__((aligned(16))) char smem[4 * TB];   // K0 V0 K1 V1
  const int nqb = (Sq + 127) / 128;
  int i0, h, b;
  xcd_grid3_lpt(i0, h, b, causal >> 1);
  const int qb = nqb - 1 - i0;   // heavy (late, causal) blocks first
  const int hk = h / (hq / hkv);
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63, r32 = lane & 31, hi = lane >> 5;
  const int q0w = qb * 128 + 32 * w;   // this wave's first query
  const int qa = q0w + r32;            // this lane's query
  const int qoff = q_offs ? q_offs[b] : 0;
  const int kvlen = min(kv_lens ? kv_lens[b] : Skv, Skv);
  const size_t tok0 = (size_t)b * Sq, ktok0 = (size_t)b * kv_rows;

  // Q as the B operand of Sᵀ = K·Qᵀ: lane (q, hi) holds Q[q][16ds + 8hi + j]
  bf16x8 qf[8];
  {
    const int qc = qa < Sq ? qa : Sq - 1;
    const bf16* qp = Q + (tok0 + qc) * ldq + h * D + 8 * hi;
#pragma unroll
    for (int ds = 0; ds < 8; ++ds) qf[ds] = *reinterpret_cast<const bf16x8*>(qp + 16 * ds);
  }
  int kend = causal ? min(Skv, qoff + qb * 128 + 128) : Skv;
  kend = min(kend, kvlen);
  const int nt = (kend + 63) / 64;
  const int wend = causal ? min(kend, qoff + q0w + 32) : kend;   // keys any query of this wave may see
  const int ntw = wend > 0 ? (wend + 63) / 64 : 0;
  const int klim = min(causal ? qoff + qa : Skv - 1, kvlen - 1);  // last key this query may see

  f32x16 acc[4];
#pragma unroll
  for (int dt = 0; dt < 4; ++dt)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[dt][r] = 0.f;
  float m_run = -INFINITY, l_run = 0.f;

  // transposed-read geometry (T10): lane 4q'+p' of 16-lane group g addresses row q' of a 4-row block,
  // chunk 2(g&1) + (p'>>1) of the 32-column d block, half p'&1 of it
  const int g = lane >> 4, qq = (lane & 15) >> 2, pp = lane & 3;
  // XOR-addressed operand bases (see attn_bwd_dkv128_k): K row r32 (+32 kh rows = 8 KB), Vᵀ rows ra0 / ra0 + 8
  // (+16 u2 rows = 4 KB, transposed chunk 4dt + c0 = base ^ 64dt)
  int ak = toff(r32, hi);
  const int ra0 = 4 * (g >> 1) + qq, c0 = 2 * (g & 1) + (pp >> 1);
  int at0 = toff(ra0, c0) + 8 * (pp & 1), at1 = toff(ra0 + 8, c0) + 8 * (pp & 1);

  // K / V tiles by LDS-DMA (as attn_bwd_dkv128_k: wave w moves image rows 16w .. 16w + 15, the swizzle applied on
  // the global side, zero past Skv), one barrier per tile, no staging VGPRs or LDS stores (row strides ldk / ldv
  // multiples of 128 elements: the binding checks)
  const uint32_t lds0 = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(lds_ptr_t)smem);
  const int wu = __builtin_amdgcn_readfirstlane(w);
  const uint32_t ldk2 = (uint32_t)ldk * 2, ldv2 = (uint32_t)ldv * 2;
  const uint32_t xs = 16u * (uint32_t)((lane & 15) ^ ((lane >> 4) << 2));
  const uint32_t vk = (16u * wu + (lane >> 4)) * ldk2 + xs, vv = (16u * wu + (lane >> 4)) * ldv2 + xs;
  auto dma_tile = [&](int t) {
    const rsrc_t rk = attn_rsrc(K + (ktok0 + t * 64) * ldk + hk * D, (size_t)max(Skv - t * 64, 0) * ldk2);
    const rsrc_t rv = attn_rsrc(V + (ktok0 + t * 64) * ldv + hk * D, (size_t)max(Skv - t * 64, 0) * ldv2);
    const uint32_t dst = lds0 + (uint32_t)(2 * TB * (t & 1) + 4096 * wu);
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      attn_dma16(rk, dst + 1024 * p, (vk + 4u * p * ldk2) ^ (16u * p));
      attn_dma16(rv, dst + TB + 1024 * p, (vv + 4u * p * ldv2) ^ (16u * p));
    }
  };
  if (nt > 0) dma_tile(0);
  for (int t2 = 0; t2 < nt; t2 += 2) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int t = t2 + u;
      if (t >= nt) break;
      __builtin_amdgcn_s_waitcnt(0xF70);   // vmcnt(0): this wave's DMAs of tile t have landed
      __syncthreads();                     // ... everyone's; every read of the other buffer is done
      if (t + 1 < nt) dma_tile(t + 1);
      if (t >= ntw) continue;   // wave-uniform: every key of the tile is above this wave's diagonal
      const char* Kl = smem + u * 2 * TB;
      const char* Vl = Kl + TB;
      const int k0 = t * 64;
      asm volatile("" : "+v"(ak), "+v"(at0), "+v"(at1));   // keep the XORs in the loop
      // ---- Sᵀ[key][q]: keys k0 + 32kh + (r&3) + 8(r>>2) + 4hi of accumulator element r
      f32x16 sc[2];
#pragma unroll
      for (int kh = 0; kh < 2; ++kh) {
#pragma unroll
        for (int r = 0; r < 16; ++r) sc[kh][r] = 0.f;
#pragma unroll
        for (int ds = 0; ds < 8; ++ds) {
          const bf16x8 kf = *reinterpret_cast<const bf16x8*>(Kl + 8192 * kh + (ak ^ (32 * ds)));
          sc[kh] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf, qf[ds], sc[kh], 0, 0, 0);
        }
      }
      const bool need_mask = (causal && k0 + 63 > qoff + q0w) || (k0 + 64 > kvlen);
      if (need_mask) {
#pragma unroll
        for (int kh = 0; kh < 2; ++kh)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int key = k0 + 32 * kh + (r & 3) + 8 * (r >> 2) + 4 * hi;
            sc[kh][r] = key <= klim ? sc[kh][r] : -INFINITY;
          }
      }
      float mx = -INFINITY;
#pragma unroll
      for (int kh = 0; kh < 2; ++kh)
#pragma unroll
        for (int r = 0; r < 16; ++r) mx = fmaxf(mx, sc[kh][r]);
      {
        float a = mx, c = mx;
        swap32(a, c);           // a = the low half's max, c = the high half's, in every lane
        mx = fmaxf(a, c);
      }
      const float mn = fmaxf(m_run, mx);
      const bool resc = (mn - m_run) * scale_log2 > 8.f;   // false while every key so far is masked (NaN)
      if (__any(resc)) {
        const float alpha = resc ? fexp2((m_run - mn) * scale_log2) : 1.f;
        m_run = resc ? mn : m_run;
        l_run *= alpha;
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) acc[dt] *= alpha;
      }
      const float mc = m_run == -INFINITY ? 0.f : m_run * scale_log2;
      float rs = 0.f;
#pragma unroll
      for (int kh = 0; kh < 2; ++kh)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float p = fexp2(fmaf(sc[kh][r], scale_log2, -mc));
          sc[kh][r] = p;
          rs += p;
        }
      l_run += rs;   // this half's keys only; the halves are summed in the epilogue
      if (DROP) {
        const uint32_t bh = (uint32_t)(b * hq + h);
#pragma unroll
        for (int kh = 0; kh < 2; ++kh)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int key = k0 + 32 * kh + (r & 3) + 8 * (r >> 2) + 4 * hi;
            sc[kh][r] = drop_hash(dp.s0, dp.s1, bh, qa, key) >= dp.thresh ? sc[kh][r] * dp.rinv : 0.f;
          }
      }
      // ---- Oᵀ[d][q] += Vᵀ[d][key]·Pᵀ[key][q], 16 keys per step: P elements 8u..8u+7 are the step's k-slots
#pragma unroll
      for (int kh = 0; kh < 2; ++kh)
#pragma unroll
        for (int u2 = 0; u2 < 2; ++u2) {
          bf16x8 pb;
#pragma unroll
          for (int j = 0; j < 8; ++j) pb[j] = (bf16)sc[kh][8 * u2 + j];
#pragma unroll
          for (int dt = 0; dt < 4; ++dt) {
            const char* p0 = Vl + 8192 * kh + 4096 * u2 + (at0 ^ (64 * dt));
            const char* p1 = Vl + 8192 * kh + 4096 * u2 + (at1 ^ (64 * dt));
            const bf16x8 vf = cat8(tr_read((const bf16*)p0), tr_read((const bf16*)p1));
            acc[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vf, pb, acc[dt], 0, 0, 0);
          }
        }
    }
  }
  // ---- epilogue: l over both halves; O rows 16 B per lane after exchanging accumulator quarters
  float la = l_run, lb = l_run;
  swap32(la, lb);
  const float lt = la + lb;
  const float inv = lt > 0.f ? 1.f / lt : 0.f;
  bf16* orow = O + (tok0 + (qa < Sq ? qa : 0)) * (size_t)(hq * D) + h * D + 8 * hi;
#pragma unroll
  for (int dt = 0; dt < 4; ++dt)
#pragma unroll
    for (int hf = 0; hf < 2; ++hf) {
      // elements 8hf + j: d = 32dt + 16hf + 4hi + j (j < 4) and + 8 (j >= 4); after the swap lane-half hi
      // holds d = 32dt + 16hf + 8hi + 0..7
      float a[4], c[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        a[j] = acc[dt][8 * hf + j] * inv;
        c[j] = acc[dt][8 * hf + 4 + j] * inv;
        swap32(a[j], c[j]);
      }
      if (qa < Sq)
        *reinterpret_cast<bf16x8*>(orow + 32 * dt + 16 * hf) =
            bf16x8{(bf16)a[0], (bf16)a[1], (bf16)a[2], (bf16)a[3], (bf16)c[0], (bf16)c[1], (bf16)c[2], (bf16)c[3]};
    }
  if (hi == 0 && qa < Sq)
    lse[((size_t)b * hq + h) * Sq + qa] = lt > 0.f ? (m_run * scale_log2 + log2f(lt)) * 0.6931471805599453f : INFINITY;
}

// ============================================================================ backward
// Two atomic-free kernels (FA2 split).  Both recompute P from the saved log-sum-exp.
//  * attn_bwd_dq_k : workgroup = 64 queries of one q-head (4 waves × 16, one query per lane, so
//    lse/delta are lane-uniform); computes delta = Σ dO·O for its queries first (written for the
//    dK/dV kernel), then sweeps key tiles: Sᵀ = K·Qᵀ, dPᵀ = V·dOᵀ, dS, dQᵀ += Kᵀ·dSᵀ with dS kept
//    in registers (permuted key order, Kᵀ via ds_read_b64_tr_b16).  dQ is written once, in bf16.
//  * attn_bwd_dkv_k: workgroup = 64 keys of one KV head (4 waves × 16 keys, K/V fragments in
//    registers) that sweeps every q-head of its GQA group × 64-query tiles, so the group's
//    dK/dV sum stays in registers: no fp32 partials, no finalize pass.  Q/dO tiles (plus
//    their lse/delta) are register-prefetched one tile ahead into double-buffered LDS.
template <int D, int PF>
__global__ __launch_bounds__(256, 2) void attn_bwd_dq_k(const bf16* __restrict__ dO, const bf16* __restrict__ O,
                                                     const bf16* __restrict__ Q, const bf16* __restrict__ K,
                                                     const bf16* __restrict__ V, const float* __restrict__ lse,
                                                     float* __restrict__ delta, const int* __restrict__ kv_lens,
                                                     int ldq, int ldk, int ldv, bf16* __restrict__ dQ, int S, int hq,
                                                     int hkv, int causal, float scale, float scale_log2,
                                                     DropParams drp) {
  constexpr int LDR = D + 16, CH = D / 8, TILE = 64 * LDR, NS = D / 32, ND = D / 16;   // D + 16: conflict-free (see attn_fwd_k)
  constexpr int LOADS = 64 * CH / 256;
  __shared__ __attribute__((aligned(16))) bf16 smem[4 * TILE];  // K0 V0 K1 V1

  const int nqb = (S + 63) / 64;
  int i0, h, b;
  xcd_grid3_lpt(i0, h, b, causal >> 1);   // causal bit 1: longest-first order
  const int qb = nqb - 1 - i0;  // heavy (late, causal) blocks first
  const int hk = h / (hq / hkv);
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, g = lane >> 4, li = lane & 15;
  const int q0 = qb * 64;
  const int qa = q0 + 16 * w + li;  // this lane's query (>= S in a tail tile: computed, never stored)
  const int qc = qa < S ? qa : S - 1;
  const int kvlen = min(kv_lens ? kv_lens[b] : S, S);
  const size_t tok0 = (size_t)b * S;
  const size_t ldo = (size_t)hq * D;

  bf16x8 qf[NS], dof[NS];
  float dsum = 0.f;
  const size_t bh = ((size_t)b * hq + h) * S;
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    const size_t off = (tok0 + qc) * ldo + h * D + 32 * s + 8 * g;
    qf[s] = *reinterpret_cast<const bf16x8*>(Q + (tok0 + qc) * ldq + h * D + 32 * s + 8 * g);
    dof[s] = *reinterpret_cast<const bf16x8*>(dO + off);
    const bf16x8 of = *reinterpret_cast<const bf16x8*>(O + off);
#pragma unroll
    for (int j = 0; j < 8; ++j) dsum += (float)dof[s][j] * (float)of[j];
  }
  dsum += __shfl_xor(dsum, 16, 64);
  dsum += __shfl_xor(dsum, 32, 64);
  if (g == 0 && qa < S) delta[bh + qa] = dsum;
  const float lse2 = lse[bh + qc] * LOG2E;
  const int klim = min(causal ? qa : S, kvlen - 1);  // last key this query may see

  int kend = causal ? min(S, q0 + 64) : S;
  kend = min(kend, kvlen);
  const int nt = (kend + 63) / 64;

  f32x4 acc[ND];
#pragma unroll
  for (int dt = 0; dt < ND; ++dt) acc[dt] = f32x4{0.f, 0.f, 0.f, 0.f};

  bf16x8 kr[PF][LOADS], vr[PF][LOADS];   // two tiles ahead, as the forward
  auto load_tile = [&](int set, int t) {
#pragma unroll
    for (int p = 0; p < LOADS; ++p) {
      const int ci = p * 256 + threadIdx.x;
      const int row = ci / CH, ch = ci % CH;
      const size_t key = tok0 + min(t * 64 + row, S - 1);
      kr[set][p] = *reinterpret_cast<const bf16x8*>(K + key * ldk + hk * D + ch * 8);
      vr[set][p] = *reinterpret_cast<const bf16x8*>(V + key * ldv + hk * D + ch * 8);
    }
  };
  auto store_tile = [&](int set, int buf) {
    bf16* Kl = smem + buf * 2 * TILE;
    bf16* Vl = Kl + TILE;
#pragma unroll
    for (int p = 0; p < LOADS; ++p) {
      const int ci = p * 256 + threadIdx.x;
      const int row = ci / CH, ch = ci % CH;
      *reinterpret_cast<bf16x8*>(Kl + row * LDR + ch * 8) = kr[set][p];
      *reinterpret_cast<bf16x8*>(Vl + row * LDR + ch * 8) = vr[set][p];
    }
  };

  if (nt > 0) load_tile(0, 0);
  if (PF == 2 && nt > 1) load_tile(PF - 1, 1);
  for (int t2 = 0; t2 < nt; t2 += 2) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
    const int t = t2 + u;
    if (t >= nt) break;
    const int set = PF == 2 ? u : 0;
    store_tile(set, u);
    __syncthreads();
    if (t + PF < nt) load_tile(set, t + PF);
    const bf16* Kl = smem + u * 2 * TILE;
    const bf16* Vl = Kl + TILE;
    const int k0 = t * 64;
    // ---- Sᵀ[key][q], dPᵀ[key][q] for 4 key-subtiles (lane: query li, keys 16kt + 4g + r)
    f32x4 sc[4], dp[4];
#pragma unroll
    for (int kt = 0; kt < 4; ++kt) {
      sc[kt] = dp[kt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < NS; ++s) {
        const bf16x8 kf = *reinterpret_cast<const bf16x8*>(Kl + (16 * kt + li) * LDR + 32 * s + 8 * g);
        const bf16x8 vf = *reinterpret_cast<const bf16x8*>(Vl + (16 * kt + li) * LDR + 32 * s + 8 * g);
        sc[kt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf, qf[s], sc[kt], 0, 0, 0);
        dp[kt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vf, dof[s], dp[kt], 0, 0, 0);
      }
    }
    const bool need_mask = (causal && k0 + 63 > q0) || (k0 + 64 > kvlen);
#pragma unroll
    for (int kt = 0; kt < 4; ++kt)
#pragma unroll
      for (int r = 0; r < 4; ++r) sc[kt][r] = fexp2(sc[kt][r] * scale_log2 - lse2);
    if (need_mask) {
#pragma unroll
      for (int kt = 0; kt < 4; ++kt)
#pragma unroll
        for (int r = 0; r < 4; ++r) sc[kt][r] = (k0 + 16 * kt + 4 * g + r <= klim) ? sc[kt][r] : 0.f;
    }
    if (drp.thresh) {   // dP = M∘dP_drop/(1-p)
      const uint32_t bh = (uint32_t)(b * hq + h);
#pragma unroll
      for (int kt = 0; kt < 4; ++kt)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          dp[kt][r] = drop_hash(drp.s0, drp.s1, bh, qa, k0 + 16 * kt + 4 * g + r) >= drp.thresh ? dp[kt][r] * drp.rinv
                                                                                              : 0.f;
    }
#pragma unroll
    for (int kt = 0; kt < 4; ++kt)
#pragma unroll
      for (int r = 0; r < 4; ++r) sc[kt][r] *= dp[kt][r] - dsum;
    // ---- dQᵀ[d][q] += Kᵀ[d][key] · dSᵀ[key][q]  (permuted key order, as the forward's PV)
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
      const bf16x8 dsf = f2b8(sc[2 * kb], sc[2 * kb + 1]);
#pragma unroll
      for (int dt = 0; dt < ND; ++dt) {
        const bf16* p0 = Kl + (32 * kb + 4 * g + (li >> 2)) * LDR + 16 * dt + 4 * (li & 3);
        const bf16x8 ktf = cat8(tr_read(p0), tr_read(p0 + 16 * LDR));
        acc[dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ktf, dsf, acc[dt], 0, 0, 0);
      }
    }
    }
  }
  // ---- dQ[q][16dt + 4g + r] = scale · acc
  if (qa >= S) return;
#pragma unroll
  for (int dt = 0; dt < ND; ++dt) {
    bf16x4 o;
#pragma unroll
    for (int r = 0; r < 4; ++r) o[r] = (bf16)(acc[dt][r] * scale);
    *reinterpret_cast<bf16x4*>(dQ + (tok0 + qa) * ldo + h * D + 16 * dt + 4 * g) = o;
  }
}


// dQ for D = 128 in the 32x32x16 form of attn_fwd128_k: 128 queries per workgroup (4 waves × 32), a lane owns
// one query (lse and delta are lane constants).  Per 64-key tile and 32-key half: Sᵀ = K·Qᵀ and dPᵀ = V·dOᵀ
// (row reads of the swizzled K / V images), dS = P∘(dP − delta) in registers, dQᵀ += Kᵀ·dSᵀ with Kᵀ from the
// transposed reads of the same K image and dS as the B operand in accumulator-row slot order (no lane
// movement).  Writes delta for the dK/dV kernel, as attn_bwd_dq_k.
template <bool DROP>
__global__ __launch_bounds__(256, 2) void attn_bwd_dq128_k(const bf16* __restrict__ dO, const bf16* __restrict__ O,
                                                        const bf16* __restrict__ Q, const bf16* __restrict__ K,
                                                        const bf16* __restrict__ V, const float* __restrict__ lse,
                                                        float* __restrict__ delta, const int* __restrict__ kv_lens,
                                                        int ldq, int ldk, int ldv, bf16* __restrict__ dQ, int S,
                                                        int hq, int hkv, int causal, float scale, float scale_log2,
                                                        DropParams drp) {
  constexpr int D = 128, TB = 64 * 256;
  __shared__ __attribute__((aligned(16))) char smem[4 * TB];   // K0 V0 K1 V1
  const int nqb = (S + 127) / 128;
  int i0, h, b;
  xcd_grid3_lpt(i0, h, b, causal >> 1);
  const int qb = nqb - 1 - i0;
  const int hk = h / (hq / hkv);
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63, r32 = lane & 31, hi = lane >> 5;
  const int q0w = qb * 128 + 32 * w, qa = q0w + r32, qc = qa < S ? qa : S - 1;
  const int kvlen = min(kv_lens ? kv_lens[b] : S, S);
  const size_t tok0 = (size_t)b * S, ldo = (size_t)hq * D;
  const size_t bh = ((size_t)b * hq + h) * S;

  bf16x8 qf[8], dof[8];
  float dsum = 0.f;
  {
    const bf16* qp = Q + (tok0 + qc) * ldq + h * D + 8 * hi;
    const size_t off = (tok0 + qc) * ldo + h * D + 8 * hi;
#pragma unroll
    for (int ds = 0; ds < 8; ++ds) {
      qf[ds] = *reinterpret_cast<const bf16x8*>(qp + 16 * ds);
      dof[ds] = *reinterpret_cast<const bf16x8*>(dO + off + 16 * ds);
      const bf16x8 of = *reinterpret_cast<const bf16x8*>(O + off + 16 * ds);
#pragma unroll
      for (int j = 0; j < 8; ++j) dsum += (float)dof[ds][j] * (float)of[j];
    }
  }
  {
    float a = dsum, c = dsum;
    swap32(a, c);
    dsum = a + c;
  }
  if (hi == 0 && qa < S) delta[bh + qa] = dsum;
  const float lse2 = lse[bh + qc] * LOG2E;
  const int klim = min(causal ? qa : S - 1, kvlen - 1);   // last key this query may see
  int kend = causal ? min(S, qb * 128 + 128) : S;
  kend = min(kend, kvlen);
  const int nt = (kend + 63) / 64;
  const int wend = causal ? min(kend, q0w + 32) : kend;
  const int ntw = wend > 0 ? (wend + 63) / 64 : 0;

  f32x16 acc[4];
#pragma unroll
  for (int dt = 0; dt < 4; ++dt)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[dt][r] = 0.f;

  const int g = lane >> 4, qq = (lane & 15) >> 2, pp = lane & 3;
  // operand rows as XOR-addressed bases (see attn_bwd_dkv128_k): K row r32 (+32 kh rows = 8 KB), Kᵀ rows
  // ra0 / ra0 + 8 (+16 u2 rows = 4 KB, transposed chunk 4dt + c0 = base ^ 64dt)
  int ak = toff(r32, hi);
  const int ra0 = 4 * (g >> 1) + qq, c0 = 2 * (g & 1) + (pp >> 1);
  int at0 = toff(ra0, c0) + 8 * (pp & 1), at1 = toff(ra0 + 8, c0) + 8 * (pp & 1);

  // K / V tiles by LDS-DMA as attn_fwd128_k (no staging VGPRs / LDS stores, one barrier per tile)
  const uint32_t lds0 = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(lds_ptr_t)smem);
  const int wu = __builtin_amdgcn_readfirstlane(w);
  const uint32_t ldk2 = (uint32_t)ldk * 2, ldv2 = (uint32_t)ldv * 2;
  const uint32_t xs = 16u * (uint32_t)((lane & 15) ^ ((lane >> 4) << 2));
  const uint32_t vk = (16u * wu + (lane >> 4)) * ldk2 + xs, vv = (16u * wu + (lane >> 4)) * ldv2 + xs;
  auto dma_tile = [&](int t) {
    const rsrc_t rk = attn_rsrc(K + (tok0 + t * 64) * ldk + hk * D, (size_t)max(S - t * 64, 0) * ldk2);
    const rsrc_t rv = attn_rsrc(V + (tok0 + t * 64) * ldv + hk * D, (size_t)max(S - t * 64, 0) * ldv2);
    const uint32_t dst = lds0 + (uint32_t)(2 * TB * (t & 1) + 4096 * wu);
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      attn_dma16(rk, dst + 1024 * p, (vk + 4u * p * ldk2) ^ (16u * p));
      attn_dma16(rv, dst + TB + 1024 * p, (vv + 4u * p * ldv2) ^ (16u * p));
    }
  };
  if (nt > 0) dma_tile(0);
  for (int t2 = 0; t2 < nt; t2 += 2) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int t = t2 + u;
      if (t >= nt) break;
      __builtin_amdgcn_s_waitcnt(0xF70);   // vmcnt(0): this wave's DMAs of tile t have landed
      __syncthreads();
      if (t + 1 < nt) dma_tile(t + 1);
      if (t >= ntw) continue;
      const char* Kl = smem + u * 2 * TB;
      const int k0 = t * 64;
      const bool need_mask = (causal && k0 + 63 > q0w) || (k0 + 64 > kvlen);
      asm volatile("" : "+v"(ak), "+v"(at0), "+v"(at1));   // keep the XORs in the loop
#pragma unroll
      for (int kh = 0; kh < 2; ++kh) {
        f32x16 s, dp;
#pragma unroll
        for (int r = 0; r < 16; ++r) s[r] = dp[r] = 0.f;
#pragma unroll
        for (int ds = 0; ds < 8; ++ds) {
          const char* pk = Kl + 8192 * kh + (ak ^ (32 * ds));
          const bf16x8 kf = *reinterpret_cast<const bf16x8*>(pk);
          const bf16x8 vf = *reinterpret_cast<const bf16x8*>(pk + TB);
          s = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf, qf[ds], s, 0, 0, 0);
          dp = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vf, dof[ds], dp, 0, 0, 0);
        }
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int key = k0 + 32 * kh + (r & 3) + 8 * (r >> 2) + 4 * hi;
          float p = fexp2(fmaf(s[r], scale_log2, -lse2));
          if (need_mask) p = key <= klim ? p : 0.f;
          float d = dp[r];
          if (DROP) d = drop_hash(drp.s0, drp.s1, (uint32_t)(b * hq + h), qa, key) >= drp.thresh ? d * drp.rinv : 0.f;
          s[r] = p * (d - dsum);
        }
        // dQᵀ[d][q] += Kᵀ[d][key]·dSᵀ[key][q]
#pragma unroll
        for (int u2 = 0; u2 < 2; ++u2) {
          bf16x8 pb;
#pragma unroll
          for (int j = 0; j < 8; ++j) pb[j] = (bf16)s[8 * u2 + j];
#pragma unroll
          for (int dt = 0; dt < 4; ++dt) {
            const char* p0 = Kl + 8192 * kh + 4096 * u2 + (at0 ^ (64 * dt));
            const char* p1 = Kl + 8192 * kh + 4096 * u2 + (at1 ^ (64 * dt));
            const bf16x8 kt = cat8(tr_read((const bf16*)p0), tr_read((const bf16*)p1));
            acc[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kt, pb, acc[dt], 0, 0, 0);
          }
        }
      }
    }
  }
  // ---- dQ = scale · acc, 16 B per lane after the permlane32 exchange (as attn_fwd128_k's epilogue)
  bf16* qrow = dQ + (tok0 + (qa < S ? qa : 0)) * ldo + h * D + 8 * hi;
#pragma unroll
  for (int dt = 0; dt < 4; ++dt)
#pragma unroll
    for (int hf = 0; hf < 2; ++hf) {
      float a[4], c[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        a[j] = acc[dt][8 * hf + j] * scale;
        c[j] = acc[dt][8 * hf + 4 + j] * scale;
        swap32(a[j], c[j]);
      }
      if (qa < S)
        *reinterpret_cast<bf16x8*>(qrow + 32 * dt + 16 * hf) =
            bf16x8{(bf16)a[0], (bf16)a[1], (bf16)a[2], (bf16)a[3], (bf16)c[0], (bf16)c[1], (bf16)c[2], (bf16)c[3]};
    }
}

// dK / dV for D = 128 in the 32x32x16 form, two waves per SIMD: a 512-thread workgroup = 64 keys of one KV
// head; wave w = (key half kw2 = w&1: 32 keys on the lanes, query half qh = (w>>1)&1: 32 of the tile's 64
// queries, head half hw = w>>2: the GQA group's q-heads split even / odd).  The K / V images of the block sit
// in LDS for the whole sweep (B operands of S = Q·Kᵀ and dP = dO·Vᵀ by row reads); each head half streams its
// Q / dO tiles by LDS-DMA into two buffers (tile it+1 lands while tile it is computed: one barrier per tile, no
// staging registers), the swizzle applied on the global side (lane l of a 1 KB DMA fetches the chunk that the
// image keeps at slot l).  lse / delta come straight from global (raw-buffer loads, zero past S, one tile ahead).
// dVᵀ += dOᵀ·P and dKᵀ += Qᵀ·dS take dOᵀ / Qᵀ from transposed reads of the same swizzled images and P / dS
// as B operands in accumulator-row slot order.  The four waves of a key half meet in LDS at the end.
// Split key blocks (nsplit) write fp32 partials as attn_bwd_dkv_k.  160 KB LDS, ≤ 256 VGPRs.
// Requires ldq % 128 == 0 (row strides in whole 256-B units: see attn_dkv128_ok).
template <bool DROP, bool TRACE = false>
__global__ __launch_bounds__(512, 1) void attn_bwd_dkv128_k(const bf16* __restrict__ dO, const bf16* __restrict__ Q,
                                                         const bf16* __restrict__ K, const bf16* __restrict__ V,
                                                         const float* __restrict__ lse,
                                                         const float* __restrict__ delta,
                                                         const int* __restrict__ kv_lens, int ldq, int ldk, int ldv,
                                                         bf16* __restrict__ dK, bf16* __restrict__ dV, int S, int hq,
                                                         int hkv, int causal, float scale, float scale_log2,
                                                         DropParams drp, float* __restrict__ ws, int nsplit) {
  constexpr int D = 128, TB = 64 * 256;
  __shared__ __attribute__((aligned(1024))) char smem[10 * TB];   // K | V | [head half][buffer][Q | dO]
  int ui, hk, b;
  xcd_grid3(ui, hk, b);
  int kbi, part;
  if (ui < 2 * nsplit) {
    kbi = ui >> 1;
    part = ui & 1;
  } else {
    kbi = ui - nsplit;
    part = -1;
  }
  const int rep = hq / hkv;
  const int tid = threadIdx.x, lane = tid & 63, r32 = lane & 31, hi = lane >> 5;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);   // wave-uniform roles
  const int kw2 = w & 1, qh = (w >> 1) & 1, hw = w >> 2, w4 = w & 3;
  const int kb0 = kbi * 64;
  const int kw = kb0 + 32 * kw2 + r32;   // this lane's key
  const int kvlen = min(kv_lens ? kv_lens[b] : S, S);
  const size_t tok0 = (size_t)b * S, ldo = (size_t)hq * D, ldkv = (size_t)hkv * D;
  const uint32_t lds0 = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(lds_ptr_t)smem);

  // K / V images of the 64 keys (512 threads × 2 chunks each per tensor)
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    const int id = p * 512 + tid, row = id >> 4, ch = id & 15;
    const size_t key = tok0 + min(kb0 + row, S - 1);
    *reinterpret_cast<bf16x8*>(smem + toff(row, ch)) = *reinterpret_cast<const bf16x8*>(K + key * ldk + hk * D + ch * 8);
    *reinterpret_cast<bf16x8*>(smem + TB + toff(row, ch)) =
        *reinterpret_cast<const bf16x8*>(V + key * ldv + hk * D + ch * 8);
  }
  f32x16 dk[4], dv[4];
#pragma unroll
  for (int dt = 0; dt < 4; ++dt)
#pragma unroll
    for (int r = 0; r < 16; ++r) dk[dt][r] = dv[dt][r] = 0.f;

  int qt0 = causal ? kbi : 0;
  const int qmin = kw < kvlen ? (causal ? kw : 0) : 1 << 30;   // first query that sees this key
  int nqt = (S + 63) / 64 - qt0;
  if (part >= 0) {
    const int h1 = (nqt + 1) / 2;
    if (part == 0) {
      nqt = h1;
    } else {
      qt0 += h1;
      nqt -= h1;
    }
  }
  const int nh = (rep + 1) / 2;
  const int n_it = kb0 < kvlen ? nh * nqt : 0;

  // DMA geometry: wave w4 of a head half moves image rows 16w4 .. 16w4 + 15 of Q and of dO (4 × 1 KB each);
  // in 1 KB chunk p lane l fills row 16w4 + 4p + (l>>4), slot l&15, i.e. logical chunk (l&15) ^ swz(row) =
  // (l&15) ^ ((l>>4)<<2) ^ p.  Row strides are multiples of 256 B, so the chunk XOR never carries into them.
  const uint32_t ldq2 = (uint32_t)ldq * 2, ldo2 = (uint32_t)ldo * 2;
  const uint32_t xs = 16u * (uint32_t)((lane & 15) ^ ((lane >> 4) << 2));
  const uint32_t vq = (16u * w4 + (lane >> 4)) * ldq2 + xs, vo = (16u * w4 + (lane >> 4)) * ldo2 + xs;
  auto dma_it = [&](int it2) {
    const int j2 = hw + 2 * (it2 / nqt);
    if (j2 >= rep) return;
    const int h2 = hk * rep + j2;
    const int qb = (qt0 + it2 % nqt) * 64;
    const rsrc_t rq = attn_rsrc(Q + (tok0 + qb) * ldq + h2 * D, (size_t)(S - qb) * ldq2);
    const rsrc_t ro = attn_rsrc(dO + (tok0 + qb) * ldo + h2 * D, (size_t)(S - qb) * ldo2);
    const uint32_t dst = lds0 + (uint32_t)(2 * TB * (1 + 2 * hw + (it2 & 1)) + 4096 * w4);
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      attn_dma16(rq, dst + 1024 * p, (vq + 4u * p * ldq2) ^ (16u * p));
      attn_dma16(ro, dst + TB + 1024 * p, (vo + 4u * p * ldo2) ^ (16u * p));
    }
  };
  const int g = lane >> 4, qq = (lane & 15) >> 2, pp = lane & 3;
  // LDS byte offsets of this lane's operand rows.  The swizzle permutes only bits 4-7 of a row's byte offset
  // (images start at multiples of 16 KB), so chunk 2ds + hi of row r is toff(r, hi) ^ 32ds and the transposed
  // chunk 4dt + c of row ra is toff(ra, c) ^ 64dt: four base registers instead of one address per read
  const int img = 2 * TB * (1 + 2 * hw);                 // this head half's buffer 0 (buffer 1: + 2 TB)
  int aq = img + toff(32 * qh + r32, hi);                // Q row (dO: + TB)
  int ak = toff(32 * kw2 + r32, hi);                     // K row (V: + TB)
  const int ra0 = 32 * qh + 4 * (g >> 1) + qq, c0 = 2 * (g & 1) + (pp >> 1);
  int at0 = img + toff(ra0, c0) + 8 * (pp & 1);          // rows ra0 (+16 u2), Qᵀ (dOᵀ: + TB)
  int at1 = img + toff(ra0 + 8, c0) + 8 * (pp & 1);      // rows ra0 + 8 (+16 u2)
  const uint32_t vst = (uint32_t)(32 * qh + 4 * hi) * 4;   // this lane's first lse / delta byte in the tile

  // TRACE (LIPA_ATTN_TRACE, attn_set_trace): lane 0 of every wave stamps s_memtime at the loop's phase
  // boundaries into ws: per wave [hw_id, xcc_id, unit, n_it, t_start, t_end, rt_start, rt_end, 4 × 64 iterations]
  unsigned long long* trc = nullptr;
  if (TRACE) {
    const int wg = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);
    trc = reinterpret_cast<unsigned long long*>(ws) + ((size_t)wg * 8 + w) * 264;
    if (lane == 0) {
      trc[0] = __builtin_amdgcn_s_getreg((31 << 11) | 4);
      trc[1] = __builtin_amdgcn_s_getreg((31 << 11) | 20);
      trc[2] = (unsigned long long)(kbi * 2 + (part + 1)) | ((unsigned long long)(hk + hkv * b) << 32);
      trc[3] = n_it;
      trc[4] = __builtin_readcyclecounter();
      trc[6] = __builtin_amdgcn_s_memrealtime();
    }
  }
  auto mark = [&](int it, int e) {
    if (TRACE && lane == 0 && it < 64) trc[8 + 4 * it + e] = __builtin_readcyclecounter();
  };
  // lse / delta of a tile: compiler-visible raw-buffer loads (zero past S), issued at the end of the previous
  // iteration and covered by the loop-top vmcnt(0) — no counted wait that would assume in-order completion
  // beside the LDS-DMAs (a vmcnt(8) "stats only" wait raced under contention: scripts/experiments/
  // attn_bwd_repeat.py, two processes)
  f32x4 L[4], Dl[4];
  auto act_of = [&](int it2) {
    const int j2 = hw + 2 * (it2 / nqt);
    const int qb = (qt0 + it2 % nqt) * 64;
    return j2 < rep && !(causal && qb + 32 * qh + 31 < kb0 + 32 * kw2);
  };
  auto stats_it = [&](int it2) {
    if (!act_of(it2)) return;
    const int j2 = hw + 2 * (it2 / nqt);
    const int qb = (qt0 + it2 % nqt) * 64;
    const size_t bh = ((size_t)b * hq + hk * rep + j2) * S + qb;
    const rsrc_t rl = attn_rsrc(lse + bh, (size_t)(S - qb) * 4);
    const rsrc_t rd = attn_rsrc(delta + bh, (size_t)(S - qb) * 4);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      L[i] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rl, vst + 32 * i, 0, 0));
      Dl[i] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rd, vst + 32 * i, 0, 0));
    }
  };
  if (n_it > 0) {
    dma_it(0);
    stats_it(0);
  }
  for (int it = 0; it < n_it; ++it) {
    mark(it, 0);
    __builtin_amdgcn_s_waitcnt(0xF70);   // vmcnt(0): this wave's DMAs and lse / delta loads of tile it have landed
    __syncthreads();   // ... everyone's; and every read of tile it-1's buffer (the next DMA target) is done
    mark(it, 1);
    const int j = hw + 2 * (it / nqt);
    const int qa0 = (qt0 + it % nqt) * 64;
    const bool act = act_of(it);
    if (it + 1 < n_it) dma_it(it + 1);
    if (act) {
    const int bo = (it & 1) * 2 * TB;
    asm volatile("" : "+v"(aq), "+v"(ak), "+v"(at0), "+v"(at1));   // keep the XORs in the loop (not 24 hoisted registers)
    f32x16 s, dp;
#pragma unroll
    for (int r = 0; r < 16; ++r) s[r] = dp[r] = 0.f;
#pragma unroll
    for (int ds = 0; ds < 8; ++ds) {
      const char* pq = smem + bo + (aq ^ (32 * ds));
      const char* pk = smem + (ak ^ (32 * ds));
      s = __builtin_amdgcn_mfma_f32_32x32x16_bf16(*reinterpret_cast<const bf16x8*>(pq),
                                                 *reinterpret_cast<const bf16x8*>(pk), s, 0, 0, 0);
      dp = __builtin_amdgcn_mfma_f32_32x32x16_bf16(*reinterpret_cast<const bf16x8*>(pq + TB),
                                                  *reinterpret_cast<const bf16x8*>(pk + TB), dp, 0, 0, 0);
    }
    // element r is row q = qa0 + 32qh + 4hi + c(r), c(r) = (r&3) + 8(r>>2); valid iff lo <= c(r) < hs (causal /
    // kv length: q >= qmin; rows past S: q < S)
    const bool need_mask = (causal && qa0 + 32 * qh < kb0 + 32 * kw2 + 32) || (kb0 + 64 > kvlen) || (qa0 + 64 > S);
    const int lo = qmin - (qa0 + 32 * qh + 4 * hi), hs = S - (qa0 + 32 * qh + 4 * hi);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int r = 4 * i + e;
        float p = fexp2(fmaf(s[r], scale_log2, L[i][e] * -LOG2E));
        if (need_mask) p = (8 * i + e >= lo && 8 * i + e < hs) ? p : 0.f;
        if (DROP) {
          const int q = qa0 + 32 * qh + 8 * i + 4 * hi + e;
          const bool keep = drop_hash(drp.s0, drp.s1, (uint32_t)(b * hq + hk * rep + j), q, kw) >= drp.thresh;
          dp[r] = p * ((keep ? dp[r] * drp.rinv : 0.f) - Dl[i][e]);
          s[r] = keep ? p * drp.rinv : 0.f;
        } else {
          dp[r] = p * (dp[r] - Dl[i][e]);
          s[r] = p;
        }
      }
    }
    mark(it, 2);
    // dVᵀ[d][key] += dOᵀ[d][q]·P[q][key] ; dKᵀ += Qᵀ·dS
#pragma unroll
    for (int u2 = 0; u2 < 2; ++u2) {
      bf16x8 pb, db;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        pb[e] = (bf16)s[8 * u2 + e];
        db[e] = (bf16)dp[8 * u2 + e];
      }
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        const char* p0 = smem + bo + (at0 ^ (64 * dt)) + 4096 * u2;
        const char* p1 = smem + bo + (at1 ^ (64 * dt)) + 4096 * u2;
        const bf16x8 ot = cat8(tr_read((const bf16*)(p0 + TB)), tr_read((const bf16*)(p1 + TB)));
        const bf16x8 qt = cat8(tr_read((const bf16*)p0), tr_read((const bf16*)p1));
        dv[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ot, pb, dv[dt], 0, 0, 0);
        dk[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(qt, db, dk[dt], 0, 0, 0);
      }
    }
    }   // act
    if (it + 1 < n_it) stats_it(it + 1);
  }
  if (TRACE && lane == 0) {
    trc[5] = __builtin_readcyclecounter();
    trc[7] = __builtin_amdgcn_s_memrealtime();
  }
  // ---- the four waves of a key half (head half × query half) sum through LDS: query half 1 → 0, then head
  // half 1 → 0, dK and dV in separate passes (a wave's 16 f32x4 per tensor = 16 KB per slot, 4 slots ≤ 96 KB)
  f32x4* red = reinterpret_cast<f32x4*>(smem);
  auto pass = [&](f32x16 (&a)[4], bool src, bool dst, int slot) {
    __syncthreads();
    if (src) {
#pragma unroll
      for (int dt = 0; dt < 4; ++dt)
#pragma unroll
        for (int i = 0; i < 4; ++i)
          red[((slot * 4 + dt) * 4 + i) * 64 + lane] = f32x4{a[dt][4 * i], a[dt][4 * i + 1], a[dt][4 * i + 2], a[dt][4 * i + 3]};
    }
    __syncthreads();
    if (dst) {
#pragma unroll
      for (int dt = 0; dt < 4; ++dt)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const f32x4 c = red[((slot * 4 + dt) * 4 + i) * 64 + lane];
#pragma unroll
          for (int e = 0; e < 4; ++e) a[dt][4 * i + e] += c[e];
        }
    }
  };
  pass(dk, qh == 1, qh == 0, hw * 2 + kw2);
  pass(dv, qh == 1, qh == 0, hw * 2 + kw2);
  pass(dk, qh == 0 && hw == 1, qh == 0 && hw == 0, kw2);
  pass(dv, qh == 0 && hw == 1, qh == 0 && hw == 0, kw2);
  if (qh != 0 || hw != 0) return;
  // ---- d = 32dt + (r&3) + 8(r>>2) + 4hi of element r
  if (part >= 0) {   // split block: raw fp32 partials, planes [part][dK | dV][T][hkv·D]
    if (kw >= S) return;
    const size_t plane = (size_t)gridDim.z * S * ldkv;
    float* wk = ws + (size_t)(2 * part) * plane + (tok0 + kw) * ldkv + hk * D + 4 * hi;
    float* wv = wk + plane;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        *reinterpret_cast<f32x4*>(wk + 32 * dt + 8 * i) =
            f32x4{dk[dt][4 * i], dk[dt][4 * i + 1], dk[dt][4 * i + 2], dk[dt][4 * i + 3]};
        *reinterpret_cast<f32x4*>(wv + 32 * dt + 8 * i) =
            f32x4{dv[dt][4 * i], dv[dt][4 * i + 1], dv[dt][4 * i + 2], dv[dt][4 * i + 3]};
      }
    return;
  }
  bf16* krow = dK + (tok0 + (kw < S ? kw : 0)) * ldkv + hk * D + 8 * hi;
  bf16* vrow = dV + (tok0 + (kw < S ? kw : 0)) * ldkv + hk * D + 8 * hi;
#pragma unroll
  for (int dt = 0; dt < 4; ++dt)
#pragma unroll
    for (int hf = 0; hf < 2; ++hf) {
      float a[4], c[4], x[4], y[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        a[e] = dk[dt][8 * hf + e] * scale;
        c[e] = dk[dt][8 * hf + 4 + e] * scale;
        swap32(a[e], c[e]);
        x[e] = dv[dt][8 * hf + e];
        y[e] = dv[dt][8 * hf + 4 + e];
        swap32(x[e], y[e]);
      }
      if (kw < S) {
        *reinterpret_cast<bf16x8*>(krow + 32 * dt + 16 * hf) =
            bf16x8{(bf16)a[0], (bf16)a[1], (bf16)a[2], (bf16)a[3], (bf16)c[0], (bf16)c[1], (bf16)c[2], (bf16)c[3]};
        *reinterpret_cast<bf16x8*>(vrow + 32 * dt + 16 * hf) =
            bf16x8{(bf16)x[0], (bf16)x[1], (bf16)x[2], (bf16)x[3], (bf16)y[0], (bf16)y[1], (bf16)y[2], (bf16)y[3]};
      }
    }
}

// HALVES = 2: a 512-thread workgroup, the two 4-wave halves sweep different q-heads of the GQA
// group over the SAME 64 keys (2 waves per SIMD instead of 1) and meet in LDS at the end.
template <int D, int HALVES, int PF>
__global__ __launch_bounds__(256 * HALVES) void attn_bwd_dkv_k(const bf16* __restrict__ dO, const bf16* __restrict__ Q,
                                                      const bf16* __restrict__ K, const bf16* __restrict__ V,
                                                      const float* __restrict__ lse, const float* __restrict__ delta,
                                                      const int* __restrict__ kv_lens, int ldq, int ldk, int ldv,
                                                      bf16* __restrict__ dK, bf16* __restrict__ dV, int S, int hq,
                                                      int hkv, int causal, float scale, float scale_log2,
                                                      DropParams drp, float* __restrict__ ws, int nsplit) {
  constexpr int LDR = D + 16, CH = D / 8, TILE = 64 * LDR, NS = D / 32, ND = D / 16;   // D + 16: conflict-free (see attn_fwd_k)
  constexpr int LOADS = 64 * CH / 256;
  __shared__ __attribute__((aligned(16))) bf16 smem_all[HALVES * 4 * TILE];  // per half: Q0 dO0 Q1 dO1
  __shared__ __attribute__((aligned(16))) float stat_all[HALVES][2][2][64];  // [half][buf][lse|delta][q]

  // causal work per key block falls off linearly (block 0 sweeps every query tile, the last one);
  // with nsplit > 0 the first nsplit blocks are each split over two workgroups by query-tile range
  // (units 2kb, 2kb+1: fp32 partials into ws, summed by attn_dkv_fin_k), the rest are whole (units
  // 2·nsplit + ...): the longest workgroup sweeps ~half as many tiles
  int ui, hk, b;
  xcd_grid3(ui, hk, b);
  int kbi, part;
  if (ui < 2 * nsplit) {
    kbi = ui >> 1;
    part = ui & 1;
  } else {
    kbi = ui - nsplit;
    part = -1;
  }
  const int rep = hq / hkv;
  const int tid = threadIdx.x & 255, hw = threadIdx.x >> 8;       // thread within half, half index
  const int hp = rep / HALVES;                                    // q-heads per half
  bf16* smem = smem_all + hw * 4 * TILE;
  float (*stat)[2][64] = stat_all[hw];
  const int w = tid >> 6, lane = threadIdx.x & 63, g = lane >> 4, li = lane & 15;
  const int kb0 = kbi * 64;
  const int kw = kb0 + 16 * w + li;  // this lane's key (column of the S / dP tiles)
  const int kwc = kw < S ? kw : S - 1;
  const int kvlen = min(kv_lens ? kv_lens[b] : S, S);
  const size_t tok0 = (size_t)b * S;
  const size_t ldo = (size_t)hq * D, ldkv = (size_t)hkv * D;

  bf16x8 kf[NS], vf[NS];
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    kf[s] = *reinterpret_cast<const bf16x8*>(K + (tok0 + kwc) * ldk + hk * D + 32 * s + 8 * g);
    vf[s] = *reinterpret_cast<const bf16x8*>(V + (tok0 + kwc) * ldv + hk * D + 32 * s + 8 * g);
  }
  f32x4 dv[ND], dk[ND];
#pragma unroll
  for (int dt = 0; dt < ND; ++dt) dv[dt] = dk[dt] = f32x4{0.f, 0.f, 0.f, 0.f};

  int qt0 = causal ? kbi : 0;
  const int qmin = kw < kvlen ? (causal ? kw : 0) : 1 << 30;  // first query that sees this key
  int nqt = (S + 63) / 64 - qt0;
  if (part >= 0) {   // this workgroup's half of the block's query tiles
    const int h1 = (nqt + 1) / 2;
    if (part == 0) {
      nqt = h1;
    } else {
      qt0 += h1;
      nqt -= h1;
    }
  }
  const int n_it = kb0 < kvlen ? hp * nqt : 0;  // keys past kv_len get zero gradient

  bf16x8 qr[PF][LOADS], dr[PF][LOADS];   // PF query tiles ahead, as the forward
  float st[PF];
  auto load_it = [&](int set, int it) {
    const int h = hk * rep + hw * hp + it / nqt;
    const int qa0 = (qt0 + it % nqt) * 64;
#pragma unroll
    for (int p = 0; p < LOADS; ++p) {
      const int ci = p * 256 + tid;
      const int row = ci / CH, ch = ci % CH;
      const size_t tq = tok0 + min(qa0 + row, S - 1);
      qr[set][p] = *reinterpret_cast<const bf16x8*>(Q + tq * ldq + h * D + ch * 8);
      dr[set][p] = *reinterpret_cast<const bf16x8*>(dO + tq * ldo + h * D + ch * 8);
    }
    if (tid < 128) {
      const size_t bh = ((size_t)b * hq + h) * S + min(qa0 + (tid & 63), S - 1);
      st[set] = tid < 64 ? lse[bh] * LOG2E : delta[bh];
    }
  };
  auto store_it = [&](int set, int buf) {
    bf16* Ql = smem + buf * 2 * TILE;
    bf16* dOl = Ql + TILE;
#pragma unroll
    for (int p = 0; p < LOADS; ++p) {
      const int ci = p * 256 + tid;
      const int row = ci / CH, ch = ci % CH;
      *reinterpret_cast<bf16x8*>(Ql + row * LDR + ch * 8) = qr[set][p];
      *reinterpret_cast<bf16x8*>(dOl + row * LDR + ch * 8) = dr[set][p];
    }
    if (tid < 128) stat[buf][tid >> 6][tid & 63] = st[set];
  };

  if (n_it > 0) load_it(0, 0);
  if (PF == 2 && n_it > 1) load_it(PF - 1, 1);
  for (int i2 = 0; i2 < n_it; i2 += 2) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
    const int it = i2 + u;
    if (it >= n_it) break;
    const int set = PF == 2 ? u : 0;
    store_it(set, u);
    __syncthreads();
    if (it + PF < n_it) load_it(set, it + PF);
    const bf16* Ql = smem + u * 2 * TILE;
    const bf16* dOl = Ql + TILE;
    const float* Ls = stat[u][0];
    const float* Dls = stat[u][1];
    const int qa0 = (qt0 + it % nqt) * 64;
    // ---- S[q][key], dP[q][key]: rows q = 16qt + 4g + r, col key = kw
    f32x4 sp[4], dp[4];
#pragma unroll
    for (int qt = 0; qt < 4; ++qt) {
      sp[qt] = dp[qt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < NS; ++s) {
        const bf16x8 qfr = *reinterpret_cast<const bf16x8*>(Ql + (16 * qt + li) * LDR + 32 * s + 8 * g);
        const bf16x8 ofr = *reinterpret_cast<const bf16x8*>(dOl + (16 * qt + li) * LDR + 32 * s + 8 * g);
        sp[qt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(qfr, kf[s], sp[qt], 0, 0, 0);
        dp[qt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ofr, vf[s], dp[qt], 0, 0, 0);
      }
    }
    const bool need_mask = (causal && qa0 < kb0 + 63) || (kb0 + 64 > kvlen) || (qa0 + 64 > S);
#pragma unroll
    for (int qt = 0; qt < 4; ++qt) {
      const f32x4 L = *reinterpret_cast<const f32x4*>(Ls + 16 * qt + 4 * g);
      const f32x4 Dl = *reinterpret_cast<const f32x4*>(Dls + 16 * qt + 4 * g);
#pragma unroll
      for (int r = 0; r < 4; ++r) sp[qt][r] = fexp2(sp[qt][r] * scale_log2 - L[r]);
      if (need_mask) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int q = qa0 + 16 * qt + 4 * g + r;
          sp[qt][r] = (q >= qmin && q < S) ? sp[qt][r] : 0.f;
        }
      }
      if (drp.thresh) {   // dV takes the dropped P, dS = P∘(M∘dP/(1-p) − delta)
        const uint32_t bh = (uint32_t)(b * hq + hk * rep + hw * hp + it / nqt);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const bool keep = drop_hash(drp.s0, drp.s1, bh, qa0 + 16 * qt + 4 * g + r, kw) >= drp.thresh;
          dp[qt][r] = sp[qt][r] * ((keep ? dp[qt][r] * drp.rinv : 0.f) - Dl[r]);
          sp[qt][r] = keep ? sp[qt][r] * drp.rinv : 0.f;
        }
      } else {
#pragma unroll
        for (int r = 0; r < 4; ++r) dp[qt][r] = sp[qt][r] * (dp[qt][r] - Dl[r]);
      }
    }
    // ---- dVᵀ[d][key] += dOᵀ[d][q]·P[q][key] ; dKᵀ += Qᵀ·dS   (permuted-q operand order)
#pragma unroll
    for (int qk = 0; qk < 2; ++qk) {
      const bf16x8 pfr = f2b8(sp[2 * qk], sp[2 * qk + 1]);
      const bf16x8 dsf = f2b8(dp[2 * qk], dp[2 * qk + 1]);
#pragma unroll
      for (int dt = 0; dt < ND; ++dt) {
        const int rr = 32 * qk + 4 * g + (li >> 2), cc = 16 * dt + 4 * (li & 3);
        const bf16x8 of = cat8(tr_read(dOl + rr * LDR + cc), tr_read(dOl + (rr + 16) * LDR + cc));
        const bf16x8 qfr = cat8(tr_read(Ql + rr * LDR + cc), tr_read(Ql + (rr + 16) * LDR + cc));
        dv[dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(of, pfr, dv[dt], 0, 0, 0);
        dk[dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(qfr, dsf, dk[dt], 0, 0, 0);
      }
    }
    }
  }
  if constexpr (HALVES == 2) {  // half 1 hands its partial sums to half 0 through LDS
    __syncthreads();
    f32x4* red = reinterpret_cast<f32x4*>(smem_all);
    if (hw == 1) {
#pragma unroll
      for (int dt = 0; dt < ND; ++dt) {
        red[(2 * dt) * 256 + tid] = dk[dt];
        red[(2 * dt + 1) * 256 + tid] = dv[dt];
      }
    }
    __syncthreads();
    if (hw == 1) return;
#pragma unroll
    for (int dt = 0; dt < ND; ++dt) {
      dk[dt] += red[(2 * dt) * 256 + tid];
      dv[dt] += red[(2 * dt + 1) * 256 + tid];
    }
  }
  // ---- dK (scaled) / dV, summed over the GQA group: lane col key = kw, rows d = 16dt + 4g + r
  if (kw >= S) return;
  if (part >= 0) {   // split block: raw fp32 partials, planes [part][dK | dV][T][hkv·D]
    const size_t plane = (size_t)gridDim.z * S * ldkv;
    float* wk = ws + (size_t)(2 * part) * plane;
    float* wv = wk + plane;
#pragma unroll
    for (int dt = 0; dt < ND; ++dt) {
      const size_t off = (tok0 + kw) * ldkv + hk * D + 16 * dt + 4 * g;
      *reinterpret_cast<f32x4*>(wk + off) = dk[dt];
      *reinterpret_cast<f32x4*>(wv + off) = dv[dt];
    }
    return;
  }
#pragma unroll
  for (int dt = 0; dt < ND; ++dt) {
    const size_t off = (tok0 + kw) * ldkv + hk * D + 16 * dt + 4 * g;
    bf16x4 ok, ov;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      ok[r] = (bf16)(dk[dt][r] * scale);
      ov[r] = (bf16)dv[dt][r];
    }
    *reinterpret_cast<bf16x4*>(dK + off) = ok;
    *reinterpret_cast<bf16x4*>(dV + off) = ov;
  }
}

// dK = scale·(P0 + P1), dV = P0 + P1 for the keys of the split blocks (keys < nsplit·64 of every batch)
__global__ __launch_bounds__(256) void attn_dkv_fin_k(const float* __restrict__ ws, bf16* __restrict__ dK,
                                                     bf16* __restrict__ dV, int B, int S, int ldkv, int rows,
                                                     float scale) {
  const size_t per_b = (size_t)rows * ldkv;
  const size_t i = ((size_t)blockIdx.x * 256 + threadIdx.x) * 4;
  if (i >= (size_t)B * per_b) return;
  const size_t b = i / per_b, r = i - b * per_b;
  const size_t off = b * (size_t)S * ldkv + r;
  const size_t plane = (size_t)B * S * ldkv;
  const f32x4 k = *reinterpret_cast<const f32x4*>(ws + off) + *reinterpret_cast<const f32x4*>(ws + 2 * plane + off);
  const f32x4 v = *reinterpret_cast<const f32x4*>(ws + plane + off) +
                  *reinterpret_cast<const f32x4*>(ws + 3 * plane + off);
  bf16x4 ok, ov;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    ok[e] = (bf16)(k[e] * scale);
    ov[e] = (bf16)v[e];
  }
  *reinterpret_cast<bf16x4*>(dK + off) = ok;
  *reinterpret_cast<bf16x4*>(dV + off) = ov;
}

}  // namespace

// key blocks of the causal dK/dV grid split over two workgroups (0: none).  Split when the grid is
// at most ~2 workgroups per CU (larger grids already balance over several waves of workgroups) and
// S >= 1024: blocks whose query-tile count exceeds half the blocks.  Measured (same box, interleaved,
// scripts/experiments/gpu_dkv_split_ab.sh): [1, 2048, 32, 8, 128] bwd 283 -> 260 us; at the bench
// shape [4, 512, ...] the 4-tile units' fixed cost and the fp32 partial round trip lose (92 -> 102 us),
// hence the S threshold (still the best after the LDS re-pad: profiles/r4/attention_knobs_ab.txt, S = 2048 bwd 236 vs 262 us unsplit).
// Also split when the unsplit grid would fill at most half the CUs (one 512-thread workgroup per CU): the
// sequential-GA micro-batch [2, 512, 8 kv-heads] is 128 workgroups (profiles/r5/attention_dkv_split_b2.txt).
// per-wave phase timestamps of the D = 128 dK/dV kernel (debug; see attn_bwd_dkv128_k TRACE): while set, the
// dK/dV launches write [grid · 8 waves · 264] u64 into this buffer instead of splitting key blocks
static float* g_attn_trace = nullptr;
void attn_set_trace(void* p) { g_attn_trace = (float*)p; }

int attn_dkv_nsplit(int B, int S, int hkv, int causal) {
  const int nb = (S + 63) / 64;
  const long grid = (long)B * hkv * nb;
  if (!causal || nb < 2) return 0;
  if (grid > 512 || (nb < 16 && grid > 128)) return 0;
  return nb - (nb + 1) / 2;   // kb with nb - kb > ceil(nb / 2)
}

static DropParams make_drop(float p, uint64_t seed) {
  DropParams d{(uint32_t)seed, (uint32_t)(seed >> 32), 0u, 1.f};
  if (p > 0.f) {
    d.thresh = (uint32_t)std::min(4294967295.0, (double)p * 4294967296.0);
    d.rinv = 1.f / (1.f - p);
  }
  return d;
}

// the head dims below 128 (128 has its own 32x32x16 forward / dQ kernels)
#define LIPA_ATTN_D3(D, ...)                \
  switch (D) {                              \
    case 32: { constexpr int DD = 32; __VA_ARGS__; } break;   \
    case 64: { constexpr int DD = 64; __VA_ARGS__; } break;   \
    default: { constexpr int DD = 96; __VA_ARGS__; } break;   \
  }

// register prefetch depth per kernel (measured, profiles/attention_fwd_bwd.txt, re-checked after the LDS
// re-pad in profiles/r4/attention_knobs_ab.txt): fwd 1 (depth 2 spills), dQ 2, dK/dV 1

void launch_attn_fwd(const void* q, const void* k, const void* v, int ldq, int ldk, int ldv, const int* kv_lens,
                     const int* q_offs, void* o, float* lse, int B, int Sq, int Skv, int kv_rows, int hq, int hkv,
                     int D, int causal, float scale, float p_drop, uint64_t seed, hipStream_t st) {
  const DropParams dp = make_drop(p_drop, seed);
  // 128-query workgroups (32 queries per wave, QT = 2) reuse each K/V tile for twice the queries;
  // 64-query ones (QT = 1) give the causal grid more, smaller blocks to balance — measured slower at
  // S = 512 / 8192 and equal at 2048 (profiles/attention_fwd_bwd.txt, profiles/r4/attention_knobs_ab.txt).
  const int qt = 2;
  dim3 grid((Sq + 64 * qt - 1) / (64 * qt), hq, B), blk(256);
  const float sl2 = scale * LOG2E;
  if (D == 128) {   // the 32x32x16 form with LDS-DMA K / V tiles (attn_fwd128_k); other head dims: attn_fwd_k
#define F128(DR)                                                                                              \
  attn_fwd128_k<DR><<<grid, blk, 0, st>>>((const bf16*)q, (const bf16*)k, (const bf16*)v, ldq, ldk, ldv, kv_lens, \
                                          q_offs, (bf16*)o, lse, Sq, Skv, kv_rows, hq, hkv,                    \
                                          causal ? 1 | (attn_lpt() << 1) : 0, sl2, dp)
    if (dp.thresh) F128(true); else F128(false);
#undef F128
    LIPA_CHECK_LAUNCH();
    return;
  }
#define FWD(PFV, QTV)                                                                                      \
  attn_fwd_k<DD, PFV, QTV><<<grid, blk, 0, st>>>((const bf16*)q, (const bf16*)k, (const bf16*)v,                 \
                                                ldq, ldk, ldv, kv_lens, q_offs, (bf16*)o, lse, Sq, Skv,          \
                                                kv_rows, hq, hkv, causal ? 1 | (attn_lpt() << 1) : 0, sl2, dp)
  LIPA_ATTN_D3(D, FWD(1, 2));
#undef FWD
  LIPA_CHECK_LAUNCH();
}

void launch_attn_bwd(const void* dout, const void* q, const void* k, const void* v, const void* o, const float* lse,
                     const int* kv_lens, int ldq, int ldk, int ldv, void* dq, void* dk, void* dv, float* delta, int B,
                     int S, int hq, int hkv, int D, int causal, float scale, float p_drop, uint64_t seed, float* ws,
                     hipStream_t st) {
  const float sl2 = scale * LOG2E;
  const DropParams dp = make_drop(p_drop, seed);
  const int nb = (S + 63) / 64;
  const bool trace = g_attn_trace && D == 128;
  const int nsplit = ws && !trace ? attn_dkv_nsplit(B, S, hkv, causal) : 0;
  dim3 gq(nb, hq, B), gkv(nb + nsplit, hkv, B), blk(256);
#define DKV(DD, PFKV)                                                                                             \
  if ((hq / hkv) % 2 == 0)                                                                                       \
    attn_bwd_dkv_k<DD, 2, PFKV><<<gkv, 512, 0, st>>>((const bf16*)dout, (const bf16*)q, (const bf16*)k,           \
                                                      (const bf16*)v, lse, delta, kv_lens, ldq, ldk, ldv, (bf16*)dk, \
                                                      (bf16*)dv, S, hq, hkv, causal, scale, sl2, dp, ws, nsplit);   \
  else                                                                                                           \
    attn_bwd_dkv_k<DD, 1, PFKV><<<gkv, 256, 0, st>>>((const bf16*)dout, (const bf16*)q, (const bf16*)k,           \
                                                      (const bf16*)v, lse, delta, kv_lens, ldq, ldk, ldv, (bf16*)dk, \
                                                      (bf16*)dv, S, hq, hkv, causal, scale, sl2, dp, ws, nsplit)
// dQ first (it writes delta), then dK/dV
#define RUN(DD, PFQ, PFKV)                                                                                        \
  attn_bwd_dq_k<DD, PFQ><<<gq, blk, 0, st>>>((const bf16*)dout, (const bf16*)o, (const bf16*)q, (const bf16*)k,   \
                                             (const bf16*)v, lse, delta, kv_lens, ldq, ldk, ldv, (bf16*)dq, S, hq, \
                                             hkv, causal ? 1 | (attn_lpt() << 1) : 0, scale, sl2, dp);            \
  DKV(DD, PFKV);
  if (D == 128) {   // the 32x32x16 forms: dQ (attn_bwd_dq128_k) and dK/dV (attn_bwd_dkv128_k), LDS-DMA operand tiles
    dim3 gq2((S + 127) / 128, hq, B);
#define DQ2(DR)                                                                                                  \
  attn_bwd_dq128_k<DR><<<gq2, blk, 0, st>>>((const bf16*)dout, (const bf16*)o, (const bf16*)q, (const bf16*)k,   \
                                            (const bf16*)v, lse, delta, kv_lens, ldq, ldk, ldv, (bf16*)dq, S, hq, \
                                            hkv, causal ? 1 | (attn_lpt() << 1) : 0, scale, sl2, dp)
    if (dp.thresh) DQ2(true); else DQ2(false);
#undef DQ2
#define DKV3(DR)                                                                                                 \
  attn_bwd_dkv128_k<DR><<<gkv, 512, 0, st>>>((const bf16*)dout, (const bf16*)q, (const bf16*)k, (const bf16*)v,   \
                                             lse, delta, kv_lens, ldq, ldk, ldv, (bf16*)dk, (bf16*)dv, S, hq, hkv, \
                                             causal, scale, sl2, dp, ws, nsplit)
    if (trace)
      attn_bwd_dkv128_k<false, true><<<gkv, 512, 0, st>>>((const bf16*)dout, (const bf16*)q, (const bf16*)k,
                                                          (const bf16*)v, lse, delta, kv_lens, ldq, ldk, ldv,
                                                          (bf16*)dk, (bf16*)dv, S, hq, hkv, causal, scale, sl2, dp,
                                                          g_attn_trace, 0);
    else if (dp.thresh) DKV3(true); else DKV3(false);
#undef DKV3
  } else {
    LIPA_ATTN_D3(D, RUN(DD, 2, 1));   // prefetch depth dQ 2, dK/dV 1
  }
#undef RUN
#undef DKV
  if (nsplit > 0) {
    const int ldkv = hkv * D, rows = std::min(nsplit * 64, S);
    const size_t n4 = (size_t)B * rows * ldkv / 4;
    attn_dkv_fin_k<<<(unsigned)((n4 + 255) / 256), 256, 0, st>>>(ws, (bf16*)dk, (bf16*)dv, B, S, ldkv, rows, scale);
  }
  LIPA_CHECK_LAUNCH();
}
