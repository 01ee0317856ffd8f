// Flash attention forward / backward for gfx950: causal, GQA by head
// broadcast (K/V never repeated), right-padding via per-batch kv length, bf16 I/O, fp32
// online softmax.  Token-major layout: q [T, Hq*D], k/v [T, Hkv*D] with arbitrary row
// stride (k/v may be strided views into the fused qkv projection).
//
// Forward: 256-thread workgroup = 4 waves × 32 queries of one (batch, head).  Scores are
// computed SWAPPED, Sᵀ = K·Qᵀ with v_mfma_f32_16x16x32_bf16 (K tile from LDS, Q fragments
// held in registers), so each lane owns ONE query: the row max / row sum are lane-local
// plus two shuffles, and the probabilities are already the B operand of Oᵀ = Vᵀ·Pᵀ in a
// permuted key order (no LDS round trip for P).  V's matching operand comes from the
// gfx950 transposed LDS read ds_read_b64_tr_b16.  K/V tiles (64 keys) are register-staged
// one tile ahead into double-buffered LDS (one barrier per tile).
//
// Backward: workgroup = 4 waves × 16 keys (a 64-key block) of one (batch, q-head); K and V
// fragments stay in registers for the whole sweep, dKᵀ/dVᵀ accumulate in registers over all
// query tiles (no atomics), P is recomputed from the saved log-sum-exp, dQ is accumulated
// with fp32 atomics (the dQ sum spans key blocks).  GQA partial dK/dV per q-head are summed
// in a finalize pass (deterministic).
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

// ============================================================================ forward
template <int D>
__global__ __launch_bounds__(256) void attn_fwd_k(const bf16* __restrict__ Q, const bf16* __restrict__ K,
                                                  const bf16* __restrict__ V, int ldq, int ldk, int ldv,
                                                  const int* __restrict__ kv_lens, bf16* __restrict__ O,
                                                  float* __restrict__ lse, int S, int hq, int hkv, int causal,
                                                  float scale_log2) {
  constexpr int LDR = D + 8;        // padded LDS row (elements)
  constexpr int CH = D / 8;         // 16-B chunks per row
  constexpr int TILE = 64 * LDR;    // elements per K or V tile
  constexpr int NS = D / 32;        // k-steps over head dim
  constexpr int ND = D / 16;        // d-subtiles of O
  constexpr int LOADS = 64 * CH / 256;
  __shared__ __attribute__((aligned(16))) bf16 smem[4 * TILE];  // K0 V0 K1 V1

  const int nqb = (S + 127) / 128;
  const int qb = nqb - 1 - blockIdx.x;  // heavy (late, causal) blocks first
  const int h = blockIdx.y, b = blockIdx.z;
  const int hk = h / (hq / hkv);
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, g = lane >> 4, li = lane & 15;
  const int q0 = qb * 128 + 32 * w;
  const int kvlen = kv_lens ? kv_lens[b] : S;
  const size_t tok0 = (size_t)b * S;

  // Q fragments (B operand of Sᵀ = K·Qᵀ): Q[q0 + 16qt + li][32s + 8g + j]
  bf16x8 qf[2][NS];
#pragma unroll
  for (int qt = 0; qt < 2; ++qt) {
    int q = q0 + 16 * qt + li;
    q = q < S ? q : S - 1;
#pragma unroll
    for (int s = 0; s < NS; ++s)
      qf[qt][s] = *reinterpret_cast<const bf16x8*>(Q + (tok0 + q) * ldq + h * D + 32 * s + 8 * g);
  }

  int kend = causal ? min(S, qb * 128 + 128) : S;
  kend = min(kend, kvlen);
  const int nt = (kend + 63) / 64;

  f32x4 acc[ND][2];
#pragma unroll
  for (int dt = 0; dt < ND; ++dt) acc[dt][0] = acc[dt][1] = f32x4{0.f, 0.f, 0.f, 0.f};
  float m_run[2] = {-INFINITY, -INFINITY}, l_run[2] = {0.f, 0.f};

  bf16x8 kr[LOADS], vr[LOADS];
  auto load_tile = [&](int t) {
#pragma unroll
    for (int p = 0; p < LOADS; ++p) {
      const int ci = p * 256 + threadIdx.x;
      const int row = ci / CH, ch = ci % CH;
      int key = t * 64 + row;
      key = key < S ? key : S - 1;
      kr[p] = *reinterpret_cast<const bf16x8*>(K + (tok0 + key) * ldk + hk * D + ch * 8);
      vr[p] = *reinterpret_cast<const bf16x8*>(V + (tok0 + key) * ldv + hk * D + ch * 8);
    }
  };
  auto store_tile = [&](int buf) {
    bf16* Kl = smem + buf * 2 * TILE;
    bf16* Vl = Kl + TILE;
#pragma unroll
    for (int p = 0; p < LOADS; ++p) {
      const int ci = p * 256 + threadIdx.x;
      const int row = ci / CH, ch = ci % CH;
      *reinterpret_cast<bf16x8*>(Kl + row * LDR + ch * 8) = kr[p];
      *reinterpret_cast<bf16x8*>(Vl + row * LDR + ch * 8) = vr[p];
    }
  };

  if (nt > 0) load_tile(0);
  for (int t = 0; t < nt; ++t) {
    store_tile(t & 1);
    __syncthreads();
    if (t + 1 < nt) load_tile(t + 1);
    const bf16* Kl = smem + (t & 1) * 2 * TILE;
    const bf16* Vl = Kl + TILE;
    const int k0 = t * 64;
    // ---- Sᵀ[key][q] for 4 key-subtiles × 2 query-subtiles
    f32x4 sc[4][2];
#pragma unroll
    for (int kt = 0; kt < 4; ++kt) {
      sc[kt][0] = sc[kt][1] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < NS; ++s) {
        const bf16x8 kf = *reinterpret_cast<const bf16x8*>(Kl + (16 * kt + li) * LDR + 32 * s + 8 * g);
        sc[kt][0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf, qf[0][s], sc[kt][0], 0, 0, 0);
        sc[kt][1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf, qf[1][s], sc[kt][1], 0, 0, 0);
      }
    }
    // ---- masks + online softmax (lane owns query q0 + 16qt + li; keys k0 + 16kt + 4g + r)
    const bool need_mask = (causal && k0 + 63 > q0) || (k0 + 64 > kvlen);
    bf16x8 pf[2][2];
#pragma unroll
    for (int qt = 0; qt < 2; ++qt) {
      const int qa = q0 + 16 * qt + li;
      float mx = -INFINITY;
#pragma unroll
      for (int kt = 0; kt < 4; ++kt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float v = sc[kt][qt][r] * scale_log2;
          if (need_mask) {
            const int ka = k0 + 16 * kt + 4 * g + r;
            if ((causal && ka > qa) || ka >= kvlen) v = -INFINITY;
          }
          sc[kt][qt][r] = v;
          mx = fmaxf(mx, v);
        }
      mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
      mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
      const float mn = fmaxf(m_run[qt], mx);
      const float alpha = (mn == -INFINITY) ? 1.f : exp2f(m_run[qt] - mn);
      float rs = 0.f;
#pragma unroll
      for (int kt = 0; kt < 4; ++kt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float p = (mn == -INFINITY) ? 0.f : exp2f(sc[kt][qt][r] - mn);
          sc[kt][qt][r] = p;
          rs += p;
        }
      rs += __shfl_xor(rs, 16, 64);
      rs += __shfl_xor(rs, 32, 64);
      l_run[qt] = l_run[qt] * alpha + rs;
      m_run[qt] = mn;
#pragma unroll
      for (int dt = 0; dt < ND; ++dt) acc[dt][qt] *= alpha;
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
        acc[dt][0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vf, pf[0][kb], acc[dt][0], 0, 0, 0);
        acc[dt][1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vf, pf[1][kb], acc[dt][1], 0, 0, 0);
      }
    }
  }
  // ---- epilogue: O[q][16dt + 4g + r] = acc / l ; lse = (m + log2 l) * ln2
#pragma unroll
  for (int qt = 0; qt < 2; ++qt) {
    const int q = q0 + 16 * qt + li;
    if (q >= S) continue;
    const float inv = l_run[qt] > 0.f ? 1.f / l_run[qt] : 0.f;
#pragma unroll
    for (int dt = 0; dt < ND; ++dt) {
      bf16x4 o;
#pragma unroll
      for (int r = 0; r < 4; ++r) o[r] = (bf16)(acc[dt][qt][r] * inv);
      *reinterpret_cast<bf16x4*>(O + (tok0 + q) * (size_t)(hq * D) + h * D + 16 * dt + 4 * g) = o;
    }
    if (g == 0)
      lse[((size_t)b * hq + h) * S + q] =
          l_run[qt] > 0.f ? (m_run[qt] + log2f(l_run[qt])) * 0.6931471805599453f : INFINITY;
  }
}

// ============================================================================ backward
// delta[b][h][q] = Σ_d dO·O
template <int D>
__global__ __launch_bounds__(256) void attn_bwd_pre_k(const bf16* __restrict__ dO, const bf16* __restrict__ O,
                                                      float* __restrict__ delta, int B, int S, int hq) {
  const int idx = blockIdx.x * 4 + (threadIdx.x >> 6);  // one wave per (token, head)
  const int lane = threadIdx.x & 63;
  if (idx >= B * S * hq) return;
  const int t = idx / hq, h = idx % hq;
  float s = 0.f;
  for (int d = lane * 2; d < D; d += 128) {
    const size_t off = (size_t)t * hq * D + h * D + d;
    s += (float)dO[off] * (float)O[off] + (float)dO[off + 1] * (float)O[off + 1];
  }
  s = wave_sum(s);
  if (lane == 0) {
    const int b = t / S, q = t % S;
    delta[((size_t)b * hq + h) * S + q] = s;
  }
}

template <int D>
__global__ __launch_bounds__(256) void attn_bwd_k(const bf16* __restrict__ dO, const bf16* __restrict__ Q,
                                                  const bf16* __restrict__ K, const bf16* __restrict__ V,
                                                  const float* __restrict__ lse, const float* __restrict__ delta,
                                                  const int* __restrict__ kv_lens, int ldq, int ldk, int ldv,
                                                  float* __restrict__ dqacc, float* __restrict__ dkf,
                                                  float* __restrict__ dvf, int S, int hq, int hkv, int causal,
                                                  float scale, float scale_log2) {
  constexpr int LDR = D + 8;
  constexpr int NS = D / 32, ND = D / 16;
  constexpr int LDS_S = 64 + 8;
  __shared__ __attribute__((aligned(16))) bf16 Kl[64 * LDR];
  __shared__ __attribute__((aligned(16))) bf16 Ql[32 * LDR];
  __shared__ __attribute__((aligned(16))) bf16 dOl[32 * LDR];
  __shared__ __attribute__((aligned(16))) bf16 dSl[32 * LDS_S];

  const int nkb = S / 64;
  const int kbi = blockIdx.x;
  const int h = blockIdx.y, b = blockIdx.z;
  const int hk = h / (hq / hkv);
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, g = lane >> 4, li = lane & 15;
  const int kb0 = kbi * 64;
  const int kw = kb0 + 16 * w + li;  // this lane's key (column of S / dP tiles)
  const int kvlen = kv_lens ? kv_lens[b] : S;
  const size_t tok0 = (size_t)b * S;
  (void)nkb;

  // K block → LDS (for dQ) ; K/V fragments (B operands) → registers
  for (int ci = threadIdx.x; ci < 64 * (D / 8); ci += 256) {
    const int row = ci / (D / 8), ch = ci % (D / 8);
    *reinterpret_cast<bf16x8*>(Kl + row * LDR + ch * 8) =
        *reinterpret_cast<const bf16x8*>(K + (tok0 + kb0 + row) * ldk + hk * D + ch * 8);
  }
  bf16x8 kf[NS], vf[NS];
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    kf[s] = *reinterpret_cast<const bf16x8*>(K + (tok0 + kw) * ldk + hk * D + 32 * s + 8 * g);
    vf[s] = *reinterpret_cast<const bf16x8*>(V + (tok0 + kw) * ldv + hk * D + 32 * s + 8 * g);
  }
  f32x4 dv[ND], dk[ND];
#pragma unroll
  for (int dt = 0; dt < ND; ++dt) dv[dt] = dk[dt] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int qt_start = causal ? kb0 / 32 : 0;
  const int nqt = S / 32;
  const float* lse_bh = lse + ((size_t)b * hq + h) * S;
  const float* del_bh = delta + ((size_t)b * hq + h) * S;

  for (int qtile = qt_start; qtile < nqt; ++qtile) {
    const int qa0 = qtile * 32;
    __syncthreads();  // previous iteration's LDS reads done
    for (int ci = threadIdx.x; ci < 32 * (D / 8); ci += 256) {
      const int row = ci / (D / 8), ch = ci % (D / 8);
      const size_t tq = tok0 + qa0 + row;
      *reinterpret_cast<bf16x8*>(Ql + row * LDR + ch * 8) =
          *reinterpret_cast<const bf16x8*>(Q + tq * ldq + h * D + ch * 8);
      *reinterpret_cast<bf16x8*>(dOl + row * LDR + ch * 8) =
          *reinterpret_cast<const bf16x8*>(dO + tq * (size_t)(hq * D) + h * D + ch * 8);
    }
    __syncthreads();
    // ---- S[q][key], dP[q][key]: rows q = 16qt + 4g + r, col key = kw
    f32x4 sp[2], dp[2];
#pragma unroll
    for (int qt = 0; qt < 2; ++qt) {
      sp[qt] = dp[qt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < NS; ++s) {
        const bf16x8 qf = *reinterpret_cast<const bf16x8*>(Ql + (16 * qt + li) * LDR + 32 * s + 8 * g);
        const bf16x8 of = *reinterpret_cast<const bf16x8*>(dOl + (16 * qt + li) * LDR + 32 * s + 8 * g);
        sp[qt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(qf, kf[s], sp[qt], 0, 0, 0);
        dp[qt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(of, vf[s], dp[qt], 0, 0, 0);
      }
    }
    f32x4 pp[2], ds[2];
#pragma unroll
    for (int qt = 0; qt < 2; ++qt) {
      const int qb4 = qa0 + 16 * qt + 4 * g;
      const f32x4 L = *reinterpret_cast<const f32x4*>(lse_bh + qb4);
      const f32x4 Dl = *reinterpret_cast<const f32x4*>(del_bh + qb4);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int qa = qb4 + r;
        float p = exp2f(sp[qt][r] * scale_log2 - L[r] * LOG2E);
        if ((causal && kw > qa) || kw >= kvlen) p = 0.f;
        pp[qt][r] = p;
        ds[qt][r] = p * (dp[qt][r] - Dl[r]);
      }
    }
    // permuted-q operand order j ↔ 16(j>>2) + 4g + (j&3)
    const bf16x8 pfr = f2b8(pp[0], pp[1]);
    const bf16x8 dsf = f2b8(ds[0], ds[1]);
    // ---- dVᵀ[d][key] += dOᵀ[d][q]·P[q][key] ; dKᵀ += Qᵀ·dS
#pragma unroll
    for (int dt = 0; dt < ND; ++dt) {
      const int rr = 4 * g + (li >> 2), cc = 16 * dt + 4 * (li & 3);
      const bf16x8 of = cat8(tr_read(dOl + rr * LDR + cc), tr_read(dOl + (rr + 16) * LDR + cc));
      const bf16x8 qf = cat8(tr_read(Ql + rr * LDR + cc), tr_read(Ql + (rr + 16) * LDR + cc));
      dv[dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(of, pfr, dv[dt], 0, 0, 0);
      dk[dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(qf, dsf, dk[dt], 0, 0, 0);
    }
    // ---- dS → LDS [q][key] for the dQ product
#pragma unroll
    for (int qt = 0; qt < 2; ++qt)
#pragma unroll
      for (int r = 0; r < 4; ++r) dSl[(16 * qt + 4 * g + r) * LDS_S + 16 * w + li] = (bf16)ds[qt][r];
    __syncthreads();
    // ---- dQ[q][d] += dS[q][key]·K[key][d] over the 64-key block; wave w: qt = w>>1, 4 d-subtiles
    {
      const int qt = w >> 1;
#pragma unroll
      for (int i = 0; i < ND / 2; ++i) {
        const int dt = (w & 1) * (ND / 2) + i;
        f32x4 a = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kb = 0; kb < 2; ++kb) {
          const bf16x8 sf = *reinterpret_cast<const bf16x8*>(dSl + (16 * qt + li) * LDS_S + 32 * kb + 8 * g);
          const int rr = 32 * kb + 8 * g + (li >> 2), cc = 16 * dt + 4 * (li & 3);
          const bf16x8 kt = cat8(tr_read(Kl + rr * LDR + cc), tr_read(Kl + (rr + 4) * LDR + cc));
          a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(sf, kt, a, 0, 0, 0);
        }
        // C layout: col d = 16dt + li, rows q = 16qt + 4g + r
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const size_t tq = tok0 + qa0 + 16 * qt + 4 * g + r;
          atomicAdd(dqacc + tq * (size_t)(hq * D) + h * D + 16 * dt + li, a[r] * scale);
        }
      }
    }
  }
  // ---- write per-q-head dK (scaled) / dV (fp32): lane col key = kw, rows d = 16dt + 4g + r
#pragma unroll
  for (int dt = 0; dt < ND; ++dt) {
    const size_t off = (tok0 + kw) * (size_t)(hq * D) + h * D + 16 * dt + 4 * g;
    *reinterpret_cast<f32x4*>(dkf + off) = dk[dt] * scale;
    *reinterpret_cast<f32x4*>(dvf + off) = dv[dt];
  }
}

// dq = bf16(dqacc); dk/dv = bf16(Σ over the GQA group of per-q-head partials)
template <int D>
__global__ __launch_bounds__(256) void attn_bwd_fin_k(const float* __restrict__ dqacc, const float* __restrict__ dkf,
                                                      const float* __restrict__ dvf, bf16* __restrict__ dq,
                                                      bf16* __restrict__ dk, bf16* __restrict__ dv, int T, int hq,
                                                      int hkv) {
  const size_t n1 = (size_t)T * hq * D;
  const size_t n2 = (size_t)T * hkv * D;
  const int rep = hq / hkv;
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n1; i += (size_t)gridDim.x * 256) {
    dq[i] = (bf16)dqacc[i];
    if (i < n2) {
      const size_t t = i / (hkv * D), rem = i % (hkv * D);
      const int hk = rem / D, d = rem % D;
      float a = 0.f, c = 0.f;
      for (int r = 0; r < rep; ++r) {
        const size_t o = t * (size_t)(hq * D) + (size_t)(hk * rep + r) * D + d;
        a += dkf[o];
        c += dvf[o];
      }
      dk[i] = (bf16)a;
      dv[i] = (bf16)c;
    }
  }
}

}  // namespace

void launch_attn_fwd(const void* q, const void* k, const void* v, int ldq, int ldk, int ldv, const int* kv_lens,
                     void* o, float* lse, int B, int S, int hq, int hkv, int D, int causal, float scale,
                     hipStream_t st) {
  dim3 grid((S + 127) / 128, hq, B), blk(256);
  const float sl2 = scale * LOG2E;
  if (D == 128)
    attn_fwd_k<128><<<grid, blk, 0, st>>>((const bf16*)q, (const bf16*)k, (const bf16*)v, ldq, ldk, ldv, kv_lens,
                                          (bf16*)o, lse, S, hq, hkv, causal, sl2);
  else
    attn_fwd_k<64><<<grid, blk, 0, st>>>((const bf16*)q, (const bf16*)k, (const bf16*)v, ldq, ldk, ldv, kv_lens,
                                         (bf16*)o, lse, S, hq, hkv, causal, sl2);
  LIPA_CHECK_LAUNCH();
}

void launch_attn_bwd(const void* dout, const void* q, const void* k, const void* v, const void* o, const float* lse,
                     const int* kv_lens, int ldq, int ldk, int ldv, void* dq, void* dk, void* dv, float* dqacc,
                     float* delta, float* dkf, float* dvf, int B, int S, int hq, int hkv, int D, int causal,
                     float scale, hipStream_t st) {
  const int rows = B * S * hq;
  const float sl2 = scale * LOG2E;
  dim3 grid(S / 64, hq, B), blk(256);
  const int T = B * S;
  size_t nfin = (size_t)T * hq * D;
  int gfin = (int)((nfin + 255) / 256 < 4096 ? (nfin + 255) / 256 : 4096);
#define RUN(DD)                                                                                                    \
  attn_bwd_pre_k<DD><<<(rows + 3) / 4, 256, 0, st>>>((const bf16*)dout, (const bf16*)o, delta, B, S, hq);          \
  attn_bwd_k<DD><<<grid, blk, 0, st>>>((const bf16*)dout, (const bf16*)q, (const bf16*)k, (const bf16*)v, lse,     \
                                       delta, kv_lens, ldq, ldk, ldv, dqacc, dkf, dvf, S, hq, hkv, causal, scale,  \
                                       sl2);                                                                       \
  attn_bwd_fin_k<DD><<<gfin, 256, 0, st>>>(dqacc, dkf, dvf, (bf16*)dq, (bf16*)dk, (bf16*)dv, T, hq, hkv)
  if (D == 128) {
    RUN(128);
  } else {
    RUN(64);
  }
#undef RUN
  LIPA_CHECK_LAUNCH();
}
