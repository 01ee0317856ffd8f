// Generation-time kernels: KV-cache decode attention and the fused
// logits → token sampler.
//
// decode attention ("flash-decoding" on CDNA4): one query token per sequence against its
// contiguous KV cache [B, Smax, Hkv*D].  Decode is HBM-bound on the cache read, so the design
// goal is to stream K/V once with 16-B loads and to spread one sequence over many CUs:
//  * grid (splits, Hkv, B); the split count is chosen on the host for occupancy (~2048
//    workgroups) and each workgroup takes 1/splits of its sequence's LIVE length (read on the
//    device), for ONE kv head and all of its G = Hq/Hkv query heads (K/V read once per group);
//  * D/8 lanes hold one key row (8 bf16 = 16 B per lane); a wave covers 64/(D/8) keys per
//    step, the dot products finish with log2(D/8) xor-shuffles; online softmax per lane slot;
//  * two keys per lane slot are loaded before either is consumed (memory-level parallelism);
//  * slots merge by xor shuffles inside the wave, waves through LDS, splits by a second tiny
//    kernel (log-sum-exp merge over the splits that had keys).
// Per-row valid lengths (right-padded batches / different prompt lengths) come from lens[B].
//
// sampler: one 1024-thread workgroup per row; repetition penalty (HF semantics: applied once
// per distinct history token), temperature, top-k and top-p by value-threshold bisection over
// the row (no sort of the 151,936-entry vocabulary), then an inverse-CDF draw from a
// counter-based RNG (splitmix64 of (key, row)) with a block prefix scan.  Greedy = argmax.
#include "common.h"

#include <algorithm>

using namespace lipa;

namespace {

constexpr int DEC_THR = 256;
constexpr int DEC_TARGET_WG = 2048;   // ≈ 8 workgroups per CU in flight

// keys per split for a sequence of `len` keys: multiple of 16 (one workgroup step)
__device__ __forceinline__ int split_chunk(int len, int nsplit) { return ((len + nsplit - 1) / nsplit + 15) & ~15; }

template <int D, int G>
__global__ __launch_bounds__(DEC_THR) void decode_attn_partial_k(const bf16* __restrict__ q,
                                                                 const bf16* __restrict__ kc,
                                                                 const bf16* __restrict__ vc,
                                                                 const int* __restrict__ lens, float* __restrict__ opart,
                                                                 float* __restrict__ mpart, float* __restrict__ lpart,
                                                                 int Smax, int hq, int hkv, int nsplit, float scale) {
  constexpr int LPK = D / 8;          // lanes per key row (16 B each)
  constexpr int KPW = 64 / LPK;       // keys per wave step
  constexpr int NSLOT = 4 * KPW;      // keys per workgroup step
  const int split = blockIdx.x, kh = blockIdx.y, b = blockIdx.z;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int sw = lane / LPK, e = lane % LPK;   // key slot within the wave, 8-element piece of the row
  const int len = lens[b];
  const int chunk = split_chunk(len, nsplit);   // splits divide the LIVE length evenly
  const int k0 = split * chunk, k1 = min(k0 + chunk, len);
  if (k0 >= len) return;              // empty split: the merge kernel never reads it

  float qf[G][8];
#pragma unroll
  for (int g = 0; g < G; ++g) {
    const bf16x8 v = *reinterpret_cast<const bf16x8*>(q + ((size_t)b * hq + kh * G + g) * D + e * 8);
#pragma unroll
    for (int j = 0; j < 8; ++j) qf[g][j] = (float)v[j] * scale;
  }
  float m[G], l[G], acc[G][8];
#pragma unroll
  for (int g = 0; g < G; ++g) {
    m[g] = -INFINITY;
    l[g] = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[g][j] = 0.f;
  }
  const size_t row_stride = (size_t)hkv * D;
  const bf16* kb = kc + (size_t)b * Smax * row_stride + kh * D + e * 8;
  const bf16* vb = vc + (size_t)b * Smax * row_stride + kh * D + e * 8;

  auto consume = [&](const bf16x8& kv, const bf16x8& vv) {
    float s[G];
#pragma unroll
    for (int g = 0; g < G; ++g) {
      float d = 0.f;
#pragma unroll
      for (int j = 0; j < 8; ++j) d += qf[g][j] * (float)kv[j];
#pragma unroll
      for (int o = LPK / 2; o > 0; o >>= 1) d += __shfl_xor(d, o, 64);
      s[g] = d;
    }
#pragma unroll
    for (int g = 0; g < G; ++g) {
      const float mn = fmaxf(m[g], s[g]);
      const float c = __expf(m[g] - mn), p = __expf(s[g] - mn);
      l[g] = l[g] * c + p;
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[g][j] = acc[g][j] * c + p * (float)vv[j];
      m[g] = mn;
    }
  };
  // two keys per lane-slot in flight: both K/V pairs are loaded before either is consumed
  const int my0 = k0 + w * KPW + sw;
  int t = my0;
  for (; t + NSLOT < k1; t += 2 * NSLOT) {
    const bf16x8 ka = *reinterpret_cast<const bf16x8*>(kb + (size_t)t * row_stride);
    const bf16x8 va = *reinterpret_cast<const bf16x8*>(vb + (size_t)t * row_stride);
    const bf16x8 kb2 = *reinterpret_cast<const bf16x8*>(kb + (size_t)(t + NSLOT) * row_stride);
    const bf16x8 vb2 = *reinterpret_cast<const bf16x8*>(vb + (size_t)(t + NSLOT) * row_stride);
    consume(ka, va);
    consume(kb2, vb2);
  }
  if (t < k1) {
    const bf16x8 ka = *reinterpret_cast<const bf16x8*>(kb + (size_t)t * row_stride);
    const bf16x8 va = *reinterpret_cast<const bf16x8*>(vb + (size_t)t * row_stride);
    consume(ka, va);
  }
  // merge the KPW slots of this wave with xor shuffles (lanes LPK apart hold the same piece e)
#pragma unroll
  for (int o = LPK; o < 64; o <<= 1) {
#pragma unroll
    for (int g = 0; g < G; ++g) {
      const float mo = __shfl_xor(m[g], o, 64), lo = __shfl_xor(l[g], o, 64);
      const float mn = fmaxf(m[g], mo);
      const float c0 = mn == -INFINITY ? 0.f : __expf(m[g] - mn), c1 = mn == -INFINITY ? 0.f : __expf(mo - mn);
      l[g] = l[g] * c0 + lo * c1;
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[g][j] = acc[g][j] * c0 + __shfl_xor(acc[g][j], o, 64) * c1;
      m[g] = mn;
    }
  }
  // then the 4 waves through LDS
  __shared__ float sm[4][G], sl[4][G];
  __shared__ float sacc[4][G][D];
  if (sw == 0) {
#pragma unroll
    for (int g = 0; g < G; ++g) {
      if (e == 0) {
        sm[w][g] = m[g];
        sl[w][g] = l[g];
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) sacc[w][g][e * 8 + j] = acc[g][j];
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < G * D; i += DEC_THR) {
    const int g = i / D, d = i % D;
    const float M = fmaxf(fmaxf(sm[0][g], sm[1][g]), fmaxf(sm[2][g], sm[3][g]));
    float L = 0.f, A = 0.f;
    if (M != -INFINITY) {
#pragma unroll
      for (int s2 = 0; s2 < 4; ++s2) {
        const float c = __expf(sm[s2][g] - M);
        L += sl[s2][g] * c;
        A += sacc[s2][g][d] * c;
      }
    }
    const size_t hrow = ((size_t)b * hq + kh * G + g) * nsplit + split;
    opart[hrow * D + d] = A;
    if (d == 0) {
      mpart[hrow] = M;
      lpart[hrow] = L;
    }
  }
}

template <int D>
__global__ __launch_bounds__(D) void decode_attn_merge_k(const float* __restrict__ opart,
                                                         const float* __restrict__ mpart,
                                                         const float* __restrict__ lpart, const int* __restrict__ lens,
                                                         bf16* __restrict__ out, int hq, int nsplit) {
  const size_t h = blockIdx.x;  // b*hq + head
  const int d = threadIdx.x;
  const int len = lens[h / hq];
  const int chunk = split_chunk(len, nsplit);
  const int nv = len > 0 ? min(nsplit, (len + chunk - 1) / chunk) : 0;   // splits that wrote partials
  float M = -INFINITY;
  for (int s = 0; s < nv; ++s) M = fmaxf(M, mpart[h * nsplit + s]);
  float L = 0.f, A = 0.f;
  if (M != -INFINITY) {
    for (int s = 0; s < nv; ++s) {
      const float c = __expf(mpart[h * nsplit + s] - M);
      L += lpart[h * nsplit + s] * c;
      A += opart[(h * nsplit + s) * D + d] * c;
    }
  }
  out[h * D + d] = (bf16)(L > 0.f ? A / L : 0.f);
}


// ------------------------------------------------------------- decode attention v2 (MFMA)
// Same split-K scheme, but the math runs on the matrix cores and the KV append is fused:
//  * a wave owns 32-key tiles of its split (tiles w, w+4, ... of the workgroup's range); the
//    G = Hq/Hkv query heads of the kv head are the 16 MFMA columns (lane li = head), scores
//    are computed swapped, Sᵀ = K·Qᵀ (K fragments straight from HBM, 16 B per lane), so the
//    online softmax is lane-local plus two shuffles and P is already Oᵀ = Vᵀ·Pᵀ's B operand;
//    V goes through a wave-private LDS tile and the gfx950 transposed read ds_read_b64_tr_b16;
//  * the new token's K/V rows are read from the projection output (not the cache), and the
//    split holding the last key writes them into the cache at pos — no separate scatter
//    kernel, no read-after-write hazard (no workgroup reads cache[pos] in this launch);
//  * lengths come from pos (int64, len = pos + 1) — no host-side lens tensor.
__device__ __forceinline__ bf16x4 dec_tr_read(const bf16* p) {
  typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4;
  return __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(p));
}
__device__ __forceinline__ int split_chunk32(int len, int nsplit) { return ((len + nsplit - 1) / nsplit + 31) & ~31; }

template <int D>
__global__ __launch_bounds__(256) void decode_attn_mfma_k(const bf16* __restrict__ q, int ldq,
                                                          const bf16* __restrict__ knew, int ldkn,
                                                          const bf16* __restrict__ vnew, int ldvn,
                                                          bf16* __restrict__ kc, bf16* __restrict__ vc,
                                                          const int64_t* __restrict__ pos, float* __restrict__ opart,
                                                          float* __restrict__ mpart, float* __restrict__ lpart,
                                                          int Smax, int hq, int hkv, int nsplit, float scale_log2) {
  constexpr int LDR = D + 8;          // padded LDS row (elements)
  constexpr int CH = D / 8;           // 16-B chunks per row
  constexpr int NS = D / 32;          // k-steps over the head dim
  constexpr int ND = D / 16;          // d-subtiles of O
  constexpr int VL = 32 * CH / 64;    // V chunks per lane per 32-key tile
  constexpr int VT = 32 * LDR;        // elements of one wave's V tile
  __shared__ __attribute__((aligned(16))) char smem[4 * VT * 2];
  __shared__ float sm[4][16], sl[4][16];
  static_assert(4 * 16 * D * 4 <= 4 * VT * 2, "merge buffer aliases the V tiles");

  const int split = blockIdx.x, kh = blockIdx.y, b = blockIdx.z;
  const int G = hq / hkv;
  const int len = (int)pos[b] + 1;
  const int chunk = split_chunk32(len, nsplit);
  const int k0 = split * chunk, k1 = min(k0 + chunk, len);
  if (k0 >= len) return;              // whole workgroup: empty split, never merged
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, g = lane >> 4, li = lane & 15;

  const size_t rs = (size_t)hkv * D;
  bf16* kcb = kc + (size_t)b * Smax * rs + kh * D;
  bf16* vcb = vc + (size_t)b * Smax * rs + kh * D;
  const bf16* knb = knew + (size_t)b * ldkn + kh * D;
  const bf16* vnb = vnew + (size_t)b * ldvn + kh * D;
  if (k1 == len && w == 0 && lane < 2 * CH) {      // append the new token's K/V rows
    const int c = lane % CH;
    if (lane < CH)
      *reinterpret_cast<bf16x8*>(kcb + (size_t)(len - 1) * rs + 8 * c) = *reinterpret_cast<const bf16x8*>(knb + 8 * c);
    else
      *reinterpret_cast<bf16x8*>(vcb + (size_t)(len - 1) * rs + 8 * c) = *reinterpret_cast<const bf16x8*>(vnb + 8 * c);
  }

  bf16x8 qf[NS];
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    if (li < G) qf[s] = *reinterpret_cast<const bf16x8*>(q + (size_t)b * ldq + (kh * G + li) * D + 32 * s + 8 * g);
    else qf[s] = bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
  }
  f32x4 acc[ND];
#pragma unroll
  for (int dt = 0; dt < ND; ++dt) acc[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
  float m_run = -INFINITY, l_run = 0.f;
  bf16* vl = reinterpret_cast<bf16*>(smem) + w * VT;

  for (int t = k0 + 32 * w; t < k1; t += 128) {
    bf16x8 kr[2][NS], vr[VL];
#pragma unroll
    for (int kt = 0; kt < 2; ++kt) {
      const int key = min(t + 16 * kt + li, k1 - 1);
      const bf16* kp = key == len - 1 ? knb : kcb + (size_t)key * rs;
#pragma unroll
      for (int s = 0; s < NS; ++s) kr[kt][s] = *reinterpret_cast<const bf16x8*>(kp + 32 * s + 8 * g);
    }
#pragma unroll
    for (int p = 0; p < VL; ++p) {
      const int ci = p * 64 + lane, row = ci / CH, ch = ci % CH;
      const int key = min(t + row, k1 - 1);
      const bf16* vp = key == len - 1 ? vnb : vcb + (size_t)key * rs;
      vr[p] = *reinterpret_cast<const bf16x8*>(vp + 8 * ch);
    }
    f32x4 sc[2];
#pragma unroll
    for (int kt = 0; kt < 2; ++kt) {
      sc[kt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < NS; ++s) sc[kt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kr[kt][s], qf[s], sc[kt], 0, 0, 0);
    }
#pragma unroll
    for (int p = 0; p < VL; ++p) {
      const int ci = p * 64 + lane, row = ci / CH, ch = ci % CH;
      *reinterpret_cast<bf16x8*>(vl + row * LDR + 8 * ch) = vr[p];
    }
    // lane owns head li; keys t + 16kt + 4g + r
    float mx = -INFINITY;
#pragma unroll
    for (int kt = 0; kt < 2; ++kt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float v = (t + 16 * kt + 4 * g + r < k1) ? sc[kt][r] * scale_log2 : -INFINITY;
        sc[kt][r] = v;
        mx = fmaxf(mx, v);
      }
    mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    const float mn = fmaxf(m_run, mx);            // finite: every tile has >= 1 valid key
    const float alpha = __builtin_amdgcn_exp2f(m_run - mn);
    float rsum = 0.f;
#pragma unroll
    for (int kt = 0; kt < 2; ++kt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float pr = __builtin_amdgcn_exp2f(sc[kt][r] - mn);
        sc[kt][r] = pr;
        rsum += pr;
      }
    rsum += __shfl_xor(rsum, 16, 64);
    rsum += __shfl_xor(rsum, 32, 64);
    l_run = l_run * alpha + rsum;
    m_run = mn;
#pragma unroll
    for (int dt = 0; dt < ND; ++dt) acc[dt] *= alpha;
    const bf16x8 pf = bf16x8{(bf16)sc[0][0], (bf16)sc[0][1], (bf16)sc[0][2], (bf16)sc[0][3],
                             (bf16)sc[1][0], (bf16)sc[1][1], (bf16)sc[1][2], (bf16)sc[1][3]};
    __builtin_amdgcn_s_waitcnt(0xc07f);          // lgkmcnt(0): this wave's V tile is in LDS
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int dt = 0; dt < ND; ++dt) {
      const bf16* p0 = vl + (4 * g + (li >> 2)) * LDR + 16 * dt + 4 * (li & 3);
      const bf16x4 a = dec_tr_read(p0), c = dec_tr_read(p0 + 16 * LDR);
      const bf16x8 vf = bf16x8{a[0], a[1], a[2], a[3], c[0], c[1], c[2], c[3]};
      acc[dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vf, pf, acc[dt], 0, 0, 0);
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);          // transposed reads done before the tile is rewritten
    __builtin_amdgcn_wave_barrier();
  }
  // ---- merge the 4 waves (Oᵀ[16dt + 4g + r][li]) through LDS, natural-log m for the merge kernel
  __syncthreads();
  float* sacc = reinterpret_cast<float*>(smem);   // [4][16][D], aliases the V tiles
  if (g == 0) {
    sm[w][li] = m_run;
    sl[w][li] = l_run;
  }
#pragma unroll
  for (int dt = 0; dt < ND; ++dt)
#pragma unroll
    for (int r = 0; r < 4; ++r) sacc[(w * 16 + li) * D + 16 * dt + 4 * g + r] = acc[dt][r];
  __syncthreads();
  for (int i = threadIdx.x; i < G * D; i += 256) {
    const int hh = i / D, d = i % D;
    const float M = fmaxf(fmaxf(sm[0][hh], sm[1][hh]), fmaxf(sm[2][hh], sm[3][hh]));
    float L = 0.f, A = 0.f;
#pragma unroll
    for (int s2 = 0; s2 < 4; ++s2) {
      const float c = __builtin_amdgcn_exp2f(sm[s2][hh] - M);   // -inf (idle wave) → 0
      L += sl[s2][hh] * c;
      A += sacc[(s2 * 16 + hh) * D + d] * c;
    }
    const size_t hrow = ((size_t)b * hq + kh * G + hh) * nsplit + split;
    opart[hrow * D + d] = A;
    if (d == 0) {
      mpart[hrow] = M * 0.6931471805599453f;
      lpart[hrow] = L;
    }
  }
}

template <int D>
__global__ __launch_bounds__(D) void decode_attn_merge2_k(const float* __restrict__ opart,
                                                          const float* __restrict__ mpart,
                                                          const float* __restrict__ lpart,
                                                          const int64_t* __restrict__ pos, bf16* __restrict__ out,
                                                          int hq, int nsplit) {
  const size_t h = blockIdx.x;  // b*hq + head
  const int d = threadIdx.x;
  const int len = (int)pos[h / hq] + 1;
  const int chunk = split_chunk32(len, nsplit);
  const int nv = min(nsplit, (len + chunk - 1) / chunk);
  float M = -INFINITY;
  for (int s = 0; s < nv; ++s) M = fmaxf(M, mpart[h * nsplit + s]);
  float L = 0.f, A = 0.f;
  for (int s = 0; s < nv; ++s) {
    const float c = __expf(mpart[h * nsplit + s] - M);
    L += lpart[h * nsplit + s] * c;
    A += opart[(h * nsplit + s) * D + d] * c;
  }
  out[h * D + d] = (bf16)(L > 0.f ? A / L : 0.f);
}

// ------------------------------------------------------------------------------ sampler
constexpr int SMP_THR = 1024;
constexpr int SMP_NW = SMP_THR / 64;

__device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

__device__ __forceinline__ float bsum(float v, float* red) { return block_sum<SMP_NW>(v, red); }

template <typename T>
__global__ __launch_bounds__(SMP_THR) void sample_k(const T* __restrict__ logits, const int* __restrict__ hist,
                                                    int hist_len, float* __restrict__ work, int64_t* __restrict__ out,
                                                    int V, float temperature, int top_k, float top_p, float penalty,
                                                    uint64_t key) {
  __shared__ float red[SMP_NW];
  __shared__ float sc[SMP_THR];
  __shared__ int si[SMP_NW];
  const int row = blockIdx.x, tid = threadIdx.x;
  const T* x = logits + (size_t)row * V;
  float* wv = work + (size_t)row * V;
  for (int i = tid; i < V; i += SMP_THR) wv[i] = (float)x[i];
  __syncthreads();
  if (hist && penalty != 1.f) {
    for (int i = tid; i < hist_len; i += SMP_THR) {
      const int id = hist[(size_t)row * hist_len + i];
      if (id >= 0 && id < V) {
        const float s = (float)x[id];  // from the ORIGINAL row: duplicates write the same value
        wv[id] = s < 0.f ? s * penalty : s / penalty;
      }
    }
  }
  __syncthreads();
  // max + argmax (lowest index wins ties)
  float best = -INFINITY;
  int bidx = 0x7FFFFFFF;
  for (int i = tid; i < V; i += SMP_THR) {
    const float v = wv[i];
    if (v > best || (v == best && i < bidx)) { best = v; bidx = i; }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float ov = __shfl_xor(best, o, 64);
    const int oi = __shfl_xor(bidx, o, 64);
    if (ov > best || (ov == best && oi < bidx)) { best = ov; bidx = oi; }
  }
  if ((tid & 63) == 0) { red[tid >> 6] = best; si[tid >> 6] = bidx; }
  __syncthreads();
  best = red[0];
  bidx = si[0];
  for (int i = 1; i < SMP_NW; ++i)
    if (red[i] > best || (red[i] == best && si[i] < bidx)) { best = red[i]; bidx = si[i]; }
  __syncthreads();
  if (!(temperature > 0.f)) {  // greedy
    if (tid == 0) out[row] = bidx;
    return;
  }
  const float invT = 1.f / temperature;
  const float mx = best * invT;
  // unnormalised probabilities p_i = exp(x_i/T - max)
  auto prob = [&](int i) { return __expf(wv[i] * invT - mx); };
  float lo = 0.f, hi = 1.f;  // threshold on p (max p == 1)
  // ---- top-k: largest threshold t with count(p >= t) >= k (bisection)
  float thr = 0.f;
  if (top_k > 0 && top_k < V) {
    lo = 0.f; hi = 1.f;
    for (int it = 0; it < 40; ++it) {
      const float mid = 0.5f * (lo + hi);
      float c = 0.f;
      for (int i = tid; i < V; i += SMP_THR) c += prob(i) >= mid ? 1.f : 0.f;
      c = bsum(c, red);
      if (c >= (float)top_k) lo = mid; else hi = mid;
    }
    thr = lo;
  }
  // ---- top-p over the kept set: largest t >= thr with mass(p >= t) >= top_p * mass(kept)
  if (top_p < 1.f) {
    float tot = 0.f;
    for (int i = tid; i < V; i += SMP_THR) { const float p = prob(i); tot += p >= thr ? p : 0.f; }
    tot = bsum(tot, red);
    lo = thr; hi = 1.f;
    for (int it = 0; it < 40; ++it) {
      const float mid = 0.5f * (lo + hi);
      float c = 0.f;
      for (int i = tid; i < V; i += SMP_THR) { const float p = prob(i); c += p >= mid ? p : 0.f; }
      c = bsum(c, red);
      if (c >= top_p * tot) lo = mid; else hi = mid;
    }
    thr = lo;
  }
  // ---- inverse-CDF draw over kept tokens in index order: contiguous chunk per thread
  const int per = (V + SMP_THR - 1) / SMP_THR;
  const int i0 = tid * per, i1 = min(i0 + per, V);
  float mine = 0.f;
  for (int i = i0; i < i1; ++i) { const float p = prob(i); mine += p >= thr ? p : 0.f; }
  sc[tid] = mine;
  __syncthreads();
  for (int off = 1; off < SMP_THR; off <<= 1) {  // inclusive Hillis-Steele scan
    const float add = tid >= off ? sc[tid - off] : 0.f;
    __syncthreads();
    sc[tid] += add;
    __syncthreads();
  }
  const float total = sc[SMP_THR - 1];
  const uint64_t r = mix64(key ^ mix64((uint64_t)row + 0x1234567ull));
  const float u = (float)((r >> 40) * (1.0 / 16777216.0)) * total;
  const float before = tid ? sc[tid - 1] : 0.f;
  if (u >= before && u < sc[tid] && mine > 0.f) {
    float run = before;
    int pick = i1 - 1;
    for (int i = i0; i < i1; ++i) {
      const float p = prob(i);
      if (p < thr) continue;
      run += p;
      if (u < run) { pick = i; break; }
    }
    out[row] = pick;
  }
  if (tid == 0 && !(total > 0.f)) out[row] = bidx;
}

}  // namespace

// Split-K plan: enough (split, kv-head, sequence) workgroups to fill the chip.  The number of
// splits depends only on (B, hkv, max_len), so a captured hipGraph stays valid as sequences
// grow; each workgroup derives its key range from the live length on the device (all splits
// busy whatever the context length, no host sync).
int decode_split_plan(int B, int hkv, int max_len) {
  const int pairs = std::max(1, B * hkv);
  int ns = std::max(1, (DEC_TARGET_WG + pairs - 1) / pairs);
  return std::min(ns, std::max(1, (max_len + 31) / 32));
}

void launch_decode_attention(const void* q, const void* kc, const void* vc, const int* lens, float* opart, float* mpart,
                             float* lpart, void* out, int B, int Smax, int hq, int hkv, int d, int nsplit,
                             float scale, hipStream_t st) {
  const int G = hq / hkv;
  dim3 grid(nsplit, hkv, B);
#define P(D_, G_)                                                                                           \
  decode_attn_partial_k<D_, G_><<<grid, DEC_THR, 0, st>>>((const bf16*)q, (const bf16*)kc, (const bf16*)vc, \
                                                          lens, opart, mpart, lpart, Smax, hq, hkv, nsplit, scale)
#define GS(D_)                          \
  switch (G) {                          \
    case 1: P(D_, 1); break;            \
    case 2: P(D_, 2); break;            \
    case 4: P(D_, 4); break;            \
    case 5: P(D_, 5); break;            \
    case 8: P(D_, 8); break;            \
    default: break;                     \
  }
  if (d == 128) { GS(128) } else if (d == 64) { GS(64) }
#undef GS
#undef P
  if (d == 128)
    decode_attn_merge_k<128><<<B * hq, 128, 0, st>>>(opart, mpart, lpart, lens, (bf16*)out, hq, nsplit);
  else
    decode_attn_merge_k<64><<<B * hq, 64, 0, st>>>(opart, mpart, lpart, lens, (bf16*)out, hq, nsplit);
  LIPA_CHECK_LAUNCH();
}


// v2: MFMA split-K decode attention with the KV append fused (see decode_attn_mfma_k)
int decode_split_plan2(int B, int hkv, int max_len) {
  const int pairs = std::max(1, B * hkv);
  int ns = std::max(1, (DEC_TARGET_WG + pairs - 1) / pairs);
  return std::min(ns, std::max(1, (max_len + 127) / 128));
}

void launch_decode_attention2(const void* q, int ldq, const void* knew, int ldkn, const void* vnew, int ldvn, void* kc,
                              void* vc, const int64_t* pos, float* opart, float* mpart, float* lpart, void* out, int B,
                              int Smax, int hq, int hkv, int d, int nsplit, float scale, hipStream_t st) {
  dim3 grid(nsplit, hkv, B);
  const float sl2 = scale * 1.4426950408889634f;
#define P(D_)                                                                                                          \
  decode_attn_mfma_k<D_><<<grid, 256, 0, st>>>((const bf16*)q, ldq, (const bf16*)knew, ldkn, (const bf16*)vnew, ldvn, \
                                               (bf16*)kc, (bf16*)vc, pos, opart, mpart, lpart, Smax, hq, hkv, nsplit, \
                                               sl2);                                                                   \
  decode_attn_merge2_k<D_><<<B * hq, D_, 0, st>>>(opart, mpart, lpart, pos, (bf16*)out, hq, nsplit)
  if (d == 128) { P(128); } else { P(64); }
#undef P
  LIPA_CHECK_LAUNCH();
}

void launch_sample(int dtype, const void* logits, const int* hist, int hist_len, float* work, int64_t* out, int B, int V,
                   float temperature, int top_k, float top_p, float penalty, uint64_t key, hipStream_t st) {
  if (dtype == 0)
    sample_k<float><<<B, SMP_THR, 0, st>>>((const float*)logits, hist, hist_len, work, out, V, temperature, top_k,
                                           top_p, penalty, key);
  else
    sample_k<bf16><<<B, SMP_THR, 0, st>>>((const bf16*)logits, hist, hist_len, work, out, V, temperature, top_k,
                                          top_p, penalty, key);
  LIPA_CHECK_LAUNCH();
}
