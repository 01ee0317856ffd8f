// Mixture-of-experts routing and token dispatch on gfx950 (the DeepSeekLike
// MoE of ``DeepSeekLike_wikitext2.py:276-309`` / ``DeepSeekLike_spare_MoE_wikitext2.py``).
//
// The reference does top-k in torch, then per (slot, expert) ``nonzero`` gathers and an
// ``index_add_`` scatter — many tiny launches, host syncs, and non-deterministic atomics.
// Here routing and dispatch are four launch-once kernels with no host round trip and no
// atomics (bitwise deterministic):
//
//  * moe_route:   one wave per token, one lane per expert (E <= 64): top-k by k rounds of
//                 wave arg-max (DPP/shuffle reductions), softmax over the k winners (or the
//                 full softmax first: "softmax_topk"), plus the full router softmax for the
//                 load-balance loss.  The backward is the same shape.
//  * moe_permute: one workgroup per expert streams the T·k expert ids: a ballot/popcount pass
//                 counts the ids below e (→ segment offset) and a second pass gives every
//                 pair routed to e its STABLE rank (token order) → pos_of[pair], perm[row],
//                 offsets[E+1].  Expert segments are contiguous, ready for per-expert GEMMs.
//  * moe_gather:  row gather x[perm/k] (optionally × gate weight) with 16-B vector loads.
//  * moe_combine: out[t] = base[t] + Σ_j w[t,j]·ys[pos_of[t,j]] — the scatter-add of the
//                 reference turned into a gather per token (fp32 accumulation), and its
//                 weight gradient dw[t,j] = <dout[t], ys[pos_of[t,j]]>.
#include "common.h"

using namespace lipa;

namespace {

__device__ __forceinline__ void wave_argmax(float& v, int& i) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float ov = __shfl_xor(v, o, 64);
    const int oi = __shfl_xor(i, o, 64);
    if (ov > v || (ov == v && oi < i)) { v = ov; i = oi; }
  }
}

// logits [T, E]; idx [T, k] int32; w [T, k] fp32; probs [T, E] fp32 (optional)
template <typename T>
__global__ __launch_bounds__(256) void moe_route_k(const T* __restrict__ logits, int* __restrict__ idx,
                                                   float* __restrict__ w, float* __restrict__ probs, int Ntok, int E,
                                                   int K, int mode) {
  const int t = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (t >= Ntok) return;
  const float x = lane < E ? to_f(logits[(size_t)t * E + lane]) : -INFINITY;
  const float mx = wave_max(x);
  const float ex = lane < E ? __expf(x - mx) : 0.f;
  const float p = ex / wave_sum(ex);
  if (probs && lane < E) probs[(size_t)t * E + lane] = p;
  float cur = mode == 0 ? x : p;
  float sel[8];
  int sid[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {          // K <= 8 (unrolled: sel/sid stay in registers)
    sel[j] = -INFINITY;
    sid[j] = 0;
    if (j >= K) continue;
    float v = lane < E ? cur : -INFINITY;
    int i = lane;
    wave_argmax(v, i);
    sel[j] = v;
    sid[j] = i;
    if (lane == i) cur = -INFINITY;
  }
  if (lane < K) {
    float val = 0.f;
    int id = 0;
    float m0 = sel[0], s = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      if (j >= K) continue;
      if (j == lane) { val = sel[j]; id = sid[j]; }
      s += __expf(sel[j] - m0);
    }
    idx[(size_t)t * K + lane] = id;
    w[(size_t)t * K + lane] = mode == 0 ? __expf(val - m0) / s : val;
  }
}

// dlogits [T, E] from dw [T, k] (w, idx from the forward; probs needed for mode 1)
template <typename T>
__global__ __launch_bounds__(256) void moe_route_bwd_k(const float* __restrict__ dw, const float* __restrict__ w,
                                                       const int* __restrict__ idx, const float* __restrict__ probs,
                                                       T* __restrict__ dlogits, int Ntok, int E, int K, int mode) {
  const int t = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (t >= Ntok) return;
  // mode 0: w = softmax(top logits): dl[idx_j] = w_j (dw_j - Σ w dw)
  // mode 1: w_j = p[idx_j], p = softmax(all): dp[idx_j] = dw_j, dl = p (dp - Σ p dp)
  float g = 0.f;   // this lane's incoming gradient on its expert (w-space)
  float dot = 0.f;
  for (int j = 0; j < K; ++j) {
    const int id = idx[(size_t)t * K + j];
    const float d = dw[(size_t)t * K + j], wj = w[(size_t)t * K + j];
    dot += wj * d;
    if (id == lane) g += d;
  }
  if (lane >= E) return;
  float out;
  if (mode == 0) {
    float wl = 0.f;
    for (int j = 0; j < K; ++j)
      if (idx[(size_t)t * K + j] == lane) wl = w[(size_t)t * K + j];
    out = wl * (g - dot);
  } else {
    out = probs[(size_t)t * E + lane] * (g - dot);
  }
  dlogits[(size_t)t * E + lane] = from_f<T>(out);
}

// one workgroup per expert e; ids [P] int32 (P = T·k pairs in token-major order)
__global__ __launch_bounds__(256) void moe_permute_k(const int* __restrict__ ids, int P, int E,
                                                     int* __restrict__ pos_of, int* __restrict__ perm,
                                                     int* __restrict__ offsets) {
  __shared__ int wsum[4];
  __shared__ int total;
  const int e = blockIdx.x, tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
  // pass 1: number of pairs routed to experts < e
  int below = 0, mine = 0;
  for (int i = tid; i < P; i += 256) {
    const int id = ids[i];
    below += id < e;
    mine += id == e;
  }
  below = (int)wave_sum((float)below);   // exact for P < 2^24
  mine = (int)wave_sum((float)mine);
  if (tid == 0) total = 0;
  __syncthreads();
  if (lane == 0) {
    atomicAdd(&total, below);
    wsum[w] = mine;
  }
  __syncthreads();
  const int off = total;
  if (tid == 0) {
    offsets[e + 1] = off + wsum[0] + wsum[1] + wsum[2] + wsum[3];
    if (e == 0) offsets[0] = 0;
  }
  // pass 2: stable rank within expert e, 256 pairs per iteration
  int base = off;
  for (int i0 = 0; i0 < P; i0 += 256) {
    const int i = i0 + tid;
    const bool hit = i < P && ids[i] == e;
    const uint64_t bal = __ballot(hit);
    const int before_in_wave = __popcll(bal & ((1ull << lane) - 1ull));
    __syncthreads();
    if (lane == 0) wsum[w] = __popcll(bal);
    __syncthreads();
    int before_waves = 0;
    for (int q = 0; q < w; ++q) before_waves += wsum[q];
    if (hit) {
      const int pos = base + before_waves + before_in_wave;
      pos_of[i] = pos;
      perm[pos] = i;
    }
    base += wsum[0] + wsum[1] + wsum[2] + wsum[3];
  }
}

// out[p] = x[perm[p] / K] (· w[perm[p]])  — rows of H elements, 8 per lane-chunk
template <typename T>
__global__ __launch_bounds__(256) void moe_gather_k(const T* __restrict__ x, const int* __restrict__ perm,
                                                    const float* __restrict__ w, T* __restrict__ out, int R, int H,
                                                    int K) {
  const int chunks = H / 8;
  const size_t n = (size_t)R * chunks;
  for (size_t g = (size_t)blockIdx.x * 256 + threadIdx.x; g < n; g += (size_t)gridDim.x * 256) {
    const int p = (int)(g / chunks), c = (int)(g % chunks);
    const int pair = perm[p];
    const int t = pair / K;
    float f[8];
    load8(x + (size_t)t * H + c * 8, f);
    if (w) {
      const float s = w[pair];
#pragma unroll
      for (int i = 0; i < 8; ++i) f[i] *= s;
    }
    store8(out + (size_t)p * H + c * 8, f);
  }
}

// out[t] = base[t] + Σ_j w[t,j] · ys[pos_of[t·K + j]]   (w optional → 1)
template <typename T>
__global__ __launch_bounds__(256) void moe_combine_k(const T* __restrict__ ys, const int* __restrict__ pos_of,
                                                     const float* __restrict__ w, const T* __restrict__ base,
                                                     T* __restrict__ out, int Ntok, int H, int K) {
  const int chunks = H / 8;
  const size_t n = (size_t)Ntok * chunks;
  for (size_t g = (size_t)blockIdx.x * 256 + threadIdx.x; g < n; g += (size_t)gridDim.x * 256) {
    const int t = (int)(g / chunks), c = (int)(g % chunks);
    float acc[8];
    if (base) load8(base + (size_t)t * H + c * 8, acc);
    else {
#pragma unroll
      for (int i = 0; i < 8; ++i) acc[i] = 0.f;
    }
    for (int j = 0; j < K; ++j) {
      const int p = pos_of[(size_t)t * K + j];
      const float s = w ? w[(size_t)t * K + j] : 1.f;
      float f[8];
      load8(ys + (size_t)p * H + c * 8, f);
#pragma unroll
      for (int i = 0; i < 8; ++i) acc[i] += s * f[i];
    }
    store8(out + (size_t)t * H + c * 8, acc);
  }
}

// dw[t,j] = <dout[t], ys[pos_of[t,j]]> — one wave per pair
template <typename T>
__global__ __launch_bounds__(256) void moe_wgrad_k(const T* __restrict__ dout, const T* __restrict__ ys,
                                                   const int* __restrict__ pos_of, float* __restrict__ dw, int Ntok,
                                                   int H, int K) {
  const int pair = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (pair >= Ntok * K) return;
  const int t = pair / K, p = pos_of[pair];
  float s = 0.f;
  for (int c = lane * 8; c < H; c += 512) {
    float a[8], b[8];
    load8(dout + (size_t)t * H + c, a);
    load8(ys + (size_t)p * H + c, b);
#pragma unroll
    for (int i = 0; i < 8; ++i) s += a[i] * b[i];
  }
  s = wave_sum(s);
  if (lane == 0) dw[pair] = s;
}

inline int grid_for(size_t n) {
  size_t g = (n + 255) / 256;
  return (int)(g < 8192 ? (g ? g : 1) : 8192);
}

}  // namespace

// dtype: 0 fp32, 1 bf16 (as every launcher in this extension)
void launch_moe_route(int dtype, const void* logits, int* idx, float* w, float* probs, int Ntok, int E, int K, int mode,
                      hipStream_t st) {
  const int g = (Ntok + 3) / 4;
  if (dtype == 1)
    moe_route_k<bf16><<<g, 256, 0, st>>>((const bf16*)logits, idx, w, probs, Ntok, E, K, mode);
  else
    moe_route_k<float><<<g, 256, 0, st>>>((const float*)logits, idx, w, probs, Ntok, E, K, mode);
}

void launch_moe_route_bwd(int dtype, const float* dw, const float* w, const int* idx, const float* probs, void* dl,
                          int Ntok, int E, int K, int mode, hipStream_t st) {
  const int g = (Ntok + 3) / 4;
  if (dtype == 1)
    moe_route_bwd_k<bf16><<<g, 256, 0, st>>>(dw, w, idx, probs, (bf16*)dl, Ntok, E, K, mode);
  else
    moe_route_bwd_k<float><<<g, 256, 0, st>>>(dw, w, idx, probs, (float*)dl, Ntok, E, K, mode);
}

void launch_moe_permute(const int* ids, int P, int E, int* pos_of, int* perm, int* offsets, hipStream_t st) {
  moe_permute_k<<<E, 256, 0, st>>>(ids, P, E, pos_of, perm, offsets);
}

void launch_moe_gather(int dtype, const void* x, const int* perm, const float* w, void* out, int R, int H, int K,
                       hipStream_t st) {
  const int g = grid_for((size_t)R * (H / 8));
  if (dtype == 1)
    moe_gather_k<bf16><<<g, 256, 0, st>>>((const bf16*)x, perm, w, (bf16*)out, R, H, K);
  else
    moe_gather_k<float><<<g, 256, 0, st>>>((const float*)x, perm, w, (float*)out, R, H, K);
}

void launch_moe_combine(int dtype, const void* ys, const int* pos_of, const float* w, const void* base, void* out,
                        int Ntok, int H, int K, hipStream_t st) {
  const int g = grid_for((size_t)Ntok * (H / 8));
  if (dtype == 1)
    moe_combine_k<bf16><<<g, 256, 0, st>>>((const bf16*)ys, pos_of, w, (const bf16*)base, (bf16*)out, Ntok, H, K);
  else
    moe_combine_k<float><<<g, 256, 0, st>>>((const float*)ys, pos_of, w, (const float*)base, (float*)out, Ntok, H, K);
}

void launch_moe_wgrad(int dtype, const void* dout, const void* ys, const int* pos_of, float* dw, int Ntok, int H, int K,
                      hipStream_t st) {
  const int g = (Ntok * K + 3) / 4;
  if (dtype == 1)
    moe_wgrad_k<bf16><<<g, 256, 0, st>>>((const bf16*)dout, (const bf16*)ys, pos_of, dw, Ntok, H, K);
  else
    moe_wgrad_k<float><<<g, 256, 0, st>>>((const float*)dout, (const float*)ys, pos_of, dw, Ntok, H, K);
}
