// Cross-entropy forward+backward in one pass over a logits chunk (K7).
//
// One 512-thread workgroup per token row of V logits (V = 151,936 for Qwen3): an online
// (max, sum-exp) reduction over 16-B vector loads, then a second sweep that overwrites the
// bf16 logits IN PLACE with dlogits = (softmax - onehot) * scale (scale = 1/n_valid), so
// the LM-head backward GEMM reads them directly.  Ignored rows (label == ignore_index)
// write zeros.  Returns per-row loss (fp32, already unscaled).
#include "common.h"

using namespace lipa;

namespace {

constexpr int NT = 512, NW = NT / 64;

template <typename T>
__global__ __launch_bounds__(NT) void ce_fwd_bwd_k(T* __restrict__ logits, const int64_t* __restrict__ labels,
                                                   float* __restrict__ row_loss, int V, int ignore_index,
                                                   const float* __restrict__ scale_ptr, float scale_val,
                                                   int rows_per_scale) {
  __shared__ float red[NW];
  const int row = blockIdx.x;
  T* lr = logits + (size_t)row * V;
  const int64_t lab = labels[row];
  // per-group scale (gradient-accumulation micro-batches fused into one pass: 1/(G·n_valid_g))
  const float scale = scale_ptr ? scale_ptr[rows_per_scale > 0 ? row / rows_per_scale : 0] : scale_val;
  if (lab == ignore_index) {
    for (int v = threadIdx.x * 8; v < V; v += NT * 8) {
      if (v + 8 <= V) {
        float z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        store8(lr + v, z);
      } else {
        for (int i = v; i < V; ++i) lr[i] = (T)0.f;
      }
    }
    if (threadIdx.x == 0) row_loss[row] = 0.f;
    return;
  }
  // pass 1: online max / sum-exp
  float m = -INFINITY, s = 0.f;
  for (int v = threadIdx.x * 8; v < V; v += NT * 8) {
    float x[8];
    int n = 8;
    if (v + 8 <= V) load8(lr + v, x);
    else {
      n = V - v;
      for (int i = 0; i < 8; ++i) x[i] = i < n ? (float)lr[v + i] : -INFINITY;
    }
    float mx = x[0];
#pragma unroll
    for (int i = 1; i < 8; ++i) mx = fmaxf(mx, x[i]);
    const float mn = fmaxf(m, mx);
    float acc = s * __expf(m - mn);
#pragma unroll
    for (int i = 0; i < 8; ++i) acc += __expf(x[i] - mn);
    m = mn;
    s = acc;
  }
  // combine (m, s) across the block
  float gm = block_max<NW>(m, red);
  __syncthreads();
  float gs = block_sum<NW>(s * __expf(m - gm), red);
  const float lse = gm + __logf(gs);
  const float xl = (float)lr[lab];
  __syncthreads();
  // pass 2: dlogits in place
  for (int v = threadIdx.x * 8; v < V; v += NT * 8) {
    if (v + 8 <= V) {
      float x[8];
      load8(lr + v, x);
#pragma unroll
      for (int i = 0; i < 8; ++i) x[i] = (__expf(x[i] - lse) - (v + i == lab ? 1.f : 0.f)) * scale;
      store8(lr + v, x);
    } else {
      for (int i = v; i < V; ++i) lr[i] = (T)((__expf((float)lr[i] - lse) - (i == lab ? 1.f : 0.f)) * scale);
    }
  }
  if (threadIdx.x == 0) row_loss[row] = lse - xl;
}

}  // namespace

void launch_ce_fwd_bwd(int dtype, void* logits, const int64_t* labels, float* row_loss, int M, int V,
                       int ignore_index, const float* scale_ptr, float scale_val, int rows_per_scale,
                       hipStream_t st) {
  if (dtype == 1)
    ce_fwd_bwd_k<bf16><<<M, NT, 0, st>>>((bf16*)logits, labels, row_loss, V, ignore_index, scale_ptr, scale_val,
                                         rows_per_scale);
  else
    ce_fwd_bwd_k<float><<<M, NT, 0, st>>>((float*)logits, labels, row_loss, V, ignore_index, scale_ptr, scale_val,
                                          rows_per_scale);
  LIPA_CHECK_LAUNCH();
}
