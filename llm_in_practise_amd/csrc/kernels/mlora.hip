// Multi-adapter LoRA serving (vLLM --enable-lora --lora-modules a=… b=…;
// reference Fine-Tuning/README.md:346-351): y[t, c0 + n] += s_a · (x[t]·A_aᵀ)·B_aᵀ[n] with a = ids[t],
// each row computing ONLY its own adapter's columns.
//
//   A_all [Σr, K], B_all [N, Σr] bf16 — every loaded adapter's factors stacked once at load time;
//   seg [n_adapters + 1] = {offset o_a into Σr, rank r_a, scale s_a}; adapter 0 = the bare base.
//
// One workgroup per (row, column chunk): the row's rank-r_a projection x·A_aᵀ (r_a ≤ 64 dot products
// of length K, 4 waves × 16 ranks, 16-B vector loads, wave reductions) is kept in LDS, then the
// chunk's columns are expanded by the same 256 threads.  Work per row is r_a·(K + N) MACs — it does
// not grow with the number of adapters loaded (the round-2 torch form computed all Σr columns for
// every row and masked the foreign ones).  Static shapes, device-side ids: captured in the decode
// hipGraph like the rest of the step.
#include "common.h"

using namespace lipa;

namespace {

constexpr int MAX_R = 64;
constexpr int CHUNK = 2048;   // output columns per workgroup (8 per thread)

struct Seg {
  int off, r;
  float scale;
};

__global__ __launch_bounds__(256) void mlora_apply_k(const bf16* __restrict__ x, int ldx, const bf16* __restrict__ A,
                                                     const bf16* __restrict__ Bm, const int64_t* __restrict__ ids,
                                                     const Seg* __restrict__ seg, int n_seg, bf16* __restrict__ y,
                                                     int ldy, int c0, int K, int N, int R) {
  const int t = blockIdx.x;
  const int64_t a = ids[t];
  if (a <= 0 || a >= n_seg) return;   // base rows (and out-of-range ids) add nothing; uniform per workgroup
  const Seg sg = seg[a];
  if (sg.r <= 0) return;
  __shared__ float xa[MAX_R];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const bf16* xr = x + (size_t)t * ldx;
  // shrink: wave w computes ranks w, w+4, … (< r); lanes stride K in 8-element vectors
  for (int r = w; r < sg.r; r += 4) {
    const bf16* ar = A + (size_t)(sg.off + r) * K;
    float acc = 0.f;
    for (int k = lane * 8; k < K; k += 64 * 8) {
      float xv[8], av[8];
      load8(xr + k, xv);
      load8(ar + k, av);
#pragma unroll
      for (int e = 0; e < 8; ++e) acc = fmaf(xv[e], av[e], acc);
    }
    acc = wave_sum(acc);
    if (lane == 0) xa[r] = acc * sg.scale;
  }
  __syncthreads();
  // expand: the row's whole column range in CHUNK-wide passes (the rank-r projection above is computed
  // once per row, not once per column chunk); thread j owns 8 consecutive columns of each pass
  for (int nb = 0; nb < N; nb += CHUNK) {
    const int n = nb + threadIdx.x * 8;
    if (n >= N) break;
    float o[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int r0 = 0; r0 < sg.r; r0 += 8) {   // ranks and offsets are multiples of 8 (host): 16-B loads
      float xv[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) xv[i] = xa[r0 + i];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        float bv[8];
        load8(Bm + (size_t)(n + e) * R + sg.off + r0, bv);
#pragma unroll
        for (int i = 0; i < 8; ++i) o[e] = fmaf(xv[i], bv[i], o[e]);
      }
    }
    bf16* yr = y + (size_t)t * ldy + c0 + n;
    float cur[8];
    load8(yr, cur);
#pragma unroll
    for (int e = 0; e < 8; ++e) cur[e] += o[e];
    store8(yr, cur);
  }
}

}  // namespace

void launch_mlora_apply(const void* x, int ldx, const void* A, const void* B, const int64_t* ids, const void* seg,
                        int n_seg, void* y, int ldy, int c0, int T, int K, int N, int R, hipStream_t st) {
  if (T <= 0) return;
  const dim3 grid(T);
  mlora_apply_k<<<grid, 256, 0, st>>>((const bf16*)x, ldx, (const bf16*)A, (const bf16*)B, ids, (const Seg*)seg,
                                      n_seg, (bf16*)y, ldy, c0, K, N, R);
  LIPA_CHECK_LAUNCH();
}
