// Token / position embedding gather and its gradient scatter-add.
//
// Forward: out[n, :] = W[ids[n], :] — a row copy, dtype-agnostic (rows moved as 16-B chunks: a
// workgroup of 256 threads covers 256·16 B of one or more rows, so a 4096-wide bf16 row is two
// wave-instructions per wave and the read of W is one 128-B line per 8 lanes).
//
// Backward: gW[ids[n], :] += dout[n, :] into an fp32 [V, D] buffer, one 8-element chunk per thread
// (16-B bf16 / 32-B fp32 loads of dout, 8 fp32 global atomics).  Token ids repeat (position tables:
// every batch row hits the same ids), so the adds meet in L2 atomics rather than a sort; the fp32
// sum makes bf16 tables exact up to the final cast.  padding_idx rows receive no gradient.
#include "common.h"

using namespace lipa;

namespace {

__global__ __launch_bounds__(256) void embedding_fwd_k(const char* __restrict__ W, const int64_t* __restrict__ ids,
                                                       char* __restrict__ out, int64_t N, int row_chunks,
                                                       int64_t V, int* __restrict__ oob) {
  const int64_t c = (int64_t)blockIdx.x * 256 + threadIdx.x;   // global 16-B chunk index
  const int64_t n = c / row_chunks;
  if (n >= N) return;
  const int ch = (int)(c - n * row_chunks);
  int64_t id = ids[n];
  if (id < 0 || id >= V) {   // out-of-range id: flag it (the host checks the word lazily) and read a valid row
    if (oob) oob[0] = 1;
    id = id < 0 ? 0 : V - 1;
  }
  const u32x4 v = *reinterpret_cast<const u32x4*>(W + (id * row_chunks + ch) * 16);
  *reinterpret_cast<u32x4*>(out + (n * row_chunks + ch) * 16) = v;
}

template <typename T>
__global__ __launch_bounds__(256) void embedding_bwd_k(const T* __restrict__ dout, const int64_t* __restrict__ ids,
                                                       float* __restrict__ gw, int64_t N, int D, int64_t V,
                                                       int64_t padding_idx) {
  const int cpr = D / 8;
  const int64_t c = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t n = c / cpr;
  if (n >= N) return;
  const int d = (int)(c - n * cpr) * 8;
  const int64_t id = ids[n];
  if (id == padding_idx || id < 0 || id >= V) return;
  float v[8];
  load8(dout + n * D + d, v);
  float* g = gw + id * D + d;
#pragma unroll
  for (int i = 0; i < 8; ++i) atomicAdd(g + i, v[i]);
}

}  // namespace

bool embedding_supported(int64_t D, int64_t elem) { return (D * elem) % 16 == 0 && D % 8 == 0; }

void launch_embedding_fwd(const void* W, const int64_t* ids, void* out, int64_t N, int64_t D, int64_t elem, int64_t V,
                          int* oob, hipStream_t st) {
  if (N == 0) return;
  const int row_chunks = (int)(D * elem / 16);
  const int64_t chunks = N * row_chunks;
  embedding_fwd_k<<<(unsigned)((chunks + 255) / 256), 256, 0, st>>>((const char*)W, ids, (char*)out, N, row_chunks, V, oob);
  LIPA_CHECK_LAUNCH();
}

// dtype: 0 bf16, 1 fp32
void launch_embedding_bwd(const void* dout, int dtype, const int64_t* ids, float* gw, int64_t N, int64_t D, int64_t V,
                          int64_t padding_idx, hipStream_t st) {
  if (N == 0) return;
  const int64_t chunks = N * (D / 8);
  const unsigned grid = (unsigned)((chunks + 255) / 256);
  if (dtype == 0)
    embedding_bwd_k<bf16><<<grid, 256, 0, st>>>((const bf16*)dout, ids, gw, N, (int)D, V, padding_idx);
  else
    embedding_bwd_k<float><<<grid, 256, 0, st>>>((const float*)dout, ids, gw, N, (int)D, V, padding_idx);
  LIPA_CHECK_LAUNCH();
}
