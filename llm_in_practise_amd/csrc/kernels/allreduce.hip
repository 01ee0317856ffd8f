// Intra-node custom all-reduce over xGMI peer memory (the reference toggles
// vLLM's custom all-reduce, Quantization/LLM-Compressor/AWQ/eval_qwen3_4b_awq.py:20).
//
// MI355X: the 8 GPUs of a node are a full xGMI mesh (7 links per GPU), so a GPU can LOAD directly
// from every peer's HBM through IPC-mapped pointers.  For the latency-bound buffers of LoRA
// fine-tuning (a few MB of adapter gradients, grad-norm partials) a ring all-reduce pays 2·(W−1)
// link hops of latency; here one kernel does it with one or two cross-GPU barriers:
//
//   one-shot (small):  every rank reads all W peers' inputs and reduces the whole buffer locally
//                      (W−1 remote reads per element, one barrier).
//   two-shot (larger): rank r reduces slice r of the buffer from all peers into its result area,
//                      barrier, then every rank gathers the W reduced slices from their owners
//                      (2·(W−1)/W remote traffic per element, two barriers).
//
// Per rank, one IPC-shared staging allocation holds (see custom_allreduce.py for the layout):
//   data[2][cap]    the caller's input, copied in by the kernel (double-buffered on call parity)
//   result[2][cap]  two-shot reduced slices
// and a separate uncached flag allocation uint32 flags[NBAR][8 src][MAXB] per rank.
//
// Barrier k of call `epoch` in block b: lane p (< W) stores `epoch` into PEER p's
// flags[k][rank][b] (a per-lane vector store, system scope), then polls its OWN flags[k][p][b]
// until it reaches `epoch`.  Epochs only grow, so flags never need resetting.  Buffers alternate
// on epoch parity: a rank rewrites data[e&1] at call e+2 only after every peer passed barrier 0 of
// call e+1, i.e. finished reading call e.  Polls are bounded: a peer that never arrives sets
// err[0] and the block proceeds, so the grid always drains (the caller raises on err).
#include <cstring>

#include "common.h"

using namespace lipa;

namespace {

constexpr int MAXW = 8;
constexpr int MAXB = 64;          // blocks per launch (one flag slot each)
constexpr int NBAR = 2;
constexpr int NT = 512;

struct ARArgs {
  const char* data[MAXW];   // peer staging bases (data[rank] = own), already offset by parity
  char* result[MAXW];       // peer result areas, offset by parity
  uint32_t* flags[MAXW];    // peer flag arrays
  int* err;
  int W, rank;
  uint32_t epoch;
  size_t nvec;              // 16-B vectors in the buffer
  float scale;              // 1 (sum) or 1/W (avg)
};

__device__ __forceinline__ void vm_drain() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

__device__ void cross_barrier(const ARArgs& a, int k) {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");   // this thread's stores visible system-wide
  vm_drain();
  __syncthreads();
  const int p = threadIdx.x;
  if (p < a.W) {
    uint32_t* dst = a.flags[p] + ((size_t)k * MAXW + a.rank) * MAXB + blockIdx.x;
    __hip_atomic_store(dst, a.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    const uint32_t* mine = a.flags[a.rank] + ((size_t)k * MAXW + p) * MAXB + blockIdx.x;
    int spins = 0;
    while (__hip_atomic_load(mine, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) < a.epoch) {
      __builtin_amdgcn_s_sleep(2);
      if (++spins > (1 << 27)) {        // ~seconds: a peer is gone; report (barrier, peer) and drain
        a.err[0] = 1 + k + 2 * p;
        break;
      }
    }
  }
  __syncthreads();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
}

template <typename T>
__device__ __forceinline__ void add16(float (&acc)[16 / sizeof(T)], const char* p) {
  if constexpr (sizeof(T) == 2) {
    const bf16x8 v = *reinterpret_cast<const bf16x8*>(p);
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[i] += (float)v[i];
  } else {
    const f32x4 v = *reinterpret_cast<const f32x4*>(p);
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[i] += v[i];
  }
}

template <typename T>
__device__ __forceinline__ void store16(char* p, const float (&acc)[16 / sizeof(T)], float s) {
  if constexpr (sizeof(T) == 2) {
    bf16x8 v;
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = (bf16)(acc[i] * s);
    *reinterpret_cast<bf16x8*>(p) = v;
  } else {
    f32x4 v;
#pragma unroll
    for (int i = 0; i < 4; ++i) v[i] = acc[i] * s;
    *reinterpret_cast<f32x4*>(p) = v;
  }
}

// Every phase walks the SAME per-block vector set {v = blockIdx·NT + tid + k·stride}: the
// barrier pairs block b with block b on every peer, so a vector may only be read from a peer by
// the block whose peer twin wrote it (copy-in, slice reduce and gather alike).
template <typename T>
__device__ __forceinline__ void sum_peers(const ARArgs& a, size_t v, float (&acc)[16 / sizeof(T)]) {
#pragma unroll
  for (int i = 0; i < 16 / (int)sizeof(T); ++i) acc[i] = 0.f;
  // rotate the start peer by rank so the W ranks do not all hit the same peer first
#pragma unroll
  for (int j = 0; j < MAXW; ++j) {
    if (j < a.W) {
      const int p = (a.rank + j) % a.W;
      add16<T>(acc, a.data[p] + v * 16);
    }
  }
}

// copy-in by the kernel itself (not a separate copy launch): the stores go through this XCD's L2
// and the barrier's release writes them back before the flag
__device__ __forceinline__ void stage_in(const ARArgs& a, const char* in) {
  char* mine = const_cast<char*>(a.data[a.rank]);
  const size_t stride = (size_t)gridDim.x * NT;
  for (size_t v = (size_t)blockIdx.x * NT + threadIdx.x; v < a.nvec; v += stride)
    *reinterpret_cast<u32x4*>(mine + v * 16) = *reinterpret_cast<const u32x4*>(in + v * 16);
}

template <typename T>
__global__ __launch_bounds__(NT) void oneshot_k(ARArgs a, T* out) {
  char* o = reinterpret_cast<char*>(out);
  stage_in(a, o);
  cross_barrier(a, 0);
  const size_t stride = (size_t)gridDim.x * NT;
  for (size_t v = (size_t)blockIdx.x * NT + threadIdx.x; v < a.nvec; v += stride) {
    float acc[16 / sizeof(T)];
    sum_peers<T>(a, v, acc);
    store16<T>(o + v * 16, acc, a.scale);
  }
}

template <typename T>
__global__ __launch_bounds__(NT) void twoshot_k(ARArgs a, T* out) {
  char* o = reinterpret_cast<char*>(out);
  const size_t per = (a.nvec + a.W - 1) / a.W;
  const size_t s0 = min(a.nvec, per * a.rank), s1 = min(a.nvec, s0 + per);
  const size_t stride = (size_t)gridDim.x * NT;
  stage_in(a, o);
  cross_barrier(a, 0);
  for (size_t v = (size_t)blockIdx.x * NT + threadIdx.x; v < a.nvec; v += stride) {
    if (v < s0 || v >= s1) continue;              // my slice, reduced, into my result area
    float acc[16 / sizeof(T)];
    sum_peers<T>(a, v, acc);
    store16<T>(a.result[a.rank] + (v - s0) * 16, acc, a.scale);
  }
  cross_barrier(a, 1);
  for (size_t v = (size_t)blockIdx.x * NT + threadIdx.x; v < a.nvec; v += stride) {
    const int owner = (int)(v / per);
    *reinterpret_cast<u32x4*>(o + v * 16) = *reinterpret_cast<const u32x4*>(a.result[owner] + (v - per * owner) * 16);
  }
}

}  // namespace

// ---- host side -------------------------------------------------------------------------------
void* car_alloc(size_t bytes, bool uncached) {
  void* p = nullptr;
  if (uncached) {
    if (hipExtMallocWithFlags(&p, bytes, hipDeviceMallocUncached) != hipSuccess) return nullptr;
  } else if (hipMalloc(&p, bytes) != hipSuccess) {
    return nullptr;
  }
  if (hipMemset(p, 0, bytes) != hipSuccess) return nullptr;
  return p;
}

void car_free(void* p) { (void)hipFree(p); }

bool car_ipc_handle(void* p, char* out64) {
  hipIpcMemHandle_t h;
  if (hipIpcGetMemHandle(&h, p) != hipSuccess) return false;
  std::memcpy(out64, &h, sizeof(h));
  return true;
}

void* car_ipc_open(const char* h64) {
  hipIpcMemHandle_t h;
  std::memcpy(&h, h64, sizeof(h));
  void* p = nullptr;
  if (hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess) != hipSuccess) return nullptr;
  return p;
}

void car_ipc_close(void* p) { (void)hipIpcCloseMemHandle(p); }

int car_max_blocks() { return MAXB; }

// data/result/flags: W peer pointers each; data/result already include the parity offset
void launch_custom_allreduce(int dtype, const void* const* data, void* const* result, uint32_t* const* flags, int* err,
                             int W, int rank, uint32_t epoch, size_t bytes, bool two_shot, float scale, void* out,
                             int blocks, hipStream_t st) {
  ARArgs a;
  for (int i = 0; i < MAXW; ++i) {
    a.data[i] = i < W ? static_cast<const char*>(data[i]) : nullptr;
    a.result[i] = i < W ? static_cast<char*>(result[i]) : nullptr;
    a.flags[i] = i < W ? flags[i] : nullptr;
  }
  a.err = err;
  a.W = W;
  a.rank = rank;
  a.epoch = epoch;
  a.nvec = bytes / 16;
  a.scale = scale;
  blocks = blocks < 1 ? 1 : (blocks > MAXB ? MAXB : blocks);
  if (dtype == 1) {
    if (two_shot) twoshot_k<bf16><<<blocks, NT, 0, st>>>(a, static_cast<bf16*>(out));
    else oneshot_k<bf16><<<blocks, NT, 0, st>>>(a, static_cast<bf16*>(out));
  } else {
    if (two_shot) twoshot_k<float><<<blocks, NT, 0, st>>>(a, static_cast<float*>(out));
    else oneshot_k<float><<<blocks, NT, 0, st>>>(a, static_cast<float*>(out));
  }
  LIPA_CHECK_LAUNCH();
}
