// Fused LoRA low-rank kernels (SURVEY.md K8 + K13): every skinny product of a LoRA branch in one
// pass over the activations, with the input dropout mask regenerated in-kernel (never stored).
//
// A rank-r branch (r <= 16) of y += s·D(x)·Aᵀ·Bᵀ needs, per training step:
//   fwd  xa_s = s·D(x)·Aᵀ                 [M, r]   (feeds the base GEMM's extra K-slice)
//   bwd  g    = s·dy_i·B                  [M, r]
//        dA   = gᵀ·D(x)                   [r, K]
//        dB   = dy_iᵀ·xa_s                [n, r]
//        dx  += D'(g·A)                   [M, K]   (dropout branches; others fold into the base GEMM)
// The previous composition (dropout kernel → hipBLASLt skinny GEMMs → scale / cast / add
// kernels → materialised g·A) cost ≈125 µs per branch per step on Qwen3-8B shapes (rocprofv3,
// profiles/bench_qwen3_8b_qlora_kernels_v2.txt) for ≈20 µs of compulsory HBM traffic.
//
// lora_proj_k  (MFMA): out[m, j] = scale·Σ_k D(X)[m,k]·W[j,k] — a workgroup = 16 rows × 1024 of K
//              (grid M/16 × K/1024 for enough memory parallelism), its 4 waves each own 256 of K with
//              all 8 fragment loads in flight, v_mfma_f32_16x16x32_bf16 with X rows as the A operand
//              (dropout applied to the fragment) and W rows as the B operand; LDS reduction of the 4
//              partials, one fp32 atomic add per output element per workgroup.
// lora_acc_k   (VALU): part[c][j][k] = Σ_{m∈chunk c} G[m,j]·D(X)[m,k]  and optionally
//              DX[m,k] += D(Σ_j G[m,j]·W[j,k]) — each thread owns 8 consecutive k of one row stream,
//              reads X and DX once; the per-chunk (64-row) partials are summed by the caller.
#include <cstdlib>

#include <algorithm>

#include "common.h"

using namespace lipa;

namespace {

// One workgroup = 16 rows × ALL of K: its NW waves each own K/NW (all fragment loads of a wave in
// flight at once), partials meet in LDS and the result is written once (fp32 and/or bf16) — no
// atomics, no zero-initialised output, no follow-up cast kernel.
template <int NW, int RW>
__device__ __forceinline__ void lora_proj_body(const bf16* __restrict__ X, int ldx, const bf16* __restrict__ W, int r,
                                               int K, float* __restrict__ outf, int ldof, bf16* __restrict__ outb,
                                               int ldob, int M, uint64_t key, uint32_t thr16, float dscale,
                                               float scale, size_t mask_ld, int bx) {
  __shared__ f32x4 red[NW][64];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int m0 = bx * RW;
  const bool rv = (lane & 15) < RW;   // RW = 8: MFMA rows 8..15 are zero padding (twice the workgroups)
  const int row = min(m0 + (lane & 15), M - 1);
  const int kw = K / NW;
  const int kbeg = w * kw;
  const bf16* xr = X + (size_t)row * ldx;
  const int n = lane & 15;
  const bf16* wr = W + (size_t)(n < r ? n : 0) * K;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  for (int k0 = kbeg; k0 < kbeg + kw; k0 += 8 * 32) {
    bf16x8 av[8], bv[8];
    const int ns = min(8, (kbeg + kw - k0) / 32);
#pragma unroll
    for (int s = 0; s < 8; ++s)
      if (s < ns) {
        const int k = k0 + s * 32 + 8 * (lane >> 4);
        av[s] = rv ? *reinterpret_cast<const bf16x8*>(xr + k) : bf16x8{};
        bv[s] = *reinterpret_cast<const bf16x8*>(wr + k);
      }
#pragma unroll
    for (int s = 0; s < 8; ++s)
      if (s < ns) {
        bf16x8 a = av[s];
        if (thr16 && rv) {
          const int k = k0 + s * 32 + 8 * (lane >> 4);
          const uint32_t keep = dropout_keep8(key, ((size_t)row * mask_ld + k) >> 3, thr16);
#pragma unroll
          for (int i = 0; i < 8; ++i) a[i] = ((keep >> i) & 1) ? (bf16)((float)a[i] * dscale) : (bf16)0.f;
        }
        const bf16x8 b = n < r ? bv[s] : bf16x8{};
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc, 0, 0, 0);
      }
  }
  red[w][lane] = acc;
  __syncthreads();
  if (w != 0) return;
  f32x4 t = red[0][lane];
#pragma unroll
  for (int i = 1; i < NW; ++i) t += red[i][lane];
  // D layout: col = lane & 15 (output j), rows 4*(lane>>4)+i (token)
  const int j = lane & 15;
  if (j >= r) return;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int ml = 4 * (lane >> 4) + i, m = m0 + ml;
    if (ml >= RW || m >= M) continue;
    const float v = t[i] * scale;
    if (outf) outf[(size_t)m * ldof + j] = v;
    if (outb) outb[(size_t)m * ldob + j] = (bf16)v;
  }
}

template <int NW, int RW>
__global__ __launch_bounds__(NW * 64) void lora_proj_k(const bf16* __restrict__ X, int ldx, const bf16* __restrict__ W,
                                                      int r, int K, float* __restrict__ outf, int ldof,
                                                      bf16* __restrict__ outb, int ldob, int M, uint64_t key,
                                                      uint32_t thr16, float dscale, float scale, size_t mask_ld) {
  lora_proj_body<NW, RW>(X, ldx, W, r, K, outf, ldof, outb, ldob, M, key, thr16, dscale, scale, mask_ld, blockIdx.x);
}

// two independent projections of one launch (blockIdx.y = branch): the backward's s·dy_i·B_i of
// q_proj and v_proj, each over its own column range of dy — one launch, one tail
struct ProjPair {
  const bf16* X[2];
  const bf16* W[2];
  float* out[2];
  int K[2];
  float scale[2];
};
template <int NW, int RW>
__global__ __launch_bounds__(NW * 64) void lora_proj_pair_k(ProjPair p, int ldx, int r, int M) {
  const int b = blockIdx.y;
  lora_proj_body<NW, RW>(p.X[b], ldx, p.W[b], r, p.K[b], p.out[b], r, nullptr, 0, M, 0, 0u, 1.f, p.scale[b], 0,
                         blockIdx.x);
}

// NRL row-lanes × 64 k-threads (8 consecutive k each); a chunk of ROWS rows is walked in passes of
// NRL·RB rows (RB rows per thread), the next pass's x / dx rows loaded before the current pass is
// used (one exposed HBM round trip per workgroup, not one per pass); the chunk's G rows are staged
// in LDS.  Taller chunks mean fewer workgroups and fewer fp32 atomics per output element.
template <int R, bool DXU, int NRL, int ROWS>
__global__ __launch_bounds__(NRL * 64) void lora_acc_k(const float* __restrict__ G, int ldg, int r,
                                                      const bf16* __restrict__ X, int ldx, bf16* __restrict__ DX,
                                                      int lddx, const bf16* __restrict__ W, int K,
                                                      float* __restrict__ out, int64_t sj, int64_t sk,
                                                      float* __restrict__ part, int M, uint64_t key, uint32_t thr16,
                                                      float dscale, size_t mask_ld) {
  constexpr int RB = (ROWS / NRL) < 8 ? (ROWS / NRL) : 8;
  constexpr int NP = ROWS / (NRL * RB);
  constexpr int NT = NRL * 64;
  __shared__ float red[64][R * 8 + 1];
  __shared__ float gs[ROWS][R];
  const int tid = threadIdx.x;
  const int kv = blockIdx.x * 64 + (tid & 63), rl = tid >> 6;
  const int k0 = kv * 8;
  const bool kin = k0 < K;
  const int mb = blockIdx.y * ROWS, me = min(mb + ROWS, M);
  for (int i = tid; i < ROWS * R; i += NT) {
    const int m = mb + i / R, j = i % R;
    gs[i / R][j] = (m < me && j < r) ? G[(size_t)m * ldg + j] : 0.f;
  }
  bf16x8 wv[DXU ? R : 1];
  if constexpr (DXU) {
#pragma unroll
    for (int j = 0; j < R; ++j) wv[j] = (kin && j < r) ? *reinterpret_cast<const bf16x8*>(W + (size_t)j * K + k0) : bf16x8{};
  }
  bf16x8 xb[2][RB], db[2][DXU ? RB : 1];
  auto load = [&](int buf, int pass) {
#pragma unroll
    for (int q = 0; q < RB; ++q) {
      const int m = min(mb + pass * NRL * RB + rl + NRL * q, M - 1);
      if (kin) {
        xb[buf][q] = *reinterpret_cast<const bf16x8*>(X + (size_t)m * ldx + k0);
        if constexpr (DXU) db[buf][q] = *reinterpret_cast<const bf16x8*>(DX + (size_t)m * lddx + k0);
      }
    }
  };
  load(0, 0);
  __syncthreads();  // gs ready
  float acc[R][8];
#pragma unroll
  for (int j = 0; j < R; ++j)
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[j][i] = 0.f;
  const float ds = thr16 ? dscale : 1.f;
#pragma unroll
  for (int pass = 0; pass < NP; ++pass) {
    const int cur = pass & 1;
    if (pass + 1 < NP) load(cur ^ 1, pass + 1);
#pragma unroll
    for (int q = 0; q < RB; ++q) {
      const int ml = pass * NRL * RB + rl + NRL * q, m = mb + ml;
      if (!kin || m >= me) continue;
      const uint32_t keep = thr16 ? dropout_keep8(key, ((size_t)m * mask_ld + k0) >> 3, thr16) : 0xFFu;
      float xv[8], g[R];
#pragma unroll
      for (int i = 0; i < 8; ++i) xv[i] = ((keep >> i) & 1) ? (float)xb[cur][q][i] * ds : 0.f;
#pragma unroll
      for (int j = 0; j < R; ++j) g[j] = gs[ml][j];
#pragma unroll
      for (int j = 0; j < R; ++j)
#pragma unroll
        for (int i = 0; i < 8; ++i) acc[j][i] += g[j] * xv[i];
      if constexpr (DXU) {
        float t[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) t[i] = 0.f;
#pragma unroll
        for (int j = 0; j < R; ++j)
#pragma unroll
          for (int i = 0; i < 8; ++i) t[i] += g[j] * (float)wv[j][i];
        bf16x8 o;
#pragma unroll
        for (int i = 0; i < 8; ++i) o[i] = (bf16)((float)db[cur][q][i] + (((keep >> i) & 1) ? t[i] * ds : 0.f));
        *reinterpret_cast<bf16x8*>(DX + (size_t)m * lddx + k0) = o;
      }
    }
  }
  // reduce the NRL row-lanes through LDS (one wave at a time), then write this chunk's partial
  for (int s2 = 0; s2 < NRL; ++s2) {
    if (rl == s2) {
#pragma unroll
      for (int j = 0; j < R; ++j)
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          float& dst = red[tid & 63][j * 8 + i];
          dst = (s2 == 0 ? 0.f : dst) + acc[j][i];
        }
    }
    __syncthreads();
  }
  // this workgroup's 512-wide k block: threads add j-rows with consecutive k per lane (full-rate
  // 256-B atomic wave instructions when sk == 1), straight into the fp32 destination (the grad)
  const int kb = blockIdx.x * 512;
  const bool jfast = sj == 1;        // order lanes along the destination's unit stride (full-rate atomics)
  for (int idx = tid; idx < r * 512; idx += NT) {
    const int j = jfast ? idx % r : idx / 512, kk = jfast ? idx / r : idx % 512;
    if (kb + kk >= K) continue;
    const float v = red[kk / 8][j * 8 + (kk & 7)];
    if (part)   // deterministic mode: per-chunk partial, summed in a fixed order by the caller
      part[((size_t)blockIdx.y * r + j) * K + kb + kk] = v;
    else
      atomicAdd(out + j * sj + (int64_t)(kb + kk) * sk, v);
  }
}


// lora_acc on the matrix cores: part[j][k] = Σ_m G[m,j]·D(X)[m,k] as v_mfma_f32_16x16x32_bf16 with
// the rank index j as the 16 MFMA rows (r <= 16), k as the columns and m as the reduction.  The
// reduction runs down the columns of the row-major X, so no LDS transpose: lane (q = l/16, n = l%16)
// loads 8 rows m0+8q+e of one 8-k chunk k8 = kb+8n (16 B each, 16 lanes = one 256-B row segment)
// and that 8x8 register block supplies the B operand of 8 MFMAs, MFMA c taking column k8+c of all
// 8 rows (so MFMA c's 16 columns are k = kb+8n+c, n = 0..15).  The VALU kernel above spent 2·R
// FMAs per element and ran VALU-bound at 1-2 TB/s; here the dA / dB product is ≈ 1 % of MFMA time.
// A workgroup = 4 waves stacked in m (SUB 32-row steps each) over one 128-wide k block; the waves'
// partials meet in LDS and leave as one fp32 atomic per output per workgroup.  With DXU, each lane
// also applies dx[m, k8..k8+7] += D(Σ_j G[m,j]·W[j,k]) to the rows it holds (VALU, R FMAs/element).
template <int R, bool DXU, int SUB>
__device__ __forceinline__ void lora_acc_mfma_body(const float* __restrict__ G, int ldg, int r,
                                                   const bf16* __restrict__ X, int ldx, bf16* __restrict__ DX,
                                                   int lddx, const bf16* __restrict__ W, int K,
                                                   float* __restrict__ out, int64_t sj, int64_t sk, int M,
                                                   uint64_t key, uint32_t thr16, float dscale, size_t mask_ld, int bx,
                                                   int by, const uint8_t* __restrict__ kbits = nullptr) {
  __shared__ float red[4][64][33];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int q = lane >> 4, n = lane & 15;
  const int kb = bx * 128;
  const int k8 = kb + 8 * n;
  const int mw = by * (128 * SUB) + w * (32 * SUB);
  bf16x8 wv[DXU ? R : 1];
  if constexpr (DXU) {
#pragma unroll
    for (int j = 0; j < R; ++j) wv[j] = j < r ? *reinterpret_cast<const bf16x8*>(W + (size_t)j * K + k8) : bf16x8{};
  }
  f32x4 acc[8];
#pragma unroll
  for (int c = 0; c < 8; ++c) acc[c] = f32x4{0.f, 0.f, 0.f, 0.f};
  const float ds = thr16 ? dscale : 1.f;
#pragma unroll
  for (int s = 0; s < SUB; ++s) {
    const int m0 = mw + 32 * s + 8 * q;
    bf16x8 xb[8], db[DXU ? 8 : 1];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int m = min(m0 + e, M - 1);
      xb[e] = *reinterpret_cast<const bf16x8*>(X + (size_t)m * ldx + k8);
      if constexpr (DXU) db[e] = *reinterpret_cast<const bf16x8*>(DX + (size_t)m * lddx + k8);
    }
    bf16x8 a;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int m = m0 + e;
      a[e] = (bf16)((m < M && n < r) ? G[(size_t)m * ldg + n] : 0.f);
    }
    uint32_t keep[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int m = m0 + e;
      keep[e] = m >= M ? 0u
                       : kbits ? (uint32_t)kbits[(size_t)m * (K >> 3) + (k8 >> 3)]   // stored by lora_proj2
                               : (thr16 ? dropout_keep8(key, ((size_t)m * mask_ld + k8) >> 3, thr16) : 0xFFu);
    }
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      bf16x8 b;
#pragma unroll
      for (int e = 0; e < 8; ++e) b[e] = ((keep[e] >> c) & 1) ? xb[e][c] : (bf16)0.f;
      acc[c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc[c], 0, 0, 0);
    }
    if constexpr (DXU) {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int m = m0 + e;
        if (m >= M) continue;
        float gr[R];
#pragma unroll
        for (int j = 0; j < R; j += 4) {
          if (j < r) {
            const f32x4 t4 = *reinterpret_cast<const f32x4*>(G + (size_t)m * ldg + j);
#pragma unroll
            for (int u = 0; u < 4; ++u) gr[j + u] = j + u < r ? t4[u] : 0.f;   // never touch padding columns
          } else {
            gr[j] = gr[j + 1] = gr[j + 2] = gr[j + 3] = 0.f;
          }
        }
        float t[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) t[i] = 0.f;
#pragma unroll
        for (int j = 0; j < R; ++j)
#pragma unroll
          for (int i = 0; i < 8; ++i) t[i] += gr[j] * (float)wv[j][i];
        bf16x8 o;
#pragma unroll
        for (int i = 0; i < 8; ++i) o[i] = (bf16)((float)db[e][i] + (((keep[e] >> i) & 1) ? t[i] * ds : 0.f));
        *reinterpret_cast<bf16x8*>(DX + (size_t)m * lddx + k8) = o;
      }
    }
  }
  // acc[c][t] = part[j = 4q + t][k = kb + 8n + c]
#pragma unroll
  for (int c = 0; c < 8; ++c)
#pragma unroll
    for (int t = 0; t < 4; ++t) red[w][lane][c * 4 + t] = acc[c][t];
  __syncthreads();
  const bool jfast = sj == 1;   // consecutive threads along the destination's unit stride
  for (int idx = threadIdx.x; idx < r * 128; idx += 256) {
    const int j = jfast ? idx % r : idx / 128, kk = jfast ? idx / r : idx % 128;
    const int ln = 16 * (j >> 2) + (kk >> 3), slot = (kk & 7) * 4 + (j & 3);
    const float v = (red[0][ln][slot] + red[1][ln][slot] + red[2][ln][slot] + red[3][ln][slot]) * ds;
    atomicAdd(out + j * sj + (int64_t)(kb + kk) * sk, v);
  }
}

template <int R, bool DXU, int SUB>
__global__ __launch_bounds__(256) void lora_acc_mfma_k(const float* __restrict__ G, int ldg, int r,
                                                      const bf16* __restrict__ X, int ldx, bf16* __restrict__ DX,
                                                      int lddx, const bf16* __restrict__ W, int K,
                                                      float* __restrict__ out, int64_t sj, int64_t sk, int M,
                                                      uint64_t key, uint32_t thr16, float dscale, size_t mask_ld) {
  lora_acc_mfma_body<R, DXU, SUB>(G, ldg, r, X, ldx, DX, lddx, W, K, out, sj, sk, M, key, thr16, dscale, mask_ld,
                                  blockIdx.x, blockIdx.y);
}

// dB_i [n_i, r] += (dy[:, c0_i : c0_i + n_i])ᵀ · xa_i for two branches in one launch (the k-blocks of
// branch 1 follow those of branch 0 along blockIdx.x)
struct AccPair {
  const float* G[2];
  const bf16* X[2];
  float* out[2];
  int K[2];
  int nblk0;
  int64_t sj[2], sk[2];
  float ds[2];            // dropout rescale 1/(1-p) (1: no dropout)
  const uint8_t* kb[2];   // keep bits [M, K/8] (null: no dropout)
};
template <int SUB>
__global__ __launch_bounds__(256) void lora_acc_pair_k(AccPair a, int ldg, int r, int ldx, int M) {
  const int b = (int)blockIdx.x >= a.nblk0;
  const int bx = blockIdx.x - (b ? a.nblk0 : 0);
  lora_acc_mfma_body<8, false, SUB>(a.G[b], ldg, r, a.X[b], ldx, nullptr, 0, nullptr, a.K[b], a.out[b], a.sj[b],
                                    a.sk[b], M, 0, a.kb[b] ? 1u : 0u, a.ds[b], 0, bx, blockIdx.y, a.kb[b]);
}

// The q+v backward's four weight-gradient products in ONE launch (job = blockIdx.x range): dB_q, dB_v
// (dy column blocks × the forward's xa) and dA_q, dA_v (x with the stored keep bits × g) — the same
// MFMA body as lora_acc_pair_k, each job with its own operands and strides; one launch, one tail
// (two back-to-back launches of ≈10 µs each left half of each launch's last wave of workgroups idle).
// The general form (AccJobs, up to 8 jobs, rank per job) serves the multi-adapter backward as well: all
// dB and dA products of a projection's 1-4 adapters (BASELINE #2: q, k, v on q|k|v and o) in one launch.
// (Grouping the dA jobs that share x so that one workgroup loads each x tile once for all members measured
// slower at BASELINE #2's shapes: q|k|v 45 -> 62 µs — a third of the workgroups, and the re-reads of x hit
// the MALL anyway; profiles/r4/lora_multi_adapter.txt.)
constexpr int kAccJobs = 8;
struct AccJobs {
  const float* G[kAccJobs];
  const bf16* X[kAccJobs];
  float* out[kAccJobs];
  int K[kAccJobs], nb[kAccJobs], ldg[kAccJobs], ldx[kAccJobs], r[kAccJobs];   // nb: first blockIdx.x of the job
  int64_t sj[kAccJobs], sk[kAccJobs];
  float ds[kAccJobs];
  const uint8_t* kb[kAccJobs];
  int njobs;
};
// XCD-aware order: the hardware deals workgroups round-robin over the 8 XCDs (each with its own L2); the
// logical order runs along k fastest, so the workgroups that read one row block's G rows and keep-bit lines
// (partial 128-B lines per workgroup) sit on ONE XCD instead of pulling the same lines into all eight L2s.
__device__ __forceinline__ void xcd_grid(int& bx, int& by) {
  const int gx = gridDim.x, nwg = gx * gridDim.y;
  const int lid = xcd_remap(blockIdx.y * gx + blockIdx.x, nwg);
  bx = lid % gx;
  by = lid / gx;
}
template <int SUB>
__global__ __launch_bounds__(256) void lora_acc_jobs_k(AccJobs a, int M) {
  int bx0, by;
  xcd_grid(bx0, by);
  int j = 0;
#pragma unroll
  for (int i = 1; i < kAccJobs; ++i)
    if (i < a.njobs && bx0 >= a.nb[i]) j = i;
  lora_acc_mfma_body<8, false, SUB>(a.G[j], a.ldg[j], a.r[j], a.X[j], a.ldx[j], nullptr, 0, nullptr, a.K[j], a.out[j],
                                    a.sj[j], a.sk[j], M, 0, a.kb[j] ? 1u : 0u, a.ds[j], 0, bx0 - a.nb[j], by,
                                    a.kb[j]);
}

// dx_lora[m, k] = Σ_i D_i[m, k]·ds_i·Σ_j G_i[m, j]·A_i[j, k] for the two branches (bf16 [M, K]): the LoRA
// input-gradient term, written once and handed to the dX GEMM as its C matrix (no read-modify-write
// pass over dx).  A thread owns 8 consecutive k of 8 rows; A's 8 k-columns are loaded once per thread.
template <int RPT>
__global__ __launch_bounds__(256) void lora_dx2_k(const float* __restrict__ G0, const float* __restrict__ G1, int ldg,
                                                  const bf16* __restrict__ A0, const bf16* __restrict__ A1, int r0,
                                                  int r1, const uint8_t* __restrict__ kb0,
                                                  const uint8_t* __restrict__ kb1, float ds0, float ds1,
                                                  bf16* __restrict__ out, int M, int K) {
  const int kv = blockIdx.x * 64 + (threadIdx.x & 63);
  const int k8 = kv * 8;
  if (k8 >= K) return;
  const int m0 = (blockIdx.y * 4 + (threadIdx.x >> 6)) * RPT;
  // every load of the thread issued up front (A columns stay packed bf16; G rows and keep bytes of
  // all RPT rows), then the math: one exposed memory round trip per thread
  bf16x8 av0[8], av1[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    av0[j] = j < r0 ? *reinterpret_cast<const bf16x8*>(A0 + (size_t)j * K + k8) : bf16x8{};
    av1[j] = j < r1 ? *reinterpret_cast<const bf16x8*>(A1 + (size_t)j * K + k8) : bf16x8{};
  }
  f32x4 gq0[RPT][2], gq1[RPT][2];
  uint32_t kp0[RPT], kp1[RPT];
#pragma unroll
  for (int e = 0; e < RPT; ++e) {
    const int m = min(m0 + e, M - 1);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      gq0[e][h] = *reinterpret_cast<const f32x4*>(G0 + (size_t)m * ldg + 4 * h);
      gq1[e][h] = *reinterpret_cast<const f32x4*>(G1 + (size_t)m * ldg + 4 * h);
    }
    kp0[e] = kb0 ? kb0[(size_t)m * (K >> 3) + kv] : 0xFFu;
    kp1[e] = kb1 ? kb1[(size_t)m * (K >> 3) + kv] : 0xFFu;
  }
#pragma unroll
  for (int e = 0; e < RPT; ++e) {
    const int m = m0 + e;
    if (m >= M) break;
    float t0[8], t1[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) t0[i] = t1[i] = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float g0 = j < r0 ? gq0[e][j >> 2][j & 3] : 0.f;
      const float g1 = j < r1 ? gq1[e][j >> 2][j & 3] : 0.f;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        t0[i] += g0 * (float)av0[j][i];
        t1[i] += g1 * (float)av1[j][i];
      }
    }
    float o[8];
#pragma unroll
    for (int i = 0; i < 8; ++i)
      o[i] = (((kp0[e] >> i) & 1) ? t0[i] * ds0 : 0.f) + (((kp1[e] >> i) & 1) ? t1[i] * ds1 : 0.f);
    store8(out + (size_t)m * K + k8, o);
  }
}

// lora_dx2 with A read once per 16 rows: a thread owns 8 consecutive k of 16 rows (workgroup = 2048 k ×
// 16 rows), the 16 rows' G values (both branches) are staged once in LDS, and every keep byte of the
// thread is loaded up front.  The 4-row form above re-read A's 8 k-columns (both adapters: 256 B per
// thread) for every 4 rows — 64 MB of L2 reads per call at the bench shape for 16 MB of output.
__global__ __launch_bounds__(256) void lora_dx2_r16_k(const float* __restrict__ G0, const float* __restrict__ G1,
                                                      int ldg, const bf16* __restrict__ A0,
                                                      const bf16* __restrict__ A1, int r0, int r1,
                                                      const uint8_t* __restrict__ kb0,
                                                      const uint8_t* __restrict__ kb1, float ds0, float ds1,
                                                      bf16* __restrict__ out, int M, int K) {
  __shared__ float gs[16][2][8];
  const int m0 = blockIdx.y * 16;
  {
    const int t = threadIdx.x, e = t >> 4, br = (t >> 3) & 1, j = t & 7;
    const int m = min(m0 + e, M - 1);
    const int rr = br ? r1 : r0;
    gs[e][br][j] = j < rr ? (br ? G1 : G0)[(size_t)m * ldg + j] : 0.f;
  }
  const int kv = blockIdx.x * 256 + threadIdx.x;
  const int k8 = kv * 8;
  const bool live = k8 < K;
  bf16x8 av0[8], av1[8];
  uint32_t kp0[16], kp1[16];
  if (live) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      av0[j] = j < r0 ? *reinterpret_cast<const bf16x8*>(A0 + (size_t)j * K + k8) : bf16x8{};
      av1[j] = j < r1 ? *reinterpret_cast<const bf16x8*>(A1 + (size_t)j * K + k8) : bf16x8{};
    }
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const int m = min(m0 + e, M - 1);
      kp0[e] = kb0 ? kb0[(size_t)m * (K >> 3) + kv] : 0xFFu;
      kp1[e] = kb1 ? kb1[(size_t)m * (K >> 3) + kv] : 0xFFu;
    }
  }
  __syncthreads();
  if (!live) return;
#pragma unroll 4
  for (int e = 0; e < 16; ++e) {
    const int m = m0 + e;
    if (m >= M) break;
    float t0[8], t1[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) t0[i] = t1[i] = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float g0 = gs[e][0][j], g1 = gs[e][1][j];
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        t0[i] += g0 * (float)av0[j][i];
        t1[i] += g1 * (float)av1[j][i];
      }
    }
    float o[8];
#pragma unroll
    for (int i = 0; i < 8; ++i)
      o[i] = (((kp0[e] >> i) & 1) ? t0[i] * ds0 : 0.f) + (((kp1[e] >> i) & 1) ? t1[i] * ds1 : 0.f);
    store8(out + (size_t)m * K + k8, o);
  }
}

// ---- two branches sharing one input (q_proj + v_proj of a fused q|k|v projection) -------------
// Each pass over x serves BOTH adapters: the x fragment is loaded once and masked twice (the two
// branches' independent dropout streams), so the activations are read once per projection instead
// of once per adapter.

// lora_proj for two branches: A0 [r0, K], A1 [r1, K] (r0 + r1 <= 16); output columns j < r0 are
// branch 0 (its mask, scale), the rest branch 1.  Two MFMAs per k-step, each against the rows of
// its own branch (the other branch's B rows are zero), accumulate into one 16-column tile.
template <int NW, int RW>
__global__ __launch_bounds__(NW * 64) void lora_proj2_k(const bf16* __restrict__ X, int ldx, const bf16* __restrict__ W0,
                                                       const bf16* __restrict__ W1, int r0, int r, int K, float* __restrict__ outf, int ldof,
                                                       bf16* __restrict__ outb, int ldob, int M, uint64_t key0,
                                                       uint64_t key1, uint32_t thr0, uint32_t thr1, float ds0,
                                                       float ds1, float scale0, float scale1, size_t mask_ld,
                                                       uint8_t* __restrict__ mko) {
  __shared__ f32x4 red[NW][64];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int m0 = blockIdx.x * RW;
  const bool rv = (lane & 15) < RW;
  const int row = min(m0 + (lane & 15), M - 1);
  const int kw = K / NW;
  const int kbeg = w * kw;
  const bf16* xr = X + (size_t)row * ldx;
  const int n = lane & 15;
  const bf16* wr = n < r0 ? W0 + (size_t)n * K : (n < r ? W1 + (size_t)(n - r0) * K : W0);
  const bool in0 = n < r0, in1 = n >= r0 && n < r;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  for (int k0 = kbeg; k0 < kbeg + kw; k0 += 8 * 32) {
    bf16x8 av[8], bv[8];
    const int ns = min(8, (kbeg + kw - k0) / 32);
#pragma unroll
    for (int s = 0; s < 8; ++s)
      if (s < ns) {
        const int k = k0 + s * 32 + 8 * (lane >> 4);
        av[s] = rv ? *reinterpret_cast<const bf16x8*>(xr + k) : bf16x8{};
        bv[s] = *reinterpret_cast<const bf16x8*>(wr + k);
      }
#pragma unroll
    for (int s = 0; s < 8; ++s)
      if (s < ns) {
        const int k = k0 + s * 32 + 8 * (lane >> 4);
        const size_t v8 = ((size_t)row * mask_ld + k) >> 3;
        // padding rows (RW = 8: lanes 8..15) draw no mask: their x fragment is zero anyway
        const uint32_t keep0 = thr0 && rv ? dropout_keep8(key0, v8, thr0) : 0xFFu;
        const uint32_t keep1 = thr1 && rv ? dropout_keep8(key1, v8, thr1) : 0xFFu;
        if (mko && rv && m0 + (lane & 15) < M) {   // the keep bits for the backward (1 bit / element)
          const size_t mi = (size_t)row * (K >> 3) + (k >> 3);
          mko[mi] = (uint8_t)keep0;
          mko[(size_t)M * (K >> 3) + mi] = (uint8_t)keep1;
        }
        const float d0 = thr0 ? ds0 : 1.f, d1 = thr1 ? ds1 : 1.f;
        bf16x8 a0, a1;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const float xv = (float)av[s][i];
          a0[i] = ((keep0 >> i) & 1) ? (bf16)(xv * d0) : (bf16)0.f;
          a1[i] = ((keep1 >> i) & 1) ? (bf16)(xv * d1) : (bf16)0.f;
        }
        const bf16x8 b0 = in0 ? bv[s] : bf16x8{};
        const bf16x8 b1 = in1 ? bv[s] : bf16x8{};
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0, b0, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1, b1, acc, 0, 0, 0);
      }
  }
  red[w][lane] = acc;
  __syncthreads();
  if (w != 0) return;
  f32x4 t = red[0][lane];
#pragma unroll
  for (int i = 1; i < NW; ++i) t += red[i][lane];
  const int j = lane & 15;
  if (j >= r) return;
  const float sc = j < r0 ? scale0 : scale1;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int ml = 4 * (lane >> 4) + i, m = m0 + ml;
    if (ml >= RW || m >= M) continue;
    const float v = t[i] * sc;
    if (outf) outf[(size_t)m * ldof + j] = v;
    if (outb) outb[(size_t)m * ldob + j] = (bf16)v;
  }
}

// Split-K form of lora_proj2 (the default when K is a multiple of 128).  lora_proj2_k above gives a
// workgroup 8 rows × all of K, so every workgroup re-reads all of [A0; A1] (128 KB at K = 4096) for
// 64 KB of x: 3× the compulsory traffic and one exposed round trip — 14 µs without dropout, 23 µs
// with it and the keep bits (rocprofv3, wait_any 0.63 of wave cycles).  Here a workgroup is 64 rows
// × KC = 4·NS·32 of K (grid K/KC × M/64 = 256 workgroups at the bench shape): each wave holds its
// NS B fragments of [A0; A1] for four 16-row MFMA blocks (A traffic 1/4 of x), every load of the
// wave is issued before the first MFMA, and the 4 waves' partials meet in LDS and leave as one
// fp32 [M, 16] slab per K chunk; lora_proj2_sum_k adds the slabs in a fixed order (deterministic).
// Lane (g = lane/16) owns NS·8 CONSECUTIVE k (MFMA step s, k-slot g ↔ k = kl + 8s): the MFMA sum
// over k is order-free, and the lane's keep bytes are contiguous → one NS-byte store per branch.
// Dropout masks the bf16 x fragment with a bitwise AND (no convert / multiply / re-round); the
// 1/(1-p) factor is folded into the output scale.
template <int NS>
__global__ __launch_bounds__(256) void lora_proj2s_k(const bf16* __restrict__ X, int ldx, const bf16* __restrict__ W0,
                                                    const bf16* __restrict__ W1, int r0, int r, int K, int M,
                                                    uint64_t key0, uint64_t key1, uint32_t thr0, uint32_t thr1,
                                                    size_t mask_ld, uint8_t* __restrict__ mko, float* __restrict__ ws) {
  constexpr int KW = NS * 32, KC = 4 * KW;
  __shared__ f32x4 red[4][4][64];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int g = lane >> 4, n = lane & 15;
  const int kc = blockIdx.x, m0 = blockIdx.y * 64;
  const int kl = kc * KC + w * KW + g * (NS * 8);
  const bool in0 = n < r0, in1 = n >= r0 && n < r;
  const bf16* wr = in0 ? W0 + (size_t)n * K : (in1 ? W1 + (size_t)(n - r0) * K : W0);
  bf16x8 bv[NS], xv[4][NS];
#pragma unroll
  for (int s = 0; s < NS; ++s) bv[s] = *reinterpret_cast<const bf16x8*>(wr + kl + 8 * s);
#pragma unroll
  for (int b = 0; b < 4; ++b) {
    const int row = min(m0 + 16 * b + n, M - 1);
#pragma unroll
    for (int s = 0; s < NS; ++s) xv[b][s] = *reinterpret_cast<const bf16x8*>(X + (size_t)row * ldx + kl + 8 * s);
  }
  f32x4 acc[4];
#pragma unroll
  for (int b = 0; b < 4; ++b) acc[b] = f32x4{0.f, 0.f, 0.f, 0.f};
  if ((thr0 | thr1) == 0) {
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      const bf16x8 bb = (in0 || in1) ? bv[s] : bf16x8{};
#pragma unroll
      for (int b = 0; b < 4; ++b) acc[b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xv[b][s], bb, acc[b], 0, 0, 0);
    }
  } else {
    // every keep byte first: the hash is independent of the loads in flight, so it runs under them
    uint32_t kp0[4], kp1[4];
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      const int row = min(m0 + 16 * b + n, M - 1);
      kp0[b] = 0;
      kp1[b] = 0;
#pragma unroll
      for (int s = 0; s < NS; ++s) {
        const size_t v8 = ((size_t)row * mask_ld + kl + 8 * s) >> 3;
        kp0[b] |= (thr0 ? dropout_keep8(key0, v8, thr0) : 0xFFu) << (8 * s);
        kp1[b] |= (thr1 ? dropout_keep8(key1, v8, thr1) : 0xFFu) << (8 * s);
      }
      const int mg = m0 + 16 * b + n;
      if (mko && mg < M) {   // the keep bits for the backward (1 bit / element), NS bytes per branch
        const size_t mi = (size_t)mg * (K >> 3) + (kl >> 3);
        if constexpr (NS == 4) {
          *reinterpret_cast<uint32_t*>(mko + mi) = kp0[b];
          *reinterpret_cast<uint32_t*>(mko + (size_t)M * (K >> 3) + mi) = kp1[b];
        } else if constexpr (NS == 2) {
          *reinterpret_cast<uint16_t*>(mko + mi) = (uint16_t)kp0[b];
          *reinterpret_cast<uint16_t*>(mko + (size_t)M * (K >> 3) + mi) = (uint16_t)kp1[b];
        } else {
          mko[mi] = (uint8_t)kp0[b];
          mko[(size_t)M * (K >> 3) + mi] = (uint8_t)kp1[b];
        }
      }
    }
    bf16x8 b0[NS], b1[NS];
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      b0[s] = in0 ? bv[s] : bf16x8{};
      b1[s] = in1 ? bv[s] : bf16x8{};
    }
#pragma unroll
    for (int b = 0; b < 4; ++b)
#pragma unroll
      for (int s = 0; s < NS; ++s) {
        const uint32_t k0 = kp0[b] >> (8 * s), k1 = kp1[b] >> (8 * s);
        const u32x4 xw = __builtin_bit_cast(u32x4, xv[b][s]);
        u32x4 a0, a1;
#pragma unroll
        for (int p = 0; p < 4; ++p) {
          const uint32_t m0w = (0u - ((k0 >> (2 * p)) & 1u)) & 0xFFFFu, m0h = (0u - ((k0 >> (2 * p + 1)) & 1u)) << 16;
          const uint32_t m1w = (0u - ((k1 >> (2 * p)) & 1u)) & 0xFFFFu, m1h = (0u - ((k1 >> (2 * p + 1)) & 1u)) << 16;
          a0[p] = xw[p] & (m0w | m0h);
          a1[p] = xw[p] & (m1w | m1h);
        }
        acc[b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a0), b0[s], acc[b], 0, 0, 0);
        acc[b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a1), b1[s], acc[b], 0, 0, 0);
      }
  }
#pragma unroll
  for (int b = 0; b < 4; ++b) red[w][b][lane] = acc[b];
  __syncthreads();
  // wave w sums row block w over the 4 waves' K ranges; D layout: col j = lane & 15, rows 4g + i
  f32x4 t = red[0][w][lane];
#pragma unroll
  for (int v = 1; v < 4; ++v) t += red[v][w][lane];
  if (n >= r) return;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int m = m0 + 16 * w + 4 * g + i;
    if (m < M) ws[((size_t)kc * M + m) * 16 + n] = t[i];
  }
}

// out[m, j] = sc_j · Σ_c ws[c][m][j] (fixed order), fp32 and / or bf16
__global__ __launch_bounds__(256) void lora_proj2_sum_k(const float* __restrict__ ws, int nkc, int M, int r, int r0,
                                                       float sc0, float sc1, float* __restrict__ outf, int ldof,
                                                       bf16* __restrict__ outb, int ldob) {
  const int idx = blockIdx.x * 256 + threadIdx.x;
  const int m = idx >> 4, j = idx & 15;
  if (m >= M || j >= r) return;
  // all slab loads in flight at once (a runtime-trip loop issues them one round trip apart)
  float v[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  for (int c0 = 0; c0 < nkc; c0 += 8) {
#pragma unroll
    for (int c = 0; c < 8; ++c)
      if (c0 + c < nkc) v[c] += ws[((size_t)(c0 + c) * M + m) * 16 + j];
  }
  float t = ((v[0] + v[1]) + (v[2] + v[3])) + ((v[4] + v[5]) + (v[6] + v[7]));
  t *= j < r0 ? sc0 : sc1;
  if (outf) outf[(size_t)m * ldof + j] = t;
  if (outb) outb[(size_t)m * ldob + j] = (bf16)t;
}

// ---- y[:, c0_i : c0_i + n_i] += xa_i · B_iᵀ for up to 4 branches, in place on the base GEMM's output ----
// (replaces the rank-Σr addmm over ALL N columns of a fused q|k|v output plus the per-call copies of
// each B into a zero-padded [N, 32] K-slice buffer: only the adapters' own column blocks are read and
// written, B is read in its natural [n, r] layout.)  xa_i is fp32 [M, r_i] and already carries the
// branch scale.  Tile: 64 rows × 256 columns per workgroup; a thread owns 8 consecutive columns
// (their 8 × r B values are 128 contiguous bytes) of 8 rows.
struct LoraApplyArgs {
  const float* xa[4];
  int ldxa[4];
  const bf16* B[4];
  bf16* Bt[4];    // optional [r, n] copy of B for the backward's dy·B projection (row-0 workgroups write it)
  int c0[4], n[4], r[4];
  int blk0[5];    // first column block of each branch (prefix sums), blk0[nb] = total
  int nb;
};

template <int R>
__global__ __launch_bounds__(256) void lora_apply_k(bf16* __restrict__ Y, int ldy, int M, LoraApplyArgs a) {
  __shared__ __attribute__((aligned(16))) float xs[64][R];
  int br = 0;
#pragma unroll
  for (int i = 1; i < 4; ++i)
    if (i < a.nb && (int)blockIdx.x >= a.blk0[i]) br = i;
  const int r = a.r[br];
  const int m0 = blockIdx.y * 64;
  const int cb = (blockIdx.x - a.blk0[br]) * 256;
  const float* xa = a.xa[br];
  for (int i = threadIdx.x; i < 64 * R; i += 256) {
    const int rr = i / R, j = i % R, m = m0 + rr;
    xs[rr][j] = (m < M && j < r) ? xa[(size_t)m * a.ldxa[br] + j] : 0.f;
  }
  __syncthreads();
  const int cl = cb + 8 * (threadIdx.x & 31);
  if (cl >= a.n[br]) return;
  // B rows of this thread's 8 columns: [8][R] bf16, contiguous when r == R (vector loads)
  float bw[8][R];
  const bf16* Bp = a.B[br] + (size_t)cl * r;
  if (r == R) {
#pragma unroll
    for (int c = 0; c < 8; ++c)
#pragma unroll
      for (int j0 = 0; j0 < R; j0 += 8) {
        const bf16x8 v = *reinterpret_cast<const bf16x8*>(Bp + c * R + j0);
#pragma unroll
        for (int e = 0; e < 8; ++e) bw[c][j0 + e] = (float)v[e];
      }
  } else {
#pragma unroll
    for (int c = 0; c < 8; ++c)
#pragma unroll
      for (int j = 0; j < R; ++j) bw[c][j] = (j < r) ? (float)Bp[c * r + j] : 0.f;
  }
  if (a.Bt[br] && blockIdx.y == 0 && threadIdx.x < 32) {
    bf16* bt = a.Bt[br] + cl;
#pragma unroll
    for (int j = 0; j < R; ++j)
      if (j < r) {
        bf16x8 v;
#pragma unroll
        for (int c = 0; c < 8; ++c) v[c] = (bf16)bw[c][j];
        *reinterpret_cast<bf16x8*>(bt + (size_t)j * a.n[br]) = v;
      }
  }
  bf16* yc = Y + a.c0[br] + cl;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int rr = (threadIdx.x >> 5) + 8 * i, m = m0 + rr;
    if (m >= M) break;
    float xv[R];
#pragma unroll
    for (int j0 = 0; j0 < R; j0 += 4) {
      const f32x4 t = *reinterpret_cast<const f32x4*>(&xs[rr][j0]);
      xv[j0] = t[0]; xv[j0 + 1] = t[1]; xv[j0 + 2] = t[2]; xv[j0 + 3] = t[3];
    }
    bf16x8 y = *reinterpret_cast<const bf16x8*>(yc + (size_t)m * ldy);
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      float acc = (float)y[c];
#pragma unroll
      for (int j = 0; j < R; ++j) acc += xv[j] * bw[c][j];
      y[c] = (bf16)acc;
    }
    *reinterpret_cast<bf16x8*>(yc + (size_t)m * ldy) = y;
  }
}

// ---- 1-4 adapters of one projection, any mix of dropout rates (BASELINE #2: q, k, v on q|k|v) ----------
// The pair kernels above pack two rank-8 adapters into one 16-column MFMA tile; with rank-16 adapters each
// branch is its own tile.  Forward: lora_projms_k reads x ONCE for all NBR branches (split-K like
// lora_proj2s_k: 64 rows × 4·NS·32 of K per workgroup, all loads issued before the first MFMA), masks the
// x fragment per branch with a bitwise AND and writes every branch's keep bits for the backward.
struct ProjM {
  const bf16* W[4];
  int r[4];
  uint64_t key[4];
  uint32_t thr[4];
  uint8_t* mko[4];   // keep-bit plane [M, K/8] per branch (null: not stored)
};
struct ProjMOut {
  float* outf[4];
  bf16* outb[4];
  int ldof[4], ldob[4], r[4];
  float sc[4];       // scale · 1/(1-p)
  int nbr;
};
template <int NS, int NBR>
__global__ __launch_bounds__(256) void lora_projms_k(const bf16* __restrict__ X, int ldx, int K, int M, ProjM p,
                                                    size_t mask_ld, float* __restrict__ ws) {
  constexpr int KW = NS * 32, KC = 4 * KW;
  __shared__ f32x4 red[4][4][64];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int g = lane >> 4, n = lane & 15;
  int kc, mbk;
  xcd_grid(kc, mbk);   // neighbouring K chunks of a row block (their keep-bit bytes share lines) on one XCD
  const int m0 = mbk * 64;
  const int kl = kc * KC + w * KW + g * (NS * 8);
  bf16x8 xv[4][NS], bv[NBR][NS];
#pragma unroll
  for (int br = 0; br < NBR; ++br) {
    const bf16* wr = p.W[br] + (size_t)(n < p.r[br] ? n : 0) * K;
#pragma unroll
    for (int s = 0; s < NS; ++s) bv[br][s] = *reinterpret_cast<const bf16x8*>(wr + kl + 8 * s);
  }
#pragma unroll
  for (int b = 0; b < 4; ++b) {
    const int row = min(m0 + 16 * b + n, M - 1);
#pragma unroll
    for (int s = 0; s < NS; ++s) xv[b][s] = *reinterpret_cast<const bf16x8*>(X + (size_t)row * ldx + kl + 8 * s);
  }
  f32x4 acc[NBR][4];
#pragma unroll
  for (int br = 0; br < NBR; ++br) {
#pragma unroll
    for (int s = 0; s < NS; ++s)
      if (n >= p.r[br]) bv[br][s] = bf16x8{};
#pragma unroll
    for (int b = 0; b < 4; ++b) acc[br][b] = f32x4{0.f, 0.f, 0.f, 0.f};
    const uint32_t thr = p.thr[br];
    if (thr == 0 && !p.mko[br]) {
#pragma unroll
      for (int s = 0; s < NS; ++s)
#pragma unroll
        for (int b = 0; b < 4; ++b) acc[br][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xv[b][s], bv[br][s], acc[br][b], 0, 0, 0);
      continue;
    }
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      const int mg = m0 + 16 * b + n;
      const int row = min(mg, M - 1);
      uint32_t kp = 0;
#pragma unroll
      for (int s = 0; s < NS; ++s)
        kp |= (thr ? dropout_keep8(p.key[br], ((size_t)row * mask_ld + kl + 8 * s) >> 3, thr) : 0xFFu) << (8 * s);
      if (p.mko[br] && mg < M) {   // NS keep bytes of the lane's row, one store
        uint8_t* dst = p.mko[br] + (size_t)mg * (K >> 3) + (kl >> 3);
        if constexpr (NS == 4) *reinterpret_cast<uint32_t*>(dst) = kp;
        else if constexpr (NS == 2) *reinterpret_cast<uint16_t*>(dst) = (uint16_t)kp;
        else *dst = (uint8_t)kp;
      }
#pragma unroll
      for (int s = 0; s < NS; ++s) {
        const uint32_t k8 = kp >> (8 * s);
        const u32x4 xw = __builtin_bit_cast(u32x4, xv[b][s]);
        u32x4 a;
#pragma unroll
        for (int q = 0; q < 4; ++q)
          a[q] = xw[q] & (((0u - ((k8 >> (2 * q)) & 1u)) & 0xFFFFu) | ((0u - ((k8 >> (2 * q + 1)) & 1u)) << 16));
        acc[br][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), bv[br][s], acc[br][b], 0, 0, 0);
      }
    }
  }
  // per branch: the 4 waves' K ranges meet in LDS, wave w sums row block w (D: col j = lane & 15, rows 4g + i)
#pragma unroll
  for (int br = 0; br < NBR; ++br) {
    if (br) __syncthreads();
#pragma unroll
    for (int b = 0; b < 4; ++b) red[w][b][lane] = acc[br][b];
    __syncthreads();
    f32x4 t = red[0][w][lane];
#pragma unroll
    for (int v = 1; v < 4; ++v) t += red[v][w][lane];
    if (n < p.r[br]) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int m = m0 + 16 * w + 4 * g + i;
        if (m < M) ws[((size_t)kc * M + m) * (16 * NBR) + 16 * br + n] = t[i];
      }
    }
  }
}

// out_b[m, j] = sc_b · Σ_c ws[c][m][16 b + j] (fixed order), fp32 and / or bf16 per branch
__global__ __launch_bounds__(256) void lora_projm_sum_k(const float* __restrict__ ws, int nkc, int M, ProjMOut o) {
  const int w16 = 16 * o.nbr;
  const int idx = blockIdx.x * 256 + threadIdx.x;
  const int m = idx / w16, c = idx % w16, b = c >> 4, j = c & 15;
  if (m >= M || j >= o.r[b]) return;
  float v[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  for (int c0 = 0; c0 < nkc; c0 += 8) {
#pragma unroll
    for (int u = 0; u < 8; ++u)
      if (c0 + u < nkc) v[u] += ws[((size_t)(c0 + u) * M + m) * w16 + c];
  }
  const float t = (((v[0] + v[1]) + (v[2] + v[3])) + ((v[4] + v[5]) + (v[6] + v[7]))) * o.sc[b];
  if (o.outf[b]) o.outf[b][(size_t)m * o.ldof[b] + j] = t;
  if (o.outb[b]) o.outb[b][(size_t)m * o.ldob[b] + j] = (bf16)t;
}

// backward projections g_b = s_b·dy[:, c0_b : c0_b + K_b]·B_b (Bᵀ [r_b, K_b]) of 1-4 adapters, blockIdx.y = branch
struct ProjMulti {
  const bf16* X[4];
  const bf16* W[4];
  float* out[4];
  int K[4], r[4];
  float scale[4];
};
template <int NW, int RW>
__global__ __launch_bounds__(NW * 64) void lora_proj_multi_k(ProjMulti p, int ldx, int M) {
  const int b = blockIdx.y;
  lora_proj_body<NW, RW>(p.X[b], ldx, p.W[b], p.r[b], p.K[b], p.out[b], p.r[b], nullptr, 0, M, 0, 0u, 1.f, p.scale[b], 0,
                         blockIdx.x);
}

// The adapters' input-gradient term as the dX GEMM's C matrix:
//   C[m, k] = Σ_b keep_b[m, k]·ds_b·Σ_j g_b[m, j]·A_b[j, k]     (bf16 [M, K], 1-4 branches, r_b <= 16)
// One MFMA per (branch, 16 k × 16 m tile): A operand = A_b columns (rows k, depth j, staged through LDS),
// B operand = the g_b row of the lane's m (depth j = rank, 16 deep).  The MFMA rows of the two tiles of a pair are mapped
// to k so that each lane's 2 × 4 accumulator rows are 8 CONSECUTIVE k of its m (tile h of pair P: row rr ↔
// k = 32 P + 8 (rr / 4) + 4 h + rr % 4): the keep bits of the lane are one byte per pair, the store is 16 B.
// A workgroup is 64 k × 4 waves × RB 16-row blocks; the A fragments are built once per workgroup and the
// next row block's g rows / keep words are loaded before the current block is computed and stored.
struct DxcArgs {
  const float* g[4];
  int ldg[4];
  const bf16* a[4];
  int r[4];
  const uint8_t* keep[4];   // [M, K/8] or null (no dropout)
  float ds[4];
  int nbr;
};
typedef short s16x4 __attribute__((ext_vector_type(4)));
template <int RB>
__global__ __launch_bounds__(256) void lora_dxc_k(DxcArgs d, bf16* __restrict__ out, int M, int K) {
  __shared__ bf16 as[4][16][64 + 8];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int q = lane >> 4, c = lane & 15;
  int bx, by;
  xcd_grid(bx, by);   // the 64 column blocks of a row block (its g rows, keep lines) on one XCD
  const int kb = bx * 64;
  const int nbr = d.nbr;
  for (int idx = threadIdx.x; idx < 4 * 16 * 8; idx += 256) {   // A_b[:, kb : kb + 64] (rows >= r_b zero)
    const int b = idx >> 7, j = (idx >> 3) & 15, cc = idx & 7;
    bf16x8 v = {};
    if (b < nbr && j < d.r[b]) v = *reinterpret_cast<const bf16x8*>(d.a[b] + (size_t)j * K + kb + 8 * cc);
    *reinterpret_cast<bf16x8*>(&as[b][j][8 * cc]) = v;
  }
  const int mb = (by * 4 + w) * RB * 16;
  // rank depth 16 = one v_mfma_f32_16x16x16_bf16: lane (q, c) holds ranks 4 q .. 4 q + 3
  f32x4 gq[2][4];      // [row-block parity][branch]: g_b[m, 4 q .. 4 q + 3]
  uint64_t kq[2][4];   // keep word of the lane's row over [kb, kb + 64)
  auto load_rb = [&](int rb, int par) {
    const int gm = min(mb + 16 * rb + c, M - 1);
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      gq[par][b] = f32x4{0.f, 0.f, 0.f, 0.f};
      kq[par][b] = ~0ull;
      if (b < nbr) {
        if (4 * q < d.r[b]) gq[par][b] = *reinterpret_cast<const f32x4*>(d.g[b] + (size_t)gm * d.ldg[b] + 4 * q);
        if (d.keep[b]) kq[par][b] = *reinterpret_cast<const uint64_t*>(d.keep[b] + (size_t)gm * (K >> 3) + (kb >> 3));
      }
    }
  };
  load_rb(0, 0);
  __syncthreads();
  s16x4 af[4][4];   // [branch][tile 2P + h]: row rr = c ↔ k = kb + 32 P + 8 (c / 4) + 4 h + c % 4, depth j = 4 q + e
#pragma unroll
  for (int b = 0; b < 4; ++b)
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int kl = 32 * (t >> 1) + 8 * (c >> 2) + 4 * (t & 1) + (c & 3);
      bf16x4 v;
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = b < nbr ? as[b][4 * q + e][kl] : (bf16)0.f;
      af[b][t] = __builtin_bit_cast(s16x4, v);
    }
#pragma unroll
  for (int rb = 0; rb < RB; ++rb) {
    const int par = rb & 1;
    if (rb + 1 < RB) load_rb(rb + 1, par ^ 1);
    const int m = mb + 16 * rb + c;
    f32x4 v[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) v[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      if (b >= nbr) break;
      const bf16x4 gb = {(bf16)gq[par][b][0], (bf16)gq[par][b][1], (bf16)gq[par][b][2], (bf16)gq[par][b][3]};
      const float ds = d.ds[b];
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const f32x4 p = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(af[b][t], __builtin_bit_cast(s16x4, gb),
                                                                  f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
        // k = kb + 32 P + 8 q + 4 h + i: byte 4 P + q of the keep word, bit 4 h + i
        const uint32_t bits = (uint32_t)(kq[par][b] >> (8 * (4 * (t >> 1) + q) + 4 * (t & 1))) & 15u;
#pragma unroll
        for (int i = 0; i < 4; ++i) v[t][i] += ((bits >> i) & 1u) ? p[i] * ds : 0.f;
      }
    }
    if (m < M) {
#pragma unroll
      for (int P = 0; P < 2; ++P) {
        bf16x8 o;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          o[i] = (bf16)v[2 * P][i];
          o[i + 4] = (bf16)v[2 * P + 1][i];
        }
        *reinterpret_cast<bf16x8*>(out + (size_t)m * K + kb + 32 * P + 8 * q) = o;
      }
    }
  }
}

}  // namespace

// X row stride ldx (elements), W [r, K] bf16 contiguous; K % 32 == 0; outf/outb may each be null.
void launch_lora_proj(const void* X, int ldx, const void* W, int r, int K, float* outf, int ldof, void* outb, int ldob,
                      int M, uint64_t key, float p, float scale, size_t mask_ld, hipStream_t st) {
  const uint32_t thr = p > 0.f ? (uint32_t)(p * 65536.0f + 0.5f) : 0u;
  const float ds = p > 0.f ? 1.f / (1.f - p) : 1.f;
  // 16-row workgroups leave half of the 256 CUs idle below M = 4096: use 8 (zero-padded MFMA rows)
  const int rw = M < 4096 ? 8 : 16;
  const int grid = (M + rw - 1) / rw;
  if (K % (16 * 32) == 0 && rw == 8)
    lora_proj_k<16, 8><<<grid, 1024, 0, st>>>((const bf16*)X, ldx, (const bf16*)W, r, K, outf, ldof, (bf16*)outb, ldob,
                                              M, key, thr, ds, scale, mask_ld);
  else if (K % (16 * 32) == 0)
    lora_proj_k<16, 16><<<grid, 1024, 0, st>>>((const bf16*)X, ldx, (const bf16*)W, r, K, outf, ldof, (bf16*)outb, ldob,
                                           M, key, thr, ds, scale, mask_ld);
  else
    lora_proj_k<1, 16><<<(M + 15) / 16, 64, 0, st>>>((const bf16*)X, ldx, (const bf16*)W, r, K, outf, ldof, (bf16*)outb, ldob, M,
                                        key, thr, ds, scale, mask_ld);
  LIPA_CHECK_LAUNCH();
}

// out[j*sj + k*sk] += Σ_m G[m,j]·D(X)[m,k] (fp32 atomics: accumulate straight into a gradient), or
// with part != null the per-chunk partials [chunks, r, K] (deterministic mode);
// with DX: DX[m,k] += D(Σ_j G[m,j]·W[j,k]).
// Chunk height: 64 rows, or 32 when that leaves fewer than 256 workgroups (narrow K).
static int lora_acc_rows(int M, int K) {
  return ((K / 8 + 63) / 64) * ((M + 63) / 64) >= 256 ? 64 : 32;
}
int lora_acc_chunks(int M, int K) { const int rows = lora_acc_rows(M, K); return (M + rows - 1) / rows; }

void launch_lora_acc(const float* G, int ldg, int r, const void* X, int ldx, void* DX, int lddx, const void* W, int K,
                     float* out, int64_t sj, int64_t sk, float* part, int M, uint64_t key, float p, size_t mask_ld,
                     hipStream_t st) {
  const uint32_t thr = p > 0.f ? (uint32_t)(p * 65536.0f + 0.5f) : 0u;
  const float ds = p > 0.f ? 1.f / (1.f - p) : 1.f;
  if (!part && r <= 16 && K % 128 == 0 && ldx % 8 == 0 && ldg % 4 == 0 && ((uintptr_t)G & 15) == 0) {
    // matrix-core path (deterministic mode keeps the VALU kernel's fixed-order partials); 32 rows per
    // wave: 2 waves/SIMD beat longer waves (-10-25 %, profiles/lora_acc_mfma_ab.txt)
    constexpr int sub = 1;
    dim3 g2(K / 128, (M + 128 * sub - 1) / (128 * sub));
#define C(R_, D_, S_)                                                                                        \
  lora_acc_mfma_k<R_, D_, S_><<<g2, 256, 0, st>>>(G, ldg, r, (const bf16*)X, ldx, (bf16*)DX, lddx,            \
                                                  (const bf16*)W, K, out, sj, sk, M, key, thr, ds, mask_ld)
#define D2(R_, D_) C(R_, D_, 1)
    if (r <= 8) {
      if (DX) { D2(8, true); } else { D2(8, false); }
    } else {
      if (DX) { D2(16, true); } else { D2(16, false); }
    }
#undef D2
#undef C
    LIPA_CHECK_LAUNCH();
    return;
  }
  const int rows = lora_acc_rows(M, K);
  dim3 grid((K / 8 + 63) / 64, (M + rows - 1) / rows);
// r <= 8: 8 row-lanes (512 threads, 2 waves/SIMD); r <= 16: 4 row-lanes (the accumulators double)
#define A(R_, D_, ROWS_)                                                                                          \
  lora_acc_k<R_, D_, (R_ > 8 ? 4 : 8), ROWS_><<<grid, (R_ > 8 ? 256 : 512), 0, st>>>(                            \
      G, ldg, r, (const bf16*)X, ldx, (bf16*)DX, lddx, (const bf16*)W, K, out, sj, sk, part, M, key, thr, ds, mask_ld)
#define B(R_, D_)       \
  if (rows == 256)      \
    A(R_, D_, 256);     \
  else if (rows == 128) \
    A(R_, D_, 128);     \
  else if (rows == 64)  \
    A(R_, D_, 64);      \
  else                  \
    A(R_, D_, 32)
  if (r <= 8) {
    if (DX) { B(8, true); } else { B(8, false); }
  } else {
    if (DX) { B(16, true); } else { B(16, false); }
  }
#undef B
#undef A
  LIPA_CHECK_LAUNCH();
}

// split-K lora_proj2s_k: NS (K per wave / 32) giving >= 256 workgroups, 0 = not applicable (old kernel)
int lora_proj2_ns(int M, int K) {
  if (M <= 0) return 0;
  const int nrb = (M + 63) / 64;
  for (int ns = 4; ns >= 1; ns /= 2)
    if (K % (128 * ns) == 0 && (nrb * (K / (128 * ns)) >= 256 || ns == 1)) return ns;
  return 0;
}
int lora_proj2_ws_floats(int M, int K) {
  const int ns = lora_proj2_ns(M, K);
  return ns ? (K / (128 * ns)) * M * 16 : 0;
}

// two branches sharing x: W = [A0; A1] ([r0 + r1 <= 16, K]); outputs [M, r0 + r1] (fp32 and/or bf16)
void launch_lora_proj2(const void* X, int ldx, const void* W0, const void* W1, int r0, int r, int K, float* outf, int ldof, void* outb,
                       int ldob, int M, uint64_t key0, float p0, float scale0, uint64_t key1, float p1, float scale1,
                       size_t mask_ld, uint8_t* mko, float* ws, hipStream_t st) {
  const uint32_t thr0 = p0 > 0.f ? (uint32_t)(p0 * 65536.0f + 0.5f) : 0u;
  const uint32_t thr1 = p1 > 0.f ? (uint32_t)(p1 * 65536.0f + 0.5f) : 0u;
  const float ds0 = p0 > 0.f ? 1.f / (1.f - p0) : 1.f, ds1 = p1 > 0.f ? 1.f / (1.f - p1) : 1.f;
  const int ns = lora_proj2_ns(M, K);
  if (ws && ns) {
    dim3 grid(K / (128 * ns), (M + 63) / 64);
#define P(NS_)                                                                                                      \
  lora_proj2s_k<NS_><<<grid, 256, 0, st>>>((const bf16*)X, ldx, (const bf16*)W0, (const bf16*)W1, r0, r, K, M, key0, \
                                           key1, thr0, thr1, mask_ld, mko, ws)
    if (ns == 4) P(4); else if (ns == 2) P(2); else P(1);
#undef P
    lora_proj2_sum_k<<<(M * 16 + 255) / 256, 256, 0, st>>>(ws, grid.x, M, r, r0, scale0 * ds0, scale1 * ds1, outf, ldof,
                                                          (bf16*)outb, ldob);
    LIPA_CHECK_LAUNCH();
    return;
  }
  const int rw = M < 4096 ? 8 : 16;
  const int grid = (M + rw - 1) / rw;
  if (K % (16 * 32) == 0 && rw == 8)
    lora_proj2_k<16, 8><<<grid, 1024, 0, st>>>((const bf16*)X, ldx, (const bf16*)W0, (const bf16*)W1, r0, r, K, outf, ldof,
                                               (bf16*)outb, ldob, M, key0, key1, thr0, thr1, ds0, ds1, scale0, scale1, mask_ld, mko);
  else if (K % (16 * 32) == 0)
    lora_proj2_k<16, 16><<<grid, 1024, 0, st>>>((const bf16*)X, ldx, (const bf16*)W0, (const bf16*)W1, r0, r, K, outf, ldof,
                                                (bf16*)outb, ldob, M, key0, key1, thr0, thr1, ds0, ds1, scale0, scale1, mask_ld, mko);
  else
    lora_proj2_k<1, 16><<<(M + 15) / 16, 64, 0, st>>>((const bf16*)X, ldx, (const bf16*)W0, (const bf16*)W1, r0, r, K, outf,
                                                      ldof, (bf16*)outb, ldob, M, key0, key1, thr0, thr1, ds0, ds1, scale0,
                                                      scale1, mask_ld, mko);
  LIPA_CHECK_LAUNCH();
}

void launch_lora_apply(void* Y, int ldy, int M, int nb, const float* const* xa, const int* ldxa, const void* const* B,
                       void* const* Bt, const int* c0, const int* n, const int* r, hipStream_t st) {
  LoraApplyArgs a{};
  a.nb = nb;
  int tot = 0;
  for (int i = 0; i < nb; ++i) {
    a.xa[i] = xa[i];
    a.ldxa[i] = ldxa[i];
    a.B[i] = static_cast<const bf16*>(B[i]);
    a.Bt[i] = Bt ? static_cast<bf16*>(Bt[i]) : nullptr;
    a.c0[i] = c0[i];
    a.n[i] = n[i];
    a.r[i] = r[i];
    a.blk0[i] = tot;
    tot += (n[i] + 255) / 256;
  }
  a.blk0[nb] = tot;
  for (int i = nb + 1; i < 5; ++i) a.blk0[i] = tot;
  dim3 grid(tot, (M + 63) / 64);
  int rmax = 0;
  for (int i = 0; i < nb; ++i) rmax = r[i] > rmax ? r[i] : rmax;
  if (rmax <= 8)
    lora_apply_k<8><<<grid, 256, 0, st>>>(static_cast<bf16*>(Y), ldy, M, a);
  else
    lora_apply_k<16><<<grid, 256, 0, st>>>(static_cast<bf16*>(Y), ldy, M, a);
  LIPA_CHECK_LAUNCH();
}

// the backward's two-branch projections g_i = s_i·dy[:, c0_i : c0_i + K_i]·B_i (fp32 [M, r]), B_i given as
// Bᵀ [r, K_i]; both branches have the same rank r
void launch_lora_proj_pair(const void* X0, const void* X1, int ldx, const void* W0, const void* W1, int r, int K0,
                           int K1, float* out0, float* out1, float s0, float s1, int M, hipStream_t st) {
  ProjPair p{{(const bf16*)X0, (const bf16*)X1}, {(const bf16*)W0, (const bf16*)W1}, {out0, out1}, {K0, K1}, {s0, s1}};
  // (a split-K form like lora_proj2s_k measured slower here: 10.4 + 5.2 us slab sum vs 11.1 us)
  const int rw = M < 4096 ? 8 : 16;
  dim3 grid((M + rw - 1) / rw, 2);
  if (rw == 8)
    lora_proj_pair_k<16, 8><<<grid, 1024, 0, st>>>(p, ldx, r, M);
  else
    lora_proj_pair_k<16, 16><<<grid, 1024, 0, st>>>(p, ldx, r, M);
  LIPA_CHECK_LAUNCH();
}

// dB_i [K_i, r] (row-major, i.e. out[k * r + j]) += Σ_m X_i[m, k]·G_i[m, j] for two branches, r <= 8
void launch_lora_acc_pair(const float* G0, const float* G1, int ldg, int r, const void* X0, const void* X1, int ldx,
                          int K0, int K1, float* out0, float* out1, int M, hipStream_t st) {
  AccPair a{{G0, G1}, {(const bf16*)X0, (const bf16*)X1}, {out0, out1}, {K0, K1}, K0 / 128, {1, 1}, {r, r},
            {1.f, 1.f}, {nullptr, nullptr}};
  dim3 g(K0 / 128 + K1 / 128, (M + 127) / 128);
  lora_acc_pair_k<1><<<g, 256, 0, st>>>(a, ldg, r, ldx, M);
  LIPA_CHECK_LAUNCH();
}

// backward of a dropout q_proj + v_proj pair from the forward's keep bits:
//   dA_i [r, K] += Σ_m G_i[m, j]·D_i(x)[m, k]·ds_i  (one launch, both branches, fp32 atomics)
void launch_lora_dA_pair(const float* G0, const float* G1, int ldg, int r, const void* X, int ldx, int K, float* out0,
                         float* out1, int64_t sj0, int64_t sk0, int64_t sj1, int64_t sk1, const uint8_t* kb0,
                         const uint8_t* kb1, float ds0, float ds1, int M, hipStream_t st) {
  AccPair a{{G0, G1}, {(const bf16*)X, (const bf16*)X}, {out0, out1}, {K, K}, K / 128, {sj0, sj1}, {sk0, sk1},
            {ds0, ds1}, {kb0, kb1}};
  dim3 g(2 * (K / 128), (M + 127) / 128);
  lora_acc_pair_k<1><<<g, 256, 0, st>>>(a, ldg, r, ldx, M);
  LIPA_CHECK_LAUNCH();
}

// jobs 0, 1: dB of the two branches (G = xa, X = dy column block, out [n, r] row-major);
// jobs 2, 3: dA (G = g, X = x, out [r, K] with strides, keep bits / rescale per branch)
// (any job count 1..8: the multi-adapter backward's dB / dA products go through the same launch)
void launch_lora_acc_jobs(int njobs, const float* const* G, const int* ldg, const int* r, const void* const* X,
                          const int* ldx, const int* K, float* const* out, const int64_t* sj, const int64_t* sk,
                          const float* ds, const uint8_t* const* kb, int M, hipStream_t st) {
  AccJobs a{};
  a.njobs = njobs;
  int nb = 0;
  for (int j = 0; j < njobs; ++j) {
    a.G[j] = G[j];
    a.X[j] = (const bf16*)X[j];
    a.out[j] = out[j];
    a.K[j] = K[j];
    a.ldg[j] = ldg[j];
    a.ldx[j] = ldx[j];
    a.r[j] = r[j];
    a.sj[j] = sj[j];
    a.sk[j] = sk[j];
    a.ds[j] = ds[j];
    a.kb[j] = kb[j];
    a.nb[j] = nb;
    nb += K[j] / 128;
  }
  // rank 16 with >= 16 row blocks of 256: two 32-row steps per wave (half the fp32 atomics; BASELINE #2's
  // q|k|v + o products 2.66 -> 2.31 ms/step, 4 steps 2.35 — profiles/r4/lora_multi_adapter.txt); rank 8
  // keeps one (the headline's quad launch, round-2 A/B)
  int rmax = 0;
  for (int j = 0; j < njobs; ++j) rmax = r[j] > rmax ? r[j] : rmax;
  const int su = rmax > 8 && (M + 255) / 256 >= 16 ? 2 : 1;
  dim3 g(nb, (M + 128 * su - 1) / (128 * su));
  if (su == 2) lora_acc_jobs_k<2><<<g, 256, 0, st>>>(a, M);
  else lora_acc_jobs_k<1><<<g, 256, 0, st>>>(a, M);
  LIPA_CHECK_LAUNCH();
}

void launch_lora_acc_quad(const float* const G[4], const int ldg[4], const void* const X[4], const int ldx[4],
                          const int K[4], float* const out[4], const int64_t sj[4], const int64_t sk[4],
                          const float ds[4], const uint8_t* const kb[4], int r, int M, hipStream_t st) {
  const int rr[4] = {r, r, r, r};
  launch_lora_acc_jobs(4, G, ldg, rr, X, ldx, K, out, sj, sk, ds, kb, M, st);
}

// N adapters sharing x: split-K projection (+ every branch's keep bits), then the fixed-order slab sum
void launch_lora_proj_m(const void* X, int ldx, int K, int M, int nbr, const void* const* W, const int* r,
                        const uint64_t* key, const float* p, const float* scale, uint8_t* const* mko, size_t mask_ld,
                        float* const* outf, const int* ldof, void* const* outb, const int* ldob, float* ws,
                        hipStream_t st) {
  ProjM pm{};
  ProjMOut po{};
  po.nbr = nbr;
  for (int b = 0; b < nbr; ++b) {
    pm.W[b] = (const bf16*)W[b];
    pm.r[b] = r[b];
    pm.key[b] = key[b];
    pm.thr[b] = p[b] > 0.f ? (uint32_t)(p[b] * 65536.0f + 0.5f) : 0u;
    pm.mko[b] = mko[b];
    po.r[b] = r[b];
    po.sc[b] = scale[b] * (p[b] > 0.f ? 1.f / (1.f - p[b]) : 1.f);
    po.outf[b] = outf[b];
    po.ldof[b] = ldof[b];
    po.outb[b] = (bf16*)outb[b];
    po.ldob[b] = ldob[b];
  }
  const int ns = lora_proj2_ns(M, K);
  dim3 grid(K / (128 * ns), (M + 63) / 64);
#define P(NS_, NB_) lora_projms_k<NS_, NB_><<<grid, 256, 0, st>>>((const bf16*)X, ldx, K, M, pm, mask_ld, ws)
#define PN(NS_) \
  if (nbr == 1) P(NS_, 1); else if (nbr == 2) P(NS_, 2); else if (nbr == 3) P(NS_, 3); else P(NS_, 4)
  if (ns == 4) { PN(4); } else if (ns == 2) { PN(2); } else { PN(1); }
#undef PN
#undef P
  lora_projm_sum_k<<<(M * 16 * nbr + 255) / 256, 256, 0, st>>>(ws, grid.x, M, po);
  LIPA_CHECK_LAUNCH();
}
int lora_proj_m_ws_floats(int M, int K, int nbr) {
  const int ns = lora_proj2_ns(M, K);
  return ns ? (K / (128 * ns)) * M * 16 * nbr : 0;
}

// the backward's g_b = s_b·dy[:, c0_b : c0_b + K_b]·B_b for 1-4 adapters of one projection (blockIdx.y = branch)
void launch_lora_proj_cols(int nbr, const void* const* X, int ldx, const void* const* W, const int* r, const int* K,
                           float* const* out, const float* scale, int M, hipStream_t st) {
  ProjMulti pm{};
  for (int b = 0; b < nbr; ++b) {
    pm.X[b] = (const bf16*)X[b];
    pm.W[b] = (const bf16*)W[b];
    pm.r[b] = r[b];
    pm.K[b] = K[b];
    pm.out[b] = out[b];
    pm.scale[b] = scale[b];
  }
  const int rw = M < 4096 ? 8 : 16;
  dim3 grid((M + rw - 1) / rw, nbr);
  if (rw == 8)
    lora_proj_multi_k<16, 8><<<grid, 1024, 0, st>>>(pm, ldx, M);
  else
    lora_proj_multi_k<16, 16><<<grid, 1024, 0, st>>>(pm, ldx, M);
  LIPA_CHECK_LAUNCH();
}

// C = Σ_b keep_b·ds_b·(g_b·A_b), bf16 [M, K] (the dX GEMM's C matrix) for 1-4 adapters
// rows per wave (16-row blocks): rb = 0 picks 4 when that still gives >= 512 workgroups, else 1
void launch_lora_dxc(int nbr, const float* const* g, const int* ldg, const void* const* a, const int* r,
                     const uint8_t* const* keep, const float* ds, void* out, int M, int K, int rb, hipStream_t st) {
  DxcArgs d{};
  d.nbr = nbr;
  for (int b = 0; b < nbr; ++b) {
    d.g[b] = g[b];
    d.ldg[b] = ldg[b];
    d.a[b] = (const bf16*)a[b];
    d.r[b] = r[b];
    d.keep[b] = keep[b];
    d.ds[b] = ds[b];
  }
  const int rbx = rb > 0 ? rb : 4;
  if (rbx == 2 && (K / 64) * ((M + 127) / 128) >= 512) {
    dim3 g2(K / 64, (M + 127) / 128);
    lora_dxc_k<2><<<g2, 256, 0, st>>>(d, (bf16*)out, M, K);
  } else if (rbx == 8 && (K / 64) * ((M + 511) / 512) >= 256) {
    dim3 g8(K / 64, (M + 511) / 512);
    lora_dxc_k<8><<<g8, 256, 0, st>>>(d, (bf16*)out, M, K);
  } else if (rbx != 1 && (K / 64) * ((M + 255) / 256) >= 512) {
    dim3 g4(K / 64, (M + 255) / 256);
    lora_dxc_k<4><<<g4, 256, 0, st>>>(d, (bf16*)out, M, K);
  } else {
    dim3 g1(K / 64, (M + 63) / 64);
    lora_dxc_k<1><<<g1, 256, 0, st>>>(d, (bf16*)out, M, K);
  }
  LIPA_CHECK_LAUNCH();
}

void launch_lora_dx2(const float* G0, const float* G1, int ldg, const void* A0, const void* A1, int r0, int r1,
                     const uint8_t* kb0, const uint8_t* kb1, float ds0, float ds1, void* out, int M, int K,
                     hipStream_t st) {
  if (r0 <= 8 && r1 <= 8) {
    dim3 g16((K / 8 + 255) / 256, (M + 15) / 16);
    lora_dx2_r16_k<<<g16, 256, 0, st>>>(G0, G1, ldg, (const bf16*)A0, (const bf16*)A1, r0, r1, kb0, kb1, ds0, ds1,
                                       (bf16*)out, M, K);
    LIPA_CHECK_LAUNCH();
    return;
  }
  dim3 g((K / 8 + 63) / 64, (M + 15) / 16);
  lora_dx2_k<4><<<g, 256, 0, st>>>(G0, G1, ldg, (const bf16*)A0, (const bf16*)A1, r0, r1, kb0, kb1, ds0, ds1, (bf16*)out,
                                M, K);
  LIPA_CHECK_LAUNCH();
}

