// Host/device description of the LoRA branches a gemm4w forward adds in its epilogue (gemm4w.hip,
// LORA = true): y[:, c0_b : c0_b + n_b] += xa[:, kofs_b : kofs_b + r_b] · B_bᵀ.  Shared by the kernels
// and the bindings (plain pointers: the bindings are compiled without HIP types).
#pragma once

struct LoraEpi {
  const void* xa;    // bf16 [M, 32·nks], row stride ldxa
  int ldxa, nks, nbr;
  const void* b[4];  // bf16 B_b [n_b, r_b]
  void* bt[4];       // optional bf16 B_bᵀ [r_b, n_b] outputs
  int c0[4], n[4], r[4], kofs[4];
};

// The LoRA input-gradient term a gemm4w dX (transposed-B) launch adds in its epilogue (LORA = true, bt):
// dx[m, k] += Σ_b keep_b[m, k] · ds_b · Σ_j g_b[m, j] · A_b[j, k]  — the adapters' dropout masks applied
// after the rank-r product, so it cannot be one more K-step of the base GEMM.
struct LoraDx {
  const float* g[2];          // fp32 g_b = s_b·dy_b·B_b [M, r_b], row stride ldg
  int ldg, nbr;
  const void* a[2];           // bf16 A_b [r_b, N]
  int r[2];                   // r_b <= 32
  const unsigned char* keep[2];   // keep bits [M, N/8] (bit e of byte (m, k/8) = element k = 8·(k/8) + e), or null
  float ds[2];                // 1 / (1 - p_b)
};
