// gemm4w with the LoRA branches in its prologue: the forward (B term as extra MFMA K-steps)
// and the transposed-B dX (the masked LoRA input-gradient term).  Kernel: gemm4w_kernel.h.
#include "gemm4w_kernel.h"

using namespace lipa;

// y = x·Wᵀ + Σ_b xa_b·B_bᵀ (LoRA branches in the epilogue) (+ residual), whole-K tiles (bm, bn from
// gemm4w_plan with splits = 1)
void launch_gemm4w_lora(const void* A, int lda, const void* B, int ldb, const float* bscale, const void* residual,
                        void* out, const LoraEpi& lx, int M, int N, int K, int bn, int bm, hipStream_t st) {
  const int tiles = tiles_of(M, N, bm, bn);
  const bf16* a = (const bf16*)A;
  const bf16* r = (const bf16*)residual;
#define G4L(BM_, BN_, W4_)                                                                                       \
  gemm4w_k<BM_, BN_, false, false, 0, W4_, true><<<tiles, NT, 0, st>>>(a, lda, B, ldb, r, out, M, N, K, 1,       \
                                                                       nullptr, nullptr, 0, nullptr, bscale, nullptr, lx, LoraDx{})
  if (bscale) {
    if (bm == 256) { if (bn == 256) G4L(256, 256, 1); else G4L(256, 128, 1); }
    else { if (bn == 256) G4L(128, 256, 1); else G4L(128, 128, 1); }
  } else if (bm == 256) {
    if (bn == 256) G4L(256, 256, 0); else if (bn == 192) G4L(256, 192, 0); else G4L(256, 128, 0);
  } else {
    if (bn == 256) G4L(128, 256, 0); else if (bn == 192) G4L(128, 192, 0); else G4L(128, 128, 0);
  }
#undef G4L
  LIPA_CHECK_LAUNCH();
}

// dX = dY·W + the adapters' masked input-gradient term (LoraDx), whole-K transposed-B tiles
void launch_gemm4w_loradx(const void* A, int lda, const void* B, int ldb, const float* bscale, const void* residual,
                          void* out, const LoraDx& ld, int M, int N, int K, int bn, int bm, hipStream_t st) {
  const int tiles = tiles_of(M, N, bm, bn);
  const bf16* a = (const bf16*)A;
  const bf16* r = (const bf16*)residual;
#define G4X(BM_, BN_, W4_)                                                                                     \
  gemm4w_k<BM_, BN_, true, false, 0, W4_, true><<<tiles, NT, 0, st>>>(a, lda, B, ldb, r, out, M, N, K, 1,       \
                                                                      nullptr, nullptr, 0, nullptr, bscale,     \
                                                                      nullptr, LoraEpi{}, ld)
  if (bscale) {
    if (bm == 256) { if (bn == 256) G4X(256, 256, 1); else G4X(256, 128, 1); }
    else { if (bn == 256) G4X(128, 256, 1); else G4X(128, 128, 1); }
  } else if (bm == 256) {
    if (bn == 256) G4X(256, 256, 0); else G4X(256, 128, 0);
  } else {
    if (bn == 256) G4X(128, 256, 0); else G4X(128, 128, 0);
  }
#undef G4X
  LIPA_CHECK_LAUNCH();
}

// gu [M, 2F] and h = silu(gate)·up [M, F] from x [M, K] and W_gu [2F, K] ([gate | up] rows), one launch
