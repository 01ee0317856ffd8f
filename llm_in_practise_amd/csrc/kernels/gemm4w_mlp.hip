// gemm4w with the SwiGLU epilogues: gate|up forward (gu + h) and the down dX with the
// SwiGLU backward.  Kernel: gemm4w_kernel.h.
#include "gemm4w_kernel.h"

using namespace lipa;

// gu [M, 2F] and h = silu(gate)·up [M, F] from x [M, K] and W_gu [2F, K] ([gate | up] rows), one launch
void launch_gemm4w_swiglu(const void* X, int ldx, const void* W, const float* wscale, void* gu, void* h, int M, int F,
                          int K, int bn, int bm, hipStream_t st) {
  const int N = 2 * F;
  const int tiles = tiles_of(M, N, bm, bn);
  const bf16* a = (const bf16*)X;
#define G4S(BM_, BN_, W4_)                                                                                        \
  gemm4w_k<BM_, BN_, false, false, 1, W4_><<<tiles, NT, 0, st>>>(a, ldx, W, K, nullptr, gu, M, N, K, 1, nullptr, \
                                                                  (bf16*)h, F, nullptr, wscale, nullptr, LoraEpi{}, LoraDx{})
  if (wscale) {
    if (bm == 256) { if (bn == 256) G4S(256, 256, 1); else G4S(256, 128, 1); }
    else { if (bn == 256) G4S(128, 256, 1); else G4S(128, 128, 1); }
  } else if (bm == 256) {
    if (bn == 256) G4S(256, 256, 0); else if (bn == 192) G4S(256, 192, 0); else G4S(256, 128, 0);
  } else {
    if (bn == 256) G4S(128, 256, 0); else if (bn == 192) G4S(128, 192, 0); else G4S(128, 128, 0);
  }
#undef G4S
  LIPA_CHECK_LAUNCH();
}

// dgu [M, 2F] = SwiGLU-backward(dh = dY·W_down, gu) with W_down [N_w, F] used as stored, one launch
void launch_gemm4w_dswiglu(const void* DY, int lddy, const void* W, const float* wscale, const void* gu, void* dgu,
                           int M, int F, int Nw, int bn, int bm, hipStream_t st) {
  const int tiles = tiles_of(M, F, bm, bn);
  const bf16* a = (const bf16*)DY;
#define G4D(BM_, BN_, W4_)                                                                                        \
  gemm4w_k<BM_, BN_, true, false, 2, W4_><<<tiles, NT, 0, st>>>(a, lddy, W, F, nullptr, dgu, M, F, Nw, 1,        \
                                                                 (const bf16*)gu, nullptr, F, nullptr, wscale, nullptr, LoraEpi{}, LoraDx{})
  if (wscale) {
    if (bm == 256) { if (bn == 256) G4D(256, 256, 1); else G4D(256, 128, 1); }
    else { if (bn == 256) G4D(128, 256, 1); else G4D(128, 128, 1); }
  } else if (bm == 256) {
    if (bn == 256) G4D(256, 256, 0); else if (bn == 192) G4D(256, 192, 0); else G4D(256, 128, 0);
  } else {
    if (bn == 256) G4D(128, 256, 0); else G4D(128, 128, 0);
  }
#undef G4D
  LIPA_CHECK_LAUNCH();
}

