// PyTorch bindings for the gfx950 kernels.  Launchers take raw pointers + the current HIP
// stream (so every op is capturable in a hipGraph and ordered with PyTorch's own work).
#include "kernels/lora_epi.h"
#include <torch/extension.h>
#include <ATen/hip/HIPContext.h>
#include <hip/hip_runtime.h>

#include <map>
#include <vector>

// ---- launcher declarations (csrc/kernels/*.hip)
void launch_rmsnorm_fwd(int, const void*, const void*, void*, float*, int, int, float, hipStream_t);
void launch_rmsnorm_bwd(int, const void*, const void*, const void*, const float*, void*, float*, float*, int, int, const void*,
                        hipStream_t);
void launch_layernorm_fwd(int, const void*, const void*, const void*, void*, float*, float*, int, int, float,
                          hipStream_t);
void launch_layernorm_bwd(int, const void*, const void*, const void*, const float*, const float*, void*, float*,
                          float*, float*, int, int, hipStream_t);
int norm_partial_rows(int M);
void launch_qk_norm_rope_fwd(const void*, const void*, const void*, const float*, const float*, void*, void*, float*,
                             float*, int, int, int, int, float, hipStream_t);
void launch_qk_norm_rope_bwd(const void*, const void*, const void*, const void*, const void*, const void*, const float*,
                             const float*, const float*, const float*, void*, int, int, int, int, hipStream_t);
void launch_rope(int, const void*, const float*, const float*, void*, int, int, int, int, int, hipStream_t);
void launch_swiglu_fwd(const void*, void*, int, int, hipStream_t);
void launch_swiglu_bwd(const void*, const void*, void*, int, int, hipStream_t);
void launch_gelu_fwd(int, const void*, void*, size_t, hipStream_t);
void launch_gelu_bwd(int, const void*, const void*, void*, size_t, hipStream_t);
void launch_ce_fwd_bwd(int, void*, const int64_t*, float*, int, int, int, const float*, float, int, hipStream_t);
void launch_grad_norm(int, const void*, size_t, float*, float*, float, int, hipStream_t);
void launch_adamw(int, float*, const void*, float*, float*, void*, size_t, float, float, float, float, float, float,
                  float, const float*, const float*, hipStream_t);
void launch_adamw8bit(int, float*, const void*, uint8_t*, uint8_t*, float*, float*, const float*, const float*, void*,
                      size_t, float, float, float, float, float, float, float, const float*, const float*,
                      hipStream_t);
void launch_unscale(int, void*, size_t, const float*, float*, hipStream_t);
void launch_nf4_quantize(const void*, uint8_t*, float*, size_t, hipStream_t);
void launch_nf4_dequant2(const uint8_t*, const float*, void*, size_t, hipStream_t);
void launch_int4_dequant(const uint8_t*, const float*, const float*, void*, size_t, int, hipStream_t);
int skinny_splits(int, int);
bool lt_gemm(bool, bool, long, long, long, const void*, long, const void*, long, const void*, void*, long, int, long,
             long, long, void*, size_t, hipStream_t, bool);
void lt_reset();
void launch_sum_slices(const void*, void*, int, size_t, size_t, hipStream_t);
void launch_gemm_skinny(const void*, int, const void*, const void*, void*, float*, int, int, int, int, hipStream_t);
bool w4mm_supported(int, int, int, int);
bool w4g_supported(int, int, int, int);
int w4g_splits(int, int, int);
void launch_w4g(const void*, int, const uint8_t*, const float*, int, const void*, void*, float*, int, int, int, int,
                hipStream_t);
int w4mm_nkb(int, int, int);
void launch_w4mm(const void*, int, const uint8_t*, const float*, int, const void*, void*, float*, int, int, int, int,
                 hipStream_t);
void set_dequant_variant(int);
void launch_nf4_dequant(const uint8_t*, const float*, const uint8_t*, const float*, const float*, const float*, void*,
                        size_t, hipStream_t);
bool gemm4w_supported(int, int, int, int, int, bool, bool);
int gemm4w_plan(int, int, int, bool, int, int, int*, int, int*, bool);
int gemm4w_tiles(int, int, int, int);
void launch_mlora_apply(const void*, int, const void*, const void*, const int64_t*, const void*, int, void*, int, int, int,
                        int, int, int, hipStream_t);
void launch_gemm4w_swiglu(const void*, int, const void*, const float*, void*, void*, int, int, int, int, int,
                          hipStream_t);
void launch_gemm4w_dswiglu(const void*, int, const void*, const float*, const void*, void*, int, int, int, int, int,
                           hipStream_t);
void launch_gemm4w(const void*, int, const void*, int, const void*, void*, float*, const float*, const float*, int, int,
                   int, int, bool, int, int, hipStream_t);
void launch_pack_g4w(const uint8_t*, void*, int, int, hipStream_t);
void launch_gemm4w_lora(const void*, int, const void*, int, const float*, const void*, void*, const LoraEpi&, int, int,
                        int, int, int, hipStream_t);
void launch_gemm4w_loradx(const void*, int, const void*, int, const float*, const void*, void*, const LoraDx&, int, int,
                          int, int, int, hipStream_t);
void launch_attn_fwd(const void*, const void*, const void*, int, int, int, const int*, const int*, void*, float*, int,
                     int, int, int, int, int, int, int, float, float, uint64_t, hipStream_t);
void launch_attn_bwd(const void*, const void*, const void*, const void*, const void*, const float*, const int*, int,
                     int, int, void*, void*, void*, float*, int, int, int, int, int, int, float, float, uint64_t,
                     float*, hipStream_t);
int attn_dkv_nsplit(int, int, int, int);
void attn_set_trace(void*);

void launch_gemv_w4(int, const void*, int, const uint8_t*, const float*, const float*, int, const void*, void*, int, int,
                    int, hipStream_t);
void launch_lora_proj(const void*, int, const void*, int, int, float*, int, void*, int, int, uint64_t, float, float,
                      size_t, hipStream_t);
void launch_moe_route(int, const void*, int*, float*, float*, int, int, int, int, hipStream_t);
void launch_moe_route_bwd(int, const float*, const float*, const int*, const float*, void*, int, int, int, int,
                          hipStream_t);
void launch_moe_permute(const int*, int, int, int*, int*, int*, hipStream_t);
void launch_moe_gather(int, const void*, const int*, const float*, void*, int, int, int, hipStream_t);
void launch_moe_combine(int, const void*, const int*, const float*, const void*, void*, int, int, int, hipStream_t);
void launch_moe_wgrad(int, const void*, const void*, const int*, float*, int, int, int, hipStream_t);
int lora_acc_chunks(int M, int K);
void launch_lora_proj2(const void*, int, const void*, const void*, int, int, int, float*, int, void*, int, int, uint64_t, float, float,
                       uint64_t, float, float, size_t, uint8_t*, float*, hipStream_t);
int lora_proj2_ws_floats(int, int);
void launch_lora_proj_pair(const void*, const void*, int, const void*, const void*, int, int, int, float*, float*, float,
                           float, int, hipStream_t);
void launch_lora_acc_pair(const float*, const float*, int, int, const void*, const void*, int, int, int, float*, float*,
                          int, hipStream_t);
void launch_lora_acc_quad(const float* const[4], const int[4], const void* const[4], const int[4], const int[4],
                          float* const[4], const int64_t[4], const int64_t[4], const float[4], const uint8_t* const[4],
                          int, int, hipStream_t);
void launch_lora_dA_pair(const float*, const float*, int, int, const void*, int, int, float*, float*, int64_t, int64_t,
                         int64_t, int64_t, const uint8_t*, const uint8_t*, float, float, int, hipStream_t);
void launch_lora_acc_jobs(int, const float* const*, const int*, const int*, const void* const*, const int*, const int*,
                          float* const*, const int64_t*, const int64_t*, const float*, const uint8_t* const*, int,
                          hipStream_t);
void launch_lora_proj_m(const void*, int, int, int, int, const void* const*, const int*, const uint64_t*, const float*,
                        const float*, uint8_t* const*, size_t, float* const*, const int*, void* const*, const int*, float*,
                        hipStream_t);
int lora_proj_m_ws_floats(int, int, int);
void launch_lora_proj_cols(int, const void* const*, int, const void* const*, const int*, const int*, float* const*,
                           const float*, int, hipStream_t);
void launch_lora_dxc(int, const float* const*, const int*, const void* const*, const int*, const uint8_t* const*,
                     const float*, void*, int, int, int, hipStream_t);
void launch_lora_dx2(const float*, const float*, int, const void*, const void*, int, int, const uint8_t*,
                     const uint8_t*, float, float, void*, int, int, hipStream_t);
void launch_lora_apply(void*, int, int, int, const float* const*, const int*, const void* const*, void* const*, const int*, const int*,
                       const int*, hipStream_t);
void launch_lora_acc(const float*, int, int, const void*, int, void*, int, const void*, int, float*, int64_t, int64_t,
                     float*, int, uint64_t, float, size_t, hipStream_t);
void launch_decode_attention(const void*, const void*, const void*, const int*, float*, float*, float*, void*, int, int,
                             int, int, int, int, float, hipStream_t);
int decode_split_plan(int, int, int);
int decode_split_plan2(int, int, int);
void launch_decode_attention2(const void*, int, const void*, int, const void*, int, void*, void*, const int64_t*, float*,
                              float*, float*, void*, int, int, int, int, int, int, float, hipStream_t);
void launch_sample(int, const void*, const int*, int, float*, int64_t*, int, int, float, int, float, float, uint64_t,
                   hipStream_t);
void* car_alloc(size_t, bool);
void car_free(void*);
bool car_ipc_handle(void*, char*);
void* car_ipc_open(const char*);
void car_ipc_close(void*);
int car_max_blocks();
void launch_custom_allreduce(int, const void* const*, void* const*, uint32_t* const*, int*, int, int, uint32_t, size_t,
                             bool, float, void*, int, hipStream_t);
void launch_dropout_fwd(const void*, void*, size_t, uint64_t, float, hipStream_t);
bool embedding_supported(int64_t, int64_t);
void launch_embedding_fwd(const void*, const int64_t*, void*, int64_t, int64_t, int64_t, int64_t, int*, hipStream_t);
void launch_embedding_bwd(const void*, int, const int64_t*, float*, int64_t, int64_t, int64_t, int64_t, hipStream_t);
void launch_dropout_bwd_add(void*, const void*, size_t, uint64_t, float, hipStream_t);

namespace {

using at::Tensor;
using c10::optional;

hipStream_t stream() { return at::hip::getCurrentHIPStream().stream(); }

#define CHECK_CUDA(x) TORCH_CHECK((x).is_cuda(), #x " must be a GPU tensor")
#define CHECK_CONTIG(x) TORCH_CHECK((x).is_contiguous(), #x " must be contiguous")
#define CHECK_BF16(x) TORCH_CHECK((x).scalar_type() == at::kBFloat16, #x " must be bf16")


int dtype_code(const Tensor& t) {
  if (t.scalar_type() == at::kBFloat16) return 1;
  TORCH_CHECK(t.scalar_type() == at::kFloat, "expected fp32 or bf16, got ", t.scalar_type());
  return 0;
}
const void* optr(const optional<Tensor>& t) { return t.has_value() && t->defined() ? t->data_ptr() : nullptr; }
template <typename T>
const T* optr_t(const optional<Tensor>& t) {
  return t.has_value() && t->defined() ? t->data_ptr<T>() : nullptr;
}

// ------------------------------------------------------------------ norms
std::vector<Tensor> rmsnorm_fwd(Tensor x, optional<Tensor> w, double eps) {
  CHECK_CUDA(x);
  CHECK_CONTIG(x);
  const int N = x.size(-1), M = x.numel() / N;
  TORCH_CHECK(N % 8 == 0, "rmsnorm: hidden size must be a multiple of 8");
  if (w) TORCH_CHECK(w->scalar_type() == x.scalar_type() && w->is_contiguous(), "rmsnorm weight dtype/layout");
  auto y = at::empty_like(x);
  auto rstd = at::empty({M}, x.options().dtype(at::kFloat));
  launch_rmsnorm_fwd(dtype_code(x), x.data_ptr(), optr(w), y.data_ptr(), rstd.data_ptr<float>(), M, N, (float)eps,
                     stream());
  return {y, rstd};
}

std::vector<Tensor> rmsnorm_bwd(Tensor dy, Tensor x, optional<Tensor> w, Tensor rstd, bool need_dw,
                                optional<Tensor> dres) {
  CHECK_CONTIG(dy);
  CHECK_CONTIG(x);
  if (dres && dres->defined()) {
    TORCH_CHECK(dres->is_contiguous() && dres->sizes() == x.sizes() && dres->scalar_type() == x.scalar_type(),
                "rmsnorm_bwd: dres must match x");
  }
  const int N = x.size(-1), M = x.numel() / N;
  auto dx = at::empty_like(x);
  Tensor part, dw;
  if (need_dw) {
    part = at::empty({norm_partial_rows(M), N}, x.options().dtype(at::kFloat));
    dw = at::empty({N}, x.options().dtype(at::kFloat));
  }
  launch_rmsnorm_bwd(dtype_code(x), dy.data_ptr(), x.data_ptr(), optr(w), rstd.data_ptr<float>(), dx.data_ptr(),
                     need_dw ? part.data_ptr<float>() : nullptr, need_dw ? dw.data_ptr<float>() : nullptr, M, N,
                     optr(dres), stream());
  return {dx, dw};
}

std::vector<Tensor> layernorm_fwd(Tensor x, optional<Tensor> w, optional<Tensor> b, double eps) {
  CHECK_CUDA(x);
  CHECK_CONTIG(x);
  const int N = x.size(-1), M = x.numel() / N;
  TORCH_CHECK(N % 8 == 0, "layernorm: hidden size must be a multiple of 8");
  auto y = at::empty_like(x);
  auto mean = at::empty({M}, x.options().dtype(at::kFloat));
  auto rstd = at::empty({M}, x.options().dtype(at::kFloat));
  launch_layernorm_fwd(dtype_code(x), x.data_ptr(), optr(w), optr(b), y.data_ptr(), mean.data_ptr<float>(),
                       rstd.data_ptr<float>(), M, N, (float)eps, stream());
  return {y, mean, rstd};
}

std::vector<Tensor> layernorm_bwd(Tensor dy, Tensor x, optional<Tensor> w, Tensor mean, Tensor rstd, bool need_dw) {
  const int N = x.size(-1), M = x.numel() / N;
  auto dx = at::empty_like(x);
  Tensor part, dw, db;
  if (need_dw) {
    part = at::empty({2 * norm_partial_rows(M), N}, x.options().dtype(at::kFloat));
    dw = at::empty({N}, x.options().dtype(at::kFloat));
    db = at::empty({N}, x.options().dtype(at::kFloat));
  }
  launch_layernorm_bwd(dtype_code(x), dy.data_ptr(), x.data_ptr(), optr(w), mean.data_ptr<float>(),
                       rstd.data_ptr<float>(), dx.data_ptr(), need_dw ? part.data_ptr<float>() : nullptr,
                       need_dw ? dw.data_ptr<float>() : nullptr, need_dw ? db.data_ptr<float>() : nullptr, M, N,
                       stream());
  return {dx, dw, db};
}

// ------------------------------------------------------------------ rope
Tensor rope(Tensor x, Tensor cos, Tensor sin, bool interleaved, bool inverse) {
  CHECK_CONTIG(x);
  TORCH_CHECK(x.dim() == 3, "rope expects [T, H, D]");
  auto y = at::empty_like(x);
  launch_rope(dtype_code(x), x.data_ptr(), cos.data_ptr<float>(), sin.data_ptr<float>(), y.data_ptr(), x.size(0),
              x.size(1), x.size(2), interleaved, inverse, stream());
  return y;
}

std::vector<Tensor> qk_norm_rope_fwd(Tensor qkv, optional<Tensor> qw, optional<Tensor> kw, Tensor cos, Tensor sin,
                                     int64_t hq, int64_t hkv, int64_t d, double eps) {
  CHECK_BF16(qkv);
  CHECK_CONTIG(qkv);
  const int T = qkv.size(0);
  TORCH_CHECK(qkv.size(1) == (hq + 2 * hkv) * d, "qkv width mismatch");
  TORCH_CHECK(cos.scalar_type() == at::kFloat && cos.size(0) == T && cos.size(1) == d / 2, "cos table [T, D/2] fp32");
  auto q = at::empty({T, hq * d}, qkv.options());
  auto k = at::empty({T, hkv * d}, qkv.options());
  auto rq = at::empty({T * hq}, qkv.options().dtype(at::kFloat));
  auto rk = at::empty({T * hkv}, qkv.options().dtype(at::kFloat));
  launch_qk_norm_rope_fwd(qkv.data_ptr(), optr(qw), optr(kw), cos.data_ptr<float>(), sin.data_ptr<float>(),
                          q.data_ptr(), k.data_ptr(), rq.data_ptr<float>(), rk.data_ptr<float>(), T, hq, hkv, d,
                          (float)eps, stream());
  return {q, k, rq, rk};
}

Tensor qk_norm_rope_bwd(Tensor dq, Tensor dk, optional<Tensor> dv, Tensor qkv, optional<Tensor> qw,
                        optional<Tensor> kw, Tensor cos, Tensor sin, Tensor rq, Tensor rk, int64_t hq, int64_t hkv,
                        int64_t d) {
  const int T = qkv.size(0);
  auto dqkv = at::empty_like(qkv);
  const void* dvp = nullptr;
  if (dv && dv->defined()) {
    CHECK_BF16((*dv));
    CHECK_CONTIG((*dv));
    TORCH_CHECK(dv->numel() == (int64_t)T * hkv * d, "qk_norm_rope_bwd: dv [T, hkv*d]");
    dvp = dv->data_ptr();
  }
  // the kernel writes all three parts of dqkv (the v rows: dv copied through, zeros without one)
  launch_qk_norm_rope_bwd(dq.data_ptr(), dk.data_ptr(), dvp, qkv.data_ptr(), optr(qw), optr(kw),
                          cos.data_ptr<float>(), sin.data_ptr<float>(), rq.data_ptr<float>(), rk.data_ptr<float>(),
                          dqkv.data_ptr(), T, hq, hkv, d, stream());
  return dqkv;
}

// ------------------------------------------------------------------ activations
Tensor swiglu_fwd(Tensor gu) {
  CHECK_BF16(gu);
  CHECK_CONTIG(gu);
  const int F = gu.size(-1) / 2, M = gu.numel() / gu.size(-1);
  TORCH_CHECK(F % 8 == 0, "swiglu: intermediate size must be a multiple of 8");
  auto sizes = gu.sizes().vec();
  sizes.back() = F;
  auto y = at::empty(sizes, gu.options());
  launch_swiglu_fwd(gu.data_ptr(), y.data_ptr(), M, F, stream());
  return y;
}
Tensor swiglu_bwd(Tensor dy, Tensor gu) {
  const int F = gu.size(-1) / 2, M = gu.numel() / gu.size(-1);
  auto dgu = at::empty_like(gu);
  launch_swiglu_bwd(dy.data_ptr(), gu.data_ptr(), dgu.data_ptr(), M, F, stream());
  return dgu;
}
Tensor gelu_fwd(Tensor x) {
  CHECK_CONTIG(x);
  auto y = at::empty_like(x);
  launch_gelu_fwd(dtype_code(x), x.data_ptr(), y.data_ptr(), x.numel(), stream());
  return y;
}
Tensor gelu_bwd(Tensor dy, Tensor x) {
  auto dx = at::empty_like(x);
  launch_gelu_bwd(dtype_code(x), dy.data_ptr(), x.data_ptr(), dx.data_ptr(), x.numel(), stream());
  return dx;
}

// ------------------------------------------------------------------ dropout (counter RNG)
// embedding gather: weight [V, D] (any dtype, D·elem % 16 == 0), ids int64 (any shape) → [*ids, D]
// oob (optional int32 [1] on the device): set to 1 when an id is outside [0, V) (that row reads clamped)
Tensor embedding_fwd(Tensor weight, Tensor ids, c10::optional<Tensor> oob) {
  CHECK_CONTIG(weight);
  TORCH_CHECK(weight.dim() == 2 && ids.scalar_type() == at::kLong, "embedding_fwd: weight [V, D], int64 ids");
  const int64_t V = weight.size(0), D = weight.size(1), el = weight.element_size();
  TORCH_CHECK(embedding_supported(D, el), "embedding_fwd: row bytes % 16");
  Tensor idc = ids.contiguous();
  auto sizes = idc.sizes().vec();
  sizes.push_back(D);
  Tensor out = at::empty(sizes, weight.options());
  int* flag = nullptr;
  if (oob.has_value() && oob->defined()) {
    TORCH_CHECK(oob->scalar_type() == at::kInt && oob->is_cuda(), "embedding_fwd: oob int32 device tensor");
    flag = oob->data_ptr<int>();
  }
  launch_embedding_fwd(weight.data_ptr(), idc.data_ptr<int64_t>(), out.data_ptr(), idc.numel(), D, el, V, flag, stream());
  return out;
}
// gradient of the gather: fp32 [V, D] (scatter-add of dout rows; padding_idx < 0: none)
Tensor embedding_bwd(Tensor dout, Tensor ids, int64_t V, int64_t padding_idx) {
  TORCH_CHECK(dout.scalar_type() == at::kBFloat16 || dout.scalar_type() == at::kFloat, "embedding_bwd: bf16/fp32");
  Tensor d = dout.contiguous(), idc = ids.contiguous();
  const int64_t D = d.size(-1);
  TORCH_CHECK(D % 8 == 0 && d.numel() == idc.numel() * D, "embedding_bwd: shapes");
  Tensor gw = at::zeros({V, D}, d.options().dtype(at::kFloat));
  launch_embedding_bwd(d.data_ptr(), d.scalar_type() == at::kFloat ? 1 : 0, idc.data_ptr<int64_t>(), gw.data_ptr<float>(),
                       idc.numel(), D, V, padding_idx, stream());
  return gw;
}

Tensor dropout_fwd(Tensor x, double p, int64_t key) {
  CHECK_BF16(x);
  CHECK_CONTIG(x);
  TORCH_CHECK(x.numel() % 8 == 0, "dropout: numel % 8");
  auto y = at::empty_like(x);
  launch_dropout_fwd(x.data_ptr(), y.data_ptr(), x.numel(), (uint64_t)key, (float)p, stream());
  return y;
}
void dropout_bwd_add(Tensor dx, Tensor t, double p, int64_t key) {
  CHECK_CONTIG(dx);
  CHECK_CONTIG(t);
  launch_dropout_bwd_add(dx.data_ptr(), t.data_ptr(), dx.numel(), (uint64_t)key, (float)p, stream());
}

// ------------------------------------------------------------------ cross entropy
Tensor ce_fwd_bwd(Tensor logits, Tensor labels, int64_t ignore_index, Tensor scale) {
  CHECK_CONTIG(logits);
  TORCH_CHECK(labels.scalar_type() == at::kLong, "labels int64");
  const int M = logits.size(0), V = logits.size(1);
  TORCH_CHECK(V % 8 == 0, "vocab must be a multiple of 8");
  auto loss = at::empty({M}, logits.options().dtype(at::kFloat));
  auto sc = scale.to(at::kFloat).contiguous();
  // scale: one value, or one per equal group of rows (fused gradient-accumulation micro-batches)
  TORCH_CHECK(sc.numel() >= 1 && M % sc.numel() == 0, "ce_fwd_bwd: scale groups must split the rows evenly");
  const int rows_per_scale = sc.numel() > 1 ? M / (int)sc.numel() : 0;
  launch_ce_fwd_bwd(dtype_code(logits), logits.data_ptr(), labels.contiguous().data_ptr<int64_t>(),
                    loss.data_ptr<float>(), M, V, ignore_index, sc.data_ptr<float>(), 1.f, rows_per_scale, stream());
  return loss;
}

// ------------------------------------------------------------------ optimizers
Tensor grad_norm(Tensor g, double max_norm, optional<Tensor> out, bool accumulate) {
  CHECK_CONTIG(g);
  Tensor o = out && out->defined() ? *out : at::zeros({3}, g.options().dtype(at::kFloat));
  auto part = at::empty({1024}, g.options().dtype(at::kFloat));
  launch_grad_norm(dtype_code(g), g.data_ptr(), g.numel(), part.data_ptr<float>(), o.data_ptr<float>(),
                   (float)max_norm, accumulate, stream());
  return o;
}

void adamw(Tensor p, Tensor g, Tensor m, Tensor v, optional<Tensor> p16, double lr, double b1, double b2, double eps,
           double wd, int64_t step, optional<Tensor> gscale, optional<Tensor> skip) {
  TORCH_CHECK(p.scalar_type() == at::kFloat && m.scalar_type() == at::kFloat && v.scalar_type() == at::kFloat,
              "adamw: fp32 master/state");
  TORCH_CHECK(p.is_contiguous() && g.is_contiguous() && m.is_contiguous() && v.is_contiguous(), "adamw: contiguous");
  const float bc1 = 1.f - std::pow((float)b1, (float)step), bc2 = 1.f - std::pow((float)b2, (float)step);
  launch_adamw(dtype_code(g), p.data_ptr<float>(), g.data_ptr(), m.data_ptr<float>(), v.data_ptr<float>(),
               (void*)optr(p16), p.numel(), lr, b1, b2, eps, wd, bc1, bc2, optr_t<float>(gscale), optr_t<float>(skip),
               stream());
}

// A device tensor whose storage is pinned, device-mapped HOST memory (hipHostMalloc mapped + its device pointer):
// kernels read and write it across the host link, nothing of it occupies HBM.  The "paged" placement of the 8-bit
// optimizer states (optim/adamw.py AdamW8bit(paged="host"), bitsandbytes paged_adamw_8bit's role).
Tensor host_mapped_empty(int64_t numel, at::ScalarType dtype) {
  TORCH_CHECK(numel > 0, "host_mapped_empty: numel > 0");
  const size_t bytes = (size_t)numel * c10::elementSize(dtype);
  void* hp = nullptr;
  TORCH_CHECK(hipHostMalloc(&hp, bytes, hipHostMallocMapped) == hipSuccess, "host_mapped_empty: hipHostMalloc failed");
  void* dp = nullptr;
  if (hipHostGetDevicePointer(&dp, hp, 0) != hipSuccess) {
    (void)hipHostFree(hp);
    TORCH_CHECK(false, "host_mapped_empty: hipHostGetDevicePointer failed");
  }
  int dev = 0;
  (void)hipGetDevice(&dev);
  return torch::from_blob(dp, {numel}, [hp](void*) { (void)hipHostFree(hp); },
                          torch::TensorOptions().dtype(dtype).device(torch::kCUDA, dev));
}

void adamw8bit(Tensor p, Tensor g, Tensor qm, Tensor qv, Tensor am, Tensor av, Tensor code_s, Tensor code_u,
               optional<Tensor> p16, double lr, double b1, double b2, double eps, double wd, int64_t step,
               optional<Tensor> gscale, optional<Tensor> skip) {
  const float bc1 = 1.f - std::pow((float)b1, (float)step), bc2 = 1.f - std::pow((float)b2, (float)step);
  launch_adamw8bit(dtype_code(g), p.data_ptr<float>(), g.data_ptr(), qm.data_ptr<uint8_t>(), qv.data_ptr<uint8_t>(),
                   am.data_ptr<float>(), av.data_ptr<float>(), code_s.data_ptr<float>(), code_u.data_ptr<float>(),
                   (void*)optr(p16), p.numel(), lr, b1, b2, eps, wd, bc1, bc2, optr_t<float>(gscale),
                   optr_t<float>(skip), stream());
}

void unscale(Tensor g, Tensor inv_scale, Tensor found_inf) {
  launch_unscale(dtype_code(g), g.data_ptr(), g.numel(), inv_scale.data_ptr<float>(), found_inf.data_ptr<float>(),
                 stream());
}

// ------------------------------------------------------------------ NF4
std::vector<Tensor> nf4_quantize(Tensor w, int64_t blocksize) {
  CHECK_BF16(w);
  CHECK_CONTIG(w);
  TORCH_CHECK(blocksize == 64, "NF4 kernel quantises with blocksize 64");
  TORCH_CHECK(w.size(-1) % 64 == 0, "in_features % 64");
  auto codes = at::empty({w.size(0), w.size(1) / 2}, w.options().dtype(at::kByte));
  auto absmax = at::empty({w.numel() / 64}, w.options().dtype(at::kFloat));
  launch_nf4_quantize(w.data_ptr(), codes.data_ptr<uint8_t>(), absmax.data_ptr<float>(), w.numel(), stream());
  return {codes, absmax};
}

// decode-shaped y = x·Wᵀ (+ residual): x [M <= 64, K] row-strided, W [N, K] contiguous bf16
// ---- hipBLASLt frozen-base GEMMs (csrc/kernels/blaslt.hip)
static void* lt_workspace(size_t& bytes) {
  static std::map<int, Tensor> ws;   // one hipBLASLt workspace per device (64 MiB; LIPA_LT_WS_MB), kept for the process
  static const size_t mb = [] { const char* e = getenv("LIPA_LT_WS_MB"); return (size_t)(e && atoi(e) > 0 ? atoi(e) : 64); }();
  const int dev = at::hip::current_device();
  bytes = mb << 20;
  Tensor& t = ws[dev];
  if (!t.defined()) t = at::empty({(int64_t)bytes}, at::TensorOptions().dtype(at::kByte).device(at::kCUDA, dev));
  return t.data_ptr();
}

// y = x·wᵀ (+ residual): x [M, K] (unit column stride), w [N, K] contiguous bf16
Tensor lt_linear(Tensor x, Tensor w, optional<Tensor> residual, bool tune) {
  CHECK_CUDA(x);
  CHECK_BF16(x);
  CHECK_BF16(w);
  CHECK_CONTIG(w);
  TORCH_CHECK(x.dim() == 2 && x.stride(1) == 1 && w.dim() == 2 && w.size(1) == x.size(1), "lt_linear: shapes");
  const int64_t M = x.size(0), K = x.size(1), N = w.size(0);
  const void* cp = nullptr;
  if (residual.has_value() && residual->defined()) {
    CHECK_BF16((*residual));
    CHECK_CONTIG((*residual));
    TORCH_CHECK(residual->size(0) == M && residual->size(1) == N, "lt_linear: residual shape");
    cp = residual->data_ptr();
  }
  Tensor out = at::empty({M, N}, x.options());
  size_t wsb;
  void* ws = lt_workspace(wsb);
  if (!lt_gemm(true, false, N, M, K, w.data_ptr(), K, x.data_ptr(), x.stride(0), cp, out.data_ptr(), N, 1, 0, 0, 0,
               ws, wsb, stream(), tune))
    return cp ? at::addmm(*residual, x, w.t()) : at::mm(x, w.t());
  return out;
}

// dx = dy·w: dy [M, N] contiguous, w [N, K] contiguous; split > 1: K-slices of the reduction dim
// as one strided-batched GEMM into bf16 partials + an fp32 slice sum
Tensor lt_dx(Tensor dy, Tensor w, int64_t split, bool tune, optional<Tensor> c) {
  CHECK_CUDA(dy);
  CHECK_BF16(dy);
  CHECK_BF16(w);
  CHECK_CONTIG(dy);
  CHECK_CONTIG(w);
  const int64_t M = dy.size(0), N = dy.size(1), K = w.size(1);
  TORCH_CHECK(w.size(0) == N, "lt_dx: shapes");
  TORCH_CHECK(split == 1 || ((split == 2 || split == 3 || split == 4 || split == 8) && N % split == 0 && K % 8 == 0),
              "lt_dx: split");
  size_t wsb;
  void* ws = lt_workspace(wsb);
  Tensor out = at::empty({M, K}, dy.options());
  const void* cp = nullptr;
  if (c.has_value() && c->defined()) {   // dx = dy·w + c (c: the LoRA input-gradient term)
    CHECK_BF16((*c));
    CHECK_CONTIG((*c));
    TORCH_CHECK(c->size(0) == M && c->size(1) == K && split == 1, "lt_dx: c [M, K], no split");
    cp = c->data_ptr();
  }
  if (split == 1) {
    if (!lt_gemm(false, false, K, M, N, w.data_ptr(), K, dy.data_ptr(), N, cp, out.data_ptr(), K, 1, 0, 0, 0, ws,
                 wsb, stream(), tune))
      return cp ? at::addmm(*c, dy, w) : at::mm(dy, w);
    return out;
  }
  const int64_t Ns = N / split;
  Tensor part = at::empty({split, M, K}, dy.options());
  if (!lt_gemm(false, false, K, M, Ns, w.data_ptr(), K, dy.data_ptr(), N, nullptr, part.data_ptr(), K, (int)split,
               Ns * K, Ns, M * K, ws, wsb, stream(), tune))
    return at::mm(dy, w);
  launch_sum_slices(part.data_ptr(), out.data_ptr(), (int)split, (size_t)(M * K), (size_t)(M * K), stream());
  return out;
}

Tensor gemm_skinny(Tensor x, Tensor w, optional<Tensor> residual) {
  CHECK_CUDA(x);
  CHECK_BF16(x);
  CHECK_BF16(w);
  CHECK_CONTIG(w);
  const int64_t M = x.size(0), K = x.size(1), N = w.size(0);
  TORCH_CHECK(x.dim() == 2 && x.stride(1) == 1 && x.stride(0) % 8 == 0 && M >= 1 && M <= 64,
              "gemm_skinny: x [M<=64, K] row-major, 16-B aligned rows");
  TORCH_CHECK(w.dim() == 2 && w.size(1) == K && K % 64 == 0 && N % 16 == 0, "gemm_skinny: W [N%16, K%64]");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0 && reinterpret_cast<uintptr_t>(w.data_ptr()) % 16 == 0,
              "gemm_skinny: 16-B aligned operands");
  const void* rp = nullptr;
  if (residual.has_value() && residual->defined()) {
    CHECK_BF16((*residual));
    CHECK_CONTIG((*residual));
    TORCH_CHECK(residual->size(0) == M && residual->size(1) == N, "gemm_skinny: residual shape");
    rp = residual->data_ptr();
  }
  const int S = skinny_splits(N, K);
  Tensor part = at::empty({S, M, N}, x.options().dtype(at::kFloat));
  Tensor out = at::empty({M, N}, x.options());
  launch_gemm_skinny(x.data_ptr(), x.stride(0), w.data_ptr(), rp, out.data_ptr(), part.data_ptr<float>(), M, N, K, S,
                     stream());
  return out;
}

// W4A16 MFMA GEMM (csrc/kernels/w4mm.hip): x [M<=64, K] bf16, codes u8 [N, K/2] (high nibble = even k),
// sc2 fp32 [N, K/gs, 2] = (scale, bias − 128·scale)
bool w4mm_ok(int64_t M, int64_t N, int64_t K, int64_t gs) { return w4mm_supported((int)M, (int)N, (int)K, (int)gs); }

Tensor w4mm(Tensor x, Tensor codes, Tensor sc2, int64_t N, int64_t gs, optional<Tensor> residual, int64_t nkb) {
  CHECK_CUDA(x); CHECK_BF16(x); CHECK_CONTIG(codes); CHECK_CONTIG(sc2);
  const int64_t M = x.size(0), K = x.size(1);
  TORCH_CHECK(x.dim() == 2 && x.stride(1) == 1 && x.stride(0) % 8 == 0, "w4mm: x row-major, 16-B aligned rows");
  TORCH_CHECK(w4mm_supported((int)M, (int)N, (int)K, (int)gs), "w4mm: M<=64, N%128, K%128, gs%128");
  TORCH_CHECK(codes.scalar_type() == at::kByte && codes.numel() == N * K / 2, "w4mm: codes [N, K/2] uint8");
  TORCH_CHECK(sc2.scalar_type() == at::kFloat && sc2.numel() == N * (K / gs) * 2, "w4mm: sc2 fp32 [N, K/gs, 2]");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0 && reinterpret_cast<uintptr_t>(codes.data_ptr()) % 16 == 0 &&
                  reinterpret_cast<uintptr_t>(sc2.data_ptr()) % 8 == 0,
              "w4mm: aligned operands");
  TORCH_CHECK((size_t)N * K / 2 < (1ull << 31) * 2, "w4mm: codes too large");
  const void* rp = nullptr;
  if (residual.has_value() && residual->defined()) {
    CHECK_BF16((*residual));
    CHECK_CONTIG((*residual));
    TORCH_CHECK(residual->size(0) == M && residual->size(1) == N, "w4mm: residual shape");
    rp = residual->data_ptr();
  }
  const int nb = nkb > 0 ? (int)nkb : w4mm_nkb((int)M, (int)N, (int)K);
  TORCH_CHECK(nb == 1 || nb == 2 || nb == 4 || nb == 8, "w4mm: nkb in 1/2/4/8");
  TORCH_CHECK((K / 128) % nb == 0, "w4mm: K/128 divisible by nkb");
  const int KS = (int)(K / (128 * nb));
  Tensor out = at::empty({M, N}, x.options());
  Tensor part;
  if (KS > 1) part = at::empty({KS, M, N}, x.options().dtype(at::kFloat));
  launch_w4mm(x.data_ptr(), (int)x.stride(0), codes.data_ptr<uint8_t>(), sc2.data_ptr<float>(), (int)gs, rp,
              out.data_ptr(), KS > 1 ? part.data_ptr<float>() : nullptr, (int)M, (int)N, (int)K, nb, stream());
  return out;
}

// The decode-batch tiling of the same W4A16 GEMM (w4mm.hip w4g_k): 1 <= M <= 64, same operands as w4mm.
bool w4g_ok(int64_t M, int64_t N, int64_t K, int64_t gs) { return w4g_supported((int)M, (int)N, (int)K, (int)gs); }

Tensor w4g(Tensor x, Tensor codes, Tensor sc2, int64_t N, int64_t gs, optional<Tensor> residual, int64_t ks) {
  CHECK_CUDA(x); CHECK_BF16(x); CHECK_CONTIG(codes); CHECK_CONTIG(sc2);
  const int64_t M = x.size(0), K = x.size(1);
  TORCH_CHECK(x.dim() == 2 && x.stride(1) == 1 && x.stride(0) % 8 == 0, "w4g: x row-major, 16-B aligned rows");
  TORCH_CHECK(w4g_supported((int)M, (int)N, (int)K, (int)gs), "w4g: M<=64, N%128, K%128, gs%128");
  TORCH_CHECK(codes.scalar_type() == at::kByte && codes.numel() == N * K / 2, "w4g: codes [N, K/2] uint8");
  TORCH_CHECK(sc2.scalar_type() == at::kFloat && sc2.numel() == N * (K / gs) * 2, "w4g: sc2 fp32 [N, K/gs, 2]");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0 && reinterpret_cast<uintptr_t>(codes.data_ptr()) % 16 == 0 &&
                  reinterpret_cast<uintptr_t>(sc2.data_ptr()) % 8 == 0,
              "w4g: aligned operands");
  const void* rp = nullptr;
  if (residual.has_value() && residual->defined()) {
    CHECK_BF16((*residual));
    CHECK_CONTIG((*residual));
    TORCH_CHECK(residual->size(0) == M && residual->size(1) == N, "w4g: residual shape");
    rp = residual->data_ptr();
  }
  const int s = ks > 0 ? (int)ks : w4g_splits((int)M, (int)N, (int)K);
  TORCH_CHECK((K / 128) % s == 0, "w4g: K/128 divisible by the K-slice count");
  Tensor out = at::empty({M, N}, x.options());
  Tensor part;
  if (s > 1) part = at::empty({s, M, N}, x.options().dtype(at::kFloat));
  launch_w4g(x.data_ptr(), (int)x.stride(0), codes.data_ptr<uint8_t>(), sc2.data_ptr<float>(), (int)gs, rp,
             out.data_ptr(), s > 1 ? part.data_ptr<float>() : nullptr, (int)M, (int)N, (int)K, s, stream());
  return out;
}

// codes [N, K/2] u8 (bnb layout), absmax fp32 [N*K/64] (decoded) → bf16 [N, K]
// affine int4 codes [N, K/2] + fp32 scale / bias tables [N, K/g] -> bf16 [N, K] (quant/int4.py layout)
Tensor int4_dequant(Tensor codes, Tensor sc, Tensor bi, int64_t N, int64_t K, int64_t group) {
  CHECK_CUDA(codes);
  CHECK_CONTIG(codes);
  CHECK_CONTIG(sc);
  CHECK_CONTIG(bi);
  TORCH_CHECK(codes.scalar_type() == at::kByte && codes.numel() * 2 == N * K && K % group == 0 && group % 8 == 0,
              "int4_dequant: codes uint8 [N, K/2], K % group, group % 8");
  TORCH_CHECK(sc.scalar_type() == at::kFloat && bi.scalar_type() == at::kFloat && sc.numel() * group == N * K &&
                  bi.numel() == sc.numel(), "int4_dequant: fp32 tables [N, K/g]");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(codes.data_ptr()) % 4 == 0, "int4_dequant: 4-B aligned codes");
  auto w = at::empty({N, K}, codes.options().dtype(at::kBFloat16));
  launch_int4_dequant(codes.data_ptr<uint8_t>(), sc.data_ptr<float>(), bi.data_ptr<float>(), w.data_ptr(),
                      (size_t)N * K, (int)group, stream());
  return w;
}

Tensor nf4_dequant_fast(Tensor codes, Tensor absmax, int64_t N, int64_t K) {
  CHECK_CUDA(codes);
  CHECK_CONTIG(codes);
  CHECK_CONTIG(absmax);
  TORCH_CHECK(codes.numel() * 2 == N * K && K % 64 == 0, "nf4_dequant_fast: codes shape");
  TORCH_CHECK(absmax.scalar_type() == at::kFloat && absmax.numel() * 64 == N * K, "nf4_dequant_fast: absmax");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(codes.data_ptr()) % 16 == 0, "nf4_dequant_fast: 16-B aligned codes");
  auto w = at::empty({N, K}, codes.options().dtype(at::kBFloat16));
  launch_nf4_dequant2(codes.data_ptr<uint8_t>(), absmax.data_ptr<float>(), w.data_ptr(), N * K, stream());
  return w;
}

// background expansion of up to 4 NF4 weights in one small persistent grid (see gemm.hip)

Tensor nf4_dequant(Tensor codes, optional<Tensor> absmax, optional<Tensor> qabs, optional<Tensor> absmax2,
                   optional<Tensor> offset, optional<Tensor> dcode, int64_t N, int64_t K) {
  auto w = at::empty({N, K}, codes.options().dtype(at::kBFloat16));
  launch_nf4_dequant(codes.data_ptr<uint8_t>(), optr_t<float>(absmax), optr_t<uint8_t>(qabs), optr_t<float>(absmax2),
                     optr_t<float>(offset), optr_t<float>(dcode), w.data_ptr(), N * K, stream());
  return w;
}

void check_ext(const optional<Tensor>& ea, const optional<Tensor>& eb, int M, int C, int& R_ext) {
  R_ext = 0;
  if (ea && ea->defined()) {
    TORCH_CHECK(eb && eb->defined(), "ext_b required with ext_a");
    CHECK_BF16(*ea);
    CHECK_BF16(*eb);
    CHECK_CONTIG(*ea);
    CHECK_CONTIG(*eb);
    R_ext = ea->size(1);
    TORCH_CHECK(R_ext % 32 == 0 && ea->size(0) == M && eb->size(0) == C && eb->size(1) == R_ext,
                "LoRA K-slice shapes: ext_a [M, R], ext_b [C, R], R % 32 == 0");
  }
}

// decode GEMV (M <= 8): codes [N, K/2] bytes (high nibble = even k), scales [N, K/blk] fp32,
// bias [N, K/blk] fp32 (affine int4) or None (NF4)
Tensor gemv_w4(Tensor x, Tensor codes, Tensor scales, optional<Tensor> bias, int64_t N, int64_t blk,
               optional<Tensor> residual) {
  CHECK_BF16(x);
  TORCH_CHECK(x.dim() == 2 && x.stride(1) == 1 && x.stride(0) % 8 == 0, "gemv_w4: x row-major");
  const int M = x.size(0), K = x.size(1);
  TORCH_CHECK(M <= 8, "gemv_w4: M <= 8");
  TORCH_CHECK(K % 32 == 0 && blk % 32 == 0 && K % blk == 0, "gemv_w4: K % 32, blk % 32");
  TORCH_CHECK(codes.numel() == N * K / 2 && scales.numel() == N * K / blk, "gemv_w4: weight size");
  if (residual) TORCH_CHECK(residual->is_contiguous() && residual->size(0) == M && residual->size(1) == N, "residual");
  auto y = at::empty({M, N}, x.options());
  const bool aff = bias.has_value() && bias->defined();
  launch_gemv_w4(aff ? 2 : 0, x.data_ptr(), x.stride(0), codes.data_ptr<uint8_t>(), scales.data_ptr<float>(),
                 aff ? bias->data_ptr<float>() : nullptr, blk, optr(residual), y.data_ptr(), M, N, K, stream());
  return y;
}


// The B operand of the gemm4w entry points: a bf16 weight, or (wscale given) the g4w-packed NF4 codes of one
// (uint8, R·C/2 bytes, NF4Weight.g4w_pack) with wscale = the decoded fp32 block absmax transposed [C/64, R].
struct G4wB {
  const void* ptr;
  const float* scale;
  int64_t ld;
};
static G4wB g4w_operand(const Tensor& w, const optional<Tensor>& wscale, int64_t rows, int64_t cols) {
  if (wscale && wscale->defined()) {
    TORCH_CHECK(w.scalar_type() == at::kByte && w.is_contiguous() && w.numel() * 2 == rows * cols,
                "gemm4w: NF4 codes [rows·cols/2] uint8");
    TORCH_CHECK(wscale->scalar_type() == at::kFloat && wscale->is_contiguous() && wscale->numel() * 64 == rows * cols,
                "gemm4w: NF4 scales [cols/64, rows] fp32");
    TORCH_CHECK(rows % 64 == 0 && cols % 64 == 0, "gemm4w: NF4 rows / cols multiples of 64");
    return {w.data_ptr(), wscale->data_ptr<float>(), cols};
  }
  CHECK_BF16(w);
  TORCH_CHECK(w.dim() == 2 && w.stride(1) == 1 && w.size(0) == rows && w.size(1) == cols, "gemm4w: weight shape");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(w.data_ptr()) % 16 == 0, "gemm4w: 16-byte aligned weight");
  return {w.data_ptr(), nullptr, w.stride(0)};
}

bool gemm4w_ok(int64_t M, int64_t N, int64_t K, int64_t lda, int64_t ldb, bool bt, bool w4) {
  return M < (1ll << 31) && N < (1ll << 31) && K < (1ll << 31) && gemm4w_supported(M, N, K, lda, ldb, bt, w4);
}

// the cost model's choice for a plain gemm4w call (host-only: no device needed): (splits, bn, bm)
std::vector<int64_t> gemm4w_plan_info(int64_t M, int64_t N, int64_t K, bool bt, bool w4) {
  int bn = 0, bm = 0;
  const int sp = gemm4w_plan((int)M, (int)N, (int)K, bt, 0, 0, &bn, 0, &bm, w4);
  return {sp, bn, bm};
}

// y = x·wᵀ (+ residual) through the one-wave-per-SIMD AGPR-accumulator MFMA GEMM (gemm4w.hip);
// x [M, K] (row stride any multiple of 8), w [N, K] contiguous rows.  bt: y = x·w with w [K, N]
// (the dX = dY·W of a frozen [N_w, K_w] weight, no transpose copy).  splits <= 0: auto split-K;
// bn: tile width 128 / 256 / 192 (bf16; the transposed-B 192 tile is 256 rows high), 0 = auto.  wscale: w is an NF4 base (g4w_operand); n_w4
// is then the GEMM N (the weight's rows for NT, its columns for bt).
Tensor gemm4w(Tensor x, Tensor w, optional<Tensor> residual, int64_t splits, bool bt, int64_t bn, int64_t bm,
              optional<Tensor> wscale, int64_t n_w4, optional<Tensor> wzero) {
  CHECK_BF16(x);
  TORCH_CHECK(x.dim() == 2 && x.stride(1) == 1, "gemm4w: x 2-D, unit inner stride");
  const bool w4 = wscale && wscale->defined();
  const int64_t M = x.size(0), K = x.size(1);
  const int64_t N = w4 ? n_w4 : (w.dim() == 2 ? (bt ? w.size(1) : w.size(0)) : 0);
  const G4wB b = bt ? g4w_operand(w, wscale, K, N) : g4w_operand(w, wscale, N, K);
  TORCH_CHECK(gemm4w_ok(M, N, K, x.stride(0), b.ld, bt, w4), "gemm4w: unsupported shape / strides");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0, "gemm4w: 16-byte aligned operands");
  const void* res = nullptr;
  if (residual && residual->defined()) {
    CHECK_BF16(*residual);
    TORCH_CHECK(residual->is_contiguous() && residual->size(0) == M && residual->size(1) == N, "gemm4w: residual [M, N]");
    res = residual->data_ptr();
  }
  TORCH_CHECK(bn == 0 || bn == 128 || bn == 256 || (bn == 192 && !w4 && !(bt && bm == 128)),
              "gemm4w: bn 0 / 128 / 256 / 192 (bf16; transposed-B 192 with 256-row tiles)");
  TORCH_CHECK(bm == 0 || bm == 128 || bm == 256, "gemm4w: bm 0 / 128 / 256");
  int bn_used = 0, bm_used = 0;
  const int sp = gemm4w_plan(M, N, K, bt, (int)bn, (int)splits, &bn_used, (int)bm, &bm_used, w4);
  auto y = at::empty({M, N}, x.options());
  Tensor ws;
  if (sp > 1) ws = at::empty({sp, M, N}, x.options().dtype(at::kFloat));
  const float* zp = nullptr;
  if (wzero && wzero->defined()) {   // affine int4 (W4A16): wscale / wzero = per-64-block fp32 s, z, [K/64, N]
    TORCH_CHECK(w4 && !bt && wzero->scalar_type() == at::kFloat && wzero->is_contiguous() &&
                    wzero->numel() == wscale->numel(), "gemm4w: wzero fp32 [K/64, N] with wscale, forward only");
    zp = wzero->data_ptr<float>();
  }
  launch_gemm4w(x.data_ptr(), x.stride(0), b.ptr, b.ld, res, y.data_ptr(), sp > 1 ? ws.data_ptr<float>() : nullptr,
                b.scale, zp, M, N, K, sp, bt, bn_used, bm_used, stream());
  return y;
}

// Fused MLP GEMMs (gemm4w.hip EPI 1 / 2).  gemm4w_swiglu: x [M, K], w_gu [2F, K] ([gate | up] rows)
// → (gu [M, 2F], h = silu(gate)·up [M, F]).  gemm4w_dswiglu: dy [M, N_w], w_down [N_w, F], gu [M, 2F]
// → dgu [M, 2F] = SwiGLU-backward(dy·w_down).  wscale: the weight is an NF4 base (g4w_operand).
std::vector<Tensor> gemm4w_swiglu(Tensor x, Tensor w, optional<Tensor> wscale, int64_t F_w4, bool want_gu,
                                  bool want_h) {
  CHECK_BF16(x);
  TORCH_CHECK(x.dim() == 2 && x.stride(1) == 1, "gemm4w_swiglu: x 2-D");
  const bool w4 = wscale && wscale->defined();
  const int64_t M = x.size(0), K = x.size(1), F = w4 ? F_w4 : w.size(0) / 2;
  const G4wB b = g4w_operand(w, wscale, 2 * F, K);
  TORCH_CHECK(F % 16 == 0 && gemm4w_ok(M, 2 * F, K, x.stride(0), K, false, w4) &&
                  (w4 || w.is_contiguous()) && reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0,
              "gemm4w_swiglu: unsupported shape / alignment");
  int bn = 0, bm = 0;
  gemm4w_plan(M, 2 * F, K, false, 0, 1, &bn, 0, &bm, w4);
  // an output the caller does not want is neither allocated nor stored (an undefined tensor is returned)
  Tensor gu, h;
  if (want_gu) gu = at::empty({M, 2 * F}, x.options());
  if (want_h) h = at::empty({M, F}, x.options());
  launch_gemm4w_swiglu(x.data_ptr(), x.stride(0), b.ptr, b.scale, want_gu ? gu.data_ptr() : nullptr,
                       want_h ? h.data_ptr() : nullptr, M, F, K, bn, bm, stream());
  return {gu, h};
}

Tensor gemm4w_dswiglu(Tensor dy, Tensor w, Tensor gu, optional<Tensor> wscale) {
  CHECK_BF16(dy);
  CHECK_BF16(gu);
  CHECK_CONTIG(gu);
  TORCH_CHECK(dy.dim() == 2 && dy.stride(1) == 1, "gemm4w_dswiglu: dy 2-D");
  const bool w4 = wscale && wscale->defined();
  const int64_t M = dy.size(0), Nw = dy.size(1), F = gu.size(1) / 2;
  const G4wB b = g4w_operand(w, wscale, Nw, F);
  TORCH_CHECK(gu.size(0) == M && gu.size(1) == 2 * F && F % 16 == 0 && gemm4w_ok(M, F, Nw, dy.stride(0), F, true, w4) &&
                  (w4 || w.is_contiguous()) && reinterpret_cast<uintptr_t>(dy.data_ptr()) % 16 == 0,
              "gemm4w_dswiglu: unsupported shape / alignment");
  int bn = 0, bm = 0;
  gemm4w_plan(M, F, Nw, true, 0, 1, &bn, 0, &bm, w4);
  auto dgu = at::empty({M, 2 * F}, dy.options());
  launch_gemm4w_dswiglu(dy.data_ptr(), dy.stride(0), b.ptr, b.scale, gu.data_ptr(), dgu.data_ptr(), M, F, Nw, bn, bm,
                        stream());
  return dgu;
}

// y = x·Wᵀ (+ residual) + Σ_b xa[:, kofs_b : kofs_b + r_b]·B_bᵀ into columns [c0_b, c0_b + n_b): the LoRA
// branches of a fused projection as extra MFMA K-steps of the base GEMM (gemm4w.hip LORA epilogue).
// xa bf16 [M, 32·nks] (zero outside the branches' slots), B_b bf16 [n_b, r_b] (r_b, kofs_b multiples of
// 8, up to 4 branches); bts[b] (optional) receives B_bᵀ [r_b, n_b].  w / wscale / n_w4 as gemm4w.
Tensor gemm4w_lora(Tensor x, Tensor w, optional<Tensor> wscale, int64_t n_w4, optional<Tensor> residual, Tensor xa,
                   std::vector<Tensor> bs, std::vector<int64_t> c0s, std::vector<int64_t> kofs,
                   std::vector<optional<Tensor>> bts) {
  CHECK_BF16(x);
  CHECK_BF16(xa);
  TORCH_CHECK(x.dim() == 2 && x.stride(1) == 1, "gemm4w_lora: x 2-D");
  const bool w4 = wscale && wscale->defined();
  const int64_t M = x.size(0), K = x.size(1);
  const int64_t N = w4 ? n_w4 : w.size(0);
  const G4wB b = g4w_operand(w, wscale, N, K);
  TORCH_CHECK(gemm4w_ok(M, N, K, x.stride(0), b.ld, false, w4) && reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0,
              "gemm4w_lora: unsupported shape / strides");
  const int nbr = (int)bs.size();
  TORCH_CHECK(nbr >= 1 && nbr <= 4 && (int)c0s.size() == nbr && (int)kofs.size() == nbr && (int)bts.size() == nbr,
              "gemm4w_lora: 1..4 branches");
  TORCH_CHECK(xa.dim() == 2 && xa.size(0) == M && xa.stride(1) == 1 && xa.size(1) % 32 == 0 && xa.size(1) <= 128 &&
                  xa.stride(0) % 8 == 0 && reinterpret_cast<uintptr_t>(xa.data_ptr()) % 16 == 0,
              "gemm4w_lora: xa bf16 [M, 32·nks], 16-B aligned rows");
  LoraEpi lx{};
  lx.xa = xa.data_ptr();
  lx.ldxa = (int)xa.stride(0);
  lx.nks = (int)(xa.size(1) / 32);
  lx.nbr = nbr;
  for (int i = 0; i < nbr; ++i) {
    const Tensor& bb = bs[i];
    CHECK_BF16(bb);
    CHECK_CONTIG(bb);
    const int64_t n = bb.size(0), r = bb.size(1);
    TORCH_CHECK(r % 8 == 0 && kofs[i] % 8 == 0 && kofs[i] + r <= xa.size(1) && c0s[i] >= 0 && c0s[i] + n <= N &&
                    reinterpret_cast<uintptr_t>(bb.data_ptr()) % 16 == 0,
                "gemm4w_lora: branch ", i, ": r, kofs multiples of 8 inside xa, columns inside N");
    lx.b[i] = bb.data_ptr();
    lx.c0[i] = (int)c0s[i];
    lx.n[i] = (int)n;
    lx.r[i] = (int)r;
    lx.kofs[i] = (int)kofs[i];
    if (bts[i] && bts[i]->defined()) {
      TORCH_CHECK(bts[i]->scalar_type() == at::kBFloat16 && bts[i]->is_contiguous() && bts[i]->size(0) == r &&
                      bts[i]->size(1) == n, "gemm4w_lora: bt [r, n] bf16");
      lx.bt[i] = bts[i]->data_ptr();
    }
  }
  const void* res = nullptr;
  if (residual && residual->defined()) {
    CHECK_BF16(*residual);
    TORCH_CHECK(residual->is_contiguous() && residual->size(0) == M && residual->size(1) == N, "gemm4w_lora: residual");
    res = residual->data_ptr();
  }
  int bn = 0, bm = 0;
  gemm4w_plan(M, N, K, false, 0, 1, &bn, 0, &bm, w4);
  auto y = at::empty({M, N}, x.options());
  launch_gemm4w_lora(x.data_ptr(), x.stride(0), b.ptr, b.ld, b.scale, res, y.data_ptr(), lx, M, N, K, bn, bm, stream());
  return y;
}

// dX = dY·W + Σ_b D_b(ds_b · g_b·A_b) for up to two dropout adapters of the projection (the LoRA input
// gradient added in the gemm4w dX epilogue: no lora_dx2 matrix, no C read).  g_b fp32 [M, r_b] (row stride
// >= r_b), A_b bf16 [r_b, N] (r_b <= 32), masks uint8 [2, M, N/8] keep bits (None: no dropout), ds_b = 1/(1-p_b).
Tensor gemm4w_loradx(Tensor dy, Tensor w, optional<Tensor> wscale, int64_t n_w4, std::vector<Tensor> gs,
                     std::vector<Tensor> as, optional<Tensor> masks, std::vector<double> ps, int64_t bn_req,
                     int64_t bm_req) {
  CHECK_BF16(dy);
  TORCH_CHECK(dy.dim() == 2 && dy.stride(1) == 1, "gemm4w_loradx: dy 2-D");
  const bool w4 = wscale && wscale->defined();
  const int64_t M = dy.size(0), K = dy.size(1);
  const int64_t N = w4 ? n_w4 : w.size(1);
  const G4wB b = g4w_operand(w, wscale, K, N);
  TORCH_CHECK(gemm4w_ok(M, N, K, dy.stride(0), b.ld, true, w4) && reinterpret_cast<uintptr_t>(dy.data_ptr()) % 16 == 0,
              "gemm4w_loradx: unsupported shape / strides");
  const int nbr = (int)gs.size();
  TORCH_CHECK(nbr >= 1 && nbr <= 2 && (int)as.size() == nbr && (int)ps.size() == nbr, "gemm4w_loradx: 1..2 branches");
  TORCH_CHECK(N % 128 == 0, "gemm4w_loradx: N % 128 (16-B keep-bit runs)");
  LoraDx ld{};
  ld.nbr = nbr;
  for (int i = 0; i < nbr; ++i) {
    const Tensor& g = gs[i];
    const Tensor& a = as[i];
    TORCH_CHECK(g.scalar_type() == at::kFloat && g.dim() == 2 && g.size(0) == M && g.stride(1) == 1 &&
                    g.size(1) <= 32 && g.size(1) % 8 == 0 && (i == 0 || g.stride(0) == gs[0].stride(0)) &&
                    reinterpret_cast<uintptr_t>(g.data_ptr()) % 16 == 0 && g.stride(0) % 4 == 0,
                "gemm4w_loradx: g fp32 [M, r], r a multiple of 8 up to 32, 16-B aligned rows");
    CHECK_BF16(a);
    CHECK_CONTIG(a);
    TORCH_CHECK(a.size(0) == g.size(1) && a.size(1) == N && reinterpret_cast<uintptr_t>(a.data_ptr()) % 16 == 0,
                "gemm4w_loradx: A [r, N]");
    ld.g[i] = g.data_ptr<float>();
    ld.ldg = (int)g.stride(0);
    ld.a[i] = a.data_ptr();
    ld.r[i] = (int)a.size(0);
    ld.ds[i] = (float)(1.0 / (1.0 - ps[i]));
  }
  // the kernel's prologue always loads the keep bits (a branch without dropout passes an all-ones plane)
  TORCH_CHECK(masks && masks->defined(), "gemm4w_loradx: keep bits required");
  {
    TORCH_CHECK(masks->scalar_type() == at::kByte && masks->is_contiguous() && masks->numel() >= nbr * M * (N / 8) &&
                    masks->numel() % (M * (N / 8)) == 0, "gemm4w_loradx: keep bits uint8 [P >= nbr, M, N/8]");
    for (int i = 0; i < nbr; ++i) ld.keep[i] = masks->data_ptr<uint8_t>() + (size_t)i * M * (N / 8);
  }
  int bn = 0, bm = 0;
  TORCH_CHECK((bn_req == 0 || bn_req == 128 || bn_req == 256) && (bm_req == 0 || bm_req == 128 || bm_req == 256),
              "gemm4w_loradx: bn / bm 0 (plan), 128 or 256");
  // the LoRA dX kernel is instantiated for 128- and 256-wide tiles only: the plan must not return 192
  gemm4w_plan(M, N, K, true, bn_req ? (int)bn_req : -1, 1, &bn, (int)bm_req, &bm, w4);
  TORCH_CHECK(bn == 128 || bn == 256, "gemm4w_loradx: planned tile width ", bn, " has no kernel");
  auto dx = at::empty({M, N}, dy.options());
  launch_gemm4w_loradx(dy.data_ptr(), dy.stride(0), b.ptr, b.ld, b.scale, nullptr, dx.data_ptr(), ld, M, N, K, bn, bm,
                       stream());
  return dx;
}

// bnb-layout NF4 codes [R, C/2] → the g4w tile layout gemm4w reads (gemm4w.hip pack_g4w_k)
Tensor g4w_pack(Tensor codes, int64_t R, int64_t C) {
  CHECK_CONTIG(codes);
  TORCH_CHECK(codes.scalar_type() == at::kByte && codes.numel() * 2 == R * C && R % 64 == 0 && C % 64 == 0,
              "g4w_pack: uint8 codes [R, C/2], R and C multiples of 64");
  auto out = at::empty({R * C / 2}, codes.options());
  launch_pack_g4w(codes.data_ptr<uint8_t>(), out.data_ptr(), (int)R, (int)C, stream());
  return out;
}

// Multi-adapter LoRA (mlora.hip): y[:, c0:c0+N] += per-row s_a·(x·A_aᵀ)·B_aᵀ, a = ids[row] (0 = base).
// x [T, K] bf16, A_all [R, K], B_all [N, R] bf16, ids [>= T] int64, seg int32 [n_adapters + 1, 3] =
// {offset, rank, float bits of the scale}; ranks / offsets multiples of 8, ranks <= 64.
void mlora_apply(Tensor x, Tensor A, Tensor B, Tensor ids, Tensor seg, Tensor y, int64_t c0) {
  CHECK_BF16(x); CHECK_BF16(A); CHECK_BF16(B); CHECK_BF16(y);
  CHECK_CONTIG(A); CHECK_CONTIG(B); CHECK_CONTIG(seg);
  TORCH_CHECK(x.dim() == 2 && x.stride(1) == 1 && y.dim() == 2 && y.stride(1) == 1, "mlora_apply: 2-D rows");
  const int64_t T = x.size(0), K = x.size(1), R = A.size(0), N = B.size(0);
  TORCH_CHECK(A.size(1) == K && B.size(1) == R && y.size(0) == T && c0 >= 0 && c0 + N <= y.size(1) && K % 8 == 0 &&
                  N % 8 == 0 && R % 8 == 0 && x.stride(0) % 8 == 0 && y.stride(0) % 8 == 0 && c0 % 8 == 0,
              "mlora_apply: shapes");
  TORCH_CHECK(ids.scalar_type() == at::kLong && ids.numel() >= T && ids.is_contiguous(), "mlora_apply: ids int64");
  TORCH_CHECK(seg.scalar_type() == at::kInt && seg.dim() == 2 && seg.size(1) == 3, "mlora_apply: seg [n, 3] int32");
  launch_mlora_apply(x.data_ptr(), x.stride(0), A.data_ptr(), B.data_ptr(), ids.data_ptr<int64_t>(), seg.data_ptr(),
                     (int)seg.size(0), y.data_ptr(), y.stride(0), (int)c0, (int)T, (int)K, (int)N, (int)R, stream());
}

// ------------------------------------------------------------------ attention
static const int* int_ptr(const optional<Tensor>& t, Tensor& keep) {
  if (!t || !t->defined()) return nullptr;
  keep = t->to(at::kInt).contiguous();
  return keep.data_ptr<int>();
}

// host-side operand checks for the attention kernels: 16-B vector loads of head rows
static void attn_check(const Tensor& t, int64_t rows, int64_t heads, int64_t d, const char* name) {
  CHECK_BF16(t);
  TORCH_CHECK(t.dim() == 2 && t.stride(-1) == 1, "attn: ", name, " must be 2-D with unit inner stride");
  TORCH_CHECK(t.stride(0) % 8 == 0 && reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0, "attn: ", name,
              " rows must be 16-byte aligned");
  TORCH_CHECK(t.size(0) >= rows && t.size(1) >= heads * d, "attn: ", name, " too small for the launch shape");
  TORCH_CHECK(d != 128 || t.stride(0) % 128 == 0, "attn: ", name,
              " row stride must be a multiple of 128 elements at head_dim 128 (LDS-DMA rows)");
}

// General forward: Sq queries per batch row (absolute positions q_offs[b] + i) over Skv keys stored
// kv_rows rows apart per batch (a KV cache), optional per-batch key lengths.
std::vector<Tensor> attn_fwd_ext(Tensor q, Tensor k, Tensor v, optional<Tensor> kv_lens, optional<Tensor> q_offs,
                                 int64_t B, int64_t Sq, int64_t Skv, int64_t kv_rows, int64_t hq, int64_t hkv,
                                 int64_t d, bool causal, double scale, double p_drop, int64_t seed) {
  TORCH_CHECK(p_drop >= 0.0 && p_drop < 1.0, "attn: dropout probability in [0, 1)");
  TORCH_CHECK(d == 32 || d == 64 || d == 96 || d == 128, "attn: head_dim in {32, 64, 96, 128}");
  TORCH_CHECK(hkv > 0 && hq % hkv == 0, "attn: GQA group");
  TORCH_CHECK(Sq > 0 && Skv > 0 && kv_rows >= Skv, "attn: shape");
  attn_check(q, B * Sq, hq, d, "q");
  attn_check(k, (B - 1) * kv_rows + Skv, hkv, d, "k");
  attn_check(v, (B - 1) * kv_rows + Skv, hkv, d, "v");
  auto o = at::empty({B * Sq, hq * d}, q.options());
  auto lse = at::empty({B, hq, Sq}, q.options().dtype(at::kFloat));
  Tensor k1, k2;
  const int* kl = int_ptr(kv_lens, k1);
  const int* qo = int_ptr(q_offs, k2);
  launch_attn_fwd(q.data_ptr(), k.data_ptr(), v.data_ptr(), q.stride(0), k.stride(0), v.stride(0), kl, qo,
                  o.data_ptr(), lse.data_ptr<float>(), B, Sq, Skv, kv_rows, hq, hkv, d, causal, scale, p_drop,
                  (uint64_t)seed, stream());
  return {o, lse};
}

std::vector<Tensor> attn_fwd(Tensor q, Tensor k, Tensor v, optional<Tensor> kv_lens, int64_t B, int64_t S, int64_t hq,
                             int64_t hkv, int64_t d, bool causal, double scale) {
  return attn_fwd_ext(q, k, v, kv_lens, c10::nullopt, B, S, S, S, hq, hkv, d, causal, scale, 0.0, 0);
}

std::vector<Tensor> attn_bwd(Tensor dout, Tensor q, Tensor k, Tensor v, Tensor o, Tensor lse,
                             optional<Tensor> kv_lens, int64_t B, int64_t S, int64_t hq, int64_t hkv, int64_t d,
                             bool causal, double scale, double p_drop, int64_t seed) {
  auto dq = at::empty({B * S, hq * d}, q.options());
  auto dk = at::empty({B * S, hkv * d}, q.options());
  auto dv = at::empty({B * S, hkv * d}, q.options());
  TORCH_CHECK(d == 32 || d == 64 || d == 96 || d == 128, "attn_bwd: head_dim in {32, 64, 96, 128}");
  attn_check(q, B * S, hq, d, "q");
  attn_check(k, B * S, hkv, d, "k");
  attn_check(v, B * S, hkv, d, "v");
  attn_check(o, B * S, hq, d, "o");
  attn_check(dout, B * S, hq, d, "dout");
  TORCH_CHECK(dout.stride(0) == hq * d && o.stride(0) == hq * d, "attn_bwd: o / dout must be dense [T, hq*d]");
  auto delta = at::empty({B, hq, S}, q.options().dtype(at::kFloat));
  Tensor ws;   // split causal dK/dV blocks: fp32 partial planes [2 parts][dK | dV][T][hkv·d]
  if (attn_dkv_nsplit(B, S, hkv, causal) > 0) ws = at::empty({4, B * S, hkv * d}, q.options().dtype(at::kFloat));
  const int* kl = nullptr;
  Tensor klc;
  if (kv_lens && kv_lens->defined()) {
    klc = kv_lens->to(at::kInt).contiguous();
    kl = klc.data_ptr<int>();
  }
  launch_attn_bwd(dout.data_ptr(), q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), lse.data_ptr<float>(), kl,
                  q.stride(0), k.stride(0), v.stride(0), dq.data_ptr(), dk.data_ptr(), dv.data_ptr(),
                  delta.data_ptr<float>(), B, S, hq, hkv, d, causal, scale, p_drop, (uint64_t)seed,
                  ws.defined() ? ws.data_ptr<float>() : nullptr, stream());
  return {dq, dk, dv};
}

// ------------------------------------------------------------------ fused LoRA branch kernels
// out = scale·D(x)·Wᵀ over x[:, c0:c0+K] (row stride = x.stride(0)); writes bf16 into outb (a column
// slice view, any row stride) and/or returns fp32 [M, r].
Tensor lora_proj(Tensor x, int64_t c0, int64_t K, Tensor w, optional<Tensor> outb, bool want_f32, double p,
                 int64_t key, double scale) {
  CHECK_BF16(x);
  CHECK_BF16(w);
  TORCH_CHECK(x.dim() == 2 && x.stride(1) == 1 && x.stride(0) % 8 == 0 && c0 % 8 == 0, "lora_proj: x layout");
  TORCH_CHECK(w.is_contiguous() && w.size(1) == K && w.size(0) <= 16 && K % 32 == 0, "lora_proj: w [r<=16, K%32]");
  const int M = x.size(0), r = w.size(0);
  Tensor of;
  if (want_f32) of = at::empty({M, r}, x.options().dtype(at::kFloat));
  void* ob = nullptr;
  int ldob = 0;
  if (outb) {
    TORCH_CHECK(outb->scalar_type() == at::kBFloat16 && outb->stride(1) == 1 && outb->size(0) == M &&
                    outb->size(1) == r, "lora_proj: outb");
    ob = outb->data_ptr();
    ldob = outb->stride(0);
  }
  TORCH_CHECK(ob || want_f32, "lora_proj: no output");
  launch_lora_proj((const char*)x.data_ptr() + c0 * 2, x.stride(0), w.data_ptr(), r, K,
                   want_f32 ? of.data_ptr<float>() : nullptr, r, ob, ldob, M, (uint64_t)key, (float)p, (float)scale,
                   (size_t)x.stride(0), stream());
  return want_f32 ? of : Tensor();
}

// out (fp32, 2-D, [r, K] or its transpose view [K, r]) += gᵀ·D(x[:, c0:c0+K]); with dx: dx += D(g·w)
// two LoRA branches sharing x (q_proj + v_proj): A0 [r0, K], A1 [r1, K] bf16, r0 + r1 <= 16
static uint8_t* keep_bits_ptr(const optional<Tensor>& m, int64_t M, int64_t K, const char* who) {
  if (!m || !m->defined()) return nullptr;
  TORCH_CHECK(m->scalar_type() == at::kByte && m->is_contiguous() && m->numel() == 2 * M * (K / 8),
              who, ": keep bits uint8 [2, M, K/8] contiguous");
  return m->data_ptr<uint8_t>();
}

// masks (optional, uint8 [2, M, K/8]): the two branches' dropout keep bits, written for the backward (lora_acc_quad, gemm4w_loradx, lora_dx2)
Tensor lora_proj2(Tensor x, Tensor a0, Tensor a1, optional<Tensor> outb, bool want_f32, double p0, int64_t key0,
                  double scale0, double p1, int64_t key1, double scale1, optional<Tensor> masks) {
  CHECK_BF16(x);
  CHECK_BF16(a0);
  CHECK_BF16(a1);
  const int64_t K = x.size(1);
  TORCH_CHECK(x.dim() == 2 && x.stride(1) == 1 && x.stride(0) % 8 == 0, "lora_proj2: x layout");
  TORCH_CHECK(a0.is_contiguous() && a1.is_contiguous() && a0.size(1) == K && a1.size(1) == K &&
                  a0.size(0) + a1.size(0) <= 16 && K % 32 == 0, "lora_proj2: A_i [r_i, K], r0 + r1 <= 16");
  const int M = x.size(0), r0 = a0.size(0), r = r0 + a1.size(0);
  Tensor of;
  if (want_f32) of = at::empty({M, r}, x.options().dtype(at::kFloat));
  void* ob = nullptr;
  int ldob = 0;
  if (outb) {
    TORCH_CHECK(outb->scalar_type() == at::kBFloat16 && outb->stride(1) == 1 && outb->size(0) == M &&
                    outb->size(1) == r, "lora_proj2: outb");
    ob = outb->data_ptr();
    ldob = outb->stride(0);
  }
  TORCH_CHECK(ob || want_f32, "lora_proj2: no output");
  const int wsf = lora_proj2_ws_floats(M, K);
  Tensor ws;
  if (wsf) ws = at::empty({wsf}, x.options().dtype(at::kFloat));
  launch_lora_proj2(x.data_ptr(), x.stride(0), a0.data_ptr(), a1.data_ptr(), r0, r, K, want_f32 ? of.data_ptr<float>() : nullptr, r,
                    ob, ldob, M, (uint64_t)key0, (float)p0, (float)scale0, (uint64_t)key1, (float)p1, (float)scale1,
                    (size_t)x.stride(0), keep_bits_ptr(masks, M, K, "lora_proj2"),
                    wsf ? ws.data_ptr<float>() : nullptr, stream());
  return want_f32 ? of : Tensor();
}

// y[:, c0_i : c0_i + n_i] += xa_i · B_iᵀ in place (xa_i fp32 [M, r_i], scale folded in; B_i bf16 [n_i, r_i])
void lora_apply(Tensor y, std::vector<Tensor> xas, std::vector<Tensor> bs, std::vector<int64_t> c0s,
                std::vector<Tensor> bts) {
  CHECK_CUDA(y);
  CHECK_BF16(y);
  const int nb = (int)xas.size();
  TORCH_CHECK(nb >= 1 && nb <= 4 && (int)bs.size() == nb && (int)c0s.size() == nb, "lora_apply: 1..4 branches");
  TORCH_CHECK(y.dim() == 2 && y.stride(1) == 1 && y.stride(0) % 8 == 0 &&
                  reinterpret_cast<uintptr_t>(y.data_ptr()) % 16 == 0, "lora_apply: y [M, N] 16-B aligned rows");
  const int M = y.size(0);
  std::vector<const float*> xp(nb);
  std::vector<const void*> bp(nb);
  std::vector<void*> btp(nb, nullptr);
  TORCH_CHECK(bts.empty() || (int)bts.size() == nb, "lora_apply: one Bt output per branch");
  std::vector<int> ld(nb), c0(nb), n(nb), r(nb);
  for (int i = 0; i < nb; ++i) {
    TORCH_CHECK(xas[i].scalar_type() == at::kFloat && xas[i].dim() == 2 && xas[i].stride(1) == 1 &&
                    xas[i].size(0) == M && xas[i].size(1) <= 16, "lora_apply: xa fp32 [M, r<=16]");
    TORCH_CHECK(bs[i].scalar_type() == at::kBFloat16 && bs[i].is_contiguous() && bs[i].size(1) == xas[i].size(1),
                "lora_apply: B bf16 [n, r] contiguous");
    TORCH_CHECK(c0s[i] % 8 == 0 && bs[i].size(0) % 8 == 0 && c0s[i] + bs[i].size(0) <= y.size(1),
                "lora_apply: column block");
    xp[i] = xas[i].data_ptr<float>();
    ld[i] = xas[i].stride(0);
    bp[i] = bs[i].data_ptr();
    if (!bts.empty()) {
      TORCH_CHECK(bts[i].scalar_type() == at::kBFloat16 && bts[i].is_contiguous() && bts[i].size(0) == bs[i].size(1) &&
                      bts[i].size(1) == bs[i].size(0) && reinterpret_cast<uintptr_t>(bts[i].data_ptr()) % 16 == 0,
                  "lora_apply: Bt bf16 [r, n] contiguous, 16-B aligned");
      btp[i] = bts[i].data_ptr();
    }
    c0[i] = c0s[i];
    n[i] = bs[i].size(0);
    r[i] = bs[i].size(1);
  }
  launch_lora_apply(y.data_ptr(), y.stride(0), M, nb, xp.data(), ld.data(), bp.data(), bts.empty() ? nullptr : btp.data(),
                    c0.data(), n.data(), r.data(), stream());
}

void lora_acc(Tensor g, Tensor x, int64_t c0, int64_t K, Tensor out, bool out_transposed, optional<Tensor> dx,
              optional<Tensor> w, double p, int64_t key, bool deterministic) {
  TORCH_CHECK(g.scalar_type() == at::kFloat && g.dim() == 2 && g.stride(1) == 1 && g.size(1) <= 16, "lora_acc: g");
  CHECK_BF16(x);
  TORCH_CHECK(x.stride(1) == 1 && x.stride(0) % 8 == 0 && c0 % 8 == 0 && K % 8 == 0, "lora_acc: x layout");
  TORCH_CHECK(out.scalar_type() == at::kFloat && out.dim() == 2, "lora_acc: out fp32 2-D");
  const int M = x.size(0), r = g.size(1);
  int64_t sj, sk;
  if (out_transposed) {
    TORCH_CHECK(out.size(0) == K && out.size(1) == r, "lora_acc: out [K, r]");
    sj = out.stride(1);
    sk = out.stride(0);
  } else {
    TORCH_CHECK(out.size(0) == r && out.size(1) == K, "lora_acc: out [r, K]");
    sj = out.stride(0);
    sk = out.stride(1);
  }
  void* dxp = nullptr;
  int lddx = 0;
  if (dx) {
    TORCH_CHECK(w.has_value() && w->is_contiguous() && w->size(0) == r && w->size(1) == K, "lora_acc: w");
    TORCH_CHECK(dx->scalar_type() == at::kBFloat16 && dx->stride(1) == 1 && dx->size(0) == M && dx->size(1) == K,
                "lora_acc: dx");
    dxp = dx->data_ptr();
    lddx = dx->stride(0);
  }
  Tensor part;
  if (deterministic) part = at::empty({lora_acc_chunks(M, K), r, K}, g.options());
  launch_lora_acc(g.data_ptr<float>(), g.stride(0), r, (const char*)x.data_ptr() + c0 * 2, x.stride(0), dxp, lddx,
                  dx ? w->data_ptr() : nullptr, K, out.data_ptr<float>(), sj, sk,
                  deterministic ? part.data_ptr<float>() : nullptr, M, (uint64_t)key, (float)p,
                  (size_t)x.stride(0), stream());
  if (deterministic) {
    Tensor s = part.sum(0);
    if (out_transposed) out.add_(s.t());
    else out.add_(s);
  }
}

// backward of a q_proj + v_proj pair, one launch per product:
//   g_i = s_i · dy[:, c0_i : c0_i + n_i] · B_i   (B_i passed as Bᵀ [r, n_i] bf16) -> fp32 [M, r]
std::vector<Tensor> lora_proj_pair(Tensor dy, int64_t c0a, Tensor bta, double sa, int64_t c0b, Tensor btb, double sb) {
  CHECK_BF16(dy);
  CHECK_BF16(bta);
  CHECK_BF16(btb);
  TORCH_CHECK(dy.dim() == 2 && dy.stride(1) == 1 && dy.stride(0) % 8 == 0 && c0a % 8 == 0 && c0b % 8 == 0,
              "lora_proj_pair: dy layout");
  TORCH_CHECK(bta.is_contiguous() && btb.is_contiguous() && bta.size(0) == btb.size(0) && bta.size(0) <= 16 &&
                  bta.size(1) % 512 == 0 && btb.size(1) % 512 == 0 && c0a + bta.size(1) <= dy.size(1) &&
                  c0b + btb.size(1) <= dy.size(1),
              "lora_proj_pair: Bt_i [r, n_i % 512] within dy");
  const int M = dy.size(0), r = bta.size(0);
  Tensor ga = at::empty({M, r}, dy.options().dtype(at::kFloat)), gb = at::empty({M, r}, dy.options().dtype(at::kFloat));
  const char* base = (const char*)dy.data_ptr();
  launch_lora_proj_pair(base + c0a * 2, base + c0b * 2, dy.stride(0), bta.data_ptr(), btb.data_ptr(), r, bta.size(1),
                        btb.size(1), ga.data_ptr<float>(), gb.data_ptr<float>(), (float)sa, (float)sb, M, stream());
  return {ga, gb};
}

//   dB_i [n_i, r] += (dy[:, c0_i : c0_i + n_i])ᵀ · xa_i   (xa_i fp32 [M, r], one row stride for both)
void lora_acc_pair(Tensor xa, Tensor xb, Tensor dy, int64_t c0a, Tensor outa, int64_t c0b, Tensor outb) {
  for (const Tensor* g : {&xa, &xb})
    TORCH_CHECK(g->scalar_type() == at::kFloat && g->dim() == 2 && g->stride(1) == 1 && g->size(1) <= 8 &&
                    g->stride(0) % 4 == 0 && reinterpret_cast<uintptr_t>(g->data_ptr()) % 16 == 0,
                "lora_acc_pair: xa fp32 [M, r<=8], 16-B aligned rows");
  TORCH_CHECK(xa.stride(0) == xb.stride(0) && xa.size(1) == xb.size(1), "lora_acc_pair: one layout for both xa");
  CHECK_BF16(dy);
  TORCH_CHECK(dy.stride(1) == 1 && dy.stride(0) % 8 == 0 && c0a % 8 == 0 && c0b % 8 == 0, "lora_acc_pair: dy layout");
  const int M = dy.size(0), r = xa.size(1);
  for (const Tensor* o : {&outa, &outb})
    TORCH_CHECK(o->scalar_type() == at::kFloat && o->is_contiguous() && o->dim() == 2 && o->size(1) == r &&
                    o->size(0) % 128 == 0, "lora_acc_pair: out fp32 [n_i % 128, r] contiguous");
  TORCH_CHECK(xa.size(0) == M && xb.size(0) == M && c0a + outa.size(0) <= dy.size(1) &&
                  c0b + outb.size(0) <= dy.size(1), "lora_acc_pair: shapes");
  const char* base = (const char*)dy.data_ptr();
  launch_lora_acc_pair(xa.data_ptr<float>(), xb.data_ptr<float>(), xa.stride(0), r, base + c0a * 2, base + c0b * 2,
                       dy.stride(0), outa.size(0), outb.size(0), outa.data_ptr<float>(), outb.data_ptr<float>(), M,
                       stream());
}

//   dA_i [r, K] += D_i(x)ᵀ-weighted G_i (keep bits from lora_proj2, masks [2, M, K/8])
void lora_dA_pair(Tensor g0, Tensor g1, Tensor x, Tensor out0, Tensor out1, Tensor masks, double p0, double p1) {
  for (const Tensor* g : {&g0, &g1})
    TORCH_CHECK(g->scalar_type() == at::kFloat && g->dim() == 2 && g->stride(1) == 1 && g->size(1) <= 8 &&
                    g->stride(0) % 4 == 0 && reinterpret_cast<uintptr_t>(g->data_ptr()) % 16 == 0,
                "lora_dA_pair: g fp32 [M, r<=8], 16-B aligned rows");
  TORCH_CHECK(g0.stride(0) == g1.stride(0) && g0.size(1) == g1.size(1), "lora_dA_pair: one layout for both g");
  CHECK_BF16(x);
  const int M = x.size(0), K = x.size(1), r = g0.size(1);
  TORCH_CHECK(x.stride(1) == 1 && x.stride(0) % 8 == 0 && K % 128 == 0, "lora_dA_pair: x layout");
  for (const Tensor* o : {&out0, &out1})
    TORCH_CHECK(o->scalar_type() == at::kFloat && o->dim() == 2 && o->size(0) == r && o->size(1) == K,
                "lora_dA_pair: out fp32 [r, K]");
  const uint8_t* kb = keep_bits_ptr(masks, M, K, "lora_dA_pair");
  TORCH_CHECK(kb, "lora_dA_pair: keep bits required");
  const size_t plane = (size_t)M * (K / 8);
  launch_lora_dA_pair(g0.data_ptr<float>(), g1.data_ptr<float>(), g0.stride(0), r, x.data_ptr(), x.stride(0), K,
                      out0.data_ptr<float>(), out1.data_ptr<float>(), out0.stride(0), out0.stride(1), out1.stride(0),
                      out1.stride(1), p0 > 0 ? kb : nullptr, p1 > 0 ? kb + plane : nullptr,
                      p0 > 0 ? (float)(1.0 / (1.0 - p0)) : 1.f, p1 > 0 ? (float)(1.0 / (1.0 - p1)) : 1.f, M, stream());
}

// dB_q, dB_v (as lora_acc_pair) and dA_q, dA_v (as lora_dA_pair) in one launch
void lora_acc_quad(Tensor xa, Tensor xb, Tensor dy, int64_t c0a, Tensor outa, int64_t c0b, Tensor outb, Tensor g0,
                   Tensor g1, Tensor x, Tensor out0, Tensor out1, Tensor masks, double p0, double p1) {
  for (const Tensor* g : {&xa, &xb, &g0, &g1})
    TORCH_CHECK(g->scalar_type() == at::kFloat && g->dim() == 2 && g->stride(1) == 1 && g->size(1) <= 8 &&
                    g->stride(0) % 4 == 0 && reinterpret_cast<uintptr_t>(g->data_ptr()) % 16 == 0,
                "lora_acc_quad: xa / g fp32 [M, r<=8], 16-B aligned rows");
  const int r = xa.size(1);
  TORCH_CHECK(xb.size(1) == r && g0.size(1) == r && g1.size(1) == r, "lora_acc_quad: one rank");
  CHECK_BF16(dy);
  CHECK_BF16(x);
  TORCH_CHECK(dy.stride(1) == 1 && dy.stride(0) % 8 == 0 && c0a % 8 == 0 && c0b % 8 == 0, "lora_acc_quad: dy layout");
  const int M = dy.size(0), K = x.size(1);
  TORCH_CHECK(x.stride(1) == 1 && x.stride(0) % 8 == 0 && K % 128 == 0 && x.size(0) == M, "lora_acc_quad: x layout");
  for (const Tensor* o : {&outa, &outb})
    TORCH_CHECK(o->scalar_type() == at::kFloat && o->is_contiguous() && o->dim() == 2 && o->size(1) == r &&
                    o->size(0) % 128 == 0, "lora_acc_quad: dB fp32 [n_i % 128, r] contiguous");
  for (const Tensor* o : {&out0, &out1})
    TORCH_CHECK(o->scalar_type() == at::kFloat && o->dim() == 2 && o->size(0) == r && o->size(1) == K,
                "lora_acc_quad: dA fp32 [r, K]");
  TORCH_CHECK(xa.size(0) == M && xb.size(0) == M && g0.size(0) == M && g1.size(0) == M &&
                  c0a + outa.size(0) <= dy.size(1) && c0b + outb.size(0) <= dy.size(1), "lora_acc_quad: shapes");
  const uint8_t* kbits = keep_bits_ptr(masks, M, K, "lora_acc_quad");
  TORCH_CHECK(kbits, "lora_acc_quad: keep bits required");
  const size_t plane = (size_t)M * (K / 8);
  const char* base = (const char*)dy.data_ptr();
  const float* G[4] = {xa.data_ptr<float>(), xb.data_ptr<float>(), g0.data_ptr<float>(), g1.data_ptr<float>()};
  const int ldg[4] = {(int)xa.stride(0), (int)xb.stride(0), (int)g0.stride(0), (int)g1.stride(0)};
  const void* X[4] = {base + c0a * 2, base + c0b * 2, x.data_ptr(), x.data_ptr()};
  const int ldx[4] = {(int)dy.stride(0), (int)dy.stride(0), (int)x.stride(0), (int)x.stride(0)};
  const int Ks[4] = {(int)outa.size(0), (int)outb.size(0), K, K};
  float* out[4] = {outa.data_ptr<float>(), outb.data_ptr<float>(), out0.data_ptr<float>(), out1.data_ptr<float>()};
  const int64_t sj[4] = {1, 1, out0.stride(0), out1.stride(0)};
  const int64_t sk[4] = {r, r, out0.stride(1), out1.stride(1)};
  const float ds[4] = {1.f, 1.f, p0 > 0 ? (float)(1.0 / (1.0 - p0)) : 1.f, p1 > 0 ? (float)(1.0 / (1.0 - p1)) : 1.f};
  const uint8_t* kb[4] = {nullptr, nullptr, p0 > 0 ? kbits : nullptr, p1 > 0 ? kbits + plane : nullptr};
  launch_lora_acc_quad(G, ldg, X, ldx, Ks, out, sj, sk, ds, kb, r, M, stream());
}

// ---- 1-4 adapters of one projection (the general multi-adapter path; BASELINE #2's q, k, v and o) ----
static uint8_t* keep_plane(const optional<Tensor>& m, int64_t plane, int64_t M, int64_t K, const char* who) {
  if (!m || !m->defined() || plane < 0) return nullptr;
  TORCH_CHECK(m->scalar_type() == at::kByte && m->is_contiguous() && m->dim() == 3 && m->size(1) == M &&
                  m->size(2) == K / 8 && plane < m->size(0), who, ": keep bits uint8 [P, M, K/8] contiguous");
  return m->data_ptr<uint8_t>() + (size_t)plane * M * (K / 8);
}

// xa_b = s_b·D_b(x)·A_bᵀ for every adapter in one pass over x: fp32 [M, r_b] returned (want_f32), bf16 into
// outbs[b] (column-slice views) when given; masks [nbr, M, K/8] (optional) receives every branch's keep bits.
std::vector<Tensor> lora_proj_m(Tensor x, std::vector<Tensor> as, std::vector<optional<Tensor>> outbs, bool want_f32,
                                std::vector<double> ps, std::vector<int64_t> keys, std::vector<double> scales,
                                optional<Tensor> masks) {
  CHECK_BF16(x);
  const int nbr = (int)as.size();
  TORCH_CHECK(nbr >= 1 && nbr <= 4 && (int)outbs.size() == nbr && (int)ps.size() == nbr && (int)keys.size() == nbr &&
                  (int)scales.size() == nbr, "lora_proj_m: 1..4 branches");
  const int64_t M = x.size(0), K = x.size(1);
  TORCH_CHECK(x.dim() == 2 && x.stride(1) == 1 && x.stride(0) % 8 == 0 && K % 128 == 0 &&
                  reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0, "lora_proj_m: x [M, K % 128], 16-B rows");
  const void* W[4] = {};
  int r[4] = {}, ldof[4] = {}, ldob[4] = {};
  uint64_t key[4] = {};
  float p[4] = {}, sc[4] = {};
  uint8_t* mko[4] = {};
  float* outf[4] = {};
  void* outb[4] = {};
  std::vector<Tensor> res;
  for (int b = 0; b < nbr; ++b) {
    const Tensor& a = as[b];
    CHECK_BF16(a);
    TORCH_CHECK(a.is_contiguous() && a.size(1) == K && a.size(0) <= 16 && reinterpret_cast<uintptr_t>(a.data_ptr()) % 16 == 0,
                "lora_proj_m: A_b [r <= 16, K]");
    W[b] = a.data_ptr();
    r[b] = (int)a.size(0);
    key[b] = (uint64_t)keys[b];
    p[b] = (float)ps[b];
    sc[b] = (float)scales[b];
    mko[b] = keep_plane(masks, masks ? b : -1, M, K, "lora_proj_m");
    if (want_f32) {
      res.push_back(at::empty({M, r[b]}, x.options().dtype(at::kFloat)));
      outf[b] = res.back().data_ptr<float>();
      ldof[b] = r[b];
    }
    if (outbs[b] && outbs[b]->defined()) {
      const Tensor& o = *outbs[b];
      TORCH_CHECK(o.scalar_type() == at::kBFloat16 && o.stride(1) == 1 && o.size(0) == M && o.size(1) == r[b],
                  "lora_proj_m: outb [M, r_b] bf16");
      outb[b] = o.data_ptr();
      ldob[b] = (int)o.stride(0);
    }
    TORCH_CHECK(outf[b] || outb[b], "lora_proj_m: no output for branch ", b);
  }
  if (masks && masks->defined()) TORCH_CHECK(masks->size(0) == nbr, "lora_proj_m: one keep-bit plane per branch");
  Tensor ws = at::empty({lora_proj_m_ws_floats((int)M, (int)K, nbr)}, x.options().dtype(at::kFloat));
  launch_lora_proj_m(x.data_ptr(), (int)x.stride(0), (int)K, (int)M, nbr, W, r, key, p, sc, mko, (size_t)x.stride(0),
                     outf, ldof, outb, ldob, ws.data_ptr<float>(), stream());
  return res;
}

// g_b = s_b·dy[:, c0_b : c0_b + n_b]·B_b for 1-4 adapters (B_b as Bᵀ [r_b, n_b] bf16, n_b % 512) -> fp32 [M, r_b]
std::vector<Tensor> lora_proj_cols(Tensor dy, std::vector<int64_t> c0s, std::vector<Tensor> bts, std::vector<double> scales) {
  CHECK_BF16(dy);
  const int nbr = (int)bts.size();
  TORCH_CHECK(nbr >= 1 && nbr <= 4 && (int)c0s.size() == nbr && (int)scales.size() == nbr, "lora_proj_cols: 1..4 branches");
  TORCH_CHECK(dy.dim() == 2 && dy.stride(1) == 1 && dy.stride(0) % 8 == 0, "lora_proj_cols: dy layout");
  const int M = dy.size(0);
  const char* base = (const char*)dy.data_ptr();
  const void* X[4] = {};
  const void* W[4] = {};
  int r[4] = {}, K[4] = {};
  float* out[4] = {};
  float sc[4] = {};
  std::vector<Tensor> res;
  for (int b = 0; b < nbr; ++b) {
    const Tensor& bt = bts[b];
    CHECK_BF16(bt);
    TORCH_CHECK(bt.is_contiguous() && bt.size(0) <= 16 && bt.size(1) % 512 == 0 && c0s[b] % 8 == 0 &&
                    c0s[b] + bt.size(1) <= dy.size(1), "lora_proj_cols: Bt_b [r <= 16, n_b % 512] within dy");
    X[b] = base + c0s[b] * 2;
    W[b] = bt.data_ptr();
    r[b] = (int)bt.size(0);
    K[b] = (int)bt.size(1);
    res.push_back(at::empty({M, r[b]}, dy.options().dtype(at::kFloat)));
    out[b] = res.back().data_ptr<float>();
    sc[b] = (float)scales[b];
  }
  launch_lora_proj_cols(nbr, X, (int)dy.stride(0), W, r, K, out, sc, M, stream());
  return res;
}

// up to 8 weight-gradient products in one launch: out_i += G_iᵀ·D_i(X_i[:, c0_i : c0_i + k_i]) (fp32 atomics);
// out_t[i]: out_i is [k_i, r_i] (a dB) rather than [r_i, k_i] (a dA); planes[i] >= 0 selects keep bits of masks
// (its K = k_i), ps[i] the matching dropout rate.
void lora_acc_jobs(std::vector<Tensor> gs, std::vector<Tensor> xs, std::vector<int64_t> c0s, std::vector<int64_t> ks,
                   std::vector<Tensor> outs, std::vector<bool> out_t, optional<Tensor> masks, std::vector<int64_t> planes,
                   std::vector<double> ps) {
  const int nj = (int)gs.size();
  TORCH_CHECK(nj >= 1 && nj <= 8 && (int)xs.size() == nj && (int)c0s.size() == nj && (int)ks.size() == nj &&
                  (int)outs.size() == nj && (int)out_t.size() == nj && (int)planes.size() == nj && (int)ps.size() == nj,
              "lora_acc_jobs: 1..8 jobs");
  const int M = gs[0].size(0);
  const float* G[8] = {};
  const void* X[8] = {};
  float* out[8] = {};
  int ldg[8] = {}, r[8] = {}, ldx[8] = {}, K[8] = {};
  int64_t sj[8] = {}, sk[8] = {};
  float ds[8] = {};
  const uint8_t* kb[8] = {};
  for (int i = 0; i < nj; ++i) {
    const Tensor& g = gs[i];
    const Tensor& x = xs[i];
    const Tensor& o = outs[i];
    TORCH_CHECK(g.scalar_type() == at::kFloat && g.dim() == 2 && g.stride(1) == 1 && g.size(0) == M && g.size(1) <= 16,
                "lora_acc_jobs: G fp32 [M, r <= 16]");
    CHECK_BF16(x);
    TORCH_CHECK(x.dim() == 2 && x.size(0) == M && x.stride(1) == 1 && x.stride(0) % 8 == 0 && c0s[i] % 8 == 0 &&
                    ks[i] % 128 == 0 && c0s[i] + ks[i] <= x.size(1), "lora_acc_jobs: X column block [M, k % 128]");
    const int64_t rr = g.size(1);
    TORCH_CHECK(o.scalar_type() == at::kFloat && o.dim() == 2 &&
                    (out_t[i] ? (o.size(0) == ks[i] && o.size(1) == rr) : (o.size(0) == rr && o.size(1) == ks[i])),
                "lora_acc_jobs: out fp32 [k, r] (out_t) or [r, k]");
    G[i] = g.data_ptr<float>();
    ldg[i] = (int)g.stride(0);
    r[i] = (int)rr;
    X[i] = (const char*)x.data_ptr() + c0s[i] * 2;
    ldx[i] = (int)x.stride(0);
    K[i] = (int)ks[i];
    out[i] = o.data_ptr<float>();
    sj[i] = out_t[i] ? o.stride(1) : o.stride(0);
    sk[i] = out_t[i] ? o.stride(0) : o.stride(1);
    kb[i] = ps[i] > 0 ? keep_plane(masks, planes[i], M, ks[i], "lora_acc_jobs") : nullptr;
    TORCH_CHECK(ps[i] <= 0 || kb[i], "lora_acc_jobs: a dropout job needs its keep bits");
    ds[i] = ps[i] > 0 ? (float)(1.0 / (1.0 - ps[i])) : 1.f;
  }
  launch_lora_acc_jobs(nj, G, ldg, r, X, ldx, K, out, sj, sk, ds, kb, M, stream());
}

// C = Σ_b keep_b·ds_b·(g_b·A_b) bf16 [M, K] for 1-4 adapters (masks [nbr, M, K/8] or None; ps_b = 0: no mask)
Tensor lora_dxc(std::vector<Tensor> gs, std::vector<Tensor> as, optional<Tensor> masks, std::vector<double> ps,
                int64_t rb) {
  const int nbr = (int)gs.size();
  TORCH_CHECK(nbr >= 1 && nbr <= 4 && (int)as.size() == nbr && (int)ps.size() == nbr, "lora_dxc: 1..4 branches");
  const int64_t M = gs[0].size(0), K = as[0].size(1);
  TORCH_CHECK(K % 64 == 0, "lora_dxc: K % 64");
  const float* g[4] = {};
  const void* a[4] = {};
  int ldg[4] = {}, r[4] = {};
  const uint8_t* kb[4] = {};
  float ds[4] = {};
  for (int b = 0; b < nbr; ++b) {
    const Tensor& gg = gs[b];
    const Tensor& aa = as[b];
    TORCH_CHECK(gg.scalar_type() == at::kFloat && gg.dim() == 2 && gg.stride(1) == 1 && gg.size(0) == M &&
                    gg.size(1) <= 16 && gg.size(1) % 4 == 0 && gg.stride(0) % 4 == 0 &&
                    reinterpret_cast<uintptr_t>(gg.data_ptr()) % 16 == 0, "lora_dxc: g fp32 [M, r <= 16, r % 4], 16-B rows");
    CHECK_BF16(aa);
    TORCH_CHECK(aa.is_contiguous() && aa.size(0) == gg.size(1) && aa.size(1) == K &&
                    reinterpret_cast<uintptr_t>(aa.data_ptr()) % 16 == 0, "lora_dxc: A_b [r_b, K]");
    g[b] = gg.data_ptr<float>();
    ldg[b] = (int)gg.stride(0);
    a[b] = aa.data_ptr();
    r[b] = (int)aa.size(0);
    kb[b] = ps[b] > 0 ? keep_plane(masks, b, M, K, "lora_dxc") : nullptr;
    TORCH_CHECK(ps[b] <= 0 || kb[b], "lora_dxc: a dropout branch needs its keep bits");
    ds[b] = ps[b] > 0 ? (float)(1.0 / (1.0 - ps[b])) : 1.f;
  }
  Tensor out = at::empty({M, K}, as[0].options());
  launch_lora_dxc(nbr, g, ldg, a, r, kb, ds, out.data_ptr(), (int)M, (int)K, (int)rb, stream());
  return out;
}

//   dx_lora [M, K] bf16 = Σ_i D_i(G_i·A_i)·ds_i  — the dX GEMM's C matrix
Tensor lora_dx2(Tensor g0, Tensor g1, Tensor a0, Tensor a1, Tensor masks, double p0, double p1) {
  TORCH_CHECK(g0.scalar_type() == at::kFloat && g1.scalar_type() == at::kFloat && g0.stride(0) == g1.stride(0) &&
                  g0.stride(1) == 1 && g1.stride(1) == 1 && g0.stride(0) % 4 == 0 && g0.stride(0) >= 8 &&
                  reinterpret_cast<uintptr_t>(g0.data_ptr()) % 16 == 0 &&
                  reinterpret_cast<uintptr_t>(g1.data_ptr()) % 16 == 0 && g0.size(1) <= 8 && g1.size(1) <= 8,
              "lora_dx2: g fp32 [M, r<=8], one row stride >= 8, 16-B aligned");
  CHECK_BF16(a0);
  CHECK_BF16(a1);
  const int M = g0.size(0), K = a0.size(1);
  TORCH_CHECK(a0.is_contiguous() && a1.is_contiguous() && a1.size(1) == K && a0.size(0) == g0.size(1) &&
                  a1.size(0) == g1.size(1) && K % 8 == 0 && g1.size(0) == M, "lora_dx2: A_i [r_i, K]");
  const uint8_t* kb = keep_bits_ptr(masks, M, K, "lora_dx2");
  TORCH_CHECK(kb, "lora_dx2: keep bits required");
  const size_t plane = (size_t)M * (K / 8);
  Tensor out = at::empty({M, K}, a0.options());
  launch_lora_dx2(g0.data_ptr<float>(), g1.data_ptr<float>(), g0.stride(0), a0.data_ptr(), a1.data_ptr(), a0.size(0),
                  a1.size(0), p0 > 0 ? kb : nullptr, p1 > 0 ? kb + plane : nullptr,
                  p0 > 0 ? (float)(1.0 / (1.0 - p0)) : 1.f, p1 > 0 ? (float)(1.0 / (1.0 - p1)) : 1.f, out.data_ptr(),
                  M, K, stream());
  return out;
}

// ------------------------------------------------------------------ generation (K16, K17)
// q [B, hq*d] bf16; kc/vc [B, Smax, hkv*d] bf16 contiguous; lens [B] int32 (valid keys per row);
// max_len >= max(lens) bounds the split count without a host sync.
Tensor decode_attention(Tensor q, Tensor kc, Tensor vc, Tensor lens, int64_t hq, int64_t hkv, int64_t d,
                        int64_t max_len, double scale) {
  CHECK_CUDA(q);
  CHECK_BF16(q);
  CHECK_BF16(kc);
  CHECK_BF16(vc);
  CHECK_CONTIG(q);
  CHECK_CONTIG(kc);
  CHECK_CONTIG(vc);
  TORCH_CHECK(lens.scalar_type() == at::kInt && lens.is_contiguous(), "lens: int32");
  TORCH_CHECK(d == 64 || d == 128, "decode_attention: head_dim 64 or 128");
  const int64_t G = hq / hkv;
  TORCH_CHECK(hq % hkv == 0 && (G == 1 || G == 2 || G == 4 || G == 5 || G == 8), "decode_attention: group size");
  const int64_t B = q.size(0), Smax = kc.size(1);
  TORCH_CHECK(kc.size(0) == B && kc.size(2) == hkv * d && vc.sizes() == kc.sizes(), "decode_attention: cache shape");
  TORCH_CHECK(max_len <= Smax, "decode_attention: max_len > cache");
  const int nsplit = decode_split_plan(B, hkv, max_len);
  auto f32 = q.options().dtype(at::kFloat);
  Tensor opart = at::empty({B * hq * nsplit, d}, f32);
  Tensor mpart = at::empty({B * hq * nsplit}, f32), lpart = at::empty({B * hq * nsplit}, f32);
  Tensor out = at::empty({B, hq * d}, q.options());
  launch_decode_attention(q.data_ptr(), kc.data_ptr(), vc.data_ptr(), lens.data_ptr<int>(), opart.data_ptr<float>(),
                          mpart.data_ptr<float>(), lpart.data_ptr<float>(), out.data_ptr(), B, Smax, hq, hkv, d,
                          nsplit, (float)scale, stream());
  return out;
}

// q [B, hq*d], knew/vnew [B, hkv*d] (row-strided views allowed), caches [B, Smax, hkv*d], pos [B] int64:
// appends knew/vnew at pos and attends over pos + 1 keys (MFMA split-K kernel)
Tensor decode_attention_append(Tensor q, Tensor knew, Tensor vnew, Tensor kc, Tensor vc, Tensor pos, int64_t hq,
                               int64_t hkv, int64_t d, int64_t max_len, double scale) {
  CHECK_CUDA(q);
  for (const Tensor* t : {&q, &knew, &vnew, &kc, &vc}) CHECK_BF16((*t));
  CHECK_CONTIG(kc);
  CHECK_CONTIG(vc);
  TORCH_CHECK(pos.scalar_type() == at::kLong && pos.is_contiguous(), "pos: int64");
  TORCH_CHECK(d == 64 || d == 128, "decode_attention_append: head_dim 64 or 128");
  TORCH_CHECK(hq % hkv == 0 && hq / hkv <= 16, "decode_attention_append: group size <= 16");
  const int64_t B = q.size(0), Smax = kc.size(1);
  for (const Tensor* t : {&q, &knew, &vnew})
    TORCH_CHECK(t->dim() == 2 && t->size(0) == B && t->stride(1) == 1 && t->stride(0) % 8 == 0,
                "decode_attention_append: 2-D row-strided q/k/v with 16-B aligned rows");
  TORCH_CHECK(q.size(1) == hq * d && knew.size(1) == hkv * d && vnew.size(1) == hkv * d, "decode_attention_append: q/k/v width");
  TORCH_CHECK(kc.size(0) == B && kc.size(2) == hkv * d && vc.sizes() == kc.sizes() && pos.numel() == B,
              "decode_attention_append: cache shape");
  TORCH_CHECK(max_len <= Smax, "decode_attention_append: max_len > cache");
  const int nsplit = decode_split_plan2(B, hkv, max_len);
  auto f32 = q.options().dtype(at::kFloat);
  Tensor opart = at::empty({B * hq * nsplit, d}, f32);
  Tensor mpart = at::empty({B * hq * nsplit}, f32), lpart = at::empty({B * hq * nsplit}, f32);
  Tensor out = at::empty({B, hq * d}, q.options());
  launch_decode_attention2(q.data_ptr(), q.stride(0), knew.data_ptr(), knew.stride(0), vnew.data_ptr(), vnew.stride(0),
                           kc.data_ptr(), vc.data_ptr(), pos.data_ptr<int64_t>(), opart.data_ptr<float>(),
                           mpart.data_ptr<float>(), lpart.data_ptr<float>(), out.data_ptr(), B, Smax, hq, hkv, d, nsplit,
                           (float)scale, stream());
  return out;
}

// logits [B, V] fp32|bf16; hist [B, L] int32 (-1 = pad) or None; temperature <= 0 → greedy
Tensor sample(Tensor logits, optional<Tensor> hist, double temperature, int64_t top_k, double top_p, double penalty,
              int64_t key) {
  CHECK_CUDA(logits);
  CHECK_CONTIG(logits);
  const int64_t B = logits.size(0), V = logits.size(1);
  Tensor work = at::empty({B, V}, logits.options().dtype(at::kFloat));
  Tensor out = at::empty({B}, logits.options().dtype(at::kLong));
  int L = 0;
  if (hist.has_value() && hist->defined()) {
    TORCH_CHECK(hist->scalar_type() == at::kInt && hist->is_contiguous() && hist->size(0) == B, "hist: [B,L] int32");
    L = hist->size(1);
  }
  launch_sample(dtype_code(logits), logits.data_ptr(), L ? hist->data_ptr<int>() : nullptr, L,
                work.data_ptr<float>(), out.data_ptr<int64_t>(), B, V, (float)temperature, (int)top_k, (float)top_p,
                (float)penalty, (uint64_t)key, stream());
  return out;
}

}  // namespace


// ---- MoE routing / dispatch (moe.hip)
std::vector<Tensor> moe_route(Tensor logits, int64_t k, int64_t mode, bool want_probs) {
  CHECK_CONTIG(logits);
  TORCH_CHECK(logits.dim() == 2 && logits.size(1) <= 64 && k >= 1 && k <= 8 && k <= logits.size(1),
              "moe_route: logits [T, E<=64], 1<=k<=min(8,E)");
  const int T = logits.size(0), E = logits.size(1);
  auto oi = logits.options();
  Tensor idx = torch::empty({T, k}, oi.dtype(at::kInt));
  Tensor w = torch::empty({T, k}, oi.dtype(at::kFloat));
  Tensor probs = want_probs ? torch::empty({T, E}, oi.dtype(at::kFloat)) : Tensor();
  if (T) launch_moe_route(dtype_code(logits), logits.data_ptr(), idx.data_ptr<int>(), w.data_ptr<float>(),
                          want_probs ? probs.data_ptr<float>() : nullptr, T, E, k, mode, stream());
  return {idx, w, probs};
}

Tensor moe_route_bwd(Tensor dw, Tensor w, Tensor idx, optional<Tensor> probs, int64_t E, int64_t mode,
                     at::ScalarType dt) {
  CHECK_CONTIG(dw); CHECK_CONTIG(w); CHECK_CONTIG(idx);
  TORCH_CHECK(dw.scalar_type() == at::kFloat && w.scalar_type() == at::kFloat && idx.scalar_type() == at::kInt,
              "moe_route_bwd: dtypes");
  TORCH_CHECK(mode == 0 || (probs.has_value() && probs->is_contiguous()), "moe_route_bwd: mode 1 needs probs");
  const int T = idx.size(0), k = idx.size(1);
  Tensor dl = torch::empty({T, E}, dw.options().dtype(dt));
  if (T) launch_moe_route_bwd(dtype_code(dl), dw.data_ptr<float>(), w.data_ptr<float>(), idx.data_ptr<int>(),
                              mode == 1 ? probs->data_ptr<float>() : nullptr, dl.data_ptr(), T, E, k, mode, stream());
  return dl;
}

std::vector<Tensor> moe_permute(Tensor ids, int64_t E) {
  CHECK_CONTIG(ids);
  TORCH_CHECK(ids.scalar_type() == at::kInt && ids.numel() < (1 << 24), "moe_permute: int32 ids, < 2^24 pairs");
  const int P = ids.numel();
  auto o = ids.options();
  Tensor pos_of = torch::empty({P}, o), perm = torch::empty({P}, o), offsets = torch::empty({E + 1}, o);
  launch_moe_permute(ids.data_ptr<int>(), P, E, pos_of.data_ptr<int>(), perm.data_ptr<int>(),
                     offsets.data_ptr<int>(), stream());
  return {pos_of, perm, offsets};
}

Tensor moe_gather(Tensor x, Tensor perm, int64_t k, optional<Tensor> w) {
  CHECK_CONTIG(x); CHECK_CONTIG(perm);
  TORCH_CHECK(x.dim() == 2 && x.size(1) % 8 == 0 && perm.scalar_type() == at::kInt, "moe_gather: x [T, H%8==0]");
  if (w.has_value()) TORCH_CHECK(w->is_contiguous() && w->scalar_type() == at::kFloat, "moe_gather: w fp32");
  const int R = perm.numel(), H = x.size(1);
  Tensor out = torch::empty({R, H}, x.options());
  if (R) launch_moe_gather(dtype_code(x), x.data_ptr(), perm.data_ptr<int>(), w.has_value() ? w->data_ptr<float>() : nullptr,
                           out.data_ptr(), R, H, k, stream());
  return out;
}

Tensor moe_combine(Tensor ys, Tensor pos_of, int64_t k, optional<Tensor> w, optional<Tensor> base) {
  CHECK_CONTIG(ys); CHECK_CONTIG(pos_of);
  TORCH_CHECK(ys.dim() == 2 && ys.size(1) % 8 == 0 && pos_of.scalar_type() == at::kInt && pos_of.numel() % k == 0,
              "moe_combine: ys [R, H%8==0], pos_of int32 [T*k]");
  if (w.has_value()) TORCH_CHECK(w->is_contiguous() && w->scalar_type() == at::kFloat, "moe_combine: w fp32");
  if (base.has_value()) TORCH_CHECK(base->is_contiguous() && base->scalar_type() == ys.scalar_type(), "moe_combine: base");
  const int T = pos_of.numel() / k, H = ys.size(1);
  Tensor out = torch::empty({T, H}, ys.options());
  if (T) launch_moe_combine(dtype_code(ys), ys.data_ptr(), pos_of.data_ptr<int>(),
                            w.has_value() ? w->data_ptr<float>() : nullptr, optr(base), out.data_ptr(), T, H, k, stream());
  return out;
}

Tensor moe_wgrad(Tensor dout, Tensor ys, Tensor pos_of, int64_t k) {
  CHECK_CONTIG(dout); CHECK_CONTIG(ys); CHECK_CONTIG(pos_of);
  TORCH_CHECK(dout.scalar_type() == ys.scalar_type() && dout.size(1) == ys.size(1) && ys.size(1) % 8 == 0,
              "moe_wgrad: shapes");
  const int T = dout.size(0), H = dout.size(1);
  Tensor dw = torch::empty({T, k}, dout.options().dtype(at::kFloat));
  if (T) launch_moe_wgrad(dtype_code(ys), dout.data_ptr(), ys.data_ptr(), pos_of.data_ptr<int>(), dw.data_ptr<float>(),
                          T, H, k, stream());
  return dw;
}

// ------------------------------------------------------------------ custom all-reduce (allreduce.hip)
int64_t car_alloc_py(int64_t bytes, bool uncached) {
  void* p = car_alloc((size_t)bytes, uncached);
  TORCH_CHECK(p != nullptr, "car_alloc: device allocation of ", bytes, " B failed");
  return reinterpret_cast<int64_t>(p);
}
void car_free_py(int64_t p) { car_free(reinterpret_cast<void*>(p)); }
pybind11::bytes car_handle_py(int64_t p) {
  char h[64] = {0};
  TORCH_CHECK(sizeof(hipIpcMemHandle_t) <= 64, "IPC handle larger than 64 B");
  TORCH_CHECK(car_ipc_handle(reinterpret_cast<void*>(p), h), "hipIpcGetMemHandle failed (is HSA_ENABLE_IPC_MODE_LEGACY=0 set?)");
  return pybind11::bytes(h, sizeof(hipIpcMemHandle_t));
}
int64_t car_open_py(pybind11::bytes h) {
  std::string s = h;
  char buf[64] = {0};
  memcpy(buf, s.data(), std::min<size_t>(s.size(), 64));
  void* p = car_ipc_open(buf);
  TORCH_CHECK(p != nullptr, "hipIpcOpenMemHandle failed");
  return reinterpret_cast<int64_t>(p);
}
void car_close_py(int64_t p) { car_ipc_close(reinterpret_cast<void*>(p)); }

void custom_allreduce(Tensor out, std::vector<int64_t> data, std::vector<int64_t> result, std::vector<int64_t> flags,
                      Tensor err, int64_t rank, int64_t epoch, bool two_shot, double scale, int64_t blocks) {
  CHECK_CUDA(out); CHECK_CONTIG(out); CHECK_CUDA(err);
  const int W = (int)data.size();
  TORCH_CHECK(W >= 1 && W <= 8 && (int)result.size() == W && (int)flags.size() == W, "custom_allreduce: 1..8 peers");
  TORCH_CHECK(rank >= 0 && rank < W, "custom_allreduce: rank");
  TORCH_CHECK(err.scalar_type() == at::kInt && err.numel() >= 1, "custom_allreduce: err must be int32");
  const size_t bytes = out.numel() * out.element_size();
  TORCH_CHECK(bytes % 16 == 0, "custom_allreduce: byte size must be a multiple of 16");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(out.data_ptr()) % 16 == 0, "custom_allreduce: out must be 16-B aligned");
  std::vector<const void*> d(W);
  std::vector<void*> r(W);
  std::vector<uint32_t*> f(W);
  for (int i = 0; i < W; ++i) {
    d[i] = reinterpret_cast<const void*>(data[i]);
    r[i] = reinterpret_cast<void*>(result[i]);
    f[i] = reinterpret_cast<uint32_t*>(flags[i]);
    TORCH_CHECK(data[i] % 16 == 0 && result[i] % 16 == 0 && flags[i] % 4 == 0, "custom_allreduce: peer alignment");
  }
  // in place: the kernel stages `out` into this rank's data area (peers read it from there)
  launch_custom_allreduce(dtype_code(out), d.data(), r.data(), f.data(), err.data_ptr<int>(), W, (int)rank,
                          (uint32_t)epoch, bytes, two_shot, (float)scale, out.data_ptr(), (int)blocks, stream());
}

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  m.doc() = "llm_in_practise_amd gfx950 (MI355X / CDNA4) kernels";
  m.def("rmsnorm_fwd", &rmsnorm_fwd);
  m.def("moe_route", &moe_route);
  m.def("moe_route_bwd", &moe_route_bwd);
  m.def("moe_permute", &moe_permute);
  m.def("moe_gather", &moe_gather);
  m.def("moe_combine", &moe_combine);
  m.def("moe_wgrad", &moe_wgrad);
  m.def("rmsnorm_bwd", &rmsnorm_bwd);
  m.def("layernorm_fwd", &layernorm_fwd);
  m.def("layernorm_bwd", &layernorm_bwd);
  m.def("rope", &rope);
  m.def("qk_norm_rope_fwd", &qk_norm_rope_fwd);
  m.def("qk_norm_rope_bwd", &qk_norm_rope_bwd);
  m.def("swiglu_fwd", &swiglu_fwd);
  m.def("swiglu_bwd", &swiglu_bwd);
  m.def("gelu_fwd", &gelu_fwd);
  m.def("gelu_bwd", &gelu_bwd);
  m.def("ce_fwd_bwd", &ce_fwd_bwd);
  m.def("dropout_fwd", &dropout_fwd);
  m.def("embedding_fwd", &embedding_fwd, py::arg("weight"), py::arg("ids"), py::arg("oob") = py::none());
  m.def("embedding_bwd", &embedding_bwd);
  m.def("dropout_bwd_add", &dropout_bwd_add);
  m.def("grad_norm", &grad_norm);
  m.def("decode_attention", &decode_attention);
  m.def("decode_attention_append", &decode_attention_append);
  m.def("lora_proj", &lora_proj);
  m.def("lora_acc", &lora_acc);
  m.def("lora_proj2", &lora_proj2);
  m.def("lora_proj_pair", &lora_proj_pair);
  m.def("lora_acc_pair", &lora_acc_pair);
  m.def("lora_dA_pair", &lora_dA_pair);
  m.def("lora_acc_quad", &lora_acc_quad);
  m.def("lora_dx2", &lora_dx2);
  m.def("lora_proj_m", &lora_proj_m);
  m.def("int4_dequant", &int4_dequant);
  m.def("lora_proj_cols", &lora_proj_cols);
  m.def("lora_acc_jobs", &lora_acc_jobs);
  m.def("lora_dxc", &lora_dxc, py::arg("gs"), py::arg("as"), py::arg("masks"), py::arg("ps"), py::arg("rb") = 0);
  m.def("lora_apply", &lora_apply);
  m.def("gemv_w4", &gemv_w4);
  m.def("sample", &sample);
  m.def("adamw", &adamw);
  m.def("adamw8bit", &adamw8bit);
  m.def("host_mapped_empty", &host_mapped_empty, py::arg("numel"), py::arg("dtype"));
  m.def("unscale", &unscale);
  m.def("nf4_quantize", &nf4_quantize);
  m.def("nf4_dequant", &nf4_dequant);
  m.def("nf4_dequant_fast", &nf4_dequant_fast);
  m.def("gemm_skinny", &gemm_skinny);
  m.def("lt_linear", &lt_linear);
  m.def("lt_dx", &lt_dx);
  m.def("lt_reset", &lt_reset);
  m.def("w4mm", &w4mm, py::arg("x"), py::arg("codes"), py::arg("sc2"), py::arg("N"), py::arg("gs"),
        py::arg("residual") = py::none(), py::arg("nkb") = 0);
  m.def("w4mm_ok", &w4mm_ok);
  m.def("w4g", &w4g, py::arg("x"), py::arg("codes"), py::arg("sc2"), py::arg("N"), py::arg("gs"),
        py::arg("residual") = py::none(), py::arg("ks") = 0);
  m.def("w4g_ok", &w4g_ok);
  m.def("w4g_splits", &w4g_splits);
  m.def("set_dequant_variant", &set_dequant_variant);
  m.def("gemm4w_ok", &gemm4w_ok);
  m.def("gemm4w_plan_info", &gemm4w_plan_info);
  m.def("g4w_pack", &g4w_pack);
  m.def("gemm4w_lora", &gemm4w_lora);
  m.def("gemm4w_loradx", &gemm4w_loradx, py::arg("dy"), py::arg("w"), py::arg("wscale"), py::arg("n_w4"), py::arg("gs"),
        py::arg("as"), py::arg("masks"), py::arg("ps"), py::arg("bn") = 0, py::arg("bm") = 0);
  m.def("gemm4w", &gemm4w, py::arg("x"), py::arg("w"), py::arg("residual") = py::none(), py::arg("splits") = 0,
        py::arg("bt") = false, py::arg("bn") = 0, py::arg("bm") = 0, py::arg("wscale") = py::none(),
        py::arg("n_w4") = 0, py::arg("wzero") = py::none());
  m.def("gemm4w_swiglu", &gemm4w_swiglu, py::arg("x"), py::arg("w"), py::arg("wscale") = py::none(),
        py::arg("f_w4") = 0, py::arg("want_gu") = true, py::arg("want_h") = true);
  m.def("mlora_apply", &mlora_apply);
  m.def("gemm4w_dswiglu", &gemm4w_dswiglu, py::arg("dy"), py::arg("w"), py::arg("gu"), py::arg("wscale") = py::none());
  m.def("attn_fwd", &attn_fwd);
  m.def("attn_fwd_ext", &attn_fwd_ext);
  m.def("attn_bwd", &attn_bwd);
  // debug: phase timestamps of the D = 128 dK/dV kernel go into `buf` (u8/i64 tensor) while set; None clears
  m.def("attn_set_trace", [](optional<Tensor> buf) { attn_set_trace(buf && buf->defined() ? buf->data_ptr() : nullptr); });
  m.def("car_alloc", &car_alloc_py);
  m.def("car_free", &car_free_py);
  m.def("car_handle", &car_handle_py);
  m.def("car_open", &car_open_py);
  m.def("car_close", &car_close_py);
  m.def("car_max_blocks", &car_max_blocks);
  m.def("custom_allreduce", &custom_allreduce);
}
