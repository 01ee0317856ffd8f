// Host AdamW for ZeRO-Offload (the DeepSpeedCPUAdam role).
//
// fp32 master params / states live in pinned host memory; the update is an OpenMP-parallel,
// compiler-vectorised (AVX-512/AVX2 via -march=native) loop.  Optionally writes the bf16
// copy that is streamed back to the GPU over PCIe, and applies a gradient scale (fp16 loss
// scale / clip coefficient) in the same pass.
#include <torch/extension.h>

#include <cmath>
#include <cstdint>
#include <cstring>

namespace {

inline uint16_t f2bf(float f) {
  uint32_t u;
  std::memcpy(&u, &f, 4);
  if ((u & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((u >> 16) | 0x40);
  u += 0x7fffu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}

void adamw_step(torch::Tensor p, torch::Tensor g, torch::Tensor m, torch::Tensor v, double lr, double b1, double b2,
                double eps, double wd, int64_t step, double grad_scale, c10::optional<torch::Tensor> p_bf16) {
  TORCH_CHECK(p.device().is_cpu() && p.scalar_type() == at::kFloat && p.is_contiguous(), "p: cpu fp32 contiguous");
  TORCH_CHECK(g.scalar_type() == at::kFloat && m.scalar_type() == at::kFloat && v.scalar_type() == at::kFloat,
              "fp32 grads/states");
  const int64_t n = p.numel();
  float* P = p.data_ptr<float>();
  const float* G = g.data_ptr<float>();
  float* M = m.data_ptr<float>();
  float* V = v.data_ptr<float>();
  uint16_t* PB = (p_bf16 && p_bf16->defined()) ? reinterpret_cast<uint16_t*>(p_bf16->data_ptr()) : nullptr;
  const float fb1 = b1, fb2 = b2, feps = eps, decay = 1.f - (float)(lr * wd), gs = grad_scale;
  const float bc1 = 1.f - std::pow(fb1, (float)step), bc2 = 1.f - std::pow(fb2, (float)step);
  const float step_size = (float)lr / bc1, inv_sqrt_bc2 = 1.f / std::sqrt(bc2);
#pragma omp parallel for simd schedule(static)
  for (int64_t i = 0; i < n; ++i) {
    const float gi = G[i] * gs;
    const float mi = fb1 * M[i] + (1.f - fb1) * gi;
    const float vi = fb2 * V[i] + (1.f - fb2) * gi * gi;
    M[i] = mi;
    V[i] = vi;
    const float pi = P[i] * decay - step_size * mi / (std::sqrt(vi) * inv_sqrt_bc2 + feps);
    P[i] = pi;
    if (PB) PB[i] = f2bf(pi);
  }
}

double sum_squares(torch::Tensor g) {
  TORCH_CHECK(g.scalar_type() == at::kFloat && g.is_contiguous(), "fp32 contiguous");
  const float* G = g.data_ptr<float>();
  const int64_t n = g.numel();
  double s = 0.0;
#pragma omp parallel for reduction(+ : s) schedule(static)
  for (int64_t i = 0; i < n; ++i) s += (double)G[i] * G[i];
  return s;
}

}  // namespace

#ifndef LIPA_SANITIZER_HARNESS  // tests/native/sanitize_host.cpp includes this file without the bindings
void register_loader(pybind11::module& m);

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  m.doc() = "llm_in_practise_amd host runtime (CPU AdamW, token loader)";
  m.def("adamw_step", &adamw_step, "fused host AdamW (ZeRO-Offload)", pybind11::arg("p"), pybind11::arg("g"),
        pybind11::arg("m"), pybind11::arg("v"), pybind11::arg("lr"), pybind11::arg("b1"), pybind11::arg("b2"),
        pybind11::arg("eps"), pybind11::arg("wd"), pybind11::arg("step"), pybind11::arg("grad_scale") = 1.0,
        pybind11::arg("p_bf16") = pybind11::none());
  m.def("sum_squares", &sum_squares);
  register_loader(m);
}
#endif  // LIPA_SANITIZER_HARNESS
