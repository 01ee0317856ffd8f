// Probe of v_permlane16_swap_b32 semantics on gfx950 (which lanes exchange): a[lane] = lane, b[lane] = 100 + lane
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(unsigned* out) {
  unsigned a = threadIdx.x, b = 100 + threadIdx.x;
  auto r = __builtin_amdgcn_permlane16_swap(a, b, false, false);
  out[threadIdx.x] = r[0];
  out[64 + threadIdx.x] = r[1];
}
int main() {
  unsigned* d;
  hipMalloc(&d, 128 * 4);
  k<<<1, 64>>>(d);
  unsigned h[128];
  hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  for (int w = 0; w < 2; ++w) {
    printf(w ? "r[1]:" : "r[0]:");
    for (int i = 0; i < 64; ++i) printf(" %u", h[64 * w + i]);
    printf("\n");
  }
  return 0;
}
