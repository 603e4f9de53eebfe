// Semantics check of v_permlane16_swap_b32 / v_permlane32_swap_b32 (gfx950): for every lane, the
// (vdst, vsrc) values after the swap, with vdst = lane, vsrc = 100 + lane before it.
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(unsigned* out) {
  const unsigned l = threadIdx.x;
  auto r = __builtin_amdgcn_permlane16_swap(l, 100u + l, false, false);
  auto s = __builtin_amdgcn_permlane32_swap(l, 100u + l, false, false);
  out[l] = r[0]; out[64 + l] = r[1]; out[128 + l] = s[0]; out[192 + l] = s[1];
}
int main() {
  unsigned* d; unsigned h[256];
  if (hipMalloc(&d, sizeof h) != hipSuccess) return 1;
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
  if (hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost) != hipSuccess) return 2;
  const char* nm[4] = {"p16 vdst", "p16 vsrc", "p32 vdst", "p32 vsrc"};
  for (int t = 0; t < 4; ++t) {
    printf("%s:", nm[t]);
    for (int l = 0; l < 64; ++l) printf(" %u", h[t * 64 + l]);
    printf("\n");
  }
  return hipFree(d) == hipSuccess ? 0 : 3;
}
