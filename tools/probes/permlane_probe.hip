// Semantics probe of v_permlane16_swap / v_permlane32_swap on gfx950 (not a test).
#include <hip/hip_runtime.h>
#include <stdio.h>
__global__ void k(unsigned* out) {
  const unsigned l = threadIdx.x;
  const unsigned v = 1000 + l;
  auto a = __builtin_amdgcn_permlane16_swap(v, v, false, false);
  auto b = __builtin_amdgcn_permlane32_swap(v, v, false, false);
  out[l * 4 + 0] = a[0];
  out[l * 4 + 1] = a[1];
  out[l * 4 + 2] = b[0];
  out[l * 4 + 3] = b[1];
}
int main() {
  unsigned* d;
  hipMalloc(&d, 64 * 4 * 4);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
  unsigned h[256];
  hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  for (int l = 0; l < 64; l += 5)
    printf("lane %2d: p16 {%u, %u}  p32 {%u, %u}\n", l, h[l * 4] - 1000, h[l * 4 + 1] - 1000, h[l * 4 + 2] - 1000,
           h[l * 4 + 3] - 1000);
  return 0;
}
