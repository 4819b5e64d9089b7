// Fixed cost of a launch (not a test): back-to-back launches of near-empty kernels, mean time per
// launch from HIP events over 200 launches, for the grid / LDS shapes of the fan-out kernels, and
// one launch's begin-to-end under hipEvents around it alone.
// Build: hipcc --offload-arch=gfx950 -O3 -o /tmp/lp launch_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void k_empty(float* out) {
  extern __shared__ float s[];
  if (threadIdx.x == 0 && blockIdx.x == 0) out[0] = 1.f;
}
__global__ void k_lds_touch(float* out) {
  extern __shared__ float s[];
  s[threadIdx.x] = threadIdx.x;
  __syncthreads();
  if (threadIdx.x == 0) out[blockIdx.x] = s[255];
}
__global__ void k_write(float* out, int n) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) out[i] = (float)i;
}

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("hip error %d line %d\n", (int)e_, __LINE__); return 1; } } while (0)

template <typename F>
int timeit(const char* name, F launch) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  for (int i = 0; i < 20; ++i) launch();
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(a, 0));
  for (int i = 0; i < 200; ++i) launch();
  CK(hipEventRecord(b, 0));
  CK(hipEventSynchronize(b));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, a, b));
  float ms1 = 0;
  CK(hipEventRecord(a, 0));
  launch();
  CK(hipEventRecord(b, 0));
  CK(hipEventSynchronize(b));
  CK(hipEventElapsedTime(&ms1, a, b));
  printf("%-44s back-to-back %6.2f us/launch, alone between events %6.2f us\n", name, ms * 1e3 / 200, ms1 * 1e3);
  return 0;
}

int main() {
  float* d;
  CK(hipMalloc(&d, 64 << 20));
  const size_t L73 = 74648, L157 = 157000;
  timeit("empty, 1 x 64", [&] { hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, 0, d); });
  timeit("empty, 256 x 256", [&] { hipLaunchKernelGGL(k_empty, dim3(256), dim3(256), 0, 0, d); });
  timeit("empty, 512 x 256", [&] { hipLaunchKernelGGL(k_empty, dim3(512), dim3(256), 0, 0, d); });
  timeit("empty, 256 x 256, 73 KB LDS", [&] { hipLaunchKernelGGL(k_empty, dim3(256), dim3(256), L73, 0, d); });
  timeit("LDS touch, 256 x 256, 73 KB LDS", [&] { hipLaunchKernelGGL(k_lds_touch, dim3(256), dim3(256), L73, 0, d); });
  timeit("LDS touch, 512 x 256, 73 KB LDS", [&] { hipLaunchKernelGGL(k_lds_touch, dim3(512), dim3(256), L73, 0, d); });
  timeit("LDS touch, 256 x 256, 157 KB LDS", [&] { hipLaunchKernelGGL(k_lds_touch, dim3(256), dim3(256), L157, 0, d); });
  timeit("write 2.6 MB, 256 x 256", [&] { hipLaunchKernelGGL(k_write, dim3(256), dim3(256), 0, 0, d, 655360); });
  timeit("write 20 MB, 256 x 256", [&] { hipLaunchKernelGGL(k_write, dim3(256), dim3(256), 0, 0, d, 5 << 20); });
  CK(hipFree(d));
  return 0;
}
