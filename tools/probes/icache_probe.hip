// Instruction-fetch cost of straight-line code (not a test): one workgroup runs N unrolled
// independent VALU ops; wall-clock per launch, cold (first launch) vs warm (relaunch) vs after
// another kernel with a different code body.  Build: hipcc --offload-arch=gfx950 -O3 -o icache_probe icache_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>

template <int N, int SALT>
__global__ void straight(float* out, float a, float b) {
  const uint64_t t0 = wall_clock64();
  float x0 = threadIdx.x, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3, x4 = x0 + 4, x5 = x0 + 5, x6 = x0 + 6, x7 = x0 + 7;
#pragma unroll
  for (int i = 0; i < N / 8; ++i) {
    x0 = __fmaf_rn(x0, a, b + SALT); x1 = __fmaf_rn(x1, a, b); x2 = __fmaf_rn(x2, a, b); x3 = __fmaf_rn(x3, a, b);
    x4 = __fmaf_rn(x4, a, b); x5 = __fmaf_rn(x5, a, b); x6 = __fmaf_rn(x6, a, b); x7 = __fmaf_rn(x7, a, b);
    asm volatile("" : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3), "+v"(x4), "+v"(x5), "+v"(x6), "+v"(x7));
  }
  const uint64_t t1 = wall_clock64();
  out[threadIdx.x] = x0 + x1 + x2 + x3 + x4 + x5 + x6 + x7;
  if (threadIdx.x == 0) out[64 + blockIdx.x] = (float)(t1 - t0);
}

template <int N, int SALT>
float run(float* d, float* h, int blocks) {
  hipLaunchKernelGGL((straight<N, SALT>), dim3(blocks), dim3(64), 0, 0, d, 1.0001f, 0.5f);
  hipDeviceSynchronize();
  hipMemcpy(h, d, (64 + blocks) * 4, hipMemcpyDeviceToHost);
  float s = 0;
  for (int i = 0; i < blocks; ++i) s += h[64 + i];
  return s / blocks * 10.f;   // ns (100 MHz wall clock)
}

int main() {
  float *d, h[64 + 256];
  hipMalloc(&d, (64 + 256) * 4);
  for (int rep = 0; rep < 3; ++rep) {
    const float c = run<4096, 0>(d, h, 256);
    const float w = run<4096, 0>(d, h, 256);
    run<4096, 1>(d, h, 256);                 // another code body of the same size
    const float a = run<4096, 0>(d, h, 256);
    const float c2 = run<512, 2>(d, h, 256);
    const float w2 = run<512, 2>(d, h, 256);
    printf("4096 ops: first %.0f ns, relaunch %.0f ns, after other kernel %.0f ns | 512 ops: first %.0f, relaunch %.0f\n",
           c, w, a, c2, w2);
  }
  return 0;
}
