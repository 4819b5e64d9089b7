// f32 MFMA issue rate on gfx950 by accumulator chains and waves per SIMD (tools/probes; not a test):
// every CU runs one workgroup of W waves, each issuing N rounds of NACC independent accumulator
// chains; prints TFLOP/s over the whole chip (HIP events) -- what the dependent-accumulator latency
// costs a GEMM's inner loop.
// hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/probes/mfma_rate_probe.hip -o /tmp/mfma_rate
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f16v __attribute__((ext_vector_type(16)));
typedef float f4v __attribute__((ext_vector_type(4)));

template <int OP, int NACC>
__global__ void k_rate(float x, float* out, int rounds) {
  const float a = x + threadIdx.x, b = x - threadIdx.x;
  if (OP == 32) {
    f16v c[NACC];
    for (int i = 0; i < NACC; ++i)
      for (int r = 0; r < 16; ++r) c[i][r] = 0.f;
    for (int it = 0; it < rounds; ++it)
#pragma unroll
      for (int i = 0; i < NACC; ++i) c[i] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c[i], 0, 0, 0);
    float s = 0.f;
    for (int i = 0; i < NACC; ++i) s += c[i][0] + c[i][15];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  } else {
    f4v c[NACC];
    for (int i = 0; i < NACC; ++i) c[i] = f4v{0.f, 0.f, 0.f, 0.f};
    for (int it = 0; it < rounds; ++it)
#pragma unroll
      for (int i = 0; i < NACC; ++i) c[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c[i], 0, 0, 0);
    float s = 0.f;
    for (int i = 0; i < NACC; ++i) s += c[i][0] + c[i][3];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  }
}

template <int OP, int NACC>
void run(float* out, int waves) {
  const int rounds = 4096 / NACC;
  const double flop_per = OP == 32 ? 32.0 * 32 * 2 * 2 : 16.0 * 16 * 4 * 2;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipLaunchKernelGGL((k_rate<OP, NACC>), dim3(256), dim3(64 * waves), 0, 0, 1.f, out, rounds);
  hipEventRecord(e0);
  for (int r = 0; r < 5; ++r)
    hipLaunchKernelGGL((k_rate<OP, NACC>), dim3(256), dim3(64 * waves), 0, 0, 1.f, out, rounds);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0.f;
  hipEventElapsedTime(&ms, e0, e1);
  const double flops = 5.0 * 256 * waves * (double)rounds * NACC * flop_per;
  printf("op %dx%d nacc %d waves/WG %2d: %.1f TFLOP/s  (%.1f cycles per mfma per SIMD at 2.4 GHz)\n", OP, OP,
         NACC, waves, flops / (ms * 1e-3) / 1e12,
         (ms * 1e-3 / 5) * 2.4e9 / ((double)rounds * NACC * waves / 4));
}

int main() {
  float* out;
  hipMalloc(&out, 256 * 1024 * sizeof(float));
  for (int waves : {4, 8}) {
    run<32, 1>(out, waves);
    run<32, 2>(out, waves);
    run<32, 4>(out, waves);
    run<16, 1>(out, waves);
    run<16, 2>(out, waves);
    run<16, 4>(out, waves);
  }
  hipFree(out);
  return 0;
}
