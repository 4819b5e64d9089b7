// Layout and issue cost of v_mfma_f32_4x4x1_16b_f32 on gfx950 (not a test).
// hipcc --offload-arch=gfx950 -O3 tools/probes/mfma4_probe.hip -o tools/probes/mfma4_probe.bin
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f4 __attribute__((ext_vector_type(4)));

__global__ void k_layout(const float* a, const float* b, float* d) {
  const int l = threadIdx.x;
  f4 c = {0.f, 0.f, 0.f, 0.f};
  c = __builtin_amdgcn_mfma_f32_4x4x1f32(a[l], b[l], c, 0, 0, 0);
  for (int r = 0; r < 4; ++r) d[l * 4 + r] = c[r];
}

template <int NACC>
__global__ void k_time(float x, float* out, long long* cyc) {
  f4 c[NACC];
  for (int i = 0; i < NACC; ++i) c[i] = f4{0.f, 0.f, 0.f, 0.f};
  const float a = x + threadIdx.x, b = x - threadIdx.x;
  long long t0 = __builtin_readcyclecounter();
  for (int it = 0; it < 256; ++it) {
#pragma unroll
    for (int i = 0; i < NACC; ++i) c[i] = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, c[i], 0, 0, 0);
  }
  long long t1 = __builtin_readcyclecounter();
  float s = 0.f;
  for (int i = 0; i < NACC; ++i) s += c[i][0] + c[i][1] + c[i][2] + c[i][3];
  out[threadIdx.x] = s;
  if (threadIdx.x == 0) *cyc = t1 - t0;
}

int main() {
  float *a, *b, *d, *o;
  long long* cyc;
  hipMallocManaged(&a, 64 * 4); hipMallocManaged(&b, 64 * 4); hipMallocManaged(&d, 256 * 4);
  hipMallocManaged(&o, 64 * 4); hipMallocManaged(&cyc, 8);
  for (int pass = 0; pass < 2; ++pass) {
    for (int l = 0; l < 64; ++l) { a[l] = pass == 0 ? (float)l : 1.f; b[l] = pass == 0 ? 1.f : (float)l; }
    hipLaunchKernelGGL(k_layout, dim3(1), dim3(64), 0, 0, a, b, d);
    hipDeviceSynchronize();
    printf("%s lane of each D[lane][reg] (reg 0..3):\n", pass == 0 ? "A" : "B");
    for (int l = 0; l < 64; ++l) {
      printf("  l%02d:", l);
      for (int r = 0; r < 4; ++r) printf(" %2.0f", d[l * 4 + r]);
      printf(l % 4 == 3 ? "\n" : " |");
    }
  }
  hipLaunchKernelGGL(k_time<1>, dim3(1), dim3(64), 0, 0, 1.f, o, cyc); hipDeviceSynchronize();
  printf("1 accumulator: %.1f cycles per mfma\n", *cyc / 256.0);
  hipLaunchKernelGGL(k_time<4>, dim3(1), dim3(64), 0, 0, 1.f, o, cyc); hipDeviceSynchronize();
  printf("4 accumulators: %.1f cycles per mfma\n", *cyc / 1024.0);
  hipLaunchKernelGGL(k_time<8>, dim3(1), dim3(64), 0, 0, 1.f, o, cyc); hipDeviceSynchronize();
  printf("8 accumulators: %.1f cycles per mfma\n", *cyc / 2048.0);
  return 0;
}
