// Probe: verify v_mfma_f32_32x32x2_f32 operand/accumulator lane maps on gfx950.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cmath>
typedef float f32x16 __attribute__((ext_vector_type(16)));
__global__ void k(const float* A, const float* B, float* D) {
  // A: 32x2 row-major [i][k], B: 2x32 [k][j]; D: 32x32 [i][j]
  int l = threadIdx.x;
  float a = A[(l & 31) * 2 + (l >> 5)];
  float b = B[(l >> 5) * 32 + (l & 31)];
  f32x16 c = {0};
  c = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
  for (int r = 0; r < 16; ++r) {
    int row = (r & 3) + 8 * (r >> 2) + 4 * (l >> 5);
    int col = l & 31;
    D[row * 32 + col] = c[r];
  }
}
int main() {
  float hA[64], hB[64], hD[1024];
  for (int i = 0; i < 32; ++i) for (int kk = 0; kk < 2; ++kk) hA[i*2+kk] = (float)(i * 3 + kk * 7 + 1);
  for (int kk = 0; kk < 2; ++kk) for (int j = 0; j < 32; ++j) hB[kk*32+j] = (float)(j * 5 - kk * 11 + 2);
  float *dA, *dB, *dD;
  hipMalloc(&dA, 256); hipMalloc(&dB, 256); hipMalloc(&dD, 4096);
  hipMemcpy(dA, hA, 256, hipMemcpyHostToDevice); hipMemcpy(dB, hB, 256, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, dA, dB, dD);
  hipMemcpy(hD, dD, 4096, hipMemcpyDeviceToHost);
  int bad = 0;
  for (int i = 0; i < 32; ++i) for (int j = 0; j < 32; ++j) {
    float ref = hA[i*2]*hB[j] + hA[i*2+1]*hB[32+j];
    if (ref != hD[i*32+j]) ++bad;
  }
  printf("mfma_32x32x2f32 layout mismatches: %d\n", bad);
  return bad != 0;
}
