// A 512 x 512 x 512 fp32 GEMM for the dense Cayley maps' backward chain (GMn = inv^T Ginv inv^T:
// two dependent 512^3 products, ~14 us each as hipBLASLt MT128x128 tiles = 16 workgroups):
// 256 workgroups of 32 x 32 output tiles, the 4 waves split K (128 each) on v_mfma_f32_16x16x4_f32
// with operands straight from L2 (16-byte loads along k for A, 64-byte rows for B), one LDS
// reduction of the 4 partials in a fixed order.  Prints us per launch and max |C - ref| (not a test).
// hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/probes/sgemm_probe.hip -o /tmp/sgemm_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cmath>
#include <vector>

typedef float f4 __attribute__((ext_vector_type(4)));
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s line %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

// C[M x N] = A[M x K] B[K x N], all row-major, M = N = K = 512 (multiples of 32 / 128)
template <int KS>     // K per wave
__global__ void __launch_bounds__(256) k_sgemm(const float* __restrict__ A, const float* __restrict__ B,
                                               float* __restrict__ C, int N, int K) {
  __shared__ float red[4][32][33];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int i = lane & 15, q = lane >> 4;
  const int tm = blockIdx.y * 32, tn = blockIdx.x * 32;
  const int k0 = w * KS;
  f4 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) acc[a][b] = f4{0.f, 0.f, 0.f, 0.f};
  // chunk kc of 16 k: step s uses k = 16 kc + 4 q + s at lane q (A: one 16-byte load per row block)
#pragma unroll 2
  for (int kc = 0; kc < KS / 16; ++kc) {
    const int kb = k0 + 16 * kc + 4 * q;
    f4 av[2], bv[2];
#pragma unroll
    for (int a = 0; a < 2; ++a) av[a] = *reinterpret_cast<const f4*>(A + (size_t)(tm + 16 * a + i) * K + kb);
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int s = 0; s < 4; ++s) bv[b][s] = B[(size_t)(kb + s) * N + tn + 16 * b + i];
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b) acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[a][s], bv[b][s], acc[a][b], 0, 0, 0);
  }
  // D[row 4q + r][col i] of block (a, b)
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int r = 0; r < 4; ++r) red[w][16 * a + 4 * q + r][16 * b + i] = acc[a][b][r];
  __syncthreads();
  for (int e = threadIdx.x; e < 32 * 32; e += 256) {
    const int r = e >> 5, c = e & 31;
    C[(size_t)(tm + r) * N + tn + c] = ((red[0][r][c] + red[1][r][c]) + red[2][r][c]) + red[3][r][c];
  }
}

int main() {
  const int n = 512;
  std::vector<float> hA(n * n), hB(n * n), hC(n * n);
  srand(3);
  for (auto& v : hA) v = (float)rand() / RAND_MAX - 0.5f;
  for (auto& v : hB) v = (float)rand() / RAND_MAX - 0.5f;
  float *A, *B, *C;
  CK(hipMalloc(&A, n * n * 4)); CK(hipMalloc(&B, n * n * 4)); CK(hipMalloc(&C, n * n * 4));
  CK(hipMemcpy(A, hA.data(), n * n * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(B, hB.data(), n * n * 4, hipMemcpyHostToDevice));
  dim3 grid(n / 32, n / 32);
  hipLaunchKernelGGL(k_sgemm<128>, grid, dim3(256), 0, 0, A, B, C, n, n);
  CK(hipDeviceSynchronize());
  CK(hipMemcpy(hC.data(), C, n * n * 4, hipMemcpyDeviceToHost));
  double md = 0;
  for (int r = 0; r < n; r += 7)
    for (int c = 0; c < n; c += 5) {
      double s = 0;
      for (int k = 0; k < n; ++k) s += (double)hA[r * n + k] * hB[k * n + c];
      md = fmax(md, fabs(s - hC[r * n + c]));
    }
  hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  for (int rep = 0; rep < 10; ++rep) hipLaunchKernelGGL(k_sgemm<128>, grid, dim3(256), 0, 0, A, B, C, n, n);
  CK(hipEventRecord(a));
  for (int rep = 0; rep < 200; ++rep) hipLaunchKernelGGL(k_sgemm<128>, grid, dim3(256), 0, 0, A, B, C, n, n);
  CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
  float ms; CK(hipEventElapsedTime(&ms, a, b));
  printf("sgemm 512^3 (256 wg, 4-wave split K): %.2f us per launch (back-to-back), max |err| %.3g\n", ms * 1e3f / 200, md);
  // a dependent pair, as GMn needs
  CK(hipEventRecord(a));
  for (int rep = 0; rep < 100; ++rep) {
    hipLaunchKernelGGL(k_sgemm<128>, grid, dim3(256), 0, 0, A, B, C, n, n);
    hipLaunchKernelGGL(k_sgemm<128>, grid, dim3(256), 0, 0, C, A, B, n, n);
  }
  CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
  CK(hipEventElapsedTime(&ms, a, b));
  printf("dependent pair: %.2f us\n", ms * 1e3f / 100);
  return 0;
}
