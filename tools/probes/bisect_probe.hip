// Cycle probe of the train_ode QP bisection variants on gfx950 (not a test): one 4-wave workgroup
// runs 20 bisection iterations of 16 rows, many times; shader-clock cycles per call, per variant.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -I include tools/probes/bisect_probe.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include "bisect_variants.h"

using namespace fiode_t16;

template <int V>
__global__ __launch_bounds__(256) void k(const float* in, unsigned long long* cyc, float* sink) {
  __shared__ float xt[2][TR][16];
  __shared__ float mu_rec[TR][33];
  const int lane = threadIdx.x & 63, p = threadIdx.x >> 6, q = lane >> 4, j = lane & 15;
  float lower[C], nom[C];
#pragma unroll
  for (int c = 0; c < C; ++c) {
    lower[c] = -0.1f * in[j * C + c];
    nom[c] = in[(j + 16) * C + c];
  }
  int xbuf = 0;
  uint32_t acc = 0;
  float lo = 0.f, hi = 0.f;
  const long long t0 = clock64();
  for (int rep = 0; rep < 1000; ++rep) {
    qp_bracket(lower, nom, lo, hi);
    if (V == 0) acc += qp_bisect_tree(lower, nom, 0, 19, 1e-4f, lo, hi, &mu_rec[j][0], q == 0, true, p, q, j, xt, xbuf);
    if (V == 1) acc += qp_bisect_range2(lower, nom, 0, 19, 1e-4f, lo, hi, &mu_rec[j][0], q == 0, true, q, j);
    if (V == 2) acc += qp_bisect_seq(lower, nom, 0, 19, 1e-4f, lo, hi, &mu_rec[j][0], q == 0, true);
    if (V == 3) {   // eps evaluations only (20 per call), no exchange
      float e = 0.f;
      for (int it = 0; it < 20; ++it) e += qp_eps(lower, nom, lo + 1e-3f * it + e * 1e-9f);
      acc += e > 0.f;
    }
    nom[rep & 7] += 1e-9f * lo;        // keep the loop from being hoisted
  }
  const long long t1 = clock64();
  if (threadIdx.x == 0) cyc[V] = (unsigned long long)(t1 - t0);
  sink[threadIdx.x] = lo + hi + (float)acc;
}

int main() {
  float h[32 * C];
  for (int i = 0; i < 32 * C; ++i) h[i] = 0.05f * (float)((i * 37) % 23) - 0.4f;
  float *din, *sink;
  unsigned long long* dc;
  hipMalloc(&din, sizeof(h));
  hipMalloc(&sink, 256 * 4);
  hipMalloc(&dc, 8 * 8);
  hipMemcpy(din, h, sizeof(h), hipMemcpyHostToDevice);
  for (int warm = 0; warm < 2; ++warm) {
    hipLaunchKernelGGL(k<0>, dim3(1), dim3(256), 0, 0, din, dc, sink);
    hipLaunchKernelGGL(k<1>, dim3(1), dim3(256), 0, 0, din, dc, sink);
    hipLaunchKernelGGL(k<2>, dim3(1), dim3(256), 0, 0, din, dc, sink);
    hipLaunchKernelGGL(k<3>, dim3(1), dim3(256), 0, 0, din, dc, sink);
  }
  unsigned long long c[8];
  hipMemcpy(c, dc, sizeof(c), hipMemcpyDeviceToHost);
  const char* nm[4] = {"tree (4 it/round, LDS + barrier)", "range2 (2 it/round, permlane)", "sequential", "20 eps evals only"};
  for (int v = 0; v < 4; ++v) printf("%-36s %8.1f cycles per 20 iterations\n", nm[v], c[v] / 1000.0);
  return 0;
}
