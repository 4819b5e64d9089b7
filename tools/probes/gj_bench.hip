// Micro-benchmark: register Gauss-Jordan variants (old k_inv_gj of cayley.hip vs fiode_gj::GJ)
// on positive-real test matrices; prints us per launch and the max |difference| (not a test).
#include "../../fi-ode_amd/csrc/cayley.hip"  // (k_inv_gj is now the gj.h kernel: old == new)
#include "../../fi-ode_amd/csrc/gj.h"
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <cmath>

template <class Ops, int NP, int TR, int TC, int NT>
__global__ void __launch_bounds__(NT) k_new(int n, const typename Ops::T* in, typename Ops::T* out) {
  typedef fiode_gj::GJ<Ops, NP, TR, TC> G;
  __shared__ typename G::Smem sm;
  typename Ops::T a[TR][TC];
  G::load(a, in + (int64_t)blockIdx.x * n * n, n, n);
  G::invert(a, n, sm);
  G::store(a, out + (int64_t)blockIdx.x * n * n, n, n);
}

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s line %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

template <class T> static T mk(float re, float im);
template <> float mk<float>(float re, float) { return re; }
template <> float2 mk<float2>(float re, float im) { return make_float2(re, im); }
static float dif(float a, float b) { return fabsf(a - b); }
static float dif(float2 a, float2 b) { return fabsf(a.x - b.x) + fabsf(a.y - b.y); }

template <class Ops, int NP, int TR, int TC>
void run(const char* tag, int n, int batch) {
  typedef typename Ops::T T;
  std::vector<T> h((size_t)batch * n * n);
  srand(1);
  auto rnd = [] { return (float)rand() / RAND_MAX - 0.5f; };
  for (int b = 0; b < batch; ++b)
    for (int i = 0; i < n; ++i)
      for (int j = 0; j < n; ++j) {
        float re = (i == j ? 1.0f : 0.0f) + 0.3f * rnd() / sqrtf((float)n) + (i < j ? 0.5f : -0.5f) * rnd();
        h[((size_t)b * n + i) * n + j] = mk<T>(re, 0.2f * rnd());
      }
  T *din, *d0, *d1;
  size_t bytes = h.size() * sizeof(T);
  CK(hipMalloc(&din, bytes)); CK(hipMalloc(&d0, bytes)); CK(hipMalloc(&d1, bytes));
  CK(hipMemcpy(din, h.data(), bytes, hipMemcpyHostToDevice));
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  const int reps = 50;
  float t_old = 0, t_new = 0;
  for (int pass = 0; pass < 2; ++pass) {
    CK(hipEventRecord(e0));
    for (int r = 0; r < reps; ++r) launch_inv<Ops>(0, batch, n, din, (int64_t)n * n, d0, (int64_t)n * n);
    CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    CK(hipEventElapsedTime(&t_old, e0, e1));
    typedef fiode_gj::GJ<Ops, NP, TR, TC> G;
    CK(hipEventRecord(e0));
    for (int r = 0; r < reps; ++r) hipLaunchKernelGGL((k_new<Ops, NP, TR, TC, G::NT>), dim3(batch), dim3(G::NT), 0, 0, n, din, d1);
    CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    CK(hipEventElapsedTime(&t_new, e0, e1));
  }
  CK(hipGetLastError());
  std::vector<T> o0(h.size()), o1(h.size());
  CK(hipMemcpy(o0.data(), d0, bytes, hipMemcpyDeviceToHost));
  CK(hipMemcpy(o1.data(), d1, bytes, hipMemcpyDeviceToHost));
  float md = 0, mx = 0;
  for (size_t i = 0; i < h.size(); ++i) { md = fmaxf(md, dif(o0[i], o1[i])); mx = fmaxf(mx, dif(o0[i], mk<T>(0, 0))); }
  printf("%-8s n=%3d batch=%4d NP=%3d tile %dx%d NT=%4d | old %8.2f us  new %8.2f us | max|diff| %.2e (max|inv| %.2e)\n",
         tag, n, batch, NP, TR, TC, fiode_gj::GJ<Ops, NP, TR, TC>::NT, t_old * 1e3 / reps, t_new * 1e3 / reps, md, mx);
  CK(hipFree(din)); CK(hipFree(d0)); CK(hipFree(d1));
}

int main() {
  using fiode_gj::RealOps; using fiode_gj::ComplexOps;
  run<RealOps, 128, 4, 8>("real", 128, 1);
  run<RealOps, 128, 8, 8>("real", 128, 1);
  run<RealOps, 128, 8, 4>("real", 128, 1);
  run<RealOps, 128, 4, 4>("real", 128, 1);

  run<RealOps, 128, 4, 8>("real", 128, 8);
  run<RealOps, 128, 8, 8>("real", 128, 8);
  run<RealOps, 64, 4, 4>("real", 64, 1);
  run<RealOps, 32, 4, 4>("real", 32, 1);
  run<RealOps, 32, 2, 2>("real", 32, 1);
  run<RealOps, 16, 2, 2>("real", 10, 3);
  run<ComplexOps, 64, 4, 4>("complex", 64, 40);
  run<ComplexOps, 64, 8, 4>("complex", 64, 40);
  run<ComplexOps, 64, 4, 8>("complex", 64, 40);
  run<ComplexOps, 64, 2, 4>("complex", 64, 40);
  run<ComplexOps, 64, 2, 2>("complex", 64, 40);

  run<ComplexOps, 32, 4, 4>("complex", 32, 144);
  run<ComplexOps, 32, 2, 4>("complex", 32, 144);
  run<ComplexOps, 32, 2, 2>("complex", 32, 144);
  run<ComplexOps, 16, 2, 2>("complex", 3, 544);
  return 0;
}
