// Where the time of one 64 x 64 blocked Gauss-Jordan inverse (gjb.h, the panel pivot of the
// 512 x 512 Cayley inverses) goes: in-kernel cycle stamps of load / each round / store (not a test).
// hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/probes/gjb_probe.hip -o /tmp/gjb_probe
#include "../../fi-ode_amd/csrc/gjb.h"
#include <cstdio>
#include <cstdlib>
#include <vector>

using namespace fiode_gjb;
namespace oldgj {
using fiode_gjb::f4v;
// the value of this lane's column in lane row qk (rows of 16 lanes), for a compile-time qk
template <int QK>
__device__ __forceinline__ float from_row(float v, int q) {
  const uint32_t u = __float_as_uint(v);
  const auto s16 = __builtin_amdgcn_permlane16_swap(u, u, false, false);
  const uint32_t x1 = (q & 1) ? s16[0] : s16[1];                // row q ^ 1
  const auto s32 = __builtin_amdgcn_permlane32_swap(u, u, false, false);
  const uint32_t x2 = (q & 2) ? s32[0] : s32[1];                // row q ^ 2
  const auto s32b = __builtin_amdgcn_permlane32_swap(x1, x1, false, false);
  const uint32_t x3 = (q & 2) ? s32b[0] : s32b[1];              // row q ^ 3
  const int d = q ^ QK;
  return __uint_as_float(d == 0 ? u : (d == 1 ? x1 : (d == 2 ? x2 : x3)));
}

template <int K>
__device__ __forceinline__ float newbcast(float v) {             // lane K of this lane's row
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x150 + K, 0xf, 0xf, false));
}

// In-register Gauss-Jordan of one 16 x 16 block held by one wave: lane (c = lane & 15, q = lane >> 4)
// holds x[r] = B[4q + r][c].  Pivot k: column entries of my rows B[4q + r][k] by row_newbcast:k,
// the pivot row entry B[k][c] from lane row k >> 2, the pivot from lane k.
template <int K>
__device__ __forceinline__ void gj16_step(float (&x)[4], int c, int q) {
  constexpr int QK = K >> 2, RK = K & 3;
  float colv[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) colv[r] = newbcast<K>(x[r]);
  const float rowv = from_row<QK>(x[RK], q);
  const float piv = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(rowv), K));
  const float p = __builtin_amdgcn_rcpf(piv);
  const float rp = rowv * p;
  const bool is_col = c == K;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const float upd = is_col ? -(colv[r] * p) : fmaf(-colv[r], rp, x[r]);
    if (r == RK) x[r] = (q == QK) ? (is_col ? p : rp) : upd;
    else x[r] = upd;
  }
}

template <int K = 0>
__device__ __forceinline__ void gj16(float (&x)[4], int c, int q) {
  if constexpr (K < 16) {
    gj16_step<K>(x, c, q);
    gj16<K + 1>(x, c, q);
  }
}

}  // namespace oldgj  (the round-2 gj16: readlane pivot, three swaps)
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s line %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

template <int NW>
__global__ void __launch_bounds__(64 * NW) k_probe(const float* in, float* out, long long* st) {
  typedef GJB<64, NW> G;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  typename G::Smem& sm = *reinterpret_cast<typename G::Smem*>(smem);
  long long t[16];
  int nt = 0;
  t[nt++] = __builtin_readcyclecounter();
  G::load(sm, in, 64, 64);
  __syncthreads();
  t[nt++] = __builtin_readcyclecounter();
  // G::invert with a stamp per phase
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int c = lane & 15, q = lane >> 4;
  if (w == 0) G::invert_block(sm, 0, c, q);
  __syncthreads();
  t[nt++] = __builtin_readcyclecounter();
  for (int kb = 0; kb < G::NB; ++kb) {
    for (int jb = w; jb < G::NB; jb += NW) {
      if (jb == kb) continue;
      f4v pa;
#pragma unroll
      for (int s = 0; s < 4; ++s) pa[s] = sm.cm[16 * kb + 4 * q + s][16 * kb + c];
      const f4v b4 = *reinterpret_cast<const f4v*>(&sm.cm[16 * jb + c][16 * kb + 4 * q]);
      f4v acc = f4v{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < 4; ++s) acc = mfma(pa[s], b4[s], acc);
      *reinterpret_cast<f4v*>(&sm.rt[16 * jb + c][4 * q]) = acc;
    }
    for (int tt = threadIdx.x; tt < 64 * 4; tt += 64 * NW) {
      const int i = tt >> 2, k4 = (tt & 3) * 4;
      *reinterpret_cast<f4v*>(&sm.cb[i][k4]) =
          f4v{sm.cm[16 * kb + k4][i], sm.cm[16 * kb + k4 + 1][i], sm.cm[16 * kb + k4 + 2][i], sm.cm[16 * kb + k4 + 3][i]};
    }
    __syncthreads();
    t[nt++] = __builtin_readcyclecounter();
    const bool ahead = kb + 1 < G::NB;
    if (ahead && w == 0) {
      G::update_block(sm, kb, kb + 1, kb + 1, c, q);
      G::invert_block(sm, kb + 1, c, q);
    } else {
      const int w0 = ahead ? 1 : 0, nw = ahead ? NW - 1 : NW;
      int n = 0;
      for (int ib = 0; ib < G::NB; ++ib)
        for (int jb = 0; jb < G::NB; ++jb) {
          if (ib == kb && jb == kb) continue;
          if (ahead && ib == kb + 1 && jb == kb + 1) continue;
          if (n++ % nw != w - w0) continue;
          if (ib == kb) *G::blk(sm, kb, jb, c, q) = *reinterpret_cast<const f4v*>(&sm.rt[16 * jb + c][4 * q]);
          else G::update_block(sm, kb, ib, jb, c, q);
        }
    }
    __syncthreads();
    t[nt++] = __builtin_readcyclecounter();
  }
  G::store(sm, out, 64, 64);
  __syncthreads();
  t[nt++] = __builtin_readcyclecounter();
  if (threadIdx.x == 0)
    for (int i = 0; i < nt; ++i) st[i] = t[i] - t[0];
}

// one 16 x 16 in-register inversion, repeated: cycles per gj16
template <bool OLD>
__global__ void k_gj16(float* io, long long* st) {
  const int lane = threadIdx.x & 63, c = lane & 15, q = lane >> 4;
  float x[4];
  for (int r = 0; r < 4; ++r) x[r] = io[lane * 4 + r];
  const long long t0 = __builtin_readcyclecounter();
  for (int it = 0; it < 64; ++it) {
    if constexpr (OLD) oldgj::gj16(x, c, q);
    else gj16(x, c, q);
  }
  const long long t1 = __builtin_readcyclecounter();
  for (int r = 0; r < 4; ++r) io[lane * 4 + r] = x[r];
  if (threadIdx.x == 0) st[0] = (t1 - t0) / 64;
}

template <int NW>
void run() {
  std::vector<float> h(64 * 64);
  srand(1);
  for (int i = 0; i < 64; ++i)
    for (int j = 0; j < 64; ++j) h[i * 64 + j] = (i == j ? 1.f : 0.f) + (i < j ? 0.05f : -0.05f) * ((float)rand() / RAND_MAX);
  float *din, *dout; long long* dst;
  CK(hipMalloc(&din, 64 * 64 * 4)); CK(hipMalloc(&dout, 64 * 64 * 4)); CK(hipMalloc(&dst, 16 * 8));
  CK(hipMemcpy(din, h.data(), 64 * 64 * 4, hipMemcpyHostToDevice));
  const size_t lds = sizeof(typename GJB<64, NW>::Smem);
  for (int rep = 0; rep < 5; ++rep) hipLaunchKernelGGL(k_probe<NW>, dim3(1), dim3(64 * NW), lds, 0, din, dout, dst);
  CK(hipDeviceSynchronize());
  long long s[16];
  CK(hipMemcpy(s, dst, sizeof(s), hipMemcpyDeviceToHost));
  printf("NW=%d cycles: load %lld, first pivot %lld", NW, s[1], s[2] - s[1]);
  for (int kb = 0; kb < 4; ++kb) printf(", round %d: R+cb %lld update %lld", kb, s[3 + 2 * kb] - s[2 + 2 * kb], s[4 + 2 * kb] - s[3 + 2 * kb]);
  printf(", store %lld, total %lld\n", s[11] - s[10], s[11]);
  hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  CK(hipEventRecord(a));
  for (int rep = 0; rep < 200; ++rep) hipLaunchKernelGGL(k_probe<NW>, dim3(1), dim3(64 * NW), lds, 0, din, dout, dst);
  CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
  float ms; CK(hipEventElapsedTime(&ms, a, b));
  printf("NW=%d us per launch (back-to-back): %.2f\n", NW, ms * 1e3f / 200);
}

int main() {
  run<4>();
  run<8>();
  float* io; long long* st;
  CK(hipMalloc(&io, 64 * 4 * 4)); CK(hipMalloc(&st, 8));
  std::vector<float> h(256);
  for (int l = 0; l < 64; ++l) for (int r = 0; r < 4; ++r) { int c = l & 15, row = 4 * (l >> 4) + r; h[l * 4 + r] = (row == c ? 1.f : 0.f) + 0.01f * (row - c); }
  CK(hipMemcpy(io, h.data(), 256 * 4, hipMemcpyHostToDevice));
  for (int old = 0; old < 2; ++old) {
    CK(hipMemcpy(io, h.data(), 256 * 4, hipMemcpyHostToDevice));
    for (int rep = 0; rep < 2; ++rep) {
      if (old) hipLaunchKernelGGL(k_gj16<true>, dim3(1), dim3(64), 0, 0, io, st);
      else hipLaunchKernelGGL(k_gj16<false>, dim3(1), dim3(64), 0, 0, io, st);
    }
    CK(hipDeviceSynchronize());
    long long c; CK(hipMemcpy(&c, st, 8, hipMemcpyDeviceToHost));
    std::vector<float> o(256); CK(hipMemcpy(o.data(), io, 256 * 4, hipMemcpyDeviceToHost));
    double cs = 0; for (float v : o) cs += v;
    printf("gj16 %s: %lld cycles per 16x16 inversion (checksum %.6f)\n", old ? "old" : "new", c, cs);
  }
  return 0;
}
