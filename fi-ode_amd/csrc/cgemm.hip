// Batched complex64 GEMM of the spectral convolutions (gfx950): the per-frequency channel products
// of CayleyConv.forward_hwcb (fiode_amd/cayley.py _SpectralConvFn; the absent libs/ortho_conv of
// models.py:12-14) -- Y[f] = Q[f] X[f] in the forward and dL/dX[f] = Q[f]^H G[f] in the backward,
// Q [F][cout][cin], X / G [F][C][B].  These are small GEMMs in a large batch (M = 32-256 channels,
// N = B = 128, K = 3-256, F = 40-544 frequencies): the library's solutions for them took 128 x 64
// tiles, one workgroup per frequency, and ran at 1-16 TFLOP/s (41 us for the n = 8 layer's forward).
//
// Here: a 32 x 32 complex output tile per workgroup (grid N/32 x M/32 x F), four waves of 16 x 16 on
// v_mfma_f32_16x16x4_f32 with the real and imaginary accumulators apart:
//   Cr += Ar Br + (-Ai) Bi,   Ci += Ar Bi + Ai Br        (4 MFMAs per 4 complex k)
// K in chunks of 32 staged through LDS, with the global loads two chunks ahead in registers.  LDS row strides: A 34 complex (lanes i = 0..15 at k, k+1 of one
// ds_read_b64 group land on 64 distinct banks), B 48 (rows k and k+1 of a group half a bank row
// apart).  Out-of-range rows / columns / k are zeros in LDS and skipped at the store, so any shape
// works (K = 3 for the 3-channel input layer).  ca: A is conj(Q)^T, read from Q [F][K][M]; cb: B is
// conj(X)^T, read from X [F][N][K] (the weight gradient G X^H, B row stride 49 then: the stores of a
// k-run spread over the banks); scale: C[f] *= scale[f] (the rfft gradient weights).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "common.h"
#include "fiode.h"

namespace {

typedef float2 c32;
typedef float f4v __attribute__((ext_vector_type(4)));

constexpr int TM = 32, TN = 32, KC = 32;
constexpr int SA = KC + 2;       // A chunk [TM][SA] (complex)
template <bool CB>
constexpr int sbs() { return CB ? TN + 17 : TN + 16; }   // B chunk [KC][SB] (complex)
constexpr int SBMAX = TN + 17;
constexpr int NTH = 256;
constexpr int PER = TM * KC / NTH;   // complex elements per thread per operand chunk (4)
constexpr int KS = KC / 4;           // MFMA k-steps per full chunk
static_assert(TM == TN, "one load shape for both operands");

struct CgArgs {
  int M, N, K;
  const float* scale;        // [F] or null
  const c32* A;
  const c32* B;
  c32* C;
  int64_t sa, sb, sc;        // per-frequency strides (complex elements)
};

__device__ __forceinline__ f4v mfma(float a, float b, f4v c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// every load is issued (out-of-range elements read element 0 of the operand and are replaced by 0):
// no per-element branch between the loads, so all of a thread's loads are in flight together
template <bool CA, bool CB>
__device__ __forceinline__ void load_chunk(const CgArgs& a, const c32* A, const c32* B, int m0, int n0, int k0,
                                           c32 (&ra)[PER], c32 (&rb)[PER]) {
  const int tid = threadIdx.x;
#pragma unroll
  for (int q = 0; q < PER; ++q) {
    const int idx = tid + NTH * q;
    if (CA) {              // opA[m][k] = conj(Q[k][m]): rows k of Q, contiguous along m
      const int k = idx / TM, m = idx % TM;
      const bool in = m0 + m < a.M && k0 + k < a.K;
      const c32 v = A[in ? (int64_t)(k0 + k) * a.M + m0 + m : 0];
      ra[q] = in ? make_float2(v.x, -v.y) : make_float2(0.f, 0.f);
    } else {               // opA[m][k] = A[m][k]: contiguous along k
      const int m = idx / KC, k = idx % KC;
      const bool in = m0 + m < a.M && k0 + k < a.K;
      const c32 v = A[in ? (int64_t)(m0 + m) * a.K + k0 + k : 0];
      ra[q] = in ? v : make_float2(0.f, 0.f);
    }
    if (CB) {              // opB[k][n] = conj(X[n][k]): rows n of X, contiguous along k
      const int n = idx / KC, k = idx % KC;
      const bool in = k0 + k < a.K && n0 + n < a.N;
      const c32 v = B[in ? (int64_t)(n0 + n) * a.K + k0 + k : 0];
      rb[q] = in ? make_float2(v.x, -v.y) : make_float2(0.f, 0.f);
    } else {
      const int k = idx / TN, n = idx % TN;
      const bool in = k0 + k < a.K && n0 + n < a.N;
      const c32 v = B[in ? (int64_t)(k0 + k) * a.N + n0 + n : 0];
      rb[q] = in ? v : make_float2(0.f, 0.f);
    }
  }
}

template <bool CA, bool CB>
__device__ __forceinline__ void store_chunk(c32* As, c32* Bs, const c32 (&ra)[PER], const c32 (&rb)[PER]) {
  const int tid = threadIdx.x;
#pragma unroll
  for (int q = 0; q < PER; ++q) {
    const int idx = tid + NTH * q;
    if (CA) {
      const int k = idx / TM, m = idx % TM;
      As[m * SA + k] = ra[q];
    } else {
      const int m = idx / KC, k = idx % KC;
      As[m * SA + k] = ra[q];
    }
    if (CB) {
      const int n = idx / KC, k = idx % KC;
      Bs[k * sbs<CB>() + n] = rb[q];
    } else {
      const int k = idx / TN, n = idx % TN;
      Bs[k * sbs<CB>() + n] = rb[q];
    }
  }
}

// one chunk's MFMAs from LDS (As / Bs at the chunk's buffer): a full chunk reads all its operands
// first and alternates two accumulator pairs; the K tail runs the plain loop
template <int SB>
__device__ __forceinline__ void chunk_mfma(const c32* As, const c32* Bs, int ks, int lane, int wm, int wn, f4v& cr0,
                                           f4v& ci0, f4v& cr1, f4v& ci1) {
  const c32* as = As + (wm + (lane & 15)) * SA + (lane >> 4);
  const c32* bs = Bs + (lane >> 4) * SB + wn + (lane & 15);
  if (ks == KS) {
    c32 av[KS], bv[KS];
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      av[s] = as[4 * s];
      bv[s] = bs[4 * s * SB];
    }
#pragma unroll
    for (int s = 0; s < KS; s += 2) {
      cr0 = mfma(av[s].x, bv[s].x, cr0);
      ci0 = mfma(av[s].x, bv[s].y, ci0);
      cr1 = mfma(av[s + 1].x, bv[s + 1].x, cr1);
      ci1 = mfma(av[s + 1].x, bv[s + 1].y, ci1);
      cr0 = mfma(-av[s].y, bv[s].y, cr0);
      ci0 = mfma(av[s].y, bv[s].x, ci0);
      cr1 = mfma(-av[s + 1].y, bv[s + 1].y, cr1);
      ci1 = mfma(av[s + 1].y, bv[s + 1].x, ci1);
    }
  } else {
    for (int s = 0; s < ks; ++s) {
      const c32 av = as[4 * s], bv = bs[4 * s * SB];
      cr0 = mfma(av.x, bv.x, cr0);
      ci0 = mfma(av.x, bv.y, ci0);
      cr0 = mfma(-av.y, bv.y, cr0);
      ci0 = mfma(av.y, bv.x, ci0);
    }
  }
}

// One LDS buffer (21 KB: seven workgroups per CU -- the many-tile products run in one round) and two
// register sets: chunk c + 2's global loads are issued when chunk c's MFMAs start.
template <bool CA, bool CB>
__global__ __launch_bounds__(NTH) void k_cgemm(CgArgs a) {
  constexpr int SB = sbs<CB>();
  __shared__ c32 As[TM * SA];
  __shared__ c32 Bs[KC * SBMAX];
  const int f = blockIdx.z;
  const int m0 = blockIdx.y * TM, n0 = blockIdx.x * TN;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int wm = (w >> 1) * 16, wn = (w & 1) * 16;
  const c32* A = a.A + (int64_t)f * a.sa;
  const c32* B = a.B + (int64_t)f * a.sb;
  const int nch = (a.K + KC - 1) / KC;       // >= 1 (K = 0 never launches)
  auto steps = [&](int c) { return (min(KC, a.K - c * KC) + 3) >> 2; };   // 4 complex k per step
  c32 ra0[PER], rb0[PER], ra1[PER], rb1[PER];
  load_chunk<CA, CB>(a, A, B, m0, n0, 0, ra0, rb0);
  if (nch > 1) load_chunk<CA, CB>(a, A, B, m0, n0, KC, ra1, rb1);
  store_chunk<CA, CB>(As, Bs, ra0, rb0);
  __syncthreads();
  const f4v z4 = {0.f, 0.f, 0.f, 0.f};
  f4v cr0 = z4, ci0 = z4, cr1 = z4, ci1 = z4;     // even / odd k-steps of a chunk
  for (int c = 0; c < nch; c += 2) {
    if (c + 2 < nch) load_chunk<CA, CB>(a, A, B, m0, n0, (c + 2) * KC, ra0, rb0);
    chunk_mfma<SB>(As, Bs, steps(c), lane, wm, wn, cr0, ci0, cr1, ci1);
    if (c + 1 >= nch) break;
    __syncthreads();
    store_chunk<CA, CB>(As, Bs, ra1, rb1);
    __syncthreads();
    if (c + 3 < nch) load_chunk<CA, CB>(a, A, B, m0, n0, (c + 3) * KC, ra1, rb1);
    chunk_mfma<SB>(As, Bs, steps(c + 1), lane, wm, wn, cr0, ci0, cr1, ci1);
    if (c + 2 >= nch) break;
    __syncthreads();
    store_chunk<CA, CB>(As, Bs, ra0, rb0);
    __syncthreads();
  }
  f4v cr = cr0 + cr1, ci = ci0 + ci1;
  if (a.scale) {
    const float sc = a.scale[f];
    cr *= sc;
    ci *= sc;
  }
  // C/D layout of 16x16x4: lane l holds rows 4 (l >> 4) + r, column l & 15
  c32* C = a.C + (int64_t)f * a.sc;
  const int n = n0 + wn + (lane & 15);
  if (n < a.N) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int m = m0 + wm + 4 * (lane >> 4) + r;
      if (m < a.M) C[(int64_t)m * a.N + n] = make_float2(cr[r], ci[r]);
    }
  }
}

}  // namespace

extern "C" int fiode_cgemm(void* stream, int32_t F, int32_t M, int32_t N, int32_t K, int32_t conj_trans_a,
                           int32_t conj_trans_b, const float* scale, const void* A, const void* B, void* C) {
  if (F < 0 || M < 0 || N < 0 || K < 0) return FIODE_EINVAL;
  if (F == 0 || M == 0 || N == 0) return FIODE_OK;
  if (!C || (K > 0 && (!A || !B))) return FIODE_EINVAL;     // K = 0: C = 0 (empty operands may be null)
  if ((int64_t)F > 65535) return FIODE_ESHAPE;
  if (conj_trans_a && conj_trans_b) return FIODE_ESHAPE;    // not needed by the convs: not instantiated
  CgArgs a;
  a.M = M;
  a.N = N;
  a.K = K;
  a.scale = scale;
  a.A = (const c32*)A;
  a.B = (const c32*)B;
  a.C = (c32*)C;
  a.sa = (int64_t)M * K;
  a.sb = (int64_t)K * N;
  a.sc = (int64_t)M * N;
  hipStream_t st = (hipStream_t)stream;
  const dim3 grid((N + TN - 1) / TN, (M + TM - 1) / TM, F);
  if (K == 0) return hipMemsetAsync(C, 0, (size_t)F * M * N * sizeof(c32), st) == hipSuccess ? FIODE_OK : FIODE_EHIP;
  if (conj_trans_a) hipLaunchKernelGGL((k_cgemm<true, false>), grid, dim3(NTH), 0, st, a);
  else if (conj_trans_b) hipLaunchKernelGGL((k_cgemm<false, true>), grid, dim3(NTH), 0, st, a);
  else hipLaunchKernelGGL((k_cgemm<false, false>), grid, dim3(NTH), 0, st, a);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? FIODE_OK : FIODE_EHIP + (int)e;
}
