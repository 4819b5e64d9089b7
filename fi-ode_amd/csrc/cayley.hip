// Batched matrix inverse for the Cayley parametrisation (gfx950).
//
// Every Cayley map in the model -- the 4 dynamics CayleyLinears (classification.py:282-293,
// convert_cayley), the backbone CayleyLinears and the per-frequency channel matrices of the
// CayleyConvs -- needs (I + A)^-1 with A = U - U^H + V^H V.  The Hermitian part of I + A is
// I + V^H V >= I, so (a) every pivot of Gauss-Jordan elimination in natural order has real part
// >= 1 (no pivoting, no singular case, ||(I+A)^-1||_2 <= 1) and (b) the elimination is a fixed
// sequence of rank-1 updates with no data-dependent control flow and no host synchronisation
// (torch.linalg.inv runs getrf + getrs with pivot search and an info check that syncs the host).
//
// One workgroup per matrix, the matrix resident in REGISTERS (<= 32 elements per thread), n <= 128,
// real f32 or complex64, eliminated two pivots per round (gj.h: 2 x 2 pivot blocks, closed-form
// inverse; the pivot blocks of a positive-real matrix are positive-real, so never singular).
// Larger matrices (the 512 x 512 backbone maps) are inverted block-wise on the host side
// (fiode_amd/cayley.py) with this kernel on the diagonal blocks.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "common.h"
#include "gj.h"
#include "fiode.h"

namespace {

using fiode_gj::ComplexOps;
using fiode_gj::RealOps;

template <class Ops, int NP, int TR, int TC, int NT>
__global__ void __launch_bounds__(NT) k_inv_gj(int n, const typename Ops::T* __restrict__ in, int64_t in_stride,
                                               typename Ops::T* __restrict__ out, int64_t out_stride) {
  typedef fiode_gj::GJ<Ops, NP, TR, TC> G;
  static_assert(G::NT == NT, "thread count");
  __shared__ typename G::Smem sm;
  typename Ops::T a[TR][TC];
  G::load(a, in + (int64_t)blockIdx.x * in_stride, n, n);
  G::invert(a, n, sm);
  G::store(a, out + (int64_t)blockIdx.x * out_stride, n, n);
}

// Tile shapes measured on MI355X (tools/gj_bench.hip): us per launch, old 2x2-pivot kernel ->
// this one: real 128: 74.6 -> 58.9 (8x4, 512 threads); real 64: 23.0 -> 16.3; real 32: 11.8 -> 6.5;
// complex 64 x 40: 60.5 -> 48.5 (2x4, 512 threads); complex 32 x 144: 22.4 -> 12.0 (2x2, 256).
template <class Ops>
int launch_inv(hipStream_t s, int batch, int n, const void* in, int64_t in_stride, void* out, int64_t out_stride);

template <>
int launch_inv<RealOps>(hipStream_t s, int batch, int n, const void* in, int64_t in_stride, void* out,
                        int64_t out_stride) {
  const float* x = (const float*)in;
  float* y = (float*)out;
  if (n <= 16) k_inv_gj<RealOps, 16, 2, 2, 64><<<batch, 64, 0, s>>>(n, x, in_stride, y, out_stride);
  else if (n <= 32) k_inv_gj<RealOps, 32, 2, 2, 256><<<batch, 256, 0, s>>>(n, x, in_stride, y, out_stride);
  else if (n <= 64) k_inv_gj<RealOps, 64, 4, 4, 256><<<batch, 256, 0, s>>>(n, x, in_stride, y, out_stride);
  else k_inv_gj<RealOps, 128, 8, 4, 512><<<batch, 512, 0, s>>>(n, x, in_stride, y, out_stride);
  return 0;
}

template <>
int launch_inv<ComplexOps>(hipStream_t s, int batch, int n, const void* in, int64_t in_stride, void* out,
                           int64_t out_stride) {
  const float2* x = (const float2*)in;
  float2* y = (float2*)out;
  if (n <= 16) k_inv_gj<ComplexOps, 16, 2, 2, 64><<<batch, 64, 0, s>>>(n, x, in_stride, y, out_stride);
  else if (n <= 32) k_inv_gj<ComplexOps, 32, 2, 2, 256><<<batch, 256, 0, s>>>(n, x, in_stride, y, out_stride);
  else if (n <= 64) k_inv_gj<ComplexOps, 64, 2, 4, 512><<<batch, 512, 0, s>>>(n, x, in_stride, y, out_stride);
  else k_inv_gj<ComplexOps, 128, 4, 4, 1024><<<batch, 1024, 0, s>>>(n, x, in_stride, y, out_stride);
  return 0;
}

// ---- large real inverses: block Gauss-Jordan over 64-wide panels --------------------------------
// For n > 64 (the 512 x 512 backbone CayleyLinears, the 128 x 128 dynamics map) the matrix lives in
// HBM (padded with I to a multiple of 64) and each of the n/64 panel steps is two launches:
//   k_panel_pivot   one workgroup: P = X_KK^-1 by the register Gauss-Jordan above (16 us at 64);
//   k_panel_update  one workgroup per 64 x 64 output tile, ping-pong buffers (no read/write race):
//                   R_Kj = P X_Kj,  X_ij -= X_iK R_Kj,  X_iK <- -X_iK P,  X_Kj <- R_Kj,  X_KK <- P.
// Smaller pivot blocks are cheaper per eliminated column (a Gauss-Jordan round costs ~0.25 us at
// 64, ~0.9 us at 128), and the update is a few us of LDS-tiled FMA on 64 workgroups.
constexpr int PB = 64;

// Batched over matrices m = blockIdx.y (pad, pivot) / blockIdx.z (update): matrix m's buffers sit
// at + m * wstride floats of the workspace, its input / output at + m * n * n.
__global__ void __launch_bounds__(256) k_panel_pad(int n, int np, const float* __restrict__ in, float* __restrict__ out,
                                                   int64_t wstride) {
  const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (idx >= (int64_t)np * np) return;
  const int64_t m = blockIdx.y;
  in += m * n * n;
  out += m * wstride;
  const int i = (int)(idx / np), j = (int)(idx % np);
  out[idx] = (i < n && j < n) ? in[(int64_t)i * n + j] : (i == j ? 1.0f : 0.0f);
}

__global__ void __launch_bounds__(256) k_panel_pivot(int np, int k0, const float* __restrict__ X, float* __restrict__ P,
                                                     int64_t wstride) {
  typedef fiode_gj::GJ<RealOps, PB, 4, 4> G;
  __shared__ typename G::Smem sm;
  float a[4][4];
  const int64_t m = blockIdx.x;
  G::load(a, X + m * wstride + (int64_t)k0 * np + k0, PB, np);
  G::invert(a, PB, sm);
  G::store(a, P + m * wstride, PB, PB);
}

// out tile (ib, jb) of the next buffer; 256 threads, 4 x 4 outputs each
__global__ void __launch_bounds__(256) k_panel_update(int np, int k0, const float* __restrict__ X,
                                                      const float* __restrict__ P, float* __restrict__ Y,
                                                      float* __restrict__ final_out, int n, int64_t wstride) {
  __shared__ float sP[PB][PB + 4];
  __shared__ float sA[PB][PB + 4];      // X_iK (rows of the tile, pivot columns)
  __shared__ float sB[PB][PB + 4];      // X_Kj, then R_Kj
  const int ib = blockIdx.x * PB, jb = blockIdx.y * PB, tid = threadIdx.x;
  const int64_t m = blockIdx.z;
  X += m * wstride;
  P += m * wstride;
  Y += m * wstride;
  if (final_out) final_out += m * (int64_t)n * n;
  const bool piv_r = ib == k0, piv_c = jb == k0;
#pragma unroll 16
  for (int idx = tid; idx < PB * PB; idx += 256) {     // 16 trips: all loads in flight together
    const int r = idx / PB, c = idx % PB;
    sP[r][c] = P[idx];
    sA[r][c] = X[(int64_t)(ib + r) * np + k0 + c];
    sB[r][c] = X[(int64_t)(k0 + r) * np + jb + c];
  }
  __syncthreads();
  const int tr = (tid / 16) * 4, tc = (tid % 16) * 4;
  float acc[4][4];
  auto gemm = [&](float (*A)[PB + 4], float (*B)[PB + 4]) {
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int c = 0; c < 4; ++c) acc[r][c] = 0.f;
#pragma unroll 8
    for (int k = 0; k < PB; ++k) {
      float x[4], y[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) x[r] = A[tr + r][k];
#pragma unroll
      for (int c = 0; c < 4; ++c) y[c] = B[k][tc + c];
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int c = 0; c < 4; ++c) acc[r][c] = fmaf(x[r], y[c], acc[r][c]);
    }
  };
  float o[4][4];
  if (piv_c) {
    if (piv_r) {
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int c = 0; c < 4; ++c) o[r][c] = sP[tr + r][tc + c];
    } else {
      gemm(sA, sP);                       // -X_iK P
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int c = 0; c < 4; ++c) o[r][c] = -acc[r][c];
    }
  } else {
    gemm(sP, sB);                         // R_Kj = P X_Kj
    if (piv_r) {
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int c = 0; c < 4; ++c) o[r][c] = acc[r][c];
    } else {
      __syncthreads();
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int c = 0; c < 4; ++c) sB[tr + r][tc + c] = acc[r][c];
      __syncthreads();
      gemm(sA, sB);                       // X_ij - X_iK R_Kj
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int c = 0; c < 4; ++c) o[r][c] = X[(int64_t)(ib + tr + r) * np + jb + tc + c] - acc[r][c];
    }
  }
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const int i = ib + tr + r, j = jb + tc + c;
      if (final_out) {
        if (i < n && j < n) final_out[(int64_t)i * n + j] = o[r][c];
      } else {
        Y[(int64_t)i * np + j] = o[r][c];
      }
    }
}

}  // namespace

extern "C" int fiode_batched_inverse(void* stream, int32_t dtype, int32_t batch, int32_t n, const void* in,
                                     int64_t in_stride, void* out, int64_t out_stride) {
  if (batch < 0 || n < 1 || n > FIODE_INV_MAX_N || (dtype != FIODE_DTYPE_F32 && dtype != FIODE_DTYPE_C64))
    return FIODE_EINVAL;
  if (!in || !out) return batch == 0 ? FIODE_OK : FIODE_EINVAL;
  if (in_stride < (int64_t)n * n || out_stride < (int64_t)n * n) return FIODE_ESHAPE;
  if (batch == 0) return FIODE_OK;
  hipStream_t s = (hipStream_t)stream;
  if (dtype == FIODE_DTYPE_F32) launch_inv<RealOps>(s, batch, n, in, in_stride, out, out_stride);
  else launch_inv<ComplexOps>(s, batch, n, in, in_stride, out, out_stride);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? FIODE_OK : FIODE_EHIP + (int)e;
}

extern "C" size_t fiode_block_inverse_workspace_bytes(int32_t n) {
  if (n < 1) return 0;
  const size_t np = (size_t)((n + PB - 1) / PB) * PB;
  return (2 * np * np + (size_t)PB * PB) * sizeof(float);
}

extern "C" int fiode_block_inverse_batched(void* stream, int32_t batch, int32_t n, const float* in, float* out,
                                           void* workspace, size_t workspace_bytes) {
  if (batch < 1 || batch > 65535 || n < 1 || n > FIODE_BLOCK_INV_MAX_N || !in || !out || !workspace)
    return FIODE_EINVAL;
  if (workspace_bytes < (size_t)batch * fiode_block_inverse_workspace_bytes(n)) return FIODE_EWORKSPACE;
  hipStream_t st = (hipStream_t)stream;
  const int np = (n + PB - 1) / PB * PB, nb = np / PB;
  const int64_t wstride = (int64_t)(fiode_block_inverse_workspace_bytes(n) / sizeof(float));
  float* A = (float*)workspace;
  float* B = A + (size_t)np * np;
  float* P = B + (size_t)np * np;
  hipLaunchKernelGGL(k_panel_pad, dim3((unsigned)(((int64_t)np * np + 255) / 256), (unsigned)batch), dim3(256), 0, st,
                     n, np, in, A, wstride);
  for (int kb = 0; kb < nb; ++kb) {
    const int k0 = kb * PB;
    hipLaunchKernelGGL(k_panel_pivot, dim3((unsigned)batch), dim3(256), 0, st, np, k0, A, P, wstride);
    const bool last = kb == nb - 1;
    hipLaunchKernelGGL(k_panel_update, dim3(nb, nb, (unsigned)batch), dim3(256), 0, st, np, k0, A, P, B,
                       last ? out : nullptr, n, wstride);
    float* t = A;
    A = B;
    B = t;
  }
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? FIODE_OK : FIODE_EHIP + (int)e;
}

extern "C" int fiode_block_inverse(void* stream, int32_t n, const float* in, float* out, void* workspace,
                                   size_t workspace_bytes) {
  return fiode_block_inverse_batched(stream, 1, n, in, out, workspace, workspace_bytes);
}
