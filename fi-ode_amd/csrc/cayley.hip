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
#include "gjb.h"
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

// Real n in (16, 128]: the blocked Gauss-Jordan of gjb.h (16-wide pivot blocks inverted in one
// wave's registers, MFMA rank-16 updates, matrix in LDS), one workgroup per matrix.
template <int NP, int NW>
__global__ void __launch_bounds__(64 * NW) k_inv_gjb(int n, const float* __restrict__ in, int64_t in_stride,
                                                     float* __restrict__ out, int64_t out_stride) {
  typedef fiode_gjb::GJB<NP, NW> G;
  extern __shared__ __attribute__((aligned(16))) char gjb_smem[];
  typename G::Smem& sm = *reinterpret_cast<typename G::Smem*>(gjb_smem);
  G::load(sm, in + (int64_t)blockIdx.x * in_stride, n, n);
  __syncthreads();
  G::invert(sm);
  G::store(sm, out + (int64_t)blockIdx.x * out_stride, n, n);
}

template <int NP, int NW>
void launch_gjb(hipStream_t s, int batch, int n, const float* x, int64_t in_stride, float* y, int64_t out_stride) {
  typedef fiode_gjb::GJB<NP, NW> G;
  hipLaunchKernelGGL((k_inv_gjb<NP, NW>), dim3(batch), dim3(G::NT), sizeof(typename G::Smem), s, n, x, in_stride, y,
                     out_stride);
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
  else if (n <= 32) launch_gjb<32, 4>(s, batch, n, x, in_stride, y, out_stride);
  else if (n <= 64) launch_gjb<64, 8>(s, batch, n, x, in_stride, y, out_stride);
  else launch_gjb<128, 16>(s, batch, n, x, in_stride, y, out_stride);
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
//   k_panel_pivot   one workgroup: P = X_KK^-1 by the blocked Gauss-Jordan of gjb.h;
//   k_panel_update  one workgroup per 64 x 64 output tile, ping-pong buffers (no read/write race):
//                   R_Kj = P X_Kj,  X_ij -= X_iK R_Kj,  X_iK <- -X_iK P,  X_Kj <- R_Kj,  X_KK <- P.
// Smaller pivot blocks are cheaper per eliminated column (a Gauss-Jordan round costs ~0.25 us at
// 64, ~0.9 us at 128), and the update is a few us of MFMA on 64 workgroups.
constexpr int PB = 64;

// Batched over matrices m = blockIdx.y (pad, pivot) / blockIdx.z (update): matrix m's buffers sit
// at + m * wstride floats of the workspace, its input / output at + m * n * n.
__global__ void __launch_bounds__(256) k_panel_pad(int n, int np, const float* __restrict__ in, float* __restrict__ out,
                                                   int64_t wstride, const int32_t* __restrict__ skip) {
  if (skip && *skip) return;                  // (uniform: the caller's inverse is already exact)
  const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (idx >= (int64_t)np * np) return;
  const int64_t m = blockIdx.y;
  in += m * n * n;
  out += m * wstride;
  const int i = (int)(idx / np), j = (int)(idx % np);
  out[idx] = (i < n && j < n) ? in[(int64_t)i * n + j] : (i == j ? 1.0f : 0.0f);
}

typedef fiode_gjb::GJB<PB, 8> PivotGJ;
__global__ void __launch_bounds__(PivotGJ::NT) k_panel_pivot(int np, int k0, const float* __restrict__ X,
                                                            int64_t xstride, float* __restrict__ P, int64_t wstride,
                                                            const int32_t* __restrict__ skip) {
  if (skip && *skip) return;
  extern __shared__ __attribute__((aligned(16))) char piv_smem[];
  PivotGJ::Smem& sm = *reinterpret_cast<PivotGJ::Smem*>(piv_smem);
  const int64_t m = blockIdx.x;
  PivotGJ::load(sm, X + m * xstride + (int64_t)k0 * np + k0, PB, np);
  __syncthreads();
  PivotGJ::invert(sm);
  PivotGJ::store(sm, P + m * wstride, PB, PB);
}

// out tile (ib, jb) of the next buffer: 256 threads, MFMA 16x16x4 (wave w: output rows 16w..16w+15,
// all 4 column blocks), operands in LDS as row-major A / column-major B so every k-chunk of 4 is
// one ds_read_b128 (k order permuted: step s of chunk kc uses k = 16 kc + 4q + s at lane q).
constexpr int LDT = PB + 4;
typedef fiode_gjb::f4v f4v;

// acc[bj] += A[16w + i][:] . B^T[16bj + j][:]  (A row-major, BT = B column-major, both [PB][LDT])
__device__ __forceinline__ void tile_gemm(const float (*A)[LDT], const float (*BT)[LDT], int w, int i, int q,
                                          f4v (&acc)[4], float sign) {
#pragma unroll 4
  for (int kc = 0; kc < PB / 16; ++kc) {
    const f4v a4 = *reinterpret_cast<const f4v*>(&A[16 * w + i][16 * kc + 4 * q]) * sign;
#pragma unroll
    for (int bj = 0; bj < 4; ++bj) {
      const f4v b4 = *reinterpret_cast<const f4v*>(&BT[16 * bj + i][16 * kc + 4 * q]);
#pragma unroll
      for (int s = 0; s < 4; ++s) acc[bj] = fiode_gjb::mfma(a4[s], b4[s], acc[bj]);
    }
  }
}

// 64 x 64 block at (r0, c0) of a row-major matrix (row stride ld) -> LDS, row-major or transposed
__device__ __forceinline__ void tile_load(float (*dst)[LDT], const float* __restrict__ src, int64_t ld, bool transpose) {
#pragma unroll
  for (int u = 0; u < PB * PB / 4 / 256; ++u) {
    const int t = threadIdx.x + 256 * u;
    const int r = t / (PB / 4), c4 = (t % (PB / 4)) * 4;
    const f4v v = *reinterpret_cast<const f4v*>(src + (int64_t)r * ld + c4);
    if (transpose) {
#pragma unroll
      for (int e = 0; e < 4; ++e) dst[c4 + e][r] = v[e];
    } else {
      *reinterpret_cast<f4v*>(&dst[r][c4]) = v;
    }
  }
}

// Look-ahead pivot: the workgroup of tile (k0 + PB, k0 + PB) -- the next panel's pivot block,
// which no other tile of this launch reads -- inverts its freshly updated tile in LDS right away
// (gjb.h, 4 waves) and writes P_next, so the next panel needs no pivot launch of its own (the chain
// of a 512 inverse: pivot + 8 updates instead of 8 pivots + 8 updates).  The values are those the
// separate pivot launch would load, so the inverse is bit-identical.
typedef fiode_gjb::GJB<PB, 4> UpdGJ;
static_assert(sizeof(UpdGJ::Smem) <= 3 * PB * LDT * sizeof(float), "pivot scratch fits the update's LDS");

__global__ void __launch_bounds__(256) k_panel_update(int np, int k0, const float* __restrict__ X, int64_t xstride,
                                                      const float* __restrict__ P, float* __restrict__ Y,
                                                      float* __restrict__ final_out, int n, int64_t wstride,
                                                      float* __restrict__ P_next, const int32_t* __restrict__ skip) {
  if (skip && *skip) return;
  __shared__ __attribute__((aligned(16))) float lds[3][PB][LDT];
  float (*sA)[LDT] = lds[0];    // P, or X_iK (row-major A operands)
  float (*sX)[LDT] = lds[1];    // X_iK for the second product
  float (*sB)[LDT] = lds[2];    // column-major B: X_Kj^T or P^T, then R^T
  const int ib = blockIdx.x * PB, jb = blockIdx.y * PB;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, i = lane & 15, q = lane >> 4;
  const int64_t m = blockIdx.z;
  X += m * xstride;
  P += m * wstride;
  Y += m * wstride;
  if (P_next) P_next += m * wstride;
  if (final_out) final_out += m * (int64_t)n * n;
  const bool piv_r = ib == k0, piv_c = jb == k0;
  f4v acc[4];
#pragma unroll
  for (int bj = 0; bj < 4; ++bj) acc[bj] = f4v{0.f, 0.f, 0.f, 0.f};
  if (piv_r && piv_c) {                       // X_KK <- P
#pragma unroll
    for (int bj = 0; bj < 4; ++bj)
#pragma unroll
      for (int r = 0; r < 4; ++r) acc[bj][r] = P[(16 * w + 4 * q + r) * PB + 16 * bj + i];
  } else if (piv_c) {                         // X_iK <- -X_iK P
    tile_load(sA, X + (int64_t)ib * np + k0, np, false);
    tile_load(sB, P, PB, true);
    __syncthreads();
    tile_gemm(sA, sB, w, i, q, acc, -1.0f);
  } else {
    // X_ij (the second product's accumulator) is loaded with the operands, so its global-load
    // latency hides behind the first product instead of following it
    f4v xij[4];
    if (!piv_r) {
#pragma unroll
      for (int bj = 0; bj < 4; ++bj)
#pragma unroll
        for (int r = 0; r < 4; ++r) xij[bj][r] = X[(int64_t)(ib + 16 * w + 4 * q + r) * np + jb + 16 * bj + i];
    }
    tile_load(sA, P, PB, false);              // R_Kj = P X_Kj
    tile_load(sB, X + (int64_t)k0 * np + jb, np, true);
    if (!piv_r) tile_load(sX, X + (int64_t)ib * np + k0, np, false);
    __syncthreads();
    tile_gemm(sA, sB, w, i, q, acc, 1.0f);
    if (!piv_r) {                             // X_ij - X_iK R_Kj
      __syncthreads();                        // every wave is done reading sB
#pragma unroll
      for (int bj = 0; bj < 4; ++bj)          // sB[col][row] = R[row][col]: rows 16w + 4q + r, col 16bj + i
        *reinterpret_cast<f4v*>(&sB[16 * bj + i][16 * w + 4 * q]) = acc[bj];
      __syncthreads();
#pragma unroll
      for (int bj = 0; bj < 4; ++bj) acc[bj] = xij[bj];
      tile_gemm(sX, sB, w, i, q, acc, -1.0f);
    }
  }
#pragma unroll
  for (int bj = 0; bj < 4; ++bj)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int gi = ib + 16 * w + 4 * q + r, gj = jb + 16 * bj + i;
      if (final_out) {
        if (gi < n && gj < n) final_out[(int64_t)gi * n + gj] = acc[bj][r];
      } else {
        Y[(int64_t)gi * np + gj] = acc[bj][r];
      }
    }
  if (P_next && ib == k0 + PB && jb == k0 + PB) {
    UpdGJ::Smem& sm = *reinterpret_cast<UpdGJ::Smem*>(&lds[0][0][0]);
    __syncthreads();                          // every wave is done with the product operands
#pragma unroll
    for (int bj = 0; bj < 4; ++bj)
#pragma unroll
      for (int r = 0; r < 4; ++r) sm.cm[16 * w + 4 * q + r][16 * bj + i] = acc[bj][r];
    __syncthreads();
    UpdGJ::invert(sm);
    UpdGJ::store(sm, P_next, PB, PB);
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
  return (2 * np * np + 2 * (size_t)PB * PB) * sizeof(float);   // ping-pong matrices + two pivot inverses
}

extern "C" int fiode_block_inverse_cond(void* stream, int32_t batch, int32_t n, const float* in, float* out,
                                        void* workspace, size_t workspace_bytes, const int32_t* skip) {
  if (batch < 1 || batch > 65535 || n < 1 || n > FIODE_BLOCK_INV_MAX_N || !in || !out || !workspace)
    return FIODE_EINVAL;
  if (workspace_bytes < (size_t)batch * fiode_block_inverse_workspace_bytes(n)) return FIODE_EWORKSPACE;
  hipStream_t st = (hipStream_t)stream;
  const int np = (n + PB - 1) / PB * PB, nb = np / PB;
  const int64_t wstride = (int64_t)(fiode_block_inverse_workspace_bytes(n) / sizeof(float));
  float* A = (float*)workspace;
  float* B = A + (size_t)np * np;
  float* Pb[2] = {B + (size_t)np * np, B + (size_t)np * np + (size_t)PB * PB};
  // n a multiple of 64 (the 512 x 512 and 128 x 128 systems): the first panel step reads the caller's
  // matrix in place (row stride n = np, matrices n * n apart) -- no padding copy, one launch fewer
  // on the dense maps' forward chain; otherwise it reads the I-padded copy in A
  const bool direct = np == n && (nb > 1 || out != in);     // (one step writing `out` must not read it)
  if (!direct)
    hipLaunchKernelGGL(k_panel_pad, dim3((unsigned)(((int64_t)np * np + 255) / 256), (unsigned)batch), dim3(256), 0,
                       st, n, np, in, A, wstride, skip);
  const float* X = direct ? in : A;
  int64_t xstride = direct ? (int64_t)n * n : wstride;
  // the first pivot block on its own; every later one is inverted by the previous update (look-ahead)
  hipLaunchKernelGGL(k_panel_pivot, dim3((unsigned)batch), dim3(PivotGJ::NT), sizeof(PivotGJ::Smem), st, np, 0, X,
                     xstride, Pb[0], wstride, skip);
  float* Yb[2] = {B, A};                      // ping-pong: a step never writes the matrix it reads
  for (int kb = 0; kb < nb; ++kb) {
    const int k0 = kb * PB;
    const bool last = kb == nb - 1;
    float* Y = Yb[kb & 1];
    hipLaunchKernelGGL(k_panel_update, dim3(nb, nb, (unsigned)batch), dim3(256), 0, st, np, k0, X, xstride,
                       Pb[kb & 1], Y, last ? out : nullptr, n, wstride, last ? nullptr : Pb[(kb + 1) & 1], skip);
    X = Y;
    xstride = wstride;
  }
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? FIODE_OK : FIODE_EHIP + (int)e;
}

extern "C" int fiode_block_inverse_batched(void* stream, int32_t batch, int32_t n, const float* in, float* out,
                                           void* workspace, size_t workspace_bytes) {
  return fiode_block_inverse_cond(stream, batch, n, in, out, workspace, workspace_bytes, nullptr);
}

extern "C" int fiode_block_inverse(void* stream, int32_t n, const float* in, float* out, void* workspace,
                                   size_t workspace_bytes) {
  return fiode_block_inverse_batched(stream, 1, n, in, out, workspace, workspace_bytes);
}
