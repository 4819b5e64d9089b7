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
// real f32 or complex64, eliminated two pivots per round (2 x 2 pivot blocks, closed-form
// inverse; the pivot blocks of a positive-real matrix are positive-real, so never singular).
// Larger matrices (the 512 x 512 backbone maps) are inverted block-wise on the host side
// (fiode_amd/cayley.py) with this kernel on the diagonal blocks.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "common.h"
#include "fiode.h"

namespace {

// Element arithmetic for the two storage types (real f32, complex64 interleaved).
struct RealOps {
  typedef float T;
  static __device__ __forceinline__ T mul(T a, T b) { return a * b; }
  static __device__ __forceinline__ T sub_mul(T o, T c, T r) { return fmaf(-c, r, o); }
  static __device__ __forceinline__ T ident(bool d) { return d ? 1.0f : 0.0f; }
  static __device__ __forceinline__ T add(T a, T b) { return a + b; }
  static __device__ __forceinline__ T sub(T a, T b) { return a - b; }
  static __device__ __forceinline__ T neg(T a) { return -a; }
  static __device__ __forceinline__ T recip(T d) { return 1.0f / d; }
};
struct ComplexOps {
  typedef float2 T;
  static __device__ __forceinline__ T mul(T a, T b) {
    return make_float2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x);
  }
  static __device__ __forceinline__ T sub_mul(T o, T c, T r) {   // o - c r, fused
    return make_float2(fmaf(c.y, r.y, fmaf(-c.x, r.x, o.x)), fmaf(-c.y, r.x, fmaf(-c.x, r.y, o.y)));
  }
  static __device__ __forceinline__ T ident(bool d) { return make_float2(d ? 1.0f : 0.0f, 0.0f); }
  static __device__ __forceinline__ T add(T a, T b) { return make_float2(a.x + b.x, a.y + b.y); }
  static __device__ __forceinline__ T sub(T a, T b) { return make_float2(a.x - b.x, a.y - b.y); }
  static __device__ __forceinline__ T neg(T a) { return make_float2(-a.x, -a.y); }
  static __device__ __forceinline__ T recip(T d) {
    const float den = d.x * d.x + d.y * d.y;
    return make_float2(d.x / den, -d.y / den);
  }
};

// Register-tiled block Gauss-Jordan on the matrix padded to NP x NP with the identity (the
// padded block stays I).  Thread t owns a TR x TC tile (rows ti*TR.., cols tj*TC..).  One round
// eliminates the 2 x 2 pivot block K = {k, k+1}: the threads holding rows / columns K stage them in
// LDS (double-buffered by round parity: one barrier per round), every thread inverts the 2 x 2
// pivot block in closed form (P = A_KK^-1), forms R = P A_K,j for its columns and applies
//   a_ij -= a_iK R_Kj  (i, j not in K),  a_iK <- -a_iK P,  a_Kj <- R_Kj,  a_KK <- P.
// n/2 rounds of latency instead of n (the elimination is a latency chain: ~0.5 us per round).
template <class Ops, int NP, int NT, int TR, int TC>
__global__ void __launch_bounds__(NT) k_inv_gj(int n, const typename Ops::T* __restrict__ in, int64_t in_stride,
                                               typename Ops::T* __restrict__ out, int64_t out_stride) {
  typedef typename Ops::T T;
  static_assert((NP / TR) * (NP / TC) == NT, "tile grid must match the thread count");
  static_assert(TR % 2 == 0 && TC % 2 == 0, "pivot pairs must not straddle tiles");
  constexpr int CT = NP / TC;  // column tiles
  __shared__ T rowk[2][2][NP];   // [parity][pivot row 0/1][col]
  __shared__ T colk[2][2][NP];   // [parity][pivot col 0/1][row]
  const int tid = threadIdx.x;
  const int ti = tid / CT, tj = tid % CT;
  const int r0 = ti * TR, c0 = tj * TC;
  const T* src = in + (int64_t)blockIdx.x * in_stride;
  T a[TR][TC];
#pragma unroll
  for (int r = 0; r < TR; ++r) {
#pragma unroll
    for (int c = 0; c < TC; ++c) {
      const int i = r0 + r, j = c0 + c;
      if (i < n && j < n) a[r][c] = src[(int64_t)i * n + j];
      else a[r][c] = Ops::ident(i == j);
    }
  }
  for (int k = 0; k < n; k += 2) {
    const int b = (k >> 1) & 1;
    const int kr = k - r0, kc = k - c0;      // pivot pair's offset inside this thread's tile
    const bool own_r = kr >= 0 && kr < TR, own_c = kc >= 0 && kc < TC;
    if (own_r) {
#pragma unroll
      for (int r = 0; r < TR; r += 2)
        if (r == kr) {
#pragma unroll
          for (int c = 0; c < TC; ++c) {
            rowk[b][0][c0 + c] = a[r][c];
            rowk[b][1][c0 + c] = a[r + 1][c];
          }
        }
    }
    if (own_c) {
#pragma unroll
      for (int c = 0; c < TC; c += 2)
        if (c == kc) {
#pragma unroll
          for (int r = 0; r < TR; ++r) {
            colk[b][0][r0 + r] = a[r][c];
            colk[b][1][r0 + r] = a[r][c + 1];
          }
        }
    }
    __syncthreads();
    T cr0[TR], cr1[TR], x0[TC], x1[TC];
#pragma unroll
    for (int r = 0; r < TR; ++r) {
      cr0[r] = colk[b][0][r0 + r];
      cr1[r] = colk[b][1][r0 + r];
    }
#pragma unroll
    for (int c = 0; c < TC; ++c) {
      x0[c] = rowk[b][0][c0 + c];
      x1[c] = rowk[b][1][c0 + c];
    }
    // P = [[p00, p01], [p10, p11]] = A_KK^-1 (closed form)
    const T q00 = rowk[b][0][k], q01 = rowk[b][0][k + 1], q10 = rowk[b][1][k], q11 = rowk[b][1][k + 1];
    const T idet = Ops::recip(Ops::sub(Ops::mul(q00, q11), Ops::mul(q01, q10)));
    const T p00 = Ops::mul(q11, idet), p11 = Ops::mul(q00, idet);
    const T p01 = Ops::neg(Ops::mul(q01, idet)), p10 = Ops::neg(Ops::mul(q10, idet));
    T r0v[TC], r1v[TC];
#pragma unroll
    for (int c = 0; c < TC; ++c) {
      r0v[c] = Ops::add(Ops::mul(p00, x0[c]), Ops::mul(p01, x1[c]));
      r1v[c] = Ops::add(Ops::mul(p10, x0[c]), Ops::mul(p11, x1[c]));
    }
#pragma unroll
    for (int r = 0; r < TR; ++r)
#pragma unroll
      for (int c = 0; c < TC; ++c) a[r][c] = Ops::sub_mul(Ops::sub_mul(a[r][c], cr0[r], r0v[c]), cr1[r], r1v[c]);
    if (own_c) {                               // pivot columns: -a_iK P
#pragma unroll
      for (int c = 0; c < TC; c += 2)
        if (c == kc) {
#pragma unroll
          for (int r = 0; r < TR; ++r) {
            a[r][c] = Ops::neg(Ops::add(Ops::mul(cr0[r], p00), Ops::mul(cr1[r], p10)));
            a[r][c + 1] = Ops::neg(Ops::add(Ops::mul(cr0[r], p01), Ops::mul(cr1[r], p11)));
          }
        }
    }
    if (own_r) {                               // pivot rows: R_Kj, pivot block P
#pragma unroll
      for (int r = 0; r < TR; r += 2)
        if (r == kr) {
#pragma unroll
          for (int c = 0; c < TC; ++c) {
            const bool c0k = own_c && c == kc, c1k = own_c && c == kc + 1;
            a[r][c] = c0k ? p00 : (c1k ? p01 : r0v[c]);
            a[r + 1][c] = c0k ? p10 : (c1k ? p11 : r1v[c]);
          }
        }
    }
  }
  T* dst = out + (int64_t)blockIdx.x * out_stride;
#pragma unroll
  for (int r = 0; r < TR; ++r) {
#pragma unroll
    for (int c = 0; c < TC; ++c) {
      const int i = r0 + r, j = c0 + c;
      if (i < n && j < n) dst[(int64_t)i * n + j] = a[r][c];
    }
  }
}

template <class Ops>
int launch_inv(hipStream_t s, int batch, int n, const void* in, int64_t in_stride, void* out, int64_t out_stride) {
  typedef typename Ops::T T;
  const T* x = (const T*)in;
  T* y = (T*)out;
  if (n <= 16) k_inv_gj<Ops, 16, 64, 2, 2><<<batch, 64, 0, s>>>(n, x, in_stride, y, out_stride);
  else if (n <= 32) k_inv_gj<Ops, 32, 64, 4, 4><<<batch, 64, 0, s>>>(n, x, in_stride, y, out_stride);
  else if (n <= 64) k_inv_gj<Ops, 64, 256, 4, 4><<<batch, 256, 0, s>>>(n, x, in_stride, y, out_stride);
  else k_inv_gj<Ops, 128, 512, 4, 8><<<batch, 512, 0, s>>>(n, x, in_stride, y, out_stride);
  return 0;
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
