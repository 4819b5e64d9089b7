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
