// Backbone elementwise kernels (gfx950): GroupSort (KWLarge_Concat's activation, the absent
// libs/ortho_conv GroupSort restated in fiode_amd/cayley.py) forward and backward as one pass each.
//
// GroupSort on [B][C][S] (S = spatial size, 1 for the linear layers): with a = x[:, :C/2],
// b = x[:, C/2:], out = cat(max(a, b), min(a, b)).  Backward follows torch.maximum / torch.minimum's
// derivative (ties split the gradient in half):
//   ga = a > b ? g_max : a < b ? g_min : g_max / 2 + g_min / 2, symmetric for gb.
// HBM-bound: 2 x 4 B read + 2 x 4 B write per pair forward, 4 reads + 2 writes backward; float4
// lanes along S (or along the pair index when S == 1).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "common.h"
#include "fiode.h"

namespace {

__device__ __forceinline__ float gmax_part(float a, float b, float gmx, float gmn) {
  return a > b ? gmx : (a < b ? gmn : gmx / 2.0f + gmn / 2.0f);
}

// pair index q over B * (C/2) * S; element of a at b*C*S + c*S + s, of b at + (C/2)*S
__global__ __launch_bounds__(256) void k_groupsort_fwd(const float* __restrict__ x, float* __restrict__ y,
                                                       int64_t npairs4, int64_t half_cs4, int64_t cs4) {
  const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= npairs4) return;
  const int64_t b = q / half_cs4, r = q - b * half_cs4;
  const int64_t ia = b * cs4 + r, ib = ia + half_cs4;
  const float4 va = reinterpret_cast<const float4*>(x)[ia];
  const float4 vb = reinterpret_cast<const float4*>(x)[ib];
  reinterpret_cast<float4*>(y)[ia] = make_float4(fmaxf(va.x, vb.x), fmaxf(va.y, vb.y), fmaxf(va.z, vb.z), fmaxf(va.w, vb.w));
  reinterpret_cast<float4*>(y)[ib] = make_float4(fminf(va.x, vb.x), fminf(va.y, vb.y), fminf(va.z, vb.z), fminf(va.w, vb.w));
}

__global__ __launch_bounds__(256) void k_groupsort_bwd(const float* __restrict__ x, const float* __restrict__ g,
                                                       float* __restrict__ gx, int64_t npairs4, int64_t half_cs4,
                                                       int64_t cs4) {
  const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= npairs4) return;
  const int64_t b = q / half_cs4, r = q - b * half_cs4;
  const int64_t ia = b * cs4 + r, ib = ia + half_cs4;
  const float4 va = reinterpret_cast<const float4*>(x)[ia];
  const float4 vb = reinterpret_cast<const float4*>(x)[ib];
  const float4 gm = reinterpret_cast<const float4*>(g)[ia];
  const float4 gn = reinterpret_cast<const float4*>(g)[ib];
  reinterpret_cast<float4*>(gx)[ia] = make_float4(gmax_part(va.x, vb.x, gm.x, gn.x), gmax_part(va.y, vb.y, gm.y, gn.y),
                                                  gmax_part(va.z, vb.z, gm.z, gn.z), gmax_part(va.w, vb.w, gm.w, gn.w));
  reinterpret_cast<float4*>(gx)[ib] = make_float4(gmax_part(vb.x, va.x, gm.x, gn.x), gmax_part(vb.y, va.y, gm.y, gn.y),
                                                  gmax_part(vb.z, va.z, gm.z, gn.z), gmax_part(vb.w, va.w, gm.w, gn.w));
}

int check_gs(int64_t B, int64_t C, int64_t S, const void* p0, const void* p1) {
  if (B <= 0 || C <= 0 || S <= 0 || (C & 1)) return FIODE_ESHAPE;
  if (((C / 2) * S) % 4 != 0) return FIODE_ESHAPE;     // float4 lanes need (C/2)*S % 4 == 0
  if (!p0 || !p1) return FIODE_EINVAL;
  return FIODE_OK;
}

// Input normalisation fused with the layout change of the conv stack (models.py:17-26 Normalize,
// then KWLargeConcat's NCHW -> spatial-major permute): y[h][w][c][b] = (x[b][c][h][w] - mu[c]) /
// std[c] (std nullable: subtraction only) -- the same two float32 roundings as torch's sub + div.
// 64 x 64 (image, pixel) tiles transposed through LDS: both the reads (along pixels) and the writes
// (along images) are coalesced.
__global__ void __launch_bounds__(256) k_normalize_hwcb(int B, int C, int HW, const float* __restrict__ x,
                                                        const float* __restrict__ mu, const float* __restrict__ sd,
                                                        float* __restrict__ y) {
  __shared__ float t[64][65];
  const int p0 = blockIdx.x * 64, b0 = blockIdx.y * 64, c = blockIdx.z, tid = threadIdx.x;
  const float m = mu[c], s = sd ? sd[c] : 1.0f;
#pragma unroll
  for (int u = 0; u < 16; ++u) {
    const int r = u * 4 + (tid >> 6), q = tid & 63;          // r: image in tile, q: pixel in tile
    const int b = b0 + r, pix = p0 + q;
    float v = 0.f;
    if (b < B && pix < HW) {
      v = x[((int64_t)b * C + c) * HW + pix] - m;
      if (sd) v = v / s;
    }
    t[r][q] = v;
  }
  __syncthreads();
#pragma unroll
  for (int u = 0; u < 16; ++u) {
    const int q = u * 4 + (tid >> 6), r = tid & 63;          // q: pixel, r: image
    const int b = b0 + r, pix = p0 + q;
    if (b < B && pix < HW) y[((int64_t)pix * C + c) * B + b] = t[r][q];
  }
}

}  // namespace

extern "C" int fiode_normalize_hwcb(void* stream, int32_t B, int32_t C, int32_t H, int32_t W, const float* x,
                                    const float* mu, const float* std, float* y) {
  if (B < 1 || C < 1 || C > 65535 || H < 1 || W < 1 || !x || !mu || !y) return FIODE_EINVAL;
  const int HW = H * W;
  hipLaunchKernelGGL(k_normalize_hwcb, dim3((unsigned)((HW + 63) / 64), (unsigned)((B + 63) / 64), (unsigned)C),
                     dim3(256), 0, (hipStream_t)stream, B, C, HW, x, mu, std, y);
  FIODE_HIP_CHECK(hipGetLastError());
  return FIODE_OK;
}

extern "C" int fiode_groupsort_forward(void* stream, int64_t B, int64_t C, int64_t S, const float* x, float* y) {
  int rc = check_gs(B, C, S, x, y);
  if (rc) return rc;
  const int64_t half_cs4 = (C / 2) * S / 4, cs4 = C * S / 4, n4 = B * half_cs4;
  hipLaunchKernelGGL(k_groupsort_fwd, dim3((unsigned)((n4 + 255) / 256)), dim3(256), 0, (hipStream_t)stream, x, y, n4,
                     half_cs4, cs4);
  FIODE_HIP_CHECK(hipGetLastError());
  return FIODE_OK;
}

extern "C" int fiode_groupsort_backward(void* stream, int64_t B, int64_t C, int64_t S, const float* x, const float* g,
                                        float* gx) {
  int rc = check_gs(B, C, S, x, gx);
  if (rc) return rc;
  if (!g) return FIODE_EINVAL;
  const int64_t half_cs4 = (C / 2) * S / 4, cs4 = C * S / 4, n4 = B * half_cs4;
  hipLaunchKernelGGL(k_groupsort_bwd, dim3((unsigned)((n4 + 255) / 256)), dim3(256), 0, (hipStream_t)stream, x, g, gx,
                     n4, half_cs4, cs4);
  FIODE_HIP_CHECK(hipGetLastError());
  return FIODE_OK;
}
