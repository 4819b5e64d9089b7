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

// ---- the linear head's output layer (KWLargeConcat's last Linear, 512 -> x_dim = 10) ------------
// out[b][j] = bias[j] + sum_k z[b][k] Q[j][k] for J <= 16 outputs: one wave per row b, lane l holds
// the k = l, l + 64, ... partial sums of all J outputs, then a fixed butterfly over the 64 lanes
// (run to run reproducible).  The library ran this 128 x 10 x 512 product on ONE workgroup (its
// 16 x 256 tile): ~15 us on the forward chain.
constexpr int HEAD_JMAX = 16;

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// JT: the unrolled output count (J <= JT at run time)
template <int JT>
__global__ __launch_bounds__(256) void k_head_out(int B, int K, int J, const float* __restrict__ z,
                                                 const float* __restrict__ Q, const float* __restrict__ bias,
                                                 float* __restrict__ out) {
  const int lane = threadIdx.x & 63, b = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (b >= B) return;
  float acc[JT];
#pragma unroll
  for (int j = 0; j < JT; ++j) acc[j] = 0.f;
  const float* zr = z + (int64_t)b * K;
  for (int k = lane; k < K; k += 64) {
    const float zv = zr[k];
#pragma unroll
    for (int j = 0; j < JT; ++j) acc[j] += zv * (j < J ? Q[(int64_t)j * K + k] : 0.f);
  }
#pragma unroll
  for (int j = 0; j < JT; ++j) acc[j] = wave_sum(acc[j]);
  if (lane < J) {
    float v = 0.f;
#pragma unroll
    for (int j = 0; j < JT; ++j) v = lane == j ? acc[j] : v;
    out[(int64_t)b * J + lane] = v + (bias ? bias[lane] : 0.f);
  }
}

// its input gradient through the preceding GroupSort: d = g Q (d[b][k] = sum_j g[b][j] Q[j][k], j in
// order), then GroupSort's backward on the pair (k, k + K/2) of its input y: one thread per pair
template <int JT>
__global__ __launch_bounds__(256) void k_head_out_bwd_gs(int B, int K, int J, const float* __restrict__ g,
                                                        const float* __restrict__ Q, const float* __restrict__ y,
                                                        float* __restrict__ gx) {
  const int half = K >> 1;
  const int64_t q = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (q >= (int64_t)B * half) return;
  const int b = (int)(q / half), r = (int)(q - (int64_t)b * half);
  float da = 0.f, db = 0.f;
#pragma unroll
  for (int j = 0; j < JT; ++j) {
    if (j < J) {
      const float gv = g[(int64_t)b * J + j];
      da += gv * Q[(int64_t)j * K + r];
      db += gv * Q[(int64_t)j * K + r + half];
    }
  }
  const float ya = y[(int64_t)b * K + r], yb = y[(int64_t)b * K + r + half];
  gx[(int64_t)b * K + r] = gmax_part(ya, yb, da, db);
  gx[(int64_t)b * K + r + half] = gmax_part(yb, ya, da, db);
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

extern "C" int fiode_head_out(void* stream, int32_t B, int32_t K, int32_t J, const float* z, const float* Q,
                              const float* bias, float* out) {
  if (B <= 0 || K <= 0 || J <= 0 || J > HEAD_JMAX) return FIODE_ESHAPE;
  if (!z || !Q || !out) return FIODE_EINVAL;
  const dim3 grid((unsigned)((B + 3) / 4));
  hipStream_t st = (hipStream_t)stream;
  if (J <= 10) hipLaunchKernelGGL(k_head_out<10>, grid, dim3(256), 0, st, B, K, (int)J, z, Q, bias, out);
  else hipLaunchKernelGGL(k_head_out<HEAD_JMAX>, grid, dim3(256), 0, st, B, K, (int)J, z, Q, bias, out);
  FIODE_HIP_CHECK(hipGetLastError());
  return FIODE_OK;
}

extern "C" int fiode_head_out_backward_gs(void* stream, int32_t B, int32_t K, int32_t J, const float* g,
                                          const float* Q, const float* y, float* gx) {
  if (B <= 0 || K <= 0 || (K & 1) || J <= 0 || J > HEAD_JMAX) return FIODE_ESHAPE;
  if (!g || !Q || !y || !gx) return FIODE_EINVAL;
  const int64_t n = (int64_t)B * (K / 2);
  const dim3 grid((unsigned)((n + 255) / 256));
  hipStream_t st = (hipStream_t)stream;
  if (J <= 10) hipLaunchKernelGGL(k_head_out_bwd_gs<10>, grid, dim3(256), 0, st, B, K, (int)J, g, Q, y, gx);
  else hipLaunchKernelGGL(k_head_out_bwd_gs<HEAD_JMAX>, grid, dim3(256), 0, st, B, K, (int)J, g, Q, y, gx);
  FIODE_HIP_CHECK(hipGetLastError());
  return FIODE_OK;
}
