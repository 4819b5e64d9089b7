// Spectral (FFT-domain) orthogonal convolution of the backbone on spatial-major activations
// (gfx950): the transforms around the per-frequency channel GEMM of CayleyConv.forward_hwcb
// (fiode_amd/cayley.py; the absent libs/ortho_conv of models.py:12-14).
//
// Activations are [n][n][C][B] (B innermost, the conv stack's HBM layout); the spectrum is
// [f][C][B] complex64 with f = ka (n/2 + 1) + kb (rfft2 over (h, w): c2c along h, r2c along w),
// which is exactly the batched-GEMM operand Q[f] (cout x cin) @ X[f] (cin x B).  torch.fft over
// the two leading dims of that layout permutes and clones the whole tensor around rocFFT (~40
// copy kernels and ~0.7 ms per training step for the four convs); here each transform is one
// kernel that reads / writes the GEMM layout directly and fuses the neighbouring elementwise work:
//   k_sconv_rfft2    X = rfft2(x); optional stride-2 space-to-channel gather of the input
//                    (channel 4c + 2dh + dw <- x[2h+dh][2w+dw][c]); optional GroupSort backward
//                    prologue (x := d/dpre from d/dout and the saved comparison codes);
//   k_sconv_irfft2   y = irfft2(Y) (torch's c2c-then-c2r order and 1/n^2 scaling), optional + bias
//                    and GroupSort (pairs c, c + C/2; codes saved for the backward), or the
//                    inverse space-to-channel scatter (the input gradient of a stride-2 conv).
// n in {8, 16, 32}, so each transform is a direct DFT per axis against an n-entry table of roots of unity
// (n^2 (n/2+1) x 2 complex MACs per image, ~17 K at n = 32) on an LDS image of BT images of one
// channel: no butterflies, no bit reversal, coalesced BT-wide loads and stores along B.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "common.h"
#include "fiode.h"

namespace {

typedef float2 c32;
constexpr int NT = 256;
constexpr int BT_F = 16;     // images per forward-transform workgroup
constexpr int BT_I = 8;      // images per inverse-transform workgroup

enum : uint8_t { GS_GT = 0, GS_LT = 1, GS_EQ = 2 };

// d/dpre of one member of a GroupSort pair from d/dmax, d/dmin (torch.maximum / minimum: ties
// split the gradient in half); `first`: the member in the lower channel half (a of max(a, b)).
__device__ __forceinline__ float gs_grad(float gmx, float gmn, uint8_t code, bool first) {
  if (code == GS_EQ) return gmx / 2.0f + gmn / 2.0f;
  const bool a_is_max = (code == GS_GT) == first;
  return a_is_max ? gmx : gmn;
}

struct SArgs {
  int n, H, C, B, ds, gs;        // H = n/2 + 1; ds: stride-2 space-to-channel; gs: GroupSort
  const float* x;                // rfft2 input [n][n][C][B] (ds: [2n][2n][C/4][B])
  const float* gy;               // rfft2 GroupSort-backward prologue: d/dout [n][n][C][B]
  const uint8_t* code;           // [n][n][C/2][B]
  c32* X;                        // rfft2 output [f][C][B]
  const c32* Y;                  // irfft2 input [f][C][B]
  const float* bias;             // [C] or null
  float* y;                      // irfft2 output [n][n][C][B] (ds: [2n][2n][C/4][B])
  uint8_t* code_out;             // [n][n][C/2][B]
};

__device__ __forceinline__ void roots_table(c32* tw, int n, float sign) {
  for (int m = threadIdx.x; m < n; m += NT) {
    float s, c;
    sincospif(2.0f * (float)m / (float)n, &s, &c);
    tw[m] = make_float2(c, sign * s);
  }
}

__device__ __forceinline__ int64_t act_index(const SArgs& a, int h, int w, int c, int b) {
  return (((int64_t)h * a.n + w) * a.C + c) * a.B + b;
}
// element (h, w, c) of the (space-to-channel) input in the raw [2n][2n][C/4][B] tensor
__device__ __forceinline__ int64_t raw_index(const SArgs& a, int h, int w, int c, int b) {
  const int cr = c >> 2, dh = (c >> 1) & 1, dw = c & 1, C4 = a.C >> 2, n2 = 2 * a.n;
  return (((int64_t)(2 * h + dh) * n2 + (2 * w + dw)) * C4 + cr) * a.B + b;
}

// LDS image strides (in elements): odd per-image strides so the BT images a wave touches at one
// (h, w) / (h, kb) land in distinct banks (a power-of-two stride put all 16 images in 1-2 banks).
template <int N>
struct Geo {
  static constexpr int H = N / 2 + 1;
  static constexpr int RS = N + 1;              // real row stride
  static constexpr int IS = N * RS + 1;         // real image stride (odd)
  static constexpr int ZS = N * H + 1;          // complex image stride (odd, in float2)
};

// ---- X[f][c][b0..b0+BT) = rfft2 of channel c ------------------------------------------------------
template <int N>
__global__ void __launch_bounds__(NT) k_sconv_rfft2(SArgs a) {
  typedef Geo<N> g;
  __shared__ float img[BT_F * g::IS];
  __shared__ c32 Z[BT_F * g::ZS];
  __shared__ c32 tw[N];
  constexpr int H = g::H;
  const int c = blockIdx.x, b0 = blockIdx.y * BT_F, tid = threadIdx.x;
  roots_table(tw, N, -1.0f);
  const int half = a.C >> 1;
  for (int idx = tid; idx < BT_F * N * N; idx += NT) {
    const int bt = idx % BT_F, hw = idx / BT_F, h = hw / N, w = hw % N;
    const int b = b0 + bt;
    float v = 0.f;
    if (b < a.B) {
      if (a.gy) {                                  // GroupSort backward: d/dpre of channel c
        const bool first = c < half;
        const int cp = first ? c + half : c - half;
        const uint8_t code = a.code[(((int64_t)h * N + w) * half + (first ? c : cp)) * a.B + b];
        v = gs_grad(a.gy[act_index(a, h, w, first ? c : cp, b)], a.gy[act_index(a, h, w, first ? cp : c, b)], code,
                    first);
      } else {
        v = a.ds ? a.x[raw_index(a, h, w, c, b)] : a.x[act_index(a, h, w, c, b)];
      }
    }
    img[bt * g::IS + h * g::RS + w] = v;
  }
  __syncthreads();
  // r2c along w
  for (int idx = tid; idx < BT_F * N * H; idx += NT) {
    const int bt = idx % BT_F, r = idx / BT_F, h = r / H, kb = r % H;
    const float* row = img + bt * g::IS + h * g::RS;
    c32 z = make_float2(0.f, 0.f);
    int m = 0;
#pragma unroll
    for (int w = 0; w < N; ++w) {
      const float v = row[w];
      const c32 e = tw[m];
      z.x = fmaf(v, e.x, z.x);
      z.y = fmaf(v, e.y, z.y);
      m = (m + kb) & (N - 1);
    }
    Z[bt * g::ZS + h * H + kb] = z;
  }
  __syncthreads();
  // c2c along h, written as X[f][c][b]
  for (int idx = tid; idx < BT_F * N * H; idx += NT) {
    const int bt = idx % BT_F, f = idx / BT_F, ka = f / H, kb = f % H;
    const c32* col = Z + bt * g::ZS + kb;
    c32 z = make_float2(0.f, 0.f);
    int m = 0;
#pragma unroll
    for (int h = 0; h < N; ++h) {
      const c32 v = col[h * H], e = tw[m];
      z.x = fmaf(v.x, e.x, fmaf(-v.y, e.y, z.x));
      z.y = fmaf(v.x, e.y, fmaf(v.y, e.x, z.y));
      m = (m + ka) & (N - 1);
    }
    const int b = b0 + bt;
    if (b < a.B) a.X[((int64_t)f * a.C + c) * a.B + b] = z;
  }
}

// irfft2 of one channel of BT_I images into out (LDS, real image stride Geo<N>::IS)
template <int N>
__device__ __forceinline__ void irfft2_channel(const SArgs& a, int c, int b0, c32* Ys, c32* Zs, float* out,
                                               const c32* tw) {
  typedef Geo<N> g;
  constexpr int H = g::H;
  const int tid = threadIdx.x;
  for (int idx = tid; idx < BT_I * N * H; idx += NT) {
    const int bt = idx % BT_I, f = idx / BT_I;
    const int b = b0 + bt;
    Ys[bt * g::ZS + f] = b < a.B ? a.Y[((int64_t)f * a.C + c) * a.B + b] : make_float2(0.f, 0.f);
  }
  __syncthreads();
  // inverse c2c along ka -> h
  for (int idx = tid; idx < BT_I * N * H; idx += NT) {
    const int bt = idx % BT_I, r = idx / BT_I, h = r / H, kb = r % H;
    const c32* col = Ys + bt * g::ZS + kb;
    c32 z = make_float2(0.f, 0.f);
    int m = 0;
#pragma unroll
    for (int ka = 0; ka < N; ++ka) {
      const c32 v = col[ka * H], e = tw[m];
      z.x = fmaf(v.x, e.x, fmaf(-v.y, e.y, z.x));
      z.y = fmaf(v.x, e.y, fmaf(v.y, e.x, z.y));
      m = (m + h) & (N - 1);
    }
    Zs[bt * g::ZS + h * H + kb] = z;
  }
  __syncthreads();
  // c2r along kb -> w: Re Z0 + Re(Z_{n/2} (-1)^w) + 2 sum_mid Re(Z_kb e^{+i..}), / n^2
  constexpr float inv = 1.0f / (float)(N * N);
  constexpr int nh = N / 2;
  for (int idx = tid; idx < BT_I * N * N; idx += NT) {
    const int bt = idx % BT_I, hw = idx / BT_I, h = hw / N, w = hw % N;
    const c32* row = Zs + bt * g::ZS + h * H;
    float s = 0.f;
    int m = w;
#pragma unroll
    for (int kb = 1; kb < nh; ++kb) {
      const c32 v = row[kb], e = tw[m];
      s = fmaf(v.x, e.x, fmaf(-v.y, e.y, s));
      m = (m + w) & (N - 1);
    }
    const float zn = row[nh].x;
    const float v = row[0].x + ((w & 1) ? -zn : zn) + 2.0f * s;
    out[bt * g::IS + h * g::RS + w] = v * inv;
  }
  __syncthreads();
}

// ---- y = irfft2(Y) (+ bias, GroupSort) or the space-to-channel scatter ---------------------------
// gs: grid.x = C/2 channel pairs; else grid.x = C channels.
template <int N>
__global__ void __launch_bounds__(NT) k_sconv_irfft2(SArgs a) {
  typedef Geo<N> g;
  __shared__ c32 Ys[BT_I * g::ZS];
  __shared__ c32 Zs[BT_I * g::ZS];
  __shared__ float o0[BT_I * g::IS];
  __shared__ float o1[BT_I * g::IS];
  __shared__ c32 tw[N];
  const int b0 = blockIdx.y * BT_I, tid = threadIdx.x;
  roots_table(tw, N, 1.0f);
  __syncthreads();
  if (a.gs) {
    const int half = a.C >> 1, c0 = blockIdx.x, c1 = c0 + half;
    irfft2_channel<N>(a, c0, b0, Ys, Zs, o0, tw);
    irfft2_channel<N>(a, c1, b0, Ys, Zs, o1, tw);
    const float bb0 = a.bias ? a.bias[c0] : 0.f, bb1 = a.bias ? a.bias[c1] : 0.f;
    for (int idx = tid; idx < BT_I * N * N; idx += NT) {
      const int bt = idx % BT_I, hw = idx / BT_I, h = hw / N, w = hw % N;
      const int b = b0 + bt;
      if (b >= a.B) continue;
      const int li = bt * g::IS + h * g::RS + w;
      const float p = o0[li] + bb0, q = o1[li] + bb1;
      a.y[act_index(a, h, w, c0, b)] = fmaxf(p, q);
      a.y[act_index(a, h, w, c1, b)] = fminf(p, q);
      a.code_out[(((int64_t)h * N + w) * half + c0) * a.B + b] = p > q ? GS_GT : (p < q ? GS_LT : GS_EQ);
    }
  } else {
    const int c = blockIdx.x;
    irfft2_channel<N>(a, c, b0, Ys, Zs, o0, tw);
    const float bb = a.bias ? a.bias[c] : 0.f;
    for (int idx = tid; idx < BT_I * N * N; idx += NT) {
      const int bt = idx % BT_I, hw = idx / BT_I, h = hw / N, w = hw % N;
      const int b = b0 + bt;
      if (b >= a.B) continue;
      const float v = o0[bt * g::IS + h * g::RS + w] + bb;
      if (a.ds) a.y[raw_index(a, h, w, c, b)] = v;
      else a.y[act_index(a, h, w, c, b)] = v;
    }
  }
}

int check(const fiode_sconv_config* cfg, SArgs& a) {
  if (!cfg) return FIODE_EINVAL;
  a = SArgs{};
  a.n = cfg->n;
  a.C = cfg->C;
  a.B = cfg->B;
  a.ds = cfg->downsample ? 1 : 0;
  if ((a.n != 8 && a.n != 16 && a.n != 32) || a.C < 1 || a.B < 1) return FIODE_ESHAPE;
  if (a.ds && (a.C & 3)) return FIODE_ESHAPE;
  a.H = a.n / 2 + 1;
  return FIODE_OK;
}

}  // namespace

extern "C" int fiode_sconv_rfft2(void* stream, const fiode_sconv_config* cfg, const float* x, const float* gy,
                                 const uint8_t* code, void* X) {
  SArgs a;
  int rc = check(cfg, a);
  if (rc) return rc;
  if (!X || (!x && !gy) || (gy && (!code || (a.C & 1) || a.ds))) return FIODE_EINVAL;
  a.x = x;
  a.gy = gy;
  a.code = code;
  a.X = (c32*)X;
  const dim3 grid(a.C, (a.B + BT_F - 1) / BT_F);
  hipStream_t st = (hipStream_t)stream;
  if (a.n == 8) hipLaunchKernelGGL(k_sconv_rfft2<8>, grid, dim3(NT), 0, st, a);
  else if (a.n == 16) hipLaunchKernelGGL(k_sconv_rfft2<16>, grid, dim3(NT), 0, st, a);
  else hipLaunchKernelGGL(k_sconv_rfft2<32>, grid, dim3(NT), 0, st, a);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? FIODE_OK : FIODE_EHIP + (int)e;
}

extern "C" int fiode_sconv_irfft2(void* stream, const fiode_sconv_config* cfg, const void* Y, const float* bias,
                                  int32_t groupsort, float* y, uint8_t* code_out) {
  SArgs a;
  int rc = check(cfg, a);
  if (rc) return rc;
  a.gs = groupsort ? 1 : 0;
  if (!Y || !y || (a.gs && (!code_out || (a.C & 1) || a.ds))) return FIODE_EINVAL;
  a.Y = (const c32*)Y;
  a.bias = bias;
  a.y = y;
  a.code_out = code_out;
  const int gx = a.gs ? a.C / 2 : a.C;
  const dim3 grid(gx, (a.B + BT_I - 1) / BT_I);
  hipStream_t st = (hipStream_t)stream;
  if (a.n == 8) hipLaunchKernelGGL(k_sconv_irfft2<8>, grid, dim3(NT), 0, st, a);
  else if (a.n == 16) hipLaunchKernelGGL(k_sconv_irfft2<16>, grid, dim3(NT), 0, st, a);
  else hipLaunchKernelGGL(k_sconv_irfft2<32>, grid, dim3(NT), 0, st, a);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? FIODE_OK : FIODE_EHIP + (int)e;
}
