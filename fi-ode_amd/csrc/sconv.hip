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
// n in {8, 16, 32}: each 1-D transform is one in-register radix-2 FFT per thread (fft.h; ~0.6 K
// VALU ops at n = 32 where the direct DFT of the first version took ~4 K FMAs), on an LDS image of
// BT images of one channel, with coalesced BT-wide loads and stores along B.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "common.h"
#include "fft.h"
#include "fiode.h"

namespace {

typedef float2 c32;
constexpr int BT_F = 16;     // images per forward-transform workgroup
constexpr int BT_I = 8;      // images per inverse-transform workgroup
// threads per workgroup (compile-time; tools/gpu_r05ar.sh sweeps 64-1024): 512 for the n = 8 / 16
// forward and inverse transforms (with 1024 half the waves idled through the FFT phases), 256 for
// the n = 8 inverse, 512 at n = 32 (the 4-image input-layer forward: 128 threads measured 11.4 us at
// best against 8.3, though steadier beside other kernels)
#ifndef SCONV_NTF8
#define SCONV_NTF8 512
#endif
#ifndef SCONV_NTF16
#define SCONV_NTF16 512
#endif
#ifndef SCONV_NTF32
#define SCONV_NTF32 512
#endif
#ifndef SCONV_NTF32S
#define SCONV_NTF32S 512
#endif
#ifndef SCONV_NTI8
#define SCONV_NTI8 256
#endif
#ifndef SCONV_NTI16
#define SCONV_NTI16 512
#endif
#ifndef SCONV_NTI32
#define SCONV_NTI32 512
#endif
// n = 32 forward transforms: 8 images per workgroup (69 KB of LDS, two workgroups per CU; 16 images
// left one per CU: k_sconv_rfft2<32> 33.1 -> 29.4 us in the step); the inverse keeps 8 (4: no gain)
#ifndef SCONV_BTF32
#define SCONV_BTF32 8
#endif
#ifndef SCONV_BTI32
#define SCONV_BTI32 8
#endif
template <int N, int BT, bool INV>
constexpr int nthreads() {
  return INV ? (N == 8 ? SCONV_NTI8 : N == 16 ? SCONV_NTI16 : SCONV_NTI32)
             : (N == 8 ? SCONV_NTF8 : N == 16 ? SCONV_NTF16 : BT == 4 ? SCONV_NTF32S : SCONV_NTF32);
}
// images per inverse-transform workgroup
template <int N>
constexpr int bt_inv() { return N == 32 ? SCONV_BTI32 : BT_I; }

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
  int nchw;                      // irfft2 output y / rfft2 gy input as [B][C][n][n], codes [B][C/2][n][n]
  const float* x;                // rfft2 input [n][n][C][B] (ds: [2n][2n][C/4][B])
  const float* gy;               // rfft2 GroupSort-backward prologue: d/dout [n][n][C][B]
  const uint8_t* code;           // [n][n][C/2][B]
  c32* X;                        // rfft2 output [f][C][B]
  const c32* Y;                  // irfft2 input [f][C][B]
  const float* bias;             // [C] or null
  float* y;                      // irfft2 output [n][n][C][B] (ds: [2n][2n][C/4][B])
  uint8_t* code_out;             // [n][n][C/2][B]
  const float* xn;               // rfft2 input in NCHW [B][C][n][n], normalised on load (the backbone's
  const float* mu;               //   first layer: Normalize fused, models.py:17-26), mu / sd [C]
  const float* sd;               //   (sd nullable)
  const c32* Q;                  // irfft2 with the channel product fused (fiode_sconv_irfft2_qx): Y[f] = Q[f] Xq[f]
  const c32* Xq;                 //   on load, Q [f][C][K], Xq [f][K][B], K <= 4 (conv 1: the 3 input channels)
};

__device__ __forceinline__ int64_t act_index(const SArgs& a, int h, int w, int c, int b) {
  return (((int64_t)h * a.n + w) * a.C + c) * a.B + b;
}
// NCHW element / GroupSort code (the last conv's output, read by the flatten as (C, h, w) features)
__device__ __forceinline__ int64_t nchw_index(const SArgs& a, int h, int w, int c, int b) {
  return (((int64_t)b * a.C + c) * a.n + h) * a.n + w;
}
__device__ __forceinline__ int64_t code_index(const SArgs& a, int h, int w, int c0, int b) {
  const int half = a.C >> 1;
  return a.nchw ? (((int64_t)b * half + c0) * a.n + h) * a.n + w : (((int64_t)h * a.n + w) * half + c0) * a.B + b;
}
// element (h, w, c) of the (space-to-channel) input in the raw [2n][2n][C/4][B] tensor
__device__ __forceinline__ int64_t raw_index(const SArgs& a, int h, int w, int c, int b) {
  const int cr = c >> 2, dh = (c >> 1) & 1, dw = c & 1, C4 = a.C >> 2, n2 = 2 * a.n;
  return (((int64_t)(2 * h + dh) * n2 + (2 * w + dw)) * C4 + cr) * a.B + b;
}

// LDS image strides (in elements) per kernel: the per-image padding that puts the lanes of every
// LDS instruction of that kernel in distinct banks as far as the gfx950 lane groups allow
// (tools/probes/sconv_lds_banks.py models each instruction's lane -> address map: e.g. k_sconv_irfft2<16>
// 824 -> 432 LDS cycles per workgroup against 428 conflict-free; the plain odd strides N (N+1) + 1 /
// N (N/2+1) + 1 left 30-70 % of the LDS cycles to conflicts in PMC).  INV: k_sconv_irfft2.
constexpr int pad_is(int n, int bt, bool inv) {
  return inv ? (n == 8 ? 76 : n == 16 ? 276 : (bt == 4 ? 1064 : 1060))
             : n == 8 ? (bt == 4 ? 72 : 74) : n == 16 ? (bt == 4 ? 280 : 274)
                                                      : (bt == 4 ? 1064 : bt == 8 ? 1060 : 1058);
}
constexpr int pad_zs(int n, int bt, bool inv) {
  return inv ? (n == 8 ? 42 : n == 16 ? 146 : (bt == 4 ? 548 : 546))
             : n == 8 ? (bt == 4 ? 44 : 41) : n == 16 ? (bt == 4 ? 148 : 145)
                                                      : (bt == 4 ? 548 : bt == 8 ? 546 : 545);
}
template <int N, int BT, bool INV>
struct Geo {
  static constexpr int H = N / 2 + 1;
  static constexpr int RS = N + 1;                  // real row stride
  static constexpr int IS = pad_is(N, BT, INV);     // real image stride
  static constexpr int ZS = pad_zs(N, BT, INV);     // complex image stride (in float2)
  static_assert(IS >= N * RS && ZS >= N * H, "image strides");
};

// ---- X[f][c][b0..b0+BT) = rfft2 of channel c ------------------------------------------------------
// One complex buffer per channel, [bt][h][kb] (row stride H, image stride ZS, channel stride BT ZS):
// the real input is stored in place (pixel (h, w) of image bt at float offset pix(ch, bt, h) + w,
// the row's first N of its 2H floats), the row transforms (r2c) overwrite their own rows, the column
// transforms (c2c) go to X.  The GroupSort backward prologue takes both channels of a pair in one
// workgroup: d/dmax, d/dmin and the codes are read once for both (round 4: a workgroup per channel
// read the pair's d/dout twice, through a separate real image buffer).
template <int N, int BT>
struct FGeo {
  typedef Geo<N, BT, false> g;
  static constexpr int H = g::H;
  static constexpr int ZS = g::ZS;
  static constexpr int CS = BT * ZS;       // channel stride (float2)
  static constexpr int NT = nthreads<N, BT, false>();
  __device__ static int pix(int ch, int bt, int h) { return 2 * (ch * CS + bt * ZS + h * H); }
};

template <int N, int BT, int NCH>
__device__ __forceinline__ void rfft2_inplace(const SArgs& a, int c0, int c1, int b0, c32* Z) {
  typedef FGeo<N, BT> G;
  constexpr int H = G::H, NT = G::NT;
  const float* img = reinterpret_cast<const float*>(Z);
  const int tid = threadIdx.x;
  // The two 1-D transforms as one length-N FFT per thread in registers (rows, then columns;
  // fft.h): a direct DFT here (N^2 complex MACs per transform) left the workgroups VALU-bound.
  // r2c along w: one (channel, image, h) row per thread (imaginary part 0, the N/2 + 1 kept
  // outputs written over the row's own floats)
  for (int row = tid; row < NCH * BT * N; row += NT) {
    const int ch = row / (BT * N), r = row - ch * (BT * N);
    const int bt = r % BT, h = r / BT;
    const float* src = img + G::pix(ch, bt, h);
    c32 x[N];
#pragma unroll
    for (int w = 0; w < N; ++w) x[w] = make_float2(src[w], 0.f);
    fiode_fft::fft_reg<N, false>(x);
    c32* dst = Z + ch * G::CS + bt * G::ZS + h * H;
#pragma unroll
    for (int kb = 0; kb < H; ++kb) dst[kb] = x[kb];
  }
  __syncthreads();
  // c2c along h: one (channel, image, kb) column per thread, written as X[f][c][b]
  for (int col = tid; col < NCH * BT * H; col += NT) {
    const int ch = col / (BT * H), r = col - ch * (BT * H);
    const int bt = r % BT, kb = r / BT;
    const c32* cp = Z + ch * G::CS + bt * G::ZS + kb;
    c32 x[N];
#pragma unroll
    for (int h = 0; h < N; ++h) x[h] = cp[h * H];
    fiode_fft::fft_reg<N, false>(x);
    const int b = b0 + bt, c = ch ? c1 : c0;
    if (b < a.B) {
#pragma unroll
      for (int ka = 0; ka < N; ++ka) a.X[((int64_t)(ka * H + kb) * a.C + c) * a.B + b] = x[ka];
    }
  }
}

// gy (GroupSort backward): grid.x = C/2 channel pairs; else grid.x = C channels
template <int N, int BT>
__global__ void __launch_bounds__((nthreads<N, BT, false>())) k_sconv_rfft2(SArgs a) {
  typedef FGeo<N, BT> G;
  constexpr int NT = G::NT;
  constexpr int NL = BT * N * N;
  constexpr int TR = (NL + NT - 1) / NT;
  __shared__ c32 Z[2 * G::CS];
  float* img = reinterpret_cast<float*>(Z);
  const int b0 = blockIdx.y * BT, tid = threadIdx.x;
  // the loads of all trips in flight together (a trip-by-trip loop waits ~1 us per trip on the
  // memory latency): a fixed trip count, unrolled, one loop per source mode
  if (a.gy) {                                      // GroupSort backward: d/dpre of both channels
    const int half = a.C >> 1, c0 = blockIdx.x, c1 = c0 + half;
#pragma unroll
    for (int t = 0; t < TR; ++t) {
      const int idx = tid + t * NT;
      if (idx < NL) {
        // lanes along b for the spatial-major layout, along w for NCHW (coalesced either way)
        const int bt = a.nchw ? idx / (N * N) : idx % BT;
        const int hw = a.nchw ? idx % (N * N) : idx / BT, h = hw / N, w = hw % N;
        const int b = min(b0 + bt, a.B - 1);
        const uint8_t code = a.code[code_index(a, h, w, c0, b)];
        const float gmx = a.gy[a.nchw ? nchw_index(a, h, w, c0, b) : act_index(a, h, w, c0, b)];
        const float gmn = a.gy[a.nchw ? nchw_index(a, h, w, c1, b) : act_index(a, h, w, c1, b)];
        const bool in = b0 + bt < a.B;
        img[G::pix(0, bt, h) + w] = in ? gs_grad(gmx, gmn, code, true) : 0.f;
        img[G::pix(1, bt, h) + w] = in ? gs_grad(gmx, gmn, code, false) : 0.f;
      }
    }
    __syncthreads();
    rfft2_inplace<N, BT, 2>(a, c0, c1, b0, Z);
    return;
  }
  const int c = blockIdx.x;
  if (a.xn) {      // NCHW input, (x - mu) / sd as fiode_normalize_hwcb computes it; lanes along w
    const float m = a.mu[c], sdv = a.sd ? a.sd[c] : 1.0f;
#pragma unroll
    for (int t = 0; t < TR; ++t) {
      const int idx = tid + t * NT;
      if (idx < NL) {
        const int w = idx % N, h = (idx / N) % N, bt = idx / (N * N);
        const int b = min(b0 + bt, a.B - 1);
        float v = a.xn[(((int64_t)b * a.C + c) * N + h) * N + w] - m;
        if (a.sd) v = v / sdv;
        img[G::pix(0, bt, h) + w] = b0 + bt < a.B ? v : 0.f;
      }
    }
  } else if (a.ds) {
#pragma unroll
    for (int t = 0; t < TR; ++t) {
      const int idx = tid + t * NT;
      if (idx < NL) {
        const int bt = idx % BT, hw = idx / BT, h = hw / N, w = hw % N;
        const int b = min(b0 + bt, a.B - 1);
        const float v = a.x[raw_index(a, h, w, c, b)];
        img[G::pix(0, bt, h) + w] = b0 + bt < a.B ? v : 0.f;
      }
    }
  } else {
#pragma unroll
    for (int t = 0; t < TR; ++t) {
      const int idx = tid + t * NT;
      if (idx < NL) {
        const int bt = idx % BT, hw = idx / BT, h = hw / N, w = hw % N;
        const int b = min(b0 + bt, a.B - 1);
        const float v = a.x[act_index(a, h, w, c, b)];
        img[G::pix(0, bt, h) + w] = b0 + bt < a.B ? v : 0.f;
      }
    }
  }
  __syncthreads();
  rfft2_inplace<N, BT, 1>(a, c, c, b0, Z);
}

// irfft2 of the workgroup's NCH channels x BTI images in place in Ys (one complex image per
// (channel, image), row stride H, channel stride BTI ZS): every channel's spectra are loaded at once,
// then the column transforms (inverse c2c along ka) of all channels, then the rows (c2r along kb; the
// row's N real outputs written over its own 2H floats).  Pixel (h, w) of image bt of channel ch ends
// at float offset pix(ch, bt, h) + w.  (Round 4 ran the two channels of a GroupSort pair one after
// the other through separate column / row / output buffers: 137 KB of LDS at n = 32, one workgroup
// per CU, two load latencies per workgroup.)
template <int N>
struct IGeo {
  typedef Geo<N, bt_inv<N>(), true> g;
  static constexpr int BTI = bt_inv<N>();
  static constexpr int H = g::H;
  static constexpr int ZS = g::ZS;
  static constexpr int CS = BTI * ZS;      // channel stride (float2)
  static constexpr int NT = nthreads<N, BTI, true>();
  __device__ static int pix(int ch, int bt, int h) { return 2 * (ch * CS + bt * ZS + h * H); }
};

// KQ > 0: Y[f][c][b] = sum_k Q[f][c][k] Xq[f][k][b] computed on load (k in order, products then
// sums in float32), instead of read from a GEMM output
template <int N, int NCH, int KQ>
__device__ __forceinline__ void irfft2_inplace(const SArgs& a, int c0, int c1, int b0, c32* Ys) {
  typedef IGeo<N> G;
  constexpr int BTI = G::BTI, H = G::H, NT = G::NT;
  constexpr int NL = NCH * BTI * N * H;
  constexpr int TR = (NL + NT - 1) / NT;
  const int tid = threadIdx.x;
  if constexpr (KQ == 0) {
    // all loads in flight together: a fixed trip count, unrolled
#pragma unroll
    for (int t = 0; t < TR; ++t) {
      const int idx = tid + t * NT;
      if (idx < NL) {
        const int ch = idx / (BTI * N * H), r = idx - ch * (BTI * N * H);
        const int bt = r % BTI, f = r / BTI;
        const int b = min(b0 + bt, a.B - 1);
        const c32 v = a.Y[((int64_t)f * a.C + (ch ? c1 : c0)) * a.B + b];
        Ys[ch * G::CS + bt * G::ZS + f] = b0 + bt < a.B ? v : make_float2(0.f, 0.f);
      }
    }
  } else {
    // one (image, frequency) per thread for every channel of the workgroup: X[f][k][b] read once
    constexpr int NL1 = BTI * N * H;
    constexpr int TR1 = (NL1 + NT - 1) / NT;
#pragma unroll
    for (int t = 0; t < TR1; ++t) {
      const int idx = tid + t * NT;
      if (idx < NL1) {
        const int bt = idx % BTI, f = idx / BTI;
        const int b = min(b0 + bt, a.B - 1);
        const c32* xq = a.Xq + (int64_t)f * KQ * a.B + b;
        c32 xk[KQ], qk[NCH][KQ];
#pragma unroll
        for (int k = 0; k < KQ; ++k) xk[k] = xq[(int64_t)k * a.B];
#pragma unroll
        for (int ch = 0; ch < NCH; ++ch) {
          const c32* q = a.Q + ((int64_t)f * a.C + (ch ? c1 : c0)) * KQ;
#pragma unroll
          for (int k = 0; k < KQ; ++k) qk[ch][k] = q[k];
        }
#pragma unroll
        for (int ch = 0; ch < NCH; ++ch) {
          c32 v = make_float2(0.f, 0.f);
#pragma unroll
          for (int k = 0; k < KQ; ++k) {
            v.x += qk[ch][k].x * xk[k].x - qk[ch][k].y * xk[k].y;
            v.y += qk[ch][k].x * xk[k].y + qk[ch][k].y * xk[k].x;
          }
          Ys[ch * G::CS + bt * G::ZS + f] = b0 + bt < a.B ? v : make_float2(0.f, 0.f);
        }
      }
    }
  }
  __syncthreads();
  // inverse c2c along ka: one (channel, image, kb) column per thread, in place
  for (int col = tid; col < NCH * BTI * H; col += NT) {
    const int ch = col / (BTI * H), r = col - ch * (BTI * H);
    const int bt = r % BTI, kb = r / BTI;
    c32* cp = Ys + ch * G::CS + bt * G::ZS + kb;
    c32 x[N];
#pragma unroll
    for (int ka = 0; ka < N; ++ka) x[ka] = cp[ka * H];
    fiode_fft::fft_reg<N, true>(x);
#pragma unroll
    for (int h = 0; h < N; ++h) cp[h * H] = x[h];
  }
  __syncthreads();
  // c2r along kb: one (channel, image, h) row per thread: the Hermitian completion X[N - k] = conj X[k]
  // (imaginary parts of X[0], X[N/2] ignored, as torch's irfft does), inverse FFT, real part, 1/n^2
  constexpr float inv = 1.0f / (float)(N * N);
  constexpr int nh = N / 2;
  for (int row = tid; row < NCH * BTI * N; row += NT) {
    const int ch = row / (BTI * N), r = row - ch * (BTI * N);
    const int bt = r % BTI, h = r / BTI;
    const c32* src = Ys + ch * G::CS + bt * G::ZS + h * H;
    c32 x[N];
    x[0] = make_float2(src[0].x, 0.f);
    x[nh] = make_float2(src[nh].x, 0.f);
#pragma unroll
    for (int kb = 1; kb < nh; ++kb) {
      const c32 v = src[kb];
      x[kb] = v;
      x[N - kb] = make_float2(v.x, -v.y);
    }
    fiode_fft::fft_reg<N, true>(x);
    float* dst = reinterpret_cast<float*>(Ys) + G::pix(ch, bt, h);
#pragma unroll
    for (int w = 0; w < N; ++w) dst[w] = x[w].x * inv;
  }
  __syncthreads();
}

// ---- y = irfft2(Y) (+ bias, GroupSort) or the space-to-channel scatter ---------------------------
// gs: grid.x = C/2 channel pairs (both channels of a pair in one workgroup); else grid.x = C channels.
template <int N, int KQ>
__global__ void __launch_bounds__((nthreads<N, bt_inv<N>(), true>())) k_sconv_irfft2(SArgs a) {
  typedef IGeo<N> G;
  constexpr int BTI = G::BTI, NT = G::NT;
  __shared__ c32 Ys[2 * G::CS];
  const float* o = reinterpret_cast<const float*>(Ys);
  const int b0 = blockIdx.y * BTI, tid = threadIdx.x;
  if (a.gs) {
    const int half = a.C >> 1, c0 = blockIdx.x, c1 = c0 + half;
    irfft2_inplace<N, 2, KQ>(a, c0, c1, b0, Ys);
    const float bb0 = a.bias ? a.bias[c0] : 0.f, bb1 = a.bias ? a.bias[c1] : 0.f;
    for (int idx = tid; idx < BTI * N * N; idx += NT) {
      const int bt = a.nchw ? idx / (N * N) : idx % BTI;
      const int hw = a.nchw ? idx % (N * N) : idx / BTI, h = hw / N, w = hw % N;
      const int b = b0 + bt;
      if (b >= a.B) continue;
      const float p = o[G::pix(0, bt, h) + w] + bb0, q = o[G::pix(1, bt, h) + w] + bb1;
      a.y[a.nchw ? nchw_index(a, h, w, c0, b) : act_index(a, h, w, c0, b)] = fmaxf(p, q);
      a.y[a.nchw ? nchw_index(a, h, w, c1, b) : act_index(a, h, w, c1, b)] = fminf(p, q);
      a.code_out[code_index(a, h, w, c0, b)] = p > q ? GS_GT : (p < q ? GS_LT : GS_EQ);
    }
    (void)half;
  } else {
    const int c = blockIdx.x;
    irfft2_inplace<N, 1, KQ>(a, c, c, b0, Ys);
    const float bb = a.bias ? a.bias[c] : 0.f;
    for (int idx = tid; idx < BTI * N * N; idx += NT) {
      const int bt = a.nchw ? idx / (N * N) : idx % BTI;
      const int hw = a.nchw ? idx % (N * N) : idx / BTI, h = hw / N, w = hw % N;
      const int b = b0 + bt;
      if (b >= a.B) continue;
      const float v = o[G::pix(0, bt, h) + w] + bb;
      if (a.ds) a.y[raw_index(a, h, w, c, b)] = v;
      else if (a.nchw) a.y[nchw_index(a, h, w, c, b)] = v;
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
  a.nchw = cfg->nchw ? 1 : 0;
  if ((a.n != 8 && a.n != 16 && a.n != 32) || a.C < 1 || a.B < 1) return FIODE_ESHAPE;
  if (a.nchw && a.ds) return FIODE_ESHAPE;
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
  hipStream_t st = (hipStream_t)stream;
  // few channels (the 3-channel input of conv 1): 4 images per workgroup to spread over the CUs
  const bool small = (int64_t)a.C * ((a.B + BT_F - 1) / BT_F) < 256;
  const int bt = small ? 4 : a.n == 32 ? SCONV_BTF32 : BT_F;
  const dim3 grid(gy ? a.C / 2 : a.C, (a.B + bt - 1) / bt);
  if (a.n == 8) {
    if (small) hipLaunchKernelGGL((k_sconv_rfft2<8, 4>), grid, dim3(nthreads<8, 4, false>()), 0, st, a);
    else hipLaunchKernelGGL((k_sconv_rfft2<8, BT_F>), grid, dim3(nthreads<8, BT_F, false>()), 0, st, a);
  } else if (a.n == 16) {
    if (small) hipLaunchKernelGGL((k_sconv_rfft2<16, 4>), grid, dim3(nthreads<16, 4, false>()), 0, st, a);
    else hipLaunchKernelGGL((k_sconv_rfft2<16, BT_F>), grid, dim3(nthreads<16, BT_F, false>()), 0, st, a);
  } else {
    if (small) hipLaunchKernelGGL((k_sconv_rfft2<32, 4>), grid, dim3(nthreads<32, 4, false>()), 0, st, a);
    else hipLaunchKernelGGL((k_sconv_rfft2<32, SCONV_BTF32>), grid, dim3(nthreads<32, SCONV_BTF32, false>()), 0, st, a);
  }
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? FIODE_OK : FIODE_EHIP + (int)e;
}

extern "C" int fiode_sconv_rfft2_nchw(void* stream, const fiode_sconv_config* cfg, const float* x, const float* mu,
                                      const float* sd, void* X) {
  SArgs a;
  int rc = check(cfg, a);
  if (rc) return rc;
  if (!X || !x || !mu || a.ds) return FIODE_EINVAL;
  a.xn = x;
  a.mu = mu;
  a.sd = sd;
  a.X = (c32*)X;
  hipStream_t st = (hipStream_t)stream;
  const bool small = (int64_t)a.C * ((a.B + BT_F - 1) / BT_F) < 256;
  const int bt = small ? 4 : a.n == 32 ? SCONV_BTF32 : BT_F;
  const dim3 grid(a.C, (a.B + bt - 1) / bt);
  if (a.n == 8) {
    if (small) hipLaunchKernelGGL((k_sconv_rfft2<8, 4>), grid, dim3(nthreads<8, 4, false>()), 0, st, a);
    else hipLaunchKernelGGL((k_sconv_rfft2<8, BT_F>), grid, dim3(nthreads<8, BT_F, false>()), 0, st, a);
  } else if (a.n == 16) {
    if (small) hipLaunchKernelGGL((k_sconv_rfft2<16, 4>), grid, dim3(nthreads<16, 4, false>()), 0, st, a);
    else hipLaunchKernelGGL((k_sconv_rfft2<16, BT_F>), grid, dim3(nthreads<16, BT_F, false>()), 0, st, a);
  } else {
    if (small) hipLaunchKernelGGL((k_sconv_rfft2<32, 4>), grid, dim3(nthreads<32, 4, false>()), 0, st, a);
    else hipLaunchKernelGGL((k_sconv_rfft2<32, SCONV_BTF32>), grid, dim3(nthreads<32, SCONV_BTF32, false>()), 0, st, a);
  }
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? FIODE_OK : FIODE_EHIP + (int)e;
}

namespace {

template <int KQ>
hipError_t launch_irfft2(const SArgs& a, hipStream_t st) {
  const int gx = a.gs ? a.C / 2 : a.C;
  const int bt = a.n == 32 ? bt_inv<32>() : BT_I;
  const dim3 grid(gx, (a.B + bt - 1) / bt);
  if (a.n == 8) hipLaunchKernelGGL((k_sconv_irfft2<8, KQ>), grid, dim3(nthreads<8, BT_I, true>()), 0, st, a);
  else if (a.n == 16) hipLaunchKernelGGL((k_sconv_irfft2<16, KQ>), grid, dim3(nthreads<16, BT_I, true>()), 0, st, a);
  else hipLaunchKernelGGL((k_sconv_irfft2<32, KQ>), grid, dim3(nthreads<32, bt_inv<32>(), true>()), 0, st, a);
  return hipGetLastError();
}

int irfft2_common(const fiode_sconv_config* cfg, const float* bias, int32_t groupsort, float* y, uint8_t* code_out,
                  SArgs& a) {
  int rc = check(cfg, a);
  if (rc) return rc;
  a.gs = groupsort ? 1 : 0;
  if (!y || (a.gs && (!code_out || (a.C & 1) || a.ds))) return FIODE_EINVAL;
  a.bias = bias;
  a.y = y;
  a.code_out = code_out;
  return FIODE_OK;
}

}  // namespace

extern "C" int fiode_sconv_irfft2(void* stream, const fiode_sconv_config* cfg, const void* Y, const float* bias,
                                  int32_t groupsort, float* y, uint8_t* code_out) {
  SArgs a;
  const int rc = irfft2_common(cfg, bias, groupsort, y, code_out, a);
  if (rc) return rc;
  if (!Y) return FIODE_EINVAL;
  a.Y = (const c32*)Y;
  const hipError_t e = launch_irfft2<0>(a, (hipStream_t)stream);
  return e == hipSuccess ? FIODE_OK : FIODE_EHIP + (int)e;
}

extern "C" int fiode_sconv_irfft2_qx(void* stream, const fiode_sconv_config* cfg, const void* Q, const void* X,
                                     int32_t K, const float* bias, int32_t groupsort, float* y, uint8_t* code_out) {
  SArgs a;
  const int rc = irfft2_common(cfg, bias, groupsort, y, code_out, a);
  if (rc) return rc;
  if (K < 1 || K > 4) return FIODE_ESHAPE;
  if (!Q || !X) return FIODE_EINVAL;
  a.Q = (const c32*)Q;
  a.Xq = (const c32*)X;
  hipStream_t st = (hipStream_t)stream;
  const hipError_t e = K == 1 ? launch_irfft2<1>(a, st) : K == 2 ? launch_irfft2<2>(a, st)
                     : K == 3 ? launch_irfft2<3>(a, st) : launch_irfft2<4>(a, st);
  return e == hipSuccess ? FIODE_OK : FIODE_EHIP + (int)e;
}
