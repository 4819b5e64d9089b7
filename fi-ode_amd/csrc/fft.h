// In-register radix-2 FFTs of length N in {8, 16, 32} for one thread (gfx950 VALU), used by the
// backbone's spectral-conv transforms (sconv.hip).  A thread holds its N complex values in
// registers; every index, every twiddle and every butterfly is resolved at compile time once the
// loops are unrolled (bit-reversal is a register renaming, twiddles 1 and -i / +i cost no
// multiply), so a length-32 transform is ~0.6 K VALU ops instead of the 4 K FMAs of a direct DFT.
//   fft_reg<N, false>(x):  X[k] = sum_n x[n] e^{-2 pi i n k / N}   (torch.fft forward, unscaled)
//   fft_reg<N, true>(x):   x[n] = sum_k X[k] e^{+2 pi i n k / N}   (inverse, unscaled)
// Twiddles: e^{-2 pi i m / 32}, m < 16, float32-rounded cos / sin (generated, hex literals); the
// shorter lengths use every 2nd / 4th entry.
#pragma once
#include <hip/hip_runtime.h>

namespace fiode_fft {

typedef float2 c32;

__device__ constexpr float kCos32[16] = {0x1.0000000000000p+0f, 0x1.f6297c0000000p-1f, 0x1.d906bc0000000p-1f, 0x1.a9b6620000000p-1f, 0x1.6a09e60000000p-1f, 0x1.1c73b40000000p-1f, 0x1.87de2a0000000p-2f, 0x1.8f8b840000000p-3f, 0x1.1a62640000000p-54f, -0x1.8f8b840000000p-3f, -0x1.87de2a0000000p-2f, -0x1.1c73b40000000p-1f, -0x1.6a09e60000000p-1f, -0x1.a9b6620000000p-1f, -0x1.d906bc0000000p-1f, -0x1.f6297c0000000p-1f};
__device__ constexpr float kSin32[16] = {0x0p+0f, 0x1.8f8b840000000p-3f, 0x1.87de2a0000000p-2f, 0x1.1c73b40000000p-1f, 0x1.6a09e60000000p-1f, 0x1.a9b6620000000p-1f, 0x1.d906bc0000000p-1f, 0x1.f6297c0000000p-1f, 0x1.0000000000000p+0f, 0x1.f6297c0000000p-1f, 0x1.d906bc0000000p-1f, 0x1.a9b6620000000p-1f, 0x1.6a09e60000000p-1f, 0x1.1c73b40000000p-1f, 0x1.87de2a0000000p-2f, 0x1.8f8b840000000p-3f};

template <int N>
__host__ __device__ constexpr int bitrev(int i) {
  int r = 0;
  for (int b = 1; b < N; b <<= 1) {
    r = (r << 1) | (i & 1);
    i >>= 1;
  }
  return r;
}

// v * e^{-+2 pi i m / N} (INV: +), m < N / 2 known at compile time after unrolling
template <int N, bool INV>
__device__ __forceinline__ c32 twiddle_mul(c32 v, int m) {
  if (m == 0) return v;
  if (4 * m == N) return INV ? make_float2(-v.y, v.x) : make_float2(v.y, -v.x);     // * (+i) / (-i)
  const int t = m * (32 / N);
  const float c = kCos32[t], s = INV ? kSin32[t] : -kSin32[t];
  return make_float2(v.x * c - v.y * s, v.x * s + v.y * c);
}

template <int N, bool INV>
__device__ __forceinline__ void fft_reg(c32 (&x)[N]) {
#pragma unroll
  for (int i = 0; i < N; ++i) {
    const int j = bitrev<N>(i);
    if (j > i) {
      const c32 t = x[i];
      x[i] = x[j];
      x[j] = t;
    }
  }
#pragma unroll
  for (int len = 2; len <= N; len <<= 1) {
#pragma unroll
    for (int i = 0; i < N; i += len) {
#pragma unroll
      for (int k = 0; k < len / 2; ++k) {
        const c32 u = x[i + k];
        const c32 v = twiddle_mul<N, INV>(x[i + k + len / 2], k * (N / len));
        x[i + k] = make_float2(u.x + v.x, u.y + v.y);
        x[i + k + len / 2] = make_float2(u.x - v.x, u.y - v.y);
      }
    }
  }
}

}  // namespace fiode_fft
