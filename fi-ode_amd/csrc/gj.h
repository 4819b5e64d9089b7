// Register-resident batched Gauss-Jordan inverse of positive-real matrices (gfx950).
//
// Shared by cayley.hip (fiode_batched_inverse) and the fused spectral Cayley kernels
// (spectral.hip).  The matrix M = I + A of a Cayley map has Hermitian part I + V^H V >= I, so
// elimination in natural order needs no pivot search and never meets a singular pivot block.
//
// Thread t of the workgroup owns a TR x TC register tile.  One round eliminates the 2 x 2 pivot
// block K = {k, k+1}: the owners of rows / columns K stage them in LDS (double-buffered by round
// parity: one barrier per round), every thread inverts the pivot block in closed form
// (P = M_KK^-1, one hardware reciprocal of the determinant) and applies
//   m_ij -= m_iK (P m_Kj)  (i, j not in K),  m_iK <- -m_iK P,  m_Kj <- P m_Kj,  m_KK <- P.
// The k loop is unrolled by U = max(TR, TC) so the tile position of every pivot row / column
// is a compile-time register index: the only run-time tests are "do I own the pivot row /
// column" (uniform across a thread's tile), no per-element selects.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace fiode_gj {

struct RealOps {
  typedef float T;
  static __device__ __forceinline__ T mul(T a, T b) { return a * b; }
  static __device__ __forceinline__ T sub_mul(T o, T c, T r) { return fmaf(-c, r, o); }
  static __device__ __forceinline__ T ident(bool d) { return d ? 1.0f : 0.0f; }
  static __device__ __forceinline__ T add(T a, T b) { return a + b; }
  static __device__ __forceinline__ T sub(T a, T b) { return a - b; }
  static __device__ __forceinline__ T neg(T a) { return -a; }
  static __device__ __forceinline__ T recip(T d) { return __builtin_amdgcn_rcpf(d); }
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
    const float r = __builtin_amdgcn_rcpf(d.x * d.x + d.y * d.y);
    return make_float2(d.x * r, -d.y * r);
  }
};

template <class Ops, int NP, int TR, int TC>
struct GJ {
  typedef typename Ops::T T;
  static constexpr int CT = NP / TC;                 // column tiles
  static constexpr int RT = NP / TR;                 // row tiles
  static constexpr int NT = RT * CT;                 // threads
  static constexpr int U = TR > TC ? TR : TC;        // unroll of the pivot loop
  static_assert(TR % 2 == 0 && TC % 2 == 0 && U % TR == 0 && U % TC == 0, "tile shape");
  // pivot rows in LDS: with 4 complex columns per thread (32 B), threads tj and tj + 8 of a 16-lane
  // group would read the same banks (2-way; LDS bank-conflict share 0.54 in k_spec_inv<64>), so every
  // 32 columns are shifted by 2 complex (4 banks)
  static constexpr bool ROW_PAD = sizeof(T) == 8 && TC == 4;
  static __device__ __forceinline__ int rc(int c) { return ROW_PAD ? c + (c >> 5) * 2 : c; }
  struct Smem {
    T rowk[2][2][ROW_PAD ? NP + NP / 16 : NP];   // [parity][pivot row 0/1][col (rc)]
    T colk[2][2][NP];                            // [parity][pivot col 0/1][row]
  };

  // Invert the n x n (n <= NP, padded with I) matrix held in a[][] by this workgroup's threads.
  static __device__ __forceinline__ void invert(T (&a)[TR][TC], int n, Smem& sm) {
    const int tid = threadIdx.x;
    const int ti = tid / CT, tj = tid % CT;
    const int r0 = ti * TR, c0 = tj * TC;
    const int kend = (n + U - 1) / U * U;
    for (int k0 = 0; k0 < kend; k0 += U) {
#pragma unroll
      for (int kk = 0; kk < U; kk += 2) {
        const int k = k0 + kk;
        const int b = (k >> 1) & 1;
        const int rr = kk % TR, cc = kk % TC;       // compile-time after unrolling
        const bool own_r = ti == (k0 + kk) / TR;
        const bool own_c = tj == (k0 + kk) / TC;
        if (own_r) {
#pragma unroll
          for (int c = 0; c < TC; ++c) {
            sm.rowk[b][0][rc(c0 + c)] = a[rr][c];
            sm.rowk[b][1][rc(c0 + c)] = a[rr + 1][c];
          }
        }
        if (own_c) {
#pragma unroll
          for (int r = 0; r < TR; ++r) {
            sm.colk[b][0][r0 + r] = a[r][cc];
            sm.colk[b][1][r0 + r] = a[r][cc + 1];
          }
        }
        __syncthreads();
        T cr0[TR], cr1[TR], x0[TC], x1[TC];
#pragma unroll
        for (int r = 0; r < TR; ++r) {
          cr0[r] = sm.colk[b][0][r0 + r];
          cr1[r] = sm.colk[b][1][r0 + r];
        }
#pragma unroll
        for (int c = 0; c < TC; ++c) {
          x0[c] = sm.rowk[b][0][rc(c0 + c)];
          x1[c] = sm.rowk[b][1][rc(c0 + c)];
        }
        const T q00 = sm.rowk[b][0][rc(k)], q01 = sm.rowk[b][0][rc(k + 1)];
        const T q10 = sm.rowk[b][1][rc(k)], q11 = sm.rowk[b][1][rc(k + 1)];
        const T idet = Ops::recip(Ops::sub(Ops::mul(q00, q11), Ops::mul(q01, q10)));
        const T p00 = Ops::mul(q11, idet), p11 = Ops::mul(q00, idet);
        const T p01 = Ops::neg(Ops::mul(q01, idet)), p10 = Ops::neg(Ops::mul(q10, idet));
        T rv0[TC], rv1[TC];
#pragma unroll
        for (int c = 0; c < TC; ++c) {
          rv0[c] = Ops::add(Ops::mul(p00, x0[c]), Ops::mul(p01, x1[c]));
          rv1[c] = Ops::add(Ops::mul(p10, x0[c]), Ops::mul(p11, x1[c]));
        }
#pragma unroll
        for (int r = 0; r < TR; ++r)
#pragma unroll
          for (int c = 0; c < TC; ++c) a[r][c] = Ops::sub_mul(Ops::sub_mul(a[r][c], cr0[r], rv0[c]), cr1[r], rv1[c]);
        if (own_c) {
#pragma unroll
          for (int r = 0; r < TR; ++r) {
            a[r][cc] = Ops::neg(Ops::add(Ops::mul(cr0[r], p00), Ops::mul(cr1[r], p10)));
            a[r][cc + 1] = Ops::neg(Ops::add(Ops::mul(cr0[r], p01), Ops::mul(cr1[r], p11)));
          }
        }
        if (own_r) {
#pragma unroll
          for (int c = 0; c < TC; ++c) {
            a[rr][c] = rv0[c];
            a[rr + 1][c] = rv1[c];
          }
          if (own_c) {
            a[rr][cc] = p00;
            a[rr][cc + 1] = p01;
            a[rr + 1][cc] = p10;
            a[rr + 1][cc + 1] = p11;
          }
        }
      }
    }
  }

  // Load a row-major n x n matrix (row stride ld) padded with the identity.
  static __device__ __forceinline__ void load(T (&a)[TR][TC], const T* __restrict__ src, int n, int64_t ld) {
    const int tid = threadIdx.x;
    const int r0 = (tid / CT) * TR, c0 = (tid % CT) * TC;
#pragma unroll
    for (int r = 0; r < TR; ++r)
#pragma unroll
      for (int c = 0; c < TC; ++c) {
        const int i = r0 + r, j = c0 + c;
        a[r][c] = (i < n && j < n) ? src[(int64_t)i * ld + j] : Ops::ident(i == j);
      }
  }

  static __device__ __forceinline__ void store(const T (&a)[TR][TC], T* __restrict__ dst, int n, int64_t ld) {
    const int tid = threadIdx.x;
    const int r0 = (tid / CT) * TR, c0 = (tid % CT) * TC;
#pragma unroll
    for (int r = 0; r < TR; ++r)
#pragma unroll
      for (int c = 0; c < TC; ++c) {
        const int i = r0 + r, j = c0 + c;
        if (i < n && j < n) dst[(int64_t)i * ld + j] = a[r][c];
      }
  }
};

}  // namespace fiode_gj
