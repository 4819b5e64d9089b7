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
#include <stdlib.h>

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
constexpr int LDT = PB + 8;     // = 8 mod 64: every ds_read_b128 lane group of the products hits 64 distinct banks
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
      for (int r = 0; r < 4; ++r) UpdGJ::at(sm, 16 * w + 4 * q + r, 16 * bj + i) = acc[bj][r];
    __syncthreads();
    UpdGJ::invert(sm);
    UpdGJ::store(sm, P_next, PB, PB);
  }
}

// ---- persistent block inverse: the whole elimination in ONE launch ---------------------------
// For n = 64 NB (NB = 2..8: the 128 x 128 dynamics map, the two 512 x 512 backbone maps) the panel
// steps above are 1 + NB dependent launches of ~13 us each; their critical path is the look-ahead
// pivot inversion plus a kernel boundary per step.  k_pinv runs them inside one launch:
//   * one "chain" workgroup (blockIdx.x 0) computes every pivot block itself,
//       X_kk^(k-1) = X_kk^(k-2) - X_k,k-1^(k-2) (P_{k-1} X_k-1,k^(k-2)),   P_k = (X_kk^(k-1))^-1
//     (two 64^3 MFMA products + the gjb.h blocked Gauss-Jordan), and publishes P_k;
//   * NB^2 tile workgroups each keep one 64 x 64 tile of X in registers and apply step k once P_k
//     is published: X_kk <- P_k,  X_ik <- -X_ik P_k,  X_kj <- P_k X_kj,
//     X_ij <- X_ij - X_ik^(k-1) (P_k X_kj^(k-1)) -- the operands of step k are tiles of version k-1,
//     published by their owners into per-version slots (written once each: no write-after-read);
//   * per step the chain's inputs are tiles of version k-2, so the tile workgroups have a whole
//     pivot inversion of slack: the step's critical path is the chain's two products + one 64 x 64
//     inversion + one hand-off of P_k, with no kernel boundary.
// Hand-offs follow cdna_hip_programming.md Guideline 16: payload tiles are 16-B sc1 (write-through)
// buffer stores, every storing wave drains vmcnt before the workgroup barrier, one lane stores the
// flag (agent-scope atomic); the consumer polls the phase's flags relaxed from one lane, takes ONE
// agent-scope acquire, drains it before the barrier, and loads (16-B sc1 buffer loads).  Correctness does
// not depend on placement or residency order (a workgroup that waits only ever waits for data of
// earlier steps, which depend on nothing later); every spin is bounded (~0.5 s: the output turns
// NaN).  The flags are zeroed by a memset node in front of every launch (cdna_hip_programming.md
// Guideline 16, "Re-initialise every call"): nothing carries over between calls, whatever else
// the caller's workspace was used for.
// Tiles travel in the MFMA accumulator layout: f4 e = (4 rw + bj) 64 + lane holds rows 16 rw + 4 q
// + (0..3), column 16 bj + i of the tile (lane = 16 q + i).  Round-5 phase timestamps of the 512
// inverse with 4-wave workgroups (fiode_debug_pinv_profile): per step the 64 x 64 inversion 8.5 us,
// the two products 2.8 us, the hand-off 0.7 us, the tile workgroups done ~4.5 us after P_k -- so the
// workgroups are 8 waves: the inversion's rank-16 updates and the products spread over twice the
// SIMDs (the tile workgroups use them too).
constexpr int PI_TILE = PB * PB;                   // floats per tile
constexpr unsigned PI_SPIN_LIMIT = 1u << 22;

struct PinvWs {                                    // per-system workspace layout (floats / words)
  static __host__ __device__ size_t flag_words(int nb) { return (size_t)nb * nb * nb + nb; }
  static __host__ __device__ size_t flag_floats(int nb) { return (flag_words(nb) + 63) / 64 * 64; }
  static __host__ __device__ size_t total_floats(int nb) {      // + an n x n copy of the input for in == out
    return flag_floats(nb) + (size_t)nb * nb * nb * PI_TILE + (size_t)nb * PI_TILE + (size_t)nb * nb * PI_TILE;
  }
  static __host__ __device__ size_t copy_offset(int nb) { return total_floats(nb) - (size_t)nb * nb * PI_TILE; }
};

__device__ __forceinline__ __amdgpu_buffer_rsrc_t pi_rsrc(const float* base, size_t floats) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(base), 0, (int)(floats * sizeof(float)), 0x00020000);
}
typedef unsigned int pi_u4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ f4v pi_load(__amdgpu_buffer_rsrc_t r, int e) {      // sc1: L2-served, fresh
  const pi_u4 u = __builtin_amdgcn_raw_buffer_load_b128(r, e * 16, 0, 16);
  return f4v{__uint_as_float(u[0]), __uint_as_float(u[1]), __uint_as_float(u[2]), __uint_as_float(u[3])};
}
__device__ __forceinline__ void pi_store(__amdgpu_buffer_rsrc_t r, int e, f4v v) {   // sc1: write-through
  const pi_u4 u = pi_u4{__float_as_uint(v[0]), __float_as_uint(v[1]), __float_as_uint(v[2]), __float_as_uint(v[3])};
  __builtin_amdgcn_raw_buffer_store_b128(u, r, e * 16, 0, 16);
}
typedef __attribute__((address_space(1))) unsigned int gu32_t;
__device__ __forceinline__ void pi_signal(unsigned* flag) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");          // every storing wave drains its stores
  __syncthreads();
  if (threadIdx.x == 0) __hip_atomic_store((gu32_t*)flag, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// one lane polls (relaxed, bounded: *dead set after the spin limit); after the last poll of a phase
// the workgroup barrier (pi_acquire), with the polling lane's agent-scope acquire in front of it only
// when `acq` (FIODE_PINV_ACQUIRE=1): every load of handed-off bytes is a 16-B sc1 buffer load of
// bytes stored sc1 and drained before the flag, the form MI355X_MICROARCH.md lists as valid without
// the acquire ("Valid forms", row 1).
__device__ __forceinline__ void pi_poll(const unsigned* flag, int& dead, unsigned limit) {
  if (threadIdx.x == 0 && !dead) {
    unsigned spins = 0;
    while (__hip_atomic_load((gu32_t*)flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0u) {
      if (++spins > limit) {
        dead = 1;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
  }
}
__device__ __forceinline__ void pi_acquire(bool acq) {
  if (acq && threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");     // (no instruction: keeps the loads below)
  __syncthreads();
}
// 512-thread workgroups (8 waves): wave w owns rows 16 (w & 3) .. + 15 and the column blocks
// bj = 2 (w >> 2) + b, b = 0, 1 of a tile, i.e. acc[b][r] = X[16 rw + 4 q + r][16 (2 ch + b) + i]
// (rw = w & 3, ch = w >> 2, lane = 16 q + i) -- a 64^3 product is 32 MFMAs per wave.
constexpr int PI_NT = 512;
// k_pinv's LDS tiles: 64 x 64, no padding, XOR-swizzled like gjb.h's image (element (a, b) of a tile at
// [a][b ^ 4 (a & 15)]): the b128 operand reads, the b128 / b32 stores of the accumulators and of the
// published tiles, and the b32 reads all conflict-free (the padded stride 72 left the stores and
// b32 accesses 2-way: bank-conflict share 0.28, r05u)
constexpr int LDTS = PB;
__device__ __forceinline__ int tsw(int a, int b) { return b ^ ((a & 15) << 2); }
// a published tile -> LDS, column-major (B operand: dst[col][row]) or row-major (A operand)
__device__ __forceinline__ void pi_put_bt(float (*dst)[LDTS], int e, f4v v) {   // f4 e of a tile, column-major
  const int w = e >> 8, bj = (e >> 6) & 3, ln = e & 63;
  const int a = 16 * bj + (ln & 15);
  *reinterpret_cast<f4v*>(&dst[a][tsw(a, 16 * w + 4 * (ln >> 4))]) = v;
}
__device__ __forceinline__ void pi_put_a(float (*dst)[LDTS], int e, f4v v) {    // f4 e of a tile, row-major
  const int w = e >> 8, bj = (e >> 6) & 3, ln = e & 63;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int a = 16 * w + 4 * (ln >> 4) + k;
    dst[a][tsw(a, 16 * bj + (ln & 15))] = v[k];
  }
}
__device__ __forceinline__ void pi_to_bt(float (*dst)[LDTS], __amdgpu_buffer_rsrc_t r) {
#pragma unroll
  for (int u = 0; u < 1024 / PI_NT; ++u) pi_put_bt(dst, threadIdx.x + PI_NT * u, pi_load(r, threadIdx.x + PI_NT * u));
}
__device__ __forceinline__ void pi_to_a(float (*dst)[LDTS], __amdgpu_buffer_rsrc_t r) {
#pragma unroll
  for (int u = 0; u < 1024 / PI_NT; ++u) pi_put_a(dst, threadIdx.x + PI_NT * u, pi_load(r, threadIdx.x + PI_NT * u));
}
// Where the matrix to invert comes from: a row-major n x n array (PlainSrc), or built on load from a
// dense Cayley map's weight (DenseSrc: M = I + s (U' - U'^T) + s^2 G with s = alpha / ||W||, the
// arithmetic of dense.hip k_dense_prep element for element -- the same M bit for bit, so the fused
// map forward needs no prep launch and no M buffer).  bind(m): the batch entry; all threads call it.
struct PlainSrc {
  const float* in;
  int64_t stride;
  int n;
  __device__ void bind(int m, float*) { in += (int64_t)m * stride; }
  __device__ float at(int r, int c) const { return in[(int64_t)r * n + c]; }
  __device__ f4v row4(int r, int c4) const { return *reinterpret_cast<const f4v*>(in + (int64_t)r * n + c4); }
};
struct DenseSrc {
  const float* W;        // [b][cout][cin]
  const float* G;        // [b][k][k] or null (square maps)
  const float* alpha;    // [b]
  const float* part;     // [b][256] squared-norm partials (fiode_dense_norm_partials*)
  float* nrm_out;        // [b]
  int cout, cin, k, wide;
  float s;
  __device__ void bind(int m, float* slot) {
    W += (int64_t)m * cout * cin;
    if (G) G += (int64_t)m * k * k;
    if (threadIdx.x < 64) {               // dense.hip dense_norm: the same fixed order
      const float* pb = part + m * 256 + 4 * threadIdx.x;
      float v = (pb[0] + pb[1]) + (pb[2] + pb[3]);
      for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
      if (threadIdx.x == 0) {
        *slot = sqrtf(v);
        if (nrm_out && blockIdx.x == 0) nrm_out[m] = *slot;
      }
    }
    __syncthreads();
    s = alpha[m] / *slot;
  }
  __device__ float wx(int r, int c) const { return wide ? W[(int64_t)c * cin + r] : W[(int64_t)r * cin + c]; }
  __device__ float at(int r, int c) const {
    float v = s * (wx(r, c) - wx(c, r));
    if (G) v = fmaf(s * s, G[(int64_t)r * k + c], v);
    if (r == c) v += 1.0f;
    return v;
  }
  __device__ f4v row4(int r, int c4) const { return f4v{at(r, c4), at(r, c4 + 1), at(r, c4 + 2), at(r, c4 + 3)}; }
};
// a 64 x 64 block of a row-major matrix (row stride ld) -> LDS, row-major or transposed
template <class Src>
__device__ __forceinline__ void pi_tile_load(float (*dst)[LDTS], const Src& src, int r0, int c0, bool transpose) {
#pragma unroll
  for (int u = 0; u < PB * PB / 4 / PI_NT; ++u) {
    const int t = threadIdx.x + PI_NT * u;
    // transposed: lanes on consecutive rows r, so the b32 stores of one column hit 32 distinct banks
    // (row-fastest lanes put 16 lanes of a group on one bank)
    const int r = transpose ? t % PB : t / (PB / 4), c4 = transpose ? (t / PB) * 4 : (t % (PB / 4)) * 4;
    const f4v v = src.row4(r0 + r, c0 + c4);
    if (transpose) {
#pragma unroll
      for (int e = 0; e < 4; ++e) dst[c4 + e][tsw(c4 + e, r)] = v[e];
    } else {
      *reinterpret_cast<f4v*>(&dst[r][tsw(r, c4)]) = v;
    }
  }
}
// this thread's accumulator registers <-> LDS (row-major A image / column-major B image)
__device__ __forceinline__ void acc_to_a(float (*dst)[LDTS], const f4v (&acc)[2], int rw, int ch, int i, int q) {
#pragma unroll
  for (int b = 0; b < 2; ++b)
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int a = 16 * rw + 4 * q + k;
      dst[a][tsw(a, 16 * (2 * ch + b) + i)] = acc[b][k];
    }
}
__device__ __forceinline__ void acc_to_bt(float (*dst)[LDTS], const f4v (&acc)[2], int rw, int ch, int i, int q) {
#pragma unroll
  for (int b = 0; b < 2; ++b) {
    const int a = 16 * (2 * ch + b) + i;
    *reinterpret_cast<f4v*>(&dst[a][tsw(a, 16 * rw + 4 * q)]) = acc[b];
  }
}
// acc[b] += sign A[16 rw + i][:] . BT[16 (2 ch + b) + i][:]  (the k order permuted as tile_gemm's)
__device__ __forceinline__ void pi_gemm(const float (*A)[LDTS], const float (*BT)[LDTS], int rw, int ch, int i, int q,
                                        f4v (&acc)[2], float sign) {
#pragma unroll
  for (int kc = 0; kc < PB / 16; ++kc) {
    const int aa = 16 * rw + i;
    const f4v a4 = *reinterpret_cast<const f4v*>(&A[aa][tsw(aa, 16 * kc + 4 * q)]) * sign;
#pragma unroll
    for (int b = 0; b < 2; ++b) {
      const int ab = 16 * (2 * ch + b) + i;
      const f4v b4 = *reinterpret_cast<const f4v*>(&BT[ab][tsw(ab, 16 * kc + 4 * q)]);
#pragma unroll
      for (int s = 0; s < 4; ++s) acc[b] = fiode_gjb::mfma(a4[s], b4[s], acc[b]);
    }
  }
}

// MFMA results consumed across control flow: hipcc (ROCm 7.2, gfx950) was seen moving an MFMA's
// accumulator (v_accvgpr_mov) at a branch join without the wait states the dependent read needs
// (k_pinv<2>: one accumulator register of the column tiles read before the last 16x16x4 MFMA had
// written it, tools/probes/pinv_probe.py).  Pinning the accumulators in AGPRs through an asm that
// holds the SIMD for the MFMA's full latency keeps every later copy behind the write.
__device__ __forceinline__ void mfma_settle(f4v (&acc)[2]) {
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 3" : "+a"(acc[0]), "+a"(acc[1]));
}

template <int NB, class Src>
__global__ void __launch_bounds__(PI_NT) k_pinv(Src src, float* __restrict__ out, float* __restrict__ qout,
                                                float* ws_all, int64_t wstride, const int32_t* __restrict__ skip,
                                                int acq, unsigned long long* prof, unsigned spin_limit, int prio) {
  if (skip && *skip) return;                  // (uniform)
  fiode_wave_prio(prio);
  constexpr int n = NB * PB;
  __shared__ __attribute__((aligned(16))) float lds[4][PB][LDTS];
  __shared__ int dead;
  __shared__ float slot;
  const int m = blockIdx.y;
  src.bind(m, &slot);
  out += (int64_t)m * n * n;
  if (qout) qout += (int64_t)m * n * n;
  float* ws = ws_all + (int64_t)m * wstride;
  unsigned* tflag = reinterpret_cast<unsigned*>(ws);                 // [NB][NB][NB]
  unsigned* pflag = tflag + NB * NB * NB;                            // [NB]
  float* V = ws + PinvWs::flag_floats(NB);                           // [NB versions][NB][NB] tiles
  float* Pt = V + (size_t)NB * NB * NB * PI_TILE;                    // [NB] tiles
  const size_t vfloats = (size_t)NB * NB * NB * PI_TILE;
  const __amdgpu_buffer_rsrc_t rV = pi_rsrc(V, vfloats), rP = pi_rsrc(Pt, (size_t)NB * PI_TILE);
  auto vtile = [&](int ver, int ti, int tj) { return ((ver * NB + ti) * NB + tj) * (PI_TILE / 4); };   // f4 index
  auto ptile = [&](int k) { return k * (PI_TILE / 4); };
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, i = lane & 15, q = lane >> 4;
  const int rw = w & 3, ch = w >> 2;
  auto own_e = [&](int b) { return (4 * rw + 2 * ch + b) * 64 + lane; };   // f4 index of acc[b]
  if (threadIdx.x == 0) dead = 0;
  // diagnostic timestamps (fiode_debug_pinv_profile; null in the product): prof[1024 + wg] start,
  // chain prof[8 k + 0..3], tile t's step k end prof[256 + t NB + k]
  auto mark = [&](int slot) {
    if (prof && threadIdx.x == 0 && m == 0) prof[slot] = wall_clock64();
  };
  mark(1024 + blockIdx.x);
  __syncthreads();
  f4v acc[2];
  auto load_in = [&](int r0, int c0) {
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int r = 0; r < 4; ++r) acc[b][r] = src.at(r0 + 16 * rw + 4 * q + r, c0 + 16 * (2 * ch + b) + i);
  };

  if (blockIdx.x == 0) {
    // ---- the chain: every pivot block and its inverse --------------------------------------------
    typedef fiode_gjb::GJB<PB, PI_NT / 64> CG;
    static_assert(sizeof(CG::Smem) <= 2 * sizeof(float) * PB * LDTS, "pivot scratch fits two LDS tiles");
    CG::Smem& sm = *reinterpret_cast<CG::Smem*>(&lds[0][0][0]);     // cm = lds[0] (same swizzle as the tiles)
    float (*sX)[LDTS] = lds[2];
    float (*sB)[LDTS] = lds[3];
    static_assert(CG::LDM == LDTS, "the pivot image doubles as the product's A operand");
    for (int t = threadIdx.x; t < PB * PB / 4; t += PI_NT) {         // X_00 (gjb.h load's layout)
      const int r = t / (PB / 4), c4 = (t % (PB / 4)) * 4;
      *CG::at4(sm, r, c4) = src.row4(r, c4);
    }
    __syncthreads();
    // the next pivot's three operand tiles (version k - 1 for step k + 1), fetched into registers
    // while the current pivot block is inverted: polled and loaded from the inversion's hook
    f4v nxt_b[2], nxt_a[2], nxt_d[2];
    for (int k = 0;; ++k) {
      const int k1 = k + 1;
      auto fetch = [&]() {
        if (k1 >= NB || k == 0) return;
        pi_poll(&tflag[((k - 1) * NB + k) * NB + k1], dead, spin_limit);
        pi_poll(&tflag[((k - 1) * NB + k1) * NB + k], dead, spin_limit);
        pi_poll(&tflag[((k - 1) * NB + k1) * NB + k1], dead, spin_limit);
        pi_acquire(acq);
        const __amdgpu_buffer_rsrc_t r0 = pi_rsrc(V + (size_t)vtile(k - 1, k, k1) * 4, PI_TILE);
        const __amdgpu_buffer_rsrc_t r1 = pi_rsrc(V + (size_t)vtile(k - 1, k1, k) * 4, PI_TILE);
        const __amdgpu_buffer_rsrc_t r2 = pi_rsrc(V + (size_t)vtile(k - 1, k1, k1) * 4, PI_TILE);
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          nxt_b[u] = pi_load(r0, threadIdx.x + PI_NT * u);
          nxt_a[u] = pi_load(r1, threadIdx.x + PI_NT * u);
          nxt_d[u] = pi_load(r2, own_e(u));
        }
      };
      mark(8 * k + 0);
      CG::invert(sm, fetch, 1);                                      // cm: P_k (row-major)
      mark(8 * k + 1);
      // a timed-out chain publishes P_k as NaN: every tile applies every step's P_k, so the whole
      // output turns NaN instead of finite values built from stale workspace tiles
      const float cpz = dead ? __builtin_nanf("") : 0.f;
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        f4v v;
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = CG::at(sm, 16 * rw + 4 * q + r, 16 * (2 * ch + b) + i) + cpz;
        pi_store(rP, ptile(k) + own_e(b), v);
      }
      pi_signal(&pflag[k]);
      mark(8 * k + 2);
      if (k1 == NB) break;
      // X_{k+1,k+1}^(k) = X_{k+1,k+1}^(k-1) - X_{k+1,k}^(k-1) (P_k X_{k,k+1}^(k-1))
      if (k == 0) {                                                  // version -1 = the input
        pi_tile_load(sB, src, 0, k1 * PB, true);                     // X_01 (column-major)
        pi_tile_load(sX, src, k1 * PB, 0, false);                    // X_10
        load_in(k1 * PB, k1 * PB);
      } else {
#pragma unroll
        for (int u = 0; u < 2; ++u) {                                // the prefetched tiles -> LDS / acc
          const int e = threadIdx.x + PI_NT * u;
          pi_put_bt(sB, e, nxt_b[u]);
          pi_put_a(sX, e, nxt_a[u]);
          acc[u] = nxt_d[u];
        }
      }
      __syncthreads();
      f4v t[2] = {f4v{0.f, 0.f, 0.f, 0.f}, f4v{0.f, 0.f, 0.f, 0.f}};
      pi_gemm(sm.cm, sB, rw, ch, i, q, t, 1.0f);                     // T = P_k X_{k,k+1}
      mfma_settle(t);
      __syncthreads();
      acc_to_bt(sB, t, rw, ch, i, q);
      __syncthreads();
      pi_gemm(sX, sB, rw, ch, i, q, acc, -1.0f);                     // X_{k+1,k+1} - X_{k+1,k} T
      mfma_settle(acc);
      __syncthreads();                                               // every wave is done with cm (A of T)
      acc_to_a(sm.cm, acc, rw, ch, i, q);
      __syncthreads();
      mark(8 * k + 3);
    }
  } else {
    // ---- one tile of X ---------------------------------------------------------------------------
    const int t = blockIdx.x - 1, ti = t / NB, tj = t % NB;
    float (*sA)[LDTS] = lds[0];
    float (*sB)[LDTS] = lds[1];
    float (*sX)[LDTS] = lds[2];
    load_in(ti * PB, tj * PB);
    for (int k = 0; k < NB; ++k) {
      if (ti == tj && k == ti - 1) continue;       // X_kk^(k-1) is the chain's; nobody reads this one
      const bool generic = ti != k && tj != k;
      pi_poll(&pflag[k], dead, spin_limit);
      if (generic && k > 0) {                      // this step's operands of version k - 1
        pi_poll(&tflag[((k - 1) * NB + k) * NB + tj], dead, spin_limit);
        pi_poll(&tflag[((k - 1) * NB + ti) * NB + k], dead, spin_limit);
      }
      pi_acquire(acq);
      const __amdgpu_buffer_rsrc_t rp = pi_rsrc(Pt + (size_t)ptile(k) * 4, PI_TILE);
      if (ti == k && tj == k) {                                      // X_kk <- P_k
#pragma unroll
        for (int b = 0; b < 2; ++b) acc[b] = pi_load(rp, own_e(b));
      } else if (tj == k) {                                          // X_ik <- -X_ik P_k
        acc_to_a(sA, acc, rw, ch, i, q);
        pi_to_bt(sB, rp);
        __syncthreads();
#pragma unroll
        for (int b = 0; b < 2; ++b) acc[b] = f4v{0.f, 0.f, 0.f, 0.f};
        pi_gemm(sA, sB, rw, ch, i, q, acc, -1.0f);
        mfma_settle(acc);
      } else if (ti == k) {                                          // X_kj <- P_k X_kj
        pi_to_a(sA, rp);
        acc_to_bt(sB, acc, rw, ch, i, q);
        __syncthreads();
#pragma unroll
        for (int b = 0; b < 2; ++b) acc[b] = f4v{0.f, 0.f, 0.f, 0.f};
        pi_gemm(sA, sB, rw, ch, i, q, acc, 1.0f);
        mfma_settle(acc);
      } else {                                                       // X_ij - X_ik (P_k X_kj)
        pi_to_a(sA, rp);
        if (k == 0) {
          pi_tile_load(sB, src, 0, tj * PB, true);                   // X_0j, column-major
          pi_tile_load(sX, src, ti * PB, 0, false);                  // X_i0
        } else {
          pi_to_bt(sB, pi_rsrc(V + (size_t)vtile(k - 1, k, tj) * 4, PI_TILE));
          pi_to_a(sX, pi_rsrc(V + (size_t)vtile(k - 1, ti, k) * 4, PI_TILE));
        }
        __syncthreads();
        f4v r4[2] = {f4v{0.f, 0.f, 0.f, 0.f}, f4v{0.f, 0.f, 0.f, 0.f}};
        pi_gemm(sA, sB, rw, ch, i, q, r4, 1.0f);                     // R_kj = P_k X_kj
        mfma_settle(r4);
        __syncthreads();                                             // every wave is done reading sB
        acc_to_bt(sB, r4, rw, ch, i, q);
        __syncthreads();
        pi_gemm(sX, sB, rw, ch, i, q, acc, -1.0f);
        mfma_settle(acc);
      }
      // publish version k where step k + 1 or the chain reads it
      const bool rowcol = (ti == k + 1) != (tj == k + 1);
      if (k + 1 < NB && (rowcol || (ti == tj && ti == k + 2))) {
        const float tpz = dead ? __builtin_nanf("") : 0.f;     // a timed-out tile poisons what it hands on
#pragma unroll
        for (int b = 0; b < 2; ++b) pi_store(rV, vtile(k, ti, tj) + own_e(b), acc[b] + tpz);
        pi_signal(&tflag[(k * NB + ti) * NB + tj]);
      }
      mark(256 + t * NB + k);
      __syncthreads();                                               // LDS images reused next step
    }
    const float poison = dead ? __builtin_nanf("") : 0.f;
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int gi = ti * PB + 16 * rw + 4 * q + r, gj = tj * PB + 16 * (2 * ch + b) + i;
        const float v = acc[b][r] + poison;
        out[(int64_t)gi * n + gj] = v;
        if (qout) {                           // a square dense map's Q = 2 inv - I (k_dense_finish's arithmetic)
          float qv = 2.0f * v;
          if (gi == gj) qv -= 1.0f;
          qout[(int64_t)gi * n + gj] = qv;
        }
      }
  }
}

// spin bound of every k_pinv poll (fiode_debug_set_pinv_spin_limit lowers it to test the timeout path)
unsigned g_pinv_spin_limit = PI_SPIN_LIMIT;

int pinv_acquire_knob() {
  static const int acq = [] {
    const char* e = getenv("FIODE_PINV_ACQUIRE");
    return e && e[0] == '1' ? 1 : 0;
  }();
  return acq;
}

template <int NB, class Src>
int launch_pinv_src(hipStream_t st, int batch, Src src, float* out, float* qout, float* ws, int64_t wstride,
                    const int32_t* skip, bool clear_flags, unsigned long long* prof = nullptr) {
  // the flag block of every system: its first flag_floats(NB) floats (a multiple of 16 bytes)
  if (clear_flags)
    FIODE_HIP_CHECK(hipMemset2DAsync(ws, (size_t)wstride * sizeof(float), 0, PinvWs::flag_floats(NB) * sizeof(float),
                                     (size_t)batch, st));
  hipLaunchKernelGGL((k_pinv<NB, Src>), dim3(1 + NB * NB, batch), dim3(PI_NT), 0, st, src, out, qout, ws, wstride, skip,
                     pinv_acquire_knob(), prof, g_pinv_spin_limit, (int)((g_fiode_prio_mask >> 3) & 1));
  return FIODE_OK;
}

template <int NB>
int launch_pinv(hipStream_t st, int batch, const float* in, int64_t in_stride, float* out, float* ws, int64_t wstride,
                const int32_t* skip, unsigned long long* prof = nullptr) {
  return launch_pinv_src<NB>(st, batch, PlainSrc{in, in_stride, NB * PB}, out, nullptr, ws, wstride, skip, true, prof);
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

namespace {
bool pinv_shape(int n) { return n % PB == 0 && n / PB >= 2 && n / PB <= 8; }
}  // namespace

extern "C" size_t fiode_block_inverse_workspace_bytes(int32_t n) {
  if (n < 1) return 0;
  if (pinv_shape(n)) return PinvWs::total_floats(n / PB) * sizeof(float);   // flags + tile versions + pivots
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
  if (pinv_shape(n)) {
    float* ws = (float*)workspace;
    int64_t in_stride = (int64_t)n * n;
    if (in == out) {        // the tile workgroups write `out` while others may still read `in`: copy it
      float* cp = ws + PinvWs::copy_offset(nb);
      FIODE_HIP_CHECK(hipMemcpy2DAsync(cp, (size_t)wstride * sizeof(float), in, (size_t)n * n * sizeof(float),
                                       (size_t)n * n * sizeof(float), (size_t)batch, hipMemcpyDeviceToDevice, st));
      in = cp;
      in_stride = wstride;
    }
    int rc = FIODE_OK;
    switch (nb) {
      case 2: rc = launch_pinv<2>(st, batch, in, in_stride, out, ws, wstride, skip); break;
      case 3: rc = launch_pinv<3>(st, batch, in, in_stride, out, ws, wstride, skip); break;
      case 4: rc = launch_pinv<4>(st, batch, in, in_stride, out, ws, wstride, skip); break;
      case 5: rc = launch_pinv<5>(st, batch, in, in_stride, out, ws, wstride, skip); break;
      case 6: rc = launch_pinv<6>(st, batch, in, in_stride, out, ws, wstride, skip); break;
      case 7: rc = launch_pinv<7>(st, batch, in, in_stride, out, ws, wstride, skip); break;
      default: rc = launch_pinv<8>(st, batch, in, in_stride, out, ws, wstride, skip); break;
    }
    if (rc) return rc;
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? FIODE_OK : FIODE_EHIP + (int)e;
  }
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

// Diagnostic (not in fiode.h): the wave-priority mask of common.h (g_fiode_prio_mask); returns the
// previous mask.  Default: the rk4 train solve's two latency chains (k_ot_fwd4, k_ot_bwd4) raised over
// the fan-out kernels sharing their CUs -- interleaved step A/B 1.2344 -> 1.2297 ms (mask 3; 1 alone
// 1.2320; the small maps / k_pinv no gain: profiles/r06/ab_wave_prio.json).  tools/ab_step.py `prio_*`.
unsigned g_fiode_prio_mask = 3;
extern "C" FIODE_API unsigned fiode_debug_set_prio_mask(unsigned mask) {
  const unsigned prev = g_fiode_prio_mask;
  g_fiode_prio_mask = mask;
  return prev;
}

// Diagnostic (not in fiode.h): the spin bound of k_pinv's polls (0 restores the default); returns the
// previous bound.  A test lowers it so that polls time out and checks that no finite output is wrong.
extern "C" FIODE_API unsigned fiode_debug_set_pinv_spin_limit(unsigned limit) {
  const unsigned prev = g_pinv_spin_limit;
  g_pinv_spin_limit = limit ? limit : PI_SPIN_LIMIT;
  return prev;
}

// Diagnostic (not in fiode.h): the one-launch inverse of one n = 512 system with phase timestamps
// (wall clock, 100 MHz) -- tools/probes/pinv_probe.py.
extern "C" FIODE_API int fiode_debug_pinv_profile(void* stream, int32_t n, const float* in, float* out, void* workspace,
                                        unsigned long long* prof) {
  if (n != 512 || !in || !out || !workspace || !prof || in == out) return FIODE_EINVAL;
  const int64_t wstride = (int64_t)(fiode_block_inverse_workspace_bytes(n) / sizeof(float));
  return launch_pinv<8>((hipStream_t)stream, 1, in, (int64_t)n * n, out, (float*)workspace, wstride, nullptr, prof);
}

// ---- the dense Cayley map's inverse, its M built on load ----------------------------------------
// fiode_dense_cayley_inverse: for each [cout][cin] matrix b of the batch (k = min(cout, cin) = 128 ..
// 512 in steps of 64): s = alpha[b] / ||W_b|| from the 256 norm partials (fiode_dense_norm_partials*),
// M = I + s (U' - U'^T) + s^2 G (G = V'^T V' for tall / wide maps, null for square ones) -- built by
// the inverse's own loads, so no prep launch and no M buffer -- and inv = M^-1 -> inv_out [b][k][k],
// ||W_b|| -> nrm_out [b]; for a square map also Q = 2 inv - I -> q_out (the whole map: no finish
// launch; tall / wide maps keep fiode_dense_cayley_finish for Q).  The workspace's flag words (the
// first fiode_dense_inverse_flag_bytes(k) bytes of each matrix's fiode_block_inverse_workspace_bytes(k)
// stride) must be zero: fiode_dense_norm_partials_clear zeroes them in the same launch as the partials.
extern "C" FIODE_API size_t fiode_dense_inverse_flag_bytes(int32_t k) {
  return pinv_shape(k) ? PinvWs::flag_floats(k / PB) * sizeof(float) : 0;
}

extern "C" FIODE_API int fiode_dense_cayley_inverse(void* stream, const fiode_dense_config* cfg, const float* W,
                                                    const float* alpha, const float* part, const float* G,
                                                    float* nrm_out, float* inv_out, float* q_out, void* workspace,
                                                    size_t workspace_bytes) {
  if (!cfg || cfg->batch < 1 || cfg->batch > 65535 || cfg->cout < 1 || cfg->cin < 1) return FIODE_EINVAL;
  const int k = cfg->cout < cfg->cin ? cfg->cout : cfg->cin, R = cfg->cout < cfg->cin ? cfg->cin : cfg->cout;
  if (!pinv_shape(k)) return FIODE_ESHAPE;
  if (!W || !alpha || !part || !nrm_out || !inv_out || !workspace || (R > k && !G) || (q_out && R > k))
    return FIODE_EINVAL;
  const size_t per = fiode_block_inverse_workspace_bytes(k);
  if (workspace_bytes < (size_t)cfg->batch * per) return FIODE_EWORKSPACE;
  DenseSrc src{W, R > k ? G : nullptr, alpha, part, nrm_out, cfg->cout, cfg->cin, k, cfg->cin > cfg->cout ? 1 : 0, 0.f};
  hipStream_t st = (hipStream_t)stream;
  float* ws = (float*)workspace;
  const int64_t wstride = (int64_t)(per / sizeof(float));
  int rc = FIODE_OK;
  switch (k / PB) {
    case 2: rc = launch_pinv_src<2>(st, cfg->batch, src, inv_out, q_out, ws, wstride, nullptr, false); break;
    case 3: rc = launch_pinv_src<3>(st, cfg->batch, src, inv_out, q_out, ws, wstride, nullptr, false); break;
    case 4: rc = launch_pinv_src<4>(st, cfg->batch, src, inv_out, q_out, ws, wstride, nullptr, false); break;
    case 5: rc = launch_pinv_src<5>(st, cfg->batch, src, inv_out, q_out, ws, wstride, nullptr, false); break;
    case 6: rc = launch_pinv_src<6>(st, cfg->batch, src, inv_out, q_out, ws, wstride, nullptr, false); break;
    case 7: rc = launch_pinv_src<7>(st, cfg->batch, src, inv_out, q_out, ws, wstride, nullptr, false); break;
    default: rc = launch_pinv_src<8>(st, cfg->batch, src, inv_out, q_out, ws, wstride, nullptr, false); break;
  }
  if (rc) return rc;
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? FIODE_OK : FIODE_EHIP + (int)e;
}
