// Blocked Gauss-Jordan inverse of positive-real f32 matrices, LDS-resident, MFMA updates (gfx950).
//
// Same algorithm family as gj.h (natural-order elimination: the pivot blocks of I + A with
// Hermitian part >= I are positive-real, never singular) but with 16-wide pivot blocks:
//   round kb (pivot block K = [16 kb, 16 kb + 16)):
//     R = P X[K, :]                      P = X[K, K]^-1, R row panel        (MFMA, 16 x 16 blocks)
//     X[i, j] -= X[i, K] R[:, j]         i, j not in K                     (MFMA, rank-16 update)
//     X[i, K] <- -X[i, K] P,  X[K, j] <- R[:, j],  X[K, K] <- P
// and the 16 x 16 pivot block inverted inside ONE wave in registers (16 pivot steps, broadcasts by
// DPP row_newbcast / v_permlane swaps: no LDS round trip, no barrier).  Look-ahead: the wave that
// updates the next round's pivot block inverts it at once, while the other waves finish the
// rank-16 update, so the per-round critical path is one 16 x 16 inversion + two barriers.
//
// Layout: the workgroup keeps the matrix "column-major" in LDS (cm[col][row]).  The kernel loads
// the row-major input straight into cm, i.e. it inverts X = M^T held column-major, and
// X^-1 = (M^-1)^T column-major is M^-1 row-major: the store is a straight copy too.
// MFMA v_mfma_f32_16x16x4_f32 with a permuted k order (step s uses k = 4q + s at lane q), so every
// operand fetch is one ds_read_b128 of 4 consecutive k.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace fiode_gjb {

typedef float f4v __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f4v mfma(float a, float b, f4v c) { return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0); }

// the value of this lane's column in lane row QK (rows of 16 lanes), for a compile-time QK: one
// v_permlane16_swap gives every row pair the value of its row with QK's bit 0, one
// v_permlane32_swap carries it to the other pair; selects only (per-lane masks, no exec branches)
template <int QK>
__device__ __forceinline__ float from_row(float v, int q) {
  const uint32_t u = __float_as_uint(v);
  const auto s16 = __builtin_amdgcn_permlane16_swap(u, u, false, false);
  const uint32_t x1 = (q & 1) ? s16[0] : s16[1];                // row q ^ 1
  const uint32_t y = ((q & 1) == (QK & 1)) ? u : x1;            // row (q & 2) | (QK & 1)
  const auto s32 = __builtin_amdgcn_permlane32_swap(y, y, false, false);
  const uint32_t y2 = (q & 2) ? s32[0] : s32[1];                // y of row q ^ 2
  return __uint_as_float(((q & 2) == (QK & 2)) ? y : y2);
}

template <int K>
__device__ __forceinline__ float newbcast(float v) {             // lane K of this lane's row
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x150 + K, 0xf, 0xf, false));
}

// In-register Gauss-Jordan of one 16 x 16 block held by one wave: lane (c = lane & 15, q = lane >> 4)
// holds x[r] = B[4q + r][c].  Pivot k: column entries of my rows B[4q + r][k] by row_newbcast:k,
// the pivot row entry B[k][c] from lane row k >> 2, the pivot B[k][k] by row_newbcast:k of that
// (every row holds the pivot row after from_row: no readlane / SGPR round trip on the chain).
template <int K>
__device__ __forceinline__ void gj16_step(float (&x)[4], int c, int q) {
  constexpr int QK = K >> 2, RK = K & 3;
  float colv[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) colv[r] = newbcast<K>(x[r]);
  const float rowv = from_row<QK>(x[RK], q);
  const float piv = newbcast<K>(rowv);
  const float p = __builtin_amdgcn_rcpf(piv);
  const float rp = rowv * p;
  const bool is_col = c == K;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const float upd = is_col ? -(colv[r] * p) : fmaf(-colv[r], rp, x[r]);
    if (r == RK) x[r] = (q == QK) ? (is_col ? p : rp) : upd;
    else x[r] = upd;
  }
}

template <int K = 0>
__device__ __forceinline__ void gj16(float (&x)[4], int c, int q) {
  if constexpr (K < 16) {
    gj16_step<K>(x, c, q);
    gj16<K + 1>(x, c, q);
  }
}

#ifndef GJB_PRIO_DEFAULT
#define GJB_PRIO_DEFAULT 0
#endif
constexpr bool GJB_PRIO = GJB_PRIO_DEFAULT != 0;

template <int NP, int NW>
struct GJB {
  static constexpr int NB = NP / 16;          // blocks per side
  static constexpr int NT = 64 * NW;
  // cm is XOR-swizzled, no padding: element (a, b) of cm[a][b] sits at cm[a][b ^ 4 (a & (NP/4 - 1))] (4-float
  // groups stay contiguous).  Against the lane groups of MI355X_MICROARCH.md's LDS table every access
  // below is conflict-free: the b128 operand reads (lane (c, q) at row 16 j + c, column 16 i + 4 q: 4-float
  // slot (4 i + q) ^ c), their b128 stores (8 contiguous lanes c: slot 4 i ^ c) and the b32 column reads
  // and stores (rows 4 q + r: the row bits flip bit 4 of the column); the padded stride 72 left the b128
  // stores and the b32 accesses 2-way (LDS bank-conflict share 0.28 in k_pinv, r05u).
  static constexpr int LDM = NP;
  static constexpr int LDP = 24;              // panel buffers' row stride (ds_read_b128 of lane (c, q) at
                                              // 24 c + 4 q: every 16-lane group of the table's grouping
                                              // covers the 64 banks; 20 was 2-way)
  struct Smem {
    float cm[NP][LDM];                        // cm[col][row] of X
    float cb[NP][LDP];                        // cb[i][k] = X[i][K0 + k] before the round's update
    float rt[NP][LDP];                        // rt[j][k] = R[k][j]
  };

  static __device__ __forceinline__ int sw(int a, int b) { return b ^ ((a & (NP / 4 - 1)) << 2); }
  static __device__ __forceinline__ float& at(Smem& sm, int a, int b) { return sm.cm[a][sw(a, b)]; }
  static __device__ __forceinline__ float at(const Smem& sm, int a, int b) { return sm.cm[a][sw(a, b)]; }
  static __device__ __forceinline__ f4v* at4(Smem& sm, int a, int b) {      // b % 4 == 0
    return reinterpret_cast<f4v*>(&sm.cm[a][sw(a, b)]);
  }
  static __device__ __forceinline__ const f4v* at4(const Smem& sm, int a, int b) {
    return reinterpret_cast<const f4v*>(&sm.cm[a][sw(a, b)]);
  }

  // the 16 x 16 block (bi, bj) of X: lane (c, q) <-> X[16 bi + 4q + r][16 bj + c]
  static __device__ __forceinline__ f4v* blk(Smem& sm, int bi, int bj, int c, int q) {
    return at4(sm, 16 * bj + c, 16 * bi + 4 * q);
  }

  // (GJB_PRIO=1 raises the pivot wave's issue priority during the elimination: measured no gain on
  // the spectral inverses and +2-3 us on the 512 block inverse, so off)
  static __device__ __forceinline__ void invert_block(Smem& sm, int b, int c, int q) {
    f4v v = *blk(sm, b, b, c, q);
    float x[4] = {v[0], v[1], v[2], v[3]};
    if constexpr (GJB_PRIO) __builtin_amdgcn_s_setprio(3);
    gj16(x, c, q);
    if constexpr (GJB_PRIO) __builtin_amdgcn_s_setprio(0);
    *blk(sm, b, b, c, q) = f4v{x[0], x[1], x[2], x[3]};
  }

  // update of block (ib, jb) in round kb (ib != kb)
  static __device__ __forceinline__ void update_block(Smem& sm, int kb, int ib, int jb, int c, int q) {
    const f4v a4 = *reinterpret_cast<const f4v*>(&sm.cb[16 * ib + c][4 * q]);   // C[i][4q + s], i = c
    f4v acc, b4;
    if (jb == kb) {
      acc = f4v{0.f, 0.f, 0.f, 0.f};
      b4 = *at4(sm, 16 * kb + c, 16 * kb + 4 * q);                                 // P[4q + s][j]
    } else {
      acc = *blk(sm, ib, jb, c, q);
      b4 = *reinterpret_cast<const f4v*>(&sm.rt[16 * jb + c][4 * q]);            // R[4q + s][j]
    }
#pragma unroll
    for (int s = 0; s < 4; ++s) acc = mfma(-a4[s], b4[s], acc);
    *blk(sm, ib, jb, c, q) = acc;
  }

  // Invert the NP x NP matrix X in sm.cm (column-major).  All NT threads.
  struct NoHook {
    __device__ void operator()() const {}
  };
  static __device__ void invert(Smem& sm) { invert(sm, NoHook{}, -1); }
  // ... calling hook() (all threads, between two workgroup barriers) after round hook_round: a caller
  // with other work for the same workgroup (e.g. issuing loads it consumes after the inversion)
  template <class Hook>
  static __device__ void invert(Smem& sm, Hook hook, int hook_round) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int c = lane & 15, q = lane >> 4;
    if (w == 0) invert_block(sm, 0, c, q);
    __syncthreads();
    for (int kb = 0; kb < NB; ++kb) {
      if (kb == hook_round) hook();
      // (c) R = P X[K, j] for j-blocks != kb (one block per wave), and the old column panel -> cb
      for (int jb = w; jb < NB; jb += NW) {
        if (jb == kb) continue;
        // A[i][k] = P[i][k] = cm[K0 + k][K0 + i] (i = c, k = 4q + s); B[k][j] = X[K0 + k][J0 + j] = cm[J0 + j][K0 + k]
        f4v pa;
#pragma unroll
        for (int s = 0; s < 4; ++s) pa[s] = at(sm, 16 * kb + 4 * q + s, 16 * kb + c);
        const f4v b4 = *at4(sm, 16 * jb + c, 16 * kb + 4 * q);
        f4v acc = f4v{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s = 0; s < 4; ++s) acc = mfma(pa[s], b4[s], acc);
        *reinterpret_cast<f4v*>(&sm.rt[16 * jb + c][4 * q]) = acc;              // rt[j][4q + r] = R[4q + r][j]
      }
      for (int t = threadIdx.x; t < NP * 4; t += NT) {
        const int i = t % NP, k4 = (t / NP) * 4;      // lanes on consecutive rows i: the b32 reads of one
                                                      // column hit 32 distinct banks (4-way before)
        *reinterpret_cast<f4v*>(&sm.cb[i][k4]) = f4v{at(sm, 16 * kb + k4, i), at(sm, 16 * kb + k4 + 1, i),
                                                     at(sm, 16 * kb + k4 + 2, i), at(sm, 16 * kb + k4 + 3, i)};
      }
      __syncthreads();
      // (e) rank-16 update; wave 0 takes the next pivot block alone and inverts it at once
      const bool ahead = kb + 1 < NB;
      if (ahead && w == 0) {
        update_block(sm, kb, kb + 1, kb + 1, c, q);
        invert_block(sm, kb + 1, c, q);
      } else {
        const int w0 = ahead ? 1 : 0, nw = ahead ? NW - 1 : NW;
        int n = 0;
        for (int ib = 0; ib < NB; ++ib)
          for (int jb = 0; jb < NB; ++jb) {
            if (ib == kb && jb == kb) continue;
            if (ahead && ib == kb + 1 && jb == kb + 1) continue;
            if (n++ % nw != w - w0) continue;
            if (ib == kb) {
              *blk(sm, kb, jb, c, q) = *reinterpret_cast<const f4v*>(&sm.rt[16 * jb + c][4 * q]);
            } else {
              update_block(sm, kb, ib, jb, c, q);
            }
          }
      }
      __syncthreads();
    }
  }

  // global row-major n x n (n <= NP, padded with I; row stride ld) -> cm, and back
  static __device__ __forceinline__ void load(Smem& sm, const float* __restrict__ src, int n, int64_t ld) {
    for (int t = threadIdx.x; t < NP * NP / 4; t += NT) {
      const int r = t / (NP / 4), c4 = (t % (NP / 4)) * 4;
      f4v v;
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int cc = c4 + u;
        v[u] = (r < n && cc < n) ? src[(int64_t)r * ld + cc] : (r == cc ? 1.0f : 0.0f);
      }
      *at4(sm, r, c4) = v;                              // row r of M = column r of X
    }
  }
  static __device__ __forceinline__ void store(const Smem& sm, float* __restrict__ dst, int n, int64_t ld) {
    for (int t = threadIdx.x; t < NP * NP / 4; t += NT) {
      const int r = t / (NP / 4), c4 = (t % (NP / 4)) * 4;
      const f4v v = *at4(sm, r, c4);
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (r < n && c4 + u < n) dst[(int64_t)r * ld + c4 + u] = v[u];
    }
  }
};

}  // namespace fiode_gjb
