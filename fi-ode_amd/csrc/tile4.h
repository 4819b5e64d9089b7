// 4-row tiles of the Cayley-MLP dynamics on v_mfma_f32_4x4x1_16b_f32, for the train_ode RK4
// forward (k_ot_fwd, odetrain.hip): a persistent solve is a latency chain per eval, and its MLP
// time is the MFMA work ONE wave issues.  With 16-row tiles (tile16.h) every wave issues the
// 16x16x4 products of 16 samples; with 4-row tiles it issues 4x4x1 products of 4 samples -- a
// quarter of the MFMA cycles per eval (measured 8.4 cycles per 4x4x1 issue with >= 4 independent
// accumulators, 12.8 on one dependent chain: tools/probes/mfma4_probe.hip), on 4x as many CUs.
//
// MFMA layout (tools/probes/mfma4_probe.hip): 16 blocks b = lane >> 2; in block b, A[i][0] comes
// from lane 4b + i, B[0][j] from lane 4b + j, and D[i][j] lands in register i of lane 4b + j.
// Here j = lane & 3 is always the SAMPLE (row of the tile), so the accumulator of a lane holds 4
// outputs of its own sample.  Wave p owns hidden units 32p .. 32p + 31 of layers 1-2:
//   layer 1: blocks b < 8: units 32p + 4b + i over inputs 0..4, blocks b >= 8 the same units over
//            inputs 5..9; the two halves meet by one v_permlane32_swap (lane l <-> l ^ 32);
//   layer 2: the same unit split, K = 128 in two halves (a1 of units 0..63 / 64..127, from LDS),
//            4 independent accumulators per half (k mod 4), summed in a fixed order;
//   layer 3: outputs c = 4 (b & 3) + i (c < 10), K = the wave's 32 units in quarters b >> 2
//            (8 steps), the quarters summed by v_permlane16_swap / v_permlane32_swap.
// The 4 waves' layer-3 partials meet in LDS and every lane sums its sample's 10 outputs over the
// parts in the same order, so the row state stays replicated (16 lanes per sample per wave).
#pragma once
#include "common.h"
#include "tile.h"

namespace fiode_t4 {
using namespace fiode_tile;

constexpr int TR4 = 4;

typedef float f32x4v __attribute__((ext_vector_type(4)));
__device__ __forceinline__ f32x4v mfma4(float a, float b, f32x4v c) {
  return __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f32x4v zero4() { return f32x4v{0.f, 0.f, 0.f, 0.f}; }

// the other half-wave's value (lane l ^ 32) / the other 16-lane row pair's (lane l ^ 16)
__device__ __forceinline__ float swap32(float v) {
  const uint32_t u = __float_as_uint(v);
  const auto s = __builtin_amdgcn_permlane32_swap(u, u, false, false);
  return __uint_as_float((threadIdx.x & 32) ? s[0] : s[1]);
}
__device__ __forceinline__ float swap16(float v) {
  const uint32_t u = __float_as_uint(v);
  const auto s = __builtin_amdgcn_permlane16_swap(u, u, false, false);
  return __uint_as_float((threadIdx.x & 16) ? s[0] : s[1]);
}

// Weight operands of wave p, in registers for the whole solve.
//   q1[s]  = Q1[32p + 4 (b & 7) + i][s + 5 (b >> 3)]           (layer 1, s = 0..4)
//   q2[s]  = Q2[32p + 4 (b & 7) + i][s + 64 (b >> 3)]          (layer 2, s = 0..63)
//   q3[s]  = Q3[4 (b & 3) + i][32p + 8 (b >> 2) + s]  (0 for rows >= C; layer 3, s = 0..7)
//   b2     = b2[32p + 4 (b & 7) + r] in accumulator order, b3 = b3[4 (b & 3) + r] on part 0
// with i = lane & 3 (the A-operand row of the lane), b = lane >> 2.
struct T4W {
  float q1[5];
  float q2[64];
  float q3[8];
  f32x4 b2;
  f32x4 b3;
};

__device__ __forceinline__ void load_t4w(const float* Q1, const float* Q2, const float* Q3, const float* b2,
                                         const float* b3, int p, int lane, T4W& w) {
  const int b = lane >> 2, i = lane & 3;
  const int u = 32 * p + 4 * (b & 7) + i;       // the unit this lane feeds as an A row
#pragma unroll
  for (int s = 0; s < 5; ++s) w.q1[s] = Q1[u * C + s + 5 * (b >> 3)];
#pragma unroll
  for (int s = 0; s < 64; s += 4) {
    const f32x4 v = *reinterpret_cast<const f32x4*>(Q2 + (size_t)u * M + s + 64 * (b >> 3));
    w.q2[s] = v[0]; w.q2[s + 1] = v[1]; w.q2[s + 2] = v[2]; w.q2[s + 3] = v[3];
  }
  const int c = 4 * (b & 3) + i;
#pragma unroll
  for (int s = 0; s < 8; ++s) w.q3[s] = c < C ? Q3[c * M + 32 * p + 8 * (b >> 2) + s] : 0.f;
  const int r0 = 32 * p + 4 * (b & 7);
  w.b2 = f32x4{b2[r0], b2[r0 + 1], b2[r0 + 2], b2[r0 + 3]};
#pragma unroll
  for (int r = 0; r < 4; ++r) w.b3[r] = (p == 0 && 4 * (b & 3) + r < C) ? b3[4 * (b & 3) + r] : 0.f;
}

// LDS of one tile's MLP: post-activations of the 4 samples (B operands), layer-3 partials.
struct Mlp4Shared {
  float a1s[TR4][M + 4];      // [sample][unit]
  float a2s[TR4][M + 4];
  float zpart[4][16][4];      // [part][lane 4 blk + j][reg]: layer-3 partial of outputs 4 blk + reg
};

// relu(dropout(z)) of units 32p + 4 blk + r (r = 0..3); keep bits from the part's word w
__device__ __forceinline__ void dropout_relu4(f32x4v& z, uint32_t w, int blk, float scale) {
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const bool keep = (w >> (4 * blk + r)) & 1u;
    z[r] = keep ? fmaxf(z[r] * scale, 0.f) : 0.f;
  }
}

// acc[t] += sum_s q[4s + t] * src[4s + t] over one K half (64 values of the lane's sample in LDS):
// the 16 B operands are read KD k-steps ahead of their MFMAs -- one step of 4 MFMAs (~34 cycles)
// does not cover a ds_read_b128's latency, and the compiler's own schedule reads one step ahead
// (the scheduling barriers keep it from sinking the reads back next to their MFMAs)
__device__ __forceinline__ void k128_half(const float* src, const float (&q)[64], f32x4v (&acc)[4]) {
  constexpr int KD = 8;
  f32x4 bv[16];
#pragma unroll
  for (int s = 0; s < KD; ++s) bv[s] = *reinterpret_cast<const f32x4*>(src + 4 * s);
#pragma unroll
  for (int s = 0; s < 16; ++s) {
    __builtin_amdgcn_sched_barrier(0);
    if (s + KD < 16) bv[s + KD] = *reinterpret_cast<const f32x4*>(src + 4 * (s + KD));
#pragma unroll
    for (int t = 0; t < 4; ++t) acc[t] = mfma4(q[4 * s + t], bv[s][t], acc[t]);
  }
  __builtin_amdgcn_sched_barrier(0);
}

// The MLP of one 4-row tile for hidden part p: uacc = u[sample][32p + 4 (b & 7) + r] (this lane's
// sample, accumulator order); h: the lane's sample input; kw1p / kw2p: the part's keep words of the
// two dropout layers.  a1row / a2row (nullable): the sample's saved rows (lanes b < 8 store their
// 4 units).  Leaves the part's layer-3 partial in sh.zpart[p]; the caller's barrier publishes it.
// Contains one workgroup barrier (a1 of all parts in LDS before layer 2).
__device__ __forceinline__ void mlp4_part(const T4W& w, const f32x4& uacc, const float (&h)[C], uint32_t kw1p,
                                          uint32_t kw2p, float scale, int p, int lane, float* a1row, float* a2row,
                                          Mlp4Shared& sh) {
  const int b = lane >> 2, j = lane & 3, hi = b >> 3, blk = b & 7;
  // layer 1: units 32p + 4 blk + r, inputs s + 5 hi
  f32x4v z = zero4();
#pragma unroll
  for (int s = 0; s < 5; ++s) z = mfma4(w.q1[s], hi ? h[s + 5] : h[s], z);
#pragma unroll
  for (int r = 0; r < 4; ++r) z[r] = uacc[r] + (z[r] + swap32(z[r]));     // (inputs 0..4 + 5..9) + u
  dropout_relu4(z, kw1p, blk, scale);
  if (b < 8) {
    const f32x4 v = f32x4{z[0], z[1], z[2], z[3]};
    *reinterpret_cast<f32x4*>(&sh.a1s[j][32 * p + 4 * blk]) = v;
    if (a1row) *reinterpret_cast<f32x4*>(a1row + 32 * p + 4 * blk) = v;
  }
  __syncthreads();
  // layer 2: units 32p + 4 blk + r, K half hi (a1 of units 64 hi + s), 4 accumulators (s mod 4)
  f32x4v acc[4] = {zero4(), zero4(), zero4(), zero4()};
  k128_half(&sh.a1s[j][64 * hi], w.q2, acc);
  f32x4v z2;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const float part = (acc[0][r] + acc[1][r]) + (acc[2][r] + acc[3][r]);
    const float other = swap32(part);                 // every lane (a cross-lane op in uniform flow)
    const float lo = hi ? other : part, up = hi ? part : other;
    z2[r] = w.b2[r] + (lo + up);
  }
  dropout_relu4(z2, kw2p, blk, scale);
  if (b < 8) {
    const f32x4 v = f32x4{z2[0], z2[1], z2[2], z2[3]};
    *reinterpret_cast<f32x4*>(&sh.a2s[j][32 * p + 4 * blk]) = v;      // read back by this wave only
    if (a2row) *reinterpret_cast<f32x4*>(a2row + 32 * p + 4 * blk) = v;
  }
  // layer 3 partial: outputs 4 (b & 3) + r, units 32p + 8 (b >> 2) + s
  f32x4v z3a = zero4(), z3b = zero4();
  const float* a2 = &sh.a2s[j][32 * p + 8 * (b >> 2)];
  const f32x4 v0 = *reinterpret_cast<const f32x4*>(a2), v1 = *reinterpret_cast<const f32x4*>(a2 + 4);
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    z3a = mfma4(w.q3[t], v0[t], z3a);
    z3b = mfma4(w.q3[4 + t], v1[t], z3b);
  }
  f32x4v z3;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const float x = z3a[r] + z3b[r];                  // this quarter (b >> 2)
    const float y = x + swap16(x);                    // quarters {0,1} / {2,3}
    z3[r] = w.b3[r] + (y + swap32(y));                // all four (the same order in every lane)
  }
  if (b < 4) *reinterpret_cast<f32x4*>(&sh.zpart[p][lane][0]) = f32x4{z3[0], z3[1], z3[2], z3[3]};
}

// After the barrier: the lane's sample j sums its 10 outputs over the 4 parts in a fixed order.
__device__ __forceinline__ void ft4_sum(const Mlp4Shared& sh, int j, float (&ft)[C]) {
#pragma unroll
  for (int g = 0; g < 3; ++g) {
    f32x4 v[4];
#pragma unroll
    for (int pp = 0; pp < 4; ++pp) v[pp] = *reinterpret_cast<const f32x4*>(&sh.zpart[pp][4 * g + j][0]);
#pragma unroll
    for (int r = 0; r < 4; ++r)
      if (4 * g + r < C) ft[4 * g + r] = ((v[0][r] + v[1][r]) + v[2][r]) + v[3][r];
  }
}

}  // namespace fiode_t4
