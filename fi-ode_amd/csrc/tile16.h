// 16-row wave tiles of the Cayley-MLP dynamics on v_mfma_f32_16x16x4_f32, shared by the
// train_ode solve (odetrain.hip) and the tile-parallel eval-mode solve (odesolve.hip): the MLP of
// one hidden part, the partial-sum combine, the resumable QP bisection with a wave-ballot
// convergence mask, and the tagged-granule exchange of the batch-global QP exit.
#pragma once
#include "common.h"
#include "tile.h"

namespace fiode_t16 {
using namespace fiode_tile;

// ---------------------------------------------------------------------------------------------
// MFMA layout: v_mfma_f32_16x16x4_f32, "hidden on M, samples on N".  A tile is TR = 16 rows
// (samples); lane l holds sample j = l & 15 of the tile and q = l >> 4 selects the K slot.
// A operand A[i = j][k = q], B operand B[k = q][col = j]; accumulator register r holds
// D[row = 4q + r][col = j].  A layer's accumulator block hb (hidden 16hb + 4q + r) is directly
// the B operand of the next layer's k-steps (hb, r), whose k index 4q' + r ... is hidden
// 16hb + 4q + r, so the A operand of that k-step is Q[out][16hb + 4q + r] (r = 0..3): one
// ds_read_b128 of 4 consecutive weights.  32-cycle issue, 40-cycle dependent latency: every
// accumulation runs >= 2 independent accumulators except the short layer-3 chain.
constexpr int TR = 16;

typedef float f32x4v __attribute__((ext_vector_type(4)));
__device__ __forceinline__ f32x4v mfma16(float a, float b, f32x4v c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f32x4v z4() { return f32x4v{0.f, 0.f, 0.f, 0.f}; }

// relu(dropout(z)) on a 16x16 block: hidden 16hb + 4q + r, keep bit from w = kw[hidden >> 5]
__device__ __forceinline__ void dropout_relu16(f32x4v& z, uint32_t w, int hb, int q, float scale) {
  const int sh = 16 * (hb & 1) + 4 * q;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const bool keep = (w >> (sh + r)) & 1u;
    z[r] = keep ? fmaxf(z[r] * scale, 0.f) : 0.f;
  }
}
__device__ __forceinline__ float sel4(const float (&v)[C], int s, int q) {   // v[4s + q], 0 past C
  const int k = 4 * s + q;
  float x = 0.f;
#pragma unroll
  for (int t = 0; t < 4; ++t)
    if (4 * s + t < C) x = (q == t) ? v[4 * s + t] : x;
  return k < C ? x : 0.f;
}

typedef __attribute__((address_space(1))) unsigned long long gu64_t;

__device__ __forceinline__ void publish_mask(unsigned long long* slot, unsigned epoch, uint32_t mask) {
  __hip_atomic_store((gu64_t*)(slot), ((unsigned long long)epoch << 32) | mask, __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}

// one wave: AND of the masks of all tiles for this epoch (lane i reads tiles i, i+64, ...).
// Bounded: after ~0.5 s without every tag (a tile not resident) it records status 4, sets the
// workgroup's sticky `dead` flag (LDS) -- later exchanges of this workgroup then stop waiting at
// once -- and returns the partial AND; the caller poisons its outputs (see k_ot_fwd).
__device__ __forceinline__ uint32_t gather_masks(unsigned long long* slots, int ntiles, unsigned epoch,
                                                 int32_t* status, int lane, int& dead) {
  uint32_t acc = 0xFFFFFFFFu;
  for (int base = 0; base < ntiles; base += 64) {
    const int t = base + lane;
    unsigned spins = 0;
    for (;;) {
      bool ok = true;
      unsigned long long x = 0;
      if (t < ntiles) {
        x = __hip_atomic_load((gu64_t*)(slots + t), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        ok = (unsigned)(x >> 32) == epoch;
      }
      if (__all(ok)) {
        if (t < ntiles) acc &= (uint32_t)x;
        break;
      }
      if (dead || ++spins > (1u << 22)) {   // ~0.5 s: a non-resident tile; record and give up
        if (lane == 0) {
          atomicMax(status, 4);
          dead = 1;
        }
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
  }
  return wave_and(acc);
}

// The bisection of FastBarrierProjectionNoUpper (qp_bisect, common.h) split so it can stop and
// resume: iterations [from, to] from the bracket state (lo, hi), recording mu per iteration.  The
// returned mask is the WAVE's: bit it set iff every valid lane converged at iteration it (ballot).
__device__ __forceinline__ void qp_bracket(const float (&lower)[C], const float (&nom)[C], float& lo, float& hi) {
  hi = nom[0] - lower[0];
  lo = nom[0];
#pragma unroll
  for (int j = 1; j < C; ++j) {
    hi = fmaxf(hi, nom[j] - lower[j]);
    lo = fminf(lo, nom[j]);
  }
}
__device__ __forceinline__ float qp_eps(const float (&lower)[C], const float (&nom)[C], float mu) {
  float eps = 0.f;
#pragma unroll
  for (int j = 0; j < C; ++j) eps = eps + fmaxf(nom[j] - mu, lower[j]);
  return eps;
}

// The bisection two iterations per round: the 4 lanes of a row (q = 0..3, lanes j + 16 q) evaluate
// the midpoint m0 (q = 0, 3) and both possible next midpoints -- the left child (q = 1, taken when
// eps(m0) < 0) and the right child (q = 2, eps(m0) > 0) -- at once, and exchange the three eps
// values by shuffles.  Every midpoint and eps is the same float32 expression the sequential loop
// evaluates (m1 = (hi' - lo') / 2 + lo' with the updated bracket), so mu, the convergence bits and
// the exit are bit-identical to qp_bisect_range; the dependent chain per iteration is halved.
__device__ __forceinline__ uint32_t qp_bisect_range2(const float (&lower)[C], const float (&nom)[C], int from, int to,
                                                     float tol, float& lo, float& hi, float* mu_rec, bool rec,
                                                     bool valid, int q, int j) {
  uint32_t conv = 0;
  int it = from;
  for (; it + 1 <= to; it += 2) {
    const float m0 = (hi - lo) / 2.0f + lo;
    const float mL = (m0 - lo) / 2.0f + lo;
    const float mR = (hi - m0) / 2.0f + m0;
    const float e = qp_eps(lower, nom, q == 1 ? mL : (q == 2 ? mR : m0));
    const float e0 = __shfl(e, j, 64);
    const float eL = __shfl(e, j + 16, 64);
    const float eR = __shfl(e, j + 32, 64);
    if (rec) mu_rec[it] = m0;
    unsigned long long open = __ballot(valid && !(fabsf(e0) < tol));
    conv |= (open == 0ull ? 1u : 0u) << it;
    const float lo1 = e0 > 0.f ? m0 : lo, hi1 = e0 < 0.f ? m0 : hi;
    const float m1 = e0 < 0.f ? mL : (e0 > 0.f ? mR : m0);
    const float e1 = e0 < 0.f ? eL : (e0 > 0.f ? eR : e0);
    if (rec) mu_rec[it + 1] = m1;
    open = __ballot(valid && !(fabsf(e1) < tol));
    conv |= (open == 0ull ? 1u : 0u) << (it + 1);
    lo = e1 > 0.f ? m1 : lo1;
    hi = e1 < 0.f ? m1 : hi1;
  }
  if (it <= to) {
    const float mu = (hi - lo) / 2.0f + lo;
    const float eps = qp_eps(lower, nom, mu);
    if (rec) mu_rec[it] = mu;
    const unsigned long long open = __ballot(valid && !(fabsf(eps) < tol));
    conv |= (open == 0ull ? 1u : 0u) << it;
    lo = eps > 0.f ? mu : lo;
    hi = eps < 0.f ? mu : hi;
  }
  return conv;
}

__device__ __forceinline__ uint32_t qp_bisect_range(const float (&lower)[C], const float (&nom)[C], int from, int to,
                                                    float tol, float& lo, float& hi, float* mu_rec, bool rec,
                                                    bool valid) {
  uint32_t conv = 0;
  for (int it = from; it <= to; ++it) {
    const float mu = (hi - lo) / 2.0f + lo;
    float eps = 0.f;
#pragma unroll
    for (int j = 0; j < C; ++j) eps = eps + fmaxf(nom[j] - mu, lower[j]);
    if (rec) mu_rec[it] = mu;
    const unsigned long long open = __ballot(valid && !(fabsf(eps) < tol));
    conv |= (open == 0ull ? 1u : 0u) << it;
    lo = eps > 0.f ? mu : lo;
    hi = eps < 0.f ? mu : hi;
  }
  return conv;
}


// The MLP of one tile for hidden part p (of 4): layer 1 in full (24 MFMA), layer-2 output blocks
// 2p, 2p+1 (64 MFMA), their layer-3 partial (8 MFMA; bias on part 0) -> zpart_lane[4] (LDS).
// Q1s: [M][C] LDS copy; Q2s / Q3s: padded LDS images (Q3s rows >= C zero or absent: masked).
// a1row / a2row (nullable): the row's saved post-activations (part p stores its blocks).
__device__ __forceinline__ void mlp16_part(const float* Q1s, const float* Q2s, const float* Q3s, const float* b2,
                                           const float* b3, const f32x4v (&uacc)[8], const float (&h)[C],
                                           const uint32_t (&kw1)[4], uint32_t kw2p, float scale, int p, int q, int j,
                                           float* a1row, float* a2row, float* zpart_lane) {
  f32x4v z1[8];
#pragma unroll
  for (int hb = 0; hb < 8; ++hb) z1[hb] = uacc[hb];
#pragma unroll
  for (int s = 0; s < 3; ++s) {
    const float bs = sel4(h, s, q);
    const bool kin = 4 * s + q < C;
#pragma unroll
    for (int hb = 0; hb < 8; ++hb) {
      const float av = kin ? Q1s[(16 * hb + j) * C + 4 * s + q] : 0.f;
      z1[hb] = mfma16(av, bs, z1[hb]);
    }
  }
#pragma unroll
  for (int hb = 0; hb < 8; ++hb) dropout_relu16(z1[hb], kw1[hb >> 1], hb, q, scale);
  if (a1row) {
#pragma unroll
    for (int hb = 0; hb < 8; ++hb)
      if ((hb >> 1) == p)
        *reinterpret_cast<f32x4*>(a1row + 16 * hb + 4 * q) = f32x4{z1[hb][0], z1[hb][1], z1[hb][2], z1[hb][3]};
  }
  f32x4v z2[2];
#pragma unroll
  for (int o = 0; o < 2; ++o) {
    const f32x4 bv = *reinterpret_cast<const f32x4*>(b2 + 16 * (2 * p + o) + 4 * q);
    z2[o] = f32x4v{bv[0], bv[1], bv[2], bv[3]};
  }
#pragma unroll
  for (int hb = 0; hb < 8; ++hb) {
#pragma unroll
    for (int o = 0; o < 2; ++o) {
      const f32x4 qv = *reinterpret_cast<const f32x4*>(Q2s + (16 * (2 * p + o) + j) * LDQ + 16 * hb + 4 * q);
#pragma unroll
      for (int t = 0; t < 4; ++t) z2[o] = mfma16(qv[t], z1[hb][t], z2[o]);
    }
  }
#pragma unroll
  for (int o = 0; o < 2; ++o) {
    dropout_relu16(z2[o], kw2p, 2 * p + o, q, scale);
    if (a2row)
      *reinterpret_cast<f32x4*>(a2row + 16 * (2 * p + o) + 4 * q) = f32x4{z2[o][0], z2[o][1], z2[o][2], z2[o][3]};
  }
  f32x4v z3 = z4();
  if (p == 0) {
#pragma unroll
    for (int t = 0; t < 4; ++t) z3[t] = 4 * q + t < C ? b3[4 * q + t] : 0.f;
  }
#pragma unroll
  for (int o = 0; o < 2; ++o) {
    const f32x4 qv = j < C ? *reinterpret_cast<const f32x4*>(Q3s + j * LDQ + 16 * (2 * p + o) + 4 * q)
                           : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int t = 0; t < 4; ++t) z3 = mfma16(qv[t], z2[o][t], z3);
  }
  *reinterpret_cast<f32x4*>(zpart_lane) = f32x4{z3[0], z3[1], z3[2], z3[3]};
}

// After the barrier: this lane's sample j sums its 10 outputs over the 4 parts in a fixed order
// (output i sits in lane 16 (i >> 2) + j, register i & 3).  zpart: [4 parts][64 lanes][4].
__device__ __forceinline__ void ft16_sum(const float (*zpart)[64][4], int j, float (&ft)[C]) {
#pragma unroll
  for (int i = 0; i < C; ++i) {
    const int ln = 16 * (i >> 2) + j, rg = i & 3;
    ft[i] = ((zpart[0][ln][rg] + zpart[1][ln][rg]) + zpart[2][ln][rg]) + zpart[3][ln][rg];
  }
}

// The batch-global QP exit of one eval with speculation: bisect to kprev + 3, publish the wave's
// mask in granule slot slots[blockIdx] (epoch), gather all tiles; only if no iteration <= kspec
// converged everywhere, resume to max_iter - 1 and exchange again in slots[ntiles + ..].  Called
// by all 4 waves (identical rows); wave 0 exchanges; shK is an LDS int.  Returns K (uniform).
__device__ __forceinline__ int qp16_exit(const float (&lower)[C], const float (&nominal)[C], float tol, int max_iter,
                                         int kprev, bool valid, int p, int q, int lane, float* mu_rec_row,
                                         unsigned long long* slots, unsigned epoch, int32_t* status, int& shK,
                                         int& dead, int drop_block = -1) {
  const int last = max_iter - 1;
  const int kspec = min(last, kprev + 3);
  float lo, hi;
  qp_bracket(lower, nominal, lo, hi);
  const int j = lane & 15;
  uint32_t conv = qp_bisect_range2(lower, nominal, 0, kspec, tol, lo, hi, mu_rec_row, q == 0, valid, q, j);
  const int ntiles = gridDim.x;
  if (p == 0) {
    // drop_block (test hook, FIODE_DEBUG_DROP_PUBLISH): that workgroup never publishes epoch 1,
    // as if it were not resident -- exercises the timeout path
    if (lane == 0 && !(epoch == 1u && (int)blockIdx.x == drop_block)) publish_mask(slots + blockIdx.x, epoch, conv);
    const uint32_t all = gather_masks(slots, ntiles, epoch, status, lane, dead);
    const uint32_t lowm = kspec >= 31 ? 0xFFFFFFFFu : ((1u << (kspec + 1)) - 1u);
    const uint32_t bits = all & lowm;
    if (lane == 0) shK = bits ? (__ffs((int)bits) - 1) : (kspec >= last ? last : -1);
  }
  __syncthreads();
  if (shK < 0) {                        // block-uniform: every tile saw the same masks
    conv |= qp_bisect_range2(lower, nominal, kspec + 1, last, tol, lo, hi, mu_rec_row, q == 0, valid, q, j);
    if (p == 0) {
      if (lane == 0) publish_mask(slots + ntiles + blockIdx.x, epoch, conv);
      const uint32_t all = gather_masks(slots + ntiles, ntiles, epoch, status, lane, dead);
      if (lane == 0) shK = qp_exit_iter(all, max_iter);
    }
    __syncthreads();
  }
  return shK;
}

}  // namespace fiode_t16
