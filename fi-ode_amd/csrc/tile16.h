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

// The batch-global QP exit is first exchanged for iterations <= previous exit + this margin; if
// no such iteration converged everywhere the bisection resumes to max_iter - 1 and exchanges
// again (same exit either way: the lowest iteration at which every row converged).
#ifndef FIODE_KSPEC_MARGIN
#define FIODE_KSPEC_MARGIN 1
#endif

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

// AND over lanes 0..n-1 of a wave (other lanes ignored; n wave-uniform): scalar readlanes while n
// is small -- the shuffle butterfly is six dependent LDS-crossbar round trips (~0.3 us).
__device__ __forceinline__ uint32_t lanes_and(uint32_t v, int n) {
  if (n <= 16) {
    uint32_t acc = 0xFFFFFFFFu;
    for (int i = 0; i < n; ++i) acc &= (uint32_t)__builtin_amdgcn_readlane((int)v, i);
    return acc;
  }
  return wave_and(v);
}

// The value of this lane's column j (= lane & 15) in each of the 4 lane rows q' (lanes j + 16 q'),
// with gfx950's cross-row swaps (VALU, no LDS round trip): v_permlane16_swap exchanges rows
// 0 <-> 1 and 2 <-> 3, v_permlane32_swap rows {0, 1} <-> {2, 3}.
__device__ __forceinline__ void rows4(float v, int q, float (&r)[4]) {
  const uint32_t u = __float_as_uint(v);
  const auto s16 = __builtin_amdgcn_permlane16_swap(u, u, false, false);
  const uint32_t x1 = (q & 1) ? s16[0] : s16[1];              // row q ^ 1
  const auto s32 = __builtin_amdgcn_permlane32_swap(u, u, false, false);
  const uint32_t x2 = (q & 2) ? s32[0] : s32[1];              // row q ^ 2
  const auto s32b = __builtin_amdgcn_permlane32_swap(x1, x1, false, false);
  const uint32_t x3 = (q & 2) ? s32b[0] : s32b[1];            // row q ^ 3
#pragma unroll
  for (int t = 0; t < 4; ++t)
    r[t] = __uint_as_float(t == q ? u : (t == (q ^ 1) ? x1 : (t == (q ^ 2) ? x2 : x3)));
}

// OR over the 64 lanes, returned wave-uniform: DPP rotations within each 16-lane row, then the
// four rows' values by scalar readlanes.
__device__ __forceinline__ uint32_t wave_or16(uint32_t x) {
  x |= (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x121, 0xf, 0xf, false);   // row_ror:1
  x |= (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x122, 0xf, 0xf, false);   // row_ror:2
  x |= (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x124, 0xf, 0xf, false);   // row_ror:4
  x |= (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x128, 0xf, 0xf, false);   // row_ror:8
  return (uint32_t)(__builtin_amdgcn_readlane((int)x, 0) | __builtin_amdgcn_readlane((int)x, 16) |
                    __builtin_amdgcn_readlane((int)x, 32) | __builtin_amdgcn_readlane((int)x, 48));
}

typedef __attribute__((address_space(1))) unsigned long long gu64_t;

__device__ __forceinline__ void publish_mask(unsigned long long* slot, unsigned epoch, uint32_t mask) {
  __hip_atomic_store((gu64_t*)(slot), ((unsigned long long)epoch << 32) | mask, __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}

// one wave: AND of the masks of all tiles for this epoch (lane i reads tiles i, i+64, ...); tile t's
// granule at slots[t * stride] (stride 16: one 128-byte line per tile, no two publishers on a line).
// Bounded: after ~0.5 s without every tag (a tile not resident) it records status 4, sets the
// workgroup's sticky `dead` flag (LDS) -- later exchanges of this workgroup then stop waiting at
// once -- and returns the partial AND; the caller poisons its outputs (see k_ot_fwd).
__device__ __forceinline__ uint32_t gather_masks(unsigned long long* slots, int ntiles, unsigned epoch,
                                                 int32_t* status, int lane, int& dead, int stride = 1) {
  uint32_t acc = 0xFFFFFFFFu;
  for (int base = 0; base < ntiles; base += 64) {
    const int t = base + lane;
    unsigned spins = 0;
    for (;;) {
      bool ok = true;
      unsigned long long x = 0;
      if (t < ntiles) {
        x = __hip_atomic_load((gu64_t*)(slots + (size_t)t * stride), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
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
  return lanes_and(acc, ntiles < 64 ? ntiles : 64);
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
// eps(mu) = sum_j max(nom_j - mu, lower_j) in the reference's order.  Only its comparisons with 0
// and tol are used, so the sum starts at term 0 (0 + t0 differs from t0 only in the sign of a zero)
// and max is vmax_f32 (common.h).
typedef float f2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ float qp_eps(const float (&lower)[C], const float (&nom)[C], float mu) {
  const f2v m2 = f2v{mu, mu};
  f2v d[C / 2];
#pragma unroll
  for (int j = 0; j < C / 2; ++j) d[j] = f2v{nom[2 * j], nom[2 * j + 1]} - m2;      // v_pk_add_f32
  float eps = vmax_f32(d[0][0], lower[0]);
#pragma unroll
  for (int j = 1; j < C; ++j) eps = eps + vmax_f32(d[j >> 1][j & 1], lower[j]);
  return eps;
}

// The sequential bisection over iterations [from, to] (barrier_projection.py:232-255), one eps per
// iteration.  Measured on gfx950 (tools/probes/bisect_probe.hip, cycles per 20 iterations of a
// 4-wave workgroup): this 4.2k, the 2-per-round permlane variant 5.4k, the 4-level workgroup tree
// 6.0k -- at one wave per SIMD the exchange and path selection of a speculative variant cost more
// than the eps evaluations they save.  Per iteration the dependent chain is mu, 5 packed
// subtracts, 10 max, the 9 ordered adds and the bracket update; everything else is kept off it:
// mu = fma(hi - lo, 0.5, lo) is (hi - lo) / 2 + lo exactly (the halving is exact for any width
// above 2^-125), the per-lane open bits are OR-reduced over the wave once per call (a ballot per
// iteration measured slower: its scalar test waits on the compare), and mu_rec (nullable) is
// written by every lane (rec: the caller's per-lane slot) with no exec-mask branch.
__device__ __forceinline__ uint32_t qp_open_seq(const float (&lower)[C], const float (&nom)[C], int from, int to,
                                                float tol, float& lo, float& hi, float* mu_rec, bool rec,
                                                bool valid) {
  uint32_t open = 0;
  for (int it = from; it <= to; ++it) {
    const float mu = __fmaf_rn(hi - lo, 0.5f, lo);
    const float eps = qp_eps(lower, nom, mu);
    if (rec) mu_rec[it] = mu;
    open |= ((valid && !(fabsf(eps) < tol)) ? 1u : 0u) << it;
    lo = eps > 0.f ? mu : lo;
    hi = eps < 0.f ? mu : hi;
  }
  return open;
}
__device__ __forceinline__ uint32_t qp_span(int from, int to) {
  const int n = to - from + 1;
  return (n >= 32 ? 0xFFFFFFFFu : ((1u << n) - 1u)) << from;
}
__device__ __forceinline__ uint32_t qp_bisect_seq(const float (&lower)[C], const float (&nom)[C], int from, int to,
                                                  float tol, float& lo, float& hi, float* mu_rec, bool rec,
                                                  bool valid) {
  if (from > to) return 0u;
  const uint32_t open = qp_open_seq(lower, nom, from, to, tol, lo, hi, mu_rec, rec, valid);
  return ~wave_or16(open) & qp_span(from, to);
}

// The same iterations, LV at a time, on the lanes that replicate a row.  A wave holding R rows has
// 64 / R copies of each (lane = m R + j: row j, copy m); copy m < 2^LV - 1 evaluates node m of the
// depth-LV tree of bisection states the next LV iterations can reach (node n's children 2n + 1 /
// 2n + 2 follow eps > 0 (lo = mu) / eps < 0 (hi = mu)), so one eps per lane replaces LV dependent
// ones.  Every node's mu is computed from the round's (lo, hi) by the sequential recurrence along
// its path, so the mus, the convergence bits and the final bracket are bit-identical to
// qp_bisect_seq's.  One ballot of the signs gives each node its place on the path (all ancestors'
// signs lead to it); the path nodes record their mu (rec: the row's shared record) and open bit, and
// the last one publishes the next bracket through LDS (bc, same wave: LDS order suffices).  A round
// in which any node's eps is 0 or NaN (the bracket would not move there) runs sequentially.
template <int R>
struct QpTree {
  static constexpr int REP = 64 / R;
  static constexpr int LV = REP >= 16 ? 4 : (REP >= 4 ? 2 : 1);
  static constexpr int NN = (1 << LV) - 1;
};

template <int R>
__device__ __forceinline__ uint32_t qp_bisect_tree(const float (&lower)[C], const float (&nom)[C], int from, int to,
                                                   float tol, float& lo, float& hi, float* rec, float* bc,
                                                   bool valid) {
  if (from > to) return 0u;
  constexpr int LV = QpTree<R>::LV;
  uint32_t open = 0;
  int it = from;
  if constexpr (LV > 1) {
    const int lane = threadIdx.x & 63;
    const int j = lane % R, m = lane / R;
    const bool owner = m < QpTree<R>::NN;
    const int n1 = (owner ? m : 0) + 1;       // heap index + 1 = binary 1 d_0 .. d_{L-1} (d = 1: eps < 0)
    const int L = 31 - __builtin_clz(n1);     // the node's level
    bool use[LV - 1], right[LV - 1];
    int pos[LV - 1];
#pragma unroll
    for (int l = 0; l < LV - 1; ++l) {
      use[l] = l < L;
      right[l] = use[l] && ((n1 >> (L - 1 - l)) & 1);
      pos[l] = (use[l] ? (n1 >> (L - l)) - 1 : 0) * R + j;       // lane of the level-l ancestor
    }
    for (; it + LV - 1 <= to; it += LV) {
      float lo_ = lo, hi_ = hi;
#pragma unroll
      for (int l = 0; l < LV - 1; ++l) {
        const float mu_l = __fmaf_rn(hi_ - lo_, 0.5f, lo_);
        lo_ = (use[l] && !right[l]) ? mu_l : lo_;
        hi_ = right[l] ? mu_l : hi_;
      }
      const float mu = __fmaf_rn(hi_ - lo_, 0.5f, lo_);
      const float eps = qp_eps(lower, nom, mu);
      if (__any(!(eps > 0.f) && !(eps < 0.f))) {       // (uniform) a node the bracket would not leave
        open |= qp_open_seq(lower, nom, it, it + LV - 1, tol, lo, hi, rec, true, valid);
        continue;
      }
      const unsigned long long P = __ballot(eps > 0.f);
      uint32_t bad = 0;
#pragma unroll
      for (int l = 0; l < LV - 1; ++l)
        bad |= use[l] ? (((uint32_t)(P >> pos[l]) & 1u) ^ (right[l] ? 0u : 1u)) : 0u;
      if (owner && bad == 0u) {
        rec[it + L] = mu;
        open |= ((valid && !(fabsf(eps) < tol)) ? 1u : 0u) << (it + L);
        if (L == LV - 1) {
          bc[0] = eps > 0.f ? mu : lo_;
          bc[1] = eps > 0.f ? hi_ : mu;
        }
      }
      lo = bc[0];
      hi = bc[1];
    }
  }
  if (it <= to) open |= qp_open_seq(lower, nom, it, to, tol, lo, hi, rec, true, valid);
  return ~wave_or16(open) & qp_span(from, to);
}

// The weights one wave (hidden part p) reads in the MLP of a tile, held in registers for the whole
// persistent kernel (108 VGPRs; the kernels run one wave per SIMD, 512 registers): no LDS reads on
// the per-eval critical path.  q1: layer-1 A operands Q1[16 hb + j][4 s + q] (0 past C); q2: the
// layer-2 A operands Q2[16 (2p + o) + j][16 hb + 4q .. + 3]; q3: layer 3's Q3[j][16 (2p + o) + 4q ..]
// (0 for j >= C); b2 of the part's output blocks; b3 on part 0.
struct T16W {
  float q1[8][3];
  f32x4 q2[2][8];
  f32x4 q3[2];
  f32x4 b2[2];
  f32x4 b3;
};

// Q1 [M][C]; Q2 / Q3 with row strides ld2 / ld3 (global: M; the padded LDS images: LDQ).
__device__ __forceinline__ void load_t16w(const float* Q1, const float* Q2, int ld2, const float* Q3, int ld3,
                                          const float* b2, const float* b3, int p, int q, int j, T16W& w) {
#pragma unroll
  for (int hb = 0; hb < 8; ++hb)
#pragma unroll
    for (int s = 0; s < 3; ++s) w.q1[hb][s] = 4 * s + q < C ? Q1[(16 * hb + j) * C + 4 * s + q] : 0.f;
#pragma unroll
  for (int o = 0; o < 2; ++o) {
#pragma unroll
    for (int hb = 0; hb < 8; ++hb)
      w.q2[o][hb] = *reinterpret_cast<const f32x4*>(Q2 + (16 * (2 * p + o) + j) * ld2 + 16 * hb + 4 * q);
    w.q3[o] = j < C ? *reinterpret_cast<const f32x4*>(Q3 + j * ld3 + 16 * (2 * p + o) + 4 * q) : f32x4{0.f, 0.f, 0.f, 0.f};
    w.b2[o] = *reinterpret_cast<const f32x4*>(b2 + 16 * (2 * p + o) + 4 * q);
  }
#pragma unroll
  for (int t = 0; t < 4; ++t) w.b3[t] = (p == 0 && 4 * q + t < C) ? b3[4 * q + t] : 0.f;
}

// Layer-1 blocks 2P, 2P+1 of one tile (part P), relu(dropout), saved row, and their LDS copy.
template <int P>
__device__ __forceinline__ void l1_pair(const T16W& w, const f32x4v (&uacc)[8], const float (&h)[C],
                                        const uint32_t (&kw1)[4], float scale, int q, int lane, float* a1row,
                                        float (*z1x)[64][4]) {
#pragma unroll
  for (int o = 0; o < 2; ++o) {
    constexpr int hb0 = 2 * P;
    const int hb = hb0 + o;
    f32x4v z = uacc[hb0 + o];
#pragma unroll
    for (int s = 0; s < 3; ++s) z = mfma16(w.q1[hb0 + o][s], sel4(h, s, q), z);
    dropout_relu16(z, kw1[P], hb, q, scale);
    if (a1row) *reinterpret_cast<f32x4*>(a1row + 16 * hb + 4 * q) = f32x4{z[0], z[1], z[2], z[3]};
    *reinterpret_cast<f32x4*>(&z1x[hb][lane][0]) = f32x4{z[0], z[1], z[2], z[3]};
  }
}

// The MLP of one tile for hidden part p (of 4): layer 1 in full (24 MFMA), layer-2 output blocks
// 2p, 2p+1 (64 MFMA), their layer-3 partial (8 MFMA; bias on part 0) -> zpart_lane[4] (LDS).
// a1row / a2row (nullable): the row's saved post-activations (part p stores its blocks).
// kShareL1 (z1x: LDS [8][64][4], all 4 waves call with the same choice): layer 1 split over the
// waves -- wave p computes blocks 2p, 2p+1 (6 MFMA instead of 24), they meet in LDS behind one
// workgroup barrier and every wave reads the 8 blocks back; bit-identical to the replicated layer 1.
template <bool kShareL1 = false>
__device__ __forceinline__ void mlp16_part(const T16W& w, const f32x4v (&uacc)[8], const float (&h)[C],
                                           const uint32_t (&kw1)[4], uint32_t kw2p, float scale, int p, int q,
                                           float* a1row, float* a2row, float* zpart_lane,
                                           float (*z1x)[64][4] = nullptr) {
  f32x4v z1[8];
  if constexpr (kShareL1) {
    const int lane = threadIdx.x & 63;
    switch (p) {              // wave-uniform: static register indices in each case
      case 0: l1_pair<0>(w, uacc, h, kw1, scale, q, lane, a1row, z1x); break;
      case 1: l1_pair<1>(w, uacc, h, kw1, scale, q, lane, a1row, z1x); break;
      case 2: l1_pair<2>(w, uacc, h, kw1, scale, q, lane, a1row, z1x); break;
      default: l1_pair<3>(w, uacc, h, kw1, scale, q, lane, a1row, z1x); break;
    }
    __syncthreads();
#pragma unroll
    for (int hb = 0; hb < 8; ++hb) {
      const f32x4 v = *reinterpret_cast<const f32x4*>(&z1x[hb][lane][0]);
      z1[hb] = f32x4v{v[0], v[1], v[2], v[3]};
    }
  } else {
#pragma unroll
    for (int hb = 0; hb < 8; ++hb) z1[hb] = uacc[hb];
#pragma unroll
    for (int s = 0; s < 3; ++s) {
      const float bs = sel4(h, s, q);
#pragma unroll
      for (int hb = 0; hb < 8; ++hb) z1[hb] = mfma16(w.q1[hb][s], bs, z1[hb]);
    }
#pragma unroll
    for (int hb = 0; hb < 8; ++hb) dropout_relu16(z1[hb], kw1[hb >> 1], hb, q, scale);
    if (a1row) {
#pragma unroll
      for (int hb = 0; hb < 8; ++hb)
        if ((hb >> 1) == p)
          *reinterpret_cast<f32x4*>(a1row + 16 * hb + 4 * q) = f32x4{z1[hb][0], z1[hb][1], z1[hb][2], z1[hb][3]};
    }
  }
  f32x4v z2[2];
#pragma unroll
  for (int o = 0; o < 2; ++o) z2[o] = f32x4v{w.b2[o][0], w.b2[o][1], w.b2[o][2], w.b2[o][3]};
#pragma unroll
  for (int hb = 0; hb < 8; ++hb) {
#pragma unroll
    for (int o = 0; o < 2; ++o) {
#pragma unroll
      for (int t = 0; t < 4; ++t) z2[o] = mfma16(w.q2[o][hb][t], z1[hb][t], z2[o]);
    }
  }
#pragma unroll
  for (int o = 0; o < 2; ++o) {
    dropout_relu16(z2[o], kw2p, 2 * p + o, q, scale);
    if (a2row)
      *reinterpret_cast<f32x4*>(a2row + 16 * (2 * p + o) + 4 * q) = f32x4{z2[o][0], z2[o][1], z2[o][2], z2[o][3]};
  }
  f32x4v z3 = f32x4v{w.b3[0], w.b3[1], w.b3[2], w.b3[3]};
#pragma unroll
  for (int o = 0; o < 2; ++o) {
#pragma unroll
    for (int t = 0; t < 4; ++t) z3 = mfma16(w.q3[o][t], z2[o][t], z3);
  }
  *reinterpret_cast<f32x4*>(zpart_lane) = f32x4{z3[0], z3[1], z3[2], z3[3]};
}

// After the barrier: this lane's sample j sums its 10 outputs over the 4 parts in a fixed order
// (outputs 4g .. 4g + 3 sit in lane 16 g + j, registers 0..3: one ds_read_b128 per part and
// group).  zpart: [4 parts][64 lanes][4].
__device__ __forceinline__ void ft16_sum(const float (*zpart)[64][4], int j, float (&ft)[C]) {
#pragma unroll
  for (int g = 0; g < 3; ++g) {
    f32x4 v[4];
#pragma unroll
    for (int pp = 0; pp < 4; ++pp) v[pp] = *reinterpret_cast<const f32x4*>(&zpart[pp][16 * g + j][0]);
#pragma unroll
    for (int r = 0; r < 4; ++r)
      if (4 * g + r < C) ft[4 * g + r] = ((v[0][r] + v[1][r]) + v[2][r]) + v[3][r];
  }
}

// The batch-global QP exit of one eval with speculation: bisect to kprev + FIODE_KSPEC_MARGIN, publish the wave's
// mask in granule slot slots[blockIdx] (epoch), gather all tiles; only if no iteration <= kspec
// converged everywhere, resume to max_iter - 1 and exchange again in slots[ntiles + ..].  Called
// by all 4 waves (identical rows); wave 0 exchanges; shK is an LDS int.  Returns K (uniform).
// allg (callers pass it for grids of <= 64 tiles, one granule per lane): every wave gathers the
// granules itself and returns K from its own registers (the rows are replicated over the waves, so
// all compute the same masks and the same K): no workgroup barrier and no LDS round trip for K;
// wave 0 still publishes, shK is left untouched.  With more tiles the 4x polling costs more than
// the barrier (B = 1024: exchange wait 2.35 -> 2.83 us per eval), so those keep the broadcast.
// R: rows per wave (16 or 4); rec: the row's mu record (shared by the row's lanes of this wave),
// bc: 2 LDS floats per (wave, row) for the tree bisection's bracket hand-over (FIODE_QP_TREE=0: the
// sequential bisection on every lane).
#ifndef FIODE_QP_TREE
#define FIODE_QP_TREE 1
#endif
template <int R>
__device__ __forceinline__ uint32_t qp_bisect_rows(const float (&lower)[C], const float (&nom)[C], int from, int to,
                                                   float tol, float& lo, float& hi, float* rec, float* bc,
                                                   bool valid) {
  // (the depth-2 tree of 16-row waves measured slower than the sequential loop: 341 -> 348 us for the
  // B = 2048 rk4 forward; depth 4 on 4-row waves: 234 -> 224 us at B = 128, dopri5 1263 -> 1171 us)
  if constexpr (FIODE_QP_TREE != 0 && QpTree<R>::LV >= 4) return qp_bisect_tree<R>(lower, nom, from, to, tol, lo, hi, rec, bc, valid);
  else return qp_bisect_seq(lower, nom, from, to, tol, lo, hi, rec, true, valid);
}

template <int R>
__device__ __forceinline__ int qp16_exit(const float (&lower)[C], const float (&nominal)[C], float tol, int max_iter,
                                         int kprev, bool valid, int p, int q, int lane, float* mu_rec_row, float* bc,
                                         unsigned long long* slots, unsigned epoch, int32_t* status, int& shK,
                                         int& dead, int drop_block = -1,
                                         unsigned long long* prof = nullptr, int stride = 1, bool allg = false) {
  const int last = max_iter - 1;
  const int kspec = min(last, kprev + FIODE_KSPEC_MARGIN);
  float lo, hi;
  const bool pr = prof && blockIdx.x == 0 && threadIdx.x == 0;      // phase timing (diagnostic builds)
  const uint64_t t0 = prof ? wall_clock64() : 0;
  qp_bracket(lower, nominal, lo, hi);
  uint32_t conv = qp_bisect_rows<R>(lower, nominal, 0, kspec, tol, lo, hi, mu_rec_row, bc, valid);
  const uint64_t t1 = prof ? wall_clock64() : 0;
  if (pr) atomicAdd(prof + 6, (unsigned long long)(t1 - t0));
  const int ntiles = gridDim.x;
  int kw = 0;
  if (allg || p == 0) {
    // drop_block (test hook, FIODE_DEBUG_DROP_PUBLISH): that workgroup never publishes epoch 1,
    // as if it were not resident -- exercises the timeout path
    if (p == 0 && lane == 0 && !(epoch == 1u && (int)blockIdx.x == drop_block))
      publish_mask(slots + (size_t)blockIdx.x * stride, epoch, conv);
    const uint32_t all = gather_masks(slots, ntiles, epoch, status, lane, dead, stride);
    const uint32_t lowm = kspec >= 31 ? 0xFFFFFFFFu : ((1u << (kspec + 1)) - 1u);
    const uint32_t bits = all & lowm;
    kw = bits ? (__ffs((int)bits) - 1) : (kspec >= last ? last : -1);
    if (!allg && lane == 0) shK = kw;
  }
  if (!allg) {                          // (uniform)
    __syncthreads();
    kw = shK;
  }
  if (pr) {
    atomicAdd(prof + 7, (unsigned long long)(wall_clock64() - t1));
    if (kw < 0) atomicAdd(prof + 8, 1ull);
  }
  if (kw < 0) {                         // block-uniform: every tile saw the same masks
    conv |= qp_bisect_rows<R>(lower, nominal, kspec + 1, last, tol, lo, hi, mu_rec_row, bc, valid);
    if (allg || p == 0) {
      unsigned long long* s2 = slots + (size_t)ntiles * stride;
      if (p == 0 && lane == 0) publish_mask(s2 + (size_t)blockIdx.x * stride, epoch, conv);
      const uint32_t all = gather_masks(s2, ntiles, epoch, status, lane, dead, stride);
      kw = qp_exit_iter(all, max_iter);
      if (!allg && lane == 0) shK = kw;
    }
    if (!allg) {
      __syncthreads();
      kw = shK;
    }
  }
  return kw;
}

}  // namespace fiode_t16
