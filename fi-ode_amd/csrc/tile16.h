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
// and max is a bare v_max_f32 (fmaxf's result for every non-signalling input; the compiler's fmaxf
// re-quiets `lower` at every use when the operand comes from another basic block: +10 VALU / eps).
__device__ __forceinline__ float vmax_f32(float a, float b) {
  float r;
  asm("v_max_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
__device__ __forceinline__ float qp_eps(const float (&lower)[C], const float (&nom)[C], float mu) {
  float eps = vmax_f32(nom[0] - mu, lower[0]);
#pragma unroll
  for (int j = 1; j < C; ++j) eps = eps + vmax_f32(nom[j] - mu, lower[j]);
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
    float E[4];
    rows4(e, q, E);
    const float e0 = E[0], eL = E[1], eR = E[2];
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

// Three iterations per round: the 4 lanes of a row (q = 0..3) evaluate TWO midpoints each -- slot a:
// m0 (q = 0, 3), the children mL (q = 1), mR (q = 2); slot b: the grandchildren mLL, mLR, mRL, mRR
// (q = 0..3) -- and rows4() (cross-row swaps, no LDS) hands every lane all seven eps values.  The
// path through the tree is then resolved exactly as the sequential loop walks it: each midpoint
// is the float32 expression (hi' - lo') / 2 + lo' of the bracket the sequential loop holds at
// that iteration (a bracket left unchanged by eps == 0 or NaN repeats its midpoint), so mu, the
// convergence bits and the exit are bit-identical to qp_bisect_range.
__device__ __forceinline__ uint32_t qp_bisect_range3(const float (&lower)[C], const float (&nom)[C], int from, int to,
                                                     float tol, float& lo, float& hi, float* mu_rec, bool rec,
                                                     bool valid, int q, int j) {
  uint32_t conv = 0;
  int it = from;
  for (; it + 2 <= to; it += 3) {
    const float m0 = (hi - lo) / 2.0f + lo;
    const float mL = (m0 - lo) / 2.0f + lo;          // bracket (lo, m0)
    const float mR = (hi - m0) / 2.0f + m0;          // bracket (m0, hi)
    const float mLL = (mL - lo) / 2.0f + lo;         // (lo, mL)
    const float mLR = (m0 - mL) / 2.0f + mL;         // (mL, m0)
    const float mRL = (mR - m0) / 2.0f + m0;         // (m0, mR)
    const float mRR = (hi - mR) / 2.0f + mR;         // (mR, hi)
    const float ma = q == 1 ? mL : (q == 2 ? mR : m0);
    const float mb = q == 0 ? mLL : (q == 1 ? mLR : (q == 2 ? mRL : mRR));
    const float ea = qp_eps(lower, nom, ma);
    const float eb = qp_eps(lower, nom, mb);
    float EA[4], EB[4];
    rows4(ea, q, EA);
    rows4(eb, q, EB);
    // iteration it: m0
    const float e0 = EA[0];
    if (rec) mu_rec[it] = m0;
    conv |= (__ballot(valid && !(fabsf(e0) < tol)) == 0ull ? 1u : 0u) << it;
    const bool l0 = e0 < 0.f, r0 = e0 > 0.f;
    const float lo1 = r0 ? m0 : lo, hi1 = l0 ? m0 : hi;
    // iteration it + 1
    const float m1 = l0 ? mL : (r0 ? mR : m0);
    const float e1 = l0 ? EA[1] : (r0 ? EA[2] : e0);
    if (rec) mu_rec[it + 1] = m1;
    conv |= (__ballot(valid && !(fabsf(e1) < tol)) == 0ull ? 1u : 0u) << (it + 1);
    const bool l1 = e1 < 0.f, r1 = e1 > 0.f;
    const float lo2 = r1 ? m1 : lo1, hi2 = l1 ? m1 : hi1;
    // iteration it + 2: a grandchild when both moves happened, else the unchanged bracket's midpoint
    float m2, e2;
    if (!(l0 || r0) || !(l1 || r1)) {
      m2 = m1;
      e2 = e1;
    } else {
      m2 = l0 ? (l1 ? mLL : mLR) : (l1 ? mRL : mRR);
      e2 = l0 ? (l1 ? EB[0] : EB[1]) : (l1 ? EB[2] : EB[3]);
    }
    if (rec) mu_rec[it + 2] = m2;
    conv |= (__ballot(valid && !(fabsf(e2) < tol)) == 0ull ? 1u : 0u) << (it + 2);
    lo = e2 > 0.f ? m2 : lo2;
    hi = e2 < 0.f ? m2 : hi2;
  }
  if (it <= to) conv |= qp_bisect_range2(lower, nom, it, to, tol, lo, hi, mu_rec, rec, valid, q, j);
  return conv;
}

// Four iterations per round over the WHOLE workgroup (the 4 waves hold the same 16 rows, so the 16
// lanes of a row -- (wave p, q) over 4 x 4 -- can split the work instead of repeating it): lane
// (p, q) evaluates node n = 4p + q + 1 of the round's bisection tree (heap order: root 1, children
// 2n (eps < 0: bracket (lo, m)) and 2n + 1 (eps > 0: (m, hi)); 15 nodes, node 16 unused), its eps
// goes to LDS (xt: two alternating [16 rows][16] buffers, one barrier per round), and every lane
// reads its row's 15 values and walks the path the sequential loop takes -- the same float32
// midpoint expressions (hi' - lo') / 2 + lo', a bracket left unchanged by eps == 0 or NaN repeating
// its midpoint -- so mu, the convergence bits and the exit are bit-identical to qp_bisect_range.
// Per lane one eps per 4 iterations instead of 2 per 3: the bisection is VALU-issue bound at one
// wave per SIMD.  Must be called by all 4 waves of the workgroup with the same (from, to).
__device__ __forceinline__ uint32_t qp_bisect_tree(const float (&lower)[C], const float (&nom)[C], int from, int to,
                                                   float tol, float& lo, float& hi, float* mu_rec, bool rec,
                                                   bool valid, int p, int q, int j, float (*xt)[TR][16], int& xbuf) {
  // this lane's node: depth dn (root 0) and the branch bits below the root (1 = right child)
  const int node = 4 * p + q + 1;
  const int dn = node >= 8 ? 3 : (node >= 4 ? 2 : (node >= 2 ? 1 : 0));
  uint32_t open = 0;      // bit it: this lane's row had |eps| >= tol at iteration it
  int it = from;
  for (; it + 3 <= to; it += 4) {
    float l = lo, h = hi, m = (hi - lo) / 2.0f + lo;
#pragma unroll
    for (int d = 1; d <= 3; ++d) {
      const bool right = (node >> (d <= dn ? dn - d : 0)) & 1;
      const float l2 = right ? m : l, h2 = right ? h : m;
      const float m2 = (h2 - l2) / 2.0f + l2;
      const bool use = d <= dn;
      l = use ? l2 : l;
      h = use ? h2 : h;
      m = use ? m2 : m;
    }
    float* row = &xt[xbuf][j][0];
    row[node - 1] = qp_eps(lower, nom, m);
    __syncthreads();
    float E[16];
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const f32x4 v = *reinterpret_cast<const f32x4*>(row + 4 * g);
      E[4 * g] = v[0]; E[4 * g + 1] = v[1]; E[4 * g + 2] = v[2]; E[4 * g + 3] = v[3];
    }
    xbuf ^= 1;
    // walk, branch-free: level k's node is 2^k + (branch bits so far); a level whose eps is 0 or
    // NaN leaves the bracket unchanged, so the next level repeats its midpoint and eps
    float mk[4], ek[4];
    mk[0] = (hi - lo) / 2.0f + lo;
    ek[0] = E[0];
    bool g[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      const bool gt = ek[k] > 0.f, lt = ek[k] < 0.f;
      g[k] = gt;
      lo = gt ? mk[k] : lo;
      hi = lt ? mk[k] : hi;
      mk[k + 1] = (hi - lo) / 2.0f + lo;
      float t;
      if (k == 0) t = gt ? E[2] : E[1];
      else if (k == 1) t = g[0] ? (gt ? E[6] : E[5]) : (gt ? E[4] : E[3]);
      else t = g[0] ? (g[1] ? (gt ? E[14] : E[13]) : (gt ? E[12] : E[11]))
                    : (g[1] ? (gt ? E[10] : E[9]) : (gt ? E[8] : E[7]));
      ek[k + 1] = (gt || lt) ? t : ek[k];
    }
    lo = ek[3] > 0.f ? mk[3] : lo;
    hi = ek[3] < 0.f ? mk[3] : hi;
#pragma unroll
    for (int k = 0; k < 4; ++k) open |= ((valid && !(fabsf(ek[k]) < tol)) ? 1u : 0u) << (it + k);
    if (rec) {
#pragma unroll
      for (int k = 0; k < 4; ++k) mu_rec[it + k] = mk[k];
    }
  }
  // converged bits of the rounds: no lane of the wave (its 16 rows) open
  const uint32_t span = (it > from) ? (((it - from) >= 32 ? 0xFFFFFFFFu : ((1u << (it - from)) - 1u)) << from) : 0u;
  uint32_t conv = ~wave_or16(open) & span;
  if (it <= to) conv |= qp_bisect_range2(lower, nom, it, to, tol, lo, hi, mu_rec, rec, valid, q, j);
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

// The MLP of one tile for hidden part p (of 4): layer 1 in full (24 MFMA), layer-2 output blocks
// 2p, 2p+1 (64 MFMA), their layer-3 partial (8 MFMA; bias on part 0) -> zpart_lane[4] (LDS).
// a1row / a2row (nullable): the row's saved post-activations (part p stores its blocks).
__device__ __forceinline__ void mlp16_part(const T16W& w, const f32x4v (&uacc)[8], const float (&h)[C],
                                           const uint32_t (&kw1)[4], uint32_t kw2p, float scale, int p, int q,
                                           float* a1row, float* a2row, float* zpart_lane) {
  f32x4v z1[8];
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

// The batch-global QP exit of one eval with speculation: bisect to kprev + 3, publish the wave's
// mask in granule slot slots[blockIdx] (epoch), gather all tiles; only if no iteration <= kspec
// converged everywhere, resume to max_iter - 1 and exchange again in slots[ntiles + ..].  Called
// by all 4 waves (identical rows); wave 0 exchanges; shK is an LDS int.  Returns K (uniform).
__device__ __forceinline__ int qp16_exit(const float (&lower)[C], const float (&nominal)[C], float tol, int max_iter,
                                         int kprev, bool valid, int p, int q, int lane, float* mu_rec_row,
                                         unsigned long long* slots, unsigned epoch, int32_t* status, int& shK,
                                         int& dead, float (*xt)[TR][16], int& xbuf, int drop_block = -1,
                                         unsigned long long* prof = nullptr) {
  const int last = max_iter - 1;
  const int kspec = min(last, kprev + 3);
  float lo, hi;
  const bool pr = prof && blockIdx.x == 0 && threadIdx.x == 0;      // phase timing (diagnostic builds)
  const uint64_t t0 = prof ? wall_clock64() : 0;
  qp_bracket(lower, nominal, lo, hi);
  const int j = lane & 15;
  uint32_t conv = qp_bisect_tree(lower, nominal, 0, kspec, tol, lo, hi, mu_rec_row, q == 0, valid, p, q, j, xt, xbuf);
  const uint64_t t1 = prof ? wall_clock64() : 0;
  if (pr) atomicAdd(prof + 6, (unsigned long long)(t1 - t0));
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
  if (pr) {
    atomicAdd(prof + 7, (unsigned long long)(wall_clock64() - t1));
    if (shK < 0) atomicAdd(prof + 8, 1ull);
  }
  if (shK < 0) {                        // block-uniform: every tile saw the same masks
    conv |= qp_bisect_tree(lower, nominal, kspec + 1, last, tol, lo, hi, mu_rec_row, q == 0, valid, p, q, j, xt, xbuf);
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
