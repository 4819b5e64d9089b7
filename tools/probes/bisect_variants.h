// Speculative bisection variants measured against the sequential one (bisect_probe.hip); kept
// here as probe code only -- the product uses qp_bisect_seq (tile16.h).
#pragma once
#include "../../fi-ode_amd/csrc/tile16.h"
namespace fiode_t16 {
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

}  // namespace fiode_t16
