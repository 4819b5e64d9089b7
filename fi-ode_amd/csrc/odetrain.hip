// Differentiable fixed-grid RK4 ODE solve of the Cayley-MLP dynamics (gfx950): the train_ode
// branch of LyapunovLearning.compute_loss (pl_modules.py:490-500):
//   y_hat = model(x, ts=linspace(0, t_max, 2), int_params={method: 'rk4', step_size}) in TRAIN
//   mode -> odeint(IVP.h_dot, (h0,), ts) (models.py:235-241) backpropagated through the stages
// (torchdiffeq 0.2.2 FixedGridODESolver + rk4_alt_step_func, the 3/8 rule; every func() call is
// eval_dot with fresh dropout masks and the QP's batch-global exit over the B rows).
//
// Forward  (k_ot_fwd, one persistent workgroup per 32-row tile, all tiles co-resident; each
//   stage's QP exit is a batch-wide AND exchanged through tagged granules, see below):
//   for each step, stage i = 1..4 (eval e = 4*step + i - 1), per row in registers:
//     Y_i = y + dt * sum_j beta_ij k_j      -> hs[b][e]
//     MLP (MFMA, hidden split over 4 waves), a1/a2 saved -> a1/a2[b][e], ft[b][e]
//     QP bisection recording mu per iteration; exit K from all tiles; k_i = v(mu_K)
//   y += (k1 + 3 (k2 + k3) + k4) dt / 8
// Backward (k_ot_bwd, one workgroup per 32 rows; rows never interact in the backward, so tiles
//   need no grid-wide synchronisation): the reverse sweep of the 3/8 rule; every stage VJP is the QP backward
//   (closed form), the sigmoid rescale, the barrier bounds' h-dependence, and the MLP input
//   gradients (Q3^T, Q2^T via LDS images, Q1^T via a zero-padded LDS image), writing the per-
//   (row, eval) activation gradients gft / gz2 / gz1.
// Weight gradients: the training step's wgrad chain over rows r = b*E + e (wgrad.h).
#include "common.h"
#include "tile.h"
#include "wgrad.h"
#include "../../include/fiode.h"

namespace {
using namespace fiode_tile;


struct OTArgs {
  int B, E, niters;
  float t0, t1, hstep;
  int dropout_mode, bit_mode;
  uint32_t thr8;
  float drop_scale;
  Rng rng;
  const uint64_t* offset_dev;
  DynScalars d;
  const float* x_feat;
  const float* h0;
  const uint8_t* masks;     // [E][2][B][M] (GIVEN)
  const float *Q1, *b1, *Qx, *bx, *Q2, *b2, *Q3, *b3;
  float* y_out;             // [B][C]
  int32_t* stats;           // [8]: nfe, steps, last exit iteration
  const float* g_y;         // [B][C] (backward)
  float* dbg_gft;           // optional [B][E][C]
  // workspace (saved by the forward for the backward)
  float* u;                 // [B][M]
  float* y;                 // [B][C]
  float* k;                 // [4][B][C]
  float* hs;                // [B][E][C] stage inputs
  float* ftw;               // [B][E][C] raw MLP outputs
  float* vw;                // [B][E][C] QP outputs (the stage derivatives k_i)
  float* muw;               // [B][E]
  float* nomw;              // [B][E][C] QP nominal (for checkers: the QP active-set test input)
  float* a1;                // [B][E][M]
  float* a2;                // [B][E][M]
  float* gz2;               // [B][E][M]
  float* gz1;               // [B][E][M]
  float* gft;               // [B][E][C]
  unsigned long long* xslots;  // [E][2 phases][ntiles] {epoch, mask} granules of the QP exit exchange
  uint32_t* kw;                // [E][2][B] uint4 dropout keep words
#ifdef OT_PROFILE
  unsigned long long* prof;    // [8] wall-clock ticks per phase (workgroup 0, lane 0)
#endif
};

// float32 grid of FixedGridODESolver: t_k = k*h + t0, last point = t1
__device__ __forceinline__ void step_times(const OTArgs& a, int it, float& ta, float& dt) {
  ta = (float)it * a.hstep + a.t0;
  const float tb = (it + 2 == a.niters) ? a.t1 : (float)(it + 1) * a.hstep + a.t0;
  dt = tb - ta;
}

__device__ __forceinline__ Rng rng_of(const OTArgs& a) {
  Rng r = a.rng;
  if (a.offset_dev) {
    const uint64_t o = (((uint64_t)r.off_hi << 32) | r.off_lo) + *a.offset_dev;
    r.off_lo = (uint32_t)o;
    r.off_hi = (uint32_t)(o >> 32);
  }
  return r;
}

// ---------------------------------------------------------------------------------------------
// forward: one workgroup per 32-row tile, persistent over all evals; 4 waves = 4 parts of the
// hidden dimension.  Per eval every wave computes layer 1 in full (20 MFMA), its 32 of the 128
// layer-2 outputs (64 MFMA) and their layer-3 partial (16 MFMA); the partials meet in LDS and
// every wave sums them in the same order, so the row state (y, k1..k4, the QP) is replicated in
// the 4 waves and needs no further exchange.  The only cross-tile coupling -- the QP's exit
// iteration, the lowest bit of the AND over ALL rows of the per-iteration convergence masks --
// is exchanged through per-eval {tag, mask} granules: each workgroup publishes its mask with ONE
// agent-scope 64-bit atomic store, then one wave sweeps the ntiles granules of that eval until
// every tag matches (relaxed agent-scope loads; the granule IS the flag, so no fence is needed).
// The spin is bounded: on timeout the status word records it and the solve completes.
struct OtShared {
  float zpart[4][64][6];      // [part][lane][valid layer-3 accumulator registers]
  float mu_rec[4][32][33];    // [wave][row][bisection iteration] (padded)
  float Q1s[M * C];
  int K;
  int Kprev;                  // previous eval's exit iteration (speculation for the next)
  int pad[2];
};

typedef __attribute__((address_space(1))) unsigned long long gu64_t;
typedef __attribute__((address_space(1))) unsigned int gu32_t;

__device__ __forceinline__ void publish_mask(unsigned long long* slot, unsigned epoch, uint32_t mask) {
  __hip_atomic_store((gu64_t*)(slot), ((unsigned long long)epoch << 32) | mask, __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}

// one wave: AND of the masks of all tiles for this epoch (lane i reads tiles i, i+64, ...)
__device__ __forceinline__ uint32_t gather_masks(unsigned long long* slots, int ntiles, unsigned epoch,
                                                 int32_t* status, int lane) {
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
      if (++spins > (1u << 22)) {           // ~0.5 s: a non-resident tile; record and give up
        if (lane == 0) atomicMax(status, 4);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
  }
  return wave_and(acc);
}

// The bisection of FastBarrierProjectionNoUpper (qp_bisect, common.h) split so it can stop and
// resume: iterations [from, to] from the bracket state (lo, hi), recording mu per iteration.
__device__ __forceinline__ void qp_bracket(const float (&lower)[C], const float (&nom)[C], float& lo, float& hi) {
  hi = nom[0] - lower[0];
  lo = nom[0];
#pragma unroll
  for (int j = 1; j < C; ++j) {
    hi = fmaxf(hi, nom[j] - lower[j]);
    lo = fminf(lo, nom[j]);
  }
}
__device__ __forceinline__ uint32_t qp_bisect_range(const float (&lower)[C], const float (&nom)[C], int from, int to,
                                                    float tol, float& lo, float& hi, float* mu_rec, bool rec) {
  uint32_t conv = 0;
  for (int it = from; it <= to; ++it) {
    const float mu = (hi - lo) / 2.0f + lo;
    float eps = 0.f;
#pragma unroll
    for (int j = 0; j < C; ++j) eps = eps + fmaxf(nom[j] - mu, lower[j]);
    if (rec) mu_rec[it] = mu;
    conv |= (fabsf(eps) < tol ? 1u : 0u) << it;
    lo = eps > 0.f ? mu : lo;
    hi = eps < 0.f ? mu : hi;
  }
  return conv;
}

#ifdef OT_PROFILE
#define OT_MARK(i) do { const uint64_t t_ = wall_clock64(); if (blockIdx.x == 0 && threadIdx.x == 0) \
    atomicAdd((unsigned long long*)&a.prof[i], (unsigned long long)(t_ - t_prev)); t_prev = t_; } while (0)
#else
#define OT_MARK(i) do { } while (0)
#endif

// one eval for this workgroup's tile: stage input h (per lane, its row) -> k (per lane)
__device__ void ot_eval(const OTArgs& a, const float* Q2s, const float* Q3s, OtShared& sh, int e, int p, int b,
                        bool valid, int lane, int half, int col, const f32x16 (&uacc)[4], const uint32_t (&kw1)[4],
                        uint32_t kw2p, const float (&h)[C], float (&k)[C]) {
  const int bb = valid ? b : a.B - 1;
  const size_t r = (size_t)bb * a.E + e;
#ifdef OT_PROFILE
  uint64_t t_prev = wall_clock64();
#endif
  if (p == 0 && valid && half == 0) store_row10(a.hs + r * C, h);
  // layer 1 (full): z1 = u[b] + Q1 h
  f32x16 z1[4];
#pragma unroll
  for (int mb = 0; mb < 4; ++mb) z1[mb] = uacc[mb];
#pragma unroll
  for (int s = 0; s < 5; ++s) {
    const float bs = half ? h[2 * s + 1] : h[2 * s];
#pragma unroll
    for (int mb = 0; mb < 4; ++mb) z1[mb] = mfma32(sh.Q1s[(32 * mb + col) * C + 2 * s + half], bs, z1[mb]);
  }
#pragma unroll
  for (int mb = 0; mb < 4; ++mb) dropout_relu(z1[mb], kw1[mb], half, a.drop_scale);
  OT_MARK(0);
  if (valid) {
#pragma unroll
    for (int mb = 0; mb < 4; ++mb)
      if (mb == p) store_acc_rows(a.a1 + r * M, mb, half, z1[mb]);
  }
  // layer 2, output block p: z2 = b2 + Q2[32p.., :] a1
  f32x16 z2;
  load_acc_rows(a.b2, p, half, z2);
#pragma unroll
  for (int kb = 0; kb < 4; ++kb) {
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const f32x4 q = *reinterpret_cast<const f32x4*>(Q2s + (32 * p + col) * LDQ + 32 * kb + 8 * g + 4 * half);
#pragma unroll
      for (int t = 0; t < 4; ++t) z2 = mfma32(q[t], z1[kb][4 * g + t], z2);
    }
  }
  dropout_relu(z2, kw2p, half, a.drop_scale);
  if (valid) store_acc_rows(a.a2 + r * M, p, half, z2);
  // layer-3 partial over hidden block p (bias on part 0)
  f32x16 z3 = f16_zero();
  if (p == 0) {
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int i = acc_row(q, half);
      z3[q] = i < C ? a.b3[i] : 0.f;
    }
  }
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    const f32x4 q = *reinterpret_cast<const f32x4*>(Q3s + col * LDQ + 32 * p + 8 * g + 4 * half);
#pragma unroll
    for (int t = 0; t < 4; ++t) z3 = mfma32(q[t], z2[4 * g + t], z3);
  }
#pragma unroll
  for (int q = 0; q < 6; ++q) sh.zpart[p][lane][q] = z3[q];
  OT_MARK(1);
  __syncthreads();
  f32x16 zs = f16_zero();
#pragma unroll
  for (int q = 0; q < 6; ++q)
    zs[q] = ((sh.zpart[0][lane][q] + sh.zpart[1][lane][q]) + sh.zpart[2][lane][q]) + sh.zpart[3][lane][q];
  float ft[C], lower[C], nominal[C], sig[C], span[C];
  gather_ft(zs, half, ft);
  barrier_nominal(a.d, h, ft, lower, nominal, sig, span);
  // Speculative exit: bisect up to the previous eval's exit + 3 and exchange; only if no iteration
  // <= that converged on every row of the batch, continue to max_iter - 1 and exchange again.
  // K is the same as the full sweep's (the lowest all-converged iteration wins either way).
  const int last = a.d.max_iter - 1;
  const int kspec = min(last, sh.Kprev + 3);
  float lo, hi;
  qp_bracket(lower, nominal, lo, hi);
  float* rec = &sh.mu_rec[p][col][0];
  uint32_t conv = qp_bisect_range(lower, nominal, 0, kspec, a.d.tol, lo, hi, rec, half == 0);
  uint32_t wconv = valid ? conv : 0xFFFFFFFFu;
  wconv = wave_and(wconv);
  OT_MARK(2);
  const int ntiles = gridDim.x;
  unsigned long long* slots = a.xslots + (size_t)e * 2 * ntiles;
  if (p == 0) {
    if (lane == 0) publish_mask(slots + blockIdx.x, (unsigned)e + 1u, wconv);
    const uint32_t all = gather_masks(slots, ntiles, (unsigned)e + 1u, a.stats + 3, lane);
    const uint32_t lowm = kspec >= 31 ? 0xFFFFFFFFu : ((1u << (kspec + 1)) - 1u);
    const uint32_t bits = all & lowm;
    if (lane == 0) sh.K = bits ? (__ffs((int)bits) - 1) : (kspec >= last ? last : -1);
  }
  __syncthreads();
  if (sh.K < 0) {                       // block-uniform: every tile saw the same masks
    conv |= qp_bisect_range(lower, nominal, kspec + 1, last, a.d.tol, lo, hi, rec, half == 0);
    wconv = valid ? conv : 0xFFFFFFFFu;
    wconv = wave_and(wconv);
    if (p == 0) {
      if (lane == 0) publish_mask(slots + ntiles + blockIdx.x, (unsigned)e + 1u, wconv);
      const uint32_t all = gather_masks(slots + ntiles, ntiles, (unsigned)e + 1u, a.stats + 3, lane);
      if (lane == 0) sh.K = qp_exit_iter(all, a.d.max_iter);
    }
    __syncthreads();
  }
  const int K = (int)sh.K;
  const float mu = sh.mu_rec[p][col][K];
#pragma unroll
  for (int j = 0; j < C; ++j) k[j] = fmaxf(nominal[j] - mu, lower[j]);
  if (p == 0 && valid && half == 0) {
    store_row10(a.ftw + r * C, ft);
    store_row10(a.nomw + r * C, nominal);
    store_row10(a.vw + r * C, k);
    a.muw[r] = mu;
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) a.stats[2] = K;
  if (threadIdx.x == 0) sh.Kprev = K;
  __syncthreads();            // zpart / mu_rec / K reused by the next eval
  OT_MARK(4);
}

// dropout keep words of every (eval, set, row): kw[e][set][b] (uint4 = the 4 words of the 128 units)
__global__ __launch_bounds__(256) void k_ot_masks(OTArgs a) {
  const int q = blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= a.E * a.B) return;
  const int e = q / a.B, b = q - e * a.B;
  const Rng rng = rng_of(a);
#pragma unroll
  for (int set = 0; set < 2; ++set) {
    const uint8_t* m = a.dropout_mode == FIODE_DROPOUT_GIVEN ? a.masks + (((size_t)e * 2 + set) * a.B + b) * M : nullptr;
    uint32_t w[4];
    dropout_keep_words(a.dropout_mode, a.bit_mode, a.thr8, rng, m, (uint32_t)b,
                       RNG_STREAM_ODE_DROP + ((uint32_t)e << 5) + ((uint32_t)set << 4), w);
    reinterpret_cast<uint4*>(a.kw)[((size_t)e * 2 + set) * a.B + b] = make_uint4(w[0], w[1], w[2], w[3]);
  }
}

__global__ __launch_bounds__(256) void k_ot_fwd(OTArgs a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* Q2s = smem;
  float* Q3s = smem + M * LDQ;
  OtShared& sh = *reinterpret_cast<OtShared*>(smem + (M + 32) * LDQ);
  load_weight_images(a.Q2, a.Q3, Q2s, Q3s, false);
  for (int q = threadIdx.x; q < M * C; q += blockDim.x) sh.Q1s[q] = a.Q1[q];
  if (threadIdx.x == 0) sh.Kprev = a.d.max_iter - 1;
  const int lane = threadIdx.x & 63, half = lane >> 5, col = lane & 31;
  const int p = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int b = blockIdx.x * 32 + col;
  const bool valid = b < a.B;
  const int bb = valid ? b : a.B - 1;
  // u[b] = U_x x_b + bx + b1 for this tile's rows (part p computes hidden block p)
  for (int q = threadIdx.x; q < 32 * M; q += blockDim.x) {
    const int rb = blockIdx.x * 32 + q / M, i = q % M;
    if (rb < a.B) {
      float s = 0.f;
#pragma unroll
      for (int c = 0; c < FIODE_X; ++c) s = __fmaf_rn(a.Qx[i * FIODE_X + c], a.x_feat[(size_t)rb * FIODE_X + c], s);
      a.u[(size_t)rb * M + i] = (s + a.bx[i]) + a.b1[i];
    }
  }
  __syncthreads();
  f32x16 uacc[4];
#pragma unroll
  for (int mb = 0; mb < 4; ++mb) load_acc_rows(a.u + (size_t)bb * M, mb, half, uacc[mb]);
  // dropout keep words of eval e (k_ot_masks), prefetched one eval ahead
  const uint4* kwp = reinterpret_cast<const uint4*>(a.kw);
  auto fetch = [&](int e, uint32_t (&w1)[4], uint32_t& w2) {
    if (a.dropout_mode == FIODE_DROPOUT_OFF) {
      w1[0] = w1[1] = w1[2] = w1[3] = w2 = 0xFFFFFFFFu;
      return;
    }
    const uint4 q1 = kwp[((size_t)e * 2 + 0) * a.B + bb];
    const uint4 q2 = kwp[((size_t)e * 2 + 1) * a.B + bb];
    w1[0] = q1.x; w1[1] = q1.y; w1[2] = q1.z; w1[3] = q1.w;
    w2 = p == 0 ? q2.x : p == 1 ? q2.y : p == 2 ? q2.z : q2.w;
  };
  uint32_t kc1[4], kc2, kn1[4], kn2;
  fetch(0, kc1, kc2);
  float y[C], k1[C], k2[C], k3[C], k4[C], hin[C];
  load_row10(a.h0 + (size_t)bb * C, y);
  const float third = 1.0f / 3.0f;
  for (int it = 0; it + 1 < a.niters; ++it) {
    float ta, dt;
    step_times(a, it, ta, dt);
    const int e0 = 4 * it;
    const int eN = 4 * (a.niters - 1);
#define OT_STAGE(E_, H_, K_)                                                       \
    {                                                                              \
      if ((E_) + 1 < eN) fetch((E_) + 1, kn1, kn2);                                \
      ot_eval(a, Q2s, Q3s, sh, (E_), p, b, valid, lane, half, col, uacc, kc1, kc2, H_, K_); \
      kc1[0] = kn1[0]; kc1[1] = kn1[1]; kc1[2] = kn1[2]; kc1[3] = kn1[3]; kc2 = kn2; \
    }
    OT_STAGE(e0, y, k1)
#pragma unroll
    for (int j = 0; j < C; ++j) hin[j] = y[j] + (dt * k1[j]) * third;
    OT_STAGE(e0 + 1, hin, k2)
#pragma unroll
    for (int j = 0; j < C; ++j) hin[j] = y[j] + dt * (k2[j] - k1[j] * third);
    OT_STAGE(e0 + 2, hin, k3)
#pragma unroll
    for (int j = 0; j < C; ++j) hin[j] = y[j] + dt * ((k1[j] - k2[j]) + k3[j]);
    OT_STAGE(e0 + 3, hin, k4)
#undef OT_STAGE
#pragma unroll
    for (int j = 0; j < C; ++j) {
      const float dy = (((k1[j] + 3.0f * (k2[j] + k3[j])) + k4[j]) * dt) * 0.125f;
      y[j] = y[j] + dy;
    }
  }
  if (p == 0 && valid && half == 0) store_row10(a.y_out + (size_t)b * C, y);
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    a.stats[0] = 4 * (a.niters - 1);
    a.stats[1] = a.niters - 1;
  }
}

// ---------------------------------------------------------------------------------------------
// backward: one workgroup per 32-row tile, 4 waves = 4 parts of the hidden dimension.  Every
// wave runs the row math (QP backward, rescale, barrier terms) and g_a2 = Q3^T g_ft in full
// (identical values in all 4 waves), then its 32 of the 128 rows of g_a1 = Q2^T g_z2 (64 MFMA)
// and their Q1^T partial; the 4 partials of g_h meet in LDS (double-buffered, one barrier per
// VJP) and every wave sums them in the same order, so the adjoint state stays replicated.
struct OtBwdShared {
  float gpart[2][4][64][6];
};

__device__ void ot_vjp(const OTArgs& a, const float* Q2Ts, const float* Q1Ts, const float (&q3t)[4][5],
                       OtBwdShared& sh, int buf, int p, int e, int b, bool valid, int lane, int half, int col,
                       const float (&g)[C], float (&gy_out)[C]) {
  const int bb = valid ? b : a.B - 1;
  const size_t r = (size_t)bb * a.E + e;
  float h[C], ft[C], v[C], lower[C], nominal[C], sig[C], span[C];
  load_row10(a.hs + r * C, h);
  load_row10(a.ftw + r * C, ft);
  load_row10(a.vw + r * C, v);
  const float mu = a.muw[r];
  barrier_nominal(a.d, h, ft, lower, nominal, sig, span);
  float g_nom[C], g_low[C], gft[C], ghb[C];
  float gin[C];
#pragma unroll
  for (int j = 0; j < C; ++j) gin[j] = valid ? g[j] : 0.f;
  qp_backward_row(gin, v, mu, nominal, g_nom, g_low);
#pragma unroll
  for (int j = 0; j < C; ++j) {
    float g_lo = g_low[j], g_up = 0.f;
    if (a.d.scale_nominal) {
      // nominal = span * sig + lower, span = upper - lower
      gft[j] = ((g_nom[j] * span[j]) * (1.0f - sig[j])) * sig[j];
      const float g_span = g_nom[j] * sig[j];
      g_lo = (g_lo + g_nom[j]) - g_span;
      g_up = g_span;
    } else {
      gft[j] = g_nom[j];
    }
    // lower = -a1 (exp(s1 h) - 1), upper = a2 (1 - h)
    ghb[j] = ((g_lo * -a.d.alpha_1) * expf(a.d.sigma_1 * h[j])) * a.d.sigma_1 + g_up * -a.d.alpha_2;
  }
  if (p == 0 && valid && half == 0) {
    store_row10(a.gft + r * C, gft);
    if (a.dbg_gft) store_row10(a.dbg_gft + r * C, gft);
  }
  // g_a2^T = Q3^T g_ft^T (all 128 rows), masked by the saved post-activation a2
  f32x16 ga[4];
#pragma unroll
  for (int mb = 0; mb < 4; ++mb) ga[mb] = f16_zero();
#pragma unroll
  for (int s = 0; s < 5; ++s) {
    const float bs = half ? gft[2 * s + 1] : gft[2 * s];
#pragma unroll
    for (int mb = 0; mb < 4; ++mb) ga[mb] = mfma32(q3t[mb][s], bs, ga[mb]);
  }
#pragma unroll
  for (int mb = 0; mb < 4; ++mb) {
    f32x16 act;
    load_acc_rows(a.a2 + r * M, mb, half, act);
#pragma unroll
    for (int q = 0; q < 16; ++q) ga[mb][q] = act[q] > 0.f ? ga[mb][q] * a.drop_scale : 0.f;
    if (valid && mb == p) store_acc_rows(a.gz2 + r * M, mb, half, ga[mb]);
  }
  // rows 32p.. of g_a1^T = Q2^T g_z2^T
  f32x16 gb = f16_zero();
#pragma unroll
  for (int kb = 0; kb < 4; ++kb) {
#pragma unroll
    for (int gg = 0; gg < 4; ++gg) {
      const f32x4 q = *reinterpret_cast<const f32x4*>(Q2Ts + (32 * p + col) * LDQ + 32 * kb + 8 * gg + 4 * half);
#pragma unroll
      for (int t = 0; t < 4; ++t) gb = mfma32(q[t], ga[kb][4 * gg + t], gb);
    }
    __builtin_amdgcn_sched_barrier(0);
  }
  {
    f32x16 act;
    load_acc_rows(a.a1 + r * M, p, half, act);
#pragma unroll
    for (int q = 0; q < 16; ++q) gb[q] = act[q] > 0.f ? gb[q] * a.drop_scale : 0.f;
    if (valid) store_acc_rows(a.gz1 + r * M, p, half, gb);
  }
  // partial g_h^T over hidden rows 32p.. (Q1^T image padded to 32 output rows)
  f32x16 gh = f16_zero();
#pragma unroll
  for (int gg = 0; gg < 4; ++gg) {
    const f32x4 q = *reinterpret_cast<const f32x4*>(Q1Ts + col * LDQ + 32 * p + 8 * gg + 4 * half);
#pragma unroll
    for (int t = 0; t < 4; ++t) gh = mfma32(q[t], gb[4 * gg + t], gh);
  }
#pragma unroll
  for (int q = 0; q < 6; ++q) sh.gpart[buf][p][lane][q] = gh[q];
  __syncthreads();
  f32x16 gs = f16_zero();
#pragma unroll
  for (int q = 0; q < 6; ++q)
    gs[q] = ((sh.gpart[buf][0][lane][q] + sh.gpart[buf][1][lane][q]) + sh.gpart[buf][2][lane][q]) +
            sh.gpart[buf][3][lane][q];
  float ghm[C];
  gather_ft(gs, half, ghm);
#pragma unroll
  for (int j = 0; j < C; ++j) gy_out[j] = ghm[j] + ghb[j];
}

__global__ __launch_bounds__(256) void k_ot_bwd(OTArgs a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* Q2Ts = smem;                 // Q2^T image [128][LDQ]
  float* Q1Ts = smem + M * LDQ;       // Q1^T image [32][LDQ] (rows >= 10 zero)
  OtBwdShared& sh = *reinterpret_cast<OtBwdShared*>(smem + (M + 32) * LDQ);
  load_weight_images(a.Q2, nullptr, Q2Ts, nullptr, true);
  for (int q = threadIdx.x; q < 32 * M; q += blockDim.x) {
    const int c = q >> 7, i = q & 127;
    Q1Ts[c * LDQ + i] = c < C ? a.Q1[i * C + c] : 0.f;
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, half = lane >> 5, col = lane & 31;
  const int p = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  float q3t[4][5];
#pragma unroll
  for (int mb = 0; mb < 4; ++mb)
#pragma unroll
    for (int s = 0; s < 5; ++s) q3t[mb][s] = a.Q3[(2 * s + half) * M + 32 * mb + col];
  const int b = blockIdx.x * 32 + col;
  const bool valid = b < a.B;
  float gy[C];
  if (valid) load_row10(a.g_y + (size_t)b * C, gy);
  else
#pragma unroll
    for (int j = 0; j < C; ++j) gy[j] = 0.f;
  const float third = 1.0f / 3.0f;
  int buf = 0;
  for (int it = a.niters - 2; it >= 0; --it) {
    float ta, dt;
    step_times(a, it, ta, dt);
    const float c8 = dt * 0.125f, c38 = 3.0f * c8;
    float gk1[C], gk2[C], gk3[C], gk4[C], acc[C], gY[C];
#pragma unroll
    for (int j = 0; j < C; ++j) {
      acc[j] = gy[j];
      gk1[j] = gy[j] * c8;
      gk2[j] = gy[j] * c38;
      gk3[j] = gy[j] * c38;
      gk4[j] = gy[j] * c8;
    }
    const int e0 = 4 * it;
    ot_vjp(a, Q2Ts, Q1Ts, q3t, sh, buf, p, e0 + 3, b, valid, lane, half, col, gk4, gY);  // Y4 = y + dt (k1 - k2 + k3)
    buf ^= 1;
#pragma unroll
    for (int j = 0; j < C; ++j) {
      acc[j] += gY[j];
      const float d = dt * gY[j];
      gk1[j] += d;
      gk2[j] -= d;
      gk3[j] += d;
    }
    ot_vjp(a, Q2Ts, Q1Ts, q3t, sh, buf, p, e0 + 2, b, valid, lane, half, col, gk3, gY);  // Y3 = y + dt (k2 - k1/3)
    buf ^= 1;
#pragma unroll
    for (int j = 0; j < C; ++j) {
      acc[j] += gY[j];
      const float d = dt * gY[j];
      gk2[j] += d;
      gk1[j] -= d * third;
    }
    ot_vjp(a, Q2Ts, Q1Ts, q3t, sh, buf, p, e0 + 1, b, valid, lane, half, col, gk2, gY);  // Y2 = y + (dt k1) / 3
    buf ^= 1;
#pragma unroll
    for (int j = 0; j < C; ++j) {
      acc[j] += gY[j];
      gk1[j] += (dt * gY[j]) * third;
    }
    ot_vjp(a, Q2Ts, Q1Ts, q3t, sh, buf, p, e0, b, valid, lane, half, col, gk1, gY);      // Y1 = y
    buf ^= 1;
#pragma unroll
    for (int j = 0; j < C; ++j) gy[j] = acc[j] + gY[j];
  }
}

inline size_t al(size_t x) { return (x + 255) & ~(size_t)255; }

int grid_iters(const fiode_odetrain_config* cfg) {
  const float t0 = (float)cfg->t0, t1 = (float)cfg->t1, h = (float)cfg->step_size;
  if (!(h > 0.f) || !(t1 > t0)) return -1;
  const float n = ceilf((t1 - t0) / h + 1.0f);
  if (!(n >= 2.f) || n > 1025.f) return -1;
  return (int)n;
}

struct OtLayout {
  size_t u, y, k, hs, ftw, vw, muw, nomw, a1, a2, gz2, gz1, gft, xs, kw, wg, total;
};
OtLayout ot_layout(int B, int E) {
  OtLayout L;
  const size_t R = (size_t)B * E;
  size_t o = 0;
  L.u = o; o += al((size_t)B * M * 4);
  L.y = o; o += al((size_t)B * C * 4);
  L.k = o; o += al(4 * (size_t)B * C * 4);
  L.hs = o; o += al(R * C * 4);
  L.ftw = o; o += al(R * C * 4);
  L.vw = o; o += al(R * C * 4);
  L.muw = o; o += al(R * 4);
  L.nomw = o; o += al(R * C * 4);
  L.a1 = o; o += al(R * M * 4);
  L.a2 = o; o += al(R * M * 4);
  L.gz2 = o; o += al(R * M * 4);
  L.gz1 = o; o += al(R * M * 4);
  L.gft = o; o += al(R * C * 4);
  L.xs = o; o += al((size_t)E * 2 * ((B + 31) / 32) * 8 + 256);
  L.kw = o; o += al((size_t)E * 2 * B * 16);
  L.wg = o; o += al(fiode_internal::wgrad_bytes(B, E));
  L.total = o;
  return L;
}

int fill_args(OTArgs& a, const fiode_odetrain_config* cfg, const fiode_dyn_config* dyn, const fiode_dyn_weights* w,
              const float* x_feat, void* workspace, size_t workspace_bytes) {
  if (!cfg || !dyn || !w || !x_feat || !workspace) return FIODE_EINVAL;
  if (dyn->n_hidden != C || dyn->mlp_size != M || dyn->x_dim != FIODE_X) return FIODE_ESHAPE;
  if (dyn->qp_max_iter < 1 || dyn->qp_max_iter > 32) return FIODE_EINVAL;
  if (!(dyn->dropout >= 0.f && dyn->dropout < 1.f)) return FIODE_EINVAL;
  if (cfg->batch <= 0 || cfg->batch > FIODE_ODE_MAX_BATCH) return FIODE_EINVAL;
  if (cfg->dropout_mode < 0 || cfg->dropout_mode > 2) return FIODE_EINVAL;
  if (!w->Q1 || !w->b1 || !w->Qx || !w->bx || !w->Q2 || !w->b2 || !w->Q3 || !w->b3) return FIODE_EINVAL;
  const int n = grid_iters(cfg);
  if (n < 0) return FIODE_EINVAL;
  a.B = cfg->batch; a.niters = n; a.E = 4 * (n - 1);
  const OtLayout L = ot_layout(a.B, a.E);
  if (workspace_bytes < L.total) return FIODE_EWORKSPACE;
  a.t0 = (float)cfg->t0; a.t1 = (float)cfg->t1; a.hstep = (float)cfg->step_size;
  a.dropout_mode = dyn->dropout > 0.f ? cfg->dropout_mode : FIODE_DROPOUT_OFF;
  a.bit_mode = dyn->dropout == 0.5f;
  a.thr8 = (uint32_t)lrintf(256.0f * (1.0f - dyn->dropout));
  a.drop_scale = a.dropout_mode == FIODE_DROPOUT_OFF ? 1.0f : 1.0f / (1.0f - dyn->dropout);
  a.rng.key = make_uint2((uint32_t)cfg->seed, (uint32_t)(cfg->seed >> 32));
  a.rng.off_lo = (uint32_t)cfg->offset; a.rng.off_hi = (uint32_t)(cfg->offset >> 32);
  a.d.alpha_1 = dyn->alpha_1; a.d.alpha_2 = dyn->alpha_2; a.d.sigma_1 = dyn->sigma_1;
  a.d.tol = dyn->qp_tol; a.d.scale_nominal = dyn->scale_nominal; a.d.max_iter = dyn->qp_max_iter;
  a.x_feat = x_feat;
  a.Q1 = w->Q1; a.b1 = w->b1; a.Qx = w->Qx; a.bx = w->bx; a.Q2 = w->Q2; a.b2 = w->b2; a.Q3 = w->Q3; a.b3 = w->b3;
  char* ws = static_cast<char*>(workspace);
  a.u = reinterpret_cast<float*>(ws + L.u);
  a.y = reinterpret_cast<float*>(ws + L.y);
  a.k = reinterpret_cast<float*>(ws + L.k);
  a.hs = reinterpret_cast<float*>(ws + L.hs);
  a.ftw = reinterpret_cast<float*>(ws + L.ftw);
  a.vw = reinterpret_cast<float*>(ws + L.vw);
  a.muw = reinterpret_cast<float*>(ws + L.muw);
  a.nomw = reinterpret_cast<float*>(ws + L.nomw);
  a.a1 = reinterpret_cast<float*>(ws + L.a1);
  a.a2 = reinterpret_cast<float*>(ws + L.a2);
  a.gz2 = reinterpret_cast<float*>(ws + L.gz2);
  a.gz1 = reinterpret_cast<float*>(ws + L.gz1);
  a.gft = reinterpret_cast<float*>(ws + L.gft);
  a.xslots = reinterpret_cast<unsigned long long*>(ws + L.xs);
  a.kw = reinterpret_cast<uint32_t*>(ws + L.kw);
#ifdef OT_PROFILE
  a.prof = reinterpret_cast<unsigned long long*>(ws + L.xs) + (size_t)a.E * 2 * ((a.B + 31) / 32) + 8;
#endif
  return FIODE_OK;
}

}  // namespace

extern "C" int32_t fiode_odetrain_evals(const fiode_odetrain_config* cfg) {
  if (!cfg) return -1;
  const int n = grid_iters(cfg);
  return n < 0 ? -1 : 4 * (n - 1);
}

extern "C" size_t fiode_odetrain_workspace_bytes(const fiode_odetrain_config* cfg) {
  if (!cfg || cfg->batch <= 0) return 0;
  const int n = grid_iters(cfg);
  if (n < 0) return 0;
  return ot_layout(cfg->batch, 4 * (n - 1)).total;
}

extern "C" int fiode_odetrain_saved_offsets(const fiode_odetrain_config* cfg, int64_t* offsets) {
  if (!cfg || !offsets || cfg->batch <= 0) return FIODE_EINVAL;
  const int n = grid_iters(cfg);
  if (n < 0) return FIODE_EINVAL;
  const OtLayout L = ot_layout(cfg->batch, 4 * (n - 1));
  const size_t o[8] = {L.hs, L.ftw, L.vw, L.muw, L.nomw, L.a1, L.a2, L.gft};
  for (int i = 0; i < 8; ++i) offsets[i] = (int64_t)o[i];
  return FIODE_OK;
}

extern "C" int fiode_odetrain_forward(void* stream, const fiode_odetrain_config* cfg, const fiode_dyn_config* dyn,
                                      const fiode_dyn_weights* w, const float* x_feat, const float* h0,
                                      const uint8_t* masks, const uint64_t* offset_dev, float* y_out, int32_t* stats,
                                      void* workspace, size_t workspace_bytes) {
  OTArgs a{};
  int rc = fill_args(a, cfg, dyn, w, x_feat, workspace, workspace_bytes);
  if (rc) return rc;
  if (!h0 || !y_out || !stats) return FIODE_EINVAL;
  if (a.dropout_mode == FIODE_DROPOUT_GIVEN && !masks) return FIODE_EINVAL;
  a.h0 = h0; a.masks = masks; a.offset_dev = offset_dev; a.y_out = y_out; a.stats = stats;
  hipStream_t st = static_cast<hipStream_t>(stream);
  const int ntiles = (a.B + 31) / 32;
  const size_t lds = (size_t)(M + 32) * LDQ * sizeof(float) + sizeof(OtShared);
  // zero the exchange granules (tags) and the status word before every launch
  FIODE_HIP_CHECK(hipMemsetAsync(a.xslots, 0, (size_t)a.E * 2 * ntiles * 8 + 256, st));
  FIODE_HIP_CHECK(hipMemsetAsync(stats, 0, 8 * sizeof(int32_t), st));
  if (a.dropout_mode != FIODE_DROPOUT_OFF) {
    hipLaunchKernelGGL(k_ot_masks, dim3((a.E * a.B + 255) / 256), dim3(256), 0, st, a);
    FIODE_HIP_CHECK(hipGetLastError());
  }
  hipLaunchKernelGGL(k_ot_fwd, dim3(ntiles), dim3(256), lds, st, a);
  FIODE_HIP_CHECK(hipGetLastError());
  return FIODE_OK;
}

extern "C" int fiode_odetrain_backward(void* stream, const fiode_odetrain_config* cfg, const fiode_dyn_config* dyn,
                                       const fiode_dyn_weights* w, const float* x_feat, const float* g_y,
                                       fiode_lyap_grads* grads, float* dbg_gft, void* workspace,
                                       size_t workspace_bytes) {
  OTArgs a{};
  int rc = fill_args(a, cfg, dyn, w, x_feat, workspace, workspace_bytes);
  if (rc) return rc;
  if (!g_y || !grads || !grads->Q1 || !grads->b1 || !grads->Qx || !grads->bx || !grads->Q2 || !grads->b2 ||
      !grads->Q3 || !grads->b3 || !grads->x_feat)
    return FIODE_EINVAL;
  a.g_y = g_y; a.dbg_gft = dbg_gft;
  hipStream_t st = static_cast<hipStream_t>(stream);
  const size_t lds = (size_t)(M + 32) * LDQ * sizeof(float) + sizeof(OtBwdShared);
  hipLaunchKernelGGL(k_ot_bwd, dim3((a.B + 31) / 32), dim3(256), lds, st, a);
  FIODE_HIP_CHECK(hipGetLastError());
  const OtLayout L = ot_layout(a.B, a.E);
  fiode_internal::WgradIO io{};
  io.B = a.B; io.S = a.E; io.x_feat = x_feat; io.Qx = w->Qx; io.h = a.hs; io.a1 = a.a1; io.a2 = a.a2;
  io.gz2 = a.gz2; io.gz1 = a.gz1; io.gft = a.gft;
  io.workspace = static_cast<char*>(workspace) + L.wg;
  io.grads = *grads;
  return fiode_internal::launch_wgrad(st, io);
}
