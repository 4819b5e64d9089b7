// Differentiable fixed-grid RK4 ODE solve of the Cayley-MLP dynamics (gfx950): the train_ode
// branch of LyapunovLearning.compute_loss (pl_modules.py:490-500):
//   y_hat = model(x, ts=linspace(0, t_max, 2), int_params={method: 'rk4', step_size}) in TRAIN
//   mode -> odeint(IVP.h_dot, (h0,), ts) (models.py:235-241) backpropagated through the stages
// (torchdiffeq 0.2.2 FixedGridODESolver + rk4_alt_step_func, the 3/8 rule; every func() call is
// eval_dot with fresh dropout masks and the QP's batch-global exit over the B rows).
//
// Forward  (k_ot_fwd, one persistent workgroup: each stage's QP exit is a batch-wide AND):
//   for each step, stage i = 1..4 (eval e = 4*step + i - 1):
//     Y_i = y + dt * sum_j beta_ij k_j      -> hs[b][e]        thread per element
//     MLP (MFMA wave tiles), a1/a2 saved    -> a1/a2[b][e], ft[b][e]
//     QP to the global exit                 -> k_i = v[b][e], mu[b][e]
//   y += (k1 + 3 (k2 + k3) + k4) dt / 8
// Backward (k_ot_bwd, one wave per 32 rows; rows never interact in the backward, so there are
//   no barriers): the reverse sweep of the 3/8 rule; every stage VJP is the QP backward
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

constexpr int OT_THREADS = 256;
constexpr int OT_WAVES = OT_THREADS / 64;

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
// forward: one eval (stage) over all B rows; stage input already in hs[:, e]
__device__ void ot_eval(const OTArgs& a, const Rng& rng, const float* Q2s, const float* Q3s,
                        const float (&q1)[4][5], int e, float* kout, uint32_t* word, int* last_exit) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, half = lane >> 5, col = lane & 31;
  const int ntiles = (a.B + 31) / 32;
  for (int tile = wave; tile < ntiles; tile += OT_WAVES) {
    const int b = tile * 32 + col;
    const bool valid = b < a.B;
    const int bb = valid ? b : a.B - 1;
    const size_t r = (size_t)bb * a.E + e;
    float h[C];
    load_row10(a.hs + r * C, h);
    uint32_t kw1[4], kw2[4];
    const uint8_t* m1 = a.dropout_mode == FIODE_DROPOUT_GIVEN ? a.masks + (((size_t)e * 2 + 0) * a.B + bb) * M : nullptr;
    const uint8_t* m2 = a.dropout_mode == FIODE_DROPOUT_GIVEN ? a.masks + (((size_t)e * 2 + 1) * a.B + bb) * M : nullptr;
    dropout_keep_words(a.dropout_mode, a.bit_mode, a.thr8, rng, m1, (uint32_t)bb,
                       RNG_STREAM_ODE_DROP + ((uint32_t)e << 5), kw1);
    dropout_keep_words(a.dropout_mode, a.bit_mode, a.thr8, rng, m2, (uint32_t)bb,
                       RNG_STREAM_ODE_DROP + ((uint32_t)e << 5) + 16u, kw2);
    f32x16 z1[4], z2[4];
    const f32x16 z3 = mlp_tile(Q2s, Q3s, q1, a.u + (size_t)bb * M, a.b2, a.b3, h, kw1, kw2, a.drop_scale, col, half,
                               z1, z2);
    float ft[C], lower[C], nominal[C], sig[C], span[C], v[C], mu;
    gather_ft(z3, half, ft);
    barrier_nominal(a.d, h, ft, lower, nominal, sig, span);
    uint32_t conv = qp_bisect(lower, nominal, a.d.max_iter - 1, a.d.tol, v, mu);
    if (!valid) conv = 0xFFFFFFFFu;
    conv = wave_and(conv);
    if (lane == 0) atomicAnd(word, conv);
    if (valid) {
#pragma unroll
      for (int mb = 0; mb < 4; ++mb) {
        store_acc_rows(a.a1 + r * M, mb, half, z1[mb]);
        store_acc_rows(a.a2 + r * M, mb, half, z2[mb]);
      }
      if (half == 0) store_row10(a.ftw + r * C, ft);
    }
  }
  __syncthreads();
  const int K = qp_exit_iter(*word, a.d.max_iter);
  for (int b = threadIdx.x; b < a.B; b += OT_THREADS) {
    const size_t r = (size_t)b * a.E + e;
    float h[C], ft[C], lower[C], nominal[C], sig[C], span[C], v[C], mu;
    load_row10(a.hs + r * C, h);
    load_row10(a.ftw + r * C, ft);
    barrier_nominal(a.d, h, ft, lower, nominal, sig, span);
    qp_bisect(lower, nominal, K, a.d.tol, v, mu);
    store_row10(a.vw + r * C, v);
    store_row10(a.nomw + r * C, nominal);
    a.muw[r] = mu;
    store_row10(kout + (size_t)b * C, v);
  }
  __syncthreads();              // every thread has read the word; k_i complete
  if (threadIdx.x == 0) {      // reset for the next eval (whose first atomicAnd follows the
    *last_exit = K;            // caller's stage-input barrier)
    *word = 0xFFFFFFFFu;
  }
}

__global__ __launch_bounds__(OT_THREADS) void k_ot_fwd(OTArgs a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* Q2s = smem;
  float* Q3s = smem + M * LDQ;
  uint32_t* word = reinterpret_cast<uint32_t*>(smem + (M + 32) * LDQ);
  int* last_exit = reinterpret_cast<int*>(word + 1);
  load_weight_images(a.Q2, a.Q3, Q2s, Q3s, false);
  if (threadIdx.x == 0) *word = 0xFFFFFFFFu;
  for (int e = threadIdx.x; e < a.B * M; e += OT_THREADS) {      // u[b] = U_x x_b + bx + b1
    const int b = e / M, i = e - b * M;
    float s = 0.f;
#pragma unroll
    for (int c = 0; c < FIODE_X; ++c) s = __fmaf_rn(a.Qx[i * FIODE_X + c], a.x_feat[(size_t)b * FIODE_X + c], s);
    a.u[e] = (s + a.bx[i]) + a.b1[i];
  }
  for (int e = threadIdx.x; e < a.B * C; e += OT_THREADS) a.y[e] = a.h0[e];
  __syncthreads();
  const Rng rng = rng_of(a);
  const int lane = threadIdx.x & 63, half = lane >> 5, col = lane & 31;
  float q1[4][5];
#pragma unroll
  for (int mb = 0; mb < 4; ++mb)
#pragma unroll
    for (int s = 0; s < 5; ++s) q1[mb][s] = a.Q1[(32 * mb + col) * C + 2 * s + half];
  const size_t BC = (size_t)a.B * C;
  float* k1 = a.k;
  float* k2 = a.k + BC;
  float* k3 = a.k + 2 * BC;
  float* k4 = a.k + 3 * BC;
  const float third = 1.0f / 3.0f;
  for (int it = 0; it + 1 < a.niters; ++it) {
    float ta, dt;
    step_times(a, it, ta, dt);
    const int e0 = 4 * it;
    for (int q = threadIdx.x; q < (int)BC; q += OT_THREADS) {
      const int b = q / C, j = q - b * C;
      a.hs[((size_t)b * a.E + e0) * C + j] = a.y[q];
    }
    __syncthreads();
    ot_eval(a, rng, Q2s, Q3s, q1, e0, k1, word, last_exit);
    for (int q = threadIdx.x; q < (int)BC; q += OT_THREADS) {
      const int b = q / C, j = q - b * C;
      a.hs[((size_t)b * a.E + e0 + 1) * C + j] = a.y[q] + (dt * k1[q]) * third;
    }
    __syncthreads();
    ot_eval(a, rng, Q2s, Q3s, q1, e0 + 1, k2, word, last_exit);
    for (int q = threadIdx.x; q < (int)BC; q += OT_THREADS) {
      const int b = q / C, j = q - b * C;
      a.hs[((size_t)b * a.E + e0 + 2) * C + j] = a.y[q] + dt * (k2[q] - k1[q] * third);
    }
    __syncthreads();
    ot_eval(a, rng, Q2s, Q3s, q1, e0 + 2, k3, word, last_exit);
    for (int q = threadIdx.x; q < (int)BC; q += OT_THREADS) {
      const int b = q / C, j = q - b * C;
      a.hs[((size_t)b * a.E + e0 + 3) * C + j] = a.y[q] + dt * ((k1[q] - k2[q]) + k3[q]);
    }
    __syncthreads();
    ot_eval(a, rng, Q2s, Q3s, q1, e0 + 3, k4, word, last_exit);
    for (int q = threadIdx.x; q < (int)BC; q += OT_THREADS) {
      const float dy = (((k1[q] + 3.0f * (k2[q] + k3[q])) + k4[q]) * dt) * 0.125f;
      a.y[q] = a.y[q] + dy;
    }
    __syncthreads();
  }
  for (int q = threadIdx.x; q < (int)BC; q += OT_THREADS) a.y_out[q] = a.y[q];
  if (threadIdx.x == 0) {
    a.stats[0] = 4 * (a.niters - 1);
    a.stats[1] = a.niters - 1;
    a.stats[2] = *last_exit;
  }
}

// ---------------------------------------------------------------------------------------------
// backward: VJP of one eval for the wave's 32 rows.  g: dL/dk (per lane, its row); returns
// dL/d(stage input) in gy_out.
__device__ void ot_vjp(const OTArgs& a, const float* Q2Ts, const float* Q1Ts, const float (&q3t)[4][5], int e,
                       int b, bool valid, int half, int col, const float (&g)[C], float (&gy_out)[C]) {
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
  if (valid && half == 0) {
    store_row10(a.gft + r * C, gft);
    if (a.dbg_gft) store_row10(a.dbg_gft + r * C, gft);
  }
  // g_a2^T = Q3^T g_ft^T, masked by the saved post-activation a2 (> 0 <=> kept and positive)
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
    if (valid) store_acc_rows(a.gz2 + r * M, mb, half, ga[mb]);
  }
  // g_a1^T = Q2^T g_z2^T
  f32x16 gb[4];
#pragma unroll
  for (int mb = 0; mb < 4; ++mb) gb[mb] = f16_zero();
#pragma unroll
  for (int kb = 0; kb < 4; ++kb) {
#pragma unroll
    for (int gg = 0; gg < 4; ++gg)
#pragma unroll
      for (int mb = 0; mb < 4; ++mb) {
        const f32x4 q = *reinterpret_cast<const f32x4*>(Q2Ts + (32 * mb + col) * LDQ + 32 * kb + 8 * gg + 4 * half);
#pragma unroll
        for (int t = 0; t < 4; ++t) gb[mb] = mfma32(q[t], ga[kb][4 * gg + t], gb[mb]);
      }
    __builtin_amdgcn_sched_barrier(0);
  }
#pragma unroll
  for (int mb = 0; mb < 4; ++mb) {
    f32x16 act;
    load_acc_rows(a.a1 + r * M, mb, half, act);
#pragma unroll
    for (int q = 0; q < 16; ++q) gb[mb][q] = act[q] > 0.f ? gb[mb][q] * a.drop_scale : 0.f;
    if (valid) store_acc_rows(a.gz1 + r * M, mb, half, gb[mb]);
  }
  // g_h^T (10 x 32, padded to 32 rows) = Q1^T g_z1^T
  f32x16 gh = f16_zero();
#pragma unroll
  for (int kb = 0; kb < 4; ++kb)
#pragma unroll
    for (int gg = 0; gg < 4; ++gg) {
      const f32x4 q = *reinterpret_cast<const f32x4*>(Q1Ts + col * LDQ + 32 * kb + 8 * gg + 4 * half);
#pragma unroll
      for (int t = 0; t < 4; ++t) gh = mfma32(q[t], gb[kb][4 * gg + t], gh);
    }
  float ghm[C];
  gather_ft(gh, half, ghm);
#pragma unroll
  for (int j = 0; j < C; ++j) gy_out[j] = ghm[j] + ghb[j];
}

__global__ __launch_bounds__(64) void k_ot_bwd(OTArgs a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* Q2Ts = smem;                 // Q2^T image [128][LDQ]
  float* Q1Ts = smem + M * LDQ;       // Q1^T image [32][LDQ] (rows >= 10 zero)
  load_weight_images(a.Q2, nullptr, Q2Ts, nullptr, true);
  for (int q = threadIdx.x; q < 32 * M; q += blockDim.x) {
    const int c = q >> 7, i = q & 127;
    Q1Ts[c * LDQ + i] = c < C ? a.Q1[i * C + c] : 0.f;
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, half = lane >> 5, col = lane & 31;
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
    ot_vjp(a, Q2Ts, Q1Ts, q3t, e0 + 3, b, valid, half, col, gk4, gY);   // Y4 = y + dt (k1 - k2 + k3)
#pragma unroll
    for (int j = 0; j < C; ++j) {
      acc[j] += gY[j];
      const float d = dt * gY[j];
      gk1[j] += d;
      gk2[j] -= d;
      gk3[j] += d;
    }
    ot_vjp(a, Q2Ts, Q1Ts, q3t, e0 + 2, b, valid, half, col, gk3, gY);   // Y3 = y + dt (k2 - k1/3)
#pragma unroll
    for (int j = 0; j < C; ++j) {
      acc[j] += gY[j];
      const float d = dt * gY[j];
      gk2[j] += d;
      gk1[j] -= d * third;
    }
    ot_vjp(a, Q2Ts, Q1Ts, q3t, e0 + 1, b, valid, half, col, gk2, gY);   // Y2 = y + (dt k1) / 3
#pragma unroll
    for (int j = 0; j < C; ++j) {
      acc[j] += gY[j];
      gk1[j] += (dt * gY[j]) * third;
    }
    ot_vjp(a, Q2Ts, Q1Ts, q3t, e0, b, valid, half, col, gk1, gY);       // Y1 = y
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
  size_t u, y, k, hs, ftw, vw, muw, nomw, a1, a2, gz2, gz1, gft, wg, total;
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
  const size_t lds = (size_t)(M + 32) * LDQ * sizeof(float) + 16;
  hipLaunchKernelGGL(k_ot_fwd, dim3(1), dim3(OT_THREADS), lds, st, a);
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
  const size_t lds = (size_t)(M + 32) * LDQ * sizeof(float);
  hipLaunchKernelGGL(k_ot_bwd, dim3((a.B + 31) / 32), dim3(64), lds, st, a);
  FIODE_HIP_CHECK(hipGetLastError());
  const OtLayout L = ot_layout(a.B, a.E);
  fiode_internal::WgradIO io{};
  io.B = a.B; io.S = a.E; io.x_feat = x_feat; io.Qx = w->Qx; io.h = a.hs; io.a1 = a.a1; io.a2 = a.a2;
  io.gz2 = a.gz2; io.gz1 = a.gz1; io.gft = a.gft;
  io.workspace = static_cast<char*>(workspace) + L.wg;
  io.grads = *grads;
  return fiode_internal::launch_wgrad(st, io);
}
