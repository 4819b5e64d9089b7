// Differentiable fixed-grid RK4 ODE solve of the Cayley-MLP dynamics (gfx950): the train_ode
// branch of LyapunovLearning.compute_loss (pl_modules.py:490-500):
//   y_hat = model(x, ts=linspace(0, t_max, 2), int_params={method: 'rk4', step_size}) in TRAIN
//   mode -> odeint(IVP.h_dot, (h0,), ts) (models.py:235-241) backpropagated through the stages
// (torchdiffeq 0.2.2 FixedGridODESolver + rk4_alt_step_func, the 3/8 rule; every func() call is
// eval_dot with fresh dropout masks and the QP's batch-global exit over the B rows).
//
// Forward  (k_ot_fwd, one persistent workgroup per 16-row tile, all tiles co-resident; each
//   stage's QP exit is a batch-wide AND exchanged through tagged granules, see below):
//   for each step, stage i = 1..4 (eval e = 4*step + i - 1), per row in registers:
//     Y_i = y + dt * sum_j beta_ij k_j      -> hs[b][e]
//     MLP (MFMA, hidden split over 4 waves), a1/a2 saved -> a1/a2[b][e], ft[b][e]
//     QP bisection recording mu per iteration; exit K from all tiles; k_i = v(mu_K)
//   y += (k1 + 3 (k2 + k3) + k4) dt / 8
// Backward (k_ot_bwd, one workgroup per 16 rows; rows never interact in the backward, so tiles
//   need no grid-wide synchronisation): the reverse sweep of the 3/8 rule; every stage VJP is the QP backward
//   (closed form), the sigmoid rescale, the barrier bounds' h-dependence, and the MLP input
//   gradients (Q3^T, Q2^T via LDS images, Q1^T via a zero-padded LDS image), writing the per-
//   (row, eval) activation gradients gft / gz2 / gz1.
// Weight gradients: the training step's wgrad chain over rows r = b*E + e (wgrad.h).
#include <type_traits>
#include "common.h"
#include "tile.h"
#include "tile16.h"
#include "tile4.h"
#include "wgrad.h"
#include "dopri5.h"
#include "../../include/fiode.h"

namespace {
using namespace fiode_tile;
using namespace fiode_t16;
using namespace fiode_t4;
using namespace fiode_dp;


// Ring of exit-exchange granule sets: eval e publishes into set e % OT_XRING with tag e + 1.  A tile
// publishes eval e + 2 only after every tile published e + 1, and every tile publishes e + 1 only
// after all its waves finished reading eval e's granules (the next eval's layer-1 barrier), so a
// set is never overwritten while it is read; 4 sets leave a margin.  The cleared region no longer
// grows with the eval count (dopri5: the attempt capacity).
constexpr int OT_XRING = 4;
constexpr int FIODE_OT_KW_PRE = 256;      // dopri5: evals whose keep words k_ot_masks draws ahead

struct OTArgs {
  int prio;                 // g_fiode_prio_mask at launch (common.h)
  int B, E, niters;
  int nslots;               // u64 words of xslots zeroed by k_ot_masks before the forward
  int kw_lazy;              // dopri5, Philox p = 0.5: the forward draws the keep words of evals >= kw_pre
                            // itself (and stores them for the backward) instead of k_ot_masks drawing
                            // the whole eval capacity up front
  int kw_pre;               // evals whose keep words k_ot_masks draws (E unless kw_lazy)
  float t0, t1, hstep;
  int dropout_mode, bit_mode;
  uint32_t thr8;
  float drop_scale;
  Rng rng;
  const uint64_t* offset_dev;
  int drop_block;           // test hook: workgroup that skips its first exit publish (-1: none)
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
  float* loww;              // [B][E][C] QP lower bound (for checkers)
  float* a1;                // [B][E][M]
  float* a2;                // [B][E][M]
  float* gz2;               // [B][E][M]
  float* gz1;               // [B][E][M]
  float* gft;               // [B][E][C]
  unsigned long long* xslots;  // [OT_XRING][2 phases][ntiles] {epoch, mask} granules of the QP exit exchange
                               // (eval e uses ring slot e % OT_XRING, tagged e + 1)
  uint32_t* kw;                // [E][2][B] uint4 dropout keep words
#ifdef OT_PROFILE
  unsigned long long* prof;    // [9] wall-clock ticks per phase (workgroup 0, lane 0); [16 + e] eval e's exit K
#endif
  // dopri5 (method FIODE_ODE_DOPRI5): E = 2 + 6 A is the eval capacity, the solve's own count is in imeta
  int method, A;
  double rtol, atol, t0d, t1d;
  float* ys;                   // [A][B][C] the state y_n attempt n starts from
  double* alog;                // [A][ALOG_W] per attempt (ALOG_*)
  double* meta;                // [META_N] initial-step scalars (META_*)
  int32_t* imeta;              // [8]: nfe, attempts, status (read by the backward and the weight chain)
  unsigned long long* xr;      // [2 parities][ntiles][2 OT_XV] float64 reduction granules
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
// forward: one workgroup per 16-row tile, persistent over all evals; 4 waves = 4 parts of the
// hidden dimension.  Per eval every wave computes layer 1 in full (24 MFMA), its 32 of the 128
// layer-2 outputs (64 MFMA) and their layer-3 partial (8 MFMA); the partials meet in LDS and
// every lane sums its sample's 10 outputs over the parts in the same order, so the row state
// (y, k1..k4, the QP) is replicated in all waves and needs no further exchange.  The QP's
// per-iteration convergence over the tile is a wave ballot (no cross-lane shuffles).  The only
// cross-tile coupling -- the QP's exit iteration, the lowest bit of the AND over ALL rows of the
// per-iteration convergence masks -- is exchanged through per-eval {tag, mask} granules: each
// workgroup publishes its mask with ONE agent-scope 64-bit atomic store, then one wave sweeps the
// ntiles granules of that eval until every tag matches (relaxed agent-scope loads; the granule
// IS the flag, so no fence is needed).  The spin is bounded: on timeout the status word records
// it and the solve completes.
#ifndef OT_SHARE_L1
#define OT_SHARE_L1 1         // layer 1 split over the 4 waves (LDS exchange) instead of replicated
#endif
struct OtShared {
  float zpart[4][64][4];      // [part][lane][layer-3 accumulator registers]
  float mu_rec[4][48][33];    // [wave][row j < 16][bisection iteration] (the row's lanes of the wave share it);
                              // [wave][32 + j][0..1]: the tree bisection's bracket hand-over
  float z1x[8][64][4];        // layer-1 blocks, one pair per wave (mlp16_part)
  int K;
  int Kprev;                  // previous eval's exit iteration (speculation for the next)
  int dead;                   // an exit exchange timed out (status 4): stop waiting, poison y_out
  int pad;
};

#ifdef OT_PROFILE
#define OT_MARK(i) do { const uint64_t t_ = wall_clock64(); if (blockIdx.x == 0 && threadIdx.x == 0) \
    atomicAdd((unsigned long long*)&a.prof[i], (unsigned long long)(t_ - t_prev)); t_prev = t_; } while (0)
#else
#define OT_MARK(i) do { } while (0)
#endif

// one eval for this workgroup's tile: stage input h (per lane, its row) -> k (per lane)
__device__ void ot_eval(const OTArgs& a, const T16W& w, OtShared& sh, int e, int p, int b, bool valid, int lane, int q,
                        int j, const f32x4v (&uacc)[8], const uint32_t (&kw1)[4], uint32_t kw2p, const float (&h)[C],
                        float (&k)[C]) {
  const int bb = valid ? b : a.B - 1;
  const size_t r = (size_t)bb * a.E + e;
#ifdef OT_PROFILE
  uint64_t t_prev = wall_clock64();
#endif
  if (p == 0 && valid && q == 0) store_row10(a.hs + r * C, h);
  // the barrier's lower bound depends on h only: interleaved with the MLP's 96 MFMAs (explicit
  // issue groups in one scheduling region), so its exp VALU work leaves the critical path
  // (same float32 expressions as barrier_nominal, common.h)
  float lower[C];
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int i = 0; i < C; ++i) {
    lower[i] = -a.d.alpha_1 * (expf(a.d.sigma_1 * h[i]) - 1.0f);
    asm volatile("" ::"v"(lower[i]));          // keep it here (IR passes would sink it to its use)
  }
  mlp16_part<OT_SHARE_L1 != 0>(w, uacc, h, kw1, kw2p, a.drop_scale, p, q, valid ? a.a1 + r * M : nullptr,
                               valid ? a.a2 + r * M : nullptr, &sh.zpart[p][lane][0], sh.z1x);
#pragma unroll
  for (int i = 0; i < (OT_SHARE_L1 ? 78 : 96); ++i) {
    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);     // one MFMA
    __builtin_amdgcn_sched_group_barrier(0x002, 3, 0);     // then up to three VALU
  }
  __builtin_amdgcn_sched_barrier(0);
  OT_MARK(1);
  __syncthreads();
  float ft[C];
  ft16_sum(sh.zpart, j, ft);
  float nominal[C];
#pragma unroll
  for (int i = 0; i < C; ++i) {
    const float upper = a.d.alpha_2 * (1.0f - h[i]);
    const float span = upper - lower[i];
    if (a.d.scale_nominal) {
      const float sig = 1.0f / (1.0f + expf(-ft[i]));
      nominal[i] = span * sig + lower[i];
    } else {
      nominal[i] = ft[i];
    }
  }
  OT_MARK(5);
  float* rec = &sh.mu_rec[p][j][0];
  qp16_exit<TR>(lower, nominal, a.d.tol, a.d.max_iter, sh.Kprev, valid, p, q, lane, rec, &sh.mu_rec[p][32 + j][0],
            a.xslots + (size_t)(e % OT_XRING) * 2 * gridDim.x, (unsigned)e + 1u, a.stats + 3, sh.K, sh.dead,
            a.drop_block,
#ifdef OT_PROFILE
            a.prof
#else
            nullptr
#endif
  );
  OT_MARK(3);
  const int K = sh.K;
  const float mu = rec[K];
#pragma unroll
  for (int i = 0; i < C; ++i) k[i] = fmaxf(nominal[i] - mu, lower[i]);
  if (p == 0 && valid && q == 0) {
    store_row10(a.ftw + r * C, ft);
    store_row10(a.nomw + r * C, nominal);
    store_row10(a.loww + r * C, lower);
    store_row10(a.vw + r * C, k);
    a.muw[r] = mu;
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) a.stats[2] = K;
#ifdef OT_PROFILE
  if (blockIdx.x == 0 && threadIdx.x == 0 && e < 96) a.prof[16 + e] = (unsigned long long)K;
#endif
  if (threadIdx.x == 0) sh.Kprev = K;
  __syncthreads();            // zpart / mu_rec / K reused by the next eval
  OT_MARK(4);
}

// dropout keep words of every (eval, set, row): kw[e][set][b] (uint4 = the 4 words of the 128 units)
// Also clears the exit-exchange granules (tags) and the status words the forward uses (one launch
// instead of two memsets ahead of it on the critical path).
__global__ __launch_bounds__(256) void k_ot_masks(OTArgs a) {
  const int q = blockIdx.x * blockDim.x + threadIdx.x;
  if (q < a.nslots) a.xslots[q] = 0ull;
  if (q < 8) a.stats[q] = 0;
  if (q < 8) a.imeta[q] = 0;       // the solve's status word (saved [12]) and the dopri5 counters
  if (a.dropout_mode == FIODE_DROPOUT_OFF || q >= a.kw_pre * a.B) return;
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
  OtShared& sh = *reinterpret_cast<OtShared*>(smem);
  if (threadIdx.x == 0) {
    sh.Kprev = a.d.max_iter - 1;
    sh.dead = 0;
  }
  const int lane = threadIdx.x & 63, q = lane >> 4, j = lane & 15;
  const int p = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int b = blockIdx.x * TR + j;
  const bool valid = b < a.B;
  const int bb = valid ? b : a.B - 1;
  T16W w;                     // this wave's weight operands, in registers for the whole solve
  load_t16w(a.Q1, a.Q2, M, a.Q3, M, a.b2, a.b3, p, q, j, w);
  // u[b] = U_x x_b + bx + b1 for this tile's rows
  for (int t = threadIdx.x; t < TR * M; t += blockDim.x) {
    const int rb = blockIdx.x * TR + t / M, i = t % M;
    if (rb < a.B) {
      float s = 0.f;
#pragma unroll
      for (int c = 0; c < FIODE_X; ++c) s = __fmaf_rn(a.Qx[i * FIODE_X + c], a.x_feat[(size_t)rb * FIODE_X + c], s);
      a.u[(size_t)rb * M + i] = (s + a.bx[i]) + a.b1[i];
    }
  }
  __syncthreads();
  f32x4v uacc[8];
#pragma unroll
  for (int hb = 0; hb < 8; ++hb) {
    const f32x4 uv = *reinterpret_cast<const f32x4*>(a.u + (size_t)bb * M + 16 * hb + 4 * q);
    uacc[hb] = f32x4v{uv[0], uv[1], uv[2], uv[3]};
  }
  // dropout keep words of eval e (k_ot_masks), prefetched one eval ahead
  const uint4* kwp = reinterpret_cast<const uint4*>(a.kw);
  auto fetch = [&](int e, uint32_t (&w1)[4], uint32_t& w2) {
    if (a.dropout_mode == FIODE_DROPOUT_OFF) {
#pragma unroll
      for (int t = 0; t < 4; ++t) w1[t] = 0xFFFFFFFFu;
      w2 = 0xFFFFFFFFu;
      return;
    }
    const uint4 q1 = kwp[((size_t)e * 2 + 0) * a.B + bb];
    w1[0] = q1.x; w1[1] = q1.y; w1[2] = q1.z; w1[3] = q1.w;
    w2 = reinterpret_cast<const uint32_t*>(kwp + ((size_t)e * 2 + 1) * a.B + bb)[p];   // layer-2 word of part p
  };
  uint32_t kc1[4], kc2, kn1[4], kn2;
  fetch(0, kc1, kc2);
  float y[C], k1[C], k2[C], k3[C], k4[C], hin[C];
  load_row10(a.h0 + (size_t)bb * C, y);
  const float third = 1.0f / 3.0f;
  const int eN = 4 * (a.niters - 1);
  for (int it = 0; it + 1 < a.niters; ++it) {
    float ta, dt;
    step_times(a, it, ta, dt);
    const int e0 = 4 * it;
#define OT_STAGE(E_, H_, K_)                                                             \
    {                                                                                    \
      if ((E_) + 1 < eN) fetch((E_) + 1, kn1, kn2);                                      \
      ot_eval(a, w, sh, (E_), p, b, valid, lane, q, j, uacc, kc1, kc2, H_, K_);     \
      _Pragma("unroll") for (int t = 0; t < 4; ++t) kc1[t] = kn1[t];                   \
      kc2 = kn2;                                                                         \
    }
    OT_STAGE(e0, y, k1)
#pragma unroll
    for (int i = 0; i < C; ++i) hin[i] = y[i] + (dt * k1[i]) * third;
    OT_STAGE(e0 + 1, hin, k2)
#pragma unroll
    for (int i = 0; i < C; ++i) hin[i] = y[i] + dt * (k2[i] - k1[i] * third);
    OT_STAGE(e0 + 2, hin, k3)
#pragma unroll
    for (int i = 0; i < C; ++i) hin[i] = y[i] + dt * ((k1[i] - k2[i]) + k3[i]);
    OT_STAGE(e0 + 3, hin, k4)
#undef OT_STAGE
#pragma unroll
    for (int i = 0; i < C; ++i) {
      const float dy = (((k1[i] + 3.0f * (k2[i] + k3[i])) + k4[i]) * dt) * 0.125f;
      y[i] = y[i] + dy;
    }
  }
  if (sh.dead) {              // this tile's QP exits came from a partial AND: make the loss NaN
#pragma unroll
    for (int i = 0; i < C; ++i) y[i] = __builtin_nanf("");
  }
  if (p == 0 && valid && q == 0) store_row10(a.y_out + (size_t)b * C, y);
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    a.stats[0] = 4 * (a.niters - 1);
    a.stats[1] = a.niters - 1;
  }
}

// ---------------------------------------------------------------------------------------------
// forward on 4-row tiles (tile4.h) for B <= 4 * FIODE_OT4_MAX_TILES: the same solve, the same
// exchanges and saved arrays as k_ot_fwd; per eval every wave issues the 4x4x1 MFMAs of its
// quarter of the hidden units for 4 samples (77 MFMAs of 8 cycles) instead of the 16x16x4
// products of 16 samples (78 of 32 cycles), on 4x as many workgroups.  The MLP's sums run in
// another order than the 16-row kernel's (both within float32 rounding of the oracle's).
constexpr int FIODE_OT4_MAX_TILES = 256;     // one persistent workgroup per CU at most
constexpr int OT4_XSTRIDE = 16;              // u64 words per exit granule: one 128-byte line per tile
struct OtShared4 {
  Mlp4Shared mlp;
  float mu_rec[4][48][33];    // [wave][row j < 16][bisection iteration] (the row's lanes of the wave share it);
                              // [wave][32 + j][0..1]: the tree bisection's bracket hand-over
  int K;
  int Kprev;
  int dead;
  int pad;
};

// end_barrier: the trailing workgroup barrier, which k_ot_fwd4 leaves out -- every LDS word this
// eval reads is either written by its own wave (mu_rec) or is next written only behind a barrier of the next
// eval that every wave reaches after its last read here: a1s / zpart behind the next layer-1
// barrier, K / Kprev by lane 0 of wave 0 behind it too, a2s by the owning wave only.  The dopri5
// solve keeps it (its caller shares the workgroup's LDS between evals).
__device__ void ot_eval4(const OTArgs& a, const T4W& w, OtShared4& sh, int e, int p, int b, bool valid, int lane,
                         int j, const f32x4& uacc, uint32_t kw1p, uint32_t kw2p, const float (&h)[C], float (&k)[C],
                         bool end_barrier = true) {
  const int bb = valid ? b : a.B - 1;
  const size_t r = (size_t)bb * a.E + e;
  const bool writer = p == 0 && valid && lane < TR4;     // lane j of wave 0 stores sample j's rows
#ifdef OT_PROFILE
  uint64_t t_prev = wall_clock64();
#endif
  if (writer) store_row10(a.hs + r * C, h);
  float lower[C];
#pragma unroll
  for (int i = 0; i < C; ++i) lower[i] = -a.d.alpha_1 * (expf(a.d.sigma_1 * h[i]) - 1.0f);
  mlp4_part(w, uacc, h, kw1p, kw2p, a.drop_scale, p, lane, valid ? a.a1 + r * M : nullptr,
            valid ? a.a2 + r * M : nullptr, sh.mlp);
  OT_MARK(1);
  __syncthreads();
  float ft[C];
  ft4_sum(sh.mlp, j, ft);
  float nominal[C];
#pragma unroll
  for (int i = 0; i < C; ++i) {
    const float upper = a.d.alpha_2 * (1.0f - h[i]);
    const float span = upper - lower[i];
    if (a.d.scale_nominal) {
      const float sig = 1.0f / (1.0f + expf(-ft[i]));
      nominal[i] = span * sig + lower[i];
    } else {
      nominal[i] = ft[i];
    }
  }
  OT_MARK(5);
  float* rec = &sh.mu_rec[p][j][0];
  const int K = qp16_exit<TR4>(lower, nominal, a.d.tol, a.d.max_iter, sh.Kprev, valid, p, 0, lane, rec,
            &sh.mu_rec[p][32 + j][0],
            a.xslots + (size_t)(e % OT_XRING) * 2 * gridDim.x * OT4_XSTRIDE, (unsigned)e + 1u, a.stats + 3, sh.K,
            sh.dead,
            a.drop_block,
#ifdef OT_PROFILE
            a.prof,
#else
            nullptr,
#endif
            OT4_XSTRIDE, gridDim.x <= 64);
  OT_MARK(3);
  const float mu = rec[K];
#pragma unroll
  for (int i = 0; i < C; ++i) k[i] = fmaxf(nominal[i] - mu, lower[i]);
  if (writer) {
    store_row10(a.ftw + r * C, ft);
    store_row10(a.nomw + r * C, nominal);
    store_row10(a.loww + r * C, lower);
    store_row10(a.vw + r * C, k);
    a.muw[r] = mu;
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) a.stats[2] = K;
#ifdef OT_PROFILE
  if (blockIdx.x == 0 && threadIdx.x == 0 && e < 96) a.prof[16 + e] = (unsigned long long)K;
#endif
  if (threadIdx.x == 0) sh.Kprev = K;
  if (end_barrier) __syncthreads();            // (uniform)
  OT_MARK(4);
}

__global__ __launch_bounds__(256) void k_ot_fwd4(OTArgs a) {
  fiode_wave_prio(a.prio & 1);
  extern __shared__ __attribute__((aligned(16))) float smem[];
  OtShared4& sh = *reinterpret_cast<OtShared4*>(smem);
  if (threadIdx.x == 0) {
    sh.Kprev = a.d.max_iter - 1;
    sh.dead = 0;
  }
  const int lane = threadIdx.x & 63, j = lane & 3;
  const int p = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int b = blockIdx.x * TR4 + j;
  const bool valid = b < a.B;
  const int bb = valid ? b : a.B - 1;
  T4W w;                      // this wave's weight operands, in registers for the whole solve
  load_t4w(a.Q1, a.Q2, a.Q3, a.b2, a.b3, p, lane, w);
  // u[b] = U_x x_b + bx + b1 for this tile's rows
  for (int t = threadIdx.x; t < TR4 * M; t += blockDim.x) {
    const int rb = blockIdx.x * TR4 + t / M, i = t % M;
    if (rb < a.B) {
      float s = 0.f;
#pragma unroll
      for (int c = 0; c < FIODE_X; ++c) s = __fmaf_rn(a.Qx[i * FIODE_X + c], a.x_feat[(size_t)rb * FIODE_X + c], s);
      a.u[(size_t)rb * M + i] = (s + a.bx[i]) + a.b1[i];
    }
  }
  __syncthreads();
  const f32x4 uacc = *reinterpret_cast<const f32x4*>(a.u + (size_t)bb * M + 32 * p + 4 * ((lane >> 2) & 7));
  // this part's keep words of eval e (k_ot_masks), prefetched one eval ahead
  const uint32_t* kwp = a.kw;
  auto fetch = [&](int e, uint32_t& w1, uint32_t& w2) {
    if (a.dropout_mode == FIODE_DROPOUT_OFF) {
      w1 = w2 = 0xFFFFFFFFu;
      return;
    }
    w1 = kwp[(((size_t)e * 2 + 0) * a.B + bb) * 4 + p];
    w2 = kwp[(((size_t)e * 2 + 1) * a.B + bb) * 4 + p];
  };
  uint32_t kc1, kc2, kn1 = 0u, kn2 = 0u;
  fetch(0, kc1, kc2);
  float y[C], k1[C], k2[C], k3[C], k4[C], hin[C];
  load_row10(a.h0 + (size_t)bb * C, y);
  const float third = 1.0f / 3.0f;
  const int eN = 4 * (a.niters - 1);
  for (int it = 0; it + 1 < a.niters; ++it) {
    float ta, dt;
    step_times(a, it, ta, dt);
    const int e0 = 4 * it;
#define OT4_STAGE(E_, H_, K_)                                                            \
    {                                                                                    \
      if ((E_) + 1 < eN) fetch((E_) + 1, kn1, kn2);                                      \
      ot_eval4(a, w, sh, (E_), p, b, valid, lane, j, uacc, kc1, kc2, H_, K_, false);    \
      kc1 = kn1;                                                                         \
      kc2 = kn2;                                                                         \
    }
    OT4_STAGE(e0, y, k1)
#pragma unroll
    for (int i = 0; i < C; ++i) hin[i] = y[i] + (dt * k1[i]) * third;
    OT4_STAGE(e0 + 1, hin, k2)
#pragma unroll
    for (int i = 0; i < C; ++i) hin[i] = y[i] + dt * (k2[i] - k1[i] * third);
    OT4_STAGE(e0 + 2, hin, k3)
#pragma unroll
    for (int i = 0; i < C; ++i) hin[i] = y[i] + dt * ((k1[i] - k2[i]) + k3[i]);
    OT4_STAGE(e0 + 3, hin, k4)
#undef OT4_STAGE
#pragma unroll
    for (int i = 0; i < C; ++i) {
      const float dy = (((k1[i] + 3.0f * (k2[i] + k3[i])) + k4[i]) * dt) * 0.125f;
      y[i] = y[i] + dy;
    }
  }
  if (sh.dead) {              // this tile's QP exits came from a partial AND: make the loss NaN
#pragma unroll
    for (int i = 0; i < C; ++i) y[i] = __builtin_nanf("");
  }
  if (p == 0 && valid && lane < TR4) store_row10(a.y_out + (size_t)b * C, y);
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    a.stats[0] = 4 * (a.niters - 1);
    a.stats[1] = a.niters - 1;
  }
}

// ---------------------------------------------------------------------------------------------
// backward: one workgroup per 16-row tile, 4 waves = 4 parts of the hidden dimension.  Every
// wave runs the row math (QP backward, rescale, barrier terms) and g_a2 = Q3^T g_ft in full
// (identical values in all waves), then its 32 of the 128 rows of g_a1 = Q2^T g_z2 (64 MFMA)
// and their Q1^T partial (8 MFMA); the 4 partials of g_h meet in LDS (double-buffered, one
// barrier per VJP) and every lane sums its sample's 10 values in the same order, so the adjoint
// state stays replicated.
struct OtBwdShared {
  float gpart[2][4][64][4];
  float gax[8][64][4];        // g_z2 blocks, one pair per wave (each wave computes its own two)
};

// The saved forward values one VJP reads (independent of the adjoint): loaded one VJP ahead, so
// their global-memory latency overlaps the previous VJP's dependent chain.
struct VjpIn {
  float h[C], ft[C], v[C], mu;
  f32x4 a2[2];        // saved post-activations of layer 2, hidden blocks 2p, 2p+1 (this lane's 4 of each)
  f32x4 a1[2];        // layer 1, hidden blocks 2p, 2p+1
};

__device__ __forceinline__ void load_vjp_in(const OTArgs& a, int p, int e, int b, bool valid, int q, VjpIn& in) {
  const int bb = valid ? b : a.B - 1;
  const size_t r = (size_t)bb * a.E + (e < 0 ? 0 : e);
  load_row10(a.hs + r * C, in.h);
  load_row10(a.ftw + r * C, in.ft);
  load_row10(a.vw + r * C, in.v);
  in.mu = a.muw[r];
#pragma unroll
  for (int o = 0; o < 2; ++o) in.a2[o] = *reinterpret_cast<const f32x4*>(a.a2 + r * M + 16 * (2 * p + o) + 4 * q);
#pragma unroll
  for (int o = 0; o < 2; ++o) in.a1[o] = *reinterpret_cast<const f32x4*>(a.a1 + r * M + 16 * (2 * p + o) + 4 * q);
}

// The backward's weight operands of one wave (part p), in registers for the whole kernel: q2t[o][hb]
// = Q2^T[16 (2p + o) + j][16 hb + 4q ..] = Q2[16 hb + 4q + t][16 (2p + o) + j]; q1t[o] =
// Q1^T[j][16 (2p + o) + 4q ..] (0 for j >= C).
struct VjpW {
  f32x4 q2t[2][8];
  f32x4 q1t[2];
};

// The adjoint-independent row math of one VJP (barrier terms of the saved stage input and MLP
// output): computed for the NEXT VJP inside the current one, between its MFMA chains, so the
// exp / sigmoid VALU work leaves the adjoint's dependent chain.
struct VjpRow {
  float nominal[C], sig[C], span[C], es[C];     // es = exp(sigma_1 h)
};
template <bool SN, class In>
__device__ __forceinline__ void vjp_row_math(const OTArgs& a, const In& in, VjpRow& rw) {
  // the expressions of barrier_nominal (common.h), branch-free for a compile-time scale_nominal
#pragma unroll
  for (int i = 0; i < C; ++i) {
    rw.es[i] = expf(a.d.sigma_1 * in.h[i]);
    const float lower = -a.d.alpha_1 * (rw.es[i] - 1.0f);
    const float upper = a.d.alpha_2 * (1.0f - in.h[i]);
    rw.span[i] = upper - lower;
    if constexpr (SN) {
      rw.sig[i] = 1.0f / (1.0f + expf(-in.ft[i]));
      rw.nominal[i] = rw.span[i] * rw.sig[i] + lower;
    } else {
      rw.sig[i] = 0.f;
      rw.nominal[i] = in.ft[i];
    }
  }
}

// g_z2 blocks 2P, 2P+1 of one VJP: Q3^T g_ft, masked by the saved a2 and the dropout scale;
// stored to gz2 (nullable row) and to the LDS exchange.
template <int P>
__device__ __forceinline__ void gz2_pair(const OTArgs& a, const float (&q3t)[8][3], const float (&gft)[C],
                                         const VjpIn& in, int q, int lane, float* gz2row, float (*gax)[64][4]) {
#pragma unroll
  for (int o = 0; o < 2; ++o) {
    constexpr int hb0 = 2 * P;
    f32x4v g = z4();
#pragma unroll
    for (int s = 0; s < 3; ++s) g = mfma16(q3t[hb0 + o][s], sel4(gft, s, q), g);
    const f32x4 act = in.a2[o];
#pragma unroll
    for (int t = 0; t < 4; ++t) g[t] = act[t] > 0.f ? g[t] * a.drop_scale : 0.f;
    if (gz2row) *reinterpret_cast<f32x4*>(gz2row + 16 * (hb0 + o) + 4 * q) = f32x4{g[0], g[1], g[2], g[3]};
    *reinterpret_cast<f32x4*>(&gax[hb0 + o][lane][0]) = f32x4{g[0], g[1], g[2], g[3]};
  }
}

template <bool SN>
__device__ void ot_vjp(const OTArgs& a, const VjpW& wv, const float (&q3t)[8][3],
                       OtBwdShared& sh, int buf, int p, int e, int b, bool valid, int lane, int q, int j,
                       const VjpIn& in, const VjpRow& rw, const VjpIn& nin, VjpRow& nrw, const float (&g)[C],
                       float (&gy_out)[C]) {
  const int bb = valid ? b : a.B - 1;
  const size_t r = (size_t)bb * a.E + e;
#ifdef OT_PROFILE
  uint64_t t_prev = wall_clock64();
#endif
  float g_nom[C], g_low[C], gft[C], ghb[C];
  float gin[C];
#pragma unroll
  for (int i = 0; i < C; ++i) gin[i] = valid ? g[i] : 0.f;
  qp_backward_row(gin, in.v, in.mu, rw.nominal, g_nom, g_low);
#pragma unroll
  for (int i = 0; i < C; ++i) {
    float g_lo = g_low[i], g_up = 0.f;
    if constexpr (SN) {
      // nominal = span * sig + lower, span = upper - lower
      gft[i] = ((g_nom[i] * rw.span[i]) * (1.0f - rw.sig[i])) * rw.sig[i];
      const float g_span = g_nom[i] * rw.sig[i];
      g_lo = (g_lo + g_nom[i]) - g_span;
      g_up = g_span;
    } else {
      gft[i] = g_nom[i];
    }
    // lower = -a1 (exp(s1 h) - 1), upper = a2 (1 - h)
    ghb[i] = ((g_lo * -a.d.alpha_1) * rw.es[i]) * a.d.sigma_1 + g_up * -a.d.alpha_2;
  }
  if (p == 0 && valid && q == 0) {
    store_row10(a.gft + r * C, gft);
    if (a.dbg_gft) store_row10(a.dbg_gft + r * C, gft);
  }
  OT_MARK(10);
  // g_z2^T = (Q3^T g_ft^T) masked by the saved a2 (K = 10 in 3 k-steps): wave p computes hidden
  // blocks 2p, 2p+1 (6 MFMA), the 8 blocks meet in LDS behind one barrier (same values as every
  // wave computing all 8)
  {
    switch (p) {              // wave-uniform: static register indices in each case
      case 0: gz2_pair<0>(a, q3t, gft, in, q, lane, valid ? a.gz2 + r * M : nullptr, sh.gax); break;
      case 1: gz2_pair<1>(a, q3t, gft, in, q, lane, valid ? a.gz2 + r * M : nullptr, sh.gax); break;
      case 2: gz2_pair<2>(a, q3t, gft, in, q, lane, valid ? a.gz2 + r * M : nullptr, sh.gax); break;
      default: gz2_pair<3>(a, q3t, gft, in, q, lane, valid ? a.gz2 + r * M : nullptr, sh.gax); break;
    }
  }
  __syncthreads();
  f32x4v ga[8];
#pragma unroll
  for (int hb = 0; hb < 8; ++hb) {
    const f32x4 v = *reinterpret_cast<const f32x4*>(&sh.gax[hb][lane][0]);
    ga[hb] = f32x4v{v[0], v[1], v[2], v[3]};
  }
  OT_MARK(11);
  // hidden blocks 2p, 2p+1 of g_a1^T = Q2^T g_z2^T (two independent accumulators), with the next
  // VJP's row math (VALU) interleaved between the 64 MFMAs: one region, explicit issue groups
  __builtin_amdgcn_sched_barrier(0);
  vjp_row_math<SN>(a, nin, nrw);
  f32x4v gb[2] = {z4(), z4()};
#pragma unroll
  for (int hb = 0; hb < 8; ++hb) {
#pragma unroll
    for (int o = 0; o < 2; ++o) {
#pragma unroll
      for (int t = 0; t < 4; ++t) gb[o] = mfma16(wv.q2t[o][hb][t], ga[hb][t], gb[o]);
    }
  }
#pragma unroll
  for (int i = 0; i < 64; ++i) {
    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);     // one MFMA
    __builtin_amdgcn_sched_group_barrier(0x002, 6, 0);     // then up to six VALU
  }
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int o = 0; o < 2; ++o) {
    const f32x4 act = in.a1[o];
#pragma unroll
    for (int t = 0; t < 4; ++t) gb[o][t] = act[t] > 0.f ? gb[o][t] * a.drop_scale : 0.f;
    if (valid)
      *reinterpret_cast<f32x4*>(a.gz1 + r * M + 16 * (2 * p + o) + 4 * q) = f32x4{gb[o][0], gb[o][1], gb[o][2], gb[o][3]};
  }
  OT_MARK(12);
  // partial g_h^T over hidden blocks 2p, 2p+1 (Q1^T image, rows >= 10 zero)
  f32x4v gh = z4();
#pragma unroll
  for (int o = 0; o < 2; ++o) {
#pragma unroll
    for (int t = 0; t < 4; ++t) gh = mfma16(wv.q1t[o][t], gb[o][t], gh);
  }
  *reinterpret_cast<f32x4*>(&sh.gpart[buf][p][lane][0]) = f32x4{gh[0], gh[1], gh[2], gh[3]};
  OT_MARK(13);
  __syncthreads();
  OT_MARK(14);
#pragma unroll
  for (int i = 0; i < C; ++i) {
    const int ln = 16 * (i >> 2) + j, rg = i & 3;
    const float ghm = ((sh.gpart[buf][0][ln][rg] + sh.gpart[buf][1][ln][rg]) + sh.gpart[buf][2][ln][rg]) +
                      sh.gpart[buf][3][ln][rg];
    gy_out[i] = ghm + ghb[i];
  }
  OT_MARK(15);
}

template <bool SN>
__global__ __launch_bounds__(256) void k_ot_bwd(OTArgs a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  OtBwdShared& sh = *reinterpret_cast<OtBwdShared*>(smem);
  const int lane = threadIdx.x & 63, q = lane >> 4, j = lane & 15;
  const int p = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  VjpW wv;
#pragma unroll
  for (int o = 0; o < 2; ++o) {
#pragma unroll
    for (int hb = 0; hb < 8; ++hb)
#pragma unroll
      for (int t = 0; t < 4; ++t) wv.q2t[o][hb][t] = a.Q2[(16 * hb + 4 * q + t) * M + 16 * (2 * p + o) + j];
#pragma unroll
    for (int t = 0; t < 4; ++t) wv.q1t[o][t] = j < C ? a.Q1[(16 * (2 * p + o) + 4 * q + t) * C + j] : 0.f;
  }
  float q3t[8][3];                    // A operand of g_a2^T: Q3^T[16hb + j][4s + q] = Q3[4s + q][16hb + j]
#pragma unroll
  for (int hb = 0; hb < 8; ++hb)
#pragma unroll
    for (int s = 0; s < 3; ++s) q3t[hb][s] = 4 * s + q < C ? a.Q3[(4 * s + q) * M + 16 * hb + j] : 0.f;
  const int b = blockIdx.x * TR + j;
  const bool valid = b < a.B;
  float gy[C];
  if (valid) load_row10(a.g_y + (size_t)b * C, gy);
  else
#pragma unroll
    for (int i = 0; i < C; ++i) gy[i] = 0.f;
  const float third = 1.0f / 3.0f;
  int buf = 0;
  VjpIn cur, nxt;
  VjpRow crw, nrw;
  load_vjp_in(a, p, a.E - 1, b, valid, q, cur);
  vjp_row_math<SN>(a, cur, crw);
  // evals are visited E-1, E-2, ..., 0: each VJP first issues the loads of the next one and
  // computes its row math between its own MFMA chains
#define OT_VJP(E_, G_)                                                                  \
  load_vjp_in(a, p, (E_) - 1, b, valid, q, nxt);                                        \
  ot_vjp<SN>(a, wv, q3t, sh, buf, p, (E_), b, valid, lane, q, j, cur, crw, nxt, nrw, G_, gY); \
  cur = nxt;                                                                            \
  crw = nrw;                                                                            \
  buf ^= 1;
  for (int it = a.niters - 2; it >= 0; --it) {
    float ta, dt;
    step_times(a, it, ta, dt);
    const float c8 = dt * 0.125f, c38 = 3.0f * c8;
    float gk1[C], gk2[C], gk3[C], gk4[C], acc[C], gY[C];
#pragma unroll
    for (int i = 0; i < C; ++i) {
      acc[i] = gy[i];
      gk1[i] = gy[i] * c8;
      gk2[i] = gy[i] * c38;
      gk3[i] = gy[i] * c38;
      gk4[i] = gy[i] * c8;
    }
    const int e0 = 4 * it;
    OT_VJP(e0 + 3, gk4)
#pragma unroll
    for (int i = 0; i < C; ++i) {
      acc[i] += gY[i];
      const float d = dt * gY[i];
      gk1[i] += d;
      gk2[i] -= d;
      gk3[i] += d;
    }
    OT_VJP(e0 + 2, gk3)
#pragma unroll
    for (int i = 0; i < C; ++i) {
      acc[i] += gY[i];
      const float d = dt * gY[i];
      gk2[i] += d;
      gk1[i] -= d * third;
    }
    OT_VJP(e0 + 1, gk2)
#pragma unroll
    for (int i = 0; i < C; ++i) {
      acc[i] += gY[i];
      gk1[i] += (dt * gY[i]) * third;
    }
    OT_VJP(e0, gk1)
#pragma unroll
    for (int i = 0; i < C; ++i) gy[i] = acc[i] + gY[i];
  }
#undef OT_VJP
}

// ---------------------------------------------------------------------------------------------
// backward on 4-row tiles (the rk4 solve for B <= 4 * FIODE_OT4_MAX_TILES): the VJPs of k_ot_bwd
// with the MFMA products of tile4.h -- wave p owns hidden units 32p .. 32p + 31:
//   g_z2 = (Q3^T g_ft) [a2 > 0] / (1 - p): K = 10 in two halves (5 steps), halves by permlane32;
//   g_a1 = Q2^T g_z2 (K = 128 from LDS, halves, 4 accumulators), g_z1 = g_a1 [a1 > 0] / (1 - p);
//   g_h partial = Q1^T g_z1 over the wave's 32 units (quarters, permlane16 / permlane32);
// the 4 parts of g_h meet in LDS (double-buffered, one barrier per VJP besides the g_z2 one).
struct OtBwdShared4 {
  float gz2s[TR4][M + 4];     // g_z2 of all units [sample][unit] (B operands of Q2^T)
  float gz1s[TR4][M + 4];     // g_z1 [sample][unit] (each wave reads back its own units)
  float gpart[2][4][16][4];   // [buffer][part][lane 4 blk + j][reg]: g_h partial of outputs 4 blk + reg
};

struct VjpIn4 {
  float h[C], ft[C], v[C], mu;
  f32x4 a2, a1;               // saved post-activations of units 32p + 4 blk + r (this lane's block)
};

__device__ __forceinline__ void load_vjp_in4(const OTArgs& a, int p, int e, int b, bool valid, int lane, VjpIn4& in) {
  const int bb = valid ? b : a.B - 1;
  const size_t r = (size_t)bb * a.E + (e < 0 ? 0 : e);
  load_row10(a.hs + r * C, in.h);
  load_row10(a.ftw + r * C, in.ft);
  load_row10(a.vw + r * C, in.v);
  in.mu = a.muw[r];
  const int u0 = 32 * p + 4 * ((lane >> 2) & 7);
  in.a2 = *reinterpret_cast<const f32x4*>(a.a2 + r * M + u0);
  in.a1 = *reinterpret_cast<const f32x4*>(a.a1 + r * M + u0);
}

// transposed weight operands of wave p (registers for the whole kernel), i = lane & 3, b = lane >> 2:
//   q3t[s] = Q3[s + 5 (b >> 3)][32p + 4 (b & 7) + i]         (g_z2, s = 0..4)
//   q2t[s] = Q2[s + 64 (b >> 3)][32p + 4 (b & 7) + i]        (g_a1, s = 0..63)
//   q1t[s] = Q1[32p + 8 (b >> 2) + s][4 (b & 3) + i]  (0 for classes >= C; g_h, s = 0..7)
struct VjpW4 {
  float q3t[5];
  float q2t[64];
  float q1t[8];
};

template <bool SN>
__device__ void ot_vjp4(const OTArgs& a, const VjpW4& wv, OtBwdShared4& sh, int buf, int p, int e, int b, bool valid,
                        int lane, int j, const VjpIn4& in, const VjpRow& rw, const float (&g)[C], float (&gy_out)[C]) {
  const int bb = valid ? b : a.B - 1;
  const size_t r = (size_t)bb * a.E + e;
  const int blk4 = lane >> 2, hi = blk4 >> 3, blk = blk4 & 7;
#ifdef OT_PROFILE
  uint64_t t_prev = wall_clock64();
#endif
  float g_nom[C], g_low[C], gft[C], ghb[C];
  float gin[C];
#pragma unroll
  for (int i = 0; i < C; ++i) gin[i] = valid ? g[i] : 0.f;
  qp_backward_row(gin, in.v, in.mu, rw.nominal, g_nom, g_low);
#pragma unroll
  for (int i = 0; i < C; ++i) {
    float g_lo = g_low[i], g_up = 0.f;
    if constexpr (SN) {
      gft[i] = ((g_nom[i] * rw.span[i]) * (1.0f - rw.sig[i])) * rw.sig[i];
      const float g_span = g_nom[i] * rw.sig[i];
      g_lo = (g_lo + g_nom[i]) - g_span;
      g_up = g_span;
    } else {
      gft[i] = g_nom[i];
    }
    ghb[i] = ((g_lo * -a.d.alpha_1) * rw.es[i]) * a.d.sigma_1 + g_up * -a.d.alpha_2;
  }
  if (p == 0 && valid && lane < TR4) {
    store_row10(a.gft + r * C, gft);
    if (a.dbg_gft) store_row10(a.dbg_gft + r * C, gft);
  }
  OT_MARK(10);
  // g_z2 of units 32p + 4 blk + r
  f32x4v gz = zero4();
#pragma unroll
  for (int s = 0; s < 5; ++s) gz = mfma4(wv.q3t[s], hi ? gft[s + 5] : gft[s], gz);
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const float v = gz[t] + swap32(gz[t]);
    gz[t] = in.a2[t] > 0.f ? v * a.drop_scale : 0.f;
  }
  if (blk4 < 8) {
    const f32x4 v = f32x4{gz[0], gz[1], gz[2], gz[3]};
    *reinterpret_cast<f32x4*>(&sh.gz2s[j][32 * p + 4 * blk]) = v;
    if (valid) *reinterpret_cast<f32x4*>(a.gz2 + r * M + 32 * p + 4 * blk) = v;
  }
  __syncthreads();
  OT_MARK(11);
  // g_a1 = Q2^T g_z2 of units 32p + 4 blk + r: K half hi, 4 accumulators
  f32x4v acc[4] = {zero4(), zero4(), zero4(), zero4()};
  k128_half(&sh.gz2s[j][64 * hi], wv.q2t, acc);
  f32x4v gb;
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const float part = (acc[0][t] + acc[1][t]) + (acc[2][t] + acc[3][t]);
    const float other = swap32(part);
    const float v = hi ? (other + part) : (part + other);
    gb[t] = in.a1[t] > 0.f ? v * a.drop_scale : 0.f;
  }
  if (blk4 < 8) {
    const f32x4 v = f32x4{gb[0], gb[1], gb[2], gb[3]};
    *reinterpret_cast<f32x4*>(&sh.gz1s[j][32 * p + 4 * blk]) = v;       // read back by this wave only
    if (valid) *reinterpret_cast<f32x4*>(a.gz1 + r * M + 32 * p + 4 * blk) = v;
  }
  OT_MARK(12);
  // g_h partial over the wave's units: outputs 4 (b & 3) + t, units 32p + 8 (b >> 2) + s
  f32x4v gha = zero4(), ghc = zero4();
  const float* g1 = &sh.gz1s[j][32 * p + 8 * (blk4 >> 2)];
  const f32x4 v0 = *reinterpret_cast<const f32x4*>(g1), v1 = *reinterpret_cast<const f32x4*>(g1 + 4);
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    gha = mfma4(wv.q1t[t], v0[t], gha);
    ghc = mfma4(wv.q1t[4 + t], v1[t], ghc);
  }
  f32x4v gh;
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const float x = gha[t] + ghc[t];
    const float y = x + swap16(x);
    gh[t] = y + swap32(y);
  }
  if (blk4 < 4) *reinterpret_cast<f32x4*>(&sh.gpart[buf][p][lane][0]) = f32x4{gh[0], gh[1], gh[2], gh[3]};
  OT_MARK(13);
  __syncthreads();
  OT_MARK(14);
#pragma unroll
  for (int i = 0; i < C; ++i) {
    const int ln = 4 * (i >> 2) + j, rg = i & 3;
    const float ghm = ((sh.gpart[buf][0][ln][rg] + sh.gpart[buf][1][ln][rg]) + sh.gpart[buf][2][ln][rg]) +
                      sh.gpart[buf][3][ln][rg];
    gy_out[i] = ghm + ghb[i];
  }
  OT_MARK(15);
}

template <bool SN>
__global__ __launch_bounds__(256) void k_ot_bwd4(OTArgs a) {
  fiode_wave_prio(a.prio & 2);
  extern __shared__ __attribute__((aligned(16))) float smem[];
  OtBwdShared4& sh = *reinterpret_cast<OtBwdShared4*>(smem);
  const int lane = threadIdx.x & 63, j = lane & 3;
  const int p = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  VjpW4 wv;
  {
    const int bq = lane >> 2, i = lane & 3;
    const int u = 32 * p + 4 * (bq & 7) + i;
#pragma unroll
    for (int s = 0; s < 5; ++s) wv.q3t[s] = a.Q3[(s + 5 * (bq >> 3)) * M + u];
#pragma unroll
    for (int s = 0; s < 64; ++s) wv.q2t[s] = a.Q2[(size_t)(s + 64 * (bq >> 3)) * M + u];
    const int c = 4 * (bq & 3) + i;
#pragma unroll
    for (int s = 0; s < 8; ++s) wv.q1t[s] = c < C ? a.Q1[(32 * p + 8 * (bq >> 2) + s) * C + c] : 0.f;
  }
  const int b = blockIdx.x * TR4 + j;
  const bool valid = b < a.B;
  float gy[C];
  if (valid) load_row10(a.g_y + (size_t)b * C, gy);
  else
#pragma unroll
    for (int i = 0; i < C; ++i) gy[i] = 0.f;
  const float third = 1.0f / 3.0f;
  int buf = 0;
  VjpIn4 cur, nxt;
  VjpRow crw;
  load_vjp_in4(a, p, a.E - 1, b, valid, lane, cur);
#define OT_VJP4(E_, G_)                                                                 \
  load_vjp_in4(a, p, (E_) - 1, b, valid, lane, nxt);                                    \
  vjp_row_math<SN>(a, cur, crw);                                                        \
  ot_vjp4<SN>(a, wv, sh, buf, p, (E_), b, valid, lane, j, cur, crw, G_, gY);          \
  cur = nxt;                                                                            \
  buf ^= 1;
  for (int it = a.niters - 2; it >= 0; --it) {
    float ta, dt;
    step_times(a, it, ta, dt);
    const float c8 = dt * 0.125f, c38 = 3.0f * c8;
    float gk1[C], gk2[C], gk3[C], gk4[C], acc[C], gY[C];
#pragma unroll
    for (int i = 0; i < C; ++i) {
      acc[i] = gy[i];
      gk1[i] = gy[i] * c8;
      gk2[i] = gy[i] * c38;
      gk3[i] = gy[i] * c38;
      gk4[i] = gy[i] * c8;
    }
    const int e0 = 4 * it;
    OT_VJP4(e0 + 3, gk4)
#pragma unroll
    for (int i = 0; i < C; ++i) {
      acc[i] += gY[i];
      const float d = dt * gY[i];
      gk1[i] += d;
      gk2[i] -= d;
      gk3[i] += d;
    }
    OT_VJP4(e0 + 2, gk3)
#pragma unroll
    for (int i = 0; i < C; ++i) {
      acc[i] += gY[i];
      const float d = dt * gY[i];
      gk2[i] += d;
      gk1[i] -= d * third;
    }
    OT_VJP4(e0 + 1, gk2)
#pragma unroll
    for (int i = 0; i < C; ++i) {
      acc[i] += gY[i];
      gk1[i] += (dt * gY[i]) * third;
    }
    OT_VJP4(e0, gk1)
#pragma unroll
    for (int i = 0; i < C; ++i) gy[i] = acc[i] + gY[i];
  }
#undef OT_VJP4
}

// =============================================================================================
// train_ode with adaptive dopri5 (cifar_train.yaml:30,32: train_ode_solver dopri5, train_ode_tol
// 1e-3; pl_modules.py:490-500 -> models.py:235-241 odeint, use_adjoint False at pl_modules.py:303):
// torchdiffeq 0.2.2's RKAdaptiveStepsizeODESolver in TRAIN mode, backpropagated directly through
// everything it computes -- the stages, the error ratio of accepted AND rejected attempts (it sets
// the next step size), the step-size controller, the initial-step selection and the interpolation
// point of the output.  oracle/dopri5_train.py restates the algorithm (dopri5_train) and this
// kernel's reverse sweep (dopri5_adjoint), checked there against torch autograd.
//
// Same tiles, MLP and QP exit as the rk4 solve (ot_eval / ot_vjp: one persistent workgroup per
// 16-row tile, hidden units split over 4 waves, rows replicated in every wave).  The solve's
// batch couplings beyond the QP exits -- the RMS norms of the initial step and every attempt's error
// ratio, and in the backward every attempt's dt adjoint -- are float64 sums over all rows that
// every workgroup forms identically (ot_batch_sum: per-tile partials exchanged through tagged
// granules and added in tile order).  The controller (dt, t, accept) runs redundantly and
// identically in every thread.  Stage derivatives k_0..k_6 of the current attempt live in LDS
// (every wave its own copy); the saved per-eval arrays (hs, a1, a2, ft, v, mu, nominal) are the rk4
// solve's, at row (b, e) = b E + e with E = 2 + 6 A the capacity; eval e of attempt n is 2 + 6n + i.
constexpr int OT_XV = 4;          // float64 values per reduction exchange (at most)
enum { ALOG_T = 0, ALOG_DT, ALOG_RATIO, ALOG_ACCEPT, ALOG_FIDX, ALOG_E0, ALOG_W = 8 };
enum { META_D0 = 0, META_D1, META_D2, META_H0, META_H1, META_CLAMP0, META_CLAMP1, META_DT0, META_R2, META_N = 16 };

// float64 sum over the 64 lanes, the same value in every lane (fixed order): a DPP prefix scan
// within each 16-lane row (VALU; the shuffle butterfly was 6 dependent LDS-crossbar round trips
// per value), then the four row totals added in row order
template <int N>
__device__ __forceinline__ double dpp_row_shr(double x) {
  const long long u = __double_as_longlong(x);
  const int lo = __builtin_amdgcn_update_dpp(0, (int)(u & 0xFFFFFFFF), 0x110 + N, 0xf, 0xf, true);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(u >> 32), 0x110 + N, 0xf, 0xf, true);
  return __longlong_as_double(((long long)(unsigned)hi << 32) | (unsigned)lo);
}
__device__ __forceinline__ double readlane_d(double x, int l) {
  const long long u = __double_as_longlong(x);
  const int lo = __builtin_amdgcn_readlane((int)(u & 0xFFFFFFFF), l);
  const int hi = __builtin_amdgcn_readlane((int)(u >> 32), l);
  return __longlong_as_double(((long long)(unsigned)hi << 32) | (unsigned)lo);
}
#ifndef FIODE_BSUM_DPP
#define FIODE_BSUM_DPP 1
#endif
__device__ __forceinline__ double wave_dsum(double x) {
  if constexpr (FIODE_BSUM_DPP == 0) {
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) x += __shfl_xor(x, o, 64);
    return x;
  }
  x += dpp_row_shr<1>(x);
  x += dpp_row_shr<2>(x);
  x += dpp_row_shr<4>(x);
  x += dpp_row_shr<8>(x);
  return ((readlane_d(x, 15) + readlane_d(x, 31)) + readlane_d(x, 47)) + readlane_d(x, 63);
}

// sum over all rows (every workgroup gets the same float64 values): the caller's per-lane values
// count only on owner lanes (the caller zeroes the others; every wave holds the same rows, so every
// wave forms the same partial).  Wave 0 publishes the partial; every wave gathers the granules
// itself and adds them in tile order, so the result needs no LDS broadcast and no barrier (the
// dopri5 forward: 1146 -> 1123 us at B = 128).
template <int NV>
__device__ void ot_batch_sum(const OTArgs& a, int& dead, unsigned& ep, const double (&mine)[NV],
                             double (&out)[NV]) {
  const int lane = threadIdx.x & 63;
#ifdef OT_PROFILE
  const uint64_t tp0 = wall_clock64();
#endif
  double w[NV];
#pragma unroll
  for (int i = 0; i < NV; ++i) w[i] = wave_dsum(mine[i]);
  const int G = gridDim.x;
  unsigned long long* buf = a.xr + (size_t)(ep & 1u) * G * 2 * OT_XV;
  if (threadIdx.x == 0) {
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      const unsigned long long bits = (unsigned long long)__double_as_longlong(w[v]);
      publish_mask(buf + (size_t)blockIdx.x * 2 * OT_XV + 2 * v, ep, (uint32_t)(bits >> 32));
      publish_mask(buf + (size_t)blockIdx.x * 2 * OT_XV + 2 * v + 1, ep, (uint32_t)bits);
    }
  }
  double acc[NV];
#pragma unroll
  for (int v = 0; v < NV; ++v) acc[v] = 0.0;
  bool timed_out = false;
  for (int base = 0; base < G; base += 64) {
    const int t = base + lane;
    unsigned spins = 0;
    for (;;) {
      bool ok = true;
      unsigned long long x[2 * NV];
#pragma unroll
      for (int g = 0; g < 2 * NV; ++g) {
        x[g] = 0;
        if (t < G) {
          x[g] = __hip_atomic_load((gu64_t*)(buf + (size_t)t * 2 * OT_XV + g), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
          ok = ok && (unsigned)(x[g] >> 32) == ep;
        }
      }
      if (__all(ok)) {
        if (t < G) {
#pragma unroll
          for (int v = 0; v < NV; ++v)
            acc[v] += __longlong_as_double((long long)(((x[2 * v] & 0xFFFFFFFFull) << 32) | (x[2 * v + 1] & 0xFFFFFFFFull)));
        }
        break;
      }
      if (dead || ++spins > (1u << 22)) {     // ~0.5 s: a workgroup is not resident
        timed_out = true;
        if (lane == 0) {
          atomicMax(a.stats ? a.stats + 3 : a.imeta + 2, 4);
          dead = 1;
        }
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
  }
  // a timed-out exchange summed only the granules that arrived: NaN, so everything computed from
  // it (y_out, the step-size controller) is poisoned instead of silently wrong.  Every wave gathers
  // for itself, so one wave can time out after another has finished with a finite sum; the
  // controller then runs on different values in different waves and their loop trip counts (with
  // the __syncthreads inside the evals) would diverge.  One barrier makes the decision uniform:
  // every timeout wrote `dead` (lane 0 of the wave) before it, every wave reads it after it.
  const double tot0 = wave_dsum(acc[0]);
  (void)timed_out;
  __syncthreads();
  const bool poisoned = dead != 0;               // (a sticky earlier timeout poisons every later sum)
#pragma unroll
  for (int v = 0; v < NV; ++v) {
    const double tot = v == 0 ? tot0 : wave_dsum(acc[v]);
    out[v] = poisoned ? __builtin_nan("") : tot;
  }
  ++ep;
#ifdef OT_PROFILE
  if (blockIdx.x == 0 && threadIdx.x == 0) atomicAdd(a.prof + 9, (unsigned long long)(wall_clock64() - tp0));
#endif
}

// The backward keeps the round-4 form: wave 0 gathers, LDS broadcast behind barriers (the form
// above measured 35 us slower there at B = 128).
template <int NV>
__device__ void ot_batch_sum_bwd(const OTArgs& a, double* red, int& dead, unsigned& ep, const double (&mine)[NV],
                             double (&out)[NV]) {
  const int lane = threadIdx.x & 63;
#ifdef OT_PROFILE
  const uint64_t tp0 = wall_clock64();
#endif
  if (threadIdx.x < 64) {
    double w[NV];
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      double s = mine[i];
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) s += __shfl_xor(s, o, 64);
      w[i] = s;
    }
    const int G = gridDim.x;
    unsigned long long* buf = a.xr + (size_t)(ep & 1u) * G * 2 * OT_XV;
    if (lane == 0) {
#pragma unroll
      for (int v = 0; v < NV; ++v) {
        const unsigned long long bits = (unsigned long long)__double_as_longlong(w[v]);
        publish_mask(buf + (size_t)blockIdx.x * 2 * OT_XV + 2 * v, ep, (uint32_t)(bits >> 32));
        publish_mask(buf + (size_t)blockIdx.x * 2 * OT_XV + 2 * v + 1, ep, (uint32_t)bits);
      }
    }
    double acc[NV];
#pragma unroll
    for (int v = 0; v < NV; ++v) acc[v] = 0.0;
    for (int base = 0; base < G; base += 64) {
      const int t = base + lane;
      unsigned spins = 0;
      for (;;) {
        bool ok = true;
        unsigned long long x[2 * NV];
#pragma unroll
        for (int g = 0; g < 2 * NV; ++g) {
          x[g] = 0;
          if (t < G) {
            x[g] = __hip_atomic_load((gu64_t*)(buf + (size_t)t * 2 * OT_XV + g), __ATOMIC_RELAXED,
                                     __HIP_MEMORY_SCOPE_AGENT);
            ok = ok && (unsigned)(x[g] >> 32) == ep;
          }
        }
        if (__all(ok)) {
          if (t < G) {
#pragma unroll
            for (int v = 0; v < NV; ++v)
              acc[v] += __longlong_as_double((long long)(((x[2 * v] & 0xFFFFFFFFull) << 32) | (x[2 * v + 1] & 0xFFFFFFFFull)));
          }
          break;
        }
        if (dead || ++spins > (1u << 22)) {     // ~0.5 s: a workgroup is not resident
          if (lane == 0) {
            atomicMax(a.stats ? a.stats + 3 : a.imeta + 2, 4);
            dead = 1;
          }
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
    }
#pragma unroll
    for (int v = 0; v < NV; ++v) {
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) acc[v] += __shfl_xor(acc[v], o, 64);
    }
    // a timed-out exchange summed only the granules that arrived: NaN, so everything computed from
    // it (y_out in the forward; g_dt and every stage adjoint upstream of it in the backward) is
    // poisoned instead of silently wrong
    if (lane == 0)
#pragma unroll
      for (int v = 0; v < NV; ++v) red[v] = dead ? __builtin_nan("") : acc[v];
  }
  ++ep;
  __syncthreads();
#pragma unroll
  for (int v = 0; v < NV; ++v) out[v] = red[v];
  __syncthreads();
#ifdef OT_PROFILE
  if (blockIdx.x == 0 && threadIdx.x == 0) atomicAdd(a.prof + 9, (unsigned long long)(wall_clock64() - tp0));
#endif
}

template <bool T4>
struct OdpShared {
  std::conditional_t<T4, OtShared4, OtShared> ot;
  float kst[4][7][T4 ? TR4 : TR][C];      // [wave][stage][row][c]: the current attempt's k_0..k_6
};

__device__ __forceinline__ double rms_of(double sumsq, double n) { return sqrt(sumsq / n); }

// T4: 4-row tiles (tile4.h MLP, ot_eval4) for B <= 4 * FIODE_OT4_MAX_TILES, else 16-row tiles
template <bool T4>
__global__ __launch_bounds__(256) void k_odp_fwd(OTArgs a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  constexpr int TRX = T4 ? TR4 : TR;
  OdpShared<T4>& S = *reinterpret_cast<OdpShared<T4>*>(smem);
  auto& sh = S.ot;
  if (threadIdx.x == 0) {
    sh.Kprev = a.d.max_iter - 1;
    sh.dead = 0;
  }
  const int lane = threadIdx.x & 63, q = lane >> 4, j = lane & (TRX - 1);
  const int p = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int b = blockIdx.x * TRX + j;
  const bool valid = b < a.B;
  const bool first = T4 ? lane < TR4 : q == 0;   // one lane per row (wave 0's are the row writers)
  const bool own = valid && first;             // lanes whose row values count in the batch sums
  const int bb = valid ? b : a.B - 1;
  std::conditional_t<T4, T4W, T16W> w;
  if constexpr (T4) load_t4w(a.Q1, a.Q2, a.Q3, a.b2, a.b3, p, lane, w);
  else load_t16w(a.Q1, a.Q2, M, a.Q3, M, a.b2, a.b3, p, q, j, w);
  for (int t = threadIdx.x; t < TRX * M; t += blockDim.x) {
    const int rb = blockIdx.x * TRX + t / M, i = t % M;
    if (rb < a.B) {
      float s = 0.f;
#pragma unroll
      for (int c = 0; c < FIODE_X; ++c) s = __fmaf_rn(a.Qx[i * FIODE_X + c], a.x_feat[(size_t)rb * FIODE_X + c], s);
      a.u[(size_t)rb * M + i] = (s + a.bx[i]) + a.b1[i];
    }
  }
  __syncthreads();
  std::conditional_t<T4, f32x4, f32x4v[8]> uacc;
  if constexpr (T4) {
    uacc = *reinterpret_cast<const f32x4*>(a.u + (size_t)bb * M + 32 * p + 4 * ((lane >> 2) & 7));
  } else {
#pragma unroll
    for (int hb = 0; hb < 8; ++hb) {
      const f32x4 uv = *reinterpret_cast<const f32x4*>(a.u + (size_t)bb * M + 16 * hb + 4 * q);
      uacc[hb] = f32x4v{uv[0], uv[1], uv[2], uv[3]};
    }
  }
  // keep words of eval e: all 4 words of layer 1 and the part's layer-2 word (16-row), or the
  // part's word of each layer (4-row)
  const uint32_t* kwp = a.kw;
  const Rng krng = rng_of(a);
  auto fetch = [&](int e, uint32_t (&w1)[4], uint32_t& w2) {
    if (a.dropout_mode == FIODE_DROPOUT_OFF) {
#pragma unroll
      for (int t = 0; t < 4; ++t) w1[t] = 0xFFFFFFFFu;
      w2 = 0xFFFFFFFFu;
      return;
    }
    if (a.kw_lazy && e >= a.kw_pre) {   // the draws k_ot_masks would make (same stream, index, offset)
      const uint4 r0 = krng.draw((uint32_t)bb, RNG_STREAM_ODE_DROP + ((uint32_t)e << 5));
      const uint4 r1 = krng.draw((uint32_t)bb, RNG_STREAM_ODE_DROP + ((uint32_t)e << 5) + (1u << 4));
      w1[0] = r0.x; w1[1] = r0.y; w1[2] = r0.z; w1[3] = r0.w;
      w2 = p == 0 ? r1.x : p == 1 ? r1.y : p == 2 ? r1.z : r1.w;
      if (p == 0 && first && valid && e < a.E) {      // saved for the backward and the weight chain
        reinterpret_cast<uint4*>(a.kw)[((size_t)e * 2 + 0) * a.B + b] = r0;
        reinterpret_cast<uint4*>(a.kw)[((size_t)e * 2 + 1) * a.B + b] = r1;
      }
      return;
    }
    const uint4 q1 = reinterpret_cast<const uint4*>(kwp)[((size_t)e * 2 + 0) * a.B + bb];
    w1[0] = q1.x; w1[1] = q1.y; w1[2] = q1.z; w1[3] = q1.w;
    w2 = kwp[(((size_t)e * 2 + 1) * a.B + bb) * 4 + p];
  };
  float (*ks)[TRX][C] = S.kst[p];
  // every lane of the row writes the same values into its wave's copy, so no lane reads another's
  auto kput = [&](int s, const float (&v)[C]) {
#pragma unroll
    for (int c = 0; c < C; ++c) ks[s][j][c] = v[c];
  };
  auto kget = [&](int s, float (&v)[C]) {
#pragma unroll
    for (int c = 0; c < C; ++c) v[c] = ks[s][j][c];
  };
  int e = 0;
  uint32_t kc1[4], kc2;
  fetch(0, kc1, kc2);
#ifdef OT_PROFILE
#define ODP_T0(V) const uint64_t V = wall_clock64();
#define ODP_T1(SLOT, V) if (blockIdx.x == 0 && threadIdx.x == 0) atomicAdd(a.prof + (SLOT), (unsigned long long)(wall_clock64() - V));
#else
#define ODP_T0(V)
#define ODP_T1(SLOT, V)
#endif
  auto eval = [&](const float (&h)[C], float (&k)[C]) {
    uint32_t kn1[4] = {0u, 0u, 0u, 0u}, kn2 = 0u;
    ODP_T0(tf0)
    if (e + 1 < a.E) fetch(e + 1, kn1, kn2);
    ODP_T1(10, tf0)
    if constexpr (T4) ot_eval4(a, w, sh, e, p, b, valid, lane, j, uacc, kc1[p], kc2, h, k);
    else ot_eval(a, w, sh, e, p, b, valid, lane, q, j, uacc, kc1, kc2, h, k);
#pragma unroll
    for (int t = 0; t < 4; ++t) kc1[t] = kn1[t];
    kc2 = kn2;
    ++e;
  };
  const double NBC = (double)a.B * C;
  const float rtol = (float)a.rtol, atol = (float)a.atol;
  unsigned rep = 1;
  const bool lead = blockIdx.x == 0 && threadIdx.x == 0;
  // ---- _select_initial_step(order 4), float32 (odesolve.hip os_dopri5's expressions) ----------
  float y[C], fcur[C];
  load_row10(a.h0 + (size_t)bb * C, y);
  eval(y, fcur);
  double s01[2] = {0.0, 0.0};
  if (own) {
#pragma unroll
    for (int c = 0; c < C; ++c) {
      const float sc = atol + fabsf(y[c]) * rtol;
      const float q0 = y[c] / sc, qq = fcur[c] / sc;
      s01[0] += (double)q0 * q0;
      s01[1] += (double)qq * qq;
    }
  }
  ot_batch_sum<2>(a, sh.dead, rep, s01, s01);
  const float d0 = (float)rms_of(s01[0], NBC), d1 = (float)rms_of(s01[1], NBC);
  const bool clamp0 = d0 < 1e-5f || d1 < 1e-5f;
  const float h0s = clamp0 ? 1e-6f : (0.01f * d0) / d1;
  double dt;
  {
    float yi[C], f1[C];
#pragma unroll
    for (int c = 0; c < C; ++c) yi[c] = y[c] + h0s * fcur[c];
    eval(yi, f1);
    double s2[1] = {0.0};
    if (own) {
#pragma unroll
      for (int c = 0; c < C; ++c) {
        const float sc = atol + fabsf(y[c]) * rtol;
        const float qv = (f1[c] - fcur[c]) / sc;
        s2[0] += (double)qv * qv;
      }
    }
    ot_batch_sum<1>(a, sh.dead, rep, s2, s2);
    const float r2 = (float)rms_of(s2[0], NBC);
    const float d2 = r2 / h0s;
    const bool clamp1 = d1 <= 1e-15f && d2 <= 1e-15f;
    const float h1 = clamp1 ? fmaxf(1e-6f, h0s * 1e-3f) : powf(0.01f / fmaxf(d1, d2), 1.0f / 5.0f);
    dt = (double)fminf(100.0f * h0s, h1);
    if (lead) {
      a.meta[META_D0] = d0; a.meta[META_D1] = d1; a.meta[META_D2] = d2; a.meta[META_H0] = h0s;
      a.meta[META_H1] = h1; a.meta[META_CLAMP0] = clamp0; a.meta[META_CLAMP1] = clamp1; a.meta[META_R2] = r2;
      a.meta[META_DT0] = dt;
    }
  }
  // ---- attempts -------------------------------------------------------------------------------
  double tcur = a.t0d, tprev = tcur, tnext = tcur;
  const double tmax = a.t1d;
  int n = 0, nacc = 0, nrej = 0, status = 0, fidx = 0;
  float yprev[C];
#pragma unroll
  for (int c = 0; c < C; ++c) yprev[c] = y[c];
  float dt32L = 0.f;
  while (tmax > tnext) {
#ifdef OT_PROFILE
    const uint64_t ta0 = wall_clock64();
#endif
    if (n >= a.A || !(tcur + dt > tcur)) {
      status = n >= a.A ? 2 : 3;           // attempt capacity exhausted / dt underflow
      break;
    }
    const float dt32 = (float)dt;
    if (p == 0 && first && valid) store_row10(a.ys + ((size_t)n * a.B + b) * C, y);
    if (lead) {
      double* lg = a.alog + (size_t)n * ALOG_W;
      lg[ALOG_T] = tcur; lg[ALOG_DT] = dt; lg[ALOG_FIDX] = fidx; lg[ALOG_E0] = e;
    }
    kput(0, fcur);
    float hin[C];
    for (int i = 0; i < 6; ++i) {
      ODP_T0(ts0)
      float acc[C];
#pragma unroll
      for (int c = 0; c < C; ++c) acc[c] = 0.f;
#pragma unroll
      for (int jj = 0; jj < 6; ++jj) {
        if (jj <= i) {          // (uniform; unrolled so the LDS reads of all terms issue together)
          float f[C];
          kget(jj, f);
          const float co = DP_BETA[i][jj] * dt32;
#pragma unroll
          for (int c = 0; c < C; ++c) acc[c] = acc[c] + f[c] * co;
        }
      }
#pragma unroll
      for (int c = 0; c < C; ++c) hin[c] = y[c] + acc[c];
      ODP_T1(11, ts0)
      float kn[C];
      eval(hin, kn);
      kput(i + 1, kn);
    }
    // y_new = the stage-5 input (FSAL); batch-global RMS error ratio
    ODP_T0(te0)
    double ps[1] = {0.0};
    if (own) {
      float err[C];
#pragma unroll
      for (int c = 0; c < C; ++c) err[c] = 0.f;
#pragma unroll
      for (int jj = 0; jj < 7; ++jj) {
        float f[C];
        kget(jj, f);
        const float co = DP_CERR[jj] * dt32;
#pragma unroll
        for (int c = 0; c < C; ++c) err[c] = err[c] + f[c] * co;
      }
#pragma unroll
      for (int c = 0; c < C; ++c) {
        const float etol = atol + rtol * fmaxf(fabsf(y[c]), fabsf(hin[c]));
        const float qv = err[c] / etol;
        ps[0] += (double)qv * qv;
      }
    }
    ODP_T1(12, te0)
    ot_batch_sum<1>(a, sh.dead, rep, ps, ps);
    ODP_T0(tc0)
    const float ratio = (float)rms_of(ps[0], NBC);
    const bool accept = ratio <= 1.0f;
    if (lead) {
      double* lg = a.alog + (size_t)n * ALOG_W;
      lg[ALOG_RATIO] = ratio;
      lg[ALOG_ACCEPT] = accept ? 1.0 : 0.0;
    }
    if (accept) {
#pragma unroll
      for (int c = 0; c < C; ++c) {
        yprev[c] = y[c];
        y[c] = hin[c];
      }
      kget(6, fcur);
      fidx = e - 1;
      dt32L = dt32;
      tprev = tcur;
      tnext = tcur + dt;
      tcur = tcur + dt;
      ++nacc;
    } else {
      ++nrej;
    }
    // _optimal_step_size (float64)
    if (ratio == 0.f) {
      dt = dt * DP_IFACTOR;
    } else {
      const double df = ratio < 1.0f ? 1.0 : DP_DFACTOR;
      dt = dt * fmin(DP_IFACTOR, fmax(DP_SAFETY / pow((double)ratio, 1.0 / 5.0), df));
    }
    ++n;
    ODP_T1(13, tc0)
#ifdef OT_PROFILE
    if (lead) atomicAdd(a.prof + 2, (unsigned long long)(wall_clock64() - ta0));
#endif
  }
  // ---- dense output at t1 (torchdiffeq _interp_evaluate of the last accepted step) -----------
  float out[C];
  if (status == 0 && nacc > 0 && !sh.dead) {
    const float x = (float)((tmax - tprev) / (tnext - tprev));
    float acc[C];
#pragma unroll
    for (int c = 0; c < C; ++c) acc[c] = 0.f;
#pragma unroll
    for (int jj = 0; jj < 7; ++jj) {
      float f[C];
      kget(jj, f);
      const float co = DP_CMID[jj] * dt32L;
#pragma unroll
      for (int c = 0; c < C; ++c) acc[c] = acc[c] + f[c] * co;
    }
    float fa[C], fb[C];
    kget(0, fa);
    kget(6, fb);
#pragma unroll
    for (int c = 0; c < C; ++c) {
      const float y0 = yprev[c], y1 = y[c], ym = y0 + acc[c];
      const float ci1 = dt32L * fa[c];
      const float ci2 = (((dt32L * (fb[c] - 4.0f * fa[c])) - 11.0f * y0) - 5.0f * y1) + 16.0f * ym;
      const float ci3 = (((dt32L * (5.0f * fa[c] - 3.0f * fb[c])) + 18.0f * y0) + 14.0f * y1) - 32.0f * ym;
      const float ci4 = ((2.0f * dt32L) * (fb[c] - fa[c]) - 8.0f * (y1 + y0)) + 16.0f * ym;
      float total = y0 + x * ci1;
      float xp = x * x;
      total = total + xp * ci2;
      xp = xp * x;
      total = total + xp * ci3;
      xp = xp * x;
      total = total + xp * ci4;
      out[c] = total;
    }
  } else {
#pragma unroll
    for (int c = 0; c < C; ++c) out[c] = __builtin_nanf("");   // failed solve: the loss turns NaN
  }
  if (p == 0 && valid && first) store_row10(a.y_out + (size_t)b * C, out);
  if (lead) {
    a.stats[0] = e;
    a.stats[1] = nacc;
    if (status) atomicMax(a.stats + 3, status);
    a.stats[4] = nacc;
    a.stats[5] = nrej;
    a.stats[6] = n;
    a.imeta[0] = e;
    a.imeta[1] = n;
    a.imeta[2] = status ? status : (sh.dead ? 4 : 0);
    a.imeta[3] = (int32_t)rep;       // next unused reduction epoch: the backward continues from it
  }
}
#undef ODP_T0
#undef ODP_T1

// ---- backward: the reverse sweep of oracle/dopri5_train.py dopri5_adjoint ---------------------
template <bool T4>
struct OdpBwdShared {
  std::conditional_t<T4, OtBwdShared4, OtBwdShared> ot;
  float gk[4][7][T4 ? TR4 : TR][C];       // [wave][stage][row][c]: adjoints of the attempt's k_0..k_6
  float kst[4][7][T4 ? TR4 : TR][C];      // [wave][stage][row][c]: the attempt's saved k_0..k_6
  double red[OT_XV];
  int dead;
};

template <bool SN, bool T4>
__global__ __launch_bounds__(256) void k_odp_bwd(OTArgs a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  constexpr int TRX = T4 ? TR4 : TR;
  OdpBwdShared<T4>& S = *reinterpret_cast<OdpBwdShared<T4>*>(smem);
  if (threadIdx.x == 0) S.dead = 0;
  const int lane = threadIdx.x & 63, q = lane >> 4, j = lane & (TRX - 1);
  const int p = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  std::conditional_t<T4, VjpW4, VjpW> wv;
  float q3t[8][3];                    // 16-row only (VjpW4 holds its own Q3^T operands)
  if constexpr (T4) {
    const int bq = lane >> 2, i = lane & 3;
    const int u = 32 * p + 4 * (bq & 7) + i;
#pragma unroll
    for (int s = 0; s < 5; ++s) wv.q3t[s] = a.Q3[(s + 5 * (bq >> 3)) * M + u];
#pragma unroll
    for (int s = 0; s < 64; ++s) wv.q2t[s] = a.Q2[(size_t)(s + 64 * (bq >> 3)) * M + u];
    const int c = 4 * (bq & 3) + i;
#pragma unroll
    for (int s = 0; s < 8; ++s) wv.q1t[s] = c < C ? a.Q1[(32 * p + 8 * (bq >> 2) + s) * C + c] : 0.f;
  } else {
#pragma unroll
    for (int o = 0; o < 2; ++o) {
#pragma unroll
      for (int hb = 0; hb < 8; ++hb)
#pragma unroll
        for (int t = 0; t < 4; ++t) wv.q2t[o][hb][t] = a.Q2[(16 * hb + 4 * q + t) * M + 16 * (2 * p + o) + j];
#pragma unroll
      for (int t = 0; t < 4; ++t) wv.q1t[o][t] = j < C ? a.Q1[(16 * (2 * p + o) + 4 * q + t) * C + j] : 0.f;
    }
#pragma unroll
    for (int hb = 0; hb < 8; ++hb)
#pragma unroll
      for (int s = 0; s < 3; ++s) q3t[hb][s] = 4 * s + q < C ? a.Q3[(4 * s + q) * M + 16 * hb + j] : 0.f;
  }
  const int b = blockIdx.x * TRX + j;
  const bool valid = b < a.B;
  const bool own = valid && (T4 ? lane < TR4 : q == 0);
  const int bb = valid ? b : a.B - 1;
  const int nfe = a.imeta[0], A = a.imeta[1];
  const bool failed = a.imeta[2] != 0 || A < 1;
  __syncthreads();
  float (*gks)[TRX][C] = S.gk[p];
  auto gadd = [&](int s, const float (&v)[C]) {
#pragma unroll
    for (int c = 0; c < C; ++c) gks[s][j][c] += v[c];
  };
  auto gget = [&](int s, float (&v)[C]) {
#pragma unroll
    for (int c = 0; c < C; ++c) v[c] = gks[s][j][c];
  };
  auto krow = [&](int e, float (&v)[C]) { load_row10(a.vw + ((size_t)bb * a.E + e) * C, v); };
  // the attempt's stage derivatives, staged in LDS once per attempt (loads issued together): read
  // from global memory term by term they cost one dependent L2 round trip each, ~28 per attempt
  float (*kss)[TRX][C] = S.kst[p];
  auto kstage = [&](int fidx, int e0) {
    float t[7][C];
#pragma unroll
    for (int jj = 0; jj < 7; ++jj) krow(jj == 0 ? fidx : e0 + jj - 1, t[jj]);
#pragma unroll
    for (int jj = 0; jj < 7; ++jj)
#pragma unroll
      for (int c = 0; c < C; ++c) kss[jj][j][c] = t[jj][c];
  };
  auto kget = [&](int s, float (&v)[C]) {
#pragma unroll
    for (int c = 0; c < C; ++c) v[c] = kss[s][j][c];
  };
  float gout[C];
  if (valid) load_row10(a.g_y + (size_t)b * C, gout);
  else
#pragma unroll
    for (int c = 0; c < C; ++c) gout[c] = 0.f;
  if (failed)
#pragma unroll
    for (int c = 0; c < C; ++c) gout[c] = __builtin_nanf("");     // a failed forward: NaN gradients
  const double NBC = (double)a.B * C;
  const float rtol = (float)a.rtol, atol = (float)a.atol;
  // the reduction granules still hold the forward's last tags (and a previous sweep's on the same
  // workspace): continue the epoch sequence where the last user of the workspace left it, so no
  // stale granule can carry a current tag.  Every workgroup reads imeta[3] before its first
  // exchange; workgroup 0 advances it only after its last exchange completed, which no workgroup
  // passes before all have published theirs (end of the kernel).
  unsigned rep = (unsigned)a.imeta[3];
  if (rep == 0u) rep = 1u;
  int buf = 0;
  std::conditional_t<T4, VjpIn4, VjpIn> cur, nxt;
  VjpRow crw, nrw;
  int ecur = nfe - 1;
  if constexpr (T4) load_vjp_in4(a, p, ecur, b, valid, lane, cur);
  else load_vjp_in(a, p, ecur, b, valid, q, cur);
  vjp_row_math<SN>(a, cur, crw);
  // evals visited nfe-1, nfe-2, ..., 0 (attempts in reverse, stages 5..0; then evals 1, 0)
#ifdef OT_PROFILE
#define ODB_T0(V) const uint64_t V = wall_clock64();
#define ODB_T1(SLOT, V) if (blockIdx.x == 0 && threadIdx.x == 0) atomicAdd(a.prof + (SLOT), (unsigned long long)(wall_clock64() - V));
#else
#define ODB_T0(V)
#define ODB_T1(SLOT, V)
#endif
  auto vjp = [&](const float (&g)[C], float (&gY)[C]) {
    ODB_T0(tv0)
    if constexpr (T4) {
      load_vjp_in4(a, p, ecur - 1, b, valid, lane, nxt);
      ot_vjp4<SN>(a, wv, S.ot, buf, p, ecur, b, valid, lane, j, cur, crw, g, gY);
      cur = nxt;
      vjp_row_math<SN>(a, cur, crw);
    } else {
      load_vjp_in(a, p, ecur - 1, b, valid, q, nxt);
      ot_vjp<SN>(a, wv, q3t, S.ot, buf, p, ecur, b, valid, lane, q, j, cur, crw, nxt, nrw, g, gY);
      cur = nxt;
      crw = nrw;
    }
    buf ^= 1;
    --ecur;
    ODB_T1(1, tv0)
  };
  float gy[C], gf[C];
#pragma unroll
  for (int c = 0; c < C; ++c) gy[c] = gf[c] = 0.f;
  double g_dt_next = 0.0, g_t_next = 0.0;
  for (int n = A - 1; n >= 0; --n) {
#ifdef OT_PROFILE
    const uint64_t tb0 = wall_clock64();
#endif
    const double* lg = a.alog + (size_t)n * ALOG_W;
    const double tn = lg[ALOG_T], dtn = lg[ALOG_DT];
    const float ratio = (float)lg[ALOG_RATIO];
    const bool accept = lg[ALOG_ACCEPT] != 0.0;
    const int fidx = (int)lg[ALOG_FIDX], e0 = (int)lg[ALOG_E0];
    const float dts = (float)dtn;
    ODB_T0(tk0)
    kstage(fidx, e0);
    // controller: dt_{n+1} = dt_n * factor(ratio_n)
    double fac, dfac = 0.0;
    if (ratio == 0.f) {
      fac = DP_IFACTOR;
    } else {
      const double df = ratio < 1.0f ? 1.0 : DP_DFACTOR;
      const double mid = DP_SAFETY / pow((double)ratio, 1.0 / 5.0);
      fac = fmin(DP_IFACTOR, fmax(mid, df));
      if (mid > df && mid < DP_IFACTOR) dfac = -0.2 * mid / (double)ratio;
    }
    const double g_ratio = g_dt_next * dtn * dfac;
    double g_dt = g_dt_next * fac;
    const bool last = n == A - 1;
    // rows
#pragma unroll
    for (int s = 0; s < 7; ++s)
#pragma unroll
      for (int c = 0; c < C; ++c) gks[s][j][c] = 0.f;
    float yn[C], ynew[C], g_yn[C], g_ynew[C];
    load_row10(a.ys + ((size_t)n * a.B + bb) * C, yn);
    load_row10(a.hs + ((size_t)bb * a.E + e0 + 5) * C, ynew);
#pragma unroll
    for (int c = 0; c < C; ++c) {
      g_yn[c] = accept ? 0.f : gy[c];
      g_ynew[c] = accept ? gy[c] : 0.f;
    }
    if (accept) gadd(6, gf);
    else gadd(0, gf);
    double pdt = 0.0, px = 0.0;
    float x = 0.f;
    double x64 = 0.0;
    if (last) {                      // the output: y_hat = interpolant of this attempt at x
      x64 = (a.t1d - tn) / ((tn + dtn) - tn);
      x = (float)x64;
      float ym[C], fa[C], fb[C];
#pragma unroll
      for (int c = 0; c < C; ++c) ym[c] = 0.f;
      for (int jj = 0; jj < 7; ++jj) {
        float f[C];
        kget(jj, f);
        const float co = DP_CMID[jj] * dts;
#pragma unroll
        for (int c = 0; c < C; ++c) ym[c] = ym[c] + f[c] * co;
      }
      kget(0, fa);
      kget(6, fb);
      const float x2 = x * x, x3 = x2 * x, x4 = x3 * x;
      float g_ym[C], gfa[C], gfb[C];
#pragma unroll
      for (int c = 0; c < C; ++c) {
        const float y0 = yn[c], y1 = ynew[c], yc = y0 + ym[c];
        const float cd = dts * fa[c];
        const float cc = (((dts * (fb[c] - 4.0f * fa[c])) - 11.0f * y0) - 5.0f * y1) + 16.0f * yc;
        const float cb = (((dts * (5.0f * fa[c] - 3.0f * fb[c])) + 18.0f * y0) + 14.0f * y1) - 32.0f * yc;
        const float ca = ((2.0f * dts) * (fb[c] - fa[c]) - 8.0f * (y1 + y0)) + 16.0f * yc;
        const float go = gout[c];
        px += (double)go * ((double)cd + 2.0 * x * cc + 3.0 * (double)x2 * cb + 4.0 * (double)x3 * ca);
        const float ga = go * x4, gb = go * x3, gc = go * x2, gd = go * x;
        g_ym[c] = (16.0f * ga - 32.0f * gb) + 16.0f * gc;
        g_yn[c] += ((((go - 8.0f * ga) + 18.0f * gb) - 11.0f * gc)) + g_ym[c];
        g_ynew[c] += (-8.0f * ga + 14.0f * gb) - 5.0f * gc;
        gfa[c] = dts * (((-2.0f * ga + 5.0f * gb) - 4.0f * gc) + gd);
        gfb[c] = dts * ((2.0f * ga - 3.0f * gb) + gc);
        pdt += (double)ga * 2.0 * (fb[c] - fa[c]) + (double)gb * (5.0 * fa[c] - 3.0 * fb[c]) +
               (double)gc * (fb[c] - 4.0 * fa[c]) + (double)gd * fa[c];
      }
      for (int jj = 0; jj < 7; ++jj) {
        float f[C], t[C];
        kget(jj, f);
        const float co = DP_CMID[jj] * dts;
#pragma unroll
        for (int c = 0; c < C; ++c) {
          t[c] = g_ym[c] * co;
          pdt += (double)g_ym[c] * f[c] * DP_CMID[jj];
        }
        gadd(jj, t);
      }
      gadd(0, gfa);
      gadd(6, gfb);
    }
    ODB_T1(5, tk0)
    ODB_T0(tr0)
    if (g_ratio != 0.0) {            // ratio = rms(err / etol), etol = atol + rtol max(|y_n|, |y_new|)
      float err[C];
#pragma unroll
      for (int c = 0; c < C; ++c) err[c] = 0.f;
      float kk[7][C];
      for (int jj = 0; jj < 7; ++jj) {
        kget(jj, kk[jj]);
        const float co = DP_CERR[jj] * dts;
#pragma unroll
        for (int c = 0; c < C; ++c) err[c] = err[c] + kk[jj][c] * co;
      }
      float g_err[C];
#pragma unroll
      for (int c = 0; c < C; ++c) {
        const float etol = atol + rtol * fmaxf(fabsf(yn[c]), fabsf(ynew[c]));
        const double qv = (double)err[c] / etol;
        const double gq = g_ratio * qv / (NBC * (double)ratio);
        g_err[c] = (float)(gq / etol);
        const float g_etol = (float)(-gq * qv / etol);
        if (fabsf(yn[c]) >= fabsf(ynew[c])) g_yn[c] += g_etol * rtol * (yn[c] > 0.f ? 1.f : (yn[c] < 0.f ? -1.f : 0.f));
        else g_ynew[c] += g_etol * rtol * (ynew[c] > 0.f ? 1.f : (ynew[c] < 0.f ? -1.f : 0.f));
      }
      for (int jj = 0; jj < 7; ++jj) {
        float t[C];
        const float co = DP_CERR[jj] * dts;
#pragma unroll
        for (int c = 0; c < C; ++c) {
          t[c] = g_err[c] * co;
          pdt += (double)g_err[c] * kk[jj][c] * DP_CERR[jj];
        }
        gadd(jj, t);
      }
    }
    ODB_T1(4, tr0)
    // stages in reverse: k_{i+1} = f(Y_i), Y_i = y_n + sum_{j <= i} k_j beta_ij dt; y_new = Y_5
    for (int i = 5; i >= 0; --i) {
      float g[C], gY[C];
      gget(i + 1, g);
      vjp(g, gY);
      ODB_T0(tj0)
      if (i == 5)
#pragma unroll
        for (int c = 0; c < C; ++c) gY[c] += g_ynew[c];
#pragma unroll
      for (int c = 0; c < C; ++c) g_yn[c] += gY[c];
#pragma unroll
      for (int jj = 0; jj < 6; ++jj) {
        if (jj <= i) {          // (uniform)
          float f[C], t[C];
          kget(jj, f);
          const float co = DP_BETA[i][jj] * dts;
#pragma unroll
          for (int c = 0; c < C; ++c) {
            t[c] = gY[c] * co;
            pdt += (double)gY[c] * f[c] * DP_BETA[i][jj];
          }
          gadd(jj, t);
        }
      }
      ODB_T1(3, tj0)
    }
    double red[2] = {own ? pdt : 0.0, own ? px : 0.0};
    ot_batch_sum_bwd<2>(a, S.red, S.dead, rep, red, red);
    g_dt += red[0];
    double g_t;
    if (last) {
      g_dt += -red[1] * x64 / dtn;   // x = (t1 - t_n) / (t_n + dt_n - t_n)
      g_t = -red[1] / dtn;
    } else {
      g_t = g_t_next;
      if (accept) g_dt += g_t_next;  // t_{n+1} = t_n + dt_n
    }
    g_t_next = g_t;
    g_dt_next = g_dt;
#pragma unroll
    for (int c = 0; c < C; ++c) gy[c] = g_yn[c];
    gget(0, gf);
#ifdef OT_PROFILE
    if (blockIdx.x == 0 && threadIdx.x == 0) atomicAdd(a.prof + 0, (unsigned long long)(wall_clock64() - tb0));
#endif
  }
  // ---- the initial step: dt_0 = min(100 h0, h1) -----------------------------------------------
  const double d1 = a.meta[META_D1], d2 = a.meta[META_D2], h0 = a.meta[META_H0], h1 = a.meta[META_H1];
  const double r2 = a.meta[META_R2];
  const bool clamp0 = a.meta[META_CLAMP0] != 0.0, clamp1 = a.meta[META_CLAMP1] != 0.0;
  double g_h0 = (100.0 * h0 <= h1) ? g_dt_next * 100.0 : 0.0;
  const double g_h1 = (h1 < 100.0 * h0) ? g_dt_next : 0.0;
  double g_d1 = 0.0, g_d2 = 0.0;
  if (clamp1) {
    if (h0 * 1e-3 > 1e-6) g_h0 += 1e-3 * g_h1;
  } else {
    const bool m2 = d2 > d1;
    const double m = m2 ? d2 : d1;
    const double g_m = g_h1 * (-0.2) * h1 / m;
    if (m2) g_d2 += g_m;
    else g_d1 += g_m;
  }
  const double g_r2 = g_d2 / h0;     // d2 = r2 / h0
  g_h0 += -g_d2 * d2 / h0;
  float y0[C], f0[C], f1[C], gf1[C], gf0[C];
  load_row10(a.hs + ((size_t)bb * a.E + 0) * C, y0);
  krow(0, f0);
  krow(1, f1);
#pragma unroll
  for (int c = 0; c < C; ++c) {
    const float sc = atol + fabsf(y0[c]) * rtol;
    const float wv_ = (f1[c] - f0[c]) / sc;
    const float gw = r2 > 0.0 ? (float)(g_r2 * wv_ / (NBC * r2)) : 0.f;
    gf1[c] = gw / sc;
    gf0[c] = gf[c] - gw / sc;
  }
  float gyi[C];
  vjp(gf1, gyi);                     // eval 1: f1 = f(y0 + h0 f0)
  double sh0 = 0.0;
#pragma unroll
  for (int c = 0; c < C; ++c) {
    gf0[c] += (float)h0 * gyi[c];
    sh0 += (double)gyi[c] * f0[c];
  }
  double red1[1] = {own ? sh0 : 0.0};
  ot_batch_sum_bwd<1>(a, S.red, S.dead, rep, red1, red1);
  g_h0 += red1[0];
  if (!clamp0) g_d1 += -g_h0 * h0 / d1;   // h0 = 0.01 d0 / d1
#pragma unroll
  for (int c = 0; c < C; ++c) {
    const float sc = atol + fabsf(y0[c]) * rtol;
    gf0[c] += (float)((g_d1 * ((double)f0[c] / sc) / (NBC * d1)) / sc);
  }
  float gy0[C];
  vjp(gf0, gy0);                     // eval 0: f0 = f(y0)
  (void)gy0;
  // Only a sweep whose every exchange completed advances the epoch word: then every workgroup has
  // published its last exchange, whose tag was computed from the imeta[3] it read at the start, so
  // no workgroup can still read the word after this store.  A sweep with a timed-out exchange (its
  // outputs are NaN) moves the word far past any tag it may have written, so a later sweep on the
  // same workspace cannot match them.
  if (blockIdx.x == 0 && threadIdx.x == 0 && !S.dead) a.imeta[3] = (int32_t)rep;
  if (threadIdx.x == 0 && S.dead) atomicMax(a.imeta + 3, (int32_t)(rep + 65536u));
}
#undef ODB_T0
#undef ODB_T1

inline size_t al(size_t x) { return (x + 255) & ~(size_t)255; }

int grid_iters(const fiode_odetrain_config* cfg) {
  const float t0 = (float)cfg->t0, t1 = (float)cfg->t1, h = (float)cfg->step_size;
  if (!(h > 0.f) || !(t1 > t0)) return -1;
  const float n = ceilf((t1 - t0) / h + 1.0f);
  if (!(n >= 2.f) || n > 1025.f) return -1;
  return (int)n;
}

// the solve's shape: E evals (rk4) or the eval capacity 2 + 6 A (dopri5); -1 if invalid
int solve_shape(const fiode_odetrain_config* cfg, int& E, int& A, int& niters) {
  if (cfg->method == FIODE_ODE_DOPRI5) {
    if (cfg->max_attempts < 1 || cfg->max_attempts > FIODE_ODETRAIN_MAX_ATTEMPTS) return -1;
    if (!(cfg->rtol > 0.0) || !(cfg->atol > 0.0) || !(cfg->t1 > cfg->t0)) return -1;
    A = cfg->max_attempts;
    E = 2 + 6 * A;
    niters = 0;
    return 0;
  }
  if (cfg->method != FIODE_ODE_RK4) return -1;
  const int n = grid_iters(cfg);
  if (n < 0) return -1;
  niters = n;
  E = 4 * (n - 1);
  A = 0;
  return 0;
}

struct OtLayout {
  size_t u, y, k, hs, ftw, vw, muw, nomw, loww, a1, a2, gz2, gz1, gft, xs, xr, kw, wg, ys, alog, meta, imeta, total;
};
// E: evals (rk4) or the eval capacity 2 + 6 A (dopri5, A > 0: attempt capacity)
OtLayout ot_layout(int B, int E, int A = 0) {
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
  L.loww = o; o += al(R * C * 4);
  L.a1 = o; o += al(R * M * 4);
  L.a2 = o; o += al(R * M * 4);
  L.gz2 = o; o += al(R * M * 4);
  L.gz1 = o; o += al(R * M * 4);
  L.gft = o; o += al(R * C * 4);
  const size_t nt4 = (size_t)(B + TR4 - 1) / TR4;     // 4-row tiles (>= the 16-row kernel's tiles)
  L.xs = o; o += (size_t)OT_XRING * 2 * nt4 * 8 * OT4_XSTRIDE + 1024;   // the reduction granules follow: one clear for both
  L.xr = o; o += al(A > 0 ? 2 * nt4 * 2 * OT_XV * 8 : 0);
  L.kw = o; o += al((size_t)E * 2 * B * 16);
  L.wg = o; o += al(fiode_internal::wgrad_bytes(B, E, A == 0));
  L.ys = o; o += al((size_t)A * B * C * 4);
  L.alog = o; o += al((size_t)A * ALOG_W * 8);
  L.meta = o; o += al(META_N * 8);
  L.imeta = o; o += al(8 * 4);
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
  int E, A, n;
  if (solve_shape(cfg, E, A, n) < 0) return FIODE_EINVAL;
  a.B = cfg->batch; a.niters = n; a.E = E; a.A = A; a.method = cfg->method;
  a.rtol = cfg->rtol; a.atol = cfg->atol; a.t0d = cfg->t0; a.t1d = cfg->t1;
  const OtLayout L = ot_layout(a.B, a.E, a.A);
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
  a.loww = reinterpret_cast<float*>(ws + L.loww);
  a.a1 = reinterpret_cast<float*>(ws + L.a1);
  a.a2 = reinterpret_cast<float*>(ws + L.a2);
  a.gz2 = reinterpret_cast<float*>(ws + L.gz2);
  a.gz1 = reinterpret_cast<float*>(ws + L.gz1);
  a.gft = reinterpret_cast<float*>(ws + L.gft);
  a.xslots = reinterpret_cast<unsigned long long*>(ws + L.xs);
  a.xr = reinterpret_cast<unsigned long long*>(ws + L.xr);
  a.kw = reinterpret_cast<uint32_t*>(ws + L.kw);
  a.ys = reinterpret_cast<float*>(ws + L.ys);
  a.alog = reinterpret_cast<double*>(ws + L.alog);
  a.meta = reinterpret_cast<double*>(ws + L.meta);
  a.imeta = reinterpret_cast<int32_t*>(ws + L.imeta);
#ifdef OT_PROFILE
  a.prof = reinterpret_cast<unsigned long long*>(ws + L.xs) + (size_t)OT_XRING * 2 * ((a.B + TR4 - 1) / TR4) * OT4_XSTRIDE + 8;
#endif
  return FIODE_OK;
}

// the adjoint sweep (weight operands in registers: VjpW): rk4 k_ot_bwd, dopri5 k_odp_bwd
hipError_t launch_sweep(const OTArgs& a, hipStream_t st) {
  const dim3 grid((a.B + TR - 1) / TR);
  const bool t4 = (a.B + TR4 - 1) / TR4 <= FIODE_OT4_MAX_TILES;
  const dim3 grid4((a.B + TR4 - 1) / TR4);
  if (a.method == FIODE_ODE_DOPRI5) {
    if (t4) {
      if (a.d.scale_nominal) hipLaunchKernelGGL((k_odp_bwd<true, true>), grid4, dim3(256), sizeof(OdpBwdShared<true>), st, a);
      else hipLaunchKernelGGL((k_odp_bwd<false, true>), grid4, dim3(256), sizeof(OdpBwdShared<true>), st, a);
    } else {
      if (a.d.scale_nominal) hipLaunchKernelGGL((k_odp_bwd<true, false>), grid, dim3(256), sizeof(OdpBwdShared<false>), st, a);
      else hipLaunchKernelGGL((k_odp_bwd<false, false>), grid, dim3(256), sizeof(OdpBwdShared<false>), st, a);
    }
  } else if (t4) {
    if (a.d.scale_nominal) hipLaunchKernelGGL(k_ot_bwd4<true>, grid4, dim3(256), sizeof(OtBwdShared4), st, a);
    else hipLaunchKernelGGL(k_ot_bwd4<false>, grid4, dim3(256), sizeof(OtBwdShared4), st, a);
  } else {
    if (a.d.scale_nominal) hipLaunchKernelGGL(k_ot_bwd<true>, grid, dim3(256), sizeof(OtBwdShared), st, a);
    else hipLaunchKernelGGL(k_ot_bwd<false>, grid, dim3(256), sizeof(OtBwdShared), st, a);
  }
  return hipGetLastError();
}

}  // namespace

extern "C" int32_t fiode_odetrain_evals(const fiode_odetrain_config* cfg) {
  if (!cfg) return -1;
  int E, A, n;
  return solve_shape(cfg, E, A, n) < 0 ? -1 : E;
}

extern "C" size_t fiode_odetrain_workspace_bytes(const fiode_odetrain_config* cfg) {
  if (!cfg || cfg->batch <= 0) return 0;
  int E, A, n;
  if (solve_shape(cfg, E, A, n) < 0) return 0;
  return ot_layout(cfg->batch, E, A).total;
}

extern "C" int fiode_odetrain_saved_offsets(const fiode_odetrain_config* cfg, int64_t* offsets) {
  if (!cfg || !offsets || cfg->batch <= 0) return FIODE_EINVAL;
  int E, A, n;
  if (solve_shape(cfg, E, A, n) < 0) return FIODE_EINVAL;
  const OtLayout L = ot_layout(cfg->batch, E, A);
  const size_t o[FIODE_ODETRAIN_NSAVED] = {L.hs, L.ftw, L.vw, L.muw, L.nomw, L.a1, L.a2, L.gft, L.loww,
                                           A ? L.ys : 0, A ? L.alog : 0, A ? L.meta : 0, L.imeta + 2 * 4, L.kw};
  for (int i = 0; i < FIODE_ODETRAIN_NSAVED; ++i) offsets[i] = (int64_t)o[i];
  return FIODE_OK;
}

extern "C" int fiode_odetrain_forward(void* stream, const fiode_odetrain_config* cfg, const fiode_dyn_config* dyn,
                                      const fiode_dyn_weights* w, const float* x_feat, const float* h0,
                                      const uint8_t* masks, const uint64_t* offset_dev, float* y_out, int32_t* stats,
                                      void* workspace, size_t workspace_bytes) {
  OTArgs a{};
  a.prio = (int)g_fiode_prio_mask;
  int rc = fill_args(a, cfg, dyn, w, x_feat, workspace, workspace_bytes);
  if (rc) return rc;
  if (!h0 || !y_out || !stats) return FIODE_EINVAL;
  if (a.dropout_mode == FIODE_DROPOUT_GIVEN && !masks) return FIODE_EINVAL;
  a.h0 = h0; a.masks = masks; a.offset_dev = offset_dev; a.y_out = y_out; a.stats = stats;
  a.drop_block = fiode_internal::debug_drop_publish();
  hipStream_t st = static_cast<hipStream_t>(stream);
  const int ntiles = (a.B + TR - 1) / TR;
  // k_ot_masks zeroes the exchange granules (tags) and the status words before every forward, and
  // draws the dropout keep words when dropout is on
  const OtLayout L = ot_layout(a.B, a.E, a.A);
  a.nslots = (int)((L.kw - L.xs) / 8);
  a.kw_lazy = a.method == FIODE_ODE_DOPRI5 && a.dropout_mode == FIODE_DROPOUT_PHILOX && a.bit_mode;
  // a dopri5 solve's first evals (a B = 128 step takes ~150) are drawn up front, off the solve's
  // dependent chain (the lazy draw cost 0.4 us per eval there); the rest of the capacity lazily
  a.kw_pre = a.kw_lazy ? std::min(a.E, FIODE_OT_KW_PRE) : a.E;
  const int nthreads = std::max(a.nslots, a.kw_pre * a.B);
  hipLaunchKernelGGL(k_ot_masks, dim3((nthreads + 255) / 256), dim3(256), 0, st, a);
  FIODE_HIP_CHECK(hipGetLastError());
  if (a.method == FIODE_ODE_DOPRI5) {
    if ((a.B + TR4 - 1) / TR4 <= FIODE_OT4_MAX_TILES)
      hipLaunchKernelGGL(k_odp_fwd<true>, dim3((a.B + TR4 - 1) / TR4), dim3(256), sizeof(OdpShared<true>), st, a);
    else
      hipLaunchKernelGGL(k_odp_fwd<false>, dim3(ntiles), dim3(256), sizeof(OdpShared<false>), st, a);
  } else if ((a.B + TR4 - 1) / TR4 <= FIODE_OT4_MAX_TILES) {
    // 4-row tiles (tile4.h T4W: weights in registers)
    hipLaunchKernelGGL(k_ot_fwd4, dim3((a.B + TR4 - 1) / TR4), dim3(256), sizeof(OtShared4), st, a);
  } else {
    // the weights live in registers (tile16.h T16W)
    hipLaunchKernelGGL(k_ot_fwd, dim3(ntiles), dim3(256), sizeof(OtShared), st, a);
  }
  FIODE_HIP_CHECK(hipGetLastError());
  return FIODE_OK;
}

namespace {
// dL/dx_feat of the solve straight from the per-row layer-1 gradients k_ot_bwd leaves in the
// workspace: g_u[b][m] = sum_e gz1[b E + e][m] (e ascending), gx[b][x] = sum_m g_u[b][m] Qx[m][x]
// (m ascending, fused multiply-adds as k_lyap_static_grads), then optionally + add[b][x] * scale[0]
// (the other loss term's x_feat gradient and its upstream scale: the combined gradient in one
// launch).  One workgroup per image, one thread per hidden unit.
__global__ __launch_bounds__(M) void k_ot_gx(int E, const int32_t* __restrict__ e_used, const float* __restrict__ gz1,
                                             const float* __restrict__ Qx, const float* __restrict__ add,
                                             const float* __restrict__ scale, float* __restrict__ gx) {
  __shared__ float gu[M];
  const int b = blockIdx.x, m = threadIdx.x;
  const float* p = gz1 + (size_t)b * E * M + m;
  const int En = e_used ? min(E, e_used[0]) : E;     // dopri5: the evals the solve made
  float s = 0.f;
#pragma unroll 8
  for (int e = 0; e < En; ++e) s += p[(size_t)e * M];
  gu[m] = s;
  __syncthreads();
  if (m < FIODE_X) {
    float d = 0.f;
#pragma unroll 16
    for (int i = 0; i < M; ++i) d = __fmaf_rn(gu[i], Qx[i * FIODE_X + m], d);
    if (add) d = d + add[(size_t)b * FIODE_X + m] * scale[0];
    gx[(size_t)b * FIODE_X + m] = d;
  }
}
}  // namespace

extern "C" int fiode_odetrain_backward_x(void* stream, const fiode_odetrain_config* cfg, const fiode_dyn_config* dyn,
                                         const fiode_dyn_weights* w, const float* x_feat, const float* g_y,
                                         float* gx, const float* gx_add, const float* gx_add_scale, float* dbg_gft,
                                         void* workspace, size_t workspace_bytes) {
  OTArgs a{};
  a.prio = (int)g_fiode_prio_mask;
  int rc = fill_args(a, cfg, dyn, w, x_feat, workspace, workspace_bytes);
  if (rc) return rc;
  if (!g_y || !gx || (gx_add && !gx_add_scale)) return FIODE_EINVAL;
  a.g_y = g_y; a.dbg_gft = dbg_gft;
  hipStream_t st = static_cast<hipStream_t>(stream);
  FIODE_HIP_CHECK(launch_sweep(a, st));
  hipLaunchKernelGGL(k_ot_gx, dim3(a.B), dim3(M), 0, st, a.E, a.method == FIODE_ODE_DOPRI5 ? (const int32_t*)a.imeta : nullptr,
                     (const float*)a.gz1, w->Qx, gx_add, gx_add_scale, gx);
  FIODE_HIP_CHECK(hipGetLastError());
  return FIODE_OK;
}

extern "C" int fiode_odetrain_backward_weights(void* stream, const fiode_odetrain_config* cfg,
                                               const fiode_dyn_config* dyn, const fiode_dyn_weights* w,
                                               const float* x_feat, fiode_lyap_grads* grads, void* workspace,
                                               size_t workspace_bytes) {
  OTArgs a{};
  a.prio = (int)g_fiode_prio_mask;
  int rc = fill_args(a, cfg, dyn, w, x_feat, workspace, workspace_bytes);
  if (rc) return rc;
  if (!grads || !grads->Q1 || !grads->b1 || !grads->Qx || !grads->bx || !grads->Q2 || !grads->b2 || !grads->Q3 ||
      !grads->b3)
    return FIODE_EINVAL;
  const OtLayout L = ot_layout(a.B, a.E, a.A);
  fiode_internal::WgradIO io{};
  io.B = a.B; io.S = a.E; io.x_feat = x_feat; io.Qx = w->Qx; io.h = a.hs; io.a1 = a.a1; io.a2 = a.a2;
  io.s_used = a.method == FIODE_ODE_DOPRI5 ? a.imeta : nullptr;     // the evals the solve made
  io.gz2 = a.gz2; io.gz1 = a.gz1; io.gft = a.gft;
  io.workspace = static_cast<char*>(workspace) + L.wg;
  io.grads = *grads;
  io.grads.x_feat = nullptr;                  // dL/dx_feat: fiode_odetrain_backward_x
  return fiode_internal::launch_wgrad(static_cast<hipStream_t>(stream), io);
}

extern "C" int fiode_odetrain_backward(void* stream, const fiode_odetrain_config* cfg, const fiode_dyn_config* dyn,
                                       const fiode_dyn_weights* w, const float* x_feat, const float* g_y,
                                       fiode_lyap_grads* grads, float* dbg_gft, void* workspace,
                                       size_t workspace_bytes) {
  // the adjoint sweep, then the weight-gradient chain whose last kernel also forms dL/dx_feat (from
  // the per-image g_u it reduces): one launch fewer than _x + _weights (k_ot_gx), so the x-gradient
  // may differ from fiode_odetrain_backward_x's in the last bits (summation order of g_u)
  OTArgs a{};
  a.prio = (int)g_fiode_prio_mask;
  int rc = fill_args(a, cfg, dyn, w, x_feat, workspace, workspace_bytes);
  if (rc) return rc;
  if (!g_y || !grads || !grads->Q1 || !grads->b1 || !grads->Qx || !grads->bx || !grads->Q2 || !grads->b2 ||
      !grads->Q3 || !grads->b3 || !grads->x_feat)
    return FIODE_EINVAL;
  a.g_y = g_y; a.dbg_gft = dbg_gft;
  hipStream_t st = static_cast<hipStream_t>(stream);
  FIODE_HIP_CHECK(launch_sweep(a, st));
  const OtLayout L = ot_layout(a.B, a.E, a.A);
  fiode_internal::WgradIO io{};
  io.B = a.B; io.S = a.E; io.x_feat = x_feat; io.Qx = w->Qx; io.h = a.hs; io.a1 = a.a1; io.a2 = a.a2;
  io.s_used = a.method == FIODE_ODE_DOPRI5 ? a.imeta : nullptr;     // the evals the solve made
  io.gz2 = a.gz2; io.gz1 = a.gz1; io.gft = a.gft;
  io.workspace = static_cast<char*>(workspace) + L.wg;
  io.grads = *grads;
  return fiode_internal::launch_wgrad(st, io);
}

// ---- the train_ode loss term: F.nll_loss(torch.log(y_hat), y) (pl_modules.py:494-497) --------
// One workgroup: loss = -(1/B) sum_b log y_hat[b, y_b] (fixed-order block sum) and its gradient
// per unit upstream gradient, g[b][c] = -1 / (B y_hat[b, y_b]) at c = y_b, else 0.  A label outside
// [0, C) makes the loss NaN (torch raises a device assert there).
namespace {
// mix (nullable): the combined loss of pl_modules.py:500, mix[0] = lyap * (1 - p) + loss_ode * p
// (the two float32 products rounded, then the sum, as torch evaluates it), and gunit scaled by p.
__global__ __launch_bounds__(256) void k_ode_nll(int B, const float* __restrict__ y_hat, const int64_t* __restrict__ y,
                                                 float* __restrict__ loss, float* __restrict__ gunit,
                                                 const float* __restrict__ lyap, float p, float* __restrict__ mix) {
  __shared__ float red[256];
  const int tid = threadIdx.x;
  float s = 0.f;
  for (int b = tid; b < B; b += 256) {
    const int64_t l = y[b];
    const bool ok = l >= 0 && l < C;
    const float v = ok ? y_hat[(size_t)b * C + l] : __builtin_nanf("");
    s = s + (-logf(v));
    const float g0 = -1.0f / ((float)B * v);
    const float g = mix ? g0 * p : g0;
#pragma unroll
    for (int c = 0; c < C; ++c) gunit[(size_t)b * C + c] = (c == l) ? g : 0.f;
  }
  red[tid] = s;
  __syncthreads();
#pragma unroll
  for (int o = 128; o > 0; o >>= 1) {
    if (tid < o) red[tid] = red[tid] + red[tid + o];
    __syncthreads();
  }
  if (tid == 0) {
    const float lo = red[0] / (float)B;
    loss[0] = lo;
    if (mix) mix[0] = lyap[0] * (1.0f - p) + lo * p;
  }
}
}  // namespace

extern "C" int fiode_ode_nll(void* stream, int32_t batch, const float* y_hat, const int64_t* labels, float* loss,
                             float* g_unit) {
  if (batch <= 0 || !y_hat || !labels || !loss || !g_unit) return FIODE_EINVAL;
  hipLaunchKernelGGL(k_ode_nll, dim3(1), dim3(256), 0, static_cast<hipStream_t>(stream), batch, y_hat, labels, loss,
                     g_unit, nullptr, 0.0f, nullptr);
  FIODE_HIP_CHECK(hipGetLastError());
  return FIODE_OK;
}

extern "C" int fiode_ode_loss_mix(void* stream, int32_t batch, const float* y_hat, const int64_t* labels,
                                  const float* lyap_loss, float portion, float* loss_ode, float* total, float* g_unit) {
  if (batch <= 0 || !y_hat || !labels || !lyap_loss || !loss_ode || !total || !g_unit) return FIODE_EINVAL;
  hipLaunchKernelGGL(k_ode_nll, dim3(1), dim3(256), 0, static_cast<hipStream_t>(stream), batch, y_hat, labels,
                     loss_ode, g_unit, lyap_loss, portion, total);
  FIODE_HIP_CHECK(hipGetLastError());
  return FIODE_OK;
}
