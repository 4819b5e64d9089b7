// Eval-mode ODE solves of the Cayley-MLP dynamics on gfx950: replaces torchdiffeq.odeint at
// models.py:235-241 (IVP.integrate) for method 'rk4' (fixed grid, 3/8 rule) and 'dopri5'
// (adaptive, torchdiffeq 0.2.2 semantics).  f(h) = eval_dot in eval mode
// (dynamics/classification.py:104-132) with the QP's batch-global exit over the B rows of each
// stage, exactly as every func() call of odeint sees it (validation forward: pl_modules.py:322-325).
//
// Tile-parallel persistent design (the train_ode forward's, odetrain.hip / tile16.h): the batch is
// cut into 16-row tiles, one workgroup owns T consecutive tiles (T = 1 while the tiles fit the
// chip's resident workgroups: B <= 4096 on 256 CUs), and inside a tile the 128 hidden units are
// split over the 4 waves (v_mfma_f32_16x16x4_f32).  The solve has three batch-wide couplings, all
// exchanged between workgroups through tagged 8-byte granules (one agent-scope atomic store per
// granule, relaxed agent-scope polls, bounded spins; tile16.h):
//   * every eval's QP exit -- the lowest iteration at which ALL rows met tol
//     (barrier_projection.py:247-249) -- as the AND of per-workgroup convergence masks, with the
//     train_ode forward's speculation (bisect to the previous exit + 3 first);
//   * dopri5's error ratio -- ONE RMS norm over the whole (B, C) state (torchdiffeq _rms_norm) --
//     and the three norms of the initial-step selection, as float64 partial sums that every
//     workgroup adds in the same (workgroup) order, so every workgroup takes the same
//     accept / reject decision and the same next step size without a host round trip.
// Per-row solver state (y, the stage derivatives k_j, the dense-output coefficients) lives in the
// workspace and is written only by the row's owner lane (wave 0, q = 0); every wave reads it after
// a workgroup barrier.  The step controller runs redundantly (and identically) in every thread.
#include "common.h"
#include "tile.h"
#include "tile16.h"
#include "dopri5.h"
#include "../../include/fiode.h"

namespace {
using namespace fiode_tile;
using namespace fiode_t16;
using namespace fiode_dp;

constexpr int OS_TMAX = 16;      // tiles per workgroup (LDS: 3.5 KB per tile)
constexpr int OS_XV = 4;         // float64 values per reduction exchange (at most)

struct OsArgs {
  int B, n_times, method, max_steps;
  int T, ntiles;                 // tiles per workgroup, tiles
  int drop_block;                // test hook: workgroup that skips its first publish (-1: none)
  double rtol, atol, step_size;
  DynScalars d;
  const float* x_feat;
  const float* h0;
  const double* times;
  const float *Q1, *b1, *Qx, *bx, *Q2, *b2, *Q3, *b3;
  float* sol;                    // [n_times][B][C]
  int32_t* stats;                // [8]: nfe, n_accept, n_reject, status, last exit iter, n_steps, workgroups,
                                 //      tiles per workgroup
  double* dstats;                // [4]: final dt, t reached, last error ratio
  // workspace
  float* u;                      // [B][M]
  float* y;                      // [B][C]
  float* K;                      // [7][B][C] stage derivatives
  float* interp;                 // [5][B][C] dopri5 dense-output coefficients
  unsigned long long* xm;        // [2 parities][grid] QP-mask granules
  unsigned long long* xr;        // [2 parities][grid][2 OS_XV] float64 partial sums (hi, lo words)
};

struct OsTile {                  // one tile's QP state kept across the exit exchange
  float mu_rec[TR][33];          // mu of every bisection iteration (owner lanes)
  float hin[TR][C];              // stage input
  float ft[TR][C];               // MLP output
  float lo[TR], hi[TR];          // bisection bracket after the speculative part
};

struct OsShared {
  float zpart[4][64][4];         // [part][lane][layer-3 accumulator registers]
  float Q1s[M * C];
  double red[OS_XV];             // broadcast of the last reduction exchange
  int K;                         // exit iteration of the current eval
  int kprev;                     // previous eval's exit (speculation)
  int dead;                      // an exchange timed out: stop waiting (status 4 recorded)
  int nx;                        // exchanges the current eval used (1, or 2 after a resume)
};

__device__ __forceinline__ bool owner_lane() { return threadIdx.x < 16; }   // wave 0, q = 0

// ---- tagged-granule exchanges (called by wave 0 of every workgroup) --------------------------
// AND of every workgroup's mask for exchange `ep` (parity buffer ep & 1; a workgroup cannot get two
// exchanges ahead of another, so two buffers suffice).
__device__ uint32_t xchg_and(const OsArgs& a, OsShared& sh, unsigned ep, uint32_t mine, int lane) {
  unsigned long long* buf = a.xm + (size_t)(ep & 1u) * gridDim.x;
  if (lane == 0 && !(ep == 1u && (int)blockIdx.x == a.drop_block)) publish_mask(buf + blockIdx.x, ep, mine);
  uint32_t acc = 0xFFFFFFFFu;
  const int G = gridDim.x;
  for (int base = 0; base < G; base += 64) {
    const int w = base + lane;
    unsigned spins = 0;
    for (;;) {
      bool ok = true;
      unsigned long long x = 0;
      if (w < G) {
        x = __hip_atomic_load((gu64_t*)(buf + w), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        ok = (unsigned)(x >> 32) == ep;
      }
      if (__all(ok)) {
        if (w < G) acc &= (uint32_t)x;
        break;
      }
      if (sh.dead || ++spins > (1u << 22)) {     // ~0.5 s: a workgroup is not resident
        if (lane == 0) {
          atomicMax(a.stats + 3, 4);
          sh.dead = 1;
        }
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
  }
  return wave_and(acc);
}

// Sum over workgroups of NV float64 values, added in workgroup order by every workgroup (same
// result everywhere).  Each value travels as two tagged granules (high, low 32 bits).
template <int NV>
__device__ void xchg_sum(const OsArgs& a, OsShared& sh, unsigned ep, const double (&mine)[NV], double (&out)[NV],
                         int lane) {
  unsigned long long* buf = a.xr + (size_t)(ep & 1u) * gridDim.x * 2 * OS_XV;
  if (lane == 0) {
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      const unsigned long long bits = (unsigned long long)__double_as_longlong(mine[v]);
      publish_mask(buf + (size_t)blockIdx.x * 2 * OS_XV + 2 * v, ep, (uint32_t)(bits >> 32));
      publish_mask(buf + (size_t)blockIdx.x * 2 * OS_XV + 2 * v + 1, ep, (uint32_t)bits);
    }
  }
  double acc[NV];
#pragma unroll
  for (int v = 0; v < NV; ++v) acc[v] = 0.0;
  const int G = gridDim.x;
  for (int base = 0; base < G; base += 64) {
    const int w = base + lane;
    unsigned spins = 0;
    for (;;) {
      bool ok = true;
      unsigned long long x[2 * NV];
#pragma unroll
      for (int g = 0; g < 2 * NV; ++g) {
        x[g] = 0;
        if (w < G) {
          x[g] = __hip_atomic_load((gu64_t*)(buf + (size_t)w * 2 * OS_XV + g), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
          ok = ok && (unsigned)(x[g] >> 32) == ep;
        }
      }
      if (__all(ok)) {
        if (w < G) {
#pragma unroll
          for (int v = 0; v < NV; ++v)
            acc[v] += __longlong_as_double((long long)(((x[2 * v] & 0xFFFFFFFFull) << 32) | (x[2 * v + 1] & 0xFFFFFFFFull)));
        }
        break;
      }
      if (sh.dead || ++spins > (1u << 22)) {
        if (lane == 0) {
          atomicMax(a.stats + 3, 4);
          sh.dead = 1;
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
    out[v] = acc[v];
  }
}

// Workgroup-wide float64 sums of per-row values (owner lanes contribute) followed by the exchange
// over workgroups; the result is broadcast to every thread.
template <int NV>
__device__ void batch_sum(const OsArgs& a, OsShared& sh, unsigned& ep, double (&v)[NV]) {
  const int lane = threadIdx.x & 63;
  if (threadIdx.x < 64) {
    double w[NV];
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      double s = v[i];
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) s += __shfl_xor(s, o, 64);
      w[i] = s;
    }
    double out[NV];
    xchg_sum<NV>(a, sh, ep, w, out, lane);
    if (lane == 0)
#pragma unroll
      for (int i = 0; i < NV; ++i) sh.red[i] = out[i];
  }
  ++ep;
  __syncthreads();
#pragma unroll
  for (int i = 0; i < NV; ++i) v[i] = sh.red[i];
  __syncthreads();
}

// ---- stage inputs (every lane of a row computes its row's from the global state) ------------
enum { IN_Y = 0, IN_RK4_2, IN_RK4_3, IN_RK4_4, IN_DP, IN_H0 };
struct StageIn {
  int kind;        // IN_*
  int i;           // dopri5 stage (IN_DP)
  float dt;        // step (rk4, dopri5) or h0 (IN_H0)
};

// The float32 expression orders of the oracle / torchdiffeq: rk4_alt_step_func (3/8 rule) and the
// dopri5 stage sums acc = sum_j k_j (beta_ij dt), y_i = y + acc.
__device__ __forceinline__ void stage_input(const OsArgs& a, const StageIn& in, int bb, float (&h)[C]) {
  const size_t BC = (size_t)a.B * C;
  const float* Kr = a.K + (size_t)bb * C;
  float y[C];
  load_row10(a.y + (size_t)bb * C, y);
  const float third = 1.0f / 3.0f, dt = in.dt;
  if (in.kind == IN_Y) {
#pragma unroll
    for (int c = 0; c < C; ++c) h[c] = y[c];
  } else if (in.kind == IN_DP) {
    float acc[C];
#pragma unroll
    for (int c = 0; c < C; ++c) acc[c] = 0.f;
    for (int jj = 0; jj <= in.i; ++jj) {
      float f[C];
      load_row10(Kr + (size_t)jj * BC, f);
      const float co = DP_BETA[in.i][jj] * dt;
#pragma unroll
      for (int c = 0; c < C; ++c) acc[c] = acc[c] + f[c] * co;
    }
#pragma unroll
    for (int c = 0; c < C; ++c) h[c] = y[c] + acc[c];
  } else {
    float f1[C], f2[C], f3[C];
    load_row10(Kr, f1);
    if (in.kind == IN_H0 || in.kind == IN_RK4_2) {
#pragma unroll
      for (int c = 0; c < C; ++c) h[c] = in.kind == IN_H0 ? y[c] + dt * f1[c] : y[c] + (dt * f1[c]) * third;
    } else {
      load_row10(Kr + BC, f2);
      if (in.kind == IN_RK4_3) {
#pragma unroll
        for (int c = 0; c < C; ++c) h[c] = y[c] + dt * (f2[c] - f1[c] * third);
      } else {
        load_row10(Kr + 2 * BC, f3);
#pragma unroll
        for (int c = 0; c < C; ++c) h[c] = y[c] + dt * ((f1[c] - f2[c]) + f3[c]);
      }
    }
  }
}

// ---- one eval: k[kdst] = eval_dot(stage input) for every row of the batch -------------------
// Uses exchange epochs ep (and ep + 1 after a resume); returns the next free epoch.
__device__ __noinline__ unsigned os_eval(const OsArgs& a, const float* Q2s, const float* Q3s, OsShared& sh, OsTile* tl,
                                    unsigned ep, int kdst, StageIn in) {
  const int lane = threadIdx.x & 63, q = lane >> 4, j = lane & 15;
  const int p = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const bool own = owner_lane();
  const int last = a.d.max_iter - 1;
  const int kspec = min(last, sh.kprev + 3);
  const uint32_t ones[4] = {0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu};
  T16W w;                     // this wave's weight operands, from the workgroup's LDS images
  load_t16w(sh.Q1s, Q2s, LDQ, Q3s, LDQ, a.b2, a.b3, p, q, j, w);
  uint32_t wconv = 0xFFFFFFFFu;
  for (int t = 0; t < a.T; ++t) {
    const int tile = blockIdx.x * a.T + t;
    const int b = tile * TR + j;
    const bool valid = b < a.B;
    const int bb = valid ? b : a.B - 1;
    float h[C];
    stage_input(a, in, bb, h);
    f32x4v uacc[8];
#pragma unroll
    for (int hb = 0; hb < 8; ++hb) {
      const f32x4 uv = *reinterpret_cast<const f32x4*>(a.u + (size_t)bb * M + 16 * hb + 4 * q);
      uacc[hb] = f32x4v{uv[0], uv[1], uv[2], uv[3]};
    }
    mlp16_part(w, uacc, h, ones, 0xFFFFFFFFu, 1.0f, p, q, nullptr, nullptr, &sh.zpart[p][lane][0]);
    __syncthreads();
    float ft[C];
    ft16_sum(sh.zpart, j, ft);
    float lower[C], nominal[C], sig[C], span[C];
    barrier_nominal(a.d, h, ft, lower, nominal, sig, span);
    float lo, hi;
    qp_bracket(lower, nominal, lo, hi);
    wconv &= qp_bisect_seq(lower, nominal, 0, kspec, a.d.tol, lo, hi, &tl[t].mu_rec[j][0], own, valid);
    if (own) {
#pragma unroll
      for (int i = 0; i < C; ++i) {
        tl[t].hin[j][i] = h[i];
        tl[t].ft[j][i] = ft[i];
      }
      tl[t].lo[j] = lo;
      tl[t].hi[j] = hi;
    }
    __syncthreads();          // zpart is reused by the next tile
  }
  // batch-global exit among the speculated iterations 0..kspec
  if (p == 0) {
    const uint32_t all = xchg_and(a, sh, ep, wconv, lane);
    const uint32_t lowm = kspec >= 31 ? 0xFFFFFFFFu : ((1u << (kspec + 1)) - 1u);
    const uint32_t bits = all & lowm;
    if (lane == 0) {
      sh.K = bits ? (__ffs((int)bits) - 1) : (kspec >= last ? last : -1);
      sh.nx = 1;
    }
  }
  __syncthreads();
  if (sh.K < 0) {             // block-uniform: no speculated iteration converged everywhere
    uint32_t wc2 = 0xFFFFFFFFu;
    for (int t = 0; t < a.T; ++t) {
      const int b = (blockIdx.x * a.T + t) * TR + j;
      const bool valid = b < a.B;
      float h[C], ft[C], lower[C], nominal[C], sig[C], span[C];
#pragma unroll
      for (int i = 0; i < C; ++i) {
        h[i] = tl[t].hin[j][i];
        ft[i] = tl[t].ft[j][i];
      }
      barrier_nominal(a.d, h, ft, lower, nominal, sig, span);
      float lo = tl[t].lo[j], hi = tl[t].hi[j];
      wc2 &= qp_bisect_seq(lower, nominal, kspec + 1, last, a.d.tol, lo, hi, &tl[t].mu_rec[j][0], own, valid);
    }
    if (p == 0) {
      const uint32_t all = xchg_and(a, sh, ep + 1, wc2, lane);
      if (lane == 0) {
        sh.K = qp_exit_iter(all, a.d.max_iter);
        sh.nx = 2;
      }
    }
    __syncthreads();
  }
  const int K = sh.K;
  const unsigned ep_next = ep + (unsigned)sh.nx;
  // finalize: k = v(mu_K) (barrier_projection.py:251-253 at the exit iteration), owner lanes store
  if (own) {
    for (int t = 0; t < a.T; ++t) {
      const int b = (blockIdx.x * a.T + t) * TR + j;
      if (b >= a.B) break;
      float h[C], ft[C], lower[C], nominal[C], sig[C], span[C], k[C];
#pragma unroll
      for (int i = 0; i < C; ++i) {
        h[i] = tl[t].hin[j][i];
        ft[i] = tl[t].ft[j][i];
      }
      barrier_nominal(a.d, h, ft, lower, nominal, sig, span);
      const float mu = tl[t].mu_rec[j][K];
#pragma unroll
      for (int i = 0; i < C; ++i) k[i] = fmaxf(nominal[i] - mu, lower[i]);
      store_row10(a.K + ((size_t)kdst * a.B + b) * C, k);
    }
  }
  if (threadIdx.x == 0) {
    sh.kprev = K;
    if (blockIdx.x == 0) a.stats[0] += 1;
  }
  __syncthreads();
  return ep_next;
}

// iterate the owner lane's valid rows: fn(b)
template <class Fn>
__device__ __forceinline__ void for_own_rows(const OsArgs& a, Fn fn) {
  if (!owner_lane()) return;
  for (int t = 0; t < a.T; ++t) {
    const int b = (blockIdx.x * a.T + t) * TR + (int)threadIdx.x;
    if (b >= a.B) return;
    fn(b);
  }
}

__device__ void os_rk4(const OsArgs& a, const float* Q2s, const float* Q3s, OsShared& sh, OsTile* tl) {
  // FixedGridODESolver grid in float32: niters = ceil((t1-t0)/h + 1), t_k = k*h + t0, last = t1
  unsigned ep = 1;
  const float t0 = (float)a.times[0], t1 = (float)a.times[a.n_times - 1], hs = (float)a.step_size;
  const int niters = (int)ceilf((t1 - t0) / hs + 1.0f);
  const size_t BC = (size_t)a.B * C;
  const float* k1 = a.K;
  const float* k2 = a.K + BC;
  const float* k3 = a.K + 2 * BC;
  const float* k4 = a.K + 3 * BC;
  int jo = 1;
  for (int it = 0; it + 1 < niters; ++it) {
    const float ta = (float)it * hs + t0;
    const float tb = (it + 2 == niters) ? t1 : (float)(it + 1) * hs + t0;
    const float dt = tb - ta;
    ep = os_eval(a, Q2s, Q3s, sh, tl, ep, 0, StageIn{IN_Y, 0, dt});
    ep = os_eval(a, Q2s, Q3s, sh, tl, ep, 1, StageIn{IN_RK4_2, 0, dt});
    ep = os_eval(a, Q2s, Q3s, sh, tl, ep, 2, StageIn{IN_RK4_3, 0, dt});
    ep = os_eval(a, Q2s, Q3s, sh, tl, ep, 3, StageIn{IN_RK4_4, 0, dt});
    const int j0 = jo;
    while (jo < a.n_times && tb >= (float)a.times[jo]) ++jo;   // outputs in (ta, tb], uniform
    for_own_rows(a, [&](int b) {
      float y[C], f1[C], f2[C], f3[C], f4[C], yn[C];
      load_row10(a.y + (size_t)b * C, y);
      load_row10(k1 + (size_t)b * C, f1);
      load_row10(k2 + (size_t)b * C, f2);
      load_row10(k3 + (size_t)b * C, f3);
      load_row10(k4 + (size_t)b * C, f4);
#pragma unroll
      for (int i = 0; i < C; ++i) {
        const float dy = (((f1[i] + 3.0f * (f2[i] + f3[i])) + f4[i]) * dt) * 0.125f;
        yn[i] = y[i] + dy;
      }
      for (int jj = j0; jj < jo; ++jj) {       // linear interpolation; exact grid hits return the grid value
        const float tj = (float)a.times[jj];
        float o[C];
#pragma unroll
        for (int i = 0; i < C; ++i)
          o[i] = tj == ta ? y[i] : (tj == tb ? yn[i] : y[i] + ((tj - ta) / (tb - ta)) * (yn[i] - y[i]));
        store_row10(a.sol + ((size_t)jj * a.B + b) * C, o);
      }
      store_row10(a.y + (size_t)b * C, yn);
    });
    if (blockIdx.x == 0 && threadIdx.x == 0) a.stats[1] += 1;
    __syncthreads();
  }
}

__device__ __forceinline__ float rms_from_sum(double sumsq, size_t n) { return (float)sqrt(sumsq / (double)n); }

__device__ void os_dopri5(const OsArgs& a, const float* Q2s, const float* Q3s, OsShared& sh, OsTile* tl) {
  unsigned ep = 1;
  const size_t BC = (size_t)a.B * C;
  const float rtol = (float)a.rtol, atol = (float)a.atol;
  const float* K0 = a.K;
  // ---- _select_initial_step(order - 1 = 4), float32 -------------------------------------------
  ep = os_eval(a, Q2s, Q3s, sh, tl, ep, 0, StageIn{IN_Y, 0, 0.f});
  double s01[2] = {0.0, 0.0};
  for_own_rows(a, [&](int b) {
    float y[C], f0[C];
    load_row10(a.y + (size_t)b * C, y);
    load_row10(K0 + (size_t)b * C, f0);
#pragma unroll
    for (int i = 0; i < C; ++i) {
      const float sc = atol + fabsf(y[i]) * rtol;
      const float q0 = y[i] / sc, qq = f0[i] / sc;
      s01[0] += (double)q0 * q0;
      s01[1] += (double)qq * qq;
    }
  });
  batch_sum<2>(a, sh, ep, s01);
  const float d0 = rms_from_sum(s01[0], BC);
  const float d1 = rms_from_sum(s01[1], BC);
  const float h0 = (d0 < 1e-5f || d1 < 1e-5f) ? 1e-6f : (0.01f * d0) / d1;
  ep = os_eval(a, Q2s, Q3s, sh, tl, ep, 1, StageIn{IN_H0, 0, h0});      // f1 at t0 + h0
  double s2[1] = {0.0};
  for_own_rows(a, [&](int b) {
    float y[C], f0[C], f1[C];
    load_row10(a.y + (size_t)b * C, y);
    load_row10(K0 + (size_t)b * C, f0);
    load_row10(a.K + BC + (size_t)b * C, f1);
#pragma unroll
    for (int i = 0; i < C; ++i) {
      const float sc = atol + fabsf(y[i]) * rtol;
      const float q = (f1[i] - f0[i]) / sc;
      s2[0] += (double)q * q;
    }
  });
  batch_sum<1>(a, sh, ep, s2);
  const float d2 = rms_from_sum(s2[0], BC) / h0;
  float h1;
  if (d1 <= 1e-15f && d2 <= 1e-15f) h1 = fmaxf(1e-6f, h0 * 1e-3f);
  else h1 = powf(0.01f / fmaxf(d1, d2), 1.0f / 5.0f);
  // controller state: identical in every thread of every workgroup
  double dt = (double)fminf(100.0f * h0, h1);
  double tcur = a.times[0], tprev = tcur, tnext = tcur;
  float ratio = 0.f;
  int nsteps = 0;
  for (int ti = 1; ti < a.n_times; ++ti) {
    const double tout = a.times[ti];
    while (tout > tnext) {
      if (nsteps >= a.max_steps || !(tcur + dt > tcur)) {
        if (blockIdx.x == 0 && threadIdx.x == 0) {
          a.stats[3] = nsteps >= a.max_steps ? 2 : 3;     // max steps / dt underflow
          a.stats[5] = nsteps;
          a.stats[4] = sh.kprev;
        }
        return;
      }
      ++nsteps;
      const float dt32 = (float)dt;
      for (int i = 0; i < 6; ++i) {
        ep = os_eval(a, Q2s, Q3s, sh, tl, ep, i + 1, StageIn{IN_DP, i, dt32});
      }
      // y1 = the stage-6 input (FSAL tableau); batch-global RMS error ratio
      double ps[1] = {0.0};
      for_own_rows(a, [&](int b) {
        const int t = b / TR - blockIdx.x * a.T;
        float y[C], err[C];
        load_row10(a.y + (size_t)b * C, y);
#pragma unroll
        for (int c = 0; c < C; ++c) err[c] = 0.f;
#pragma unroll
        for (int jj = 0; jj < 7; ++jj) {
          float f[C];
          load_row10(a.K + (size_t)jj * BC + (size_t)b * C, f);
          const float co = DP_CERR[jj] * dt32;
#pragma unroll
          for (int c = 0; c < C; ++c) err[c] = err[c] + f[c] * co;
        }
#pragma unroll
        for (int c = 0; c < C; ++c) {
          const float y1 = tl[t].hin[threadIdx.x][c];
          const float etol = atol + rtol * fmaxf(fabsf(y[c]), fabsf(y1));
          const float q = err[c] / etol;
          ps[0] += (double)q * q;
        }
      });
      batch_sum<1>(a, sh, ep, ps);
      ratio = rms_from_sum(ps[0], BC);
      const bool accept = ratio <= 1.0f;
      if (accept) {
        for_own_rows(a, [&](int b) {
          const int t = b / TR - blockIdx.x * a.T;
          float y0[C], acc[C], fa[C], fb[C];
          load_row10(a.y + (size_t)b * C, y0);
          load_row10(a.K + (size_t)b * C, fa);
          load_row10(a.K + 6 * BC + (size_t)b * C, fb);
#pragma unroll
          for (int c = 0; c < C; ++c) acc[c] = 0.f;
#pragma unroll
          for (int jj = 0; jj < 7; ++jj) {
            float f[C];
            load_row10(a.K + (size_t)jj * BC + (size_t)b * C, f);
            const float co = DP_CMID[jj] * dt32;
#pragma unroll
            for (int c = 0; c < C; ++c) acc[c] = acc[c] + f[c] * co;
          }
          float y1[C], ci[5][C];
#pragma unroll
          for (int c = 0; c < C; ++c) {
            y1[c] = tl[t].hin[threadIdx.x][c];
            const float ym = y0[c] + acc[c];
            ci[0][c] = y0[c];
            ci[1][c] = dt32 * fa[c];
            ci[2][c] = (((dt32 * (fb[c] - 4.0f * fa[c])) - 11.0f * y0[c]) - 5.0f * y1[c]) + 16.0f * ym;
            ci[3][c] = (((dt32 * (5.0f * fa[c] - 3.0f * fb[c])) + 18.0f * y0[c]) + 14.0f * y1[c]) - 32.0f * ym;
            ci[4][c] = ((2.0f * dt32) * (fb[c] - fa[c]) - 8.0f * (y1[c] + y0[c])) + 16.0f * ym;
          }
#pragma unroll
          for (int m = 0; m < 5; ++m) store_row10(a.interp + (size_t)m * BC + (size_t)b * C, ci[m]);
          store_row10(a.y + (size_t)b * C, y1);
          store_row10(a.K + (size_t)b * C, fb);                 // FSAL
        });
        tprev = tcur;
        tnext = tcur + dt;
        tcur = tcur + dt;
      }
      if (blockIdx.x == 0 && threadIdx.x == 0) a.stats[accept ? 1 : 2] += 1;
      // _optimal_step_size (float64)
      if (ratio == 0.f) {
        dt = dt * 10.0;
      } else {
        const double df = ratio < 1.0f ? 1.0 : 0.2;
        dt = dt * fmin(10.0, fmax(0.9 / pow((double)ratio, 1.0 / 5.0), df));
      }
      __syncthreads();
    }
    // dense output at tout (torchdiffeq _interp_evaluate: power sum over x = (tout - t0)/(t1 - t0))
    const float x = (float)((tout - tprev) / (tnext - tprev));
    for_own_rows(a, [&](int b) {
      float total[C], cm[C];
      load_row10(a.interp + (size_t)b * C, total);
      load_row10(a.interp + BC + (size_t)b * C, cm);
#pragma unroll
      for (int c = 0; c < C; ++c) total[c] = total[c] + x * cm[c];
      float xp = x;
#pragma unroll
      for (int m = 2; m < 5; ++m) {
        xp = xp * x;
        load_row10(a.interp + (size_t)m * BC + (size_t)b * C, cm);
#pragma unroll
        for (int c = 0; c < C; ++c) total[c] = total[c] + xp * cm[c];
      }
      store_row10(a.sol + ((size_t)ti * a.B + b) * C, total);
    });
    __syncthreads();
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    a.dstats[0] = dt;
    a.dstats[1] = tcur;
    a.dstats[2] = (double)ratio;
    a.stats[5] = nsteps;
  }
}

// clears the exchange granules (tags) and the stats ahead of the solve
__global__ __launch_bounds__(256) void k_os_clear(OsArgs a, int nslots) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < nslots) a.xm[i] = 0ull;     // xm and xr are contiguous
  if (i < 8) a.stats[i] = 0;
  if (i < 4) a.dstats[i] = 0.0;
}

__global__ __launch_bounds__(256) void k_ode_tiles(OsArgs a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* Q2s = smem;
  float* Q3s = smem + M * LDQ;
  OsShared& sh = *reinterpret_cast<OsShared*>(smem + (M + 32) * LDQ);
  OsTile* tl = reinterpret_cast<OsTile*>(reinterpret_cast<char*>(&sh) + sizeof(OsShared));
  load_weight_images(a.Q2, a.Q3, Q2s, Q3s);
  for (int t = threadIdx.x; t < M * C; t += blockDim.x) sh.Q1s[t] = a.Q1[t];
  if (threadIdx.x == 0) {
    sh.kprev = a.d.max_iter - 1;
    sh.dead = 0;
  }
  // u[b] = U_x x_b + bx + b1 for this workgroup's rows; y = h0; sol[0] = h0
  const int r0 = blockIdx.x * a.T * TR;
  const int nr = min(a.T * TR, a.B - r0);
  for (int e = threadIdx.x; e < nr * M; e += blockDim.x) {
    const int rb = r0 + e / M, i = e % M;
    float s = 0.f;
#pragma unroll
    for (int c = 0; c < FIODE_X; ++c) s = __fmaf_rn(a.Qx[i * FIODE_X + c], a.x_feat[(size_t)rb * FIODE_X + c], s);
    a.u[(size_t)rb * M + i] = (s + a.bx[i]) + a.b1[i];
  }
  for (int e = threadIdx.x; e < nr * C; e += blockDim.x) {
    const size_t o = (size_t)r0 * C + e;
    a.y[o] = a.h0[o];
    a.sol[o] = a.h0[o];
  }
  __syncthreads();
  if (a.method == FIODE_ODE_RK4) os_rk4(a, Q2s, Q3s, sh, tl);
  else os_dopri5(a, Q2s, Q3s, sh, tl);
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    a.stats[4] = sh.kprev;
    a.stats[6] = (int)gridDim.x;
    a.stats[7] = a.T;
  }
}

inline size_t al(size_t x) { return (x + 255) & ~(size_t)255; }

struct OsLayout {
  size_t u, y, K, interp, xm, xr, total;
};
OsLayout os_layout(int B) {
  const size_t BC = (size_t)B * C * 4;
  const size_t nt = (size_t)(B + TR - 1) / TR;
  OsLayout L;
  size_t o = 0;
  L.u = o; o += al((size_t)B * M * 4);
  L.y = o; o += al(BC);
  L.K = o; o += al(7 * BC);
  L.interp = o; o += al(5 * BC);
  L.xm = o; o += 2 * nt * 8;                 // xr follows xm directly (one clear)
  L.xr = o; o += al(2 * nt * 2 * OS_XV * 8);
  L.total = al(o);
  return L;
}

size_t os_lds_bytes(int T) {
  return (size_t)(M + 32) * LDQ * sizeof(float) + sizeof(OsShared) + (size_t)T * sizeof(OsTile);
}

// resident workgroups of k_ode_tiles on this device (cached per device): CUs x occupancy
int os_capacity(size_t lds) {
  static int cached[64][2];
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0) return -1;
  if (dev < 64 && cached[dev][0] > 0 && (size_t)cached[dev][1] == lds) return cached[dev][0];
  int cus = 0, occ = 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return -1;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k_ode_tiles, 256, lds) != hipSuccess) return -1;
  const int cap = cus * (occ > 0 ? occ : 0);
  if (dev < 64) {
    cached[dev][0] = cap;
    cached[dev][1] = (int)lds;
  }
  return cap;
}

}  // namespace

extern "C" size_t fiode_odeint_workspace_bytes(int32_t batch) {
  if (batch <= 0) return 256;
  return os_layout(batch).total;
}

extern "C" int fiode_odeint(void* stream, const fiode_ode_config* cfg, const fiode_dyn_config* dyn,
                            const fiode_dyn_weights* w, const float* x_feat, const float* h0, const double* times,
                            float* solution, int32_t* stats, double* dstats, void* workspace, size_t workspace_bytes) {
  if (!cfg || !dyn || !w) return FIODE_EINVAL;
  if (dyn->n_hidden != C || dyn->mlp_size != M || dyn->x_dim != FIODE_X) return FIODE_ESHAPE;
  if (dyn->qp_max_iter < 1 || dyn->qp_max_iter > 32) return FIODE_EINVAL;
  if (cfg->batch <= 0 || cfg->batch > FIODE_ODEINT_MAX_BATCH || cfg->n_times < 2) return FIODE_EINVAL;
  if (cfg->method != FIODE_ODE_RK4 && cfg->method != FIODE_ODE_DOPRI5) return FIODE_EINVAL;
  if (cfg->method == FIODE_ODE_RK4 && !(cfg->step_size > 0)) return FIODE_EINVAL;
  if (cfg->method == FIODE_ODE_DOPRI5 && !(cfg->rtol > 0 && cfg->atol > 0)) return FIODE_EINVAL;
  if (!x_feat || !h0 || !times || !solution || !stats || !dstats || !workspace) return FIODE_EINVAL;
  if (!w->Q1 || !w->b1 || !w->Qx || !w->bx || !w->Q2 || !w->b2 || !w->Q3 || !w->b3) return FIODE_EINVAL;
  if (workspace_bytes < fiode_odeint_workspace_bytes(cfg->batch)) return FIODE_EWORKSPACE;
  OsArgs a{};
  a.B = cfg->batch; a.n_times = cfg->n_times; a.method = cfg->method;
  a.max_steps = cfg->max_steps > 0 ? cfg->max_steps : 100000;
  a.rtol = cfg->rtol; a.atol = cfg->atol; a.step_size = cfg->step_size;
  a.d.alpha_1 = dyn->alpha_1; a.d.alpha_2 = dyn->alpha_2; a.d.sigma_1 = dyn->sigma_1;
  a.d.tol = dyn->qp_tol; a.d.scale_nominal = dyn->scale_nominal; a.d.max_iter = dyn->qp_max_iter;
  a.x_feat = x_feat; a.h0 = h0; a.times = times;
  a.Q1 = w->Q1; a.b1 = w->b1; a.Qx = w->Qx; a.bx = w->bx; a.Q2 = w->Q2; a.b2 = w->b2; a.Q3 = w->Q3; a.b3 = w->b3;
  a.sol = solution; a.stats = stats; a.dstats = dstats;
  a.drop_block = fiode_internal::debug_drop_publish();
  // tiles -> workgroups: one tile per workgroup while they fit the resident capacity, else T each
  a.ntiles = (a.B + TR - 1) / TR;
  const int cap = os_capacity(os_lds_bytes(OS_TMAX));
  if (cap <= 0) return FIODE_EHIP;
  a.T = (a.ntiles + cap - 1) / cap;
  if (a.T > OS_TMAX) return FIODE_EINVAL;
  const int grid = (a.ntiles + a.T - 1) / a.T;
  const OsLayout L = os_layout(a.B);
  char* ws = static_cast<char*>(workspace);
  a.u = reinterpret_cast<float*>(ws + L.u);
  a.y = reinterpret_cast<float*>(ws + L.y);
  a.K = reinterpret_cast<float*>(ws + L.K);
  a.interp = reinterpret_cast<float*>(ws + L.interp);
  a.xm = reinterpret_cast<unsigned long long*>(ws + L.xm);
  a.xr = reinterpret_cast<unsigned long long*>(ws + L.xr);
  hipStream_t st = static_cast<hipStream_t>(stream);
  const int nslots = (int)((L.total - L.xm) / 8);
  hipLaunchKernelGGL(k_os_clear, dim3((nslots + 255) / 256), dim3(256), 0, st, a, nslots);
  FIODE_HIP_CHECK(hipGetLastError());
  hipLaunchKernelGGL(k_ode_tiles, dim3(grid), dim3(256), os_lds_bytes(a.T), st, a);
  FIODE_HIP_CHECK(hipGetLastError());
  return FIODE_OK;
}
