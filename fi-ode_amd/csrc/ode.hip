// ODE solves of the Cayley-MLP dynamics on gfx950: replaces torchdiffeq.odeint at
// models.py:235-241 (IVP.integrate) for method 'rk4' (fixed grid, 3/8 rule) and 'dopri5'
// (adaptive, torchdiffeq 0.2.2 semantics).  f(h) = eval_dot in eval mode
// (dynamics/classification.py:104-132) with the QP's batch-global exit over the B rows of each
// stage, exactly as every func() call of odeint sees it.
//
// One persistent workgroup owns the whole batch: every stage needs two batch-wide reductions
// (the QP exit word, and for dopri5 the RMS error norm shared by all samples), which inside one
// workgroup are LDS reductions + barriers -- no host syncs, no grid barriers.  Per stage:
//   (1) stage input  y_i = y + sum_j k_j (beta_ij dt)           thread per row
//   (2) MLP + barrier + QP convergence mask                      wave per 32-row tile (MFMA)
//   (3) QP to the global exit, k_{i+1} = v                      thread per row
// The step-size controller (float64) runs on thread 0; all branches are block-uniform.
#include "common.h"
#include "tile.h"
#include "../../include/fiode.h"

namespace {
using namespace fiode_tile;

constexpr int ODE_THREADS = 256;
constexpr int ODE_WAVES = ODE_THREADS / 64;

struct OdeArgs {
  int B, n_times, method, max_steps;
  double rtol, atol, step_size;
  DynScalars d;
  const float* x_feat;
  const float* h0;
  const double* times;
  const float *Q1, *b1, *Qx, *bx, *Q2, *b2, *Q3, *b3;
  float* sol;         // [n_times][B][C]
  int32_t* stats;     // [8]: nfe, n_accept, n_reject, status, last exit iter, n_steps
  double* dstats;     // [4]: final dt, t reached, last error ratio
  // workspace
  float* u;           // [B][M]
  float* y;           // [B][C]
  float* yi;          // [B][C] stage input
  float* ft;          // [B][C] MLP output of the stage
  float* k;           // [7][B][C]
  float* interp;      // [5][B][C]
  float* ynew;        // [B][C]
};

struct Shared {            // lives in the dynamic LDS region after the weight images (16-B aligned)
  double red[ODE_THREADS];
  double dt, tcur, tprev, tnext;
  uint32_t word;
  int last_exit;
  int pad[2];
};

__device__ __forceinline__ double block_sum(double v, Shared& sh) {
  sh.red[threadIdx.x] = v;
  __syncthreads();
  for (int o = ODE_THREADS / 2; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) sh.red[threadIdx.x] += sh.red[threadIdx.x + o];
    __syncthreads();
  }
  const double r = sh.red[0];
  __syncthreads();
  return r;
}

// f = eval_dot(yin) for all B rows -> fout.  Two phases separated by the global exit word.
__device__ void eval_f(const OdeArgs& a, const float* Q2s, const float* Q3s, const float (&q1)[4][5],
                       const float* yin, float* fout, Shared& sh) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, half = lane >> 5, col = lane & 31;
  if (threadIdx.x == 0) sh.word = 0xFFFFFFFFu;
  __syncthreads();
  const uint32_t kw[4] = {0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu};
  const int ntiles = (a.B + 31) / 32;
  for (int tile = wave; tile < ntiles; tile += ODE_WAVES) {
    const int row = tile * 32 + col;
    const bool valid = row < a.B;
    const int rr = valid ? row : a.B - 1;
    float h[C];
    load_row10(yin + (size_t)rr * C, h);
    f32x16 z1[4], z2[4];
    const f32x16 z3 = mlp_tile(Q2s, Q3s, q1, a.u + (size_t)rr * M, a.b2, a.b3, h, kw, kw, 1.0f, col, half, z1, z2);
    float ft[C], lower[C], nominal[C], sig[C], span[C], v[C], mu;
    gather_ft(z3, half, ft);
    barrier_nominal(a.d, h, ft, lower, nominal, sig, span);
    uint32_t conv = qp_bisect(lower, nominal, a.d.max_iter - 1, a.d.tol, v, mu);
    if (!valid) conv = 0xFFFFFFFFu;
    conv = wave_and(conv);
    if (lane == 0) atomicAnd(&sh.word, conv);
    if (valid && half == 0) store_row10(a.ft + (size_t)row * C, ft);
  }
  __syncthreads();
  const int K = qp_exit_iter(sh.word, a.d.max_iter);
  for (int r = threadIdx.x; r < a.B; r += ODE_THREADS) {
    float h[C], ft[C], lower[C], nominal[C], sig[C], span[C], v[C], mu;
    load_row10(yin + (size_t)r * C, h);
    load_row10(a.ft + (size_t)r * C, ft);
    barrier_nominal(a.d, h, ft, lower, nominal, sig, span);
    qp_bisect(lower, nominal, K, a.d.tol, v, mu);
    store_row10(fout + (size_t)r * C, v);
  }
  if (threadIdx.x == 0) {
    sh.last_exit = K;
    a.stats[0] += 1;
  }
  __syncthreads();
}

__device__ __forceinline__ void copy_rows(const float* src, float* dst, int B) {
  for (int e = threadIdx.x; e < B * C; e += ODE_THREADS) dst[e] = src[e];
}

__device__ void solve_rk4(const OdeArgs& a, const float* Q2s, const float* Q3s, const float (&q1)[4][5], Shared& sh) {
  // FixedGridODESolver grid in float32: niters = ceil((t1-t0)/h + 1), t_k = k*h + t0, last = t1
  const float t0 = (float)a.times[0], t1 = (float)a.times[a.n_times - 1], hs = (float)a.step_size;
  const int niters = (int)ceilf((t1 - t0) / hs + 1.0f);
  const float third = 1.0f / 3.0f;
  float* k1 = a.k;
  float* k2 = a.k + (size_t)a.B * C;
  float* k3 = a.k + 2 * (size_t)a.B * C;
  float* k4 = a.k + 3 * (size_t)a.B * C;
  int j = 1;
  for (int it = 0; it + 1 < niters; ++it) {
    const float ta = (float)it * hs + t0;
    const float tb = (it + 2 == niters) ? t1 : (float)(it + 1) * hs + t0;
    const float dt = tb - ta;
    eval_f(a, Q2s, Q3s, q1, a.y, k1, sh);
    for (int e = threadIdx.x; e < a.B * C; e += ODE_THREADS) a.yi[e] = a.y[e] + (dt * k1[e]) * third;
    __syncthreads();
    eval_f(a, Q2s, Q3s, q1, a.yi, k2, sh);
    for (int e = threadIdx.x; e < a.B * C; e += ODE_THREADS) a.yi[e] = a.y[e] + dt * (k2[e] - k1[e] * third);
    __syncthreads();
    eval_f(a, Q2s, Q3s, q1, a.yi, k3, sh);
    for (int e = threadIdx.x; e < a.B * C; e += ODE_THREADS) a.yi[e] = a.y[e] + dt * ((k1[e] - k2[e]) + k3[e]);
    __syncthreads();
    eval_f(a, Q2s, Q3s, q1, a.yi, k4, sh);
    for (int e = threadIdx.x; e < a.B * C; e += ODE_THREADS) {
      const float dy = (((k1[e] + 3.0f * (k2[e] + k3[e])) + k4[e]) * dt) * 0.125f;
      a.ynew[e] = a.y[e] + dy;
    }
    __syncthreads();
    // outputs falling in (ta, tb]: linear interpolation (exact hits return the grid value)
    while (j < a.n_times && tb >= (float)a.times[j]) {
      const float tj = (float)a.times[j];
      float* out = a.sol + (size_t)j * a.B * C;
      for (int e = threadIdx.x; e < a.B * C; e += ODE_THREADS) {
        if (tj == ta) out[e] = a.y[e];
        else if (tj == tb) out[e] = a.ynew[e];
        else out[e] = a.y[e] + ((tj - ta) / (tb - ta)) * (a.ynew[e] - a.y[e]);
      }
      ++j;
    }
    copy_rows(a.ynew, a.y, a.B);
    if (threadIdx.x == 0) a.stats[1] += 1;
    __syncthreads();
  }
}

// torchdiffeq 0.2.2 dopri5 tableau (float32 copies, as RKAdaptiveStepsizeODESolver casts it)
__device__ const float DP_BETA[6][6] = {
    {1.0f / 5, 0, 0, 0, 0, 0},
    {3.0f / 40, 9.0f / 40, 0, 0, 0, 0},
    {(float)(44.0 / 45), (float)(-56.0 / 15), (float)(32.0 / 9), 0, 0, 0},
    {(float)(19372.0 / 6561), (float)(-25360.0 / 2187), (float)(64448.0 / 6561), (float)(-212.0 / 729), 0, 0},
    {(float)(9017.0 / 3168), (float)(-355.0 / 33), (float)(46732.0 / 5247), (float)(49.0 / 176),
     (float)(-5103.0 / 18656), 0},
    {(float)(35.0 / 384), 0, (float)(500.0 / 1113), (float)(125.0 / 192), (float)(-2187.0 / 6784),
     (float)(11.0 / 84)}};
__device__ const float DP_CERR[7] = {(float)(35.0 / 384 - 1951.0 / 21600), 0, (float)(500.0 / 1113 - 22642.0 / 50085),
                                     (float)(125.0 / 192 - 451.0 / 720), (float)(-2187.0 / 6784 - -12231.0 / 42400),
                                     (float)(11.0 / 84 - 649.0 / 6300), (float)(-1.0 / 60.0)};
__device__ const float DP_CMID[7] = {(float)(6025192743.0 / 30085553152.0 / 2), 0,
                                     (float)(51252292925.0 / 65400821598.0 / 2),
                                     (float)(-2691868925.0 / 45128329728.0 / 2),
                                     (float)(187940372067.0 / 1594534317056.0 / 2),
                                     (float)(-1776094331.0 / 19743644256.0 / 2), (float)(11237099.0 / 235043384.0 / 2)};

__device__ float rms_from_sum(double sumsq, int n) { return (float)sqrt(sumsq / (double)n); }

__device__ void solve_dopri5(const OdeArgs& a, const float* Q2s, const float* Q3s, const float (&q1)[4][5],
                             Shared& sh) {
  const int BC = a.B * C;
  const float rtol = (float)a.rtol, atol = (float)a.atol;
  float* K[7];
#pragma unroll
  for (int i = 0; i < 7; ++i) K[i] = a.k + (size_t)i * BC;
  double& s_dt = sh.dt;
  double& s_tcur = sh.tcur;
  double& s_tprev = sh.tprev;
  double& s_tnext = sh.tnext;
  // ---- _select_initial_step(order - 1 = 4), float32 -------------------------------------------
  eval_f(a, Q2s, Q3s, q1, a.y, K[0], sh);                  // f0
  double p0 = 0, p1 = 0;
  for (int e = threadIdx.x; e < BC; e += ODE_THREADS) {
    const float sc = atol + fabsf(a.y[e]) * rtol;
    const float q0 = a.y[e] / sc, qq = K[0][e] / sc;
    p0 += (double)q0 * q0;
    p1 += (double)qq * qq;
  }
  const float d0 = rms_from_sum(block_sum(p0, sh), BC);
  const float d1 = rms_from_sum(block_sum(p1, sh), BC);
  const float h0 = (d0 < 1e-5f || d1 < 1e-5f) ? 1e-6f : (0.01f * d0) / d1;
  for (int e = threadIdx.x; e < BC; e += ODE_THREADS) a.yi[e] = a.y[e] + h0 * K[0][e];
  __syncthreads();
  eval_f(a, Q2s, Q3s, q1, a.yi, K[1], sh);                 // f1 at t0 + h0
  double p2 = 0;
  for (int e = threadIdx.x; e < BC; e += ODE_THREADS) {
    const float sc = atol + fabsf(a.y[e]) * rtol;
    const float q = (K[1][e] - K[0][e]) / sc;
    p2 += (double)q * q;
  }
  const float d2 = rms_from_sum(block_sum(p2, sh), BC) / h0;
  float h1;
  if (d1 <= 1e-15f && d2 <= 1e-15f) h1 = fmaxf(1e-6f, h0 * 1e-3f);
  else h1 = powf(0.01f / fmaxf(d1, d2), 1.0f / 5.0f);
  if (threadIdx.x == 0) {
    s_dt = (double)fminf(100.0f * h0, h1);
    s_tcur = s_tprev = s_tnext = a.times[0];
  }
  __syncthreads();
  int nsteps = 0;
  for (int ti = 1; ti < a.n_times; ++ti) {
    const double tout = a.times[ti];
    while (tout > s_tnext) {
      if (nsteps >= a.max_steps || !(s_tcur + s_dt > s_tcur)) {
        if (threadIdx.x == 0) a.stats[3] = nsteps >= a.max_steps ? 2 : 3;   // max steps / dt underflow
        __syncthreads();
        return;
      }
      ++nsteps;
      const double dt = s_dt, tcur = s_tcur;
      const float dt32 = (float)dt;
      for (int i = 0; i < 6; ++i) {
        for (int e = threadIdx.x; e < BC; e += ODE_THREADS) {
          float acc = 0.f;
          for (int j = 0; j <= i; ++j) acc = acc + K[j][e] * (DP_BETA[i][j] * dt32);
          a.yi[e] = a.y[e] + acc;
        }
        __syncthreads();
        eval_f(a, Q2s, Q3s, q1, a.yi, K[i + 1], sh);
      }
      // y1 = stage-6 input (FSAL tableau), error estimate, batch-global RMS ratio
      double ps = 0;
      for (int e = threadIdx.x; e < BC; e += ODE_THREADS) {
        float err = 0.f;
#pragma unroll
        for (int j = 0; j < 7; ++j) err = err + K[j][e] * (DP_CERR[j] * dt32);
        const float y1 = a.yi[e];
        const float etol = atol + rtol * fmaxf(fabsf(a.y[e]), fabsf(y1));
        const float q = err / etol;
        ps += (double)q * q;
      }
      const float ratio = rms_from_sum(block_sum(ps, sh), BC);
      const bool accept = ratio <= 1.0f;
      if (accept) {
        for (int e = threadIdx.x; e < BC; e += ODE_THREADS) {
          float acc = 0.f;
#pragma unroll
          for (int j = 0; j < 7; ++j) acc = acc + K[j][e] * (DP_CMID[j] * dt32);
          const float y0 = a.y[e], y1 = a.yi[e], ym = y0 + acc, fa = K[0][e], fb = K[6][e];
          const float ca = ((2.0f * dt32) * (fb - fa) - 8.0f * (y1 + y0)) + 16.0f * ym;
          const float cb = (((dt32 * (5.0f * fa - 3.0f * fb)) + 18.0f * y0) + 14.0f * y1) - 32.0f * ym;
          const float cc = (((dt32 * (fb - 4.0f * fa)) - 11.0f * y0) - 5.0f * y1) + 16.0f * ym;
          a.interp[e] = y0;
          a.interp[(size_t)BC + e] = dt32 * fa;
          a.interp[2 * (size_t)BC + e] = cc;
          a.interp[3 * (size_t)BC + e] = cb;
          a.interp[4 * (size_t)BC + e] = ca;
          a.y[e] = y1;
          K[0][e] = fb;                                    // FSAL
        }
      }
      if (threadIdx.x == 0) {
        if (accept) {
          s_tprev = tcur;
          s_tnext = tcur + dt;
          s_tcur = tcur + dt;
          a.stats[1] += 1;
        } else {
          a.stats[2] += 1;
        }
        double nd;
        if (ratio == 0.f) {
          nd = dt * 10.0;
        } else {
          const double df = ratio < 1.0f ? 1.0 : 0.2;
          nd = dt * fmin(10.0, fmax(0.9 / pow((double)ratio, 1.0 / 5.0), df));
        }
        s_dt = nd;
        a.dstats[2] = (double)ratio;
      }
      __syncthreads();
    }
    // dense output at tout: x = (tout - t0)/(t1 - t0), Horner-free power sum (torchdiffeq _interp_evaluate)
    const float x = (float)((tout - s_tprev) / (s_tnext - s_tprev));
    float* out = a.sol + (size_t)ti * BC;
    for (int e = threadIdx.x; e < BC; e += ODE_THREADS) {
      float total = a.interp[e] + x * a.interp[(size_t)BC + e];
      float xp = x;
#pragma unroll
      for (int c = 2; c < 5; ++c) {
        xp = xp * x;
        total = total + xp * a.interp[(size_t)c * BC + e];
      }
      out[e] = total;
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    a.dstats[0] = s_dt;
    a.dstats[1] = s_tcur;
    a.stats[5] = nsteps;
  }
}

__global__ __launch_bounds__(ODE_THREADS) void k_ode_solve(OdeArgs a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* Q2s = smem;
  float* Q3s = smem + M * LDQ;
  Shared& sh = *reinterpret_cast<Shared*>(smem + (M + 32) * LDQ);
  load_weight_images(a.Q2, a.Q3, Q2s, Q3s, false);
  if (threadIdx.x < 8) a.stats[threadIdx.x] = 0;
  if (threadIdx.x < 4) a.dstats[threadIdx.x] = 0.0;
  // u[b] = U_x x_b + bx + b1 ; y = h0 ; sol[0] = h0
  for (int e = threadIdx.x; e < a.B * M; e += ODE_THREADS) {
    const int b = e / M, i = e - b * M;
    float s = 0.f;
#pragma unroll
    for (int c = 0; c < FIODE_X; ++c) s = __fmaf_rn(a.Qx[i * FIODE_X + c], a.x_feat[(size_t)b * FIODE_X + c], s);
    a.u[e] = (s + a.bx[i]) + a.b1[i];
  }
  for (int e = threadIdx.x; e < a.B * C; e += ODE_THREADS) {
    a.y[e] = a.h0[e];
    a.sol[e] = a.h0[e];
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, half = lane >> 5, col = lane & 31;
  float q1[4][5];
#pragma unroll
  for (int mb = 0; mb < 4; ++mb)
#pragma unroll
    for (int s = 0; s < 5; ++s) q1[mb][s] = a.Q1[(32 * mb + col) * C + 2 * s + half];
  if (a.method == 0) solve_rk4(a, Q2s, Q3s, q1, sh);
  else solve_dopri5(a, Q2s, Q3s, q1, sh);
  if (threadIdx.x == 0) a.stats[4] = sh.last_exit;
}

inline size_t al(size_t x) { return (x + 255) & ~(size_t)255; }

}  // namespace

extern "C" size_t fiode_odeint_workspace_bytes(int32_t batch) {
  if (batch <= 0) return 256;
  const size_t BC = (size_t)batch * C * 4;
  return al((size_t)batch * M * 4) + 4 * al(BC) + al(7 * BC) + al(5 * BC) + al(64);
}

extern "C" int fiode_odeint(void* stream, const fiode_ode_config* cfg, const fiode_dyn_config* dyn,
                            const fiode_dyn_weights* w, const float* x_feat, const float* h0, const double* times,
                            float* solution, int32_t* stats, double* dstats, void* workspace, size_t workspace_bytes) {
  if (!cfg || !dyn || !w) return FIODE_EINVAL;
  if (dyn->n_hidden != C || dyn->mlp_size != M || dyn->x_dim != FIODE_X) return FIODE_ESHAPE;
  if (dyn->qp_max_iter < 1 || dyn->qp_max_iter > 32) return FIODE_EINVAL;
  if (cfg->batch <= 0 || cfg->batch > FIODE_ODE_MAX_BATCH || cfg->n_times < 2) return FIODE_EINVAL;
  if (cfg->method != FIODE_ODE_RK4 && cfg->method != FIODE_ODE_DOPRI5) return FIODE_EINVAL;
  if (cfg->method == FIODE_ODE_RK4 && !(cfg->step_size > 0)) return FIODE_EINVAL;
  if (cfg->method == FIODE_ODE_DOPRI5 && !(cfg->rtol > 0 && cfg->atol > 0)) return FIODE_EINVAL;
  if (!x_feat || !h0 || !times || !solution || !stats || !dstats || !workspace) return FIODE_EINVAL;
  if (workspace_bytes < fiode_odeint_workspace_bytes(cfg->batch)) return FIODE_EWORKSPACE;
  OdeArgs a{};
  a.B = cfg->batch; a.n_times = cfg->n_times; a.method = cfg->method;
  a.max_steps = cfg->max_steps > 0 ? cfg->max_steps : 100000;
  a.rtol = cfg->rtol; a.atol = cfg->atol; a.step_size = cfg->step_size;
  a.d.alpha_1 = dyn->alpha_1; a.d.alpha_2 = dyn->alpha_2; a.d.sigma_1 = dyn->sigma_1;
  a.d.tol = dyn->qp_tol; a.d.scale_nominal = dyn->scale_nominal; a.d.max_iter = dyn->qp_max_iter;
  a.x_feat = x_feat; a.h0 = h0; a.times = times;
  a.Q1 = w->Q1; a.b1 = w->b1; a.Qx = w->Qx; a.bx = w->bx; a.Q2 = w->Q2; a.b2 = w->b2; a.Q3 = w->Q3; a.b3 = w->b3;
  a.sol = solution; a.stats = stats; a.dstats = dstats;
  char* ws = static_cast<char*>(workspace);
  const size_t BC = (size_t)a.B * C * 4;
  size_t o = 0;
  a.u = reinterpret_cast<float*>(ws + o); o += al((size_t)a.B * M * 4);
  a.y = reinterpret_cast<float*>(ws + o); o += al(BC);
  a.yi = reinterpret_cast<float*>(ws + o); o += al(BC);
  a.ft = reinterpret_cast<float*>(ws + o); o += al(BC);
  a.ynew = reinterpret_cast<float*>(ws + o); o += al(BC);
  a.k = reinterpret_cast<float*>(ws + o); o += al(7 * BC);
  a.interp = reinterpret_cast<float*>(ws + o); o += al(5 * BC);
  hipStream_t st = static_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(k_ode_solve, dim3(1), dim3(ODE_THREADS), (size_t)(M + 32) * LDQ * sizeof(float) + sizeof(Shared),
                     st, a);
  FIODE_HIP_CHECK(hipGetLastError());
  return FIODE_OK;
}
