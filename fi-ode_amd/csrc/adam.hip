// Adam / AdamW parameter update over every parameter tensor of the model in ONE launch (gfx950):
// the optimizer step that closes each training step (pl_modules.py:97-147 configure_optimizers ->
// torch.optim.Adam; fiode_amd/optim.py FiodeAdam).  torch's fused multi-tensor Adam takes ~45 us
// for the KWLarge model's 2.6 M parameters (33 tensors, 73 MB of p/g/m/v traffic) on the step's
// critical path; this kernel is plain HBM streaming: each workgroup owns 1024 consecutive elements
// of one tensor (float4 per thread), the tensor table travels in the kernel arguments (captured by
// value in a hipGraph), and the per-element arithmetic is torch's fused Adam formula in the same
// operation order (fp32 element math; the scalar factors formed in double from the host's values):
//   g  = maximize ? -grad : grad;  AdamW: p -= lr wd p;  Adam: g += wd p
//   m  = b1 m + (1 - b1) g;        v = b2 v + (1 - b2) g g
//   p -= (lr / (1 - b1^t)) m / (sqrt(v) / sqrt(1 - b2^t) + eps)
// t is the tensor's step count AFTER this step's increment, read from the device (capturable) or
// given by the host.
// Step guard (fiode_step_guard): a step whose train_ode solve failed (status word) or whose loss is
// not finite -- or, on N ranks, any rank's such step (the guard slot of the all-reduced gradient
// bucket) -- leaves p, m, v and the step counts as they were, like torch.cuda.amp's found_inf skip
// but decided on the device; k_adam_steps counts the skipped steps in a sticky word.  Unlike
// found_inf the guard does not scan the gradients: a finite loss with a non-finite gradient still
// updates; a caller that needs that check writes it into the guard's flag word.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "common.h"
#include "fiode.h"

namespace {

constexpr int NT = 256;
constexpr int PER_BLOCK = NT * 4;
constexpr int MAXT = FIODE_ADAM_MAX_TENSORS;

struct AdamArgs {
  int n;                       // tensors
  int decoupled, maximize;
  float lr, b1, omb1, b2, omb2, eps, wd;   // fp32 operands; 1 - beta formed in double
  double lr_d, b1_d, b2_d;     // for the bias corrections of device step counts
  float step_size_h, bc2_sqrt_h;  // bias-corrected factors of a host step count
  double step_h;
  int blk0[MAXT + 1];          // first workgroup of each tensor (prefix sum)
  int64_t numel[MAXT];
  float* p[MAXT];
  const float* g[MAXT];
  float* m[MAXT];
  float* v[MAXT];
  const float* t_dev[MAXT];     // per-tensor step count on the device (capturable Adam)
  const void* lr_dev;          // device learning rate (tensor lr) or null
  int lr_dev_is_double;
  fiode_step_guard guard;      // all-null: no guard
};

__device__ __forceinline__ bool guard_skip(const fiode_step_guard& g) {
  bool bad = false;
  if (g.flag) bad = bad || !(*g.flag == 0.f);            // nonzero or NaN
  if (g.loss) bad = bad || !isfinite(*g.loss);
#pragma unroll
  for (int i = 0; i < FIODE_GUARD_MAX_STATUS; ++i)
    if (g.status[i]) bad = bad || *g.status[i] != 0;
  return bad;
}

// the step counts of a guarded step: +1 unless the guard skips it (then the sticky count +1)
__global__ __launch_bounds__(64) void k_adam_steps(const AdamArgs a) {
  const bool skip = guard_skip(a.guard);
  for (int t = threadIdx.x; t < a.n; t += blockDim.x)
    if (!skip && a.t_dev[t]) *const_cast<float*>(a.t_dev[t]) += 1.0f;
  if (threadIdx.x == 0 && skip && a.guard.skipped) *a.guard.skipped += 1;
}

__global__ void k_guard_flag(const fiode_step_guard g, float* out) {
  if (threadIdx.x == 0) out[0] = guard_skip(g) ? 1.0f : 0.0f;
}

struct Coef {
  float lr, b1, omb1, b2, omb2, eps, wd, step_size, bc2_sqrt;
  int decoupled, maximize;
};

__device__ __forceinline__ void adam_elem(const Coef& c, float& p, float g, float& m, float& v) {
  if (c.maximize) g = -g;
  if (c.wd != 0.f) {
    if (c.decoupled) p -= c.lr * c.wd * p;
    else g += p * c.wd;
  }
  m = c.b1 * m + c.omb1 * g;
  v = c.b2 * v + c.omb2 * g * g;
  const float denom = (sqrtf(v) / c.bc2_sqrt) + c.eps;
  p -= c.step_size * m / denom;
}

__global__ __launch_bounds__(NT) void k_adam(const AdamArgs a) {
  if (guard_skip(a.guard)) return;
  const int b = blockIdx.x;
  int t = 0;
  while (t + 1 < a.n && a.blk0[t + 1] <= b) ++t;
  Coef c;
  double lr_d = a.lr_d;
  float lr = a.lr;
  if (a.lr_dev) {
    lr_d = a.lr_dev_is_double ? *(const double*)a.lr_dev : (double)*(const float*)a.lr_dev;
    lr = (float)lr_d;
  }
  c.lr = lr; c.b1 = a.b1; c.omb1 = a.omb1; c.b2 = a.b2; c.omb2 = a.omb2; c.eps = a.eps; c.wd = a.wd;
  c.decoupled = a.decoupled; c.maximize = a.maximize;
  if (a.t_dev[t]) {
    const double step = (double)*a.t_dev[t];
    c.step_size = (float)(lr_d / (1.0 - pow(a.b1_d, step)));
    c.bc2_sqrt = (float)sqrt(1.0 - pow(a.b2_d, step));
  } else {
    c.step_size = a.lr_dev ? (float)(lr_d / (1.0 - pow(a.b1_d, a.step_h))) : a.step_size_h;
    c.bc2_sqrt = a.bc2_sqrt_h;
  }

  const int64_t n = a.numel[t];
  const int64_t e0 = (int64_t)(b - a.blk0[t]) * PER_BLOCK + 4 * threadIdx.x;
  float* P = a.p[t];
  const float* G = a.g[t];
  float* M = a.m[t];
  float* V = a.v[t];
  const bool vec = ((((uintptr_t)P) | ((uintptr_t)G) | ((uintptr_t)M) | ((uintptr_t)V)) & 15) == 0;
  if (vec && e0 + 4 <= n) {
    float4 p = *(const float4*)(P + e0), g = *(const float4*)(G + e0);
    float4 m = *(const float4*)(M + e0), v = *(const float4*)(V + e0);
    adam_elem(c, p.x, g.x, m.x, v.x);
    adam_elem(c, p.y, g.y, m.y, v.y);
    adam_elem(c, p.z, g.z, m.z, v.z);
    adam_elem(c, p.w, g.w, m.w, v.w);
    *(float4*)(P + e0) = p;
    *(float4*)(M + e0) = m;
    *(float4*)(V + e0) = v;
  } else {
    for (int64_t e = e0; e < e0 + 4 && e < n; ++e) {
      float p = P[e], m = M[e], v = V[e];
      adam_elem(c, p, G[e], m, v);
      P[e] = p; M[e] = m; V[e] = v;
    }
  }
}

}  // namespace

extern "C" int fiode_adam_step(void* stream, const fiode_adam_config* cfg, float* const* params,
                               const float* const* grads, float* const* exp_avg, float* const* exp_avg_sq,
                               const int64_t* numel, float* const* step, const fiode_step_guard* guard) {
  if (!cfg || cfg->n_tensors < 0 || cfg->n_tensors > MAXT) return FIODE_EINVAL;
  if (cfg->n_tensors == 0) return FIODE_OK;
  if (!params || !grads || !exp_avg || !exp_avg_sq || !numel) return FIODE_EINVAL;
  AdamArgs a{};
  a.n = cfg->n_tensors;
  a.decoupled = cfg->decoupled != 0; a.maximize = cfg->maximize != 0;
  a.lr = (float)cfg->lr; a.eps = (float)cfg->eps; a.wd = (float)cfg->weight_decay;
  a.b1 = (float)cfg->beta1; a.omb1 = (float)(1.0 - cfg->beta1);
  a.b2 = (float)cfg->beta2; a.omb2 = (float)(1.0 - cfg->beta2);
  a.lr_d = cfg->lr; a.b1_d = cfg->beta1; a.b2_d = cfg->beta2;
  a.step_size_h = (float)(cfg->lr / (1.0 - pow(cfg->beta1, cfg->step)));
  a.bc2_sqrt_h = (float)sqrt(1.0 - pow(cfg->beta2, cfg->step));
  a.step_h = cfg->step;
  a.lr_dev = cfg->lr_dev;
  a.lr_dev_is_double = cfg->lr_dev_is_double != 0;
  if (guard) a.guard = *guard;
  if (cfg->increment_steps && !step) return FIODE_EINVAL;
  int64_t blocks = 0;
  for (int i = 0; i < a.n; ++i) {
    if (numel[i] < 0 || (numel[i] > 0 && (!params[i] || !grads[i] || !exp_avg[i] || !exp_avg_sq[i])))
      return FIODE_EINVAL;
    a.blk0[i] = (int)blocks;
    blocks += (numel[i] + PER_BLOCK - 1) / PER_BLOCK;
    if (blocks > INT32_MAX / 2) return FIODE_ESHAPE;
    a.numel[i] = numel[i];
    a.p[i] = params[i]; a.g[i] = grads[i]; a.m[i] = exp_avg[i]; a.v[i] = exp_avg_sq[i];
    a.t_dev[i] = step ? step[i] : nullptr;
  }
  a.blk0[a.n] = (int)blocks;
  // the step counts advance even when every tensor is empty (torch's Adam counts such steps too)
  if (cfg->increment_steps) {
    hipLaunchKernelGGL(k_adam_steps, dim3(1), dim3(64), 0, (hipStream_t)stream, a);
    const hipError_t e0 = hipGetLastError();
    if (e0 != hipSuccess) return FIODE_EHIP + (int)e0;
  }
  if (blocks == 0) return FIODE_OK;
  hipLaunchKernelGGL(k_adam, dim3((unsigned)blocks), dim3(NT), 0, (hipStream_t)stream, a);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? FIODE_OK : FIODE_EHIP + (int)e;
}

extern "C" int fiode_step_guard_flag(void* stream, const fiode_step_guard* guard, float* flag_out) {
  if (!guard || !flag_out) return FIODE_EINVAL;
  fiode_step_guard g = *guard;
  g.flag = nullptr;
  g.skipped = nullptr;
  hipLaunchKernelGGL(k_guard_flag, dim3(1), dim3(64), 0, (hipStream_t)stream, g, flag_out);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? FIODE_OK : FIODE_EHIP + (int)e;
}
