// Standalone FastBarrierProjectionNoUpper (barrier_projection.py:217-313) and eval-mode
// eval_dot (dynamics/classification.py:104-132) for gfx950.
//
// The reference's bisection stops every row at the first iteration where max|eps| < tol over the
// whole batch, reading that max on the host each iteration (barrier_projection.py:247-249).  Each
// row's bisection path is independent of the others, so the same exit is found without host
// syncs in two passes: pass 1 runs all max_iter iterations per row and AND-reduces the per-row
// 32-bit "converged at iteration i" masks into one word; pass 2 reads the word's lowest set bit K
// and re-runs each row to exactly iteration K.
#include "common.h"
#include "tile.h"
#include "../../include/fiode.h"

namespace {
using namespace fiode_tile;

__global__ __launch_bounds__(256) void k_qp_mask(int n, const float* lower, const float* nominal, int max_iter,
                                                 float tol, uint32_t* word) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t conv = 0xFFFFFFFFu;
  if (r < n) {
    float lo[C], nm[C], v[C], mu;
    load_row10(lower + (size_t)r * C, lo);
    load_row10(nominal + (size_t)r * C, nm);
    conv = qp_bisect(lo, nm, max_iter - 1, tol, v, mu);
  }
  conv = wave_and(conv);
  if ((threadIdx.x & 63) == 0) atomicAnd(word, conv);
}

__global__ __launch_bounds__(256) void k_qp_final(int n, const float* lower, const float* nominal, int max_iter,
                                                  float tol, const uint32_t* word, float* v_out, float* mu_out,
                                                  int32_t* exit_iter) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  const int K = qp_exit_iter(*word, max_iter);
  if (r == 0 && exit_iter) *exit_iter = K;
  if (r >= n) return;
  float lo[C], nm[C], v[C], mu;
  load_row10(lower + (size_t)r * C, lo);
  load_row10(nominal + (size_t)r * C, nm);
  qp_bisect(lo, nm, K, tol, v, mu);
  store_row10(v_out + (size_t)r * C, v);
  if (mu_out) mu_out[r] = mu;
}

__global__ __launch_bounds__(256) void k_qp_bwd(int n, const float* g, const float* v, const float* mu,
                                                const float* nominal, float* g_lower, float* g_nominal) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= n) return;
  float gg[C], vv[C], nm[C], gn[C], gl[C];
  load_row10(g + (size_t)r * C, gg);
  load_row10(v + (size_t)r * C, vv);
  load_row10(nominal + (size_t)r * C, nm);
  qp_backward_row(gg, vv, mu[r], nm, gn, gl);
  if (g_lower) store_row10(g_lower + (size_t)r * C, gl);
  if (g_nominal) store_row10(g_nominal + (size_t)r * C, gn);
}

// ---- eval_dot (eval mode) ------------------------------------------------------------------------
struct DynEvalArgs {
  int N, S, B;
  DynScalars d;
  const float* x_feat;
  const float* h;
  const float *Q1, *b1, *Qx, *bx, *Q2, *b2, *Q3, *b3;
  uint32_t* word;
  float* u;      // [B][M]
  float* ft;     // [N][C]
  float* f;      // [N][C]
  int32_t* exit_iter;
};

__global__ __launch_bounds__(128) void k_dyn_static(DynEvalArgs a) {
  const int b = blockIdx.x, i = threadIdx.x;
  if (b == 0 && i == 0) *a.word = 0xFFFFFFFFu;
  float s = 0.f;
  const float* xb = a.x_feat + (size_t)b * FIODE_X;
#pragma unroll
  for (int c = 0; c < FIODE_X; ++c) s = __fmaf_rn(a.Qx[i * FIODE_X + c], xb[c], s);
  a.u[(size_t)b * M + i] = (s + a.bx[i]) + a.b1[i];
}

__global__ __launch_bounds__(256) void k_dyn_fwd(DynEvalArgs a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* Q2s = smem;
  float* Q3s = smem + M * LDQ;
  load_weight_images(a.Q2, a.Q3, Q2s, Q3s);
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, half = lane >> 5, col = lane & 31;
  float q1[4][5];
#pragma unroll
  for (int mb = 0; mb < 4; ++mb)
#pragma unroll
    for (int s = 0; s < 5; ++s) q1[mb][s] = a.Q1[(32 * mb + col) * C + 2 * s + half];
  const uint32_t kw[4] = {0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu};
  const int ntiles = (a.N + 31) / 32;
  for (int tile = blockIdx.x * FIODE_WAVES + wave; tile < ntiles; tile += gridDim.x * FIODE_WAVES) {
    const int row = tile * 32 + col;
    const bool valid = row < a.N;
    const int rr = valid ? row : a.N - 1;
    const int b = rr / a.S;
    float h[C];
    load_row10(a.h + (size_t)rr * C, h);
    f32x16 z1[4], z2[4];
    const f32x16 z3 = mlp_tile<false>(Q2s, Q3s, q1, a.u + (size_t)b * M, a.b2, a.b3, h, kw, kw, 1.0f, col, half, z1, z2);
    float ft[C], lower[C], nominal[C], sig[C], span[C], v[C], mu;
    gather_ft(z3, half, ft);
    barrier_nominal(a.d, h, ft, lower, nominal, sig, span);
    uint32_t conv = qp_bisect(lower, nominal, a.d.max_iter - 1, a.d.tol, v, mu);
    if (!valid) conv = 0xFFFFFFFFu;
    conv = wave_and(conv);
    if (lane == 0) atomicAnd(a.word, conv);
    if (valid && half == 0) store_row10(a.ft + (size_t)row * C, ft);
  }
}

__global__ __launch_bounds__(256) void k_dyn_final(DynEvalArgs a) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  const int K = qp_exit_iter(*a.word, a.d.max_iter);
  if (r == 0 && a.exit_iter) *a.exit_iter = K;
  if (r >= a.N) return;
  float h[C], ft[C], lower[C], nominal[C], sig[C], span[C], v[C], mu;
  load_row10(a.h + (size_t)r * C, h);
  load_row10(a.ft + (size_t)r * C, ft);
  barrier_nominal(a.d, h, ft, lower, nominal, sig, span);
  qp_bisect(lower, nominal, K, a.d.tol, v, mu);
  store_row10(a.f + (size_t)r * C, v);
}

inline size_t al(size_t x) { return (x + 255) & ~(size_t)255; }

}  // namespace

extern "C" int fiode_qp_forward(void* stream, int32_t n, int32_t c, const float* lower, const float* nominal,
                                int32_t max_iter, float tol, float* v, float* mu, int32_t* exit_iter,
                                void* workspace, size_t workspace_bytes) {
  if (c != C) return FIODE_ESHAPE;
  if (n < 0 || max_iter < 1 || max_iter > 32 || !workspace || workspace_bytes < 16) return FIODE_EINVAL;
  if (n == 0) return FIODE_OK;
  if (!lower || !nominal || !v) return FIODE_EINVAL;
  hipStream_t st = static_cast<hipStream_t>(stream);
  uint32_t* word = static_cast<uint32_t*>(workspace);
  FIODE_HIP_CHECK(hipMemsetAsync(word, 0xFF, 4, st));
  const int blocks = (n + 255) / 256;
  hipLaunchKernelGGL(k_qp_mask, dim3(blocks), dim3(256), 0, st, n, lower, nominal, max_iter, tol, word);
  FIODE_HIP_CHECK(hipGetLastError());
  hipLaunchKernelGGL(k_qp_final, dim3(blocks), dim3(256), 0, st, n, lower, nominal, max_iter, tol, word, v, mu,
                     exit_iter);
  FIODE_HIP_CHECK(hipGetLastError());
  return FIODE_OK;
}

extern "C" int fiode_qp_backward(void* stream, int32_t n, int32_t c, const float* g, const float* v,
                                 const float* mu, const float* lower, const float* nominal, float* g_lower,
                                 float* g_nominal) {
  (void)lower;   // the reference's Jacobian depends on lower only through v (barrier_projection.py:288)
  if (c != C) return FIODE_ESHAPE;
  if (n < 0) return FIODE_EINVAL;
  if (n == 0) return FIODE_OK;
  if (!g || !v || !mu || !nominal) return FIODE_EINVAL;
  hipStream_t st = static_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(k_qp_bwd, dim3((n + 255) / 256), dim3(256), 0, st, n, g, v, mu, nominal, g_lower, g_nominal);
  FIODE_HIP_CHECK(hipGetLastError());
  return FIODE_OK;
}

extern "C" size_t fiode_dyn_eval_workspace_bytes(int32_t n) {
  if (n <= 0) return 256;
  return al(16) + al((size_t)n * M * 4) + al((size_t)n * C * 4);
}

extern "C" int fiode_dyn_eval(void* stream, const fiode_dyn_config* dyn, const fiode_dyn_weights* w, int32_t batch,
                              int32_t rows_per_image, const float* x_feat, const float* h, float* f,
                              int32_t* exit_iter, void* workspace, size_t workspace_bytes) {
  if (!dyn || !w) return FIODE_EINVAL;
  if (dyn->n_hidden != C || dyn->mlp_size != M || dyn->x_dim != FIODE_X) return FIODE_ESHAPE;
  if (dyn->qp_max_iter < 1 || dyn->qp_max_iter > 32) return FIODE_EINVAL;
  if (batch < 0 || rows_per_image <= 0) return FIODE_EINVAL;
  const long long nl = (long long)batch * rows_per_image;
  if (nl > (1LL << 30)) return FIODE_EINVAL;
  const int n = (int)nl;
  if (n == 0) return FIODE_OK;
  if (!x_feat || !h || !f || !workspace) return FIODE_EINVAL;
  if (workspace_bytes < fiode_dyn_eval_workspace_bytes(n)) return FIODE_EWORKSPACE;
  char* ws = static_cast<char*>(workspace);
  DynEvalArgs a{};
  a.N = n; a.S = rows_per_image; a.B = batch;
  a.d.alpha_1 = dyn->alpha_1; a.d.alpha_2 = dyn->alpha_2; a.d.sigma_1 = dyn->sigma_1;
  a.d.tol = dyn->qp_tol; a.d.scale_nominal = dyn->scale_nominal; a.d.max_iter = dyn->qp_max_iter;
  a.x_feat = x_feat; a.h = h;
  a.Q1 = w->Q1; a.b1 = w->b1; a.Qx = w->Qx; a.bx = w->bx; a.Q2 = w->Q2; a.b2 = w->b2; a.Q3 = w->Q3; a.b3 = w->b3;
  a.word = reinterpret_cast<uint32_t*>(ws);
  a.u = reinterpret_cast<float*>(ws + al(16));
  a.ft = reinterpret_cast<float*>(ws + al(16) + al((size_t)n * M * 4));
  a.f = f;
  a.exit_iter = exit_iter;
  hipStream_t st = static_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(k_dyn_static, dim3(batch), dim3(128), 0, st, a);
  FIODE_HIP_CHECK(hipGetLastError());
  const int ntiles = (n + 31) / 32;
  hipLaunchKernelGGL(k_dyn_fwd, dim3((ntiles + FIODE_WAVES - 1) / FIODE_WAVES), dim3(256),
                     (size_t)(M + 32) * LDQ * sizeof(float), st, a);
  FIODE_HIP_CHECK(hipGetLastError());
  hipLaunchKernelGGL(k_dyn_final, dim3((n + 255) / 256), dim3(256), 0, st, a);
  FIODE_HIP_CHECK(hipGetLastError());
  return FIODE_OK;
}

extern "C" const char* fiode_error_string(int code) {
  switch (code) {
    case FIODE_OK: return "ok";
    case FIODE_EINVAL: return "invalid argument";
    case FIODE_ESHAPE: return "unsupported shape (dynamics: n_hidden=10, mlp_size=128, x_dim=10; spectral: 3x3 taps, min(cout, cin) <= 64, n <= 64; transforms: n in {8, 16, 32})";
    case FIODE_EWORKSPACE: return "workspace too small";
    default: return code >= FIODE_EHIP ? hipGetErrorString((hipError_t)(code - FIODE_EHIP)) : "unknown error";
  }
}

extern "C" int fiode_abi_version(void) { return FIODE_ABI_VERSION; }
