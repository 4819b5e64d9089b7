/*
 * fiode.h -- C-ABI of the MI355X (gfx950) FI-ODE hot path (libfiode.so).
 *
 * The reference (yjhuangcd/FI-ODE) has no FFI: its seams are hydra `_target_` classes and
 * duck-typed nn.Module / autograd.Function objects.  Each entry point
 * below replaces one of those seams; the Python host mirror (fi-ode_amd/fiode_amd) binds them
 * with ctypes (INTEGRATION.md shows the binding a maintainer would add to the reference).
 *
 * Conventions
 *   - every pointer is a device pointer to caller-owned memory (PyTorch caching allocator),
 *     fp32 row-major, nn.Linear layout [out][in]; the library never allocates or frees;
 *   - work is stream-ordered on `stream` (a hipStream_t passed as void*), with no host syncs;
 *   - entry points return 0 on success, a FIODE_E* code otherwise; they never throw.
 *   - shapes: C (classes = n_hidden = ODE state) = 10, M (mlp_size) = 128, X (x_dim) = 10.
 */
#ifndef FIODE_H_
#define FIODE_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ABI 4 (round 6): fiode_sconv_config gained `nchw` (20 bytes, was 16), the one-launch block inverse
   (n = 128 .. 512) needs a larger workspace (fiode_block_inverse_workspace_bytes), fiode_gemm added.
   ABI 5: fiode_gemm_desc gained `max_workgroups` (in what was its tail padding; the size is unchanged,
   so a caller built against ABI 4 would pass an undefined value there). */
#define FIODE_ABI_VERSION 5

#if defined(__GNUC__)
#define FIODE_API __attribute__((visibility("default")))
#else
#define FIODE_API
#endif

enum {
  FIODE_OK = 0,
  FIODE_EINVAL = 1,       /* bad argument / NULL where required                   */
  FIODE_ESHAPE = 2,       /* C, M or X not supported by this build                */
  FIODE_EWORKSPACE = 3,   /* workspace smaller than fiode_*_workspace_bytes()     */
  FIODE_EHIP = 100        /* a HIP runtime error; FIODE_EHIP + hipError_t         */
};

/* TRAJECTORY: rows s < n_uniform are UniformSimplex draws (as COMPOSITE), rows s >= n_uniform are
   read from io->h laid out [B][S - n_uniform][C] (TrajectorySampler, sampler.py:156-166).          */
enum { FIODE_SAMPLER_GIVEN = 0, FIODE_SAMPLER_COMPOSITE = 1, FIODE_SAMPLER_DECISION_BOUNDARY = 2,
       FIODE_SAMPLER_TRAJECTORY = 3 };
enum { FIODE_DROPOUT_OFF = 0, FIODE_DROPOUT_GIVEN = 1, FIODE_DROPOUT_PHILOX = 2 };

/* Effective (post-Cayley) dynamics weights of OrthoClassDynProjectSimplexLips
 * (dynamics/classification.py:68-75): hidden_to_mlp, U_x, mlp_to_mlp, mlp_to_hidden. */
typedef struct fiode_dyn_weights {
  const float* Q1; const float* b1; /* hidden_to_mlp  [M][C], [M] */
  const float* Qx; const float* bx; /* U_x            [M][X], [M] */
  const float* Q2; const float* b2; /* mlp_to_mlp     [M][M], [M] */
  const float* Q3; const float* b3; /* mlp_to_hidden  [C][M], [C] */
} fiode_dyn_weights;

/* Constructor fields of OrthoClassDynProjectSimplexLips read by the hot path
 * (classification.py:32-66) and of its FastBarrierProjectionNoUpper (classification.py:63). */
typedef struct fiode_dyn_config {
  int32_t n_hidden;      /* C, must be 10   */
  int32_t mlp_size;      /* M, must be 128  */
  int32_t x_dim;         /* X, must be 10   */
  float alpha_1, alpha_2, sigma_1;
  int32_t scale_nominal; /* sigmoid rescale of the nominal velocity (classification.py:110-112) */
  float dropout;         /* p of nn.Dropout (classification.py:49)                             */
  int32_t qp_max_iter;   /* 1..32 (reference: 30)                                              */
  float qp_tol;          /* reference: 1e-4                                                    */
} fiode_dyn_config;

/* One LyapunovLearning.compute_loss (pl_modules.py:390-502): B images x S samples. */
typedef struct fiode_lyap_config {
  int32_t batch;         /* B                                                                  */
  int32_t sample_size;   /* S (h_sample_size); rows N = B*S, row = b*S + s                     */
  int32_t n_uniform;     /* S1: UniformSimplex rows per image (first S1); S-S1 CorrectCone     */
  int32_t sampler;       /* FIODE_SAMPLER_*                                                    */
  int32_t dropout_mode;  /* FIODE_DROPOUT_*                                                    */
  float kappa;           /* current_kappa (pl_modules.py:447-451)                              */
  uint64_t seed;         /* Philox key (sampler + dropout)                                     */
  uint64_t offset;       /* Philox counter offset (advance per step)                           */
} fiode_lyap_config;

typedef struct fiode_lyap_io {
  const float* x_feat;   /* [B][X] static features = param_map(x) (init_coordinates.py:35)     */
  const int64_t* y;      /* [B] labels                                                         */
  const float* h;        /* [N][C] samples (GIVEN) or [B][S-n_uniform][C] trajectory rows (TRAJECTORY) */
  const uint8_t* masks;  /* [4][N][M] keep masks (loss L1, loss L2, log L1, log L2), GIVEN mode */
  float* scalars;        /* [8] out: loss, eff_count, mean_active, qp_exit_loss, qp_exit_log,
                            viol_sum, active_count, rows                                       */
  /* optional per-row outputs (NULL = not written) */
  float* h_out;          /* [N][C] samples used                                                */
  float* V;              /* [N] DecisionBoundary V                                             */
  float* Vdot;           /* [N] jvp V-dot                                                      */
  float* f;              /* [N][C] loss-pass eval_dot                                          */
  float* f_log;          /* [N][C] logging-pass eval_dot                                       */
  float* qp_lower;       /* [N][C] QP lower bound                                              */
  float* qp_nominal;     /* [2][N][C] QP nominal (loss pass, logging pass)                     */
  float* g_ftilde;       /* [N][C] d loss / d mlp_to_hidden output                             */
  /* optional profiling: hipEvent_t handles recorded on `stream` before the first kernel and
   * after each of the FIODE_LYAP_NKERNELS kernels (needs n_events >= FIODE_LYAP_NKERNELS + 1) */
  void* const* events;
  int32_t n_events;
  /* optional device-resident Philox offset addend (NULL = 0): offset = cfg.offset + *offset_dev,
   * so a captured hipGraph of the step draws fresh samples / dropout masks on every replay when
   * the graph also advances the counter */
  const uint64_t* offset_dev;
  /* optional sampler draws (parity checks): NULL = in-kernel Philox.  Exp(1) variates in the
   * reference's draw shapes (sampler.py:36, 116, 142): COMPOSITE / TRAJECTORY: UniformSimplex
   * [n_uniform][C] followed by CorrectCone [B][S - n_uniform][C] (TRAJECTORY: the uniform part
   * only); DECISION_BOUNDARY: [B][S][C - 1]. */
  const float* exp_draws;
  float* exp_draws_out;     /* optional out: the Exp(1) variates the sampler used, same layout  */
  uint32_t* keep_words_out; /* optional out: [4][N][4] dropout keep words of the 4 mask sets
                               (bit t of word mb = keep hidden unit 32 mb + t)                  */
  /* optional device-resident kappa (NULL = cfg.kappa): the kappa ramp of pl_modules.py:447-448
   * (global_step / kappa_length * kappa while global_step < kappa_length) computed on the device,
   * so a captured step follows it on every replay */
  const float* kappa_dev;
} fiode_lyap_io;

/* kernels of one fiode_lyap_step, in launch order (for the profiling events) */
#define FIODE_LYAP_NKERNELS 6
/* static_proj, prep (sampler + dropout words), fwd (2 eval_dot passes), bwd (QP finalize + loss +
 * activation grads + weight-gradient GEMMs, one partial slab per workgroup), reduce, static_grads */

typedef struct fiode_lyap_grads {  /* outputs, overwritten: d loss / d (effective weights) */
  float *Q1, *b1, *Qx, *bx, *Q2, *b2, *Q3, *b3;
  float* x_feat;                   /* [B][X] gradient into the backbone */
} fiode_lyap_grads;

/* Workspace bytes for fiode_lyap_step (depends on B, S only). */
FIODE_API size_t fiode_lyap_workspace_bytes(const fiode_lyap_config* cfg, const fiode_dyn_config* dyn);

/* The fused forward-invariance training step: sampler fan-out, two eval_dot passes (loss pass
 * with dropout masks 0/1, logging pass with masks 2/3), DecisionBoundary V / V-dot, hinge loss,
 * logging statistics and the gradient of mean(relu(Vdot + kappa V)) w.r.t. the effective
 * weights and the static features.  Replaces LyapunovLearning.compute_loss + loss.backward()
 * below the Cayley maps (pl_modules.py:394-484; classification.py:96-115;
 * barrier_projection.py:217-313; lya_cands.py:79-94; sampler.py:195-216). */
FIODE_API int fiode_lyap_step(void* stream, const fiode_lyap_config* cfg, const fiode_dyn_config* dyn,
                    const fiode_dyn_weights* w, const fiode_lyap_io* io, fiode_lyap_grads* grads,
                    void* workspace, size_t workspace_bytes);

/* FastBarrierProjectionNoUpper forward (barrier_projection.py:220-269) with the reference's
 * batch-global exit.  exit_iter: device int32[1] (0-based exit iteration).  workspace: >= 16 B. */
FIODE_API int fiode_qp_forward(void* stream, int32_t n, int32_t c, const float* lower, const float* nominal,
                     int32_t max_iter, float tol, float* v, float* mu, int32_t* exit_iter,
                     void* workspace, size_t workspace_bytes);

/* FastBarrierProjectionNoUpper backward (barrier_projection.py:271-311), O(C) per row. */
FIODE_API int fiode_qp_backward(void* stream, int32_t n, int32_t c, const float* g, const float* v,
                      const float* mu, const float* lower, const float* nominal, float* g_lower,
                      float* g_nominal);

/* eval_dot / eval_dot_light / ode_forward in eval mode (no dropout; classification.py:104-132):
 * f[N][C] for h[N][C], rows grouped S per image of x_feat[B][X] (N = B*S).  The QP exit is
 * global over the N rows of the call.  workspace: fiode_dyn_eval_workspace_bytes(). */
FIODE_API size_t fiode_dyn_eval_workspace_bytes(int32_t n);
FIODE_API int fiode_dyn_eval(void* stream, const fiode_dyn_config* dyn, const fiode_dyn_weights* w,
                   int32_t batch, int32_t rows_per_image, const float* x_feat, const float* h,
                   float* f, int32_t* exit_iter, void* workspace, size_t workspace_bytes);

/* ---- ODE solves (models.py:211-242 IVP.integrate -> torchdiffeq.odeint) ------------------- */
enum { FIODE_ODE_RK4 = 0, FIODE_ODE_DOPRI5 = 1 };
#define FIODE_ODE_MAX_BATCH 4096          /* the differentiable train_ode solve (fiode_odetrain_*) */
#define FIODE_ODEINT_MAX_BATCH 65536      /* the eval-mode solve (fiode_odeint); also <= 256 x CUs */

typedef struct fiode_ode_config {
  int32_t method;        /* FIODE_ODE_RK4 (fixed grid, 3/8 rule) or FIODE_ODE_DOPRI5          */
  int32_t batch;         /* B rows (one per image), <= FIODE_ODEINT_MAX_BATCH                  */
  int32_t n_times;       /* >= 2 output times (device float64 array, increasing)              */
  int32_t max_steps;     /* dopri5 step cap (<= 0: 100000)                                     */
  double rtol, atol;     /* dopri5 (make_solver_params: rtol = atol = ode_tol, pl_modules.py:26) */
  double step_size;      /* rk4 (make_solver_params: options.step_size = ode_tol, :27-33)       */
} fiode_ode_config;

FIODE_API size_t fiode_odeint_workspace_bytes(int32_t batch);

/* odeint(IVP.h_dot, (h0,), times, method, rtol/atol | step_size) with f = ode_forward in eval
 * mode (no dropout), static_state = x_feat.  solution: [n_times][B][C] (solution[0] = h0).
 * stats (device int32[8]): nfe, n_accept (rk4: steps), n_reject, status (0 ok, 2 max_steps,
 * 3 dt underflow, 4 a cross-workgroup exchange timed out: results invalid), last QP exit
 * iteration, dopri5 attempted steps, workgroups of the solve, 16-row tiles per workgroup.  dstats
 * (device double[4]): next dt, final t, last error ratio.  One persistent workgroup per 16-row tile (several tiles each past the chip's resident
 * capacity); the batch-global QP exit and the dopri5 RMS error norm are exchanged between
 * workgroups on the device (no host sync). */
FIODE_API int fiode_odeint(void* stream, const fiode_ode_config* cfg, const fiode_dyn_config* dyn,
                           const fiode_dyn_weights* w, const float* x_feat, const float* h0,
                           const double* times, float* solution, int32_t* stats, double* dstats,
                           void* workspace, size_t workspace_bytes);

/* ---- Differentiable solve for train_ode (pl_modules.py:490-500; models.py:235-241) -----------
 * y_hat = odeint(IVP.h_dot, (h0,), [t0, t1], method, ...) with the dynamics in TRAIN mode (fresh
 * dropout masks per func() call), backpropagated directly through the solve (use_adjoint False):
 *   FIODE_ODE_RK4:    options.step_size; evals E = 4 * (niters - 1), niters = ceil((t1 - t0) /
 *                     step_size + 1) in float32;
 *   FIODE_ODE_DOPRI5: rtol, atol (make_solver_params('dopri5', tol): rtol = atol = tol), torchdiffeq
 *                     0.2.2's adaptive solver incl. the gradient through its step-size controller;
 *                     E = 2 + 6 max_attempts is the eval CAPACITY (the solve's count: stats[0]);
 *                     more attempts than max_attempts (torchdiffeq: unbounded) -> stats[3] = 2 and a
 *                     NaN y_out.  Eval e of attempt n is 2 + 6 n + i (evals 0, 1: initial step). */
typedef struct fiode_odetrain_config {
  int32_t batch;         /* B (<= FIODE_ODE_MAX_BATCH)                                          */
  int32_t dropout_mode;  /* FIODE_DROPOUT_*; GIVEN: masks [E][2][B][M] uint8 0/1               */
  uint64_t seed;         /* Philox key                                                          */
  uint64_t offset;       /* Philox counter offset                                               */
  double t0, t1;         /* ts = [t0, t1] (linspace(0, t_max, 2))                               */
  double step_size;      /* rk4: make_solver_params('rk4', tol): options.step_size = tol        */
  int32_t method;        /* FIODE_ODE_RK4 (0) or FIODE_ODE_DOPRI5                               */
  int32_t max_attempts;  /* dopri5: attempt capacity (1 .. FIODE_ODETRAIN_MAX_ATTEMPTS)         */
  double rtol, atol;     /* dopri5                                                              */
} fiode_odetrain_config;
#define FIODE_ODETRAIN_MAX_ATTEMPTS 1024

FIODE_API int32_t fiode_odetrain_evals(const fiode_odetrain_config* cfg);
/* The workspace also carries the forward's saved activations to the backward. */
FIODE_API size_t fiode_odetrain_workspace_bytes(const fiode_odetrain_config* cfg);
/* y_out [B][C] = y(t1); stats (device int32[8]): nfe, accepted steps, last QP exit iteration, status
 * (0 ok, 2 attempt capacity exhausted, 3 dt underflow, 4 a cross-workgroup exchange timed out), and
 * for dopri5 n_accept, n_reject, attempts.  offset_dev: optional device addend of the Philox offset
 * (graph replay).  The forward is one persistent workgroup per tile whose workgroups exchange the
 * batch-global QP exits, so all of them must be resident at once: 4-row tiles up to B = 1,024
 * (ceil(B / 4) workgroups), 16-row tiles beyond (ceil(B / 16), B <= FIODE_ODE_MAX_BATCH). */
FIODE_API int fiode_odetrain_forward(void* stream, const fiode_odetrain_config* cfg, const fiode_dyn_config* dyn,
                                     const fiode_dyn_weights* w, const float* x_feat, const float* h0,
                                     const uint8_t* masks, const uint64_t* offset_dev, float* y_out,
                                     int32_t* stats, void* workspace, size_t workspace_bytes);
/* Byte offsets inside the workspace of the forward's saved arrays, for checkers (offsets:
 * int64[FIODE_ODETRAIN_NSAVED]): [0] stage inputs [B][E][C], [1] MLP outputs [B][E][C], [2] QP
 * outputs v [B][E][C], [3] QP mu [B][E], [4] QP nominal [B][E][C], [5] a1 [B][E][M], [6] a2
 * [B][E][M], [7] dL/d mlp output [B][E][C] (after the backward), [8] QP lower bound [B][E][C];
 * dopri5 only (else 0): [9] y_n of every attempt [A][B][C] float, [10] the attempt log [A][8]
 * double (t_n, dt_n, error ratio, accepted, eval of k_0, eval of stage 0), [11] the initial step
 * [16] double (d0, d1, d2, h0, h1, clamp0, clamp1, dt0, rms(f1 - f0)), [12] the solve's int32
 * status word (rk4: always 0, its status is stats[3]; dopri5: 0 ok; 2 attempt capacity exhausted; 3 dt underflow; 4 a cross-workgroup exchange of
 * the forward or the backward timed out -- the outputs are NaN then), [13] the dropout keep words uint32 [E][2][B][4] (bit t of word q =
 * keep hidden unit 32 q + t; the evals the solve made).  Row (b, e) = b*E + e. */
#define FIODE_ODETRAIN_NSAVED 14
FIODE_API int fiode_odetrain_saved_offsets(const fiode_odetrain_config* cfg, int64_t* offsets);
/* Given g_y = dL/dy(t1) [B][C]: all weight gradients and dL/dx_feat (overwritten).  Must follow
 * fiode_odetrain_forward on the same workspace.  dbg_gft: optional [B][E][C] dL/d mlp output. */
/* The train_ode loss term F.nll_loss(torch.log(y_hat), y) (pl_modules.py:494-497) in one launch:
 * loss[0] = -(1/B) sum_b log y_hat[b, y_b]; g_unit [B][C] = d loss / d y_hat (times the upstream
 * gradient in the caller's backward).  labels int64 [B] in [0, C). */
FIODE_API int fiode_ode_nll(void* stream, int32_t batch, const float* y_hat, const int64_t* labels, float* loss,
                            float* g_unit);
/* The same fused with the loss mix of pl_modules.py:500: total[0] = lyap_loss[0] * (1 - portion) +
 * loss_ode * portion; g_unit = portion * d loss_ode / d y_hat (= d total / d y_hat per unit). */
FIODE_API int fiode_ode_loss_mix(void* stream, int32_t batch, const float* y_hat, const int64_t* labels,
                                 const float* lyap_loss, float portion, float* loss_ode, float* total, float* g_unit);
FIODE_API int fiode_odetrain_backward(void* stream, const fiode_odetrain_config* cfg, const fiode_dyn_config* dyn,
                                      const fiode_dyn_weights* w, const float* x_feat, const float* g_y,
                                      fiode_lyap_grads* grads, float* dbg_gft, void* workspace,
                                      size_t workspace_bytes);
/* fiode_odetrain_backward in two parts, so the backbone's backward (which needs only dL/dx_feat)
 * can start before the weight gradients are summed (these may then run on another stream):
 *   _x:       the adjoint sweep (k_ot_bwd) and gx [B][X] = dL/dx_feat, plus gx_add [B][X] times
 *             gx_add_scale[0] (device scalar) when gx_add is given;
 *   _weights: the weight gradients (grads->x_feat ignored); after _x on the same workspace.
 * fiode_odetrain_backward = the same work with dL/dx_feat formed inside the weight-gradient chain
 * (one launch fewer; its x-gradient may differ from _x's in the last bits: g_u summation order). */
FIODE_API int fiode_odetrain_backward_x(void* stream, const fiode_odetrain_config* cfg, const fiode_dyn_config* dyn,
                                        const fiode_dyn_weights* w, const float* x_feat, const float* g_y, float* gx,
                                        const float* gx_add, const float* gx_add_scale, float* dbg_gft,
                                        void* workspace, size_t workspace_bytes);
FIODE_API int fiode_odetrain_backward_weights(void* stream, const fiode_odetrain_config* cfg,
                                              const fiode_dyn_config* dyn, const fiode_dyn_weights* w,
                                              const float* x_feat, fiode_lyap_grads* grads, void* workspace,
                                              size_t workspace_bytes);

/* ---- Certification grid (robustness/eval_utils.py:31-89, certify_lipschitz.py:37-143) ------ */
typedef struct fiode_certify_config {
  int32_t n_classes;     /* 10                                                                   */
  int32_t T;             /* grid density (reference: 40)                                         */
  int32_t batches;       /* cfg.batches: G // batches rows per batch, +1 tail batch (ref: 10)     */
  int32_t label;         /* the image's label (selects the column swap of get_grid_for_label)    */
  float eps;             /* cfg.eps (0.141): kappa = sqrt(2) * Lfx * eps                         */
  float min_std;         /* min(Normalize.std): Lfx = (scale_nominal ? alpha_1 : 1) / min_std    */
} fiode_certify_config;

/* Rows G of the decision-boundary grid {v in Z>=0^n : sum v = T, v_0 = max_{i>=1} v_i}; -1 if
 * unsupported (n <= 16, T <= 64, G < 2^32).  Host only. */
FIODE_API int64_t fiode_certify_grid_rows(int32_t n, int32_t T);
/* Build grid_label_0 as uint8 counts [G][n] (eta = v/T) in sample_decision_boundary's row order. */
FIODE_API int fiode_certify_grid(void* stream, int32_t n, int32_t T, uint8_t* grid);
FIODE_API size_t fiode_certify_workspace_bytes(int64_t G, int32_t batches);
/* One image: per batch of grid rows, out[b] = (max violation, max violation_larger_T) with the
 * QP exit global over the batch (eval_dot_light on the batch), exit_iters[b] its exit iteration.
 * x_feat: [X] the image's static features.  nb = batches + (G % batches != 0). */
FIODE_API int fiode_certify(void* stream, const fiode_certify_config* cfg, const fiode_dyn_config* dyn,
                            const fiode_dyn_weights* w, const float* x_feat, const uint8_t* grid, int64_t G,
                            float* out, int32_t* exit_iters, void* workspace, size_t workspace_bytes);

/* ---- Batched inverse of the Cayley maps (classification.py:282-293 convert_cayley ->
 * cayley(): (I + A)^-1 with A = U - U^H + V^H V; replaces torch.inverse / torch.linalg.inv) ---- */
#define FIODE_DTYPE_F32 0
#define FIODE_DTYPE_C64 1   /* complex64, interleaved (re, im) */
#define FIODE_INV_MAX_N 128
/* out[b] = in[b]^-1 for b < batch, n x n row-major matrices at element strides in_stride /
 * out_stride (in == out allowed).  Gauss-Jordan in natural pivot order: valid for matrices whose
 * Hermitian part is positive definite (every I + A above); no pivoting, no host sync. */
FIODE_API int fiode_batched_inverse(void* stream, int32_t dtype, int32_t batch, int32_t n, const void* in,
                                    int64_t in_stride, void* out, int64_t out_stride);

/* ---- Backbone GroupSort (KWLarge_Concat activation; absent libs/ortho_conv, restated) --------
 * x, y: [B][C][S] float32 (S = spatial size, 1 for linear layers); C even, (C/2)*S % 4 == 0.
 * y = cat(max(x[:, :C/2], x[:, C/2:]), min(...)); backward splits ties in half (torch.maximum). */
/* Normalize (models.py:17-26) fused with the backbone's NCHW -> spatial-major layout change:
 * y [H][W][C][B] = (x [B][C][H][W] - mu[c]) / std[c] (std may be NULL: no division). */
FIODE_API int fiode_normalize_hwcb(void* stream, int32_t B, int32_t C, int32_t H, int32_t W, const float* x,
                                   const float* mu, const float* std, float* y);
FIODE_API int fiode_groupsort_forward(void* stream, int64_t B, int64_t C, int64_t S, const float* x, float* y);
FIODE_API int fiode_groupsort_backward(void* stream, int64_t B, int64_t C, int64_t S, const float* x, const float* g,
                                       float* gx);

/* The linear head's output layer (KWLargeConcat's last Linear, 512 -> 10; F.linear's addmm in
 * models.py's head): out [B][J] = z [B][K] Q^T + bias (Q [J][K], bias [J] or NULL), J <= 16, one
 * wave per row with a fixed-order lane reduction.  fiode_head_out_backward_gs: its input gradient
 * through the preceding GroupSort, gx = GroupSort backward of y [B][K] (pairs k, k + K/2) applied to
 * g [B][J] Q (K even). */
FIODE_API int fiode_head_out(void* stream, int32_t B, int32_t K, int32_t J, const float* z, const float* Q,
                             const float* bias, float* out);
FIODE_API int fiode_head_out_backward_gs(void* stream, int32_t B, int32_t K, int32_t J, const float* g,
                                         const float* Q, const float* y, float* gx);

/* Error text for a return code. */
/* Inverse of one real n x n matrix with positive-definite symmetric part (the Cayley systems of the
 * 512 x 512 backbone CayleyLinears and the 128 x 128 dynamics map): block Gauss-Jordan over
 * 64-wide panels, no pivot search, no host sync.  n = 128, 192, ..., 512: ONE persistent launch
 * (cayley.hip k_pinv: a chain workgroup inverts every pivot block, one workgroup per 64 x 64 tile
 * applies the panel steps, hand-offs through flags in the workspace, zeroed by a memset in front of
 * the launch); other n: one update launch per panel (the next pivot block is inverted inside it).
 * in may equal out. */
#define FIODE_BLOCK_INV_MAX_N 4096
FIODE_API size_t fiode_block_inverse_workspace_bytes(int32_t n);
FIODE_API int fiode_block_inverse(void* stream, int32_t n, const float* in, float* out, void* workspace,
                                  size_t workspace_bytes);
/* The same for a batch of n x n matrices (in / out [batch][n][n] contiguous, workspace
 * batch * fiode_block_inverse_workspace_bytes(n)): one launch sequence for all of them, so the
 * Cayley systems of several layers share the n/64 + 1 dependent launches. */
FIODE_API int fiode_block_inverse_batched(void* stream, int32_t batch, int32_t n, const float* in, float* out,
                                          void* workspace, size_t workspace_bytes);
/* The same, skipped on the device when *skip != 0 (device int32; NULL = never): every launch of the
 * sequence returns at once and `out` keeps its contents -- for a caller that decides on the device
 * whether an inverse it already holds is still exact (no host sync). */
FIODE_API int fiode_block_inverse_cond(void* stream, int32_t batch, int32_t n, const float* in, float* out,
                                       void* workspace, size_t workspace_bytes, const int32_t* skip);

/* ---- small Cayley maps in one launch (k = min(cout, cin) <= 16, max(cout, cin) * k <= 8192): the
 * backbone's 512 -> 10 CayleyLinear and the dynamics' 128 x 10 maps (classification.py:282-293
 * convert_cayley).  Q = cayley(alpha W / ||W||) for a batch of [cout][cin] matrices (per-matrix
 * alpha [b]); the forward also writes ||W|| [b] and the inverse [b][k][k] the backward reads.
 * One workgroup per matrix (small_cayley.hip). */
#define FIODE_SMALL_CAYLEY_MAX_K 16
#define FIODE_SMALL_CAYLEY_MAX_RK 8192
FIODE_API int fiode_small_cayley_forward(void* stream, int32_t batch, int32_t cout, int32_t cin, const float* W,
                                         const float* alpha, float* Q, float* inv, float* nrm);
FIODE_API int fiode_small_cayley_backward(void* stream, int32_t batch, int32_t cout, int32_t cin, const float* W,
                                          const float* alpha, const float* nrm, const float* inv, const float* gQ,
                                          float* gW, float* galpha);

/* ---- dense Cayley map stages (CayleyLinear; classification.py:282-293 convert_cayley): the
 * elementwise steps between the library GEMMs and the inverse of Q = cayley(alpha W / ||W||) for a
 * batch of [cout][cin] matrices with per-matrix alpha [b] and ||W|| [b] (see dense.hip).  The
 * [R-k] x k blocks P, P1, P2 and gX are in W's layout (wide W: [k][R-k]). */
typedef struct fiode_dense_config {
  int32_t batch, cout, cin;
} fiode_dense_config;
FIODE_API int fiode_dense_cayley_prep(void* stream, const fiode_dense_config* cfg, const float* W, const float* alpha,
                                      const float* nrm, const float* G, float* M);
/* ||W[b]|| in two stream-ordered steps around the G GEMM (replaces torch.linalg.vector_norm on the
 * map's forward chain): fiode_dense_norm_partials writes 256 fixed-order partial sums of squares per
 * matrix into the workspace; fiode_dense_cayley_prep_normed = fiode_dense_cayley_prep with the norm
 * finished from those partials (same order in every workgroup), also written to nrm_out [b]. */
FIODE_API size_t fiode_dense_norm_workspace_bytes(const fiode_dense_config* cfg);
FIODE_API int fiode_dense_norm_partials(void* stream, const fiode_dense_config* cfg, const float* W, void* workspace,
                                        size_t workspace_bytes);
FIODE_API int fiode_dense_cayley_prep_normed(void* stream, const fiode_dense_config* cfg, const float* W,
                                             const float* alpha, const void* workspace, float* nrm_out,
                                             const float* G, float* M);
/* The norm partials, zeroing `clear_words` 32-bit words at clear + b * clear_stride_bytes for every
 * matrix b in the same launch (the flag words of fiode_dense_cayley_inverse's workspace). */
FIODE_API int fiode_dense_norm_partials_clear(void* stream, const fiode_dense_config* cfg, const float* W,
                                              void* workspace, size_t workspace_bytes, void* clear,
                                              size_t clear_words, size_t clear_stride_bytes);
/* The dense map's inverse in ONE launch with M built on load (no prep launch, no M buffer):
 * k = min(cout, cin) = 128 .. 512 in steps of 64; s = alpha / ||W|| from the norm partials,
 * M = I + s (U' - U'^T) + s^2 G (G = V'^T V' when cout != cin, else NULL), inv_out [b][k][k] = M^-1,
 * nrm_out [b] = ||W||; q_out (square maps only, else NULL): Q = 2 inv - I.  Workspace: batch x
 * fiode_block_inverse_workspace_bytes(k), whose first fiode_dense_inverse_flag_bytes(k) bytes per
 * matrix must be zero (fiode_dense_norm_partials_clear). */
FIODE_API size_t fiode_dense_inverse_flag_bytes(int32_t k);
FIODE_API int fiode_dense_cayley_inverse(void* stream, const fiode_dense_config* cfg, const float* W,
                                         const float* alpha, const float* part, const float* G, float* nrm_out,
                                         float* inv_out, float* q_out, void* workspace, size_t workspace_bytes);
FIODE_API int fiode_dense_cayley_finish(void* stream, const fiode_dense_config* cfg, const float* alpha,
                                        const float* nrm, const float* inv, const float* P, float* Q);
FIODE_API int fiode_dense_cayley_ginv(void* stream, const fiode_dense_config* cfg, const float* alpha,
                                      const float* nrm, const float* gQ, const float* A, float* Ginv);
FIODE_API int fiode_dense_cayley_h(void* stream, const fiode_dense_config* cfg, const float* GMn, float* gX, float* H);
FIODE_API size_t fiode_dense_cayley_workspace_bytes(const fiode_dense_config* cfg);
FIODE_API int fiode_dense_cayley_grad(void* stream, const fiode_dense_config* cfg, const float* W, const float* alpha,
                                      const float* nrm, const float* P1, const float* P2, float* gX, float* gW,
                                      float* galpha, void* workspace, size_t workspace_bytes);
/* C[b] = op(A[b]) op(B[b]) for a batch of n x n row-major float matrices (op = transpose when
 * trans_a / trans_b), n % 64 == 0, A and B 16-byte aligned (FIODE_ESHAPE otherwise): the two
 * dependent k x k products of the dense maps' backward, GMn = inv^T (Ginv inv^T) (cayley.py
 * _dense_backward; the reference's autograd through torch.inverse, classification.py:282-293). */
FIODE_API int fiode_dense_gemm(void* stream, int32_t batch, int32_t n, int32_t trans_a, int32_t trans_b,
                               const float* A, const float* B, float* C);

/* ---- real f32 GEMM of the Cayley layers (gemm.hip) ---------------------------------------------
 * C[b] = alpha opA(A[b]) opB(B[b]) + beta C[b] + bias (bias [N] added to every row, or NULL), all
 * row-major: opA [M][K] is A [M][lda] (trans_a 0) or the transpose of A [K][lda] (trans_a 1); opB
 * [K][N] is B [K][ldb] (trans_b 0) or the transpose of B [N][ldb] (trans_b 1).  Replaces the library
 * GEMMs of the dense Cayley maps (cayley_scaled's V'^T V', V' inv and their backward products,
 * classification.py:282-293) and the head's CayleyLinear products (F.linear / addmm and autograd's
 * mm of KWLarge_Concat, models.py:29-35).  K is split over workgroups when the output has too few
 * 64 x 64 tiles to fill the chip (split_k 0: the library's choice, fiode_gemm_splits); the partial
 * tiles are summed in split order by the last workgroup of each tile (deterministic).  Workspace:
 * fiode_gemm_workspace_bytes (0 when unsplit); its first fiode_gemm_counter_bytes must be zero
 * before the first call, and every completed call leaves them zero (one workspace per stream). */
typedef struct fiode_gemm_desc {
  int32_t batch, M, N, K;
  int32_t trans_a, trans_b;
  int64_t lda, ldb, ldc;
  int64_t stride_a, stride_b, stride_c;   /* elements between batch entries */
  float alpha, beta;
  int32_t split_k;                        /* 0: the library's choice */
  int32_t max_workgroups;                 /* 0: one workgroup per 64 x 64 tile (x split); else at most
                                             this many (rounded down to a multiple of 8, >= 8), each
                                             looping over tiles: a narrow launch that leaves the other
                                             CUs to concurrent work (ABI 5) */
} fiode_gemm_desc;
FIODE_API int32_t fiode_gemm_splits(const fiode_gemm_desc* d);
FIODE_API size_t fiode_gemm_counter_bytes(const fiode_gemm_desc* d);
FIODE_API size_t fiode_gemm_workspace_bytes(const fiode_gemm_desc* d);
FIODE_API int fiode_gemm(void* stream, const fiode_gemm_desc* d, const float* A, const float* B, const float* bias,
                         float* C, void* workspace, size_t workspace_bytes);
/* Two independent products in one launch (the dense maps' backward A = V'^T Gb beside P2 = Gb inv^T),
 * each bit-identical to its own fiode_gemm call; shapes the one-launch kernel does not take run as
 * two launches.  Workspace: fiode_gemm_pair_workspace_bytes (counters zero before the first call). */
FIODE_API size_t fiode_gemm_pair_workspace_bytes(const fiode_gemm_desc* d0, const fiode_gemm_desc* d1);
FIODE_API int fiode_gemm_pair(void* stream, const fiode_gemm_desc* d0, const float* A0, const float* B0,
                              const float* bias0, float* C0, const fiode_gemm_desc* d1, const float* A1,
                              const float* B1, const float* bias1, float* C1, void* workspace,
                              size_t workspace_bytes);

/* ---- spectral convolution transforms on spatial-major activations [n][n][C][B] (CayleyConv
 * forward_hwcb; fiode_amd/cayley.py).  Spectrum layout [f][C][B] complex64, f = ka (n/2+1) + kb. */
typedef struct fiode_sconv_config {
  int32_t n;             /* spatial size after any space-to-channel: 8, 16 or 32                */
  int32_t C;             /* channels of the transformed tensor (after space-to-channel)         */
  int32_t B;             /* batch                                                               */
  int32_t downsample;    /* rfft2: gather x from [2n][2n][C/4][B]; irfft2: scatter y to it       */
  int32_t nchw;          /* irfft2's y and rfft2's gy in NCHW [B][C][n][n], the GroupSort codes in
                          * [B][C/2][n][n] (the last conv, whose output the flatten reads as (C, h, w)
                          * features); not with downsample                                          */
} fiode_sconv_config;
/* X = rfft2(x) over (h, w).  With gy != NULL the input is the GroupSort backward of gy (d/dout
 * [n][n][C][B]) with the comparison codes [n][n][C/2][B] of the forward (x unused). */
FIODE_API int fiode_sconv_rfft2(void* stream, const fiode_sconv_config* cfg, const float* x, const float* gy,
                                const uint8_t* code, void* X);
/* X = rfft2((x - mu) / std) for an NCHW input x [B][C][n][n] (the backbone's first conv with its
 * Normalize fused, models.py:17-26; std nullable: x - mu; downsample must be 0). */
FIODE_API int fiode_sconv_rfft2_nchw(void* stream, const fiode_sconv_config* cfg, const float* x, const float* mu,
                                     const float* std, void* X);
/* y = irfft2(Y) (c2c over h, c2r over w, 1/n^2), + bias[C] if given; groupsort != 0: y = GroupSort
 * of it over the channel halves and code_out [n][n][C/2][B] records max/min/tie. */
FIODE_API int fiode_sconv_irfft2(void* stream, const fiode_sconv_config* cfg, const void* Y, const float* bias,
                                 int32_t groupsort, float* y, uint8_t* code_out);
/* fiode_sconv_irfft2 with the per-frequency channel product of a few-input-channel conv fused into
 * its loads: Y[f] = Q[f] X[f] is formed on the fly (conv 1: K = 3 input channels), no [f][C][B]
 * GEMM output.  Q [f][C][K], X [f][K][B] complex64 (f = n (n/2 + 1)), 1 <= K <= 4 (else
 * FIODE_ESHAPE); bias / groupsort / y / code_out as fiode_sconv_irfft2 (cfg->C = output channels). */
FIODE_API int fiode_sconv_irfft2_qx(void* stream, const fiode_sconv_config* cfg, const void* Q, const void* X,
                                    int32_t K, const float* bias, int32_t groupsort, float* y, uint8_t* code_out);

/* Batched complex64 GEMM of the spectral convolutions' per-frequency channel products (CayleyConv
 * forward_hwcb; replaces torch.matmul on complex64 in fiode_amd/cayley.py _SpectralConvFn):
 * C[f] = scale[f] opA(A[f]) opB(B[f]) for f < F, C [F][M][N] (row-major, contiguous);
 * conj_trans_a == 0: A [F][M][K], opA = A; else A [F][K][M], opA = conj(A)^T (dL/dX = Q^H G);
 * conj_trans_b == 0: B [F][K][N], opB = B; else B [F][N][K], opB = conj(B)^T (dL/dQ = w G X^H);
 * not both; scale [F] float32 or NULL (1). */
FIODE_API int fiode_cgemm(void* stream, int32_t F, int32_t M, int32_t N, int32_t K, int32_t conj_trans_a,
                          int32_t conj_trans_b, const float* scale, const void* A, const void* B, void* C);

/* ---- spectral Cayley map of an orthogonal convolution (CayleyConv; libs/ortho_conv, absent:
 * restated in fiode_amd/cayley.py).  Replaces CayleyConv.spectral_weight + cayley_scaled
 * (rfft2 of the taps, shift, conj, ||.||, the per-frequency Cayley map) and its autograd. */
typedef struct fiode_spectral_config {
  int32_t cout, cin;     /* weight [cout][cin][ks][ks] (cin after a stride-2 space-to-channel)   */
  int32_t ks;            /* kernel size: 3 (KWLarge); other sizes return FIODE_ESHAPE           */
  int32_t n;             /* even input size n <= 64: nf = n (n/2 + 1) rFFT frequencies          */
} fiode_spectral_config;

/* Workspace (norm partials, backward scratch): keep the forward's until the backward. */
FIODE_API size_t fiode_spectral_workspace_bytes(const fiode_spectral_config* cfg);
/* Q: complex64 [nf][cout][cin] = cayley(alpha Wf / ||Wf||) per frequency; inv: complex64 [nf][K][K]
 * (K = min(cout, cin)) saved for the backward.  min(cout, cin) <= 64. */
FIODE_API int fiode_spectral_cayley_forward(void* stream, const fiode_spectral_config* cfg, const float* weight,
                                            const float* alpha, void* Q, void* inv, void* workspace,
                                            size_t workspace_bytes);
/* gQ: dL/dQ (torch's complex-gradient convention); grad_weight [cout][cin][ks][ks], grad_alpha [1]
 * are overwritten. */
FIODE_API int fiode_spectral_cayley_backward(void* stream, const fiode_spectral_config* cfg, const float* weight,
                                             const float* alpha, const void* gQ, const void* inv,
                                             float* grad_weight, float* grad_alpha, void* workspace,
                                             size_t workspace_bytes);

/* ---- optimizer step (pl_modules.py:97-147 configure_optimizers -> torch.optim.Adam / AdamW;
 * fiode_amd/optim.py FiodeAdam): one launch updates every parameter tensor (adam.hip).  The host
 * arrays hold n_tensors device pointers each; tensors are contiguous float32 of numel[i] elements.
 * step: host array of device pointers to each tensor's step count (capturable Adam; an entry or
 * the array may be NULL: cfg->step is used), incremented by this call when cfg->increment_steps
 * (one small kernel ahead of the update, skipped with it), else already incremented by the caller.
 * guard (nullable): see fiode_step_guard.  lr_dev (may be NULL):
 * a device scalar holding the learning rate (torch's tensor lr, which LR schedulers update in
 * place; float32, or float64 when lr_dev_is_double): read by the kernel at run time, so a captured
 * step follows schedule changes; else cfg->lr (a value baked into a captured launch). */
#define FIODE_ADAM_MAX_TENSORS 64
/* Step guard (AMP's found_inf, without a host sync): a training step whose solve failed or whose
 * loss is not finite must not reach the parameters.  Every non-NULL source is read on the device:
 *   flag      nonzero or NaN = skip (e.g. the guard slot of the all-reduced gradient bucket, where
 *             fiode_step_guard_flag wrote this rank's verdict: any rank's bad step skips on all);
 *   loss      non-finite = skip;
 *   status[i] nonzero = skip (solve status words: fiode_odetrain_forward stats[3], saved [12]).
 * A skipped update leaves p, m, v and the step counts untouched; `skipped` (nullable) counts the
 * skipped steps (sticky, for the host to read now and then). */
#define FIODE_GUARD_MAX_STATUS 4
typedef struct fiode_step_guard {
  const float* flag;
  const float* loss;
  const int32_t* status[FIODE_GUARD_MAX_STATUS];
  int32_t* skipped;
} fiode_step_guard;
/* flag_out[0] = 1 if the guard's sources (loss, status words; `flag` ignored) say skip, else 0. */
FIODE_API int fiode_step_guard_flag(void* stream, const fiode_step_guard* guard, float* flag_out);

typedef struct fiode_adam_config {
  int32_t n_tensors;
  int32_t decoupled;     /* AdamW: p -= lr wd p before the moments (else g += wd p)             */
  int32_t maximize;
  int32_t increment_steps;  /* 1: the device step counts are incremented here (guarded), before
                               the update reads them; 0: the caller already incremented them   */
  /* hyper-parameters as the host holds them (Python floats): 1 - beta, the bias corrections and
   * lr / (1 - beta1^t) are formed in double, then rounded to the fp32 the update runs in */
  double lr, beta1, beta2, eps, weight_decay;
  double step;
  const void* lr_dev;
  int32_t lr_dev_is_double;
  int32_t pad2_;
} fiode_adam_config;
FIODE_API int fiode_adam_step(void* stream, const fiode_adam_config* cfg, float* const* params,
                              const float* const* grads, float* const* exp_avg, float* const* exp_avg_sq,
                              const int64_t* numel, float* const* step, const fiode_step_guard* guard);

FIODE_API const char* fiode_error_string(int code);
FIODE_API int fiode_abi_version(void);

#ifdef __cplusplus
}
#endif
#endif /* FIODE_H_ */
