// FI-ODE forward-invariance training step on gfx950 (MI355X).
//
// Replaces, below the Cayley maps, LyapunovLearning.compute_loss + loss.backward()
// (pl_modules.py:390-502) and everything it calls on the per-sample path:
//   sampler fan-out         sampling/sampler.py:34-38, 113-128, 139-153, 195-216
//   dynamics f(h, x)        dynamics/classification.py:96-115
//   QP projection fwd/bwd   barrier_projection/barrier_projection.py:217-313
//   V, V-dot (jvp)          lya_cands.py:79-94, pl_modules.py:403-412
//   hinge loss + logs       pl_modules.py:444-484
//
// Layout ("hidden on M, samples on N"): one wave owns a tile of 32 rows (samples).  Every layer
// is computed transposed, Z^T[hidden x samples] = Q[hidden x in] * A^T[in x samples], with
// v_mfma_f32_32x32x2_f32.  The accumulator of one layer (hidden index in registers, sample on
// the lane) is directly the B operand of the next layer's MFMA (the K index of a k-step is the
// register's row), so activations never leave registers between layers.  Weights live in LDS
// (128x132-padded images read with ds_read_b128: 4 k-steps per read, conflict-free).
//
// Kernels of one step (stream-ordered, no host sync):
//   k_static_proj  u[b] = U_x x_b + bx + b1, reset the QP exit words
//   k_lyap_fwd     sampler, both eval_dot passes (loss pass + logging pass), per-row QP
//                  convergence masks AND-reduced into one word per pass (batch-global exit,
//                  barrier_projection.py:247-249), activations of the loss pass to HBM
//   k_lyap_bwd     QP to the global exit, V / V-dot / hinge / logging stats, QP backward,
//                  sigmoid backward, dL/da2 -> dL/dz2 -> dL/da1 -> dL/dz1 (MFMA)
//   k_lyap_wgrad   weight gradients dQ2 = gz2^T a1, dQ3 = gft^T a2, dQ1 = gz1^T h (MFMA, K =
//                  samples), split per image part into partial slabs (deterministic)
//   k_lyap_reduce  slab sum, per-image g_u, scalars;  k_lyap_static_grads: dQx, dbx, dx
//   (the train_ode weight-gradient chain: k_lyap_wgrad also sums g_u from the gz1 rows, and its
//   k_lyap_reduce runs the static gradients beside the slab sums -- two launches)
#include "common.h"
#include "tile.h"
#include "../../include/fiode.h"
#include "wgrad.h"

namespace {
using namespace fiode_tile;

typedef float f32x4q __attribute__((ext_vector_type(4)));
__device__ __forceinline__ f32x4q mfma16q(float a, float b, f32x4q c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f32x4q q4_zero() { return f32x4q{0.f, 0.f, 0.f, 0.f}; }

// Phase timing (OT_PROFILE builds, tools/lyap_probe.py): lane 0 of every wave of workgroups 0..7
// adds the wall-clock ticks (100 MHz) of each phase into prof[i] (a sample: all workgroups' atomics
// on one word would time their own contention); LY_COUNT(i) counts the sampled waves.
#ifdef OT_PROFILE
#define LY_T0() uint64_t ly_t_ = wall_clock64()
#define LY_T(i) do { const uint64_t n_ = wall_clock64(); if ((threadIdx.x & 63) == 0 && blockIdx.x < 8) \
    atomicAdd(a.prof + (i), (unsigned long long)(n_ - ly_t_)); ly_t_ = n_; } while (0)
#define LY_COUNT(i) do { if ((threadIdx.x & 63) == 0 && blockIdx.x < 8) atomicAdd(a.prof + (i), 1ull); } while (0)
// per-workgroup start / end stamps of wave 0 (slot base: fwd 64, bwd 64 + 2 * 1024)
#define LY_STAMP(base, k) do { if (threadIdx.x == 0 && blockIdx.x < 1024) \
    a.prof[(base) + 2 * blockIdx.x + (k)] = wall_clock64(); } while (0)
// k_lyap_wgrad: per-workgroup stamps of wave 0 (start, staged, MFMA done, end) in a device array
// read by fiode_debug_wgrad_stamps (tools/probes/wgrad_probe.py)
__device__ unsigned long long g_wg_stamps[4 * 1024];
#define WG_STAMP(k) do { if (threadIdx.x == 0 && blockIdx.x < 1024) g_wg_stamps[4 * blockIdx.x + (k)] = wall_clock64(); } while (0)
#else
#define WG_STAMP(k) do { } while (0)
#define LY_STAMP(base, k) do { } while (0)
#define LY_T0() do { } while (0)
#define LY_T(i) do { } while (0)
#define LY_COUNT(i) do { } while (0)
#endif

constexpr int SLAB = 16384 + 1280 + 1280 + 128 + 128 + 16;   // floats per wgrad partial slab
// The batch-global QP exit words (one AND per pass) are spread over CONV_SLOTS words per pass:
// 2,048 waves AND-ing into ONE word serialise at the memory-side atomic unit (~88 ops/us per word,
// MI355X_MICROARCH.md: ~23 us -- the tail of k_lyap_fwd); consumers AND the slots (conv_word).
constexpr int CONV_SLOTS = 32;
constexpr int SLAB_Q2 = 0, SLAB_Q3 = 16384, SLAB_Q1 = 16384 + 1280, SLAB_B2 = 16384 + 2560,
              SLAB_B1 = 16384 + 2560 + 128, SLAB_B3 = 16384 + 2560 + 256;

struct LyapArgs {
  const int32_t* s_used;   // launch_wgrad: optional device count of the rows per image that are data
  int N, S, B, S1;
  int sampler, dropout_mode, bit_mode;
  uint32_t thr8;
  float drop_scale;
  Rng rng;
  const uint64_t* offset_dev;   // optional device-resident addend of the Philox offset
  DynScalars d;
  float kappa, invN;
  const float* kappa_dev;    // optional device kappa (the ramp of a captured step), else kappa
  int parts, chunk, ipw;   // k_lyap_wgrad: parts per image, rows per part, images per workgroup
  const float* x_feat;
  const int64_t* y;
  const float* h_in;
  const uint8_t* masks;
  const float *Q1, *b1, *Qx, *bx, *Q2, *b2, *Q3, *b3;
  // workspace
  uint32_t* conv;      // [2][CONV_SLOTS] QP exit words (AND of the slots = the pass's word)
  float* u;            // [B][M]
  float* h_ws;         // [N][C]
  float* ft_ws;        // [2][N][C]
  float *a1, *a2, *gz2, *gz1;   // [N][M]
  float* gft;          // [N][C]
  uint4* kw;           // [4][N] dropout keep words (bit t of word mb = keep hidden 32mb+t)
  float* tile_sc;      // [ntiles][4]
  float* slabs;        // [nslab][SLAB]
  int nslab;           // partial slabs summed by k_lyap_reduce
  float* g_u;          // [B][M]
  float* gu_tiles;     // fused backward: per-(tile, image segment) partial g_u [ntiles][nseg][M] (else null)
  unsigned long long* prof;   // OT_PROFILE builds: per-phase wall-clock ticks summed over waves
  int nseg;            // image segments per 32-row tile (images a tile's rows can span)
  // outputs
  float* scalars;
  float *h_out, *V, *Vdot, *f, *f_log, *qp_lower, *qp_nominal, *g_ftilde;
  const float* exp_draws;    // optional given Exp(1) variates (parity), else Philox
  float* exp_draws_out;      // optional: the variates used
  uint32_t* kw_out;          // optional: [4][N][4] keep words
  fiode_lyap_grads grads;
};

__device__ __forceinline__ uint32_t conv_word(const LyapArgs& a, int pass) {
  uint32_t w = 0xFFFFFFFFu;
#pragma unroll
  for (int s = 0; s < CONV_SLOTS; ++s) w &= a.conv[pass * CONV_SLOTS + s];
  return w;
}

// ---- sampler (one lane computes one row) ----------------------------------------------------
__device__ __forceinline__ void draws10(const Rng& rng, uint32_t index, uint32_t stream, float (&e)[C]) {
  const uint4 r0 = rng.draw(index, stream), r1 = rng.draw(index, stream + 1), r2 = rng.draw(index, stream + 2);
  const uint32_t w[12] = {r0.x, r0.y, r0.z, r0.w, r1.x, r1.y, r1.z, r1.w, r2.x, r2.y, r2.z, r2.w};
#pragma unroll
  for (int j = 0; j < C; ++j) e[j] = exp1_from_bits(w[j]);
}

// The n (<= C) Exp(1) variates of one sampler draw row: read from the caller's draws (parity
// mode) or drawn from Philox (index, stream); draw_row indexes the reference's draw tensor (see
// fiode_lyap_io.exp_draws), `publish` = this lane owns the row of exp_draws_out.
__device__ __forceinline__ void row_draws(const LyapArgs& a, size_t draw_row, int n, bool publish, uint32_t index,
                                          uint32_t stream, float (&e)[C]) {
  if (a.exp_draws) {
    const float* p = a.exp_draws + draw_row * n;
#pragma unroll
    for (int j = 0; j < C; ++j) e[j] = j < n ? p[j] : 0.f;
  } else {
    draws10(a.rng, index, stream, e);
  }
  if (a.exp_draws_out && publish) {
    float* q = a.exp_draws_out + draw_row * n;
#pragma unroll
    for (int j = 0; j < C; ++j)
      if (j < n) q[j] = e[j];
  }
}

__device__ void sample_row(const LyapArgs& a, int row, int label, float (&h)[C]) {
  if (a.sampler == FIODE_SAMPLER_GIVEN) {
    load_row10(a.h_in + (size_t)row * C, h);
    return;
  }
  const int b = row / a.S, s = row - b * a.S;
  if (a.sampler == FIODE_SAMPLER_COMPOSITE || a.sampler == FIODE_SAMPLER_TRAJECTORY) {
    if (s < a.S1) {                      // UniformSimplexSampling, shared over the batch (sampler.py:209-210)
      row_draws(a, (size_t)s, C, b == 0, (uint32_t)s, RNG_STREAM_UNIFORM, h);
      l1_normalize(h);
    } else if (a.sampler == FIODE_SAMPLER_TRAJECTORY) {
      // TrajectorySampler (sampler.py:156-166): the solve's states at linspace(0, t_max, S - S1),
      // given as [B][S - S1][C] (the per-image trajectory, transpose(0, 1) of odeint's output)
      load_row10(a.h_in + ((size_t)b * (a.S - a.S1) + (s - a.S1)) * C, h);
    } else {                             // CorrectConeSampling (sampler.py:113-128)
      row_draws(a, (size_t)a.S1 + (size_t)b * (a.S - a.S1) + (s - a.S1), C, true, (uint32_t)row, RNG_STREAM_CONE, h);
      l1_normalize(h);
      int am = 0;
      float mx = h[0];
#pragma unroll
      for (int j = 1; j < C; ++j)
        if (h[j] > mx) { mx = h[j]; am = j; }
      float hl = 0.f;
#pragma unroll
      for (int j = 0; j < C; ++j) hl = (j == label) ? h[j] : hl;
#pragma unroll
      for (int j = 0; j < C; ++j) {
        const float o = h[j];
        h[j] = (j == label) ? mx : ((j == am) ? hl : o);
      }
    }
  } else {                               // DecisionBoundarySampling (sampler.py:139-153)
    float z[C];
    row_draws(a, (size_t)row, C - 1, true, (uint32_t)row, RNG_STREAM_DB, z);
    float raw[C];
    float zm = z[0];
#pragma unroll
    for (int j = 1; j < C - 1; ++j) zm = fmaxf(zm, z[j]);
    raw[0] = zm;
#pragma unroll
    for (int j = 0; j < C - 1; ++j) raw[j + 1] = z[j];
    l1_normalize(raw);
#pragma unroll
    for (int c = 0; c < C; ++c) {
      const float below = raw[c + 1 < C ? c + 1 : C - 1];   // classes before the label keep raw[c+1]
      const float above = raw[c];                          // classes after it take raw[c]
      h[c] = (c == label) ? raw[0] : ((c < label) ? below : above);
    }
  }
}

__device__ __forceinline__ void keep_words(const LyapArgs& a, int row, int set, uint32_t (&kw)[4]) {
  const uint8_t* m = a.dropout_mode == FIODE_DROPOUT_GIVEN ? a.masks + ((size_t)set * a.N + row) * M : nullptr;
  dropout_keep_words(a.dropout_mode, a.bit_mode, a.thr8, a.rng, m, (uint32_t)row,
                     RNG_STREAM_DROP + ((uint32_t)set << 4), kw);
}

// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(128) void k_static_proj(LyapArgs a) {
  const int b = blockIdx.x, i = threadIdx.x;
  if (b == 0 && i < 2 * CONV_SLOTS) a.conv[i] = 0xFFFFFFFFu;
  if (b == 0 && a.prof && i < 64) a.prof[i] = 0ull;
  if (b >= a.B) return;
  float s = 0.f;
  const float* xb = a.x_feat + (size_t)b * FIODE_X;
#pragma unroll
  for (int c = 0; c < FIODE_X; ++c) s = __fmaf_rn(a.Qx[i * FIODE_X + c], xb[c], s);
  a.u[(size_t)b * M + i] = (s + a.bx[i]) + a.b1[i];
}

// Per-row preparation: sampler fan-out (h -> h_ws) and the dropout keep words of the 4 mask sets.
__global__ __launch_bounds__(256) void k_lyap_prep(LyapArgs a) {
  const int row = blockIdx.x * blockDim.x + threadIdx.x;
  if (row >= a.N) return;
  if (a.offset_dev) {            // graph replay: the step counter lives in device memory
    const uint64_t o = (((uint64_t)a.rng.off_hi << 32) | a.rng.off_lo) + *a.offset_dev;
    a.rng.off_lo = (uint32_t)o;
    a.rng.off_hi = (uint32_t)(o >> 32);
  }
  if (a.sampler != FIODE_SAMPLER_GIVEN || a.h_out) {
    const int label = (int)a.y[row / a.S];
    float h[C];
    sample_row(a, row, label, h);
    if (a.sampler != FIODE_SAMPLER_GIVEN) store_row10(a.h_ws + (size_t)row * C, h);
    if (a.h_out) store_row10(a.h_out + (size_t)row * C, h);
  }
  for (int set = 0; set < 4; ++set) {
    uint32_t kw[4];
    keep_words(a, row, set, kw);
    a.kw[(size_t)set * a.N + row] = make_uint4(kw[0], kw[1], kw[2], kw[3]);
    if (a.kw_out)
      reinterpret_cast<uint4*>(a.kw_out)[(size_t)set * a.N + row] = make_uint4(kw[0], kw[1], kw[2], kw[3]);
  }
}

// One wave per 32-row tile, both passes: the loss pass's MLP (dropout masks 0/1) and the logging
// pass's (masks 2/3) on the MFMA, then ONE QP per lane -- lanes 0..31 take the loss pass of their
// row, lanes 32..63 the logging pass (a 32x32 accumulator tile leaves every row's outputs on both
// halves, so one pass per wave would run each row's QP twice).  Per wave: ft -> HBM, the QP to
// max_iter - 1 for its convergence bits, AND-ed per pass into CONV_SLOTS words (the batch-global
// exit, barrier_projection.py:247-249).  Persistent: two workgroups per CU (LDS 72.9 KB each), the
// weight images staged once per workgroup; with more than one tile per SIMD, one wave's QP (VALU)
// overlaps the other's MFMA.
#ifndef FWD_WAVES
#define FWD_WAVES 4           // waves (tiles in flight) per workgroup
#endif
__global__ __launch_bounds__(64 * FWD_WAVES, 8 / FWD_WAVES) void k_lyap_fwd(LyapArgs a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  LY_T0();
  LY_COUNT(6);
  LY_STAMP(64, 0);
  float* Q2s = smem;
  float* Q3s = smem + M * LDQ;
  load_weight_images(a.Q2, a.Q3, Q2s, Q3s, C);
  __syncthreads();
  LY_T(0);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, half = lane >> 5, col = lane & 31;
  float q1[4][5];
#pragma unroll
  for (int mb = 0; mb < 4; ++mb)
#pragma unroll
    for (int s = 0; s < 5; ++s) q1[mb][s] = a.Q1[(32 * mb + col) * C + 2 * s + half];
  const int ntiles = (a.N + 31) / 32;
  const int pass = half;                    // this lane's pass in the QP phase
  for (int tile = FWD_WAVES * blockIdx.x + wave; tile < ntiles; tile += FWD_WAVES * gridDim.x) {
    const int row = tile * 32 + col;
    const bool valid = row < a.N;
    const int rr = valid ? row : a.N - 1;
    const int b = rr / a.S;
    float h[C];
    load_row10(((a.sampler == FIODE_SAMPLER_GIVEN) ? a.h_in : a.h_ws) + (size_t)rr * C, h);
    uint4 kq[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) kq[q] = a.kw[(size_t)q * a.N + rr];
    LY_T(1);
    float ft[C] = {};
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      const uint32_t kw1[4] = {kq[2 * p].x, kq[2 * p].y, kq[2 * p].z, kq[2 * p].w};
      const uint32_t kw2[4] = {kq[2 * p + 1].x, kq[2 * p + 1].y, kq[2 * p + 1].z, kq[2 * p + 1].w};
      f32x16 z1[4], z2[4];
      const f32x16 z3 = mlp_tile(Q2s, Q3s, q1, a.u + (size_t)b * M, a.b2, a.b3, h, kw1, kw2, a.drop_scale,
                                 col, half, z1, z2);
      float fp[C];
      gather_ft(z3, half, fp);
#pragma unroll
      for (int j = 0; j < C; ++j) ft[j] = (p == pass) ? fp[j] : ft[j];
    }
    LY_T(2);
    float lower[C], nominal[C], sig[C], span[C], v[C], mu;
    barrier_nominal(a.d, h, ft, lower, nominal, sig, span);
    LY_T(3);
    uint32_t conv = qp_bisect(lower, nominal, a.d.max_iter - 1, a.d.tol, v, mu);
    LY_T(4);
    if (!valid) conv = 0xFFFFFFFFu;
#pragma unroll
    for (int o = 16; o > 0; o >>= 1) conv &= (uint32_t)__shfl_xor((int)conv, o, 64);   // AND within each half
    if (col == 0) atomicAnd(a.conv + pass * CONV_SLOTS + (blockIdx.x % CONV_SLOTS), conv);
    if (valid) {
      store_row10(a.ft_ws + ((size_t)pass * a.N + row) * C, ft);
      if (a.qp_nominal) store_row10(a.qp_nominal + ((size_t)pass * a.N + row) * C, nominal);
      if (pass == 0 && a.qp_lower) store_row10(a.qp_lower + (size_t)row * C, lower);
    }
    LY_T(5);
  }
  LY_STAMP(64, 1);
}

// One tile's operands of the backward's second half and of the weight gradients, staged
// row-major (row n = sample of the tile): the samples are the K dimension of dQ2 = gz2^T a1,
// dQ3 = gft^T a2, dQ1 = gz1^T h; g_a1 = Q2^T g_z2 reads gz2 of all 128 units from here.
struct BwdStage {
  float g2[32][LDQ];    // gz2[n][i]
  float a1[32][LDQ];    // a1[n][k]
  float a2[32][LDQ];    // a2[n][k]
  float g1[32][LDQ];    // gz1[n][i]
  float gf[4][32][12];  // gft[n][c] of the round's 4 tiles (phase A)
  float hh[4][32][12];  // h[n][c]
  uint32_t kw[4][32][8];  // keep words of both dropout layers (phase A loads them behind its QP work)
};
constexpr size_t BWD_LDS = (size_t)(M + C) * LDQ * sizeof(float) + sizeof(BwdStage);

// Backward of the loss pass fused with the weight gradients: no activation reaches HBM.
// A workgroup takes 4 consecutive 32-row tiles per round.
//   Phase A (wave w, tile w; VALU): the loss-pass QP to the global exit K0 (ft from the forward),
//     V / V-dot / hinge, the QP backward -> g_ft; the logging-pass QP to K1; g_ft and h -> LDS.
//   Phase B (each tile in turn, all 4 waves; wave w owns hidden units 32w..32w+31): recompute
//     layer 1 (all units) and wave w's block of layer 2 (a1, a2), g_a2 = Q3^T g_ft and
//     g_z2 = g_a2 [a2 > 0] / (1 - p) for its block -> LDS; g_a1 = Q2^T g_z2 for its block (the A
//     operand Q2[i][k] read transposed from the one Q2 image, g_z2 of all units from LDS) -> g_z1;
//     then its quarter of the weight gradients over the staged tile (dQ2 rows 32w.. : 4 blocks,
//     dQ3 columns 32w.., dQ1 rows 32w..; MFMA with K = the tile's samples); db2 / db3 ride on the
//     A operand reads; the tile's per-image g_u partial (fixed-order sum) -> gu_tiles.
// One partial slab per workgroup (k_lyap_reduce sums them in a fixed order).
__global__ __launch_bounds__(256, 1) void k_lyap_bwd(LyapArgs a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* Q2s = smem;                         // Q2[i][k] (not transposed)
  float* Q3s = smem + M * LDQ;               // Q3 rows 0..C-1 (unused here: the layout of k_lyap_fwd)
  (void)Q3s;
  BwdStage& st = *reinterpret_cast<BwdStage*>(smem + (M + C) * LDQ);
  LY_T0();
  LY_COUNT(18);
  LY_STAMP(64 + 2048, 0);
  load_weight_images(a.Q2, nullptr, Q2s, nullptr);
  __syncthreads();
  LY_T(8);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, half = lane >> 5, col = lane & 31;
  float q1[4][5], q3t[5];
#pragma unroll
  for (int mb = 0; mb < 4; ++mb)
#pragma unroll
    for (int s = 0; s < 5; ++s) q1[mb][s] = a.Q1[(32 * mb + col) * C + 2 * s + half];
#pragma unroll
  for (int s = 0; s < 5; ++s) q3t[s] = a.Q3[(2 * s + half) * M + 32 * w + col];   // A operand of Q3^T g_ft^T, block w
  f32x4 b2w[4];                              // b2 of block w in accumulator order
#pragma unroll
  for (int g = 0; g < 4; ++g) b2w[g] = *reinterpret_cast<const f32x4*>(a.b2 + 32 * w + 8 * g + 4 * half);
  const float kappa = a.kappa_dev ? *a.kappa_dev : a.kappa;
  const int K0 = qp_exit_iter(conv_word(a, 0), a.d.max_iter);
  const int K1 = qp_exit_iter(conv_word(a, 1), a.d.max_iter);
  const float* hsrc = (a.sampler == FIODE_SAMPLER_GIVEN) ? a.h_in : a.h_ws;
  const int ntiles = (a.N + 31) / 32;
  f32x16 dq2[4];
#pragma unroll
  for (int kb = 0; kb < 4; ++kb) dq2[kb] = f16_zero();
  // dQ3 (10 x 32 block w) and dQ1 (32 x 10 block w) on 16x16x4 tiles: the 10 classes pad to 16,
  // not 32 (lane l: j = l & 15, q = l >> 4; A[i = j][k = q], B[k = q][j], D[4q + r][j])
  f32x4q dq3[2] = {q4_zero(), q4_zero()}, dq1[2] = {q4_zero(), q4_zero()};
  const int j16 = lane & 15, q16 = lane >> 4;
  float db2 = 0.f, db3 = 0.f;
  // u[b] rows of the layer-1 accumulators, loaded one tile ahead (the global-load latency of the
  // first tile hides behind phase A, of tile t + 1 behind tile t's MFMA work)
  f32x16 un[4];
  auto load_u = [&](int tile) {
    const int row = tile * 32 + col;
    const int b = (row < a.N ? row : a.N - 1) / a.S;
#pragma unroll
    for (int mb = 0; mb < 4; ++mb) load_acc_rows(a.u + (size_t)b * M, mb, half, un[mb]);
  };
  for (int base = 4 * blockIdx.x; base < ntiles; base += 4 * gridDim.x) {
    load_u(base);
    // ---------------- phase A: wave w, tile base + w: the row math of the loss and logging passes
    {
      const int tile = base + w;
      const int row = tile * 32 + col;
      const bool valid = row < a.N;
      const int rr = valid ? row : a.N - 1;
      float h[C], gft[C];
#pragma unroll
      for (int j = 0; j < C; ++j) gft[j] = 0.f;
      load_row10(hsrc + (size_t)rr * C, h);
      const uint4 kwa = a.kw[rr], kwb = a.kw[(size_t)a.N + rr];
      if (tile < ntiles) {
        // lanes 0..31: the loss pass of their row (QP to K0, V / V-dot / hinge, QP backward);
        // lanes 32..63: the logging pass (QP to K1, active-constraint count) -- one QP per lane
        const int label = (int)a.y[rr / a.S];
        const bool loss_half = half == 0;
        float ft[C], lower[C], nominal[C], sig[C], span[C], v[C], mu;
        load_row10(a.ft_ws + ((size_t)half * a.N + rr) * C, ft);
        barrier_nominal(a.d, h, ft, lower, nominal, sig, span);
        qp_bisect(lower, nominal, loss_half ? K0 : K1, a.d.tol, v, mu);
        float viol = 0.f, active = 0.f;
        if (loss_half) {
          // V = (1 + max_{j != y} h_j) - h_y ; j* first index (lya_cands.py:84-94)
          int js = label == 0 ? 1 : 0;
          float hm = h[js];
#pragma unroll
          for (int j = 0; j < C; ++j)
            if (j != label && h[j] > hm) { hm = h[j]; js = j; }
          float hy = 0.f, fy = 0.f, fj = 0.f;
#pragma unroll
          for (int j = 0; j < C; ++j) {
            hy = (j == label) ? h[j] : hy;
            fy = (j == label) ? v[j] : fy;
            fj = (j == js) ? v[j] : fj;
          }
          const float Vv = (1.0f + hm) - hy;
          const float Vd = fj - fy;                  // jvp of the piecewise-linear V along f
          const float pre = Vd + kappa * Vv;         // vdot + kappa * V.detach() (pl_modules.py:455-457)
          viol = pre > 0.f ? pre : 0.f;
          const float gp = (pre > 0.f && valid) ? a.invN : 0.f;
          float g[C], g_nom[C], g_low[C];
#pragma unroll
          for (int j = 0; j < C; ++j) g[j] = (j == js) ? gp : ((j == label) ? -gp : 0.f);
          qp_backward_row(g, v, mu, nominal, g_nom, g_low);
#pragma unroll
          for (int j = 0; j < C; ++j)
            gft[j] = a.d.scale_nominal ? ((g_nom[j] * span[j]) * (1.0f - sig[j])) * sig[j] : g_nom[j];
          if (valid) {
            if (a.V) a.V[row] = Vv;
            if (a.Vdot) a.Vdot[row] = Vd;
            if (a.f) store_row10(a.f + (size_t)row * C, v);
            if (a.g_ftilde) store_row10(a.g_ftilde + (size_t)row * C, gft);
          }
        } else {
          // logging pass: active-constraint count (pl_modules.py:476-482)
#pragma unroll
          for (int j = 0; j < C; ++j) {
            const float lin = -a.d.alpha_1 * h[j];
            const float up = a.d.alpha_2 * (1.0f - h[j]);
            active += (fabsf(v[j] - lin) <= 1e-6f || fabsf(v[j] - up) <= 1e-6f) ? 1.f : 0.f;
          }
          if (valid && a.f_log) store_row10(a.f_log + (size_t)row * C, v);
        }
        const float s0 = wave_sum(valid && loss_half ? viol : 0.f);
        const float s1 = wave_sum(valid && loss_half && viol > 0.f ? 1.f : 0.f);
        const float s2 = wave_sum(valid && !loss_half ? active : 0.f);
        if (lane == 0) *reinterpret_cast<f32x4*>(a.tile_sc + 4 * tile) = f32x4{s0, s1, s2, 0.f};
      }
      if (half == 0) {
#pragma unroll
        for (int c = 0; c < C; ++c) {
          st.gf[w][col][c] = gft[c];
          st.hh[w][col][c] = valid ? h[c] : 0.f;
        }
        *reinterpret_cast<uint4*>(&st.kw[w][col][0]) = kwa;
        *reinterpret_cast<uint4*>(&st.kw[w][col][4]) = kwb;
      }
    }
    __syncthreads();
    LY_T(9);
    // ---------------- phase B: the round's tiles in turn, all waves
#pragma unroll 1
    for (int t = 0; t < 4; ++t) {
      const int tile = base + t;
      if (tile >= ntiles) break;                   // block-uniform
      // h and the keep words from phase A's LDS copy (rows past N: h = 0; their gradients are 0)
      const uint4 k1 = *reinterpret_cast<const uint4*>(&st.kw[t][col][0]);
      const uint32_t kw1[4] = {k1.x, k1.y, k1.z, k1.w};
      const uint32_t kw2w = st.kw[t][col][4 + w];
      // layer 1 (all units): z1 = u[b] + Q1 h, dropout-ReLU
      f32x16 z1[4] = {un[0], un[1], un[2], un[3]};
      if (t + 1 < 4 && tile + 1 < ntiles) load_u(tile + 1);
#pragma unroll
      for (int s = 0; s < 5; ++s) {
        const float bs = st.hh[t][col][2 * s + half];
#pragma unroll
        for (int mb = 0; mb < 4; ++mb) z1[mb] = mfma32(q1[mb][s], bs, z1[mb]);
      }
#pragma unroll
      for (int mb = 0; mb < 4; ++mb) dropout_relu(z1[mb], kw1[mb], half, a.drop_scale);
      f32x16 z1w;                                  // this wave's block of a1 (w is wave-uniform)
      if (w == 0) z1w = z1[0];
      else if (w == 1) z1w = z1[1];
      else if (w == 2) z1w = z1[2];
      else z1w = z1[3];
      // layer 2, block w: z2 = b2 + Q2 a1
      f32x16 z2;
#pragma unroll
      for (int g = 0; g < 4; ++g)
#pragma unroll
        for (int e = 0; e < 4; ++e) z2[4 * g + e] = b2w[g][e];
      // the LDS operands of step kk + 1 are read before the MFMAs of step kk (software pipeline: the
      // compiler otherwise waits on every read right before its MFMA -- one wave per SIMD, nothing
      // else hides the ~100-cycle LDS latency)
      {
        const float* q2row = Q2s + (32 * w + col) * LDQ + 4 * half;
        f32x4 q = *reinterpret_cast<const f32x4*>(q2row);
#pragma unroll
        for (int kk = 0; kk < 16; ++kk) {                // kk = 4 kb + g
          const f32x4 qn = kk + 1 < 16 ? *reinterpret_cast<const f32x4*>(q2row + 32 * ((kk + 1) >> 2) + 8 * ((kk + 1) & 3))
                                       : q;
#pragma unroll
          for (int e = 0; e < 4; ++e) z2 = mfma32(q[e], z1[kk >> 2][4 * (kk & 3) + e], z2);
          q = qn;
        }
      }
      dropout_relu(z2, kw2w, half, a.drop_scale);
      // g_a2^T block w = Q3^T g_ft^T ; g_z2 = g_a2 [a2 > 0] * scale
      f32x16 ga = f16_zero();
#pragma unroll
      for (int s = 0; s < 5; ++s) ga = mfma32(q3t[s], st.gf[t][col][2 * s + half], ga);
#pragma unroll
      for (int r = 0; r < 16; ++r) ga[r] = z2[r] > 0.f ? ga[r] * a.drop_scale : 0.f;
      store_acc_rows(&st.a1[col][0], w, half, z1w);
      store_acc_rows(&st.a2[col][0], w, half, z2);
      store_acc_rows(&st.g2[col][0], w, half, ga);
      LY_T(10);
      __syncthreads();
      LY_T(11);
      // g_a1^T block w = Q2^T g_z2^T: A = Q2[32kb + 8g + 4half + e][32w + col], B = g_z2[n = col][32kb + 8g + 4half + e]
      f32x16 gb = f16_zero();
      {
        auto ld = [&](int kk, float (&qa)[4], f32x4& gz) {   // kk = 4 kb + g
          const int k0 = 32 * (kk >> 2) + 8 * (kk & 3) + 4 * half;
          gz = *reinterpret_cast<const f32x4*>(&st.g2[col][k0]);
#pragma unroll
          for (int e = 0; e < 4; ++e) qa[e] = Q2s[(k0 + e) * LDQ + 32 * w + col];
        };
        float qa[4];
        f32x4 gz;
        ld(0, qa, gz);
#pragma unroll
        for (int kk = 0; kk < 16; ++kk) {
          float qn[4] = {0.f, 0.f, 0.f, 0.f};
          f32x4 gn = gz;
          if (kk + 1 < 16) ld(kk + 1, qn, gn);
#pragma unroll
          for (int e = 0; e < 4; ++e) gb = mfma32(qa[e], gz[e], gb);
#pragma unroll
          for (int e = 0; e < 4; ++e) qa[e] = qn[e];
          gz = gn;
        }
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) gb[r] = z1w[r] > 0.f ? gb[r] * a.drop_scale : 0.f;
      store_acc_rows(&st.g1[col][0], w, half, gb);
      LY_T(12);
      __syncthreads();
      LY_T(13);
      // weight gradients of this tile: wave w's quarter
      {
        float av = st.g2[half][32 * w + col], bv[4];
#pragma unroll
        for (int kb = 0; kb < 4; ++kb) bv[kb] = st.a1[half][32 * kb + col];
#pragma unroll
        for (int s = 0; s < 16; ++s) {
          const int n1 = 2 * (s + 1) + half;
          float avn = av, bvn[4] = {bv[0], bv[1], bv[2], bv[3]};
          if (s + 1 < 16) {
            avn = st.g2[n1][32 * w + col];
#pragma unroll
            for (int kb = 0; kb < 4; ++kb) bvn[kb] = st.a1[n1][32 * kb + col];
          }
          db2 += av;
#pragma unroll
          for (int kb = 0; kb < 4; ++kb) dq2[kb] = mfma32(av, bv[kb], dq2[kb]);
          av = avn;
#pragma unroll
          for (int kb = 0; kb < 4; ++kb) bv[kb] = bvn[kb];
        }
      }
      {
        // operands of step s + 1 read ahead of step s's MFMAs (as above)
        float o[6], on[6];
        auto ld = [&](int s, float (&v)[6]) {
          const int n = 4 * s + q16;
          v[0] = j16 < C ? st.gf[t][n][j16] : 0.f;
          v[1] = j16 < C ? st.hh[t][n][j16] : 0.f;
#pragma unroll
          for (int hb = 0; hb < 2; ++hb) {
            v[2 + hb] = st.a2[n][32 * w + 16 * hb + j16];
            v[4 + hb] = st.g1[n][32 * w + 16 * hb + j16];
          }
        };
        ld(0, o);
#pragma unroll
        for (int s = 0; s < 8; ++s) {
#pragma unroll
          for (int e = 0; e < 6; ++e) on[e] = o[e];
          if (s + 1 < 8) ld(s + 1, on);
          if (w == 0) db3 += o[0];
#pragma unroll
          for (int hb = 0; hb < 2; ++hb) {
            dq3[hb] = mfma16q(o[0], o[2 + hb], dq3[hb]);
            dq1[hb] = mfma16q(o[4 + hb], o[1], dq1[hb]);
          }
#pragma unroll
          for (int e = 0; e < 6; ++e) o[e] = on[e];
        }
      }
      LY_T(14);
      // this tile's per-image partial of g_u: rows in order, one segment per image (threads 0..127)
      if (threadIdx.x < M) {
        const int i = threadIdx.x;
        const int r0 = tile * 32;
        const int nrow = a.N - r0 < 32 ? a.N - r0 : 32;
        float g[32];
#pragma unroll
        for (int n = 0; n < 32; ++n) g[n] = st.g1[n][i];
        int next = (r0 / a.S + 1) * a.S - r0;        // first row of the next image
        float acc = 0.f;
        int seg = 0;
#pragma unroll
        for (int n = 0; n < 32; ++n) {
          if (n < nrow) {
            if (n == next) {
              a.gu_tiles[((size_t)tile * a.nseg + seg) * M + i] = acc;
              acc = 0.f;
              ++seg;
              next += a.S;
            }
            acc += g[n];
          }
        }
        a.gu_tiles[((size_t)tile * a.nseg + seg) * M + i] = acc;
      }
      LY_T(15);
      __syncthreads();
      LY_T(16);
    }
  }
  // ---- this workgroup's partial: its own fp32 slab (plain stores), summed by k_lyap_reduce in a
  // fixed order -- bit-reproducible.  (Round 2 added the partials into 8 per-XCD float64 sums with
  // atomics instead; float atomics execute at the memory side, not in L2 (MI355X_MICROARCH.md,
  // Global float atomics: ~1.3 TB/s of added bytes), so the 4.9 M adds cost ~20 us more per step
  // than these 19.7 MB of slab stores and their reduce: k_lyap_bwd 103 -> 83 us.)
  db2 += shfl_xor32(db2);
  db3 += __shfl_xor(db3, 16, 64);
  db3 += shfl_xor32(db3);
  float* slab = a.slabs + (size_t)blockIdx.x * SLAB;
#pragma unroll
  for (int kb = 0; kb < 4; ++kb)
#pragma unroll
    for (int r = 0; r < 16; ++r) slab[SLAB_Q2 + (32 * w + acc_row(r, half)) * M + 32 * kb + col] = dq2[kb][r];
#pragma unroll
  for (int hb = 0; hb < 2; ++hb)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int i = 4 * q16 + r;
      if (i < C) slab[SLAB_Q3 + i * M + 32 * w + 16 * hb + j16] = dq3[hb][r];
      if (j16 < C) slab[SLAB_Q1 + (32 * w + 16 * hb + i) * C + j16] = dq1[hb][r];
    }
  if (half == 0) {
    slab[SLAB_B2 + 32 * w + col] = db2;
    if (w == 0 && col < C) slab[SLAB_B3 + col] = db3;
  }
  LY_STAMP(64 + 2048, 1);
}

// Weight gradients (the train_ode solve's rows; fiode_internal::launch_wgrad).  A row group is
// ipw images (part p of each; with a device row count only rows s < s_used[0] of an image) -- about
// 80 rows -- and each group is split over four workgroups by column block cb: dQ2[:, 32cb:+32] (wave
// w: the 32 x 32 block of rows 32w), dQ3[:, 32cb:+32] (wave 2) and dQ1[32cb:+32, :] (wave 3) on
// 16x16x4 tiles (C = 10 pads to 16, not 32), db2[32cb:+32] (wave cb), db3 (wave 2 of cb 0).  The
// four column blocks write disjoint quarters of their group's partial slab, summed by k_lyap_reduce
// in a fixed order (bit-reproducible).  Round 3 gave each workgroup all columns of 20 rows: the same
// MFMA cycles per wave (dQ3 / dQ1 were padded 32 x 32 blocks), 4x the slabs (19.7 MB written and
// re-read per RK4 step).  Rows are staged WG_CH at a time, every load of a chunk in flight at once.
// Blocks past 4 x nslab sum g_u[b] = the image's gz1 rows in row order (independent of the slabs).
constexpr int WG_CH = 40;       // rows per staged chunk (the RK4 solve's 40 evals of an image)
constexpr int WG_LDA = 160;     // gz2 row stride: a row pair's two halves on disjoint banks
constexpr int WG_LDN = 32;      // 32-column rows (a1, a2, gz1 of the column block): likewise
struct WgStage {
  float gz2[WG_CH][WG_LDA];
  float a1[WG_CH][WG_LDN], a2[WG_CH][WG_LDN], gz1[WG_CH][WG_LDN];
  float gft[WG_CH][12], h[WG_CH][12];
};
constexpr size_t WG_LDS = sizeof(WgStage);
static_assert(WG_LDS <= 160 * 1024, "wgrad stage fits the LDS");
__global__ __launch_bounds__(256, 1) void k_lyap_wgrad(LyapArgs a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  WgStage& S = *reinterpret_cast<WgStage*>(smem);
  if ((int)blockIdx.x >= 4 * a.nslab) {      // g_u[b][i] = sum of image b's gz1 rows, in row order
    const int q = ((int)blockIdx.x - 4 * a.nslab) * 256 + threadIdx.x;
    if (q < a.B * M) {
      const int b = q / M, i = q - b * M;
      const int n = a.s_used ? min(a.S, a.s_used[0]) : a.S;
      const float* gz = a.gz1 + (size_t)b * a.S * M + i;
      float acc[4] = {0.f, 0.f, 0.f, 0.f};
      int r = 0;
      for (; r + 4 <= n; r += 4)
#pragma unroll
        for (int u = 0; u < 4; ++u) acc[u] += gz[(size_t)(r + u) * M];
      for (; r < n; ++r) acc[0] += gz[(size_t)r * M];
      a.g_u[q] = (acc[0] + acc[1]) + (acc[2] + acc[3]);
    }
    return;
  }
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, half = lane >> 5, col = lane & 31;
  const int j16 = lane & 15, q16 = lane >> 4;
  // the four column blocks of a group are blocks grp + k * nslab: with nslab % 8 == 0 they share an
  // XCD (blocks are dealt round-robin over the 8 XCDs), so three of the four gz2 reads hit its L2
  const int grp = (int)blockIdx.x % a.nslab, cb = (int)blockIdx.x / a.nslab;
  const int g = grp / a.parts, p = grp - g * a.parts;
  const float* hsrc = (a.sampler == FIODE_SAMPLER_GIVEN) ? a.h_in : a.h_ws;
  WG_STAMP(0);
  f32x16 acc2 = f16_zero();
  f32x4q dq[2] = {q4_zero(), q4_zero()};     // wave 2: dQ3 tiles, wave 3: dQ1 tiles
  float db2 = 0.f, db3 = 0.f;
  // stage registers: gz2 32 float4 per row, the column block of a1 / a2 / gz1 8 float4 each, gft /
  // h rows; rows past n load row n - 1 and are stored as zeros (A and B operands)
  constexpr int NW = WG_CH * 32 / 256;                        // gz2 float4 per thread
  constexpr int NN = (WG_CH * 24 + 255) / 256;                // narrow float4 per thread
  constexpr int NS = WG_CH * C * 2, NST = (NS + 255) / 256;
  f32x4 vw[NW], vn[NN];
  float sv[NST];
  const int k4 = threadIdx.x & 31;
  auto load = [&](int c0, int n) {            // rows c0 .. c0 + n - 1 (n <= WG_CH) -> registers
#pragma unroll
    for (int u = 0; u < NW; ++u) {
      const int r = (threadIdx.x >> 5) + 8 * u;
      vw[u] = *reinterpret_cast<const f32x4*>(a.gz2 + (size_t)(c0 + min(r, n - 1)) * M + 4 * k4);
    }
#pragma unroll
    for (int u = 0; u < NN; ++u) {
      const int e = threadIdx.x + 256 * u;
      const int r = e / 24, rem = e - r * 24, arr = rem >> 3, c4 = rem & 7;
      const float* src = arr == 0 ? a.a1 : arr == 1 ? a.a2 : a.gz1;
      vn[u] = e < WG_CH * 24 ? *reinterpret_cast<const f32x4*>(src + (size_t)(c0 + min(r, n - 1)) * M + 32 * cb + 4 * c4)
                             : f32x4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int u = 0; u < NST; ++u) {
      const int e = threadIdx.x + u * 256;
      const int r = (e >> 1) / C, c = (e >> 1) - r * C;
      const int rs = min(r, n - 1);
      const float t = e < NS ? ((e & 1) ? hsrc[(size_t)(c0 + rs) * C + c] : a.gft[(size_t)(c0 + rs) * C + c]) : 0.f;
      sv[u] = (e < NS && r < n) ? t : 0.f;
    }
  };
  auto store = [&](int n) {                   // registers -> LDS (the previous chunk's readers are done)
#pragma unroll
    for (int u = 0; u < NW; ++u) {
      const int r = (threadIdx.x >> 5) + 8 * u;
      *reinterpret_cast<f32x4*>(&S.gz2[r][4 * k4]) = r < n ? vw[u] : f32x4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int u = 0; u < NN; ++u) {
      const int e = threadIdx.x + 256 * u;
      if (e < WG_CH * 24) {
        const int r = e / 24, rem = e - r * 24, arr = rem >> 3, c4 = rem & 7;
        float* dst = arr == 0 ? &S.a1[r][4 * c4] : arr == 1 ? &S.a2[r][4 * c4] : &S.gz1[r][4 * c4];
        *reinterpret_cast<f32x4*>(dst) = r < n ? vn[u] : f32x4{0.f, 0.f, 0.f, 0.f};
      }
    }
#pragma unroll
    for (int u = 0; u < NST; ++u) {
      const int e = threadIdx.x + u * 256;
      if (e < NS) {
        const int r = (e >> 1) / C, c = (e >> 1) - r * C;
        if (e & 1) S.h[r][c] = sv[u];
        else S.gft[r][c] = sv[u];
      }
    }
  };
  auto compute = [&](int n) {
    // dQ2 block (rows 32w, columns 32cb): row pairs, LDS operands of pair j + 2 read before the
    // MFMA of pair j (one wave per SIMD: nothing else hides the LDS latency)
    {
      float av = S.gz2[half][32 * w + col], bv = S.a1[half][col];
      for (int j = 0; j < n; j += 2) {
        float an = av, bn = bv;
        if (j + 2 < n) {
          an = S.gz2[j + 2 + half][32 * w + col];
          bn = S.a1[j + 2 + half][col];
        }
        acc2 = mfma32(av, bv, acc2);
        if (w == cb) db2 += av;
        av = an;
        bv = bn;
      }
    }
    if (w >= 2) {                             // dQ3 (wave 2) / dQ1 (wave 3) on 16x16x4 tiles, row quads
      const int nq = (n + 3) >> 2;
      auto ld = [&](int s4, float (&o)[3]) {
        const int r = 4 * s4 + q16;
        if (w == 2) {
          o[0] = j16 < C ? S.gft[r][j16] : 0.f;
          o[1] = S.a2[r][j16];
          o[2] = S.a2[r][16 + j16];
        } else {
          o[0] = j16 < C ? S.h[r][j16] : 0.f;
          o[1] = S.gz1[r][j16];
          o[2] = S.gz1[r][16 + j16];
        }
      };
      float o[3], on[3];
      ld(0, o);
      for (int s4 = 0; s4 < nq; ++s4) {
        on[0] = o[0]; on[1] = o[1]; on[2] = o[2];
        if (s4 + 1 < nq) ld(s4 + 1, on);
        if (w == 2) {
          db3 += o[0];
          dq[0] = mfma16q(o[0], o[1], dq[0]);
          dq[1] = mfma16q(o[0], o[2], dq[1]);
        } else {
          dq[0] = mfma16q(o[1], o[0], dq[0]);
          dq[1] = mfma16q(o[2], o[0], dq[1]);
        }
        o[0] = on[0]; o[1] = on[1]; o[2] = on[2];
      }
    }
  };
  // the group's chunks: images g * ipw .. (g + 1) * ipw - 1, rows r0 .. r1 of each (part p, and
  // with a device row count only rows s < s_used[0]), WG_CH rows at a time; the next chunk's loads
  // are in flight while the current chunk's MFMAs run
  const int b_end = min(a.B, (g + 1) * a.ipw);
  auto rows_of = [&](int b, int& r0, int& r1) {
    r0 = b * a.S + p * a.chunk;
    r1 = min(r0 + a.chunk, (b + 1) * a.S);
    if (a.s_used) r1 = min(r1, b * a.S + a.s_used[0]);        // rows past the device count are not data
  };
  auto next = [&](int& b, int& c0, int& r1) {   // first chunk at or after (b, c0) that has rows
    while (b < b_end && c0 >= r1) {
      if (++b < b_end) rows_of(b, c0, r1);
    }
  };
  int b = g * a.ipw, c0 = 0, r1 = 0;
  if (b < b_end) rows_of(b, c0, r1);
  next(b, c0, r1);
  if (b < b_end) {
    int n = min(WG_CH, r1 - c0);
    load(c0, n);
    store(n);
    __syncthreads();
    WG_STAMP(1);
    while (true) {
      int bn = b, cn = c0 + WG_CH, rn = r1;
      next(bn, cn, rn);
      const bool more = bn < b_end;
      const int nn = more ? min(WG_CH, rn - cn) : 0;
      if (more) load(cn, nn);                 // in flight during this chunk's MFMAs
      compute(n);
      __syncthreads();
      if (!more) break;
      store(nn);
      __syncthreads();
      b = bn; c0 = cn; r1 = rn; n = nn;
    }
  }
  WG_STAMP(2);
  float* slab = a.slabs + (size_t)grp * SLAB;
#pragma unroll
  for (int r = 0; r < 16; ++r) slab[SLAB_Q2 + (32 * w + acc_row(r, half)) * M + 32 * cb + col] = acc2[r];
  if (w == 2) {
#pragma unroll
    for (int hb = 0; hb < 2; ++hb)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int i = 4 * q16 + r;
        if (i < C) slab[SLAB_Q3 + i * M + 32 * cb + 16 * hb + j16] = dq[hb][r];
      }
  } else if (w == 3) {
#pragma unroll
    for (int hb = 0; hb < 2; ++hb)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        if (j16 < C) slab[SLAB_Q1 + (32 * cb + 16 * hb + 4 * q16 + r) * C + j16] = dq[hb][r];
  }
  if (w == cb) {
    db2 += shfl_xor32(db2);
    if (half == 0) slab[SLAB_B2 + 32 * cb + col] = db2;
  }
  if (w == 2 && cb == 0) {
    db3 += __shfl_xor(db3, 16, 64);
    db3 += shfl_xor32(db3);
    if (q16 == 0 && j16 < C) slab[SLAB_B3 + j16] = db3;
  }
  WG_STAMP(3);
}

// one item of the static gradients (k_lyap_static_grads; the wgrad chain's k_lyap_reduce)
__device__ __forceinline__ void static_grads_item(const LyapArgs& a, int e) {
  if (e < M * FIODE_X) {
    const int i = e / FIODE_X, c = e - i * FIODE_X;
    float s = 0.f;
#pragma unroll 16
    for (int b = 0; b < a.B; ++b) s = __fmaf_rn(a.g_u[(size_t)b * M + i], a.x_feat[(size_t)b * FIODE_X + c], s);
    a.grads.Qx[e] = s;
  } else if (e < M * FIODE_X + M) {
    const int i = e - M * FIODE_X;
    float s = 0.f;
#pragma unroll 16
    for (int b = 0; b < a.B; ++b) s += a.g_u[(size_t)b * M + i];
    a.grads.bx[i] = s;
    a.grads.b1[i] = s;
  } else if (a.grads.x_feat && e < M * FIODE_X + M + a.B * FIODE_X) {
    const int q = e - M * FIODE_X - M, b = q / FIODE_X, c = q - b * FIODE_X;
    float s = 0.f;
#pragma unroll 16
    for (int i = 0; i < M; ++i) s = __fmaf_rn(a.g_u[(size_t)b * M + i], a.Qx[i * FIODE_X + c], s);
    a.grads.x_feat[q] = s;
  }
}

// Sum of the slabs (fixed order, deterministic) -> dQ2, dQ3, dQ1, db2, db3; then per-image g_u
// and the scalars (fused fan-out backward) or the static gradients (weight-gradient chain).  Workgroup w < n_el_blocks sums 64 consecutive slab entries: its 4 waves each add a
// quarter of the slabs (8 independent loads in flight per lane), then combine through LDS.
// The last workgroup reduces the per-tile scalars.
constexpr int RED_COLS = 64;
__global__ __launch_bounds__(256) void k_lyap_reduce(LyapArgs a) {
  __shared__ float part[4][RED_COLS];
  __shared__ double dpart[3][256];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int nwg = a.nslab;
  const int n_el_blocks = (SLAB + RED_COLS - 1) / RED_COLS;
  const int n_gu_blocks = (a.B * M + RED_COLS - 1) / RED_COLS;
  if ((int)blockIdx.x < n_el_blocks) {
    const int e = blockIdx.x * RED_COLS + lane;
    float s = 0.f;
    if (e < SLAB) {
      const int k0 = (nwg * wv) / 4, k1 = (nwg * (wv + 1)) / 4;
      float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      int k = k0;
      for (; k + 8 <= k1; k += 8)
#pragma unroll
        for (int u = 0; u < 8; ++u) acc[u] += a.slabs[(size_t)(k + u) * SLAB + e];
      for (; k < k1; ++k) acc[0] += a.slabs[(size_t)k * SLAB + e];
      s = ((acc[0] + acc[1]) + (acc[2] + acc[3])) + ((acc[4] + acc[5]) + (acc[6] + acc[7]));
    }
    part[wv][lane] = s;
    __syncthreads();
    if (wv == 0 && e < SLAB) {
      const float t = (part[0][lane] + part[1][lane]) + (part[2][lane] + part[3][lane]);
      if (e < SLAB_Q3) a.grads.Q2[e] = t;
      else if (e < SLAB_Q1) a.grads.Q3[e - SLAB_Q3] = t;
      else if (e < SLAB_B2) a.grads.Q1[e - SLAB_Q1] = t;
      else if (e < SLAB_B1) a.grads.b2[e - SLAB_B2] = t;
      else if (e >= SLAB_B3 && e < SLAB_B3 + C) a.grads.b3[e - SLAB_B3] = t;
    }
  } else if (!a.gu_tiles) {       // weight-gradient chain: g_u is final (k_lyap_wgrad) -> static grads
    static_grads_item(a, ((int)blockIdx.x - n_el_blocks) * 256 + threadIdx.x);
  } else if ((int)blockIdx.x < n_el_blocks + n_gu_blocks) {      // g_u[b][i] = sum over the image's tiles
    const int q = (blockIdx.x - n_el_blocks) * RED_COLS + (threadIdx.x & (RED_COLS - 1));
    if (threadIdx.x < RED_COLS && q < a.B * M) {
      const int b = q / M, i = q - b * M;
      float s = 0.f;
      {                           // fused backward: the tiles holding rows of image b, in order
        const int t0 = (int)(((size_t)b * a.S) / 32), t1 = (int)(((size_t)(b + 1) * a.S - 1) / 32);
        for (int t = t0; t <= t1; ++t) {
          const int seg = b - (int)(((size_t)t * 32) / a.S);
          s += a.gu_tiles[((size_t)t * a.nseg + seg) * M + i];
        }
      }
      a.g_u[q] = s;
    }
  } else if (a.tile_sc) {                                           // scalars
    const int ntiles = (a.N + 31) / 32;
    double v = 0.0, ef = 0.0, ac = 0.0;
    for (int t = threadIdx.x; t < ntiles; t += 256) {
      const f32x4 q = *reinterpret_cast<const f32x4*>(a.tile_sc + 4 * t);
      v += q[0]; ef += q[1]; ac += q[2];
    }
    dpart[0][threadIdx.x] = v; dpart[1][threadIdx.x] = ef; dpart[2][threadIdx.x] = ac;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
      if ((int)threadIdx.x < o)
        for (int c = 0; c < 3; ++c) dpart[c][threadIdx.x] += dpart[c][threadIdx.x + o];
      __syncthreads();
    }
    if (threadIdx.x == 0) {
      v = dpart[0][0]; ef = dpart[1][0]; ac = dpart[2][0];
      a.scalars[0] = (float)(v / a.N);
      a.scalars[1] = (float)ef;
      a.scalars[2] = (float)(ac / ((double)a.N * C));
      a.scalars[3] = (float)qp_exit_iter(conv_word(a, 0), a.d.max_iter);
      a.scalars[4] = (float)qp_exit_iter(conv_word(a, 1), a.d.max_iter);
      a.scalars[5] = (float)v;
      a.scalars[6] = (float)ac;
      a.scalars[7] = (float)a.N;
    }
  }
}

// dQx = g_u^T x ; dbx = db1 = sum_b g_u ; dx = g_u Qx   (expand backward, pl_modules.py:400)
// (the fixed-order sums are unrolled so their loads are in flight together: 33 -> ~10 us)
__global__ __launch_bounds__(256) void k_lyap_static_grads(LyapArgs a) {
  static_grads_item(a, blockIdx.x * blockDim.x + threadIdx.x);
}

// ---- workspace ----------------------------------------------------------------------------------
struct WsLayout {
  size_t conv, u, h, ft, kw, tsc, slabs, gut, gu, total;
  int nslab, nseg;
};
inline size_t al(size_t x) { return (x + 255) & ~(size_t)255; }
inline void parts_for(int B, int S, int& parts, int& chunk) {
  parts = (256 + B - 1) / B;
  const int maxp = S / 16 > 0 ? S / 16 : 1;        // >= 16 rows per part
  if (parts > maxp) parts = maxp;
  if (parts < 1) parts = 1;
  chunk = (S + parts - 1) / parts;
  chunk = (chunk + 1) & ~1;
}
// fused backward: one workgroup per 4 tiles up to one per CU (BWD_LDS: one resident per CU); its
// partial slab count is the grid size
constexpr int BWD_MAX_WG = 256;
inline int bwd_grid(size_t N) {
  const int ntiles = (int)((N + 31) / 32);
  const int g = (ntiles + 3) / 4;
  return g < BWD_MAX_WG ? g : BWD_MAX_WG;
}
inline WsLayout ws_layout(int B, int S) {
  const size_t N = (size_t)B * S;
  const size_t ntiles = (N + 31) / 32;
  WsLayout L;
  L.nslab = bwd_grid(N);
  L.nseg = S >= 32 ? 2 : (31 / S + 2 > 32 ? 32 : 31 / S + 2);   // images one 32-row tile can span
  size_t o = 0;
  L.conv = o; o = al(o + 2 * CONV_SLOTS * 4);
  L.u = o; o = al(o + (size_t)B * M * 4);
  L.h = o; o = al(o + N * C * 4);
  L.ft = o; o = al(o + 2 * N * C * 4);
  L.kw = o; o = al(o + 4 * N * 16);
  L.tsc = o; o = al(o + ntiles * 16);
  L.slabs = o; o = al(o + (size_t)L.nslab * SLAB * 4);
  L.gut = o; o = al(o + ntiles * L.nseg * M * 4);
  L.gu = o; o = al(o + (size_t)B * M * 4);
#ifdef OT_PROFILE
  o += (64 + 4096) * 8;                      // phase timers + per-workgroup stamps (the tail)
#endif
  L.total = o;
  return L;
}

int check_dyn(const fiode_dyn_config* d) {
  if (!d) return FIODE_EINVAL;
  if (d->n_hidden != C || d->mlp_size != M || d->x_dim != FIODE_X) return FIODE_ESHAPE;
  if (d->qp_max_iter < 1 || d->qp_max_iter > 32) return FIODE_EINVAL;
  if (!(d->dropout >= 0.f && d->dropout < 1.f)) return FIODE_EINVAL;
  return FIODE_OK;
}

}  // namespace

extern "C" size_t fiode_lyap_workspace_bytes(const fiode_lyap_config* cfg, const fiode_dyn_config* dyn) {
  (void)dyn;
  if (!cfg || cfg->batch <= 0 || cfg->sample_size <= 0) return 0;
  return ws_layout(cfg->batch, cfg->sample_size).total;
}

extern "C" int fiode_lyap_step(void* stream, const fiode_lyap_config* cfg, const fiode_dyn_config* dyn,
                               const fiode_dyn_weights* w, const fiode_lyap_io* io, fiode_lyap_grads* grads,
                               void* workspace, size_t workspace_bytes) {
  int rc = check_dyn(dyn);
  if (rc) return rc;
  if (!cfg || !w || !io || !grads || !workspace) return FIODE_EINVAL;
  const int B = cfg->batch, S = cfg->sample_size;
  if (B <= 0 || S <= 0 || (long long)B * S > (1LL << 30)) return FIODE_EINVAL;
  if (cfg->n_uniform < 0 || cfg->n_uniform > S) return FIODE_EINVAL;
  if (cfg->sampler < 0 || cfg->sampler > 3 || cfg->dropout_mode < 0 || cfg->dropout_mode > 2) return FIODE_EINVAL;
  if (!io->x_feat || !io->y || !io->scalars) return FIODE_EINVAL;
  if (cfg->sampler == FIODE_SAMPLER_GIVEN && !io->h) return FIODE_EINVAL;
  if (cfg->sampler == FIODE_SAMPLER_TRAJECTORY && cfg->n_uniform < S && !io->h) return FIODE_EINVAL;
  if (cfg->dropout_mode == FIODE_DROPOUT_GIVEN && !io->masks) return FIODE_EINVAL;
  if (!w->Q1 || !w->b1 || !w->Qx || !w->bx || !w->Q2 || !w->b2 || !w->Q3 || !w->b3) return FIODE_EINVAL;
  if (!grads->Q1 || !grads->b1 || !grads->Qx || !grads->bx || !grads->Q2 || !grads->b2 || !grads->Q3 ||
      !grads->b3 || !grads->x_feat)
    return FIODE_EINVAL;
  const WsLayout L = ws_layout(B, S);
  if (workspace_bytes < L.total) return FIODE_EWORKSPACE;
  char* ws = static_cast<char*>(workspace);

  LyapArgs a{};
  a.N = B * S; a.S = S; a.B = B; a.S1 = cfg->n_uniform;
  a.sampler = cfg->sampler;
  const float p = cfg->dropout_mode == FIODE_DROPOUT_OFF ? 0.f : dyn->dropout;
  a.dropout_mode = (p == 0.f) ? FIODE_DROPOUT_OFF : cfg->dropout_mode;
  a.bit_mode = (p == 0.5f);
  a.thr8 = (uint32_t)lrintf((1.0f - p) * 256.0f);
  a.drop_scale = (a.dropout_mode == FIODE_DROPOUT_OFF) ? 1.0f : 1.0f / (1.0f - p);
  a.rng.key = make_uint2((uint32_t)cfg->seed, (uint32_t)(cfg->seed >> 32));
  a.rng.off_lo = (uint32_t)cfg->offset; a.rng.off_hi = (uint32_t)(cfg->offset >> 32);
  a.offset_dev = io->offset_dev;
  a.d.alpha_1 = dyn->alpha_1; a.d.alpha_2 = dyn->alpha_2; a.d.sigma_1 = dyn->sigma_1;
  a.d.tol = dyn->qp_tol; a.d.scale_nominal = dyn->scale_nominal; a.d.max_iter = dyn->qp_max_iter;
  a.kappa = cfg->kappa;
  a.kappa_dev = io->kappa_dev;
  a.invN = 1.0f / (float)a.N;
  parts_for(B, S, a.parts, a.chunk);
  a.x_feat = io->x_feat; a.y = io->y; a.h_in = io->h; a.masks = io->masks;
  a.Q1 = w->Q1; a.b1 = w->b1; a.Qx = w->Qx; a.bx = w->bx; a.Q2 = w->Q2; a.b2 = w->b2; a.Q3 = w->Q3; a.b3 = w->b3;
  a.conv = reinterpret_cast<uint32_t*>(ws + L.conv);
  a.u = reinterpret_cast<float*>(ws + L.u);
  a.h_ws = reinterpret_cast<float*>(ws + L.h);
  a.ft_ws = reinterpret_cast<float*>(ws + L.ft);
  a.kw = reinterpret_cast<uint4*>(ws + L.kw);
  a.tile_sc = reinterpret_cast<float*>(ws + L.tsc);
  a.slabs = reinterpret_cast<float*>(ws + L.slabs);
  a.nslab = L.nslab;
#ifdef OT_PROFILE
  a.prof = reinterpret_cast<unsigned long long*>(ws + L.total - (64 + 4096) * 8);
#endif
  a.gu_tiles = reinterpret_cast<float*>(ws + L.gut);
  a.nseg = L.nseg;
  a.g_u = reinterpret_cast<float*>(ws + L.gu);
  a.scalars = io->scalars;
  a.h_out = io->h_out; a.V = io->V; a.Vdot = io->Vdot; a.f = io->f; a.f_log = io->f_log;
  a.qp_lower = io->qp_lower; a.qp_nominal = io->qp_nominal; a.g_ftilde = io->g_ftilde;
  a.exp_draws = io->exp_draws; a.exp_draws_out = io->exp_draws_out; a.kw_out = io->keep_words_out;
  a.grads = *grads;

  hipStream_t st = static_cast<hipStream_t>(stream);
  const bool prof = io->events && io->n_events >= FIODE_LYAP_NKERNELS + 1;
  int ev = 0;
  auto mark = [&]() -> int {
    if (prof) {
      hipError_t e = hipEventRecord(static_cast<hipEvent_t>(io->events[ev++]), st);
      if (e != hipSuccess) return 100 + (int)e;
    }
    return 0;
  };
  const int ntiles = (a.N + 31) / 32;
  int fwd_blocks = (ntiles + FWD_WAVES - 1) / FWD_WAVES;                    // one tile (both passes) per wave
  {
    int dev = 0, ncu = 256;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        ncu <= 0)
      ncu = 256;
    if (fwd_blocks > (8 / FWD_WAVES) * ncu) fwd_blocks = (8 / FWD_WAVES) * ncu;   // persistent: resident workgroups
  }
  const size_t lds_fwd = (size_t)(M + C) * LDQ * sizeof(float);
  if ((rc = mark())) return rc;
  hipLaunchKernelGGL(k_static_proj, dim3(B), dim3(128), 0, st, a);
  FIODE_HIP_CHECK(hipGetLastError());
  if ((rc = mark())) return rc;
  hipLaunchKernelGGL(k_lyap_prep, dim3((a.N + 255) / 256), dim3(256), 0, st, a);
  FIODE_HIP_CHECK(hipGetLastError());
  if ((rc = mark())) return rc;
  hipLaunchKernelGGL(k_lyap_fwd, dim3(fwd_blocks), dim3(64 * FWD_WAVES), lds_fwd, st, a);
  FIODE_HIP_CHECK(hipGetLastError());
  if ((rc = mark())) return rc;
  hipLaunchKernelGGL(k_lyap_bwd, dim3(L.nslab), dim3(256), BWD_LDS, st, a);
  FIODE_HIP_CHECK(hipGetLastError());
  if ((rc = mark())) return rc;
  const int red_blocks = (SLAB + RED_COLS - 1) / RED_COLS + (B * M + RED_COLS - 1) / RED_COLS + 1;
  hipLaunchKernelGGL(k_lyap_reduce, dim3(red_blocks), dim3(256), 0, st, a);
  FIODE_HIP_CHECK(hipGetLastError());
  if ((rc = mark())) return rc;
  const int sg_items = M * FIODE_X + M + B * FIODE_X;
  hipLaunchKernelGGL(k_lyap_static_grads, dim3((sg_items + 255) / 256), dim3(256), 0, st, a);
  FIODE_HIP_CHECK(hipGetLastError());
  if ((rc = mark())) return rc;
  return FIODE_OK;
}

#ifdef OT_PROFILE
extern "C" FIODE_API int fiode_debug_wgrad_stamps(unsigned long long* host, int n) {
  if (n > 4 * 1024) n = 4 * 1024;
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_wg_stamps), (size_t)n * 8, 0, hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}
#endif

// ---- shared with the ODE training path (odetrain.hip): weight gradients of rows (b, s) ------
namespace fiode_internal {
// Weight-gradient grid: row groups of ~80 rows (ipw images, or one part of an image), at most 256,
// each on four workgroups (column blocks, k_lyap_wgrad) that fill one 77 KB partial slab together.
// S is the exact rows per image (rk4) or, with a device row count (dopri5: S = the eval capacity),
// an upper bound: the estimate then takes 64 rows per image.  nwg = the row groups (= slabs).
struct WgGrid { int parts, chunk, ipw, nwg; };
WgGrid wgrad_grid(int B, int S, bool exact_rows) {
  WgGrid g{};
  const long long se = exact_rows ? S : (S < 64 ? S : 64);
  long long t = (long long)B * se / 80;
  if (t < 1) t = 1;
  if (t > 256) t = 256;
  g.parts = 1;
  g.ipw = 1;
  if (t >= B) {
    const int maxp = (int)(se / 80 > 0 ? se / 80 : 1);
    g.parts = (int)(t / B) < maxp ? (int)(t / B) : maxp;
  } else {
    g.ipw = (int)((B + t - 1) / t);
  }
  g.chunk = (S + g.parts - 1) / g.parts;
  g.chunk = (g.chunk + 1) & ~1;
  g.nwg = (B + g.ipw - 1) / g.ipw * g.parts;
  return g;
}

size_t wgrad_bytes(int B, int S, bool exact_rows) {
  const WgGrid g = wgrad_grid(B, S, exact_rows);
  return al((size_t)g.nwg * SLAB * 4) + al((size_t)B * M * 4);
}

int launch_wgrad(hipStream_t st, const WgradIO& io) {
  LyapArgs a{};
  a.B = io.B; a.S = io.S; a.N = io.B * io.S;
  a.s_used = io.s_used;
  const WgGrid g = wgrad_grid(a.B, a.S, io.s_used == nullptr);
  a.parts = g.parts; a.chunk = g.chunk; a.ipw = g.ipw;
  a.sampler = FIODE_SAMPLER_GIVEN;
  a.h_in = io.h; a.x_feat = io.x_feat; a.Qx = io.Qx;
  a.a1 = const_cast<float*>(io.a1); a.a2 = const_cast<float*>(io.a2);
  a.gz2 = const_cast<float*>(io.gz2); a.gz1 = const_cast<float*>(io.gz1); a.gft = const_cast<float*>(io.gft);
  char* ws = static_cast<char*>(io.workspace);
  a.slabs = reinterpret_cast<float*>(ws);
  a.g_u = reinterpret_cast<float*>(ws + al((size_t)g.nwg * SLAB * 4));
  a.tile_sc = nullptr;
  a.nslab = g.nwg;
  a.gu_tiles = nullptr;
  a.grads = io.grads;
  // one launch: the slab workgroups + g_u blocks (independent: g_u reads the gz1 rows); then one
  // launch for the slab sums beside the static gradients, which need only the finished g_u
  hipLaunchKernelGGL(k_lyap_wgrad, dim3(4 * g.nwg + (a.B * M + 255) / 256), dim3(256), WG_LDS, st, a);
  FIODE_HIP_CHECK(hipGetLastError());
  const int sg_items = M * FIODE_X + M + a.B * FIODE_X;
  const int red_blocks = (SLAB + RED_COLS - 1) / RED_COLS + (sg_items + 255) / 256;
  hipLaunchKernelGGL(k_lyap_reduce, dim3(red_blocks), dim3(256), 0, st, a);
  FIODE_HIP_CHECK(hipGetLastError());
  return FIODE_OK;
}
}  // namespace fiode_internal
