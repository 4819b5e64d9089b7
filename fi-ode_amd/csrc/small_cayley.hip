// One-launch Cayley maps for small k = min(cout, cin) <= 16 (gfx950): the backbone's last
// CayleyLinear (512 -> 10) and the dynamics' three 128 x 10 maps (classification.py:282-293
// convert_cayley; fiode_amd/cayley.py _SmallCayleyFn).  For these the dense path
// (_DenseCayleyFn: library GEMMs + dense.hip stages + Gauss-Jordan) is ~10 dependent launches
// forward and ~12 backward of a few us each; here each direction is ONE workgroup per matrix:
//
// X = s Wx (Wx = W, or W^T when cin > cout: the "tall" orientation, R = max(cout, cin) rows),
// s = alpha / ||W||, U = X[:k], V = X[k:]:
//   forward   M = I + (U - U^T) + V^T V,  inv = M^-1 (wave-0 Gauss-Jordan in registers, natural
//             order: M's symmetric part is I + V^T V >= I, no pivoting),  Q = [2 inv - I ; -2 V inv]
//   backward  G = dL/dQ (tall), Ginv = 2 Gt - 2 V^T Gb,  GM = -(inv^T Ginv) inv^T,
//             gU = GM - GM^T,  gV = V (GM + GM^T) - 2 Gb inv^T,
//             D = <gX, Wx>,  dL/dW = s gX - alpha D / ||W||^3 W,  dL/dalpha = D / ||W||
// -- the same formula and operation order as _CayleyScaledFn.  Every sum runs in a fixed order
// (no float atomics): the Frobenius norm and D as 256 per-thread partials + a fixed tree, the
// k x k Gram products over row parts with 8 accumulators each, added in order.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "common.h"
#include "fiode.h"

namespace {

constexpr int NT = 256;
constexpr int KM = FIODE_SMALL_CAYLEY_MAX_K;      // 16

struct SCArgs {
  int prio;             // g_fiode_prio_mask bit 2 at launch
  int cout, cin, k, R, wide;
  const float* W;       // [b][cout][cin]
  const float* alpha;   // [b]
  float* nrm;           // [b]      (forward writes, backward reads)
  float* inv;           // [b][k][k] (forward writes, backward reads)
  float* Q;             // [b][cout][cin] (forward)
  const float* gQ;      // [b][cout][cin] (backward)
  float* gW;            // [b][cout][cin] (backward)
  float* galpha;        // [b]            (backward)
};

__device__ __forceinline__ int64_t wpos(const SCArgs& a, int r, int c) {   // tall (r, c) -> W offset
  return a.wide ? (int64_t)c * a.cin + r : (int64_t)r * a.cin + c;
}

// Fixed-order block sum of one value per thread (256 threads): result in every thread.
__device__ __forceinline__ float block_sum(float v, float* red) {
  red[threadIdx.x] = v;
  __syncthreads();
#pragma unroll
  for (int o = NT / 2; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) red[threadIdx.x] = red[threadIdx.x] + red[threadIdx.x + o];
    __syncthreads();
  }
  const float r = red[0];
  __syncthreads();
  return r;
}

// In-register Gauss-Jordan inverse of the k x k (k <= 16, padded with I) matrix in LDS m[16][17],
// by wave 0: lane l owns row l >> 2, columns 4 (l & 3) .. + 3; pivot rows / columns travel by
// shuffles (no workgroup barriers).  Result written back to m.
__device__ __forceinline__ void wave_gj16(float (*m)[KM + 1], int k) {
  const int l = threadIdx.x;          // caller: l < 64
  const int i = l >> 2, cg = l & 3;
  float x[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int j = 4 * cg + e;
    x[e] = (i < k && j < k) ? m[i][j] : (i == j ? 1.0f : 0.0f);
  }
#pragma unroll
  for (int p = 0; p < KM; ++p) {
    const int pc = p >> 2, pe = p & 3;
    float r[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) r[e] = __shfl(x[e], (p << 2) | cg, 64);
    const float cval = __shfl(x[pe], (i << 2) | pc, 64);
    const float piv = __shfl(x[pe], (p << 2) | pc, 64);
    const float d = 1.0f / piv;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int j = 4 * cg + e;
      const float rd = r[e] * d;
      if (i == p) x[e] = (j == p) ? d : rd;
      else x[e] = (j == p) ? -(cval * d) : fmaf(-cval, rd, x[e]);
    }
  }
#pragma unroll
  for (int e = 0; e < 4; ++e) m[i][4 * cg + e] = x[e];
}

// Copy the n = R k floats (n <= FIODE_SMALL_CAYLEY_MAX_RK = 32 x 256) of one or two matrices (W
// layout) into LDS in the tall layout with every load in flight at once (one memory round trip:
// the 512 -> 10 map's backward took six dependent round trips with 8 loads per thread in flight).
// Returns this thread's sum of squares of the first matrix's values it loaded (fixed order).
constexpr int LMAX = FIODE_SMALL_CAYLEY_MAX_RK / NT;
__device__ __forceinline__ float load_tall(const SCArgs& a, const float* __restrict__ src, float* dst,
                                           const float* __restrict__ src2 = nullptr, float* dst2 = nullptr) {
  const int tid = threadIdx.x, k = a.k, n = a.R * a.k;
  float v[LMAX], v2[LMAX];
#pragma unroll
  for (int u = 0; u < LMAX; ++u) {
    const int w = u * NT + tid;
    v[u] = w < n ? src[w] : 0.f;
    v2[u] = (src2 && w < n) ? src2[w] : 0.f;
  }
  float ss = 0.f;
#pragma unroll
  for (int u = 0; u < LMAX; ++u) {
    const int w = u * NT + tid;
    if (w < n) {
      const int r = a.wide ? w % a.cin : w / a.cin, c = a.wide ? w / a.cin : w % a.cin;
      dst[r * k + c] = v[u];
      if (dst2) dst2[r * k + c] = v2[u];
      ss = fmaf(v[u], v[u], ss);
    }
  }
  return ss;
}
static_assert(FIODE_SMALL_CAYLEY_MAX_RK % NT == 0, "load_tall: whole trips");

// Sum over rows r in [k, R) of X[r][i] * Y[r][j] for the k*k entries (i, j), fixed order: the
// rows are split into P = 256 / k^2 contiguous parts, each summed with 8 independent accumulators
// (LDS loads of 8 rows in flight), the parts added in order.  Result for entry e in red[e]
// (valid after the call's final barrier).
__device__ __forceinline__ void rows_gram(const float* X, const float* Y, int k, int R, float* red) {
  const int tid = threadIdx.x, kk = k * k;
  const int P = NT / kk > 0 ? NT / kk : 1;
  const int nrows = R - k, chunk = (nrows + P - 1) / P;
  float tot = 0.f;
  if (tid < kk * P) {
    const int e = tid % kk, part = tid / kk, i = e / k, j = e - (e / k) * k;
    const int r0 = k + part * chunk, r1 = min(R, r0 + chunk);
    float acc[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) acc[u] = 0.f;
    int r = r0;
    for (; r + 8 <= r1; r += 8) {
#pragma unroll
      for (int u = 0; u < 8; ++u) acc[u] = fmaf(X[(r + u) * k + i], Y[(r + u) * k + j], acc[u]);
    }
    for (; r < r1; ++r) acc[0] = fmaf(X[r * k + i], Y[r * k + j], acc[0]);
    tot = ((acc[0] + acc[1]) + (acc[2] + acc[3])) + ((acc[4] + acc[5]) + (acc[6] + acc[7]));
  }
  __syncthreads();                       // red may still be read by the caller's previous step
  if (tid < kk * P) red[tid] = tot;
  __syncthreads();
  if (tid < kk) {
    float v = red[tid];
    for (int part = 1; part < P; ++part) v = v + red[part * kk + tid];
    tot = v;
  }
  __syncthreads();
  if (tid < kk) red[tid] = tot;
  __syncthreads();
}

// LDS: X tall [R][k] | red [256] | m [16][17]
__global__ void __launch_bounds__(NT) k_small_cayley_fwd(SCArgs a) {
  fiode_wave_prio(a.prio);
  extern __shared__ float smem[];
  const int b = blockIdx.x, k = a.k, R = a.R, tid = threadIdx.x;
  float* X = smem;
  float* red = X + R * k;
  float (*m)[KM + 1] = reinterpret_cast<float (*)[KM + 1]>(red + NT);
  const float* Wb = a.W + (int64_t)b * a.cout * a.cin;
  const float nrm = sqrtf(block_sum(load_tall(a, Wb, X), red));   // (its barriers publish X)
  const float s = a.alpha[b] / nrm;
  for (int idx = tid; idx < R * k; idx += NT) X[idx] = X[idx] * s;
  __syncthreads();
  rows_gram(X, X, k, R, red);                     // V^T V
  if (tid < k * k) {
    const int i = tid / k, j = tid - i * k;
    float mm = (X[i * k + j] - X[j * k + i]) + red[tid];
    if (i == j) mm += 1.0f;
    m[i][j] = mm;
  }
  __syncthreads();
  if (tid < 64) wave_gj16(m, k);
  __syncthreads();
  if (tid == 0) a.nrm[b] = nrm;
  if (tid < k * k) a.inv[(int64_t)b * k * k + tid] = m[tid / k][tid % k];
  float* Qb = a.Q + (int64_t)b * a.cout * a.cin;
  for (int r = tid; r < R; r += NT) {             // one tall row per thread (W column when wide)
    if (r < k) {
      for (int c = 0; c < k; ++c) Qb[wpos(a, r, c)] = m[r][c] * 2.0f - (r == c ? 1.0f : 0.0f);
    } else {
      float x[KM];
#pragma unroll
      for (int j = 0; j < KM; ++j) x[j] = j < k ? X[r * k + j] : 0.f;
      for (int c = 0; c < k; ++c) {
        float acc = 0.f;
#pragma unroll
        for (int j = 0; j < KM; ++j)
          if (j < k) acc = fmaf(x[j], m[j][c], acc);
        Qb[wpos(a, r, c)] = acc * -2.0f;
      }
    }
  }
}

// LDS: X tall [R][k] | G tall [R][k] | gX tall [R][k] | W tall [R][k] | red [256] |
//      inv, Ginv, P1, GM [16][17] each
__global__ void __launch_bounds__(NT) k_small_cayley_bwd(SCArgs a) {
  fiode_wave_prio(a.prio);
  extern __shared__ float smem[];
  const int b = blockIdx.x, k = a.k, R = a.R, tid = threadIdx.x;
  float* X = smem;
  float* G = X + R * k;
  float* gX = G + R * k;
  float* Wt = gX + R * k;
  float* red = Wt + R * k;
  float (*iv)[KM + 1] = reinterpret_cast<float (*)[KM + 1]>(red + NT);
  float (*gi)[KM + 1] = iv + KM;
  float (*p1)[KM + 1] = gi + KM;
  float (*gm)[KM + 1] = p1 + KM;
  const float* Wb = a.W + (int64_t)b * a.cout * a.cin;
  const float* Gq = a.gQ + (int64_t)b * a.cout * a.cin;
  const float nrm = a.nrm[b], al = a.alpha[b];
  const float s = al / nrm;
  load_tall(a, Wb, Wt, Gq, G);
  if (tid < k * k) iv[tid / k][tid % k] = a.inv[(int64_t)b * k * k + tid];
  __syncthreads();
  for (int idx = tid; idx < R * k; idx += NT) X[idx] = Wt[idx] * s;
  __syncthreads();
  const int i = tid / k, j = tid - (tid / k) * k;
  const bool own = tid < k * k;
  rows_gram(X, G, k, R, red);                  // V^T Gb
  if (own) gi[i][j] = 2.0f * G[i * k + j] - 2.0f * red[tid];   // Ginv = 2 Gt - 2 V^T Gb
  __syncthreads();
  if (own) {                                   // P1 = inv^T Ginv
    float acc = 0.f;
    for (int q = 0; q < k; ++q) acc = fmaf(iv[q][i], gi[q][j], acc);
    p1[i][j] = acc;
  }
  __syncthreads();
  if (own) {                                   // GM = -(P1 inv^T)
    float acc = 0.f;
    for (int q = 0; q < k; ++q) acc = fmaf(p1[i][q], iv[j][q], acc);
    gm[i][j] = -acc;
  }
  __syncthreads();
  float dpart = 0.f;                           // D = <gX, Wx>, per-thread partials (rows tid, tid + 256, ..)
  for (int r = tid; r < R; r += NT) {
    if (r < k) {
      for (int c = 0; c < k; ++c) {
        const float gx = gm[r][c] - gm[c][r];
        gX[r * k + c] = gx;
        dpart = fmaf(gx, Wt[r * k + c], dpart);
      }
    } else {                                   // V (GM + GM^T) - 2 Gb inv^T
      float x[KM], g[KM];
#pragma unroll
      for (int q = 0; q < KM; ++q) {
        x[q] = q < k ? X[r * k + q] : 0.f;
        g[q] = q < k ? G[r * k + q] : 0.f;
      }
      for (int c = 0; c < k; ++c) {
        float v1 = 0.f, v2 = 0.f;
#pragma unroll
        for (int q = 0; q < KM; ++q)
          if (q < k) {
            v1 = fmaf(x[q], gm[q][c] + gm[c][q], v1);
            v2 = fmaf(g[q], iv[c][q], v2);
          }
        const float gx = v1 - 2.0f * v2;
        gX[r * k + c] = gx;
        dpart = fmaf(gx, Wt[r * k + c], dpart);
      }
    }
  }
  const float D = block_sum(dpart, red);       // (its barriers also publish gX)
  const float cw = al * D / (nrm * nrm * nrm);
  float* gWb = a.gW + (int64_t)b * a.cout * a.cin;
  for (int w = tid; w < R * k; w += NT) {       // coalesced over W's layout
    const int r = a.wide ? w % a.cin : w / a.cin, c = a.wide ? w / a.cin : w % a.cin;
    gWb[w] = s * gX[r * k + c] - cw * Wt[r * k + c];
  }
  if (tid == 0) a.galpha[b] = D / nrm;
}

size_t fwd_lds(int R, int k) { return ((size_t)R * k + NT + KM * (KM + 1)) * sizeof(float); }
size_t bwd_lds(int R, int k) { return ((size_t)4 * R * k + NT + 4 * KM * (KM + 1)) * sizeof(float); }

int check(int32_t batch, int32_t cout, int32_t cin) {
  const int k = cout < cin ? cout : cin, R = cout < cin ? cin : cout;
  if (batch < 0 || k < 1 || k > KM || (int64_t)R * k > FIODE_SMALL_CAYLEY_MAX_RK) return FIODE_EINVAL;
  return FIODE_OK;
}

SCArgs make_args(int32_t cout, int32_t cin, const float* W, const float* alpha) {
  SCArgs a{};
  a.prio = (g_fiode_prio_mask >> 2) & 1;
  a.cout = cout; a.cin = cin;
  a.wide = cin > cout;
  a.k = a.wide ? cout : cin;
  a.R = a.wide ? cin : cout;
  a.W = W; a.alpha = alpha;
  return a;
}

}  // namespace

extern "C" int fiode_small_cayley_forward(void* stream, int32_t batch, int32_t cout, int32_t cin, const float* W,
                                          const float* alpha, float* Q, float* inv, float* nrm) {
  int rc = check(batch, cout, cin);
  if (rc) return rc;
  if (batch == 0) return FIODE_OK;
  if (!W || !alpha || !Q || !inv || !nrm) return FIODE_EINVAL;
  SCArgs a = make_args(cout, cin, W, alpha);
  a.Q = Q; a.inv = inv; a.nrm = nrm;
  hipLaunchKernelGGL(k_small_cayley_fwd, dim3(batch), dim3(NT), fwd_lds(a.R, a.k), (hipStream_t)stream, a);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? FIODE_OK : FIODE_EHIP + (int)e;
}

extern "C" int fiode_small_cayley_backward(void* stream, int32_t batch, int32_t cout, int32_t cin, const float* W,
                                           const float* alpha, const float* nrm, const float* inv, const float* gQ,
                                           float* gW, float* galpha) {
  int rc = check(batch, cout, cin);
  if (rc) return rc;
  if (batch == 0) return FIODE_OK;
  if (!W || !alpha || !nrm || !inv || !gQ || !gW || !galpha) return FIODE_EINVAL;
  SCArgs a = make_args(cout, cin, W, alpha);
  a.nrm = const_cast<float*>(nrm); a.inv = const_cast<float*>(inv);
  a.gQ = gQ; a.gW = gW; a.galpha = galpha;
  hipLaunchKernelGGL(k_small_cayley_bwd, dim3(batch), dim3(NT), bwd_lds(a.R, a.k), (hipStream_t)stream, a);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? FIODE_OK : FIODE_EHIP + (int)e;
}
