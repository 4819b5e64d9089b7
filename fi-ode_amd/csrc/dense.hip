// Elementwise stages of the dense Cayley map Q = cayley(alpha W / ||W||) (gfx950): the
// CayleyLinears of the backbone (4096 -> 512 -> 512 -> 10) and of the dynamics (classification.py:
// 282-293 convert_cayley; fiode_amd/cayley.py _DenseCayleyFn).  The GEMMs of the map stay library
// GEMMs (hipBLASLt through torch.matmul) and the inverse is fiode_block_inverse / the batched
// Gauss-Jordan; everything between them -- ~30 PyTorch elementwise / copy / reduction kernels per
// map forward + backward -- is one kernel per stage here:
//
// X = s Wx (Wx = W, or W^T when cin > cout), s = alpha / ||W||, U = X[:k], V = X[k:], k = min(cout, cin),
// primes denote the unscaled blocks (U', V' of Wx):
//   prep    M = I + s (U' - U'^T) + s^2 G,                  G = V'^T V'           (GEMM)
//   finish  Q = [2 inv - I ; -2 s P] in W's orientation,     P = V' inv            (GEMM)
//   ginv    G_inv = 2 Gt - 2 s A,                            A = V'^T Gb           (GEMM)
//           (G_M' = inv^T G_inv inv^T by two GEMMs; G_M = -G_M')
//   h       gU = G_M - G_M^T, H = G_M + G_M^T
//   gv      gV = s P1 - 2 P2, D partials of <gX, Wx>,        P1 = V' H, P2 = Gb inv^T (GEMMs)
//   gw      dL/dW = s gX - alpha D / ||W||^3 W, dL/dalpha = D / ||W||  (fixed-order D sum)
// Every [R-k] x k block (P, P1, P2) and gX are passed in W's layout -- for a wide W (cin > cout)
// that is the transposed block, [k][R-k] (the host forms it with the GEMM operands swapped) --
// so every stage streams W-layout rows: no strided gathers over the 4096 x 512 matrices.
// with the matrices batched over a leading index (the dynamics' three 128 x 10 maps share one
// launch, per-matrix norms and alphas).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "common.h"
#include "fiode.h"

namespace {

constexpr int NT = 256;
constexpr int DPARTS = 256;     // D partial sums per matrix (grid.x of k_dense_gv)

struct DArgs {
  int cout, cin, k, R, wide;
  const float* W;       // [b][cout][cin]
  const float* alpha;   // [b]
  const float* nrm;     // [b]
};

__device__ __forceinline__ float wx(const DArgs& a, const float* Wb, int r, int c) {
  return a.wide ? Wb[(int64_t)c * a.cin + r] : Wb[(int64_t)r * a.cin + c];
}
__device__ __forceinline__ int64_t wpos(const DArgs& a, int r, int c) {   // X (r, c) -> W offset
  return a.wide ? (int64_t)c * a.cin + r : (int64_t)r * a.cin + c;
}

// Squared Frobenius norm partials of each W[b] (NPART per matrix, each a fixed-order sum over its
// block's float4 stride): the norm the prep kernel finishes in a fixed order -- one 2-8 MB streaming
// read over NPART x batch workgroups in place of torch's vector_norm reduction (~10 us on the dense
// maps' forward chain).
constexpr int NPART = 256;      // 8 float4 per thread of the 4096 x 512 map: two load round trips
__global__ void __launch_bounds__(NT) k_dense_sumsq(DArgs a, float* __restrict__ part, unsigned* __restrict__ clear,
                                                    int clear_words, int64_t clear_stride) {
  __shared__ float red[NT / 64];
  const int b = blockIdx.y;
  // (optional) zero the next kernel's hand-off flags: the one-launch inverse of this map
  // (fiode_dense_cayley_inverse) runs two launches later on the same stream
  if (clear && blockIdx.x == 0)
    for (int t = threadIdx.x; t < clear_words; t += NT) clear[(int64_t)b * clear_stride + t] = 0u;
  const int64_t n = (int64_t)a.cout * a.cin;
  const float* Wb = a.W + (int64_t)b * n;
  float acc = 0.f;
  if ((n & 3) == 0 && ((uintptr_t)Wb & 15u) == 0) {
    const f32x4* W4 = reinterpret_cast<const f32x4*>(Wb);
#pragma unroll 4
    for (int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x; i < (n >> 2); i += (int64_t)NPART * NT) {
      const f32x4 v = W4[i];
      acc = fmaf(v[0], v[0], acc);
      acc = fmaf(v[1], v[1], acc);
      acc = fmaf(v[2], v[2], acc);
      acc = fmaf(v[3], v[3], acc);
    }
  } else {
    for (int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x; i < n; i += (int64_t)NPART * NT) acc = fmaf(Wb[i], Wb[i], acc);
  }
  for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) part[b * NPART + blockIdx.x] = (red[0] + red[1]) + (red[2] + red[3]);
}

// ||W[b]|| from the NPART partials, the same fixed order in every workgroup (wave 0's lanes, then a
// butterfly); block 0 also writes it to nrm_out
__device__ __forceinline__ float dense_norm(const float* __restrict__ part, int b, float* nrm_out) {
  __shared__ float sn;
  if (threadIdx.x < 64) {
    const float* pb = part + b * NPART + 4 * threadIdx.x;
    float v = (pb[0] + pb[1]) + (pb[2] + pb[3]);
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    if (threadIdx.x == 0) {
      sn = sqrtf(v);
      if (nrm_out && blockIdx.x == 0) nrm_out[b] = sn;
    }
  }
  __syncthreads();
  return sn;
}
static_assert(NPART == 256, "dense_norm: four partials per lane of wave 0");

__global__ void __launch_bounds__(NT) k_dense_prep(DArgs a, const float* __restrict__ G, float* __restrict__ M,
                                                   const float* __restrict__ part, float* __restrict__ nrm_out) {
  const int b = blockIdx.y, k = a.k;
  const float* Wb = a.W + (int64_t)b * a.cout * a.cin;
  const float s = a.alpha[b] / (part ? dense_norm(part, b, nrm_out) : a.nrm[b]);
  for (int idx = blockIdx.x * NT + threadIdx.x; idx < k * k; idx += gridDim.x * NT) {
    const int i = idx / k, j = idx % k;
    float m = s * (wx(a, Wb, i, j) - wx(a, Wb, j, i));
    if (G) m = fmaf(s * s, G[(int64_t)b * k * k + idx], m);
    if (i == j) m += 1.0f;
    M[(int64_t)b * k * k + idx] = m;
  }
}

__global__ void __launch_bounds__(NT) k_dense_finish(DArgs a, const float* __restrict__ inv,
                                                     const float* __restrict__ P, float* __restrict__ Q) {
  const int b = blockIdx.y, k = a.k;
  const float s = a.alpha[b] / a.nrm[b];
  float* Qb = Q + (int64_t)b * a.cout * a.cin;
  // walk Q in its own (W) layout so the stores are coalesced
  for (int idx = blockIdx.x * NT + threadIdx.x; idx < a.cout * a.cin; idx += gridDim.x * NT) {
    const int o = idx / a.cin, c = idx % a.cin;
    const int r = a.wide ? c : o, j = a.wide ? o : c;      // X element (r, j)
    float q;
    if (r < k) {
      q = 2.0f * inv[((int64_t)b * k + r) * k + j];
      if (r == j) q -= 1.0f;
    } else {
      q = -2.0f * s * P[(int64_t)b * (a.R - k) * k + (a.wide ? (int64_t)j * (a.R - k) + (r - k) : (int64_t)(r - k) * k + j)];
    }
    Qb[idx] = q;
  }
}

// Wide maps (cin > cout): Q[o][c] = 2 inv[c][o] - [c == o] for c < k reads inv transposed, so Q is
// written in 32 x 32 tiles with the inv tile staged through LDS (both sides coalesced); the
// columns c >= k read P row-major along c.  grid (cin / 32, cout / 32, batch).
__global__ void __launch_bounds__(NT) k_dense_finish_wide(DArgs a, const float* __restrict__ inv,
                                                          const float* __restrict__ P, float* __restrict__ Q) {
  __shared__ float t[32][33];
  const int b = blockIdx.z, k = a.k, o0 = blockIdx.y * 32, c0 = blockIdx.x * 32;
  const int x = threadIdx.x & 31, y0 = threadIdx.x >> 5;        // 8 rows of 32 per pass
  float* Qb = Q + (int64_t)b * a.cout * a.cin;
  if (c0 < k) {                                                  // (k % 32 == 0: whole tile inside)
    const float* ib = inv + (int64_t)b * k * k;
#pragma unroll
    for (int y = y0; y < 32; y += 8) t[y][x] = ib[(int64_t)(c0 + y) * k + o0 + x];   // t[c][o]
    __syncthreads();
#pragma unroll
    for (int y = y0; y < 32; y += 8) {
      float q = 2.0f * t[x][y];                                  // inv[c0 + x][o0 + y]
      if (c0 + x == o0 + y) q -= 1.0f;
      Qb[(int64_t)(o0 + y) * a.cin + c0 + x] = q;
    }
  } else {
    const float s = a.alpha[b] / a.nrm[b];
    const int RV = a.R - k;
    const float* Pb = P + (int64_t)b * RV * k;
#pragma unroll
    for (int y = y0; y < 32; y += 8)
      Qb[(int64_t)(o0 + y) * a.cin + c0 + x] = -2.0f * s * Pb[(int64_t)(o0 + y) * RV + (c0 + x - k)];
  }
}

__global__ void __launch_bounds__(NT) k_dense_ginv(DArgs a, const float* __restrict__ Gq, const float* __restrict__ A,
                                                   float* __restrict__ Ginv) {
  const int b = blockIdx.y, k = a.k;
  const float s = a.alpha[b] / a.nrm[b];
  const float* Gb = Gq + (int64_t)b * a.cout * a.cin;
  for (int idx = blockIdx.x * NT + threadIdx.x; idx < k * k; idx += gridDim.x * NT) {
    const int i = idx / k, j = idx % k;
    float g = 2.0f * Gb[wpos(a, i, j)];
    if (A) g = fmaf(-2.0f * s, A[(int64_t)b * k * k + idx], g);
    Ginv[(int64_t)b * k * k + idx] = g;
  }
}

// GMn = -G_M: gU = G_M - G_M^T -> gX (W layout); H = G_M + G_M^T
__global__ void __launch_bounds__(NT) k_dense_h(DArgs a, const float* __restrict__ GMn, float* __restrict__ gX,
                                                float* __restrict__ H) {
  const int b = blockIdx.y, k = a.k;
  const float* Gm = GMn + (int64_t)b * k * k;
  for (int idx = blockIdx.x * NT + threadIdx.x; idx < k * k; idx += gridDim.x * NT) {
    const int i = idx / k, j = idx % k;
    const float g = -Gm[idx], gt = -Gm[(int64_t)j * k + i];
    gX[(int64_t)b * a.cout * a.cin + wpos(a, i, j)] = g - gt;
    H[(int64_t)b * k * k + idx] = g + gt;
  }
}

// gV = s P1 - 2 P2 -> gX (W layout); D partials of sum gX * W over the whole matrix
__global__ void __launch_bounds__(NT) k_dense_gv(DArgs a, const float* __restrict__ P1, const float* __restrict__ P2,
                                                 float* __restrict__ gX, float* __restrict__ dpart) {
  __shared__ float red[NT / 64];
  const int b = blockIdx.y, k = a.k, n = a.cout * a.cin, RV = a.R - k;
  const float s = a.alpha[b] / a.nrm[b];
  const float* Wb = a.W + (int64_t)b * n;
  const float* P1b = P1 ? P1 + (int64_t)b * RV * k : nullptr;
  const float* P2b = P2 ? P2 + (int64_t)b * RV * k : nullptr;
  float* gXb = gX + (int64_t)b * n;
  float d = 0.f;
#pragma unroll 4
  for (int idx = blockIdx.x * NT + threadIdx.x; idx < n; idx += DPARTS * NT) {
    const int o = idx / a.cin, c = idx % a.cin;
    const int r = a.wide ? c : o;
    float g;
    if (r < k) {
      g = gXb[idx];
    } else {                                  // P blocks in W layout: wide [k][RV] (o, c-k), tall [RV][k] (o-k, c)
      const int64_t pi = a.wide ? (int64_t)o * RV + (c - k) : (int64_t)(o - k) * k + c;
      g = s * P1b[pi] - 2.0f * P2b[pi];
      gXb[idx] = g;
    }
    d = fmaf(g, Wb[idx], d);
  }
  for (int o = 32; o > 0; o >>= 1) d += __shfl_xor(d, o);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = d;
  __syncthreads();
  if (threadIdx.x == 0) {
    float t = 0.f;
    for (int q = 0; q < NT / 64; ++q) t += red[q];
    dpart[b * DPARTS + blockIdx.x] = t;
  }
}

// k_dense_gv with float4 rows (cin % 4 == 0, k % 4 == 0): block x walks rows x, x + DPARTS, ...
// and a row's float4 columns in order -- no per-element division, every access 16 bytes wide
__global__ void __launch_bounds__(NT) k_dense_gv4(DArgs a, const float* __restrict__ P1, const float* __restrict__ P2,
                                                  float* __restrict__ gX, float* __restrict__ dpart) {
  __shared__ float red[NT / 64];
  const int b = blockIdx.y, k = a.k, n = a.cout * a.cin, RV = a.R - k, c4n = a.cin >> 2;
  const float s = a.alpha[b] / a.nrm[b];
  const float* Wb = a.W + (int64_t)b * n;
  const float* P1b = P1 ? P1 + (int64_t)b * RV * k : nullptr;
  const float* P2b = P2 ? P2 + (int64_t)b * RV * k : nullptr;
  float* gXb = gX + (int64_t)b * n;
  float d = 0.f;
  for (int o = blockIdx.x; o < a.cout; o += DPARTS) {
    for (int c4 = threadIdx.x; c4 < c4n; c4 += NT) {
      const int c = 4 * c4;
      const int r = a.wide ? c : o;                 // the 4 columns share r < k or r >= k
      const int64_t idx = (int64_t)o * a.cin + c;
      f32x4 g;
      if (r < k) {
        g = *reinterpret_cast<const f32x4*>(gXb + idx);
      } else {
        const int64_t pi = a.wide ? (int64_t)o * RV + (c - k) : (int64_t)(o - k) * k + c;
        const f32x4 p1 = *reinterpret_cast<const f32x4*>(P1b + pi), p2 = *reinterpret_cast<const f32x4*>(P2b + pi);
#pragma unroll
        for (int e = 0; e < 4; ++e) g[e] = s * p1[e] - 2.0f * p2[e];
        *reinterpret_cast<f32x4*>(gXb + idx) = g;
      }
      const f32x4 w = *reinterpret_cast<const f32x4*>(Wb + idx);
#pragma unroll
      for (int e = 0; e < 4; ++e) d = fmaf(g[e], w[e], d);
    }
  }
  for (int o = 32; o > 0; o >>= 1) d += __shfl_xor(d, o);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = d;
  __syncthreads();
  if (threadIdx.x == 0) {
    float t = 0.f;
    for (int q = 0; q < NT / 64; ++q) t += red[q];
    dpart[b * DPARTS + blockIdx.x] = t;
  }
}

__global__ void __launch_bounds__(NT) k_dense_gw(DArgs a, const float* __restrict__ gX, const float* __restrict__ dpart,
                                                 float* __restrict__ gW, float* __restrict__ galpha, int vec) {
  __shared__ float sD;
  const int b = blockIdx.y;
  if (threadIdx.x < 64) {                     // fixed-order sum of the D partials
    float v = 0.f;
#pragma unroll
    for (int q = threadIdx.x; q < DPARTS; q += 64) v += dpart[b * DPARTS + q];
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    if (threadIdx.x == 0) sD = v;
  }
  __syncthreads();
  const float D = sD, n = a.nrm[b], al = a.alpha[b];
  const float s = al / n, cw = al * D / (n * n * n);
  if (blockIdx.x == 0 && threadIdx.x == 0) galpha[b] = D / n;
  const float* Wb = a.W + (int64_t)b * a.cout * a.cin;
  const float* gXb = gX + (int64_t)b * a.cout * a.cin;
  float* gWb = gW + (int64_t)b * a.cout * a.cin;
  const int ne = a.cout * a.cin;
  if (vec) {                                  // float4: ne % 4 == 0 and 16-byte aligned matrices (host check)
    for (int i4 = blockIdx.x * NT + threadIdx.x; i4 < (ne >> 2); i4 += gridDim.x * NT) {
      const f32x4 g = reinterpret_cast<const f32x4*>(gXb)[i4], w = reinterpret_cast<const f32x4*>(Wb)[i4];
      f32x4 o;
#pragma unroll
      for (int e = 0; e < 4; ++e) o[e] = s * g[e] - cw * w[e];
      reinterpret_cast<f32x4*>(gWb)[i4] = o;
    }
    return;
  }
  for (int idx = blockIdx.x * NT + threadIdx.x; idx < ne; idx += gridDim.x * NT)
    gWb[idx] = s * gXb[idx] - cw * Wb[idx];
}

// C[b] = op(A[b]) op(B[b]) for n x n matrices (n % 64 == 0), op = transpose when TA / TB: the
// dense maps' backward chain GMn = inv^T (Ginv inv^T), two dependent 512^3 products that the
// library runs as 16 workgroups of 128 x 128 tiles (~14 us each).  Here 32 x 32 output tiles
// (256 workgroups at n = 512), the 4 waves split K (n / 4 each) on v_mfma_f32_16x16x4_f32 with
// operands straight from L2 (16-byte loads along k where the layout allows, 64-byte rows
// otherwise), the 4 partials summed in LDS in a fixed order (tools/probes/sgemm_probe.hip).
template <bool TA, bool TB>
__global__ void __launch_bounds__(256) k_dense_gemm(int n, const float* __restrict__ A, const float* __restrict__ B,
                                                    float* __restrict__ C) {
  __shared__ float red[4][32][33];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int i = lane & 15, q = lane >> 4;
  const int tm = blockIdx.y * 32, tn = blockIdx.x * 32;
  const int64_t mo = (int64_t)blockIdx.z * n * n;
  A += mo;
  B += mo;
  C += mo;
  const int ks = n >> 2, k0 = w * ks;
  f32x4 acc[2][2];
#pragma unroll
  for (int x = 0; x < 2; ++x)
#pragma unroll
    for (int y = 0; y < 2; ++y) acc[x][y] = f32x4{0.f, 0.f, 0.f, 0.f};
  // chunk of 16 k: step s uses k = kb + s, kb = k0 + 16 kc + 4 q at lane q
  for (int kc = 0; kc < ks / 16; ++kc) {
    const int kb = k0 + 16 * kc + 4 * q;
    f32x4 av[2], bv[2];
#pragma unroll
    for (int x = 0; x < 2; ++x) {
      const int m = tm + 16 * x + i;
      if (TA) {
#pragma unroll
        for (int s = 0; s < 4; ++s) av[x][s] = A[(int64_t)(kb + s) * n + m];
      } else {
        av[x] = *reinterpret_cast<const f32x4*>(A + (int64_t)m * n + kb);
      }
    }
#pragma unroll
    for (int y = 0; y < 2; ++y) {
      const int c = tn + 16 * y + i;
      if (TB) {
        bv[y] = *reinterpret_cast<const f32x4*>(B + (int64_t)c * n + kb);
      } else {
#pragma unroll
        for (int s = 0; s < 4; ++s) bv[y][s] = B[(int64_t)(kb + s) * n + c];
      }
    }
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int x = 0; x < 2; ++x)
#pragma unroll
        for (int y = 0; y < 2; ++y)
          acc[x][y] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[x][s], bv[y][s], acc[x][y], 0, 0, 0);
  }
#pragma unroll
  for (int x = 0; x < 2; ++x)
#pragma unroll
    for (int y = 0; y < 2; ++y)
#pragma unroll
      for (int r = 0; r < 4; ++r) red[w][16 * x + 4 * q + r][16 * y + i] = acc[x][y][r];   // D[4q + r][i]
  __syncthreads();
  for (int e = threadIdx.x; e < 32 * 32; e += 256) {
    const int r = e >> 5, c = e & 31;
    C[(int64_t)(tm + r) * n + tn + c] = ((red[0][r][c] + red[1][r][c]) + red[2][r][c]) + red[3][r][c];
  }
}

int mk(const fiode_dense_config* cfg, DArgs& a, int& batch) {
  if (!cfg || cfg->batch < 1 || cfg->cout < 1 || cfg->cin < 1) return FIODE_EINVAL;
  a = DArgs{};
  a.cout = cfg->cout;
  a.cin = cfg->cin;
  a.wide = a.cin > a.cout;
  a.k = a.wide ? a.cout : a.cin;
  a.R = a.wide ? a.cin : a.cout;
  batch = cfg->batch;
  return FIODE_OK;
}

dim3 grid_for(int64_t n, int batch) {
  int64_t g = (n + NT - 1) / NT;
  if (g > 1024) g = 1024;
  return dim3((unsigned)g, (unsigned)batch);
}

#define DENSE_RET()                                            \
  do {                                                         \
    const hipError_t e = hipGetLastError();                    \
    return e == hipSuccess ? FIODE_OK : FIODE_EHIP + (int)e;   \
  } while (0)

}  // namespace

extern "C" int fiode_dense_cayley_prep(void* stream, const fiode_dense_config* cfg, const float* W, const float* alpha,
                                       const float* nrm, const float* G, float* M) {
  DArgs a;
  int batch, rc = mk(cfg, a, batch);
  if (rc) return rc;
  if (!W || !alpha || !nrm || !M || (a.R > a.k && !G)) return FIODE_EINVAL;
  a.W = W;
  a.alpha = alpha;
  a.nrm = nrm;
  hipLaunchKernelGGL(k_dense_prep, grid_for((int64_t)a.k * a.k, batch), dim3(NT), 0, (hipStream_t)stream, a,
                     a.R > a.k ? G : nullptr, M, (const float*)nullptr, (float*)nullptr);
  DENSE_RET();
}

extern "C" size_t fiode_dense_norm_workspace_bytes(const fiode_dense_config* cfg) {
  return cfg && cfg->batch > 0 ? (size_t)cfg->batch * NPART * sizeof(float) : 0;
}

extern "C" int fiode_dense_norm_partials(void* stream, const fiode_dense_config* cfg, const float* W, void* workspace,
                                         size_t workspace_bytes) {
  DArgs a;
  int batch, rc = mk(cfg, a, batch);
  if (rc) return rc;
  if (!W || !workspace) return FIODE_EINVAL;
  if (workspace_bytes < fiode_dense_norm_workspace_bytes(cfg)) return FIODE_EWORKSPACE;
  a.W = W;
  hipLaunchKernelGGL(k_dense_sumsq, dim3(NPART, batch), dim3(NT), 0, (hipStream_t)stream, a, (float*)workspace,
                     (unsigned*)nullptr, 0, (int64_t)0);
  DENSE_RET();
}

extern "C" int fiode_dense_norm_partials_clear(void* stream, const fiode_dense_config* cfg, const float* W,
                                               void* workspace, size_t workspace_bytes, void* clear,
                                               size_t clear_words, size_t clear_stride_bytes) {
  DArgs a;
  int batch, rc = mk(cfg, a, batch);
  if (rc) return rc;
  if (!W || !workspace || (clear_words && !clear) || clear_words > (1u << 20) || clear_stride_bytes % 4)
    return FIODE_EINVAL;
  if (workspace_bytes < fiode_dense_norm_workspace_bytes(cfg)) return FIODE_EWORKSPACE;
  a.W = W;
  hipLaunchKernelGGL(k_dense_sumsq, dim3(NPART, batch), dim3(NT), 0, (hipStream_t)stream, a, (float*)workspace,
                     clear_words ? (unsigned*)clear : (unsigned*)nullptr, (int)clear_words,
                     (int64_t)(clear_stride_bytes / 4));
  DENSE_RET();
}

extern "C" int fiode_dense_cayley_prep_normed(void* stream, const fiode_dense_config* cfg, const float* W,
                                              const float* alpha, const void* workspace, float* nrm_out,
                                              const float* G, float* M) {
  DArgs a;
  int batch, rc = mk(cfg, a, batch);
  if (rc) return rc;
  if (!W || !alpha || !workspace || !nrm_out || !M || (a.R > a.k && !G)) return FIODE_EINVAL;
  a.W = W;
  a.alpha = alpha;
  a.nrm = nullptr;
  hipLaunchKernelGGL(k_dense_prep, grid_for((int64_t)a.k * a.k, batch), dim3(NT), 0, (hipStream_t)stream, a,
                     a.R > a.k ? G : nullptr, M, (const float*)workspace, nrm_out);
  DENSE_RET();
}

extern "C" int fiode_dense_cayley_finish(void* stream, const fiode_dense_config* cfg, const float* alpha,
                                         const float* nrm, const float* inv, const float* P, float* Q) {
  DArgs a;
  int batch, rc = mk(cfg, a, batch);
  if (rc) return rc;
  if (!alpha || !nrm || !inv || !Q || (a.R > a.k && !P)) return FIODE_EINVAL;
  a.alpha = alpha;
  a.nrm = nrm;
  if (a.wide && a.cout % 32 == 0 && a.cin % 32 == 0)
    hipLaunchKernelGGL(k_dense_finish_wide, dim3(a.cin / 32, a.cout / 32, batch), dim3(NT), 0, (hipStream_t)stream, a,
                       inv, P, Q);
  else
    hipLaunchKernelGGL(k_dense_finish, grid_for((int64_t)a.cout * a.cin, batch), dim3(NT), 0, (hipStream_t)stream, a,
                       inv, P, Q);
  DENSE_RET();
}

extern "C" int fiode_dense_cayley_ginv(void* stream, const fiode_dense_config* cfg, const float* alpha,
                                       const float* nrm, const float* gQ, const float* A, float* Ginv) {
  DArgs a;
  int batch, rc = mk(cfg, a, batch);
  if (rc) return rc;
  if (!alpha || !nrm || !gQ || !Ginv || (a.R > a.k && !A)) return FIODE_EINVAL;
  a.alpha = alpha;
  a.nrm = nrm;
  hipLaunchKernelGGL(k_dense_ginv, grid_for((int64_t)a.k * a.k, batch), dim3(NT), 0, (hipStream_t)stream, a, gQ,
                     a.R > a.k ? A : nullptr, Ginv);
  DENSE_RET();
}

extern "C" int fiode_dense_cayley_h(void* stream, const fiode_dense_config* cfg, const float* GMn, float* gX,
                                    float* H) {
  DArgs a;
  int batch, rc = mk(cfg, a, batch);
  if (rc) return rc;
  if (!GMn || !gX || !H) return FIODE_EINVAL;
  hipLaunchKernelGGL(k_dense_h, grid_for((int64_t)a.k * a.k, batch), dim3(NT), 0, (hipStream_t)stream, a, GMn, gX, H);
  DENSE_RET();
}

extern "C" size_t fiode_dense_cayley_workspace_bytes(const fiode_dense_config* cfg) {
  return cfg && cfg->batch > 0 ? (size_t)cfg->batch * DPARTS * sizeof(float) : 0;
}

extern "C" int fiode_dense_cayley_grad(void* stream, const fiode_dense_config* cfg, const float* W, const float* alpha,
                                       const float* nrm, const float* P1, const float* P2, float* gX, float* gW,
                                       float* galpha, void* workspace, size_t workspace_bytes) {
  DArgs a;
  int batch, rc = mk(cfg, a, batch);
  if (rc) return rc;
  if (!W || !alpha || !nrm || !gX || !gW || !galpha || !workspace || (a.R > a.k && (!P1 || !P2)))
    return FIODE_EINVAL;
  if (workspace_bytes < fiode_dense_cayley_workspace_bytes(cfg)) return FIODE_EWORKSPACE;
  a.W = W;
  a.alpha = alpha;
  a.nrm = nrm;
  hipStream_t st = (hipStream_t)stream;
  float* dpart = (float*)workspace;
  auto al16 = [](const void* q) { return ((uintptr_t)q & 15u) == 0; };
  const bool vec = a.cin % 4 == 0 && a.k % 4 == 0 && al16(W) && al16(gX) && al16(gW) && (!P1 || al16(P1)) &&
                   (!P2 || al16(P2));
  if (vec)
    hipLaunchKernelGGL(k_dense_gv4, dim3(DPARTS, batch), dim3(NT), 0, st, a, P1, P2, gX, dpart);
  else
    hipLaunchKernelGGL(k_dense_gv, dim3(DPARTS, batch), dim3(NT), 0, st, a, P1, P2, gX, dpart);
  hipLaunchKernelGGL(k_dense_gw, grid_for((int64_t)a.cout * a.cin, batch), dim3(NT), 0, st, a, (const float*)gX, dpart,
                     gW, galpha, vec ? 1 : 0);
  DENSE_RET();
}

extern "C" int fiode_dense_gemm(void* stream, int32_t batch, int32_t n, int32_t trans_a, int32_t trans_b,
                                const float* A, const float* B, float* C) {
  if (batch < 1 || batch > 65535 || n < 64 || !A || !B || !C) return FIODE_EINVAL;
  if (n % 64 != 0) return FIODE_ESHAPE;
  if ((((uintptr_t)A | (uintptr_t)B) & 15u) != 0) return FIODE_ESHAPE;   // 16-byte operand loads
  const dim3 grid((unsigned)(n / 32), (unsigned)(n / 32), (unsigned)batch);
  hipStream_t st = (hipStream_t)stream;
  if (trans_a && trans_b) hipLaunchKernelGGL((k_dense_gemm<true, true>), grid, dim3(256), 0, st, n, A, B, C);
  else if (trans_a) hipLaunchKernelGGL((k_dense_gemm<true, false>), grid, dim3(256), 0, st, n, A, B, C);
  else if (trans_b) hipLaunchKernelGGL((k_dense_gemm<false, true>), grid, dim3(256), 0, st, n, A, B, C);
  else hipLaunchKernelGGL((k_dense_gemm<false, false>), grid, dim3(256), 0, st, n, A, B, C);
  DENSE_RET();
}

