// Lipschitz certification on the decision-boundary grid (BASELINE config 4), gfx950.
//
// Replaces robustness/eval_utils.py:31-69 (sample_decision_boundary + get_grid_for_label: the
// grid, G(10,40) = 41,320,837 rows per label) and the per-image body of certify_lipschitz.py:104-143:
//   for each batch of grid rows:  f = eval_dot_light(eta, static)       (QP exit global per batch)
//                                 h_vdot = max_{runner-up} f - f_label   (certify_lipschitz.py:37-42)
//                                 violation = h_vdot + sqrt2*Lf_eta*dist + kappa
//   certified <=> max violation < 0.
// The grid is built once on the device in the reference's exact row order (unranking the
// construction's case split, so every batch holds the same rows as the reference's slices), kept
// resident in HBM as uint8 counts v (eta = v/T); the label's column swap is applied on the fly --
// no per-batch host->device grid copies.
#include "common.h"
#include "tile.h"
#include "../../include/fiode.h"

namespace {
using namespace fiode_tile;

constexpr int MAXN = 16;
constexpr int MAXT = 64;

struct CountTable {
  uint32_t f[MAXT + 1][MAXN + 1];
  uint32_t comb[MAXN + 1][MAXN + 1];
};

// Row r of the decision-boundary grid (sum T, dim n, coordinate 0 = max of the others), in the
// construction order of eval_utils.py:39-58: blocks by the number l of zero coordinates among
// 1..k-1, then the lexicographic set c of non-zero positions, then the sub-block's row order.
__device__ void db_unrank(uint32_t r, int n, int T, const CountTable& t, uint8_t* out) {
  int idx[MAXN];
  for (int p = 0; p < n; ++p) idx[p] = p;
  int add = 0, j = T, k = n;
  while (true) {
    if (j == 0) {
      for (int p = 0; p < k; ++p) out[idx[p]] = (uint8_t)add;
      return;
    }
    if (k == 2) {
      out[idx[0]] = out[idx[1]] = (uint8_t)(add + j / 2);
      return;
    }
    int l = 0;
    uint32_t sub = 1;
    for (l = 0; l < k - 1; ++l) {
      if (j - k + l < 0) continue;
      sub = t.f[j - k + l][k - l];
      const uint32_t blk = t.comb[k - 1][k - l - 1] * sub;
      if (r < blk) break;
      r -= blk;
    }
    const int m = k - l - 1;
    uint32_t ci = r / sub;
    r -= ci * sub;
    int keep[MAXN];
    keep[0] = 0;
    int nk = 1;
    for (int e = 1; nk < m + 1; ++e) {        // lexicographic combination of m positions from 1..k-1
      const uint32_t cnt = t.comb[k - 1 - e][m - nk];
      if (ci < cnt) keep[nk++] = e;
      else ci -= cnt;
    }
    int q = 0;
    for (int p = 0; p < k; ++p) {
      if (q < nk && keep[q] == p) ++q;
      else out[idx[p]] = (uint8_t)add;
    }
    for (int p = 0; p < nk; ++p) idx[p] = idx[keep[p]];
    add += 1;
    j = j - k + l;
    k = k - l;
  }
}

__global__ __launch_bounds__(256) void k_cert_grid(CountTable t, int n, int T, uint32_t G, uint8_t* grid) {
  const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= G) return;
  uint8_t v[MAXN];
  db_unrank(r, n, T, t, v);
  for (int p = 0; p < n; ++p) grid[(size_t)r * n + p] = v[p];
}

struct CertArgs {
  uint32_t G, ebs;
  int nb, label, T;
  float eps_g, dist, kappa, sqrt_n, sa, sqrt2;
  float etab[MAXT + 1];   // float32(v / T) for the counts v = 0..T (double quotient, host-rounded)
  DynScalars d;
  const float* x_feat;
  const uint8_t* grid;
  const float *Q1, *b1, *Qx, *bx, *Q2, *b2, *Q3, *b3;
  float* u;          // [M]
  float* ft;         // [G][C]
  uint32_t* words;   // [nb] QP exit AND words
  uint32_t* keys;    // [nb][2] order-preserving max keys
  float* out;        // [nb][2]
  int32_t* exit_iters;
};

__device__ __forceinline__ uint32_t fkey(float x) {
  const uint32_t b = __float_as_uint(x);
  return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}
__device__ __forceinline__ float unkey(uint32_t k) {
  return __uint_as_float((k & 0x80000000u) ? (k & 0x7FFFFFFFu) : ~k);
}
// batch of row r (certify_lipschitz.py:100-102, 115-119): b*ebs.., the last batch takes the tail
__device__ __forceinline__ int batch_of(const CertArgs& a, uint32_t r) {
  const uint32_t b = r / a.ebs;
  return (int)(b < (uint32_t)(a.nb - 1) ? b : (uint32_t)(a.nb - 1));
}

// eta row: float32(v / T) with the label's column swapped with column 0 (eval_utils.py:64-69);
// the T + 1 possible values come from a table in LDS (stage_etab) -- the per-element float64
// division they replace was ~14 f64 instructions per value
__device__ __forceinline__ void stage_etab(const CertArgs& a, float* tab) {
  for (int v = threadIdx.x; v <= a.T; v += blockDim.x) tab[v] = a.etab[v];
}
__device__ __forceinline__ void eta_row(const CertArgs& a, const float* tab, uint32_t r, float (&h)[C]) {
  const uint8_t* g = a.grid + (size_t)r * C;
  float v[C];
#pragma unroll
  for (int j = 0; j < C; ++j) v[j] = tab[g[j]];
  float v0 = v[0], vl = v[0];
#pragma unroll
  for (int j = 0; j < C; ++j) vl = (j == a.label) ? v[j] : vl;
#pragma unroll
  for (int j = 0; j < C; ++j) h[j] = (j == 0) ? vl : ((j == a.label) ? v0 : v[j]);
}

__global__ __launch_bounds__(256) void k_cert_prep(CertArgs a) {
  const int i = threadIdx.x;
  if (i < FIODE_M) {
    float s = 0.f;
#pragma unroll
    for (int c = 0; c < FIODE_X; ++c) s = __fmaf_rn(a.Qx[i * FIODE_X + c], a.x_feat[c], s);
    a.u[i] = (s + a.bx[i]) + a.b1[i];
  }
  for (int b = i; b < a.nb; b += blockDim.x) {
    a.words[b] = 0xFFFFFFFFu;
    a.keys[2 * b] = 0u;
    a.keys[2 * b + 1] = 0u;
  }
}

// Batch-wise reductions are accumulated in registers and flushed to the per-batch words only when
// a wave moves to another batch (and at its end): one wave-level atomic per (wave, batch visited),
// not one per tile or per 64 rows -- hundreds of thousands of same-word atomics serialise at the
// memory-side atomic unit (~88 ops/us per word, MI355X_MICROARCH.md), which was most of
// k_cert_final's 13 ms and a share of k_cert_fwd's time.
// AND `conv` into the exit word of each lane's batch (a 32-row tile spans at most a few batches)
__device__ __forceinline__ void and_by_batch(const CertArgs& a, int batch, bool valid, uint32_t conv) {
  bool pending = valid;
  while (__any(pending)) {
    const unsigned long long m = __ballot(pending);
    const int leader = __ffsll((long long)m) - 1;
    const int b0 = __shfl(batch, leader, 64);
    const bool mine = pending && batch == b0;
    const uint32_t w = wave_and(mine ? conv : 0xFFFFFFFFu);
    if ((int)(threadIdx.x & 63) == leader) atomicAnd(a.words + b0, w);
    pending = pending && !mine;
  }
}

// Two workgroups per CU (LDS: the Q2 image + Q3's C rows, 72.9 KB each; <= 256 registers): the
// two waves of a SIMD run many tile pairs each and drift apart, so one wave's QP / barrier VALU
// work overlaps the other's MFMAs (one resident workgroup per CU left the matrix pipe idle during
// them).  A wave takes two consecutive 32-row tiles: both MLPs (dropout off: plain relu), then one
// QP per lane -- lanes 0..31 the first tile's rows, 32..63 the second's (a 32x32 accumulator tile
// leaves each row's outputs on both lane halves, so a wave per tile ran every row's QP twice).
__global__ __launch_bounds__(256, 2) void k_cert_fwd(CertArgs a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* Q2s = smem;
  float* Q3s = smem + M * LDQ;
  float* tab = smem + (M + C) * LDQ;
  load_weight_images(a.Q2, a.Q3, Q2s, Q3s, C);
  stage_etab(a, tab);
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, half = lane >> 5, col = lane & 31;
  float q1[4][5];
#pragma unroll
  for (int mb = 0; mb < 4; ++mb)
#pragma unroll
    for (int s = 0; s < 5; ++s) q1[mb][s] = a.Q1[(32 * mb + col) * C + 2 * s + half];
  const uint32_t kw[4] = {0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu};
  const uint32_t npairs = (a.G + 63) / 64;
  int cur_b = -1;                    // the batch whose AND this wave accumulates (wave-uniform)
  uint32_t cur_and = 0xFFFFFFFFu;
  for (uint32_t pair = blockIdx.x * FIODE_WAVES + wave; pair < npairs; pair += gridDim.x * FIODE_WAVES) {
    float h[C] = {}, ft[C] = {};
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const uint32_t rt = pair * 64 + 32 * t + col;          // row of tile t on this lane (both halves)
      const uint32_t rrt = rt < a.G ? rt : a.G - 1;
      float ht[C];
      eta_row(a, tab, rrt, ht);
      f32x16 z1[4], z2[4];
      const f32x16 z3 = mlp_tile<false>(Q2s, Q3s, q1, a.u, a.b2, a.b3, ht, kw, kw, 1.0f, col, half, z1, z2);
      float ftt[C];
      gather_ft(z3, half, ftt);
#pragma unroll
      for (int j = 0; j < C; ++j) {
        h[j] = (t == half) ? ht[j] : h[j];
        ft[j] = (t == half) ? ftt[j] : ft[j];
      }
    }
    const uint32_t row = pair * 64 + lane;                     // this lane's row in the QP phase
    const bool valid = row < a.G;
    const uint32_t rr = valid ? row : a.G - 1;
    float lower[C], nominal[C], sig[C], span[C], v[C], mu;
    barrier_nominal(a.d, h, ft, lower, nominal, sig, span);
    const uint32_t conv = qp_bisect(lower, nominal, a.d.max_iter - 1, a.d.tol, v, mu);
    const int bt = batch_of(a, rr);
    const int b_first = __shfl(bt, 0, 64), b_last = __shfl(bt, 63, 64);
    if (b_first == b_last) {          // the whole pair in one batch (all but a few boundary pairs)
      if (b_first != cur_b) {
        if (cur_b >= 0 && (threadIdx.x & 63) == 0) atomicAnd(a.words + cur_b, cur_and);
        cur_b = b_first;
        cur_and = 0xFFFFFFFFu;
      }
      cur_and &= wave_and(valid ? conv : 0xFFFFFFFFu);
    } else {
      and_by_batch(a, bt, valid, conv);
    }
    if (valid) store_row10(a.ft + (size_t)row * C, ft);
  }
  if (cur_b >= 0 && (threadIdx.x & 63) == 0) atomicAnd(a.words + cur_b, cur_and);
}

// one row: the violation and violation_larger_T of grid row rr (certify_lipschitz.py:120-136)
__device__ __forceinline__ void cert_row(const CertArgs& a, const float* tab, uint32_t rr, int b, float& viol,
                                         float& violT) {
  float h[C], ft[C], lower[C], nominal[C], sig[C], span[C], v[C], mu;
  eta_row(a, tab, rr, h);
  load_row10(a.ft + (size_t)rr * C, ft);
  barrier_nominal(a.d, h, ft, lower, nominal, sig, span);
  qp_bisect(lower, nominal, qp_exit_iter(a.words[b], a.d.max_iter), a.d.tol, v, mu);
  // runner-up set: eta == max eta, label excluded (certify_lipschitz.py:126-128)
  float mx = h[0];
#pragma unroll
  for (int j = 1; j < C; ++j) mx = fmaxf(mx, h[j]);
  float fw = -INFINITY, fy = 0.f;
#pragma unroll
  for (int j = 0; j < C; ++j) {
    if (j == a.label) fy = v[j];
    else if (h[j] == mx) fw = fmaxf(fw, v[j]);
  }
  const float hv = -fy + fw;
  const float ub = mx + a.eps_g;
  const float lf = a.sqrt_n * (a.sa * expf(a.d.sigma_1 * ub)) + 1.0f;
  const float perturb = (a.sqrt2 * lf) * a.dist;
  viol = (hv + perturb) + a.kappa;
  violT = hv + a.kappa;
}

// per-batch max of one wave's lanes (several batches possible) -> one atomic per (wave, batch)
__device__ __forceinline__ void max_by_batch(const CertArgs& a, int b, bool valid, float viol, float violT) {
  bool pending = valid;
  while (__any(pending)) {
    const unsigned long long m = __ballot(pending);
    const int leader = __ffsll((long long)m) - 1;
    const int b0 = __shfl(b, leader, 64);
    const bool mine = pending && b == b0;
    float m0 = mine ? viol : -INFINITY, m1 = mine ? violT : -INFINITY;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      m0 = fmaxf(m0, __shfl_xor(m0, o, 64));
      m1 = fmaxf(m1, __shfl_xor(m1, o, 64));
    }
    if ((int)(threadIdx.x & 63) == leader) {
      atomicMax(a.keys + 2 * b0, fkey(m0));
      atomicMax(a.keys + 2 * b0 + 1, fkey(m1));
    }
    pending = pending && !mine;
  }
}

// Persistent grid-stride loop over the rows (one row per lane per pass); each lane keeps the
// running maxima of the batch its wave is in, flushed when the wave moves on (see and_by_batch).
__global__ __launch_bounds__(256) void k_cert_final(CertArgs a) {
  __shared__ float tab[MAXT + 1];
  stage_etab(a, tab);
  __syncthreads();
  int cur_b = -1;
  float acc0 = -INFINITY, acc1 = -INFINITY;
  auto flush = [&]() {
    if (cur_b < 0) return;
    float m0 = acc0, m1 = acc1;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      m0 = fmaxf(m0, __shfl_xor(m0, o, 64));
      m1 = fmaxf(m1, __shfl_xor(m1, o, 64));
    }
    if ((threadIdx.x & 63) == 0) {
      atomicMax(a.keys + 2 * cur_b, fkey(m0));
      atomicMax(a.keys + 2 * cur_b + 1, fkey(m1));
    }
  };
  const uint32_t stride = gridDim.x * blockDim.x;
  const uint32_t nrounds = (a.G + stride - 1) / stride;
  for (uint32_t k = 0; k < nrounds; ++k) {                 // wave-uniform trip count
    const uint32_t r = k * stride + blockIdx.x * blockDim.x + threadIdx.x;
    const bool valid = r < a.G;
    const uint32_t rr = valid ? r : a.G - 1;
    const int b = batch_of(a, rr);
    float viol, violT;
    cert_row(a, tab, rr, b, viol, violT);
    const int b_first = __shfl(b, 0, 64), b_last = __shfl(b, 63, 64);
    if (b_first == b_last && __all(valid)) {
      if (b_first != cur_b) {
        flush();
        cur_b = b_first;
        acc0 = acc1 = -INFINITY;
      }
      acc0 = fmaxf(acc0, viol);
      acc1 = fmaxf(acc1, violT);
    } else {
      max_by_batch(a, b, valid, viol, violT);
    }
  }
  flush();
}

__global__ void k_cert_decode(CertArgs a) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= a.nb) return;
  a.out[2 * b] = unkey(a.keys[2 * b]);
  a.out[2 * b + 1] = unkey(a.keys[2 * b + 1]);
  if (a.exit_iters) a.exit_iters[b] = qp_exit_iter(a.words[b], a.d.max_iter);
}

bool count_table(int n, int T, CountTable& t, uint64_t& G) {
  if (n < 2 || n > MAXN || T < 0 || T > MAXT) return false;
  uint64_t f[MAXT + 1][MAXN + 1] = {};
  uint64_t comb[MAXN + 1][MAXN + 1] = {};
  for (int a = 0; a <= MAXN; ++a) {
    comb[a][0] = 1;
    for (int b = 1; b <= a; ++b) comb[a][b] = comb[a - 1][b - 1] + (b <= a - 1 ? comb[a - 1][b] : 0);
  }
  for (int j = 0; j <= T; ++j)
    for (int k = 0; k <= n; ++k) {
      if (j == 0) f[j][k] = 1;
      else if (k < 2 || j == 1) f[j][k] = 0;
      else if (k == 2) f[j][k] = (j % 2 == 0) ? 1 : 0;
      else {
        uint64_t s = 0;
        for (int l = 0; l < k - 1; ++l)
          if (j - k + l >= 0) s += f[j - k + l][k - l] * comb[k - 1][l];
        f[j][k] = s;
      }
    }
  G = f[T][n];
  if (G >= (1ull << 32)) return false;
  for (int j = 0; j <= MAXT; ++j)
    for (int k = 0; k <= MAXN; ++k) t.f[j][k] = (uint32_t)f[j][k];
  for (int a = 0; a <= MAXN; ++a)
    for (int b = 0; b <= MAXN; ++b) t.comb[a][b] = (uint32_t)comb[a][b];
  return true;
}

inline size_t al(size_t x) { return (x + 255) & ~(size_t)255; }

}  // namespace

extern "C" int64_t fiode_certify_grid_rows(int32_t n, int32_t T) {
  CountTable t;
  uint64_t G = 0;
  if (!count_table(n, T, t, G)) return -1;
  return (int64_t)G;
}

extern "C" int fiode_certify_grid(void* stream, int32_t n, int32_t T, uint8_t* grid) {
  CountTable t;
  uint64_t G = 0;
  if (!grid || !count_table(n, T, t, G)) return FIODE_EINVAL;
  if (G == 0) return FIODE_OK;
  hipStream_t st = static_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(k_cert_grid, dim3((unsigned)((G + 255) / 256)), dim3(256), 0, st, t, n, T, (uint32_t)G, grid);
  FIODE_HIP_CHECK(hipGetLastError());
  return FIODE_OK;
}

extern "C" size_t fiode_certify_workspace_bytes(int64_t G, int32_t batches) {
  if (G <= 0 || batches <= 0) return 256;
  const size_t nb = (size_t)batches + 1;
  return al(FIODE_M * 4) + al((size_t)G * C * 4) + al(nb * 4) + al(nb * 8);
}

extern "C" int fiode_certify(void* stream, const fiode_certify_config* cfg, const fiode_dyn_config* dyn,
                             const fiode_dyn_weights* w, const float* x_feat, const uint8_t* grid, int64_t G,
                             float* out, int32_t* exit_iters, void* workspace, size_t workspace_bytes) {
  if (!cfg || !dyn || !w || !x_feat || !grid || !out || !workspace) return FIODE_EINVAL;
  if (dyn->n_hidden != C || dyn->mlp_size != M || dyn->x_dim != FIODE_X) return FIODE_ESHAPE;
  if (cfg->n_classes != C) return FIODE_ESHAPE;
  if (dyn->qp_max_iter < 1 || dyn->qp_max_iter > 32) return FIODE_EINVAL;
  if (cfg->label < 0 || cfg->label >= C || cfg->T <= 0 || cfg->batches <= 0 || !(cfg->min_std > 0.f)) return FIODE_EINVAL;
  if (G < cfg->batches || G >= (1LL << 32)) return FIODE_EINVAL;
  if (workspace_bytes < fiode_certify_workspace_bytes(G, cfg->batches)) return FIODE_EWORKSPACE;
  CertArgs a{};
  a.G = (uint32_t)G;
  a.ebs = (uint32_t)(G / cfg->batches);
  a.nb = cfg->batches + ((G % cfg->batches) != 0 ? 1 : 0);
  a.label = cfg->label;
  a.T = cfg->T;
  if (cfg->T > MAXT) return FIODE_EINVAL;
  for (int v = 0; v <= cfg->T; ++v) a.etab[v] = (float)((double)v / (double)cfg->T);
  a.eps_g = (float)(1.0 / cfg->T);                                   // certify_lipschitz.py:78
  a.dist = (float)(sqrt((double)C) / cfg->T);                        // :81
  const double lfx = (dyn->scale_nominal ? (double)dyn->alpha_1 : 1.0) / (double)cfg->min_std;   // :67-70
  a.kappa = (float)(sqrt(2.0) * lfx * (double)cfg->eps);            // :72
  a.sqrt_n = (float)sqrt((double)C);
  a.sa = (float)((double)dyn->sigma_1 * (double)dyn->alpha_1);
  a.sqrt2 = (float)sqrt(2.0);
  a.d.alpha_1 = dyn->alpha_1; a.d.alpha_2 = dyn->alpha_2; a.d.sigma_1 = dyn->sigma_1;
  a.d.tol = dyn->qp_tol; a.d.scale_nominal = dyn->scale_nominal; a.d.max_iter = dyn->qp_max_iter;
  a.x_feat = x_feat; a.grid = grid;
  a.Q1 = w->Q1; a.b1 = w->b1; a.Qx = w->Qx; a.bx = w->bx; a.Q2 = w->Q2; a.b2 = w->b2; a.Q3 = w->Q3; a.b3 = w->b3;
  char* ws = static_cast<char*>(workspace);
  size_t o = 0;
  a.u = reinterpret_cast<float*>(ws + o); o += al(FIODE_M * 4);
  a.ft = reinterpret_cast<float*>(ws + o); o += al((size_t)G * C * 4);
  a.words = reinterpret_cast<uint32_t*>(ws + o); o += al((size_t)(cfg->batches + 1) * 4);
  a.keys = reinterpret_cast<uint32_t*>(ws + o);
  a.out = out;
  a.exit_iters = exit_iters;
  hipStream_t st = static_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(k_cert_prep, dim3(1), dim3(256), 0, st, a);
  FIODE_HIP_CHECK(hipGetLastError());
  const uint32_t npairs = (a.G + 63) / 64;
  uint32_t blocks = (npairs + FIODE_WAVES - 1) / FIODE_WAVES;
  // persistent: two workgroups per CU, each loading the weight images once
  int dev = 0, ncu = 256;
  if (hipGetDevice(&dev) == hipSuccess && hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    ncu = 256;
  const uint32_t cap = 2u * (uint32_t)(ncu > 0 ? ncu : 256);
  if (blocks > cap) blocks = cap;
  hipLaunchKernelGGL(k_cert_fwd, dim3(blocks), dim3(256), ((size_t)(M + C) * LDQ + MAXT + 1) * sizeof(float), st, a);
  FIODE_HIP_CHECK(hipGetLastError());
  uint32_t fblocks = (a.G + 255) / 256;
  if (fblocks > 8u * (uint32_t)ncu) fblocks = 8u * (uint32_t)ncu;      // persistent: 8 workgroups per CU
  hipLaunchKernelGGL(k_cert_final, dim3(fblocks), dim3(256), 0, st, a);
  FIODE_HIP_CHECK(hipGetLastError());
  hipLaunchKernelGGL(k_cert_decode, dim3(1), dim3(64), 0, st, a);
  FIODE_HIP_CHECK(hipGetLastError());
  return FIODE_OK;
}
