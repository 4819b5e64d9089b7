// Real f32 GEMM of the Cayley-orthogonal layers (gfx950): the products of the dense Cayley maps'
// forward / backward (fiode_amd/cayley.py _dense_forward_fused / _dense_backward: G = V'^T V',
// P = V' inv, A = V'^T Gb, P1 = V' H, P2 = Gb inv^T, the GMn chain) and of the KWLarge head's
// CayleyLinear layers (cayley.py _LinearHeadFn: x Q^T + b, g Q, g^T x), i.e. the
// `cayley(alpha W / ||W||)` parametrisation of convert_cayley (dynamics/classification.py:282-293)
// and the CayleyLinear 4096 -> 512 -> 512 -> 10 head of KWLarge_Concat (models.py:29-35,
// ExpConfig.py:131-138).  These are latency-bound shapes: 512 x 512 outputs over K = 3,584, 128 x 512
// over K = 4,096, 512 x 3,584 over K = 512 -- far too few 64 x 64 output tiles to fill 256 CUs, so
// the K dimension is split over workgroups and the partial tiles are summed in a fixed order by the
// workgroup that finishes a tile last (one launch, deterministic, no float atomics).
//
// C[b] = alpha opA(A[b]) opB(B[b]) + beta C[b] + bias   (row-major; opA = A or A^T, opB = B or B^T)
//
// Workgroup: 256 threads, one 64 x 64 output tile, four waves of 32 x 32 on v_mfma_f32_32x32x2_f32
// (exact f32: a k-ordered fmaf chain per output).  K in chunks of 32 staged through LDS, double-
// buffered, with the next chunk's global loads in flight during the current chunk's MFMAs (one
// barrier per chunk).  LDS operand images are [row][k] with a 36-float row stride for BOTH operands:
// a lane (i, h) reads row i, k = 8 t + 4 h .. + 3 with one ds_read_b128 and feeds MFMA steps
// s = 0..3 of group t from its four registers (the MFMA's k index is a summation dummy: half h at
// step s stands for k = 8 t + 4 h + s in both operands).  Row stride 36: rows i map to bank groups
// 9 i mod 16 -- a bijection on the 16 lanes of every ds_read_b128 lane group (MI355X_MICROARCH.md
// LDS table), so the operand reads are conflict-free; the k-contiguous fills are 8 lanes x 16 B of
// one row (conflict-free ds_write_b128); the transposed fills are 4 b32 stores per float4.
//
// Split-K hand-off (MI355X_MICROARCH.md "Hand-offs measured with sc1 loads", row 1): each split
// stores its raw 64 x 64 partial with 16-B sc1 buffer stores, every storing wave drains vmcnt, a
// workgroup barrier, then ONE lane adds to the tile's counter (agent-scope atomic); the workgroup
// whose add returns S - 1 is the last: its other waves load after a barrier it joins, every load of
// the partials is a 16-B sc1 buffer load, the S partials are added in split order 0..S-1 (the same
// sum whatever the arrival order), and it resets the counter to 0 for the next call.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include "common.h"
#include "fiode.h"

namespace {

constexpr int BM = 64, BN = 64, KC = 64, SL = KC + 4;
constexpr int NT = 256;
constexpr int TILE_F = BM * BN;                 // floats per partial tile
constexpr int LPT = BM * KC / 4 / NT;           // float4 loads per thread per operand chunk (4)
// split-K counters: a FIXED block at the start of every workspace (the same words for every call,
// whatever its shape: a call never reads another call's partials as counters), then the partials
constexpr int64_t CNT_WORDS = 16384;
constexpr int64_t CNT_BYTES = CNT_WORDS * 4;

struct GArgs {
  int M, N, K;
  const float* A;
  const float* B;
  float* C;
  const float* bias;
  int64_t lda, ldb, ldc, sa, sb, sc;
  float alpha, beta;
  int tiles_m, tiles_n, tiles;  // output tiles per matrix
  int S, cps, nch;            // K splits, chunks per split, chunks
  int units, per;             // work units (batch x S x tiles) and units per XCD
  int nvb;                    // virtual blocks (8 per)
  float* part;                // [batch][tiles][S][TILE_F]
  unsigned* cnt;              // [batch][tiles]
  int dbg;                    // probe knob (FIODE_GEMM_VARIANT 4: return at once; 5: no K loop; 6: no
                              // LDS reads in the loop; 7: no global loads in the loop)
};

typedef unsigned int u4v __attribute__((ext_vector_type(4)));

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const float* base, int64_t floats) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(base), 0, (int)(floats * sizeof(float)), 0x00020000);
}
__device__ __forceinline__ f32x4 ld_sc1(__amdgpu_buffer_rsrc_t r, int e) {       // 16-B sc1 load
  const u4v u = __builtin_amdgcn_raw_buffer_load_b128(r, e * 16, 0, 16);
  return f32x4{__uint_as_float(u[0]), __uint_as_float(u[1]), __uint_as_float(u[2]), __uint_as_float(u[3])};
}
__device__ __forceinline__ void st_sc1(__amdgpu_buffer_rsrc_t r, int e, f32x4 v) { // 16-B sc1 store
  const u4v u = u4v{__float_as_uint(v[0]), __float_as_uint(v[1]), __float_as_uint(v[2]), __float_as_uint(v[3])};
  __builtin_amdgcn_raw_buffer_store_b128(u, r, e * 16, 0, 16);
}
typedef __attribute__((address_space(1))) unsigned int gu32_t;

// LDS column of element (row, k) of an operand image: k-contiguous images are plain (their fill is
// 16 lanes x 16 B along one row: conflict-free ds_write_b128); images filled from row-contiguous
// memory (transposed operands: 4 ds_write_b32 per float4, lanes l = 0..15 on rows 4 l + c) XOR the
// k-quad with (row >> 4) & 3, which spreads those 16 lanes over 16 banks; both keep every aligned
// 4-float k-quad contiguous, so the operand reads stay one ds_read_b128
template <bool KC_>
__device__ __forceinline__ int lcol(int row, int k) {
  return KC_ ? k : (k ^ (((row >> 4) & 3) << 2));
}

// one operand's chunk: 64 rows (m or n) x 64 k.  KC_: the operand's k index is contiguous in memory
// (A not transposed / B transposed); else its row index is.  VEC: float4 loads (the contiguous extent
// and the leading dimension multiples of 4, 16-B aligned bases); else element loads.  Every load is
// issued, from a clamped address when out of range, and the range mask is applied when the chunk is
// written to LDS: a select on a loaded value right after its load would make the compiler wait for
// that load there (vmcnt(0) in front of the MFMAs -- cdna_hip_programming.md, the split-K pitfalls)
template <bool KC_, bool VEC>
struct Operand {
  f32x4 r[LPT];
  uint32_t ok;                                   // in-range bits: q (VEC) or 4 q + c (element loads)
  __device__ __forceinline__ void load(const float* P, int64_t ld, int rows, int K, int r0, int k0) {
    ok = 0;
#pragma unroll
    for (int q = 0; q < LPT; ++q) {
      const int idx = threadIdx.x + NT * q;
      int row, k;
      if (KC_) {
        row = r0 + (idx >> 4);
        k = k0 + (idx & 15) * 4;
      } else {
        k = k0 + (idx >> 4);
        row = r0 + (idx & 15) * 4;
      }
      if (VEC) {
        const bool in = row < rows && k < K;
        ok |= (uint32_t)in << q;
        const int64_t off = KC_ ? (int64_t)row * ld + k : (int64_t)k * ld + row;
        r[q] = *reinterpret_cast<const f32x4*>(P + (in ? off : 0));
      } else {
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const int rr = KC_ ? row : row + c, kk = KC_ ? k + c : k;
          const bool in = rr < rows && kk < K;
          ok |= (uint32_t)in << (4 * q + c);
          r[q][c] = P[in ? (KC_ ? (int64_t)rr * ld + kk : (int64_t)kk * ld + rr) : 0];
        }
      }
    }
  }
  __device__ __forceinline__ float pick(int q, int c) const {
    const bool in = VEC ? ((ok >> q) & 1u) : ((ok >> (4 * q + c)) & 1u);
    return in ? r[q][c] : 0.f;
  }
  __device__ __forceinline__ void store(float (*S)[SL]) const {
#pragma unroll
    for (int q = 0; q < LPT; ++q) {
      const int idx = threadIdx.x + NT * q;
      if (KC_) {
        *reinterpret_cast<f32x4*>(&S[idx >> 4][(idx & 15) * 4]) = f32x4{pick(q, 0), pick(q, 1), pick(q, 2), pick(q, 3)};
      } else {
        const int kk = idx >> 4, r4 = (idx & 15) * 4;
#pragma unroll
        for (int c = 0; c < 4; ++c) S[r4 + c][lcol<false>(r4 + c, kk)] = pick(q, c);
      }
    }
  }
};

// split-K hand-off (the last workgroup of a tile sums the S partials in split order) and the
// epilogue C = alpha acc + beta C + bias[n]; shared by both K loops
__device__ __forceinline__ void gemm_finish(const GArgs& a, f32x16 acc, int z, int tile, int s, int m0, int n0,
                                            int* lastp) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int j = lane & 31, h = lane >> 5;
  const int wm = w & 1, wn = w >> 1;
  if (a.S > 1) {
    // ---- split-K: publish the raw partial, the last workgroup of the tile sums them in order ----
    float* slab = a.part + ((int64_t)z * a.tiles + tile) * a.S * TILE_F;
    const __amdgpu_buffer_rsrc_t rs = rsrc(slab, (int64_t)a.S * TILE_F);
#pragma unroll
    for (int g = 0; g < 4; ++g)
      st_sc1(rs, s * (TILE_F / 4) + (w * 4 + g) * 64 + lane, f32x4{acc[4 * g], acc[4 * g + 1], acc[4 * g + 2], acc[4 * g + 3]});
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");       // every storing wave drains its stores
    __syncthreads();
    unsigned* cnt = a.cnt + (int64_t)z * a.tiles + tile;          // < CNT_WORDS (plan_of)
    if (threadIdx.x == 0) {
      const unsigned old = __hip_atomic_fetch_add((gu32_t*)cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      *lastp = old == (unsigned)(a.S - 1);
    }
    __syncthreads();
    if (!*lastp) return;                              // (uniform)
    f32x4 sum[4];
#pragma unroll
    for (int g = 0; g < 4; ++g) sum[g] = ld_sc1(rs, (w * 4 + g) * 64 + lane);
    for (int p = 1; p < a.S; ++p) {
      f32x4 v[4];
#pragma unroll
      for (int g = 0; g < 4; ++g) v[g] = ld_sc1(rs, p * (TILE_F / 4) + (w * 4 + g) * 64 + lane);
#pragma unroll
      for (int g = 0; g < 4; ++g) sum[g] = sum[g] + v[g];
    }
#pragma unroll
    for (int g = 0; g < 4; ++g)
#pragma unroll
      for (int c = 0; c < 4; ++c) acc[4 * g + c] = sum[g][c];
    if (threadIdx.x == 0) __hip_atomic_store((gu32_t*)cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }

  // ---- epilogue: C = alpha acc + beta C + bias[n] ------------------------------------------------
  float* C = a.C + (int64_t)z * a.sc;
  const int n = n0 + 32 * wn + j;
  if (n >= a.N) return;
  const float bn = a.bias ? a.bias[n] : 0.f;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int m = m0 + 32 * wm + acc_row(r, h);
    if (m < a.M) {
      float* cp = C + (int64_t)m * a.ldc + n;
      float v = a.alpha * acc[r];
      if (a.beta != 0.f) v = v + a.beta * *cp;
      if (a.bias) v = v + bn;
      *cp = v;
    }
  }
}

template <bool AK, bool BK, bool VEC>
__device__ __forceinline__ void gemm_unit(const GArgs& a, int vb, float (*sA)[BM][SL], float (*sB)[BN][SL],
                                          int* lastp) {
  // XCD-aware work mapping: blocks are dealt round-robin over the 8 XCDs (block b on XCD b % 8,
  // MI355X_MICROARCH.md; for speed only), so XCD x takes the contiguous run of work units
  // [x per, (x + 1) per) of the order (batch, split, column tile, row tile): the units of one XCD
  // share their K range (split) and B column block, which its L2 then holds once, instead of every
  // XCD streaming the whole operand (W2 of the 4096 -> 512 map: 7.3 MB per XCD).  vb: the virtual
  // block (= blockIdx.x, or one of a capped grid's trips, which keep vb % 8 and so the XCD)
  const int u = (vb & 7) * a.per + (vb >> 3);
  if (u >= a.units) return;                        // (uniform; no barrier yet)
  const int tm_ = u % a.tiles_m, rest = u / a.tiles_m;
  const int tn_ = rest % a.tiles_n, rest2 = rest / a.tiles_n;
  const int s = rest2 % a.S, z = rest2 / a.S;
  const int tile = tm_ * a.tiles_n + tn_;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int j = lane & 31, h = lane >> 5;
  const int wm = w & 1, wn = w >> 1;
  const int m0 = tm_ * BM, n0 = tn_ * BN;
  const float* A = a.A + (int64_t)z * a.sa;
  const float* B = a.B + (int64_t)z * a.sb;
  const int c0 = s * a.cps, c1 = min(a.nch, c0 + a.cps);

  // K loop: LDS double buffer + two register stages, so a chunk's global loads are issued two
  // chunks (two MFMA phases of 32 MFMAs per wave) before they are stored to LDS
  Operand<AK, VEC> oa0, oa1;
  Operand<BK, VEC> ob0, ob1;
  f32x16 acc = f16_zero(), acc1 = f16_zero();     // two interleaved chains (see k_gemm_dma)
  const int ra = 32 * wm + j, rb = 32 * wn + j;
  auto compute = [&](int buf) {
#pragma unroll
    for (int t = 0; t < KC / 8; ++t) {
      const f32x4 av = *reinterpret_cast<const f32x4*>(&sA[buf][ra][lcol<AK>(ra, 8 * t + 4 * h)]);
      const f32x4 bv = *reinterpret_cast<const f32x4*>(&sB[buf][rb][lcol<BK>(rb, 8 * t + 4 * h)]);
#pragma unroll
      for (int q = 0; q < 4; q += 2) {
        acc = mfma32(av[q], bv[q], acc);
        acc1 = mfma32(av[q + 1], bv[q + 1], acc1);
      }
    }
  };
  // every chunk load is unconditional (a chunk index past the split is clamped to its last chunk and
  // the copy goes unused), so the count of loads in flight is the same on every path and the
  // compiler's vmcnt waits in front of the LDS stores are counted, not vmcnt(0)
  const int cl = max(c0, c1 - 1);
  if (c0 < c1) {
    oa0.load(A, a.lda, a.M, a.K, m0, c0 * KC);
    ob0.load(B, a.ldb, a.N, a.K, n0, c0 * KC);
    oa1.load(A, a.lda, a.M, a.K, m0, min(c0 + 1, cl) * KC);
    ob1.load(B, a.ldb, a.N, a.K, n0, min(c0 + 1, cl) * KC);
    oa0.store(sA[0]);
    ob0.store(sB[0]);
  }
  __syncthreads();
  for (int c = c0; c < c1; c += 2) {              // (uniform trip count)
    // even: buf 0 holds chunk c, stage 1 chunk c + 1
    oa0.load(A, a.lda, a.M, a.K, m0, min(c + 2, cl) * KC);
    ob0.load(B, a.ldb, a.N, a.K, n0, min(c + 2, cl) * KC);
    compute(0);
    if (c + 1 < c1) {
      oa1.store(sA[1]);
      ob1.store(sB[1]);
    }
    __syncthreads();
    if (c + 1 >= c1) break;
    // odd: buf 1 holds chunk c + 1, stage 0 chunk c + 2
    oa1.load(A, a.lda, a.M, a.K, m0, min(c + 3, cl) * KC);
    ob1.load(B, a.ldb, a.N, a.K, n0, min(c + 3, cl) * KC);
    compute(1);
    if (c + 2 < c1) {
      oa0.store(sA[0]);
      ob0.store(sB[0]);
    }
    __syncthreads();
  }

  gemm_finish(a, acc + acc1, z, tile, s, m0, n0, lastp);
}

// one workgroup per work unit, or (max_workgroups) a capped grid whose workgroups loop over the
// virtual blocks b, b + grid, ... -- a narrow launch that leaves the other CUs to concurrent work
template <bool AK, bool BK, bool VEC>
__global__ void __launch_bounds__(NT) k_gemm(GArgs a) {
  __shared__ __attribute__((aligned(16))) float sA[2][BM][SL];
  __shared__ __attribute__((aligned(16))) float sB[2][BN][SL];
  __shared__ int last;
  for (int vb = blockIdx.x; vb < a.nvb; vb += gridDim.x) {
    gemm_unit<AK, BK, VEC>(a, vb, sA, sB, &last);
    __syncthreads();                               // (uniform) LDS and `last` reused by the next trip
  }
}

// ---- the LDS-DMA K loop (aligned shapes: M, N multiples of 64, K of 32, 16-B aligned operands) ----
// Each 64 x 32 operand chunk is eight global_load_lds_dwordx4 wave instructions (1 KiB each, two per
// wave), written straight into LDS (no VGPR staging, so no register hazard can force the compiler
// into a vmcnt(0) wait -- which is what bounded the register-staged loop), into a ring of NS = 4
// stages: chunk c + 3 is in flight while chunk c is computed.  Per chunk, each wave waits with a
// COUNTED vmcnt (its two newer chunks' 8 loads stay in flight), joins a raw s_barrier (a
// __syncthreads would drain every DMA: cdna_hip_programming.md, "Pipelining across barriers"), then
// restages the slot read one chunk earlier and computes.  All LDS is one __shared__ array (a second
// object can make the compiler wait vmcnt(0) in front of the ds_reads).
// Images: a k-contiguous operand is [64 rows][32 k] (128-B rows), its 4-float quads XOR-swizzled
// by (row >> 1) & 7 on the SOURCE address (the DMA destination is lane-linear), so a ds_read_b128 of
// 16 rows hits 16 distinct bank quads; a row-contiguous operand is [32 k][64 rows] as it lies in
// memory, read with ds_read_b32 (lanes on consecutive rows: conflict-free).
constexpr int DKC = 32;                                   // the default chunk k (plan_of's unit)
typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(1))) void glob_void;

// k-quad swizzle of a k-contiguous image row: 32-float rows (two rows per 64-bank line) by
// (row >> 1) & 7, 64-float rows by row & 15 -- either way the 16 rows of a ds_read_b128 lane group
// land on 16 distinct bank quads
template <int KCH>
__device__ __forceinline__ int qswz(int row) { return KCH == 32 ? ((row >> 1) & 7) : (row & 15); }

template <bool KC_, int KCH>
__device__ __forceinline__ void dma_chunk(float* img, const float* P, int64_t ld, int r0, int k0, int w, int lane) {
  constexpr int NI = 64 * KCH / 256;                       // wave instructions per operand chunk
#pragma unroll
  for (int u = 0; u < NI / 4; ++u) {
    const int q = w + 4 * u;
    const float* src;
    if (KC_) {                                             // 1 KiB = 256 / KCH rows of KCH floats
      constexpr int RPI = 256 / KCH, QPR = KCH / 4;
      const int r = RPI * q + lane / QPR, p = lane % QPR;
      src = P + (int64_t)(r0 + r) * ld + k0 + 4 * (p ^ qswz<KCH>(r));
    } else {                                               // k rows 4 q .. 4 q + 3, 16 quads each
      src = P + (int64_t)(k0 + 4 * q + (lane >> 4)) * ld + r0 + 4 * (lane & 15);
    }
    __builtin_amdgcn_global_load_lds((glob_void*)src, (lds_void*)(img + 256 * q), 16, 0, 0);
  }
}

template <bool AK, bool BK, int NSG, int KCH, bool PF>
__device__ __forceinline__ void gemm_dma_unit(const GArgs& a, int vb, float* sm) {
  constexpr int IMG = 64 * KCH;                             // floats per operand image
  constexpr int PER_CHUNK = 2 * (64 * KCH / 256) / 4;       // glds per wave per chunk
  int* lastp = reinterpret_cast<int*>(&sm[NSG * 2 * IMG]);
  const int u = (vb & 7) * a.per + (vb >> 3);               // XCD-aware, as gemm_unit
  if (u >= a.units || a.dbg == 4) return;
  const int tm_ = u % a.tiles_m, rest = u / a.tiles_m;
  const int tn_ = rest % a.tiles_n, rest2 = rest / a.tiles_n;
  const int s = rest2 % a.S, z = rest2 / a.S;
  const int tile = tm_ * a.tiles_n + tn_;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int j = lane & 31, h = lane >> 5;
  const int wm = w & 1, wn = w >> 1;
  const int m0 = tm_ * BM, n0 = tn_ * BN;
  const float* A = a.A + (int64_t)z * a.sa;
  const float* B = a.B + (int64_t)z * a.sb;
  // chunks of KCH k (a.cps / a.nch count DKC-chunks: KCH / DKC of them per chunk here)
  constexpr int R = KCH / DKC;
  const int c0 = s * a.cps / R, c1 = (min(a.nch, s * a.cps + a.cps) + R - 1) / R, cl = max(c0, c1 - 1);
  auto slot_of = [&](int c) { return NSG == 4 ? ((c - c0) & 3) : ((c - c0) % NSG); };
  auto issue = [&](int c) {              // chunk min(c, cl) into ring slot (c - c0) % NSG
    const int slot = slot_of(c), cc = min(c, cl);
    dma_chunk<AK, KCH>(&sm[(slot * 2 + 0) * IMG], A, a.lda, m0, cc * KCH, w, lane);
    dma_chunk<BK, KCH>(&sm[(slot * 2 + 1) * IMG], B, a.ldb, n0, cc * KCH, w, lane);
  };
  const int ra = 32 * wm + j, rb = 32 * wn + j;
  auto rd = [&](const float* ia, const float* ib, int t, f32x4& av, f32x4& bv) {
    const int qd = 2 * t + h;                              // k quad of this lane half
    if (AK) av = *reinterpret_cast<const f32x4*>(ia + ra * KCH + 4 * (qd ^ qswz<KCH>(ra)));
    else {
#pragma unroll
      for (int e = 0; e < 4; ++e) av[e] = ia[(4 * qd + e) * 64 + ra];
    }
    if (BK) bv = *reinterpret_cast<const f32x4*>(ib + rb * KCH + 4 * (qd ^ qswz<KCH>(rb)));
    else {
#pragma unroll
      for (int e = 0; e < 4; ++e) bv[e] = ib[(4 * qd + e) * 64 + rb];
    }
  };
  // two accumulators, the k-steps alternating between them (summed once at the end)
  f32x16 acc = f16_zero(), acc1 = f16_zero();
  if (c0 < c1 && a.dbg != 5) {
#pragma unroll
    for (int i = 0; i < NSG - 1; ++i) issue(c0 + i);
    for (int c = c0; c < c1; ++c) {
      // this wave's loads of chunk c are in LDS (its NSG - 2 newer chunks' loads stay in flight)
      if constexpr ((NSG - 2) * PER_CHUNK == 12) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
      else if constexpr ((NSG - 2) * PER_CHUNK == 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
      else if constexpr ((NSG - 2) * PER_CHUNK == 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // (and its reads of chunk c - 1 retired)
      __builtin_amdgcn_s_barrier();                       // ... and every other wave's
      if (a.dbg != 7) issue(c + NSG - 1);                 // into the slot chunk c - 1 used
      const float* ia = &sm[(slot_of(c) * 2 + 0) * IMG];
      const float* ib = &sm[(slot_of(c) * 2 + 1) * IMG];
      if (a.dbg == 6) {
        const float xa = __int_as_float(threadIdx.x), xb = __int_as_float(c);
#pragma unroll
        for (int t = 0; t < KCH / 4; ++t) {
          acc = mfma32(xa, xb, acc);
          acc1 = mfma32(xa, xb, acc1);
        }
      } else if (PF) {
        // the operands of k-group t + 1 read from LDS before group t's MFMAs are issued (two register
        // sets), so an MFMA never waits on the read that feeds it
        f32x4 av[2], bv[2];
        rd(ia, ib, 0, av[0], bv[0]);
#pragma unroll
        for (int t = 0; t < KCH / 8; ++t) {
          if (t + 1 < KCH / 8) rd(ia, ib, t + 1, av[(t + 1) & 1], bv[(t + 1) & 1]);
#pragma unroll
          for (int e = 0; e < 4; e += 2) {
            acc = mfma32(av[t & 1][e], bv[t & 1][e], acc);
            acc1 = mfma32(av[t & 1][e + 1], bv[t & 1][e + 1], acc1);
          }
          // keep the schedule in that order: group t + 1's LDS reads, then group t's 4 MFMAs
          __builtin_amdgcn_sched_group_barrier(0x100, 8, 0);
          __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);
        }
      } else {
#pragma unroll
        for (int t = 0; t < KCH / 8; ++t) {
          f32x4 av, bv;
          rd(ia, ib, t, av, bv);
#pragma unroll
          for (int e = 0; e < 4; e += 2) {
            acc = mfma32(av[e], bv[e], acc);
            acc1 = mfma32(av[e + 1], bv[e + 1], acc1);
          }
        }
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");      // the clamped tail loads land before exit
    __syncthreads();
  }
  gemm_finish(a, acc + acc1, z, tile, s, m0, n0, lastp);
}

template <bool AK, bool BK, int NSG, int KCH, bool PF = false>
__global__ void __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(1, 2))) k_gemm_dma(GArgs a) {
  __shared__ __attribute__((aligned(16))) float sm[NSG * 2 * 64 * KCH + 4];
  for (int vb = blockIdx.x; vb < a.nvb; vb += gridDim.x) {   // (see k_gemm)
    gemm_dma_unit<AK, BK, NSG, KCH, PF>(a, vb, sm);
    __syncthreads();
  }
}

// A capped (narrow) grid claims each CU's whole LDS: the dispatcher then puts no other LDS-using
// workgroup on its CUs, so the concurrent kernels it is meant to leave room for land on the other CUs
// instead of sharing SIMDs with it (measured: a 40-workgroup spectral inverse beside a 64-workgroup
// capped GEMM ran 2.3x slower when both packed onto the same CUs).
constexpr size_t LDS_PER_CU = 163840;
template <typename Kern>
void launch_gemm(Kern kern, dim3 grid, size_t static_lds, bool excl, hipStream_t st, const GArgs& a) {
  size_t dyn = 0;
  if (excl && static_lds + 512 < LDS_PER_CU) {
    dyn = LDS_PER_CU - static_lds - 512;
    hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize, (int)dyn);
  }
  hipLaunchKernelGGL(kern, grid, dim3(NT), dyn, st, a);
}

// Two independent products in ONE launch (fiode_gemm_pair): virtual blocks [0, a0.nvb) are problem
// 0's, the rest problem 1's (a0.nvb is a multiple of 8, so every block keeps its XCD's share of
// either problem).  Each tile is computed exactly as fiode_gemm computes it (same k order, same
// split order): the pair is bit-identical to the two calls.  The 64-k, two-stage, prefetching K loop
// only; other shapes take two launches.
template <bool AK0, bool BK0, bool AK1, bool BK1>
__global__ void __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(1, 2))) k_gemm_dma_pair(GArgs a0, GArgs a1) {
  __shared__ __attribute__((aligned(16))) float sm[2 * 2 * 64 * 64 + 4];
  const int n0 = a0.nvb, n = n0 + a1.nvb;
  for (int vb = blockIdx.x; vb < n; vb += gridDim.x) {
    if (vb < n0) gemm_dma_unit<AK0, BK0, 2, 64, true>(a0, vb, sm);
    else gemm_dma_unit<AK1, BK1, 2, 64, true>(a1, vb - n0, sm);
    __syncthreads();
  }
}

int gemm_variant() {
  const char* e = getenv("FIODE_GEMM_VARIANT");           // probe knob: 0 = default
  return e && *e ? atoi(e) : 0;
}

struct Plan {
  int tiles_m, tiles_n, tiles, nch, S, cps;
  bool dma;
};

bool dma_shape(const fiode_gemm_desc* d) {       // the k_gemm_dma path (shape conditions; pointers apart)
  const bool ak = !d->trans_a, bk = d->trans_b != 0;
  (void)ak; (void)bk;
  return d->M % BM == 0 && d->N % BN == 0 && d->K % DKC == 0 && d->K > 0 && d->lda % 4 == 0 && d->ldb % 4 == 0 &&
         d->stride_a % 4 == 0 && d->stride_b % 4 == 0;
}

bool plan_of(const fiode_gemm_desc* d, Plan& p, bool force_reg = false) {
  if (!d || d->batch < 1 || d->batch > 65535 || d->M < 0 || d->N < 0 || d->K < 0) return false;
  p.dma = !force_reg && dma_shape(d);
  const int kc = p.dma ? DKC : KC;
  p.tiles_m = (d->M + BM - 1) / BM;
  p.tiles_n = (d->N + BN - 1) / BN;
  p.tiles = p.tiles_m * p.tiles_n;
  p.nch = (d->K + kc - 1) / kc;
  const int64_t wgs = (int64_t)p.tiles * d->batch;
  int S = d->split_k;
  if (S <= 0) {
    // the library's choice: about one workgroup per CU (a block's latency, not the MFMA rate, sets
    // these launches' time), at least 4 k-steps of 32 per split, and at most 8 splits so that the
    // last workgroup of a tile reads <= 128 KB of partials (cdna_hip_programming.md, split-K)
    S = 1;
    if (wgs > 0 && wgs < 256) S = (int)((256 + wgs - 1) / wgs);
    S = min(S, max(1, d->K / 128));
    S = min(S, 8);
  }
  S = max(1, min(S, max(1, p.nch)));
  if (wgs > CNT_WORDS) S = 1;  // (the counter block's capacity)
  p.cps = p.nch > 0 ? (p.nch + S - 1) / S : 0;
  p.S = p.cps > 0 ? (p.nch + p.cps - 1) / p.cps : 1;     // no empty split
  return true;
}

}  // namespace

extern "C" FIODE_API int32_t fiode_gemm_splits(const fiode_gemm_desc* d) {
  Plan p;
  return plan_of(d, p) ? p.S : 0;
}

extern "C" FIODE_API size_t fiode_gemm_counter_bytes(const fiode_gemm_desc* d) {
  Plan p, q;
  if (!plan_of(d, p) || !plan_of(d, q, true) || (p.S <= 1 && q.S <= 1)) return 0;
  return CNT_BYTES;
}

// (the larger of the two K loops' plans: which one runs also depends on the operands' alignment)
extern "C" FIODE_API size_t fiode_gemm_workspace_bytes(const fiode_gemm_desc* d) {
  Plan p, q;
  if (!plan_of(d, p) || !plan_of(d, q, true) || (p.S <= 1 && q.S <= 1)) return 0;
  const int S = p.S > q.S ? p.S : q.S;
  return CNT_BYTES + (size_t)d->batch * p.tiles * S * TILE_F * sizeof(float);
}

extern "C" FIODE_API int fiode_gemm(void* stream, const fiode_gemm_desc* d, const float* A, const float* B,
                                    const float* bias, float* C, void* workspace, size_t workspace_bytes) {
  Plan p;
  if (!plan_of(d, p)) return FIODE_EINVAL;
  if (d->M == 0 || d->N == 0) return FIODE_OK;
  if (!C || (d->K > 0 && (!A || !B))) return FIODE_EINVAL;
  const bool ta = d->trans_a != 0, tb = d->trans_b != 0;
  // leading dimensions: opA [M][K] is A [M][lda] (ta = 0) or A [K][lda] (ta = 1)
  if (d->ldc < d->N || d->lda < (ta ? d->M : d->K) || d->ldb < (tb ? d->K : d->N)) return FIODE_ESHAPE;
  if (p.S > 1 && (!workspace || workspace_bytes < fiode_gemm_workspace_bytes(d))) return FIODE_EWORKSPACE;
  const bool ak = !ta, bk = tb;                  // k contiguous in memory
  auto al16 = [](const void* q) { return ((uintptr_t)q & 15u) == 0; };
  const bool vec = al16(A) && al16(B) && d->lda % 4 == 0 && d->ldb % 4 == 0 && d->stride_a % 4 == 0 &&
                   d->stride_b % 4 == 0 && (ak ? d->K % 4 == 0 : d->M % 4 == 0) && (bk ? d->K % 4 == 0 : d->N % 4 == 0);
  const bool dma = p.dma && al16(A) && al16(B);
  if (p.dma && !dma) plan_of(d, p, true);       // unaligned operands: the register loop's plan
  GArgs a;
  a.M = d->M; a.N = d->N; a.K = d->K;
  a.A = A; a.B = B; a.C = C; a.bias = bias;
  a.lda = d->lda; a.ldb = d->ldb; a.ldc = d->ldc;
  a.sa = d->stride_a; a.sb = d->stride_b; a.sc = d->stride_c;
  a.alpha = d->alpha; a.beta = d->beta;
  a.tiles_m = p.tiles_m; a.tiles_n = p.tiles_n; a.tiles = p.tiles;
  a.S = p.S; a.cps = p.cps; a.nch = p.nch;
  a.units = d->batch * p.S * p.tiles;
  a.per = (a.units + 7) / 8;
  a.nvb = 8 * a.per;
  a.cnt = p.S > 1 ? (unsigned*)workspace : nullptr;
  a.part = p.S > 1 ? (float*)((char*)workspace + CNT_BYTES) : nullptr;
  a.dbg = gemm_variant();
  // max_workgroups: a persistent grid (a multiple of 8, so every trip keeps its XCD) that loops
  int nb = a.nvb;
  if (d->max_workgroups > 0 && d->max_workgroups < nb) nb = d->max_workgroups < 8 ? 8 : d->max_workgroups & ~7;
  const dim3 grid((unsigned)nb);
  const bool excl = nb < a.nvb;
  hipStream_t st = (hipStream_t)stream;
  if (dma) {
    const int v = gemm_variant();
#define FIODE_DMA(NS_, KC2_, PF_)                                                                           \
  do {                                                                                                      \
    const size_t sl = (size_t)(NS_ * 2 * 64 * KC2_ + 4) * sizeof(float);                                     \
    if (ak && bk) launch_gemm(k_gemm_dma<true, true, NS_, KC2_, PF_>, grid, sl, excl, st, a);                \
    else if (ak) launch_gemm(k_gemm_dma<true, false, NS_, KC2_, PF_>, grid, sl, excl, st, a);                \
    else if (bk) launch_gemm(k_gemm_dma<false, true, NS_, KC2_, PF_>, grid, sl, excl, st, a);                \
    else launch_gemm(k_gemm_dma<false, false, NS_, KC2_, PF_>, grid, sl, excl, st, a);                       \
  } while (0)
    // 64-k chunks in two stages where every split holds whole ones, the LDS operands read one k-group
    // ahead (measured fastest on the step's shapes: tools/probes/gemm_probe.py, profiles/r06/
    // gemm_probe_prefetch.log), else 32-k chunks in a ring of four
    const bool k64 = d->K % 64 == 0 && p.cps % 2 == 0;
    if (v == 1 && k64) FIODE_DMA(3, 64, false);
    else if (v == 3) FIODE_DMA(3, 32, false);
    else if (v == 8 && k64) FIODE_DMA(2, 64, true);
    else if (v == 9) FIODE_DMA(4, 32, true);
    else if (v == 2) FIODE_DMA(2, 64, false);
    else if (v == 0 && k64) FIODE_DMA(2, 64, true);
    else FIODE_DMA(4, 32, false);
#undef FIODE_DMA
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? FIODE_OK : FIODE_EHIP + (int)e;
  }
  const size_t sl = (size_t)(2 * 2 * BM * SL + 4) * sizeof(float);
#define FIODE_GEMM_LAUNCH(AK_, BK_, V_) launch_gemm(k_gemm<AK_, BK_, V_>, grid, sl, excl, st, a)
  if (vec) {
    if (ak && bk) FIODE_GEMM_LAUNCH(true, true, true);
    else if (ak) FIODE_GEMM_LAUNCH(true, false, true);
    else if (bk) FIODE_GEMM_LAUNCH(false, true, true);
    else FIODE_GEMM_LAUNCH(false, false, true);
  } else {
    if (ak && bk) FIODE_GEMM_LAUNCH(true, true, false);
    else if (ak) FIODE_GEMM_LAUNCH(true, false, false);
    else if (bk) FIODE_GEMM_LAUNCH(false, true, false);
    else FIODE_GEMM_LAUNCH(false, false, false);
  }
#undef FIODE_GEMM_LAUNCH
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? FIODE_OK : FIODE_EHIP + (int)e;
}

namespace {
// The checks and kernel arguments of one fiode_gemm product; cnt / part: its counter words and
// partial-tile region.  ok_pair: the product takes the 64-k prefetching DMA loop (the pair kernel's).
int gemm_prepare(const fiode_gemm_desc* d, const float* A, const float* B, const float* bias, float* C, unsigned* cnt,
                 float* part, GArgs& a, bool& ok_pair, bool& ak, bool& bk) {
  Plan p;
  if (!plan_of(d, p)) return FIODE_EINVAL;
  if (!C || (d->K > 0 && (!A || !B))) return FIODE_EINVAL;
  const bool ta = d->trans_a != 0, tb = d->trans_b != 0;
  if (d->ldc < d->N || d->lda < (ta ? d->M : d->K) || d->ldb < (tb ? d->K : d->N)) return FIODE_ESHAPE;
  ak = !ta;
  bk = tb;
  auto al16 = [](const void* q) { return ((uintptr_t)q & 15u) == 0; };
  const bool k64 = d->K % 64 == 0 && p.cps % 2 == 0;
  ok_pair = p.dma && al16(A) && al16(B) && k64 && gemm_variant() == 0 && d->max_workgroups == 0 && d->M > 0 &&
            d->N > 0;
  a.M = d->M; a.N = d->N; a.K = d->K;
  a.A = A; a.B = B; a.C = C; a.bias = bias;
  a.lda = d->lda; a.ldb = d->ldb; a.ldc = d->ldc;
  a.sa = d->stride_a; a.sb = d->stride_b; a.sc = d->stride_c;
  a.alpha = d->alpha; a.beta = d->beta;
  a.tiles_m = p.tiles_m; a.tiles_n = p.tiles_n; a.tiles = p.tiles;
  a.S = p.S; a.cps = p.cps; a.nch = p.nch;
  a.units = d->batch * p.S * p.tiles;
  a.per = (a.units + 7) / 8;
  a.nvb = 8 * a.per;
  a.cnt = p.S > 1 ? cnt : nullptr;
  a.part = p.S > 1 ? part : nullptr;
  a.dbg = 0;
  return FIODE_OK;
}
}  // namespace

extern "C" FIODE_API size_t fiode_gemm_pair_workspace_bytes(const fiode_gemm_desc* d0, const fiode_gemm_desc* d1) {
  const size_t w0 = fiode_gemm_workspace_bytes(d0), w1 = fiode_gemm_workspace_bytes(d1);
  if (!w0 && !w1) return 0;
  return CNT_BYTES + (w0 ? w0 - CNT_BYTES : 0) + (w1 ? w1 - CNT_BYTES : 0);
}

extern "C" FIODE_API int fiode_gemm_pair(void* stream, const fiode_gemm_desc* d0, const float* A0, const float* B0,
                                         const float* bias0, float* C0, const fiode_gemm_desc* d1, const float* A1,
                                         const float* B1, const float* bias1, float* C1, void* workspace,
                                         size_t workspace_bytes) {
  if (!d0 || !d1) return FIODE_EINVAL;
  const size_t need = fiode_gemm_pair_workspace_bytes(d0, d1);
  if (need && (!workspace || workspace_bytes < need)) return FIODE_EWORKSPACE;
  const size_t w0 = fiode_gemm_workspace_bytes(d0);
  Plan p0;
  if (!plan_of(d0, p0)) return FIODE_EINVAL;
  unsigned* cnt = reinterpret_cast<unsigned*>(workspace);
  float* part = workspace ? reinterpret_cast<float*>(static_cast<char*>(workspace) + CNT_BYTES) : nullptr;
  // problem 1's counters follow problem 0's tiles in the fixed block; its partials follow problem 0's
  const int64_t c1 = (int64_t)d0->batch * p0.tiles;
  GArgs a0, a1;
  bool ok0, ok1, ak0, bk0, ak1, bk1;
  int rc = gemm_prepare(d0, A0, B0, bias0, C0, cnt, part, a0, ok0, ak0, bk0);
  if (rc != FIODE_OK) return rc;
  rc = gemm_prepare(d1, A1, B1, bias1, C1, cnt ? cnt + c1 : nullptr,
                    part ? part + (w0 ? (w0 - CNT_BYTES) / sizeof(float) : 0) : nullptr, a1, ok1, ak1, bk1);
  if (rc != FIODE_OK) return rc;
  Plan p1;
  plan_of(d1, p1);
  const bool fits = c1 + (int64_t)d1->batch * p1.tiles <= CNT_WORDS;
  hipStream_t st = (hipStream_t)stream;
  if (ok0 && ok1 && fits) {
    const dim3 grid((unsigned)(a0.nvb + a1.nvb));
#define FIODE_PAIR(X0, Y0, X1, Y1)                                                                     \
    if (ak0 == X0 && bk0 == Y0 && ak1 == X1 && bk1 == Y1) {                                         \
      hipLaunchKernelGGL((k_gemm_dma_pair<X0, Y0, X1, Y1>), grid, dim3(NT), 0, st, a0, a1);        \
      const hipError_t e = hipGetLastError();                                                        \
      return e == hipSuccess ? FIODE_OK : FIODE_EHIP + (int)e;                                       \
    }
    // the dense maps' backward pair A = V'^T Gb with P2 = inv Gb^T (wide maps; tall: the mirror)
    FIODE_PAIR(true, true, true, false)
    FIODE_PAIR(false, false, true, true)
#undef FIODE_PAIR
  }
  // any other pair: the two products one after the other (the same results)
  rc = fiode_gemm(stream, d0, A0, B0, bias0, C0, workspace, workspace_bytes);
  if (rc != FIODE_OK) return rc;
  return fiode_gemm(stream, d1, A1, B1, bias1, C1, workspace, workspace_bytes);
}
