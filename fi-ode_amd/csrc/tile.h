// Wave-tile building blocks of the Cayley-MLP dynamics (classification.py:96-102) shared by
// the training-step, eval and ODE kernels.  See lyap.hip for the layout.
#pragma once
#include "common.h"

namespace fiode_tile {
constexpr int C = FIODE_C;
constexpr int M = FIODE_M;
constexpr int LDQ = FIODE_LDQ;

__device__ __forceinline__ void load_row10(const float* p, float (&v)[C]) {
  const float2* q = reinterpret_cast<const float2*>(p);
#pragma unroll
  for (int j = 0; j < 5; ++j) {
    const float2 t = q[j];
    v[2 * j] = t.x;
    v[2 * j + 1] = t.y;
  }
}
__device__ __forceinline__ void store_row10(float* p, const float (&v)[C]) {
  float2* q = reinterpret_cast<float2*>(p);
#pragma unroll
  for (int j = 0; j < 5; ++j) q[j] = make_float2(v[2 * j], v[2 * j + 1]);
}

// relu(dropout(z)) on one accumulator tile, in place (classification.py:98,100); DROP = false:
// plain relu (dropout off: keep = 1, scale = 1 -- the same values, without the per-element mask work)
template <bool DROP = true>
__device__ __forceinline__ void dropout_relu(f32x16& z, uint32_t kw, int half, float scale) {
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    if (DROP) {
      const bool keep = (kw >> acc_row(r, half)) & 1u;
      z[r] = keep ? fmaxf(z[r] * scale, 0.f) : 0.f;
    } else {
      z[r] = fmaxf(z[r], 0.f);
    }
  }
}

// store one [32 hidden x 32 samples] accumulator block as rows of a sample-major [N][M] array
__device__ __forceinline__ void store_acc_rows(float* base_row, int mb, int half, const f32x16& z) {
#pragma unroll
  for (int g = 0; g < 4; ++g)
    *reinterpret_cast<f32x4*>(base_row + 32 * mb + 8 * g + 4 * half) =
        f32x4{z[4 * g], z[4 * g + 1], z[4 * g + 2], z[4 * g + 3]};
}
__device__ __forceinline__ void load_acc_rows(const float* base_row, int mb, int half, f32x16& z) {
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    const f32x4 t = *reinterpret_cast<const f32x4*>(base_row + 32 * mb + 8 * g + 4 * half);
    z[4 * g] = t[0]; z[4 * g + 1] = t[1]; z[4 * g + 2] = t[2]; z[4 * g + 3] = t[3];
  }
}

// gather the 10 outputs of the (M padded to 32) layer-3 accumulator into every lane of the row
__device__ __forceinline__ void gather_ft(const f32x16& z3, int half, float (&ft)[C]) {
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const float o = shfl_xor32(z3[t]);
    ft[t] = half ? o : z3[t];
    ft[4 + t] = half ? z3[t] : o;
  }
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const float o = shfl_xor32(z3[4 + t]);
    ft[8 + t] = half ? o : z3[4 + t];
  }
}

// Layers 1-2 of the MLP of one wave tile: z1/z2 become the post-dropout-ReLU activations a1^T,
// a2^T.  q1: hoisted layer-1 A operands.
template <bool DROP = true>
__device__ __forceinline__ void mlp12_tile(const float* Q2s, const float (&q1)[4][5], const float* u_row,
                                           const float* b2, const float (&h)[C], const uint32_t (&kw1)[4],
                                           const uint32_t (&kw2)[4], float scale, int col, int half, f32x16 (&z1)[4],
                                           f32x16 (&z2)[4]) {
  // layer 1: z1 = u[b] + Q1 h   (hidden_to_mlp(h) + U_x(x), classification.py:97)
#pragma unroll
  for (int mb = 0; mb < 4; ++mb) load_acc_rows(u_row, mb, half, z1[mb]);
#pragma unroll
  for (int s = 0; s < 5; ++s) {
    const float bs = half ? h[2 * s + 1] : h[2 * s];
#pragma unroll
    for (int mb = 0; mb < 4; ++mb) z1[mb] = mfma32(q1[mb][s], bs, z1[mb]);
  }
#pragma unroll
  for (int mb = 0; mb < 4; ++mb) dropout_relu<DROP>(z1[mb], kw1[mb], half, scale);
  // layer 2: z2 = b2 + Q2 a1
#pragma unroll
  for (int mb = 0; mb < 4; ++mb) load_acc_rows(b2, mb, half, z2[mb]);
#pragma unroll
  for (int kb = 0; kb < 4; ++kb) {
#pragma unroll
    for (int g = 0; g < 4; ++g)
#pragma unroll
      for (int mb = 0; mb < 4; ++mb) {
        const f32x4 q = *reinterpret_cast<const f32x4*>(Q2s + (32 * mb + col) * LDQ + 32 * kb + 8 * g + 4 * half);
#pragma unroll
        for (int t = 0; t < 4; ++t) z2[mb] = mfma32(q[t], z1[kb][4 * g + t], z2[mb]);
      }
    __builtin_amdgcn_sched_barrier(0);   // bound the LDS-read hoisting window to one k-block
  }
#pragma unroll
  for (int mb = 0; mb < 4; ++mb) dropout_relu<DROP>(z2[mb], kw2[mb], half, scale);
}

// The MLP of one wave tile: layers 1-3, returns the layer-3 accumulator (mlp12_tile + layer 3).
template <bool DROP = true>
__device__ __forceinline__ f32x16 mlp_tile(const float* Q2s, const float* Q3s, const float (&q1)[4][5],
                                           const float* u_row, const float* b2, const float* b3,
                                           const float (&h)[C], const uint32_t (&kw1)[4], const uint32_t (&kw2)[4],
                                           float scale, int col, int half, f32x16 (&z1)[4], f32x16 (&z2)[4]) {
  mlp12_tile<DROP>(Q2s, q1, u_row, b2, h, kw1, kw2, scale, col, half, z1, z2);
  // layer 3: z3 = b3 + Q3 a2 (rows >= 10 of the 32-row tile are zero weights)
  f32x16 z3;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int i = acc_row(r, half);
    z3[r] = i < C ? b3[i] : 0.f;
  }
#pragma unroll
  for (int kb = 0; kb < 4; ++kb)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      // rows >= C of the layer-3 A operand are zero (the image may hold only C rows)
      const f32x4 q = col < C ? *reinterpret_cast<const f32x4*>(Q3s + col * LDQ + 32 * kb + 8 * g + 4 * half)
                              : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int t = 0; t < 4; ++t) z3 = mfma32(q[t], z2[kb][4 * g + t], z3);
    }
  return z3;
}

// Stage the 128x128 mlp_to_mlp weight and the 10x128 mlp_to_hidden weight (zero rows up to
// q3_rows) into padded LDS images: 16-byte global loads, all of a thread's loads in flight
// together (a dependent 4-byte load loop took ~15 us of L2 latency at kernel start).
__device__ __forceinline__ void load_weight_images(const float* Q2, const float* Q3, float* Q2s, float* Q3s,
                                                   int q3_rows = 32) {
  const f32x4* Q2v = reinterpret_cast<const f32x4*>(Q2);
  constexpr int N2 = M * M / 4;                        // 4096 float4
  for (int e0 = threadIdx.x; e0 < N2; e0 += 8 * blockDim.x) {
    f32x4 v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int e = e0 + u * blockDim.x;
      if (e < N2) v[u] = Q2v[e];
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int e = e0 + u * blockDim.x;
      if (e < N2) *reinterpret_cast<f32x4*>(Q2s + (e >> 5) * LDQ + (e & 31) * 4) = v[u];
    }
  }
  if (Q3s) {
    const f32x4* Q3v = reinterpret_cast<const f32x4*>(Q3);
    for (int e = threadIdx.x; e < q3_rows * M / 4; e += blockDim.x) {
      const int i = e >> 5;
      *reinterpret_cast<f32x4*>(Q3s + i * LDQ + (e & 31) * 4) = i < C ? Q3v[e] : f32x4{0.f, 0.f, 0.f, 0.f};
    }
  }
}
}  // namespace fiode_tile
