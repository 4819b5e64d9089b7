// Internal (not exported) entry shared by the training-step and ODE-training kernels: weight
// gradients of the Cayley-MLP dynamics summed over rows r = b*S + s, from the per-row
// activations and activation gradients (the k_lyap_wgrad / k_lyap_reduce / k_lyap_static_grads
// chain of lyap.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>

#include "../../include/fiode.h"

namespace fiode_internal {
struct WgradIO {
  int B, S;                       // rows r = b*S + s
  const float* x_feat;            // [B][X]
  const float* Qx;                // [M][X]
  const float* h;                 // [B*S][C] layer-1 inputs
  const float *a1, *a2;           // [B*S][M] post-dropout-ReLU activations
  const float *gz2, *gz1;         // [B*S][M] gradients at the layer-2 / layer-1 pre-activations
  const float* gft;               // [B*S][C] gradient at the MLP output
  void* workspace;                // wgrad_bytes(B, S, s_used == nullptr)
  const int32_t* s_used;          // optional device count: only rows s < s_used[0] of each image count
  fiode_lyap_grads grads;         // outputs (all overwritten)
};
size_t wgrad_bytes(int B, int S, bool exact_rows);   // exact_rows: S rows per image (else a bound, s_used set)
int launch_wgrad(hipStream_t st, const WgradIO& io);
}  // namespace fiode_internal
