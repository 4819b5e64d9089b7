// Does a CU-masked HIP stream (hipExtStreamCreateWithCUMask) keep its mask when its work is
// captured into a hipGraph and replayed?  (tools/probes; not a test -- VERDICT r05 item 3 asks for
// the answer before placing the train_ode solve on one XCD.)  Each workgroup of a 1024-block grid
// records its XCC_ID and HW_ID (CU / SH / SE); the probe counts the distinct CUs used by
//   (1) a plain stream, (2) a stream masked to the first 32 mask bits, eager, (3) the same masked
// stream captured into a graph and replayed, (4) a masked stream captured while the capture ORIGIN is
// a plain stream that forks to it (the way torch side streams join a capture).
// hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/probes/cumask_probe.hip -o tools/probes/cumask_probe.bin
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <cstdio>
#include <set>
#include <vector>

__global__ void k_where(unsigned* out) {
  if (threadIdx.x == 0) {
    unsigned xcc, hw;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    out[2 * blockIdx.x] = xcc;
    out[2 * blockIdx.x + 1] = hw;
  }
  // keep the workgroup busy a little so the grid spreads
  float x = threadIdx.x;
  for (int i = 0; i < 2000; ++i) x = x * 0.999f + 1.0f;
  if (x == -1.f) out[0] = 0;
}

static void report(const char* what, const unsigned* h, int n) {
  std::set<unsigned> cus, xccs;
  for (int b = 0; b < n; ++b) {
    const unsigned xcc = h[2 * b] & 0xF, hw = h[2 * b + 1];
    const unsigned cu = (hw >> 8) & 0xF, sh = (hw >> 12) & 1, se = (hw >> 13) & 7;
    cus.insert((xcc << 16) | (se << 8) | (sh << 4) | cu);
    xccs.insert(xcc);
  }
  printf("%-40s distinct CUs %3zu, XCDs %zu:", what, cus.size(), xccs.size());
  for (unsigned x : xccs) printf(" %u", x);
  printf("\n");
}

int main() {
  const int n = 1024;
  unsigned *d, *h = new unsigned[2 * n];
  hipMalloc(&d, 2 * n * sizeof(unsigned));
  hipStream_t plain, masked, masked2, origin;
  hipStreamCreate(&plain);
  hipStreamCreate(&origin);
  std::vector<uint32_t> mask(8, 0u);
  mask[0] = 0xFFFFFFFFu;                       // the first 32 mask bits
  if (hipExtStreamCreateWithCUMask(&masked, (uint32_t)mask.size(), mask.data()) != hipSuccess) {
    printf("hipExtStreamCreateWithCUMask failed\n");
    return 1;
  }
  hipExtStreamCreateWithCUMask(&masked2, (uint32_t)mask.size(), mask.data());
  auto run = [&](hipStream_t s, const char* what) {
    hipMemsetAsync(d, 0xFF, 2 * n * sizeof(unsigned), s);
    hipLaunchKernelGGL(k_where, dim3(n), dim3(256), 0, s, d);
    hipStreamSynchronize(s);
    hipMemcpy(h, d, 2 * n * sizeof(unsigned), hipMemcpyDeviceToHost);
    report(what, h, n);
  };
  run(plain, "plain stream");
  run(masked, "masked stream (eager)");
  // captured on the masked stream itself
  hipGraph_t g;
  hipGraphExec_t ge;
  hipStreamBeginCapture(masked, hipStreamCaptureModeThreadLocal);
  hipLaunchKernelGGL(k_where, dim3(n), dim3(256), 0, masked, d);
  hipStreamEndCapture(masked, &g);
  hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
  hipMemset(d, 0xFF, 2 * n * sizeof(unsigned));
  hipGraphLaunch(ge, plain);
  hipStreamSynchronize(plain);
  hipMemcpy(h, d, 2 * n * sizeof(unsigned), hipMemcpyDeviceToHost);
  report("graph captured on masked, launched plain", h, n);
  hipGraphLaunch(ge, masked);
  hipStreamSynchronize(masked);
  hipMemcpy(h, d, 2 * n * sizeof(unsigned), hipMemcpyDeviceToHost);
  report("graph captured on masked, launched masked", h, n);
  // origin plain, forked to masked2 (event join), joined back
  hipEvent_t e1, e2;
  hipEventCreate(&e1);
  hipEventCreate(&e2);
  hipGraph_t g2;
  hipGraphExec_t ge2;
  hipStreamBeginCapture(origin, hipStreamCaptureModeThreadLocal);
  hipEventRecord(e1, origin);
  hipStreamWaitEvent(masked2, e1, 0);
  hipLaunchKernelGGL(k_where, dim3(n), dim3(256), 0, masked2, d);
  hipEventRecord(e2, masked2);
  hipStreamWaitEvent(origin, e2, 0);
  hipStreamEndCapture(origin, &g2);
  hipGraphInstantiate(&ge2, g2, nullptr, nullptr, 0);
  hipMemset(d, 0xFF, 2 * n * sizeof(unsigned));
  hipGraphLaunch(ge2, plain);
  hipStreamSynchronize(plain);
  hipMemcpy(h, d, 2 * n * sizeof(unsigned), hipMemcpyDeviceToHost);
  report("fork to masked inside a plain capture", h, n);
  // how mask bits map to XCDs: every 8th bit (i % 8 == 0), and its complement
  for (int pat = 0; pat < 3; ++pat) {
    std::vector<uint32_t> m(8, 0u);
    for (int i = 0; i < 256; ++i) {
      const bool on = pat == 0 ? (i % 8 == 0) : pat == 1 ? (i % 8 != 0) : (i / 32 != 0);
      if (on) m[i / 32] |= 1u << (i % 32);
    }
    hipStream_t s;
    if (hipExtStreamCreateWithCUMask(&s, (uint32_t)m.size(), m.data()) != hipSuccess) {
      printf("mask pattern %d refused\n", pat);
      continue;
    }
    run(s, pat == 0 ? "mask bits i%8==0 (eager)" : pat == 1 ? "mask bits i%8!=0 (eager)" : "mask bits 32..255 (eager)");
  }
  return 0;
}
