// probe_latency.hip — diagnostic: what a dependent global-load level and a kernel boundary cost on
// this GPU, for tiny latency-bound kernels like the p2p window pipeline's.
// (a) K back-to-back launches of a 64-block kernel whose thread chases a pointer chain of length L
//     through a buffer the previous launch rewrote (from other blocks, i.e. other XCDs / L2s);
// (b) the same with L = 0 (launch + boundary only); (c) in-kernel s_memrealtime per level.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <stdlib.h>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

__global__ void chase(uint32_t *buf, int L, int n, uint64_t *ticks, int rewrite) {
  const uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x;
  uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  uint32_t x = tid % n;
  for (int l = 0; l < L; l++) x = buf[x];
  uint64_t t1 = __builtin_amdgcn_s_memrealtime();
  if (rewrite) buf[(tid * 7919u) % n] = (buf[(tid * 7919u) % n] + 0u);  // dirty lines for the next launch
  if (threadIdx.x == 0 && blockIdx.x == 0) ticks[0] += (t1 - t0);
  if (x == 0xffffffffu) buf[0] = 1;  // keep the chain live
}

__global__ void clk(uint64_t *out) {
  if (threadIdx.x == 0) {
    out[0] = __builtin_amdgcn_s_memrealtime();
    out[1] = __builtin_amdgcn_s_memtime();
  }
}

int main() {
  const int n = 1 << 16;
  uint32_t *buf;
  uint64_t *ticks;
  CK(hipMalloc(&buf, n * 4));
  CK(hipMalloc(&ticks, 64));
  uint32_t *h = (uint32_t *)malloc(n * 4);
  for (int i = 0; i < n; i++) h[i] = (uint32_t)((i * 40503ull + 12345) % n);  // a permutation-ish chain
  CK(hipMemcpy(buf, h, n * 4, hipMemcpyHostToDevice));
  hipStream_t s;
  CK(hipStreamCreate(&s));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  // clock rates: s_memrealtime is 100 MHz
  uint64_t *o;
  CK(hipMalloc(&o, 32));
  const int K = 2000;
  for (int rewrite = 0; rewrite < 2; rewrite++)
    for (int L : {0, 1, 2, 4, 8, 16}) {
      CK(hipMemset(ticks, 0, 64));
      for (int w = 0; w < 50; w++) hipLaunchKernelGGL(chase, dim3(64), dim3(64), 0, s, buf, L, n, ticks, rewrite);
      CK(hipMemset(ticks, 0, 64));
      CK(hipEventRecord(a, s));
      for (int k = 0; k < K; k++) hipLaunchKernelGGL(chase, dim3(64), dim3(64), 0, s, buf, L, n, ticks, rewrite);
      CK(hipEventRecord(b, s));
      CK(hipEventSynchronize(b));
      float ms;
      CK(hipEventElapsedTime(&ms, a, b));
      uint64_t t;
      CK(hipMemcpy(&t, ticks, 8, hipMemcpyDeviceToHost));
      printf("rewrite=%d L=%2d: %.2f us per launch (event span), in-kernel chain %.3f us (%.3f us/level)\n", rewrite, L,
             1e3 * ms / K, t / 100.0 / K, L ? t / 100.0 / K / L : 0.0);
    }
  // graph of the same: 64 launches per replay
  for (int L : {0, 4}) {
    hipGraph_t g;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
    for (int k = 0; k < 64; k++) hipLaunchKernelGGL(chase, dim3(64), dim3(64), 0, s, buf, L, n, ticks, 1);
    CK(hipStreamEndCapture(s, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    for (int r = 0; r < 5; r++) CK(hipGraphLaunch(ge, s));
    CK(hipEventRecord(a, s));
    for (int r = 0; r < 50; r++) CK(hipGraphLaunch(ge, s));
    CK(hipEventRecord(b, s));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    printf("graph L=%d: %.2f us per kernel\n", L, 1e3 * ms / (50 * 64));
  }
  return 0;
}
