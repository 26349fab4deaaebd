// probe_graph.hip — diagnostic: does a hipGraph run a side branch concurrently with the main chain, and
// what does a cross-branch join cost?  Per "window": a main chain of spin kernels (a, b, c[, d]); variant
// SIDE forks s(n) after a(n+1) on a second captured stream and joins it before a(n+2) — the shape a
// deferred per-window scan would have.  Spin kernels hold their blocks for T us (s_memrealtime, 100 MHz).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <stdlib.h>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

__global__ void spin(uint32_t ticks, uint32_t *sink) {
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  uint32_t x = 0;
  while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) x++;
  if (x == 0xffffffffu) sink[0] = x;
}

static float run(hipGraphExec_t ge, hipStream_t s, int reps) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int i = 0; i < 3; i++) CK(hipGraphLaunch(ge, s));
  CK(hipStreamSynchronize(s));
  CK(hipEventRecord(a, s));
  for (int i = 0; i < reps; i++) CK(hipGraphLaunch(ge, s));
  CK(hipEventRecord(b, s));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  return ms;
}

int main(int argc, char **argv) {
  const int NW = 32, REPS = 20;
  const uint32_t T = argc > 1 ? atoi(argv[1]) : 8;   // us per main kernel
  const uint32_t TS = argc > 2 ? atoi(argv[2]) : 12;  // us of the side kernel
  uint32_t *sink;
  CK(hipMalloc(&sink, 64));
  hipStream_t s, s2;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
  hipEvent_t ev[2 * NW + 4];
  for (int i = 0; i < 2 * NW + 4; i++) CK(hipEventCreateWithFlags(&ev[i], hipEventDisableTiming));
  for (int variant = 0; variant < 5; variant++) {
    // 0: a,b,c,d chain   1: a,b,c chain   2: a,b,c + side s(n) (fork after a(n+1), join before a(n+2))
    // 3: a,b,c + side s(n) forked after a(n+1), joined only at the end of the graph
    // 4: a,b,c with s inline after a (a,s,b,c)
    hipGraph_t g;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
    int ne = 0;
    hipEvent_t pend_join = nullptr;
    for (int w = 0; w < NW; w++) {
      if (variant == 2 && pend_join) CK(hipStreamWaitEvent(s, pend_join, 0));
      hipLaunchKernelGGL(spin, dim3(256), dim3(256), 0, s, T * 100, sink);
      if (variant == 4) hipLaunchKernelGGL(spin, dim3(1), dim3(1024), 0, s, TS * 100, sink);
      if ((variant == 2 || variant == 3) && w > 0) {
        hipEvent_t f = ev[ne++];
        CK(hipEventRecord(f, s));
        CK(hipStreamWaitEvent(s2, f, 0));
        hipLaunchKernelGGL(spin, dim3(1), dim3(1024), 0, s2, TS * 100, sink);
        hipEvent_t j = ev[ne++];
        CK(hipEventRecord(j, s2));
        pend_join = j;
      }
      hipLaunchKernelGGL(spin, dim3(1024), dim3(64), 0, s, T * 100, sink);
      hipLaunchKernelGGL(spin, dim3(1024), dim3(256), 0, s, T * 100, sink);
      if (variant == 0) hipLaunchKernelGGL(spin, dim3(1), dim3(1024), 0, s, T * 100, sink);
    }
    if ((variant == 2 || variant == 3) && pend_join) CK(hipStreamWaitEvent(s, pend_join, 0));
    CK(hipStreamEndCapture(s, &g));
    size_t nn = 0;
    CK(hipGraphGetNodes(g, nullptr, &nn));
    hipGraphExec_t ge;
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    const float ms = run(ge, s, REPS);
    printf("variant %d: T=%u TS=%u  nodes %zu  %.2f us per window\n", variant, T, TS, nn, ms * 1000.f / (REPS * NW));
    CK(hipGraphExecDestroy(ge));
    CK(hipGraphDestroy(g));
  }
  return 0;
}
