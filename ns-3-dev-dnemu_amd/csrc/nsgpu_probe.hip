// nsgpu_probe.hip — the latency constants of the window pipeline's roofline (include/nsgpu.h
// nsgpu_probe_latency).  The p2p window is a chain of small kernels, each a few dependent memory trips
// long: its speed of light is (boundaries x boundary cost) + (dependent trips x trip latency), not HBM
// bandwidth.  Both constants are measured here, the way the pipeline meets them:
//  * boundary: an empty 64-block kernel replayed 64 times from a graph (us per kernel);
//  * trip: 64 blocks chase pointers through a 128-MB table (random jumps: every level is a line no L2 holds,
//    served from the Infinity Cache or HBM, as the window kernels' reads of the previous kernel's writes are).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <vector>

#include "nsgpu.h"
#include "nsgpu_internal.h"

namespace nsgpu {
namespace {
constexpr int PN = 1 << 25;  // chain table entries (128 MB: 32x the L2s)
constexpr int LV = 32;       // chase levels per launch

__global__ __launch_bounds__(64) void k_probe_chase(uint32_t *buf, int levels, uint32_t salt) {
  const uint32_t tid = blockIdx.x * 64 + threadIdx.x;
  uint32_t x = (uint32_t)(((uint64_t)(tid + 1) * 0x9e3779b97f4a7c15ull + salt * 0x632be59bd9b4e019ull) >> 39) % PN;
  for (int l = 0; l < levels; l++) x = buf[x];
  if (x == 0xffffffffu) buf[0] = 1;  // (keeps the chain live)
}
}  // namespace
}  // namespace nsgpu

using namespace nsgpu;

extern "C" int nsgpu_probe_latency(void *stream, double *boundary_us, double *trip_us) {
  if (!boundary_us || !trip_us) return set_error(NSGPU_EINVAL, "nsgpu_probe_latency: null");
  hipStream_t s = (hipStream_t)stream;
  uint32_t *buf = nullptr;
  hipStream_t cs = nullptr;
  hipEvent_t a = nullptr, b = nullptr;
  hipGraph_t g[3] = {nullptr, nullptr, nullptr};
  hipGraphExec_t ge[3] = {nullptr, nullptr, nullptr};
  float ms[3] = {0, 0, 0};
  constexpr int NK = 64, REPS = 20;
  std::vector<uint32_t> h(PN);
  for (int i = 0; i < PN; i++) {  // a random jump per entry
    uint64_t z = (uint64_t)i * 0x9e3779b97f4a7c15ull + 0x2545f4914f6cdd1dull;
    z = (z ^ (z >> 31)) * 0xbf58476d1ce4e5b9ull;
    h[i] = (uint32_t)((z ^ (z >> 29)) % PN);
  }
  hipError_t e = hipSuccess;
  const char *what = "";
#define PROBE(x, w)                  \
  if (e == hipSuccess) {             \
    e = (x);                         \
    if (e != hipSuccess) what = (w); \
  }
  PROBE(hipMalloc(&buf, PN * sizeof(uint32_t)), "hipMalloc");
  PROBE(hipMemcpy(buf, h.data(), PN * sizeof(uint32_t), hipMemcpyHostToDevice), "copy");
  PROBE(hipEventCreate(&a), "event");
  PROBE(hipEventCreate(&b), "event");
  PROBE(hipStreamCreateWithFlags(&cs, hipStreamNonBlocking), "stream");
  // v = 0: empty kernels; v = 1: the same (the chase's baseline); v = 2: LV levels each
  for (int v = 0; v < 3 && e == hipSuccess; v++) {
    PROBE(hipStreamBeginCapture(cs, hipStreamCaptureModeThreadLocal), "capture");
    if (e != hipSuccess) break;
    for (int k = 0; k < NK; k++)
      hipLaunchKernelGGL(k_probe_chase, dim3(64), dim3(64), 0, cs, buf, v == 2 ? LV : 0, (uint32_t)k);
    hipError_t ec = hipStreamEndCapture(cs, &g[v]);
    PROBE(ec, "capture end");
    PROBE(hipGraphInstantiate(&ge[v], g[v], nullptr, nullptr, 0), "instantiate");
    for (int r = 0; r < 3; r++) PROBE(hipGraphLaunch(ge[v], s), "launch");
    PROBE(hipEventRecord(a, s), "record");
    for (int r = 0; r < REPS; r++) PROBE(hipGraphLaunch(ge[v], s), "launch");
    PROBE(hipEventRecord(b, s), "record");
    PROBE(hipEventSynchronize(b), "run");
    PROBE(hipEventElapsedTime(&ms[v], a, b), "elapsed");
  }
#undef PROBE
  for (int v = 0; v < 3; v++) {
    if (ge[v]) (void)hipGraphExecDestroy(ge[v]);
    if (g[v]) (void)hipGraphDestroy(g[v]);
  }
  if (a) (void)hipEventDestroy(a);
  if (b) (void)hipEventDestroy(b);
  if (cs) (void)hipStreamDestroy(cs);
  if (buf) (void)hipFree(buf);
  (void)hipGetLastError();  // (nothing of the probe's is left as the thread's last error)
  if (e != hipSuccess) return set_error(NSGPU_EHIP, "nsgpu_probe_latency: %s: %s", what, hipGetErrorString(e));
  const double per0 = 1e3 * ms[0] / (NK * REPS), per1 = 1e3 * ms[1] / (NK * REPS), per2 = 1e3 * ms[2] / (NK * REPS);
  *boundary_us = per0;
  *trip_us = std::max(0.0, (per2 - per1) / LV);
  return NSGPU_OK;
}
