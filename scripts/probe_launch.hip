// probe_launch.hip — diagnostic: what a host round trip through the GPU costs on MI355X, for the closed-loop
// Wi-Fi epoch (nsgpu_wifil), whose host waits for each epoch's close before the next launch.
//   (A) launch a 1-block kernel that writes a flag into mapped host memory; the host spins on the flag
//   (B) the same with a 10000-wave grid whose last block (a ticket) writes the flag
//   (C) a 1-block gate kernel queued beforehand spins on a "go" word the host writes, then the flag kernel
//       (queued behind it) writes the flag: the round trip without a launch on the critical path
//   (D) as (C) with the 10000-wave grid behind the gate
// Every spin is bounded (s_memrealtime, 100 MHz: 0.2 s) so no wave outlives a lost host.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <algorithm>
#include <chrono>
#include <vector>
#define CK(x)                                                           \
  do {                                                                  \
    hipError_t e = (x);                                                 \
    if (e != hipSuccess) {                                              \
      printf("%s: %s\n", #x, hipGetErrorString(e));                     \
      exit(1);                                                          \
    }                                                                   \
  } while (0)

struct Big {
  uint64_t w[64];  // (a kernel argument the size of the epoch's)
};

__global__ void k_flag(Big a, uint32_t *hflag, uint32_t seq) {
  if (threadIdx.x == 0) __hip_atomic_store(hflag, seq + (uint32_t)(a.w[0] & 0), __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}
__global__ void k_grid(Big a, uint32_t *hflag, uint32_t seq, uint32_t *ticket) {
  __shared__ uint32_t last;
  if (threadIdx.x == 0) last = (atomicAdd(ticket, 1u) == gridDim.x - 1);
  __syncthreads();
  if (last && threadIdx.x == 0) {
    *ticket = 0;
    __hip_atomic_store(hflag, seq + (uint32_t)(a.w[0] & 0), __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}
__global__ void k_gate(const uint32_t *hgo, uint32_t seq, uint32_t *timeouts) {
  if (threadIdx.x != 0) return;
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  while (__hip_atomic_load(hgo, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) != seq) {
    __builtin_amdgcn_s_sleep(1);
    if (__builtin_amdgcn_s_memrealtime() - t0 > 20000000ull) {
      atomicAdd(timeouts, 1u);
      return;
    }
  }
}

using clk = std::chrono::steady_clock;
static double us(clk::time_point a, clk::time_point b) {
  return std::chrono::duration<double, std::micro>(b - a).count();
}
static void report(const char *name, std::vector<double> &v, std::vector<double> &api) {
  std::sort(v.begin(), v.end());
  double m = 0, ma = 0;
  for (double x : v) m += x;
  for (double x : api) ma += x;
  printf("%-44s round trip us: mean %.2f p10 %.2f p50 %.2f p90 %.2f | launch API us mean %.2f\n", name, m / v.size(),
         v[v.size() / 10], v[v.size() / 2], v[v.size() * 9 / 10], api.empty() ? 0.0 : ma / api.size());
}

__global__ void k_noop(Big a, uint32_t *out) {
  if (a.w[1] == 1 && threadIdx.x == 0) out[blockIdx.x] = 1;  // (never: keeps the kernel from being empty)
}

struct Mode {
  const char *name;
  unsigned grid, block;  // 0: the 1-block flag kernel alone
  int ticket;            // 1: k_grid (last block flags); 0: k_noop then k_flag behind it
  int gate;
};

int main() {
  const int N = 2000;
  uint32_t *h, *d, *ticket, *tmo, *sink;
  CK(hipHostMalloc((void **)&h, 64, hipHostMallocMapped | hipHostMallocCoherent));
  CK(hipHostGetDevicePointer((void **)&d, h, 0));
  CK(hipMalloc(&ticket, 4));
  CK(hipMalloc(&tmo, 4));
  CK(hipMalloc(&sink, 1 << 20));
  CK(hipMemset(ticket, 0, 4));
  CK(hipMemset(tmo, 0, 4));
  volatile uint32_t *flag = h, *go = h + 16;
  uint32_t *dflag = d, *dgo = d + 16;
  h[0] = 0;
  h[16] = 0;
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  Big a{};
  uint32_t seq = 0;
  const Mode modes[] = {
      {"(A) 1 block flags", 0, 0, 0, 0},
      {"(B) 2500x256, last block (ticket) flags", 2500, 256, 1, 0},
      {"(C) gate ahead, 1 block flags", 0, 0, 0, 1},
      {"(D) gate ahead, 2500x256 ticket", 2500, 256, 1, 1},
      {"(E) no-op 10000x64, flag kernel behind", 10000, 64, 0, 0},
      {"(F) no-op 2500x256, flag kernel behind", 2500, 256, 0, 0},
      {"(G) no-op 625x1024, flag kernel behind", 625, 1024, 0, 0},
      {"(H) no-op 256x64, flag kernel behind", 256, 64, 0, 0},
      {"(I) no-op 1x64, flag kernel behind", 1, 64, 0, 0},
      {"(J) gate ahead, no-op 10000x64, flag behind", 10000, 64, 0, 1},
      {"(K) gate ahead, no-op 2500x256, flag behind", 2500, 256, 0, 1},
      {"(L) gate ahead, no-op 1x64, flag behind", 1, 64, 0, 1},
  };
  for (const Mode &m : modes) {
    std::vector<double> rt, api;
    auto enqueue = [&](uint32_t q) {
      if (m.gate) hipLaunchKernelGGL(k_gate, dim3(1), dim3(64), 0, s, dgo, q, tmo);
      if (m.grid && m.ticket) {
        hipLaunchKernelGGL(k_grid, dim3(m.grid), dim3(m.block), 0, s, a, dflag, q, ticket);
      } else {
        if (m.grid) hipLaunchKernelGGL(k_noop, dim3(m.grid), dim3(m.block), 0, s, a, sink);
        hipLaunchKernelGGL(k_flag, dim3(1), dim3(64), 0, s, a, dflag, q);
      }
    };
    CK(hipStreamSynchronize(s));
    if (m.gate) {  // two epochs queued ahead
      enqueue(seq + 1);
      enqueue(seq + 2);
    }
    for (int i = 0; i < N + 100; i++) {
      const uint32_t q = ++seq;
      const clk::time_point t0 = clk::now();
      if (m.gate) {
        *go = q;
      } else {
        enqueue(q);
      }
      const clk::time_point t1 = clk::now();
      while (*flag != q) {
      }
      const clk::time_point t2 = clk::now();
      if (m.gate) enqueue(q + 2);  // (the host's wait for the next epoch hides this)
      if (i >= 100) {
        rt.push_back(us(t0, t2));
        if (!m.gate) api.push_back(us(t0, t1));
      }
    }
    if (m.gate) {  // release the two queued gates
      *go = seq + 1;
      while (*flag != seq + 1) {
      }
      *go = seq + 2;
      seq += 2;
    }
    CK(hipStreamSynchronize(s));
    report(m.name, rt, api);
  }
  uint32_t t = 0;
  CK(hipMemcpy(&t, tmo, 4, hipMemcpyDeviceToHost));
  printf("gate timeouts: %u\n", t);
  return 0;
}
