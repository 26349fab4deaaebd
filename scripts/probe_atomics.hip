// probe_atomics.hip — diagnostic: what the p2p window kernels' same-word device-scope atomics cost.
// A 256 x 256 grid (k2_pa's shape) where (a) every block folds a min into two shared words (publish_min),
// (b) `nw` waves each add to two shared counters (window slot / fresh-buffer allocation), (c) 64 waves
// add a digest; against the same kernel with per-block partial slots (plain stores) instead.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <stdlib.h>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

__global__ __launch_bounds__(256) void k(unsigned long long *w, unsigned long long *part, int mode, int nw) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int gw = blockIdx.x * 4 + wid;
  unsigned long long v = 1000000ull + (blockIdx.x * 7919u + threadIdx.x) % 4096u;
  for (int o = 32; o > 0; o >>= 1) {
    unsigned long long x = __shfl_xor(v, o);
    v = x < v ? x : v;
  }
  __shared__ unsigned long long s[4];
  if (lane == 0) s[wid] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long m = s[0];
    for (int i = 1; i < 4; i++) m = s[i] < m ? s[i] : m;
    if (mode & 1) {
      atomicMin(&w[0], m);
      atomicMin(&w[1], m + 5);
    } else {
      part[blockIdx.x * 2] = m;
      part[blockIdx.x * 2 + 1] = m + 5;
    }
  }
  if ((mode & 2) && lane == 0 && gw < nw) {
    unsigned long long a = atomicAdd(&w[2], 3ull);
    unsigned long long b = atomicAdd(&w[3], 2ull);
    if (a == 0xffffffffffffull && b == 1) w[5] = 1;
  }
  if ((mode & 4) && lane == 0 && gw < 64) atomicAdd(&w[4], v);
}

int main() {
  unsigned long long *w, *part;
  CK(hipMalloc(&w, 64));
  CK(hipMalloc(&part, 256 * 16));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int modes[] = {0, 1, 2, 4, 7, 6};
  for (int nw : {64, 170, 512}) {
    for (int mode : modes) {
      for (int rep = 0; rep < 3; rep++) k<<<256, 256>>>(w, part, mode, nw);
      CK(hipDeviceSynchronize());
      const int N = 200;
      CK(hipEventRecord(e0));
      for (int rep = 0; rep < N; rep++) k<<<256, 256>>>(w, part, mode, nw);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      printf("nw=%3d mode=%d (min-atomics %d, alloc-atomics %d, digest-atomics %d): %.2f us per kernel\n", nw, mode,
             mode & 1, (mode >> 1) & 1, (mode >> 2) & 1, 1e3 * ms / N);
    }
  }
  return 0;
}
