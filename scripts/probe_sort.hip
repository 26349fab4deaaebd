// Probe: cycle cost of the workgroup window sort (run_rank_sort) in isolation, 512 threads.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include "../ns-3-dev-dnemu_amd/csrc/nsgpu_sort.h"
using namespace nsgpu;
#ifndef ALG
#define ALG 1
#endif
__global__ __launch_bounds__(512) void k(const uint64_t *in, uint32_t n, uint64_t *out, uint64_t *cyc, int reps) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  SortLds &L = *reinterpret_cast<SortLds *>(smem);
  uint64_t t0 = 0, acc = 0;
  for (int r = 0; r < reps; r++) {
    for (int i = threadIdx.x; i < (int)n; i += 512) {
      L.k[0][i] = in[i];
      L.v[0][i] = i;
    }
    __syncthreads();
    t0 = __builtin_amdgcn_s_memtime();
    if (ALG == 0) run_rank_sort<512>(L, n);
    else merge_sort<512>(L, n);
    acc += __builtin_amdgcn_s_memtime() - t0;
  }
  for (int i = threadIdx.x; i < (int)n; i += 512) out[i] = L.k[0][i];
  if (threadIdx.x == 0) cyc[0] = acc / reps;
}
int main(int argc, char **argv) {
  const uint32_t n = argc > 1 ? atoi(argv[1]) : 2000;
  const int distinct = argc > 2 ? atoi(argv[2]) : 8;
  uint64_t *h = (uint64_t *)malloc(8 * n), *o = (uint64_t *)malloc(8 * n);
  srand(1);
  for (uint32_t i = 0; i < n; i++) h[i] = ((uint64_t)(rand() % distinct) << 32) | (uint32_t)(i * 7919u % 100003u);
  uint64_t *din, *dout, *dc, c;
  hipMalloc(&din, 8 * n); hipMalloc(&dout, 8 * n); hipMalloc(&dc, 8);
  hipMemcpy(din, h, 8 * n, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(1), dim3(512), sizeof(SortLds), 0, din, n, dout, dc, 20);
  hipMemcpy(o, dout, 8 * n, hipMemcpyDeviceToHost);
  hipMemcpy(&c, dc, 8, hipMemcpyDeviceToHost);
  int ok = 1;
  for (uint32_t i = 1; i < n; i++) ok &= o[i - 1] < o[i];
  printf("alg %d n %u distinct %d: sorted %d, %llu cycles/sort\n", ALG, n, distinct, ok, (unsigned long long)c);
  return 0;
}
