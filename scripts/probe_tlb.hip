// probe_tlb.hip — diagnostic: the latency of one dependent global load on MI355X by where the line and its
// translation sit: (A) lines of one 64 KB block, caches flushed (HBM latency, translation cached);
// (B) every level on another 2 MB page of a 4 GB buffer, caches flushed (+ translation misses);
// (C) the same chain as (B) run again at once (lines and translations warm); (D) every level on another
// 4 KB page of one 2 MB page, flushed.  One lane chases; s_memrealtime (100 MHz) brackets the chain.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#define CK(x)                                                           \
  do {                                                                  \
    hipError_t e = (x);                                                 \
    if (e != hipSuccess) {                                              \
      printf("%s: %s\n", #x, hipGetErrorString(e));                     \
      exit(1);                                                          \
    }                                                                   \
  } while (0)

__global__ void chase(const uint64_t *buf, uint64_t start, int L, uint64_t *out) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  uint64_t x = start;
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  for (int l = 0; l < L; l++) x = __builtin_nontemporal_load(&buf[x]);
  const uint64_t t1 = __builtin_amdgcn_s_memrealtime();
  out[0] = t1 - t0;
  out[1] = x;
}

// streams `n` words (evicts L2 / MALL lines and many translations)
__global__ void flush(uint64_t *b, uint64_t n) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    b[i] += 1;
}

int main() {
  const uint64_t BYTES = 4ull << 30, NW = BYTES / 8;
  uint64_t *buf, *out, *fl;
  CK(hipMalloc(&buf, BYTES));
  CK(hipMalloc(&fl, 1ull << 30));
  CK(hipMalloc(&out, 64));
  CK(hipMemset(fl, 0, 1ull << 30));
  const int L = 16;
  uint64_t *h = (uint64_t *)calloc(NW, 8);
  // chain A: 16 lines 4 KB apart inside one 64 KB block
  // chain B: levels 2 MB + 4 KB apart over the 4 GB buffer (distinct 2 MB pages, spread)
  // chain D: levels 4 KB apart inside one 2 MB page
  const uint64_t a0 = 0, b0 = 8ull << 20, d0 = 460ull << 20;  // (word indices)
  for (int l = 0; l < L; l++) {
    h[a0 + (uint64_t)l * 512] = a0 + (uint64_t)(l + 1) * 512;  // 4 KB apart (inside 64 KB)
    h[b0 + (uint64_t)l * ((200ull << 20) / 8)] = b0 + (uint64_t)(l + 1) * ((200ull << 20) / 8);  // 200 MB apart
    h[d0 + (uint64_t)l * 512 * 3] = d0 + (uint64_t)(l + 1) * 512 * 3;                            // 12 KB apart
  }
  CK(hipMemcpy(buf, h, BYTES, hipMemcpyHostToDevice));
  uint64_t r[2];
  const char *names[3] = {"A: one 64 KB block, flushed", "B: a new 2 MB page per level (200 MB apart), flushed",
                          "D: a new 4 KB page per level inside 2 MB, flushed"};
  const uint64_t starts[3] = {a0, b0, d0};
  for (int rep = 0; rep < 3; rep++)
    for (int c = 0; c < 3; c++) {
      hipLaunchKernelGGL(flush, dim3(2048), dim3(256), 0, 0, fl, (1ull << 30) / 8);
      CK(hipDeviceSynchronize());
      hipLaunchKernelGGL(chase, dim3(1), dim3(64), 0, 0, buf, starts[c], L, out);
      CK(hipDeviceSynchronize());
      CK(hipMemcpy(r, out, 16, hipMemcpyDeviceToHost));
      const double cold = r[0] * 10.0 / L;
      hipLaunchKernelGGL(chase, dim3(1), dim3(64), 0, 0, buf, starts[c], L, out);
      CK(hipDeviceSynchronize());
      CK(hipMemcpy(r, out, 16, hipMemcpyDeviceToHost));
      printf("rep %d %-55s cold %7.1f ns/level, warm (again at once) %7.1f ns/level\n", rep, names[c], cold,
             r[0] * 10.0 / L);
    }
  return 0;
}
