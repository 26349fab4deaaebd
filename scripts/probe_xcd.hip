// probe_xcd.hip — diagnostic: does a line written by one kernel read faster in the next kernel on the XCD that
// wrote it?  Kernel W: block b writes a pointer chain through its own 256 lines (128 B apart, shuffled) with
// plain stores and records its XCC id.  Kernel R (the next launch): block b chases the chain of block
// (b + shift) % NB, one lane, dependent loads; the chase time / 256 is the load latency.  Blocks whose source
// was written on their own XCD and on another XCD are reported apart (placement is read, not assumed).  The
// values are checked (a stale line would break the chain).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>
#define CK(x)                                                           \
  do {                                                                  \
    hipError_t e = (x);                                                 \
    if (e != hipSuccess) {                                              \
      printf("%s: %s\n", #x, hipGetErrorString(e));                     \
      exit(1);                                                          \
    }                                                                   \
  } while (0)

constexpr int NB = 512, L = 256, STRIDE = 32;  // blocks, lines per block, words (4 B) per line

__device__ __forceinline__ uint32_t xcc_id() {
  uint32_t v;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(v));
  return v;
}

// perm: L entries per block (host-made shuffle); buf[b][line * STRIDE] = next line index + tag
__global__ void k_write(uint32_t *buf, const uint16_t *perm, uint32_t tag, uint32_t *wx) {
  const uint32_t b = blockIdx.x;
  for (uint32_t i = threadIdx.x; i < (uint32_t)L; i += blockDim.x) {
    const uint32_t cur = perm[b * L + i], nxt = perm[b * L + (i + 1) % L];
    buf[((uint64_t)b * L + cur) * STRIDE] = nxt | (tag << 16);
  }
  if (threadIdx.x == 0) wx[b] = xcc_id();
}
__global__ void k_read(const uint32_t *buf, const uint16_t *perm, uint32_t tag, int shift, uint64_t *out,
                       uint32_t *rx, uint32_t *bad) {
  const uint32_t b = blockIdx.x, src = (b + shift) % NB;
  if (threadIdx.x != 0) return;
  rx[b] = xcc_id();
  uint32_t x = perm[src * L];
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  uint32_t nbad = 0;
  for (int l = 0; l < L; l++) {
    const uint32_t v = __builtin_nontemporal_load(&buf[((uint64_t)src * L + x) * STRIDE]);
    if ((v >> 16) != tag) nbad++;
    x = v & 0xffffu;
    x = x < (uint32_t)L ? x : 0u;
  }
  const uint64_t t1 = __builtin_amdgcn_s_memrealtime();
  out[b] = t1 - t0;
  if (nbad) atomicAdd(bad, nbad);
}
// every block reads every line once (puts stale copies into every XCD's L2 before the next write)
__global__ void k_touch(const uint32_t *buf, uint32_t *sink) {
  uint32_t acc = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < (uint64_t)NB * L; i += (uint64_t)gridDim.x * blockDim.x)
    acc += buf[i * STRIDE];
  if (acc == 0x12345678u) sink[0] = acc;
}

int main() {
  uint32_t *buf, *wx, *rx, *bad, *sink;
  uint16_t *perm;
  uint64_t *out;
  CK(hipMalloc(&buf, (size_t)NB * L * STRIDE * 4));
  CK(hipMalloc(&perm, (size_t)NB * L * 2));
  CK(hipMalloc(&wx, NB * 4));
  CK(hipMalloc(&rx, NB * 4));
  CK(hipMalloc(&bad, 4));
  CK(hipMalloc(&sink, 4));
  CK(hipMalloc(&out, NB * 8));
  CK(hipMemset(bad, 0, 4));
  std::vector<uint16_t> hp((size_t)NB * L);
  srand(7);
  for (int b = 0; b < NB; b++) {
    for (int i = 0; i < L; i++) hp[b * L + i] = (uint16_t)i;
    for (int i = L - 1; i > 0; i--) {
      const int j = rand() % (i + 1);
      std::swap(hp[b * L + i], hp[b * L + j]);
    }
  }
  CK(hipMemcpy(perm, hp.data(), hp.size() * 2, hipMemcpyHostToDevice));
  std::vector<uint32_t> hw(NB), hr(NB);
  std::vector<uint64_t> ho(NB);
  const int shifts[] = {0, 1, 8, 3};
  for (int touch = 0; touch < 2; touch++)
    for (int si = 0; si < 4; si++) {
      double same = 0, cross = 0;
      int ns = 0, nc = 0;
      for (int it = 0; it < 20; it++) {
        const uint32_t tag = (uint32_t)(1 + (it + si * 20 + touch * 80) % 60000);
        if (touch) hipLaunchKernelGGL(k_touch, dim3(1024), dim3(256), 0, 0, buf, sink);
        hipLaunchKernelGGL(k_write, dim3(NB), dim3(256), 0, 0, buf, perm, tag, wx);
        hipLaunchKernelGGL(k_read, dim3(NB), dim3(64), 0, 0, buf, perm, tag, shifts[si], out, rx, bad);
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(hw.data(), wx, NB * 4, hipMemcpyDeviceToHost));
        CK(hipMemcpy(hr.data(), rx, NB * 4, hipMemcpyDeviceToHost));
        CK(hipMemcpy(ho.data(), out, NB * 8, hipMemcpyDeviceToHost));
        if (it < 2) continue;
        for (int b = 0; b < NB; b++) {
          const int src = (b + shifts[si]) % NB;
          const double ns_per = ho[b] * 10.0 / L;
          if (hr[b] == hw[src]) same += ns_per, ns++;
          else cross += ns_per, nc++;
        }
      }
      printf("touch %d shift %d: same-XCD reads %5d blocks %7.1f ns/load | cross-XCD %5d blocks %7.1f ns/load\n", touch,
             shifts[si], ns, ns ? same / ns : 0.0, nc, nc ? cross / nc : 0.0);
    }
  uint32_t hb = 0;
  CK(hipMemcpy(&hb, bad, 4, hipMemcpyDeviceToHost));
  printf("stale values read: %u\n", hb);
  return 0;
}
