// Probe: semantics of the gfx950 cross-lane primitives used by the wave sort (run on the GPU box).
#include <hip/hip_runtime.h>
#include <stdio.h>
__global__ void k(unsigned *out) {
  const unsigned v = threadIdx.x;
  out[0 * 64 + v] = __builtin_amdgcn_mov_dpp(v, 0xB1, 0xf, 0xf, false);
  out[1 * 64 + v] = __builtin_amdgcn_mov_dpp(v, 0x4E, 0xf, 0xf, false);
  out[2 * 64 + v] = __builtin_amdgcn_mov_dpp(v, 0x104, 0xf, 0xf, false);
  out[3 * 64 + v] = __builtin_amdgcn_mov_dpp(v, 0x114, 0xf, 0xf, false);
  out[4 * 64 + v] = __builtin_amdgcn_mov_dpp(v, 0x128, 0xf, 0xf, false);
  out[5 * 64 + v] = __builtin_amdgcn_ds_swizzle(v, 0x401f);
  auto r = __builtin_amdgcn_permlane16_swap(v, v, false, false);
  out[6 * 64 + v] = r[0];
  out[7 * 64 + v] = r[1];
  auto s = __builtin_amdgcn_permlane32_swap(v, v, false, false);
  out[8 * 64 + v] = s[0];
  out[9 * 64 + v] = s[1];
}
int main() {
  unsigned *d, h[640];
  hipMalloc(&d, sizeof(h));
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
  hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  const char *nm[] = {"qp B1", "qp 4E", "row_shl4", "row_shr4", "row_ror8", "swz x16", "pl16 r0", "pl16 r1", "pl32 r0", "pl32 r1"};
  for (int t = 0; t < 10; t++) {
    printf("%-9s", nm[t]);
    for (int i = 0; i < 64; i++) printf(" %d", h[t * 64 + i]);
    printf("\n");
  }
  return 0;
}
