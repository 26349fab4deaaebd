// nsgpu_sort.h — workgroup-wide bitonic sort of SORT_N = 4096 (u64 key, u32 value) pairs.
//
// Layout for a workgroup of THREADS threads (E = SORT_N / THREADS elements per lane): wave w owns
// elements [64 E w, 64 E (w + 1)); lane l holds element 64 E w + 64 q + l in register slot q.
// Stages with j < 64 exchange through wave shuffles, stages with 64 <= j < 64 E swap between the
// lane's own registers (compile-time slots: a runtime register index would send the arrays to
// scratch, cdna_hip_programming.md §5.4 rule 20), and only the stages with j >= 64 E go through
// LDS (one barrier each, double-buffered).  Ascending order.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace nsgpu {

constexpr int SORT_N = 4096;

struct SortLds {
  uint64_t k[2][SORT_N];
  uint32_t v[2][SORT_N];
};

__device__ __forceinline__ void cswap(uint64_t &ak, uint32_t &av, uint64_t &bk, uint32_t &bv, bool asc) {
  const bool sw = asc ? (ak > bk) : (ak < bk);
  if (sw) {
    uint64_t tk = ak;
    ak = bk;
    bk = tk;
    uint32_t tv = av;
    av = bv;
    bv = tv;
  }
}

template <int E, int QJ>
__device__ __forceinline__ void reg_stage(uint64_t (&key)[E], uint32_t (&val)[E], int base, int k) {
#pragma unroll
  for (int q = 0; q < E; q++)
    if ((q & QJ) == 0) cswap(key[q], val[q], key[q | QJ], val[q | QJ], ((base + 64 * q) & k) == 0);
}

template <int THREADS>
__device__ __forceinline__ void bitonic_sort(uint64_t (&key)[SORT_N / THREADS], uint32_t (&val)[SORT_N / THREADS],
                                             SortLds &L) {
  constexpr int E = SORT_N / THREADS;
  constexpr int CHUNK = 64 * E;  // elements per wave
  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  const int base = CHUNK * wid + lane;
  int buf = 0;
#pragma unroll 1
  for (int k = 2; k <= SORT_N; k <<= 1) {
#pragma unroll 1
    for (int j = k >> 1; j > 0; j >>= 1) {
      if (j >= CHUNK) {
#pragma unroll
        for (int q = 0; q < E; q++) {
          L.k[buf][base + 64 * q] = key[q];
          L.v[buf][base + 64 * q] = val[q];
        }
        __syncthreads();
#pragma unroll
        for (int q = 0; q < E; q++) {
          const int i = base + 64 * q;
          const int p = i ^ j;
          const uint64_t pk = L.k[buf][p];
          const uint32_t pv = L.v[buf][p];
          const bool asc = (i & k) == 0;
          const bool lower = (i & j) == 0;
          const bool take = lower ? (asc ? (pk < key[q]) : (pk > key[q])) : (asc ? (pk > key[q]) : (pk < key[q]));
          if (take) {
            key[q] = pk;
            val[q] = pv;
          }
        }
        buf ^= 1;
      } else if (j >= 64) {
        if (j == 64) reg_stage<E, 1>(key, val, base, k);
        else if (j == 128) reg_stage<E, (E > 2 ? 2 : 1)>(key, val, base, k);
        else if (j == 256) reg_stage<E, (E > 4 ? 4 : 1)>(key, val, base, k);
        else if (j == 512) reg_stage<E, (E > 8 ? 8 : 1)>(key, val, base, k);
      } else {
#pragma unroll
        for (int q = 0; q < E; q++) {
          const int i = base + 64 * q;
          const uint64_t pk = __shfl_xor(key[q], j);
          const uint32_t pv = __shfl_xor(val[q], j);
          const bool asc = (i & k) == 0;
          const bool lower = (i & j) == 0;
          const bool take = lower ? (asc ? (pk < key[q]) : (pk > key[q])) : (asc ? (pk > key[q]) : (pk < key[q]));
          if (take) {
            key[q] = pk;
            val[q] = pv;
          }
        }
      }
    }
  }
  __syncthreads();  // the last LDS buffer may still be read by a slow wave
}

}  // namespace nsgpu
