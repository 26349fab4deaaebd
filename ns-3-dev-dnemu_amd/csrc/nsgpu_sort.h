// nsgpu_sort.h — workgroup-wide bitonic sort of 4096 (u64 key, u32 value) pairs for 1024 threads.
//
// Layout: wave w owns elements [256 w, 256 w + 256); lane l holds element 256 w + 64 q + l in
// register slot q (q = 0..3).  Stages with j < 64 exchange through wave shuffles, stages with
// 64 <= j < 256 swap between the lane's own registers, and only the 10 stages with j >= 256
// go through LDS (one barrier each, double-buffered).  Ascending order.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace nsgpu {

constexpr int SORT_N = 4096;
constexpr int SORT_THREADS = 1024;

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

// k[q], v[q]: this lane's 4 elements (global index i_q = 256*wid + 64*q + lane).  Sorted in place.
__device__ __forceinline__ void bitonic_sort_4096(uint64_t (&key)[4], uint32_t (&val)[4], SortLds &L) {
  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  int buf = 0;
  for (int k = 2; k <= SORT_N; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      if (j >= 256) {
        // cross-wave: publish, barrier, read partner
#pragma unroll
        for (int q = 0; q < 4; q++) {
          const int i = 256 * wid + 64 * q + lane;
          L.k[buf][i] = key[q];
          L.v[buf][i] = val[q];
        }
        __syncthreads();
#pragma unroll
        for (int q = 0; q < 4; q++) {
          const int i = 256 * wid + 64 * q + lane;
          const int p = i ^ j;
          const uint64_t pk = L.k[buf][p];
          const uint32_t pv = L.v[buf][p];
          const bool asc = (i & k) == 0;
          const bool lower = (i & j) == 0;
          // lower keeps min (asc) / max (desc); upper keeps the other
          const bool take = lower ? (asc ? (pk < key[q]) : (pk > key[q])) : (asc ? (pk > key[q]) : (pk < key[q]));
          if (take) {
            key[q] = pk;
            val[q] = pv;
          }
        }
        buf ^= 1;
      } else if (j >= 64) {
        const int qj = j >> 6;  // 1 or 2
#pragma unroll
        for (int q = 0; q < 4; q++) {
          if ((q & qj) == 0) {
            const int i = 256 * wid + 64 * q + lane;
            const bool asc = (i & k) == 0;
            cswap(key[q], val[q], key[q | qj], val[q | qj], asc);
          }
        }
      } else {
#pragma unroll
        for (int q = 0; q < 4; q++) {
          const int i = 256 * wid + 64 * q + lane;
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
