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

// Value of lane (lane ^ J) of the wave, without the LDS crossbar: DPP for J < 16 (quad_perm for 1 and
// 2, row shifts for 4, row rotate for 8) and the gfx950 permlane swaps for 16 and 32.
template <int J>
__device__ __forceinline__ uint32_t xlane(uint32_t v) {
  const int lane = threadIdx.x & 63;
  if constexpr (J == 1) {
    return __builtin_amdgcn_mov_dpp(v, 0xB1, 0xf, 0xf, false);  // quad_perm [1,0,3,2]
  } else if constexpr (J == 2) {
    return __builtin_amdgcn_mov_dpp(v, 0x4E, 0xf, 0xf, false);  // quad_perm [2,3,0,1]
  } else if constexpr (J == 4) {
    const uint32_t up = __builtin_amdgcn_mov_dpp(v, 0x104, 0xf, 0xf, false);  // row_shl:4 (lane + 4)
    const uint32_t dn = __builtin_amdgcn_mov_dpp(v, 0x114, 0xf, 0xf, false);  // row_shr:4 (lane - 4)
    return (lane & 4) ? dn : up;
  } else if constexpr (J == 8) {
    return __builtin_amdgcn_mov_dpp(v, 0x128, 0xf, 0xf, false);  // row_ror:8
  } else if constexpr (J == 16) {
    const auto r = __builtin_amdgcn_permlane16_swap(v, v, false, false);  // r[0]: even rows, r[1]: odd rows
    return (lane & 16) ? r[0] : r[1];
  } else {
    const auto r = __builtin_amdgcn_permlane32_swap(v, v, false, false);  // r[0]: low half, r[1]: high half
    return (lane & 32) ? r[0] : r[1];
  }
}

template <int E, int J>
__device__ __forceinline__ void lane_stage(uint64_t (&key)[E], uint32_t (&val)[E], int k) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int q = 0; q < E; q++) {
    const int i = 64 * q + lane;
    const uint64_t pk = ((uint64_t)xlane<J>((uint32_t)(key[q] >> 32)) << 32) | xlane<J>((uint32_t)key[q]);
    const uint32_t pv = xlane<J>(val[q]);
    const bool asc = (i & k) == 0;
    const bool lower = (i & J) == 0;
    const bool take = (lower == asc) ? (pk < key[q]) : (pk > key[q]);
    if (take) {
      key[q] = pk;
      val[q] = pv;
    }
  }
}

// Wave-local bitonic sort of the wave's 64 E elements (same register layout as bitonic_sort):
// lane stages exchange through DPP / permlane (VALU, no LDS traffic), slot stages swap registers.
template <int E>
__device__ __forceinline__ void wave_sort(uint64_t (&key)[E], uint32_t (&val)[E]) {
  constexpr int CHUNK = 64 * E;
  const int lane = threadIdx.x & 63;
#pragma unroll 1
  for (int k = 2; k <= CHUNK; k <<= 1) {
#pragma unroll 1
    for (int j = k >> 1; j > 0; j >>= 1) {
      switch (j) {
        case 1: lane_stage<E, 1>(key, val, k); break;
        case 2: lane_stage<E, 2>(key, val, k); break;
        case 4: lane_stage<E, 4>(key, val, k); break;
        case 8: lane_stage<E, 8>(key, val, k); break;
        case 16: lane_stage<E, 16>(key, val, k); break;
        case 32: lane_stage<E, 32>(key, val, k); break;
        case 64: reg_stage<E, 1>(key, val, lane, k); break;
        case 128: reg_stage<E, (E > 2 ? 2 : 1)>(key, val, lane, k); break;
        case 256: reg_stage<E, (E > 4 ? 4 : 1)>(key, val, lane, k); break;
        default: reg_stage<E, (E > 8 ? 8 : 1)>(key, val, lane, k); break;
      }
    }
  }
}

// Workgroup sort of n <= SORT_N keys held in L.k[0]/L.v[0][0, n) (keys distinct and < ~0): each
// wave sorts its run of 64 E keys in registers, then sorted blocks are merged pairwise (every key's
// position in the merged block = its index in its own block + its lower bound in the partner
// block).  Result in L.k[0]/L.v[0][0, n).
template <int THREADS>
__device__ __forceinline__ void run_rank_sort(SortLds &L, uint32_t n) {
  constexpr int E = SORT_N / THREADS;
  constexpr int CHUNK = 64 * E;
  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  const int base = CHUNK * wid + lane;
  const int nruns = (int)((n + CHUNK - 1) / CHUNK);
  if (wid < nruns) {
    uint64_t key[E];
    uint32_t val[E];
#pragma unroll
    for (int q = 0; q < E; q++) {
      const int i = base + 64 * q;
      key[q] = i < (int)n ? L.k[0][i] : ~0ull;
      val[q] = i < (int)n ? L.v[0][i] : 0xffffffffu;
    }
    wave_sort<E>(key, val);
#pragma unroll
    for (int q = 0; q < E; q++) {
      L.k[1][base + 64 * q] = key[q];
      L.v[1][base + 64 * q] = val[q];
    }
  }
  __syncthreads();
  // merge rounds: blocks of `blk` sorted keys in buffer `src` -> blocks of 2 blk in buffer src ^ 1
  int src = 1;
  const int used = nruns * CHUNK;  // slots in use (keys at n..used-1 are padding ~0)
#pragma unroll 1
  for (int blk = CHUNK; blk < used; blk <<= 1) {
#pragma unroll 1
    for (int q = 0; q < E; q++) {
      const int i = base + 64 * q;  // any slot (keys are re-read from LDS)
      if (i >= used) continue;
      const uint64_t x = L.k[src][i];
      const uint32_t xv = L.v[src][i];
      const int me = i / blk, own = i - me * blk;
      const int pb = (me ^ 1) * blk;  // partner block start
      const int mstart = (me & ~1) * blk;
      const int plen = pb < used ? (used - pb < blk ? used - pb : blk) : 0;
      // position in the partner block: # keys < x for the left block, # keys <= x for the right one
      // (ties are padding keys ~0, which keeps every slot of the merged block written)
      const bool right = me & 1;
      int lo = 0, len = plen;
#pragma unroll 1
      while (len > 0) {
        const int half = len >> 1;
        const uint64_t y = L.k[src][pb + lo + half];
        if (y < x || (right && y == x)) {
          lo += half + 1;
          len -= half + 1;
        } else {
          len = half;
        }
      }
      L.k[src ^ 1][mstart + own + lo] = x;
      L.v[src ^ 1][mstart + own + lo] = xv;
    }
    src ^= 1;
    __syncthreads();
  }
  if (src == 1) {
    for (int i = threadIdx.x; i < (int)n; i += THREADS) {
      L.k[0][i] = L.k[1][i];
      L.v[0][i] = L.v[1][i];
    }
    __syncthreads();
  }
}

// Workgroup merge sort of n <= SORT_N keys in L.k[0]/L.v[0][0, n) (ascending; equal keys keep no
// particular order).  Work-efficient for a CU (16-lane SIMDs: a wave64 VALU op is 4 cycles), unlike a
// bitonic network: each thread sorts 8 keys in registers, then log2(n / 8) merge rounds in which a
// thread finds its 8-output diagonal of the merged block by a merge-path search and merges serially.
// Only the first pow2ceil(n) / 8 threads work.  Result in L.k[0]/L.v[0][0, n).
template <int THREADS>
__device__ __forceinline__ void merge_sort(SortLds &L, uint32_t n) {
  constexpr int VT = 8;
  int npad = VT;
  while (npad < (int)n) npad <<= 1;
  const int t = threadIdx.x;
  const bool act = t * VT < npad;
  if (act) {
    uint64_t k[VT];
    uint32_t v[VT];
#pragma unroll
    for (int q = 0; q < VT; q++) {
      const int i = t * VT + q;
      k[q] = i < (int)n ? L.k[0][i] : ~0ull;
      v[q] = i < (int)n ? L.v[0][i] : 0xffffffffu;
    }
    // odd-even transposition network, 8 passes
#pragma unroll
    for (int pass = 0; pass < VT; pass++) {
#pragma unroll
      for (int q = pass & 1; q + 1 < VT; q += 2) cswap(k[q], v[q], k[q + 1], v[q + 1], true);
    }
#pragma unroll
    for (int q = 0; q < VT; q++) {
      L.k[0][t * VT + q] = k[q];
      L.v[0][t * VT + q] = v[q];
    }
  }
  __syncthreads();
  int src = 0;
#pragma unroll 1
  for (int blk = VT; blk < npad; blk <<= 1) {
    if (act) {
      const uint64_t *sk = L.k[src];
      const uint32_t *sv = L.v[src];
      const int d = (t * VT) & (2 * blk - 1);  // output diagonal inside the merged block
      const int s0 = t * VT - d;                // merged block start; A = [s0, s0+blk), B = [s0+blk, s0+2blk)
      int lo = d > blk ? d - blk : 0, hi = d < blk ? d : blk;
      while (lo < hi) {  // merge path: # of A keys among the first d outputs (A first on ties)
        const int mid = (lo + hi) >> 1;
        if (!(sk[s0 + blk + d - 1 - mid] < sk[s0 + mid])) lo = mid + 1;
        else hi = mid;
      }
      int ia = s0 + lo, ib = s0 + blk + d - lo;
      const int ea = s0 + blk, eb = s0 + 2 * blk;
      uint64_t ka = ia < ea ? sk[ia] : ~0ull, kb = ib < eb ? sk[ib] : ~0ull;
      uint64_t *dk = L.k[src ^ 1];
      uint32_t *dv = L.v[src ^ 1];
#pragma unroll
      for (int q = 0; q < VT; q++) {
        const bool takea = ib >= eb || (ia < ea && !(kb < ka));
        if (takea) {
          dk[t * VT + q] = ka;
          dv[t * VT + q] = sv[ia];
          ia++;
          ka = ia < ea ? sk[ia] : ~0ull;
        } else {
          dk[t * VT + q] = kb;
          dv[t * VT + q] = sv[ib];
          ib++;
          kb = ib < eb ? sk[ib] : ~0ull;
        }
      }
    }
    src ^= 1;
    __syncthreads();
  }
  if (src == 1) {
    for (int i = t; i < (int)n; i += THREADS) {
      L.k[0][i] = L.k[1][i];
      L.v[0][i] = L.v[1][i];
    }
    __syncthreads();
  }
}

}  // namespace nsgpu
