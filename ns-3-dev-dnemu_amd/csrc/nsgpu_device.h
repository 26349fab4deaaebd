// nsgpu_device.h — device-side arithmetic shared by the nsgpu kernels (gfx950).
//
// Everything here must round exactly like the reference's x86-64 -O2 build:
//   * compiled with -ffp-contract=off (no FMA contraction),
//   * IEEE double '/' and sqrt (correctly rounded on gfx950),
//   * 64.64 fixed point in __int128 exactly as src/core/model/int64x64-128.{h,cc}.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "../../include/nsgpu_types.h"

namespace nsgpu {

typedef __int128 i128;
typedef unsigned __int128 u128;

// int64x64_t (double) — src/core/model/int64x64-128.h:26-36
__host__ __device__ __forceinline__ i128 i64x64_from_double(double value) {
  bool neg = value < 0;
  value = neg ? -value : value;
  double hi = floor(value);
  double lo = (value - hi) * 18446744073709551615.0;  // HP128_MAX_64 (== 2^64 as a double)
  i128 v = (i128)hi;
  v <<= 64;
  v += (i128)lo;
  return neg ? -v : v;
}

// Seconds (double).GetTimeStep () at NS resolution: GetHigh (int64x64_t (s) * int64x64_t (1e9)).
// int64x64_t::Mul/Umul (int64x64-128.cc:20-57) specialised to b = 1e9 << 64 (bL = 0):
//   loPart = 0, midPart = aL * 1e9, hiPart = aH * 1e9,
//   result = (mid & LO) | ((hi & LO) << 64) + (mid & HI)   — the low word of the OR is mid's low word
//   GetHigh = (hi + (mid >> 64)) mod 2^64, sign applied after.
// The overflow abort of Umul (hiPart >> 64 != 0) cannot trigger for |s| < 2^63/1e9 s (292 years).
__host__ __device__ __forceinline__ int64_t seconds_to_ts(double s) {
  i128 v = i64x64_from_double(s);
  bool neg = v < 0;
  u128 a = neg ? (u128)(-v) : (u128)v;
  uint64_t aL = (uint64_t)a;
  uint64_t aH = (uint64_t)(a >> 64);
  u128 mid = (u128)aL * 1000000000ull;
  u128 hi = (u128)aH * 1000000000ull;
  u128 high = hi + (mid >> 64);   // (result >> 64) before the final int128 truncation
  u128 res = (high << 64) | (u128)(uint64_t)mid;
  i128 r = neg ? -(i128)res : (i128)res;
  // GetHigh (int64x64-128.h:98-105)
  bool rn = r < 0;
  i128 x = rn ? -r : r;
  x >>= 64;
  int64_t out = (int64_t)x;
  return rn ? -out : out;
}

// CalculateDistance — src/core/model/vector.cc:63-70 (b - a).
__host__ __device__ __forceinline__ double distance3(double ax, double ay, double az, double bx, double by,
                                                      double bz) {
  double dx = bx - ax;
  double dy = by - ay;
  double dz = bz - az;
  return sqrt(dx * dx + dy * dy + dz * dz);
}

// One PropagationLossModel link's DoCalcRxPower (src/propagation/model/propagation-loss-model.cc).
__host__ __device__ __forceinline__ double loss_link(const nsgpu_loss_model &m, double tx, double distance) {
  const double PI = 3.14159265358979323846;
  switch (m.kind) {
    case NSGPU_LOSS_LOG_DISTANCE: {  // :464-491
      if (distance <= m.p1) return tx;
      double pathLossDb = 10 * m.p0 * log10(distance / m.p1);
      double rxc = -m.p2 - pathLossDb;
      return tx + rxc;
    }
    case NSGPU_LOSS_FRIIS: {  // :197-239
      if (distance <= m.p2) return tx;
      double numerator = m.p0 * m.p0;
      double denominator = 16 * PI * PI * distance * distance * m.p1;
      double pr = 10 * log10(numerator / denominator);
      return tx + pr;
    }
    case NSGPU_LOSS_FIXED_RSS:  // :718-723
      return m.p0;
    case NSGPU_LOSS_RANGE:  // :822-834
      return distance <= m.p0 ? tx : -1000.0;
    default:
      return tx;
  }
}

// PropagationLossModel::CalcRxPower chain (:64-74).
__host__ __device__ __forceinline__ double calc_rx_power(const nsgpu_loss_chain &c, double tx, double distance) {
  double self = tx;
  for (int i = 0; i < c.n; i++) self = loss_link(c.m[i], self, distance);
  return self;
}

// Event key order (scheduler.h:105-121): (ts, uid).
__host__ __device__ __forceinline__ bool key_less(uint64_t ats, uint32_t auid, uint64_t bts, uint32_t buid) {
  return ats < bts || (ats == bts && auid < buid);
}

__host__ __device__ __forceinline__ uint64_t mix64(uint64_t z) { return nsgpu_mix64(z); }
__host__ __device__ __forceinline__ uint64_t digest_term(uint64_t rank, uint64_t ts, uint32_t uid) {
  return nsgpu_dispatch_digest_term(rank, ts, uid);
}

}  // namespace nsgpu
