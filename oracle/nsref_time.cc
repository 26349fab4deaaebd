// nsref_time.cc — CPU ORACLE (test infrastructure only; see nsref.h header).
// Restatement of ns-3's 64.64 fixed point (src/core/model/int64x64-128.{h,cc}) and of
// Time at the default NS resolution (src/core/model/nstime.h, src/core/model/time.cc).
#include "nsref.h"
#include <math.h>
#include <string.h>
#include <stdlib.h>
#include <stdio.h>

typedef __int128 i128;
typedef unsigned __int128 u128;

static const u128 MASK_LO = (((u128)1) << 64) - 1;
static const u128 MASK_HI = ~MASK_LO;

static inline i128 load(const uint64_t w[2]) { return (i128)(((u128)w[1] << 64) | (u128)w[0]); }
static inline void store(i128 v, uint64_t w[2]) { u128 u = (u128)v; w[0] = (uint64_t)u; w[1] = (uint64_t)(u >> 64); }

// int64x64_t (double) — int64x64-128.h:26-36.  HP128_MAX_64 = 18446744073709551615.0 (== 2^64 as a double).
static i128 from_double(double value) {
  bool is_negative = value < 0;
  value = is_negative ? -value : value;
  double hi = floor(value);
  double lo = (value - hi) * 18446744073709551615.0;
  i128 v = (i128)hi;
  v <<= 64;
  v += (i128)lo;
  return is_negative ? -v : v;
}

// int64x64_t::Umul — int64x64-128.cc:30-57.  Note the '|=' combining step, restated as-is.
static u128 umul(u128 a, u128 b) {
  u128 aL = a & MASK_LO, bL = b & MASK_LO;
  u128 aH = (a >> 64) & MASK_LO, bH = (b >> 64) & MASK_LO;
  u128 loPart = aL * bL;
  u128 midPart = aL * bH + aH * bL;
  u128 result = (loPart >> 64) + (midPart & MASK_LO);
  u128 hiPart = aH * bH;
  result |= ((hiPart & MASK_LO) << 64) + (midPart & MASK_HI);
  if ((hiPart & MASK_HI) != 0) {
    fprintf(stderr, "nsref: High precision 128 bits multiplication error: multiplication overflow.\n");
    abort();  // NS_ABORT_MSG_IF (int64x64-128.cc:54-55)
  }
  return result;
}

// int64x64_t::Mul — int64x64-128.cc:20-29 (OUTPUT_SIGN macro :7-14).
static i128 mul(i128 x, i128 y) {
  bool negA = x < 0, negB = y < 0;
  u128 a = negA ? -x : x, b = negB ? -y : y;
  bool neg = (negA && !negB) || (!negA && negB);
  i128 r = (i128)umul(a, b);
  return neg ? -r : r;
}

// int64x64_t::Divu — int64x64-128.cc:67-92.
static u128 divu(u128 a, u128 b) {
  u128 quo = a / b;
  u128 rem = a % b;
  u128 result = quo << 64;
  u128 tmp = rem >> 64;
  u128 div;
  if (tmp == 0) {
    rem = rem << 64;
    div = b;
  } else {
    div = b >> 64;
  }
  quo = rem / div;
  result = result + quo;
  return result;
}

static i128 div_(i128 x, i128 y) {  // int64x64-128.cc:58-66
  bool negA = x < 0, negB = y < 0;
  u128 a = negA ? -x : x, b = negB ? -y : y;
  bool neg = (negA && !negB) || (!negA && negB);
  i128 r = (i128)divu(a, b);
  return neg ? -r : r;
}

// int64x64_t::UmulByInvert — int64x64-128.cc:103-118
static u128 umul_by_invert(u128 a, u128 b) {
  u128 ah = a >> 64, bh = b >> 64, al = a & MASK_LO, bl = b & MASK_LO;
  u128 hi = ah * bh;
  u128 mid = ah * bl + al * bh;
  mid >>= 64;
  return hi + mid;
}
// int64x64_t::MulByInvert — int64x64-128.cc:94-102
static i128 mul_by_invert(i128 v, i128 o) {
  bool neg = v < 0;
  u128 a = neg ? -v : v;
  u128 r = umul_by_invert(a, (u128)o);
  return neg ? -(i128)r : (i128)r;
}

static int64_t get_high(i128 v) {  // int64x64-128.h:98-105
  bool negative = v < 0;
  i128 x = negative ? -v : v;
  x >>= 64;
  int64_t r = (int64_t)x;
  return negative ? -r : r;
}

// int64x64_t::Invert — int64x64-128.cc:119-134
static i128 invert(uint64_t v) {
  u128 a = 1;
  a <<= 64;
  i128 result = (i128)divu(a, v);
  i128 tmp = ((i128)(int64_t)v) << 64;  // int64x64_t (v, false)
  tmp = mul_by_invert(tmp, result);
  if (get_high(tmp) != 1) result += 1;
  return result;
}

extern "C" {

void nsref_i64x64_from_double(double v, uint64_t out[2]) { store(from_double(v), out); }
void nsref_i64x64_from_int(int64_t v, uint64_t out[2]) { store(((i128)v) << 64, out); }
void nsref_i64x64_from_parts(int64_t hi, uint64_t lo, uint64_t out[2]) {
  // int64x64-128.h:67-74
  bool is_negative = hi < 0;
  i128 v = is_negative ? -hi : hi;
  v <<= 64;
  v += lo;
  store(is_negative ? -v : v, out);
}
void nsref_i64x64_mul(const uint64_t a[2], const uint64_t b[2], uint64_t out[2]) { store(mul(load(a), load(b)), out); }
void nsref_i64x64_div(const uint64_t a[2], const uint64_t b[2], uint64_t out[2]) { store(div_(load(a), load(b)), out); }
void nsref_i64x64_invert(uint64_t v, uint64_t out[2]) { store(invert(v), out); }
void nsref_i64x64_mul_by_invert(const uint64_t a[2], const uint64_t b[2], uint64_t out[2]) {
  store(mul_by_invert(load(a), load(b)), out);
}
int64_t nsref_i64x64_get_high(const uint64_t a[2]) { return get_high(load(a)); }
uint64_t nsref_i64x64_get_low(const uint64_t a[2]) {  // int64x64-128.h:106-113
  i128 v = load(a);
  bool negative = v < 0;
  i128 x = negative ? -v : v;
  return (uint64_t)(x & (i128)MASK_LO);
}
double nsref_i64x64_get_double(const uint64_t a[2]) {  // int64x64-128.h:85-97
  i128 v = load(a);
  bool is_negative = v < 0;
  u128 value = is_negative ? -v : v;
  uint64_t hi = (uint64_t)(value >> 64);
  uint64_t lo = (uint64_t)value;
  double flo = (double)lo;
  flo /= 18446744073709551615.0;
  double retval = (double)hi;
  retval += flo;
  return is_negative ? -retval : retval;
}

// Seconds (double) = Time::FromDouble (v, Time::S) = Time::From (int64x64_t (v), S):
// with NS resolution, S has shift = 15 - 6 = 9 > 0 -> fromMul, timeFrom = int64x64_t (1e9)
// (time.cc:106-126), so the value is int64x64_t (v) * int64x64_t (1000000000), and the
// Time is its GetHigh () (nstime.h:433-435).
int64_t nsref_seconds(double s) {
  i128 r = mul(from_double(s), ((i128)1000000000) << 64);
  return get_high(r);
}
void nsref_seconds_batch(const double *s, int64_t *out, int64_t n) {
  for (int64_t i = 0; i < n; i++) out[i] = nsref_seconds(s[i]);
}
// GetSeconds = ToDouble (S) = To (S).GetDouble (); To(S): toMul false -> MulByInvert (Invert (1e9)).
double nsref_get_seconds(int64_t ts) {
  i128 v = ((i128)ts) << 64;
  v = mul_by_invert(v, invert(1000000000ULL));
  uint64_t w[2];
  store(v, w);
  return nsref_i64x64_get_double(w);
}
// Time::FromInteger (nstime.h:344-353) at NS resolution; power table of time.cc:104.
int64_t nsref_from_integer(int64_t v, int unit) {
  static const int power[6] = {15, 12, 9, 6, 3, 0};
  int shift = power[unit] - power[3];
  uint64_t factor = (uint64_t)pow(10, fabs((double)shift));
  uint64_t value = (uint64_t)v;
  if (shift >= 0) value *= factor;  // fromMul (shift == 0 -> factor 1)
  else value /= factor;
  return (int64_t)value;
}

uint64_t nsref_distribution_ns(double seconds) { return (uint64_t)(seconds * 1000000000); }

}  // extern "C"
