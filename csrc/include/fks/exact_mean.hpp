// Exact mean of doubles, correctly rounded -- the value Python's
// statistics.mean returns (reference simulator/evaluator.py:83-89).
//
// Every value the evaluator averages is a ratio  k / T  of integers with
// |T| <= 2^44, so each double is a multiple of 2^-96 (its lowest mantissa bit
// weighs >= 2^(-44-52)).  Summing them in a signed 128-bit fixed-point word
// with 96 fractional bits is therefore EXACT; the mean is the correctly
// rounded quotient of that word by the count.  A value that is not a
// multiple of 2^-96 (or would overflow the 31 integer bits) sets `inexact`,
// and callers recompute that policy with an arbitrary-precision path.
//
// Plain C++17 (host).  The HIP replay kernel carries its own device copy of
// the same arithmetic (csrc/hip/exact_mean_dev.hip.h).
#pragma once

#include <cmath>
#include <cstdint>

namespace fks {

using i128 = __int128;
using u128 = unsigned __int128;

constexpr int kFixedFracBits = 96;

struct FixedAcc {
  i128 sum = 0;
  int64_t count = 0;
  bool inexact = false;

  void add(double v) {
    ++count;
    if (v == 0.0) return;
    if (!std::isfinite(v)) { inexact = true; return; }
    int e;
    double m = std::frexp(v, &e);                 // v = m * 2^e, 0.5 <= |m| < 1
    int64_t mi = (int64_t)std::ldexp(m, 53);      // exact 53-bit integer mantissa
    int shift = e - 53 + kFixedFracBits;          // v * 2^96 = mi * 2^shift
    if (shift < 0) {
      // representable only if the dropped bits are zero
      int64_t mask = (shift <= -63) ? -1 : (((int64_t)1 << (-shift)) - 1);
      uint64_t am = (uint64_t)(mi < 0 ? -mi : mi);
      if (shift <= -63 || (am & (uint64_t)mask)) { inexact = true; return; }
      mi >>= (-shift);  // exact (arithmetic shift of a multiple)
      shift = 0;
    }
    if (shift > 126 - 53) { inexact = true; return; }
    sum += (i128)mi << shift;
    // guard the 31 integer bits (|sum| < 2^127 always; keep headroom)
    u128 mag = sum < 0 ? (u128)(-sum) : (u128)sum;
    if (mag >> 126) inexact = true;
  }
};

// Correctly rounded (round-half-even) value of  A * 2^-frac_bits / n.
inline double fixed_div_round(i128 A, uint64_t n, int frac_bits = kFixedFracBits) {
  if (A == 0 || n == 0) return 0.0;
  const bool neg = A < 0;
  u128 a = neg ? (u128)(-A) : (u128)A;
  u128 q = a / n;
  u128 r = a % n;
  int exp2 = -frac_bits;  // result = (q + r/n) * 2^exp2
  // Normalise q to exactly 64 significant bits (top bit 63), collecting sticky.
  bool sticky = false;
  if (q >> 64) {
    int extra = 0;
    while (q >> (64 + extra)) ++extra;
    u128 dropped = q & (((u128)1 << extra) - 1);
    sticky = dropped != 0 || r != 0;
    q >>= extra;
    exp2 += extra;
    r = 0;
  } else {
    while (!(q >> 63)) {
      r <<= 1;
      u128 bit = (r >= n) ? 1 : 0;
      if (bit) r -= n;
      q = (q << 1) | bit;
      --exp2;
    }
    sticky = r != 0;
  }
  uint64_t M = (uint64_t)q;  // 64 significant bits
  uint64_t low = M & 0x7FFull;
  uint64_t m53 = M >> 11;
  exp2 += 11;
  const uint64_t half = 0x400ull;
  if (low > half || (low == half && (sticky || (m53 & 1)))) {
    ++m53;
    if (m53 >> 53) { m53 >>= 1; ++exp2; }
  } else if (low == half && !sticky && !(m53 & 1)) {
    // tie, even: keep
  }
  double v = std::ldexp((double)m53, exp2);
  return neg ? -v : v;
}

inline double fixed_mean(const FixedAcc& acc) {
  return acc.count ? fixed_div_round(acc.sum, (uint64_t)acc.count) : 0.0;
}

}  // namespace fks
