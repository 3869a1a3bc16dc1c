// exp / log / pow, bit-identical to the glibc that CPython calls.
//
// CPython evaluates `**` (float_pow), math.pow, math.exp and math.log with
// libm (reference: funsearch/safe_execution.py:25,112-116 exposes `math`;
// every candidate program runs through it).  glibc >= 2.28 computes them
// with the table-driven algorithms of sysdeps/ieee754/dbl-64/e_exp.c, e_log.c
// and e_pow.c, and on x86-64 hosts with FMA + AVX2 its IFUNCs pick builds of
// those sources compiled with fused multiply-adds (__exp_fma, __log_fma,
// __pow_fma).  This header re-implements exactly those builds: the same
// tables (glibc_math_tables.inc, extracted from the host's libm by
// tools/gen_glibc_math_tables.py), the same operation order, and a fused
// multiply-add exactly where GCC contracted one in the libm binary (read off
// its disassembly; the comments give each contraction).  IEEE double add,
// mul and fma are correctly rounded on gfx950 and on the host, so the device
// returns glibc's bits -- including glibc's occasional 0.52-ULP roundings --
// and no result needs deferring to the host.
//
// The equality is checked, not assumed: tests/test_glibc_math.py compares
// the host build of these functions with Python's `math` on >= 10M
// arguments per function, the extension re-checks 200k at import
// (`glibc_math_selfcheck`; on a mismatch -- a host whose libm is another
// build -- the device defers transcendental calls to the CPU VM, which calls
// the host libm), and tests/test_gpu_glibc_math.py checks device == host.
//
// Only the inputs CPython hands to libm are supported (CPython's float_pow /
// math_1 / m_log handle the rest before calling libm): exp(x) x finite,
// log(x) x > 0 finite, pow(x, y) x > 0 finite, x != 1, y finite non-zero.
// Status: 0 ok, 1 overflow (glibc returns inf with ERANGE: OverflowError).
// Underflow returns 0 / a subnormal, as glibc (CPython ignores ERANGE there).
//
// ---------------------------------------------------------------------------
// Provenance and licence.  The algorithms, operation order and polynomial
// coefficients below are those of glibc's sysdeps/ieee754/dbl-64/e_exp.c,
// e_log.c and e_pow.c (with e_exp_data.c, e_log_data.c, e_pow_log_data.c),
// which glibc took from Arm's Optimized Routines:
//
//   Copyright (C) 2018-2022 Free Software Foundation, Inc.
//   This file is part of the GNU C Library.  The GNU C Library is free
//   software; you can redistribute it and/or modify it under the terms of the
//   GNU Lesser General Public License as published by the Free Software
//   Foundation; either version 2.1 of the License, or (at your option) any
//   later version.  It is distributed WITHOUT ANY WARRANTY; see the GNU
//   Lesser General Public License (https://www.gnu.org/licenses/) for details.
//
//   Copyright (c) 2018, Arm Limited.
//   SPDX-License-Identifier: MIT (Arm Optimized Routines, exp / log / pow)
//
// This is an independent re-implementation for HIP (host and gfx950), written
// from the algorithm descriptions and checked bit for bit against the host's
// libm; the data tables are read from the installed libm.so.6 itself
// (tools/gen_glibc_math_tables.py), not copied from glibc sources.
// ---------------------------------------------------------------------------
#pragma once

#include "jit_env.h"

namespace fksd {
namespace gm {

#include "glibc_math_tables.inc"

__host__ __device__ __forceinline__ uint64_t asu(double x) { return __builtin_bit_cast(uint64_t, x); }
__host__ __device__ __forceinline__ double asd(uint64_t u) { return __builtin_bit_cast(double, u); }
__host__ __device__ __forceinline__ uint32_t top12(double x) { return (uint32_t)(asu(x) >> 52); }

constexpr int kN = 128;   // table entries (EXP_TABLE_BITS = LOG_TABLE_BITS = POW_LOG_TABLE_BITS = 7)

// exp.c specialcase(): the scale's exponent over- or underflowed (|x| > 512).
// exp and pow share it (pow's sign handling is moot: CPython passes x > 0).
__host__ __device__ inline double exp_special(double tmp, uint64_t sbits, uint64_t ki) {
  if ((ki & 0x80000000u) == 0) {
    // k > 0: the exponent of scale may have overflowed by <= 460
    sbits -= 1009ull << 52;
    const double scale = asd(sbits);
    return 0x1p1009 * fma(scale, tmp, scale);            // scale + scale * tmp: contracted
  }
  // k < 0: subnormal range
  sbits += 1022ull << 52;
  const double scale = asd(sbits);
  const double st = scale * tmp;                         // two uses: not contracted
  double y = scale + st;
  if (y < 1.0) {
    double lo = scale - y + st;
    const double hi = 1.0 + y;
    lo = 1.0 - hi + y + lo;
    y = (lo + hi) - 1.0;
    if (y == 0.0) y = 0.0;
  }
  return 0x1p-1022 * y;
}

// exp.c; with TAIL, pow.c's exp_inline (xtail added to r).  `out` = exp(x + xtail).
template <bool TAIL>
__host__ __device__ inline int exp_core(double x, double xtail, double& out) {
  uint32_t abstop = top12(x) & 0x7ff;
  if (abstop - 0x3c9u >= 0x3fu) {          // top12(512) - top12(0x1p-54)
    if (abstop - 0x3c9u >= 0x80000000u) {  // |x| < 2^-54
      out = 1.0 + x;
      return 0;
    }
    if (abstop >= 0x409u) {                // |x| >= 1024 (finite): over- / underflow
      if (asu(x) >> 63) { out = 0.0; return 0; }
      out = INFINITY;
      return 1;
    }
    abstop = 0;                            // large |x|: special-cased below
  }
  const double InvLn2N = kExpHdr[0], Shift = kExpHdr[1], NegLn2hiN = kExpHdr[2], NegLn2loN = kExpHdr[3];
  const double C2 = kExpHdr[4], C3 = kExpHdr[5], C4 = kExpHdr[6], C5 = kExpHdr[7];
  double kd = fma(x, InvLn2N, Shift);      // z + Shift with z = InvLn2N * x: contracted
  const uint64_t ki = asu(kd);
  kd -= Shift;
  double r = fma(kd, NegLn2hiN, x);        // x + kd * NegLn2hiN + kd * NegLn2loN: both contracted
  r = fma(kd, NegLn2loN, r);
  if constexpr (TAIL) r = xtail + r;
  const uint64_t idx = 2 * (ki % kN);
  const uint64_t top = ki << 45;
  const double tail = asd(kExpTab[idx]);
  const uint64_t sbits = kExpTab[idx + 1] + top;
  const double r2 = r * r;
  // tail + r + r2 * (C2 + r * C3) + r2 * r2 * (C4 + r * C5)
  const double t0 = r + tail;
  const double p23 = fma(r, C3, C2);
  const double p45 = fma(r, C5, C4);
  const double t1 = fma(p23, r2, t0);
  const double tmp = fma(r2 * r2, p45, t1);
  if (abstop == 0) {
    out = exp_special(tmp, sbits, ki);
    if (out == INFINITY) return 1;
    return 0;
  }
  const double scale = asd(sbits);
  out = fma(scale, tmp, scale);           // scale + scale * tmp: contracted
  return 0;
}

// math.exp(x), x finite
__host__ __device__ inline int exp(double x, double& out) { return exp_core<false>(x, 0.0, out); }

// math.log(x), x > 0 finite (log.c)
__host__ __device__ inline int log(double x, double& out) {
  uint64_t ix = asu(x);
  const uint32_t top = (uint32_t)(ix >> 48);
  constexpr uint64_t LO = 0x3fee000000000000ull;   // asuint64(1.0 - 0x1p-4)
  constexpr uint64_t HI = 0x3ff1090000000000ull;   // asuint64(1.0 + 0x1.09p-4)
  if (ix - LO < HI - LO) {
    if (ix == 0x3ff0000000000000ull) { out = 0.0; return 0; }
    const double* B = kLogB;
    const double r = x - 1.0;
    const double r2 = r * r;
    const double r3 = r * r2;
    // y = r3 * (B1 + r B2 + r2 B3 + r3 (B4 + r B5 + r2 B6 + r3 (B7 + r B8 + r2 B9 + r3 B10)))
    const double q1 = fma(r2, B[3], fma(r, B[2], B[1]));
    const double q2 = fma(r2, B[6], fma(r, B[5], B[4]));
    double q3 = fma(r2, B[9], fma(r, B[8], B[7]));
    q3 = fma(r3, B[10], q3);
    const double p = fma(fma(q3, r3, q2), r3, q1);
    // w = r * 0x1p27; rhi = r + w - w: the product contracted into both uses
    const double rhi = fma(-0x1p27, r, fma(r, 0x1p27, r));
    const double rlo = r - rhi;
    const double rr = rhi * rhi;
    const double hi = fma(rr, B[0], r);              // r + w, w = rhi * rhi * B0
    double lo = fma(rr, B[0], r - hi);               // r - hi + w
    lo = fma(B[0] * rlo, rhi + r, lo);               // lo += B0 * rlo * (rhi + r)
    const double y = fma(p, r3, lo);                 // y = r3 * (...); y += lo
    out = hi + y;                                    // y += hi
    return 0;
  }
  if (top - 0x0010u >= 0x7ff0u - 0x0010u) {
    // x is subnormal here (CPython passes x > 0 finite): normalise
    ix = asu(x * 0x1p52);
    ix -= 52ull << 52;
  }
  constexpr uint64_t OFF = 0x3fe6000000000000ull;
  const uint64_t tmp = ix - OFF;
  const int i = (int)((tmp >> 45) % kN);
  const int k = (int)((int64_t)tmp >> 52);
  const uint64_t iz = ix - (tmp & (0xfffull << 52));
  const double invc = kLogTab[2 * i], logc = kLogTab[2 * i + 1];
  const double z = asd(iz);
  const double kd = (double)k;
  const double r = fma(z, invc, -1.0);
  const double Ln2hi = kLogLn2[0], Ln2lo = kLogLn2[1];
  const double* A = kLogA;
  const double w = fma(kd, Ln2hi, logc);             // kd * Ln2hi + logc
  const double hi = w + r;
  const double lo = fma(kd, Ln2lo, (w - hi) + r);    // w - hi + r + kd * Ln2lo
  const double r2 = r * r;
  // y = lo + r2 * A0 + r * r2 * (A1 + r A2 + r2 (A3 + r A4)) + hi
  const double a12 = fma(r, A[2], A[1]);
  const double a34 = fma(r, A[4], A[3]);
  const double t = fma(r2, A[0], lo);
  const double q = fma(a34, r2, a12);
  out = fma(r * r2, q, t) + hi;
  return 0;
}

// pow.c log_inline: log(x) as hi + tail, |tail| <~ 2^-65 |hi|
__host__ __device__ inline double pow_log(uint64_t ix, double& tail) {
  constexpr uint64_t OFF = 0x3fe6955500000000ull;
  const uint64_t tmp = ix - OFF;
  const int i = (int)((tmp >> 45) % kN);
  const int k = (int)((int64_t)tmp >> 52);
  const uint64_t iz = ix - (tmp & (0xfffull << 52));
  const double z = asd(iz);
  const double kd = (double)k;
  const double invc = kPowTab[3 * i], logc = kPowTab[3 * i + 1], logctail = kPowTab[3 * i + 2];
  const double Ln2hi = kPowHdr[0], Ln2lo = kPowHdr[1];
  const double* A = kPowHdr + 2;
  const double r = fma(z, invc, -1.0);
  const double t1 = fma(kd, Ln2hi, logc);            // kd * Ln2hi + logc
  const double t2 = t1 + r;
  const double lo1 = fma(kd, Ln2lo, logctail);       // kd * Ln2lo + logctail
  const double lo2 = t1 - t2 + r;
  const double ar = A[0] * r;                        // A[0] = -0.5
  const double ar2 = r * ar;
  const double ar3 = r * ar2;
  const double hi = t2 + ar2;
  const double lo3 = fma(ar, r, -ar2);
  const double lo4 = t2 - hi + ar2;
  // p = ar3 * (A1 + r A2 + ar2 (A3 + r A4 + ar2 (A5 + r A6)))
  const double a12 = fma(r, A[2], A[1]);
  const double a34 = fma(r, A[4], A[3]);
  const double a56 = fma(r, A[6], A[5]);
  const double q = fma(ar2, fma(a56, ar2, a34), a12);
  const double lo = fma(ar3, q, lo1 + lo2 + lo3 + lo4);   // lo1 + lo2 + lo3 + lo4 + p: p contracted
  const double y = hi + lo;
  tail = hi - y + lo;
  return y;
}

// pow(x, y) for what CPython's float_pow / math.pow hand to libm here:
// x > 0 finite, x != 1, y finite and non-zero (negative bases are folded by
// the caller: glibc's result for -x is exactly the negation)
__host__ __device__ inline int pow(double x, double y, double& out) {
  uint64_t ix = asu(x);
  const uint64_t iy = asu(y);
  const uint32_t topx = top12(x);
  const uint32_t topy = top12(y);
  if (topx - 0x001u >= 0x7ffu - 0x001u || (topy & 0x7ff) - 0x3beu >= 0x43eu - 0x3beu) {
    if ((topy & 0x7ff) - 0x3beu >= 0x43eu - 0x3beu) {
      if (ix == 0x3ff0000000000000ull) { out = 1.0; return 0; }
      if ((topy & 0x7ff) < 0x3beu) {            // |y| < 2^-65: x^y ~= 1 + y log(x)
        out = ix > 0x3ff0000000000000ull ? 1.0 + y : 1.0 - y;
        return 0;
      }
      if ((ix > 0x3ff0000000000000ull) == (topy < 0x800u)) { out = INFINITY; return 1; }
      out = 0.0;
      return 0;
    }
    if (topx == 0) {                            // subnormal x: normalise
      ix = asu(x * 0x1p52);
      ix &= 0x7fffffffffffffffull;
      ix -= 52ull << 52;
    }
  }
  (void)iy;
  double lo;
  const double hi = pow_log(ix, lo);
  const double ehi = y * hi;
  const double elo = fma(y, lo, fma(y, hi, -ehi));   // y * lo + fma(y, hi, -ehi): contracted
  return exp_core<true>(ehi, elo, out);
}

}  // namespace gm
}  // namespace fksd
