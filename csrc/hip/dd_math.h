// Correctly rounded exp / log / pow for the device (VM runtime and the
// native programs' rt_binop / rt_unop).
//
// CPython delegates `**`, math.exp, math.log and math.pow to glibc.  The
// device evaluates them in double-double arithmetic (~2^-100 relative error)
// and rounds once, so it returns the correctly rounded double; results that
// land within 2^-84..2^-90 of a rounding midpoint (exact ties such as small
// integer powers) are reported as `defer` and the policy is re-run on the
// host, where glibc decides.
//
// Measured (csrc/tools/dd_math_check.cpp, tests/test_dd_math.py): glibc's pow
// and exp are NOT correctly rounded (<= 0.52 ULP), so ~0.08% of calls differ
// from CPython by one ULP (log: a few per million); in every such case the
// device holds the correctly rounded value.  A one-ULP difference only
// matters if it moves a node's int(score) across an integer or flips a
// comparison between values within one ULP of each other.
//
// __host__ __device__ so the identical code is checked on the host.
#pragma once

#include "jit_env.h"

namespace fksd {

struct dd { double hi, lo; };

__host__ __device__ inline dd two_sum(double a, double b) {
  double s = a + b;
  double bb = s - a;
  double e = (a - (s - bb)) + (b - bb);
  return {s, e};
}
__host__ __device__ inline dd quick_two_sum(double a, double b) {
  double s = a + b;
  return {s, b - (s - a)};
}
__host__ __device__ inline dd two_prod(double a, double b) {
  double p = a * b;
  return {p, fma(a, b, -p)};
}
__host__ __device__ inline dd dd_add(dd a, dd b) {
  dd s = two_sum(a.hi, b.hi);
  dd t = two_sum(a.lo, b.lo);
  s.lo += t.hi;
  s = quick_two_sum(s.hi, s.lo);
  s.lo += t.lo;
  return quick_two_sum(s.hi, s.lo);
}
// a + b where the two do not cancel (same sign, or |b| far below |a|): one
// two_sum plus the low parts (~2^-104 relative, the cancellation-free case of dd_add)
__host__ __device__ inline dd dd_add_nc(dd a, dd b) {
  dd s = two_sum(a.hi, b.hi);
  s.lo += a.lo + b.lo;
  return quick_two_sum(s.hi, s.lo);
}
__host__ __device__ inline dd dd_mul(dd a, dd b) {
  dd p = two_prod(a.hi, b.hi);
  p.lo += a.hi * b.lo + a.lo * b.hi;
  return quick_two_sum(p.hi, p.lo);
}
__host__ __device__ inline dd dd_mul_d(dd a, double b) {
  dd p = two_prod(a.hi, b);
  p.lo += a.lo * b;
  return quick_two_sum(p.hi, p.lo);
}
__host__ __device__ inline dd dd_ldexp(dd a, int e) { return {ldexp(a.hi, e), ldexp(a.lo, e)}; }

// 1/n! as double-doubles, n = 2..7 (the terms of e^r - 1 that need ~106 bits)
struct DdConst { double hi, lo; };
#define FKS_INV_FACT_DD                                                   \
  {{0.5, 0.0}, {0.16666666666666666, 9.25185853854297e-18},               \
   {0.041666666666666664, 2.3129646346357427e-18},                        \
   {0.008333333333333333, 1.1564823173178714e-19},                        \
   {0.001388888888888889, -5.300543954373577e-20},                        \
   {0.0001984126984126984, 1.7209558293420705e-22}}

// exp of a double-double argument; |a| <= 700 required (caller checks).
// a = k ln2 + 32 r, |r| <= ln2 / 64; e^r - 1 by a degree-12 polynomial whose
// terms r^8..r^12 (< 2^-68 of the sum) are summed in double and r^2..r^7 in
// double-double Horner steps with exact 1/n! constants (no divisions); then
// five squarings (1+s)^32 and the 2^k scale.  Relative error ~2^-100 (the
// rounding check of dd_round keeps a 2^-84 margin for pow, 2^-90 for exp/log).
__host__ __device__ inline dd dd_exp(dd a) {
  const dd ln2 = {6.931471805599452862e-01, 2.319046813846299558e-17};
  const double k = nearbyint(a.hi * 1.4426950408889634);
  dd r = dd_add(a, dd_mul_d({-ln2.hi, -ln2.lo}, k));
  r = dd_ldexp(r, -5);  // |r| < 0.0109
  const double rh = r.hi;
  // r^8 .. r^12 tail in double: ((((c12 r + c11) r + c10) r + c9) r + c8)
  double q = 2.08767569878681e-09;
  q = q * rh + 2.505210838544172e-08;
  q = q * rh + 2.755731922398589e-07;
  q = q * rh + 2.7557319223985893e-06;
  q = q * rh + 2.48015873015873e-05;
  const DdConst c[6] = FKS_INV_FACT_DD;
  dd p = {q, 0.0};
  // no step below cancels (|p r| <= 0.02 |c_n|, |r^2 p| <= 0.006 |r|, |s^2| <= 0.006 |2 s|,
  // |s| < 0.35 in 1 + s), so the short double-double add is exact enough
#pragma unroll
  for (int n = 5; n >= 0; --n) p = dd_add_nc(dd{c[n].hi, c[n].lo}, dd_mul(p, r));
  // p = 1/2 + r/6 + ... ; s = r + r^2 p = e^r - 1
  dd s = dd_add_nc(r, dd_mul(dd_mul(r, r), p));
  // (1+s)^(2^5): s <- 2s + s^2
  for (int i = 0; i < 5; ++i) s = dd_add_nc(dd_ldexp(s, 1), dd_mul(s, s));
  dd res = dd_add_nc({1.0, 0.0}, s);
  return dd_ldexp(res, (int)k);
}

// natural log of a positive finite double, ~106 bits (one Newton step on exp)
__host__ __device__ inline dd dd_log(double x) {
  const double y0 = log(x);
  dd e = dd_exp({-y0, 0.0});
  dd t = dd_mul_d(e, x);               // x * exp(-y0) ~ 1
  t = dd_add(t, {-1.0, 0.0});
  return dd_add({y0, 0.0}, t);         // y0 + (x e^-y0 - 1)
}

// round a double-double to double; returns false when too close to a
// rounding midpoint to trust (|distance| < 2^-90 relative)
__host__ __device__ inline bool dd_round(dd v, double& out, int rel_bits = 90, double abs_err = 0.0) {
  dd n = quick_two_sum(v.hi, v.lo);
  out = n.hi;
  if (n.hi == 0.0 || !isfinite(n.hi)) return true;
  int e;
  frexp(n.hi, &e);
  const double half_ulp = ldexp(1.0, e - 54);
  const double d1 = fabs(fabs(n.lo) - half_ulp);
  const double margin = fmax(ldexp(fabs(n.hi), -rel_bits), abs_err);
  return !(d1 <= margin);
}

// pow(x, y) for x > 0 finite, y finite, x != 1 (CPython already handled the
// special cases).  status: 0 ok, 1 overflow (inf), 2 defer to host.
__host__ __device__ inline int dd_pow(double x, double y, double& out) {
  if (y == 1.0) { out = x; return 0; }
  if (y == 2.0) { out = x * x; return isinf(out) ? 1 : 0; }
  if (y == 0.5) { out = sqrt(x); return 0; }
  dd L = dd_log(x);
  dd P = dd_mul_d(L, y);
  if (P.hi > 709.9) { out = INFINITY; return 1; }
  if (P.hi > 700.0 || P.hi < -700.0) return 2;   // near overflow / subnormal range: host
  dd r = dd_exp(P);
  return dd_round(r, out, 84) ? 0 : 2;
}

// exp(x), x finite: status 0 ok, 1 overflow, 2 defer
__host__ __device__ inline int dd_exp_d(double x, double& out) {
  if (x == 0.0) { out = 1.0; return 0; }
  if (x > 709.9) { out = INFINITY; return 1; }
  if (x > 700.0 || x < -700.0) return 2;
  return dd_round(dd_exp({x, 0.0}), out) ? 0 : 2;
}

// log(x), x > 0 finite: status 0 ok, 2 defer
__host__ __device__ inline int dd_log_d(double x, double& out) {
  if (x == 1.0) { out = 0.0; return 0; }
  return dd_round(dd_log(x), out, 90, 1e-30) ? 0 : 2;
}

}  // namespace fksd
