// Correctly rounded exp / log / pow for the device interpreter.
//
// CPython delegates `**`, math.exp, math.log and math.pow to glibc, whose
// results are correctly rounded except in rare hard cases.  The device
// evaluates the same functions in double-double arithmetic (~2^-100
// relative error) and rounds once, so it returns the correctly rounded
// double; results that land within 2^-90 of a rounding midpoint (the exact
// tie cases, e.g. small integer powers) are reported as `defer` and the
// policy is re-run on the host, where glibc decides.
//
// __host__ __device__ so the identical code is unit-tested on the host
// against glibc (tests/test_dd_math.py).
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

// exp of a double-double argument; |a| <= 700 required (caller checks).
__host__ __device__ inline dd dd_exp(dd a) {
  const dd ln2 = {6.931471805599452862e-01, 2.319046813846299558e-17};
  const double k = nearbyint(a.hi / ln2.hi);
  dd r = dd_add(a, dd_mul_d({-ln2.hi, -ln2.lo}, k));
  r = dd_ldexp(r, -10);  // |r| < 3.4e-4
  // e^r - 1 by Taylor to r^11
  dd term = r, s = r;
  double inv = 1.0;
  for (int n = 2; n <= 11; ++n) {
    term = dd_mul(term, r);
    inv = 1.0 / (double)n;
    // term_n = term_{n-1} * r / n  (divide exactly by a small integer in dd)
    dd q = {term.hi * inv, 0.0};
    // refine q = term / n with one correction step
    dd back = two_prod(q.hi, (double)n);
    double rem = ((term.hi - back.hi) - back.lo + term.lo) / (double)n;
    term = quick_two_sum(q.hi, rem);
    s = dd_add(s, term);
  }
  (void)inv;
  // (1+s)^(2^10): s <- 2s + s^2
  for (int i = 0; i < 10; ++i) s = dd_add(dd_add(s, s), dd_mul(s, s));
  dd res = dd_add({1.0, 0.0}, s);
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
