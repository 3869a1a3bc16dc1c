// CPython 3 numeric semantics for int64/double values (host side).
//
// Each function mirrors the CPython implementation it names
// (Objects/longobject.c, Objects/floatobject.c, Modules/mathmodule.c) for
// operands that fit the native subset; anything that would need a Python
// bigint or produce a complex number returns EXC_UNSUPPORTED so the caller
// re-runs the policy on the exact object engine.
#pragma once

#include <cerrno>
#include <cmath>
#include <cstdint>
#include <limits>

#include "fks/types.hpp"

namespace fks {

struct PyNum {
  int64_t i;
  double f;
  bool fl;  // true: float
};

inline PyNum pyi(int64_t v) { return PyNum{v, 0.0, false}; }
inline PyNum pyf(double v) { return PyNum{0, v, true}; }
inline double as_f(const PyNum& x) { return x.fl ? x.f : (double)x.i; }

constexpr double kTwo63 = 9223372036854775808.0;
constexpr int64_t kTwo53 = (int64_t)1 << 53;

inline bool truthy(const PyNum& x) { return x.fl ? (x.f != 0.0) : (x.i != 0); }

// ---- int helpers -------------------------------------------------------------
inline int py_add(const PyNum& a, const PyNum& b, PyNum& r) {
  if (!a.fl && !b.fl) {
    int64_t v;
    if (__builtin_add_overflow(a.i, b.i, &v)) return EXC_UNSUPPORTED;
    r = pyi(v); return EXC_NONE;
  }
  r = pyf(as_f(a) + as_f(b)); return EXC_NONE;
}
inline int py_sub(const PyNum& a, const PyNum& b, PyNum& r) {
  if (!a.fl && !b.fl) {
    int64_t v;
    if (__builtin_sub_overflow(a.i, b.i, &v)) return EXC_UNSUPPORTED;
    r = pyi(v); return EXC_NONE;
  }
  r = pyf(as_f(a) - as_f(b)); return EXC_NONE;
}
inline int py_mul(const PyNum& a, const PyNum& b, PyNum& r) {
  if (!a.fl && !b.fl) {
    int64_t v;
    if (__builtin_mul_overflow(a.i, b.i, &v)) return EXC_UNSUPPORTED;
    r = pyi(v); return EXC_NONE;
  }
  r = pyf(as_f(a) * as_f(b)); return EXC_NONE;
}
inline int py_tdiv(const PyNum& a, const PyNum& b, PyNum& r) {
  if (!a.fl && !b.fl) {
    if (b.i == 0) return EXC_ZERO_DIVISION;
    // exact operands => one correctly rounded division == long_true_divide
    if (a.i > kTwo53 || a.i < -kTwo53 || b.i > kTwo53 || b.i < -kTwo53) return EXC_UNSUPPORTED;
    r = pyf((double)a.i / (double)b.i); return EXC_NONE;
  }
  double y = as_f(b);
  if (y == 0.0) return EXC_ZERO_DIVISION;
  r = pyf(as_f(a) / y); return EXC_NONE;
}
// float_divmod (Objects/floatobject.c)
inline void py_float_divmod(double vx, double wx, double& floordiv, double& mod) {
  mod = std::fmod(vx, wx);
  double div = (vx - mod) / wx;
  if (mod != 0.0) {
    if ((wx < 0) != (mod < 0)) { mod += wx; div -= 1.0; }
  } else {
    mod = std::copysign(0.0, wx);
  }
  if (div != 0.0) {
    floordiv = std::floor(div);
    if (div - floordiv > 0.5) floordiv += 1.0;
  } else {
    floordiv = std::copysign(0.0, vx / wx);
  }
}
inline int py_fdiv(const PyNum& a, const PyNum& b, PyNum& r) {
  if (!a.fl && !b.fl) {
    if (b.i == 0) return EXC_ZERO_DIVISION;
    if (a.i == std::numeric_limits<int64_t>::min() && b.i == -1) return EXC_UNSUPPORTED;
    int64_t q = a.i / b.i, m = a.i % b.i;
    if (m != 0 && ((m < 0) != (b.i < 0))) q -= 1;
    r = pyi(q); return EXC_NONE;
  }
  double y = as_f(b);
  if (y == 0.0) return EXC_ZERO_DIVISION;
  double fd, md;
  py_float_divmod(as_f(a), y, fd, md);
  r = pyf(fd); return EXC_NONE;
}
inline int py_mod(const PyNum& a, const PyNum& b, PyNum& r) {
  if (!a.fl && !b.fl) {
    if (b.i == 0) return EXC_ZERO_DIVISION;
    if (b.i == -1) { r = pyi(0); return EXC_NONE; }
    int64_t m = a.i % b.i;
    if (m != 0 && ((m < 0) != (b.i < 0))) m += b.i;
    r = pyi(m); return EXC_NONE;
  }
  double vx = as_f(a), wx = as_f(b);
  if (wx == 0.0) return EXC_ZERO_DIVISION;
  double mod = std::fmod(vx, wx);
  if (mod != 0.0) {
    if ((wx < 0) != (mod < 0)) mod += wx;
  } else {
    mod = std::copysign(0.0, wx);
  }
  r = pyf(mod); return EXC_NONE;
}

inline bool dbl_is_odd_integer(double x) { return std::fmod(std::fabs(x), 2.0) == 1.0; }

// float_pow (Objects/floatobject.c, CPython 3.10)
inline int py_float_pow(double iv, double iw, PyNum& r) {
  if (iw == 0.0) { r = pyf(1.0); return EXC_NONE; }
  if (std::isnan(iv)) { r = pyf(iv); return EXC_NONE; }
  if (std::isnan(iw)) { r = pyf(iv == 1.0 ? 1.0 : iw); return EXC_NONE; }
  if (std::isinf(iw)) {
    double av = std::fabs(iv);
    if (av == 1.0) r = pyf(1.0);
    else if ((iw > 0.0) == (av > 1.0)) r = pyf(std::fabs(iw));
    else r = pyf(0.0);
    return EXC_NONE;
  }
  if (std::isinf(iv)) {
    bool odd = dbl_is_odd_integer(iw);
    if (iw > 0.0) r = pyf(odd ? iv : std::fabs(iv));
    else r = pyf(odd ? std::copysign(0.0, iv) : 0.0);
    return EXC_NONE;
  }
  if (iv == 0.0) {
    bool odd = dbl_is_odd_integer(iw);
    if (iw < 0.0) return EXC_ZERO_DIVISION;
    r = pyf(odd ? iv : 0.0);
    return EXC_NONE;
  }
  bool neg = false;
  if (iv < 0.0) {
    if (iw != std::floor(iw)) return EXC_UNSUPPORTED;  // complex result
    iv = -iv;
    neg = dbl_is_odd_integer(iw);
  }
  if (iv == 1.0) { r = pyf(neg ? -1.0 : 1.0); return EXC_NONE; }
  errno = 0;
  double ix = std::pow(iv, iw);
  bool overflow = std::isinf(ix);
  if (neg) ix = -ix;
  if (overflow) return EXC_OVERFLOW;
  r = pyf(ix);
  return EXC_NONE;
}

inline int py_pow(const PyNum& a, const PyNum& b, PyNum& r) {
  if (!a.fl && !b.fl) {
    if (b.i < 0) {
      if (a.i == 0) return EXC_ZERO_DIVISION;
      return py_float_pow((double)a.i, (double)b.i, r);
    }
    // exponentiation by squaring with overflow detection
    int64_t base = a.i, e = b.i, acc = 1;
    while (e > 0) {
      if (e & 1) { if (__builtin_mul_overflow(acc, base, &acc)) return EXC_UNSUPPORTED; }
      e >>= 1;
      if (e > 0 && __builtin_mul_overflow(base, base, &base)) return EXC_UNSUPPORTED;
    }
    r = pyi(acc);
    return EXC_NONE;
  }
  return py_float_pow(as_f(a), as_f(b), r);
}

// exact comparison (int vs float compared mathematically)
// returns -1, 0, 1, or 2 for unordered (nan)
inline int py_cmp(const PyNum& a, const PyNum& b) {
  if (!a.fl && !b.fl) return a.i < b.i ? -1 : (a.i > b.i ? 1 : 0);
  if (a.fl && b.fl) {
    if (std::isnan(a.f) || std::isnan(b.f)) return 2;
    return a.f < b.f ? -1 : (a.f > b.f ? 1 : 0);
  }
  const bool swap = !a.fl;  // make x the float, y the int
  const double x = swap ? b.f : a.f;
  const int64_t y = swap ? a.i : b.i;
  int c;
  if (std::isnan(x)) return 2;
  if (std::isinf(x)) c = x > 0 ? 1 : -1;
  else if (x >= kTwo63) c = 1;
  else if (x < -kTwo63) c = -1;
  else {
    double t = std::trunc(x);
    int64_t ti = (int64_t)t;
    if (ti != y) c = ti < y ? -1 : 1;
    else c = (x > t) ? 1 : ((x < t) ? -1 : 0);
  }
  return swap ? -c : c;
}

// int(x)
inline int py_int(const PyNum& a, PyNum& r) {
  if (!a.fl) { r = a; return EXC_NONE; }
  if (std::isnan(a.f)) return EXC_VALUE;
  if (std::isinf(a.f)) return EXC_OVERFLOW;
  double t = std::trunc(a.f);
  if (t >= kTwo63 || t < -kTwo63) return EXC_UNSUPPORTED;
  r = pyi((int64_t)t);
  return EXC_NONE;
}

// round(x) with one argument -> int (float___round___impl, ndigits None)
inline int py_round(const PyNum& a, PyNum& r) {
  if (!a.fl) { r = a; return EXC_NONE; }
  double x = a.f;
  double rounded = std::round(x);
  if (std::fabs(x - rounded) == 0.5) rounded = 2.0 * std::round(x / 2.0);
  return py_int(pyf(rounded), r);
}

// math module functions (math_1 / m_log / math_pow semantics)
inline int py_sqrt(const PyNum& a, PyNum& r) {
  double x = as_f(a);
  if (std::isnan(x)) { r = pyf(x); return EXC_NONE; }
  if (x < 0.0) return EXC_VALUE;
  r = pyf(std::sqrt(x)); return EXC_NONE;
}
inline int py_log_helper(const PyNum& a, double& out) {
  if (!a.fl) {
    if (a.i <= 0) return EXC_VALUE;
    out = std::log((double)a.i);
    return EXC_NONE;
  }
  double x = a.f;
  if (std::isnan(x)) { out = x; return EXC_NONE; }
  if (std::isinf(x)) { if (x > 0) { out = x; return EXC_NONE; } return EXC_VALUE; }
  if (x <= 0.0) return EXC_VALUE;
  out = std::log(x);
  return EXC_NONE;
}
inline int py_log(const PyNum& a, PyNum& r) {
  double v; int e = py_log_helper(a, v); if (e) return e; r = pyf(v); return EXC_NONE;
}
inline int py_logb(const PyNum& a, const PyNum& b, PyNum& r) {
  double num, den; int e = py_log_helper(a, num); if (e) return e;
  e = py_log_helper(b, den); if (e) return e;
  if (den == 0.0) return EXC_ZERO_DIVISION;
  r = pyf(num / den); return EXC_NONE;
}
inline int py_exp(const PyNum& a, PyNum& r) {
  double x = as_f(a);
  double v = std::exp(x);
  if (std::isinf(v) && std::isfinite(x)) return EXC_OVERFLOW;
  r = pyf(v); return EXC_NONE;
}
inline int py_trig(int op, const PyNum& a, PyNum& r) {  // 0 sin 1 cos 2 tan
  double x = as_f(a);
  if (std::isinf(x)) return EXC_VALUE;
  double v = op == 0 ? std::sin(x) : (op == 1 ? std::cos(x) : std::tan(x));
  r = pyf(v); return EXC_NONE;
}
inline int py_mpow(const PyNum& a, const PyNum& b, PyNum& r) {
  double x = as_f(a), y = as_f(b), v;
  if (!std::isfinite(x) || !std::isfinite(y)) {
    if (std::isnan(x)) v = (y == 0.0) ? 1.0 : x;
    else if (std::isnan(y)) v = (x == 1.0) ? 1.0 : y;
    else if (std::isinf(x)) {
      bool odd_y = std::isfinite(y) && std::fmod(std::fabs(y), 2.0) == 1.0;
      if (y > 0.) v = odd_y ? x : std::fabs(x);
      else if (y == 0.) v = 1.;
      else v = odd_y ? std::copysign(0., x) : 0.;
    } else {  // y infinite
      if (std::fabs(x) == 1.0) v = 1.;
      else if (y > 0. && std::fabs(x) > 1.0) v = y;
      else if (y < 0. && std::fabs(x) < 1.0) v = -y;
      else v = 0.;
    }
    r = pyf(v); return EXC_NONE;
  }
  v = std::pow(x, y);
  if (std::isnan(v)) return EXC_VALUE;
  if (std::isinf(v)) return x == 0.0 ? EXC_VALUE : EXC_OVERFLOW;
  r = pyf(v); return EXC_NONE;
}

}  // namespace fks
