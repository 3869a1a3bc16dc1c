// Python number semantics on the device (int64 / double with CPython's
// int/float rules, floor division, modulo, pow, math.exp/log/pow, exact
// int-vs-float comparison), shared by the bytecode VM (vm_dev.hip.h) and the
// native program backend (policy/native_codegen.py emits C++ that calls these
// helpers; ops/jit.py compiles it for gfx950 at run time).  Executable spec:
// csrc/include/fks/pyops.hpp + csrc/cpu/vm_cpu.hpp.
//
// Builds in three environments (jit_env.h): hipcc (the replay kernels), the
// standalone device-only JIT compile (no HIP headers, FKS_JIT) and a host g++
// build of generated programs (FKS_HOST_JIT, tests / CPU-native path).
#pragma once

#include "jit_env.h"
#include "exc_codes.h"
#include "glibc_math.h"

namespace fksd {

enum VmOp : int {
  OP_NOP = 0, OP_CONST = 1, OP_MOV = 2, OP_POD = 3, OP_NODE = 4, OP_GPU = 5, OP_GLIST_ALL = 6,
  OP_GLIST_LEN = 7, OP_GLIST_GET = 8, OP_GLIST_SLICE = 9, OP_GLIST_NEW = 10, OP_GLIST_APPEND = 11,
  OP_GLIST_INSERT = 12, OP_ADD = 20, OP_SUB = 21, OP_MUL = 22, OP_TDIV = 23, OP_FDIV = 24, OP_MOD = 25,
  OP_POW = 26, OP_NEG = 27, OP_POS = 28, OP_NOT = 29, OP_TRUTH = 30, OP_LT = 31, OP_LE = 32, OP_GT = 33,
  OP_GE = 34, OP_EQ = 35, OP_NE = 36, OP_ABS = 40, OP_INT = 41, OP_FLOAT = 42, OP_ROUND = 43,
  OP_MIN2 = 44, OP_MAX2 = 45, OP_SQRT = 46, OP_LOG = 47, OP_LOGB = 48, OP_EXP = 49, OP_MPOW = 50,
  OP_SIN = 51, OP_COS = 52, OP_TAN = 53, OP_IF = 60, OP_ELSE = 61, OP_ENDIF = 62, OP_LOOP_BEGIN = 63,
  OP_LOOP_TEST = 64, OP_LOOP_CONT = 65, OP_LOOP_NEXT = 66, OP_LOOP_EXIT = 67, OP_BREAK = 68,
  OP_CONTINUE = 69, OP_RET = 70, OP_RAISE = 71, OP_END = 72, OP_ISINT = 73,
};

#if defined(FKS_HOST_JIT)
struct Ret2 { int64_t x, y; };
#else
typedef long long Ret2 __attribute__((ext_vector_type(2)));
#endif

// ---- Python numbers ------------------------------------------------------------
struct PyN {
  int64_t b;  // int value or double bits
  bool fl;
};
__device__ __forceinline__ PyN pi(int64_t v) { return {v, false}; }
__device__ __forceinline__ PyN pf(double v) { return {__double_as_longlong(v), true}; }
__device__ __forceinline__ double fv(const PyN& x) { return x.fl ? __longlong_as_double(x.b) : (double)x.b; }
__device__ __forceinline__ bool truthy(const PyN& x) { return x.fl ? (__longlong_as_double(x.b) != 0.0) : (x.b != 0); }

constexpr double kTwo63d = 9223372036854775808.0;
constexpr int64_t kTwo53i = (int64_t)1 << 53;

// int-vs-float comparison (exact, CPython float_richcompare): out of line
// (scalar arguments: a struct passed by value to an out-of-line function
// travels through scratch memory on AMDGPU)
__device__ inline __noinline__ int d_cmp_mixed_s(int64_t ab, int64_t bb, bool swap) {
  const double x = __longlong_as_double(swap ? bb : ab);
  const int64_t y = swap ? ab : bb;
  int c;
  if (isnan(x)) return 2;
  if (isinf(x)) c = x > 0 ? 1 : -1;
  else if (x >= kTwo63d) c = 1;
  else if (x < -kTwo63d) c = -1;
  else {
    const double t = trunc(x);
    const int64_t ti = (int64_t)t;
    if (ti != y) c = ti < y ? -1 : 1;
    else c = (x > t) ? 1 : ((x < t) ? -1 : 0);
  }
  return swap ? -c : c;
}

__device__ __forceinline__ int d_cmp(const PyN& a, const PyN& b) {
  if (!a.fl && !b.fl) return a.b < b.b ? -1 : (a.b > b.b ? 1 : 0);
  if (a.fl && b.fl) {
    const double x = __longlong_as_double(a.b), y = __longlong_as_double(b.b);
    if (isnan(x) || isnan(y)) return 2;
    return x < y ? -1 : (x > y ? 1 : 0);
  }
  return d_cmp_mixed_s(a.b, b.b, !a.fl);
}

__device__ __forceinline__ bool dbl_odd_int(double x) { return fmod(fabs(x), 2.0) == 1.0; }

__device__ __forceinline__ int d_float_pow_impl(double iv, double iw, PyN& r) {
  if (iw == 0.0) { r = pf(1.0); return EXC_NONE; }
  if (isnan(iv)) { r = pf(iv); return EXC_NONE; }
  if (isnan(iw)) { r = pf(iv == 1.0 ? 1.0 : iw); return EXC_NONE; }
  if (isinf(iw)) {
    const double av = fabs(iv);
    if (av == 1.0) r = pf(1.0);
    else if ((iw > 0.0) == (av > 1.0)) r = pf(fabs(iw));
    else r = pf(0.0);
    return EXC_NONE;
  }
  if (isinf(iv)) {
    const bool odd = dbl_odd_int(iw);
    if (iw > 0.0) r = pf(odd ? iv : fabs(iv));
    else r = pf(odd ? copysign(0.0, iv) : 0.0);
    return EXC_NONE;
  }
  if (iv == 0.0) {
    const bool odd = dbl_odd_int(iw);
    if (iw < 0.0) return EXC_ZERO_DIVISION;
    r = pf(odd ? iv : 0.0);
    return EXC_NONE;
  }
  bool neg = false;
  if (iv < 0.0) {
    if (iw != floor(iw)) return EXC_UNSUPPORTED;  // complex
    iv = -iv;
    neg = dbl_odd_int(iw);
  }
  if (iv == 1.0) { r = pf(neg ? -1.0 : 1.0); return EXC_NONE; }
  double ix;
  const int st = gm::pow(iv, iw, ix);   // glibc's pow, bit for bit (glibc_math.h)
  if (st == 1) return EXC_OVERFLOW;
  r = pf(neg ? -ix : ix);
  return EXC_NONE;
}

__device__ inline __noinline__ Ret2 d_float_pow_s(double iv, double iw) {
  PyN r = pi(0);
  const int e = d_float_pow_impl(iv, iw, r);
  Ret2 o;
  o.x = r.b;
  o.y = (r.fl ? 1 : 0) | ((int64_t)e << 8);
  return o;
}
__device__ __forceinline__ int d_float_pow(double iv, double iw, PyN& r) {
  const Ret2 o = d_float_pow_s(iv, iw);
  r = PyN{(int64_t)o.x, (o.y & 1) != 0};
  return (int)(o.y >> 8);
}

// Full Python binary-operator semantics.  The interpreter inlines the common
// cases (int/int and float add, sub, mul, true division) and calls this out
// of line for the rest, which keeps the dispatch loop small enough for the
// instruction cache.
__device__ __forceinline__ int d_binop_impl(int op, const PyN& a, const PyN& b, PyN& r) {
  const bool ii = !a.fl && !b.fl;
  switch (op) {
    case OP_ADD: {
      if (ii) { int64_t v; if (__builtin_add_overflow(a.b, b.b, &v)) return EXC_UNSUPPORTED; r = pi(v); return EXC_NONE; }
      r = pf(fv(a) + fv(b)); return EXC_NONE;
    }
    case OP_SUB: {
      if (ii) { int64_t v; if (__builtin_sub_overflow(a.b, b.b, &v)) return EXC_UNSUPPORTED; r = pi(v); return EXC_NONE; }
      r = pf(fv(a) - fv(b)); return EXC_NONE;
    }
    case OP_MUL: {
      if (ii) { int64_t v; if (__builtin_mul_overflow(a.b, b.b, &v)) return EXC_UNSUPPORTED; r = pi(v); return EXC_NONE; }
      r = pf(fv(a) * fv(b)); return EXC_NONE;
    }
    case OP_TDIV: {
      if (ii) {
        if (b.b == 0) return EXC_ZERO_DIVISION;
        if (a.b > kTwo53i || a.b < -kTwo53i || b.b > kTwo53i || b.b < -kTwo53i) return EXC_UNSUPPORTED;
        r = pf((double)a.b / (double)b.b); return EXC_NONE;
      }
      const double y = fv(b);
      if (y == 0.0) return EXC_ZERO_DIVISION;
      r = pf(fv(a) / y); return EXC_NONE;
    }
    case OP_FDIV: {
      if (ii) {
        if (b.b == 0) return EXC_ZERO_DIVISION;
        if (a.b == INT64_MIN && b.b == -1) return EXC_UNSUPPORTED;
        int64_t q = a.b / b.b, m = a.b % b.b;
        if (m != 0 && ((m < 0) != (b.b < 0))) q -= 1;
        r = pi(q); return EXC_NONE;
      }
      const double vx = fv(a), wx = fv(b);
      if (wx == 0.0) return EXC_ZERO_DIVISION;
      double mod = fmod(vx, wx);
      double div = (vx - mod) / wx;
      if (mod != 0.0) { if ((wx < 0) != (mod < 0)) { mod += wx; div -= 1.0; } }
      double fd;
      if (div != 0.0) { fd = floor(div); if (div - fd > 0.5) fd += 1.0; }
      else fd = copysign(0.0, vx / wx);
      r = pf(fd); return EXC_NONE;
    }
    case OP_MOD: {
      if (ii) {
        if (b.b == 0) return EXC_ZERO_DIVISION;
        if (b.b == -1) { r = pi(0); return EXC_NONE; }
        int64_t m = a.b % b.b;
        if (m != 0 && ((m < 0) != (b.b < 0))) m += b.b;
        r = pi(m); return EXC_NONE;
      }
      const double vx = fv(a), wx = fv(b);
      if (wx == 0.0) return EXC_ZERO_DIVISION;
      double mod = fmod(vx, wx);
      if (mod != 0.0) { if ((wx < 0) != (mod < 0)) mod += wx; }
      else mod = copysign(0.0, wx);
      r = pf(mod); return EXC_NONE;
    }
    case OP_POW: {
      if (ii) {
        if (b.b < 0) {
          if (a.b == 0) return EXC_ZERO_DIVISION;
          return d_float_pow((double)a.b, (double)b.b, r);
        }
        int64_t base = a.b, e = b.b, acc = 1;
        while (e > 0) {
          if (e & 1) { if (__builtin_mul_overflow(acc, base, &acc)) return EXC_UNSUPPORTED; }
          e >>= 1;
          if (e > 0 && __builtin_mul_overflow(base, base, &base)) return EXC_UNSUPPORTED;
        }
        r = pi(acc); return EXC_NONE;
      }
      return d_float_pow(fv(a), fv(b), r);
    }
    case OP_LOGB: {
      double num = 0.0, den = 1.0;
      for (int k = 0; k < 2; ++k) {
        const PyN& x = k == 0 ? a : b;
        double out;
        if (!x.fl) {
          if (x.b <= 0) return EXC_VALUE;
          gm::log((double)x.b, out);
        } else {
          const double v = __longlong_as_double(x.b);
          if (isnan(v)) out = v;
          else if (isinf(v)) { if (v > 0) out = v; else return EXC_VALUE; }
          else if (v <= 0.0) return EXC_VALUE;
          else gm::log(v, out);
        }
        (k == 0 ? num : den) = out;
      }
      if (den == 0.0) return EXC_ZERO_DIVISION;
      r = pf(num / den); return EXC_NONE;
    }
    case OP_MPOW: {
      const double x = fv(a), y = fv(b);
      double v;
      if (!isfinite(x) || !isfinite(y)) {
        if (isnan(x)) v = (y == 0.0) ? 1.0 : x;
        else if (isnan(y)) v = (x == 1.0) ? 1.0 : y;
        else if (isinf(x)) {
          const bool odd_y = isfinite(y) && fmod(fabs(y), 2.0) == 1.0;
          if (y > 0.) v = odd_y ? x : fabs(x);
          else if (y == 0.) v = 1.;
          else v = odd_y ? copysign(0., x) : 0.;
        } else {
          if (fabs(x) == 1.0) v = 1.;
          else if (y > 0. && fabs(x) > 1.0) v = y;
          else if (y < 0. && fabs(x) < 1.0) v = -y;
          else v = 0.;
        }
        r = pf(v); return EXC_NONE;
      }
      // finite ** finite through libm semantics: reuse the float_pow core
      if (x == 0.0) {
        if (y < 0.0) return EXC_VALUE;            // pow(0, neg) = inf -> EDOM
        r = pf(dbl_odd_int(y) ? x : (y == 0.0 ? 1.0 : 0.0)); return EXC_NONE;
      }
      if (x < 0.0 && y != floor(y)) return EXC_VALUE;  // nan -> EDOM
      PyN t;
      const int e = d_float_pow(x, y, t);
      if (e == EXC_ZERO_DIVISION) return EXC_VALUE;
      if (e) return e;
      r = t; return EXC_NONE;
    }
  }
  return EXC_UNSUPPORTED;
}

__device__ __forceinline__ int d_unop_impl(int op, const PyN& a, PyN& r) {
  switch (op) {
    case OP_NEG:
      if (a.fl) { r = pf(-__longlong_as_double(a.b)); return EXC_NONE; }
      if (a.b == INT64_MIN) return EXC_UNSUPPORTED;
      r = pi(-a.b); return EXC_NONE;
    case OP_POS: r = a; return EXC_NONE;
    case OP_NOT: r = pi(truthy(a) ? 0 : 1); return EXC_NONE;
    case OP_TRUTH: r = pi(truthy(a) ? 1 : 0); return EXC_NONE;
    case OP_ISINT: r = pi(a.fl ? 0 : 1); return EXC_NONE;
    case OP_ABS:
      if (a.fl) { r = pf(fabs(__longlong_as_double(a.b))); return EXC_NONE; }
      if (a.b == INT64_MIN) return EXC_UNSUPPORTED;
      r = pi(a.b < 0 ? -a.b : a.b); return EXC_NONE;
    case OP_FLOAT: r = pf(fv(a)); return EXC_NONE;
    case OP_INT:
    case OP_ROUND: {
      if (!a.fl) { r = a; return EXC_NONE; }
      double x = __longlong_as_double(a.b);
      if (op == OP_ROUND) {
        double rd = round(x);
        if (fabs(x - rd) == 0.5) rd = 2.0 * round(x / 2.0);
        x = rd;
      }
      if (isnan(x)) return EXC_VALUE;
      if (isinf(x)) return EXC_OVERFLOW;
      const double t = trunc(x);
      if (t >= kTwo63d || t < -kTwo63d) return EXC_UNSUPPORTED;
      r = pi((int64_t)t); return EXC_NONE;
    }
    case OP_SQRT: {
      const double x = fv(a);
      if (isnan(x)) { r = pf(x); return EXC_NONE; }
      if (x < 0.0) return EXC_VALUE;
      r = pf(sqrt(x)); return EXC_NONE;
    }
    case OP_LOG: {
      double out;
      if (!a.fl) {
        if (a.b <= 0) return EXC_VALUE;
        gm::log((double)a.b, out);
      } else {
        const double v = __longlong_as_double(a.b);
        if (isnan(v)) out = v;
        else if (isinf(v)) { if (v > 0) out = v; else return EXC_VALUE; }
        else if (v <= 0.0) return EXC_VALUE;
        else gm::log(v, out);
      }
      r = pf(out); return EXC_NONE;
    }
    case OP_EXP: {
      const double x = fv(a);
      if (isnan(x)) { r = pf(x); return EXC_NONE; }
      if (isinf(x)) { r = pf(x > 0 ? x : 0.0); return EXC_NONE; }
      double out;
      if (gm::exp(x, out) == 1) return EXC_OVERFLOW;
      r = pf(out); return EXC_NONE;
    }
    case OP_SIN: case OP_COS: case OP_TAN:
      return EXC_UNSUPPORTED;  // no correctly rounded device version: host decides
  }
  return EXC_UNSUPPORTED;
}

// Out-of-line entry points: arguments and results travel by value (registers),
// so the interpreter's result slot never has to live in scratch memory.
struct PyR {
  int64_t b;
  int32_t fl;
  int32_t e;
};
// Out-of-line entry points with scalar arguments and a two-register vector
// result (value bits, fl | exc << 8): nothing goes through scratch memory.
// These are also the runtime library of natively compiled programs
// (jit_abi.h rt_binop / rt_unop).
__device__ __forceinline__ Ret2 mk_ret2(const PyN& r, int e) {
  Ret2 o;
  o.x = r.b;
  o.y = (r.fl ? 1 : 0) | ((int64_t)e << 8);
  return o;
}
__device__ __forceinline__ PyR from_ret2(Ret2 o) { return PyR{(int64_t)o.x, (int32_t)(o.y & 1), (int32_t)(o.y >> 8)}; }
__device__ inline __noinline__ Ret2 d_binop_s(int op, int64_t ab, int32_t afl, int64_t bb, int32_t bfl) {
  PyN r = pi(0);
  const int e = d_binop_impl(op, PyN{ab, afl != 0}, PyN{bb, bfl != 0}, r);
  return mk_ret2(r, e);
}
__device__ inline __noinline__ Ret2 d_unop_s(int op, int64_t ab, int32_t afl) {
  PyN r = pi(0);
  const int e = d_unop_impl(op, PyN{ab, afl != 0}, r);
  return mk_ret2(r, e);
}
__device__ __forceinline__ PyR d_binop(int op, PyN a, PyN b) { return from_ret2(d_binop_s(op, a.b, a.fl, b.b, b.fl)); }
__device__ __forceinline__ PyR d_unop(int op, PyN a) { return from_ret2(d_unop_s(op, a.b, a.fl)); }

}  // namespace fksd
