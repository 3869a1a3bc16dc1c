// Build environment of the device math / Python-number headers.
//
//   (default)     hipcc: HIP runtime headers, ocml math.
//   FKS_JIT       standalone device-only clang compile of generated policy
//                 programs (ops/jit.py): no HIP headers and no device
//                 libraries, so a batch compiles in tens of milliseconds.
//                 Math comes from LLVM intrinsics (floor, trunc, sqrt, fma,
//                 ... are exact or correctly rounded) plus the exact integer
//                 fmod below (exp / log / pow: glibc_math.h).
//   FKS_HOST_JIT  the same generated C++ built for the host with g++
//                 (CPU-native program path and codegen tests).
#pragma once

#if defined(FKS_JIT)

#define __device__ __attribute__((device))
#define __host__ __attribute__((host))
#define __global__ __attribute__((global))
#define __forceinline__ inline __attribute__((always_inline))
#define __noinline__ __attribute__((noinline))
typedef signed char int8_t;
typedef short int16_t;
typedef int int32_t;
typedef long long int64_t;
typedef unsigned char uint8_t;
typedef unsigned short uint16_t;
typedef unsigned int uint32_t;
typedef unsigned long long uint64_t;
#define INT64_MAX 0x7fffffffffffffffLL
#define INT64_MIN (-INT64_MAX - 1)
#define INT32_MAX 0x7fffffff
#define INFINITY (__builtin_inff())

namespace fksd {
__device__ inline bool isnan(double x) { return __builtin_isnan(x); }
__device__ inline bool isinf(double x) { return __builtin_isinf(x); }
__device__ inline bool isfinite(double x) { return __builtin_isfinite(x); }
__device__ inline double fabs(double x) { return __builtin_fabs(x); }
__device__ inline double floor(double x) { return __builtin_floor(x); }
__device__ inline double trunc(double x) { return __builtin_trunc(x); }
__device__ inline double round(double x) { return __builtin_round(x); }
__device__ inline double nearbyint(double x) { return __builtin_nearbyint(x); }
__device__ inline double copysign(double x, double y) { return __builtin_copysign(x, y); }
__device__ inline double sqrt(double x) { return __builtin_sqrt(x); }
__device__ inline double fma(double a, double b, double c) { return __builtin_fma(a, b, c); }
__device__ inline double fmax(double a, double b) { return __builtin_fmax(a, b); }
__device__ inline double ldexp(double x, int e) { return __builtin_ldexp(x, e); }
__device__ inline double frexp(double x, int* e) { return __builtin_frexp(x, e); }
__device__ inline long long __double_as_longlong(double x) { return __builtin_bit_cast(long long, x); }
__device__ inline double __longlong_as_double(long long x) { return __builtin_bit_cast(double, x); }
}  // namespace fksd

#elif defined(FKS_HOST_JIT)

#include <cmath>
#include <cstdint>
#include <cstring>
#define __device__
#define __host__
#define __global__
#define __forceinline__ inline __attribute__((always_inline))
#define __noinline__ __attribute__((noinline))
namespace fksd {
using std::copysign; using std::fabs; using std::floor; using std::fma; using std::fmax; using std::frexp;
using std::isfinite; using std::isinf; using std::isnan; using std::ldexp; using std::log; using std::nearbyint;
using std::round; using std::sqrt; using std::trunc;
inline long long __double_as_longlong(double x) { long long v; std::memcpy(&v, &x, 8); return v; }
inline double __longlong_as_double(long long x) { double v; std::memcpy(&v, &x, 8); return v; }
}  // namespace fksd

#else

#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#endif

namespace fksd {

// Exact IEEE fmod by shift-and-subtract on the significands (the result of
// fmod is always representable, so every correct algorithm returns the same
// bits as glibc / ocml).  Used where no device library is linked.
__host__ __device__ inline double exact_fmod(double x, double y) {
  uint64_t ux = (uint64_t)__double_as_longlong(x), uy = (uint64_t)__double_as_longlong(y);
  int ex = (int)((ux >> 52) & 0x7FF), ey = (int)((uy >> 52) & 0x7FF);
  const uint64_t sx = ux >> 63;
  if ((uy << 1) == 0 || (ey == 0x7FF && (uy << 12) != 0) || ex == 0x7FF) return (x * y) / (x * y);
  if ((ux << 1) <= (uy << 1)) return (ux << 1) == (uy << 1) ? 0.0 * x : x;
  uint64_t i;
  if (!ex) {
    for (i = ux << 12; (i >> 63) == 0; --ex, i <<= 1) {}
    ux <<= -ex + 1;
  } else {
    ux &= ~0ull >> 12;
    ux |= 1ull << 52;
  }
  if (!ey) {
    for (i = uy << 12; (i >> 63) == 0; --ey, i <<= 1) {}
    uy <<= -ey + 1;
  } else {
    uy &= ~0ull >> 12;
    uy |= 1ull << 52;
  }
  for (; ex > ey; --ex) {
    i = ux - uy;
    if ((i >> 63) == 0) {
      if (i == 0) return 0.0 * x;
      ux = i;
    }
    ux <<= 1;
  }
  i = ux - uy;
  if ((i >> 63) == 0) {
    if (i == 0) return 0.0 * x;
    ux = i;
  }
  for (; (ux >> 52) == 0; ux <<= 1, --ex) {}
  if (ex > 0) {
    ux -= 1ull << 52;
    ux |= (uint64_t)ex << 52;
  } else {
    ux >>= -ex + 1;
  }
  ux |= sx << 63;
  return __longlong_as_double((long long)ux);
}

#if defined(FKS_JIT)
__device__ inline double fmod(double x, double y) { return exact_fmod(x, y); }
#endif

}  // namespace fksd
