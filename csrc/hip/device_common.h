// Device-side building blocks shared by the MI355X kernels: wave-64
// reductions, the 128-bit fixed-point exact accumulator and the packed
// event-key layout of the LDS heap.
#pragma once

#ifndef __HIPCC_RTC__   // hiprtc (policy JIT) provides these itself
#include <hip/hip_runtime.h>
#include <stdint.h>
#else
using __hip_internal::int8_t;
using __hip_internal::int16_t;
using __hip_internal::int32_t;
using __hip_internal::int64_t;
using __hip_internal::uint8_t;
using __hip_internal::uint16_t;
using __hip_internal::uint32_t;
using __hip_internal::uint64_t;
#ifndef INT64_MAX
#define INT64_MAX 0x7fffffffffffffffLL
#endif
#ifndef INT64_MIN
#define INT64_MIN (-INT64_MAX - 1)
#endif
#ifndef INT32_MAX
#define INT32_MAX 0x7fffffff
#endif
#endif

namespace fksd {

constexpr int kWave = 64;

// Address-space qualified pointers: generic pointers make the compiler emit
// FLAT memory instructions (one path for LDS and global, both counters, the
// slower one's latency).  LDS data goes through ds_*, HBM through global_*,
// and read-only launch data through scalar s_load.
#define FKS_LDS __attribute__((address_space(3)))
#define FKS_GLOBAL __attribute__((address_space(1)))
#define FKS_CONST __attribute__((address_space(4)))
template <class T>
__device__ __forceinline__ FKS_LDS T* lds_ptr(T* p) { return (FKS_LDS T*)p; }
template <class T>
__device__ __forceinline__ FKS_GLOBAL T* global_ptr(T* p) { return (FKS_GLOBAL T*)p; }
template <class T>
__device__ __forceinline__ const FKS_CONST T* const_ptr(const T* p) { return (const FKS_CONST T*)p; }

__device__ __forceinline__ int lane_id() { return __lane_id(); }

__device__ __forceinline__ int uni(int x) { return __builtin_amdgcn_readfirstlane(x); }
__device__ __forceinline__ uint32_t uni(uint32_t x) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)x); }
__device__ __forceinline__ int64_t uni64(int64_t x) {
  uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)x);
  uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)((uint64_t)x >> 32));
  return (int64_t)(((uint64_t)hi << 32) | lo);
}
__device__ __forceinline__ uint64_t uniu64(uint64_t x) { return (uint64_t)uni64((int64_t)x); }
__device__ __forceinline__ int readlane(int x, int l) { return __builtin_amdgcn_readlane(x, l); }
__device__ __forceinline__ int64_t readlane64(int64_t x, int l) {
  uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)x, l);
  uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)((uint64_t)x >> 32), l);
  return (int64_t)(((uint64_t)hi << 32) | lo);
}
__device__ __forceinline__ double readlane_f64(double x, int l) {
  return __longlong_as_double(readlane64(__double_as_longlong(x), l));
}

__device__ __forceinline__ int64_t shfl_xor64(int64_t v, int m) {
  int lo = __shfl_xor((int)(uint32_t)v, m, kWave);
  int hi = __shfl_xor((int)(uint32_t)((uint64_t)v >> 32), m, kWave);
  return (int64_t)(((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo);
}
__device__ __forceinline__ int64_t wave_max64(int64_t v) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) { int64_t o = shfl_xor64(v, m); v = o > v ? o : v; }
  return v;
}
__device__ __forceinline__ int64_t wave_sum64(int64_t v) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) v += shfl_xor64(v, m);
  return v;
}
// ---- DPP (register-crossbar) reductions: no LDS round trip --------------------
// Classic GFX9 wave64 reduction ladder: row_shr 1/2/3, row_shr 4 (bank mask),
// row_shr 8 (bank mask), row_bcast 15, row_bcast 31; the full result lands in
// lane 63.  Lanes without a DPP source keep `old` = the identity.
template <int CTRL, int ROW_MASK, int BANK_MASK>
__device__ __forceinline__ uint64_t dpp64(uint64_t v, uint64_t ident) {
  const int lo = __builtin_amdgcn_update_dpp((int)(uint32_t)ident, (int)(uint32_t)v, CTRL, ROW_MASK, BANK_MASK, false);
  const int hi = __builtin_amdgcn_update_dpp((int)(uint32_t)(ident >> 32), (int)(uint32_t)(v >> 32), CTRL, ROW_MASK,
                                             BANK_MASK, false);
  return ((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo;
}
struct OpMaxU64 {
  static constexpr uint64_t ident = 0;
  __device__ static uint64_t f(uint64_t a, uint64_t b) { return a > b ? a : b; }
};
struct OpSumU64 {
  static constexpr uint64_t ident = 0;
  __device__ static uint64_t f(uint64_t a, uint64_t b) { return a + b; }
};
template <class Op>
__device__ __forceinline__ uint64_t wave_reduce_dpp(uint64_t v) {
  const uint64_t x = v;                                // first three read the ORIGINAL values
  v = Op::f(v, dpp64<0x111, 0xF, 0xF>(x, Op::ident));  // row_shr:1
  v = Op::f(v, dpp64<0x112, 0xF, 0xF>(x, Op::ident));  // row_shr:2
  v = Op::f(v, dpp64<0x113, 0xF, 0xF>(x, Op::ident));  // row_shr:3
  v = Op::f(v, dpp64<0x114, 0xF, 0xE>(v, Op::ident));  // row_shr:4 bank_mask 0xe
  v = Op::f(v, dpp64<0x118, 0xF, 0xC>(v, Op::ident));  // row_shr:8 bank_mask 0xc
  v = Op::f(v, dpp64<0x142, 0xA, 0xF>(v, Op::ident));  // row_bcast:15 row_mask 0xa
  v = Op::f(v, dpp64<0x143, 0xC, 0xF>(v, Op::ident));  // row_bcast:31 row_mask 0xc
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, 63);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), 63);
  return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ uint64_t wave_max_u64(uint64_t v) { return wave_reduce_dpp<OpMaxU64>(v); }
__device__ __forceinline__ int64_t wave_sum_i64(int64_t v) { return (int64_t)wave_reduce_dpp<OpSumU64>((uint64_t)v); }
// swap adjacent lane pairs (quad_perm [1,0,3,2])
__device__ __forceinline__ uint64_t swap_pairs64(uint64_t v) {
  const int lo = __builtin_amdgcn_mov_dpp((int)(uint32_t)v, 0xB1, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_mov_dpp((int)(uint32_t)(v >> 32), 0xB1, 0xF, 0xF, false);
  return ((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo;
}

// Vector load whose address the compiler must treat as divergent: the result
// stays in VGPRs and is waited for (vmcnt) only where it is first used, so a
// uniform load can be issued early and overlap LDS work instead of being
// hoisted into SGPRs with an immediate wait.
__device__ __forceinline__ int4 load_vgpr(const int4* p) {
  const uint64_t a = (uint64_t)p;
  uint32_t lo = (uint32_t)a;
  asm volatile("v_mov_b32 %0, %0" : "+v"(lo));
  typedef int v4i __attribute__((ext_vector_type(4)));
  const FKS_GLOBAL v4i* q = reinterpret_cast<const FKS_GLOBAL v4i*>((a & 0xFFFFFFFF00000000ull) | lo);
  const v4i v = *q;   // global_load_dwordx4
  return make_int4(v.x, v.y, v.z, v.w);
}

__device__ __forceinline__ uint64_t ballot(bool p) { return __ballot(p); }
__device__ __forceinline__ int first_lane(uint64_t m) { return __ffsll((unsigned long long)m) - 1; }

// ---- exact accumulator (host twin: csrc/include/fks/exact_mean.hpp) --------
using i128 = __int128;
using u128 = unsigned __int128;

struct FixedAccD {
  i128 sum;
  int64_t count;
  int32_t inexact;
  __device__ void init() { sum = 0; count = 0; inexact = 0; }
  // v is wave-uniform; all lanes do the same (scalarised) work.
  __device__ void add(double v) {
    ++count;
    uint64_t bits = (uint64_t)__double_as_longlong(v);
    int E = (int)((bits >> 52) & 0x7FF);
    uint64_t frac = bits & ((1ull << 52) - 1);
    if (E == 0 && frac == 0) return;
    if (E == 0x7FF || E == 0) { inexact = 1; return; }  // inf/nan, subnormal
    uint64_t M = frac | (1ull << 52);
    int shift = E - 979;  // v * 2^96 = M * 2^(E-1075+96)
    if (shift < 0) {
      if (shift <= -53 || (M & ((1ull << (-shift)) - 1))) { inexact = 1; return; }
      M >>= (-shift);
      shift = 0;
    }
    if (shift > 126 - 53) { inexact = 1; return; }
    i128 t = (i128)(u128)M << shift;
    if (bits >> 63) t = -t;
    sum += t;
    u128 mag = sum < 0 ? (u128)(-sum) : (u128)sum;
    if (mag >> 126) inexact = 1;
  }
};

// The replay's five exact accumulators (4 utilisation means + fragmentation)
// spread over lanes: accumulator k lives in lane k, so the whole set costs a
// handful of VGPRs instead of ~35 loop-carried SGPRs (which the compiler
// would otherwise spill through v_writelane / v_readlane on every event).
// Same arithmetic as FixedAccD.
struct LaneAcc {
  i128 sum;
  int64_t count;
  int32_t inexact;
  __device__ void init() { sum = 0; count = 0; inexact = 0; }
  // v is wave-uniform; adds it to accumulator k
  __device__ void add(int k, double v) {
    const bool mine = lane_id() == k;
    uint64_t bits = (uint64_t)__double_as_longlong(v);
    const int E = (int)((bits >> 52) & 0x7FF);
    const uint64_t frac = bits & ((1ull << 52) - 1);
    if (mine) ++count;
    if (E == 0 && frac == 0) return;
    bool bad = (E == 0x7FF || E == 0);   // inf/nan, subnormal
    uint64_t M = frac | (1ull << 52);
    int shift = E - 979;  // v * 2^96 = M * 2^(E-1075+96)
    if (!bad && shift < 0) {
      if (shift <= -53 || (M & ((1ull << (-shift)) - 1))) bad = true;
      else { M >>= (-shift); shift = 0; }
    }
    if (!bad && shift > 126 - 53) bad = true;
    if (bad) { if (mine) inexact = 1; return; }
    i128 t = (i128)(u128)M << shift;
    if (bits >> 63) t = -t;
    if (mine) {
      sum += t;
      const u128 mag = sum < 0 ? (u128)(-sum) : (u128)sum;
      if (mag >> 126) inexact = 1;
    }
  }
};

// Correctly rounded A * 2^-96 / n  (bit-serial long division; no libcalls).
__device__ inline double fixed_div_round_dev(i128 A, uint64_t n) {
  if (A == 0 || n == 0) return 0.0;
  const bool neg = A < 0;
  u128 a = neg ? (u128)(-A) : (u128)A;
  // q = a / n, r = a % n by restoring division (128 iterations)
  u128 q = 0, r = 0;
  for (int i = 127; i >= 0; --i) {
    r = (r << 1) | ((a >> i) & 1);
    if (r >= n) { r -= n; q |= ((u128)1 << i); }
  }
  int exp2 = -96;
  bool sticky = false;
  if (q >> 64) {
    int extra = 0;
    while (q >> (64 + extra)) ++extra;
    u128 dropped = q & (((u128)1 << extra) - 1);
    sticky = dropped != 0 || r != 0;
    q >>= extra;
    exp2 += extra;
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
  uint64_t M = (uint64_t)q;
  uint64_t low = M & 0x7FFull;
  uint64_t m53 = M >> 11;
  exp2 += 11;
  if (low > 0x400ull || (low == 0x400ull && (sticky || (m53 & 1)))) {
    ++m53;
    if (m53 >> 53) { m53 >>= 1; ++exp2; }
  }
  double v = ldexp((double)m53, exp2);
  return neg ? -v : v;
}

// ---- FNV-style event hash (host twin: fks::mix_event) -----------------------
__device__ __forceinline__ uint64_t mix_event(uint64_t h, uint64_t a, uint64_t b) {
  h ^= a + 0x9E3779B97F4A7C15ull + (h << 6) + (h >> 2);
  h *= 0x100000001B3ull;
  h ^= b + 0x9E3779B97F4A7C15ull + (h << 6) + (h >> 2);
  h *= 0x100000001B3ull;
  return h;
}

}  // namespace fksd
