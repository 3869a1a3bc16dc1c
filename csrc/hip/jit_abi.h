// ABI between the precompiled replay kernels and natively compiled policy
// programs (policy/native_codegen.py -> ops/jit.py -> hipModuleLoadData).
//
// A program is `int64_t fks_prog_<i>(FKS_PROG_ARGS)`: it scores ONE
// (pod, node) pair for the calling lane and returns the reference's
// `int(max(0, priority_function(pod, node)))` (>= 0) or -ExcCode.  The replay
// kernel (k_replay_native, replay_kernels.hip FKS_KIND 4) calls it through a
// function pointer read from the launch's per-policy pointer table: the JIT
// code object is loaded next to the extension's code object and reached with
// an ordinary indirect call (s_swappc), so only the small scorer is compiled
// per generation, never the replay loop.  The caller kernel's register
// allocation is raised to kJitVgprs / kJitSgprs (fks_reg_floor below) and
// ops/jit.py verifies each program's resource use against those limits.
#pragma once

#include "pyops_dev.h"

namespace fksd {

constexpr int kJitVgprs = 128;   // VGPRs the calling kernel allocates (register floor)
constexpr int kJitSgprs = 102;   // numbered SGPRs the calling kernel allocates (all of s0-s101)

// pod fields: p_gpu = gpu_milli | num_gpu << 16 (the device pod record's packing);
// kc = [instruction budget, constant payloads...] of the policy (int64, float bits)
// n_gpu_ng = (uint16)free GPUs | GPU count << 16: the argument list is 31
// dwords, all in VGPRs (v31 holds the work-item ids; a 32nd dword would be
// passed through scratch memory on every call)
__device__ __forceinline__ int32_t pack_gpu_ng(int32_t gpu_left, int32_t ngpus) {
  return (int32_t)(((uint32_t)gpu_left & 0xFFFFu) | ((uint32_t)ngpus << 16));
}
// kc = the policy's constant block, copied into the calling wave's LDS when the
// policy starts (a constant read is one ds_read_b64 instead of a dependent
// global load on every use); a program may hold at most kKcLds entries
// (native_codegen rejects larger blocks, which then run on the VM engines)
constexpr int kKcLds = 256;
#if defined(FKS_HOST_JIT)
typedef const int64_t* KcPtr;
#else
typedef const __attribute__((address_space(3))) int64_t* KcPtr;
#endif
typedef int64_t (*ProgFn)(int32_t n_cpu_left, int32_t n_cpu_total, int32_t n_mem_left, int32_t n_mem_total,
                          int32_t n_gpu_ng, int32_t gl0, int32_t gl1, int32_t gl2, int32_t gl3,
                          int32_t gl4, int32_t gl5, int32_t gl6, int32_t gl7, int32_t gt0, int32_t gt1, int32_t gt2,
                          int32_t gt3, int32_t gt4, int32_t gt5, int32_t gt6, int32_t gt7, const int64_t* gmem,
                          int32_t p_cpu, int32_t p_mem, int32_t p_gpu, int64_t p_ctime, int32_t p_dur,
                          KcPtr kc);

// A launch's per-policy function table entry: the scorer's device address with
// bit 0 set when the program opens with the template's feasibility prologue
// (CompiledPolicy.feasibility_prologue): it then scores 0, with no other
// effect, exactly where the kernels' feasible() is false, so the kernels call
// it only for feasible nodes (function addresses are at least 4-byte aligned).
constexpr uint64_t kFnFeasBit = 1;
__host__ __device__ __forceinline__ ProgFn prog_of(uint64_t e) { return reinterpret_cast<ProgFn>(e & ~kFnFeasBit); }
__host__ __device__ __forceinline__ bool prog_feas(uint64_t e) { return (e & kFnFeasBit) != 0; }

// ---- runtime library -------------------------------------------------------------
// The float // and %, **, math.log / exp / sqrt / pow machinery (glibc's
// exp / log / pow, glibc_math.h; CPython float_pow) is compiled once, into the extension, and the
// generated code reaches it through `fks_rt_table` (filled by the loader with
// the addresses k_native_rt_table reports).  Keeps every JIT compile small.
typedef Ret2 (*RtBinFn)(int op, int64_t ab, int32_t afl, int64_t bb, int32_t bfl);
typedef Ret2 (*RtUnFn)(int op, int64_t ab, int32_t afl);
#if defined(FKS_JIT)
extern "C" __device__ uint64_t fks_rt_table[4];
#define FKS_JIT_RT_TABLE_DEFINITION extern "C" __device__ uint64_t fks_rt_table[4] = {0, 0, 0, 0};
__device__ __forceinline__ PyR rt_binop(int op, PyN a, PyN b) {
  return from_ret2(((RtBinFn)fks_rt_table[0])(op, a.b, a.fl, b.b, b.fl));
}
__device__ __forceinline__ PyR rt_unop(int op, PyN a) { return from_ret2(((RtUnFn)fks_rt_table[1])(op, a.b, a.fl)); }
#else
#define FKS_JIT_RT_TABLE_DEFINITION
__device__ __forceinline__ PyR rt_binop(int op, PyN a, PyN b) { return d_binop(op, a, b); }
__device__ __forceinline__ PyR rt_unop(int op, PyN a) { return d_unop(op, a); }
#endif

// ---- helpers the generated code calls ------------------------------------------
__device__ __forceinline__ int32_t sel8(int j, int32_t a0, int32_t a1, int32_t a2, int32_t a3, int32_t a4, int32_t a5,
                                        int32_t a6, int32_t a7) {
  int32_t v = a0;
  v = j == 1 ? a1 : v; v = j == 2 ? a2 : v; v = j == 3 ? a3 : v; v = j == 4 ? a4 : v;
  v = j == 5 ? a5 : v; v = j == 6 ? a6 : v; v = j == 7 ? a7 : v;
  return v;
}

// GPU lists are packed in one int64: bits 0-3 length, 4 bits per GPU index.
__device__ __forceinline__ int64_t glist_all(int32_t ngp) {
  return (int64_t)ngp | ((int64_t)(0x76543210u & (uint32_t)((1ull << (4 * ngp)) - 1)) << 4);
}
__device__ __forceinline__ int glist_get(const PyN& a, const PyN& i, PyN& r) {
  const int64_t lst = a.b;
  const int n = (int)(lst & 0xF);
  if (i.fl) return EXC_TYPE;
  const int64_t k = i.b < 0 ? i.b + n : i.b;
  if (k < 0 || k >= n) return EXC_INDEX;
  r = pi((lst >> (4 + 4 * k)) & 0xF);
  return EXC_NONE;
}

__device__ __forceinline__ int glist_slice(const PyN& a, const PyN& lo_v, int has_lo, const PyN& hi_v, int has_hi,
                                           PyN& r) {
  const int64_t lst = a.b;
  const int n = (int)(lst & 0xF);
  int64_t lo = 0, hi = n;
  if (has_lo) { if (lo_v.fl) return EXC_TYPE; lo = lo_v.b; }
  if (has_hi) { if (hi_v.fl) return EXC_TYPE; hi = hi_v.b; }
  if (lo < 0) { lo += n; if (lo < 0) lo = 0; } else if (lo > n) lo = n;
  if (hi < 0) { hi += n; if (hi < 0) hi = 0; } else if (hi > n) hi = n;
  int64_t outv = 0;
  int m = 0;
  for (int64_t k = lo; k < hi; ++k, ++m) outv |= ((lst >> (4 + 4 * k)) & 0xF) << (4 + 4 * m);
  r = pi(outv | m);
  return EXC_NONE;
}

__device__ __forceinline__ int glist_append(const PyN& a, const PyN& item, PyN& r) {
  int64_t lst = a.b;
  const int n = (int)(lst & 0xF);
  if (n >= 15) return EXC_UNSUPPORTED;
  lst = (lst & ~(int64_t)0xF) | (n + 1);
  lst |= (item.b & 0xF) << (4 + 4 * n);
  r = pi(lst);
  return EXC_NONE;
}

__device__ __forceinline__ int glist_insert(const PyN& a, const PyN& item, const PyN& pos_v, PyN& r) {
  const int64_t lst = a.b;
  const int n = (int)(lst & 0xF);
  if (n >= 15) return EXC_UNSUPPORTED;
  if (pos_v.fl) return EXC_TYPE;
  int64_t pos = pos_v.b;
  if (pos < 0) { pos += n; if (pos < 0) pos = 0; } else if (pos > n) pos = n;
  const int64_t it = item.b & 0xF;
  const int64_t body = lst >> 4;
  const int64_t lowmask = (pos == 0) ? 0 : (((int64_t)1 << (4 * pos)) - 1);
  const int64_t nb = (body & lowmask) | (it << (4 * pos)) | ((body & ~lowmask) << 4);
  r = pi((nb << 4) | (n + 1));
  return EXC_NONE;
}

// int * int with overflow -> EXC_UNSUPPORTED (bigint: the host decides).
// Operands in int32 range (the common case) multiply exactly in int64;
// only the rest goes through the 128-bit check, out of line (LLVM's inline
// expansion of a 64-bit __builtin_mul_overflow is large and very slow to
// compile -- it dominated JIT compile time).
__device__ inline __noinline__ bool mul_ovf_slow(int64_t a, int64_t b, int64_t* r) { return __builtin_mul_overflow(a, b, r); }
__device__ __forceinline__ bool mul_ovf(int64_t a, int64_t b, int64_t* r) {
  if ((((uint64_t)a + 0x80000000ull) | ((uint64_t)b + 0x80000000ull)) >> 32 == 0) { *r = a * b; return false; }
  return mul_ovf_slow(a, b, r);
}

// int // int and int % int (CPython floor semantics); the float cases go out
// of line through d_binop.
__device__ __forceinline__ int int_floordiv(int64_t a, int64_t b, PyN& r) {
  if (b == 0) return EXC_ZERO_DIVISION;
  if (a == INT64_MIN && b == -1) return EXC_UNSUPPORTED;
  int64_t q = a / b;
  const int64_t m = a % b;
  if (m != 0 && ((m < 0) != (b < 0))) q -= 1;
  r = pi(q);
  return EXC_NONE;
}
__device__ __forceinline__ int int_mod(int64_t a, int64_t b, PyN& r) {
  if (b == 0) return EXC_ZERO_DIVISION;
  if (b == -1) { r = pi(0); return EXC_NONE; }
  int64_t m = a % b;
  if (m != 0 && ((m < 0) != (b < 0))) m += b;
  r = pi(m);
  return EXC_NONE;
}

// int(max(0, v)) of the returned value (FunSearchScheduler.__call__,
// funsearch/funsearch_integration.py:96), or -exception.
__device__ __forceinline__ int64_t finish_score(const PyN& v) {
  if (!v.fl) return v.b > 0 ? v.b : 0;
  const double x = __longlong_as_double(v.b);
  if (!(x > 0.0)) return 0;
  if (isinf(x)) return -(int64_t)EXC_OVERFLOW;
  if (x >= kTwo63d) return -(int64_t)EXC_UNSUPPORTED;
  return (int64_t)x;
}

}  // namespace fksd
