// Device interpreter of the policy bytecode (ISA: csrc/include/fks/bytecode.hpp,
// executable spec: csrc/cpu/vm_cpu.hpp).
//
// SIMT over nodes: the 64 lanes of the policy's wave evaluate
// priority(pod, node) for 64 nodes at once under ONE wave-uniform program
// counter (instructions are fetched with scalar loads and dispatched by a
// scalar branch); structured control flow is realised with per-lane mask
// counters, exactly as the CPU VM does.  The virtual register file lives in
// LDS behind the policy's event heap, lane-major ([reg][64 lanes] of 8 B: a
// ds_read_b64 per operand, conflict-free), the int/float tags in one 64-bit
// VGPR mask per lane.  exp/log/pow are the correctly rounded double-double
// versions of dd_math.h; trigonometry defers to the host.
#pragma once

#include "dd_math.h"
#include "replay.hip.h"

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
constexpr int kNoRegDev = 255;

struct DevProgramTable {
  const uint64_t* code;   // all programs, 8-byte instructions
  const int32_t* meta;    // per policy: code offset (insns), length, constant offset
  const int64_t* kpay;    // constant payloads (double bits for floats)
  const uint8_t* ktag;    // 0 int, 1 float
};

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
__device__ __noinline__ int d_cmp_mixed(PyN a, PyN b) {
  const bool swap = !a.fl;
  const double x = __longlong_as_double(swap ? b.b : a.b);
  const int64_t y = swap ? a.b : b.b;
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
  return d_cmp_mixed(a, b);
}

__device__ __forceinline__ bool dbl_odd_int(double x) { return fmod(fabs(x), 2.0) == 1.0; }

__device__ __noinline__ int d_float_pow(double iv, double iw, PyN& r) {
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
  const int st = dd_pow(iv, iw, ix);
  if (st == 2) return EXC_UNSUPPORTED;
  if (st == 1) return EXC_OVERFLOW;
  r = pf(neg ? -ix : ix);
  return EXC_NONE;
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
      double num, den;
      for (int k = 0; k < 2; ++k) {
        const PyN& x = k == 0 ? a : b;
        double out;
        if (!x.fl) {
          if (x.b <= 0) return EXC_VALUE;
          if (dd_log_d((double)x.b, out) == 2) return EXC_UNSUPPORTED;
        } else {
          const double v = __longlong_as_double(x.b);
          if (isnan(v)) out = v;
          else if (isinf(v)) { if (v > 0) out = v; else return EXC_VALUE; }
          else if (v <= 0.0) return EXC_VALUE;
          else if (dd_log_d(v, out) == 2) return EXC_UNSUPPORTED;
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
        if (dd_log_d((double)a.b, out) == 2) return EXC_UNSUPPORTED;
      } else {
        const double v = __longlong_as_double(a.b);
        if (isnan(v)) out = v;
        else if (isinf(v)) { if (v > 0) out = v; else return EXC_VALUE; }
        else if (v <= 0.0) return EXC_VALUE;
        else if (dd_log_d(v, out) == 2) return EXC_UNSUPPORTED;
      }
      r = pf(out); return EXC_NONE;
    }
    case OP_EXP: {
      const double x = fv(a);
      if (isnan(x)) { r = pf(x); return EXC_NONE; }
      if (isinf(x)) { r = pf(x > 0 ? x : 0.0); return EXC_NONE; }
      double out;
      const int st = dd_exp_d(x, out);
      if (st == 1) return EXC_OVERFLOW;
      if (st == 2) return EXC_UNSUPPORTED;
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
__device__ __noinline__ PyR d_binop(int op, PyN a, PyN b) {
  PyN r = pi(0);
  const int e = d_binop_impl(op, a, b, r);
  return PyR{r.b, r.fl ? 1 : 0, e};
}
__device__ __noinline__ PyR d_unop(int op, PyN a) {
  PyN r = pi(0);
  const int e = d_unop_impl(op, a, r);
  return PyR{r.b, r.fl ? 1 : 0, e};
}

// ---- the interpreter ---------------------------------------------------------------
constexpr uint32_t kBrk = 1, kCont = 2, kDone = 4;

// Scalar (SMEM) load of a wave-uniform 64-bit word.  The program table is
// reached through a generic pointer, which the compiler would fetch with a
// vector flat_load per instruction; the scalar cache path is much shorter.
__device__ __forceinline__ uint64_t sload64(const uint64_t* p) {
  uint64_t v;
  asm volatile("s_load_dwordx2 %0, %1, 0x0\n\ts_waitcnt lgkmcnt(0)" : "=s"(v) : "s"(p) : "memory");
  return v;
}
// The 16 most-used virtual registers (the compiler numbers them by use count)
// live in VGPRs, the rest in LDS.  (A 32-register all-VGPR file measured
// slower: 32-bit halves double the relative-addressing work and the extra
// VGPRs cost spills; the interpreter is dispatch-bound, not register-bound.)
struct VmScorerDev {
  static constexpr int kVgprRegs = 16;
  const uint64_t* code;
  const int64_t* kpay;
  const uint8_t* ktag;
  const int64_t* gmem_total;
  int32_t n_nodes;
  int64_t budget_call;  // instruction budget of one priority evaluation (<= 0: unlimited)
  bool limited;
  uint64_t* vregs;     // LDS: [reg][64]

  __device__ void init(const DevProgramTable& T, int p, const DevWorkload& W, int64_t bud, uint64_t* vreg_base) {
    const int off = T.meta[3 * p], koff = T.meta[3 * p + 2];
    code = T.code + off;
    kpay = T.kpay + koff;
    ktag = T.ktag + koff;
    gmem_total = W.gmem_total;
    n_nodes = W.n_nodes;
    budget_call = bud;
    limited = bud > 0;
    vregs = vreg_base;
  }

  template <int NPASS>
  __device__ int64_t score(int ps, const NodeRegs<NPASS>& nr, const PodView& pod, int& exc) {
    const int lane = lane_id();
    const int node = ps * kWave + lane;
    int off = 0;
    uint32_t st = node < n_nodes ? 0u : kDone;
    uint64_t ftag = 0;
    int lexc = EXC_NONE;
    PyN result = pi(0);
    bool has_result = false;
    FKS_LDS uint64_t* R = lds_ptr(vregs) + lane;
    // registers [0, kVgprRegs) live in VGPRs (uniform index -> s_set_gpr_idx
    // relative addressing, no LDS round trip); the compiler numbers registers
    // by use count, so the hot ones land here.  The rest live in LDS.
    typedef long long VRegs __attribute__((ext_vector_type(kVgprRegs)));
    VRegs RV = (VRegs)0;   // vector value: dynamic element access stays in registers
    auto rd = [&](int r) -> int64_t { return r < kVgprRegs ? (int64_t)RV[r] : (int64_t)R[r * kWave]; };
    auto wr = [&](int r, int64_t v) {
      if (r < kVgprRegs) RV[r] = v;
      else R[r * kWave] = (uint64_t)v;
    };
    auto get = [&](int r) -> PyN { return PyN{rd(r), ((ftag >> r) & 1) != 0}; };
    auto put = [&](int r, const PyN& v) {
      wr(r, v.b);
      ftag = v.fl ? (ftag | (1ull << r)) : (ftag & ~(1ull << r));
    };
    auto put_raw = [&](int r, int64_t v) { wr(r, v); ftag &= ~(1ull << r); };

    // per-lane node view (pass ps), copied into registers once per call
    // (score() is out of line, so `nr` arrives through memory)
    int32_t gml[kGmax], gmt[kGmax];
#pragma unroll
    for (int j = 0; j < kGmax; ++j) { gml[j] = nr.gml[ps][j]; gmt[j] = nr.gmt[ps][j]; }
    const int ngp = nr.ngpus[ps];
    const int64_t n_cpu_left = nr.cpu_left[ps], n_cpu_total = nr.cpu_total[ps];
    const int64_t n_mem_left = nr.mem_left[ps], n_mem_total = nr.mem_total[ps], n_gpu_left = nr.gpu_left[ps];
    const int64_t p_cpu = pod.cpu, p_mem = pod.mem, p_ngpu = pod.ngpu, p_gmilli = pod.gmilli;
    const int64_t p_ctime = pod.ctime, p_dur = pod.dur;

    int pc = 0;
    int64_t budget = budget_call;   // runaway programs end here, so every wave drains
    const uint64_t* cp = reinterpret_cast<const uint64_t*>(uniu64(reinterpret_cast<uint64_t>(code)));
    for (;;) {
      if (limited && --budget < 0) { exc = EXC_BUDGET; return 0; }
      // pc is wave-uniform by construction; say so, so the fetch is a scalar load
      pc = uni(pc);
      const uint64_t in = sload64(cp + pc);
      const int op = uni((int)(in & 0xFF));
      const int d = uni((int)((in >> 8) & 0xFF));
      const int a = uni((int)((in >> 16) & 0xFF));
      const int b = uni((int)((in >> 24) & 0xFF));
      const int imm = uni((int)(in >> 32));
      const bool act = off == 0 && st == 0;
      // Every case computes at most one result; it is written back once, after
      // the switch (one write site keeps the VGPR register file from being
      // copied along every arm).  wmode: 0 none, 1 active lanes, 2 all lanes.
      PyN res = pi(0);
      int wmode = 0;
      int jump = -1;   // >= 0: uniform branch target
      bool fin = false;
      switch (op) {
        case OP_NOP: break;
        case OP_CONST:
          res = PyN{kpay[imm], ktag[imm] != 0};
          wmode = 1;
          break;
        case OP_MOV:
          res = get(a);
          wmode = 1;
          break;
        case OP_POD: {
          int64_t v;
          switch (imm) {
            case 0: v = p_cpu; break;
            case 1: v = p_mem; break;
            case 2: v = p_ngpu; break;
            case 3: v = p_gmilli; break;
            case 4: v = p_ctime; break;
            default: v = p_dur; break;
          }
          res = pi(v);
          wmode = 1;
          break;
        }
        case OP_NODE: {
          int64_t v;
          switch (imm) {
            case 0: v = n_cpu_left; break;
            case 1: v = n_cpu_total; break;
            case 2: v = n_mem_left; break;
            case 3: v = n_mem_total; break;
            case 4: v = n_gpu_left; break;
            default: v = ngp; break;
          }
          res = pi(v);
          wmode = 1;
          break;
        }
        case OP_GPU:
          if (act) {
            const int j = (int)(get(a).b & 0xF);
            int64_t v = 0;
            if (imm == 0) {
#pragma unroll
              for (int jj = 0; jj < kGmax; ++jj) v = (jj == j) ? gml[jj] : v;
            } else if (imm == 1) {
#pragma unroll
              for (int jj = 0; jj < kGmax; ++jj) v = (jj == j) ? gmt[jj] : v;
            } else {
              v = gmem_total[node * kGmax + j];
            }
            res = pi(v);
          }
          wmode = 1;
          break;
        case OP_GLIST_ALL:
          res = pi((int64_t)ngp | ((int64_t)(0x76543210u & (uint32_t)((1ull << (4 * ngp)) - 1)) << 4));
          wmode = 1;
          break;
        case OP_GLIST_LEN:
          res = pi(get(a).b & 0xF);
          wmode = 1;
          break;
        case OP_GLIST_GET:
          if (act) {
            const PyN i = get(b);
            const int64_t lst = get(a).b;
            const int n = (int)(lst & 0xF);
            const int64_t k = i.b < 0 ? i.b + n : i.b;
            if (i.fl) { lexc = EXC_TYPE; st |= kDone; }
            else if (k < 0 || k >= n) { lexc = EXC_INDEX; st |= kDone; }
            else res = pi((lst >> (4 + 4 * k)) & 0xF);
          }
          wmode = 1;
          break;
        case OP_GLIST_SLICE:
          if (act) {
            const int64_t lst = get(a).b;
            const int n = (int)(lst & 0xF);
            int64_t lo = 0, hi = n;
            bool bad = false;
            if (b != kNoRegDev) { const PyN s_ = get(b); bad |= s_.fl; lo = s_.b; }
            if (imm != kNoRegDev) { const PyN s_ = get(imm); bad |= s_.fl; hi = s_.b; }
            if (bad) {
              lexc = EXC_TYPE; st |= kDone;
            } else {
              if (lo < 0) { lo += n; if (lo < 0) lo = 0; } else if (lo > n) lo = n;
              if (hi < 0) { hi += n; if (hi < 0) hi = 0; } else if (hi > n) hi = n;
              int64_t outv = 0;
              int m = 0;
              for (int64_t k = lo; k < hi; ++k, ++m) outv |= ((lst >> (4 + 4 * k)) & 0xF) << (4 + 4 * m);
              res = pi(outv | m);
            }
          }
          wmode = 1;
          break;
        case OP_GLIST_NEW:
          wmode = 1;
          break;
        case OP_GLIST_APPEND:
          if (act) {
            int64_t lst = get(a).b;
            const int n = (int)(lst & 0xF);
            if (n >= 15) {
              lexc = EXC_UNSUPPORTED; st |= kDone;
            } else {
              lst = (lst & ~(int64_t)0xF) | (n + 1);
              lst |= (get(b).b & 0xF) << (4 + 4 * n);
              res = pi(lst);
            }
          }
          wmode = 1;
          break;
        case OP_GLIST_INSERT:
          if (act) {
            const int64_t lst = get(a).b;
            const int n = (int)(lst & 0xF);
            const PyN ps_ = get(imm);
            if (n >= 15) { lexc = EXC_UNSUPPORTED; st |= kDone; }
            else if (ps_.fl) { lexc = EXC_TYPE; st |= kDone; }
            else {
              int64_t pos = ps_.b;
              if (pos < 0) { pos += n; if (pos < 0) pos = 0; } else if (pos > n) pos = n;
              const int64_t item = get(b).b & 0xF;
              const int64_t body = lst >> 4;
              const int64_t lowmask = (pos == 0) ? 0 : (((int64_t)1 << (4 * pos)) - 1);
              const int64_t nb = (body & lowmask) | (item << (4 * pos)) | ((body & ~lowmask) << 4);
              res = pi((nb << 4) | (n + 1));
            }
          }
          wmode = 1;
          break;
        case OP_ADD: case OP_SUB: case OP_MUL:
          if (act) {
            const PyN x = get(a), y = get(b);
            if (!x.fl && !y.fl) {
              int64_t v;
              const bool ovf = op == OP_ADD ? __builtin_add_overflow(x.b, y.b, &v)
                             : op == OP_SUB ? __builtin_sub_overflow(x.b, y.b, &v)
                                            : __builtin_mul_overflow(x.b, y.b, &v);
              if (ovf) { lexc = EXC_UNSUPPORTED; st |= kDone; }   // bigint: host decides
              else res = pi(v);
            } else {
              const double p = fv(x), q = fv(y);
              res = pf(op == OP_ADD ? p + q : op == OP_SUB ? p - q : p * q);
            }
          }
          wmode = 1;
          break;
        case OP_TDIV:
          if (act) {
            const PyN x = get(a), y = get(b);
            const bool big = !x.fl && !y.fl && (x.b > kTwo53i || x.b < -kTwo53i || y.b > kTwo53i || y.b < -kTwo53i);
            const double q = fv(y);
            if (q == 0.0) { lexc = EXC_ZERO_DIVISION; st |= kDone; }
            else if (big) { lexc = EXC_UNSUPPORTED; st |= kDone; }
            else res = pf(fv(x) / q);
          }
          wmode = 1;
          break;
        case OP_FDIV: case OP_MOD: case OP_POW: case OP_LOGB: case OP_MPOW:
          if (act) {
            const PyR o = d_binop(op, get(a), get(b));
            if (o.e) { lexc = o.e; st |= kDone; }
            else res = PyN{o.b, o.fl != 0};
          }
          wmode = 1;
          break;
        case OP_NOT:
          res = pi(truthy(get(a)) ? 0 : 1);
          wmode = 1;
          break;
        case OP_TRUTH:
          res = pi(truthy(get(a)) ? 1 : 0);
          wmode = 1;
          break;
        case OP_ISINT:
          res = pi(get(a).fl ? 0 : 1);
          wmode = 1;
          break;
        case OP_FLOAT:
          res = pf(fv(get(a)));
          wmode = 1;
          break;
        case OP_NEG: case OP_POS: case OP_ABS: case OP_INT: case OP_ROUND: case OP_SQRT: case OP_LOG: case OP_EXP:
        case OP_SIN: case OP_COS: case OP_TAN:
          if (act) {
            const PyR o = d_unop(op, get(a));
            if (o.e) { lexc = o.e; st |= kDone; }
            else res = PyN{o.b, o.fl != 0};
          }
          wmode = 1;
          break;
        case OP_LT: case OP_LE: case OP_GT: case OP_GE: case OP_EQ: case OP_NE: {
          const int c = d_cmp(get(a), get(b));
          bool v;
          switch (op) {
            case OP_LT: v = c == -1; break;
            case OP_LE: v = c == -1 || c == 0; break;
            case OP_GT: v = c == 1; break;
            case OP_GE: v = c == 1 || c == 0; break;
            case OP_EQ: v = c == 0; break;
            default: v = c != 0; break;
          }
          res = pi(v ? 1 : 0);
          wmode = 1;
          break;
        }
        case OP_MIN2: case OP_MAX2: {
          const PyN x = get(a), y = get(b);
          const int c = d_cmp(y, x);
          const bool take = op == OP_MAX2 ? c == 1 : c == -1;
          res = take ? y : x;
          wmode = 1;
          break;
        }
        case OP_IF:
          if (act) { if (!truthy(get(a))) off = 1; }
          else off += 1;
          if (!ballot(off == 0 && st == 0)) jump = imm;
          break;
        case OP_ELSE:
          if (off == 1) off = 0; else if (off == 0) off = 1;
          if (!ballot(off == 0 && st == 0)) jump = imm;
          break;
        case OP_ENDIF:
          if (off > 0) off -= 1;
          break;
        case OP_LOOP_BEGIN:
          res = pi((int64_t)(st & (kBrk | kCont)));
          wmode = 2;
          if (!act) off += 1;
          st &= ~(kBrk | kCont);
          break;
        case OP_LOOP_TEST:
          if (act && !truthy(get(a))) st |= kBrk;
          if (!ballot(off == 0 && st == 0)) jump = imm;
          break;
        case OP_LOOP_CONT:
          st &= ~kCont;
          break;
        case OP_LOOP_NEXT:
          jump = imm;
          break;
        case OP_LOOP_EXIT: {
          if (off > 0) off -= 1;
          const uint32_t s_ = (uint32_t)get(a).b & (kBrk | kCont);
          st = (st & kDone) | s_;
          break;
        }
        case OP_BREAK:
          if (act) st |= kBrk;
          break;
        case OP_CONTINUE:
          if (act) st |= kCont;
          break;
        case OP_RET:
          if (act) { result = get(a); has_result = true; st |= kDone; }
          fin = !ballot((st & kDone) == 0);
          break;
        case OP_RAISE:
          if (act) { lexc = imm; st |= kDone; }
          break;
        case OP_END:
          fin = true;
          break;
        default:
          lexc = EXC_UNSUPPORTED;
          fin = true;
          break;
      }
      // single write-back (lanes that raised above are no longer active)
      if (wmode == 2 || (wmode == 1 && act && st == 0)) put(d, res);
      if (fin) break;
      pc = jump >= 0 ? jump : pc + 1;
    }
    // finished
    if (node >= n_nodes) return 0;
    if (lexc != EXC_NONE) { exc = lexc; return 0; }
    if (!has_result) { exc = EXC_TYPE; return 0; }  // returned None
    // int(max(0, v))
    if (!result.fl) return result.b > 0 ? result.b : 0;
    const double x = __longlong_as_double(result.b);
    if (!(x > 0.0)) return 0;
    if (isinf(x)) { exc = EXC_OVERFLOW; return 0; }
    if (x >= kTwo63d) { exc = EXC_UNSUPPORTED; return 0; }
    return (int64_t)x;
  }
};

}  // namespace fksd
