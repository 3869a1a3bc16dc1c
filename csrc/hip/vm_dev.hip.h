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
// VGPR mask per lane.  exp/log/pow are glibc's own algorithms
// (glibc_math.h, CPython's bits); trigonometry defers to the host.
#pragma once

#include "pyops_dev.h"
#include "replay.hip.h"

namespace fksd {

constexpr int kNoRegDev = 255;

struct DevProgramTable {
  const uint64_t* code;   // all programs, 8-byte instructions
  const int32_t* meta;    // per policy: code offset (insns), length, constant offset
  const int64_t* kpay;    // constant payloads (double bits for floats)
  const uint8_t* ktag;    // 0 int, 1 float
};

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

  template <int NPASS, bool GP>
  __device__ int64_t score(int ps, const NodeRegs<NPASS, GP>& nr, const PodView& pod, int& exc) {
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
    for (int j = 0; j < kGmax; ++j) { gml[j] = nr.g(ps, j); gmt[j] = nr.gt(ps, j); }
    const int ngp = nr.ngp(ps);
    const int64_t n_cpu_left = nr.cpu_left[ps], n_cpu_total = nr.ctot(ps);
    const int64_t n_mem_left = nr.mem_left[ps], n_mem_total = nr.mtot(ps), n_gpu_left = nr.gpu_left[ps];
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
