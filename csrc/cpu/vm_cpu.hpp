// CPU interpreter of the policy bytecode (csrc/include/fks/bytecode.hpp).
//
// It executes the program for all nodes at once with exactly the lane/mask
// semantics of the device interpreter, so it doubles as the executable
// specification of the device VM: any divergence between the two is a bug in
// one of them, and tests diff them event by event (trace_hash).
#pragma once

#include <algorithm>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

#include "engine.hpp"
#include "fks/bytecode.hpp"
#include "fks/pyops.hpp"

namespace fks {

struct Program {
  std::vector<Insn> code;
  std::vector<int64_t> kpay;  // constant payloads (double bits for floats)
  std::vector<uint8_t> ktag;
  int nregs = 0;
};

inline Program make_program(const std::string& s, const std::vector<double>& fconst,
                            const std::vector<int64_t>& iconst, const std::vector<uint8_t>& ctag) {
  Program p;
  if (s.size() % sizeof(Insn)) throw std::invalid_argument("bytecode length must be a multiple of 8");
  p.code.resize(s.size() / sizeof(Insn));
  std::memcpy(p.code.data(), s.data(), s.size());
  const size_t nk = ctag.size();
  if (fconst.size() != nk || iconst.size() != nk) throw std::invalid_argument("constant pool size mismatch");
  p.kpay.resize(nk);
  p.ktag = ctag;
  for (size_t i = 0; i < nk; ++i) {
    if (ctag[i] == TAG_FLOAT) std::memcpy(&p.kpay[i], &fconst[i], 8);
    else p.kpay[i] = iconst[i];
  }
  int mx = 0;
  for (const Insn& in : p.code) {
    if (in.op == OP_NOP) continue;
    if (in.d != kNoReg) mx = std::max(mx, (int)in.d + 1);
  }
  p.nregs = std::max(mx, 1);
  if (p.nregs > kMaxRegs) throw std::invalid_argument("program uses too many registers");
  // validate jump targets and register indices once, so the hot loop can trust them
  const int32_t n = (int32_t)p.code.size();
  for (const Insn& in : p.code) {
    switch (in.op) {
      case OP_IF: case OP_ELSE: case OP_LOOP_TEST: case OP_LOOP_NEXT:
        if (in.imm < 0 || in.imm >= n) throw std::invalid_argument("jump target out of range");
        break;
      case OP_CONST:
        if (in.imm < 0 || (size_t)in.imm >= nk) throw std::invalid_argument("constant index out of range");
        break;
      default: break;
    }
  }
  if (p.code.empty() || p.code.back().op != OP_END) throw std::invalid_argument("program must end with END");
  return p;
}

// Packed GPU list helpers
inline int glist_len(int64_t v) { return (int)(v & 0xF); }
inline int glist_at(int64_t v, int k) { return (int)((v >> (4 + 4 * k)) & 0xF); }
inline int64_t glist_make(const int* idx, int n) {
  int64_t v = n;
  for (int k = 0; k < n; ++k) v |= (int64_t)(idx[k] & 0xF) << (4 + 4 * k);
  return v;
}

// Lane-parallel interpreter.  Evaluates the program for nodes [0, L).
struct VmCore {
  const Program& P;
  int64_t budget;      // remaining instruction budget (<= 0 -> unlimited)
  bool limited;
  int32_t exc = EXC_NONE;

  // lane state (SoA)
  int L = 0;
  std::vector<int64_t> pay;   // [R][L]
  std::vector<uint8_t> isf;   // [R][L]
  std::vector<int32_t> off;
  std::vector<uint8_t> brk, cont, done;
  std::vector<PyNum> result;
  std::vector<uint8_t> has_result;

  VmCore(const Program& p, int64_t b) : P(p), budget(b), limited(b > 0) {}
  int64_t executed = 0;   // instructions dispatched (one per wave-uniform step)

  void resize(int lanes) {
    L = lanes;
    pay.assign((size_t)P.nregs * L, 0);
    isf.assign((size_t)P.nregs * L, 0);
    off.assign(L, 0); brk.assign(L, 0); cont.assign(L, 0); done.assign(L, 0);
    result.assign(L, pyi(0)); has_result.assign(L, 0);
  }

  inline bool active(int l) const { return off[l] == 0 && !brk[l] && !cont[l] && !done[l]; }
  inline PyNum get(int r, int l) const {
    size_t k = (size_t)r * L + l;
    PyNum v; v.fl = isf[k];
    if (v.fl) { std::memcpy(&v.f, &pay[k], 8); v.i = 0; } else { v.i = pay[k]; v.f = 0; }
    return v;
  }
  inline void put(int r, int l, const PyNum& v) {
    size_t k = (size_t)r * L + l;
    isf[k] = v.fl;
    if (v.fl) std::memcpy(&pay[k], &v.f, 8); else pay[k] = v.i;
  }
  inline int64_t raw(int r, int l) const { return pay[(size_t)r * L + l]; }
  inline void put_raw(int r, int l, int64_t v) { size_t k = (size_t)r * L + l; pay[k] = v; isf[k] = 0; }

  // Accessors into the simulated world, supplied by the caller.
  struct World {
    // pod (uniform)
    int64_t pod[6];
    // node fields per lane
    const int64_t* cpu_left; const int64_t* cpu_total; const int64_t* mem_left; const int64_t* mem_total;
    const int32_t* gpu_left; const int32_t* ngpus; const int32_t* gpu_start;
    const int32_t* gmilli_left; const int32_t* gmilli_total; const int64_t* gmem_left; const int64_t* gmem_total;
  };

  bool any_active() const {
    for (int l = 0; l < L; ++l) if (active(l)) return true;
    return false;
  }

  // Runs the program; returns false if an exception was raised (exc set).
  bool run(const World& W) {
    const Insn* code = P.code.data();
    int pc = 0;
    for (;;) {
      if (limited && --budget < 0) { exc = EXC_BUDGET; return false; }
      ++executed;
      const Insn in = code[pc];
      switch (in.op) {
        case OP_NOP: break;
        case OP_CONST: {
          PyNum k; k.fl = P.ktag[in.imm] == TAG_FLOAT;
          if (k.fl) { std::memcpy(&k.f, &P.kpay[in.imm], 8); k.i = 0; } else { k.i = P.kpay[in.imm]; k.f = 0; }
          for (int l = 0; l < L; ++l) if (active(l)) put(in.d, l, k);
          break;
        }
        case OP_MOV:
          for (int l = 0; l < L; ++l) if (active(l)) { size_t s = (size_t)in.a * L + l, d = (size_t)in.d * L + l; pay[d] = pay[s]; isf[d] = isf[s]; }
          break;
        case OP_POD:
          for (int l = 0; l < L; ++l) if (active(l)) put(in.d, l, pyi(W.pod[in.imm]));
          break;
        case OP_NODE:
          for (int l = 0; l < L; ++l) if (active(l)) {
            int64_t v = 0;
            switch (in.imm) {
              case NF_CPU_LEFT: v = W.cpu_left[l]; break;
              case NF_CPU_TOTAL: v = W.cpu_total[l]; break;
              case NF_MEM_LEFT: v = W.mem_left[l]; break;
              case NF_MEM_TOTAL: v = W.mem_total[l]; break;
              case NF_GPU_LEFT: v = W.gpu_left[l]; break;
              default: v = W.ngpus[l]; break;
            }
            put(in.d, l, pyi(v));
          }
          break;
        case OP_GPU:
          for (int l = 0; l < L; ++l) if (active(l)) {
            int g = W.gpu_start[l] + (int)raw(in.a, l);
            int64_t v = in.imm == GF_MILLI_LEFT ? W.gmilli_left[g]
                      : in.imm == GF_MILLI_TOTAL ? W.gmilli_total[g]
                      : in.imm == GF_MEM_LEFT ? W.gmem_left[g] : W.gmem_total[g];
            put(in.d, l, pyi(v));
          }
          break;
        case OP_GLIST_ALL:
          for (int l = 0; l < L; ++l) if (active(l)) {
            int n = W.ngpus[l];
            if (n > kMaxListLen) { exc = EXC_UNSUPPORTED; return false; }
            int idx[kMaxListLen];
            for (int k = 0; k < n; ++k) idx[k] = k;
            put_raw(in.d, l, glist_make(idx, n));
          }
          break;
        case OP_GLIST_LEN:
          for (int l = 0; l < L; ++l) if (active(l)) put(in.d, l, pyi(glist_len(raw(in.a, l))));
          break;
        case OP_GLIST_GET:
          for (int l = 0; l < L; ++l) if (active(l)) {
            PyNum i = get(in.b, l);
            if (i.fl) { exc = EXC_TYPE; return false; }
            int64_t lst = raw(in.a, l); int n = glist_len(lst);
            int64_t k = i.i < 0 ? i.i + n : i.i;
            if (k < 0 || k >= n) { exc = EXC_INDEX; return false; }
            put_raw(in.d, l, glist_at(lst, (int)k));
          }
          break;
        case OP_GLIST_SLICE:
          for (int l = 0; l < L; ++l) if (active(l)) {
            int64_t lst = raw(in.a, l); int n = glist_len(lst);
            int64_t lo = 0, hi = n;
            if (in.b != kNoReg) { PyNum s = get(in.b, l); if (s.fl) { exc = EXC_TYPE; return false; } lo = s.i; }
            if (in.imm != kNoReg) { PyNum s = get(in.imm, l); if (s.fl) { exc = EXC_TYPE; return false; } hi = s.i; }
            if (lo < 0) { lo += n; if (lo < 0) lo = 0; } else if (lo > n) lo = n;
            if (hi < 0) { hi += n; if (hi < 0) hi = 0; } else if (hi > n) hi = n;
            int idx[kMaxListLen]; int m = 0;
            for (int64_t k = lo; k < hi; ++k) idx[m++] = glist_at(lst, (int)k);
            put_raw(in.d, l, glist_make(idx, m));
          }
          break;
        case OP_GLIST_NEW:
          for (int l = 0; l < L; ++l) if (active(l)) put_raw(in.d, l, 0);
          break;
        case OP_GLIST_APPEND:
          for (int l = 0; l < L; ++l) if (active(l)) {
            int64_t lst = raw(in.a, l); int n = glist_len(lst);
            if (n >= kMaxListLen) { exc = EXC_UNSUPPORTED; return false; }
            lst = (lst & ~(int64_t)0xF) | (n + 1);
            lst |= (raw(in.b, l) & 0xF) << (4 + 4 * n);
            put_raw(in.d, l, lst);
          }
          break;
        case OP_GLIST_INSERT:
          for (int l = 0; l < L; ++l) if (active(l)) {
            int64_t lst = raw(in.a, l); int n = glist_len(lst);
            if (n >= kMaxListLen) { exc = EXC_UNSUPPORTED; return false; }
            PyNum ps = get(in.imm, l);
            if (ps.fl) { exc = EXC_TYPE; return false; }
            int64_t pos = ps.i;
            if (pos < 0) { pos += n; if (pos < 0) pos = 0; } else if (pos > n) pos = n;
            int idx[kMaxListLen + 1]; int m = 0;
            for (int k = 0; k < n; ++k) { if (k == pos) idx[m++] = (int)(raw(in.b, l) & 0xF); idx[m++] = glist_at(lst, k); }
            if (pos == n) idx[m++] = (int)(raw(in.b, l) & 0xF);
            put_raw(in.d, l, glist_make(idx, m));
          }
          break;

#define FKS_BINOP(OPC, FN)                                               \
  case OPC:                                                              \
    for (int l = 0; l < L; ++l) if (active(l)) {                         \
      PyNum r; int e = FN(get(in.a, l), get(in.b, l), r);                \
      if (e) { exc = e; return false; }                                  \
      put(in.d, l, r);                                                   \
    }                                                                    \
    break;
        FKS_BINOP(OP_ADD, py_add)
        FKS_BINOP(OP_SUB, py_sub)
        FKS_BINOP(OP_MUL, py_mul)
        FKS_BINOP(OP_TDIV, py_tdiv)
        FKS_BINOP(OP_FDIV, py_fdiv)
        FKS_BINOP(OP_MOD, py_mod)
        FKS_BINOP(OP_POW, py_pow)
        FKS_BINOP(OP_LOGB, py_logb)
        FKS_BINOP(OP_MPOW, py_mpow)
#undef FKS_BINOP
        case OP_NEG:
          for (int l = 0; l < L; ++l) if (active(l)) {
            PyNum a = get(in.a, l);
            if (a.fl) put(in.d, l, pyf(-a.f));
            else { if (a.i == std::numeric_limits<int64_t>::min()) { exc = EXC_UNSUPPORTED; return false; } put(in.d, l, pyi(-a.i)); }
          }
          break;
        case OP_POS:
          for (int l = 0; l < L; ++l) if (active(l)) put(in.d, l, get(in.a, l));
          break;
        case OP_NOT:
          for (int l = 0; l < L; ++l) if (active(l)) put(in.d, l, pyi(truthy(get(in.a, l)) ? 0 : 1));
          break;
        case OP_TRUTH:
          for (int l = 0; l < L; ++l) if (active(l)) put(in.d, l, pyi(truthy(get(in.a, l)) ? 1 : 0));
          break;
        case OP_LT: case OP_LE: case OP_GT: case OP_GE: case OP_EQ: case OP_NE:
          for (int l = 0; l < L; ++l) if (active(l)) {
            int c = py_cmp(get(in.a, l), get(in.b, l));
            bool v;
            switch (in.op) {
              case OP_LT: v = c == -1; break;
              case OP_LE: v = c == -1 || c == 0; break;
              case OP_GT: v = c == 1; break;
              case OP_GE: v = c == 1 || c == 0; break;
              case OP_EQ: v = c == 0; break;
              default: v = c != 0; break;
            }
            put(in.d, l, pyi(v ? 1 : 0));
          }
          break;
        case OP_ABS:
          for (int l = 0; l < L; ++l) if (active(l)) {
            PyNum a = get(in.a, l);
            if (a.fl) put(in.d, l, pyf(std::fabs(a.f)));
            else { if (a.i == std::numeric_limits<int64_t>::min()) { exc = EXC_UNSUPPORTED; return false; } put(in.d, l, pyi(a.i < 0 ? -a.i : a.i)); }
          }
          break;
#define FKS_UNOP(OPC, FN)                                                \
  case OPC:                                                              \
    for (int l = 0; l < L; ++l) if (active(l)) {                         \
      PyNum r; int e = FN(get(in.a, l), r);                              \
      if (e) { exc = e; return false; }                                  \
      put(in.d, l, r);                                                   \
    }                                                                    \
    break;
        FKS_UNOP(OP_INT, py_int)
        FKS_UNOP(OP_ROUND, py_round)
        FKS_UNOP(OP_SQRT, py_sqrt)
        FKS_UNOP(OP_LOG, py_log)
        FKS_UNOP(OP_EXP, py_exp)
#undef FKS_UNOP
        case OP_SIN: case OP_COS: case OP_TAN:
          for (int l = 0; l < L; ++l) if (active(l)) {
            PyNum r; int e = py_trig(in.op - OP_SIN, get(in.a, l), r);
            if (e) { exc = e; return false; }
            put(in.d, l, r);
          }
          break;
        case OP_ISINT:
          for (int l = 0; l < L; ++l) if (active(l)) put(in.d, l, pyi(get(in.a, l).fl ? 0 : 1));
          break;
        case OP_FLOAT:
          for (int l = 0; l < L; ++l) if (active(l)) put(in.d, l, pyf(as_f(get(in.a, l))));
          break;
        case OP_MIN2: case OP_MAX2:
          for (int l = 0; l < L; ++l) if (active(l)) {
            PyNum a = get(in.a, l), b = get(in.b, l);
            int c = py_cmp(b, a);
            bool take_b = in.op == OP_MAX2 ? c == 1 : c == -1;
            put(in.d, l, take_b ? b : a);
          }
          break;

        // ---- structured control flow
        case OP_IF: {
          bool any = false;
          for (int l = 0; l < L; ++l) {
            if (active(l)) { if (!truthy(get(in.a, l))) off[l] = 1; else any = true; }
            else off[l] += 1;
          }
          if (!any) { pc = in.imm; continue; }
          break;
        }
        case OP_ELSE: {
          for (int l = 0; l < L; ++l) { if (off[l] == 1) off[l] = 0; else if (off[l] == 0) off[l] = 1; }
          if (!any_active()) { pc = in.imm; continue; }
          break;
        }
        case OP_ENDIF:
          for (int l = 0; l < L; ++l) if (off[l] > 0) off[l] -= 1;
          break;
        case OP_LOOP_BEGIN:
          for (int l = 0; l < L; ++l) {
            bool was = active(l);
            put_raw(in.d, l, (int64_t)brk[l] | ((int64_t)cont[l] << 1));
            if (!was) off[l] += 1;
            brk[l] = 0; cont[l] = 0;
          }
          break;
        case OP_LOOP_TEST: {
          bool any = false;
          for (int l = 0; l < L; ++l) if (active(l)) { if (!truthy(get(in.a, l))) brk[l] = 1; else any = true; }
          if (!any) { pc = in.imm; continue; }
          break;
        }
        case OP_LOOP_CONT:
          for (int l = 0; l < L; ++l) cont[l] = 0;
          break;
        case OP_LOOP_NEXT:
          pc = in.imm;
          continue;
        case OP_LOOP_EXIT:
          for (int l = 0; l < L; ++l) {
            if (off[l] > 0) off[l] -= 1;
            int64_t s = raw(in.a, l);
            brk[l] = s & 1; cont[l] = (s >> 1) & 1;
          }
          break;
        case OP_BREAK:
          for (int l = 0; l < L; ++l) if (active(l)) brk[l] = 1;
          break;
        case OP_CONTINUE:
          for (int l = 0; l < L; ++l) if (active(l)) cont[l] = 1;
          break;
        case OP_RET:
          for (int l = 0; l < L; ++l) if (active(l)) { result[l] = get(in.a, l); has_result[l] = 1; done[l] = 1; }
          if (!any_active()) {
            // fast exit when every lane has returned and no structure can re-enable one
            bool all_done = true;
            for (int l = 0; l < L; ++l) all_done &= done[l] != 0;
            if (all_done) return true;
          }
          break;
        case OP_RAISE:
          for (int l = 0; l < L; ++l) if (active(l)) { exc = in.imm; return false; }
          break;
        case OP_END:
          for (int l = 0; l < L; ++l) if (!done[l]) { has_result[l] = 0; done[l] = 1; }
          return true;
        default:
          exc = EXC_UNSUPPORTED;
          return false;
      }
      ++pc;
    }
  }
};

// Scorer adaptor: evaluates all nodes at the first call for a pod (lane
// parallel), serves the cached results for the following nodes.
struct VmScorer {
  const Program& prog;
  int64_t budget_total;
  int64_t budget_left;
  int32_t exc = EXC_NONE;
  int cached_pod = -1;
  int64_t cached_time = -1;
  std::vector<PyNum> res;
  std::vector<uint8_t> has;
  VmScorer(const Program& p, int64_t budget) : prog(p), budget_total(budget), budget_left(budget) {}
  int64_t insns = 0;   // VM instructions executed over the replay

  ScoreOut operator()(const ScoreCtx& c, int n) {
    ScoreOut o;
    if (n == 0 || c.pod != cached_pod || c.pod_ctime != cached_time) {
      const Workload& w = c.w;
      VmCore vm(prog, budget_total);   // the budget bounds one priority evaluation
      vm.resize(w.n_nodes);
      VmCore::World W;
      W.pod[PF_CPU] = w.pcpu[c.pod]; W.pod[PF_MEM] = w.pmem[c.pod];
      W.pod[PF_NGPU] = w.pngpu[c.pod]; W.pod[PF_GMILLI] = w.pgmilli[c.pod];
      W.pod[PF_CTIME] = c.pod_ctime; W.pod[PF_DUR] = w.pdur[c.pod];
      W.cpu_left = c.s.cpu_left.data(); W.cpu_total = w.cpu_total.data();
      W.mem_left = c.s.mem_left.data(); W.mem_total = w.mem_total.data();
      W.gpu_left = c.s.gpu_left.data(); W.ngpus = w.ngpus.data(); W.gpu_start = w.gpu_start.data();
      W.gmilli_left = c.s.gmilli_left.data(); W.gmilli_total = w.gmilli_total.data();
      W.gmem_left = w.gmem_left0.data(); W.gmem_total = w.gmem_total.data();
      bool ok = vm.run(W);
      insns += vm.executed;
      if (!ok) { o.exc = vm.exc; exc = vm.exc; return o; }
      res = vm.result; has = vm.has_result;
      cached_pod = c.pod; cached_time = c.pod_ctime;
    }
    if (!has[n]) { o.exc = EXC_TYPE; return o; }  // returned None
    const PyNum& v = res[n];
    o.v = v.fl ? Num::F(v.f) : Num::I(v.i);
    return o;
  }
};

}  // namespace fks
