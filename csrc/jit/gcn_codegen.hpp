// Baseline program JIT: policy bytecode -> gfx950 machine instructions.
//
// The LLVM path (policy/native_codegen.py -> ops/jit.py) produces tight code
// but costs ~140 ms of clang + llc per program, which is more than a whole
// replay of a new LLM program is worth.  This generator lowers the same
// bytecode (ISA: csrc/include/fks/bytecode.hpp) directly, in tens of
// microseconds, to a function with the same ABI (jit_abi.h ProgFn): it is
// called from the precompiled replay kernels with the node in v0-v22, the pod
// in v23-v28 and the LDS constant block in v29, and returns
// int(max(0, priority)) or -exception in v[0:1].
//
// Design (SIMT over nodes, like the VMs):
//  * static types from the same forward analysis as native_codegen.py: most
//    operations are emitted for int64 or f64 operands; genuinely mixed
//    operands call the precompiled runtime (rt_binop / rt_unop, d_binop_impl
//    semantics) or use tag bits kept per lane in one VGPR;
//  * registers: virtual registers get even-aligned VGPR pairs by liveness
//    (interference colouring); only caller-saved registers are used, so the
//    function needs no prologue saves; pod fields are wave-uniform and live
//    in SGPR pairs;
//  * control flow: structured, with EXEC masks -- IF saves EXEC, ELSE switches
//    to the saved complement, ENDIF restores EXEC minus the lanes that left
//    (returned / raised / broke / continued); loops keep their entry mask, a
//    break mask and a continue mask, and every back edge charges the per-call
//    iteration budget (EXC_BUDGET), so every loop ends;
//  * exceptions are "soft" per lane, exactly as the C++ codegen: the first
//    exception is kept, the lane keeps running until the next RET / back edge;
//  * register pressure beyond the caller-saved pairs: the virtual registers
//    with the highest interference per use live in per-lane scratch slots at
//    [s32, s32 + 8k); every instruction that touches one reloads it into a
//    reserved pair first and stores it back after (a runtime call's save area
//    starts above the slots);
//  * anything the baseline tier does not lower (an unknown opcode, more than
//    kMaxSpills spilled registers) throws CodegenError and the program goes to
//    the LLVM tier or the VMs.
#pragma once

#include <array>
#include <cmath>
#include <cstdlib>
#include <functional>
#include <map>
#include <set>
#include <stdexcept>
#include <vector>

#include "fks/bytecode.hpp"
#include "fks/types.hpp"
#include "gcn_lower.hpp"

namespace fks {
namespace gcn {

class CodegenError : public std::runtime_error {
 public:
  using std::runtime_error::runtime_error;
};

enum : uint8_t { TY_I = 1, TY_F = 2, TY_IF = 3 };

struct ProgIn {
  const Insn* code = nullptr;
  int n = 0;
  const uint8_t* ctag = nullptr;
  const uint8_t* is_lit = nullptr;   // constant slot read from the kc block at run time
  const int64_t* iconst = nullptr;
  const double* fconst = nullptr;
  int n_const = 0;
  // [elide_lo, elide_hi): the template's feasibility prologue, compiled out
  // when every caller calls only for nodes its own feasible() accepts (the
  // prologue then falls through with no effect); 0, 0: none
  int elide_lo = 0, elide_hi = 0;
  bool no_unroll = false;   // keep node.gpus loops rolled (the fallback when unrolled code does not fit)
};

struct GenStats {
  int vregs = 0, vgprs_used = 0, sgprs_used = 0, calls = 0, tagged = 0, spills = 0, unrolled = 0;
};

// Test hook: at most this many VGPR pairs for virtual registers (0: no cap),
// so CPU tests can force the spill path on ordinary programs.
inline int& pair_cap() {
  static int cap = 0;
  return cap;
}
constexpr int kMaxSpills = 16;   // 128 B of scratch per lane

// Unrolling of the compiler's node.gpus loop skeletons (Codegen::unroll_gpu_loops):
// a loop whose expanded body would exceed this many bytecode instructions stays
// rolled; 0 disables unrolling (A/B: FKS_JIT_UNROLL=0, or this hook in tests).
inline int& unroll_cap() {
  static int cap = [] {
    const char* e = std::getenv("FKS_JIT_UNROLL");
    return e ? std::atoi(e) : 1600;
  }();
  return cap;
}
constexpr int kUnrollTotalCap = 6000;   // bytecode instructions of the whole unrolled program

class Codegen {
 public:
  explicit Codegen(const ProgIn& p) : P_(p), n_(p.n) {
    if (p.elide_lo >= 0 && p.elide_lo < p.elide_hi && p.elide_hi <= p.n) {
      own_code_.assign(p.code, p.code + p.n);
      for (int pc = p.elide_lo; pc < p.elide_hi; ++pc) {
        if (defines(own_code_[(size_t)pc].op) && own_code_[(size_t)pc].d != kNoReg)
          elided_defs_ |= 1ull << own_code_[(size_t)pc].d;
        own_code_[(size_t)pc] = Insn{};   // OP_NOP
        own_code_[(size_t)pc].op = OP_NOP;
        own_code_[(size_t)pc].d = own_code_[(size_t)pc].a = own_code_[(size_t)pc].b = kNoReg;
      }
      P_.code = own_code_.data();
    }
  }

  Func run(GenStats* st = nullptr) {
    if (n_ <= 0) throw CodegenError("empty program");
    if (P_.n_const + 1 > 256) throw CodegenError("constant block larger than the LDS staging area");
    elide_hi_ = P_.elide_hi;
    if (unroll_cap() > 0 && !P_.no_unroll) unroll_gpu_loops();
    analyse_flow();
    for (int round = 0; round < 6; ++round) {
      list_facts();
      value_facts();
      const_facts();
      bool_facts();
      if (!prune_static_ifs()) break;
    }
    infer_types();
    fold_masks();
    liveness();
    // a value the elided prologue would have computed (e.g. its GPU count)
    // must not be read afterwards: the caller then compiles the whole program
    if (elided_defs_ && elide_hi_ < n_ && (live_in_[(size_t)elide_hi_] & elided_defs_))
      throw CodegenError("elided prologue defines a value the body reads");
    simt_liveness();
    layout_registers();
    arg_liveness();
    emit_all();
    if (st) {
      st->vregs = n_vregs_;
      st->calls = (int)F_.calls.size();
      st->tagged = n_tagged_;
      st->vgprs_used = max_vgpr_ + 1;
      st->sgprs_used = max_sgpr_ + 1;
      st->spills = __builtin_popcountll(spilled_);
      st->unrolled = n_unrolled_;
    }
    return F_;
  }

 private:
  ProgIn P_;
  std::vector<Insn> own_code_;   // the bytecode with the elided prologue as NOPs
  uint64_t elided_defs_ = 0;     // registers the elided prologue defined
  int elide_hi_ = 0;             // P_.elide_hi in the (unrolled) code
  int n_;
  // ---- unrolled node.gpus loops (unroll_gpu_loops): the rewritten code and the
  // constant pool extended by the GPU indices 0-7
  std::vector<Insn> unrolled_code_;
  std::vector<uint8_t> own_ctag_, own_lit_;
  std::vector<int64_t> own_iconst_;
  std::vector<double> own_fconst_;
  int n_unrolled_ = 0;
  Func F_;
  // ---- flow
  std::vector<int> brk_t_, cont_t_;
  std::vector<std::array<int, 2>> succ_;
  // ---- GPU-list facts per pc entry: registers holding node.gpus unchanged on
  // every path (all_in_), and elements of such lists read by a kLoopIndex GET
  // in the current iteration (uni_in_: the loop counter, equal in every lane
  // still in the loop)
  std::vector<uint64_t> all_in_, uni_in_;
  // ---- value facts per pc entry (every path, per lane): ints with |x| < 2^31
  // (i32_in_) / |x| <= 2^53 (ex_in_), and small non-negative constants (kin_:
  // value 0-15, or -1) -- overflow / exactness checks and list indexing they make moot
  std::vector<uint64_t> i32_in_, ex_in_, acc_in_;
  // ints with |x| < 2^32 (i33_in_: a sum / difference of two int32), and values
  // that are > 0 or NaN -- never zero, so a division by them cannot raise
  // (pos_in_: positive compiled-in constants and max / min built from them)
  std::vector<uint64_t> i33_in_, pos_in_;
  using MagRow = std::array<uint8_t, kMaxRegs>;
  std::vector<MagRow> mag_in_;   // |x| < 2^m of int registers per pc entry (64: unknown; value_facts)
  int mag(int r) const { return cur_pc_ >= 0 && r != kNoReg && !mag_in_.empty() ? mag_in_[cur_pc_][r] : 64; }
  std::vector<std::array<int8_t, kMaxRegs>> kin_;
  // registers holding a constant compiled into the code (pool index, -1: unknown)
  // and, per pc, the operands folded into the instruction as inline constants
  std::vector<std::array<int16_t, kMaxRegs>> kpool_;
  std::vector<uint64_t> fold_;
  int cur_pc_ = -1;
  bool i32(int r) const { return cur_pc_ >= 0 && r != kNoReg && (i32_in_[cur_pc_] >> r & 1); }
  bool exact(int r) const { return cur_pc_ >= 0 && r != kNoReg && (ex_in_[cur_pc_] >> r & 1); }
  bool acc(int r) const { return cur_pc_ >= 0 && r != kNoReg && (acc_in_[cur_pc_] >> r & 1); }
  bool i33(int r) const { return cur_pc_ >= 0 && r != kNoReg && (i33_in_[cur_pc_] >> r & 1); }
  bool acc_term_i33_ = false;   // accumulators may take |term| < 2^32 (few enough ADD / SUB sites)
  // int64 ADD / SUB / MUL of a and b that cannot overflow: both int32, or an
  // accumulator plus / minus a bounded term
  bool no_int_overflow(uint8_t op, int a, int b) const {
    if (i32(a) && i32(b)) return true;
    if (op == OP_MUL) return false;   // (the unchecked product is v_mad_i64_i32: int32 operands only)
    const int ma = mag(a), mb = mag(b);
    if (ma < 64 && mb < 64 && std::max(ma, mb) + 1 <= 63) return true;
    auto term = [&](int r) { return acc_term_i33_ ? i33(r) : i32(r); };
    return (acc(a) && term(b)) || (term(a) && acc(b));
  }
  bool nonzero(int r) const { return cur_pc_ >= 0 && r != kNoReg && (pos_in_[cur_pc_] >> r & 1); }
  // Loop iterations per call are capped at kJitLoopCap (more -> EXC_BUDGET, the
  // next engine decides), so a static ADD / SUB runs at most 2 * cap + 1 times
  // a call; with at most kAccSites of them, a value built from int32 terms by
  // ADD / SUB with an int32 operand stays below 1024 * (2^21 + 1) * 2^31 < 2^63.
  static constexpr uint32_t kJitLoopCap = 1u << 20;
  static constexpr int kAccSites = 1024;
  int kval(int r) const { return cur_pc_ >= 0 && r != kNoReg ? kin_[cur_pc_][r] : -1; }
  // ---- types: per pc entry state
  std::vector<std::array<uint8_t, kMaxRegs>> ty_;
  std::vector<char> reached_;
  // ---- liveness (per lane: register allocation) and SIMT liveness (spills)
  std::vector<uint64_t> live_in_, live_out_;
  std::vector<uint64_t> slive_out_;
  // ---- registers
  int n_vregs_ = 0, n_tagged_ = 0;
  std::array<int, kMaxRegs> base_{};      // VGPR pair base per virtual register (-1 unused)
  std::array<int, kMaxRegs> tagbit_{};    // tag bit index (-1: untagged)
  uint64_t tagged_ = 0;
  bool use_node_ = false, use_gl_ = false, use_gmem_ = false, use_kc_ = false, has_loop_ = false;
  std::array<int, 6> pod_s_{};            // argument VGPR of each pod field the program reads (-1 unused)
  int v_exc_ = -1, v_out_ = -1, v_spill_ = -1;
  int v_tag_[2] = {-1, -1};
  int T_[3] = {-1, -1, -1};               // temp VGPR pairs
  int s_entry_ = -1, s_dead_ = -1, ST_[3] = {-1, -1, -1}, S_LIT_ = -1;
  int s_bud_ = -1;   // loop iterations left this call (wave-level: the SGPR pair's low half)
  std::vector<int> free_spairs_;
  std::vector<int> ctl_spairs_;           // SGPR pairs held by open control frames
  std::vector<int> held_spairs_;          // SGPR pairs an instruction keeps across its own runtime call
  int max_vgpr_ = 0, max_sgpr_ = 0;
  // ---- spills: registers in scratch slots, reloaded per instruction
  uint64_t spilled_ = 0;
  std::array<int, kMaxRegs> slot_{};      // byte offset of a spilled register's slot
  std::array<int, kMaxRegs> map_{};       // reload pair of a spilled register in the current instruction (-1)
  int rl_[4] = {-1, -1, -1, -1};          // reload pairs (operands a, b, imm and the destination)
  int m_tmp_ = -1;                        // pair for writes outside an instruction (bools, zero init)

  struct Frame {
    bool loop;
    int pc;
    int s_save = -1, s_else = -1;         // IF
    int s_entry = -1, s_brk = -1, s_cont = -1;   // LOOP
    bool static_branch = false;           // IF with a known condition: one branch, no mask
    int l_exit = -1, l_head = -1;
  };
  std::vector<Frame> frames_;
  std::map<int, int> label_at_pc_;        // pc -> label placed before its code
  int skip_to_ = 0;                       // emission resumes at this pc (a dead branch)

  // ============================================================ unrolling
  // The compiler's loop over node.gpus (policy/compiler.py _for_glist /
  // _gen_loop; bytecode LOOP_INDEX):
  //
  //   GLIST_LEN n, src; CONST idx (0); CONST one (1); LOOP_BEGIN s
  //   LT c, idx, n [LOOP_INDEX]; LOOP_TEST c; GLIST_GET g, src, idx [LOOP_INDEX]
  //   body; LOOP_CONT; ADD idx, idx, one [LOOP_INDEX]; LOOP_NEXT; LOOP_EXIT s
  //
  // with src = node.gpus unchanged runs at most 8 iterations (a node has at
  // most kGmax GPUs), so it becomes eight guarded copies of the body:
  //
  //   LOOP_BEGIN s
  //   { CONST idx (k); LT c, idx, n; IF c; CONST g (k); body; ENDIF; [LOOP_CONT] } k = 0..7
  //   LOOP_EXIT s
  //
  // Same lanes, same order, same values: a lane runs copy k iff k < len(its
  // node.gpus), g is GPU k there (node.gpus[k] == k), and BREAK / CONTINUE /
  // RET keep their loop-frame meaning (a CONTINUE leaves the copy; LOOP_CONT,
  // kept only when the body continues, takes the lane back for the next one).
  // What it buys: the counter, the per-iteration test / back edge / budget
  // charge go away, and every GPU field read gets a constant index -- one move
  // from the argument VGPR instead of a readfirstlane + GPR-index-mode move.
  // The loop budget is charged by the back edges of the loops that remain (an
  // unrolled loop has none: it is bounded by construction).
  struct LoopPat {
    int b = -1, e = -1;                  // LOOP_BEGIN / LOOP_EXIT pcs
    int idx = -1, n = -1, g = -1, src = -1;
    bool cont = false;                   // the body CONTINUEs this loop
    int body_size = 0;                   // expanded size of the body (inner unrolled loops counted)
    bool unroll = false;
  };
  int pool_int(int64_t v) {
    // a non-literal int constant of the (own) pool with value v
    for (int k = 0; k < (int)own_iconst_.size(); ++k)
      if (!own_lit_[(size_t)k] && own_ctag_[(size_t)k] != TAG_FLOAT && own_iconst_[(size_t)k] == v) return k;
    own_ctag_.push_back(TAG_INT);
    own_lit_.push_back(0);
    own_iconst_.push_back(v);
    own_fconst_.push_back(0.0);
    return (int)own_iconst_.size() - 1;
  }
  void unroll_gpu_loops() {
    analyse_flow();
    list_facts();
    liveness();
    std::map<int, LoopPat> pats;   // by LOOP_BEGIN pc: loops that match the skeleton
    {
      std::vector<int> stk;
      std::map<int, int> exit_of;
      for (int pc = 0; pc < n_; ++pc) {
        if (P_.code[pc].op == OP_LOOP_BEGIN) stk.push_back(pc);
        else if (P_.code[pc].op == OP_LOOP_EXIT) { exit_of[stk.back()] = pc; stk.pop_back(); }
      }
      for (const auto& kv : exit_of) {
        const int b = kv.first, e = kv.second;
        if (b < 3 || e - b < 7) continue;
        const Insn* c = P_.code;
        const Insn &len = c[b - 3], &k0 = c[b - 2], &k1 = c[b - 1], &lt = c[b + 1], &tst = c[b + 2], &get = c[b + 3];
        const Insn &lc = c[e - 3], &add = c[e - 2], &nxt = c[e - 1];
        auto int_const = [&](const Insn& in, int64_t v) {
          return in.op == OP_CONST && in.imm >= 0 && in.imm < P_.n_const && !P_.is_lit[in.imm] &&
                 P_.ctag[in.imm] != TAG_FLOAT && P_.iconst[in.imm] == v;
        };
        if (len.op != OP_GLIST_LEN || !int_const(k0, 0) || !int_const(k1, 1)) continue;
        if (lt.op != OP_LT || lt.imm != kLoopIndex || lt.a != k0.d || lt.b != len.d) continue;
        if (tst.op != OP_LOOP_TEST || tst.a != lt.d || tst.imm != e) continue;
        if (get.op != OP_GLIST_GET || get.imm != kLoopIndex || get.a != len.a || get.b != k0.d) continue;
        if (lc.op != OP_LOOP_CONT || add.op != OP_ADD || add.imm != kLoopIndex || add.d != k0.d || add.a != k0.d ||
            add.b != k1.d || nxt.op != OP_LOOP_NEXT || nxt.imm != b + 1)
          continue;
        if (!(all_in_[(size_t)b + 3] >> get.a & 1)) continue;   // node.gpus itself
        if (k0.d == k1.d || k0.d == len.d || get.d == k0.d || get.d == len.d || get.d == get.a) continue;
        LoopPat L;
        L.b = b; L.e = e; L.idx = k0.d; L.n = len.d; L.g = get.d; L.src = get.a;
        // the counter, its step, the length and the list are the skeleton's own:
        // nothing in the body writes them, and the counter / step are dead after the loop
        bool ok = true;
        int inner_conts = 0;
        for (int pc = b + 4; pc < e - 3 && ok; ++pc) {
          const Insn& in = c[pc];
          if (defines(in.op) && in.d != kNoReg && (in.d == L.idx || in.d == k1.d || in.d == L.n || in.d == L.src))
            ok = false;
          if (in.op == OP_CONTINUE && cont_t_[(size_t)pc] == e - 3) L.cont = true;
          if (in.op == OP_LOOP_CONT) ++inner_conts;
        }
        (void)inner_conts;
        if (!ok) continue;
        if (e + 1 < n_ && (live_in_[(size_t)e + 1] >> L.idx & 1 || live_in_[(size_t)e + 1] >> k1.d & 1)) continue;
        pats[b] = L;
      }
    }
    if (pats.empty()) return;
    // sizes, innermost first: a loop is unrolled when its eight copies stay under the cap
    std::function<int(int, int)> size_of = [&](int lo, int hi) {
      int sz = 0;
      for (int pc = lo; pc < hi; ++pc) {
        auto it = pats.find(pc);
        if (it == pats.end()) { ++sz; continue; }
        LoopPat& L = it->second;
        L.body_size = size_of(L.b + 4, L.e - 3);
        const int unrolled = 2 + 8 * (L.body_size + 5 + (L.cont ? 1 : 0));
        L.unroll = 8 * L.body_size <= unroll_cap();
        sz += L.unroll ? unrolled : (L.e - L.b + 1 - (L.e - 3 - (L.b + 4)) + L.body_size);
        pc = L.e;
      }
      return sz;
    };
    if (size_of(0, n_) > kUnrollTotalCap) return;
    bool any = false;
    for (const auto& kv : pats) any = any || kv.second.unroll;
    if (!any) return;
    own_ctag_.assign(P_.ctag, P_.ctag + P_.n_const);
    own_lit_.assign(P_.is_lit, P_.is_lit + P_.n_const);
    own_iconst_.assign(P_.iconst, P_.iconst + P_.n_const);
    own_fconst_.assign(P_.fconst, P_.fconst + P_.n_const);
    int kidx[8];
    for (int k = 0; k < 8; ++k) kidx[k] = pool_int(k);
    std::vector<Insn> out;
    out.reserve((size_t)n_ * 2);
    auto mk_insn = [](uint8_t op, int d, int a, int b, int32_t imm) {
      Insn in{};
      in.op = op; in.d = (uint8_t)d; in.a = (uint8_t)a; in.b = (uint8_t)b; in.imm = imm;
      return in;
    };
    auto has_target = [](uint8_t op) {
      return op == OP_IF || op == OP_ELSE || op == OP_LOOP_TEST || op == OP_LOOP_NEXT;
    };
    // copy old pcs [lo, hi) (structured: every jump target of the range lies in
    // it, or is hi itself for the top level's end); top: record elide_hi
    std::function<void(int, int, bool)> emit_range = [&](int lo, int hi, bool top) {
      std::map<int, int> at;              // old pc -> new pc
      std::vector<size_t> fix;
      for (int pc = lo; pc < hi; ++pc) {
        at[pc] = (int)out.size();
        if (top && pc == P_.elide_hi) elide_hi_ = (int)out.size();
        auto it = pats.find(pc);
        if (it != pats.end() && it->second.unroll) {
          const LoopPat& L = it->second;
          out.push_back(P_.code[L.b]);    // LOOP_BEGIN
          const Insn& lt = P_.code[L.b + 1];
          // a body that never CONTINUEs: copy k + 1 nested in copy k (a lane
          // that reaches it ran every copy before it -- the analyses see that
          // path, e.g. a max()'s "seen" flag is a constant from copy 1 on --
          // and the wave skips every remaining copy once no lane has more GPUs);
          // otherwise flat copies, each ended by LOOP_CONT at loop level
          std::vector<size_t> open_ifs;
          for (int k = 0; k < 8; ++k) {
            out.push_back(mk_insn(OP_CONST, L.idx, kNoReg, kNoReg, kidx[k]));
            out.push_back(mk_insn(OP_LT, lt.d, L.idx, L.n, 0));
            open_ifs.push_back(out.size());
            out.push_back(mk_insn(OP_IF, kNoReg, lt.d, kNoReg, 0));
            out.push_back(mk_insn(OP_CONST, L.g, kNoReg, kNoReg, kidx[k]));
            emit_range(L.b + 4, L.e - 3, false);
            if (L.cont) {
              out[open_ifs.back()].imm = (int32_t)out.size();
              open_ifs.pop_back();
              out.push_back(mk_insn(OP_ENDIF, kNoReg, kNoReg, kNoReg, 0));
              out.push_back(mk_insn(OP_LOOP_CONT, kNoReg, kNoReg, kNoReg, 0));
            }
          }
          while (!open_ifs.empty()) {
            out[open_ifs.back()].imm = (int32_t)out.size();
            open_ifs.pop_back();
            out.push_back(mk_insn(OP_ENDIF, kNoReg, kNoReg, kNoReg, 0));
          }
          at[L.e] = (int)out.size();
          out.push_back(P_.code[L.e]);    // LOOP_EXIT
          for (int q = L.b + 1; q < L.e; ++q) at.erase(q);   // (nothing outside jumps into the loop)
          pc = L.e;
          ++n_unrolled_;
          continue;
        }
        out.push_back(P_.code[pc]);
        if (has_target(P_.code[pc].op)) fix.push_back(out.size() - 1);
      }
      at[hi] = (int)out.size();
      if (top && hi == P_.elide_hi) elide_hi_ = (int)out.size();
      for (size_t i : fix) {
        auto t = at.find(out[i].imm);
        if (t == at.end()) throw CodegenError("internal: jump out of an unrolled range");
        out[i].imm = t->second;
      }
    };
    emit_range(0, n_, true);
    unrolled_code_ = std::move(out);
    P_.code = unrolled_code_.data();
    n_ = (int)unrolled_code_.size();
    P_.ctag = own_ctag_.data();
    P_.is_lit = own_lit_.data();
    P_.iconst = own_iconst_.data();
    P_.fconst = own_fconst_.data();
    P_.n_const = (int)own_iconst_.size();
    // (the analyses run again on the new code)
    all_in_.clear(); uni_in_.clear(); live_in_.clear(); live_out_.clear();
  }

  // ============================================================ analysis
  static bool defines(uint8_t op) {
    switch (op) {
      case OP_NOP: case OP_IF: case OP_ELSE: case OP_ENDIF: case OP_LOOP_BEGIN: case OP_LOOP_TEST:
      case OP_LOOP_CONT: case OP_LOOP_NEXT: case OP_LOOP_EXIT: case OP_BREAK: case OP_CONTINUE: case OP_RET:
      case OP_RAISE: case OP_END:
        return false;
      default:
        return true;
    }
  }
  // truth value of node.gpus (register r unchanged on every path) read at pc
  bool list_truth(int pc, int r) const {
    if (pc < 0 || r == kNoReg || all_in_.empty() || !(all_in_[(size_t)pc] >> r & 1)) return false;
    const uint8_t op = P_.code[pc].op;
    return (op == OP_IF || op == OP_LOOP_TEST || op == OP_NOT || op == OP_TRUTH) && P_.code[pc].a == r;
  }
  uint64_t uses(int pc) const {
    const Insn& in = P_.code[pc];
    uint64_t u = 0;
    if (in.op == OP_LOOP_BEGIN || in.op == OP_LOOP_EXIT || in.op == OP_CONST || in.op == OP_POD ||
        in.op == OP_NODE || in.op == OP_RAISE)
      return 0;
    // node.gpus itself is not read by its length or a loop-counter get (all_in_)
    const bool all_list_read = (in.op == OP_GLIST_LEN || (in.op == OP_GLIST_GET && in.imm == kLoopIndex)) &&
                               in.a != kNoReg && !all_in_.empty() && (all_in_[pc] >> in.a & 1);
    // a GPU index known to be a constant is not read either (emit_gpu: a direct move)
    const bool const_gpu = in.op == OP_GPU && (in.imm == 0 || in.imm == 1) && in.a != kNoReg && !kin_.empty() &&
                           kin_[(size_t)pc][in.a] >= 0 && kin_[(size_t)pc][in.a] < 8;
    if (in.a != kNoReg && !all_list_read && !const_gpu && !list_truth(pc, in.a)) u |= 1ull << in.a;
    if (in.b != kNoReg) u |= 1ull << in.b;
    if (!fold_.empty()) u &= ~fold_[pc];   // read as inline constants
    if ((in.op == OP_GLIST_SLICE || in.op == OP_GLIST_INSERT) && in.imm != kNoReg) u |= 1ull << in.imm;
    return u;
  }
  uint64_t defs(int pc) const {
    const Insn& in = P_.code[pc];
    return (defines(in.op) && in.d != kNoReg) ? (1ull << in.d) : 0ull;
  }

  void analyse_flow() {
    brk_t_.assign(n_, -1);
    cont_t_.assign(n_, -1);
    std::vector<int> stack;
    std::map<int, int> exit_of;
    std::map<int, std::vector<int>> conts;
    std::map<int, int> pend_b, pend_c;
    for (int pc = 0; pc < n_; ++pc) {
      const Insn& in = P_.code[pc];
      if (in.a != kNoReg && in.a >= kMaxRegs) throw CodegenError("register out of range");
      if (in.op == OP_LOOP_BEGIN) { stack.push_back(pc); conts[pc]; }
      else if (in.op == OP_LOOP_EXIT) {
        if (stack.empty()) throw CodegenError("LOOP_EXIT without LOOP_BEGIN");
        exit_of[stack.back()] = pc;
        stack.pop_back();
      } else if (in.op == OP_LOOP_CONT) {
        if (stack.empty()) throw CodegenError("LOOP_CONT outside a loop");
        conts[stack.back()].push_back(pc);
      } else if (in.op == OP_BREAK || in.op == OP_CONTINUE) {
        if (stack.empty()) throw CodegenError("BREAK / CONTINUE outside a loop");
        (in.op == OP_BREAK ? pend_b : pend_c)[pc] = stack.back();
      }
    }
    if (!stack.empty()) throw CodegenError("unterminated loop");
    for (auto& kv : pend_b) brk_t_[kv.first] = exit_of[kv.second];
    for (auto& kv : pend_c) {
      int t = -1;
      for (int c : conts[kv.second])
        if (c > kv.first) { t = c; break; }
      if (t < 0) throw CodegenError("CONTINUE without a following LOOP_CONT");
      cont_t_[kv.first] = t;
    }
    succ_.assign(n_, {-1, -1});
    for (int pc = 0; pc < n_; ++pc) {
      const Insn& in = P_.code[pc];
      std::array<int, 2> sc{-1, -1};
      switch (in.op) {
        case OP_IF: sc = {pc + 1, in.imm + 1}; break;
        case OP_ELSE: case OP_LOOP_NEXT: sc = {in.imm, -1}; break;
        case OP_LOOP_TEST: sc = {pc + 1, in.imm}; break;
        case OP_BREAK: sc = {brk_t_[pc], -1}; break;
        case OP_CONTINUE: sc = {cont_t_[pc], -1}; break;
        case OP_RET: case OP_RAISE: case OP_END: break;
        default: sc = {pc + 1, -1};
      }
      for (int t : sc)
        if (t != -1 && (t < 0 || t >= n_)) throw CodegenError("jump target out of range");
      succ_[pc] = sc;
    }
  }

  // Forward must-analyses over the CFG (meet = intersection).  A lane follows
  // one CFG path, so "on every path" holds per lane.  uni_in_ is cleared at
  // every LOOP_CONT / LOOP_EXIT: an element is uniform only inside the
  // iteration that read it (after the loop, lanes hold different last GPUs).
  template <class F>
  void must_solve(std::vector<uint64_t>& st, F transfer) {
    st.assign(n_, ~0ull);
    std::vector<char> seen(n_, 0);
    st[0] = 0;
    seen[0] = 1;
    std::vector<int> work{0};
    while (!work.empty()) {
      const int pc = work.back();
      work.pop_back();
      const uint64_t out = transfer(pc, st[pc]);
      for (int t : succ_[pc]) {
        if (t < 0) continue;
        const uint64_t nw = seen[t] ? (st[t] & out) : out;
        if (!seen[t] || nw != st[t]) {
          st[t] = nw;
          seen[t] = 1;
          work.push_back(t);
        }
      }
    }
  }
  void list_facts() {
    must_solve(all_in_, [&](int pc, uint64_t s) {
      const Insn& in = P_.code[pc];
      if (!defines(in.op) || in.d == kNoReg) return s;
      const uint64_t bit = 1ull << in.d;
      if (in.op == OP_GLIST_ALL || (in.op == OP_MOV && in.a != kNoReg && (s >> in.a & 1))) return s | bit;
      return s & ~bit;
    });
    // the loop (LOOP_BEGIN pc) each pc belongs to, and the registers the
    // counter-indexed GETs of each loop define: they stop being uniform at
    // that loop's LOOP_CONT / LOOP_EXIT (an inner loop keeps an outer element)
    std::vector<int> loop_of(n_, -1);
    std::map<int, uint64_t> gen_of;
    {
      std::vector<int> stk;
      for (int pc = 0; pc < n_; ++pc) {
        const Insn& in = P_.code[pc];
        if (in.op == OP_LOOP_BEGIN) stk.push_back(pc);
        loop_of[pc] = stk.empty() ? -1 : stk.back();
        if (in.op == OP_LOOP_EXIT && !stk.empty()) stk.pop_back();
        if (in.op == OP_GLIST_GET && in.imm == kLoopIndex && in.d != kNoReg && loop_of[pc] >= 0)
          gen_of[loop_of[pc]] |= 1ull << in.d;
      }
    }
    must_solve(uni_in_, [&](int pc, uint64_t s) {
      const Insn& in = P_.code[pc];
      if (in.op == OP_LOOP_CONT || in.op == OP_LOOP_EXIT) {
        const auto it = gen_of.find(loop_of[pc]);
        return it == gen_of.end() ? s : (s & ~it->second);
      }
      if (!defines(in.op) || in.d == kNoReg) return s;
      const uint64_t bit = 1ull << in.d;
      if (in.op == OP_GLIST_GET && in.imm == kLoopIndex && in.a != kNoReg && (all_in_[pc] >> in.a & 1))
        return s | bit;
      return s & ~bit;
    });
  }

  void value_facts() {
    // constants compiled into the code only: a data literal (is_lit) takes
    // other values in other programs of the same shape
    auto fixed_int = [&](int k) { return k >= 0 && k < P_.n_const && !P_.is_lit[k] && P_.ctag[k] != TAG_FLOAT; };
    auto small_k = [&](int k) { return fixed_int(k) && P_.iconst[k] > -(1ll << 31) && P_.iconst[k] < (1ll << 31); };
    auto is_bool_op = [](uint8_t op) {
      return op == OP_LT || op == OP_LE || op == OP_GT || op == OP_GE || op == OP_EQ || op == OP_NE ||
             op == OP_NOT || op == OP_TRUTH || op == OP_ISINT;
    };
    // does the definition at pc give an int with |x| < 2^31 (i: i32 facts on entry)?
    auto i32_def = [&](const Insn& in, uint64_t i) {
      switch (in.op) {
        case OP_CONST: return small_k(in.imm);
        case OP_MOV: case OP_POS: return (i >> in.a & 1) != 0;
        case OP_NODE: case OP_GLIST_LEN: case OP_GLIST_GET: return true;   // int32 argument fields / [0, 15]
        case OP_POD: return in.imm >= 0 && in.imm <= 3;                     // creation / duration: int64
        case OP_GPU: return in.imm == 0 || in.imm == 1;                     // GPU memory: int64
        case OP_MIN2: case OP_MAX2: return (i >> in.a & 1) && (i >> in.b & 1);
        default: return is_bool_op(in.op);
      }
    };
    // magnitudes: per pc entry and register, m with |x| < 2^m for an int value
    // (64: not known to be a bounded int -- a float, a mixed type, or grown
    // around a loop).  Forward, join = max; at a loop head a register that
    // grows is widened to 64 (an unrolled node.gpus loop has no back edge, so
    // a sum over the GPUs keeps its bound).  i32 / i33 / exact are its views.
    {
      std::vector<MagRow>& mag = mag_in_;
      mag.assign(n_, MagRow{});
      std::vector<char> seen(n_, 0), head(n_, 0);
      for (int pc = 0; pc < n_; ++pc)
        if (P_.code[pc].op == OP_LOOP_NEXT && P_.code[pc].imm >= 0 && P_.code[pc].imm < n_) head[P_.code[pc].imm] = 1;
      auto bits_of = [](int64_t v) {
        const uint64_t a = v < 0 ? (uint64_t)(-(v + 1)) + 1 : (uint64_t)v;
        int m = 0;
        while (m < 64 && (a >> m) != 0) ++m;
        return (uint8_t)(m < 1 ? 1 : m);   // |v| < 2^m (0 and 1: 1)
      };
      auto cap = [](int m) { return (uint8_t)(m > 64 ? 64 : m); };
      mag[0].fill(64);
      seen[0] = 1;
      std::vector<int> work{0};
      while (!work.empty()) {
        const int pc = work.back();
        work.pop_back();
        MagRow out = mag[pc];
        const Insn& in = P_.code[pc];
        if (defines(in.op) && in.d != kNoReg) {
          const uint8_t ma = in.a != kNoReg && in.a < kMaxRegs ? mag[pc][in.a] : 64;
          const uint8_t mb = in.b != kNoReg && in.b < kMaxRegs ? mag[pc][in.b] : 64;
          uint8_t m = 64;
          switch (in.op) {
            case OP_CONST: if (fixed_int(in.imm)) m = bits_of(P_.iconst[in.imm]); break;
            case OP_MOV: case OP_POS: case OP_NEG: case OP_ABS: m = ma; break;
            case OP_NODE: m = 31; break;                                 // int32 argument fields
            case OP_GLIST_LEN: case OP_GLIST_GET: m = 4; break;          // [0, 15]
            case OP_POD: m = in.imm >= 0 && in.imm <= 3 ? 31 : 64; break;   // creation / duration: int64
            case OP_GPU: m = in.imm == 0 || in.imm == 1 ? 31 : 64; break;   // GPU memory: int64
            case OP_ADD: case OP_SUB: m = (ma < 64 && mb < 64) ? cap(std::max(ma, mb) + 1) : 64; break;
            case OP_MUL: m = (ma < 64 && mb < 64) ? cap(ma + mb) : 64; break;
            case OP_MIN2: case OP_MAX2: m = std::max(ma, mb); break;
            case OP_FDIV: m = (ma < 64 && mb < 64) ? ma : 64; break;     // |a // b| <= |a| (b != 0 int)
            case OP_MOD: m = (ma < 64 && mb < 64) ? mb : 64; break;      // |a % b| < |b|
            default: m = is_bool_op(in.op) ? 1 : 64; break;
          }
          out[in.d] = m;
        }
        for (int t : succ_[pc]) {
          if (t < 0) continue;
          bool changed = !seen[t];
          for (int r = 0; r < kMaxRegs; ++r) {
            uint8_t nv = !seen[t] ? out[r] : std::max(mag[t][r], out[r]);
            if (seen[t] && head[t] && nv > mag[t][r]) nv = 64;   // widen around a loop
            if (nv != mag[t][r]) { mag[t][r] = nv; changed = true; }
          }
          seen[t] = 1;
          if (changed) work.push_back(t);
        }
      }
      i32_in_.assign(n_, ~0ull);
      ex_in_.assign(n_, ~0ull);
      i33_in_.assign(n_, ~0ull);
      for (int pc = 0; pc < n_; ++pc) {
        if (!seen[pc]) continue;   // unreached: every fact (as must_solve)
        uint64_t a = 0, b = 0, c = 0;
        for (int r = 0; r < kMaxRegs; ++r) {
          if (mag[pc][r] <= 31) a |= 1ull << r;
          if (mag[pc][r] <= 32) c |= 1ull << r;
          if (mag[pc][r] <= 53) b |= 1ull << r;
        }
        i32_in_[pc] = a;
        ex_in_[pc] = b;
        i33_in_[pc] = c;
      }
    }
    int add_sites = 0;
    for (int pc = 0; pc < n_; ++pc)
      if (P_.code[pc].op == OP_ADD || P_.code[pc].op == OP_SUB) ++add_sites;
    // an accumulator: built from int32 terms by ADD / SUB with an int32 operand
    // (<= kAccSites sites: below 2^62, see kJitLoopCap) -- or with |term| < 2^32
    // when there are at most half as many sites (the same bound)
    acc_term_i33_ = add_sites <= kAccSites / 2;
    must_solve(acc_in_, [&](int pc, uint64_t st) {
      const Insn& in = P_.code[pc];
      if (!defines(in.op) || in.d == kNoReg) return st;
      const uint64_t bit = 1ull << in.d;
      const uint64_t i = add_sites <= kAccSites / 2 ? i33_in_[pc] : i32_in_[pc];
      bool r = i32_def(in, i32_in_[pc]);
      if (add_sites <= kAccSites) {
        switch (in.op) {
          case OP_MOV: case OP_POS: case OP_NEG: case OP_ABS: r = r || (st >> in.a & 1); break;
          case OP_ADD: case OP_SUB:
            r = r || ((st >> in.a & 1) && (i >> in.b & 1)) || ((i >> in.a & 1) && (st >> in.b & 1));
            break;
          case OP_MIN2: case OP_MAX2: r = r || ((st >> in.a & 1) && (st >> in.b & 1)); break;
          default: break;
        }
      }
      return r ? (st | bit) : (st & ~bit);
    });
    must_solve(pos_in_, [&](int pc, uint64_t st) {
      const Insn& in = P_.code[pc];
      if (!defines(in.op) || in.d == kNoReg) return st;
      const uint64_t bit = 1ull << in.d;
      bool r = false;
      switch (in.op) {
        case OP_CONST: r = fixed_int(in.imm) && P_.iconst[in.imm] > 0; break;
        case OP_MOV: case OP_POS: r = (st >> in.a & 1) != 0; break;
        // max(a, b) is b only where b > a: a > 0 (or NaN) -> the result is too;
        // b > 0 and a an int (never NaN) or > 0 -> likewise; a NaN a stays NaN
        case OP_MAX2: r = (st >> in.a & 1) || (st >> in.b & 1); break;
        case OP_MIN2: r = (st >> in.a & 1) && (st >> in.b & 1); break;   // one of the two
        default: break;
      }
      return r ? (st | bit) : (st & ~bit);
    });
    // small constants: per register 0-15, -1 unknown, -2 not reached yet
    kin_.assign(n_, {});
    for (auto& a : kin_) a.fill(-2);
    kin_[0].fill(-1);
    std::vector<char> seen(n_, 0);
    seen[0] = 1;
    std::vector<int> work{0};
    while (!work.empty()) {
      const int pc = work.back();
      work.pop_back();
      std::array<int8_t, kMaxRegs> out = kin_[pc];
      const Insn& in = P_.code[pc];
      if (defines(in.op) && in.d != kNoReg) {
        int8_t v = -1;
        if (in.op == OP_CONST && fixed_int(in.imm) && P_.iconst[in.imm] >= 0 && P_.iconst[in.imm] <= 15)
          v = (int8_t)P_.iconst[in.imm];
        else if ((in.op == OP_MOV || in.op == OP_POS) && in.a != kNoReg)
          v = kin_[pc][in.a];
        else if (in.op == OP_GLIST_GET && in.a != kNoReg && in.b != kNoReg && (all_in_[pc] >> in.a & 1) &&
                 kin_[pc][in.b] >= 0)
          v = kin_[pc][in.b];   // node.gpus[k] is GPU k (lanes with k >= len raised)
        out[in.d] = v < 0 ? -1 : v;
      }
      for (int t : succ_[pc]) {
        if (t < 0) continue;
        bool changed = !seen[t];
        for (int r = 0; r < kMaxRegs; ++r) {
          const int8_t nv = !seen[t] ? out[r] : (kin_[t][r] == out[r] ? out[r] : (int8_t)-1);
          if (nv != kin_[t][r]) { kin_[t][r] = nv; changed = true; }
        }
        seen[t] = 1;
        if (changed) work.push_back(t);
      }
    }
  }

  // ---- truth values known at compile time (kbool_: per pc entry and register,
  // -1 unknown, 0 / 1): compiled-in constants, and NOT / TRUTH / copies of them
  std::vector<std::array<int8_t, kMaxRegs>> kbool_;
  std::vector<int8_t> static_if_;   // per IF pc: -1 dynamic, 0 never taken, 1 always taken
  void bool_facts() {
    kbool_.assign(n_, {});
    for (auto& a : kbool_) a.fill(-2);
    kbool_[0].fill(-1);
    std::vector<char> seen(n_, 0);
    seen[0] = 1;
    std::vector<int> work{0};
    while (!work.empty()) {
      const int pc = work.back();
      work.pop_back();
      std::array<int8_t, kMaxRegs> out = kbool_[pc];
      const Insn& in = P_.code[pc];
      if (defines(in.op) && in.d != kNoReg) {
        int8_t v = -1;
        if (in.op == OP_CONST && in.imm >= 0 && in.imm < P_.n_const && !P_.is_lit[in.imm])
          v = P_.ctag[in.imm] == TAG_FLOAT ? (int8_t)(P_.fconst[in.imm] != 0.0 || std::isnan(P_.fconst[in.imm]))
                                           : (int8_t)(P_.iconst[in.imm] != 0);
        else if ((in.op == OP_MOV || in.op == OP_POS || in.op == OP_TRUTH) && in.a != kNoReg)
          v = kbool_[pc][in.a] >= 0 ? kbool_[pc][in.a] : -1;
        else if (in.op == OP_NOT && in.a != kNoReg)
          v = kbool_[pc][in.a] >= 0 ? (int8_t)(1 - kbool_[pc][in.a]) : -1;
        out[in.d] = v;
      }
      for (int t : succ_[pc]) {
        if (t < 0) continue;
        bool changed = !seen[t];
        for (int r = 0; r < kMaxRegs; ++r) {
          const int8_t nv = !seen[t] ? out[r] : (kbool_[t][r] == out[r] ? out[r] : (int8_t)-1);
          if (nv != kbool_[t][r]) { kbool_[t][r] = nv; changed = true; }
        }
        seen[t] = 1;
        if (changed) work.push_back(t);
      }
    }
  }
  // IFs whose condition is a known truth value: the dead branch leaves the
  // CFG (the next round of analyses is more precise); true: a change
  bool prune_static_ifs() {
    if (static_if_.empty()) static_if_.assign(n_, -1);
    bool changed = false;
    for (int pc = 0; pc < n_; ++pc) {
      const Insn& in = P_.code[pc];
      if (in.op != OP_IF || static_if_[pc] >= 0 || in.a == kNoReg) continue;
      const int8_t v = kbool_[pc][in.a];
      if (v < 0) continue;
      static_if_[pc] = v;
      succ_[pc] = v ? std::array<int, 2>{pc + 1, -1} : std::array<int, 2>{in.imm + 1, -1};
      changed = true;
    }
    return changed;
  }

  void const_facts() {
    kpool_.assign(n_, {});
    for (auto& a : kpool_) a.fill(-1);
    std::vector<char> seen(n_, 0);
    seen[0] = 1;
    std::vector<int> work{0};
    while (!work.empty()) {
      const int pc = work.back();
      work.pop_back();
      std::array<int16_t, kMaxRegs> out = kpool_[pc];
      const Insn& in = P_.code[pc];
      if (defines(in.op) && in.d != kNoReg) {
        int16_t v = -1;
        if (in.op == OP_CONST && in.imm >= 0 && in.imm < P_.n_const && !P_.is_lit[in.imm]) v = (int16_t)in.imm;
        else if ((in.op == OP_MOV || in.op == OP_POS) && in.a != kNoReg) v = kpool_[pc][in.a];
        out[in.d] = v;
      }
      for (int t : succ_[pc]) {
        if (t < 0) continue;
        bool changed = !seen[t];
        for (int r = 0; r < kMaxRegs; ++r) {
          const int16_t nv = !seen[t] ? out[r] : (kpool_[t][r] == out[r] ? out[r] : (int16_t)-1);
          if (nv != kpool_[t][r]) { kpool_[t][r] = nv; changed = true; }
        }
        seen[t] = 1;
        if (changed) work.push_back(t);
      }
    }
  }
  // inline operand code of register r's constant at pc (NONE: not foldable):
  // int context -- a sign-extended integer in [-16, 64]; float context -- one
  // of the float inline constants (0, +-0.5, +-1, +-2, +-4; an integer inline
  // constant in a float operand is a bit pattern, not a converted value)
  uint16_t fold_code(int pc, int r, bool as_float) const {
    if (r == kNoReg || pc < 0 || kpool_.empty()) return NONE;
    const int k = kpool_[pc][r];
    if (k < 0) return NONE;
    if (!as_float) return P_.ctag[k] != TAG_FLOAT ? ic(P_.iconst[k]) : NONE;
    const double x = P_.ctag[k] == TAG_FLOAT ? P_.fconst[k] : (double)P_.iconst[k];
    if (P_.ctag[k] != TAG_FLOAT && (P_.iconst[k] < -4 || P_.iconst[k] > 4)) return NONE;
    if (x == 0.0) return std::signbit(x) ? NONE : ic(0);
    static const double kF[8] = {0.5, -0.5, 1.0, -1.0, 2.0, -2.0, 4.0, -4.0};
    for (int i = 0; i < 8; ++i)
      if (x == kF[i]) return (uint16_t)(F_HALF + i);
    return NONE;
  }
  // which operands the lowering below takes as inline constants (so their
  // CONST need not be materialised when nothing else reads it)
  void fold_masks() {
    fold_.assign(n_, 0);
    for (int pc = 0; pc < n_; ++pc) {
      const Insn& in = P_.code[pc];
      const uint8_t ta = in.a != kNoReg ? ty_[pc][in.a] : TY_I, tb = in.b != kNoReg ? ty_[pc][in.b] : TY_I;
      uint64_t m = 0;
      auto f = [&](int r, bool fl) { if (fold_code(pc, r, fl) != NONE) m |= 1ull << r; };
      switch (in.op) {
        case OP_LT: case OP_LE: case OP_GT: case OP_GE: case OP_EQ: case OP_NE:
          if (in.imm == kLoopIndex && ta == TY_I && tb == TY_I) break;
          if (ta == TY_I && tb == TY_I) { f(in.a, false); f(in.b, false); }
          else if (ta != TY_IF && tb != TY_IF) { f(in.a, true); f(in.b, true); }
          break;
        case OP_ADD: case OP_SUB: case OP_MUL:
          if (ta == TY_I && tb == TY_I) {
            cur_pc_ = pc;
            const bool no_ovf = no_int_overflow(in.op, in.a, in.b);
            cur_pc_ = -1;
            if (no_ovf && !(in.op == OP_ADD && in.imm == kLoopIndex)) { f(in.a, false); f(in.b, false); }
          } else if (ta != TY_IF && tb != TY_IF) {
            f(in.a, true);
            f(in.b, true);
          }
          break;
        default: break;
      }
      if (in.a != kNoReg && in.a == in.b) m &= ~(1ull << in.a);   // (both operands: keep it simple)
      fold_[pc] = m;
    }
  }

  static uint8_t result_type(uint8_t op, uint8_t ta, uint8_t tb, uint8_t ct) {
    switch (op) {
      case OP_CONST: return ct;
      case OP_MOV: case OP_POS: return ta;
      case OP_POD: case OP_NODE: case OP_GPU: case OP_GLIST_ALL: case OP_GLIST_LEN: case OP_GLIST_GET:
      case OP_GLIST_SLICE: case OP_GLIST_NEW: case OP_GLIST_APPEND: case OP_GLIST_INSERT: case OP_NOT:
      case OP_TRUTH: case OP_ISINT: case OP_LT: case OP_LE: case OP_GT: case OP_GE: case OP_EQ: case OP_NE:
      case OP_INT: case OP_ROUND: case OP_LOOP_BEGIN:
        return TY_I;
      case OP_TDIV: case OP_FLOAT: case OP_SQRT: case OP_LOG: case OP_LOGB: case OP_EXP: case OP_MPOW:
      case OP_SIN: case OP_COS: case OP_TAN:
        return TY_F;
      case OP_ADD: case OP_SUB: case OP_MUL: case OP_FDIV: case OP_MOD:
        return (uint8_t)(((ta & TY_I) && (tb & TY_I) ? TY_I : 0) | ((ta & TY_F) || (tb & TY_F) ? TY_F : 0));
      case OP_POW:
        return (uint8_t)(((ta & TY_I) && (tb & TY_I) ? TY_IF : 0) | ((ta & TY_F) || (tb & TY_F) ? TY_F : 0));
      case OP_NEG: case OP_ABS: return ta;
      case OP_MIN2: case OP_MAX2: return (uint8_t)(ta | tb);
      default: return 0;
    }
  }

  void infer_types() {
    ty_.assign(n_, {});
    reached_.assign(n_, 0);
    for (auto& a : ty_) a.fill(TY_I);
    reached_[0] = 1;
    std::vector<int> work{0};
    std::vector<char> on(n_, 0);
    on[0] = 1;
    while (!work.empty()) {
      const int pc = work.back();
      work.pop_back();
      on[pc] = 0;
      const Insn& in = P_.code[pc];
      std::array<uint8_t, kMaxRegs> out = ty_[pc];
      if (in.d != kNoReg && defines(in.op)) {
        uint8_t ct = 0;
        if (in.op == OP_CONST) {
          if (in.imm < 0 || in.imm >= P_.n_const) throw CodegenError("constant index out of range");
          ct = P_.ctag[in.imm] == TAG_FLOAT ? TY_F : TY_I;
        }
        const uint8_t ta = in.a != kNoReg ? ty_[pc][in.a] : TY_I;
        const uint8_t tb = in.b != kNoReg ? ty_[pc][in.b] : TY_I;
        uint8_t t = result_type(in.op, ta, tb, ct);
        if (t == 0) t = TY_IF;
        out[in.d] = t;
      }
      for (int s : succ_[pc]) {
        if (s < 0) continue;
        bool changed = false;
        if (!reached_[s]) {
          reached_[s] = 1;
          ty_[s] = out;
          changed = true;
        } else {
          for (int r = 0; r < kMaxRegs; ++r) {
            const uint8_t u = (uint8_t)(ty_[s][r] | out[r]);
            if (u != ty_[s][r]) { ty_[s][r] = u; changed = true; }
          }
        }
        if (changed && !on[s]) { on[s] = 1; work.push_back(s); }
      }
    }
  }

  // side-effect-free definitions that emit nothing when their result is dead
  // (emit_op): they read nothing then either (strong liveness -- a chain of
  // dead copies, e.g. node.gpus built only for an unrolled loop, is dead as a whole)
  bool elidable_def(int pc) const {
    const Insn& in = P_.code[pc];
    if (in.d == kNoReg) return false;
    switch (in.op) {
      case OP_CONST: case OP_MOV: case OP_POS: case OP_POD: case OP_NODE: case OP_GLIST_ALL: case OP_GLIST_LEN:
        return true;
      case OP_GPU: return in.imm <= 1;
      default: return false;
    }
  }
  void liveness() {
    live_in_.assign(n_, 0);
    live_out_.assign(n_, 0);
    bool changed = true;
    while (changed) {
      changed = false;
      for (int pc = n_ - 1; pc >= 0; --pc) {
        uint64_t out = 0;
        for (int s : succ_[pc])
          if (s >= 0) out |= live_in_[s];
        const bool dead = elidable_def(pc) && !(out >> P_.code[pc].d & 1);
        const uint64_t in = (dead ? 0 : uses(pc)) | (out & ~defs(pc));
        if (out != live_out_[pc] || in != live_in_[pc]) {
          live_out_[pc] = out;
          live_in_[pc] = in;
          changed = true;
        }
      }
    }
  }

  // SIMT liveness: what ANY lane may still read.  The wave walks structured
  // code linearly (then-branch, then else-branch; code after a break or a
  // return still runs for the other lanes), so a register the suspended lanes
  // need later is live here even if no path of the active lanes reads it.
  // A runtime call clobbers every lane of the caller-saved registers, so its
  // spill set comes from this relation.
  void simt_liveness() {
    std::vector<uint64_t> in(n_, 0);
    slive_out_.assign(n_, 0);
    bool changed = true;
    while (changed) {
      changed = false;
      for (int pc = n_ - 1; pc >= 0; --pc) {
        const Insn& ins = P_.code[pc];
        uint64_t out = 0;
        if (ins.op != OP_END && pc + 1 < n_) out |= in[pc + 1];
        int t = -1;
        if (ins.op == OP_IF || ins.op == OP_ELSE || ins.op == OP_LOOP_TEST || ins.op == OP_LOOP_NEXT) t = ins.imm;
        if (t >= 0 && t < n_) out |= in[t];
        const bool dead = elidable_def(pc) && !(live_out_[pc] >> ins.d & 1);   // emits nothing
        const uint64_t li = (dead ? 0 : uses(pc)) | (out & ~defs(pc));
        if (out != slive_out_[pc] || li != in[pc]) {
          slive_out_[pc] = out;
          in[pc] = li;
          changed = true;
        }
      }
    }
  }

  // ============================================================ registers
  void layout_registers() {
    uint64_t used = 0;
    for (int pc = 0; pc < n_; ++pc) {
      const Insn& in = P_.code[pc];
      used |= uses(pc) | defs(pc);
      if (in.op == OP_NODE) use_node_ = true;
      if (in.op == OP_GLIST_ALL || in.op == OP_GLIST_LEN) use_node_ = true;
      if (in.op == OP_GPU) {
        if (in.imm == 0 || in.imm == 1) use_gl_ = true;
        else use_gmem_ = true;
      }
      if (in.op == OP_CONST && P_.is_lit[in.imm]) use_kc_ = true;
      if (in.op == OP_LOOP_BEGIN) has_loop_ = true;
      if (in.op == OP_POD) {
        const int f = (in.imm >= 0 && in.imm <= 5) ? in.imm : 5;
        pod_s_[f] = 1;
      }
    }
    // tagged registers: read somewhere while their type is mixed
    for (int pc = 0; pc < n_; ++pc) {
      if (!reached_[pc]) continue;
      const uint64_t u = uses(pc);
      for (int r = 0; r < kMaxRegs; ++r)
        if ((u >> r & 1) && ty_[pc][r] == TY_IF) tagged_ |= 1ull << r;
    }
    // interference
    std::vector<uint64_t> adj(kMaxRegs, 0);
    auto clique = [&](uint64_t set) {
      for (int r = 0; r < kMaxRegs; ++r)
        if (set >> r & 1) adj[r] |= set & ~(1ull << r);
    };
    clique(live_in_[0]);
    for (int pc = 0; pc < n_; ++pc) {
      clique(live_in_[pc]);
      const uint64_t d = defs(pc);
      if (d) {
        const int r = __builtin_ctzll(d);
        adj[r] |= live_out_[pc] & ~d;
        for (int q = 0; q < kMaxRegs; ++q)
          if (live_out_[pc] >> q & 1 && q != r) adj[q] |= d;
      }
    }
    // VGPR pools (caller-saved only; v0-v22 and v29 are the node arguments / kc).
    // The pod arguments (v23-v28) a program reads stay in place for its whole
    // run: they are per-lane, not wave-uniform -- in the four-programs-per-wave
    // row kernel one call can cover several DPP rows (programs of one shape),
    // each with its own pod.
    const bool pv23 = pod_s_[0] > 0, pv24 = pod_s_[1] > 0, pv25 = pod_s_[2] > 0 || pod_s_[3] > 0;
    const bool pv26 = pod_s_[4] > 0, pv28 = pod_s_[5] > 0;
    std::vector<int> pairs;
    if (!pv24 && !pv25) pairs.push_back(24);
    if (!pv26) pairs.push_back(26);
    for (int b : {30, 32, 34, 36, 38, 48, 50, 52, 54, 64, 66, 68, 70, 80, 82, 84, 86, 96, 98, 100, 102, 112, 114, 116,
                  118})
      pairs.push_back(b);
    std::vector<int> singles;
    if (!pv28) singles.push_back(28);
    if (pv24 && !pv25) singles.push_back(25);
    if (pv25 && !pv24) singles.push_back(24);
    if (!use_gl_) {
      for (int b = 6; b <= 18; b += 2) pairs.push_back(b);
      singles.push_back(5);
      singles.push_back(20);
    }
    if (!use_gmem_) {
      if (!pv23) pairs.push_back(22);
      else singles.push_back(22);
    } else if (!pv23) {
      singles.push_back(23);
    }
    if (!use_node_ && !use_gl_ && !use_gmem_) {
      // node fields unused: v0-v4 are free too (v0-v1 also carry the result)
      pairs.push_back(2);
      singles.push_back(4);
    }
    auto take_pair = [&]() {
      if (pairs.empty()) throw CodegenError("out of VGPR pairs");
      const int b = pairs.front();
      pairs.erase(pairs.begin());
      max_vgpr_ = std::max(max_vgpr_, b + 1);
      return b;
    };
    auto take_single = [&]() {
      if (singles.empty()) {
        const int b = take_pair();
        singles.push_back(b + 1);
        return b;
      }
      const int s1 = singles.front();
      singles.erase(singles.begin());
      max_vgpr_ = std::max(max_vgpr_, s1);
      return s1;
    };
    for (int i = 0; i < 4; ++i) F_.mr.x[i] = take_pair();
    for (int i = 0; i < 3; ++i) T_[i] = take_pair();
    v_out_ = take_pair();
    v_exc_ = take_single();
    n_tagged_ = __builtin_popcountll(tagged_);
    tagbit_.fill(-1);
    {
      int k = 0;
      for (int r = 0; r < kMaxRegs; ++r)
        if (tagged_ >> r & 1) tagbit_[r] = k++;
      if (k > 0) v_tag_[0] = take_single();
      if (k > 32) v_tag_[1] = take_single();
    }
    v_spill_ = take_single();
    // colour virtual registers (most-constrained first)
    base_.fill(-1);
    map_.fill(-1);
    slot_.fill(-1);
    std::vector<int> regs;
    for (int r = 0; r < kMaxRegs; ++r)
      if (used >> r & 1) regs.push_back(r);
    n_vregs_ = (int)regs.size();
    if (pair_cap() > 0 && (int)pairs.size() > pair_cap()) pairs.resize((size_t)pair_cap() + 5);
    // colours for the registers outside `spill` from `pool`; false: not enough pairs
    auto colour_with = [&](uint64_t spill, const std::vector<int>& pool, size_t cap) {
      std::vector<int> order;
      for (int r : regs)
        if (!(spill >> r & 1)) order.push_back(r);
      std::stable_sort(order.begin(), order.end(),
                       [&](int a, int b) { return __builtin_popcountll(adj[a]) > __builtin_popcountll(adj[b]); });
      std::vector<int> colour(kMaxRegs, -1);
      size_t n_col = 0;
      for (int r : order) {
        std::vector<char> busy(n_col, 0);
        for (int q = 0; q < kMaxRegs; ++q)
          if ((adj[r] >> q & 1) && colour[q] >= 0) busy[(size_t)colour[q]] = 1;
        int c = -1;
        for (size_t k = 0; k < busy.size(); ++k)
          if (!busy[k]) { c = (int)k; break; }
        if (c < 0) {
          if (n_col >= std::min(cap, pool.size())) return false;
          c = (int)n_col++;
        }
        colour[r] = c;
      }
      for (int r : order) base_[r] = pool[(size_t)colour[r]];
      for (size_t k = 0; k < n_col; ++k) max_vgpr_ = std::max(max_vgpr_, pool[k] + 1);
      return true;
    };
    const size_t cap0 = pair_cap() > 0 ? (size_t)pair_cap() : pairs.size();
    if (!colour_with(0, pairs, cap0)) {
      // spill: reserve the reload pairs, then move registers to scratch -- most
      // interference per static use first -- until the rest colour
      if (pairs.size() < 6) throw CodegenError("out of VGPR pairs");
      std::vector<int> pool(pairs.begin(), pairs.end());
      for (int k = 0; k < 4; ++k) rl_[k] = pool[(size_t)k];
      m_tmp_ = pool[4];
      for (int k = 0; k < 5; ++k) max_vgpr_ = std::max(max_vgpr_, pool[(size_t)k] + 1);
      pool.erase(pool.begin(), pool.begin() + 5);
      std::array<int, kMaxRegs> nuse{};
      for (int pc = 0; pc < n_; ++pc) {
        const uint64_t ud = uses(pc) | defs(pc);
        for (int r = 0; r < kMaxRegs; ++r) nuse[r] += (int)(ud >> r & 1);
      }
      // (control-flow instructions are safe too: labels inside ELSE / ENDIF /
      // LOOP_EXIT precede no register access, IF / LOOP_TEST read their
      // condition right after the reload, LOOP_BEGIN places the loop head
      // before the next instruction's reloads)
      std::vector<int> cand(regs);
      std::stable_sort(cand.begin(), cand.end(), [&](int a, int b) {
        return (int64_t)__builtin_popcountll(adj[a]) * (1 + nuse[b]) > (int64_t)__builtin_popcountll(adj[b]) * (1 + nuse[a]);
      });
      const size_t cap1 = pair_cap() > 0 ? (size_t)pair_cap() : pool.size();
      bool ok = false;
      for (int r : cand) {
        if (__builtin_popcountll(spilled_) >= kMaxSpills) break;
        slot_[r] = 8 * __builtin_popcountll(spilled_);
        spilled_ |= 1ull << r;
        base_.fill(-1);
        if (colour_with(spilled_, pool, cap1)) { ok = true; break; }
      }
      if (!ok) throw CodegenError("out of VGPR pairs");
      F_.spill_bytes = 8 * __builtin_popcountll(spilled_);
    }
    // SGPR pairs: s[24:25] and s[28:29] are macro scratch; s30-s33 ABI; callee-saved ones untouched
    free_spairs_ = {0, 2, 4, 6, 8, 10, 12, 14, 16, 18, 20, 22, 26, 40, 42, 44, 46, 56, 58, 60, 62, 72, 74, 76, 78,
                    88, 90, 92, 94};
    s_entry_ = take_spair();
    s_dead_ = take_spair();
    if (has_loop_) s_bud_ = take_spair();
    for (int i = 0; i < 3; ++i) ST_[i] = take_spair();
    S_LIT_ = take_spair();
    bm_pair_[0] = take_spair();
    bm_pair_[1] = take_spair();
    bm_of_.fill(-1);
    static const int pod_arg[6] = {23, 24, 25, 25, 26, 28};
    for (int f = 0; f < 6; ++f) pod_s_[f] = pod_s_[f] > 0 ? pod_arg[f] : -1;   // now: the argument VGPR
  }
  int take_spair() {
    if (free_spairs_.empty()) throw CodegenError("out of SGPR pairs");
    const int b = free_spairs_.front();
    free_spairs_.erase(free_spairs_.begin());
    max_sgpr_ = std::max(max_sgpr_, b + 1);
    return b;
  }
  void give_spair(int b) {
    free_spairs_.insert(free_spairs_.begin(), b);
  }

  // ============================================================ emission helpers
  // Emission.  LDS loads (constant reads) are waited for lazily: right before
  // the first instruction that touches their destination, or at any label /
  // branch / call (so every control-flow merge starts with nothing pending).
  std::vector<uint16_t> lds_pending_;
  uint8_t cur_bc_ = 255;   // bytecode opcode being lowered (MI::bc)
  void e(const MI& m) {
    if (!lds_pending_.empty()) {
      bool need = m.op == LABEL || is_branch(m.op) || m.op == S_SETPC_B64 || m.op == M_RTCALL || m.op == S_WAITCNT;
      for (uint16_t b : lds_pending_)
        for (uint16_t c : {m.s0, m.s1, m.s2, m.d, m.sd})
          if (c != NONE && c + 1 >= b && c <= b + 1) need = true;
      if (need) {
        lds_pending_.clear();
        if (m.op != S_WAITCNT) {
          F_.mi.push_back(mkimm(S_WAITCNT, 0xC07F));
          F_.mi.back().bc = cur_bc_;
        }
      }
    }
    F_.mi.push_back(m);
    F_.mi.back().bc = cur_bc_;
    if (m.op == DS_READ_B64) lds_pending_.push_back(m.d);
  }
  // Bool-mask cache: a register that holds a 0 / 1 produced in the current
  // basic block also has its lane mask in one of two SGPR pairs, so IF /
  // NOT / TRUTH / LOOP_TEST of it need no VALU compare.  Invalidated at every
  // label, structural op, call and redefinition.
  //
  // Bools are materialised lazily: a compare only records its mask; the 0 / 1
  // value is written to the register when something reads it as a number,
  // when its mask slot is reused, or -- if it is still live -- before EXEC
  // changes (structural ops, leaving lanes, calls), always under the EXEC it
  // was computed with.
  int bm_pair_[2] = {-1, -1};
  std::array<int8_t, kMaxRegs> bm_of_{};
  int bm_next_ = 0;
  uint64_t pend_ = 0;   // registers whose value is only in their mask slot
  void materialize(int r) {
    if (!(pend_ >> r & 1)) return;
    pend_ &= ~(1ull << r);
    if (spilled_ >> r & 1) {   // into the register's reload pair (if mapped) and its slot
      const int p = map_[r] >= 0 ? map_[r] : m_tmp_;
      e(mk(V_CNDMASK_B32, v(p), ic(0), ic(1), s(bm_pair_[bm_of_[r]])));
      e(mk(V_MOV_B32, v(p + 1), ic(0)));
      spill_store(r, p);
      return;
    }
    e(mk(V_CNDMASK_B32, R(r), ic(0), ic(1), s(bm_pair_[bm_of_[r]])));
    e(mk(V_MOV_B32, Rh(r), ic(0)));
  }
  // scratch slot of spilled register r <-> VGPR pair p (active lanes)
  void spill_store(int r, int p) {   // dword accesses (scratch is swizzled per lane in dwords)
    for (int h = 0; h < 2; ++h) {
      MI st = mk(SCRATCH_STORE_DWORD, NONE, NONE, s(32), v(p + h));
      st.imm = slot_[r] + 4 * h;
      e(st);
    }
  }
  void spill_load(int r, int p) {
    for (int h = 0; h < 2; ++h) {
      MI ld = mk(SCRATCH_LOAD_DWORD, v(p + h), NONE, s(32));
      ld.imm = slot_[r] + 4 * h;
      e(ld);
    }
  }
  // before instruction pc: its spilled operands (and destination: partial
  // writes keep the inactive lanes' value) in reload pairs
  void spill_in(int pc) {
    const uint64_t need = (uses(pc) | defs(pc)) & spilled_;
    if (!need) return;
    int k = 0;
    for (int r = 0; r < kMaxRegs; ++r)
      if (need >> r & 1) {
        if (k >= 4) throw CodegenError("internal: more than four spilled registers in one instruction");
        map_[r] = rl_[k++];
        spill_load(r, map_[r]);
      }
    e(mkimm(S_WAITCNT, 0x0F70));   // vmcnt(0)
  }
  // after it: the destination back to its slot (a bool still only in its
  // mask is stored when it is materialised)
  void spill_out(int pc) {
    if (!spilled_) return;
    const uint64_t dd = defs(pc) & spilled_;
    for (int r = 0; r < kMaxRegs; ++r)
      if ((dd >> r & 1) && !(pend_ >> r & 1) && map_[r] >= 0) spill_store(r, map_[r]);
    map_.fill(-1);
  }
  void materialize_live(uint64_t live) {
    for (int r = 0; r < kMaxRegs; ++r)
      if ((pend_ >> r & 1) && (live >> r & 1)) materialize(r);
    pend_ = 0;
  }
  void bm_clear() {
    if (pend_) throw CodegenError("internal: pending bools at an EXEC change");
    bm_of_.fill(-1);
  }
  void bm_set(int r, uint16_t mask) {
    const int slot = bm_next_++ & 1;
    for (int q = 0; q < kMaxRegs; ++q)
      if (bm_of_[q] == slot && q != r) {
        if (mask == s(bm_pair_[slot])) continue;   // the source mask itself stays
        materialize(q);
        bm_of_[q] = -1;
      }
    if (mask != s(bm_pair_[slot])) e(mk(S_MOV_B64, s(bm_pair_[slot]), mask));
    bm_of_[r] = (int8_t)slot;
  }
  uint16_t R(int r) const {
    if (spilled_ >> r & 1) {
      if (map_[r] < 0) throw CodegenError("spilled register used outside its instruction");
      return v(map_[r]);
    }
    if (base_[r] < 0) throw CodegenError("register without a home");
    return v(base_[r]);
  }
  uint16_t Rh(int r) const { return (uint16_t)(R(r) + 1); }
  uint16_t T(int i) const { return v(T_[i]); }
  uint16_t Th(int i) const { return v(T_[i] + 1); }
  uint16_t X(int i) const { return v(F_.mr.x[i]); }
  uint16_t ST(int i) const { return s(ST_[i]); }
  uint16_t TAGV(int r) const { return v(v_tag_[tagbit_[r] >> 5]); }
  int label() { return F_.new_label(); }
  void place(int lab) {
    e(mkimm(LABEL, lab));
    bm_clear();
  }
  int label_for_pc(int pc) {
    auto it = label_at_pc_.find(pc);
    if (it != label_at_pc_.end()) return it->second;
    const int l = label();
    label_at_pc_[pc] = l;
    return l;
  }

  // VOPC into an SGPR pair
  void cmp(Opc op, uint16_t dst, uint16_t a, uint16_t b, uint8_t abs = 0) {
    MI m = mk(op, NONE, a, b);
    m.sd = dst;
    m.abs = abs;
    e(m);
  }
  void movk64(uint16_t dst_pair, uint64_t x) {   // SGPR pair constant
    for (int h = 0; h < 2; ++h) {
      const uint32_t w = (uint32_t)(x >> (32 * h));
      const uint16_t c = ic((int32_t)w);
      if (c != NONE) e(mk(S_MOV_B32, (uint16_t)(dst_pair + h), c));
      else e(mklit(S_MOV_B32, (uint16_t)(dst_pair + h), w));
    }
  }
  void vmov32(uint16_t d, uint32_t x) {
    const uint16_t c = ic((int32_t)x);
    if (c != NONE) e(mk(V_MOV_B32, d, c));
    else e(mklit(V_MOV_B32, d, x));
  }
  // exc = (exc == 0 && lanes(mask)) ? code : exc
  // Raising lanes record their code and leave EXEC at once (s_dead_), so every
  // active lane has no exception yet and a raise is one v_cndmask: codes >= 100
  // are held as code - 44 (56-59, inline constants) and mapped back in the
  // epilogue.  Every EXEC restore excludes s_dead_.
  static int exc_internal(int code) { return code >= 100 ? code - 44 : code; }
  void kill_vcc() {
    e(mk(S_OR_B64, s(s_dead_), s(s_dead_), VCC));
    e(mk(S_ANDN2_B64, EXEC, EXEC, VCC));
  }
  void soft_raise(uint16_t mask, int code) {
    const int c = exc_internal(code);
    e(mk(S_AND_B64, VCC, EXEC, mask));
    if (ic(c) != NONE) e(mk(V_CNDMASK_B32, v(v_exc_), v(v_exc_), ic(c), VCC));
    else {
      vmov32(Th(2), (uint32_t)c);
      e(mk(V_CNDMASK_B32, v(v_exc_), v(v_exc_), Th(2), VCC));
    }
    kill_vcc();
  }
  // same with the (external) code in a VGPR
  void soft_raise_v(uint16_t mask, uint16_t code_v) {
    e(mklit(S_MOV_B32, s(S_LIT_), 100u));
    cmp(V_CMP_GE_U32, ST(2), code_v, s(S_LIT_));
    e(mklit(V_ADD_U32, Th(2), (uint32_t)-44, code_v));
    e(mk(V_CNDMASK_B32, Th(2), code_v, Th(2), ST(2)));
    e(mk(S_AND_B64, VCC, EXEC, mask));
    e(mk(V_CNDMASK_B32, v(v_exc_), v(v_exc_), Th(2), VCC));
    kill_vcc();
  }
  // lanes where register r holds a float -> SGPR pair
  void tag_mask(int r, uint16_t dst) {
    if (tagbit_[r] < 0) throw CodegenError("dynamic type of an untagged register");
    e(mk(V_BFE_U32, Th(2), TAGV(r), ic(tagbit_[r] & 31), ic(1)));
    cmp(V_CMP_NE_U32, dst, ic(0), Th(2));
  }
  // float flag of register r (type t at this pc) as an operand (inline 0 / 1 or a VGPR)
  uint16_t flag_of(int r, uint8_t t, uint16_t tmpv) {
    if (t == TY_I) return ic(0);
    if (t == TY_F) return ic(1);
    if (tagbit_[r] < 0) throw CodegenError("dynamic type of an untagged register");
    e(mk(V_BFE_U32, tmpv, TAGV(r), ic(tagbit_[r] & 31), ic(1)));
    return tmpv;
  }
  void set_tag_static(int r, bool fl) {
    if (tagbit_[r] < 0) return;
    const uint32_t bit = 1u << (tagbit_[r] & 31);
    if (fl) {
      if (ic(bit) != NONE) e(mk(V_OR_B32, TAGV(r), ic(bit), TAGV(r)));
      else e(mklit(V_OR_B32, TAGV(r), bit, TAGV(r)));
    } else {
      e(mklit(V_AND_B32, TAGV(r), ~bit, TAGV(r)));
    }
  }
  void set_tag_flag(int r, uint16_t flag_v) {   // flag_v: VGPR holding 0 / 1
    if (tagbit_[r] < 0) return;
    set_tag_static(r, false);
    e(mk(V_LSHLREV_B32, Th(2), ic(tagbit_[r] & 31), flag_v));
    e(mk(V_OR_B32, TAGV(r), TAGV(r), Th(2)));
  }
  void set_tag_mask(int r, uint16_t mask) {     // lanes of mask: float
    if (tagbit_[r] < 0) return;
    e(mk(V_CNDMASK_B32, Th(1), ic(0), ic(1), mask));
    set_tag_flag(r, Th(1));
  }
  void copy_tag(int d, int a, uint8_t ta) {
    if (tagbit_[d] < 0) return;
    if (ta == TY_I) set_tag_static(d, false);
    else if (ta == TY_F) set_tag_static(d, true);
    else {
      const uint16_t f = flag_of(a, ta, Th(1));
      set_tag_flag(d, f);
    }
  }
  // f64 value of register r (type t) -> operand code of a pair
  // operand r of the instruction being lowered as an inline constant (fold_), or NONE
  uint16_t fold_of(int r, bool as_float) const {
    if (cur_pc_ < 0 || fold_.empty() || r == kNoReg || !(fold_[cur_pc_] >> r & 1)) return NONE;
    return fold_code(cur_pc_, r, as_float);
  }
  uint16_t opi(int r) const { const uint16_t c = fold_of(r, false); return c != NONE ? c : R(r); }
  uint16_t opih(int r) const {   // high dword (sign of an inline integer)
    const uint16_t c = fold_of(r, false);
    if (c == NONE) return Rh(r);
    return (c >= 193 && c <= 208) ? ic(-1) : ic(0);
  }
  uint16_t as_f64(int r, uint8_t t, int tmp) {
    if (t != TY_IF) {
      const uint16_t c = fold_of(r, true);
      if (c != NONE) return c;
    }
    if (t == TY_F) return R(r);
    if (t == TY_I && i32(r)) {   // exact from the low dword
      e(mk(V_CVT_F64_I32, T(tmp), R(r)));
      return T(tmp);
    }
    e(mk(M_CVT_F64_I64, T(tmp), R(r)));
    if (t == TY_I) return T(tmp);
    tag_mask(r, ST(1));
    e(mk(V_CNDMASK_B32, T(tmp), T(tmp), R(r), ST(1)));
    e(mk(V_CNDMASK_B32, Th(tmp), Th(tmp), Rh(r), ST(1)));
    return T(tmp);
  }
  // lanes (of `lanes_mask`) whose int64 operand (pair p) is outside [-2^53, 2^53] -> EXC_UNSUPPORTED
  void check_exact_int(uint16_t p, uint16_t lanes_mask) {
    e(mk(S_MOV_B32, s(S_LIT_), ic(0)));
    e(mklit(S_MOV_B32, s(S_LIT_ + 1), 0x00200000u));
    e(mk(V_LSHL_ADD_U64, T(0), p, ic(0), s(S_LIT_)));   // x + 2^53
    e(mklit(S_MOV_B32, s(S_LIT_ + 1), 0x00400000u));
    cmp(V_CMP_GT_U64, ST(1), T(0), s(S_LIT_));
    if (lanes_mask != EXEC) e(mk(S_AND_B64, ST(1), ST(1), lanes_mask));
    soft_raise(ST(1), EXC_UNSUPPORTED);
  }
  // SGPR pairs live across a runtime call
  std::vector<int> live_sgprs() const {
    std::vector<int> out = {30, 31, s_entry_, s_entry_ + 1, s_dead_, s_dead_ + 1};
    if (s_bud_ >= 0) out.push_back(s_bud_);
    for (int b : held_spairs_) { out.push_back(b); out.push_back(b + 1); }
    for (const Frame& fr : frames_)
      for (int b : {fr.s_save, fr.s_else, fr.s_entry, fr.s_brk, fr.s_cont})
        if (b >= 0) { out.push_back(b); out.push_back(b + 1); }
    return out;
  }
  // Argument VGPRs are read only by NODE / GLIST_ALL / GLIST_LEN / GPU / POD
  // instructions; past the last such read (a read inside a loop counts up to
  // the loop's exit) a class of them is dead and a runtime call need not save
  // it.  The code is structured and emitted in pc order, so this pc bound is
  // exact for the wave (SIMT) as well.
  enum ArgClass { AC_NODE, AC_GL, AC_GMEM, AC_POD, AC_N };
  std::array<int, AC_N> arg_last_{};
  void arg_liveness() {
    arg_last_.fill(-1);
    std::vector<std::pair<int, int>> loops;   // (LOOP_BEGIN pc, LOOP_EXIT pc)
    std::vector<int> open;
    for (int pc = 0; pc < n_; ++pc) {
      const Insn& in = P_.code[pc];
      if (in.op == OP_LOOP_BEGIN) open.push_back(pc);
      else if (in.op == OP_LOOP_EXIT && !open.empty()) { loops.push_back({open.back(), pc}); open.pop_back(); }
    }
    auto mark = [&](int cls, int pc) {
      int end = pc;
      for (const auto& l : loops)
        if (l.first <= pc && pc <= l.second) end = std::max(end, l.second);
      arg_last_[cls] = std::max(arg_last_[cls], end);
    };
    for (int pc = 0; pc < n_; ++pc) {
      const Insn& in = P_.code[pc];
      if (in.op == OP_NODE || in.op == OP_GLIST_ALL || in.op == OP_GLIST_LEN || list_truth(pc, in.a))
        mark(AC_NODE, pc);
      if (in.op == OP_GPU) mark(in.imm == 0 || in.imm == 1 ? AC_GL : AC_GMEM, pc);
      if (in.op == OP_GPU) mark(AC_NODE, pc);   // (GPU j exists: the count in v4)
      if (in.op == OP_POD) mark(AC_POD, pc);
    }
  }
  std::vector<int> live_vgprs(int pc, int d) const {
    std::vector<int> out;
    if ((use_node_ || use_gl_ || use_gmem_) && arg_last_[AC_NODE] > pc)
      for (int g = 0; g <= 4; ++g) out.push_back(g);
    if (use_gl_ && arg_last_[AC_GL] > pc)
      for (int g = 5; g <= 20; ++g) out.push_back(g);
    if (use_gmem_ && arg_last_[AC_GMEM] > pc) { out.push_back(21); out.push_back(22); }
    for (int f = 0; f < 6; ++f)   // pod arguments the program still reads
      if (pod_s_[f] >= 0 && arg_last_[AC_POD] > pc) {
        out.push_back(pod_s_[f]);
        if (f == 4) out.push_back(pod_s_[f] + 1);
      }
    out.push_back(29);
    out.push_back(v_exc_);
    out.push_back(v_out_);
    out.push_back(v_out_ + 1);
    for (int t : v_tag_)
      if (t >= 0) out.push_back(t);
    // the destination is included: lanes outside EXEC keep its old value
    const uint64_t live = slive_out_[pc] | live_out_[pc] | (d >= 0 ? (1ull << d) : 0ull);
    std::set<int> bases;
    for (int r = 0; r < kMaxRegs; ++r)
      if ((live >> r & 1) && base_[r] >= 0) bases.insert(base_[r]);
    for (int b : bases) { out.push_back(b); out.push_back(b + 1); }
    for (int r = 0; r < kMaxRegs; ++r)   // spilled operands reloaded for this instruction
      if (map_[r] >= 0) { out.push_back(map_[r]); out.push_back(map_[r] + 1); }
    std::sort(out.begin(), out.end());
    out.erase(std::unique(out.begin(), out.end()), out.end());
    return out;
  }
  // d = rt_binop / rt_unop(op, a[, b]) with Python semantics for any operand types
  void rtcall(int kind, int op, int pc, int d, int a, uint8_t ta, int b = -1, uint8_t tb = TY_I) {
    materialize_live(slive_out_[pc] | live_out_[pc]);
    e(mk(V_MOV_B64, X(0), R(a)));
    CallInfo c;
    c.kind = kind;
    c.op = op;
    c.a = X(0);
    c.afl = flag_of(a, ta, X(3));
    if (kind == 0) {
      e(mk(V_MOV_B64, X(1), R(b)));
      c.b = X(1);
      c.bfl = flag_of(b, tb, (uint16_t)(X(3) + 1));
    }
    c.res = X(2);
    c.resy = X(3);
    c.spill_vgpr = v(v_spill_);
    c.vgprs = live_vgprs(pc, d);
    c.sgprs = live_sgprs();
    if (c.sgprs.size() > 64) throw CodegenError("too many SGPRs live across a call");
    MI m;
    m.op = M_RTCALL;
    m.ext = (int)F_.calls.size();
    F_.calls.push_back(c);
    e(m);
    bm_clear();   // the callee clobbers the mask registers
    // exception code: fl | e << 8
    e(mk(V_LSHRREV_B32, Th(0), ic(8), X(3)));
    cmp(V_CMP_NE_U32, ST(0), ic(0), Th(0));
    soft_raise_v(ST(0), Th(0));
    e(mk(V_MOV_B64, R(d), X(2)));
    if (tagbit_[d] >= 0) {
      e(mk(V_AND_B32, T(0), ic(1), X(3)));
      set_tag_flag(d, T(0));
    }
  }

  Frame* innermost_loop() {
    for (auto it = frames_.rbegin(); it != frames_.rend(); ++it)
      if (it->loop) return &*it;
    return nullptr;
  }
  // EXEC = base & ~(lanes that left the construct)
  void restore_exec(uint16_t base) {
    e(mk(S_ANDN2_B64, EXEC, base, s(s_dead_)));
    if (Frame* l = innermost_loop()) {
      if (l->s_brk >= 0) e(mk(S_ANDN2_B64, EXEC, EXEC, s(l->s_brk)));
      if (l->s_cont >= 0) e(mk(S_ANDN2_B64, EXEC, EXEC, s(l->s_cont)));
    }
  }
  // lanes of EXEC leave the function here
  void leave_function() {
    e(mk(S_OR_B64, s(s_dead_), s(s_dead_), EXEC));
    e(mk(S_MOV_B64, EXEC, ic(0)));
  }
  // truth(r) -> SGPR pair
  uint16_t truth(int r, uint8_t t, uint16_t dst) {
    if (bm_of_[r] >= 0) return s(bm_pair_[bm_of_[r]]);
    if (list_truth(cur_pc_, r)) {   // node.gpus: nonempty = a GPU count above 0 (the list itself unread)
      e(mk(V_LSHRREV_B32, Th(1), ic(16), v(4)));
      cmp(V_CMP_NE_U32, dst, ic(0), Th(1));
      return dst;
    }
    if (t == TY_I) { cmp(V_CMP_NE_I64, dst, ic(0), R(r)); return dst; }
    if (t == TY_F) { cmp(V_CMP_NEQ_F64, dst, ic(0), R(r)); return dst; }
    tag_mask(r, ST(1));
    cmp(V_CMP_NE_I64, dst, ic(0), R(r));
    cmp(V_CMP_NEQ_F64, ST(2), ic(0), R(r));
    e(mk(S_AND_B64, ST(2), ST(2), ST(1)));
    e(mk(S_ANDN2_B64, dst, dst, ST(1)));
    e(mk(S_OR_B64, dst, dst, ST(2)));
    return dst;
  }
  void set_bool(int d, uint16_t mask) {   // d = int(mask), materialised lazily
    set_tag_static(d, false);
    bm_set(d, mask);
    pend_ |= 1ull << d;
  }
  // the mask slot a new bool d is computed into directly (no copy from a
  // scratch pair): its other occupants are materialised first; commit_bool
  // then makes d pending in it
  uint16_t bool_slot(int d) {
    const int slot = bm_next_ & 1;
    for (int q = 0; q < kMaxRegs; ++q)
      if (bm_of_[q] == slot && q != d) {
        materialize(q);
        bm_of_[q] = -1;
      }
    return s(bm_pair_[slot]);
  }
  void commit_bool(int d) {
    const int slot = bm_next_++ & 1;
    set_tag_static(d, false);
    bm_of_[d] = (int8_t)slot;
    pend_ |= 1ull << d;
  }

  // ============================================================ per-op lowering
  void emit_all() {
    // prologue
    e(mkimm(S_WAITCNT, 0));
    e(mk(S_MOV_B64, s(s_entry_), EXEC));
    e(mk(S_MOV_B64, s(s_dead_), ic(0)));
    e(mk(V_MOV_B32, v(v_exc_), ic(0)));
    e(mk(V_MOV_B64, v(v_out_), ic(0)));
    for (int t : v_tag_)
      if (t >= 0) e(mk(V_MOV_B32, v(t), ic(0)));
    if (s_bud_ >= 0) {
      // kc[0] = the iteration budget, capped; one counter for the wave: a lane
      // never runs more iterations than the wave
      MI ld = mk(DS_READ_B64, T(0), v(29));
      ld.imm = 0;
      e(ld);
      e(mkimm(S_WAITCNT, 0xC07F));
      // min(kc[0], cap) with kc[0] <= 0 (unlimited) -> the cap: (x - 1 as unsigned) min (cap - 1), + 1
      e(mklit(V_ADD_U32, T(0), 0xFFFFFFFFu, T(0)));
      e(mklit(V_MIN_U32, T(0), kJitLoopCap - 1, T(0)));
      e(mk(V_ADD_U32, T(0), ic(1), T(0)));
      e(mk(V_READFIRSTLANE_B32, s(s_bud_), T(0)));
    }
    for (int r = 0; r < kMaxRegs; ++r) {
      if (!(live_in_[0] >> r & 1)) continue;
      if (spilled_ >> r & 1) {
        e(mk(V_MOV_B64, v(m_tmp_), ic(0)));
        spill_store(r, m_tmp_);
      } else if (base_[r] >= 0) {
        e(mk(V_MOV_B64, R(r), ic(0)));
      }
    }
    const int l_end = label();
    for (int pc = 0; pc < n_; ++pc) {
      if (pc < skip_to_) continue;   // the dead branch of a known condition
      auto it = label_at_pc_.find(pc);
      if (it != label_at_pc_.end() && P_.code[pc].op != OP_ENDIF && P_.code[pc].op != OP_ELSE &&
          P_.code[pc].op != OP_LOOP_EXIT)
        place(it->second);
      // unreached code is skipped, but structural ops still open / close
      // their EXEC frames (an ENDIF after a then-branch that always returns
      // is unreached by flow, yet the IF branches to it)
      if (!reached_[pc] && !structural(P_.code[pc].op)) continue;
      cur_bc_ = P_.code[pc].op;
      cur_pc_ = pc;
      spill_in(pc);
      emit_op(pc);
      spill_out(pc);
      cur_bc_ = 255;
      cur_pc_ = -1;
    }
    if (!frames_.empty()) throw CodegenError("unbalanced control flow");
    // epilogue: v[0:1] = exc ? -exc : out
    place(l_end);
    e(mk(S_MOV_B64, EXEC, s(s_entry_)));
    cmp(V_CMP_GE_U32, ST(0), v(v_exc_), ic(56));                  // internal code -> EXC_*
    e(mk(V_ADD_U32, T(1), ic(44), v(v_exc_)));
    e(mk(V_CNDMASK_B32, v(v_exc_), v(v_exc_), T(1), ST(0)));
    cmp(V_CMP_NE_U32, ST(0), ic(0), v(v_exc_));
    e(mk(V_SUB_U32, T(0), ic(0), v(v_exc_)));
    e(mk(V_CNDMASK_B32, v(0), v(v_out_), T(0), ST(0)));
    e(mk(V_CNDMASK_B32, v(1), v(v_out_ + 1), ic(-1), ST(0)));
    e(mk(S_SETPC_B64, NONE, s(30)));
  }

  void emit_op(int pc) {
    const Insn& in = P_.code[pc];
    const auto& st = ty_[pc];
    const uint8_t ta = in.a != kNoReg ? st[in.a] : TY_I;
    const uint8_t tb = in.b != kNoReg ? st[in.b] : TY_I;
    const int d = in.d, a = in.a, b = in.b;
    // a side-effect-free definition nothing reads (e.g. node.gpus built for a
    // len() or an unrolled loop) emits nothing -- its operands are not read
    // either (strong liveness: they need not even hold a value)
    if (elidable_def(pc) && !(live_out_[pc] >> d & 1)) {
      pend_ &= ~(1ull << d);
      bm_of_[d] = -1;
      return;
    }
    const bool exec_change = structural(in.op) || in.op == OP_BREAK || in.op == OP_CONTINUE || in.op == OP_RET ||
                             in.op == OP_RAISE || in.op == OP_END;
    const bool via_mask = in.op == OP_IF || in.op == OP_LOOP_TEST || in.op == OP_NOT || in.op == OP_TRUTH;
    // operands read as numbers must hold their value
    if (!(in.op == OP_MOV || in.op == OP_POS || via_mask)) {
      const uint64_t u = uses(pc) & pend_;
      for (int r = 0; r < kMaxRegs; ++r)
        if (u >> r & 1) materialize(r);
    }
    // bools still live must be written before EXEC changes (IF / LOOP_TEST
    // take their operand's mask first, then materialise)
    uint16_t mask_a = NONE;
    if (exec_change) {
      if ((in.op == OP_IF && static_if_[pc] < 0) || in.op == OP_LOOP_TEST) mask_a = truth(a, ta, ST(0));
      // (a bool's mask pair survives the materialisation below: used in place)
      materialize_live(slive_out_[pc] | live_out_[pc]);
      bm_clear();
    } else if (defines(in.op) && d != kNoReg && !via_mask) {
      // (NOT / TRUTH read their operand's mask first and set d's state themselves)
      if (!(in.op == OP_MOV || in.op == OP_POS)) bm_of_[d] = -1;
      if (!((in.op == OP_MOV || in.op == OP_POS) && (pend_ >> a & 1))) pend_ &= ~(1ull << d);
    }
    switch (in.op) {
      case OP_NOP: break;
      case OP_CONST: {
        const int k = in.imm;
        const bool fl = P_.ctag[k] == TAG_FLOAT;
        if (P_.is_lit[k]) {
          MI ld = mk(DS_READ_B64, R(d), v(29));
          ld.imm = 8 * (1 + k);
          e(ld);   // waited for at the first use (e())
        } else {
          uint64_t bits;
          if (fl) std::memcpy(&bits, &P_.fconst[k], 8);
          else bits = (uint64_t)P_.iconst[k];
          vmov32(R(d), (uint32_t)bits);
          vmov32(Rh(d), (uint32_t)(bits >> 32));
        }
        set_tag_static(d, fl);
        break;
      }
      case OP_MOV: case OP_POS:
        if (pend_ >> a & 1) {          // a bool still in its mask: d shares it
          bm_of_[d] = bm_of_[a];
          pend_ |= 1ull << d;
          set_tag_static(d, false);
          break;
        }
        if (R(d) != R(a)) e(mk(V_MOV_B64, R(d), R(a)));
        copy_tag(d, a, ta);
        bm_of_[d] = bm_of_[a];
        break;
      case OP_POD: {   // from the (per-lane) argument VGPRs, kept intact
        const int f = (in.imm >= 0 && in.imm <= 5) ? in.imm : 5;
        const int a = pod_s_[f];
        switch (f) {
          case 0: case 1: case 5:
            e(mk(V_MOV_B32, R(d), v(a)));
            e(mk(V_ASHRREV_I32, Rh(d), ic(31), v(a)));
            break;
          case 2:
            e(mk(V_LSHRREV_B32, R(d), ic(16), v(a)));
            e(mk(V_MOV_B32, Rh(d), ic(0)));
            break;
          case 3:
            e(mklit(V_AND_B32, R(d), 0xFFFFu, v(a)));
            e(mk(V_MOV_B32, Rh(d), ic(0)));
            break;
          default:
            e(mk(V_MOV_B64, R(d), v(a)));
            break;
        }
        set_tag_static(d, false);
        break;
      }
      case OP_NODE: {
        const int f = (in.imm >= 0 && in.imm <= 5) ? in.imm : 5;
        if (f <= 3) {
          e(mk(V_MOV_B32, R(d), v(f)));
          e(mk(V_ASHRREV_I32, Rh(d), ic(31), v(f)));
        } else if (f == 4) {
          e(mk(V_BFE_I32, R(d), v(4), ic(0), ic(16)));
          e(mk(V_ASHRREV_I32, Rh(d), ic(31), R(d)));
        } else {
          e(mk(V_LSHRREV_B32, R(d), ic(16), v(4)));
          e(mk(V_MOV_B32, Rh(d), ic(0)));
        }
        set_tag_static(d, false);
        break;
      }
      case OP_GPU: emit_gpu(in, ta, (uni_in_[pc] >> a & 1) != 0); break;
      case OP_GLIST_ALL:
        e(mk(V_LSHRREV_B32, T(1), ic(16), v(4)));                 // n
        e(mk(V_LSHLREV_B32, Th(1), ic(2), T(1)));                 // 4n
        e(mk(V_LSHLREV_B64, T(0), Th(1), ic(1)));                 // 1 << 4n (64-bit)
        e(mk(V_LSHL_ADD_U64, T(0), T(0), ic(0), ic(-1)));         // - 1
        e(mklit(V_AND_B32, T(0), 0x76543210u, T(0)));
        e(mk(V_LSHLREV_B32, R(d), ic(4), T(0)));
        e(mk(V_OR_B32, R(d), R(d), T(1)));
        e(mk(V_LSHRREV_B32, Rh(d), ic(28), T(0)));
        set_tag_static(d, false);
        break;
      case OP_GLIST_LEN:
        if (all_in_[pc] >> a & 1) e(mk(V_LSHRREV_B32, R(d), ic(16), v(4)));   // len(node.gpus): the GPU count
        else e(mk(V_AND_B32, R(d), ic(15), R(a)));
        e(mk(V_MOV_B32, Rh(d), ic(0)));
        set_tag_static(d, false);
        break;
      case OP_GLIST_GET:
        if (in.imm == kLoopIndex && tb == TY_I) {
          // the compiler's loop counter: 0 <= b < len(a), no checks
          if (all_in_[pc] >> a & 1) {   // node.gpus: element b is GPU b
            if (R(d) != R(b)) e(mk(V_MOV_B64, R(d), R(b)));
          } else {
            e(mk(V_LSHLREV_B32, Th(1), ic(2), R(b)));
            e(mk(V_ADD_U32, Th(1), ic(4), Th(1)));
            e(mk(V_LSHRREV_B64, T(2), Th(1), R(a)));
            e(mk(V_AND_B32, R(d), ic(15), T(2)));
            e(mk(V_MOV_B32, Rh(d), ic(0)));
          }
          set_tag_static(d, false);
          break;
        }
        if (tb == TY_I && kval(b) >= 0 && (all_in_[pc] >> a & 1)) {
          // node.gpus[k], k a small constant: GPU k where k < len, else IndexError
          e(mk(V_LSHRREV_B32, Th(1), ic(16), v(4)));
          cmp(V_CMP_GE_U32, ST(0), ic(kval(b)), Th(1));
          soft_raise(ST(0), EXC_INDEX);
          e(mk(V_MOV_B64, R(d), ic(kval(b))));
          set_tag_static(d, false);
          break;
        }
        emit_glist_get(in, tb);
        break;
      case OP_GLIST_SLICE: emit_glist_slice(in, st); break;
      case OP_GLIST_NEW:
        e(mk(V_MOV_B64, R(d), ic(0)));
        set_tag_static(d, false);
        break;
      case OP_GLIST_APPEND: emit_glist_append(in); break;
      case OP_GLIST_INSERT: emit_glist_insert(in, st); break;
      case OP_ADD: case OP_SUB: case OP_MUL:
        if (in.op == OP_ADD && in.imm == kLoopIndex && ta == TY_I && tb == TY_I) {
          // loop counter step: counter + 1 <= 15, no overflow; the high half stays 0
          e(mk(V_ADD_U32, R(d), R(a), R(b)));
          if (R(d) != R(a)) e(mk(V_MOV_B32, Rh(d), ic(0)));
          set_tag_static(d, false);
          break;
        }
        if (ta == TY_IF || tb == TY_IF) { rtcall(0, in.op, pc, d, a, ta, b, tb); break; }
        if (ta == TY_I && tb == TY_I) { emit_int_arith(in); break; }
        {
          const uint16_t fa = as_f64(a, ta, 0), fb = as_f64(b, tb, 1);
          MI m = mk(in.op == OP_MUL ? V_MUL_F64 : V_ADD_F64, R(d), fa, fb);
          if (in.op == OP_SUB) m.neg = 2;
          e(m);
          set_tag_static(d, true);
        }
        break;
      case OP_TDIV:
        if (ta == TY_IF || tb == TY_IF) { rtcall(0, in.op, pc, d, a, ta, b, tb); break; }
        if (ta == TY_I && tb == TY_I) {
          if (!nonzero(b)) {
            cmp(V_CMP_EQ_I64, ST(0), ic(0), R(b));
            soft_raise(ST(0), EXC_ZERO_DIVISION);
          }
          if (!exact(a)) check_exact_int(R(a), EXEC);
          if (!exact(b)) check_exact_int(R(b), EXEC);
        }
        {
          const uint16_t fa = as_f64(a, ta, 0), fb = as_f64(b, tb, 1);
          if (!(ta == TY_I && tb == TY_I) && !nonzero(b)) {
            cmp(V_CMP_EQ_F64, ST(0), ic(0), fb);
            soft_raise(ST(0), EXC_ZERO_DIVISION);
          }
          e(mk(M_FDIV64, R(d), fa, fb));
          set_tag_static(d, true);
        }
        break;
      case OP_FDIV: case OP_MOD:
        if (ta == TY_I && tb == TY_I) { emit_int_divmod(in); break; }
        rtcall(0, in.op, pc, d, a, ta, b, tb);
        break;
      case OP_POW: case OP_LOGB: case OP_MPOW:
        if (in.op == OP_POW && ta == TY_F && tb == TY_I && in.imm >= 1 && in.imm <= 3) {
          emit_small_pow(in, pc);
          break;
        }
        rtcall(0, in.op, pc, d, a, ta, b, tb);
        break;
      case OP_SQRT: case OP_LOG: case OP_EXP: case OP_SIN: case OP_COS: case OP_TAN:
        rtcall(1, in.op, pc, d, a, ta);
        break;
      case OP_NEG: case OP_ABS:
        if (ta == TY_IF) { rtcall(1, in.op, pc, d, a, ta); break; }
        if (ta == TY_F) {
          if (R(d) != R(a)) e(mk(V_MOV_B32, R(d), R(a)));
          if (in.op == OP_NEG) e(mklit(V_XOR_B32, Rh(d), 0x80000000u, Rh(a)));
          else e(mklit(V_AND_B32, Rh(d), 0x7FFFFFFFu, Rh(a)));
          set_tag_static(d, true);
        } else {
          movk64(s(S_LIT_), 0x8000000000000000ull);
          cmp(V_CMP_EQ_I64, ST(0), R(a), s(S_LIT_));
          soft_raise(ST(0), EXC_UNSUPPORTED);
          MI lo = mk(V_SUB_CO_U32, T(0), ic(0), R(a)); lo.sd = ST(0); e(lo);
          MI hi = mk(V_SUBB_CO_U32, Th(0), ic(0), Rh(a), ST(0)); hi.sd = ST(0); e(hi);
          if (in.op == OP_NEG) {
            e(mk(V_MOV_B64, R(d), T(0)));
          } else {
            cmp(V_CMP_LT_I32, ST(1), Rh(a), ic(0));
            e(mk(V_CNDMASK_B32, R(d), R(a), T(0), ST(1)));
            e(mk(V_CNDMASK_B32, Rh(d), Rh(a), Th(0), ST(1)));
          }
          set_tag_static(d, false);
        }
        break;
      case OP_INT: case OP_ROUND:
        if (ta == TY_IF) { rtcall(1, in.op, pc, d, a, ta); break; }
        if (ta == TY_I) {
          if (R(d) != R(a)) e(mk(V_MOV_B64, R(d), R(a)));
          set_tag_static(d, false);
          break;
        }
        {
          uint16_t x = R(a);
          if (in.op == OP_ROUND) { e(mk(V_RNDNE_F64, T(1), R(a))); x = T(1); }
          cmp(V_CMP_CLASS_F64, ST(0), x, ic(3));
          soft_raise(ST(0), EXC_VALUE);
          e(mklit(S_MOV_B32, s(S_LIT_), 0x204u));
          cmp(V_CMP_CLASS_F64, ST(0), x, s(S_LIT_));
          soft_raise(ST(0), EXC_OVERFLOW);
          e(mk(V_TRUNC_F64, T(0), x));
          movk64(s(S_LIT_), 0x43E0000000000000ull);
          cmp(V_CMP_GE_F64, ST(0), T(0), s(S_LIT_), 1);
          soft_raise(ST(0), EXC_UNSUPPORTED);
          e(mk(M_CVT_I64_F64, R(d), T(0)));
          set_tag_static(d, false);
        }
        break;
      case OP_FLOAT: {
        const uint16_t f = as_f64(a, ta, 0);
        if (f != R(d)) e(mk(V_MOV_B64, R(d), f));
        set_tag_static(d, true);
        break;
      }
      case OP_NOT: case OP_TRUTH: {
        if (in.op == OP_TRUTH && bm_of_[a] >= 0) {   // truth of a bool: the same bool
          if (pend_ >> a & 1) {
            pend_ |= 1ull << d;
          } else {
            pend_ &= ~(1ull << d);
            if (R(d) != R(a)) e(mk(V_MOV_B64, R(d), R(a)));
          }
          bm_of_[d] = bm_of_[a];
          set_tag_static(d, false);
          break;
        }
        const uint16_t m = truth(a, ta, ST(0));
        if (in.op == OP_NOT) {
          // (the operand's own slot may be the one d takes: read before written)
          const uint16_t slot = bool_slot(d);
          e(mk(S_ANDN2_B64, slot, EXEC, m));
          commit_bool(d);
        } else {
          set_bool(d, m);
        }
        break;
      }
      case OP_ISINT:
        if (ta == TY_IF) {
          tag_mask(a, ST(0));
          e(mk(S_ANDN2_B64, ST(0), EXEC, ST(0)));
          set_bool(d, ST(0));
        } else {
          e(mk(V_MOV_B64, R(d), ic(ta == TY_I ? 1 : 0)));
          set_tag_static(d, false);
        }
        break;
      case OP_LT: case OP_LE: case OP_GT: case OP_GE: case OP_EQ: case OP_NE: {
        const uint16_t slot = bool_slot(d);   // the compare writes d's mask slot itself
        if (in.op == OP_LT && in.imm == kLoopIndex && ta == TY_I && tb == TY_I)
          cmp(V_CMP_LT_I32, slot, R(a), R(b));   // counter < length, both in [0, 15]
        else
          emit_compare(in.op, a, ta, b, tb, slot);
        commit_bool(d);
        break;
      }
      case OP_MIN2: case OP_MAX2: emit_minmax(in, ta, tb); break;
      // ---- control flow
      case OP_IF: {
        const int t = in.imm;
        if (t <= pc || t >= n_) throw CodegenError("bad IF target");
        if (static_if_[pc] >= 0) {
          // a known condition: no mask, no branch; the dead branch is not emitted
          const bool has_else = P_.code[t].op == OP_ELSE;
          if (!static_if_[pc] && !has_else) {   // never taken: nothing at all
            skip_to_ = t + 1;
            break;
          }
          Frame fr{};
          fr.loop = false;
          fr.pc = pc;
          fr.s_save = take_spair();            // (the ENDIF still drops lanes that left inside)
          fr.static_branch = true;
          e(mk(S_MOV_B64, s(fr.s_save), EXEC));
          frames_.push_back(fr);
          if (!static_if_[pc]) skip_to_ = t + 1;   // straight to the else-branch
          break;
        }
        Frame fr{};
        fr.loop = false;
        fr.pc = pc;
        fr.s_save = take_spair();
        if (P_.code[t].op == OP_ELSE) {
          fr.s_else = take_spair();
          e(mk(S_ANDN2_B64, s(fr.s_else), EXEC, mask_a));
        } else if (P_.code[t].op != OP_ENDIF) {
          throw CodegenError("IF target is neither ELSE nor ENDIF");
        }
        e(mk(S_AND_SAVEEXEC_B64, s(fr.s_save), mask_a));
        e(mkimm(S_CBRANCH_EXECZ, label_for_pc(t)));
        frames_.push_back(fr);
        break;
      }
      case OP_ELSE: {
        if (!frames_.empty() && !frames_.back().loop && frames_.back().static_branch) {
          skip_to_ = in.imm;   // end of an always-taken then-branch: the else-branch is dead
          break;
        }
        if (frames_.empty() || frames_.back().loop || frames_.back().s_else < 0) throw CodegenError("stray ELSE");
        place(label_for_pc(pc));
        e(mk(S_MOV_B64, EXEC, s(frames_.back().s_else)));
        e(mkimm(S_CBRANCH_EXECZ, label_for_pc(in.imm)));
        break;
      }
      case OP_ENDIF: {
        if (frames_.empty() || frames_.back().loop) throw CodegenError("stray ENDIF");
        place(label_for_pc(pc));
        Frame fr = frames_.back();
        frames_.pop_back();
        restore_exec(s(fr.s_save));
        give_spair(fr.s_save);
        if (fr.s_else >= 0) give_spair(fr.s_else);
        break;
      }
      case OP_LOOP_BEGIN: {
        Frame fr{};
        fr.loop = true;
        fr.pc = pc;
        fr.s_entry = take_spair();
        // break / continue masks only for loops that break / continue (the
        // others skip their upkeep at every ENDIF and LOOP_CONT)
        bool brk = false, cont = false;
        {
          int depth = 0, q = pc + 1;
          std::set<int> conts;
          for (; q < n_; ++q) {
            const uint8_t o = P_.code[q].op;
            if (o == OP_LOOP_BEGIN) ++depth;
            else if (o == OP_LOOP_EXIT) { if (depth == 0) break; --depth; }
            else if (o == OP_LOOP_CONT && depth == 0) conts.insert(q);
          }
          for (int r = pc + 1; r < q; ++r) {
            if (P_.code[r].op == OP_BREAK && brk_t_[(size_t)r] == q) brk = true;
            if (P_.code[r].op == OP_CONTINUE && conts.count(cont_t_[(size_t)r])) cont = true;
          }
        }
        e(mk(S_MOV_B64, s(fr.s_entry), EXEC));
        if (brk) {
          fr.s_brk = take_spair();
          e(mk(S_MOV_B64, s(fr.s_brk), ic(0)));
        }
        if (cont) {
          fr.s_cont = take_spair();
          e(mk(S_MOV_B64, s(fr.s_cont), ic(0)));
        }
        fr.l_head = label();
        place(fr.l_head);
        frames_.push_back(fr);
        break;
      }
      case OP_LOOP_TEST: {
        Frame* l = innermost_loop();
        if (!l || frames_.back().pc != l->pc) throw CodegenError("LOOP_TEST not at loop level");
        e(mk(S_AND_B64, EXEC, EXEC, mask_a));
        e(mkimm(S_CBRANCH_EXECZ, label_for_pc(in.imm)));
        break;
      }
      case OP_LOOP_CONT: {
        Frame* l = innermost_loop();
        if (!l || frames_.back().pc != l->pc) throw CodegenError("LOOP_CONT not at loop level");
        if (l->s_cont >= 0) {
          e(mk(S_OR_B64, EXEC, EXEC, s(l->s_cont)));
          e(mk(S_MOV_B64, s(l->s_cont), ic(0)));
        }
        break;
      }
      case OP_LOOP_NEXT: {
        Frame* l = innermost_loop();
        if (!l || frames_.back().pc != l->pc) throw CodegenError("LOOP_NEXT not at loop level");
        if (in.imm != l->pc + 1) throw CodegenError("loop back edge not to the loop head");
        {   // budget: s_bud -= 1; on a borrow every lane still looping raises BUDGET,
          // and the counter stays exhausted (0: the next back edge borrows again),
          // so lanes outside EXEC here -- done with this loop, in another branch or
          // an outer loop -- raise at their next back edge instead of continuing
          // with a wrapped ~2^32 budget (kJitLoopCap is what value_facts relies on)
          e(mk(S_SUB_U32, s(s_bud_), s(s_bud_), ic(1)));
          const int ok = label();
          e(mkimm(S_CBRANCH_SCC0, ok));
          soft_raise(EXEC, EXC_BUDGET);
          e(mk(S_MOV_B32, s(s_bud_), ic(0)));
          place(ok);
        }
        e(mkimm(S_CBRANCH_EXECNZ, l->l_head));   // (lanes that raised in the body left EXEC already)
        if (pc + 1 >= n_ || P_.code[pc + 1].op != OP_LOOP_EXIT) e(mkimm(S_BRANCH, label_for_pc(l_exit_of(pc))));
        break;
      }
      case OP_LOOP_EXIT: {
        if (frames_.empty() || !frames_.back().loop) throw CodegenError("stray LOOP_EXIT");
        place(label_for_pc(pc));
        Frame fr = frames_.back();
        frames_.pop_back();
        e(mk(S_ANDN2_B64, EXEC, s(fr.s_entry), s(s_dead_)));
        give_spair(fr.s_entry);
        if (fr.s_brk >= 0) give_spair(fr.s_brk);
        if (fr.s_cont >= 0) give_spair(fr.s_cont);
        break;
      }
      case OP_BREAK: {
        Frame* l = innermost_loop();
        if (!l || l->s_brk < 0) throw CodegenError("internal: BREAK of a loop without a break mask");
        e(mk(S_OR_B64, s(l->s_brk), s(l->s_brk), EXEC));
        e(mk(S_MOV_B64, EXEC, ic(0)));
        break;
      }
      case OP_CONTINUE: {
        Frame* l = innermost_loop();
        if (!l || l->s_cont < 0) throw CodegenError("internal: CONTINUE of a loop without a continue mask");
        e(mk(S_OR_B64, s(l->s_cont), s(l->s_cont), EXEC));
        e(mk(S_MOV_B64, EXEC, ic(0)));
        break;
      }
      case OP_RET:
        emit_finish(a, ta);
        leave_function();
        break;
      case OP_RAISE:
        soft_raise(EXEC, in.imm);
        leave_function();
        break;
      case OP_END:
        soft_raise(EXEC, EXC_TYPE);
        leave_function();
        break;
      default:
        throw CodegenError("opcode " + std::to_string((int)in.op) + " has no baseline lowering");
    }
  }
  static bool structural(uint8_t op) {
    return op == OP_IF || op == OP_ELSE || op == OP_ENDIF || op == OP_LOOP_BEGIN || op == OP_LOOP_TEST ||
           op == OP_LOOP_CONT || op == OP_LOOP_NEXT || op == OP_LOOP_EXIT;
  }

  int l_exit_of(int pc_next) const {
    // the LOOP_EXIT that closes the loop whose LOOP_NEXT is at pc_next
    int depth = 0;
    for (int q = pc_next + 1; q < n_; ++q) {
      if (P_.code[q].op == OP_LOOP_BEGIN) ++depth;
      if (P_.code[q].op == OP_LOOP_EXIT) {
        if (depth == 0) return q;
        --depth;
      }
    }
    throw CodegenError("loop without LOOP_EXIT");
  }

  // ---- int64 add / sub / mul with overflow -> EXC_UNSUPPORTED
  void emit_int_arith(const Insn& in) {
    const int d = in.d, a = in.a, b = in.b;
    const bool no_ovf = no_int_overflow(in.op, a, b);
    if (no_ovf) {   // |a|, |b| < 2^31, or an accumulator plus an int32: no int64 overflow
      if (in.op == OP_MUL) {
        e(mk3b(V_MAD_I64_I32, R(d), VCC, opi(a), opi(b), ic(0)));
      } else {
        MI lo = mk(in.op == OP_ADD ? V_ADD_CO_U32 : V_SUB_CO_U32, R(d), opi(a), opi(b));
        lo.sd = ST(0);
        e(lo);
        MI hi = mk(in.op == OP_ADD ? V_ADDC_CO_U32 : V_SUBB_CO_U32, Rh(d), opih(a), opih(b), ST(0));
        hi.sd = ST(0);
        e(hi);
      }
      set_tag_static(d, false);
      return;
    }
    if (in.op == OP_MUL) {
      // operands in int32 range multiply exactly with v_mad_i64_i32; anything
      // wider is left to the next engine (EXC_UNSUPPORTED)
      e(mk(V_ASHRREV_I32, T(1), ic(31), R(a)));
      cmp(V_CMP_EQ_U32, ST(0), T(1), Rh(a));
      e(mk(V_ASHRREV_I32, Th(1), ic(31), R(b)));
      cmp(V_CMP_EQ_U32, ST(1), Th(1), Rh(b));
      e(mk(S_AND_B64, ST(0), ST(0), ST(1)));
      e(mk(S_ANDN2_B64, ST(1), EXEC, ST(0)));
      soft_raise(ST(1), EXC_UNSUPPORTED);
      e(mk3b(V_MAD_I64_I32, R(d), VCC, R(a), R(b), ic(0)));
      set_tag_static(d, false);
      return;
    }
    MI lo = mk(in.op == OP_ADD ? V_ADD_CO_U32 : V_SUB_CO_U32, T(0), R(a), R(b));
    lo.sd = ST(0);
    e(lo);
    MI hi = mk(in.op == OP_ADD ? V_ADDC_CO_U32 : V_SUBB_CO_U32, Th(0), Rh(a), Rh(b), ST(0));
    hi.sd = ST(0);
    e(hi);
    if (in.op == OP_ADD) {
      e(mk(V_XOR_B32, T(1), Rh(a), Th(0)));
      e(mk(V_XOR_B32, Th(1), Rh(b), Th(0)));
    } else {
      e(mk(V_XOR_B32, T(1), Rh(a), Rh(b)));
      e(mk(V_XOR_B32, Th(1), Rh(a), Th(0)));
    }
    e(mk(V_AND_B32, T(1), T(1), Th(1)));
    cmp(V_CMP_LT_I32, ST(1), T(1), ic(0));
    soft_raise(ST(1), EXC_UNSUPPORTED);
    e(mk(V_MOV_B64, R(d), T(0)));
    set_tag_static(d, false);
  }

  // ---- int // int and int % int (CPython floor semantics), exact for
  // |a|, |b| <= 2^53: q0 = floor(fl(a / b)) is the true floor or one above it
  // (a / b can round up onto the next integer, never below its floor), and
  // r = a - q0 * b, corrected once when r and b differ in sign.  Wider
  // operands -> EXC_UNSUPPORTED (the next engine decides).
  void emit_int_divmod(const Insn& in) {
    const int d = in.d, a = in.a, b = in.b;
    if (!nonzero(b)) {
      cmp(V_CMP_EQ_I64, ST(0), ic(0), R(b));
      soft_raise(ST(0), EXC_ZERO_DIVISION);
    }
    if (!exact(a)) check_exact_int(R(a), EXEC);
    if (!exact(b)) check_exact_int(R(b), EXEC);
    const uint16_t fa = as_f64(a, TY_I, 0), fb = as_f64(b, TY_I, 1);
    e(mk(M_FDIV64, T(2), fa, fb));
    e(mk(V_FLOOR_F64, T(2), T(2)));
    e(mk(M_CVT_I64_F64, T(2), T(2)));                                   // q0
    // q0 * b (low 64 bits; |q0 * b| < 2^54)
    e(mk3b(V_MAD_U64_U32, X(0), VCC, T(2), R(b), ic(0)));
    e(mk(V_MUL_LO_U32, X(1), Th(2), R(b)));
    e(mk(V_MUL_LO_U32, (uint16_t)(X(1) + 1), T(2), Rh(b)));
    e(mk(V_ADD_U32, (uint16_t)(X(0) + 1), (uint16_t)(X(0) + 1), X(1)));
    e(mk(V_ADD_U32, (uint16_t)(X(0) + 1), (uint16_t)(X(0) + 1), (uint16_t)(X(1) + 1)));
    // r = a - q0 b
    MI lo = mk(V_SUB_CO_U32, X(1), R(a), X(0)); lo.sd = ST(0); e(lo);
    MI hi = mk(V_SUBB_CO_U32, (uint16_t)(X(1) + 1), Rh(a), (uint16_t)(X(0) + 1), ST(0)); hi.sd = ST(0); e(hi);
    // fix = r != 0 && sign(r) != sign(b)
    cmp(V_CMP_NE_I64, ST(0), ic(0), X(1));
    e(mk(V_XOR_B32, X(2), (uint16_t)(X(1) + 1), Rh(b)));
    cmp(V_CMP_LT_I32, ST(1), X(2), ic(0));
    e(mk(S_AND_B64, ST(0), ST(0), ST(1)));
    if (in.op == OP_FDIV) {
      e(mk(V_LSHL_ADD_U64, X(2), T(2), ic(0), ic(-1)));                 // q0 - 1
      e(mk(V_CNDMASK_B32, R(d), T(2), X(2), ST(0)));
      e(mk(V_CNDMASK_B32, Rh(d), Th(2), (uint16_t)(X(2) + 1), ST(0)));
    } else {
      e(mk(V_LSHL_ADD_U64, X(2), X(1), ic(0), R(b)));                   // r + b
      e(mk(V_CNDMASK_B32, R(d), X(1), X(2), ST(0)));
      e(mk(V_CNDMASK_B32, Rh(d), (uint16_t)(X(1) + 1), (uint16_t)(X(2) + 1), ST(0)));
    }
    set_tag_static(d, false);
  }

  // ---- float ** k for a literal k in {1, 2, 3} (bytecode POW imm = k):
  // glibc's pow is within 0.52 ULP of the exact power, so where the exact
  // value x**k (as hi + residual, error-free products) lies within 0.4375 ULP
  // of hi = fl(x**k) -- every neighbour of hi is then over 0.56 ULP away --
  // pow returns hi.  hi must be normal, not a power of two (an exact value
  // just below one sits in the finer binade) and well above the underflow
  // range (exact error terms).  Other lanes call the runtime pow as before.
  void small_pow_mask(int k, uint16_t x, uint16_t mask) {
    // mask = lanes whose x ** k is hi (hi into T(0), residual into T(1))
    auto normal_far = [&](uint16_t h, uint16_t out) {
      e(mklit(S_MOV_B32, s(S_LIT_), 0x108u));                      // -normal | +normal
      cmp(V_CMP_CLASS_F64, out, h, s(S_LIT_));
      e(mk(V_BFE_U32, Th(2), (uint16_t)(h + 1), ic(20), ic(11)));    // biased exponent
      e(mklit(S_MOV_B32, s(S_LIT_), 123u));
      cmp(V_CMP_GT_U32, ST(2), Th(2), s(S_LIT_));
      e(mk(S_AND_B64, out, out, ST(2)));
    };
    if (k == 1) {
      normal_far(x, mask);
      e(mklit(V_AND_B32, T(2), 0xFFFFFu, (uint16_t)(x + 1)));
      e(mk(V_OR_B32, T(2), T(2), x));
      cmp(V_CMP_NE_U32, ST(1), ic(0), T(2));
      e(mk(S_AND_B64, mask, mask, ST(1)));
      return;
    }
    e(mk(V_MUL_F64, T(0), x, x));                                    // h2
    if (k == 2) {
      MI f = mk(V_FMA_F64, T(1), x, x, T(0)); f.neg = 4; e(f);      // x*x - h2 (exact)
    } else {
      normal_far(T(0), mask);                                        // h2 normal, far from underflow
      MI f = mk(V_FMA_F64, T(1), x, x, T(0)); f.neg = 4; e(f);      // l2
      e(mk(V_MUL_F64, T(2), T(0), x));                               // h3
      MI g = mk(V_FMA_F64, T(0), T(0), x, T(2)); g.neg = 4; e(g);   // e3 = h2*x - h3 (exact)
      e(mk(V_FMA_F64, T(1), T(1), x, T(0)));                         // residual = l2*x + e3
      e(mk(V_MOV_B64, T(0), T(2)));                                  // hi = h3
    }
    normal_far(T(0), k == 2 ? mask : ST(1));
    if (k == 3) e(mk(S_AND_B64, mask, mask, ST(1)));
    // hi's mantissa nonzero
    e(mklit(V_AND_B32, T(2), 0xFFFFFu, Th(0)));
    e(mk(V_OR_B32, T(2), T(2), T(0)));
    cmp(V_CMP_NE_U32, ST(1), ic(0), T(2));
    e(mk(S_AND_B64, mask, mask, ST(1)));
    // |residual| <= 1.75 * 2^(eb - 1077) = 0.4375 ulp(hi): bits ((eb - 54) << 20 | 0xC0000, 0)
    e(mk(V_BFE_U32, Th(2), Th(0), ic(20), ic(11)));
    e(mk(V_LSHLREV_B32, Th(2), ic(20), Th(2)));
    e(mklit(V_ADD_U32, Th(2), (uint32_t)(0xC0000 - (54 << 20)), Th(2)));
    e(mk(V_MOV_B32, T(2), ic(0)));
    cmp(V_CMP_LE_F64, ST(1), T(1), T(2), 1);
    e(mk(S_AND_B64, mask, mask, ST(1)));
  }
  void emit_small_pow(const Insn& in, int pc) {
    const int d = in.d, a = in.a, b = in.b, k = in.imm;
    materialize_live(slive_out_[pc] | live_out_[pc]);   // both paths of the branch below see the same state
    const int P = take_spair(), Q = take_spair();
    held_spairs_ = {P, Q};
    small_pow_mask(k, R(a), s(P));
    // the other lanes: the runtime pow (inactive lanes' registers survive the call)
    e(mk(S_ANDN2_B64, ST(0), EXEC, s(P)));
    e(mk(S_AND_SAVEEXEC_B64, s(Q), ST(0)));
    const int skip = label();
    e(mkimm(S_CBRANCH_EXECZ, skip));
    rtcall(0, OP_POW, pc, d, a, TY_F, b, TY_I);
    place(skip);
    e(mk(S_ANDN2_B64, EXEC, s(Q), s(s_dead_)));   // lanes the runtime pow raised in stay out
    held_spairs_.clear();
    // fast lanes: hi (recomputed from x, which those lanes kept)
    uint16_t hi = R(a);
    if (k >= 2) {
      e(mk(V_MUL_F64, T(0), R(a), R(a)));
      if (k == 3) e(mk(V_MUL_F64, T(0), T(0), R(a)));
      hi = T(0);
    }
    e(mk(V_CNDMASK_B32, R(d), R(d), hi, s(P)));
    e(mk(V_CNDMASK_B32, Rh(d), Rh(d), (uint16_t)(hi + 1), s(P)));
    set_tag_static(d, true);
    give_spair(Q);
    give_spair(P);
  }

  // ---- node.gpus[j].field
  void emit_gpu(const Insn& in, uint8_t ta, bool uniform) {
    (void)ta;
    const int d = in.d, a = in.a;
    if ((in.imm == 0 || in.imm == 1) && kval(a) >= 0 && kval(a) < 8) {   // a constant GPU index
      e(mk(V_MOV_B32, R(d), v((in.imm == 0 ? 5 : 13) + kval(a))));
      e(mk(V_ASHRREV_I32, Rh(d), ic(31), R(d)));
      set_tag_static(d, false);
      return;
    }
    if (uniform && (in.imm == 0 || in.imm == 1)) {
      // j is the same in every active lane: one indexed move (GPR index mode)
      // instead of a 3-level v_cndmask tree; j & 7 keeps an empty-exec read in range
      const int base = in.imm == 0 ? 5 : 13;
      e(mk(V_READFIRSTLANE_B32, s(S_LIT_), R(a)));
      e(mk(S_AND_B32, s(S_LIT_), s(S_LIT_), ic(7)));
      MI on = mk(S_SET_GPR_IDX_ON, NONE, s(S_LIT_));
      on.s1 = 1;   // the mode field: index SRC0
      e(on);
      e(mkimm(S_NOP, 0));
      e(mk(V_MOV_B32, R(d), v(base)));
      e(mkimm(S_SET_GPR_IDX_OFF, 0));
      e(mk(V_ASHRREV_I32, Rh(d), ic(31), R(d)));
      set_tag_static(d, false);
      return;
    }
    e(mk(V_AND_B32, T(1), ic(15), R(a)));   // j
    if (in.imm == 0 || in.imm == 1) {
      const int base = in.imm == 0 ? 5 : 13;
      // select by the bits of j: 3 levels of v_cndmask
      e(mk(V_AND_B32, Th(1), ic(1), T(1)));
      cmp(V_CMP_NE_U32, ST(0), ic(0), Th(1));
      e(mk(V_AND_B32, Th(1), ic(2), T(1)));
      cmp(V_CMP_NE_U32, ST(1), ic(0), Th(1));
      e(mk(V_AND_B32, Th(1), ic(4), T(1)));
      cmp(V_CMP_NE_U32, ST(2), ic(0), Th(1));
      e(mk(V_CNDMASK_B32, T(0), v(base + 0), v(base + 1), ST(0)));
      e(mk(V_CNDMASK_B32, Th(0), v(base + 2), v(base + 3), ST(0)));
      e(mk(V_CNDMASK_B32, T(2), v(base + 4), v(base + 5), ST(0)));
      e(mk(V_CNDMASK_B32, Th(2), v(base + 6), v(base + 7), ST(0)));
      e(mk(V_CNDMASK_B32, T(0), T(0), Th(0), ST(1)));
      e(mk(V_CNDMASK_B32, T(2), T(2), Th(2), ST(1)));
      e(mk(V_CNDMASK_B32, R(d), T(0), T(2), ST(2)));
      e(mk(V_ASHRREV_I32, Rh(d), ic(31), R(d)));
    } else {
      // gmem[j]: 64-bit load from the node's row (v[21:22], 8 entries)
      e(mk(V_LSHLREV_B32, Th(1), ic(3), T(1)));
      MI lo = mk(V_ADD_CO_U32, T(0), v(21), Th(1)); lo.sd = ST(0); e(lo);
      MI hi = mk(V_ADDC_CO_U32, Th(0), v(22), ic(0), ST(0)); hi.sd = ST(0); e(hi);
      e(mk(GLOBAL_LOAD_DWORDX2, R(d), T(0)));
      e(mkimm(S_WAITCNT, 0x0F70));
    }
    set_tag_static(d, false);
  }

  // ---- GPU lists (int64: bits 0-3 length, 4 bits per entry)
  void emit_glist_get(const Insn& in, uint8_t tb) {
    const int d = in.d, a = in.a, b = in.b;
    // float index -> TypeError
    if (tb == TY_F) soft_raise(EXEC, EXC_TYPE);
    else if (tb == TY_IF) { tag_mask(b, ST(0)); soft_raise(ST(0), EXC_TYPE); }
    e(mk(V_AND_B32, T(1), ic(15), R(a)));                    // n
    e(mk(V_MOV_B32, Th(1), ic(0)));
    // k = i < 0 ? i + n : i
    e(mk(V_LSHL_ADD_U64, T(0), R(b), ic(0), T(1)));
    cmp(V_CMP_LT_I64, ST(0), R(b), ic(0));
    e(mk(V_CNDMASK_B32, T(0), R(b), T(0), ST(0)));
    e(mk(V_CNDMASK_B32, Th(0), Rh(b), Th(0), ST(0)));
    // k < 0 || k >= n -> IndexError
    cmp(V_CMP_LT_I64, ST(0), T(0), ic(0));
    cmp(V_CMP_GE_I64, ST(1), T(0), T(1));
    e(mk(S_OR_B64, ST(0), ST(0), ST(1)));
    soft_raise(ST(0), EXC_INDEX);   // a lane that raised TypeError above keeps it
    // (lst >> (4 + 4k)) & 15
    e(mk(V_LSHLREV_B32, Th(1), ic(2), T(0)));
    e(mk(V_ADD_U32, Th(1), ic(4), Th(1)));
    e(mk(V_LSHRREV_B64, T(2), Th(1), R(a)));
    e(mk(V_AND_B32, R(d), ic(15), T(2)));
    e(mk(V_MOV_B32, Rh(d), ic(0)));
    set_tag_static(d, false);
  }
  // clamp a Python slice / insert position (int64 pair p) into [0, n] (n: VGPR) -> 32-bit VGPR out
  void clamp_pos(uint16_t p, uint16_t nv, uint16_t out, uint16_t tmp_pair) {
    // x < 0: x += n, then max(x, 0); x > n: n
    e(mk(V_MOV_B32, (uint16_t)(tmp_pair + 1), ic(0)));
    e(mk(V_MOV_B32, tmp_pair, nv));
    e(mk(V_LSHL_ADD_U64, tmp_pair, p, ic(0), tmp_pair));       // x + n
    cmp(V_CMP_LT_I64, ST(0), tmp_pair, ic(0));                  // x + n < 0
    cmp(V_CMP_LT_I64, ST(1), p, ic(0));                         // x < 0
    e(mk(V_CNDMASK_B32, out, tmp_pair, ic(0), ST(0)));           // max(x + n, 0)
    e(mk(V_MOV_B32, tmp_pair, nv));
    e(mk(V_MOV_B32, (uint16_t)(tmp_pair + 1), ic(0)));
    cmp(V_CMP_GT_I64, ST(0), p, tmp_pair);                      // x > n
    e(mk(V_CNDMASK_B32, (uint16_t)(tmp_pair + 1), p, nv, ST(0))); // min(x, n) (low word)
    e(mk(V_CNDMASK_B32, out, (uint16_t)(tmp_pair + 1), out, ST(1)));
  }
  void emit_glist_slice(const Insn& in, const std::array<uint8_t, kMaxRegs>& st) {
    const int d = in.d, a = in.a, b = in.b, h = in.imm;
    // float bounds -> TypeError
    for (int r : {b, h}) {
      if (r == kNoReg) continue;
      if (st[r] == TY_F) soft_raise(EXEC, EXC_TYPE);
      else if (st[r] == TY_IF) { tag_mask(r, ST(0)); soft_raise(ST(0), EXC_TYPE); }
    }
    e(mk(V_AND_B32, X(3), ic(15), R(a)));                       // n
    if (b != kNoReg) clamp_pos(R(b), X(3), (uint16_t)(X(3) + 1), T(2));
    else e(mk(V_MOV_B32, (uint16_t)(X(3) + 1), ic(0)));           // lo
    if (h != kNoReg) clamp_pos(R(h), X(3), T(1), T(2));
    else e(mk(V_MOV_B32, T(1), X(3)));                           // hi
    // m = max(hi - lo, 0)
    e(mk(V_SUB_U32, Th(1), T(1), (uint16_t)(X(3) + 1)));
    cmp(V_CMP_LT_I32, ST(0), Th(1), ic(0));
    e(mk(V_CNDMASK_B32, Th(1), Th(1), ic(0), ST(0)));
    // out = (((lst >> (4 + 4 lo)) & ((1 << 4m) - 1)) << 4) | m
    e(mk(V_LSHLREV_B32, T(1), ic(2), (uint16_t)(X(3) + 1)));
    e(mk(V_ADD_U32, T(1), ic(4), T(1)));
    e(mk(V_LSHRREV_B64, T(0), T(1), R(a)));
    e(mk(V_LSHLREV_B32, T(1), ic(2), Th(1)));
    e(mk(V_LSHLREV_B64, T(2), T(1), ic(1)));
    e(mk(V_LSHL_ADD_U64, T(2), T(2), ic(0), ic(-1)));
    e(mk(V_AND_B32, T(0), T(0), T(2)));
    e(mk(V_AND_B32, Th(0), Th(0), Th(2)));
    e(mk(V_LSHLREV_B64, T(0), ic(4), T(0)));
    e(mk(V_OR_B32, R(d), T(0), Th(1)));
    e(mk(V_MOV_B32, Rh(d), Th(0)));
    set_tag_static(d, false);
  }
  void emit_glist_append(const Insn& in) {
    const int d = in.d, a = in.a, b = in.b;
    e(mk(V_AND_B32, T(1), ic(15), R(a)));                       // n
    cmp(V_CMP_GE_U32, ST(0), T(1), ic(15));
    soft_raise(ST(0), EXC_UNSUPPORTED);
    // item & 15 << (4 + 4n)
    e(mk(V_AND_B32, T(2), ic(15), R(b)));
    e(mk(V_MOV_B32, Th(2), ic(0)));
    e(mk(V_LSHLREV_B32, Th(1), ic(2), T(1)));
    e(mk(V_ADD_U32, Th(1), ic(4), Th(1)));
    e(mk(V_LSHLREV_B64, T(2), Th(1), T(2)));
    // (lst & ~15) | (n + 1)
    e(mk(V_ADD_U32, T(1), ic(1), T(1)));
    e(mk(V_AND_B32, T(0), ic(-16), R(a)));
    e(mk(V_OR_B32, T(0), T(0), T(1)));
    e(mk(V_OR_B32, R(d), T(0), T(2)));
    e(mk(V_OR_B32, Rh(d), Rh(a), Th(2)));
    set_tag_static(d, false);
  }
  void emit_glist_insert(const Insn& in, const std::array<uint8_t, kMaxRegs>& st) {
    const int d = in.d, a = in.a, b = in.b, p = in.imm;
    e(mk(V_AND_B32, X(3), ic(15), R(a)));                       // n
    cmp(V_CMP_GE_U32, ST(0), X(3), ic(15));
    soft_raise(ST(0), EXC_UNSUPPORTED);
    if (st[p] == TY_F) soft_raise(EXEC, EXC_TYPE);
    else if (st[p] == TY_IF) { tag_mask(p, ST(0)); soft_raise(ST(0), EXC_TYPE); }
    clamp_pos(R(p), X(3), (uint16_t)(X(3) + 1), T(2));             // pos
    // body = lst >> 4; low = (1 << 4pos) - 1
    e(mk(V_LSHRREV_B64, T(0), ic(4), R(a)));
    e(mk(V_LSHLREV_B32, T(1), ic(2), (uint16_t)(X(3) + 1)));     // 4 pos
    e(mk(V_LSHLREV_B64, T(2), T(1), ic(1)));
    e(mk(V_LSHL_ADD_U64, T(2), T(2), ic(0), ic(-1)));            // low mask
    // nb = (body & low) | (item << 4pos) | ((body & ~low) << 4)
    e(mk(V_NOT_B32, X(2), T(2)));
    e(mk(V_NOT_B32, (uint16_t)(X(2) + 1), Th(2)));
    e(mk(V_AND_B32, X(2), X(2), T(0)));
    e(mk(V_AND_B32, (uint16_t)(X(2) + 1), (uint16_t)(X(2) + 1), Th(0)));
    e(mk(V_LSHLREV_B64, X(2), ic(4), X(2)));                     // (body & ~low) << 4
    e(mk(V_AND_B32, T(0), T(0), T(2)));
    e(mk(V_AND_B32, Th(0), Th(0), Th(2)));                       // body & low
    e(mk(V_OR_B32, T(0), T(0), X(2)));
    e(mk(V_OR_B32, Th(0), Th(0), (uint16_t)(X(2) + 1)));
    e(mk(V_AND_B32, T(2), ic(15), R(b)));
    e(mk(V_MOV_B32, Th(2), ic(0)));
    e(mk(V_LSHLREV_B64, T(2), T(1), T(2)));                      // item << 4pos
    e(mk(V_OR_B32, T(0), T(0), T(2)));
    e(mk(V_OR_B32, Th(0), Th(0), Th(2)));
    // (nb << 4) | (n + 1)
    e(mk(V_LSHLREV_B64, T(0), ic(4), T(0)));
    e(mk(V_ADD_U32, X(3), ic(1), X(3)));
    e(mk(V_OR_B32, R(d), T(0), X(3)));
    e(mk(V_MOV_B32, Rh(d), Th(0)));
    set_tag_static(d, false);
  }

  // ---- comparisons: result mask (lanes where true) in dst
  void emit_compare(uint8_t op, int a, uint8_t ta, int b, uint8_t tb, uint16_t dst) {
    static const Opc ci[6] = {V_CMP_LT_I64, V_CMP_LE_I64, V_CMP_GT_I64, V_CMP_GE_I64, V_CMP_EQ_I64, V_CMP_NE_I64};
    static const Opc cf[6] = {V_CMP_LT_F64, V_CMP_LE_F64, V_CMP_GT_F64, V_CMP_GE_F64, V_CMP_EQ_F64, V_CMP_NEQ_F64};
    const int k = op - OP_LT;
    if (ta == TY_I && tb == TY_I) { cmp(ci[k], dst, opi(a), opi(b)); return; }
    if (ta == TY_F && tb == TY_F) { cmp(cf[k], dst, as_f64(a, ta, 0), as_f64(b, tb, 1)); return; }
    // mixed: int operands within +-2^53 convert exactly; others -> EXC_UNSUPPORTED
    if (ta != TY_F) int_lanes_exact(a, ta);
    if (tb != TY_F) int_lanes_exact(b, tb);
    const uint16_t fa = as_f64(a, ta, 0), fb = as_f64(b, tb, 1);
    if (ta == TY_IF || tb == TY_IF) {
      // lanes where both are ints compare as int64 (exact for any value)
      both_int_mask(a, ta, b, tb, ST(1));
      cmp(cf[k], dst, fa, fb);
      cmp(ci[k], ST(2), R(a), R(b));
      e(mk(S_AND_B64, ST(2), ST(2), ST(1)));
      e(mk(S_ANDN2_B64, dst, dst, ST(1)));
      e(mk(S_OR_B64, dst, dst, ST(2)));
    } else {
      cmp(cf[k], dst, fa, fb);
    }
  }
  // lanes where register r (type t) holds an int outside +-2^53 -> EXC_UNSUPPORTED
  // (conservative for the int / int lanes of a dynamic pair: the next engine decides them)
  void int_lanes_exact(int r, uint8_t t) {
    if (t == TY_I) {
      if (!exact(r) && fold_of(r, true) == NONE) check_exact_int(R(r), EXEC);
      return;
    }
    tag_mask(r, ST(0));
    e(mk(S_ANDN2_B64, ST(0), EXEC, ST(0)));
    check_exact_int(R(r), ST(0));
  }
  void both_int_mask(int a, uint8_t ta, int b, uint8_t tb, uint16_t dst) {
    // dst = lanes where a and b are both ints
    e(mk(S_MOV_B64, dst, EXEC));
    if (ta == TY_F || tb == TY_F) { e(mk(S_MOV_B64, dst, ic(0))); return; }
    if (ta == TY_IF) { tag_mask(a, ST(2)); e(mk(S_ANDN2_B64, dst, dst, ST(2))); }
    if (tb == TY_IF) { tag_mask(b, ST(2)); e(mk(S_ANDN2_B64, dst, dst, ST(2))); }
  }
  void emit_minmax(const Insn& in, uint8_t ta, uint8_t tb) {
    const int d = in.d, a = in.a, b = in.b;
    // max(a, b): b replaces a only if b > a (min: b < a); NaNs never replace
    const uint8_t op = in.op == OP_MAX2 ? OP_GT : OP_LT;
    emit_compare(op, b, tb, a, ta, ST(0));
    // tags first (the value select may overwrite a / b when d aliases them)
    if (tagbit_[d] >= 0) {
      if (ta == tb && ta != TY_IF) set_tag_static(d, ta == TY_F);
      else {
        const uint16_t fa = flag_of(a, ta, X(2)), fb = flag_of(b, tb, (uint16_t)(X(2) + 1));
        e(mk(V_CNDMASK_B32, X(3), fa, fb, ST(0)));
        set_tag_flag(d, X(3));
      }
    }
    e(mk(V_CNDMASK_B32, R(d), R(a), R(b), ST(0)));
    e(mk(V_CNDMASK_B32, Rh(d), Rh(a), Rh(b), ST(0)));
  }

  // ---- return: out = int(max(0, value)) (soft exceptions for inf / >= 2^63)
  void emit_finish(int a, uint8_t ta) {
    auto finish_int = [&](uint16_t lanes) {
      cmp(V_CMP_GT_I64, ST(0), R(a), ic(0));
      if (lanes != EXEC) e(mk(S_AND_B64, ST(0), ST(0), lanes));
      e(mk(V_CNDMASK_B32, T(0), ic(0), R(a), ST(0)));
      e(mk(V_CNDMASK_B32, Th(0), ic(0), Rh(a), ST(0)));
    };
    auto finish_float = [&](uint16_t lanes) {
      cmp(V_CMP_GT_F64, ST(0), R(a), ic(0));                       // !(x > 0) -> 0
      if (lanes != EXEC) e(mk(S_AND_B64, ST(0), ST(0), lanes));
      e(mklit(S_MOV_B32, s(S_LIT_), 0x200u));                      // +inf
      cmp(V_CMP_CLASS_F64, ST(1), R(a), s(S_LIT_));
      e(mk(S_AND_B64, ST(1), ST(1), ST(0)));
      soft_raise(ST(1), EXC_OVERFLOW);
      movk64(s(S_LIT_), 0x43E0000000000000ull);
      cmp(V_CMP_GE_F64, ST(1), R(a), s(S_LIT_));
      e(mk(S_AND_B64, ST(1), ST(1), ST(0)));
      soft_raise(ST(1), EXC_UNSUPPORTED);
      e(mk(M_CVT_I64_F64, T(1), R(a)));
      e(mk(V_CNDMASK_B32, T(0), T(0), T(1), ST(0)));
      e(mk(V_CNDMASK_B32, Th(0), Th(0), Th(1), ST(0)));
    };
    e(mk(V_MOV_B64, T(0), ic(0)));
    if (ta == TY_I) finish_int(EXEC);
    else if (ta == TY_F) finish_float(EXEC);
    else {
      // keep the float lanes in an SGPR pair of their own (finish_* use ST 0-2)
      tag_mask(a, ST(1));
      const int keep = take_spair();
      e(mk(S_MOV_B64, s(keep), ST(1)));
      e(mk(S_ANDN2_B64, s(S_LIT_), EXEC, s(keep)));
      finish_int(s(S_LIT_));
      finish_float(s(keep));
      give_spair(keep);
    }
    e(mk(V_MOV_B64, v(v_out_), T(0)));
  }
};

}  // namespace gcn
}  // namespace fks
