// Macro expansion, gfx950 hazard padding, branch resolution and encoding of a
// baseline-JIT function (gcn_isa.hpp).
#pragma once

#include <algorithm>
#include <unordered_map>

#include "gcn_isa.hpp"

namespace fks {
namespace gcn {

// Registers reserved for macro expansion (gcn_codegen.hpp never allocates them
// to values that live across a macro).
struct MacroRegs {
  int x[4] = {-1, -1, -1, -1};  // four VGPR pairs (even indices)
  int st = 24;                  // SGPR pair: fdiv scale flag / conversion constant
  int sc = 28;                  // SGPR pair: call scratch (exec save, callee address)
};

struct Func {
  std::vector<MI> mi;
  std::vector<CallInfo> calls;
  int n_labels = 0;
  int spill_bytes = 0;          // per-lane scratch [s32, s32 + spill_bytes): spilled registers
  MacroRegs mr;
  int new_label() { return n_labels++; }
};

inline MI mk(Opc op, uint16_t d = NONE, uint16_t s0 = NONE, uint16_t s1 = NONE, uint16_t s2 = NONE) {
  MI m;
  m.op = op; m.d = d; m.s0 = s0; m.s1 = s1; m.s2 = s2;
  return m;
}
inline MI mk3b(Opc op, uint16_t d, uint16_t sd, uint16_t s0, uint16_t s1, uint16_t s2 = NONE) {
  MI m = mk(op, d, s0, s1, s2);
  m.sd = sd;
  return m;
}
inline MI mkimm(Opc op, int32_t imm, uint16_t d = NONE) {
  MI m;
  m.op = op; m.imm = imm; m.d = d;
  return m;
}
// 32-bit constant operand: an inline constant when the value has one (the
// canonical encoding), a literal otherwise
inline MI mklit(Opc op, uint16_t d, uint32_t lit, uint16_t s1 = NONE) {
  const uint16_t c = ic((int32_t)lit);
  MI m = mk(op, d, c != NONE ? c : LIT, s1);
  m.lit = c != NONE ? 0u : lit;
  return m;
}

// ---- macro expansion -------------------------------------------------------------------
inline void expand(const Func& f, std::vector<MI>& out, int& next_label) {
  const MacroRegs& r = f.mr;
  auto X = [&](int i) { return v(r.x[i]); };
  for (const MI& m : f.mi) {
    switch (m.op) {
      case M_FDIV64: {
        // LLVM's correctly rounded f64 division (v_div_scale / v_rcp / 2 Newton
        // steps / v_div_fmas / v_div_fixup); num = s0, den = s1
        const uint16_t num = m.s0, den = m.s1;
        out.push_back(mk3b(V_DIV_SCALE_F64, X(0), s(r.st), den, den, num));
        out.push_back(mk(V_RCP_F64, X(1), X(0)));
        out.push_back(mk3b(V_DIV_SCALE_F64, X(2), VCC, num, den, num));
        MI a = mk(V_FMA_F64, X(3), X(0), X(1), F_ONE); a.neg = 1; out.push_back(a);
        out.push_back(mk(V_FMA_F64, X(1), X(1), X(3), X(1)));
        out.push_back(a);
        out.push_back(mk(V_FMA_F64, X(1), X(1), X(3), X(1)));
        out.push_back(mk(V_MUL_F64, X(3), X(2), X(1)));
        MI b = mk(V_FMA_F64, X(0), X(0), X(3), X(2)); b.neg = 1; out.push_back(b);
        out.push_back(mk(V_DIV_FMAS_F64, X(0), X(0), X(1), X(3)));
        out.push_back(mk(V_DIV_FIXUP_F64, m.d, X(0), den, num));
        break;
      }
      case M_CVT_F64_I64: {
        const uint16_t lo = m.s0, hi = (uint16_t)(m.s0 + 1);
        out.push_back(mk(V_CVT_F64_I32, X(0), hi));
        out.push_back(mk(V_LDEXP_F64, X(0), X(0), ic(32)));
        out.push_back(mk(V_CVT_F64_U32, X(1), lo));
        out.push_back(mk(V_ADD_F64, m.d, X(0), X(1)));
        break;
      }
      case M_CVT_I64_F64: {
        out.push_back(mk(V_TRUNC_F64, X(0), m.s0));
        out.push_back(mkimm(S_MOVK_I32, (int32_t)0xFFE0, s(r.st)));             // -32
        out.push_back(mk(V_LDEXP_F64, X(1), X(0), s(r.st)));
        out.push_back(mk(V_FLOOR_F64, X(1), X(1)));
        out.push_back(mk(S_MOV_B32, s(r.st), ic(0)));
        out.push_back(mklit(S_MOV_B32, s(r.st + 1), 0xC1F00000u));                // -2^32
        out.push_back(mk(V_FMA_F64, X(0), X(1), s(r.st), X(0)));
        out.push_back(mk(V_CVT_U32_F64, m.d, X(0)));
        out.push_back(mk(V_CVT_I32_F64, (uint16_t)(m.d + 1), X(1)));
        break;
      }
      case M_RTCALL: {
        const CallInfo& c = f.calls[(size_t)m.ext];
        const int skip = next_label++;
        out.push_back(mkimm(S_CBRANCH_EXECZ, skip));
        MI sav = mk(S_OR_SAVEEXEC_B64, s(r.sc), ic(-1));
        out.push_back(sav);
        int off = f.spill_bytes;   // the save area sits above the spill slots
        // one dword per live VGPR: scratch is swizzled per lane in dwords, and
        // paired / quad accesses measured ~9% slower on evolved populations
        // (tools/population_bench.py, profiles/r4_jit_rtcall_save_ab.txt)
        for (int g : c.vgprs) {
          MI st = mk(SCRATCH_STORE_DWORD, NONE, NONE, s(32), v(g));
          st.imm = off; off += 4;
          out.push_back(st);
        }
        // v_writelane writes its lane whatever EXEC holds, and the caller may
        // keep values in the inactive lanes of any VGPR across the call (the
        // ABI: a callee preserves them) -- LLVM does, e.g. an `if` result
        // zeroed before the branch in a caller-saved register.  So the spill
        // VGPR's own contents are saved first and reloaded after the readlanes.
        const int orig = off;
        {
          MI st = mk(SCRATCH_STORE_DWORD, NONE, NONE, s(32), c.spill_vgpr);
          st.imm = orig; off += 4;
          out.push_back(st);
        }
        int lane = 0;
        for (int sg : c.sgprs) {
          MI wl = mk(V_WRITELANE_B32, c.spill_vgpr, s(sg), ic(lane++));
          out.push_back(wl);
        }
        {
          MI st = mk(SCRATCH_STORE_DWORD, NONE, NONE, s(32), c.spill_vgpr);
          st.imm = off; off += 4;
          out.push_back(st);
        }
        out.push_back(mk(S_MOV_B64, EXEC, s(r.sc)));
        // arguments: v0 = op, v[1:2] = a, v3 = a.fl, v[4:5] = b, v6 = b.fl (the
        // operands were copied to macro temps by the code generator, so these
        // moves never read a register they already overwrote)
        out.push_back(mk(V_MOV_B32, v(0), ic(c.op)));
        out.push_back(mk(V_MOV_B32, v(1), c.a));
        out.push_back(mk(V_MOV_B32, v(2), (uint16_t)(c.a + 1)));
        out.push_back(mk(V_MOV_B32, v(3), c.afl));
        if (c.kind == 0) {
          out.push_back(mk(V_MOV_B32, v(4), c.b));
          out.push_back(mk(V_MOV_B32, v(5), (uint16_t)(c.b + 1)));
          out.push_back(mk(V_MOV_B32, v(6), c.bfl));
        }
        const int frame = (off + 15) & ~15;
        {
          MI a = mklit(S_ADD_I32, s(32), (uint32_t)frame, s(32));
          std::swap(a.s0, a.s1);   // s32 + frame
          out.push_back(a);
        }
        out.push_back(mk(S_GETPC_B64, s(r.sc)));
        {
          MI lo = mk(S_ADD_U32, s(r.sc), s(r.sc), LIT);
          MI hi = mk(S_ADDC_U32, s(r.sc + 1), s(r.sc + 1), LIT);
          lo.reloc = 0;
          hi.reloc = 1;
          out.push_back(lo);
          out.push_back(hi);
        }
        MI ld = mk(S_LOAD_DWORDX2, s(r.sc), s(r.sc));
        ld.imm = 8 * c.kind;
        out.push_back(ld);
        out.push_back(mkimm(S_WAITCNT, 0xC07F));   // lgkmcnt(0)
        out.push_back(mk(S_SWAPPC_B64, s(30), s(r.sc)));
        {
          MI a = mklit(S_ADD_I32, s(32), (uint32_t)(-frame), s(32));
          std::swap(a.s0, a.s1);
          out.push_back(a);
        }
        out.push_back(mk(V_MOV_B32, c.res, v(0)));
        out.push_back(mk(V_MOV_B32, (uint16_t)(c.res + 1), v(1)));
        out.push_back(mk(V_MOV_B32, c.resy, v(2)));
        out.push_back(mk(S_OR_SAVEEXEC_B64, s(r.sc), ic(-1)));
        off = f.spill_bytes;
        for (int g : c.vgprs) {
          MI ldv = mk(SCRATCH_LOAD_DWORD, v(g), NONE, s(32));
          ldv.imm = off; off += 4;
          out.push_back(ldv);
        }
        off += 4;   // the spill VGPR's own contents (orig)
        {
          MI ldv = mk(SCRATCH_LOAD_DWORD, c.spill_vgpr, NONE, s(32));
          ldv.imm = off;
          out.push_back(ldv);
        }
        out.push_back(mkimm(S_WAITCNT, 0x0F70));   // vmcnt(0)
        lane = 0;
        for (int sg : c.sgprs) out.push_back(mk(V_READLANE_B32, s(sg), c.spill_vgpr, ic(lane++)));
        {
          MI ldv = mk(SCRATCH_LOAD_DWORD, c.spill_vgpr, NONE, s(32));
          ldv.imm = orig;
          out.push_back(ldv);
        }
        out.push_back(mkimm(S_WAITCNT, 0x0F70));   // vmcnt(0)
        out.push_back(mk(S_MOV_B64, EXEC, s(r.sc)));
        out.push_back(mkimm(LABEL, skip));
        break;
      }
      default:
        out.push_back(m);
    }
  }
}

// ---- hazards ----------------------------------------------------------------------------
// Registers an instruction writes / reads, as (first, count) ranges of operand codes.
struct Span {
  uint16_t c;
  int n;
};
inline bool overlaps(Span a, uint16_t c, int n) {
  return a.c != NONE && c != NONE && a.c < c + n && c < a.c + a.n;
}

inline int dst_width(const MI& m) {
  switch (m.op) {
    case V_MOV_B64: case V_CVT_F64_I32: case V_CVT_F64_U32: case V_TRUNC_F64: case V_RNDNE_F64:
    case V_FLOOR_F64: case V_RCP_F64: case V_ADD_F64: case V_MUL_F64: case V_FMA_F64: case V_LDEXP_F64:
    case V_DIV_SCALE_F64: case V_DIV_FMAS_F64: case V_DIV_FIXUP_F64: case V_MAD_U64_U32: case V_MAD_I64_I32:
    case V_LSHLREV_B64: case V_LSHRREV_B64: case V_ASHRREV_I64: case V_LSHL_ADD_U64: case DS_READ_B64:
    case GLOBAL_LOAD_DWORDX2: case SCRATCH_LOAD_DWORDX2:
      return 2;
    case SCRATCH_LOAD_DWORDX4:
      return 4;
    default:
      return 1;
  }
}

// Wait states the gfx950 hazard rules need between `prod` (an earlier VALU)
// and `cons` (LLVM GCNHazardRecognizer's rules for the instructions emitted
// here; checked against the padding hipcc puts in the same sequences).
inline int needed_wait(const MI& prod, const MI& cons) {
  if (!is_valu(prod.op)) return 0;
  int w = 0;
  uint16_t sdst = NONE;
  if (info(prod.op).fmt == VOPC || is_vop3b(prod.op)) sdst = prod.sd;
  else if (prod.op == V_READFIRSTLANE_B32 || prod.op == V_READLANE_B32) sdst = prod.d;
  if (sdst != NONE) {
    if (cons.op == V_CNDMASK_B32 && cons.s2 == sdst) w = std::max(w, 2);        // lane mask
    if (cons.op == V_DIV_FMAS_F64 && sdst == VCC) w = std::max(w, 4);
    if ((cons.op == V_READLANE_B32 || cons.op == V_WRITELANE_B32) && cons.s1 == sdst) w = std::max(w, 4);
    if ((prod.op == V_READFIRSTLANE_B32 || prod.op == V_READLANE_B32) && is_valu(cons.op) &&
        (cons.s0 == sdst || cons.s1 == sdst || cons.s2 == sdst))
      w = std::max(w, 1);
  }
  // VALU writes a VGPR that v_readfirstlane / v_readlane reads
  if (is_v(prod.d) && (cons.op == V_READFIRSTLANE_B32 || cons.op == V_READLANE_B32) &&
      overlaps(Span{prod.d, dst_width(prod)}, cons.s0, 1))
    w = std::max(w, 1);
  // transcendental result consumed by the next VALU
  if (prod.op == V_RCP_F64 && is_valu(cons.op))
    for (uint16_t c : {cons.s0, cons.s1, cons.s2})
      if (overlaps(Span{prod.d, 2}, c, 2)) w = std::max(w, 1);
  return w;
}

inline std::vector<MI> pad_hazards(const std::vector<MI>& in) {
  std::vector<MI> out;
  out.reserve(in.size() + in.size() / 4);
  for (const MI& m : in) {
    if (m.op != LABEL && info(m.op).fmt != PSEUDO) {
      // scan back over the last few issued instructions (labels cost nothing)
      int need = 0, dist = 0;
      for (size_t k = out.size(); k-- > 0 && dist < 5;) {
        const MI& p = out[k];
        if (p.op == LABEL) continue;
        if (p.op == S_BRANCH || p.op == S_SETPC_B64 || p.op == S_SWAPPC_B64) break;
        const int w = needed_wait(p, m) - dist;
        if (w > need) need = w;
        dist += p.op == S_NOP ? p.imm + 1 : 1;
      }
      if (need > 0) out.push_back(mkimm(S_NOP, need - 1));
    }
    out.push_back(m);
  }
  return out;
}

// ---- assemble ------------------------------------------------------------------------------
inline bool is_branch(Opc o) {
  return o == S_BRANCH || o == S_CBRANCH_SCC0 || o == S_CBRANCH_SCC1 || o == S_CBRANCH_VCCZ ||
         o == S_CBRANCH_VCCNZ || o == S_CBRANCH_EXECZ || o == S_CBRANCH_EXECNZ;
}

inline Code assemble(const Func& f) {
  std::vector<MI> lowered;
  int n_labels = f.n_labels;
  expand(f, lowered, n_labels);
  const std::vector<MI> fin = pad_hazards(lowered);
  // layout
  std::vector<int> label_word((size_t)n_labels, -1);
  std::vector<int> word_of(fin.size());
  int w = 0;
  for (size_t i = 0; i < fin.size(); ++i) {
    word_of[i] = w;
    if (fin[i].op == LABEL) label_word[(size_t)fin[i].imm] = w;
    else w += size_words(fin[i]);
  }
  Code out;
  out.words.reserve((size_t)w);
  int pending_lo = -1;
  uint32_t pc_after_getpc = 0;
  for (size_t i = 0; i < fin.size(); ++i) {
    MI m = fin[i];
    if (m.op == LABEL) continue;
    if (is_branch(m.op)) {
      const int t = label_word[(size_t)m.imm];
      if (t < 0) throw std::logic_error("branch to an unplaced label");
      const int rel = t - (word_of[i] + 1);
      if (rel < -32768 || rel > 32767) throw std::runtime_error("branch out of range");
      m.imm = rel;
    }
    if (m.op == S_GETPC_B64) pc_after_getpc = (uint32_t)(word_of[i] + 1) * 4;
    encode_one(m, out.words);
    ++out.n_insns;
    if (m.reloc == 0) pending_lo = (int)out.words.size() - 1;
    if (m.reloc == 1) {
      if (pending_lo < 0) throw std::logic_error("unpaired relocation");
      out.relocs.push_back(Reloc{(uint32_t)pending_lo, (uint32_t)out.words.size() - 1, pc_after_getpc});
      pending_lo = -1;
    }
  }
  return out;
}

}  // namespace gcn
}  // namespace fks
