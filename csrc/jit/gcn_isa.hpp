// gfx950 (CDNA4) machine instructions for the baseline program JIT.
//
// The baseline JIT (gcn_codegen.hpp) turns a policy's bytecode straight into
// gfx950 machine code: no LLVM, no subprocess, tens of microseconds per
// program.  This header is its instruction layer:
//
//  * `MI`: one machine instruction (or a macro that lower() expands: the
//    correctly rounded f64 division, int64 <-> f64 conversions, the runtime
//    call with its spill / restore sequence);
//  * `lower()`: macros -> real instructions, s_nop padding for the gfx950
//    VALU hazards the code can create, branch resolution;
//  * `encode()`: SOP1/SOP2/SOPK/SOPC/SOPP/SMEM/VOP1/VOP2/VOPC/VOP3(B)/DS/FLAT
//    words.  Opcode numbers come from the ROCm assembler itself
//    (tools/gen_gcn_opcodes.py -> gcn_opcodes.inc) and tests/test_gcn_jit.py
//    re-assembles every emitted form with llvm-mc.
//
// Operands use the hardware's 9-bit source encoding: 0-101 SGPRs, 106 VCC,
// 126 EXEC, 128-192 the integers 0..64, 193-208 -1..-16, 240-247 the float
// constants, 255 a 32-bit literal, 256 + n VGPR n.
#pragma once

#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

namespace fks {
namespace gcn {

enum Fmt : uint8_t { SOP1, SOP2, SOPK, SOPC, SOPP, SMEM, VOP1, VOP2, VOPC, VOP3, VOP3B, DS, FLAT, PSEUDO };

enum Opc : uint16_t {
#define FKS_GCN_OP(n, f, o) n,
#include "gcn_opcodes.inc"
#undef FKS_GCN_OP
  LABEL,          // imm = label id
  M_FDIV64,       // d = s0 / s1 (IEEE, correctly rounded)
  M_CVT_F64_I64,  // d = (double)(int64)s0 (correctly rounded)
  M_CVT_I64_F64,  // d = (int64)s0 (s0 integral, |s0| < 2^63)
  M_RTCALL,       // runtime-library call (CallInfo ext)
  NUM_OPC
};

struct OpInfo {
  const char* name;
  Fmt fmt;
  uint16_t code;
};

inline const OpInfo& info(Opc o) {
  static const OpInfo tab[] = {
#define FKS_GCN_OP(n, f, o) {#n, f, o},
#include "gcn_opcodes.inc"
#undef FKS_GCN_OP
      {"LABEL", PSEUDO, 0},        {"M_FDIV64", PSEUDO, 0}, {"M_CVT_F64_I64", PSEUDO, 0},
      {"M_CVT_I64_F64", PSEUDO, 0}, {"M_RTCALL", PSEUDO, 0},
  };
  return tab[o];
}

// ---- operand codes -------------------------------------------------------------
constexpr uint16_t VCC = 106, EXEC = 126, M0 = 124, LIT = 255, NONE = 0xFFFF;
constexpr uint16_t F_HALF = 240, F_ONE = 242, F_TWO = 244;
constexpr uint16_t v(int n) { return (uint16_t)(256 + n); }
constexpr uint16_t s(int n) { return (uint16_t)n; }
constexpr bool is_v(uint16_t c) { return c >= 256 && c != NONE; }
constexpr bool is_s(uint16_t c) { return c < 128 && c != NONE; }   // SGPR / VCC / EXEC / M0
constexpr int vidx(uint16_t c) { return (int)c - 256; }
// inline integer constant, or NONE
constexpr uint16_t ic(int64_t x) {
  return (x >= 0 && x <= 64) ? (uint16_t)(128 + x) : (x >= -16 && x < 0) ? (uint16_t)(192 - x) : NONE;
}
inline bool is_inline(uint16_t c) { return c >= 128 && c <= 208; }
inline bool is_fconst(uint16_t c) { return c >= 240 && c <= 248; }

// ---- machine instruction ----------------------------------------------------------
struct MI {
  Opc op = S_NOP;
  uint16_t d = NONE;    // vdst / sdst
  uint16_t sd = NONE;   // VOP3B / VOPC e64 scalar destination
  uint16_t s0 = NONE, s1 = NONE, s2 = NONE;
  uint32_t lit = 0;     // literal (when a source is LIT)
  int32_t imm = 0;      // SOPP / SOPK simm16, offsets, label id
  uint8_t neg = 0, abs = 0;
  int32_t ext = -1;     // M_RTCALL: CallInfo index
  int8_t reloc = -1;    // 0 / 1: literal of the s_add_u32 / s_addc_u32 of a runtime-table address
  uint8_t bc = 255;     // bytecode opcode this instruction lowers (emulator profiles; 255: prologue / epilogue)
};

// Runtime-library call (jit_abi.h rt_binop / rt_unop): arguments, result and
// everything that must survive the call (the callee may clobber every
// caller-saved register: v0-v39, v48-55, ..., s0-s29, s40-47, ...).
struct CallInfo {
  int kind = 0;                    // 0 binop, 1 unop
  int op = 0;                      // bytecode opcode
  uint16_t a = NONE, afl = NONE;   // operand a (VGPR pair) and its float flag (VGPR or inline 0 / 1)
  uint16_t b = NONE, bfl = NONE;
  uint16_t res = NONE, resy = NONE;  // result value pair / (fl | exc << 8) word: temps, never spilled
  uint16_t spill_vgpr = NONE;      // VGPR that carries the preserved SGPRs
  std::vector<int> vgprs;          // VGPRs to preserve (indices)
  std::vector<int> sgprs;          // SGPRs to preserve (indices; s30 / s31 always)
};

// Relocation of a PC-relative runtime-table address: rel = target - (code + pc_off)
struct Reloc {
  uint32_t lo_word, hi_word;  // word indices of the s_add_u32 / s_addc_u32 literals
  uint32_t pc_off;            // byte offset of the instruction after s_getpc_b64
};

struct Code {
  std::vector<uint32_t> words;
  std::vector<Reloc> relocs;
  int n_insns = 0;
};

// ---- helpers -------------------------------------------------------------------------
inline bool is_valu(Opc o) {
  const Fmt f = info(o).fmt;
  return f == VOP1 || f == VOP2 || f == VOPC || f == VOP3 || f == VOP3B;
}
inline bool is_vop3b(Opc o) {
  return info(o).fmt == VOP3B || o == V_ADD_CO_U32 || o == V_SUB_CO_U32 || o == V_ADDC_CO_U32 ||
         o == V_SUBB_CO_U32;
}
inline bool uses_lit(const MI& m) { return m.s0 == LIT || m.s1 == LIT || m.s2 == LIT; }

// e32 (VOP1 / VOP2 / VOPC) encodable?  Otherwise VOP3.
inline bool use_e32(const MI& m) {
  const Fmt f = info(m.op).fmt;
  if (m.neg || m.abs) return false;
  if (f == VOP1) return true;
  if (f == VOP2) {
    if (!is_v(m.s1) || !is_v(m.d) || m.s2 == LIT) return false;
    if (m.op == V_CNDMASK_B32) return m.s2 == VCC;
    if (m.op == V_ADD_CO_U32 || m.op == V_SUB_CO_U32) return m.sd == VCC;
    if (m.op == V_ADDC_CO_U32 || m.op == V_SUBB_CO_U32) return m.sd == VCC && m.s2 == VCC;
    return true;
  }
  if (f == VOPC) return m.sd == VCC && is_v(m.s1);
  return false;
}

inline int size_words(const MI& m) {
  const Fmt f = info(m.op).fmt;
  switch (f) {
    case SOP1: case SOP2: case SOPC: return 1 + (uses_lit(m) ? 1 : 0);
    case SOPK: case SOPP: return 1;
    case SMEM: case DS: case FLAT: return 2;
    case VOP1: case VOP2: case VOPC: case VOP3: case VOP3B:
      if (use_e32(m)) return 1 + (uses_lit(m) ? 1 : 0);
      if (uses_lit(m)) throw std::logic_error(std::string("literal in VOP3 form: ") + info(m.op).name);
      return 2;
    case PSEUDO: return 0;
  }
  return 0;
}

inline uint32_t f8(uint16_t c) {
  if (c == NONE) return 0;
  if (c >= 256) throw std::logic_error("VGPR in a scalar operand");
  return c;
}
inline uint32_t f9(uint16_t c) { return c == NONE ? 0u : (uint32_t)c; }

// Encode one real instruction; branch immediates must already be resolved.
inline void encode_one(const MI& m, std::vector<uint32_t>& out) {
  const OpInfo& oi = info(m.op);
  const uint32_t op = oi.code;
  switch (oi.fmt) {
    case SOP1:
      out.push_back(0xBE800000u | f8(m.d) << 16 | op << 8 | f8(m.s0));
      if (uses_lit(m)) out.push_back(m.lit);
      return;
    case SOP2:
      out.push_back(0x80000000u | op << 23 | f8(m.d) << 16 | f8(m.s1) << 8 | f8(m.s0));
      if (uses_lit(m)) out.push_back(m.lit);
      return;
    case SOPK:
      out.push_back(0xB0000000u | op << 23 | f8(m.d) << 16 | ((uint32_t)m.imm & 0xFFFF));
      return;
    case SOPC:
      out.push_back(0xBF000000u | op << 16 | f8(m.s1) << 8 | f8(m.s0));
      if (uses_lit(m)) out.push_back(m.lit);
      return;
    case SOPP:
      out.push_back(0xBF800000u | op << 16 | ((uint32_t)m.imm & 0xFFFF));
      return;
    case SMEM:   // s_load: sdata = d, sbase = s0 (pair), immediate byte offset
      out.push_back(0xC0000000u | op << 18 | 1u << 17 | f8(m.d) << 6 | (f8(m.s0) >> 1));
      out.push_back((uint32_t)m.imm & 0x1FFFFF);
      return;
    case DS:     // ds_read: vdst = d, addr = s0
      out.push_back(0xD8000000u | op << 17 | ((uint32_t)m.imm & 0xFFFF));
      out.push_back((uint32_t)vidx(m.d) << 24 | (uint32_t)vidx(m.s0));
      return;
    case FLAT: {
      // global: vaddr pair s0, saddr off; scratch: saddr s1 (s32), vaddr off,
      // data s2 (stores) / vdst d (loads)
      const bool scratch = m.op != GLOBAL_LOAD_DWORDX2;
      const uint32_t seg = scratch ? 1u : 2u;
      out.push_back(0xDC000000u | op << 18 | seg << 14 | ((uint32_t)m.imm & 0x1FFF));
      const uint32_t vd = m.d == NONE ? 0u : (uint32_t)vidx(m.d);
      const uint32_t data = m.s2 == NONE ? 0u : (uint32_t)vidx(m.s2);
      const uint32_t saddr = scratch ? f8(m.s1) : 0x7Fu;
      const uint32_t addr = scratch ? 0u : (uint32_t)vidx(m.s0);
      out.push_back(vd << 24 | saddr << 16 | data << 8 | addr);
      return;
    }
    case VOP1: case VOP2: case VOPC: case VOP3: case VOP3B: {
      if (use_e32(m)) {
        if (oi.fmt == VOP1) {
          const uint32_t dst = m.d == NONE ? 0u : (is_v(m.d) ? (uint32_t)vidx(m.d) : (uint32_t)m.d);
          out.push_back(0x7E000000u | dst << 17 | op << 9 | f9(m.s0));
        } else if (oi.fmt == VOP2) {
          out.push_back(op << 25 | (uint32_t)vidx(m.d) << 17 | (uint32_t)vidx(m.s1) << 9 | f9(m.s0));
        } else {
          out.push_back(0x7C000000u | op << 17 | (uint32_t)vidx(m.s1) << 9 | f9(m.s0));
        }
        if (uses_lit(m)) out.push_back(m.lit);
        return;
      }
      uint32_t op3 = op;
      if (oi.fmt == VOP1) op3 = 0x140 + op;
      else if (oi.fmt == VOP2) op3 = 0x100 + op;
      uint32_t w0 = 0xD0000000u | op3 << 16;
      if (oi.fmt == VOPC) {
        w0 |= f8(m.sd) | (uint32_t)(m.abs & 3) << 8;   // VOP3A: sdst in the vdst field, abs still encoded
      } else {
        const uint32_t dst = m.d == NONE ? 0u : (is_v(m.d) ? (uint32_t)vidx(m.d) : (uint32_t)m.d);
        w0 |= dst;
        if (is_vop3b(m.op)) w0 |= f8(m.sd) << 8;
        else w0 |= (uint32_t)(m.abs & 7) << 8;
      }
      out.push_back(w0);
      out.push_back((uint32_t)(m.neg & 7) << 29 | f9(m.s2) << 18 | f9(m.s1) << 9 | f9(m.s0));
      return;
    }
    case PSEUDO:
      return;
  }
}

}  // namespace gcn
}  // namespace fks
