// Wave64 emulator of the baseline JIT's machine-instruction stream (before
// macro expansion), for CPU-side validation: tests replay whole traces with
// the emulated program as the scorer and compare against the CPU VM and the
// host build of the LLVM-path code (tests/test_gcn_jit.py).  It models exactly
// the instruction subset the code generator emits: per-lane VALU under EXEC,
// VOPC results (0 in inactive lanes), SALU with SCC, structured branches,
// LDS / global / scratch memory.  Macros run with their defined semantics
// (M_RTCALL evaluates the runtime library's host build, pyops_dev.h).
#pragma once

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "gcn_lower.hpp"
#include "../hip/jit_abi.h"

namespace fks {
namespace gcn {

struct Emu {
  static constexpr int kW = 64;
  uint32_t vg[256][kW];
  uint32_t sg[128];
  bool scc = false;
  int gidx = -1;   // GPR index mode (SRC0) offset, -1: off
  int64_t* hist = nullptr;   // executed instructions per opcode (profiling), or null
  int64_t* hist_bc = nullptr;   // ... per bytecode opcode they lower (256 entries), or null
  std::vector<uint8_t> lds;
  std::vector<uint8_t> scratch[kW];
  int64_t steps = 0;
  int trace_lane = std::getenv("FKS_EMU_TRACE_LANE") ? std::atoi(std::getenv("FKS_EMU_TRACE_LANE")) : -1;

  uint64_t rd64s(uint16_t c) const { return (uint64_t)sg[c] | (uint64_t)sg[c + 1] << 32; }
  void wr64s(uint16_t c, uint64_t x) { sg[c] = (uint32_t)x; sg[c + 1] = (uint32_t)(x >> 32); }
  uint64_t exec() const { return rd64s(EXEC); }
  void set_exec(uint64_t x) { wr64s(EXEC, x); }

  // 32-bit source value in lane l
  uint32_t r32(uint16_t c, int l, uint32_t lit, bool f64ctx = false) const {
    if (c < 128) return sg[c];
    if (c >= 128 && c <= 192) return (uint32_t)(c - 128);
    if (c >= 193 && c <= 208) return (uint32_t)(int32_t)(192 - (int)c);
    if (c == LIT) return lit;
    if (c >= 256) return vg[c - 256][l];
    (void)f64ctx;
    throw std::logic_error("emu: unsupported 32-bit operand");
  }
  // 64-bit source: integer context
  uint64_t r64(uint16_t c, int l, uint32_t lit) const {
    if (c < 128) return rd64s(c);
    if (c >= 128 && c <= 192) return (uint64_t)(c - 128);
    if (c >= 193 && c <= 208) return (uint64_t)(int64_t)(192 - (int)c);
    if (c == LIT) return (uint64_t)lit;
    if (c >= 256) return (uint64_t)vg[c - 256][l] | (uint64_t)vg[c - 255][l] << 32;
    throw std::logic_error("emu: unsupported 64-bit operand");
  }
  // 64-bit source: double context (inline float constants are doubles, a literal is the high half)
  double rf(uint16_t c, int l, uint32_t lit) const {
    double x;
    if (c >= 240 && c <= 247) {
      static const double k[8] = {0.5, -0.5, 1.0, -1.0, 2.0, -2.0, 4.0, -4.0};
      return k[c - 240];
    }
    uint64_t b;
    // (an integer inline constant, 128-208, is its sign-extended bit pattern
    // in a 64-bit float operand -- not converted -- as on the hardware)
    if (c == LIT) b = (uint64_t)lit << 32;
    else b = r64(c, l, lit);
    std::memcpy(&x, &b, 8);
    return x;
  }
  static uint64_t dbits(double x) { uint64_t b; std::memcpy(&b, &x, 8); return b; }
  void w32(uint16_t d, int l, uint32_t x) {
    if (d >= 256) vg[d - 256][l] = x;
    else sg[d] = x;
  }
  void w64v(uint16_t d, int l, uint64_t x) {
    vg[d - 256][l] = (uint32_t)x;
    vg[d - 255][l] = (uint32_t)(x >> 32);
  }
  static double mod_f(double x, uint8_t neg, uint8_t abs, int i) {
    if (abs >> i & 1) x = std::fabs(x);
    if (neg >> i & 1) x = -x;
    return x;
  }

  // Run `fn` (with labels resolved to indices) from index 0 until it executes
  // s_setpc_b64 to `ret` (the emulated caller's return address).
  const Func* labels_of = nullptr;
  std::vector<int> label_at;

  void run(const Func& f, uint64_t ret, int64_t max_steps = 200000000) {
    if (labels_of != &f) {
      label_at.assign((size_t)f.n_labels, -1);
      for (size_t i = 0; i < f.mi.size(); ++i)
        if (f.mi[i].op == LABEL) label_at[(size_t)f.mi[i].imm] = (int)i;
      labels_of = &f;
    }
    size_t pc = 0;
    steps = 0;
    for (;;) {
      if (pc >= f.mi.size()) throw std::logic_error("emu: ran off the end");
      if (++steps > max_steps) throw std::runtime_error("emu: step limit");
      const MI& m = f.mi[pc];
      if (hist) ++hist[m.op];
      if (hist_bc) ++hist_bc[m.bc];
      const uint64_t ex = exec();
      size_t next = pc + 1;
      auto lanes = [&](auto fn) {
        for (uint64_t b = ex; b; b &= b - 1) fn(__builtin_ctzll(b));
      };
      auto jump = [&](int lab) { next = (size_t)label_at[(size_t)lab]; };
      if (gidx >= 0 && is_valu(m.op) && m.op != V_MOV_B32)
        throw std::logic_error("emu: VALU other than v_mov_b32 in GPR index mode");
      switch (m.op) {
        case LABEL: case S_NOP: case S_WAITCNT: break;
        case S_ENDPGM: throw std::logic_error("emu: s_endpgm in a function");
        case S_BRANCH: jump(m.imm); break;
        case S_CBRANCH_EXECZ: if (ex == 0) jump(m.imm); break;
        case S_CBRANCH_EXECNZ: if (ex != 0) jump(m.imm); break;
        case S_CBRANCH_SCC0: if (!scc) jump(m.imm); break;
        case S_CBRANCH_SCC1: if (scc) jump(m.imm); break;
        case S_CBRANCH_VCCZ: if (rd64s(VCC) == 0) jump(m.imm); break;
        case S_CBRANCH_VCCNZ: if (rd64s(VCC) != 0) jump(m.imm); break;
        case S_SETPC_B64:
          if (rd64s(m.s0) == ret) return;
          throw std::logic_error("emu: s_setpc to an unknown address");
        // ---- SALU
        case S_MOV_B32: sg[m.d] = r32(m.s0, 0, m.lit); break;
        case S_MOVK_I32: sg[m.d] = (uint32_t)(int32_t)(int16_t)(m.imm & 0xFFFF); break;
        case S_MOV_B64: wr64s(m.d, r64(m.s0, 0, m.lit)); break;
        case S_NOT_B64: { const uint64_t x = ~r64(m.s0, 0, m.lit); wr64s(m.d, x); scc = x != 0; break; }
        case S_AND_SAVEEXEC_B64: { const uint64_t e = ex; set_exec(r64(m.s0, 0, m.lit) & e); wr64s(m.d, e); scc = exec() != 0; break; }
        case S_OR_SAVEEXEC_B64: { const uint64_t e = ex; set_exec(r64(m.s0, 0, m.lit) | e); wr64s(m.d, e); scc = exec() != 0; break; }
        case S_AND_B64: { const uint64_t x = r64(m.s0, 0, m.lit) & r64(m.s1, 0, m.lit); wr64s(m.d, x); scc = x != 0; break; }
        case S_OR_B64: { const uint64_t x = r64(m.s0, 0, m.lit) | r64(m.s1, 0, m.lit); wr64s(m.d, x); scc = x != 0; break; }
        case S_XOR_B64: { const uint64_t x = r64(m.s0, 0, m.lit) ^ r64(m.s1, 0, m.lit); wr64s(m.d, x); scc = x != 0; break; }
        case S_ANDN2_B64: { const uint64_t x = r64(m.s0, 0, m.lit) & ~r64(m.s1, 0, m.lit); wr64s(m.d, x); scc = x != 0; break; }
        case S_ORN2_B64: { const uint64_t x = r64(m.s0, 0, m.lit) | ~r64(m.s1, 0, m.lit); wr64s(m.d, x); scc = x != 0; break; }
        case S_CSELECT_B64: wr64s(m.d, scc ? r64(m.s0, 0, m.lit) : r64(m.s1, 0, m.lit)); break;
        case S_AND_B32: { const uint32_t x = r32(m.s0, 0, m.lit) & r32(m.s1, 0, m.lit); sg[m.d] = x; scc = x != 0; break; }
        case S_LSHR_B32: { const uint32_t x = r32(m.s0, 0, m.lit) >> (r32(m.s1, 0, m.lit) & 31); sg[m.d] = x; scc = x != 0; break; }
        case S_ASHR_I32: { const uint32_t x = (uint32_t)((int32_t)r32(m.s0, 0, m.lit) >> (r32(m.s1, 0, m.lit) & 31)); sg[m.d] = x; scc = x != 0; break; }
        case S_ADD_U32: { const uint64_t x = (uint64_t)r32(m.s0, 0, m.lit) + r32(m.s1, 0, m.lit); sg[m.d] = (uint32_t)x; scc = x >> 32; break; }
        case S_ADDC_U32: { const uint64_t x = (uint64_t)r32(m.s0, 0, m.lit) + r32(m.s1, 0, m.lit) + (scc ? 1 : 0); sg[m.d] = (uint32_t)x; scc = x >> 32; break; }
        case S_SUB_U32: { const uint32_t a = r32(m.s0, 0, m.lit), b = r32(m.s1, 0, m.lit); sg[m.d] = a - b; scc = b > a; break; }
        case S_ADD_I32: { const int64_t x = (int64_t)(int32_t)r32(m.s0, 0, m.lit) + (int32_t)r32(m.s1, 0, m.lit); sg[m.d] = (uint32_t)x; scc = x != (int32_t)x; break; }
        case S_SET_GPR_IDX_ON:
          if (m.s1 != 1) throw std::logic_error("emu: GPR index mode other than SRC0");
          gidx = (int)(sg[m.s0] & 0xFF);
          break;
        case S_SET_GPR_IDX_OFF: gidx = -1; break;
        case S_CMP_EQ_U32: scc = r32(m.s0, 0, m.lit) == r32(m.s1, 0, m.lit); break;
        case S_CMP_LG_U32: scc = r32(m.s0, 0, m.lit) != r32(m.s1, 0, m.lit); break;
        case S_CMP_EQ_U64: scc = r64(m.s0, 0, m.lit) == r64(m.s1, 0, m.lit); break;
        case S_CMP_LG_U64: scc = r64(m.s0, 0, m.lit) != r64(m.s1, 0, m.lit); break;
        // ---- VALU
        case V_MOV_B32:
          if (gidx >= 0) {
            if (m.s0 < 256 || m.s0 - 256 + gidx >= 256) throw std::logic_error("emu: indexed move out of range");
            lanes([&](int l) { w32(m.d, l, vg[m.s0 - 256 + gidx][l]); });
          } else {
            lanes([&](int l) { w32(m.d, l, r32(m.s0, l, m.lit)); });
          }
          break;
        case V_MOV_B64: lanes([&](int l) { w64v(m.d, l, r64(m.s0, l, m.lit)); }); break;
        case V_NOT_B32: lanes([&](int l) { w32(m.d, l, ~r32(m.s0, l, m.lit)); }); break;
        case V_READFIRSTLANE_B32: {
          int l0 = 0;
          while (l0 < kW && !(ex >> l0 & 1)) ++l0;
          sg[m.d] = r32(m.s0, l0 < kW ? l0 : 0, m.lit);
          break;
        }
        case V_READLANE_B32: sg[m.d] = r32(m.s0, (int)(r32(m.s1, 0, m.lit) & 63), m.lit); break;
        case V_WRITELANE_B32: vg[m.d - 256][r32(m.s1, 0, m.lit) & 63] = r32(m.s0, 0, m.lit); break;
        case V_CVT_F64_I32: lanes([&](int l) { w64v(m.d, l, dbits((double)(int32_t)r32(m.s0, l, m.lit))); }); break;
        case V_CVT_F64_U32: lanes([&](int l) { w64v(m.d, l, dbits((double)r32(m.s0, l, m.lit))); }); break;
        case V_TRUNC_F64: lanes([&](int l) { w64v(m.d, l, dbits(std::trunc(mod_f(rf(m.s0, l, m.lit), m.neg, m.abs, 0)))); }); break;
        case V_RNDNE_F64: lanes([&](int l) { w64v(m.d, l, dbits(std::nearbyint(mod_f(rf(m.s0, l, m.lit), m.neg, m.abs, 0)))); }); break;
        case V_FLOOR_F64: lanes([&](int l) { w64v(m.d, l, dbits(std::floor(mod_f(rf(m.s0, l, m.lit), m.neg, m.abs, 0)))); }); break;
        case V_CNDMASK_B32: {
          const uint64_t mask = r64(m.s2, 0, m.lit);
          lanes([&](int l) { w32(m.d, l, (mask >> l & 1) ? r32(m.s1, l, m.lit) : r32(m.s0, l, m.lit)); });
          break;
        }
        case V_AND_B32: lanes([&](int l) { w32(m.d, l, r32(m.s0, l, m.lit) & r32(m.s1, l, m.lit)); }); break;
        case V_OR_B32: lanes([&](int l) { w32(m.d, l, r32(m.s0, l, m.lit) | r32(m.s1, l, m.lit)); }); break;
        case V_XOR_B32: lanes([&](int l) { w32(m.d, l, r32(m.s0, l, m.lit) ^ r32(m.s1, l, m.lit)); }); break;
        case V_LSHLREV_B32: lanes([&](int l) { w32(m.d, l, r32(m.s1, l, m.lit) << (r32(m.s0, l, m.lit) & 31)); }); break;
        case V_LSHRREV_B32: lanes([&](int l) { w32(m.d, l, r32(m.s1, l, m.lit) >> (r32(m.s0, l, m.lit) & 31)); }); break;
        case V_ASHRREV_I32: lanes([&](int l) { w32(m.d, l, (uint32_t)((int32_t)r32(m.s1, l, m.lit) >> (r32(m.s0, l, m.lit) & 31))); }); break;
        case V_ADD_U32: lanes([&](int l) { w32(m.d, l, r32(m.s0, l, m.lit) + r32(m.s1, l, m.lit)); }); break;
        case V_SUB_U32: lanes([&](int l) { w32(m.d, l, r32(m.s0, l, m.lit) - r32(m.s1, l, m.lit)); }); break;
        case V_MAX_U32: lanes([&](int l) { w32(m.d, l, std::max(r32(m.s0, l, m.lit), r32(m.s1, l, m.lit))); }); break;
        case V_MIN_U32: lanes([&](int l) { w32(m.d, l, std::min(r32(m.s0, l, m.lit), r32(m.s1, l, m.lit))); }); break;
        case V_ADD_CO_U32: case V_SUB_CO_U32: case V_ADDC_CO_U32: case V_SUBB_CO_U32: {
          const uint64_t cin = (m.op == V_ADDC_CO_U32 || m.op == V_SUBB_CO_U32) ? r64(m.s2, 0, m.lit) : 0;
          uint64_t cout = 0;
          lanes([&](int l) {
            const uint64_t a = r32(m.s0, l, m.lit), b = r32(m.s1, l, m.lit), ci = cin >> l & 1;
            uint64_t x;
            bool c;
            if (m.op == V_ADD_CO_U32 || m.op == V_ADDC_CO_U32) { x = a + b + ci; c = x >> 32; }
            else { x = a - b - ci; c = b + ci > a; }
            w32(m.d, l, (uint32_t)x);
            if (c) cout |= 1ull << l;
          });
          wr64s(m.sd, cout);
          break;
        }
        case V_CMP_CLASS_F64: case V_CMP_LT_F64: case V_CMP_EQ_F64: case V_CMP_LE_F64: case V_CMP_GT_F64:
        case V_CMP_GE_F64: case V_CMP_NEQ_F64: case V_CMP_U_F64: case V_CMP_LT_I32: case V_CMP_EQ_U32:
        case V_CMP_NE_U32: case V_CMP_GT_U32: case V_CMP_GE_U32: case V_CMP_LT_U32: case V_CMP_LT_I64:
        case V_CMP_EQ_I64: case V_CMP_LE_I64: case V_CMP_GT_I64: case V_CMP_NE_I64: case V_CMP_GE_I64:
        case V_CMP_LT_U64: case V_CMP_GT_U64: {
          uint64_t res = 0;
          lanes([&](int l) {
            bool t = false;
            switch (m.op) {
              case V_CMP_CLASS_F64: {
                const double x = mod_f(rf(m.s0, l, m.lit), m.neg, m.abs, 0);
                const uint32_t k = r32(m.s1, l, m.lit);
                int cls;
                if (std::isnan(x)) cls = 1;   // quiet NaN (signalling NaNs never arise here)
                else if (std::isinf(x)) cls = x < 0 ? 2 : 9;
                else if (x == 0) cls = std::signbit(x) ? 5 : 6;
                else if (std::fpclassify(x) == FP_SUBNORMAL) cls = x < 0 ? 4 : 7;
                else cls = x < 0 ? 3 : 8;
                t = (k >> cls) & 1;
                break;
              }
              case V_CMP_LT_F64: t = mod_f(rf(m.s0, l, m.lit), m.neg, m.abs, 0) < mod_f(rf(m.s1, l, m.lit), m.neg, m.abs, 1); break;
              case V_CMP_EQ_F64: t = mod_f(rf(m.s0, l, m.lit), m.neg, m.abs, 0) == mod_f(rf(m.s1, l, m.lit), m.neg, m.abs, 1); break;
              case V_CMP_LE_F64: t = mod_f(rf(m.s0, l, m.lit), m.neg, m.abs, 0) <= mod_f(rf(m.s1, l, m.lit), m.neg, m.abs, 1); break;
              case V_CMP_GT_F64: t = mod_f(rf(m.s0, l, m.lit), m.neg, m.abs, 0) > mod_f(rf(m.s1, l, m.lit), m.neg, m.abs, 1); break;
              case V_CMP_GE_F64: t = mod_f(rf(m.s0, l, m.lit), m.neg, m.abs, 0) >= mod_f(rf(m.s1, l, m.lit), m.neg, m.abs, 1); break;
              case V_CMP_NEQ_F64: t = !(mod_f(rf(m.s0, l, m.lit), m.neg, m.abs, 0) == mod_f(rf(m.s1, l, m.lit), m.neg, m.abs, 1)); break;
              case V_CMP_U_F64: t = std::isnan(rf(m.s0, l, m.lit)) || std::isnan(rf(m.s1, l, m.lit)); break;
              case V_CMP_LT_I32: t = (int32_t)r32(m.s0, l, m.lit) < (int32_t)r32(m.s1, l, m.lit); break;
              case V_CMP_EQ_U32: t = r32(m.s0, l, m.lit) == r32(m.s1, l, m.lit); break;
              case V_CMP_NE_U32: t = r32(m.s0, l, m.lit) != r32(m.s1, l, m.lit); break;
              case V_CMP_GT_U32: t = r32(m.s0, l, m.lit) > r32(m.s1, l, m.lit); break;
              case V_CMP_GE_U32: t = r32(m.s0, l, m.lit) >= r32(m.s1, l, m.lit); break;
              case V_CMP_LT_U32: t = r32(m.s0, l, m.lit) < r32(m.s1, l, m.lit); break;
              case V_CMP_LT_I64: t = (int64_t)r64(m.s0, l, m.lit) < (int64_t)r64(m.s1, l, m.lit); break;
              case V_CMP_EQ_I64: t = r64(m.s0, l, m.lit) == r64(m.s1, l, m.lit); break;
              case V_CMP_LE_I64: t = (int64_t)r64(m.s0, l, m.lit) <= (int64_t)r64(m.s1, l, m.lit); break;
              case V_CMP_GT_I64: t = (int64_t)r64(m.s0, l, m.lit) > (int64_t)r64(m.s1, l, m.lit); break;
              case V_CMP_NE_I64: t = r64(m.s0, l, m.lit) != r64(m.s1, l, m.lit); break;
              case V_CMP_GE_I64: t = (int64_t)r64(m.s0, l, m.lit) >= (int64_t)r64(m.s1, l, m.lit); break;
              case V_CMP_LT_U64: t = r64(m.s0, l, m.lit) < r64(m.s1, l, m.lit); break;
              case V_CMP_GT_U64: t = r64(m.s0, l, m.lit) > r64(m.s1, l, m.lit); break;
              default: break;
            }
            if (t) res |= 1ull << l;
          });
          wr64s(m.sd, res);
          break;
        }
        case V_ADD_F64: lanes([&](int l) { w64v(m.d, l, dbits(mod_f(rf(m.s0, l, m.lit), m.neg, m.abs, 0) + mod_f(rf(m.s1, l, m.lit), m.neg, m.abs, 1))); }); break;
        case V_MUL_F64: lanes([&](int l) { w64v(m.d, l, dbits(mod_f(rf(m.s0, l, m.lit), m.neg, m.abs, 0) * mod_f(rf(m.s1, l, m.lit), m.neg, m.abs, 1))); }); break;
        case V_FMA_F64: lanes([&](int l) { w64v(m.d, l, dbits(std::fma(mod_f(rf(m.s0, l, m.lit), m.neg, m.abs, 0), mod_f(rf(m.s1, l, m.lit), m.neg, m.abs, 1), mod_f(rf(m.s2, l, m.lit), m.neg, m.abs, 2)))); }); break;
        case V_LDEXP_F64: lanes([&](int l) { w64v(m.d, l, dbits(std::ldexp(rf(m.s0, l, m.lit), (int32_t)r32(m.s1, l, m.lit)))); }); break;
        case V_MAD_U64_U32: case V_MAD_I64_I32: {
          uint64_t cout = 0;
          lanes([&](int l) {
            uint64_t x;
            if (m.op == V_MAD_U64_U32) {
              const unsigned __int128 p = (unsigned __int128)r32(m.s0, l, m.lit) * r32(m.s1, l, m.lit) + r64(m.s2, l, m.lit);
              x = (uint64_t)p;
              if (p >> 64) cout |= 1ull << l;
            } else {
              const __int128 p = (__int128)(int32_t)r32(m.s0, l, m.lit) * (int32_t)r32(m.s1, l, m.lit) + (int64_t)r64(m.s2, l, m.lit);
              x = (uint64_t)p;
            }
            w64v(m.d, l, x);
          });
          if (m.sd != NONE) wr64s(m.sd, cout);
          break;
        }
        case V_MUL_LO_U32: lanes([&](int l) { w32(m.d, l, r32(m.s0, l, m.lit) * r32(m.s1, l, m.lit)); }); break;
        case V_MUL_HI_U32: lanes([&](int l) { w32(m.d, l, (uint32_t)(((uint64_t)r32(m.s0, l, m.lit) * r32(m.s1, l, m.lit)) >> 32)); }); break;
        case V_LSHLREV_B64: lanes([&](int l) { w64v(m.d, l, r64(m.s1, l, m.lit) << (r32(m.s0, l, m.lit) & 63)); }); break;
        case V_LSHRREV_B64: lanes([&](int l) { w64v(m.d, l, r64(m.s1, l, m.lit) >> (r32(m.s0, l, m.lit) & 63)); }); break;
        case V_ASHRREV_I64: lanes([&](int l) { w64v(m.d, l, (uint64_t)((int64_t)r64(m.s1, l, m.lit) >> (r32(m.s0, l, m.lit) & 63))); }); break;
        case V_BFE_U32: lanes([&](int l) {
          const uint32_t off = r32(m.s1, l, m.lit) & 31, w = r32(m.s2, l, m.lit) & 31;
          w32(m.d, l, w == 0 ? 0u : (r32(m.s0, l, m.lit) >> off) & (w == 32 ? ~0u : ((1u << w) - 1)));
        }); break;
        case V_BFE_I32: lanes([&](int l) {
          const uint32_t off = r32(m.s1, l, m.lit) & 31, w = r32(m.s2, l, m.lit) & 31;
          if (w == 0) { w32(m.d, l, 0); return; }
          const int32_t x = (int32_t)(r32(m.s0, l, m.lit) << (32 - off - w));
          w32(m.d, l, (uint32_t)(x >> (32 - w)));
        }); break;
        case V_LSHL_ADD_U64: lanes([&](int l) { w64v(m.d, l, (r64(m.s0, l, m.lit) << (r32(m.s1, l, m.lit) & 7)) + r64(m.s2, l, m.lit)); }); break;
        case V_CVT_I32_F64: case V_CVT_U32_F64: case V_RCP_F64: case V_DIV_SCALE_F64: case V_DIV_FMAS_F64:
        case V_DIV_FIXUP_F64:
          throw std::logic_error("emu: instruction only valid inside a macro expansion");
        // ---- memory
        case DS_READ_B64: lanes([&](int l) {
          const uint32_t a = r32(m.s0, l, m.lit) + (uint32_t)m.imm;
          uint64_t x;
          if (a + 8 > lds.size()) throw std::runtime_error("emu: LDS read out of range");
          std::memcpy(&x, lds.data() + a, 8);
          w64v(m.d, l, x);
        }); break;
        case GLOBAL_LOAD_DWORDX2: lanes([&](int l) {
          const uint64_t a = r64(m.s0, l, m.lit) + (uint64_t)(int64_t)m.imm;
          uint64_t x;
          std::memcpy(&x, reinterpret_cast<const void*>(a), 8);
          w64v(m.d, l, x);
        }); break;
        case SCRATCH_LOAD_DWORD: case SCRATCH_STORE_DWORD: case SCRATCH_LOAD_DWORDX2: case SCRATCH_STORE_DWORDX2:
        case SCRATCH_LOAD_DWORDX4: lanes([&](int l) {
          const int n = (m.op == SCRATCH_LOAD_DWORDX4) ? 4
                        : (m.op == SCRATCH_LOAD_DWORDX2 || m.op == SCRATCH_STORE_DWORDX2) ? 2 : 1;
          const size_t a = (size_t)sg[m.s1] + (size_t)m.imm;
          if (scratch[l].size() < a + 4 * n) scratch[l].resize(a + 4 * n + 64);
          for (int k = 0; k < n; ++k) {
            if (m.op == SCRATCH_STORE_DWORD || m.op == SCRATCH_STORE_DWORDX2) {
              const uint32_t x = r32((uint16_t)(m.s2 + k), l, m.lit);
              std::memcpy(scratch[l].data() + a + 4 * k, &x, 4);
            } else {
              uint32_t x;
              std::memcpy(&x, scratch[l].data() + a + 4 * k, 4);
              w32((uint16_t)(m.d + k), l, x);
            }
          }
        }); break;
        // ---- macros
        case M_FDIV64: lanes([&](int l) { w64v(m.d, l, dbits(rf(m.s0, l, m.lit) / rf(m.s1, l, m.lit))); }); break;
        case M_CVT_F64_I64: lanes([&](int l) { w64v(m.d, l, dbits((double)(int64_t)r64(m.s0, l, m.lit))); }); break;
        case M_CVT_I64_F64: lanes([&](int l) {
          const double x = std::trunc(rf(m.s0, l, m.lit));
          w64v(m.d, l, (std::fabs(x) < 9.2233720368547758e18) ? (uint64_t)(int64_t)x : 0x8000000000000000ull);
        }); break;
        case M_RTCALL: {
          const CallInfo& c = f.calls[(size_t)m.ext];
          lanes([&](int l) {
            const int64_t ab = (int64_t)r64(c.a, l, 0);
            const int32_t afl = (int32_t)r32(c.afl, l, 0);
            fksd::Ret2 o;
            if (c.kind == 0) {
              const int64_t bb = (int64_t)r64(c.b, l, 0);
              const int32_t bfl = (int32_t)r32(c.bfl, l, 0);
              o = fksd::d_binop_s(c.op, ab, afl, bb, bfl);
            } else {
              o = fksd::d_unop_s(c.op, ab, afl);
            }
            w64v(c.res, l, (uint64_t)o.x);
            w32(c.resy, l, (uint32_t)o.y);
            if (std::getenv("FKS_EMU_TRACE_RT") && (o.y >> 8) != 0)
              std::fprintf(stderr, "rt kind=%d op=%d a=%016llx afl=%d b=%016llx bfl=%d -> x=%016llx y=%llx\n", c.kind,
                           c.op, (unsigned long long)ab, afl,
                           c.kind == 0 ? (unsigned long long)r64(c.b, l, 0) : 0ull,
                           c.kind == 0 ? (int)r32(c.bfl, l, 0) : 0, (unsigned long long)o.x, (unsigned long long)o.y);
          });
          if (trace_lane >= 0) {
            std::fprintf(stderr, "RTCALL sgprs:");
            for (int x : c.sgprs) std::fprintf(stderr, " %d", x);
            std::fprintf(stderr, " vgprs:");
            for (int x : c.vgprs) std::fprintf(stderr, " %d", x);
            std::fprintf(stderr, " res=%d resy=%d spill=%d\n", c.res - 256, c.resy - 256, c.spill_vgpr - 256);
          }
          // the callee may clobber every caller-saved register: model the ones
          // the spill set does not cover as garbage, so a missing spill shows
          for (int g = 0; g < 128; ++g) {
            const bool cs = g < 40 || ((g - 40) % 16) >= 8;   // v0-39, v48-55, v64-71, ...
            if (!cs) continue;
            if (std::find(c.vgprs.begin(), c.vgprs.end(), g) != c.vgprs.end()) continue;
            if (g == c.res - 256 || g == c.res - 255 || g == c.resy - 256 || g == c.spill_vgpr - 256) continue;
            // (active lanes only: a callee preserves the inactive lanes of every
            // VGPR -- its whole-wave code saves them, see fks_rt_binop's v34)
            for (uint64_t b = ex; b; b &= b - 1) vg[g][__builtin_ctzll(b)] = 0xDEADBEEFu;
          }
          for (int sgi = 0; sgi < 96; ++sgi) {
            const bool cs = sgi < 30 || (sgi >= 40 && ((sgi - 40) % 16) < 8);   // s0-29, s40-47, s56-63, ...
            if (!cs) continue;
            if (std::find(c.sgprs.begin(), c.sgprs.end(), sgi) != c.sgprs.end()) continue;
            sg[sgi] = 0xDEADBEEFu;
          }
          wr64s(VCC, 0xDEADBEEFDEADBEEFull);
          break;
        }
        default:
          throw std::logic_error(std::string("emu: unhandled ") + info(m.op).name);
      }
      if (trace_lane >= 0) {
        std::fprintf(stderr, "%4zu %-22s exec=%d", pc, info(m.op).name, (int)(ex >> trace_lane & 1));
        if (m.d != NONE && m.d >= 256) std::fprintf(stderr, " v%d=%08x", m.d - 256, vg[m.d - 256][trace_lane]);
        else if (m.d != NONE && m.d < 128) std::fprintf(stderr, " s%d=%08x", m.d, sg[m.d]);
        if (m.sd != NONE && m.sd < 128) std::fprintf(stderr, " s%d=%08x:%08x", m.sd, sg[m.sd], sg[m.sd + 1]);
        std::fprintf(stderr, "\n");
      }
      pc = next;
    }
  }
};

}  // namespace gcn
}  // namespace fks
