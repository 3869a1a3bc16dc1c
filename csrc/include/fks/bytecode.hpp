// Policy bytecode ISA shared by the compiler (policy/bytecode.py), the CPU
// VM (csrc/cpu/vm_cpu.hpp) and the device VM (csrc/hip/vm_dev.hip.h).
//
// Execution model: SIMT over nodes.  One program evaluates priority(pod,node)
// for every node of the cluster at once, one LANE per node; the program
// counter is UNIFORM (wave-wide on the device), control flow is structured
// and realised with per-lane masks:
//
//   lane state: off (nesting counter, 0 = enabled), brk, cont, done
//   active  <=>  off == 0 && !brk && !cont && !done
//   IF a    : active && !truthy(a) -> off = 1 ; inactive -> off += 1
//             (if no lane is active afterwards: jump to imm = the ELSE/ENDIF)
//   ELSE    : off == 1 -> 0 ; off == 0 -> 1     (jump to imm = ENDIF if none active)
//   ENDIF   : off > 0 -> off -= 1
//   LOOP_BEGIN d : d = brk | cont<<1 (saved) ; inactive -> off += 1 ; brk = cont = 0
//   LOOP_TEST a  : active && !truthy(a) -> brk = 1 ; jump to imm (LOOP_EXIT) if none active
//   LOOP_CONT    : cont = 0
//   LOOP_NEXT    : jump to imm (the loop's test block)
//   LOOP_EXIT a  : off > 0 -> off -= 1 ; (brk, cont) = saved a
//   BREAK / CONTINUE : active -> brk / cont = 1
//   RET a   : active -> result = a, done = 1
//   END     : active lanes fell off the function: result = None
//
// Every register write and every exception is masked by `active`, so code in
// untaken branches has no effect (Python short-circuit semantics hold).
//
// Values are Python numbers with a per-register runtime tag (int64 / double)
// implementing CPython's int/float rules; GPU lists are packed in one
// register: bits 0-3 length, then 4 bits per GPU index (<= 15 entries).
#pragma once

#include <cstdint>

namespace fks {

struct Insn {
  uint8_t op, d, a, b;
  int32_t imm;
};
static_assert(sizeof(Insn) == 8, "Insn must be 8 bytes");

constexpr int kMaxRegs = 64;
constexpr int kNoReg = 255;
constexpr int kMaxListLen = 15;
// imm of GLIST_GET / LT / ADD in the compiler's GPU-list loop skeletons (policy/bytecode.py LOOP_INDEX)
constexpr int32_t kLoopIndex = 1;

enum Op : uint8_t {
  OP_NOP = 0,
  OP_CONST = 1,       // d = K[imm]
  OP_MOV = 2,         // d = a
  OP_POD = 3,         // d = pod.<imm>
  OP_NODE = 4,        // d = node.<imm>
  OP_GPU = 5,         // d = node.gpus[a].<imm>      (a holds a GPU index)
  OP_GLIST_ALL = 6,   // d = node.gpus
  OP_GLIST_LEN = 7,   // d = len(a)
  OP_GLIST_GET = 8,   // d = a[b]                     (IndexError / TypeError)
  OP_GLIST_SLICE = 9, // d = a[b:imm]  (b / imm = register or kNoReg for None)
  OP_GLIST_NEW = 10,  // d = []
  OP_GLIST_APPEND = 11,  // d = a + [b]
  OP_GLIST_INSERT = 12,  // d = a with b inserted at position reg[imm] (list.insert)

  OP_ADD = 20, OP_SUB = 21, OP_MUL = 22, OP_TDIV = 23, OP_FDIV = 24, OP_MOD = 25, OP_POW = 26,
  OP_NEG = 27, OP_POS = 28, OP_NOT = 29, OP_TRUTH = 30,
  OP_LT = 31, OP_LE = 32, OP_GT = 33, OP_GE = 34, OP_EQ = 35, OP_NE = 36,

  OP_ABS = 40, OP_INT = 41, OP_FLOAT = 42, OP_ROUND = 43, OP_MIN2 = 44, OP_MAX2 = 45,
  OP_SQRT = 46, OP_LOG = 47, OP_LOGB = 48, OP_EXP = 49, OP_MPOW = 50,
  OP_SIN = 51, OP_COS = 52, OP_TAN = 53,

  OP_IF = 60, OP_ELSE = 61, OP_ENDIF = 62,
  OP_LOOP_BEGIN = 63, OP_LOOP_TEST = 64, OP_LOOP_CONT = 65, OP_LOOP_NEXT = 66, OP_LOOP_EXIT = 67,
  OP_BREAK = 68, OP_CONTINUE = 69,
  OP_RET = 70,
  OP_RAISE = 71,      // raise exception class imm (ExcCode)
  OP_END = 72,
  OP_ISINT = 73,     // d = 1 if a holds an int else 0
};

// pod fields (OP_POD imm)
enum PodField : int32_t { PF_CPU = 0, PF_MEM = 1, PF_NGPU = 2, PF_GMILLI = 3, PF_CTIME = 4, PF_DUR = 5 };
// node fields (OP_NODE imm)
enum NodeField : int32_t {
  NF_CPU_LEFT = 0, NF_CPU_TOTAL = 1, NF_MEM_LEFT = 2, NF_MEM_TOTAL = 3, NF_GPU_LEFT = 4, NF_NGPUS = 5
};
// gpu fields (OP_GPU imm)
enum GpuField : int32_t { GF_MILLI_LEFT = 0, GF_MILLI_TOTAL = 1, GF_MEM_LEFT = 2, GF_MEM_TOTAL = 3 };

// Constant-pool tags
enum ConstTag : uint8_t { TAG_INT = 0, TAG_FLOAT = 1 };

}  // namespace fks
