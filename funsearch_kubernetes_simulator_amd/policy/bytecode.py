"""Opcode table of the policy bytecode (mirror of csrc/include/fks/bytecode.hpp).

`tests/test_compiler.py` parses the C++ header and checks that every value
here matches, so the Python compiler and both interpreters can never drift.
"""

from __future__ import annotations

import enum
import struct


class Op(enum.IntEnum):
    NOP = 0
    CONST = 1
    MOV = 2
    POD = 3
    NODE = 4
    GPU = 5
    GLIST_ALL = 6
    GLIST_LEN = 7
    GLIST_GET = 8
    GLIST_SLICE = 9
    GLIST_NEW = 10
    GLIST_APPEND = 11
    GLIST_INSERT = 12
    ADD = 20
    SUB = 21
    MUL = 22
    TDIV = 23
    FDIV = 24
    MOD = 25
    POW = 26
    NEG = 27
    POS = 28
    NOT = 29
    TRUTH = 30
    LT = 31
    LE = 32
    GT = 33
    GE = 34
    EQ = 35
    NE = 36
    ABS = 40
    INT = 41
    FLOAT = 42
    ROUND = 43
    MIN2 = 44
    MAX2 = 45
    SQRT = 46
    LOG = 47
    LOGB = 48
    EXP = 49
    MPOW = 50
    SIN = 51
    COS = 52
    TAN = 53
    IF = 60
    ELSE = 61
    ENDIF = 62
    LOOP_BEGIN = 63
    LOOP_TEST = 64
    LOOP_CONT = 65
    LOOP_NEXT = 66
    LOOP_EXIT = 67
    BREAK = 68
    CONTINUE = 69
    RET = 70
    RAISE = 71
    END = 72
    ISINT = 73


POD_FIELDS = {"cpu_milli": 0, "memory_mib": 1, "num_gpu": 2, "gpu_milli": 3,
              "creation_time": 4, "duration_time": 5}
NODE_FIELDS = {"cpu_milli_left": 0, "cpu_milli_total": 1, "memory_mib_left": 2,
               "memory_mib_total": 3, "gpu_left": 4}
NODE_NGPUS = 5  # len(node.gpus)
GPU_FIELDS = {"gpu_milli_left": 0, "gpu_milli_total": 1, "memory_mib_left": 2, "memory_mib_total": 3}

TAG_INT, TAG_FLOAT = 0, 1
MAX_REGS = 64
NO_REG = 255
MAX_LIST_LEN = 15
#: `imm` of GLIST_GET / LT / ADD in the compiler's own GPU-list loop skeletons
#: (hidden list snapshot, length and counter): the counter runs 0 .. len-1, so
#: the GET is in range, the LT compares two ints in [0, 15] and the ADD is
#: counter + 1 <= 15.  Interpreters ignore it (their checks pass anyway); the
#: baseline JIT drops the checks, and when the list is ``node.gpus`` unchanged
#: indexes the GPU fields with the counter (uniform across the lanes in the loop).
LOOP_INDEX = 1


class Exc(enum.IntEnum):
    """Mirror of fks::ExcCode (csrc/include/fks/types.hpp)."""
    NONE = 0
    ZERO_DIVISION = 1
    VALUE = 2
    OVERFLOW = 3
    TYPE = 4
    INDEX = 5
    ALLOC = 6
    NAME = 7
    UNSUPPORTED = 100
    BUDGET = 101
    INVARIANT = 102
    TIMEOUT = 103
    EVENTS = 104        # the replay passed the caller's event budget (a resource limit): not scored


_INSN = struct.Struct("<BBBBi")


def pack_insn(op: int, d: int = NO_REG, a: int = NO_REG, b: int = NO_REG, imm: int = 0) -> bytes:
    return _INSN.pack(int(op), d, a, b, imm)


def unpack_code(code: bytes):
    return [_INSN.unpack_from(code, i) for i in range(0, len(code), _INSN.size)]


def disassemble(code: bytes) -> str:
    lines = []
    for pc, (op, d, a, b, imm) in enumerate(unpack_code(code)):
        regs = ", ".join(f"r{x}" for x in (d, a, b) if x != NO_REG)
        lines.append(f"{pc:4d}  {Op(op).name:<13} {regs}{'' if not imm else f'  #{imm}'}")
    return "\n".join(lines)
