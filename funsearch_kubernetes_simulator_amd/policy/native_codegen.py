"""Native program backend: policy bytecode -> per-lane C++ (SURVEY section 7.1 backend B).

The bytecode (`policy.compiler`) is a SIMT program: one uniform program
counter, per-lane masks for structured control flow.  Per lane that is plain
sequential execution, so each program lowers to an ordinary C++ function that
scores ONE (pod, node) pair -- `if` / loops become real branches (the GPU's
exec mask handles divergence between the nodes of a wave), virtual registers
become locals the compiler keeps in VGPRs, and every operation follows the
same Python-number rules as the VMs (`csrc/hip/pyops_dev.h`, executable spec
`csrc/include/fks/pyops.hpp`).  Results are bit-identical to the VMs and to
the reference (`funsearch/funsearch_integration.py:91-101`): CPython int/float
rules, exceptions -> the replay's exception code, ``int(max(0, s))`` applied
on return.

Speed (of the compile and of the code):

* a forward type analysis over the bytecode's control-flow graph proves most
  registers int-only or float-only at each use, so arithmetic and compares are
  emitted for the static types (no tag tests); only genuinely mixed uses keep
  the tagged path;
* the float ``//`` / ``%`` / ``**``, ``math.log/exp/sqrt/pow`` machinery is not
  compiled per program: the generated code calls the runtime copies inside the
  precompiled extension (``rt_binop`` / ``rt_unop``, jit_abi.h) through a table
  the loader fills in;
* numeric constants are data (``kc[1 + i]``), not code: programs that differ
  only in constants -- most offline mutations, and every member of a
  constant-polish sweep -- share one compiled function ("shape").

Control-flow mapping (bytecode pcs become labels):

* ``IF a -> t``        false: ``goto L(t+1)`` (t is the ELSE or the ENDIF)
* ``ELSE -> e``        ``goto L(e)`` (the then-branch skips the else-branch)
* ``LOOP_TEST a -> x`` false: ``goto L(x)`` (x = LOOP_EXIT)
* ``LOOP_NEXT -> h``   back edge to the loop's test block, with an iteration budget
* ``BREAK``            ``goto`` the innermost loop's LOOP_EXIT
* ``CONTINUE``         ``goto`` the next LOOP_CONT of the innermost loop
* ``RET a`` / ``RAISE e`` / ``END`` leave the function.
"""

from __future__ import annotations

import hashlib
import math
import struct
from typing import Dict, List, Sequence, Tuple

import numpy as np

from .bytecode import NO_REG, TAG_FLOAT, Op, unpack_code
from .compiler import CompiledPolicy

#: parameter list shared by every generated program (keep in sync with jit_abi.h ProgFn)
#: (31 argument dwords: v0-v30 -- v31 carries the work-item ids, so a 32nd
#: dword would travel through the stack, i.e. a scratch store + load per call;
#: the node's free-GPU count and GPU count share one dword)
PROG_PARAMS = ("int32_t n_cpu_left, int32_t n_cpu_total, int32_t n_mem_left, int32_t n_mem_total, "
               "int32_t n_gpu_ng, "
               "int32_t gl0, int32_t gl1, int32_t gl2, int32_t gl3, int32_t gl4, int32_t gl5, int32_t gl6, "
               "int32_t gl7, int32_t gt0, int32_t gt1, int32_t gt2, int32_t gt3, int32_t gt4, int32_t gt5, "
               "int32_t gt6, int32_t gt7, const int64_t* gmem, "
               "int32_t p_cpu, int32_t p_mem, int32_t p_gpu, int64_t p_ctime, int32_t p_dur, KcPtr kc")
#: constant-block entries the replay kernels stage in LDS per policy (jit_abi.h kKcLds)
KC_LDS = 256

I, F = 1, 2          # type lattice bits: may be int / may be float
IF_ = I | F

_POD = {0: "p_cpu", 1: "p_mem", 2: "(p_gpu >> 16)", 3: "(p_gpu & 0xFFFF)", 4: "p_ctime", 5: "p_dur"}
_NODE = {0: "n_cpu_left", 1: "n_cpu_total", 2: "n_mem_left", 3: "n_mem_total", 4: "n_gpu_left", 5: "n_ngpus"}
_OPNAME = {Op.FDIV: "OP_FDIV", Op.MOD: "OP_MOD", Op.POW: "OP_POW", Op.LOGB: "OP_LOGB", Op.MPOW: "OP_MPOW",
           Op.NEG: "OP_NEG", Op.POS: "OP_POS", Op.ABS: "OP_ABS", Op.INT: "OP_INT", Op.ROUND: "OP_ROUND",
           Op.SQRT: "OP_SQRT", Op.LOG: "OP_LOG", Op.EXP: "OP_EXP", Op.SIN: "OP_SIN", Op.COS: "OP_COS",
           Op.TAN: "OP_TAN"}
_RT_BIN = {Op.POW, Op.LOGB, Op.MPOW}
_RT_UN = {Op.SQRT, Op.LOG, Op.EXP, Op.SIN, Op.COS, Op.TAN}
_CMP_C = {Op.LT: "<", Op.LE: "<=", Op.GT: ">", Op.GE: ">=", Op.EQ: "==", Op.NE: "!="}
_CMP_C3 = {Op.LT: "c_ == -1", Op.LE: "(c_ == -1 || c_ == 0)", Op.GT: "c_ == 1", Op.GE: "(c_ == 1 || c_ == 0)",
           Op.EQ: "c_ == 0", Op.NE: "c_ != 0"}
_ARITH = {Op.ADD: ("__builtin_add_overflow", "+"), Op.SUB: ("__builtin_sub_overflow", "-"),
          Op.MUL: ("mul_ovf", "*")}
_INT_RESULT = {Op.POD, Op.NODE, Op.GPU, Op.GLIST_ALL, Op.GLIST_LEN, Op.GLIST_GET, Op.GLIST_SLICE, Op.GLIST_NEW,
               Op.GLIST_APPEND, Op.GLIST_INSERT, Op.NOT, Op.TRUTH, Op.ISINT, Op.LT, Op.LE, Op.GT, Op.GE, Op.EQ,
               Op.NE, Op.INT, Op.ROUND, Op.LOOP_BEGIN}
_FLOAT_RESULT = {Op.TDIV, Op.FLOAT, Op.SQRT, Op.LOG, Op.LOGB, Op.EXP, Op.MPOW, Op.SIN, Op.COS, Op.TAN}


class CodegenError(ValueError):
    """The bytecode has a shape the native backend does not lower."""


def data_literal(tag: int, fval: float, ival: int) -> bool:
    """A source literal kept as run-time data (read from the constant block):
    the values constant polish tunes (funsearch/polish.py tunable_literals) --
    ints of magnitude >= 2, finite nonzero floats.  0, +-1, 0.0 and non-finite
    literals are compiled in as immediates instead (no dependent LDS read per
    use) and, like compiler-generated constants, are part of the shape key."""
    if tag == TAG_FLOAT:
        return fval != 0.0 and math.isfinite(fval)
    return abs(int(ival)) >= 2


def _literal_slots(prog: CompiledPolicy) -> set:
    """Pool entries read from the constant block at run time (the data of a
    shape); the rest -- compiler-generated constants (loop start / step, ...)
    and the literals data_literal() pins -- are immediates in the code."""
    return {k for k in (int(lit[0]) for lit in getattr(prog, "literals", ()) or ())
            if data_literal(int(prog.ctag[k]), float(prog.fconst[k]), int(prog.iconst[k]))}


def _all_list_at(code, flow) -> List[set]:
    """Must-analysis over the bytecode CFG: for every pc, the registers that hold
    ``node.gpus`` unchanged on every path reaching it (defined by GLIST_ALL, or a
    MOV of such a register, and not overwritten since).  For those lists an
    element is its own index and the length is the GPU count, so ``for g in
    node.gpus`` loops index the GPU fields with the (wave-uniform) loop counter
    instead of unpacking the 4-bit list."""
    n = len(code)
    succ: List[List[int]] = []
    for pc, (op, d, a, b, imm) in enumerate(code):
        if op == Op.IF:
            nxt = [pc + 1, imm + 1]
        elif op in (Op.ELSE, Op.LOOP_NEXT):
            nxt = [imm]
        elif op == Op.LOOP_TEST:
            nxt = [pc + 1, imm]
        elif op == Op.BREAK:
            nxt = [flow["break"][pc]]
        elif op == Op.CONTINUE:
            nxt = [flow["continue"][pc]]
        elif op in (Op.RET, Op.RAISE, Op.END):
            nxt = []
        else:
            nxt = [pc + 1]
        succ.append([x for x in nxt if 0 <= x < n])
    TOP = None   # "every register" (not yet reached)
    state_in: List[object] = [TOP] * n
    state_in[0] = frozenset()
    work = [0]
    while work:
        pc = work.pop()
        cur = state_in[pc]
        op, d, a, b, imm = code[pc]
        out = set(cur)
        if d != NO_REG:
            if op == Op.GLIST_ALL or (op == Op.MOV and a in cur):
                out.add(d)
            else:
                out.discard(d)
        out = frozenset(out)
        for t in succ[pc]:
            old = state_in[t]
            new = out if old is TOP else (old & out)
            if new != old:
                state_in[t] = new
                work.append(t)
    return [set() if x is TOP else set(x) for x in state_in]


def _inline_constants(prog: CompiledPolicy) -> List[Tuple[int, int, float, int]]:
    lits = _literal_slots(prog)
    return [(k, int(prog.ctag[k]), float(prog.fconst[k]), int(prog.iconst[k])) for k in range(len(prog.ctag))
            if k not in lits]


def shape_key(prog: CompiledPolicy) -> str:
    """Programs with equal keys share one compiled function: source literals are
    data (read from the constant block), so programs that differ only in them
    share a shape; compiler-generated constants are immediates in the code and
    part of the key.  Cached on the program."""
    v = prog.__dict__.get("_shape_key")
    if v is None:
        v = prog.__dict__["_shape_key"] = _shape_key_uncached(prog)
    return v


def _shape_key_uncached(prog: CompiledPolicy) -> str:
    h = hashlib.sha1(b"imm-literals-1")
    h.update(prog.code)
    h.update(bytes(prog.ctag))
    h.update(repr(_inline_constants(prog)).encode())
    return h.hexdigest()


def constant_payload(prog: CompiledPolicy) -> np.ndarray:
    """The constant payloads of one program as int64 (float constants as their
    bits), in pool order -- cached on the program (a producer process fills
    the cache before the program is pickled to the dispatcher)."""
    v = prog.__dict__.get("_kc")   # (bytes: pickles in a fraction of an array's time)
    if v is None:
        n = len(prog.ctag)
        tags = np.asarray(prog.ctag, dtype=np.uint8).reshape(n)
        f = np.asarray(prog.fconst, dtype=np.float64).reshape(n).view(np.int64)
        i = np.asarray(prog.iconst, dtype=np.int64).reshape(n)
        v = prog.__dict__["_kc"] = np.where(tags == TAG_FLOAT, f, i).astype(np.int64).tobytes()
    return np.frombuffer(v, dtype=np.int64)


def constant_block(prog: CompiledPolicy, budget: int) -> np.ndarray:
    """``kc`` of one program: [budget, constant payloads...] as int64 (float bits)."""
    kc = constant_payload(prog)
    out = np.empty(1 + kc.size, dtype=np.int64)
    out[0] = budget
    out[1:] = kc
    return out


def constant_blocks(progs: Sequence[CompiledPolicy], budget: int) -> Tuple[np.ndarray, np.ndarray]:
    """(kc, koff) of a batch: every program's `constant_block`, concatenated,
    and the offset of each -- one numpy concatenation instead of a loop over
    the constants of every program."""
    P = len(progs)
    if not P:
        return np.zeros(1, np.int64), np.zeros(0, np.int32)
    head = np.array([budget], dtype=np.int64)
    parts = []
    lens = np.empty(P, dtype=np.int64)
    for j, p in enumerate(progs):
        kc = constant_payload(p)
        parts.append(head)
        parts.append(kc)
        lens[j] = 1 + kc.size
    koff = np.zeros(P, dtype=np.int64)
    np.cumsum(lens[:-1], out=koff[1:])
    return np.concatenate(parts), koff.astype(np.int32)


# ---------------------------------------------------------------------------- analysis
def _loop_structure(code) -> Dict[str, Dict[int, int]]:
    """For every BREAK / CONTINUE: its jump target; checks the nesting."""
    stack: List[int] = []
    exit_of: Dict[int, int] = {}
    conts: Dict[int, List[int]] = {}
    pend_b: Dict[int, int] = {}
    pend_c: Dict[int, int] = {}
    for pc, (op, d, a, b, imm) in enumerate(code):
        if op == Op.LOOP_BEGIN:
            stack.append(pc)
            conts[pc] = []
        elif op == Op.LOOP_EXIT:
            if not stack:
                raise CodegenError(f"LOOP_EXIT without LOOP_BEGIN at {pc}")
            exit_of[stack.pop()] = pc
        elif op == Op.LOOP_CONT:
            if not stack:
                raise CodegenError(f"LOOP_CONT outside a loop at {pc}")
            conts[stack[-1]].append(pc)
        elif op in (Op.BREAK, Op.CONTINUE):
            if not stack:
                raise CodegenError(f"{Op(op).name} outside a loop at {pc}")
            (pend_b if op == Op.BREAK else pend_c)[pc] = stack[-1]
    if stack:
        raise CodegenError("unterminated loop")
    cont = {}
    for pc, lp in pend_c.items():
        nxt = [c for c in conts[lp] if c > pc]
        if not nxt:
            raise CodegenError(f"CONTINUE at {pc} has no following LOOP_CONT")
        cont[pc] = nxt[0]
    return {"break": {pc: exit_of[lp] for pc, lp in pend_b.items()}, "continue": cont}


def _successors(code, flow) -> List[Tuple[int, ...]]:
    n = len(code)
    succ = []
    for pc, (op, d, a, b, imm) in enumerate(code):
        if op == Op.IF:
            s = (pc + 1, imm + 1)
        elif op in (Op.ELSE, Op.LOOP_NEXT):
            s = (imm,)
        elif op == Op.LOOP_TEST:
            s = (pc + 1, imm)
        elif op == Op.BREAK:
            s = (flow["break"][pc],)
        elif op == Op.CONTINUE:
            s = (flow["continue"][pc],)
        elif op in (Op.RET, Op.RAISE, Op.END):
            s = ()
        else:
            s = (pc + 1,)
        for t in s:
            if not 0 <= t < n:
                raise CodegenError(f"jump target {t} out of range at {pc}")
        succ.append(s)
    return succ


def _result_type(op, ta: int, tb: int, ctag_t: int) -> int:
    if op == Op.CONST:
        return ctag_t
    if op == Op.MOV or op == Op.POS:
        return ta
    if op in _INT_RESULT:
        return I
    if op in _FLOAT_RESULT:
        return F
    if op in (Op.ADD, Op.SUB, Op.MUL, Op.FDIV, Op.MOD):
        return (I if (ta & I and tb & I) else 0) | (F if (ta & F or tb & F) else 0)
    if op == Op.POW:   # int ** negative int -> float
        return ((I | F) if (ta & I and tb & I) else 0) | (F if (ta & F or tb & F) else 0)
    if op in (Op.NEG, Op.ABS):
        return ta
    if op in (Op.MIN2, Op.MAX2):
        return ta | tb
    return 0


def infer_types(code, flow, ctag) -> List[Dict[int, int]]:
    """Type lattice state (register -> I/F bits) on entry to every pc."""
    n = len(code)
    succ = _successors(code, flow)
    state: List[Dict[int, int]] = [None] * n  # type: ignore[list-item]
    state[0] = {}
    work = [0]
    on = {0}
    while work:
        pc = work.pop()
        on.discard(pc)
        st = state[pc]
        op, d, a, b, imm = code[pc]
        get = lambda r: st.get(r, I)     # registers start as int 0
        out = st
        if d != NO_REG and op not in (Op.IF, Op.ELSE, Op.LOOP_TEST, Op.LOOP_NEXT, Op.RET, Op.RAISE, Op.END,
                                      Op.LOOP_EXIT):
            ct = (F if ctag[imm] == TAG_FLOAT else I) if op == Op.CONST else 0
            t = _result_type(Op(op), get(a) if a != NO_REG else I, get(b) if b != NO_REG else I, ct)
            if t == 0:
                t = IF_
            out = dict(st)
            out[d] = t
        for s in succ[pc]:
            cur = state[s]
            if cur is None:
                state[s] = dict(out)
                changed = True
            else:
                changed = False
                for r, t in out.items():
                    u = cur.get(r, I) | t
                    if u != cur.get(r, I):
                        cur[r] = u
                        changed = True
                for r in list(cur):
                    if r not in out:
                        u = cur[r] | I
                        if u != cur[r]:
                            cur[r] = u
                            changed = True
            if changed and s not in on:
                work.append(s)
                on.add(s)
    return [s if s is not None else {} for s in state]


# ---------------------------------------------------------------------------- emission
def program_source(prog: CompiledPolicy, name: str, lift_consts: bool = True) -> str:
    """C++ of one program: ``extern "C" int64_t name(PROG_PARAMS)``."""
    if lift_consts and 1 + len(prog.ctag) > KC_LDS:
        raise CodegenError(f"{len(prog.ctag)} constants > {KC_LDS - 1} (the LDS constant block)")
    code = unpack_code(prog.code)
    literal_slots = _literal_slots(prog)
    flow = _loop_structure(code)
    all_lists_at = _all_list_at(code, flow)
    types = infer_types(code, flow, prog.ctag)
    regs = set()
    for op, d, a, b, imm in code:
        if op in (Op.LOOP_BEGIN, Op.LOOP_EXIT):
            continue
        for r in (d, a, b):
            if r != NO_REG:
                regs.add(r)
        if op in (Op.GLIST_SLICE, Op.GLIST_INSERT) and imm != NO_REG:
            regs.add(imm)
    targets = set()
    for pc, (op, d, a, b, imm) in enumerate(code):
        if op == Op.IF:
            targets.add(imm + 1)
        elif op in (Op.ELSE, Op.LOOP_TEST, Op.LOOP_NEXT):
            targets.add(imm)
    targets.update(flow["break"].values())
    targets.update(flow["continue"].values())

    out: List[str] = []
    w = out.append
    w(f'extern "C" __device__ __noinline__ int64_t {name}({PROG_PARAMS}) {{')
    if regs:
        w("  PyN " + ", ".join(f"r{r} = pi(0)" for r in sorted(regs)) + ";")
    w("  PyN res_ = pi(0);")
    w("  int exc_ = EXC_NONE;")
    w("  int64_t bud_ = kc[0];")
    w("  (void)bud_; (void)gmem;")
    w("  const int32_t n_gpu_left = (int16_t)(n_gpu_ng & 0xFFFF), n_ngpus = n_gpu_ng >> 16;")
    w("  (void)n_gpu_left; (void)n_ngpus;")

    def R(r: int) -> str:
        if r == NO_REG:
            raise CodegenError("missing register operand")
        return f"r{r}"

    def RAISE(e: str) -> str:
        # "soft" raise: remember the FIRST exception and keep going (no branch:
        # later results are discarded, loops stop at their back edge, RET and the
        # end check exc_) -- far fewer basic blocks, so shorter compiles and no
        # divergence on the common no-exception path
        return f"{{ exc_ = exc_ ? exc_ : ({e}); }}"

    def HARD_RAISE(e: str) -> str:
        return f"{{ exc_ = exc_ ? exc_ : ({e}); goto L_done; }}"

    for pc, (op, d, a, b, imm) in enumerate(code):
        if pc in targets:
            w(f" L{pc}:;")
        op = Op(op)
        st = types[pc]
        ta = st.get(a, I) if a != NO_REG else I
        tb = st.get(b, I) if b != NO_REG else I

        def iv(r):   # int value of a statically int register
            return f"{R(r)}.b"

        def dv(r, t):   # double value of a register of static type t
            if t == I:
                return f"(double){R(r)}.b"
            if t == F:
                return f"__longlong_as_double({R(r)}.b)"
            return f"fv({R(r)})"

        def truth(r, t):
            if t == I:
                return f"({R(r)}.b != 0)"
            if t == F:
                return f"(__longlong_as_double({R(r)}.b) != 0.0)"
            return f"truthy({R(r)})"

        if op in (Op.NOP, Op.ENDIF, Op.LOOP_BEGIN, Op.LOOP_CONT, Op.LOOP_EXIT):
            continue
        if op == Op.CONST:
            fl = prog.ctag[imm] == TAG_FLOAT
            # source literals come from the constant block; compiler-generated
            # constants (loop start / step, ...) are immediates the optimiser sees
            if lift_consts and imm in literal_slots:
                w(f"  {R(d)} = PyN{{kc[{1 + imm}], {'true' if fl else 'false'}}};")
            elif fl:
                bits = struct.unpack("<q", struct.pack("<d", prog.fconst[imm]))[0]
                w(f"  {R(d)} = PyN{{(int64_t){bits}LL, true}};")
            else:
                v = int(prog.iconst[imm])
                w(f"  {R(d)} = pi({'INT64_MIN' if v == -(1 << 63) else f'(int64_t){v}LL'});")
        elif op == Op.MOV:
            if d != a:
                w(f"  {R(d)} = {R(a)};")
        elif op == Op.POD:
            w(f"  {R(d)} = pi((int64_t){_POD.get(imm, 'p_dur')});")
        elif op == Op.NODE:
            w(f"  {R(d)} = pi((int64_t){_NODE.get(imm, 'n_ngpus')});")
        elif op == Op.GPU:
            j = f"(int)({R(a)}.b & 0xF)"
            if imm == 0:
                w(f"  {R(d)} = pi((int64_t)sel8({j}, gl0, gl1, gl2, gl3, gl4, gl5, gl6, gl7));")
            elif imm == 1:
                w(f"  {R(d)} = pi((int64_t)sel8({j}, gt0, gt1, gt2, gt3, gt4, gt5, gt6, gt7));")
            else:
                w(f"  {R(d)} = pi(gmem[{j}]);")
        elif op == Op.GLIST_ALL:
            w(f"  {R(d)} = pi(glist_all(n_ngpus));")
        elif op == Op.GLIST_LEN:
            if a in all_lists_at[pc]:
                w(f"  {R(d)} = pi((int64_t)n_ngpus);")
            else:
                w(f"  {R(d)} = pi({R(a)}.b & 0xF);")
        elif op == Op.GLIST_GET:
            if a in all_lists_at[pc]:   # node.gpus[i] is GPU i (glist_get's checks, no unpacking)
                w(f"  if ({R(b)}.fl) {RAISE('EXC_TYPE')} else {{ const int64_t k_ = {R(b)}.b < 0 ? {R(b)}.b + n_ngpus : "
                  f"{R(b)}.b; if (k_ < 0 || k_ >= n_ngpus) {RAISE('EXC_INDEX')} else {R(d)} = pi(k_); }}")
            else:
                w(f"  {{ const int e_ = glist_get({R(a)}, {R(b)}, {R(d)}); if (e_) {RAISE('e_')} }}")
        elif op == Op.GLIST_SLICE:
            lo = R(b) if b != NO_REG else "pi(0)"
            hi = R(imm) if imm != NO_REG else "pi(0)"
            w(f"  {{ const int e_ = glist_slice({R(a)}, {lo}, {int(b != NO_REG)}, {hi}, {int(imm != NO_REG)}, {R(d)});"
              f" if (e_) {RAISE('e_')} }}")
        elif op == Op.GLIST_NEW:
            w(f"  {R(d)} = pi(0);")
        elif op == Op.GLIST_APPEND:
            w(f"  {{ const int e_ = glist_append({R(a)}, {R(b)}, {R(d)}); if (e_) {RAISE('e_')} }}")
        elif op == Op.GLIST_INSERT:
            w(f"  {{ const int e_ = glist_insert({R(a)}, {R(b)}, {R(imm)}, {R(d)}); if (e_) {RAISE('e_')} }}")
        elif op in _ARITH:
            fn, sym = _ARITH[op]
            if ta == I and tb == I:
                w(f"  {{ int64_t v_; if ({fn}({iv(a)}, {iv(b)}, &v_)) {RAISE('EXC_UNSUPPORTED')} {R(d)} = pi(v_); }}")
            elif ta != IF_ and tb != IF_:
                w(f"  {R(d)} = pf({dv(a, ta)} {sym} {dv(b, tb)});")
            else:
                w(f"  {{ const PyN x_ = {R(a)}, y_ = {R(b)};"
                  f" if (!x_.fl && !y_.fl) {{ int64_t v_; if ({fn}(x_.b, y_.b, &v_)) {RAISE('EXC_UNSUPPORTED')}"
                  f" {R(d)} = pi(v_); }} else {R(d)} = pf(fv(x_) {sym} fv(y_)); }}")
        elif op == Op.TDIV:
            if ta == I and tb == I:
                w(f"  {{ const int64_t x_ = {iv(a)}, y_ = {iv(b)}; if (y_ == 0) {RAISE('EXC_ZERO_DIVISION')}"
                  f" if (x_ > kTwo53i || x_ < -kTwo53i || y_ > kTwo53i || y_ < -kTwo53i) {RAISE('EXC_UNSUPPORTED')}"
                  f" {R(d)} = pf((double)x_ / (double)y_); }}")
            elif ta != IF_ and tb != IF_:
                w(f"  {{ const double q_ = {dv(b, tb)}; if (q_ == 0.0) {RAISE('EXC_ZERO_DIVISION')}"
                  f" {R(d)} = pf({dv(a, ta)} / q_); }}")
            else:
                w(f"  {{ const PyN x_ = {R(a)}, y_ = {R(b)};"
                  f" const bool big_ = !x_.fl && !y_.fl && (x_.b > kTwo53i || x_.b < -kTwo53i || y_.b > kTwo53i || y_.b < -kTwo53i);"
                  f" const double q_ = fv(y_); if (q_ == 0.0) {RAISE('EXC_ZERO_DIVISION')}"
                  f" if (big_) {RAISE('EXC_UNSUPPORTED')} {R(d)} = pf(fv(x_) / q_); }}")
        elif op in (Op.FDIV, Op.MOD):
            fast = "int_floordiv" if op == Op.FDIV else "int_mod"
            if ta == I and tb == I:
                w(f"  {{ PyN t_ = pi(0); const int e_ = {fast}({iv(a)}, {iv(b)}, t_); if (e_) {RAISE('e_')} {R(d)} = t_; }}")
            else:
                w(f"  {{ const PyN x_ = {R(a)}, y_ = {R(b)}; PyN t_ = pi(0); int e_;"
                  f" if (!x_.fl && !y_.fl) e_ = {fast}(x_.b, y_.b, t_);"
                  f" else {{ const PyR o_ = rt_binop({_OPNAME[op]}, x_, y_); e_ = o_.e; t_ = PyN{{o_.b, o_.fl != 0}}; }}"
                  f" if (e_) {RAISE('e_')} {R(d)} = t_; }}")
        elif op in _RT_BIN:
            w(f"  {{ const PyR o_ = rt_binop({_OPNAME[op]}, {R(a)}, {R(b)});"
              f" if (o_.e) {RAISE('o_.e')} {R(d)} = PyN{{o_.b, o_.fl != 0}}; }}")
        elif op in _RT_UN:
            w(f"  {{ const PyR o_ = rt_unop({_OPNAME[op]}, {R(a)});"
              f" if (o_.e) {RAISE('o_.e')} {R(d)} = PyN{{o_.b, o_.fl != 0}}; }}")
        elif op == Op.NOT:
            w(f"  {R(d)} = pi({truth(a, ta)} ? 0 : 1);")
        elif op == Op.TRUTH:
            w(f"  {R(d)} = pi({truth(a, ta)} ? 1 : 0);")
        elif op == Op.ISINT:
            if ta == IF_:
                w(f"  {R(d)} = pi({R(a)}.fl ? 0 : 1);")
            else:
                w(f"  {R(d)} = pi({1 if ta == I else 0});")
        elif op == Op.FLOAT:
            w(f"  {R(d)} = pf({dv(a, ta)});")
        elif op == Op.POS:
            if d != a:
                w(f"  {R(d)} = {R(a)};")
        elif op in (Op.NEG, Op.ABS) and ta != IF_:
            if ta == I:
                expr = f"-{iv(a)}" if op == Op.NEG else f"({iv(a)} < 0 ? -{iv(a)} : {iv(a)})"
                w(f"  {{ if ({iv(a)} == INT64_MIN) {RAISE('EXC_UNSUPPORTED')} {R(d)} = pi({expr}); }}")
            else:
                expr = f"-{dv(a, F)}" if op == Op.NEG else f"fabs({dv(a, F)})"
                w(f"  {R(d)} = pf({expr});")
        elif op in (Op.INT, Op.ROUND) and ta == I:
            if d != a:
                w(f"  {R(d)} = {R(a)};")
        elif op in _OPNAME:   # NEG / ABS / INT / ROUND with float or mixed operands: shared inline helper
            w(f"  {{ PyN t_ = pi(0); const int e_ = d_unop_impl({_OPNAME[op]}, {R(a)}, t_);"
              f" if (e_) {RAISE('e_')} {R(d)} = t_; }}")
        elif op in _CMP_C:
            if ta == I and tb == I:
                w(f"  {R(d)} = pi({iv(a)} {_CMP_C[op]} {iv(b)} ? 1 : 0);")
            elif ta == F and tb == F:   # IEEE compares have Python's NaN behaviour
                w(f"  {R(d)} = pi({dv(a, F)} {_CMP_C[op]} {dv(b, F)} ? 1 : 0);")
            else:
                w(f"  {{ const int c_ = d_cmp({R(a)}, {R(b)}); {R(d)} = pi({_CMP_C3[op]} ? 1 : 0); }}")
        elif op in (Op.MIN2, Op.MAX2):
            # max(x, y): y replaces x only if y > x (min: y < x); NaNs never replace
            rel = ">" if op == Op.MAX2 else "<"
            # (field-wise selects: a ?: of two structs leaves them in scratch memory)
            if ta == I and tb == I:
                cond = f"{iv(b)} {rel} {iv(a)}"
            elif ta == F and tb == F:
                cond = f"{dv(b, F)} {rel} {dv(a, F)}"
            else:
                cond = f"d_cmp({R(b)}, {R(a)}) == {'1' if op == Op.MAX2 else '-1'}"
            w(f"  {{ const bool t_ = {cond}; const PyN x_ = {R(a)}, y_ = {R(b)};"
              f" {R(d)} = PyN{{t_ ? y_.b : x_.b, t_ ? y_.fl : x_.fl}}; }}")
        elif op == Op.IF:
            w(f"  if (!{truth(a, ta)}) goto L{imm + 1};")
        elif op == Op.ELSE:
            w(f"  goto L{imm};")
        elif op == Op.LOOP_TEST:
            w(f"  if (!{truth(a, ta)}) goto L{imm};")
        elif op == Op.LOOP_NEXT:
            w(f"  if (exc_) goto L_done; if (--bud_ < 0) {HARD_RAISE('EXC_BUDGET')} goto L{imm};")
        elif op == Op.BREAK:
            w(f"  goto L{flow['break'][pc]};")
        elif op == Op.CONTINUE:
            w(f"  goto L{flow['continue'][pc]};")
        elif op == Op.RET:
            w(f"  res_ = {R(a)}; goto L_ret;")
        elif op == Op.RAISE:
            w(f"  {HARD_RAISE(str(int(imm)))}")
        elif op == Op.END:
            w(f"  {HARD_RAISE('EXC_TYPE')}")   # fell off the function: returned None
        else:
            raise CodegenError(f"opcode {op.name} has no native lowering")
    w(" L_ret:")
    w("  if (exc_) return -(int64_t)exc_;")
    w("  return finish_score(res_);")
    w(" L_done:")
    w("  return -(int64_t)exc_;")
    w("}")
    return "\n".join(out)


MODULE_PRELUDE = """// generated by policy/native_codegen.py -- do not edit
#include "jit_abi.h"
using namespace fksd;
FKS_JIT_RT_TABLE_DEFINITION
"""

#: argument list of a probe kernel's direct call (values from memory so nothing folds)
_PROBE_ARGS = ", ".join([f"a[{k + 1}]" for k in range(22)] + ["g", "a[23]", "a[24]", "a[25]", "g[1]", "a[26]", "(KcPtr)g"])


def module_source(progs: Sequence[CompiledPolicy], with_probes: bool = True, host: bool = False,
                  lift_consts: bool = True) -> str:
    """One compile unit: the programs ``fks_prog_<i>``, the pointer table kernel
    ``fks_jit_table`` and one resource probe kernel per program (its metadata
    gives that program's register / stack use; `ops.jit` checks it against the
    calling replay kernel's allocation).  ``host=True``: the g++ variant with a
    plain pointer table ``fks_host_table``."""
    parts = [MODULE_PRELUDE]
    for i, p in enumerate(progs):
        parts.append(program_source(p, f"fks_prog_{i}", lift_consts))
    if host:
        parts.append('extern "C" {\nconst void* fks_host_table[] = {' +
                     ", ".join(f"(const void*)&fks_prog_{i}" for i in range(len(progs))) + "};\n" +
                     f"int fks_host_count = {len(progs)};\n}}")
        return "\n\n".join(parts) + "\n"
    parts.append('extern "C" __global__ void fks_jit_table(uint64_t* out) {\n' +
                 "".join(f"  out[{i}] = (uint64_t)&fks_prog_{i};\n" for i in range(len(progs))) + "}")
    if with_probes:
        for i in range(len(progs)):
            parts.append(f'extern "C" __global__ void fks_jit_probe_{i}(const int32_t* a, const int64_t* g, int64_t* o) {{\n'
                         f"  if (a[0] == 0x5EED) o[0] = fks_prog_{i}({_PROBE_ARGS});\n}}")
    return "\n\n".join(parts) + "\n"


__all__ = ["CodegenError", "PROG_PARAMS", "constant_block", "constant_blocks", "constant_payload", "infer_types", "module_source", "program_source",
           "shape_key"]
