"""Policy compiler: Python ``priority_function`` source -> SIMT bytecode.

The accepted grammar *is* the sandbox of the batched engines: only the
constructs below are lowered, everything else raises `CompileError` and the
program is evaluated by the exact object engine instead (so results never
depend on what the compiler supports, only speed does).

Supported (covers every program shipped with the reference and the template
the LLM fills in, SURVEY §2.4 rule 10):

* statements: assignment (names, tuple unpacking of tuple literals),
  augmented assignment, if/elif/else, for over ``node.gpus`` / GPU lists /
  ``range(...)`` / ``enumerate(gpu list)`` / literal number lists, while,
  break, continue, pass, return;
* expressions: int/float/bool constants, + - * / // % ** (CPython int/float
  rules), unary - + not, and/or (short-circuit, value-returning), chained
  comparisons, conditional expressions, ``pod.*``, ``node.*``, ``gpu.*``
  fields, ``len``, ``sum``, ``min``, ``max``, ``abs``, ``int``, ``float``,
  ``round(x)``, ``bool``, ``sorted(gpus, key=lambda g: ..., reverse=...)``,
  ``math.sqrt/log/exp/pow/sin/cos/tan``, ``operator.add/sub/mul/truediv/mod``,
  GPU-list comprehensions / generator expressions with filters, GPU-list
  indexing and slicing, literal number lists with constant indices.

Semantics are Python's, lane by lane: short-circuit evaluation is real
control flow (a masked branch), so an expression Python would not evaluate
cannot raise; reads of possibly-unassigned variables are checked at run time
(UnboundLocalError); unknown names raise NameError when reached.
"""

from __future__ import annotations

import ast
import hashlib
import struct
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

from .bytecode import (GPU_FIELDS, LOOP_INDEX, MAX_REGS, NO_REG, NODE_FIELDS, NODE_NGPUS, POD_FIELDS, TAG_FLOAT,
                       TAG_INT, Exc, Op, pack_insn)


#: AST node types that never matter to the analysis passes (see `_index_tree`)
_LEAF_NODES = frozenset(c for base in (ast.expr_context, ast.operator, ast.unaryop, ast.cmpop, ast.boolop)
                        for c in base.__subclasses__())


class CompileError(Exception):
    """The program uses a construct outside the native subset."""


# value kinds
NUM, GPU, GLIST, SLIST = "num", "gpu", "glist", "slist"

MATH_FUNCS = {"sqrt": Op.SQRT, "log": Op.LOG, "exp": Op.EXP, "pow": Op.MPOW,
              "sin": Op.SIN, "cos": Op.COS, "tan": Op.TAN}
OPERATOR_FUNCS = {"add": Op.ADD, "sub": Op.SUB, "mul": Op.MUL, "truediv": Op.TDIV, "mod": Op.MOD}
BIN_OPS = {ast.Add: Op.ADD, ast.Sub: Op.SUB, ast.Mult: Op.MUL, ast.Div: Op.TDIV,
           ast.FloorDiv: Op.FDIV, ast.Mod: Op.MOD, ast.Pow: Op.POW}
CMP_OPS = {ast.Lt: Op.LT, ast.LtE: Op.LE, ast.Gt: Op.GT, ast.GtE: Op.GE, ast.Eq: Op.EQ, ast.NotEq: Op.NE}
SAFE_BUILTINS = {"abs", "min", "max", "sum", "len", "range", "enumerate", "int", "float", "bool",
                 "str", "round", "sorted"}
INT64_MIN, INT64_MAX = -(1 << 63), (1 << 63) - 1


@dataclass
class Val:
    kind: str
    reg: int = NO_REG
    regs: Tuple["Val", ...] = ()   # SLIST elements
    temp: bool = False


#: operations CPython evaluates with libm (exp / log / pow: glibc_math.h on the device)
_LIBM_OPS = frozenset({Op.POW, Op.LOG, Op.LOGB, Op.EXP, Op.MPOW})


@dataclass
class CompiledPolicy:
    """Bytecode + constant pool of one program."""

    code: bytes
    fconst: List[float]
    iconst: List[int]
    ctag: List[int]
    nregs: int
    source: str
    features: frozenset = field(default_factory=frozenset)
    #: numeric source literals: (pool index, line, col, end line, end col)
    literals: list = field(default_factory=list)
    #: bytecode range [lo, hi) of the body's first two statements -- the
    #: template's feasibility prologue when `feasibility_prologue` holds
    #: (ops/gcnjit.py compiles it out for kernels that call feasible nodes only)
    prologue: Optional[Tuple[int, int]] = None

    @property
    def n_insns(self) -> int:
        return len(self.code) // 8

    @property
    def device_ok(self) -> bool:
        """False when the program uses functions the device interpreter routes
        back to the host (trigonometry: no correctly rounded device version)."""
        return "trig" not in self.features

    @property
    def uses_libm(self) -> bool:
        """The program may call libm's exp / log / pow (`**`, math.exp / log / pow)."""
        return "libm" in self.features

    @property
    def feasibility_prologue(self) -> bool:
        """The scoring function opens with the template's feasibility prologue
        (`policy.template.FEASIBILITY_PROLOGUE`, AST-equal, literals included):
        it then scores 0 -- with no other effect -- exactly on the (pod, node)
        pairs the replay kernels' own `feasible()` rejects, so a kernel may skip
        the call for those nodes."""
        v = self.__dict__.get("_feas_prologue")
        if v is None:
            v = self.__dict__["_feas_prologue"] = starts_with_feasibility_prologue(self.source)
        return v

    def digest(self) -> str:
        h = hashlib.sha1(self.code)
        h.update(struct.pack(f"<{len(self.fconst)}d", *self.fconst))
        h.update(struct.pack(f"<{len(self.iconst)}q", *self.iconst))
        h.update(bytes(self.ctag))
        return h.hexdigest()


class _Scope:
    def __init__(self):
        self.vars: Dict[str, Val] = {}
        self.flags: Dict[str, int] = {}   # defined-flag registers of maybe-unbound variables


class Compiler:
    def __init__(self, source: str):
        self.source = source
        self.code: List[list] = []         # [op, d, a, b, imm]
        self.consts: Dict[Tuple[int, object], int] = {}
        self.literals: List[Tuple[int, int, int, int, int]] = []   # (pool index, line, col, end line, end col)
        self.fconst: List[float] = []
        self.iconst: List[int] = []
        self.ctag: List[int] = []
        self.free: List[int] = list(range(MAX_REGS - 1, -1, -1))
        self.features = set()
        self.globals: Dict[str, Val] = {}
        self._order: list = []
        self._span: Dict[int, tuple] = {}
        self.scope = _Scope()
        self.pod_name = self.node_name = None
        self.loop_depth = 0
        # common subexpressions (see `expr`): text -> register holding the value
        self._cse: Dict[str, Val] = {}
        self._cse_memo: Dict[int, tuple] = {}
        self._cond = 0                      # > 0: inside a branch (no new cache entries)
        self._lines: Optional[List[str]] = None

    # ------------------------------------------------------------------ regs
    def alloc(self) -> int:
        if not self.free:
            raise CompileError("program needs more than 64 registers")
        return self.free.pop()

    def release(self, v: Optional[Val]) -> None:
        if v is not None and v.kind == SLIST:
            for r in v.regs:
                self.release(r)
            return
        if v is not None and v.temp and v.reg != NO_REG:
            self.free.append(v.reg)
            v.temp = False

    def tmp(self, kind: str = NUM) -> Val:
        return Val(kind, self.alloc(), temp=True)

    # ------------------------------------------------------------------ emit
    def emit(self, op: Op, d: int = NO_REG, a: int = NO_REG, b: int = NO_REG, imm: int = 0) -> int:
        if op in _LIBM_OPS:
            self.features.add("libm")
        self.code.append([int(op), d, a, b, imm])
        return len(self.code) - 1

    def patch(self, at: int, target: int) -> None:
        self.code[at][4] = target

    def const(self, value, literal: Optional[ast.Constant] = None) -> int:
        """Pool index of a constant.  Compiler-made constants are shared by
        value; every numeric *literal of the source* gets a pool entry of its own
        (recorded in `literals` with its source span), so the constants a
        program author wrote can be changed as data -- one compiled shape, many
        weight settings (funsearch/polish.py) -- without touching the loop
        counters and flags the compiler itself emits."""
        if literal is not None and isinstance(value, (int, float)) and not isinstance(value, bool):
            if isinstance(value, int) and not INT64_MIN <= value <= INT64_MAX:
                raise CompileError("integer constant outside int64")
            idx = len(self.ctag)
            fl = isinstance(value, float)
            self.ctag.append(TAG_FLOAT if fl else TAG_INT)
            self.fconst.append(float(value) if fl else 0.0)
            self.iconst.append(0 if fl else value)
            self.literals.append((idx, literal.lineno, literal.col_offset, literal.end_lineno, literal.end_col_offset))
            return idx
        if isinstance(value, bool):
            value = int(value)
        if isinstance(value, int):
            if not INT64_MIN <= value <= INT64_MAX:
                raise CompileError("integer constant outside int64")
            key = (TAG_INT, value)
        elif isinstance(value, float):
            key = (TAG_FLOAT, struct.pack("<d", value))
        else:
            raise CompileError(f"unsupported constant {value!r}")
        if key not in self.consts:
            self.consts[key] = len(self.ctag)
            self.ctag.append(key[0])
            self.fconst.append(float(value) if key[0] == TAG_FLOAT else 0.0)
            self.iconst.append(value if key[0] == TAG_INT else 0)
        return self.consts[key]

    def load_const(self, value, into: Optional[Val] = None, literal: Optional[ast.Constant] = None) -> Val:
        v = into or self.tmp()
        self.emit(Op.CONST, v.reg, imm=self.const(value, literal))
        return v

    def raise_(self, exc: Exc) -> None:
        self.emit(Op.RAISE, imm=int(exc))

    # ------------------------------------------------------------------ top level
    def compile(self) -> CompiledPolicy:
        from .sandbox import take_parsed
        tree = take_parsed(self.source)   # the validator's parse of this very string
        if tree is None:
            try:
                tree = ast.parse(self.source)
            except SyntaxError as exc:
                raise CompileError(f"syntax error: {exc}")
        fn = None
        for stmt in tree.body:
            if isinstance(stmt, ast.FunctionDef) and stmt.name == "priority_function":
                fn = stmt
            elif isinstance(stmt, ast.Expr) and isinstance(stmt.value, ast.Constant):
                continue
            elif isinstance(stmt, ast.Assign) and len(stmt.targets) == 1 \
                    and isinstance(stmt.targets[0], ast.Name):
                value = self._fold_constant(stmt.value)
                self.globals[stmt.targets[0].id] = value
            else:
                raise CompileError(f"unsupported top-level statement {type(stmt).__name__}")
        if fn is None:
            raise CompileError("no priority_function defined")
        args = fn.args
        if (len(args.args) != 2 or args.vararg or args.kwarg or args.kwonlyargs or args.defaults
                or getattr(args, "posonlyargs", [])):
            raise CompileError("priority_function must take exactly (pod, node)")
        if fn.decorator_list:
            raise CompileError("decorators are not supported")
        self.pod_name, self.node_name = args.args[0].arg, args.args[1].arg
        self._check_names(fn)
        self._plan_kinds(fn.body)
        for name, kind in sorted(self.kinds.items()):
            if kind != SLIST:
                self.scope.vars[name] = Val(kind, self.alloc())
        self._maybe_unbound = self._unbound_analysis(fn.body, set(self.kinds))
        for name in sorted(self._maybe_unbound):
            flag = self.alloc()
            self.scope.flags[name] = flag
            self.emit(Op.CONST, flag, imm=self.const(0))
        body = fn.body
        n_doc = 1 if (body and isinstance(body[0], ast.Expr) and isinstance(body[0].value, ast.Constant)
                      and isinstance(body[0].value.value, str)) else 0
        prologue = None
        lo = len(self.code)
        for j, st in enumerate(body):
            self.stmt(st)
            if j == n_doc + 1 and len(body) > n_doc + 2:
                prologue = (lo, len(self.code))
        self.emit(Op.END)
        self._renumber_registers()
        nregs = max((c[1] for c in self.code if c[1] != NO_REG), default=0) + 1
        return CompiledPolicy(b"".join(pack_insn(*c) for c in self.code), self.fconst, self.iconst,
                              self.ctag, nregs, self.source, frozenset(self.features), list(self.literals),
                              prologue)

    #: ops whose `imm` field names a register (or NO_REG)
    _IMM_REG_OPS = (Op.GLIST_SLICE, Op.GLIST_INSERT)

    def _renumber_registers(self) -> None:
        """Renumber virtual registers by static use count (most used -> 0).

        The device VM keeps the lowest-numbered registers in VGPRs and the
        rest in LDS, so hot temporaries and loop variables get the fast file.
        A pure renaming: both VMs execute the same instructions."""
        from collections import Counter
        imm_ops = self._IMM_REG_OPS
        uses = Counter(r for op, d, a, b, imm in self.code
                       for r in ((d, a, b, imm) if op in imm_ops else (d, a, b)))
        uses.pop(NO_REG, None)
        order = sorted(uses, key=lambda r: (-uses[r], r))
        perm = {r: i for i, r in enumerate(order)}
        perm[NO_REG] = NO_REG
        self.code = [(op, perm[d], perm[a], perm[b], perm[imm] if op in imm_ops else imm)
                     for op, d, a, b, imm in self.code]

    def _fold_constant(self, node: ast.AST):
        """Module-level ``NAME = <numeric literal expression>``."""
        try:
            value = eval(compile(ast.Expression(node), "<const>", "eval"), {"__builtins__": {}}, {})
        except Exception:
            raise CompileError("module-level assignment is not a numeric constant")
        if isinstance(value, bool) or not isinstance(value, (int, float)):
            raise CompileError("module-level assignment is not a numeric constant")
        for sub in ast.walk(node):
            if isinstance(sub, (ast.Name, ast.Call, ast.Attribute)):
                raise CompileError("module-level constant must be a literal expression")
        return value

    #: constructs the compiler rejects anywhere inside the policy function
    _BANNED = frozenset((ast.Global, ast.Nonlocal, ast.FunctionDef, ast.AsyncFunctionDef,
                         ast.ClassDef, ast.With, ast.Try, ast.Raise, ast.Assert, ast.Delete,
                         ast.Yield, ast.YieldFrom, ast.Await, ast.NamedExpr, ast.Starred,
                         ast.DictComp, ast.SetComp, ast.Dict, ast.Set, ast.JoinedStr))

    def _check_names(self, fn: ast.FunctionDef) -> None:
        self._index_tree(fn)
        reserved = {self.pod_name, self.node_name, "math", "operator"} | SAFE_BUILTINS
        banned, Name, Store = self._BANNED, ast.Name, ast.Store
        for node in self._walk(fn):
            t = type(node)
            if t is Name and type(node.ctx) is Store and node.id in reserved:
                raise CompileError(f"assignment to reserved name {node.id}")
            if t in banned and node is not fn:
                raise CompileError(f"unsupported construct {t.__name__}")

    # ------------------------------------------------------------------ analysis
    def _index_tree(self, root) -> None:
        """One pre-order pass over the function: every subtree is then a slice
        of `self._order`.  The analysis passes re-walk the same statements
        (kind planning runs three rounds, the unbound analysis nests per
        statement); walking them afresh each time was over half of compile
        time, and a per-subtree memo still paid O(size x depth).  Operator and
        load/store context nodes carry nothing the passes look at and are left
        out (they are a third of a typical tree)."""
        order, span, AST, leaf = [], {}, ast.AST, _LEAF_NODES

        def visit(n):
            i = len(order)
            order.append(n)
            for f in n._fields:
                v = getattr(n, f, None)
                if type(v) is list:
                    for x in v:
                        if isinstance(x, AST) and type(x) not in leaf:
                            visit(x)
                elif isinstance(v, AST) and type(v) not in leaf:
                    visit(v)
            span[id(n)] = (n, i, len(order))

        visit(root)
        self._order, self._span = order, span

    def _walk(self, node) -> list:
        """The nodes of `node`'s subtree in pre-order: `ast.walk` up to order,
        without operator and context nodes."""
        hit = self._span.get(id(node))
        if hit is not None and hit[0] is node:
            return self._order[hit[1]:hit[2]]
        return list(ast.walk(node))

    @staticmethod
    def _assigned_names(body) -> set:
        names = set()
        for stmt in body:
            for node in ast.walk(stmt):
                if isinstance(node, ast.Name) and isinstance(node.ctx, ast.Store):
                    names.add(node.id)
        return names

    def _plan_kinds(self, body) -> None:
        """Fix each local's kind from its assignments (a name must keep one kind)."""
        self.kinds: Dict[str, str] = {}
        kinds = (ast.Assign, ast.AnnAssign, ast.AugAssign, ast.For)
        sites = [node for stmt in body for node in self._walk(stmt) if type(node) in kinds]
        for _ in range(3):
            for node in sites:
                t = type(node)
                if t is ast.Assign:
                    for tgt in node.targets:
                        self._plan_target(tgt, node.value)
                elif t is ast.AnnAssign:
                    self._plan_target(node.target, node.value)
                elif t is ast.AugAssign:
                    self._plan_set(node.target, NUM)
                else:
                    self._plan_for(node)

    def _plan_set(self, target, kind) -> None:
        if not isinstance(target, ast.Name):
            raise CompileError("only simple names can be assigned")
        prev = self.kinds.get(target.id)
        if prev is not None and prev != kind:
            raise CompileError(f"variable {target.id} changes kind ({prev} -> {kind})")
        self.kinds[target.id] = kind

    def _plan_target(self, target, value) -> None:
        if isinstance(target, (ast.Tuple, ast.List)):
            if not isinstance(value, (ast.Tuple, ast.List)) or len(value.elts) != len(target.elts):
                raise CompileError("tuple unpacking needs a literal of the same length")
            for t, v in zip(target.elts, value.elts):
                self._plan_target(t, v)
            return
        self._plan_set(target, self._guess_kind(value))

    def _plan_for(self, node: ast.For) -> None:
        it = node.iter
        if isinstance(it, ast.Call) and isinstance(it.func, ast.Name) and it.func.id == "enumerate":
            if not isinstance(node.target, ast.Tuple) or len(node.target.elts) != 2:
                raise CompileError("enumerate() needs two loop targets")
            self._plan_set(node.target.elts[0], NUM)
            self._plan_set(node.target.elts[1], GPU)
            return
        if isinstance(it, ast.Call) and isinstance(it.func, ast.Name) and it.func.id == "range":
            self._plan_set(node.target, NUM)
            return
        k = self._guess_kind(it)
        if k == GLIST:
            self._plan_set(node.target, GPU)
        elif k == SLIST:
            self._plan_set(node.target, NUM)
        else:
            raise CompileError("unsupported for-loop iterable")

    def _guess_kind(self, e) -> str:
        if isinstance(e, ast.Attribute) and e.attr == "gpus":
            return GLIST
        if isinstance(e, ast.Name):
            return self.kinds.get(e.id, NUM)
        if isinstance(e, ast.ListComp):
            return GLIST
        if isinstance(e, (ast.List, ast.Tuple)):
            return SLIST
        if isinstance(e, ast.Subscript):
            base = self._guess_kind(e.value)
            if isinstance(e.slice, ast.Slice):
                return base
            return GPU if base == GLIST else NUM
        if isinstance(e, ast.Call) and isinstance(e.func, ast.Name) and e.func.id == "sorted":
            return GLIST
        if isinstance(e, ast.IfExp):
            a, b = self._guess_kind(e.body), self._guess_kind(e.orelse)
            if a != b:
                raise CompileError("conditional expression mixes kinds")
            return a
        return NUM

    def _unbound_analysis(self, body, assigned) -> set:
        """Names that some path may read before assigning."""
        risky = set()

        def expr_reads(e, defined):
            for n in self._walk(e):
                if isinstance(n, ast.Name) and isinstance(n.ctx, ast.Load) and n.id in assigned \
                        and n.id not in defined:
                    risky.add(n.id)

        def comp_locals(e):
            out = set()
            for n in self._walk(e):
                if isinstance(n, (ast.ListComp, ast.GeneratorExp)):
                    for g in n.generators:
                        for t in self._walk(g.target):
                            if isinstance(t, ast.Name):
                                out.add(t.id)
                if isinstance(n, ast.Lambda):
                    out.update(a.arg for a in n.args.args)
            return out

        def visit(stmts, defined):
            defined = set(defined)
            for s in stmts:
                local = comp_locals(s)
                if isinstance(s, ast.Assign):
                    expr_reads(s.value, defined | local)
                    for t in s.targets:
                        for n in self._walk(t):
                            if isinstance(n, ast.Name):
                                defined.add(n.id)
                elif isinstance(s, ast.AugAssign):
                    expr_reads(s.value, defined | local)
                    if s.target.id not in defined:
                        risky.add(s.target.id)
                    defined.add(s.target.id)
                elif isinstance(s, ast.If):
                    expr_reads(s.test, defined | local)
                    a = visit(s.body, defined)
                    b = visit(s.orelse, defined)
                    defined = a & b
                elif isinstance(s, (ast.For, ast.While)):
                    if isinstance(s, ast.For):
                        expr_reads(s.iter, defined | local)
                        tgt = {n.id for n in self._walk(s.target) if isinstance(n, ast.Name)}
                        visit(s.body, defined | tgt)
                        visit(s.body, defined | tgt | set())
                    else:
                        expr_reads(s.test, defined | local)
                        visit(s.body, defined)
                    visit(s.orelse, defined)
                elif isinstance(s, (ast.Return, ast.Expr)):
                    if s.value is not None:
                        expr_reads(s.value, defined | local)
                else:
                    for n in self._walk(s):
                        if isinstance(n, ast.expr):
                            expr_reads(n, defined | local)
            return defined

        visit(body, set())
        # a name assigned only inside a loop body and read after it is also risky;
        # approximate: names whose first assignment is inside a loop or branch
        return risky

    # ------------------------------------------------------------------ statements
    def block(self, stmts: Sequence[ast.stmt]) -> None:
        for s in stmts:
            self.stmt(s)

    def stmt(self, s: ast.stmt) -> None:
        if isinstance(s, ast.Expr):
            if isinstance(s.value, ast.Constant):
                return
            self.release(self.expr(s.value))
        elif isinstance(s, ast.Pass):
            return
        elif isinstance(s, ast.Assign):
            self.assign_stmt(s.targets, s.value)
        elif isinstance(s, ast.AnnAssign):
            if s.value is None:
                return
            self.assign_stmt([s.target], s.value)
        elif isinstance(s, ast.AugAssign):
            if not isinstance(s.target, ast.Name):
                raise CompileError("augmented assignment needs a name target")
            op = BIN_OPS.get(type(s.op))
            if op is None:
                raise CompileError("unsupported augmented operator")
            cur = self.load_name(s.target.id)
            if cur.kind != NUM:
                raise CompileError("augmented assignment on a non-number")
            rhs = self.num(s.value)
            dst = self.var_val(s.target.id, NUM)
            self.emit(op, dst.reg, cur.reg, rhs.reg)
            self.mark_defined(s.target.id)
            self.release(rhs)
            self.release(cur)
        elif isinstance(s, ast.If):
            self.if_stmt(s)
        elif isinstance(s, ast.For):
            self.for_stmt(s)
        elif isinstance(s, ast.While):
            self.while_stmt(s)
        elif isinstance(s, ast.Break):
            if not self.loop_depth:
                raise CompileError("break outside loop")
            self.emit(Op.BREAK)
        elif isinstance(s, ast.Continue):
            if not self.loop_depth:
                raise CompileError("continue outside loop")
            self.emit(Op.CONTINUE)
        elif isinstance(s, ast.Return):
            if s.value is None:
                self.raise_(Exc.TYPE)       # returns None -> int(max(0, None)) fails
                return
            v = self.expr(s.value)
            if v.kind != NUM:
                self.raise_(Exc.TYPE)
            else:
                self.emit(Op.RET, a=v.reg)
            self.release(v)
        else:
            raise CompileError(f"unsupported statement {type(s).__name__}")

    def var_val(self, name: str, kind: str) -> Val:
        v = self.scope.vars.get(name)
        if v is None:
            planned = self.kinds.get(name, kind)
            if planned != kind:
                raise CompileError(f"variable {name} changes kind")
            v = Val(kind, self.alloc())
            self.scope.vars[name] = v
        elif v.kind != kind:
            raise CompileError(f"variable {name} changes kind ({v.kind} -> {kind})")
        return v

    def mark_defined(self, name: str) -> None:
        flag = self.scope.flags.get(name)
        if flag is not None:
            self.emit(Op.CONST, flag, imm=self.const(1))

    def assign_stmt(self, targets, value) -> None:
        if len(targets) == 1 and isinstance(targets[0], (ast.Tuple, ast.List)):
            t = targets[0]
            if not isinstance(value, (ast.Tuple, ast.List)) or len(value.elts) != len(t.elts):
                raise CompileError("tuple unpacking needs a literal of the same length")
            vals = [self.expr(e) for e in value.elts]
            held = []
            for v in vals:   # snapshot RHS before any store (a, b = b, a)
                if v.kind in (NUM, GPU, GLIST):
                    c = self.tmp(v.kind)
                    self.emit(Op.MOV, c.reg, v.reg)
                    self.release(v)
                    held.append(c)
                else:
                    held.append(v)
            for tgt, v in zip(t.elts, held):
                self.store(tgt, v)
                self.release(v)
            return
        v = self.expr(value)
        for tgt in targets:
            self.store(tgt, v)
        self.release(v)

    def store(self, target, v: Val) -> None:
        if not isinstance(target, ast.Name):
            raise CompileError("only simple names can be assigned")
        name = target.id
        if v.kind == SLIST:
            # literal number lists: bind element registers (copied, so later
            # changes of the source variables cannot alias)
            if name in self.scope.vars and self.scope.vars[name].kind != SLIST:
                raise CompileError(f"variable {name} changes kind")
            old = self.scope.vars.get(name)
            if old is not None and len(old.regs) != len(v.regs):
                raise CompileError("literal list variables must keep their length")
            elems = old.regs if old is not None else tuple(Val(NUM, self.alloc()) for _ in v.regs)
            for dst, src in zip(elems, v.regs):
                self.emit(Op.MOV, dst.reg, src.reg)
            self.scope.vars[name] = Val(SLIST, regs=elems)
            self.mark_defined(name)
            return
        dst = self.var_val(name, v.kind)
        if dst.reg != v.reg:
            self.emit(Op.MOV, dst.reg, v.reg)
        self.mark_defined(name)

    def if_stmt(self, s: ast.If) -> None:
        t = self.truth(s.test)
        at_if = self.emit(Op.IF, a=t.reg)
        self.release(t)
        self._cond += 1
        self.block(s.body)
        if s.orelse:
            at_else = self.emit(Op.ELSE)
            self.patch(at_if, at_else)
            self.block(s.orelse)
            at_end = self.emit(Op.ENDIF)
            self.patch(at_else, at_end)
        else:
            at_end = self.emit(Op.ENDIF)
            self.patch(at_if, at_end)
        self._cond -= 1

    def _loop(self, header, body_fn, step_fn=None) -> None:
        """Masked loop skeleton: BEGIN; test: header() -> cond; TEST; body; CONT; step; NEXT; EXIT."""
        save = self.tmp()
        self.emit(Op.LOOP_BEGIN, save.reg)
        test_pc = len(self.code)
        cond = header()
        at_test = self.emit(Op.LOOP_TEST, a=cond.reg)
        self.release(cond)
        self.loop_depth += 1
        body_fn()
        self.loop_depth -= 1
        self.emit(Op.LOOP_CONT)
        if step_fn:
            step_fn()
        self.emit(Op.LOOP_NEXT, imm=test_pc)
        at_exit = self.emit(Op.LOOP_EXIT, a=save.reg)
        self.patch(at_test, at_exit)
        self.release(save)

    def for_stmt(self, s: ast.For) -> None:
        if s.orelse:
            raise CompileError("for/else is not supported")
        it = s.iter
        if isinstance(it, ast.Call) and isinstance(it.func, ast.Name) and it.func.id == "range" \
                and "range" not in self.scope.vars:
            self._for_range(it, s.target, s.body)
            return
        if isinstance(it, ast.Call) and isinstance(it.func, ast.Name) and it.func.id == "enumerate":
            if it.keywords or len(it.args) != 1:
                raise CompileError("enumerate(list) only")
            lst = self.expr(it.args[0])
            if lst.kind != GLIST:
                raise CompileError("enumerate over a GPU list only")
            idx_t, gpu_t = s.target.elts
            self._for_glist(lst, gpu_t, s.body, idx_target=idx_t)
            self.release(lst)
            return
        lst = self.expr(it)
        if lst.kind == GLIST:
            self._for_glist(lst, s.target, s.body)
            self.release(lst)
        elif lst.kind == SLIST:
            self._for_slist(lst, s.target, s.body)
        else:
            raise CompileError("unsupported for-loop iterable")

    def _for_glist(self, lst: Val, target, body, idx_target=None) -> None:
        # snapshot the list (the iterable is evaluated once)
        src = self.tmp(GLIST)
        self.emit(Op.MOV, src.reg, lst.reg)
        n = self.tmp()
        self.emit(Op.GLIST_LEN, n.reg, src.reg)
        idx = self.load_const(0)
        one = self.load_const(1)

        def header():
            c = self.tmp()
            self.emit(Op.LT, c.reg, idx.reg, n.reg, LOOP_INDEX)
            return c

        def body_fn():
            g = self.var_val(target.id, GPU) if isinstance(target, ast.Name) else None
            if g is None:
                raise CompileError("loop target must be a name")
            self.emit(Op.GLIST_GET, g.reg, src.reg, idx.reg, LOOP_INDEX)
            self.mark_defined(target.id)
            if idx_target is not None:
                iv = self.var_val(idx_target.id, NUM)
                self.emit(Op.MOV, iv.reg, idx.reg)
                self.mark_defined(idx_target.id)
            self.block(body)

        def step():
            self.emit(Op.ADD, idx.reg, idx.reg, one.reg, LOOP_INDEX)

        self._loop(header, body_fn, step)
        for v in (src, n, idx, one):
            self.release(v)

    def _for_range(self, call: ast.Call, target, body) -> None:
        if call.keywords or not 1 <= len(call.args) <= 3:
            raise CompileError("range() takes 1-3 positional arguments")
        args = [self.num(a) for a in call.args]
        if len(args) == 1:
            start, stop, step = self.load_const(0), args[0], self.load_const(1)
        elif len(args) == 2:
            start, stop, step = args[0], args[1], self.load_const(1)
        else:
            start, stop, step = args
        for v in (start, stop, step):   # range() accepts ints only
            chk = self.tmp()
            self.emit(Op.ISINT, chk.reg, v.reg)
            self.emit(Op.NOT, chk.reg, chk.reg)
            at = self.emit(Op.IF, a=chk.reg)
            self.raise_(Exc.TYPE)
            self.patch(at, self.emit(Op.ENDIF))
            self.release(chk)
        zero = self.load_const(0)
        chk = self.tmp()
        self.emit(Op.EQ, chk.reg, step.reg, zero.reg)
        at = self.emit(Op.IF, a=chk.reg)
        self.raise_(Exc.VALUE)
        self.patch(at, self.emit(Op.ENDIF))
        self.release(chk)
        i = self.tmp()
        self.emit(Op.MOV, i.reg, start.reg)
        stop_c, step_c = self.tmp(), self.tmp()
        self.emit(Op.MOV, stop_c.reg, stop.reg)
        self.emit(Op.MOV, step_c.reg, step.reg)
        for v in (start, stop, step):
            self.release(v)
        if not isinstance(target, ast.Name):
            raise CompileError("loop target must be a name")

        def header():
            pos, a, b = self.tmp(), self.tmp(), self.tmp()
            self.emit(Op.GT, pos.reg, step_c.reg, zero.reg)
            self.emit(Op.LT, a.reg, i.reg, stop_c.reg)
            self.emit(Op.GT, b.reg, i.reg, stop_c.reg)
            # cond = a if step > 0 else b  (selected with a masked branch)
            c = self.tmp()
            self.emit(Op.MOV, c.reg, b.reg)
            at = self.emit(Op.IF, a=pos.reg)
            self.emit(Op.MOV, c.reg, a.reg)
            self.patch(at, self.emit(Op.ENDIF))
            for v in (pos, a, b):
                self.release(v)
            return c

        def body_fn():
            tv = self.var_val(target.id, NUM)
            self.emit(Op.MOV, tv.reg, i.reg)
            self.mark_defined(target.id)
            self.block(body)

        def step_fn():
            self.emit(Op.ADD, i.reg, i.reg, step_c.reg)

        self._loop(header, body_fn, step_fn)
        for v in (zero, i, stop_c, step_c):
            self.release(v)

    def _for_slist(self, lst: Val, target, body) -> None:
        if not isinstance(target, ast.Name):
            raise CompileError("loop target must be a name")
        save = self.tmp()
        self.emit(Op.LOOP_BEGIN, save.reg)
        self.loop_depth += 1
        for elem in lst.regs:
            tv = self.var_val(target.id, NUM)
            self.emit(Op.MOV, tv.reg, elem.reg)
            self.mark_defined(target.id)
            self.block(body)
            self.emit(Op.LOOP_CONT)
        self.loop_depth -= 1
        self.emit(Op.LOOP_EXIT, a=save.reg)
        self.release(save)

    def while_stmt(self, s: ast.While) -> None:
        if s.orelse:
            raise CompileError("while/else is not supported")
        self._loop(lambda: self.truth(s.test), lambda: self.block(s.body))

    # ------------------------------------------------------------------ expressions
    def num(self, e) -> Val:
        v = self.expr(e)
        if v.kind != NUM:
            raise CompileError("a number was expected")
        return v

    def truth(self, e) -> Val:
        """Register holding 0/1 = bool(e)."""
        v = self.expr(e)
        t = self.tmp()
        if v.kind == NUM:
            self.emit(Op.TRUTH, t.reg, v.reg)
        elif v.kind == GLIST:
            self.emit(Op.GLIST_LEN, t.reg, v.reg)
            self.emit(Op.TRUTH, t.reg, t.reg)
        elif v.kind == SLIST:
            self.emit(Op.CONST, t.reg, imm=self.const(1 if v.regs else 0))
        else:  # GPU objects are always truthy
            self.emit(Op.CONST, t.reg, imm=self.const(1))
        self.release(v)
        return t

    def load_name(self, name: str) -> Val:
        if name in self.scope.vars:
            v = self.scope.vars[name]
            flag = self.scope.flags.get(name)
            if flag is not None:
                chk = self.tmp()
                self.emit(Op.NOT, chk.reg, flag)
                at = self.emit(Op.IF, a=chk.reg)
                self.raise_(Exc.NAME)
                self.patch(at, self.emit(Op.ENDIF))
                self.release(chk)
            return v
        if name in self.kinds:
            # assigned somewhere but never before this point in program order
            self.raise_(Exc.NAME)
            return self.load_const(0)
        if name in self.globals:
            return self.load_const(self.globals[name])
        if name in ("True", "False"):
            return self.load_const(1 if name == "True" else 0)
        # never assigned anywhere: NameError when (and only when) reached
        self.raise_(Exc.NAME)
        return self.load_const(0)

    def expr(self, e) -> Val:
        m = getattr(self, "e_" + type(e).__name__, None)
        if m is None:
            raise CompileError(f"unsupported expression {type(e).__name__}")
        key = self._cse_key(e) if self.CSE_MAX else None
        if key is not None:
            hit = self._cse.get(key)
            if hit is not None:
                return hit
        v = m(e)
        if key is not None and v.kind == NUM and v.temp and not self._cond and not self.loop_depth \
                and len(self._cse) < self.CSE_MAX:
            v.temp = False                  # held for the rest of the function
            self._cse[key] = v
        return v

    #: cached values per program (each holds a register to the end).  Off: on
    #: an evolved population (data/populations/config3_steady_r4_islands.json,
    #: 512 children) 16 held values made the baseline JIT decline 371 programs
    #: for VGPR pressure (4: 154; 0: 2) -- a declined program replays on the
    #: device VM at a fraction of native speed, far more than the saved work
    CSE_MAX = 0
    _CSE_NODES = (ast.BinOp, ast.UnaryOp, ast.Compare, ast.BoolOp, ast.IfExp, ast.Call, ast.Attribute,
                  ast.Subscript, ast.GeneratorExp, ast.ListComp, ast.comprehension, ast.Lambda, ast.Name,
                  ast.Constant, ast.Slice, ast.arguments, ast.arg, ast.keyword)

    def _cse_key(self, e) -> Optional[str]:
        """Common-subexpression elimination for what is invariant within a call:
        an expression that reads only pod / node fields (and names it binds
        itself, as a comprehension does), calls only the pure builtins and
        `math` functions, and holds no numeric literal other than int 0 / 1.
        The first evaluation of such an expression at an unconditional point of
        the function (not in a branch, loop or conditional operand) keeps its
        register; later occurrences with the same source text reuse it.  Exact:
        the value cannot change within the call, and if the first evaluation
        raises, the call ends there as in CPython.  Literal-free, so a
        program's bytecode never depends on its tunable constants (constant
        polish and `same_shape_child` change values, not shapes).  None: not
        eligible."""
        if not isinstance(e, (ast.BinOp, ast.UnaryOp, ast.Compare, ast.BoolOp, ast.IfExp, ast.Call,
                              ast.Subscript)):
            return None
        ok, used, bound, size, has_call = self._cse_info(e)
        if not ok or size < 4 and not has_call:
            return None
        if not (used - bound) <= {self.pod_name, self.node_name, "math"} | SAFE_BUILTINS:
            return None
        if e.lineno != e.end_lineno:
            return None
        if self._lines is None:
            self._lines = self.source.split("\n")
        line = self._lines[e.lineno - 1]
        if not line.isascii():
            return None                     # (offsets are UTF-8 bytes)
        return line[e.col_offset:e.end_col_offset]

    def _cse_info(self, e) -> tuple:
        """(eligible, names read, names bound, nodes, has a call) of a subtree, memoised."""
        hit = self._cse_memo.get(id(e))
        if hit is not None and hit[0] is e:
            return hit[1]
        t = type(e)
        ok = isinstance(e, self._CSE_NODES)
        used, bound, size, has_call = set(), set(), 1, t is ast.Call or t is ast.GeneratorExp or t is ast.ListComp
        if t is ast.Constant:
            ok = type(e.value) is int and e.value in (0, 1)
        elif t is ast.Name:
            if type(e.ctx) is ast.Load:
                used.add(e.id)
            else:
                bound.add(e.id)             # a comprehension target
        elif t is ast.arg:
            bound.add(e.arg)
        elif t is ast.Call and not (isinstance(e.func, ast.Name) and e.func.id in SAFE_BUILTINS
                                    or isinstance(e.func, ast.Attribute) and isinstance(e.func.value, ast.Name)
                                    and e.func.value.id == "math"):
            ok = False
        if ok:
            for f in e._fields:
                v = getattr(e, f, None)
                for c in (v if type(v) is list else (v,)):
                    if isinstance(c, ast.AST) and type(c) not in _LEAF_NODES:
                        cok, cu, cb, cs, cc = self._cse_info(c)
                        if not cok:
                            ok = False
                            break
                        used |= cu
                        bound |= cb
                        size += cs
                        has_call = has_call or cc
                if not ok:
                    break
        res = (ok, used, bound, size, has_call)
        self._cse_memo[id(e)] = (e, res)
        return res

    def e_Constant(self, e: ast.Constant) -> Val:
        if isinstance(e.value, (bool, int, float)):
            return self.load_const(e.value, literal=e)
        raise CompileError(f"unsupported constant {e.value!r}")

    def e_Name(self, e: ast.Name) -> Val:
        if e.id in (self.pod_name, self.node_name, "math", "operator"):
            raise CompileError(f"bare use of {e.id}")
        if e.id in SAFE_BUILTINS and e.id not in self.scope.vars:
            raise CompileError(f"bare use of builtin {e.id}")
        return self.load_name(e.id)

    def e_Attribute(self, e: ast.Attribute) -> Val:
        base = e.value
        if isinstance(base, ast.Name) and base.id == self.pod_name and base.id not in self.scope.vars:
            if e.attr not in POD_FIELDS:
                raise CompileError(f"unsupported pod field {e.attr}")
            v = self.tmp()
            self.emit(Op.POD, v.reg, imm=POD_FIELDS[e.attr])
            return v
        if isinstance(base, ast.Name) and base.id == self.node_name and base.id not in self.scope.vars:
            if e.attr == "gpus":
                v = self.tmp(GLIST)
                self.emit(Op.GLIST_ALL, v.reg)
                return v
            if e.attr not in NODE_FIELDS:
                raise CompileError(f"unsupported node field {e.attr}")
            v = self.tmp()
            self.emit(Op.NODE, v.reg, imm=NODE_FIELDS[e.attr])
            return v
        g = self.expr(base)
        if g.kind != GPU:
            raise CompileError(f"attribute {e.attr} of a non-GPU value")
        if e.attr not in GPU_FIELDS:
            raise CompileError(f"unsupported gpu field {e.attr}")
        v = self.tmp()
        self.emit(Op.GPU, v.reg, g.reg, imm=GPU_FIELDS[e.attr])
        self.release(g)
        return v

    def e_BinOp(self, e: ast.BinOp) -> Val:
        op = BIN_OPS.get(type(e.op))
        if op is None:
            raise CompileError(f"unsupported operator {type(e.op).__name__}")
        a = self.num(e.left)
        r = e.right
        if op == Op.POW and isinstance(r, ast.Constant) and type(r.value) is int and r.value in (1, 2, 3):
            # x ** 1 / 2 / 3: the exponent is part of the code (not a tunable
            # literal) and named in imm, so the baseline JIT can inline the
            # power (POW semantics unchanged; interpreters ignore imm)
            b = self.load_const(r.value)
            d = self.tmp()
            self.emit(op, d.reg, a.reg, b.reg, r.value)
        else:
            b = self.num(r)
            d = self.tmp()
            self.emit(op, d.reg, a.reg, b.reg)
        self.release(a)
        self.release(b)
        return d

    def e_UnaryOp(self, e: ast.UnaryOp) -> Val:
        if isinstance(e.op, ast.Not):
            t = self.truth(e.operand)
            self.emit(Op.NOT, t.reg, t.reg)
            return t
        a = self.num(e.operand)
        d = self.tmp()
        op = {ast.USub: Op.NEG, ast.UAdd: Op.POS}.get(type(e.op))
        if op is None:
            raise CompileError("unsupported unary operator")
        self.emit(op, d.reg, a.reg)
        self.release(a)
        return d

    def e_BoolOp(self, e: ast.BoolOp) -> Val:
        r = self.tmp()
        first = self.num(e.values[0])
        self.emit(Op.MOV, r.reg, first.reg)
        self.release(first)
        ifs = []
        self._cond += 1
        for v in e.values[1:]:
            t = self.tmp()
            self.emit(Op.TRUTH, t.reg, r.reg)
            if isinstance(e.op, ast.Or):
                self.emit(Op.NOT, t.reg, t.reg)
            ifs.append(self.emit(Op.IF, a=t.reg))
            self.release(t)
            nv = self.num(v)
            self.emit(Op.MOV, r.reg, nv.reg)
            self.release(nv)
        self._cond -= 1
        for at in reversed(ifs):
            self.patch(at, self.emit(Op.ENDIF))
        return r

    def e_Compare(self, e: ast.Compare) -> Val:
        r = self.tmp()
        left = self.num(e.left)
        ifs = []
        for i, (op, comp) in enumerate(zip(e.ops, e.comparators)):
            code = CMP_OPS.get(type(op))
            if code is None:
                raise CompileError(f"unsupported comparison {type(op).__name__}")
            right = self.num(comp)
            self.emit(code, r.reg, left.reg, right.reg)
            self.release(left)
            left = right
            if i < len(e.ops) - 1:
                ifs.append(self.emit(Op.IF, a=r.reg))
                self._cond += 1             # the rest of a chain is conditional
        self._cond -= len(ifs)
        self.release(left)
        for at in reversed(ifs):
            self.patch(at, self.emit(Op.ENDIF))
        return r

    def e_IfExp(self, e: ast.IfExp) -> Val:
        t = self.truth(e.test)
        at_if = self.emit(Op.IF, a=t.reg)
        self.release(t)
        self._cond += 1
        a = self.expr(e.body)
        r = self.tmp(a.kind)
        self.emit(Op.MOV, r.reg, a.reg)
        self.release(a)
        at_else = self.emit(Op.ELSE)
        self.patch(at_if, at_else)
        b = self.expr(e.orelse)
        self._cond -= 1
        if b.kind != r.kind:
            raise CompileError("conditional expression mixes kinds")
        self.emit(Op.MOV, r.reg, b.reg)
        self.release(b)
        self.patch(at_else, self.emit(Op.ENDIF))
        return r

    def e_List(self, e) -> Val:
        elems = []
        for x in e.elts:
            v = self.num(x)
            c = self.tmp()
            self.emit(Op.MOV, c.reg, v.reg)
            self.release(v)
            elems.append(c)
        return Val(SLIST, regs=tuple(elems), temp=False)

    e_Tuple = e_List

    def e_Subscript(self, e: ast.Subscript) -> Val:
        base = self.expr(e.value)
        sl = e.slice
        if isinstance(sl, ast.Index):  # py<3.9 compat
            sl = sl.value
        if base.kind == GLIST:
            if isinstance(sl, ast.Slice):
                if sl.step is not None:
                    raise CompileError("slice steps are not supported")
                lo = self.num(sl.lower) if sl.lower is not None else None
                hi = self.num(sl.upper) if sl.upper is not None else None
                d = self.tmp(GLIST)
                self.emit(Op.GLIST_SLICE, d.reg, base.reg, lo.reg if lo else NO_REG,
                          hi.reg if hi else NO_REG)
                self.release(lo)
                self.release(hi)
                self.release(base)
                return d
            idx = self.num(sl)
            d = self.tmp(GPU)
            self.emit(Op.GLIST_GET, d.reg, base.reg, idx.reg)
            self.release(idx)
            self.release(base)
            return d
        if base.kind == SLIST:
            if isinstance(sl, ast.Constant) and isinstance(sl.value, int) and not isinstance(sl.value, bool):
                k = sl.value
                n = len(base.regs)
                if not -n <= k < n:
                    self.raise_(Exc.INDEX)
                    return self.load_const(0)
                src = base.regs[k]
                d = self.tmp()
                self.emit(Op.MOV, d.reg, src.reg)
                self._release_slist(base)
                return d
            raise CompileError("literal lists support constant indices only")
        raise CompileError("subscript of a non-list value")

    def _release_slist(self, v: Val) -> None:
        # element temporaries of a literal list (variable-bound elements are not temps)
        self.release(v)

    # ------------------------------------------------------------------ comprehensions
    def _comp_iter(self, comp) -> Tuple[ast.comprehension, Val]:
        if len(comp.generators) != 1:
            raise CompileError("nested comprehensions are not supported")
        g = comp.generators[0]
        if g.is_async:
            raise CompileError("async comprehension")
        return g, None

    def _gen_loop(self, comp, per_item) -> None:
        """Drive a one-generator comprehension: per_item(elem_val) runs for
        every item that passes the filters (masked)."""
        g, _ = self._comp_iter(comp)
        target = g.target
        if not isinstance(target, ast.Name):
            raise CompileError("comprehension target must be a name")
        saved = self.scope.vars.get(target.id)
        saved_flag = self.scope.flags.pop(target.id, None)
        it = g.iter
        if isinstance(it, ast.Call) and isinstance(it.func, ast.Name) and it.func.id == "range":
            kind, lst = NUM, None
        else:
            lst = self.expr(it)
            if lst.kind == GLIST:
                kind = GPU
            elif lst.kind == SLIST:
                kind = NUM
            else:
                raise CompileError("unsupported comprehension iterable")
        elem = Val(kind, self.alloc())
        self.scope.vars[target.id] = elem

        def body():
            ifs = []
            for cond in g.ifs:
                t = self.truth(cond)
                ifs.append(self.emit(Op.IF, a=t.reg))
                self.release(t)
            per_item()
            for at in reversed(ifs):
                self.patch(at, self.emit(Op.ENDIF))

        try:
            if lst is None:
                self._range_items(it, elem, body)
            elif lst.kind == GLIST:
                src = self.tmp(GLIST)
                self.emit(Op.MOV, src.reg, lst.reg)
                self.release(lst)
                n = self.tmp()
                self.emit(Op.GLIST_LEN, n.reg, src.reg)
                idx = self.load_const(0)
                one = self.load_const(1)

                def header():
                    c = self.tmp()
                    self.emit(Op.LT, c.reg, idx.reg, n.reg, LOOP_INDEX)
                    return c

                def body_fn():
                    self.emit(Op.GLIST_GET, elem.reg, src.reg, idx.reg, LOOP_INDEX)
                    body()

                self._loop(header, body_fn, lambda: self.emit(Op.ADD, idx.reg, idx.reg, one.reg, LOOP_INDEX))
                for v in (src, n, idx, one):
                    self.release(v)
            else:
                for r in lst.regs:
                    self.emit(Op.MOV, elem.reg, r.reg)
                    body()
                self._release_slist(lst)
        finally:
            self.free.append(elem.reg)
            if saved is not None:
                self.scope.vars[target.id] = saved
            else:
                self.scope.vars.pop(target.id, None)
            if saved_flag is not None:
                self.scope.flags[target.id] = saved_flag

    def _range_items(self, call, elem: Val, body) -> None:
        if call.keywords or not 1 <= len(call.args) <= 2:
            raise CompileError("comprehension range() takes 1-2 arguments")
        args = [self.num(a) for a in call.args]
        start, stop = (self.load_const(0), args[0]) if len(args) == 1 else (args[0], args[1])
        i = self.tmp()
        self.emit(Op.MOV, i.reg, start.reg)
        stop_c = self.tmp()
        self.emit(Op.MOV, stop_c.reg, stop.reg)
        self.release(start)
        self.release(stop)
        one = self.load_const(1)

        def header():
            c = self.tmp()
            self.emit(Op.LT, c.reg, i.reg, stop_c.reg)
            return c

        def body_fn():
            self.emit(Op.MOV, elem.reg, i.reg)
            body()

        self._loop(header, body_fn, lambda: self.emit(Op.ADD, i.reg, i.reg, one.reg))
        for v in (i, stop_c, one):
            self.release(v)

    def e_ListComp(self, e: ast.ListComp) -> Val:
        """Materialise a GPU list (element must be a GPU)."""
        out = self.tmp(GLIST)
        self.emit(Op.GLIST_NEW, out.reg)

        def item():
            v = self.expr(e.elt)
            if v.kind != GPU:
                raise CompileError("only lists of GPUs can be materialised")
            self.emit(Op.GLIST_APPEND, out.reg, out.reg, v.reg)
            self.release(v)

        self._gen_loop(e, item)
        return out

    # ------------------------------------------------------------------ calls
    def e_Call(self, e: ast.Call) -> Val:
        f = e.func
        if isinstance(f, ast.Attribute) and isinstance(f.value, ast.Name) \
                and f.value.id in ("math", "operator") and f.value.id not in self.scope.vars:
            table = MATH_FUNCS if f.value.id == "math" else OPERATOR_FUNCS
            if f.attr not in table or e.keywords:
                raise CompileError(f"unsupported {f.value.id}.{f.attr}")
            op = table[f.attr]
            if f.value.id == "math" and f.attr == "log" and len(e.args) == 2:
                op = Op.LOGB
            arity = 2 if op in (Op.MPOW, Op.LOGB, Op.ADD, Op.SUB, Op.MUL, Op.TDIV, Op.MOD) else 1
            if len(e.args) != arity:
                raise CompileError(f"{f.value.id}.{f.attr} arity")
            if op in (Op.SIN, Op.COS, Op.TAN):
                self.features.add("trig")
            args = [self.num(a) for a in e.args]
            d = self.tmp()
            self.emit(op, d.reg, args[0].reg, args[1].reg if arity == 2 else NO_REG)
            for a in args:
                self.release(a)
            return d
        if not isinstance(f, ast.Name):
            raise CompileError("unsupported call target")
        name = f.id
        if name in self.scope.vars or name in self.kinds:
            raise CompileError(f"calling local variable {name}")
        if name not in SAFE_BUILTINS:
            # NameError when (and only when) this call is reached
            self.raise_(Exc.NAME)
            return self.load_const(0)
        m = getattr(self, "call_" + name, None)
        if m is None:
            raise CompileError(f"unsupported builtin {name}()")
        return m(e)

    def _unary_builtin(self, e, op) -> Val:
        if e.keywords or len(e.args) != 1:
            raise CompileError("unsupported builtin arguments")
        a = self.num(e.args[0])
        d = self.tmp()
        self.emit(op, d.reg, a.reg)
        self.release(a)
        return d

    def call_abs(self, e):
        return self._unary_builtin(e, Op.ABS)

    def call_int(self, e):
        if e.keywords or len(e.args) != 1:
            raise CompileError("int() with base is not supported")
        return self._unary_builtin(e, Op.INT)

    def call_float(self, e):
        if not e.args:
            return self.load_const(0.0)
        return self._unary_builtin(e, Op.FLOAT)

    def call_bool(self, e):
        if not e.args:
            return self.load_const(0)
        if e.keywords or len(e.args) != 1:
            raise CompileError("bool() arguments")
        return self.truth(e.args[0])

    def call_round(self, e):
        if e.keywords or len(e.args) != 1:
            raise CompileError("round() with ndigits is not supported")
        return self._unary_builtin(e, Op.ROUND)

    def call_len(self, e):
        if e.keywords or len(e.args) != 1:
            raise CompileError("len() arguments")
        arg = e.args[0]
        if isinstance(arg, (ast.ListComp, ast.GeneratorExp)):
            if isinstance(arg, ast.GeneratorExp):
                self.raise_(Exc.TYPE)  # len(generator) is a TypeError
                return self.load_const(0)
            cnt = self.load_const(0)
            one = self.load_const(1)

            def item():
                v = self.expr(arg.elt)
                self.release(v)
                self.emit(Op.ADD, cnt.reg, cnt.reg, one.reg)

            self._gen_loop(arg, item)
            self.release(one)
            return cnt
        v = self.expr(arg)
        if v.kind == GLIST:
            d = self.tmp()
            self.emit(Op.GLIST_LEN, d.reg, v.reg)
            self.release(v)
            return d
        if v.kind == SLIST:
            n = len(v.regs)
            self._release_slist(v)
            return self.load_const(n)
        self.release(v)
        self.raise_(Exc.TYPE)
        return self.load_const(0)

    def call_sum(self, e):
        if e.keywords or not 1 <= len(e.args) <= 2:
            raise CompileError("sum() arguments")
        acc = self.tmp()
        if len(e.args) == 2:
            s = self.num(e.args[1])
            self.emit(Op.MOV, acc.reg, s.reg)
            self.release(s)
        else:
            self.emit(Op.CONST, acc.reg, imm=self.const(0))
        self._fold_iterable(e.args[0], lambda v: self.emit(Op.ADD, acc.reg, acc.reg, v.reg))
        return acc

    def _fold_iterable(self, arg, on_item) -> None:
        if isinstance(arg, (ast.ListComp, ast.GeneratorExp)):
            def item():
                v = self.expr(arg.elt)
                if v.kind != NUM:
                    raise CompileError("reduction over non-numbers")
                on_item(v)
                self.release(v)
            self._gen_loop(arg, item)
            return
        v = self.expr(arg)
        if v.kind == SLIST:
            for r in v.regs:
                on_item(r)
            self._release_slist(v)
            return
        raise CompileError("unsupported reduction iterable")

    def _minmax(self, e, op) -> Val:
        default = None
        for kw in e.keywords:
            if kw.arg == "default":
                default = kw.value
            else:
                raise CompileError(f"{op.name.lower()}() keyword {kw.arg}")
        if len(e.args) > 1:
            if default is not None:
                raise CompileError("default with multiple arguments")
            r = self.tmp()
            first = self.num(e.args[0])
            self.emit(Op.MOV, r.reg, first.reg)
            self.release(first)
            for a in e.args[1:]:
                v = self.num(a)
                self.emit(op, r.reg, r.reg, v.reg)
                self.release(v)
            return r
        if len(e.args) != 1:
            raise CompileError("min/max need arguments")
        arg = e.args[0]
        r = self.tmp()
        seen = self.load_const(0)
        one = self.load_const(1)

        def on_item(v):
            t = self.tmp()
            self.emit(Op.NOT, t.reg, seen.reg)
            at_if = self.emit(Op.IF, a=t.reg)
            self.emit(Op.MOV, r.reg, v.reg)
            self.emit(Op.MOV, seen.reg, one.reg)
            at_else = self.emit(Op.ELSE)
            self.patch(at_if, at_else)
            self.emit(op, r.reg, r.reg, v.reg)
            self.patch(at_else, self.emit(Op.ENDIF))
            self.release(t)

        self._fold_iterable(arg, on_item)
        t = self.tmp()
        self.emit(Op.NOT, t.reg, seen.reg)
        at = self.emit(Op.IF, a=t.reg)
        if default is None:
            self.raise_(Exc.VALUE)   # max() arg is an empty sequence
        else:
            dv = self.num(default)
            self.emit(Op.MOV, r.reg, dv.reg)
            self.release(dv)
        self.patch(at, self.emit(Op.ENDIF))
        for v in (t, seen, one):
            self.release(v)
        return r

    def call_max(self, e):
        return self._minmax(e, Op.MAX2)

    def call_min(self, e):
        return self._minmax(e, Op.MIN2)

    def call_sorted(self, e):
        if len(e.args) != 1:
            raise CompileError("sorted() takes one iterable")
        key = None
        reverse = False
        for kw in e.keywords:
            if kw.arg == "key":
                key = kw.value
            elif kw.arg == "reverse":
                if not isinstance(kw.value, ast.Constant):
                    raise CompileError("sorted(reverse=...) must be a constant")
                reverse = bool(kw.value.value)
            else:
                raise CompileError(f"sorted() keyword {kw.arg}")
        src = self.expr(e.args[0])
        if src.kind != GLIST:
            raise CompileError("sorted() over GPU lists only")
        if key is None:
            # GPU objects are unorderable: TypeError as soon as two are compared
            n = self.tmp()
            self.emit(Op.GLIST_LEN, n.reg, src.reg)
            two = self.load_const(2)
            self.emit(Op.GE, n.reg, n.reg, two.reg)
            at = self.emit(Op.IF, a=n.reg)
            self.raise_(Exc.TYPE)
            self.patch(at, self.emit(Op.ENDIF))
            self.release(n)
            self.release(two)
            return src
        if not (isinstance(key, ast.Lambda) and len(key.args.args) == 1 and not key.args.defaults):
            raise CompileError("sorted(key=...) must be a one-argument lambda")
        lam_arg = key.args.args[0].arg
        # stable insertion sort: g goes after every element whose key <= key(g)
        # (>= with reverse=True); keys recomputed, lists have <= 15 entries
        out = self.tmp(GLIST)
        self.emit(Op.GLIST_NEW, out.reg)
        srcc = self.tmp(GLIST)
        self.emit(Op.MOV, srcc.reg, src.reg)
        self.release(src)

        def key_of(gpu_reg: int) -> Val:
            saved = self.scope.vars.get(lam_arg)
            saved_flag = self.scope.flags.pop(lam_arg, None)
            self.scope.vars[lam_arg] = Val(GPU, gpu_reg)
            try:
                k = self.num(key.body)
            finally:
                if saved is not None:
                    self.scope.vars[lam_arg] = saved
                else:
                    self.scope.vars.pop(lam_arg, None)
                if saved_flag is not None:
                    self.scope.flags[lam_arg] = saved_flag
            kc = self.tmp()
            self.emit(Op.MOV, kc.reg, k.reg)
            self.release(k)
            return kc

        n = self.tmp()
        self.emit(Op.GLIST_LEN, n.reg, srcc.reg)
        i = self.load_const(0)
        one = self.load_const(1)
        g = self.tmp(GPU)

        def outer_header():
            c = self.tmp()
            self.emit(Op.LT, c.reg, i.reg, n.reg)
            return c

        def outer_body():
            self.emit(Op.GLIST_GET, g.reg, srcc.reg, i.reg)
            kg = key_of(g.reg)
            nan_chk = self.tmp()
            self.emit(Op.NE, nan_chk.reg, kg.reg, kg.reg)   # NaN keys: CPython's order differs
            at = self.emit(Op.IF, a=nan_chk.reg)
            self.raise_(Exc.UNSUPPORTED)
            self.patch(at, self.emit(Op.ENDIF))
            self.release(nan_chk)
            pos = self.load_const(0)
            m = self.tmp()
            self.emit(Op.GLIST_LEN, m.reg, out.reg)
            j = self.load_const(0)
            e_ = self.tmp(GPU)

            def inner_header():
                c = self.tmp()
                self.emit(Op.LT, c.reg, j.reg, m.reg)
                return c

            def inner_body():
                self.emit(Op.GLIST_GET, e_.reg, out.reg, j.reg)
                ke = key_of(e_.reg)
                c = self.tmp()
                self.emit(Op.GE if reverse else Op.LE, c.reg, ke.reg, kg.reg)
                at2 = self.emit(Op.IF, a=c.reg)
                self.emit(Op.ADD, pos.reg, pos.reg, one.reg)
                self.patch(at2, self.emit(Op.ENDIF))
                self.release(c)
                self.release(ke)

            self._loop(inner_header, inner_body, lambda: self.emit(Op.ADD, j.reg, j.reg, one.reg))
            self.emit(Op.GLIST_INSERT, out.reg, out.reg, g.reg, pos.reg)
            for v in (kg, pos, m, j, e_):
                self.release(v)

        self._loop(outer_header, outer_body, lambda: self.emit(Op.ADD, i.reg, i.reg, one.reg))
        for v in (srcc, n, i, one, g):
            self.release(v)
        return out

    def call_str(self, e):
        raise CompileError("strings are not supported")

    def call_range(self, e):
        raise CompileError("range() outside a for loop")

    def call_enumerate(self, e):
        raise CompileError("enumerate() outside a for loop")


_PROLOGUE_DUMPS: Optional[List[str]] = None


def starts_with_feasibility_prologue(source: str) -> bool:
    """True when the program's `priority_function(pod, node)` body (after an
    optional docstring) starts with the template's feasibility prologue."""
    global _PROLOGUE_DUMPS
    from .template import FEASIBILITY_PROLOGUE, PolicyTemplate
    # fast path (template-filled programs): the template's own head verbatim, the
    # only priority_function, and the line after the prologue back at the
    # function body's indentation -- then the body's first statements are the
    # prologue's, token for token (no AST parse on the batch-preparation path)
    head = PolicyTemplate.TEMPLATE.split("\n    \n    # LLM fills in this part")[0]
    i = source.find(head)
    if i >= 0 and source.count("def priority_function") == 1:
        rest = source[i + len(head):]
        if rest == "" or rest.startswith("\n"):
            nxt = next((ln for ln in rest.split("\n")[1:] if ln.strip()), "")
            if len(nxt) - len(nxt.lstrip(" ")) <= 4 and not nxt.startswith("\t"):
                return True
    if _PROLOGUE_DUMPS is None:
        ref = ast.parse("def priority_function(pod, node):\n" + FEASIBILITY_PROLOGUE + "\n")
        _PROLOGUE_DUMPS = [ast.dump(st) for st in ref.body[0].body]
    try:
        tree = ast.parse(source)
    except (SyntaxError, ValueError, RecursionError):
        return False
    fn = None
    for st in tree.body:
        if isinstance(st, ast.FunctionDef) and st.name == "priority_function":
            fn = st
    if fn is None or [a.arg for a in fn.args.args] != ["pod", "node"]:
        return False
    body = list(fn.body)
    if body and isinstance(body[0], ast.Expr) and isinstance(body[0].value, ast.Constant) \
            and isinstance(body[0].value.value, str):
        body = body[1:]
    k = len(_PROLOGUE_DUMPS)
    return len(body) > k and [ast.dump(st) for st in body[:k]] == _PROLOGUE_DUMPS


def compile_policy(source: str) -> CompiledPolicy:
    """Compile one program; raises `CompileError` outside the native subset."""
    return Compiler(source).compile()


_NUM_TOKEN = None


def same_shape_child(parent: CompiledPolicy, child: str) -> Optional[CompiledPolicy]:
    """`child` compiled without the compiler when it is `parent.source` with only
    the digits of numeric literals changed (an offline mutator's constant
    perturbation): the parent's bytecode with the child's literal values and
    spans.  Exact by construction -- same token stream, every changed token a
    literal of the same int / float kind; anything else (a changed non-literal
    digit, a literal the token scan does not see, a kind change) returns None
    and the caller compiles."""
    import re
    global _NUM_TOKEN
    if _NUM_TOKEN is None:
        _NUM_TOKEN = re.compile(r"(?<![\w.])(\d+\.\d+|\d+)(?![\w.])")
    src = parent.source
    if len(child) > 2 * len(src) + 64:
        return None
    tp = parent.__dict__.get("_num_tokens")   # a parent serves many children
    if tp is None:
        tp = parent.__dict__["_num_tokens"] = [(m.start(), m.end()) for m in _NUM_TOKEN.finditer(src)]
    tc = [(m.start(), m.end()) for m in _NUM_TOKEN.finditer(child)]
    if len(tp) != len(tc):
        return None
    # text between the tokens must be identical
    prev_p = prev_c = 0
    for (ps, pe), (cs, ce) in zip(tp, tc):
        if src[prev_p:ps] != child[prev_c:cs]:
            return None
        prev_p, prev_c = pe, ce
    if src[prev_p:] != child[prev_c:]:
        return None
    # literal spans of the parent -> token positions
    starts = [0]
    for line in src.split("\n"):
        starts.append(starts[-1] + len(line) + 1)
    lit_at = {}
    for idx, ln, col, eln, ecol in parent.literals:
        if ln != eln:
            return None
        lit_at[starts[ln - 1] + col] = (idx, starts[ln - 1] + ecol)
    cstarts = [0]
    for line in child.split("\n"):
        cstarts.append(cstarts[-1] + len(line) + 1)
    f, i = list(parent.fconst), list(parent.iconst)
    lits, seen = [], 0
    line_c = 0
    for (ps, pe), (cs, ce) in zip(tp, tc):
        hit = lit_at.get(ps)
        ptxt, ctxt = src[ps:pe], child[cs:ce]
        if hit is None or hit[1] != pe:
            if ptxt != ctxt:
                return None        # a changed digit outside a literal the compiler saw
            continue
        idx = hit[0]
        seen += 1
        is_float = "." in ctxt
        if is_float != (parent.ctag[idx] == TAG_FLOAT):
            return None
        if is_float:
            f[idx] = float(ctxt)
        else:
            if len(ctxt) > 1 and ctxt[0] == "0":
                return None        # `007`: a SyntaxError in Python 3 (int() would accept it)
            i[idx] = int(ctxt)
            if not INT64_MIN <= i[idx] <= INT64_MAX:
                return None        # Compiler.const's range check (the compile path reports it)
            if ptxt != ctxt and (parent.iconst[idx] in (0, 1) or i[idx] in (0, 1)):
                return None        # int 0 / 1 decide common-subexpression eligibility (Compiler._cse_key)
        while cstarts[line_c + 1] <= cs:
            line_c += 1
        lits.append((idx, line_c + 1, cs - cstarts[line_c], line_c + 1, ce - cstarts[line_c]))
    if seen != len(parent.literals):
        return None
    span = {lt[0]: lt for lt in lits}
    # the parent's bytecode range of the opening statements (whether they are the
    # template's feasibility prologue is decided on the child's own text)
    return CompiledPolicy(parent.code, f, i, list(parent.ctag), parent.nregs, child, parent.features,
                          [span[lt[0]] for lt in parent.literals],   # the compiler's order
                          prologue=parent.prologue)


def try_compile(source: str) -> Tuple[Optional[CompiledPolicy], Optional[str]]:
    try:
        return compile_policy(source), None
    except CompileError as exc:
        return None, str(exc)
    except RecursionError:
        return None, "program too deeply nested"
