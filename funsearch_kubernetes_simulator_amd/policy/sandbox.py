"""Host-side sandbox for policy programs (reference-compatible validator).

`SafeExecutor` reproduces the reference's checks
(`funsearch/safe_execution.py:15-168`) because they decide which LLM
candidates survive, and therefore what a search run does:

* `validate_code_content` - case-insensitive *substring* blacklist (so
  ``direction`` is rejected for containing ``dir``);
* `validate_code_structure` - AST: no imports, no ``__*`` attributes, bare-name
  calls only to whitelisted builtins / math / operator names;
* `create_safe_environment` - restricted ``__builtins__`` plus fake ``math`` and
  ``operator`` namespaces;
* `execute_policy_function` - one guarded call with a SIGALRM timeout.

This validator is *not* the real isolation boundary of this framework: the
policy compiler (`policy.compiler`) only lowers a whitelisted grammar to
bytecode, and the device interpreter enforces an instruction budget, so a
candidate that passes here but loops forever is stopped on the device rather
than hanging a worker (the reference has no eval-time timeout).
"""

from __future__ import annotations

import ast
import builtins
import math
import operator
import signal
import threading
from contextlib import contextmanager
from typing import Any, Dict


#: the tree of the last program that passed `validate_code_structure` on this
#: thread, handed once to the compiler (`take_parsed`): a child is validated
#: and then compiled, and parsing a few KB of source twice was ~15% of a
#: producer's time
_last = threading.local()


def take_parsed(code: str):
    """The validated tree of `code` if it was the last one validated on this
    thread (single use: the compiler may annotate it), else None."""
    hit = getattr(_last, "entry", None)
    if hit is not None and hit[0] is code:
        _last.entry = None
        return hit[1]
    return None


#: node types without children that the structure check never inspects
_LEAF_NODES = frozenset(c for base in (ast.expr_context, ast.operator, ast.unaryop, ast.cmpop, ast.boolop)
                        for c in base.__subclasses__())


class SafeExecutor:
    ALLOWED_BUILTINS = {
        "abs", "min", "max", "sum", "len", "range", "enumerate",
        "int", "float", "bool", "str", "round", "sorted",
    }
    ALLOWED_MODULES = {
        "math": ["sqrt", "log", "exp", "pow", "sin", "cos", "tan"],
        "operator": ["add", "sub", "mul", "truediv", "mod"],
    }
    FORBIDDEN_PATTERNS = [
        "import", "__", "exec", "eval", "open", "file", "input",
        "raw_input", "compile", "globals", "locals", "vars",
        "dir", "hasattr", "getattr", "setattr", "delattr",
    ]

    def __init__(self, timeout_seconds: int = 10):
        self.timeout_seconds = timeout_seconds

    # -- static checks -------------------------------------------------------
    def _is_allowed_function_call(self, func_name: str) -> bool:
        return any(func_name in names for names in self.ALLOWED_MODULES.values())

    def validate_code_structure(self, code: str) -> bool:
        try:
            tree = ast.parse(code)
        except SyntaxError as exc:
            raise ValueError(f"Syntax error in generated code: {exc}")
        allowed = self._allowed_calls()
        queue, i = [tree], 0
        while i < len(queue):                   # breadth-first: ast.walk's order
            node = queue[i]
            i += 1
            t = type(node)
            if t is ast.Call:
                if type(node.func) is ast.Name and node.func.id not in allowed:
                    raise ValueError(f"Function {node.func.id} not allowed")
            elif t is ast.Attribute:
                if node.attr.startswith("__"):
                    raise ValueError(f"Access to {node.attr} not allowed")
            elif t is ast.Import or t is ast.ImportFrom:
                raise ValueError("Import statements not allowed")
            for f in node._fields:
                v = getattr(node, f, None)
                if type(v) is list:
                    queue.extend(x for x in v if isinstance(x, ast.AST) and type(x) not in _LEAF_NODES)
                elif isinstance(v, ast.AST) and type(v) not in _LEAF_NODES:
                    queue.append(v)
        _last.entry = (code, tree)
        return True

    def _allowed_calls(self) -> frozenset:
        key = (frozenset(self.ALLOWED_BUILTINS), tuple((m, tuple(n)) for m, n in self.ALLOWED_MODULES.items()))
        if getattr(self, "_allowed_key", None) != key:
            self._allowed_key = key
            self._allowed = frozenset(self.ALLOWED_BUILTINS).union(
                *(set(names) for names in self.ALLOWED_MODULES.values()))
        return self._allowed

    def validate_code_content(self, code: str) -> bool:
        lowered = code.lower()
        hit = next((p for p in self.FORBIDDEN_PATTERNS if p in lowered), None)
        if hit is not None:
            raise ValueError(f"Forbidden pattern '{hit}' found in code")
        return True

    def validate(self, code: str) -> bool:
        """Both checks, content first (the order the reference generator uses)."""
        return self.validate_code_content(code) and self.validate_code_structure(code)

    # -- execution -----------------------------------------------------------
    @contextmanager
    def timeout_handler(self, seconds: int):
        """SIGALRM-based timeout; a no-op off the main thread (signals are
        main-thread only), where the device step budget is the guard."""
        if threading.current_thread() is not threading.main_thread() or seconds <= 0:
            yield
            return

        def _expire(signum, frame):
            raise TimeoutError(f"Code execution timed out after {seconds} seconds")

        previous = signal.signal(signal.SIGALRM, _expire)
        signal.alarm(int(seconds))
        try:
            yield
        finally:
            signal.alarm(0)
            signal.signal(signal.SIGALRM, previous)

    def create_safe_environment(self) -> Dict[str, Any]:
        safe_builtins = {n: getattr(builtins, n) for n in self.ALLOWED_BUILTINS if hasattr(builtins, n)}

        def namespace(label, module, names):
            return type(label, (), {n: getattr(module, n) for n in names})()

        return {
            "__builtins__": safe_builtins,
            "math": namespace("SafeMath", math, self.ALLOWED_MODULES["math"]),
            "operator": namespace("SafeOperator", operator, self.ALLOWED_MODULES["operator"]),
        }

    def execute_policy_function(self, code: str, pod, node) -> float:
        self.validate_code_content(code)
        self.validate_code_structure(code)
        env = self.create_safe_environment()
        env.update({"pod": pod, "node": node})
        try:
            with self.timeout_handler(self.timeout_seconds):
                exec(code, env)
                if "priority_function" not in env:
                    raise ValueError("Generated code must define 'priority_function'")
                result = env["priority_function"](pod, node)
                if not isinstance(result, (int, float)):
                    raise ValueError(f"Priority function must return a number, got {type(result)}")
                if math.isnan(result) or math.isinf(result):
                    raise ValueError("Priority function returned NaN or infinite value")
                return float(result)
        except TimeoutError:
            raise ValueError("Code execution timed out")
        except Exception as exc:
            raise ValueError(f"Error executing generated code: {exc}")


def compile_priority_function(code: str, executor: "SafeExecutor | None" = None):
    """``exec`` a policy program in the restricted namespace and return its
    ``priority_function`` (no validation, no timeout: the reference's
    `FunSearchScheduler._compile_policy` semantics)."""
    env = (executor or SafeExecutor()).create_safe_environment()
    exec(code, env)
    fn = env.get("priority_function")
    if not fn:
        raise ValueError("No priority_function found in evolved code")
    return fn
