"""LLM backends for program generation.

Every backend exposes the tiny slice of the OpenAI client that the generator
uses -- ``client.chat.completions.create(model=..., messages=[...],
temperature=..., max_tokens=...)`` returning ``resp.choices[0].message.content``
-- so `LLMCodeGenerator` (reference `funsearch/safe_execution.py:273-317`) works
unchanged with any of them:

* `OpenAICompatibleClient` -- HTTP POST to ``{base_url}/chat/completions``
  (OpenRouter, vLLM, any OpenAI-compatible server) with retry + exponential
  backoff; the API key comes from the config or the ``FKS_LLM_API_KEY`` /
  ``OPENROUTER_API_KEY`` / ``OPENAI_API_KEY`` environment variables (never from
  committed files).  The reference has no retries.
* `MutationClient` -- deterministic, offline: parses the parent programs out of
  the prompt and returns a mutated policy body: constant perturbation, term
  insertion (a fixed library, or new terms from a feature grammar that covers
  every template field), ast-level operator / aggregation swaps, wrapping a
  subexpression (abs / min / max / square / power), subexpression crossover
  between the two parents, statement deletion, line crossover.  Used for
  tests, benchmarks and air-gapped runs.
* `ScriptedClient` -- replays a fixed list of responses (tests).
* `LatencyClient` -- wraps any client and answers after a delay drawn from
  ``latency_s`` = [lo, hi] seconds: a remote LLM's response time, to size and
  measure the search's request fan-out (``llm.concurrency``, steady mode)
  without a network.
"""

from __future__ import annotations

import ast
import functools
import json
import os
import random
import re
import textwrap
import threading
import time
from dataclasses import dataclass
from typing import Callable, List, Optional, Sequence


# ---------------------------------------------------------------- response shape
@dataclass
class _Message:
    content: str


@dataclass
class _Choice:
    message: _Message


@dataclass
class ChatResponse:
    choices: List[_Choice]
    latency_s: float = 0.0


def _response(text: str, latency: float = 0.0) -> ChatResponse:
    return ChatResponse([_Choice(_Message(text))], latency)


class _Completions:
    def __init__(self, fn: Callable[..., ChatResponse]):
        self._fn = fn

    def create(self, **kw) -> ChatResponse:
        return self._fn(**kw)


class _Chat:
    def __init__(self, fn):
        self.completions = _Completions(fn)


class BaseClient:
    """OpenAI-client-shaped object: ``client.chat.completions.create(...)``."""

    def __init__(self):
        self.chat = _Chat(self._create)
        self.calls = 0
        self.failures = 0
        self._lock = threading.Lock()

    def _create(self, model=None, messages=None, temperature=0.7, max_tokens=400, **_) -> ChatResponse:
        raise NotImplementedError


# ---------------------------------------------------------------- HTTP backend
class OpenAICompatibleClient(BaseClient):
    def __init__(self, api_key: Optional[str] = None, base_url: str = "https://openrouter.ai/api/v1",
                 timeout_s: float = 60.0, max_retries: int = 4, backoff_s: float = 1.0):
        super().__init__()
        if not api_key or api_key in ("OPENROUTER_API_KEY", "API_KEY"):
            api_key = (os.environ.get("FKS_LLM_API_KEY") or os.environ.get("OPENROUTER_API_KEY")
                       or os.environ.get("OPENAI_API_KEY"))
        self.api_key = api_key
        self.base_url = base_url.rstrip("/")
        self.timeout_s = timeout_s
        self.max_retries = max_retries
        self.backoff_s = backoff_s

    def _create(self, model=None, messages=None, temperature=0.7, max_tokens=400, **_) -> ChatResponse:
        import requests
        if not self.api_key:
            raise RuntimeError("no API key: set FKS_LLM_API_KEY (or OPENROUTER_API_KEY / OPENAI_API_KEY)")
        body = {"model": model, "messages": messages, "temperature": temperature, "max_tokens": max_tokens}
        headers = {"Authorization": f"Bearer {self.api_key}", "Content-Type": "application/json"}
        err: Optional[Exception] = None
        for attempt in range(self.max_retries + 1):
            t0 = time.time()
            try:
                r = requests.post(f"{self.base_url}/chat/completions", headers=headers, data=json.dumps(body),
                                  timeout=self.timeout_s)
            except Exception as exc:  # network errors are retried
                err = exc
            else:
                if r.status_code == 200:
                    text = r.json()["choices"][0]["message"]["content"]
                    with self._lock:
                        self.calls += 1
                    return _response(text, time.time() - t0)
                if r.status_code not in (408, 409, 425, 429, 500, 502, 503, 504):
                    with self._lock:
                        self.failures += 1
                    raise RuntimeError(f"LLM HTTP {r.status_code}: {r.text[:200]}")   # not retryable
                err = RuntimeError(f"LLM HTTP {r.status_code}")
            if attempt < self.max_retries:
                time.sleep(self.backoff_s * (2 ** attempt) * (0.5 + random.random()))
        with self._lock:
            self.failures += 1
        raise RuntimeError(f"LLM request failed after {self.max_retries + 1} attempts: {err}")


# ---------------------------------------------------------------- scripted backend
class ScriptedClient(BaseClient):
    def __init__(self, responses: Sequence[str]):
        super().__init__()
        self.responses = list(responses)

    def _create(self, **_) -> ChatResponse:
        with self._lock:
            text = self.responses[self.calls % len(self.responses)]
            self.calls += 1
        return _response(text)


# ---------------------------------------------------------------- offline mutation backend
_PARENT_RE = re.compile(r"\nPolicy v_\d+ \(score: [-\d.]+\):\n(.*?)(?=\nPolicy v_\d+ \(score:|\n\nPerformance feedback:)",
                        re.S)

#: policy-body fragments the mutation backend can insert (each defines nothing
#: new, only updates ``score``; all are valid inside the template)
TERM_LIBRARY = [
    "score += {c} * (node.cpu_milli_total - node.cpu_milli_left + pod.cpu_milli) / max(1, node.cpu_milli_total)",
    "score += {c} * (node.memory_mib_total - node.memory_mib_left + pod.memory_mib) / max(1, node.memory_mib_total)",
    "score -= {c} * abs((node.cpu_milli_left - pod.cpu_milli) / max(1, node.cpu_milli_total) - "
    "(node.memory_mib_left - pod.memory_mib) / max(1, node.memory_mib_total))",
    "score -= {c} * (sum(g.gpu_milli_left for g in node.gpus) % max(1, pod.gpu_milli)) / 1000",
    "score += {c} * (node.gpu_left - pod.num_gpu) / max(1, len(node.gpus))",
    "score -= {c} * (node.gpu_left - pod.num_gpu) / max(1, len(node.gpus))",
    "if pod.num_gpu == 0 and len(node.gpus) > 0:\n    score -= {c}",
    "if pod.num_gpu > 0:\n    score += {c} * (1 - min(g.gpu_milli_left for g in node.gpus if g.gpu_milli_left >= pod.gpu_milli) / 1000)",
    "score += {c} * sum(1 for g in node.gpus if 0 < g.gpu_milli_left < g.gpu_milli_total) / max(1, len(node.gpus))",
    "if node.cpu_milli_left > pod.cpu_milli * 2 and node.memory_mib_left > pod.memory_mib * 2:\n    score += {c}",
    "score += {c} * min(node.cpu_milli_left - pod.cpu_milli, node.memory_mib_left - pod.memory_mib) / "
    "max(node.cpu_milli_total, node.memory_mib_total)",
    # piecewise utilisation (a free fraction that counts only below / above a load level)
    "if node.cpu_milli_left > 0.3 * node.cpu_milli_total:\n    score += {c} * node.cpu_milli_left / max(1, node.cpu_milli_total)",
    "if node.memory_mib_left > 0.3 * node.memory_mib_total:\n    score += {c} * node.memory_mib_left / max(1, node.memory_mib_total)",
    "if pod.num_gpu > 0 and len(node.gpus) > 0:\n    score += {c} * sum(g.gpu_milli_left for g in node.gpus) / "
    "max(1, sum(g.gpu_milli_total for g in node.gpus))",
    "if node.cpu_milli_left < 0.1 * node.cpu_milli_total or node.memory_mib_left < 0.1 * node.memory_mib_total:\n"
    "    score -= {c}",
    # GPU fragmentation: spread of the per-GPU free compute, partially used GPUs left behind
    "if pod.num_gpu > 0 and len(node.gpus) > 0:\n    score -= {c} * (max(g.gpu_milli_left for g in node.gpus) - "
    "min(g.gpu_milli_left for g in node.gpus)) / 1000",
    "score -= {c} * sum(1 for g in node.gpus if 0 < g.gpu_milli_left - pod.gpu_milli < 200) / max(1, len(node.gpus))",
    # node scale and the balance of what the pod leaves behind
    "score += {c} * min(1.0, node.cpu_milli_total / 100000)",
    "score -= {c} * abs(node.cpu_milli_left / max(1, node.memory_mib_left) - pod.cpu_milli / max(1, pod.memory_mib)) / 100",
]


#: normalised (pod, node) features for freshly built terms (`_random_expr`):
#: every template field appears in at least one, so a structural mutation can
#: bring a field into a program that never used it
FEATURES = [
    "node.cpu_milli_left / max(1, node.cpu_milli_total)",
    "node.memory_mib_left / max(1, node.memory_mib_total)",
    "(node.cpu_milli_left - pod.cpu_milli) / max(1, node.cpu_milli_total)",
    "(node.memory_mib_left - pod.memory_mib) / max(1, node.memory_mib_total)",
    "pod.cpu_milli / max(1, node.cpu_milli_left)",
    "pod.memory_mib / max(1, node.memory_mib_left)",
    "node.gpu_left / max(1, len(node.gpus))",
    "(node.gpu_left - pod.num_gpu) / max(1, len(node.gpus))",
    "sum(g.gpu_milli_left for g in node.gpus) / max(1, 1000 * len(node.gpus))",
    "(max(g.gpu_milli_left for g in node.gpus) if node.gpus else 0) / 1000",
    "(min(g.gpu_milli_left for g in node.gpus) if node.gpus else 1000) / 1000",
    "sum(1 for g in node.gpus if g.gpu_milli_left >= pod.gpu_milli) / max(1, len(node.gpus))",
    "len([g for g in node.gpus if 0 < g.gpu_milli_left < g.gpu_milli_total]) / max(1, len(node.gpus))",
    "sum(g.gpu_milli_left - pod.gpu_milli for g in node.gpus if g.gpu_milli_left >= pod.gpu_milli) / 1000",
    "pod.gpu_milli / 1000",
    "pod.num_gpu",
    "min(node.cpu_milli_left / max(1, pod.cpu_milli), node.memory_mib_left / max(1, pod.memory_mib)) / 100",
    "(1.0 if node.cpu_milli_left < 0.3 * node.cpu_milli_total else 0.0)",
    "(1.0 if node.memory_mib_left < 0.3 * node.memory_mib_total else 0.0)",
    "(1.0 if node.gpu_left == len(node.gpus) else 0.0)",
]

#: names a moved subexpression may mention (anything else is a local of its parent)
_FREE_OK = frozenset({"pod", "node", "math", "abs", "min", "max", "sum", "len", "int", "float", "round", "sorted"})
_NUMERIC_FIELDS = frozenset({"cpu_milli", "memory_mib", "num_gpu", "gpu_milli", "cpu_milli_left", "memory_mib_left",
                             "gpu_left", "cpu_milli_total", "memory_mib_total"})


def _free_names(node: ast.AST) -> set:
    """Names read in `node` that no comprehension inside it binds."""
    bound, used = set(), set()
    for n in ast.walk(node):
        if isinstance(n, ast.comprehension):
            for t in ast.walk(n.target):
                if isinstance(t, ast.Name):
                    bound.add(t.id)
        elif isinstance(n, ast.Lambda):
            bound.update(a.arg for a in n.args.args)
        elif isinstance(n, ast.Name) and isinstance(n.ctx, ast.Load):
            used.add(n.id)
    return used - bound


def _numeric_subexprs(tree: ast.AST, portable: bool) -> list:
    """Expression nodes that hold a number and may be swapped for another
    numeric expression: arithmetic, numeric literals, pod / node scalar fields,
    abs / min / max / sum calls -- never inside a comprehension's iterable
    (keeps `for g in node.gpus` intact), an assignment target or a called
    name.  `portable`: only those that mention no parent-local name (they may
    move into another program).  One pass, pre-order."""
    out = []
    Name, Load, Constant, Attribute, Call = ast.Name, ast.Load, ast.Constant, ast.Attribute, ast.Call
    arith = (ast.BinOp, ast.UnaryOp)

    def visit(n, skipped):
        # returns (names read, names bound) of the subtree when `portable`
        used, bound = (set(), set()) if portable else (None, None)
        t = type(n)
        ok = False
        if not skipped:
            ok = (t in arith
                  or (t is Constant and isinstance(n.value, (int, float)) and not isinstance(n.value, bool))
                  or (t is Attribute and type(n.value) is Name and n.value.id in ("pod", "node")
                      and n.attr in _NUMERIC_FIELDS)
                  or (t is Call and type(n.func) is Name and n.func.id in ("abs", "min", "max", "sum")))
        if ok:
            slot = len(out)
            out.append(n)
        if portable:
            if t is Name:
                if type(n.ctx) is Load:
                    used.add(n.id)
            elif t is ast.comprehension:
                bound.update(x.id for x in ast.walk(n.target) if isinstance(x, ast.Name))
            elif t is ast.Lambda:
                bound.update(a.arg for a in n.args.args)
        for f in n._fields:
            v = getattr(n, f, None)
            kids = v if type(v) is list else (v,)
            sk = skipped or (t is ast.comprehension and f == "iter") or (t is Call and f == "func") \
                or (t is ast.Assign and f == "targets") or (t is ast.AugAssign and f == "target")
            for c in kids:
                if isinstance(c, ast.AST):
                    u, bd = visit(c, sk)
                    if portable:
                        used |= u
                        bound |= bd
        if ok and portable and not (used - bound <= _FREE_OK):
            out[slot] = None
        return used, bound

    visit(tree, False)
    return [n for n in out if n is not None]


def _scope_sets(tree: ast.AST) -> dict:
    """id(node) -> (names read, names bound by comprehensions / lambdas) over
    the node's subtree, in one bottom-up pass (`_free_names` of every node
    without re-walking each subtree)."""
    memo = {}

    def rec(n):
        used, bound = set(), set()
        t = type(n)
        if t is ast.Name:
            if type(n.ctx) is ast.Load:
                used.add(n.id)
        elif t is ast.comprehension:
            bound.update(x.id for x in ast.walk(n.target) if isinstance(x, ast.Name))
        elif t is ast.Lambda:
            bound.update(a.arg for a in n.args.args)
        for c in ast.iter_child_nodes(n):
            u, b = rec(c)
            used |= u
            bound |= b
        memo[id(n)] = (used, bound)
        return used, bound

    rec(tree)
    return memo


def _replace(tree: ast.AST, target: ast.AST, new: ast.AST) -> ast.AST:
    """`tree` with the (single) occurrence of node `target` swapped for `new`."""
    if tree is target:
        return new
    for parent in ast.walk(tree):
        for f in parent._fields:
            v = getattr(parent, f, None)
            if v is target:
                setattr(parent, f, new)
                return tree
            if type(v) is list:
                for i, x in enumerate(v):
                    if x is target:
                        v[i] = new
                        return tree
    return tree


@functools.lru_cache(maxsize=4096)   # parents repeat across thousands of children
def _extract_body(program: str) -> Optional[str]:
    """The logic between ``score = 0.0`` and the final return of a
    template-shaped program, dedented to 4 spaces; else the whole function
    body after the feasibility prologue."""
    from ..policy.template import PolicyTemplate
    try:
        return PolicyTemplate.extract_logic(program)
    except ValueError:
        pass
    try:
        fn = next(n for n in ast.parse(program).body if isinstance(n, ast.FunctionDef))
    except Exception:
        return None
    lines = program.splitlines()
    body = fn.body
    # skip docstring + feasibility checks (leading `if ...: return 0` blocks)
    start = 0
    while start < len(body) and (isinstance(body[start], ast.Expr) or
                                 (isinstance(body[start], ast.If) and _returns_zero(body[start]))):
        start += 1
    if start >= len(body):
        return None
    seg = lines[body[start].lineno - 1: body[-1].end_lineno]
    # turn a trailing `return <expr>` into `score = <expr>` (template adds the return)
    text = "\n".join(seg)
    text = re.sub(r"\n\s*return max\(1, int\((.*)\)\)\s*$", r"\n    score = \1", "\n" + text).lstrip("\n")
    text = re.sub(r"^(\s*)return max\(1, int\((.*)\)\)\s*$", r"\1score = \2", text, flags=re.M)
    text = re.sub(r"^(\s*)return (.+)$", r"\1score = \2", text, flags=re.M)
    return text


def _returns_zero(node: ast.If) -> bool:
    return any(isinstance(n, ast.Return) and isinstance(n.value, ast.Constant) and n.value.value == 0
               for n in ast.walk(node))


class MutationClient(BaseClient):
    """Deterministic offline program mutator (seeded)."""

    def __init__(self, seed: int = 0, temperature_scale: float = 1.0):
        super().__init__()
        self.rng = random.Random(seed)
        self.scale = temperature_scale

    def _create(self, model=None, messages=None, temperature=0.7, **_) -> ChatResponse:
        prompt = messages[-1]["content"] if messages else ""
        parents = [p.strip("\n") + "\n" for p in _PARENT_RE.findall(prompt + "\n\nPerformance feedback:")]
        with self._lock:
            self.calls += 1
            rng = random.Random(self.rng.random())
        bodies = [textwrap.dedent(b).strip("\n") for b in (_extract_body(p) for p in parents) if b]
        other = None
        if not bodies:
            body = "score = 1000.0"
        elif len(bodies) >= 2 and rng.random() < 0.25:
            body = self._crossover(bodies[0], bodies[1], rng)
        else:
            k = rng.randrange(len(bodies))
            body = bodies[k]
            other = bodies[1 - k] if len(bodies) >= 2 else None
        if len(body) > self.max_body_chars:
            # bloat control: a parent grown past the size of LLM-written policies
            # loses random score terms first (children of ever-growing parents
            # cost the producers, the JIT's registers and the host fallbacks)
            body = self._prune(body, rng, int(0.8 * self.max_body_chars))
        for _ in range(1 + int(rng.random() < 0.5 * max(0.2, temperature))):
            body = self._mutate(body, rng, other)
        return _response(self._indent(body))

    #: body size (characters) past which a parent is pruned before mutation; the
    #: longest LLM-found champion bodies in data/policies are ~2,300 characters
    max_body_chars = 2400

    @staticmethod
    def _score_only(stmt: ast.stmt) -> bool:
        """A statement that only updates ``score`` (droppable without leaving a
        later read of a name it defined)."""
        def upd(s):
            if isinstance(s, ast.AugAssign):
                return isinstance(s.target, ast.Name) and s.target.id == "score"
            if isinstance(s, ast.Assign):
                return len(s.targets) == 1 and isinstance(s.targets[0], ast.Name) and s.targets[0].id == "score"
            if isinstance(s, ast.If):
                return all(upd(x) for x in s.body + s.orelse)
            return False
        return upd(stmt)

    def _prune(self, body: str, rng: random.Random, limit: int) -> str:
        """Drop random score-only top-level statements until the body is at most
        `limit` characters; removes their source lines, so the rest of the text
        is kept verbatim (no unparse)."""
        try:
            tree = ast.parse(body)
        except SyntaxError:
            return body
        lines = body.split("\n")
        line_of = {}
        for i, st in enumerate(tree.body):
            for ln in range(st.lineno, (st.end_lineno or st.lineno) + 1):
                line_of.setdefault(ln, []).append(i)
        cands = [i for i, st in enumerate(tree.body)
                 if i > 0 and self._score_only(st)
                 and all(line_of[ln] == [i] for ln in range(st.lineno, (st.end_lineno or st.lineno) + 1))]
        drop, size = set(), len(body)
        while size > limit and cands:
            i = cands.pop(rng.randrange(len(cands)))
            st = tree.body[i]
            for ln in range(st.lineno, (st.end_lineno or st.lineno) + 1):
                drop.add(ln)
                size -= len(lines[ln - 1]) + 1
        return "\n".join(l for k, l in enumerate(lines, 1) if k not in drop)

    # -- operators ----------------------------------------------------------------------
    #: (cumulative probability, operator).  Structural operators (new terms from
    #: the feature grammar, operator / aggregation swaps, subexpression crossover,
    #: wrapping) change a program's shape; constant perturbations keep it.
    OPERATORS = ((0.30, "constants"), (0.42, "library_term"), (0.57, "random_term"), (0.66, "swap_binop"),
                 (0.74, "swap_aggregate"), (0.84, "subexpr_crossover"), (0.90, "wrap"), (0.96, "drop"),
                 (1.00, "swap_comparison"))

    def _mutate(self, body: str, rng: random.Random, other: Optional[str] = None) -> str:
        op = rng.random()
        name = next(n for p, n in self.OPERATORS if op < p)
        self.last_op = name
        if name == "constants":
            return self._perturb_constants(body, rng)
        if name == "library_term":
            term = rng.choice(TERM_LIBRARY).format(c=self._const(rng))
            return body.rstrip("\n") + "\n" + term
        if name == "random_term":
            return body.rstrip("\n") + "\n" + self._random_term(rng)
        if name == "drop":
            return self._drop_statement(body, rng)
        if name == "swap_comparison":
            return self._swap_comparison(body, rng)
        out = self._structural(name, body, rng, other)
        return out if out is not None else self._perturb_constants(body, rng)

    # -- structural operators (ast) -------------------------------------------------------
    def _random_expr(self, rng: random.Random, depth: int = 0) -> str:
        r = rng.random()
        if depth >= 2 or r < 0.45:
            return f"({rng.choice(FEATURES)})"
        a, b = self._random_expr(rng, depth + 1), self._random_expr(rng, depth + 1)
        if r < 0.65:
            return f"({a} {rng.choice(['+', '-', '*'])} {b})"
        if r < 0.8:
            return f"{rng.choice(['min', 'max'])}({a}, {b})"
        if r < 0.9:
            return f"abs({a} - {b})"
        # a square as a product: `x ** 2` is a libm pow call per node on the device
        # (and for CPython), x * x one multiply
        return f"({a}) * ({a})"

    def _random_term(self, rng: random.Random) -> str:
        e = self._random_expr(rng)
        c = self._const(rng)
        form = rng.random()
        if form < 0.45:
            return f"score += {c} * {e}"
        if form < 0.9:
            return f"score -= {c} * {e}"
        return f"if {e} > {round(rng.uniform(0, 1), 3)}:\n    score += {c}"

    def _structural(self, name: str, body: str, rng: random.Random, other: Optional[str]) -> Optional[str]:
        try:
            tree = ast.parse(body)
        except SyntaxError:
            return None
        if name == "swap_binop":
            ops = [n for n in ast.walk(tree) if isinstance(n, ast.BinOp)
                   and isinstance(n.op, (ast.Add, ast.Sub, ast.Mult, ast.Div))]
            if not ops:
                return None
            n = rng.choice(ops)
            swap = {ast.Add: ast.Sub, ast.Sub: ast.Add, ast.Mult: ast.Div, ast.Div: ast.Mult}
            n.op = swap[type(n.op)]()
            if isinstance(n.op, ast.Div):   # never divide by a possibly-zero right operand
                n.right = ast.Call(ast.Name("max", ast.Load()), [ast.Constant(1), n.right], [])
        elif name == "swap_aggregate":
            calls = [n for n in ast.walk(tree) if isinstance(n, ast.Call) and isinstance(n.func, ast.Name)
                     and n.func.id in ("min", "max", "sum") and not n.keywords]
            if not calls:
                return None
            n = rng.choice(calls)
            if len(n.args) == 1 and isinstance(n.args[0], ast.GeneratorExp):
                n.func.id = rng.choice([f for f in ("min", "max", "sum") if f != n.func.id])
                if n.func.id in ("min", "max"):   # an empty GPU list would raise: guard like the features do
                    node = ast.IfExp(ast.Attribute(ast.Name("node", ast.Load()), "gpus", ast.Load()), n,
                                     ast.Constant(0))
                    tree = _replace(tree, n, node)
            elif len(n.args) >= 2 and n.func.id in ("min", "max"):
                n.func.id = "max" if n.func.id == "min" else "min"
            else:
                return None
        elif name == "subexpr_crossover":
            if not other:
                return None
            try:
                donor = ast.parse(other)
            except SyntaxError:
                return None
            targets = _numeric_subexprs(tree, portable=False)
            pieces = [n for n in _numeric_subexprs(donor, portable=True) if not isinstance(n, ast.Constant)]
            if not targets or not pieces:
                return None
            tree = _replace(tree, rng.choice(targets), rng.choice(pieces))
        elif name == "wrap":
            targets = [n for n in _numeric_subexprs(tree, portable=False) if not isinstance(n, ast.Constant)]
            if not targets:
                return None
            t = rng.choice(targets)
            c = ast.Constant(float(self._const(rng)))
            u = rng.random()   # abs / min-max / square 30% each, a fractional power 10%
            form = 0 if u < 0.3 else 1 if u < 0.6 else 2 if u < 0.9 else 3
            if form == 0:
                new = ast.Call(ast.Name("abs", ast.Load()), [t], [])
            elif form == 1:
                new = ast.Call(ast.Name(rng.choice(["min", "max"]), ast.Load()), [t, c], [])
            elif form == 2:
                new = ast.BinOp(t, ast.Mult(), t)
            else:
                new = ast.BinOp(ast.Call(ast.Name("abs", ast.Load()), [t], []), ast.Pow(),
                                ast.Constant(round(rng.uniform(0.3, 2.0), 2)))
            tree = _replace(tree, t, new)
        else:
            return None
        try:
            out = ast.unparse(tree)             # unparse needs no source locations
            ast.parse(out)
        except Exception:
            return None
        return out

    @staticmethod
    def _const(rng: random.Random) -> str:
        return repr(round(10 ** rng.uniform(-1, 3), 3))

    def _perturb_constants(self, body: str, rng: random.Random) -> str:
        nums = list(re.finditer(r"(?<![\w.])(\d+\.\d+|\d+)(?![\w.])", body))
        if not nums:
            return body
        m = rng.choice(nums)
        v = float(m.group(1))
        nv = v * (1 + rng.gauss(0, 0.3 * self.scale)) if v != 0 else rng.uniform(0, 1)
        text = repr(round(nv, 4)) if "." in m.group(1) else str(max(0, int(round(nv))))
        return body[:m.start()] + text + body[m.end():]

    @staticmethod
    def _drop_statement(body: str, rng: random.Random) -> str:
        lines = body.split("\n")
        cands = [i for i, l in enumerate(lines) if re.match(r"^score\s*[-+*/]?=", l.strip())
                 and not l.startswith(" ")]
        if len(cands) <= 1:
            return body
        i = rng.choice(cands)
        return "\n".join(lines[:i] + lines[i + 1:])

    @staticmethod
    def _swap_comparison(body: str, rng: random.Random) -> str:
        swaps = [(" < ", " <= "), (" > ", " >= "), (" <= ", " < "), (" >= ", " > "), (" * 0.", " * 1.")]
        a, b = rng.choice(swaps)
        return body.replace(a, b, 1) if a in body else body

    @staticmethod
    def _crossover(a: str, b: str, rng: random.Random) -> str:
        la, lb = a.split("\n"), b.split("\n")
        cut_a = rng.randint(1, max(1, len(la)))
        top = [l for l in lb if l.startswith("score")]
        return "\n".join(la[:cut_a] + top[-2:])

    @staticmethod
    def _indent(body: str) -> str:
        lines = [l for l in body.split("\n")]
        # normalise: the template inserts the body after 4 spaces on the first line
        base = min((len(l) - len(l.lstrip()) for l in lines if l.strip()), default=0)
        out = []
        for l in lines:
            if not l.strip():
                continue
            out.append("    " + l[base:])
        return "\n".join(out).lstrip()


class FaultInjectingClient(BaseClient):
    """Wraps a client and fails a fraction of requests (SURVEY section 5.3
    fault-injection hook): the search must treat them like real LLM errors."""

    def __init__(self, inner: BaseClient, rate: float, seed: int = 0):
        super().__init__()
        self.inner, self.rate = inner, float(rate)
        self._rng = random.Random(seed)
        self.injected = 0

    def _create(self, **kw) -> ChatResponse:
        with self._lock:
            fail = self._rng.random() < self.rate
            if fail:
                self.injected += 1
        if fail:
            raise RuntimeError("injected LLM failure")
        return self.inner._create(**kw)


class LatencyClient(BaseClient):
    """The inner client's reply after a delay drawn uniformly from [lo, hi]
    seconds (thread-safe; the wait releases the GIL, as an HTTP request does)."""

    def __init__(self, inner: BaseClient, lo: float, hi: float, seed: int = 0):
        super().__init__()
        if not 0 <= lo <= hi:
            raise ValueError(f"latency range [{lo}, {hi}]")
        self.inner, self.lo, self.hi = inner, float(lo), float(hi)
        self._rng = random.Random(seed)
        self.waited_s = 0.0

    def _create(self, **kw) -> ChatResponse:
        with self._lock:
            d = self._rng.uniform(self.lo, self.hi)
            self.waited_s += d
            self.calls += 1
        time.sleep(d)
        r = self.inner._create(**kw)
        r.latency_s += d
        return r


def make_client(cfg: dict) -> BaseClient:
    """Client from the ``llm`` / ``openrouter`` section of a config
    (``fault_rate`` > 0 wraps it in a `FaultInjectingClient`; ``latency_s``
    = [lo, hi] in a `LatencyClient`)."""
    backend = cfg.get("backend", "openai")
    if backend in ("mutation", "offline"):
        client: BaseClient = MutationClient(int(cfg.get("seed", 0)))
    elif backend == "scripted":
        client = ScriptedClient(cfg["responses"])
    else:
        client = OpenAICompatibleClient(cfg.get("api_key"), cfg.get("base_url", "https://openrouter.ai/api/v1"),
                                        float(cfg.get("timeout_s", 60)), int(cfg.get("max_retries", 4)))
    if float(cfg.get("fault_rate", 0) or 0) > 0:
        client = FaultInjectingClient(client, float(cfg["fault_rate"]), int(cfg.get("seed", 0)) + 17)
    lat = cfg.get("latency_s")
    if lat:
        lo, hi = (float(lat), float(lat)) if isinstance(lat, (int, float)) else (float(lat[0]), float(lat[1]))
        client = LatencyClient(client, lo, hi, int(cfg.get("seed", 0)) + 29)
    return client


def remote_like(cfg: dict) -> bool:
    """Requests to this backend spend their time waiting (HTTP, or a modelled
    latency), not computing: worth many in flight per process."""
    return cfg.get("backend", "openai") not in ("mutation", "offline", "scripted") or bool(cfg.get("latency_s"))
