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
  the prompt and returns a mutated policy body (constant perturbation,
  operator / comparison swaps, term insertion from a feature library, term
  deletion, crossover of two parents).  Used for tests, benchmarks and
  air-gapped runs.
* `ScriptedClient` -- replays a fixed list of responses (tests).
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
]


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
        if not bodies:
            body = "score = 1000.0"
        elif len(bodies) >= 2 and rng.random() < 0.25:
            body = self._crossover(bodies[0], bodies[1], rng)
        else:
            body = rng.choice(bodies)
        for _ in range(1 + int(rng.random() < 0.5 * max(0.2, temperature))):
            body = self._mutate(body, rng)
        return _response(self._indent(body))

    # -- operators ----------------------------------------------------------------------
    def _mutate(self, body: str, rng: random.Random) -> str:
        op = rng.random()
        if op < 0.45:
            return self._perturb_constants(body, rng)
        if op < 0.75:
            term = rng.choice(TERM_LIBRARY).format(c=self._const(rng))
            return body.rstrip("\n") + "\n" + term
        if op < 0.9:
            return self._drop_statement(body, rng)
        return self._swap_comparison(body, rng)

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


def make_client(cfg: dict) -> BaseClient:
    """Client from the ``llm`` / ``openrouter`` section of a config
    (``fault_rate`` > 0 wraps it in a `FaultInjectingClient`)."""
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
    return client
