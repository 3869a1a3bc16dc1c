"""Constant polish: batched device search over the numeric literals of a
program (couples program islands to the device).

An LLM (or the offline mutator) proposes program *structure*; the numbers in
it -- weights, thresholds -- are guesses.  Every numeric literal of a compiled
program is its own constant-pool entry (`policy.compiler`), and the native
backend compiles a program's *shape* once with constants as data
(`policy.native_codegen`), so thousands of constant settings of one program
replay on the MI355X in a single k_replay_native launch with one JIT compile.

`polish` runs a few rounds of a (1 + lambda) evolution strategy over the
literals (log-normal multiplicative steps for floats, relative steps for
integers >= 2; 0/1 literals, which usually encode structure, stay fixed),
keeps the best-scoring setting, and writes it back into the program TEXT at
the literals' source spans -- the result is an ordinary program, re-scored
exactly through the normal evaluation path before it enters a population.
"""

from __future__ import annotations

import math
import random
from dataclasses import dataclass, replace
from typing import List, Optional, Sequence, Tuple

import numpy as np

from ..policy.bytecode import TAG_FLOAT
from ..policy.compiler import CompiledPolicy, try_compile


@dataclass
class PolishResult:
    code: str
    score: float
    base_score: float
    evaluated: int
    rounds: int
    improved: bool


def tunable_literals(prog: CompiledPolicy) -> List[int]:
    """Positions (in `prog.literals`) of the literals worth tuning."""
    out = []
    for j, (idx, *_span) in enumerate(prog.literals):
        if prog.ctag[idx] == TAG_FLOAT:
            if prog.fconst[idx] != 0.0 and math.isfinite(prog.fconst[idx]):
                out.append(j)
        elif abs(int(prog.iconst[idx])) >= 2:
            out.append(j)
    return out


def with_values(prog: CompiledPolicy, values: dict) -> CompiledPolicy:
    """Same bytecode and shape, other literal values ({pool index: value})."""
    f, i = list(prog.fconst), list(prog.iconst)
    for idx, v in values.items():
        if prog.ctag[idx] == TAG_FLOAT:
            f[idx] = float(v)
        else:
            i[idx] = int(v)
    out = replace(prog, fconst=f, iconst=i)
    for k in ("_shape_key", "_jit_key"):   # literals are data: the variant keeps its shape
        if k in prog.__dict__:
            out.__dict__[k] = prog.__dict__[k]
    return out


def _literal_text(prog: CompiledPolicy, idx: int, v) -> str:
    if prog.ctag[idx] == TAG_FLOAT:
        t = repr(float(v))
        return t if ("e" in t or "." in t or "n" in t) else t + ".0"
    return str(int(v))


def rewrite_source(prog: CompiledPolicy, values: dict) -> str:
    """Program text with the literals at their source spans replaced."""
    lines = prog.source.split("\n")
    spans = sorted(((ln, col, eln, ecol, idx) for idx, ln, col, eln, ecol in prog.literals if idx in values),
                   reverse=True)
    for ln, col, eln, ecol, idx in spans:
        if ln != eln:
            continue   # literals never span lines; be safe
        row = lines[ln - 1]
        lines[ln - 1] = row[:col] + _literal_text(prog, idx, values[idx]) + row[ecol:]
    return "\n".join(lines)


def _perturb(prog: CompiledPolicy, base: dict, tune: Sequence[int], sigma: float, rng: random.Random) -> dict:
    vals = dict(base)
    k = max(1, min(len(tune), int(rng.expovariate(1.0)) + 1))   # mostly 1-2 literals per variant
    for j in rng.sample(list(tune), k):
        idx = prog.literals[j][0]
        v = vals[idx]
        if prog.ctag[idx] == TAG_FLOAT:
            nv = v * math.exp(rng.gauss(0.0, sigma))
            if rng.random() < 0.1:
                nv = -nv
            vals[idx] = float(f"{nv:.6g}")
        else:
            step = max(1, int(round(abs(v) * sigma * abs(rng.gauss(0.0, 1.0)))))
            vals[idx] = int(v + (step if rng.random() < 0.5 else -step))
    return vals


def polish(score_fn, code: str, base_score: Optional[float] = None, variants: int = 1024, rounds: int = 3,
           sigma: float = 0.35, seed: int = 0) -> PolishResult:
    """(1 + lambda) search over the literals of `code`.

    ``score_fn(list[CompiledPolicy]) -> np.ndarray`` scores a batch exactly
    (one device launch: `DeviceEvaluator.evaluate_native(...)[:, 0]`, or a CPU
    engine in tests).  Returns the best program text found and its score."""
    prog, err = try_compile(code)
    if prog is None:
        return PolishResult(code, base_score or 0.0, base_score or 0.0, 0, 0, False)
    tune = tunable_literals(prog)
    if not tune:
        return PolishResult(code, base_score or 0.0, base_score or 0.0, 0, 0, False)
    rng = random.Random(seed)
    best_vals = {prog.literals[j][0]: (prog.fconst[prog.literals[j][0]] if prog.ctag[prog.literals[j][0]] == TAG_FLOAT
                                       else prog.iconst[prog.literals[j][0]]) for j in range(len(prog.literals))}
    evaluated = 0
    if base_score is None:
        base_score = float(score_fn([prog])[0])
        evaluated += 1
    best = base_score
    for r in range(rounds):
        cands = [_perturb(prog, best_vals, tune, sigma * (0.6 ** r), rng) for _ in range(variants)]
        scores = np.asarray(score_fn([with_values(prog, v) for v in cands]), dtype=np.float64)
        evaluated += len(cands)
        j = int(np.argmax(scores))
        if scores[j] > best:
            best, best_vals = float(scores[j]), cands[j]
    improved = best > base_score
    text = rewrite_source(prog, best_vals) if improved else code
    return PolishResult(text, best, base_score, evaluated, rounds, improved)


__all__ = ["PolishResult", "polish", "rewrite_source", "tunable_literals", "with_values"]
