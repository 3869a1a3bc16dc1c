"""Parametric policy families: weights <-> program text.

Each family has (a) a native twin in both engines (`csrc/cpu/builtin_scorers.hpp`,
`csrc/hip/scorers.hip.h`) that evaluates a weight vector with exactly the same
IEEE operations, and (b) a `to_program` that renders the weight vector as an
ordinary policy program (``repr`` floats round-trip exactly), so a member
found by fast batched search can be exported, re-evaluated by the object
engine or handed to the LLM loop with a bit-identical score.

* ``random_linear`` -- the reference's `_create_random_policy`
  (`funsearch/funsearch_integration.py:403-431`): base + cpu_left*cf +
  mem_left*mf (+ gpu_left*gf for GPU pods on nodes with free GPUs), with the
  reference's sampling ranges.  These are the "random-weight candidate
  policies" of the headline benchmark.
* ``feature_linear`` -- a 12-feature linear score (remaining-capacity
  fractions, balance, GPU fragmentation / slack / idle-GPU terms, node size)
  used by the evolutionary search.
"""

from __future__ import annotations

from typing import List, Sequence

import numpy as np

from ..policy.template import FEASIBILITY_PROLOGUE

WEIGHTS = 16

_HEAD = "\ndef priority_function(pod, node):\n" + FEASIBILITY_PROLOGUE + "\n    \n"

# ---------------------------------------------------------------- random_linear
RANDOM_LINEAR_RANGES = ((1000.0, 5000.0), (0.0001, 0.01), (0.00001, 0.001), (10.0, 1000.0))


def sample_random_linear(n: int, rng: np.random.Generator) -> np.ndarray:
    """[n, 4] weights drawn like `_create_random_policy` (base, cpu, mem, gpu)."""
    cols = [rng.uniform(lo, hi, n) for lo, hi in
            (RANDOM_LINEAR_RANGES[1], RANDOM_LINEAR_RANGES[2], RANDOM_LINEAR_RANGES[3], RANDOM_LINEAR_RANGES[0])]
    cpu, mem, gpu, base = cols
    return np.stack([base, cpu, mem, gpu], axis=1)


def random_linear_program(w: Sequence[float]) -> str:
    base, cf, mf, gf = (float(x) for x in w[:4])
    return (_HEAD +
            f"    score = {base!r} + node.cpu_milli_left * {cf!r} + node.memory_mib_left * {mf!r}\n"
            "    \n"
            "    if pod.num_gpu > 0 and node.gpu_left > 0:\n"
            f"        score += node.gpu_left * {gf!r}\n"
            "    \n"
            "    return max(1, int(score))\n")


# ---------------------------------------------------------------- feature_linear
#: (name, python expression) in evaluation order; must match the native twins.
FEATURES: List[tuple] = [
    ("bias", "1.0"),
    ("cpu_remaining", "(node.cpu_milli_left - pod.cpu_milli) / max(1, node.cpu_milli_total)"),
    ("mem_remaining", "(node.memory_mib_left - pod.memory_mib) / max(1, node.memory_mib_total)"),
    ("gpu_remaining", "(node.gpu_left - pod.num_gpu) / max(1, len(node.gpus))"),
    ("cpu_mem_imbalance",
     "abs((node.cpu_milli_left - pod.cpu_milli) / max(1, node.cpu_milli_total)"
     " - (node.memory_mib_left - pod.memory_mib) / max(1, node.memory_mib_total))"),
    ("free_gpu_milli", "sum(g.gpu_milli_left for g in node.gpus) / 1000"),
    ("gpu_milli_fragment", "sum(g.gpu_milli_left for g in node.gpus) % max(1, pod.gpu_milli) / 1000"),
    ("idle_gpu_fraction",
     "sum(1 for g in node.gpus if g.gpu_milli_left == g.gpu_milli_total) / max(1, len(node.gpus))"),
    ("partial_gpu_fraction",
     "sum(1 for g in node.gpus if 0 < g.gpu_milli_left < g.gpu_milli_total) / max(1, len(node.gpus))"),
    ("cpu_pod_on_gpu_node", "(1.0 if pod.num_gpu == 0 and len(node.gpus) > 0 else 0.0)"),
    ("best_fit_gpu_slack",
     "(min(g.gpu_milli_left - pod.gpu_milli for g in node.gpus if g.gpu_milli_left >= pod.gpu_milli) / 1000"
     " if pod.num_gpu > 0 else 0.0)"),
    ("node_cpu_size", "node.cpu_milli_total / 100000"),
]
N_FEATURES = len(FEATURES)


def feature_linear_program(w: Sequence[float]) -> str:
    lines = ["    score = 0.0"]
    for (name, expr), wk in zip(FEATURES, w):
        wk = float(wk)
        if wk != 0.0:
            lines.append(f"    score += {wk!r} * ({expr})  # {name}")
    return _HEAD + "\n".join(lines) + "\n    \n    return max(1, int(score))\n"


def sample_feature_linear(n: int, rng: np.random.Generator, scale: float = 1000.0) -> np.ndarray:
    w = rng.normal(0.0, scale, size=(n, N_FEATURES))
    w[:, 0] = np.abs(w[:, 0]) + 5 * scale   # keep most scores >= 1 (feasible nodes score)
    return w


def to_program(family: str, w: Sequence[float]) -> str:
    if family == "random_linear":
        return random_linear_program(w)
    if family == "feature_linear":
        return feature_linear_program(w)
    raise KeyError(family)


def pad_weights(w: np.ndarray) -> np.ndarray:
    w = np.atleast_2d(np.asarray(w, dtype=np.float64))
    out = np.zeros((w.shape[0], WEIGHTS))
    out[:, :w.shape[1]] = w
    return out
