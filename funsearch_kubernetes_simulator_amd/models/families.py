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
* ``composite_linear`` -- a 16-term basis that contains the reference
  champion's scoring terms (piecewise utilisation, GPU-milli remainder,
  ratio balance, bonuses/penalties), so search starts next to 0.4901 and
  explores around it.
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


# ---------------------------------------------------------------- composite_linear
#: Shared sub-expressions of the composite family (evaluated once per call,
#: never raise: every divisor is clamped with max(1, .)).
COMPOSITE_PREAMBLE = (
    "    cpu_u = (node.cpu_milli_total - node.cpu_milli_left) / max(1, node.cpu_milli_total)\n"
    "    mem_u = (node.memory_mib_total - node.memory_mib_left) / max(1, node.memory_mib_total)\n"
    "    gpu_u = ((node.gpu_left * node.gpus[0].gpu_milli_total - sum(g.gpu_milli_left for g in node.gpus))"
    " / max(1, node.gpu_left * node.gpus[0].gpu_milli_total)) if pod.num_gpu > 0 else 0.0\n")

#: The champion's decomposition (reference `tests/test_scheduler.py:21-99`,
#: score 0.4901): piecewise utilisation scores, GPU-milli remainder, cpu/mem
#: ratio balance, "ample resources" / "big node" bonuses, GPU imbalance and
#: the nearly-full penalty -- plus three best-fit style GPU terms.
COMPOSITE_FEATURES: List[tuple] = [
    ("bias", "1.0"),
    ("cpu_free_lo", "(1.0 - cpu_u) if cpu_u < 0.7 else 0.0"),
    ("cpu_free_hi", "(1.0 - cpu_u) if cpu_u >= 0.7 else 0.0"),
    ("mem_free_lo", "(1.0 - mem_u) if mem_u < 0.7 else 0.0"),
    ("mem_free_hi", "(1.0 - mem_u) if mem_u >= 0.7 else 0.0"),
    ("gpu_free_lo", "((1.0 - gpu_u) if gpu_u < 0.7 else 0.0) if pod.num_gpu > 0 else 0.0"),
    ("gpu_free_hi", "((1.0 - gpu_u) if gpu_u >= 0.7 else 0.0) if pod.num_gpu > 0 else 0.0"),
    ("gpu_milli_remainder",
     "(sum(g.gpu_milli_left for g in node.gpus) % max(1, pod.gpu_milli)) if pod.num_gpu > 0 else 0"),
    ("cpu_mem_ratio_gap",
     "abs(node.cpu_milli_left / max(1, node.memory_mib_left) - pod.cpu_milli / max(1, pod.memory_mib))"),
    ("ample_resources",
     "1.0 if (node.cpu_milli_left > pod.cpu_milli * 2 and node.memory_mib_left > pod.memory_mib * 2) else 0.0"),
    ("gpu_imbalance",
     "(max(g.gpu_milli_left for g in node.gpus) - min(g.gpu_milli_left for g in node.gpus))"
     " if pod.num_gpu > 0 else 0"),
    ("big_node", "1.0 if (node.cpu_milli_total > 10000 and node.memory_mib_total > 64) else 0.0"),
    ("nearly_full", "1.0 if (cpu_u > 0.9 or mem_u > 0.9) else 0.0"),
    ("best_fit_gpu_slack", FEATURES[10][1]),
    ("idle_gpu_fraction", FEATURES[7][1]),
    ("cpu_pod_on_gpu_node", FEATURES[9][1]),
]
N_COMPOSITE = len(COMPOSITE_FEATURES)

#: The champion's weights in this basis (its scores differ only by the float
#: summation order of the terms).
CHAMPION_COMPOSITE = np.array([0.0, 100.0, 50.0, 100.0, 50.0, 200.0, 100.0, -0.2, -0.5, 25.0, -0.05, 15.0, -20.0,
                               0.0, 0.0, 0.0])
_COMPOSITE_SCALE = np.array([20.0, 50.0, 25.0, 50.0, 25.0, 100.0, 50.0, 0.1, 0.25, 12.0, 0.025, 8.0, 10.0,
                             50.0, 50.0, 20.0])


def composite_linear_program(w: Sequence[float]) -> str:
    lines = [COMPOSITE_PREAMBLE + "    score = 0.0"]
    for (name, expr), wk in zip(COMPOSITE_FEATURES, w):
        wk = float(wk)
        if wk != 0.0:
            lines.append(f"    score += {wk!r} * ({expr})  # {name}")
    return _HEAD + "\n".join(lines) + "\n    \n    return max(1, int(score))\n"


def sample_composite_linear(n: int, rng: np.random.Generator) -> np.ndarray:
    """Prior around the champion: log-normal rescaling of its terms, Gaussian
    values for the terms it does not use, occasional sign flips."""
    w = CHAMPION_COMPOSITE * np.exp(rng.normal(0.0, 0.6, size=(n, N_COMPOSITE)))
    unused = CHAMPION_COMPOSITE == 0.0
    w[:, unused] = rng.normal(0.0, 1.0, size=(n, int(unused.sum()))) * _COMPOSITE_SCALE[unused]
    flip = rng.random(w.shape) < 0.05
    w[flip] = -w[flip]
    return w


SAMPLERS = {"random_linear": sample_random_linear, "feature_linear": sample_feature_linear,
            "composite_linear": sample_composite_linear}


def to_program(family: str, w: Sequence[float]) -> str:
    if family == "random_linear":
        return random_linear_program(w)
    if family == "feature_linear":
        return feature_linear_program(w)
    if family == "composite_linear":
        return composite_linear_program(w)
    raise KeyError(family)


def pad_weights(w: np.ndarray) -> np.ndarray:
    w = np.atleast_2d(np.asarray(w, dtype=np.float64))
    out = np.zeros((w.shape[0], WEIGHTS))
    out[:, :w.shape[1]] = w
    return out
