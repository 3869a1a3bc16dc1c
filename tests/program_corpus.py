"""Shared corpus of compiled policy programs for the engine differential tests:
the reference's 5 programs, the seed policies, feature/random-linear family
members lowered to program text, and every compiler snippet wrapped in the
template's feasibility prologue (tests/test_compiler.py SNIPPETS)."""
import numpy as np

from funsearch_kubernetes_simulator_amd.models import families as fam
from funsearch_kubernetes_simulator_amd.models.library import reference_policies, seed_policies
from funsearch_kubernetes_simulator_amd.policy.compiler import CompileError, compile_policy

from test_compiler import SNIPPETS

PROLOGUE = ("def priority_function(pod, node):\n    if (pod.cpu_milli > node.cpu_milli_left or "
            "pod.memory_mib > node.memory_mib_left or pod.num_gpu > node.gpu_left):\n        return 0\n"
            "    if pod.num_gpu > 0 and sum(1 for g in node.gpus if g.gpu_milli_left >= pod.gpu_milli) "
            "< pod.num_gpu:\n        return 0\n    ")


def program_codes():
    codes = list(reference_policies().values()) + list(seed_policies().values())
    rng = np.random.default_rng(9)
    codes += [fam.to_program("feature_linear", w) for w in fam.sample_feature_linear(6, rng)]
    codes += [fam.to_program("random_linear", w) for w in fam.sample_random_linear(4, rng)]
    for s in SNIPPETS:
        body = s if "return" in s else s + "\n    return 1"
        codes.append(PROLOGUE + body + "\n")
    return codes


def programs():
    progs = []
    for c in program_codes():
        try:
            progs.append(compile_policy(c))
        except CompileError:
            pass
    return progs
