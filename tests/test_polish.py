"""Constant polish (funsearch/polish.py): literals are data, the best setting
is written back into the program text and re-scores identically."""
import numpy as np

from funsearch_kubernetes_simulator_amd.core.arrays import Workload
from funsearch_kubernetes_simulator_amd.funsearch.polish import polish, rewrite_source, tunable_literals, with_values
from funsearch_kubernetes_simulator_amd.models.library import reference_policies
from funsearch_kubernetes_simulator_amd.ops import cpu_engine as ce
from funsearch_kubernetes_simulator_amd.policy.compiler import compile_policy
from funsearch_kubernetes_simulator_amd.policy.native_codegen import shape_key


def test_literals_are_separate_pool_entries():
    p = compile_policy("def priority_function(pod, node):\n    s = 0.5 * node.cpu_milli_left + 0.5\n"
                       "    for g in node.gpus:\n        s += 1\n    return s\n")
    vals = [p.fconst[i] if p.ctag[i] else p.iconst[i] for i, *_ in p.literals]
    assert vals == [0.5, 0.5, 1]                      # two 0.5 literals: two entries
    assert len(tunable_literals(p)) == 2               # the int 1 (structure-like) stays fixed
    q = with_values(p, {p.literals[0][0]: 0.25})
    assert shape_key(q) == shape_key(p)
    text = rewrite_source(p, {p.literals[0][0]: 0.25, p.literals[1][0]: -2.0})
    assert "0.25 * node.cpu_milli_left + -2.0" in text
    r = compile_policy(text)
    # a negative value is written as unary minus + literal: same number, exact
    assert [r.fconst[i] for i, *_ in r.literals[:2]] == [0.25, 2.0]


def test_polish_improves_and_text_rescoring_is_exact(default_workload):
    w = default_workload
    sub = Workload(w.cluster, w.pods.subset(np.arange(2000, 2600)))
    score = lambda progs: ce.simulate_program_batch(sub, progs, threads=8)[:, 0]
    code = reference_policies()["funsearch_4816"]
    res = polish(score, code, variants=24, rounds=2, seed=1)
    assert res.evaluated == 1 + 48
    assert res.score >= res.base_score
    again = score([compile_policy(res.code)])[0]
    assert again == res.score                           # the rewritten program IS the polished setting
    if res.improved:
        assert res.code != code
