"""Native CPU oracle: golden scores, families <-> program text, exact means, options."""
import copy
import statistics

import numpy as np
import pytest

from funsearch_kubernetes_simulator_amd.core import load_default_workload
from funsearch_kubernetes_simulator_amd.core.arrays import Workload
from funsearch_kubernetes_simulator_amd.engine import Evaluator, object_engine_eval
from funsearch_kubernetes_simulator_amd.models import families as fam
from funsearch_kubernetes_simulator_amd.models.library import reference_policies, reference_scores
from funsearch_kubernetes_simulator_amd.ops import cpu_engine as ce
from funsearch_kubernetes_simulator_amd.ops.hip_engine import snapshot_schedule
from funsearch_kubernetes_simulator_amd.policy.compiler import compile_policy

GOLD = {"first_fit": (47, 3152, 19456), "best_fit": (40, 79, 16383), "funsearch_4901": (67, 11259, 27563),
        "funsearch_4816": (45, 2353, 18657), "funsearch_4800": (45, 2299, 18603)}


@pytest.mark.parametrize("family", ["first_fit", "best_fit"])
def test_builtin_golden(default_workload, family):
    r = ce.simulate_builtin(default_workload, family)
    assert r["score"] == reference_scores()[family]
    assert (r["n_snapshots"], r["n_frag_events"], r["n_events"]) == GOLD[family]


@pytest.mark.parametrize("name", list(GOLD))
def test_vm_golden(default_workload, name):
    r = ce.simulate_program(default_workload, compile_policy(reference_policies()[name]))
    assert r["score"] == reference_scores()[name]
    assert (r["n_snapshots"], r["n_frag_events"], r["n_events"]) == GOLD[name]
    assert r["exc"] == 0 and not r["inexact"]


def test_builtin_equals_vm_trace(default_workload):
    b = ce.simulate_builtin(default_workload, "best_fit")
    v = ce.simulate_program(default_workload, compile_policy(reference_policies()["best_fit"]))
    assert b["trace_hash"] == v["trace_hash"]


@pytest.mark.parametrize("family", ["random_linear", "feature_linear", "composite_linear"])
def test_family_text_matches_builtin(default_workload, family):
    rng = np.random.default_rng(42)
    W = fam.SAMPLERS[family](6, rng)
    tab = ce.simulate_builtin_batch(default_workload, family, W, threads=4)
    progs = [compile_policy(fam.to_program(family, w)) for w in W]
    tab2 = ce.simulate_program_batch(default_workload, progs, threads=4)
    assert np.array_equal(tab, tab2)
    # and the object engine (CPython exec) agrees on one member
    assert object_engine_eval(fam.to_program(family, W[0]), default_workload).score == tab[0, 0]


def test_composite_basis_contains_champion(default_workload):
    """The champion (reference tests/test_scheduler.py:21) is a member of the composite basis."""
    r = ce.simulate_builtin(default_workload, "composite_linear", list(fam.CHAMPION_COMPOSITE))
    assert r["score"] == reference_scores()["funsearch_4901"]


def test_exact_mean_matches_statistics():
    rng = np.random.default_rng(0)
    for _ in range(300):
        T = int(rng.integers(1, 10 ** 9))
        vals = [int(x) / T for x in rng.integers(-T // 10, T + 1, int(rng.integers(1, 400)))]
        got, inexact = ce.native().exact_mean(vals)
        assert not inexact
        assert got == statistics.mean(vals)


def test_exact_mean_flags_unrepresentable():
    got, inexact = ce.native().exact_mean([1e-30, 0.5])
    assert inexact


def test_record_values_reproduce_means(default_workload):
    r = ce.simulate_builtin(default_workload, "first_fit", options=ce.SimOptions(record_values=True))
    snaps = np.array(r["snap_values"]).reshape(-1, 4)
    assert statistics.mean(snaps[:, 0].tolist()) == r["avg_cpu"]
    assert statistics.mean(r["frag_values"]) == r["frag"]


def test_snapshot_schedule_brute_force():
    for N in (1, 7, 19, 20, 21, 8152):
        fire, _ = snapshot_schedule(N, 0.05, 60)
        got, processed, thr = [], 0, 0.05
        while len(got) < 60:
            processed += 1
            if processed / N >= thr:
                got.append(processed)
                thr += 0.05
        assert list(fire) == got


def test_repush_earliest_and_first_fit_alloc_options(default_workload):
    base = ce.simulate_builtin(default_workload, "first_fit")
    e = ce.simulate_builtin(default_workload, "first_fit", options=ce.SimOptions(repush="earliest"))
    assert e["score"] != base["score"]    # SURVEY: FF 0.4311 under the earliest-deletion rule
    assert abs(e["score"] - 0.4311) < 5e-4
    f = ce.simulate_builtin(default_workload, "best_fit", options=ce.SimOptions(gpu_alloc="first_fit"))
    assert f["exc"] == 0


def test_unknown_model_nodes_and_overcommit(default_workload):
    """Q12 (gpus == [] but gpu_left > 0) and a policy that over-commits CPU."""
    from funsearch_kubernetes_simulator_amd.core.arrays import Workload
    cluster, pods = default_workload.to_objects()
    first = next(iter(cluster.nodes_dict.values()))
    first.gpus = []                       # model missing from the mapping
    pods = sorted(pods, key=lambda p: p.creation_time)[:600]
    w = Workload.from_objects(cluster, pods)
    code = "def priority_function(pod, node):\n    return 1 + node.cpu_milli_left // 1000\n"
    ev = Evaluator(w, device="cpu")
    assert ev.evaluate_programs([code])[0].score == object_engine_eval(code, w).score


def test_exception_semantics(default_workload):
    ev = Evaluator(default_workload, device="cpu")
    codes = ["def priority_function(pod, node):\n    return 1 / 0\n",
             "def priority_function(pod, node):\n    return int(float('inf'))\n",
             "def priority_function(pod, node):\n    return node.gpus[5].gpu_milli_left\n",
             "def priority_function(pod, node):\n    return 1000 if pod.num_gpu == 0 else 0\n",
             "def priority_function(pod, node):\n    return 1000\n"]
    res = ev.evaluate_programs(codes)
    assert [r.score for r in res[:3]] == [0.0, 0.0, 0.0]
    assert all(r.exc != 0 for r in res[:3])
    # GPU pods never placed -> dropped -> unassigned -> score 0, no exception
    assert res[3].score == 0 and res[3].exc == 0
    # no feasibility check: a GPU pod lands on a node without enough GPUs -> allocator raises
    assert res[4].score == 0 and res[4].exc == 6


def test_invariant_checker_passes_and_is_transparent(default_workload):
    """`check_invariants` (reference _validate_cluster_invariants) holds at every event of real replays."""
    sub = Workload(default_workload.cluster, default_workload.pods.subset(np.arange(0, 1500)))
    opts = ce.SimOptions(check_invariants=1)
    for name in ("first_fit", "best_fit"):
        a = ce.simulate_builtin(sub, name, options=opts)
        b = ce.simulate_builtin(sub, name)
        assert a["exc"] == 0 and a["score"] == b["score"] and a["trace_hash"] == b["trace_hash"]
    prog = compile_policy(reference_policies()["funsearch_4901"])
    a = ce.simulate_program(sub, prog, options=opts)
    assert a["exc"] == 0 and a["score"] == ce.simulate_program(sub, prog)["score"]


def test_native_sequence_matcher_equals_difflib():
    """The evolution loop's similarity gate (reference `_is_too_similar`) uses the
    native SequenceMatcher: ratio and threshold decision must equal difflib's."""
    import difflib
    import random
    from funsearch_kubernetes_simulator_amd.ops import _fks_cpu
    rng = random.Random(3)
    texts = list(reference_policies().values())
    pairs = [("", ""), ("a", ""), ("", "b"), ("abc", "abc")]
    for _ in range(60):
        a = rng.choice(texts)
        b = list(a)
        for _ in range(rng.randint(0, 40)):
            i = rng.randrange(len(b))
            b[i:i + rng.randint(0, 3)] = rng.choice(["", "x", " ", "\n", "é", "score += 1"])
        pairs.append((a.strip(), "".join(b).strip()))
    for _ in range(400):   # short strings over small alphabets: many ties and popular elements
        alpha = rng.choice(["ab", "abcd", "ab \n", "xyzé"])
        pairs.append(("".join(rng.choice(alpha) for _ in range(rng.randint(0, 450))),
                      "".join(rng.choice(alpha) for _ in range(rng.randint(0, 450)))))
    for a, b in pairs:
        ref = difflib.SequenceMatcher(None, a, b).ratio()
        assert _fks_cpu.seq_ratio(a, b) == ref
        for t in (0.5, 0.85, ref):
            assert _fks_cpu.similar_at_least(a, b, t) == (ref >= t)
