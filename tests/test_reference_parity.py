"""Differential test against the reference implementation itself.

Runs the reference's own simulator (read-only checkout, imported with a
3-line ``enum.StrEnum`` shim for Python 3.10) on random sub-traces and random
policies in a subprocess, and compares its scores with the native engine.
Skipped when the reference checkout is not mounted (e.g. on the GPU box).
"""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

from funsearch_kubernetes_simulator_amd.core import load_default_workload
from funsearch_kubernetes_simulator_amd.engine import Evaluator
from funsearch_kubernetes_simulator_amd.models import families as fam

REF = "/root/reference"

DRIVER = r'''
import enum, json, sys, copy
if not hasattr(enum, "StrEnum"):
    class StrEnum(str, enum.Enum):
        @staticmethod
        def _generate_next_value_(name, start, count, last_values):
            return name.lower()
    enum.StrEnum = StrEnum
sys.path.insert(0, sys.argv[1])
from benchmarks.parser import TraceParser
from simulator.event_simulator import DiscreteEventSimulator
from simulator.main import KubernetesSimulator
from simulator.evaluator import SchedulingEvaluator
job = json.load(open(sys.argv[2]))
parser = TraceParser(sys.argv[1] + "/benchmarks/traces")
cluster0, pods0 = parser.parse_workload()
by_id = {p.pod_id: p for p in pods0}
out = []
for case in job:
    cluster = copy.deepcopy(cluster0)
    pods = [copy.deepcopy(by_id[i]) for i in case["pods"]]
    env = {"__builtins__": __builtins__}
    exec(case["code"], env)
    fn = env["priority_function"]
    sched = lambda pod, node: int(max(0, fn(pod, node)))
    ev = SchedulingEvaluator(cluster, enabled=True)
    sim = KubernetesSimulator(cluster, pods, DiscreteEventSimulator(pods), sched, evaluator=ev)
    try:
        sim.run_schedule()
        out.append(ev.get_policy_score(pods))
    except Exception:
        out.append(0)
print(json.dumps(out))
'''


@pytest.mark.skipif(not os.path.isdir(REF), reason="reference checkout not mounted")
@pytest.mark.slow
def test_random_subtraces_random_policies_match_reference(tmp_path):
    w = load_default_workload()
    rng = np.random.default_rng(2024)
    cases = []
    for k in range(8):
        n = int(rng.integers(200, 900))
        start = int(rng.integers(0, w.pods.n_pods - n))
        idx = np.arange(start, start + n)
        family = "random_linear" if k % 2 else "feature_linear"
        W = (fam.sample_random_linear if family == "random_linear" else fam.sample_feature_linear)(1, rng)[0]
        cases.append({"pods": [w.pods.pod_ids[i] for i in idx], "code": fam.to_program(family, W), "idx": idx})
    job = tmp_path / "job.json"
    job.write_text(json.dumps([{"pods": c["pods"], "code": c["code"]} for c in cases]))
    drv = tmp_path / "drv.py"
    drv.write_text(DRIVER)
    r = subprocess.run([sys.executable, str(drv), REF, str(job)], capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stderr[-2000:]
    ref_scores = json.loads(r.stdout.strip().splitlines()[-1])
    from funsearch_kubernetes_simulator_amd.core.arrays import Workload
    for c, ref in zip(cases, ref_scores):
        sub = Workload(w.cluster, w.pods.subset(c["idx"]))
        got = Evaluator(sub, device="cpu").scores([c["code"]])[0]
        assert got == ref, (got, ref)
