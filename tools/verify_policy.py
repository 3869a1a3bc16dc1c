#!/usr/bin/env python3
"""Re-score saved policy programs on every engine and, when the reference
checkout is mounted, on the reference implementation itself.

    python tools/verify_policy.py data/policies/discovered/*.json [--no-reference] [--no-object]

For each results-JSON (reference `save_best_policy` schema) prints the
recorded score, the native CPU VM score, the object-engine score (CPython
exec over this framework's Python simulator) and the reference's own
`get_policy_score` (run from the read-only checkout in a subprocess, with a
3-line `enum.StrEnum` shim for Python 3.10) -- all must be identical.
"""
import argparse
import json
import os
import subprocess
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

REF = "/root/reference"
DRIVER = r'''
import enum, json, sys
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
codes = json.load(open(sys.argv[2]))
out = []
for code in codes:
    cluster, pods = TraceParser(sys.argv[1] + "/benchmarks/traces").parse_workload()
    env = {"__builtins__": __builtins__}
    exec(code, env)
    fn = env["priority_function"]
    ev = SchedulingEvaluator(cluster, enabled=True)
    sim = KubernetesSimulator(cluster, pods, DiscreteEventSimulator(pods), lambda p, n: int(max(0, fn(p, n))),
                              evaluator=ev)
    try:
        sim.run_schedule()
        r = ev.get_evaluation_results()
        out.append([ev.get_policy_score(pods), r.avg_cpu_utilization, r.avg_memory_utilization,
                    r.avg_gpu_count_utilization, r.gpu_fragmentation_score])
    except Exception as e:
        out.append([0, repr(e)])
print(json.dumps(out))
'''


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("files", nargs="+")
    ap.add_argument("--no-reference", action="store_true")
    ap.add_argument("--no-object", action="store_true")
    a = ap.parse_args()
    from funsearch_kubernetes_simulator_amd.core import load_default_workload
    from funsearch_kubernetes_simulator_amd.engine import Evaluator, object_engine_eval
    w = load_default_workload()
    recs = [json.load(open(f)) for f in a.files]
    codes = [r["code"] for r in recs]
    t = time.perf_counter()
    vm = Evaluator(w, device="cpu").evaluate_programs(codes)
    print(f"native CPU VM: {time.perf_counter() - t:.2f} s")
    obj = [None] * len(codes)
    if not a.no_object:
        t = time.perf_counter()
        obj = [object_engine_eval(c, w) for c in codes]
        print(f"object engine: {time.perf_counter() - t:.2f} s")
    ref = [None] * len(codes)
    if not a.no_reference and os.path.isdir(REF):
        with tempfile.TemporaryDirectory() as d:
            drv, job = os.path.join(d, "drv.py"), os.path.join(d, "codes.json")
            open(drv, "w").write(DRIVER)
            json.dump(codes, open(job, "w"))
            t = time.perf_counter()
            r = subprocess.run([sys.executable, drv, REF, job], capture_output=True, text=True, timeout=7200)
            print(f"reference implementation: {time.perf_counter() - t:.2f} s")
            if r.returncode != 0:
                print(r.stderr[-2000:])
            else:
                ref = json.loads(r.stdout.strip().splitlines()[-1])
    ok = True
    for f, rec, v, o, rf in zip(a.files, recs, vm, obj, ref):
        line = {"file": os.path.basename(f), "recorded": rec.get("score"), "cpu_vm": v.score,
                "object": None if o is None else o.score, "reference": None if rf is None else rf[0]}
        if rf is not None and len(rf) == 5:
            line["reference_util_frag"] = rf[1:]
        same = {x for x in (line["recorded"], line["cpu_vm"], line["object"], line["reference"]) if x is not None}
        line["identical"] = len(same) == 1
        ok &= line["identical"]
        print(json.dumps(line))
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
