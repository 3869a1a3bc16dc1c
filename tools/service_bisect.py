"""Bisect a service-only mismatch: the same programs through the resident
program service under variants (default; JIT with node.gpus loops rolled; a
small grid; programs one per submission), each compared with the CPU VM.

    python tools/service_bisect.py data/diag/r6i_population.json
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np


def main() -> None:
    path = sys.argv[1]
    from funsearch_kubernetes_simulator_amd.core.traces import load_default_workload
    from funsearch_kubernetes_simulator_amd.ops import cpu_engine as ce
    from funsearch_kubernetes_simulator_amd.ops import hip_engine as he
    from funsearch_kubernetes_simulator_amd.policy.compiler import try_compile
    d = json.load(open(path))
    progs = [p for p in (try_compile(x["code"])[0] for x in d["programs"]) if p is not None]
    w = load_default_workload()
    vm = np.asarray(ce.simulate_program_batch(w, progs, threads=8))
    dev = he.DeviceEvaluator(w)
    dev.set_options(max_events=2_000_000)

    def report(name, tab, ids=None):
        ids = list(range(len(progs))) if ids is None else ids
        bad = [i for r, i in enumerate(ids) if int(tab[r, 10]) not in (100, 101, 103)
               and not (tab[r, 0] == vm[i, 0] and tab[r, 8] == vm[i, 8])]
        print(json.dumps({"variant": name, "compared": len(ids), "mismatch": len(bad), "bad": bad[:12],
                          "exc": sorted({int(tab[r, 10]) for r in range(len(ids))})}), flush=True)

    def service(share=0.875, one_by_one=False, ids=None):
        ids = list(range(len(progs))) if ids is None else ids
        dev.start_service(slots=1024, share=share)
        try:
            if one_by_one:
                return np.concatenate([dev.evaluate_native([progs[i]]) for i in ids])
            return dev.evaluate_native([progs[i] for i in ids])
        finally:
            dev.stop_service()

    report("service_default", service())
    report("service_small_grid", service(share=0.05))
    report("service_one_by_one", service(one_by_one=True, ids=list(range(0, len(progs), 4))),
           list(range(0, len(progs), 4)))
    # node.gpus loops rolled: a fresh compiler (empty shape cache) with unrolling off
    ce.native().gcn_set_unroll_cap(0)
    dev._jit = None
    report("service_rolled", service())
    report("batch_rolled_single", np.concatenate([dev.evaluate_native([progs[i]]) for i in range(0, len(progs), 4)]),
           list(range(0, len(progs), 4)))


if __name__ == "__main__":
    main()
