"""Re-score a saved population on every device path and the CPU VM:
batch launches (row kernel / two-wave kernel), the resident program service,
and the CPU VM (the reference-exact oracle); prints per program which paths
disagree.  Used to pin down the round-6 steady-run mismatch (data/diag/).

    python tools/mismatch_probe.py data/diag/r6i_population.json [--max-events N]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("--max-events", type=int, default=2_000_000)
    a = ap.parse_args()
    from funsearch_kubernetes_simulator_amd.core.traces import load_default_workload
    from funsearch_kubernetes_simulator_amd.ops import cpu_engine as ce
    from funsearch_kubernetes_simulator_amd.ops import hip_engine as he
    from funsearch_kubernetes_simulator_amd.policy.compiler import try_compile
    d = json.load(open(a.path))
    codes = [p["code"] for p in d["programs"]]
    rec = [p.get("device_score") for p in d["programs"]]
    progs = [try_compile(c)[0] for c in codes]
    keep = [i for i, p in enumerate(progs) if p is not None]
    progs = [progs[i] for i in keep]
    w = load_default_workload()
    t0 = time.time()
    vm = np.asarray(ce.simulate_program_batch(w, progs, threads=8))
    print(json.dumps({"cpu_vm_s": round(time.time() - t0, 2), "programs": len(progs)}), flush=True)
    dev = he.DeviceEvaluator(w)
    dev.set_options(max_events=a.max_events)
    out = {}
    # one program per launch: the two-wave kernel (which honours max_events; a
    # larger batch would take the row kernel, which has no event budget)
    sel = list(range(0, len(progs), max(1, len(progs) // 12)))[:12]
    t0 = time.time()
    out["batch_single"] = (sel, np.concatenate([dev.evaluate_native([progs[i]]) for i in sel]))
    print(json.dumps({"batch_single_s": round(time.time() - t0, 2)}), flush=True)
    # the two-wave batch kernel with the service's heap layout: a small LDS heap
    # top (most of each heap in HBM), forced through the in-flight size it is sized for
    dev.set_options(native_inflight=1 << 16)
    t0 = time.time()
    out["batch_small_top"] = (sel, np.concatenate([dev.evaluate_native([progs[i]]) for i in sel]))
    print(json.dumps({"batch_small_top_s": round(time.time() - t0, 2),
                      "duo_top": dev.info().get("native_duo_top_last")}), flush=True)
    dev.set_options(native_inflight=0)
    dev.start_service(slots=1024, share=0.875)
    try:
        t0 = time.time()
        out["service"] = (list(range(len(progs))), dev.evaluate_native(progs))
        print(json.dumps({"service_s": round(time.time() - t0, 2), "service": dev.info().get("service")}), flush=True)
    finally:
        dev.stop_service()
    for k, (ids, tab) in out.items():
        bad = [(r, i) for r, i in enumerate(ids) if not (int(tab[r, 10]) in (100, 101, 103) or
                                                        (tab[r, 0] == vm[i, 0] and tab[r, 8] == vm[i, 8]))]
        print(json.dumps({"path": k, "compared": len(ids), "mismatch": len(bad),
                          "examples": [{"i": keep[i], "recorded": rec[keep[i]], "vm": [float(vm[i, 0]), int(vm[i, 8])],
                                        "dev": [float(tab[r, 0]), int(tab[r, 8]), int(tab[r, 10])]} for r, i in bad[:8]]}),
              flush=True)


if __name__ == "__main__":
    main()
