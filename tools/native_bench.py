"""Program-evaluation throughput at LLM-sized batches: native JIT on the
MI355X vs the native CPU VM (the path round 1 used for config 3).

Programs are offline-mutation children (funsearch/llm.py MutationClient) of
the reference / seed programs, i.e. what the evolution loop evaluates.  For
each batch size: JIT compile wall time (fresh shapes and shape-cache hits
counted separately), device replay time, end-to-end evals/s, the CPU VM's
evals/s on the same programs, and a bit-exactness check of every row.

    python tools/native_bench.py --batch 60 --batches 4 --threads 16
"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from funsearch_kubernetes_simulator_amd.bench.programs import mutation_children  # noqa: E402
from funsearch_kubernetes_simulator_amd.core import load_default_workload  # noqa: E402
from funsearch_kubernetes_simulator_amd.ops import cpu_engine as ce  # noqa: E402


def children(n, seed):
    return mutation_children(n, seed)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=60)
    ap.add_argument("--batches", type=int, default=4)
    ap.add_argument("--threads", type=int, default=0)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--cpu", action="store_true", help="also time the CPU VM on the same programs")
    ap.add_argument("--single", type=int, default=0, help="also time K programs one per launch (replay latency)")
    ap.add_argument("--options", default="{}", help="DeviceEvaluator options (JSON), e.g. '{\"row_kernel\": \"off\"}'")
    a = ap.parse_args()
    from funsearch_kubernetes_simulator_amd.ops import hip_engine as he
    w = load_default_workload()
    dev = he.DeviceEvaluator(w, options=json.loads(a.options))
    threads = a.threads or ce.default_threads()
    progs = children(a.batch * a.batches, a.seed)
    # warm the compiler / module loader (first hipModuleLoadData, clang page-in)
    dev.evaluate_native(progs[:1])
    for b in range(a.batches):
        batch = progs[b * a.batch:(b + 1) * a.batch]
        t0 = time.perf_counter()
        nb = dev.submit_native(0, batch)
        t1 = time.perf_counter()
        tab = dev.wait(0)
        t2 = time.perf_counter()
        rec = {"batch": b, "P": len(batch), "new_shapes": nb.compiled, "compile_s": round(t1 - t0, 3),
               "device_s": round(t2 - t1, 3), "evals_per_s": round(len(batch) / (t2 - t0), 1),
               "native": int(nb.ok.sum()), "events": int(tab[:, 8].sum())}
        if a.cpu:
            t3 = time.perf_counter()
            cpu = ce.simulate_program_batch(w, batch, threads=threads)
            t4 = time.perf_counter()
            rec["cpu_vm_s"] = round(t4 - t3, 3)
            rec["cpu_vm_evals_per_s"] = round(len(batch) / (t4 - t3), 1)
            ok = nb.ok
            rec["exact"] = bool(np.array_equal(tab[ok], cpu[ok]))
        # the same batch again: every shape cached -> pure device time
        t5 = time.perf_counter()
        dev.submit_native(0, batch)
        tab2 = dev.wait(0)
        t6 = time.perf_counter()
        rec["cached_evals_per_s"] = round(len(batch) / (t6 - t5), 1)
        rec["repeat_identical"] = bool(np.array_equal(tab, tab2))
        print(json.dumps(rec), flush=True)
    for i, p in enumerate(progs[:a.single]):
        dev.evaluate_native([p])   # compiled already; warm
        t0 = time.perf_counter()
        tab = dev.evaluate_native([p])
        dt = time.perf_counter() - t0
        ev = int(tab[0, 8])
        print(json.dumps({"single": i, "n_insns": p.n_insns, "events": ev, "replay_ms": round(dt * 1e3, 2),
                          "us_per_event": round(dt * 1e6 / max(1, ev), 3), "exc": int(tab[0, 10])}), flush=True)
    print(json.dumps({"jit_stats": dev.native_compiler.stats}), flush=True)


if __name__ == "__main__":
    main()
