"""Staged MI355X check of the baseline program JIT (ops/gcnjit.py).

    python tools/gcn_probe.py simple     # one arithmetic program, no runtime calls
    python tools/gcn_probe.py reference  # the reference / seed policies
    python tools/gcn_probe.py children N # N offline-mutation children (runtime calls, loops, lists)
    python tools/gcn_probe.py bench N    # novel-program throughput: baseline vs LLVM tier vs CPU VM

Every stage compares device rows with the CPU VM bit for bit and prints one
JSON line per step (flushed), so a hang or a fault names its stage.
"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from funsearch_kubernetes_simulator_amd.core import load_default_workload  # noqa: E402
from funsearch_kubernetes_simulator_amd.ops import cpu_engine as ce  # noqa: E402
from funsearch_kubernetes_simulator_amd.policy.compiler import compile_policy  # noqa: E402

SKIP = (100, 101)


def say(**kw):
    print(json.dumps(kw), flush=True)


def compare(tab, vm):
    bad = []
    for i in range(len(tab)):
        if int(tab[i, 10]) in SKIP or int(vm[i, 10]) in SKIP:
            continue
        if not np.array_equal(tab[i], vm[i]):
            bad.append(i)
    return bad


def evaluator(tier):
    from funsearch_kubernetes_simulator_amd.ops import hip_engine as he
    w = load_default_workload()
    dev = he.DeviceEvaluator(w)
    from funsearch_kubernetes_simulator_amd.ops.jit import NativeCompiler
    dev._jit = NativeCompiler(dev._eng, dev.device, budget=int(dev.options["budget"]), tier=tier)
    return w, dev


def run(dev, w, progs, label):
    t0 = time.perf_counter()
    nb = dev.submit_native(0, progs)
    t1 = time.perf_counter()
    tab = dev.wait(0)
    t2 = time.perf_counter()
    vm = ce.simulate_program_batch(w, progs, threads=16)
    bad = compare(tab, vm)
    say(stage=label, P=len(progs), native=int(nb.ok.sum()), new_shapes=nb.compiled, compile_s=round(t1 - t0, 4),
        device_s=round(t2 - t1, 4), bad=bad[:10], n_bad=len(bad), reasons=list(nb.reasons.values())[:3],
        exc=sorted(set(int(x) for x in tab[:, 10])))
    return tab, vm, bad


def main():
    stage = sys.argv[1]
    tier = os.environ.get("FKS_JIT_TIER", "baseline")
    if stage == "simple":
        w, dev = evaluator(tier)
        progs = [compile_policy("def priority_function(pod, node):\n    return 5000 - node.cpu_milli_left * 0.25\n"),
                 compile_policy("def priority_function(pod, node):\n    if pod.cpu_milli > node.cpu_milli_left:\n"
                                "        return 0\n    return node.cpu_milli_left - pod.cpu_milli + 1\n")]
        for i, p in enumerate(progs):
            _, _, bad = run(dev, w, [p], f"simple{i}")
            if bad:
                sys.exit(1)
    elif stage == "reference":
        from funsearch_kubernetes_simulator_amd.models.library import reference_policies, seed_policies
        w, dev = evaluator(tier)
        progs = [compile_policy(s) for s in list(reference_policies().values()) + list(seed_policies().values())]
        _, _, bad = run(dev, w, progs, "reference")
        if bad:
            sys.exit(1)
    elif stage == "children":
        from funsearch_kubernetes_simulator_amd.bench.programs import mutation_children
        n = int(sys.argv[2]) if len(sys.argv) > 2 else 64
        w, dev = evaluator(tier)
        progs = mutation_children(n, 11)
        _, _, bad = run(dev, w, progs, f"children{n}")
        if bad:
            sys.exit(1)
    elif stage == "bench":
        from funsearch_kubernetes_simulator_amd.bench.programs import mutation_children
        n = int(sys.argv[2]) if len(sys.argv) > 2 else 64
        seed = int(sys.argv[3]) if len(sys.argv) > 3 else 21
        progs = mutation_children(n, seed)
        tabs = {}
        for t in ("baseline", "llvm"):
            w, dev = evaluator(t)
            dev.submit_native(0, progs[:1])
            dev.wait(0)   # warm: module loader, first launch
            t0 = time.perf_counter()
            nb = dev.submit_native(0, progs)
            t1 = time.perf_counter()
            tab = dev.wait(0)
            t2 = time.perf_counter()
            dev.submit_native(0, progs)
            dev.wait(0)
            t3 = time.perf_counter()
            tabs[t] = tab
            say(stage="bench", tier=t, P=n, native=int(nb.ok.sum()), compile_s=round(t1 - t0, 4),
                device_s=round(t2 - t1, 4), evals_per_s_incl_jit=round(n / (t2 - t0), 1),
                evals_per_s_cached=round(n / (t3 - t2), 1), stats=dev.native_compiler.stats)
            # one program per launch: replay latency (the latency-bound regime)
            lat = []
            for p in progs[:6]:
                dev.evaluate_native([p])
                s0 = time.perf_counter()
                r = dev.evaluate_native([p])
                lat.append((round((time.perf_counter() - s0) * 1e3, 2), int(r[0, 8])))
            say(stage="latency", tier=t, ms_events=lat)
        t0 = time.perf_counter()
        vm = ce.simulate_program_batch(w, progs, threads=16)
        t1 = time.perf_counter()
        say(stage="bench", tier="cpu_vm", P=n, evals_per_s=round(n / (t1 - t0), 1),
            bad_baseline=compare(tabs["baseline"], vm)[:10], bad_llvm=compare(tabs["llvm"], vm)[:10])
    elif stage == "overlap":
        # a JIT compile + module load must not wait for batches replaying on other slots
        from funsearch_kubernetes_simulator_amd.bench.programs import novel_children
        w, dev = evaluator(os.environ.get("FKS_JIT_TIER", "auto"))
        progs = novel_children(256 + 3 * 64, 41)
        dev.submit_native(0, progs[:1])
        dev.wait(0)
        t0 = time.perf_counter()
        dev.submit_native(0, progs[:256])
        t1 = time.perf_counter()
        loads = []
        for i in range(3):
            s0 = time.perf_counter()
            nb = dev.native_compiler.prepare(progs[256 + 64 * i:256 + 64 * (i + 1)])
            loads.append((round(time.perf_counter() - s0, 4), int(nb.compiled), bool(dev.ready(0))))
        dev.submit_native(1, progs[256:320])
        t2 = time.perf_counter()
        busy = not dev.ready(0)
        dev.wait(0)
        t3 = time.perf_counter()
        dev.wait(1)
        say(stage="overlap", submit0_s=round(t1 - t0, 4), loads_s_shapes_ready0=loads, submit1_s=round(t2 - t1, 4),
            slot0_still_busy_after=busy, slot0_total_s=round(t3 - t0, 4))
    else:
        raise SystemExit(f"unknown stage {stage}")


if __name__ == "__main__":
    main()
