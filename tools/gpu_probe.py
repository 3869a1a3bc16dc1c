"""Quick device probe: correctness + timing of the replay kernels (prints JSON lines)."""
import json, sys, time, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from funsearch_kubernetes_simulator_amd.core import load_default_workload
from funsearch_kubernetes_simulator_amd.ops import cpu_engine as ce
from funsearch_kubernetes_simulator_amd.ops.hip_engine import DeviceEvaluator
from funsearch_kubernetes_simulator_amd.models.library import reference_policies, reference_scores
from funsearch_kubernetes_simulator_amd.policy.compiler import compile_policy

w = load_default_workload()
dev = DeviceEvaluator(w)
print(json.dumps({"info": dev.info()}), flush=True)
rng = np.random.default_rng(0)
def rl(P):
    return np.stack([rng.uniform(1000, 5000, P), rng.uniform(1e-4, 1e-2, P), rng.uniform(1e-5, 1e-3, P), rng.uniform(10, 1000, P)], 1)
ref = None
for mode in ("lds", "hbm"):
    dev.set_options(heap_mode=mode)
    for P in ((512, 1024) if mode == "lds" else (1024, 2048, 4096, 8192)):
        wts = rl(P)
        dev.evaluate_builtin("random_linear", wts[:8])
        t = time.time(); tab = dev.evaluate_builtin("random_linear", wts); dt = time.time() - t
        cpu = ce.simulate_builtin_batch(w, "random_linear", wts[:32])
        print(json.dumps({"mode": mode, "P": P, "s": round(dt, 4), "evals_per_s": round(P / dt, 1),
                          "exact_vs_cpu32": bool(np.array_equal(cpu, tab[:32]))}), flush=True)
dev.set_options(heap_mode="auto")
names = list(reference_policies()); progs = [compile_policy(reference_policies()[n]) for n in names]
for mode in ("lds", "hbm"):
    dev.set_options(heap_mode=mode)
    tv = dev.evaluate_programs(progs)
    progs1k = [progs[i % 5] for i in range(1024)]
    t = time.time(); tv = dev.evaluate_programs(progs1k); dt = time.time() - t
    print(json.dumps({"mode": mode, "vm_1024_s": round(dt, 3), "vm_evals_per_s": round(1024 / dt, 1),
                      "ok": bool(all(tv[i, 0] == reference_scores()[names[i % 5]] for i in range(1024)))}), flush=True)
