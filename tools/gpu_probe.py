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
t = time.time(); tab = dev.evaluate_builtin(["first_fit", "best_fit"]); dt = time.time() - t
print(json.dumps({"ff": tab[0, 0], "bf": tab[1, 0], "ff_counts": tab[0, 6:10].tolist(), "first_call_s": dt}), flush=True)
rng = np.random.default_rng(0)
for P in (256, 1024, 2048):
    wts = np.stack([rng.uniform(1000, 5000, P), rng.uniform(1e-4, 1e-2, P), rng.uniform(1e-5, 1e-3, P), rng.uniform(10, 1000, P)], 1)
    dev.evaluate_builtin("random_linear", wts)
    t = time.time(); tab = dev.evaluate_builtin("random_linear", wts); dt = time.time() - t
    print(json.dumps({"P": P, "random_linear_s": dt, "evals_per_s": P / dt, "mean_score": float(tab[:, 0].mean()), "exc": int((tab[:, 10] != 0).sum())}), flush=True)
cpu = ce.simulate_builtin_batch(w, "random_linear", wts[:64])
print(json.dumps({"cpu_gpu_equal_64": bool(np.array_equal(cpu, tab[:64]))}), flush=True)
names = list(reference_policies()); progs = [compile_policy(reference_policies()[n]) for n in names]
t = time.time(); tv = dev.evaluate_programs(progs); dt = time.time() - t
print(json.dumps({"vm": {n: [float(tv[i, 0]), bool(tv[i, 0] == reference_scores()[n]), int(tv[i, 10])] for i, n in enumerate(names)}, "vm_s": dt}), flush=True)
progs256 = [progs[i % 5] for i in range(1024)]
dev.evaluate_programs(progs256[:8])
t = time.time(); tv = dev.evaluate_programs(progs256); dt = time.time() - t
print(json.dumps({"vm_1024_s": dt, "vm_evals_per_s": 1024 / dt, "ok": bool(all(tv[i, 0] == reference_scores()[names[i % 5]] for i in range(1024)))}), flush=True)
