"""Per-phase cycle breakdown of k_replay (s_memtime instrumented build)."""
import json, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from funsearch_kubernetes_simulator_amd.core import load_default_workload
from funsearch_kubernetes_simulator_amd.ops.hip_engine import DeviceEvaluator
from funsearch_kubernetes_simulator_amd.models.library import reference_policies
from funsearch_kubernetes_simulator_amd.policy.compiler import compile_policy

w = load_default_workload()
dev = DeviceEvaluator(w)
rng = np.random.default_rng(0)
def report(tag, tab, prof):
    ev = tab[:, 8]
    out = {"tag": tag, "cycles_per_event": round(float((prof.sum(1) / ev).mean()), 1),
           "phases": {ph: round(float((prof[:, i] / ev).mean()), 1) for i, ph in enumerate(DeviceEvaluator.PHASES)}}
    print(json.dumps(out), flush=True)
for mode, P in (("lds", 512), ("hbm", 512), ("hbm", 3072)):
    dev.set_options(heap_mode=mode)
    wts = np.stack([rng.uniform(1000, 5000, P), rng.uniform(1e-4, 1e-2, P), rng.uniform(1e-5, 1e-3, P), rng.uniform(10, 1000, P)], 1)
    tab, prof = dev.profile_builtin("random_linear", wts); report(f"random_linear/{mode}/P{P}", tab, prof)
dev.set_options(heap_mode="lds")
progs = [compile_policy(c) for c in reference_policies().values()]
tab, prof = dev.profile_programs(progs * 8); report("vm_reference/lds", tab, prof)
