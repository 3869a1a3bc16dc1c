"""Device bytecode-VM throughput: P compiled programs per launch (reference + seed + family programs)."""
import json, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from funsearch_kubernetes_simulator_amd.core import load_default_workload
from funsearch_kubernetes_simulator_amd.models import families as fam
from funsearch_kubernetes_simulator_amd.models.library import reference_policies, seed_policies
from funsearch_kubernetes_simulator_amd.ops import cpu_engine as ce
from funsearch_kubernetes_simulator_amd.ops.hip_engine import DeviceEvaluator
from funsearch_kubernetes_simulator_amd.policy.compiler import compile_policy

w = load_default_workload()
rng = np.random.default_rng(1)
codes = list(reference_policies().values()) + list(seed_policies().values())
codes += [fam.to_program("composite_linear", x) for x in fam.sample_composite_linear(4, rng)]
progs = [compile_policy(c) for c in codes]
cpu = ce.simulate_program_batch(w, progs, threads=os.cpu_count() or 8)
for mode, P in [(m, p) for m in ("lds", "hbm") for p in (512, 2048)]:
    dev = DeviceEvaluator(w, options={"heap_mode": mode})
    batch = [progs[i % len(progs)] for i in range(P)]
    dev.evaluate_programs(batch[:64])   # warm
    t = time.perf_counter()
    tab = dev.evaluate_programs(batch)
    dt = time.perf_counter() - t
    ok = all(np.array_equal(tab[i], cpu[i % len(progs)]) for i in range(P))
    print(json.dumps({"mode": mode, "P": P, "s": round(dt, 3), "evals_per_s": round(P / dt, 1),
                      "events_per_s": round(float(tab[:, 8].sum()) / dt, 1), "exact": ok}), flush=True)
