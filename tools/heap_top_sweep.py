"""Time one P-policy launch for several LDS heap-top sizes (HBM heap mode)."""
import json, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from funsearch_kubernetes_simulator_amd.core import load_default_workload
from funsearch_kubernetes_simulator_amd.models import families as fam
from funsearch_kubernetes_simulator_amd.ops.hip_engine import DeviceEvaluator

w = load_default_workload()
dev = DeviceEvaluator(w, options={"heap_mode": "hbm"})
rng = np.random.default_rng(0)
P = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
for family in ("random_linear", "composite_linear"):
    W = fam.SAMPLERS[family](P, rng)
    ref = None
    for top in (0, 255, 1023, 2047, -1):
        dev.set_options(heap_top=top)
        dev.evaluate_builtin(family, W)   # warm
        t = time.perf_counter()
        tab = dev.evaluate_builtin(family, W)
        dt = time.perf_counter() - t
        if ref is None:
            ref = tab
        assert np.array_equal(tab, ref), "heap_top changed results"
        print(json.dumps({"family": family, "P": P, "heap_top": top, "s": round(dt, 4),
                          "evals_per_s": round(P / dt, 1), "events_per_s": round(float(tab[:, 8].sum()) / dt, 1)}),
              flush=True)
print(json.dumps(dev.info()))
