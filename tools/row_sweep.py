"""Wave kernel (1 policy / wave) vs row kernel (4 policies / wave) at several
LDS heap-top sizes: one P-policy launch each, results must agree bit-exactly.

    python tools/row_sweep.py [P] [families...]
"""
import json, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from funsearch_kubernetes_simulator_amd.core import load_default_workload
from funsearch_kubernetes_simulator_amd.models import families as fam
from funsearch_kubernetes_simulator_amd.ops.hip_engine import DeviceEvaluator

Ps = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "6144").split(",")]
families = sys.argv[2:] or ["random_linear", "composite_linear"]
tops = [int(x) for x in os.environ.get("ROW_TOPS", "127,255,511,1023").split(",")]
w = load_default_workload()
dev = DeviceEvaluator(w)
rng = np.random.default_rng(0)
wave = os.environ.get("ROW_WAVE", "1") == "1"
for family, P in [(f, p) for f in families for p in Ps]:
    W = fam.SAMPLERS[family](P, rng)
    ref = None
    for cfg in [{"row_kernel": "off"}] * wave + [{"row_kernel": "on", "row_heap_top": t} for t in tops]:
        dev.set_options(**cfg)
        dev.evaluate_builtin(family, W[:256])   # warm
        t0 = time.perf_counter()
        tab = dev.evaluate_builtin(family, W)
        dt = time.perf_counter() - t0
        if ref is None:
            ref = tab
        same = bool(np.array_equal(tab, ref))
        print(json.dumps({"family": family, "P": P, **cfg, "s": round(dt, 4), "evals_per_s": round(P / dt, 1),
                          "events_per_s": round(float(tab[:, 8].sum()) / dt, 1), "same": same}), flush=True)
        assert same, "row kernel differs from the wave kernel"
print(json.dumps(dev.info()))
