"""MFMA surrogate screening throughput and surrogate quality on the default trace."""
import json, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from funsearch_kubernetes_simulator_amd.core import load_default_workload
from funsearch_kubernetes_simulator_amd.models import families as fam
from funsearch_kubernetes_simulator_amd.ops import screening as scr
from funsearch_kubernetes_simulator_amd.ops.hip_engine import native

w = load_default_workload()
sc = scr.Screener(w, device="auto")
rng = np.random.default_rng(0)
for P in (1024, 4096, 16384):
    W = fam.sample_composite_linear(P, rng)
    Wt = scr.weights_matrix(W)
    native().screen_linear(sc.X, Wt, sc.R, sc.Rfail, sc.Np, 0)    # warm
    t = time.perf_counter()
    for _ in range(5):
        native().screen_linear(sc.X, Wt, sc.R, sc.Rfail, sc.Np, 0)
    dt = (time.perf_counter() - t) / 5
    M = sc.X.shape[0]
    print(json.dumps({"candidates": P, "states": sc.states.n_states, "rows": M, "s_per_call_incl_copies": round(dt, 5),
                      "candidates_per_s": round(P / dt, 1), "gflops": round(2 * M * scr.KP * P / dt / 1e9, 1)}),
          flush=True)
