"""s_memtime phase split of the 256-node wave kernel (BASELINE config-5 shape).

One launch of P composite policies on the 65,536-pod / 256-node synthetic
workload through the profiled twin of the production instance
(k_replay_c5_prof: NPASS 4, HBM heap, same launch bounds); prints cycles per
policy-event by phase (replay.hip.h Phase) as one JSON line.

    python tools/wave_phase_c5.py 2048
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from funsearch_kubernetes_simulator_amd.core import synthetic_workload  # noqa: E402
from funsearch_kubernetes_simulator_amd.models import families as fam  # noqa: E402
from funsearch_kubernetes_simulator_amd.ops.hip_engine import DeviceEvaluator  # noqa: E402

P = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
w = synthetic_workload(n_nodes=256, n_pods=65536, seed=0)
dev = DeviceEvaluator(w)
W = fam.sample_composite_linear(P, np.random.default_rng(0))
ref = dev.evaluate_builtin("composite_linear", W)
tab, prof = dev.profile_builtin("composite_linear", W)
assert np.array_equal(np.asarray(tab), np.asarray(ref)), "profiled kernel differs from the production kernel"
ev = float(np.asarray(tab)[:, 8].sum())
cyc = np.asarray(prof, dtype=np.float64).sum(0)
out = {"P": P, "events": ev, "cycles_per_event": {k: round(cyc[i] / ev, 1) for i, k in enumerate(DeviceEvaluator.PHASES)},
       "total_per_event": round(cyc[:6].sum() / ev, 1),
       "creations": float(cyc[7]), "feasible_node_slots_per_creation": round(cyc[6] / max(cyc[7], 1.0), 2)}
print(json.dumps(out))
