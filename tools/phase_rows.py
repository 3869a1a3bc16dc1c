"""Wave-level phase breakdown of the row kernel (s_memtime build): for each
region, the share of wave time spent in it, and cycles per wave step."""
import json, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from funsearch_kubernetes_simulator_amd.core import load_default_workload
from funsearch_kubernetes_simulator_amd.models import families as fam
from funsearch_kubernetes_simulator_amd.ops.hip_engine import DeviceEvaluator

P = int(sys.argv[1]) if len(sys.argv) > 1 else 12288
w = load_default_workload()
dev = DeviceEvaluator(w)
for family in sys.argv[2:] or ["random_linear", "composite_linear"]:
    W = fam.SAMPLERS[family](P, np.random.default_rng(0))
    plain = dev.evaluate_builtin(family, W)
    tab, prof = dev.profile_rows(family, W)
    assert np.array_equal(tab, plain), "profiled build changed results"
    tot = prof[:, :7].sum()
    events = float(tab[:, 8].sum())
    names = {m: "".join(c for b, c in ((1, "D"), (2, "P"), (4, "F")) if m & b) for m in range(1, 8)}
    steps = float(prof[:, 9:16].sum())
    mix = {names[m]: round(float(prof[:, 8 + m].sum()) / max(1.0, steps), 4) for m in range(1, 8)}
    print(json.dumps({"family": family, "P": P, "waves": int(prof.shape[0]),
                      "wave_cycles_per_policy_event": round(float(tot) / events, 1),
                      "share": {ph: round(float(prof[:, i].sum() / tot), 4)
                                for i, ph in enumerate(DeviceEvaluator.ROW_PHASES)},
                      # wave-steps by the set of event kinds its four rows ran (D deletion,
                      # P creation placed, F creation failed): the wave issues the union
                      "wave_steps": int(steps), "kind_mix": mix,
                      "mean_distinct_kinds": round(sum(bin(m).count("1") * float(prof[:, 8 + m].sum())
                                                       for m in range(1, 8)) / max(1.0, steps), 3)}), flush=True)
