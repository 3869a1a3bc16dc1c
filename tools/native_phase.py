"""s_memtime phase split of the native-program row kernel (latency regime:
a few dozen programs, one program per wave).  Prints wave cycles per event by
phase (the profiled build is a diagnostics kernel: s_memtime itself adds cost).

    python tools/native_phase.py --programs 48
"""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from funsearch_kubernetes_simulator_amd.bench.programs import mutation_children  # noqa: E402
from funsearch_kubernetes_simulator_amd.core import load_default_workload  # noqa: E402
from funsearch_kubernetes_simulator_amd.models.library import reference_policies  # noqa: E402
from funsearch_kubernetes_simulator_amd.policy.compiler import compile_policy  # noqa: E402

PH = ("pop", "delete", "score", "fail", "commit", "eval", "next_policy")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--programs", type=int, default=48)
    ap.add_argument("--rows", type=int, default=0, help="programs per wave (0: auto)")
    a = ap.parse_args()
    from funsearch_kubernetes_simulator_amd.ops import hip_engine as he
    dev = he.DeviceEvaluator(load_default_workload(), options={"native_rows": a.rows})
    sets = {"first_fit": [compile_policy(reference_policies()["first_fit"])],
            "funsearch_4901": [compile_policy(reference_policies()["funsearch_4901"])],
            "children": mutation_children(a.programs, 0)}
    for name, progs in sets.items():
        dev.profile_native(progs)   # compile + warm
        tab, prof = dev.profile_native(progs)
        ev = float(tab[:, 8].sum())
        tot = prof[:, :7].sum()
        print(json.dumps({"set": name, "P": len(progs), "events": int(ev),
                          "cycles_per_event": round(float(tot) / ev, 1),
                          "phases_per_event": {PH[i]: round(float(prof[:, i].sum()) / ev, 1) for i in range(7)}}),
              flush=True)


if __name__ == "__main__":
    main()
