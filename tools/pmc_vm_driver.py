"""One launch of P compiled reference programs on the device VM (for rocprofv3 --pmc).
Prints the number of VM instructions the CPU VM executes for the same batch."""
import json, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from funsearch_kubernetes_simulator_amd.core import load_default_workload
from funsearch_kubernetes_simulator_amd.models.library import reference_policies
from funsearch_kubernetes_simulator_amd.ops import cpu_engine as ce
from funsearch_kubernetes_simulator_amd.ops.hip_engine import DeviceEvaluator
from funsearch_kubernetes_simulator_amd.policy.compiler import compile_policy

P = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
mode = sys.argv[2] if len(sys.argv) > 2 else "hbm"
w = load_default_workload()
progs = [compile_policy(c) for c in reference_policies().values()]
insns = [ce.simulate_program(w, p)["vm_insns"] for p in progs]
dev = DeviceEvaluator(w, options={"heap_mode": mode})
batch = [progs[i % len(progs)] for i in range(P)]
tab = dev.evaluate_programs(batch)
print(json.dumps({"P": P, "mode": mode, "events": float(tab[:, 8].sum()),
                  "vm_insns": float(sum(insns[i % len(progs)] for i in range(P)))}))
