"""One P-policy composite launch at the BASELINE config-5 shape (65,536 pods /
256 nodes, wave kernel NPASS = 4, HBM heaps) for PMC counter collection.

    rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU ... --kernel-trace -d gpurun_out/pmc5 -o run --output-format csv \\
        -- python3 tools/pmc_c5_driver.py 2048
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
top = int(sys.argv[2]) if len(sys.argv) > 2 else -1
w = synthetic_workload(n_nodes=256, n_pods=65536, seed=0)
dev = DeviceEvaluator(w, options={} if top < 0 else {"heap_top": top})
W = fam.sample_composite_linear(P, np.random.default_rng(0))
tab = dev.evaluate_builtin("composite_linear", W)
print(json.dumps({"P": P, "events": float(tab[:, 8].sum()), "info": {k: v for k, v in dev.info().items()
                                                                     if k in ("npass", "heap_top_hbm")}}))
