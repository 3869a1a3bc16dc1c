"""One P-policy builtin launch (plus a small warm-up) for PMC counter collection.

    rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU ... -d gpurun_out/pmc -o run --output-format csv \
        -- python3 tools/pmc_driver.py random_linear 4096
"""
import json, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from funsearch_kubernetes_simulator_amd.core import load_default_workload
from funsearch_kubernetes_simulator_amd.models import families as fam
from funsearch_kubernetes_simulator_amd.ops.hip_engine import DeviceEvaluator

family = sys.argv[1] if len(sys.argv) > 1 else "random_linear"
P = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
w = load_default_workload()
dev = DeviceEvaluator(w)
W = fam.SAMPLERS[family](P, np.random.default_rng(0))
dev.evaluate_builtin(family, W[:64])
tab = dev.evaluate_builtin(family, W)
print(json.dumps({"family": family, "P": P, "events": float(tab[:, 8].sum()), "info": dev.info()}))
