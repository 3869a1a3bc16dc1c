"""Cycles per wave-parallel heap push / pop (s_memtime inside k_test_heap)."""
import heapq, json, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from funsearch_kubernetes_simulator_amd.ops.hip_engine import native
m = native()
rng = np.random.default_rng(0)
for n0 in (100, 1000, 2000):
    keys = sorted(int(x) << 7 for x in rng.integers(0, 2**40, n0))
    ops = []
    for i in range(2000):
        ops.append(-1 if i % 2 else (int(rng.integers(0, 2**40)) << 7))
    out, pops = m.test_heap(np.array(keys, np.uint64), np.array(ops, np.int64), 7)
    print(json.dumps({"n0": n0, "cycles_push": int(pops[-2]), "cycles_pop": int(pops[-1])}), flush=True)
