"""How many events of each candidate's replay precede its first failed placement?

Until then every policy pops the same, policy-independent event sequence (the
"no-failure" stream: heap order depends only on (time, pod rank) keys), which
is what the shared-prefix kernel (csrc/hip/replay_prefix.hip.h) skips through
without a heap.  Prints per-policy prefix lengths and the mean share of replay
events they cover.

    python tools/prefix_stats.py composite_linear 16
"""
import heapq
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from funsearch_kubernetes_simulator_amd.core import load_default_workload  # noqa: E402
from funsearch_kubernetes_simulator_amd.models import families as fam  # noqa: E402
from funsearch_kubernetes_simulator_amd.ops import cpu_engine as ce  # noqa: E402

w = load_default_workload()
p = w.pods
h = [(int(p.pod_ctime[i]), int(p.pod_rank[i]), i, 0) for i in range(p.n_pods)]
heapq.heapify(h)
ev = 0
create_ev = []
run = maxrun = 0
while h:
    t, r, i, k = heapq.heappop(h)
    if k == 0:
        create_ev.append(ev)
        heapq.heappush(h, (t + int(p.pod_dur[i]), r, i, 1))
        run += 1
        maxrun = max(maxrun, run)
    else:
        run -= 1
    ev += 1
print("no-failure stream events", ev, "max running pods", maxrun)
family = sys.argv[1] if len(sys.argv) > 1 else "composite_linear"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 16
W = fam.SAMPLERS[family](n, np.random.default_rng(0))
tab = ce.simulate_builtin_batch(w, family, fam.pad_weights(W))
fr, share = [], []
for wv, row in zip(W, tab):
    r = ce.simulate_builtin(w, family, list(wv), ce.SimOptions(record_states=True))
    N, G = w.cluster.n_nodes, int(w.cluster.gpu_start[-1])
    decision = np.asarray(r["states"], dtype=np.int64).reshape(-1, 2 + 3 * N + G)[:, 1]
    fails = np.nonzero(decision < 0)[0]
    c = int(fails[0]) if fails.size else len(decision)
    e = create_ev[c] if c < len(create_ev) else ev
    fr.append(e)
    share.append(e / max(1.0, row[8]))
    print(f"first failure at creation {c} = event {e}; replay events {int(row[8])}; failures {fails.size}", flush=True)
print(f"prefix events mean {np.mean(fr):.0f} median {np.median(fr):.0f} min {min(fr)} max {max(fr)}; "
      f"mean share of replay events {np.mean(share):.3f}")
