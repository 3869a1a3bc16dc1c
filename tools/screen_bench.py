"""MFMA behavioural screening (ops/screen.py, k_score_linear_mfma) on the
MI355X: throughput over P feature_linear candidates x S recorded states, and
how many candidates of a batch are behavioural duplicates -- for random
family samples and for the children of one elite (the family search's
mutation step: Gaussian perturbation of 1-2 weights).

    python tools/screen_bench.py [--P 65536] [--S 512]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--P", type=int, default=65536)
    ap.add_argument("--S", type=int, default=512)
    a = ap.parse_args()
    from funsearch_kubernetes_simulator_amd.core import load_default_workload
    from funsearch_kubernetes_simulator_amd.models.families import sample_feature_linear
    from funsearch_kubernetes_simulator_amd.ops import screen
    w = load_default_workload()
    rng = np.random.default_rng(0)
    w0 = sample_feature_linear(1, rng)[0]
    t0 = time.perf_counter()
    st = screen.record_states(w, w0, every=8, max_states=a.S)
    rec_s = time.perf_counter() - t0
    out = {"states": st.S, "record_s": round(rec_s, 2)}
    W = sample_feature_linear(a.P, rng)
    screen.screen(st, W[:1024])                      # warm-up (module load, first launch)
    sig, _, ms = screen.screen(st, W)
    flops = 2.0 * a.P * st.S * 16 * 16
    out["random"] = {"P": a.P, "kernel_ms": round(ms, 3), "candidate_states_per_s": round(a.P * st.S / (ms / 1e3)),
                     "mfma_tflops": round(flops / (ms / 1e3) / 1e12, 2),
                     "distinct_fraction": round(len(screen.unique_by_signature(sig)) / a.P, 4)}
    # children of one elite: 1-2 weights perturbed (log-normal, sigma 0.35), as the family search mutates
    kids = np.repeat(w0[None, :], a.P, axis=0)
    for i in range(a.P):
        for j in rng.choice(12, size=1 + int(rng.random() < 0.5), replace=False):
            kids[i, j] *= np.exp(rng.normal(0.0, 0.35))
    sig_k, _, ms_k = screen.screen(st, kids)
    parent_sig, _, _ = screen.screen(st, w0[None, :])
    keep = screen.unique_by_signature(sig_k, exclude=[parent_sig[0]])
    out["children_of_one_elite"] = {"P": a.P, "kernel_ms": round(ms_k, 3),
                                    "same_as_parent_fraction": round(float((sig_k == parent_sig[0]).mean()), 4),
                                    "distinct_new_fraction": round(len(keep) / a.P, 4)}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
