"""Behavioural screening of linear-family candidates on the matrix cores.

A `feature_linear` / `composite_linear` candidate is a weight vector over the
family's node features (`models.families.FEATURES`, `COMPOSITE_FEATURES`).  Replays diverge after the first
placement, so the per-event products are per-policy (VALU work, see
docs/ARCHITECTURE.md "Considered and not built"); but scored on one common set
of *recorded* cluster states, every candidate shares the same feature blocks
and the scoring is a real GEMM -- `k_score_linear_mfma`
(`csrc/hip/screen_mfma.hip.h`, v_mfma_f32_16x16x4_f32), SURVEY section 7.4
item 3's shared-operand case.

What it is for: a candidate's *decisions* on the recorded states (which node
each recorded pod would go to) give a behavioural signature; candidates with
equal signatures place every recorded pod alike and mostly replay alike, so a
search can replay one of each (`unique_by_signature`).  It is a screen, not a
score: f32 products may differ from the replay's f64 arithmetic at near-ties,
and the exact replay stays the only fitness.

    states = record_states(workload, seed_weights, family)   # object-engine replay, every k-th creation
    sig, dec, ms = screen(states, W)                    # MFMA on the device
    keep = unique_by_signature(sig)
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional, Sequence, Tuple

import numpy as np

from ..models import families as fam

STEPS = 5        # MFMA k-steps of 4 (csrc/hip/screen_mfma.hip.h kScreenSteps)
K = 4 * STEPS    # feature slots: the family's features, zero pads, the feasibility bias (last)
NODES = 16       # nodes per state (the row-kernel cluster size)
MASK = -1e30     # bias of an infeasible (or padding) node


@dataclass
class States:
    """Recorded states: node features [S, 16, F] (float64), feasibility
    [S, 16] and the node the recording policy chose (-1: none)."""
    feats: np.ndarray
    feasible: np.ndarray
    chosen: np.ndarray

    @property
    def S(self) -> int:
        return int(self.feats.shape[0])


FAMILIES = ("feature_linear", "composite_linear")


def _features(family: str):
    if family == "feature_linear":
        return fam.FEATURES, ""
    if family == "composite_linear":
        return fam.COMPOSITE_FEATURES, fam.COMPOSITE_PREAMBLE
    raise ValueError(f"screening covers {FAMILIES}, not {family!r}")


def n_features(family: str) -> int:
    return len(_features(family)[0])


def _feature_fn(family: str):
    # the family's own expressions (models/families.py, our constants only),
    # evaluated per (pod, node) after the family's preamble
    feats, pre = _features(family)
    src = "def _f(pod, node):\n" + pre + "    return (" + ", ".join(e for _, e in feats) + ",)\n"
    env = {"min": min, "max": max, "sum": sum, "abs": abs, "len": len}
    exec(compile(src, "<screen-features>", "exec"), env)
    return env["_f"]


def _feasible(pod, node) -> bool:
    # the template's feasibility prologue (policy/template.py)
    if pod.cpu_milli > node.cpu_milli_left or pod.memory_mib > node.memory_mib_left or pod.num_gpu > node.gpu_left:
        return False
    if pod.num_gpu > 0:
        return sum(1 for g in node.gpus if g.gpu_milli_left >= pod.gpu_milli) >= pod.num_gpu
    return True


def record_states(workload, weights: Sequence[float], family: str = "feature_linear", every: int = 16,
                  max_states: int = 512) -> States:
    """Replay the `family` policy `weights` on the object engine and record
    the node features, feasibility and the chosen node at every `every`-th
    creation event (up to `max_states`; the replay stops there)."""
    from ..funsearch.scheduler import FunSearchScheduler
    from ..simulator import DiscreteEventSimulator, KubernetesSimulator
    if workload.cluster.n_nodes > NODES:
        raise ValueError(f"screening records clusters of <= {NODES} nodes")
    feat = _feature_fn(family)
    F_n = n_features(family)
    if F_n > K - 1:
        raise ValueError(f"{family}: {F_n} features do not fit {K - 1} slots")
    sched = FunSearchScheduler(fam.to_program(family, weights))
    cluster, pods = workload.to_objects()
    F, M, C = [], [], []
    count = [0]

    class Recorder(KubernetesSimulator):
        def _select_node(self, pod):
            best = super()._select_node(pod)
            count[0] += 1
            if count[0] % every == 0 and len(F) < max_states:
                f = np.zeros((NODES, F_n))
                m = np.zeros(NODES, dtype=bool)
                ch = -1
                for j, node in enumerate(self.cluster.nodes_dict.values()):
                    if _feasible(pod, node):
                        m[j] = True
                        f[j] = feat(pod, node)
                    if node is best:
                        ch = j
                F.append(f)
                M.append(m)
                C.append(ch)
                if len(F) >= max_states:
                    raise _Done
            return best

    try:
        Recorder(cluster, pods, DiscreteEventSimulator(pods), sched).run_schedule()
    except _Done:
        pass
    return States(np.asarray(F), np.asarray(M), np.asarray(C, dtype=np.int64))


class _Done(Exception):
    """Enough states recorded: the replay stops."""


def arrange_states(st: States) -> np.ndarray:
    """X in the kernel's A-fragment layout: float32 [S, STEPS, 64], element
    (s, t, l) = feature 4t + (l >> 4) of node l & 15 (slot K - 1: the bias)."""
    S, F_n = st.S, st.feats.shape[2]
    full = np.zeros((S, NODES, K), dtype=np.float64)
    full[:, :, :F_n] = st.feats
    full[:, :, K - 1] = np.where(st.feasible, 0.0, MASK)
    lanes = np.arange(64)
    out = np.empty((S, STEPS, 64), dtype=np.float32)
    for t in range(STEPS):
        out[:, t, :] = full[:, lanes & 15, 4 * t + (lanes >> 4)]
    return out


def arrange_weights(W: np.ndarray, F_n: int) -> Tuple[np.ndarray, int]:
    """W [P, >= F_n] in the B-fragment layout: float32 [tiles, STEPS, 64],
    element (tile, t, l) = weight 4t + (l >> 4) of candidate 16 tile + (l & 15);
    slot K - 1 = 1 (the feasibility bias), padding candidates all zero."""
    W = np.asarray(W, dtype=np.float64)
    P = W.shape[0]
    tiles = (P + 15) // 16
    full = np.zeros((tiles * 16, K), dtype=np.float64)
    full[:P, :F_n] = W[:, :F_n]
    full[:P, K - 1] = 1.0
    lanes = np.arange(64)
    out = np.empty((tiles, STEPS, 64), dtype=np.float32)
    for t in range(STEPS):
        out[:, t, :] = full.reshape(tiles, 16, K)[:, lanes & 15, 4 * t + (lanes >> 4)]
    return out, P


def decisions_reference(st: States, W: np.ndarray, dtype=np.float64) -> np.ndarray:
    """[P, S] node the family's rule picks on each recorded state (255: none
    feasible): score = max(1, int(w . f)) on feasible nodes, the first maximum
    wins.  float64: the replay's arithmetic; float32: the kernel's."""
    f = st.feats.astype(dtype)
    W = np.asarray(W, dtype=dtype)[:, :f.shape[2]]
    v = np.einsum("snf,pf->psn", f, W)                         # [P, S, 16]
    sc = np.maximum(1.0, np.trunc(v))
    sc = np.where(st.feasible[None, :, :], sc, -2.0)
    best = sc.argmax(axis=2)                                   # first maximum
    none = ~st.feasible.any(axis=1)
    best = np.where(none[None, :], 255, best)
    return best.astype(np.uint8)


#: states per signature chunk: fixed, so a signature does not depend on the
#: batch it was computed in (an elite screened alone must match its copy in a
#: batch of 65,536); the launch runs one wave per (16 candidates, chunk), which
#: also gives small batches enough waves to cover the MFMA chain's latency
CHUNK = 16


def chunks_for(P: int, S: int) -> int:
    """State chunks of a launch (grid y): ceil(S / CHUNK), whatever P."""
    return int(-(-S // CHUNK))


def signature(dec: np.ndarray, chunks: int = 1) -> np.ndarray:
    """The kernel's signature of a [P, S] decision matrix (host twin): an
    FNV-1a fold of the decisions within each chunk of states, then of the
    chunk signatures in order."""
    P, S = dec.shape
    spc = -(-S // max(1, chunks))
    prime = np.uint64(0x100000001b3)
    basis = np.uint64(0xcbf29ce484222325)
    d = dec.astype(np.uint64)
    out = np.full(P, basis, dtype=np.uint64)
    for s0 in range(0, S, spc):
        h = np.full(P, basis, dtype=np.uint64)
        # 255 (none) folds as 256, like the kernel's (d + 1) with d = 255
        for s in range(s0, min(S, s0 + spc)):
            h = (h ^ (d[:, s] + np.uint64(1))) * prime
        out = (out ^ h) * prime
    return out


def screen(st: States, W: np.ndarray, want_dec: bool = False, device: int = 0):
    """(sig [P] uint64, dec [P, S] uint8 or None, kernel ms) on the MI355X
    (signature(dec, chunks_for(P, S)) is the signature's host twin)."""
    from . import hip_engine
    mod = hip_engine.native()
    X = arrange_states(st)
    Wt, P = arrange_weights(W, st.feats.shape[2])
    sig, dec, ms = mod.screen_linear(X.reshape(-1), Wt.reshape(-1), st.S, P, want_dec, device, chunks_for(P, st.S))
    return np.asarray(sig), (None if dec is None else np.asarray(dec)), float(ms)


def unique_by_signature(sig: np.ndarray, exclude: Optional[Sequence[int]] = None) -> np.ndarray:
    """Indices of the first candidate of every distinct signature (in order),
    without the signatures in `exclude` (e.g. the parents already scored)."""
    seen = set(int(x) for x in (exclude or ()))
    keep = []
    for i, x in enumerate(np.asarray(sig, dtype=np.uint64).tolist()):
        if x not in seen:
            seen.add(x)
            keep.append(i)
    return np.asarray(keep, dtype=np.int64)
