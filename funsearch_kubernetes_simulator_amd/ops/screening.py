"""MFMA surrogate screening of linear policy candidates.

Exact replay is block-diagonal: every candidate drives its own cluster state,
so its per-event feature x weight products are a batched GEMV.  Matrix cores
pay where states are *shared* (SURVEY.md section 7.4): record the S
(pod, cluster-state) pairs one reference replay visits, build the composite
feature matrix X[S*Np, K] once, and score P candidate weight vectors on all of
them with one GEMM, Y = X W, in `k_screen_linear` (fp32 MFMA
`v_mfma_f32_32x32x2_f32`, csrc/hip/screen.hip).  The kernel's epilogue takes
each candidate's argmax node per state (first node wins ties, like the
reference's strict `>` scan; best <= 0 means "not placed") and sums a reward
for that decision, giving a fitness surrogate for thousands of candidates in
about a millisecond.  It is a *pre-filter*: the evolutionary search proposes
k x more candidates, keeps the best-screened 1/k, and scores those with exact
replay (`models/families.py` + `engine.Evaluator`).

Rewards (per state s and node n):
* ``myopic``: packing quality of putting the pod on n -- mean post-placement
  cpu / memory / GPU-count utilisation of the node minus twice the GPU-milli
  it strands (free milli on partially used GPUs), normalised per node;
* ``imitation``: 1 where n is the reference replay's own decision.
"""

from __future__ import annotations

from dataclasses import dataclass
from typing import Optional

import numpy as np

from ..core.arrays import Workload
from ..models import families as fam

KP = 18          # 16 composite features + infeasibility bias + zero pad (MFMA K steps of 2)
INFEASIBLE = -1.0e30


@dataclass
class RecordedStates:
    pod: np.ndarray        # [S] pod index (trace order)
    decision: np.ndarray   # [S] chosen node, -1 failed
    cpu_left: np.ndarray   # [S, N]
    mem_left: np.ndarray
    gpu_left: np.ndarray
    gml: np.ndarray        # [S, G] GPU milli left (cluster GPU order)

    @property
    def n_states(self) -> int:
        return int(self.pod.size)


def record_states(w: Workload, family: str = "composite_linear", weights=None) -> RecordedStates:
    """Replay one policy on the CPU oracle and record every creation event's state."""
    from . import cpu_engine as ce
    if weights is None and family == "composite_linear":
        weights = fam.CHAMPION_COMPOSITE
    r = ce.simulate_builtin(w, family, [] if weights is None else list(weights),
                            ce.SimOptions(record_states=True))
    N, G = w.cluster.n_nodes, int(w.cluster.gpu_start[-1])
    rec = np.asarray(r["states"], dtype=np.int64).reshape(-1, 2 + 3 * N + G)
    return RecordedStates(rec[:, 0], rec[:, 1], rec[:, 2:2 + N], rec[:, 2 + N:2 + 2 * N],
                          rec[:, 2 + 2 * N:2 + 3 * N], rec[:, 2 + 3 * N:])


def _pad_nodes(n: int) -> int:
    return max(32, (n + 31) // 32 * 32)


def _per_node_gpu(w: Workload, gml: np.ndarray):
    """[S, N, GMAX] left / total arrays with -1 padding for absent GPUs."""
    c = w.cluster
    N = c.n_nodes
    gmax = max(1, int(c.node_ngpus.max(initial=0)))
    left = np.full((gml.shape[0], N, gmax), -1, dtype=np.int64)
    tot = np.full((N, gmax), -1, dtype=np.int64)
    for n in range(N):
        a, b = int(c.gpu_start[n]), int(c.gpu_start[n + 1])
        left[:, n, :b - a] = gml[:, a:b]
        tot[n, :b - a] = c.gpu_milli_total[a:b]
    return left, tot


def composite_features(w: Workload, st: RecordedStates) -> np.ndarray:
    """X [S * Np, KP] float32: the composite family's 16 features per (state, node)
    (models/families.py COMPOSITE_FEATURES), column 16 = infeasibility bias."""
    c, p = w.cluster, w.pods
    S, N = st.n_states, c.n_nodes
    Np = _pad_nodes(N)
    pc, pm = p.pod_cpu[st.pod][:, None].astype(np.float64), p.pod_mem[st.pod][:, None].astype(np.float64)
    png, pgm = p.pod_ngpu[st.pod][:, None], p.pod_gmilli[st.pod][:, None]
    ct, mt = c.node_cpu_total[None, :].astype(np.float64), c.node_mem_total[None, :].astype(np.float64)
    cl, ml, gl = st.cpu_left.astype(np.float64), st.mem_left.astype(np.float64), st.gpu_left
    ng = c.node_ngpus[None, :]
    gleft, gtot = _per_node_gpu(w, st.gml)
    present = gleft >= 0
    lft = np.where(present, gleft, 0)
    free_m = lft.sum(-1)
    fits = present & (gleft >= pgm[:, :, None])
    feasible = (pc <= cl) & (pm <= ml) & (png <= gl) & ((png == 0) | (fits.sum(-1) >= png))
    gpod = png > 0
    cpu_u = (ct - cl) / np.maximum(1, ct)
    mem_u = (mt - ml) / np.maximum(1, mt)
    cap = gl * gtot[None, :, 0]
    gpu_u = np.where(gpod, (cap - free_m) / np.maximum(1, cap), 0.0)
    gmax_ = np.where(present, gleft, np.iinfo(np.int64).min).max(-1)
    gmin_ = np.where(present, gleft, np.iinfo(np.int64).max).min(-1)
    slack = np.where(fits, gleft - pgm[:, :, None], np.iinfo(np.int64).max).min(-1)
    idle = (present & (gleft == gtot[None])).sum(-1)
    F = np.zeros((S, N, 16))
    F[..., 0] = 1.0
    F[..., 1] = np.where(cpu_u < 0.7, 1.0 - cpu_u, 0.0)
    F[..., 2] = np.where(cpu_u >= 0.7, 1.0 - cpu_u, 0.0)
    F[..., 3] = np.where(mem_u < 0.7, 1.0 - mem_u, 0.0)
    F[..., 4] = np.where(mem_u >= 0.7, 1.0 - mem_u, 0.0)
    F[..., 5] = np.where(gpod, np.where(gpu_u < 0.7, 1.0 - gpu_u, 0.0), 0.0)
    F[..., 6] = np.where(gpod, np.where(gpu_u >= 0.7, 1.0 - gpu_u, 0.0), 0.0)
    F[..., 7] = np.where(gpod, free_m % np.maximum(1, pgm), 0)
    F[..., 8] = np.abs(cl / np.maximum(1, ml) - pc / np.maximum(1, pm))
    F[..., 9] = ((cl > 2 * pc) & (ml > 2 * pm)).astype(np.float64)
    F[..., 10] = np.where(gpod & (ng > 0), gmax_ - gmin_, 0)
    F[..., 11] = ((ct > 10000) & (mt > 64)).astype(np.float64) * np.ones_like(cl)
    F[..., 12] = ((cpu_u > 0.9) | (mem_u > 0.9)).astype(np.float64)
    F[..., 13] = np.where(gpod & (slack < np.iinfo(np.int64).max), slack / 1000.0, 0.0)
    F[..., 14] = idle / np.maximum(1, ng)
    F[..., 15] = ((~gpod) & (ng > 0)).astype(np.float64)
    X = np.zeros((S, Np, KP), dtype=np.float32)
    X[:, :N, :16] = np.where(feasible[..., None], F, 0.0)
    X[:, :, 16] = INFEASIBLE
    X[:, :N, 16] = np.where(feasible, 0.0, INFEASIBLE)
    return X.reshape(S * Np, KP)


def rewards(w: Workload, st: RecordedStates, kind: str = "myopic"):
    """R [S * Np], Rfail [S] float32."""
    c, p = w.cluster, w.pods
    S, N = st.n_states, c.n_nodes
    Np = _pad_nodes(N)
    R = np.zeros((S, Np), dtype=np.float32)
    if kind == "imitation":
        ok = st.decision >= 0
        R[np.nonzero(ok)[0], st.decision[ok]] = 1.0
        return R.reshape(-1), np.where(st.decision < 0, 1.0, 0.0).astype(np.float32)
    pc, pm = p.pod_cpu[st.pod][:, None], p.pod_mem[st.pod][:, None]
    png, pgm = p.pod_ngpu[st.pod][:, None], p.pod_gmilli[st.pod][:, None]
    ct, mt, ng = c.node_cpu_total[None, :], c.node_mem_total[None, :], c.node_ngpus[None, :]
    gleft, gtot = _per_node_gpu(w, st.gml)
    present = gleft >= 0
    util = ((ct - st.cpu_left + pc) / np.maximum(1, ct) + (mt - st.mem_left + pm) / np.maximum(1, mt)
            + np.where(ng > 0, (ng - st.gpu_left + png) / np.maximum(1, ng), 0.0)) / 3.0
    # stranded milli after a best-fit placement of the pod's GPUs
    after = gleft.copy()
    fits = present & (gleft >= pgm[:, :, None])
    key = np.where(fits, gleft, np.iinfo(np.int64).max)
    order = np.argsort(key, axis=-1, kind="stable")
    rank = np.argsort(order, axis=-1, kind="stable")
    take = fits & (rank < png[:, :, None])
    after = np.where(take, after - pgm[:, :, None], after)
    tot_node = np.maximum(1, np.where(present, gtot[None], 0).sum(-1))
    stranded = np.where(present & (after > 0) & (after < np.where(present, gtot[None], 0)), after, 0).sum(-1)
    R[:, :N] = util - 2.0 * stranded / tot_node
    return R.reshape(-1), np.full(S, -1.0, dtype=np.float32)


def weights_matrix(weights: np.ndarray) -> np.ndarray:
    """Wt [KP, Ppad] float32 (candidate weights as columns, bias row = 1)."""
    W = np.atleast_2d(np.asarray(weights, dtype=np.float64))
    P = W.shape[0]
    Ppad = (P + 31) // 32 * 32
    Wt = np.zeros((KP, Ppad), dtype=np.float32)
    Wt[:16, :P] = W[:, :16].T
    Wt[16, :] = 1.0
    return Wt


def screen_numpy(X, Wt, R, Rfail, Np: int, chunk: int = 256) -> np.ndarray:
    """fp32 reference of k_screen_linear (same argmax / tie / reward rules)."""
    M = X.shape[0]
    S = M // Np
    fit = np.zeros(Wt.shape[1], dtype=np.float64)
    for s0 in range(0, S, chunk):
        s1 = min(S, s0 + chunk)
        Y = (X[s0 * Np:s1 * Np] @ Wt).reshape(s1 - s0, Np, -1)
        best = Y.argmax(axis=1)                                   # first max
        bv = np.take_along_axis(Y, best[:, None, :], axis=1)[:, 0]
        Rs = R[s0 * Np:s1 * Np].reshape(s1 - s0, Np)
        rew = np.take_along_axis(Rs, best, axis=1)
        fit += np.where(bv > 0, rew, Rfail[s0:s1, None]).sum(0)
    return fit.astype(np.float32)


class Screener:
    """Surrogate fitness of composite-family candidates on one recorded trajectory.

    ``state_stride`` keeps every k-th recorded state (the surrogate is a sum
    over states, so a subsample ranks candidates almost identically at 1/k of
    the MFMA work).  On a HIP device the features / rewards are uploaded once
    (``_fks_hip.ScreenDevice``) and every `score` call moves only the
    candidates' weights and their fitness."""

    def __init__(self, w: Workload, reference_weights=None, kind: str = "myopic", device="auto",
                 state_stride: int = 1):
        self.workload = w
        self.kind = kind
        self.state_stride = int(state_stride)
        self.Np = _pad_nodes(w.cluster.n_nodes)
        self.device = None
        self._dev = None
        self.refreshes = 0
        if device != "cpu":
            from . import hip_engine
            if hip_engine.device_available():
                self.device = 0 if device == "auto" else int(device)
            elif device not in ("auto",):
                raise RuntimeError("HIP device requested but none is visible")
        self._load([reference_weights])

    def _load(self, weight_list) -> None:
        parts = []
        stride = self.state_stride * max(1, len(weight_list))   # same state budget for any trajectory count
        for i, wt in enumerate(weight_list):
            st = record_states(self.workload, "composite_linear", wt)
            keep = np.arange(i % stride, st.n_states, stride)
            parts.append(RecordedStates(st.pod[keep], st.decision[keep], st.cpu_left[keep], st.mem_left[keep],
                                        st.gpu_left[keep], st.gml[keep]))
        self.states = RecordedStates(*(np.concatenate([getattr(q, f) for q in parts])
                                       for f in ("pod", "decision", "cpu_left", "mem_left", "gpu_left", "gml")))
        self.X = composite_features(self.workload, self.states)
        self.R, self.Rfail = rewards(self.workload, self.states, self.kind)
        if self.device is not None:
            from . import hip_engine
            self._dev = hip_engine.native().ScreenDevice(self.X, self.R, self.Rfail, self.Np, self.device)

    def refresh(self, weight_list) -> None:
        """Re-draw the surrogate states from the given candidates' own
        trajectories (e.g. the islands' current elites, every migration epoch):
        the surrogate then scores proposals on states the search actually
        visits, not on one fixed policy's."""
        self._load([np.asarray(wt, dtype=np.float64) for wt in weight_list])
        self.refreshes += 1

    @staticmethod
    def spearman(surrogate: np.ndarray, exact: np.ndarray) -> float:
        """Rank correlation of surrogate and exact scores (average ranks for ties)."""
        from scipy.stats import spearmanr
        r = spearmanr(np.asarray(surrogate, dtype=np.float64), np.asarray(exact, dtype=np.float64)).correlation
        return float(r) if r == r else 0.0

    @property
    def n_states(self) -> int:
        return self.states.n_states

    def score(self, weights: np.ndarray) -> np.ndarray:
        P = np.atleast_2d(weights).shape[0]
        Wt = weights_matrix(weights)
        if self._dev is not None:
            fit = self._dev.score(Wt)
        else:
            fit = screen_numpy(self.X, Wt, self.R, self.Rfail, self.Np)
        return np.asarray(fit[:P], dtype=np.float64)

    def select(self, weights: np.ndarray, keep: int) -> np.ndarray:
        """Indices of the `keep` best-screened candidates, in their input order
        (the proposer's longest-replay-first order survives the filter)."""
        fit = self.score(weights)
        if keep >= len(fit):
            return np.arange(len(fit))
        top = np.argpartition(-fit, keep - 1)[:keep]
        return np.sort(top)
