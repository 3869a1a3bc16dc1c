"""Island evolution over parametric policy families (weights as genomes).

Each island keeps an elite set of weight vectors and proposes a generation of
candidates by Gaussian mutation of elites (multiplicative noise per weight,
occasional sign flips / zeroing), uniform crossover between elites, and fresh
samples from the family prior.  All islands of all ranks are evaluated in
batched device launches; every `migrate_every` generations each island's best
members are all-gathered across ranks (RCCL) and injected into the next
island (ring topology over the global island index).

This is the high-throughput half of the search: it finds good members of a
family at 10^4+ evaluations/s; every member converts to an ordinary program
(`models.families.to_program`) for the program-level FunSearch loop.
"""

from __future__ import annotations

from dataclasses import dataclass, field
from typing import Callable, List, Optional, Tuple

import numpy as np

from ..models import families as fam


@dataclass
class ParamIsland:
    family: str
    n_candidates: int
    elite_size: int
    rng: np.random.Generator
    sampler: Callable[[int, np.random.Generator], np.ndarray]
    sigma: float = 0.15
    fresh_fraction: float = 0.1
    elites: np.ndarray = field(default=None)       # [E, K]
    elite_scores: np.ndarray = field(default=None)  # [E]
    elite_events: np.ndarray = field(default=None)  # [E] replay events of each elite (NaN: unknown)
    generation: int = 0
    #: behavioural screen (ops/screen.py, k_score_linear_mfma): weights [P, K] ->
    #: signatures [P]; with it a generation draws `screen_factor` x the
    #: candidates and keeps those whose decisions on the recorded states differ
    #: from every elite's and from each other's (None: no screen)
    screener: Optional[Callable[[np.ndarray], np.ndarray]] = None
    screen_factor: int = 4
    screened: int = 0          # candidates drawn for the screen
    screen_kept: int = 0       # of those, behaviourally new (replayed)

    def __post_init__(self):
        k = self.sampler(1, self.rng).shape[1]
        self.elites = np.zeros((0, k))
        self.elite_scores = np.zeros(0)
        self.elite_events = np.zeros(0)

    @property
    def best(self) -> Tuple[Optional[np.ndarray], float]:
        if not len(self.elite_scores):
            return None, float("-inf")
        i = int(np.argmax(self.elite_scores))
        return self.elites[i], float(self.elite_scores[i])

    def propose(self, n: Optional[int] = None) -> np.ndarray:
        """A generation of candidates, longest predicted replay first.

        The device drains a batch through a persistent queue in index order,
        so handing out the long replays first and the short ones last (LPT
        scheduling) keeps the rows of a wave finishing close together.  A
        mutant is predicted to replay as many events as its parent, a
        crossover as its longer parent; fresh samples (unknown) go first."""
        n = self.n_candidates if n is None else int(n)
        if self.screener is not None and len(self.elites):
            from ..ops.screen import unique_by_signature
            draw = self._propose(n * max(1, int(self.screen_factor)))
            sig = np.asarray(self.screener(draw))
            known = np.asarray(self.screener(self.elites))
            keep = unique_by_signature(sig, exclude=known.tolist())[:n]   # LPT order kept
            self.screened += len(draw)
            self.screen_kept += len(keep)
            if len(keep):
                return draw[keep]
        return self._propose(n)

    def _propose(self, n: int) -> np.ndarray:
        if len(self.elites) == 0:
            return self.sampler(n, self.rng)
        n_fresh = max(1, int(n * self.fresh_fraction))
        n_cross = n // 4
        n_mut = n - n_fresh - n_cross
        E = len(self.elites)
        # rank-weighted parent choice
        order = np.argsort(-self.elite_scores)
        p = 1.0 / (np.arange(E) + 1.0)
        p /= p.sum()
        ia = order[self.rng.choice(E, n_mut, p=p)]
        pa = self.elites[ia]
        scale = self.sigma * self.rng.standard_normal(pa.shape)
        mut = pa * np.exp(scale) + self.rng.normal(0, self.sigma * 0.05, pa.shape) * np.abs(pa).mean(0)
        flip = self.rng.random(pa.shape) < 0.02
        mut[flip] = -mut[flip]
        zero = self.rng.random(pa.shape) < 0.02
        mut[zero] = 0.0
        ca = order[self.rng.choice(E, n_cross, p=p)]
        cb = order[self.rng.choice(E, n_cross, p=p)]
        a, b = self.elites[ca], self.elites[cb]
        mask = self.rng.random(a.shape) < 0.5
        cross = np.where(mask, a, b)
        fresh = self.sampler(n_fresh, self.rng)
        ev = self.elite_events
        pred = np.concatenate([ev[ia], np.fmax(ev[ca], ev[cb]), np.full(n_fresh, np.nan)])
        pred = np.where(np.isnan(pred), np.inf, pred)
        lpt = np.argsort(-pred, kind="stable")
        return np.concatenate([mut, cross, fresh])[lpt]

    def update(self, weights: np.ndarray, scores: np.ndarray, events: Optional[np.ndarray] = None) -> None:
        self.generation += 1
        if events is None:
            events = np.full(len(scores), np.nan)
        allw = np.concatenate([self.elites, weights])
        alls = np.concatenate([self.elite_scores, scores])
        alle = np.concatenate([self.elite_events, np.asarray(events, dtype=np.float64)])
        # dedup exact duplicates, keep the best elite_size
        _, uniq = np.unique(np.round(allw, 12), axis=0, return_index=True)
        allw, alls, alle = allw[uniq], alls[uniq], alle[uniq]
        keep = np.argsort(-alls, kind="stable")[:self.elite_size]
        self.elites, self.elite_scores, self.elite_events = allw[keep], alls[keep], alle[keep]

    def migrants(self, k: int) -> np.ndarray:
        """[k, 1 + K] records: score, weights (best first; -inf padded)."""
        K = self.elites.shape[1]
        out = np.full((k, 1 + K), -np.inf)
        order = np.argsort(-self.elite_scores)[:k]
        out[:len(order), 0] = self.elite_scores[order]
        out[:len(order), 1:] = self.elites[order]
        out[len(order):, 1:] = 0.0
        return out

    def accept(self, records: np.ndarray) -> None:
        rec = records[np.isfinite(records[:, 0])]
        if len(rec):
            self.update(rec[:, 1:], rec[:, 0])
            self.generation -= 1


def make_islands(n: int, family: str, n_candidates: int, elite_size: int, seed: int) -> List[ParamIsland]:
    sampler = fam.SAMPLERS[family]
    return [ParamIsland(family, n_candidates, elite_size, np.random.default_rng(seed + 7919 * i), sampler)
            for i in range(n)]


def migration_records(islands: List[ParamIsland], k: int) -> np.ndarray:
    """[I, k, 1 + K]: every local island's best k members (score, weights)."""
    return np.stack([isl.migrants(k) for isl in islands])


def inject(islands: List[ParamIsland], glob: np.ndarray, rank: int = 0) -> None:
    """Ring migration over the global island index (rank-major): island g
    receives island g-1's migrants.  glob: [W, I, k, R] all-gathered records."""
    for li in range(len(islands)):
        inject_one(islands, li, glob, rank)


def inject_one(islands: List[ParamIsland], li: int, glob: np.ndarray, rank: int = 0) -> None:
    """inject() for local island `li` alone (asynchronous migration: each
    island takes its ring predecessor's migrants when it reaches a boundary)."""
    W, I, k = glob.shape[0], glob.shape[1], glob.shape[2]
    flat = glob.reshape(W * I, k, -1)
    islands[li].accept(flat[(rank * I + li - 1) % (W * I)])


def migrate(islands: List[ParamIsland], k: int, all_gather=None) -> None:
    """Synchronous ring migration (an RCCL all-gather across ranks)."""
    local = migration_records(islands, k)
    glob = all_gather(local) if all_gather is not None else local[None]   # [W, I, k, R]
    from ..parallel.dist import context
    inject(islands, glob, context().rank if all_gather is not None else 0)
