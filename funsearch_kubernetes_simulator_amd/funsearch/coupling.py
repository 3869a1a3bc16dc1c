"""Family coupling: a device family search that feeds program islands.

Program islands evaluate LLM-sized batches (a few dozen programs per island
step, one wave each), which leaves most of the MI355X's 256 CUs idle while the
slowest replay of the batch finishes.  The coupler fills that idle capacity: it
runs a parametric island search (`param_islands.ParamIsland`, tens of
thousands of exact replays per second on the row kernel) on its own HIP slot,
renders the family champion as ordinary program text
(`models.families.to_program`), re-scores that TEXT through the normal program
path (compile -> native JIT -> replay) and hands it to the program islands as a
migrant.  Program islands then mutate / polish it like any other elite.

Default family: ``random_linear`` -- the reference's own `_create_random_policy`
(`/root/reference/funsearch/funsearch_integration.py:403-431`), whose seeding
loop the reference ships disabled (``for _ in range(0)``, `:185-186`); with
``feature_linear`` (12 generic capacity / fragmentation features) as a second
family.  Neither family is derived from the reference champion, so a run seeded
with first-fit / best-fit only stays a from-scratch run.

The coupler is a plain object driven by `IslandFunSearch` (`islands.py`):
``round()`` runs a few generations of every family's island and returns the
new champion programs (if any improved); its state goes into checkpoints.
"""

from __future__ import annotations

import time
from typing import Dict, List, Optional

import numpy as np

from ..models import families as fam
from .param_islands import ParamIsland, make_islands

DEFAULT_FAMILIES = ("random_linear", "feature_linear")


class FamilyCoupler:
    def __init__(self, evaluator, cfg: Optional[dict] = None, slot: int = 0, seed: int = 0):
        cfg = dict(cfg or {})
        self.evaluator = evaluator
        self.slot = int(slot)
        self.every = int(cfg.get("every", 0))                       # program generations between rounds
        self.generations = int(cfg.get("generations", 4))            # family generations per round
        self.candidates = int(cfg.get("candidates", 4096))
        self.elite = int(cfg.get("elite", 32))
        self.families = tuple(cfg.get("families", DEFAULT_FAMILIES))
        for f in self.families:
            if f not in fam.SAMPLERS:
                raise ValueError(f"coupling: unknown family {f!r}")
        self.islands: Dict[str, ParamIsland] = {
            f: make_islands(1, f, self.candidates, self.elite, seed=seed + 31 * k)[0]
            for k, f in enumerate(self.families)}
        self.exported: Dict[str, float] = {f: float("-inf") for f in self.families}   # best score handed out
        #: behavioural screen on the matrix cores (``coupling.screen``: {"factor",
        #: "states", "every"}): linear families draw factor x the candidates and
        #: replay only those that place the recorded pods differently from the
        #: elites and each other (ops/screen.py)
        self.screen_cfg = cfg.get("screen")
        self._screen_ready = False
        self.rounds = 0
        self.evaluated = 0
        self.seconds = 0.0

    @property
    def enabled(self) -> bool:
        return self.every > 0

    def due(self, generation: int) -> bool:
        return self.enabled and generation > 0 and generation % self.every == 0

    def _evaluate(self, family: str, weights: np.ndarray) -> np.ndarray:
        ev = self.evaluator
        if getattr(ev, "device", None) is not None:
            ev.submit_family(self.slot, family, weights)   # its own stream: program islands keep running
            return ev.wait(self.slot)
        return ev.evaluate_family(family, weights)

    def _setup_screen(self) -> None:
        self._screen_ready = True
        sc = self.screen_cfg
        ev = self.evaluator
        if not sc or getattr(ev, "device", None) is None:
            return
        from ..ops import screen
        w = ev.workload
        if w.cluster.n_nodes > screen.NODES:
            return
        sc = sc if isinstance(sc, dict) else {}
        dev_index = int(getattr(ev.device, "device", 0) or 0)
        for f, isl in self.islands.items():
            if f not in screen.FAMILIES:
                continue
            seed = fam.CHAMPION_COMPOSITE if f == "composite_linear" else fam.SAMPLERS[f](1, np.random.default_rng(0))[0]
            st = screen.record_states(w, seed, family=f, every=int(sc.get("every", 8)),
                                      max_states=int(sc.get("states", 512)))
            isl.screener = (lambda W, st=st: screen.screen(st, W, device=dev_index)[0])
            isl.screen_factor = int(sc.get("factor", 4))

    def round(self) -> List[dict]:
        """Advance every family island by ``generations``; return one record
        per family whose champion beat what was exported before:
        ``{"family", "weights", "family_score", "code", "score"}`` where
        ``score`` is the exact re-score of the rendered program text."""
        from ..engine import COLS
        t0 = time.time()
        if not self._screen_ready:
            self._setup_screen()
        out = []
        for f, isl in self.islands.items():
            for _ in range(self.generations):
                w = isl.propose()
                tab = self._evaluate(f, w)
                isl.update(w, tab[:, COLS["score"]], tab[:, COLS["n_events"]])
                self.evaluated += len(w)
            wbest, sbest = isl.best
            if wbest is None or not sbest > self.exported[f]:
                continue
            self.exported[f] = sbest
            k = fam.SAMPLERS[f](1, np.random.default_rng(0)).shape[1]
            code = fam.to_program(f, wbest[:k])
            res = self.evaluator.evaluate_programs([code], slot=self.slot)[0]   # the TEXT, normal path
            self.evaluated += 1
            out.append({"family": f, "weights": [float(x) for x in wbest[:k]], "family_score": sbest,
                        "code": code, "score": res.score})
        self.rounds += 1
        self.seconds += time.time() - t0
        return out

    # -- checkpoint ----------------------------------------------------------------------
    def state_dict(self) -> dict:
        return {"rounds": self.rounds, "evaluated": self.evaluated, "exported": dict(self.exported),
                "islands": {f: {"elites": isl.elites.tolist(), "scores": isl.elite_scores.tolist(),
                                "events": np.nan_to_num(isl.elite_events, nan=-1.0).tolist(),
                                "generation": isl.generation}
                            for f, isl in self.islands.items()}}

    def load_state_dict(self, st: dict) -> None:
        self.rounds = int(st.get("rounds", 0))
        self.evaluated = int(st.get("evaluated", 0))
        for f, v in (st.get("exported") or {}).items():
            if f in self.exported:
                self.exported[f] = float(v)
        for f, d in (st.get("islands") or {}).items():
            isl = self.islands.get(f)
            if isl is None or not d.get("elites"):
                continue
            isl.elites = np.asarray(d["elites"], dtype=np.float64)
            isl.elite_scores = np.asarray(d["scores"], dtype=np.float64)
            ev = np.asarray(d.get("events") or [-1.0] * len(isl.elite_scores), dtype=np.float64)
            isl.elite_events = np.where(ev < 0, np.nan, ev)
            isl.generation = int(d.get("generation", 0))
