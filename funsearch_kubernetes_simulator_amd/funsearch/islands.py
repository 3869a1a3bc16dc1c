"""Multi-island FunSearch over program text: `run_funsearch`.

Layout: one process per GPU (`parallel.dist`), ``islands.per_rank``
populations per process.  Each generation:

1. every island asks the LLM backend for children of two random elites
   (one shared thread pool -> concurrent LLM requests across islands);
2. all children of all islands are evaluated in ONE batched engine call
   (one k_replay wave per program on the MI355X);
3. each island merges its own children with the reference's rules
   (similarity filter, elites + children, truncate);
4. every ``migrate_every`` generations the best ``migrants`` programs of every
   island are all-gathered across ranks (`funsearch/migration.py`: one
   compressed variable-length blob per rank over RCCL, posted asynchronously
   in the pipelined and steady modes) and injected into the next island of a
   global ring;
5. global best / early stop: every migration payload carries the rank's best
   score and stop vote, so ranks agree at migration points without a
   per-generation all-reduce.

With ``islands.per_rank = 1`` on one process this is exactly `SimpleFunSearch`.
Checkpoints (``checkpoint.dir``) hold every island's population so a run can
`resume` after a crash, which the reference cannot.

Failure handling (the reference has none): a collective that
fails because a peer rank died makes the survivors checkpoint, log a
``rank_failure`` record and continue as single-rank jobs
(``islands.elastic``, on by default).  ``--resume`` is elastic: it re-shards
the saved islands of a run with any world size / islands-per-rank onto the
current layout (surplus islands are merged, missing ones are cloned), so a
job restarted on fewer or more GPUs (e.g. by ``torchrun --max-restarts``)
keeps every population.
"""

from __future__ import annotations

import concurrent.futures
import glob
import json
import os
import threading
import time
from typing import List, Optional, Tuple

from ..engine import Evaluator
from ..parallel import dist
from ..utils.metrics import MetricsLog
from ..utils.trace import roctx_range
from .llm import make_client
from .search import FEEDBACK, SimpleFunSearch, load_config


class IslandFunSearch:
    def __init__(self, config, evaluator: Optional[Evaluator] = None, verbose: bool = False):
        self.config = load_config(config)
        self.ctx = dist.init_distributed(use_gpu=(self.config.get("device") or {}).get("kind", "auto") != "cpu")
        isl = self.config.get("islands") or {}
        self.n_islands = int(isl.get("per_rank", 1))
        self.migrate_every = int(isl.get("migrate_every", 50))
        self.n_migrants = int(isl.get("migrants", 2))
        self.elastic = bool(isl.get("elastic", True))
        # FunSearch-style island resets (off by default; the reference has one
        # population): every `reset_every` generations the weakest
        # `reset_fraction` of this rank's islands restart from the best program
        # of a random surviving island, so the islands do not all converge on
        # one lineage through migration
        self.reset_every = int(isl.get("reset_every", 0))
        self.reset_fraction = float(isl.get("reset_fraction", 0.5))
        # reset_diverse: a reset island restarts from the best program of the
        # surviving islands' populations that is NOT similar (the dedup ratio) to
        # any program another island already leads with -- so resets keep
        # lineages apart instead of cloning one island's champion
        self.reset_diverse = bool(isl.get("reset_diverse", False))
        # migrants enter only if no equal-or-better member is too similar
        # (the island's own dedup rule) and they beat its worst member
        self.migrant_dedup = bool(isl.get("migrant_dedup", False))
        import random as _random
        self._reset_rng = _random.Random(int((self.config.get("llm") or {}).get("seed", 0)) * 31 + 7)
        self.resets = 0
        # constant polish of island champions on the device (funsearch/polish.py)
        pol = self.config.get("polish") or {}
        self.polish_every = int(pol.get("every", 0))
        self.polish_variants = int(pol.get("variants", 1024))
        self.polish_rounds = int(pol.get("rounds", 3))
        # repeat: polish the island champion at every due generation with fresh
        # random variants, even when it has been polished before (a (1 + lambda)
        # strategy over its constants that keeps running on the device)
        self.polish_repeat = bool(pol.get("repeat", False))
        #: steady mode: also polish island champions on HIP slots that would
        #: otherwise idle while the producers refill the child queue
        self.polish_idle = bool(pol.get("idle", False))
        self._polished = set()
        # islands step independently (LLM / JIT / device stages overlap across islands)
        self.pipeline = bool(isl.get("pipeline", False))
        # steady-state mode (funsearch/steady.py): hundreds of programs in flight,
        # children sampled from the islands' current populations, no lockstep
        self.mode = str(isl.get("mode", "steady" if isl.get("steady") else ("pipeline" if self.pipeline else "sync")))
        self.steady_cfg = dict(isl.get("steady") or {})
        self.failures: List[dict] = []
        self._count_lock = threading.Lock()
        self._ck_due = False
        dev = (self.config.get("device") or {}).get("kind", "auto")
        if dev == "auto" and self.ctx.backend == "nccl":
            dev = self.ctx.local_rank
        opts = {}
        if "min_batch" in (self.config.get("device") or {}):
            opts["device_min_batch"] = int(self.config["device"]["min_batch"])
        if "compile_workers" in (self.config.get("device") or {}):
            opts["compile_workers"] = int(self.config["device"]["compile_workers"])
        fi = self.config.get("fault_injection") or {}
        if fi.get("eval_failure_rate"):
            opts["fault_rate"] = float(fi["eval_failure_rate"])
            opts["fault_seed"] = int(fi.get("seed", 0))
        if fi.get("llm_failure_rate"):
            self.config.setdefault("llm", {})["fault_rate"] = float(fi["llm_failure_rate"])
        # one HIP stream (slot) per island, so pipelined islands never share one,
        # plus one for the family coupler (funsearch/coupling.py)
        cpl = dict(self.config.get("coupling") or {})
        # steady mode may ask for more slots than islands: more batches in flight
        # than the chip holds, so one batch's slowest programs never idle the CUs
        # the rest of it has left (each slot is a stream: run with
        # GPU_MAX_HW_QUEUES >= slots so the launches overlap)
        st_slots = int(((self.config.get("islands") or {}).get("steady") or {}).get("slots") or 0)
        self.evaluator = evaluator or Evaluator(device=dev, options=opts,
                                                n_slots=max(4, self.n_islands, st_slots) +
                                                (1 if cpl.get("every") else 0))
        llm_cfg = dict(self.config.get("llm") or {})
        base_seed = int(llm_cfg.get("seed", 0)) + 1000003 * self.ctx.rank
        self.islands: List[SimpleFunSearch] = []
        for i in range(self.n_islands):
            cfg = json.loads(json.dumps(self.config))
            cfg.setdefault("llm", dict(llm_cfg))
            if cfg["llm"].get("backend") in ("mutation", "offline"):
                cfg["llm"]["seed"] = base_seed + 7919 * i
            cfg["checkpoint"] = {}
            self.islands.append(SimpleFunSearch(cfg, evaluator=self.evaluator, seed=base_seed + i,
                                                llm_client=None if cfg.get("llm") else make_client(cfg["llm"]),
                                                verbose=verbose))
        self.generation = 0
        self.evaluations = 0
        self.verbose = verbose
        log_path = self.config.get("log_path")
        if log_path and self.ctx.world_size > 1:
            root, ext = os.path.splitext(log_path)
            log_path = f"{root}.rank{self.ctx.rank}{ext}"
        self.log = MetricsLog(log_path)
        ck = self.config.get("checkpoint") or {}
        self.ck_dir = ck.get("dir")
        self.ck_every = int(ck.get("every", 0))
        self.coupler = None
        if cpl.get("every"):
            from .coupling import FamilyCoupler
            self.coupler = FamilyCoupler(self.evaluator, cpl, slot=self._n_slots() - 1,
                                         seed=int(cpl.get("seed", 0)) + 7907 * self.ctx.rank)

    # -- helpers --------------------------------------------------------------------------
    @property
    def _threshold(self) -> float:
        return self.islands[0].early_stop_threshold

    @property
    def best(self) -> Tuple[Optional[str], float]:
        b = max(self.islands, key=lambda s: s.best_score)
        return b.best_policy, b.best_score

    def initialize(self) -> None:
        first = self.islands[0]
        if not first.population:
            first.initialize_population()
        for s in self.islands[1:]:
            if not s.population:
                s.population = list(first.population)
                s.best_policy, s.best_score = first.best_policy, first.best_score

    def evolve(self) -> dict:
        t0 = time.time()
        self.generation += 1
        plans = []
        for s in self.islands:
            s.generation += 1
            s.population.sort(key=lambda x: x[1], reverse=True)
            elites = s.population[:s.elite_size]
            n_new = min(s.policies_per_generation, s.population_size - len(elites))
            plans.append((s, elites, max(0, n_new)))
        jobs = [(k, i) for k, (s, el, n) in enumerate(plans) if el for i in range(n)]
        workers = max(1, min(64, sum(s.max_workers for s in self.islands)))
        with concurrent.futures.ThreadPoolExecutor(max_workers=workers) as ex:
            outs = list(ex.map(lambda ki: (ki[0],) + plans[ki[0]][0]._generate_single_policy(
                ki[1], plans[ki[0]][1], FEEDBACK), jobs))
        children = [(k, code) for k, _, code in outs if code]
        t_gen = time.time()
        with roctx_range(f"funsearch.evaluate gen {self.generation} ({len(children)} programs)"):
            results = self.evaluator.evaluate_programs([c for _, c in children]) if children else []
        t_eval = time.time()
        self.evaluations += len(children)
        for k, (s, elites, _) in enumerate(plans):
            new = []
            for (kk, code), res in zip(children, results):
                if kk != k or s._is_too_similar(code, res.score):
                    continue
                new.append((code, res.score))
                if res.score > s.best_score:
                    s.best_score, s.best_policy = res.score, code
            s.population = sorted(elites + new, key=lambda x: x[1], reverse=True)[:s.population_size]
        for i in range(len(self.islands)):
            self.maybe_polish(i)
        if self.reset_every and self.generation % self.reset_every == 0:
            self.reset_weak_islands()
        if self.coupler is not None and self.coupler.due(self.generation):
            for rec in self.run_coupling():
                self.inject_coupled(rec)
        best_local = self.best[1]
        chan = self._sync_channel()
        stop = best_local >= self._threshold and not chan.active
        if chan.every and self.generation % chan.every == 0:
            # lock-step mode: a blocking gather; its header carries every rank's
            # best and stop vote (no per-generation all-reduce)
            with roctx_range(f"funsearch.migrate gen {self.generation}"):
                chan.post(self.generation, best_local >= self._threshold)
                for res in chan.poll(self._threshold, block=True):
                    for li, inc in res.incoming.items():
                        self.apply_migrants(li, inc)
                    stop = stop or chan.stopping
            chan.stop_at = None    # lock-step: nobody posted ahead, the decision is `stop`
        best_global = max(chan.best_global, best_local)
        rec = dict(kind="generation", rank=self.ctx.rank, generation=self.generation, best=best_local,
                   best_global=best_global, stop=bool(stop), collective_wait_s=round(chan.wait_s, 4),
                   children=len(children),
                   islands=[round(s.best_score, 6) for s in self.islands],
                   llm_s=round(t_gen - t0, 4), eval_s=round(t_eval - t_gen, 4),
                   evals_per_s=round(len(children) / max(1e-9, t_eval - t_gen), 2))
        self.log.write(**rec)
        if self.ck_dir and self.ck_every and self.generation % self.ck_every == 0:
            self.save_checkpoint()
        return rec

    def _sync_channel(self):
        if getattr(self, "_chan", None) is None:
            from .migration import MigrationChannel
            self._chan = MigrationChannel(self, self.migrate_every, self.generation)
        return self._chan

    def _collective(self, what: str, fn, fallback):
        """Run a collective; if a peer is gone, survive as a single-rank job."""
        if not self.ctx.distributed:
            return fn()
        try:
            return fn()
        except Exception as exc:        # DistBackendError / RuntimeError from a dead or timed-out peer
            self.rank_lost(what, exc)
            return fn() if fallback is None else fallback

    def rank_lost(self, what: str, exc: BaseException) -> None:
        """A collective failed (dead or timed-out peer): log it, leave the
        group and continue as a single-rank job (raises unless elastic)."""
        if not self.elastic:
            raise exc
        rec = dict(kind="rank_failure", rank=self.ctx.rank, generation=self.generation, collective=what,
                   world_size=self.ctx.world_size, error=f"{type(exc).__name__}: {str(exc)[:300]}")
        self.failures.append(rec)
        self.log.write(**rec)
        if self.verbose:
            print(json.dumps(rec), flush=True)
        self.ctx = dist.degrade_to_local(what)
        if self.ck_dir:
            self.save_checkpoint()

    def migrant_blob(self):
        """This rank's migrants (each island's top ``n_migrants``) as one
        variable-length record blob (`dist.pack_migrants`; drops are logged)."""
        recs = []
        for li, s in enumerate(self.islands):
            for code, score in sorted(s.population, key=lambda x: x[1], reverse=True)[:self.n_migrants]:
                recs.append((li, code, score))
        recs.sort(key=lambda r: r[2], reverse=True)
        return dist.pack_migrants(recs, log=lambda rec: self.log.write(rank=self.ctx.rank, **rec))

    def incoming_migrants(self, glob) -> dict:
        """Ring migration: global island g receives island g - 1's migrants.
        glob: [world, blob] -> {local island: [(code, score)]}."""
        W, I = glob.shape[0], len(self.islands)
        by_island = {}
        for r in range(W):
            for li, code, score in dist.unpack_migrants(glob[r]):
                by_island.setdefault(r * I + li, []).append((code, score))
        return {li: by_island.get((self.ctx.rank * I + li - 1) % (W * I), []) for li in range(I)}

    def apply_migrants(self, li: int, incoming) -> None:
        s = self.islands[li]
        known = {c for c, _ in s.population}
        for code, score in incoming:
            if code in known:
                continue
            if self.migrant_dedup:
                # replace only a worse member, never one the island already has in kind
                full = len(s.population) >= s.population_size
                if (full and score <= min(sc for _, sc in s.population)) or s._is_too_similar(code, score):
                    continue
            s.population.append((code, score))
            known.add(code)
            if score > s.best_score:
                s.best_score, s.best_policy = score, code
        s.population = sorted(s.population, key=lambda x: x[1], reverse=True)[:s.population_size]

    def reset_weak_islands(self) -> List[int]:
        """FunSearch island reset: the weakest `reset_fraction` of this rank's
        islands (by best score; ties: higher index first) are emptied and
        re-seeded with the best program of a random surviving island.  Returns
        the reset island indices (logged as an ``island_reset`` record)."""
        k = len(self.islands)
        n = int(k * self.reset_fraction)
        if k < 2 or n < 1:
            return []
        order = sorted(range(k), key=lambda i: (self.islands[i].best_score, -i))
        weak, keep = order[:n], order[n:]
        if self.reset_diverse:
            from .search import _similar_at_least
            thr = self.islands[0].similarity_threshold
            leads = [self.islands[j].best_policy.strip() for j in keep if self.islands[j].best_policy]
            pool = sorted({(c, sc) for j in keep for c, sc in self.islands[j].population}, key=lambda x: -x[1])
        for i in weak:
            s = self.islands[i]
            pick = None
            if self.reset_diverse:
                for c, sc in pool:
                    cs = c.strip()
                    if not any(_similar_at_least(cs, t, thr) for t in leads):
                        pick = (c, sc)
                        leads.append(cs)
                        break
            if pick is not None:
                s.population = [pick]
                s.best_policy, s.best_score = pick
                continue
            src = self.islands[self._reset_rng.choice(keep)]
            s.population = [(src.best_policy, src.best_score)] if src.best_policy else list(src.population[:1])
            s.best_policy, s.best_score = src.best_policy, src.best_score
        self.resets += 1
        self.log.write(kind="island_reset", rank=self.ctx.rank, generation=self.generation, reset=weak,
                       bests=[round(s.best_score, 6) for s in self.islands])
        return weak

    def absorb_migrants(self, glob) -> None:
        for li, inc in self.incoming_migrants(glob).items():
            self.apply_migrants(li, inc)

    def migrate(self) -> None:
        """Ring migration of each island's best programs across all ranks."""
        self.absorb_migrants(dist.all_gather_array(self.migrant_blob()))

    # -- pipelined generations ---------------------------------------
    def _plan(self, s: SimpleFunSearch):
        s.population.sort(key=lambda x: x[1], reverse=True)
        elites = s.population[:s.elite_size]
        n_new = max(0, min(s.policies_per_generation, s.population_size - len(elites)))
        return elites, n_new

    def _merge(self, s: SimpleFunSearch, elites, children: List[str], results) -> None:
        new = []
        for code, res in zip(children, results):
            if s._is_too_similar(code, res.score):
                continue
            new.append((code, res.score))
            if res.score > s.best_score:
                s.best_score, s.best_policy = res.score, code
        s.population = sorted(elites + new, key=lambda x: x[1], reverse=True)[:s.population_size]

    # -- family coupling (funsearch/coupling.py) -----------------------------------------------
    def run_coupling(self) -> List[dict]:
        """One coupler round: family search on the device, champion rendered as
        program text and re-scored exactly.  Safe to run in a worker thread
        (touches no island population)."""
        with roctx_range(f"funsearch.coupling round {self.coupler.rounds}"):
            return self.coupler.round()

    def inject_coupled(self, rec: dict, idle: Optional[List[int]] = None) -> Optional[int]:
        """Put a coupled family champion into the island with the lowest best
        score (among `idle`); returns the island index, or None if every
        candidate island already holds the program or would drop it."""
        cand = list(range(len(self.islands))) if idle is None else list(idle)
        if not cand:
            return None
        i = min(cand, key=lambda k: self.islands[k].best_score)
        s = self.islands[i]
        code, score = rec["code"], float(rec["score"])
        known = {c for c, _ in s.population}
        accepted = code not in known and (len(s.population) < s.population_size
                                          or score > min(sc for _, sc in s.population))
        if accepted:
            s.population = sorted(s.population + [(code, score)], key=lambda x: x[1],
                                  reverse=True)[:s.population_size]
            if score > s.best_score:
                s.best_score, s.best_policy = score, code
        self.evaluations += 1
        self.log.write(kind="coupling", rank=self.ctx.rank, island=i, generation=s.generation,
                       family=rec["family"], family_score=rec["family_score"], score=score,
                       accepted=accepted, coupler_rounds=self.coupler.rounds,
                       coupler_evaluated=self.coupler.evaluated, coupler_s=round(self.coupler.seconds, 3))
        if self.verbose and self.ctx.is_main:
            print(json.dumps(dict(kind="coupling", island=i, family=rec["family"], score=score,
                                  accepted=accepted)), flush=True)
        return i if accepted else None

    def polish_due(self, i: int) -> bool:
        s = self.islands[i]
        if not self.polish_every or s.generation % self.polish_every or not s.population:
            return False
        code, _ = max(s.population, key=lambda x: x[1])
        return self.polish_repeat or code not in self._polished

    def maybe_polish(self, i: int, log: bool = True) -> Optional[dict]:
        """Every ``polish.every`` generations: tune the numeric literals of island
        i's best program with one batched device search (thousands of constant
        settings, one JIT compile), re-score the rewritten text through the normal
        evaluation path, and put it into the population if it is better.  Runs
        on the island's own HIP slot (the pipelined loop calls it from a worker
        thread, so the other islands keep stepping meanwhile)."""
        if not self.polish_due(i):
            return None
        s = self.islands[i]
        code, score = max(s.population, key=lambda x: x[1])
        self._polished.add(code)
        from .polish import polish
        slot = i % max(1, self._n_slots())
        t0 = time.time()
        res = polish(lambda progs: self.evaluator.score_compiled(progs, slot), code, base_score=score,
                     variants=self.polish_variants, rounds=self.polish_rounds,
                     seed=hash((self.ctx.rank, i, s.generation)) & 0xFFFF)
        rec = dict(kind="polish", rank=self.ctx.rank, island=i, generation=s.generation, base=score,
                   polished=res.score, evaluated=res.evaluated, seconds=round(time.time() - t0, 3))
        if res.improved:
            exact = self.evaluator.evaluate_programs([res.code], slot=slot)[0]   # the rewritten TEXT, normal path
            rec["rescored"] = exact.score
            if exact.score > score and res.code not in {c for c, _ in s.population}:
                s.population = sorted(s.population + [(res.code, exact.score)], key=lambda x: x[1],
                                      reverse=True)[:s.population_size]
                if exact.score > s.best_score:
                    s.best_score, s.best_policy = exact.score, res.code
                self._polished.add(res.code)
        with self._count_lock:       # polish runs in a worker thread in pipelined mode
            self.evaluations += res.evaluated
        if log:
            self.log.write(**rec)
        return rec

    def run_pipelined(self, generations: int, threshold: float) -> None:
        """Every island runs its own generation loop -- LLM requests (thread
        pool), JIT compile + device launch on the island's own HIP stream,
        merge -- so one island's LLM round trips and compiles overlap the other
        islands' device replays instead of the whole rank waiting on each stage
        in turn.  Each island's generation g+1 still samples from its own
        generation-g population (per-island semantics of `evolve`); islands
        meet only at migration points and at the end.  The JSONL log gets one
        ``island_generation`` record per island step (llm_s / jit_s / eval_s
        wall intervals) and one ``generation`` record per completed global
        generation (with the device-busy fraction of the wall time)."""
        k = len(self.islands)
        stop = [False]
        target = self.generation + generations
        gen = [self.generation] * k
        phase = ["idle"] * k
        fut: List[object] = [None] * k
        plan: List[object] = [None] * k
        stamp = [dict() for _ in range(k)]
        done_children = {}
        workers = max(2, min(64, sum(s.max_workers for s in self.islands) + k))
        busy_since = [None]
        busy_total = [0.0]
        t_start = time.time()
        inflight = [False] * k
        global_rec = {}   # generation -> partial aggregate
        cpl = {"fut": None, "inbox": [], "last": self.generation}
        from .migration import MigrationChannel
        chan = MigrationChannel(self, self.migrate_every, self.generation)
        self._chan = chan
        inbox = [[] for _ in range(k)]     # migrants waiting for their island to be between generations
        vote = [False]                     # this rank wants to stop (threshold reached)

        def landed(results) -> bool:
            for res in results:
                for li, inc in res.incoming.items():
                    inbox[li].extend(inc)
                self.log.write(kind="migration", rank=self.ctx.rank, generation=res.generation,
                               bests=[round(x, 6) for x in res.bests], stop_votes=res.votes,
                               collective_wait_s=round(chan.wait_s, 4))
            return bool(results)

        def set_busy():
            now = time.time()
            any_on = any(inflight)
            if any_on and busy_since[0] is None:
                busy_since[0] = now
            elif not any_on and busy_since[0] is not None:
                busy_total[0] += now - busy_since[0]
                busy_since[0] = None

        def gen_children(i):
            s = self.islands[i]
            elites, n_new = plan[i]
            if not elites or n_new == 0:
                return []
            with concurrent.futures.ThreadPoolExecutor(max_workers=max(1, min(n_new, s.max_workers))) as ex:
                outs = list(ex.map(lambda j: s._generate_single_policy(j, elites, FEEDBACK), range(n_new)))
            return [code for _, code in outs if code]

        def launch(i, children):
            return self.evaluator.submit_programs(children, slot=i % max(1, self._n_slots()))

        with concurrent.futures.ThreadPoolExecutor(max_workers=workers) as pool:
            while True:
                progressed = False
                if chan.every:
                    # post a gather once the slowest island reaches a migration
                    # generation; nobody waits for it (lookahead-bounded)
                    with roctx_range("funsearch.migrate"):
                        if chan.post_due(min(gen) if not stop[0] else -1, vote[0]):
                            progressed = True
                        if landed(chan.poll(threshold)):
                            progressed = True
                    if chan.stopping:
                        stop[0] = True
                if self._ck_due and all(ph == "idle" for ph in phase) and cpl["fut"] is None:
                    # every island between generations, no polish / coupler thread touching a
                    # population: a consistent cut (the islands' own generation counters are saved)
                    self._ck_due = False
                    self.save_checkpoint()
                for i in range(k):
                    if inbox[i] and phase[i] == "idle":     # between generations: elites not captured
                        self.apply_migrants(i, inbox[i])
                        inbox[i] = []
                if self.coupler is not None:
                    # the family coupler runs on its own slot in a worker; its
                    # champions wait in an inbox until an island is idle
                    if cpl["fut"] is not None and cpl["fut"].done():
                        cpl["inbox"].extend(cpl["fut"].result())
                        cpl["fut"] = None
                        progressed = True
                    g_min = min(gen)
                    if (cpl["fut"] is None and g_min > cpl["last"] and self.coupler.due(g_min)
                            and g_min < target and not stop[0] and not self._ck_due):
                        cpl["last"] = g_min
                        cpl["fut"] = pool.submit(self.run_coupling)
                    idle = [j for j in range(k) if phase[j] == "idle"]
                    while cpl["inbox"] and idle:
                        self.inject_coupled(cpl["inbox"].pop(0), idle)
                        progressed = True
                for i in range(k):
                    s = self.islands[i]
                    if phase[i] == "idle":
                        if gen[i] >= target or stop[0] or self._ck_due:
                            # a due checkpoint holds idle islands back until every
                            # island is between generations (the consistent cut above)
                            continue
                        s.generation += 1
                        plan[i] = self._plan(s)
                        stamp[i] = {"t0": time.time()}
                        fut[i] = pool.submit(gen_children, i)
                        phase[i] = "llm"
                        progressed = True
                    elif phase[i] == "llm" and fut[i].done():
                        children = fut[i].result()
                        stamp[i]["t_llm"] = time.time()
                        done_children[i] = children
                        fut[i] = pool.submit(launch, i, children)
                        phase[i] = "launch"
                        progressed = True
                    elif phase[i] == "launch" and fut[i].done():
                        fut[i] = fut[i].result()        # PendingPrograms
                        stamp[i]["t_launch"] = time.time()
                        inflight[i] = bool(fut[i].native_idx)
                        set_busy()
                        phase[i] = "eval"
                        progressed = True
                    elif phase[i] == "eval" and self.evaluator.ready(fut[i]):
                        pend = fut[i]
                        results = self.evaluator.collect(pend)
                        inflight[i] = False
                        set_busy()
                        t_end = time.time()
                        children = done_children.pop(i)
                        self._merge(s, plan[i][0], children, results)
                        with self._count_lock:
                            self.evaluations += len(children)
                        gen[i] += 1
                        st = stamp[i]
                        rec = dict(kind="island_generation", rank=self.ctx.rank, island=i, generation=gen[i],
                                   children=len(children), best=round(s.best_score, 6),
                                   llm_s=round(st["t_llm"] - st["t0"], 4), jit_s=round(pend.jit_s, 4),
                                   eval_s=round(t_end - st["t_launch"], 4), wall_s=round(t_end - st["t0"], 4),
                                   new_shapes=pend.new_shapes, t0=round(st["t0"] - t_start, 4),
                                   t_end=round(t_end - t_start, 4))
                        self.log.write(**rec)
                        agg = global_rec.setdefault(gen[i], {"children": 0, "islands": 0, "llm_s": 0.0, "jit_s": 0.0,
                                                             "eval_s": 0.0, "t0": st["t0"]})
                        agg["children"] += len(children)
                        agg["islands"] += 1
                        agg["llm_s"] += rec["llm_s"]
                        agg["jit_s"] += rec["jit_s"]
                        agg["eval_s"] += rec["eval_s"]
                        agg["t0"] = min(agg["t0"], st["t0"])
                        if agg["islands"] == k:
                            self._finish_generation(gen[i], global_rec.pop(gen[i]), busy_total, busy_since,
                                                    t_start, threshold, stop, chan, vote)
                        if self.polish_due(i):
                            # constant polish on the island's slot, in a worker: the
                            # other islands keep stepping; this island resumes after it
                            fut[i] = pool.submit(self.maybe_polish, i, False)
                            inflight[i] = True
                            set_busy()
                            phase[i] = "polish"
                        else:
                            phase[i] = "idle"
                        progressed = True
                    elif phase[i] == "polish" and fut[i].done():
                        rec = fut[i].result()
                        if rec:
                            self.log.write(**rec)
                        inflight[i] = False
                        set_busy()
                        phase[i] = "idle"
                        progressed = True
                if (all(phase[i] == "idle" and (gen[i] >= target or stop[0]) for i in range(k))
                        and cpl["fut"] is None and not cpl["inbox"]):
                    due = chan.every and chan.next is not None and (
                        chan.next <= chan.stop_at if chan.stopping else (chan.next <= min(gen) and not stop[0]))
                    if not due:
                        if not chan.pending:
                            for i in range(k):
                                if inbox[i]:
                                    self.apply_migrants(i, inbox[i])
                                    inbox[i] = []
                            break
                        landed(chan.poll(threshold, block=True))
                        continue
                if not progressed:
                    time.sleep(0.0005)

    def _n_slots(self) -> int:
        dev = getattr(self.evaluator, "device", None)
        return dev.n_slots if dev is not None else max(1, len(self.islands))

    def _finish_generation(self, g: int, agg: dict, busy_total, busy_since, t_start: float, threshold: float,
                           stop, chan, vote) -> None:
        self.generation = g
        best_local = self.best[1]
        # the global best is known from the last finished migration gather (no all-reduce here)
        best_global = max(best_local, chan.best_global)
        now = time.time()
        busy = busy_total[0] + (now - busy_since[0] if busy_since[0] is not None else 0.0)
        wall = now - agg["t0"]
        rec = dict(kind="generation", rank=self.ctx.rank, generation=g, best=best_local, best_global=best_global,
                   children=agg["children"], islands=[round(s.best_score, 6) for s in self.islands],
                   llm_s=round(agg["llm_s"], 4), jit_s=round(agg["jit_s"], 4), eval_s=round(agg["eval_s"], 4),
                   wall_s=round(wall, 4), pipelined=True, collective_wait_s=round(chan.wait_s, 4),
                   collective_wait_frac=round(chan.wait_s / max(1e-9, now - t_start), 5),
                   device_busy=round(busy / max(1e-9, now - t_start), 4),
                   evals_per_s=round(self.evaluations / max(1e-9, now - t_start), 2),
                   engines={k: v for k, v in self.evaluator.stats.items() if k in
                            ("device_native", "device", "cpu_vm", "object", "compile_errors", "jit_shapes")})
        self.log.write(**rec)
        if self.verbose and self.ctx.is_main:
            print(json.dumps(rec), flush=True)
        if self.ck_dir and self.ck_every and g % self.ck_every == 0:
            self._ck_due = True      # written when every island is idle (a consistent cut)
        if best_local >= threshold:
            vote[0] = True
            if not chan.active:
                stop[0] = True       # alone: nobody to agree with

    def run(self, generations: Optional[int] = None, resume: bool = False) -> Tuple[Optional[str], float]:
        if resume and self.ck_dir:
            self.load_elastic(self.ck_dir)
        self.initialize()
        generations = generations or self.islands[0].max_generations
        threshold = self._threshold
        start = self.generation
        if self.mode == "steady":
            from .steady import SteadyStateSearch
            sc = self.steady_cfg
            self.steady = SteadyStateSearch(self, batch=int(sc.get("batch", 256)), slots=sc.get("slots"),
                                            producers=int(sc.get("producers", 0)),
                                            task_size=int(sc.get("task_size", 8)),
                                            status_every_s=float(sc.get("status_every_s", 5.0)),
                                            tierup=bool(sc.get("tierup", False)),
                                            ahead=int(sc.get("ahead", 2)),
                                            stagers=int(sc.get("stagers", 1)),
                                            host_object=bool(sc.get("host_object", False)),
                                            service=sc.get("service"))
            self.steady.run(generations, threshold, wall_s=float(sc.get("wall_s", 0.0)))
            return self.global_best()
        if self.pipeline:
            self.run_pipelined(generations, threshold)
            if self._ck_due:
                self._ck_due = False
                self.save_checkpoint()
            return self.global_best()
        while self.generation - start < generations:
            rec = self.evolve()
            if self.verbose and self.ctx.is_main:
                print(json.dumps(rec), flush=True)
            if rec["stop"]:
                break
        return self.global_best()

    def global_best(self) -> Tuple[Optional[str], float]:
        """(code, score) of the best program on any rank.  Programs of any
        length travel (`dist.all_gather_bytes`, as the reference saves any
        program, funsearch_integration.py:599-679); ties go to the lowest rank,
        so every rank returns the same program."""
        code, score = self.best
        if not self.ctx.distributed:
            return code, score
        mine = json.dumps({"code": code, "score": float(score)}).encode("utf-8")
        allb = self._collective("global_best", lambda: dist.all_gather_bytes(mine), [mine])
        recs = [json.loads(b.decode("utf-8")) for b in allb]
        best = max(recs, key=lambda r: r["score"])      # first (lowest rank) of equal scores
        return best["code"], float(best["score"])

    # -- checkpoint ----------------------------------------------------------------------
    def save_checkpoint(self) -> str:
        os.makedirs(self.ck_dir, exist_ok=True)
        path = os.path.join(self.ck_dir, f"islands_rank{self.ctx.rank}.json")
        state = {"format": "fks-islands-checkpoint-v1", "generation": self.generation,
                 "rank": self.ctx.rank, "world_size": self.ctx.world_size,
                 "evaluations": self.evaluations, "islands": [s.state_dict() for s in self.islands]}
        if self.coupler is not None:
            state["coupling"] = self.coupler.state_dict()
        tmp = path + ".tmp"
        with open(tmp, "w") as fh:
            json.dump(state, fh)
        os.replace(tmp, path)
        return path

    def load_checkpoint(self, path: str) -> None:
        with open(path) as fh:
            st = json.load(fh)
        if st.get("format") != "fks-islands-checkpoint-v1":
            raise ValueError(f"not an island checkpoint: {path}")
        self.generation = int(st["generation"])
        self.evaluations = int(st.get("evaluations", 0))
        for s, ss in zip(self.islands, st["islands"]):
            s.generation = int(ss["generation"])
            s.population = [(p["code"], float(p["score"])) for p in ss["population"]]
            s.best_policy, s.best_score = ss["best_policy"], float(ss["best_score"])
        if self.coupler is not None and st.get("coupling"):
            self.coupler.load_state_dict(st["coupling"])

    def load_elastic(self, ck_dir: str) -> bool:
        """Resume from the newest complete checkpoint set in `ck_dir`, whatever
        world size and islands-per-rank wrote it.  Saved islands are numbered
        globally (rank-major); with T islands now, saved island j goes to global
        island j % T (populations merged: union, best first, truncated), and
        when fewer were saved than exist now, island g clones saved island
        g % J.  Returns False when there is nothing to resume."""
        sets = {}
        for path in glob.glob(os.path.join(ck_dir, "islands_rank*.json")):
            try:
                with open(path) as fh:
                    st = json.load(fh)
            except (OSError, ValueError):
                continue
            if st.get("format") != "fks-islands-checkpoint-v1":
                continue
            rank = int(st.get("rank", os.path.basename(path)[len("islands_rank"):-len(".json")]))
            key = (int(st["generation"]), int(st.get("world_size", 1)))
            sets.setdefault(key, {})[rank] = st
        if not sets:
            return False
        complete = [k for k, v in sets.items() if len(v) >= k[1]]
        gen, ws = max(complete or sets)
        saved = sets[(gen, ws)]
        own = saved.get(self.ctx.rank)
        cst = (own or saved[min(saved)]).get("coupling")
        if self.coupler is not None and cst:
            self.coupler.load_state_dict(cst)
        if ws == self.ctx.world_size and own is not None and len(own["islands"]) == len(self.islands):
            self.generation = gen
            self.evaluations = int(own.get("evaluations", 0))
            for s, ss in zip(self.islands, own["islands"]):
                self._load_island(s, [ss])
            return True
        flat = [ss for r in sorted(saved) for ss in saved[r]["islands"]]
        T, I = self.ctx.world_size * len(self.islands), len(self.islands)
        self.generation = gen
        self.evaluations = sum(int(st.get("evaluations", 0)) for r, st in saved.items()
                               if r % self.ctx.world_size == self.ctx.rank)
        for li, s in enumerate(self.islands):
            g = self.ctx.rank * I + li
            src = flat[g::T] if len(flat) >= T else [flat[g % len(flat)]]
            self._load_island(s, src)
        return True

    @staticmethod
    def _load_island(s: SimpleFunSearch, states: List[dict]) -> None:
        pop, seen = [], set()
        for ss in states:
            for p in ss["population"]:
                if p["code"] not in seen:
                    seen.add(p["code"])
                    pop.append((p["code"], float(p["score"])))
        pop.sort(key=lambda x: x[1], reverse=True)
        s.population = pop[:s.population_size]
        s.generation = max(int(ss["generation"]) for ss in states)
        best = max(states, key=lambda ss: float(ss["best_score"]))
        s.best_policy, s.best_score = best["best_policy"], float(best["best_score"])


def run_funsearch(config="configs/offline_islands.json", generations: Optional[int] = None, resume: bool = False,
                  evaluator: Optional[Evaluator] = None, verbose: bool = False) -> Tuple[Optional[str], float]:
    """Run the (multi-island, multi-GPU) FunSearch loop; returns (best_code, best_score)."""
    return IslandFunSearch(config, evaluator=evaluator, verbose=verbose).run(generations, resume)
