"""Asynchronous steady-state island search: keep the MI355X full of programs.

The reference evolves one population in lockstep generations of
``min(8, population_size - elites)`` children (`funsearch/funsearch_integration.py:
487-572`): every generation waits for its LLM calls, then for its slowest
replay.  The generation-synchronous island modes here keep that contract
(`islands.py`); this mode drops the lockstep to keep hundreds of programs in
flight on one GPU:

* **producers** -- a process pool (spawn: no HIP state) turns tasks (island,
  current elites, n) into children: LLM (or offline mutation) call, template
  fill, sandbox validation and bytecode compile, all off the main process;
  parents are sampled from each island's population *at submission time*;
* **dispatcher** -- the main thread packs ready children into batches of up to
  ``batch`` programs; a stager thread JIT-compiles their new shapes with the
  baseline tier (`ops/gcnjit.py`, ~0.2 ms per program) and loads the modules
  up to ``ahead`` batches before a slot frees, and the main thread launches a
  staged batch the moment a HIP slot is free (up to ``slots`` in flight);
* **merge** -- results land per batch and merge into their island one by one
  with the reference's rules (dedup by difflib ratio against equal-or-better
  members, keep the top ``population_size``): a steady-state GA instead of
  generational replacement.  An island's *generation* is its merged-children
  count divided by ``policies_per_generation``;
* **migration without lockstep** -- when the slowest island passes a multiple
  of ``migrate_every`` generations the rank *starts* an asynchronous
  all-gather of its migrant blob (`dist.pack_migrants`: variable-length,
  compressed, carrying each rank's best score -- so early stop needs no extra
  all-reduce) and keeps evaluating; the incoming migrants merge when the
  gather completes.  Ranks meet only inside collectives they have all posted,
  never at a per-generation barrier;
* **checkpoints** are written at migration points from the main thread, the
  only thread that touches populations (a consistent cut).

JSONL records: ``steady_batch`` (per batch: programs, new shapes, JIT and
device seconds, programs in flight) and ``steady_status`` (every few seconds:
evals/s, device busy fraction, new-shape fraction, best per island).
"""

from __future__ import annotations

import collections
import concurrent.futures
import multiprocessing
import os
import random
import time
from dataclasses import dataclass, field
from typing import List, Optional, Tuple

import numpy as np

from ..parallel import dist
from ..utils.trace import roctx_range
from .search import FEEDBACK

from ..policy.bytecode import Exc as _Exc

_EXC_EVENTS = int(_Exc.EVENTS)

#: device cost of a child scored on the host engines (the JIT declined it):
#: the selection treats it as the costliest kind of program
HOST_COST = -1.0
_POLISH_SIGMAS = (0.6, 0.35, 0.15, 0.06, 0.02)   # constant-polish step sizes (log-normal sigma)

# ---------------------------------------------------------------------------- producer processes
_W: dict = {}


def _producer_init(llm_cfg: dict, timeout_s: int, seed: int, fanout: int = 0) -> None:
    from ..policy.sandbox import SafeExecutor
    from .generator import LLMCodeGenerator
    from .llm import make_client
    cfg = dict(llm_cfg)
    cfg["seed"] = int(cfg.get("seed", 0)) * 7919 + seed + os.getpid()
    client = make_client(cfg)
    _W["gen"] = LLMCodeGenerator(client, SafeExecutor(timeout_seconds=timeout_s), cfg.get("model"),
                                 cfg.get("max_tokens", 400), cfg.get("temperature", 0.7))
    _W["rng"] = random.Random(cfg["seed"])
    if fanout > 1:
        # a remote LLM: a task's requests wait concurrently (threads; the wait
        # releases the GIL), so `producers x task_size` requests are in flight
        _W["fanout"] = concurrent.futures.ThreadPoolExecutor(max_workers=fanout, thread_name_prefix="fks-llm")
        _W["fanout_n"] = fanout


def _produce(task):
    """(island, elites [(code, score)], n[, weights]) -> ([(island, code, CompiledPolicy | None)], cpu s, wall s,
    gap s).
    weights: per-elite parent weights (the steady search's device-cost
    weighting, `_parent_weights`), or None for uniform sampling.

    With a request fan-out (a remote LLM, `_producer_init` fanout > 1) a task
    does not wait for its own requests: it starts its n requests on the
    process's threads once at most `fanout - n` are still in flight, and
    returns the children whose requests have completed by then -- so every
    producer keeps ~fanout requests waiting at all times instead of idling on
    the slowest of each task's n (16 requests of 2-8 s: a task would last the
    maximum, ~7.6 s, not the mean).  n = 0 flushes: waits for every request in
    flight and returns their children (the end of a run)."""
    island, elites, n = task[:3]
    weights = task[3] if len(task) > 3 else None
    t0 = time.process_time()
    w0 = time.perf_counter()
    # the producer's gap since its previous task ended: its last result's
    # trip to the dispatcher plus this task's trip to the process (idle time
    # the pool's hand-offs cost; reported with the task)
    last = _W.get("t_end")
    gap = w0 - last if last is not None else 0.0
    pool = _W.get("fanout")
    if pool is not None:
        pend = _W.setdefault("pending", [])
        cap = _W["fanout_n"]
        out = []

        def harvest():
            done = [f for f in pend if f.done()]
            if done:
                pend[:] = [f for f in pend if not f.done()]
                out.extend(f.result() for f in done)

        if n <= 0:
            concurrent.futures.wait(pend)
        while len(pend) + n > cap:
            concurrent.futures.wait(pend, return_when=concurrent.futures.FIRST_COMPLETED)
            harvest()
        harvest()
        pend.extend(pool.submit(_produce_one, island, elites, weights) for _ in range(max(0, n)))
    else:
        out = [_produce_one(island, elites, weights) for _ in range(n)]
    for _, code, prog in out:
        # the program's source is the child's text: sent once (results travel
        # through one pipe read by the pool's result thread in the GIL-bound
        # dispatcher; the duplicate text was ~half of the ~6.6 KB per child)
        if prog is not None and prog.source == code:
            prog.source = None
    _W["t_end"] = time.perf_counter()
    return out, time.process_time() - t0, _W["t_end"] - w0, gap


def _produce_one(island, elites, weights):
    from ..ops.jit import launch_key
    from ..policy.compiler import same_shape_child, try_compile
    gen, rng = _W["gen"], _W["rng"]
    pcache = _W.setdefault("parents", {})   # parent text -> CompiledPolicy (elites repeat)
    parents = _sample_parents(rng, elites, weights)
    reuse = []

    def same_shape(child, parents=parents, reuse=reuse):
        # a constant-only mutation keeps its parent's shape: bytecode reused,
        # and -- the parent having passed validation, only digits differing --
        # the sandbox checks need not run again
        for pc, _ in parents:
            pp = pcache.get(pc)
            if pp is None:
                if len(pcache) > 256:
                    pcache.clear()
                try:   # the parent itself passes the sandbox checks (once per parent text)
                    gen.safe_executor.validate(pc)
                    pp = try_compile(pc)[0] or False
                except Exception:
                    pp = False
                pcache[pc] = pp
            if pp:
                prog = same_shape_child(pp, child)
                if prog is not None:
                    reuse.append(prog)
                    return True
        return False

    code = gen.generate_policy(parent_policies=parents, performance_feedback=FEEDBACK, prevalidated=same_shape)
    if not code:             # LLM / validation failure: the child slot is spent
        return island, None, None
    if reuse:
        prog = reuse[0]
        _W["reused"] = _W.get("reused", 0) + 1
    else:
        prog, _ = try_compile(code)
    if prog is not None:
        # the JIT cache key and constant payload travel with the child: the
        # dispatcher process's stagers only look them up
        launch_key(prog)
    return island, code, prog


def _sample_parents(rng, elites, weights, k: int = 2):
    """k distinct parents: uniform (the reference's `random.sample`) or by weight."""
    if not weights or len(elites) <= k:
        return rng.sample(elites, min(k, len(elites)))
    idx = list(range(len(elites)))
    w = list(weights)
    out = []
    for _ in range(k):
        j = rng.choices(range(len(idx)), weights=w)[0]
        out.append(elites[idx.pop(j)])
        w.pop(j)
    return out


@dataclass
class _Polish:
    """A constant-polish batch: literal settings of one island champion (one
    shape: one JIT compile, then data only; funsearch/polish.py)."""
    island: int
    code: str
    prog: object                   # the champion's CompiledPolicy
    base: float
    cands: list                    # {constant-pool index: value} per variant
    progs: Optional[list] = None   # the variants' CompiledPolicy (until staged)


@dataclass
class _Batch:
    slot: int
    items: list                    # [(island, code, prog)]
    pend: object
    t_launch: float
    new_shapes: int = 0
    jit_s: float = 0.0
    polish: Optional[_Polish] = None
    results: Optional[list] = None   # streaming (program service): results so far
    left: int = 0                    # programs not merged yet
    aborted: bool = False            # in flight at a grid rollover's abort: no host fallbacks


class _Slots:
    """Batch slots (a list of `_Batch` or None) that keeps its occupied indices:
    the program service runs with ~1,000 slots (a straggler holds its batch's
    slot until its last program is merged), and the dispatcher loop visits
    only the occupied ones."""

    def __init__(self, n: int):
        self._b: List[Optional[_Batch]] = [None] * n
        self._free = collections.deque(range(n))
        self._active: dict = {}          # slot -> batch (insertion order: launch order)

    def __len__(self) -> int:
        return len(self._b)

    def __getitem__(self, si: int) -> Optional["_Batch"]:
        return self._b[si]

    def __setitem__(self, si: int, b: Optional["_Batch"]) -> None:
        old = self._b[si]
        self._b[si] = b
        if b is None and old is not None:
            del self._active[si]
            self._free.append(si)
        elif b is not None and old is None:
            self._active[si] = b
            self._free.remove(si) if self._free and self._free[0] != si else self._free.popleft()
        elif b is not None:
            self._active[si] = b

    def live(self) -> list:
        return list(self._active.values())

    def active_ids(self) -> list:
        return list(self._active)

    def empty(self) -> bool:
        return not self._active

    def has_free(self) -> bool:
        return bool(self._free)

    def next_free(self) -> Optional[int]:
        return self._free[0] if self._free else None


@dataclass
class SteadyStats:
    evaluations: int = 0
    batches: int = 0
    new_shapes: int = 0
    native: int = 0
    jit_s: float = 0.0
    busy_s: float = 0.0
    produced: int = 0
    rejected: int = 0
    migrations: int = 0
    fallback: int = 0                # programs scored by the host engines (async)
    shed: int = 0                    # children only CPython could score, not evaluated (host_object off)
    abandoned: int = 0               # host fallbacks still queued when the run stopped
    producer_cpu_s: float = 0.0
    task_turnaround_s: float = 0.0   # producer tasks: submit -> result collected (wall), summed
    task_n: int = 0
    producer_gap_s: float = 0.0      # producers idle between tasks (result out + next task in), summed
    producer_wall_s: float = 0.0     # wall seconds the producers spent on tasks (CPU / wall: their core share)
    polish_batches: int = 0          # constant-polish batches (variants of an island champion)
    polish_evals: int = 0            # their device evaluations (not children)
    polish_improved: int = 0         # polished champions re-entered as children
    polish_idle: int = 0             # of the polish batches: run on a slot that would have idled
    coupled: int = 0                 # family-coupler champions offered to the islands
    inflight_sum: float = 0.0        # programs in flight x seconds
    inflight_n: float = 0.0          # seconds observed
    cost_rejected: int = 0           # children not merged by the bloat control (device cost)
    event_capped: int = 0            # children whose replay passed the event budget (not scored)
    cost_sum: float = 0.0            # device cycles of the children replayed on the service ...
    cost_n: int = 0                  # ... and their number
    rollovers: int = 0               # grid rollovers (module unloads while the service runs)
    rollover_s: float = 0.0          # wall seconds the rollovers took (drain + restart)
    history: List[dict] = field(default_factory=list)


class SteadyStateSearch:
    """Steady-state driver over an `IslandFunSearch` (its islands, evaluator,
    distributed context, log and checkpoint settings)."""

    def __init__(self, fs, batch: int = 256, slots: Optional[int] = None, producers: int = 0,
                 task_size: int = 8, status_every_s: float = 5.0, tierup: bool = False, ahead: int = 2,
                 host_object: bool = False, service=None, stagers: int = 1):
        self.fs = fs
        #: children only CPython can score (bigint / complex intermediates, ~1% of
        #: mutated programs, ~3 s each on one core) go to the object engine only
        #: when True; else they are shed (counted, never merged) -- the search
        #: loses ~1% of its children instead of its host cores
        self.host_object = bool(host_object)
        self.batch = int(batch)
        #: batches compiled and loaded ahead of a free slot (the stager thread)
        self.ahead = max(1, int(ahead))
        #: stager threads: a batch's module load overlaps the next batch's code
        #: generation (NativeCompiler.prepare is thread-safe); batches still
        #: launch in staging order
        self.stagers = max(1, int(stagers))
        #: constant polish of island champions as device batches (the islands'
        #: ``polish`` config: every / variants; 0 = off)
        self.polish_every = int(getattr(fs, "polish_every", 0) or 0)
        self.polish_variants = int(getattr(fs, "polish_variants", 512) or 512)
        self.polish_idle = bool(getattr(fs, "polish_idle", False)) and self.polish_every > 0
        self._idle_rr = -1
        self._polish_count: dict = {}
        dev = getattr(fs.evaluator, "device", None)
        if dev is not None and not tierup:
            # background LLVM recompiles of hot shapes compete with the producer
            # processes for the host's cores and with the batches' module loads;
            # at steady state almost every shape is evaluated once or twice
            dev.native_compiler.tierup_after = 0
        # host fallbacks run at low priority: the producers come first
        fs.evaluator.fallback_nice = 15
        n_slots = dev.n_slots if dev is not None else 1
        if getattr(fs, "coupler", None) is not None:
            n_slots = max(1, n_slots - 1)   # the last slot is the family coupler's
        self.slots = max(1, min(int(slots or n_slots), n_slots))
        #: resident program service (ops/hip_engine.py start_service): batches are
        #: queued to one persistent grid instead of launched per slot, so the
        #: number of batches in flight is no longer the engine's stream count
        svc = service if isinstance(service, dict) else ({} if service else None)
        self.service_cfg = None
        self.slot_base = 0
        #: host collectives: with the grid resident RCCL collectives cannot
        #: progress (tools/grid_coexist_probe.py), so a service configuration
        #: sends the migrations' small host arrays over the gloo group opened
        #: beside RCCL -- decided from the configuration, the same on every rank
        self.host_collectives = dist.use_host_collectives(svc is not None)
        if svc is not None and dev is not None and hasattr(dev, "start_service"):
            self.service_cfg = dict(svc)
            # batches in flight at once (a batch holds its entry until its
            # slowest program is done; results stream out before that) and the
            # programs kept queued on the grid (`inflight`, default 1.5 x its
            # resident workgroups, set when the service starts)
            self.slots = max(1, int(svc.get("slots", slots or 1024)))
            self.slot_base = dev.SERVICE_SLOT_BASE
        self.service_inflight = 0
        #: producer tasks kept submitted per producer process (FKS_TASKS_PER_PRODUCER;
        #: the pool hands a finished producer its next task from this backlog)
        self.tasks_per_producer = max(1, int(os.environ.get("FKS_TASKS_PER_PRODUCER", "2")))
        #: device-cost selection (service runs: every child's replay cycles are
        #: measured on the grid): parents are sampled with weight median / cost
        #: (clipped to [1/4, 4]) among an island's elites, and a child costing more
        #: than `bloat` x the island's median member is not merged unless it
        #: beats the island's best.  Scores are never touched.
        cc = dict((svc or {}).get("cost") or {}) if isinstance(svc, dict) else {}
        self.cost_parents = bool(cc.get("parents", True))
        self.cost_bloat = float(cc.get("bloat", 3.0))
        #: and an absolute anchor: the median cost of the run's first
        #: `anchor_children` replays; a child costing more than `anchor_cap` x it
        #: enters only as a new island best (the population median alone drifts
        #: with the population: every step within `bloat` x, the run 2-3x
        #: costlier after a few minutes)
        self.cost_anchor_cap = float(cc.get("anchor_cap", 3.0))
        self.cost_anchor_children = int(cc.get("anchor_children", 4096))
        self._anchor_samples: list = []
        self.cost_anchor = 0.0
        #: grid rollover: retired JIT modules stay loaded while the grid runs
        #: (an unload waits for the device); past this many the loop drains the
        #: grid (launches paused, stragglers aborted after `rollover_grace_s`),
        #: unloads them and starts it again
        self.rollover_deferred = int((svc or {}).get("rollover_modules", 2048)) if isinstance(svc, dict) else 2048
        self.rollover_grace_s = float((svc or {}).get("rollover_grace_s", 3.0)) if isinstance(svc, dict) else 3.0
        #: replay event budget on the device (a resource limit, like the
        #: reference's per-call timeout but per replay): a child whose replay passes
        #: it is not scored.  A normal replay of the OpenB trace is 20-45k events;
        #: some evolved policies re-queue failed placements for 15M events -- tens
        #: of seconds of a workgroup each, and they exploit the evaluator's
        #: event-count snapshot schedule (docs/ARCHITECTURE.md).  0: no budget
        self.max_events = int((svc or {}).get("max_events", 400_000)) if isinstance(svc, dict) else 0
        #: programs waiting for (or in) a host-engine fallback at most; more are shed
        self.fallback_cap = int((svc or {}).get("fallback_cap", 64)) if isinstance(svc, dict) else 1 << 30
        self._cost: dict = {}            # island -> {code: device cycles}
        if dev is not None:
            # the two-wave kernel sizes its LDS heap top so that every slot's batch
            # stays resident at once (csrc/hip/engine_host.hip.h duo_top)
            dev.set_options(native_inflight=min(self.batch * self.slots, 1 << 14))
            if self.service_cfg is not None:
                dev.set_options(max_events=self.max_events)
            if not tierup:
                # shapes the baseline generator declines (~0.1%) go to the host
                # engines asynchronously instead of a ~0.2 s LLVM compile on the
                # dispatcher thread
                dev.native_compiler.tier = "baseline"
        from ..ops.cpu_engine import default_threads
        local = max(1, int(os.environ.get("LOCAL_WORLD_SIZE", "1")))
        self.producers = int(producers or max(1, min(16, default_threads() // local - 1)))
        self.task_size = int(task_size)
        self.status_every_s = float(status_every_s)
        self.stats = SteadyStats()
        self.llm_concurrency = 0
        self._pending_merges: collections.deque = collections.deque()   # deferred similarity scans
        self._asked = 0                  # children requested from the producers ...
        self._got = 0                    # ... and returned (fan-out tasks return what is ready)
        self._sim_pool = None
        # main-thread wall time by phase (the dispatcher is one thread: its busy
        # fraction bounds the steady-state rate)
        self.phase = {"receive": 0.0, "submit": 0.0, "collect": 0.0, "merge": 0.0}

    # -- helpers ------------------------------------------------------------------------
    def _elites(self, s):
        s.population.sort(key=lambda x: x[1], reverse=True)
        return list(s.population[:s.elite_size])

    def _parent_weights(self, i: int, elites) -> Optional[list]:
        """Parent weights of island i's elites: median cost / cost, in [1/4, 4]
        (unknown cost: 1) -- cheaper parents breed more, so the population does
        not drift toward ever costlier programs (a costlier parent still breeds)."""
        if not self.cost_parents or self.service_cfg is None:
            return None
        cmap = self._cost.get(i) or {}
        costs = [cmap.get(c) for c, _ in elites]
        known = sorted(x for x in costs if x and x > 0)
        if not any(x is not None and x < 0 for x in costs) and len(known) < 2:
            return None
        med = known[len(known) // 2] if known else 1.0
        # a host-scored elite (HOST_COST: its same-shape children replay on the
        # CPU VM, seconds of a core each) breeds least
        return [1.0 if not x else 0.25 if x < 0 else min(4.0, max(0.25, med / x)) for x in costs]

    def _merge_one(self, s, code: str, score: float, cost: float = 0.0, island: Optional[int] = None,
                   defer: bool = False) -> bool:
        """Merge one scored child into island `s` (the reference's rules: dedup by
        difflib ratio against equal-or-better members, keep the top
        population_size).  defer: the similarity scan (milliseconds of C++ per
        evolved child, the dispatcher's largest cost) runs on a worker thread
        against a snapshot of the population and the child is appended when it
        returns (`_finish_merges`), after a scan of the members added since;
        returns True when the child was appended now."""
        if len(s.population) >= s.population_size and score <= min(sc for _, sc in s.population):
            # truncation would drop it anyway (a tie sorts after the members it
            # ties with): skip the similarity scan, same resulting population
            return False
        cmap = self._cost.setdefault(island, {}) if island is not None else None
        if cost != 0 and cmap is not None and self.cost_bloat > 0 and score <= s.best_score:
            if cost < 0:
                # scored on the host (the device JIT declined it): enters only as a
                # new island best -- its constant-only children would all replay
                # on the CPU VM
                self.stats.cost_rejected += 1
                return False
            known = sorted(cmap[c] for c, _ in s.population if cmap.get(c, 0) > 0)
            if len(known) >= 3 and cost > self.cost_bloat * known[len(known) // 2]:
                self.stats.cost_rejected += 1
                return False
            if self.cost_anchor and self.cost_anchor_cap > 0 and cost > self.cost_anchor_cap * self.cost_anchor:
                self.stats.cost_rejected += 1
                return False
        if defer:
            others = [c.strip() for c, sc in s.population if sc >= score]
            if others:
                from .search import _similar_to_any
                fut = self._simpool().submit(_similar_to_any, code.strip(), others, s.similarity_threshold,
                                             s.similarity_threads if len(others) > 2 else 1)
                self._pending_merges.append((fut, s, code, score, cost, island, getattr(s, "_pop_version", 0)))
                return False
        elif s._is_too_similar(code, score):
            return False
        self._append(s, code, score, cost, cmap)
        return True

    def _append(self, s, code: str, score: float, cost: float, cmap) -> None:
        if cost != 0 and cmap is not None:
            cmap[code] = cost
            if len(cmap) > 4 * s.population_size:   # forget programs that left the population
                live = {c for c, _ in s.population}
                live.add(code)
                for c in [c for c in cmap if c not in live]:
                    del cmap[c]
        s.population.append((code, score))
        # (population version + recent appends: a deferred merge scans the members
        # added after its snapshot)
        s._pop_version = getattr(s, "_pop_version", 0) + 1
        added = s.__dict__.setdefault("_added", collections.deque(maxlen=256))
        added.append((s._pop_version, code, score))
        if score > s.best_score:
            s.best_score, s.best_policy = score, code
        s.population.sort(key=lambda x: x[1], reverse=True)
        del s.population[s.population_size:]

    def _simpool(self):
        if self._sim_pool is None:
            self._sim_pool = concurrent.futures.ThreadPoolExecutor(max_workers=2, thread_name_prefix="fks-similar")
        return self._sim_pool

    def _finish_merges(self, block: bool = False) -> bool:
        """Deferred merges whose similarity scan finished (in submission order):
        drop the child when the scan found a similar member; else scan the
        members added since the snapshot (usually none), re-check the
        truncation rule and append."""
        done = False
        pend = self._pending_merges
        while pend and (block or pend[0][0].done()):
            fut, s, code, score, cost, island, ver = pend.popleft()
            done = True
            if fut.result() >= 0:
                continue
            if len(s.population) >= s.population_size and score <= min(sc for _, sc in s.population):
                continue
            if getattr(s, "_pop_version", 0) != ver:
                from .search import _similar_to_any
                live = {c for c, _ in s.population}
                newer = [c.strip() for v, c, sc in s.__dict__.get("_added", ()) if v > ver and sc >= score and c in live]
                if newer and _similar_to_any(code.strip(), newer, s.similarity_threshold, 1) >= 0:
                    continue
            self._append(s, code, score, cost, self._cost.setdefault(island, {}) if island is not None else None)
        return done

    def _absorb(self, results) -> bool:
        """Merge finished migrations into the islands (main thread only)."""
        fs = self.fs
        for res in results:
            for li, inc in res.incoming.items():
                fs.apply_migrants(li, inc)
            self.stats.migrations += 1
            fs.log.write(kind="steady_migration", rank=fs.ctx.rank, generation=res.generation,
                         best_global=self.channel.best_global, bests=[round(x, 6) for x in res.bests],
                         stop_votes=res.votes, collective_wait_s=round(self.channel.wait_s, 4),
                         gather_s=round(self.channel.last_gather_s, 4), max_stall_s=round(self.channel.max_stall_s, 4))
            if fs.ck_dir:
                fs.save_checkpoint()
        return bool(results)

    def _polish_job(self, merged, start_gen, polish_next, idle: bool = False) -> Optional[_Polish]:
        """The next due constant polish (round robin over the islands): variants
        of the island champion's literals, one (1 + lambda) round per polish with
        the step size cycling through the schedule of funsearch/polish.py.
        idle: not due -- a slot would idle (the next island in turn)."""
        from ..policy.bytecode import TAG_FLOAT
        from ..policy.compiler import try_compile
        from .polish import _perturb, tunable_literals, with_values
        fs = self.fs
        gens = self._gen_of(merged)
        order = list(range(len(gens)))
        if idle:
            self._idle_rr = (self._idle_rr + 1) % max(1, len(gens))
            order = order[self._idle_rr:] + order[:self._idle_rr]
        for i in order:
            g = start_gen + gens[i]
            if not idle:
                if g < polish_next[i]:
                    continue
                polish_next[i] = g + self.polish_every
            s = fs.islands[i]
            if not s.population:
                continue
            n_done = self._polish_count.get(i, 0)
            # every third polish of an island takes its second or third best
            # member instead of the champion: a champion polished over and over
            # sits on a plateau its literals no longer leave, while a runner-up's
            # basin may hold a better setting
            ranked = sorted(s.population, key=lambda x: -x[1])
            pick = 0 if n_done % 3 != 2 or len(ranked) < 2 else 1 + (n_done // 3) % min(2, len(ranked) - 1)
            code, score = ranked[pick]
            if not fs.polish_repeat and code in fs._polished:
                continue
            fs._polished.add(code)
            prog, _ = try_compile(code)
            if prog is None or not prog.device_ok:
                continue
            from ..ops.jit import launch_key
            launch_key(prog)   # (the variants inherit the shape key: one compile, then data)
            tune = tunable_literals(prog)
            if not tune:
                continue
            base = {prog.literals[j][0]: (prog.fconst[prog.literals[j][0]] if prog.ctag[prog.literals[j][0]] == TAG_FLOAT
                                          else prog.iconst[prog.literals[j][0]]) for j in range(len(prog.literals))}
            self._polish_count[i] = n_done + 1
            # step sizes cycle from coarse (a new basin) to fine (the last digits)
            sigma = _POLISH_SIGMAS[n_done % len(_POLISH_SIGMAS)]
            rng = random.Random(hash((fs.ctx.rank, i, g)) & 0xFFFFFFFF)
            cands = [_perturb(prog, base, tune, sigma, rng) for _ in range(self.polish_variants)]
            return _Polish(i, code, prog, score, cands, [with_values(prog, v) for v in cands])
        return None

    def _polish_done(self, job: _Polish, results, ready: list) -> None:
        """Best variant better than the champion -> its rewritten text enters the
        island as an ordinary child (re-scored exactly, merged by the usual rules)."""
        from ..policy.compiler import try_compile
        from .polish import rewrite_source
        st = self.stats
        st.polish_batches += 1
        st.polish_evals += sum(r is not None for r in results)
        self.fs.evaluations += sum(r is not None for r in results)
        scores = [r.score if r is not None and r.exc == 0 else -1.0 for r in results]
        j = max(range(len(scores)), key=scores.__getitem__) if scores else -1
        rec = dict(kind="steady_polish", rank=self.fs.ctx.rank, island=job.island, base=round(job.base, 6),
                   best=round(scores[j], 6) if j >= 0 else None, variants=len(results))
        if j >= 0 and scores[j] > job.base:
            text = rewrite_source(job.prog, job.cands[j])
            prog, _ = try_compile(text)
            if prog is not None:
                ready.insert(0, (job.island, text, prog))
                st.polish_improved += 1
                rec["improved"] = True
                # (only the improving batches: ~15 polish batches/s would put a
                # JSON record per batch on the dispatcher thread; the status
                # records carry polish_batches / polish_improved)
                self.fs.log.write(**rec)

    def _stream(self, b: _Batch, merged: List[int], islands, ready: list) -> bool:
        """Program service: merge the batch's programs that finished since the
        last look (a straggler -- a replay of millions of events -- holds its
        own workgroup only, never the other results); on completion the
        programs left to the host engines are in ``b.pend.fallback_idx``."""
        t_ph = time.perf_counter()
        got, complete = self.fs.evaluator.collect_partial(b.pend)
        for i, r in got:
            b.results[i] = r
            b.left -= 1
            if b.polish is None:
                isl, code, _ = b.items[i]
                if r.exc == _EXC_EVENTS:
                    self.stats.event_capped += 1
                if r.device_cycles > 0:
                    self.stats.cost_sum += r.device_cycles
                    self.stats.cost_n += 1
                    if not self.cost_anchor and self.cost_anchor_children > 0:
                        self._anchor_samples.append(r.device_cycles)
                        if len(self._anchor_samples) >= self.cost_anchor_children:
                            xs = sorted(self._anchor_samples)
                            self.cost_anchor = xs[len(xs) // 2]
                            self._anchor_samples = []
                            self.fs.log.write(kind="steady_cost_anchor", rank=self.fs.ctx.rank,
                                              mcycles=round(self.cost_anchor / 1e6, 3))
                self._merge_one(islands[isl], code, r.score, r.device_cycles, isl, defer=True)
                merged[isl] += 1
                self.stats.native += int(r.engine == "hip-native")
        if b.polish is None:
            self.stats.evaluations += len(got)
            self.fs.evaluations += len(got)
        if complete:
            b.left = 0
            if b.polish is not None:
                # declined variants are not replayed on the host: the best device-scored setting
                self._polish_done(b.polish, b.results, ready)
        self.phase["merge"] += time.perf_counter() - t_ph
        return bool(got) or complete

    def _log_batch(self, log, ctx, si: int, b: _Batch, ready) -> None:
        ev_n = [r.n_events for r in b.results if r is not None and r.engine == "hip-native"]
        cyc = [r.device_cycles for r in b.results if r is not None and r.device_cycles > 0]
        log.write(kind="steady_batch", rank=ctx.rank, slot=si, programs=len(b.items), new_shapes=b.new_shapes,
                  jit_s=round(b.jit_s, 4), device_s=round(time.time() - b.t_launch, 4),
                  inflight_after=self._left, queued=len(ready),
                  events_mean=round(sum(ev_n) / len(ev_n), 1) if ev_n else 0, events_max=max(ev_n) if ev_n else 0,
                  # device cycles per replay (program service): mean and the longest
                  mcycles_mean=round(sum(cyc) / len(cyc) / 1e6, 3) if cyc else 0,
                  mcycles_max=round(max(cyc) / 1e6, 3) if cyc else 0)

    def _gen_of(self, merged: List[int]) -> List[int]:
        return [m // max(1, s.policies_per_generation) for m, s in zip(merged, self.fs.islands)]

    # -- main loop --------------------------------------------------------------------------
    def run(self, generations: int, threshold: float, wall_s: float = 0.0) -> Tuple[Optional[str], float]:
        fs = self.fs
        islands = fs.islands
        k = len(islands)
        ev = fs.evaluator
        log = fs.log
        ctx = fs.ctx
        start_gen = fs.generation
        merged = [0] * k
        target_children = [generations * max(1, s.policies_per_generation) for s in islands]
        from .migration import MigrationChannel
        dev = getattr(ev, "device", None)
        if dev is not None and hasattr(dev, "warm_native"):
            # first-use JIT set-up (every code-object skeleton's layout probe) before
            # the replays fill the chip: a probe queued behind them waits seconds
            fs.log.write(kind="steady_warm", rank=ctx.rank, warm_s=round(dev.warm_native(), 3))
        svc_started = False
        svc_aborted = False
        if self.service_cfg is not None:
            sc = self.service_cfg
            # (not the whole chip: JIT module loads and copies run as kernels of
            # their own, and at full share they waited for workgroups to leave --
            # tens of seconds of a stalled dispatcher)
            share = float(sc.get("share", 0.75 if fs.coupler is not None else 0.875))
            # data slots: the programs queued or running, stragglers included
            if fs.coupler is not None:
                # the coupler's row-kernel batches take part of what the grid
                # leaves, not all of it: JIT module loads need free slots too
                dev.set_options(row_wave_share=float(sc.get("coupler_share", 0.25)))
            info = dev.start_service(slots=int(sc.get("data_slots", 16384)), share=share)
            svc_started = True
            self.service_inflight = int(sc.get("inflight", 0)) or int(1.5 * info["blocks"])
            fs.log.write(kind="steady_service", rank=ctx.rank, batch_slots=self.slots, share=share,
                         inflight=self.service_inflight, **info)
        chan = MigrationChannel(fs, fs.migrate_every, start_gen)
        self.channel = chan
        stop = False             # no more children: drain and finish
        want_stop = False        # this rank's vote (threshold reached / wall time up)
        global_best = fs.best[1]
        llm_cfg = dict(fs.config.get("llm") or {})
        if not llm_cfg:
            llm_cfg = dict(fs.config.get("openrouter", {}))
            llm_cfg.setdefault("backend", "openai")
        timeout_s = int((fs.config.get("safe_execution") or {}).get("timeout_seconds", 3))
        # LLM request fan-out (``llm.concurrency``): a remote model answers in
        # seconds, so its requests are spread over producers x task_size threads
        # instead of one request per producer process at a time
        from .llm import remote_like
        conc = int(llm_cfg.get("concurrency", 0) or 0)
        fanout = 0
        if conc > 0 and remote_like(llm_cfg):
            # each producer keeps `fanout` requests in flight; a task tops them
            # up by a quarter of that and returns what completed meanwhile (a
            # task of the full fanout would wait for every request in flight --
            # the slowest of 16 at 2-8 s: 7.5 s per task, 33 children/s of 51)
            fanout = max(1, -(-conc // self.producers))
            self.task_size = max(1, fanout // 4)
        self.llm_concurrency = fanout * self.producers
        if fanout:
            fs.log.write(kind="steady_llm", rank=ctx.rank, concurrency=self.llm_concurrency, producers=self.producers,
                         task_size=self.task_size, latency_s=llm_cfg.get("latency_s"))
        ctx_mp = multiprocessing.get_context("spawn")
        pool = concurrent.futures.ProcessPoolExecutor(
            max_workers=self.producers, mp_context=ctx_mp, initializer=_producer_init,
            initargs=(llm_cfg, timeout_s, 1000 * ctx.rank + 1, fanout))
        inflight_tasks: List[concurrent.futures.Future] = []
        fallbacks: list = []             # (batch items, future of the host-engine fallback, programs)
        polish_next = [start_gen + self.polish_every] * k   # generation of each island's next polish
        staged: collections.deque = collections.deque()   # (batch items, future of prepare_compiled, polish job)
        stager = concurrent.futures.ThreadPoolExecutor(max_workers=self.stagers, thread_name_prefix="fks-stage")
        # family coupler (funsearch/coupling.py, `coupling.every` > 0): device family
        # search rounds on a worker thread and the evaluator's last HIP slot, next to
        # the program batches; each round's improved champions enter the islands as
        # program text (re-scored exactly through the normal program path)
        coupler = fs.coupler
        cpl_exec = (concurrent.futures.ThreadPoolExecutor(max_workers=1, thread_name_prefix="fks-couple")
                    if coupler is not None else None)
        cpl_fut = None
        cpl_next = start_gen
        ready: List[tuple] = []          # produced children waiting for a batch
        batches = _Slots(self.slots)
        # children requested per island: production stops at the island's target
        requested = [0] * k
        rr = 0
        t_start = time.time()
        self._cpu0 = time.process_time()
        # per-thread breakdown of the host side (FKS_THREAD_PROFILE=path: CPU
        # seconds per thread group + sampled Python stacks, written at the end)
        sampler = None
        if os.environ.get("FKS_THREAD_PROFILE"):
            from ..utils.trace import ThreadSampler
            sampler = ThreadSampler().start()
        # the dispatcher process runs several Python threads (this loop, the
        # stagers, the similarity scans, the process pool's result thread); at
        # CPython's default 5 ms GIL switch interval a thread that only needs
        # the GIL for a moment (the pool thread handing a finished task back)
        # waits up to 5 ms per hand-off behind the busy ones
        import sys as _sys
        gil_prev = _sys.getswitchinterval()
        _sys.setswitchinterval(float(os.environ.get("FKS_GIL_SWITCH_S", "0.0005")))
        t_status = t_start
        t_prev = t_start
        busy_since = None
        want_buffer = self.batch * (self.slots + self.ahead + 1)
        if self.service_inflight:
            # streaming: the grid's queue, plus the batches being staged
            want_buffer = self.service_inflight + self.batch * (self.ahead + 1)
        next_reset = ((start_gen // fs.reset_every) + 1) * fs.reset_every if fs.reset_every else 0
        rolling = 0.0            # a grid rollover in progress: its start time (launches paused)
        svc_share = share if svc_started else 0.0
        try:
            while True:
                progressed = False
                live = batches.live()
                self._left = sum(b.left for b in live)   # programs not merged yet
                # 1) keep producers busy (children from the islands' CURRENT elites);
                # children only: polish variants filling the grid's spare room must
                # not hold the producers back (they did: polish kept ~2/3 of the
                # in-flight count, the producers idled at ~40 % busy, and the
                # emptier child queue then let in more polish)
                left_children = sum(b.left for b in live if b.polish is None)
                queued = len(ready) + left_children + \
                    sum(len(t) for t, _, pj in staged if pj is None) + self.task_size * len(inflight_tasks)
                while (not stop and queued < want_buffer + self.task_size * self.producers
                       and len(inflight_tasks) < self.tasks_per_producer * self.producers):
                    cands = [i for i in range(k) if requested[i] < target_children[i]]
                    if not cands:
                        break
                    i = cands[rr % len(cands)]
                    rr += 1
                    elites = self._elites(islands[i])
                    if not elites:
                        requested[i] = target_children[i]
                        continue
                    n = min(self.task_size, target_children[i] - requested[i])
                    requested[i] += n
                    fut = pool.submit(_produce, (i, elites, n, self._parent_weights(i, elites)))
                    fut.t_sub = time.perf_counter()
                    inflight_tasks.append(fut)
                    self._asked += n
                    queued += n
                    progressed = True
                # 2) collect produced children
                still = []
                for f in inflight_tasks:
                    if f.done():
                        t_ph = time.perf_counter()
                        items, cpu_s, task_wall_s, gap_s = f.result()
                        self.stats.producer_gap_s += gap_s
                        self.phase["receive"] += time.perf_counter() - t_ph
                        self.stats.producer_cpu_s += cpu_s
                        self.stats.producer_wall_s += task_wall_s
                        t_sub = getattr(f, "t_sub", None)
                        if t_sub is not None:   # submit -> collected, beyond the task itself
                            self.stats.task_turnaround_s += t_ph - t_sub
                            self.stats.task_n += 1
                        self._got += len(items)
                        for isl, code, prog in items:
                            self.stats.produced += 1
                            if prog is not None and prog.source is None:
                                prog.source = code       # (stripped for the trip: _produce)
                            if prog is None:     # no program: counts toward the island's generation
                                self.stats.rejected += 1
                                if code is not None:
                                    fs.evaluator._bump("compile_errors")
                                merged[isl] += 1
                                continue
                            ready.append((isl, code, prog))
                        progressed = True
                    else:
                        still.append(f)
                inflight_tasks = still
                # 3a) stage the next batches: JIT compile + module loads on the stager
                # thread while the slots are busy, so a freed slot relaunches at once
                # (a partial batch when nothing else is coming); a due constant polish
                # of an island champion goes first
                if self.polish_every and not stop and len(staged) < self.ahead:
                    job = self._polish_job(merged, start_gen, polish_next)
                    if job is None and self.polish_idle and len(ready) < self.batch and batches.has_free() and (
                            # stream slots: one would idle; the program service: the grid
                            # has room the children (not a full batch yet) leave
                            not staged if not self.service_inflight
                            else self._left + sum(len(t) for t, _, _ in staged) < (3 * self.service_inflight) // 4):
                        # a slot would idle until the producers refill a batch
                        job = self._polish_job(merged, start_gen, polish_next, idle=True)
                        if job is not None:
                            self.stats.polish_idle += 1
                    if job is not None:
                        items = [(job.island, job.code, pv) for pv in job.progs]
                        staged.append((items, stager.submit(ev.prepare_compiled, [job.code] * len(items),
                                                            job.progs, False), job))
                        job.progs = None
                        progressed = True
                while ready and len(staged) < self.ahead:
                    tail = not inflight_tasks and all(requested[i] >= target_children[i] for i in range(k))
                    if len(ready) < self.batch and not (
                            tail or stop or (batches.empty() and not staged)):
                        break
                    take, ready = ready[:self.batch], ready[self.batch:]
                    staged.append((take, stager.submit(ev.prepare_compiled, [c for _, c, _ in take],
                                                       [p for _, _, p in take]), None))
                    progressed = True
                # 3b) launch staged batches on free slots: in staging order on the
                # stream slots; on the program service any batch whose staging is
                # done (a batch of cached shapes does not wait behind one still
                # generating code), and none while a grid rollover drains it
                while staged and not rolling and batches.has_free():
                    si = batches.next_free()
                    if self.service_inflight:
                        if self._left >= self.service_inflight:
                            break   # the grid has enough queued: results stream back first
                        j = next((j for j, st in enumerate(staged) if st[1].done()), -1)
                        if j < 0:
                            break
                        staged.rotate(-j)
                        take, fut, pjob = staged.popleft()
                        staged.rotate(j)
                    else:
                        if not staged[0][1].done():
                            break
                        take, fut, pjob = staged.popleft()
                    pend = fut.result()
                    with roctx_range(f"steady.launch slot {si} ({len(take)} programs)"):
                        t_ph = time.perf_counter()
                        ev.launch_prepared(pend, self.slot_base + si)
                        self.phase["submit"] += time.perf_counter() - t_ph
                    b = _Batch(si, take, pend, time.time(), pend.new_shapes, pend.jit_s, pjob,
                               [None] * len(take), len(take))
                    batches[si] = b
                    self._left += len(take)
                    self.stats.jit_s += pend.jit_s
                    self.stats.new_shapes += pend.new_shapes
                    if busy_since is None:
                        busy_since = time.time()
                    progressed = True
                # 4a) host-engine fallbacks that finished -> merge
                still_fb = []
                for items, fut, nfb in fallbacks:
                    if not fut.done():
                        still_fb.append((items, fut, nfb))
                        continue
                    if fut.cancelled():
                        continue
                    idx, res = fut.result()
                    t_m = time.perf_counter()
                    for i, r in zip(idx, res):
                        isl, code, _ = items[i]
                        merged[isl] += 1
                        if r.engine == "shed":
                            self.stats.shed += 1
                            continue
                        if self.service_cfg is not None:   # (device-cost selection on)
                            self._merge_one(islands[isl], code, r.score, HOST_COST, isl)
                        else:
                            self._merge_one(islands[isl], code, r.score)
                    self.stats.fallback += len(idx)
                    self.phase["merge"] += time.perf_counter() - t_m
                    progressed = True
                fallbacks = still_fb
                # 4b) finished batches -> merge (programs the device did not score go
                # to the host engines in a worker thread: the dispatcher never runs a
                # CPU-VM or CPython replay itself).  On the program service one scan
                # of the done flags names the batches with rows to take
                news = dev.service_news() if svc_started and dev.service is not None else None
                for si in batches.active_ids():
                    b = batches[si]
                    if self.service_cfg is not None:
                        if news is not None and b.pend.native_idx and b.pend.slot not in news:
                            continue
                        if self._stream(b, merged, islands, ready):
                            progressed = True
                        if b.left > 0:
                            continue
                        # complete: its host fallbacks and the batch record
                        batches[si] = None
                        if busy_since is not None and batches.empty():
                            self.stats.busy_s += time.time() - busy_since
                            busy_since = None
                        if b.polish is None and b.pend.fallback_idx:
                            nfb = len(b.pend.fallback_idx)
                            if svc_aborted or b.aborted:   # (aborted replays and the rest: not needed)
                                self.stats.abandoned += nfb
                            elif sum(x[2] for x in fallbacks) + nfb > self.fallback_cap:
                                # the host engines are behind (a CPU-VM replay of an evolved
                                # program takes seconds of a core, and the producers need the
                                # cores): shed instead of queueing
                                self.stats.shed += nfb
                                for i in b.pend.fallback_idx:
                                    merged[b.items[i][0]] += 1
                            else:             # (merged when their fallback completes)
                                self.stats.evaluations += nfb
                                fs.evaluations += nfb
                                fallbacks.append((b.items, ev.fallback_async(b.pend, object_ok=self.host_object),
                                                  nfb))
                        if b.polish is None:
                            self.stats.batches += 1
                            self._log_batch(log, ctx, si, b, ready)
                        progressed = True
                        continue
                    if not ev.ready(b.pend):
                        continue
                    t_ph = time.perf_counter()
                    # (no device: a polish batch is scored here, on the host engines)
                    results = ev.collect(b.pend, defer_fallback=b.polish is None or ev.device is not None)
                    if b.polish is not None:
                        # declined variants are not replayed on the host: the polish
                        # takes the best device-scored setting
                        batches[si] = None
                        if busy_since is not None and batches.empty():
                            self.stats.busy_s += time.time() - busy_since
                            busy_since = None
                        self._polish_done(b.polish, results, ready)
                        self.phase["collect"] += time.perf_counter() - t_ph
                        progressed = True
                        continue
                    if b.pend.fallback_idx:
                        fallbacks.append((b.items, ev.fallback_async(b.pend, object_ok=self.host_object),
                                          len(b.pend.fallback_idx)))
                    t_m = time.perf_counter()
                    self.phase["collect"] += t_m - t_ph
                    t_done = time.time()
                    batches[si] = None
                    if busy_since is not None and batches.empty():
                        self.stats.busy_s += t_done - busy_since
                        busy_since = None
                    for (isl, code, _), res in zip(b.items, results):
                        if res is None:          # merged when its fallback completes
                            continue
                        self._merge_one(islands[isl], code, res.score)
                        merged[isl] += 1
                        if res.engine == "hip-native":
                            self.stats.native += 1
                    self.phase["merge"] += time.perf_counter() - t_m
                    self.stats.evaluations += len(b.items)
                    self.stats.batches += 1
                    fs.evaluations += len(b.items)
                    inflight = sum(len(x.items) for x in batches.live())
                    ev_n = [r.n_events for r in results if r is not None and r.engine == "hip-native"]
                    log.write(kind="steady_batch", rank=ctx.rank, slot=si, programs=len(b.items),
                              new_shapes=b.new_shapes, jit_s=round(b.jit_s, 4),
                              device_s=round(t_done - b.t_launch, 4), inflight_after=inflight,
                              queued=len(ready),
                              # replayed events per program: the batch's mean and its longest (tail)
                              events_mean=round(sum(ev_n) / len(ev_n), 1) if ev_n else 0,
                              events_max=max(ev_n) if ev_n else 0)
                    progressed = True
                # deferred merges whose similarity scans finished
                if self._pending_merges:
                    t_m = time.perf_counter()
                    if self._finish_merges():
                        progressed = True
                    self.phase["merge"] += time.perf_counter() - t_m
                gens = self._gen_of(merged)
                g_min = start_gen + min(gens)
                fs.generation = g_min
                for s, g in zip(islands, gens):
                    s.generation = start_gen + g
                # island resets (islands.reset_every): at each multiple the slowest island passes
                if fs.reset_every and g_min >= next_reset:
                    fs.reset_weak_islands()
                    next_reset = (g_min // fs.reset_every + 1) * fs.reset_every
                # 5) migration: post async gathers; absorb finished ones (in order)
                if chan.every:
                    if chan.post_due(g_min if not stop else -1, want_stop):
                        progressed = True
                    if self._absorb(chan.poll(threshold)):
                        progressed = True
                    if chan.stopping:
                        stop = True
                # 5b) family coupling: start a round when one is due, merge a finished one
                if coupler is not None:
                    if cpl_fut is not None and cpl_fut.done():
                        for rec in cpl_fut.result():
                            fs.inject_coupled(rec)
                            self.stats.coupled += 1
                        cpl_fut = None
                        progressed = True
                    if cpl_fut is None and not stop and g_min >= cpl_next:
                        cpl_fut = cpl_exec.submit(fs.run_coupling)
                        cpl_next = g_min + coupler.every
                global_best = max(chan.best_global, fs.best[1])
                want_stop = want_stop or global_best >= threshold or bool(wall_s and time.time() - t_start > wall_s)
                if want_stop and not chan.active:
                    stop = True        # alone (or no migrations): nobody to agree with
                if stop and svc_started and not svc_aborted:
                    # the replays still in flight are not needed: a straggler of
                    # millions of events would hold the end of the run
                    dev.abort_service()
                    svc_aborted = True
                # 5c) grid rollover: JIT modules retired while the grid runs stay
                # loaded (an unload waits for the device); past `rollover_modules`
                # pause launches, let the grid drain (stragglers aborted after the
                # grace period), unload, and start the grid again
                if svc_started and not svc_aborted and not stop and self.rollover_deferred > 0:
                    nc = dev.native_compiler
                    if not rolling and nc.deferred >= self.rollover_deferred:
                        rolling = time.time()
                        fs.log.write(kind="steady_rollover_begin", rank=ctx.rank, deferred=nc.deferred,
                                     inflight=self._left)
                    if rolling:
                        busy = batches.live()
                        if busy and time.time() - rolling > self.rollover_grace_s and not any(b.aborted for b in busy):
                            dev.abort_service()
                            for b in busy:
                                b.aborted = True
                        if not busy:
                            t_r = time.time()
                            flushed = nc.deferred
                            dev.stop_service()
                            dev.start_service(slots=int(self.service_cfg.get("data_slots", 16384)), share=svc_share)
                            self.stats.rollovers += 1
                            self.stats.rollover_s += time.time() - rolling
                            fs.log.write(kind="steady_rollover", rank=ctx.rank, unloaded=flushed,
                                         drain_s=round(t_r - rolling, 3), restart_s=round(time.time() - t_r, 3),
                                         live_modules=nc.stats.get("live_modules"),
                                         loaded_mb=nc.stats.get("loaded_mb"))
                            rolling = 0.0
                            progressed = True
                # 6) status (time-weighted programs in flight, for the occupancy figure)
                now = time.time()
                self.stats.inflight_sum += sum(b.left for b in batches.live()) * (now - t_prev)
                self.stats.inflight_n += now - t_prev
                t_prev = now
                if now - t_status >= self.status_every_s:
                    t_status = now
                    self._status(now, t_start, busy_since, batches, ready, inflight_tasks, merged, global_best)
                # stopping: host fallbacks not started yet are abandoned (a CPU-VM
                # replay of a large program takes seconds of a core)
                if stop and fallbacks and batches.empty() and not staged:
                    kept = []
                    for items, fut, nfb in fallbacks:
                        if fut.cancel():
                            self.stats.abandoned += nfb
                        else:
                            kept.append((items, fut, nfb))
                    fallbacks = kept
                # 7) done?  (every child merged, or stopping; then every agreed gather finished)
                all_launched = all(requested[i] >= target_children[i] for i in range(k))
                if fanout and all_launched and not stop and not inflight_tasks and self._got < self._asked:
                    # children still waiting on their requests inside the producers
                    # (fan-out tasks return what is ready): flush every process
                    inflight_tasks.extend(pool.submit(_produce, (0, [], 0, None)) for _ in range(self.producers))
                    progressed = True
                idle = (not inflight_tasks and batches.empty() and not fallbacks and not self._pending_merges
                        and not staged and cpl_fut is None)
                if idle and (stop or (all_launched and not ready)):
                    ready.clear()
                    due = chan.every and chan.next is not None and (
                        chan.next <= chan.stop_at if chan.stopping else (chan.next <= g_min and not stop))
                    if not due:
                        if not chan.pending:
                            break
                        self._absorb(chan.poll(threshold, block=True))
                        continue
                if not progressed:
                    time.sleep(0.0005)
        finally:
            _sys.setswitchinterval(gil_prev)
            if sampler is not None:
                sampler.stop()
                rep = sampler.report()
                rep["main_phase_s"] = {k: round(v, 3) for k, v in self.phase.items()}
                log.write(kind="steady_threads", rank=ctx.rank, **rep)
                import json
                path = os.environ["FKS_THREAD_PROFILE"]
                if ctx.world_size > 1:
                    path = f"{path}.rank{ctx.rank}"
                with open(path, "w") as fh:
                    json.dump(rep, fh, indent=1)
            pool.shutdown(wait=False, cancel_futures=True)
            stager.shutdown(wait=True, cancel_futures=True)
            if self._pending_merges:
                self._finish_merges(block=True)
            if self._sim_pool is not None:
                self._sim_pool.shutdown(wait=True)
                self._sim_pool = None
            if cpl_exec is not None:
                cpl_exec.shutdown(wait=True, cancel_futures=True)
            for _, fut, _pj in staged:   # compiled but never launched: give the modules back
                if fut.done() and not fut.cancelled() and fut.exception() is None:
                    ev.discard_prepared(fut.result())
            if svc_started:
                dev.stop_service()
        now = time.time()
        rec = self._status(now, t_start, busy_since, batches, ready, inflight_tasks, merged, global_best, final=True)
        if fs.ck_dir:
            fs.save_checkpoint()
        if fs.verbose and ctx.is_main:
            import json
            print(json.dumps(rec), flush=True)
        return fs.best

    def _status(self, now, t_start, busy_since, batches, ready, tasks, merged, best_global, final=False) -> dict:
        st = self.stats
        wall = max(1e-9, now - t_start)
        busy = st.busy_s + (now - busy_since if busy_since is not None else 0.0)
        fs = self.fs
        inflight = sum(b.left for b in batches.live())
        self._left = inflight
        # programs of batches launched more than 5 s ago that are still replaying:
        # the grid's workgroups held by long replays (a 15M-event policy takes ~30 s)
        stragglers = sum(b.left for b in batches.live() if now - b.t_launch > 5.0)
        # occupancy: programs in flight / programs the device holds resident at the
        # current heap top (device_busy only says that *some* batch was in flight)
        capacity = 0
        info = {}
        dev = getattr(fs.evaluator, "device", None)
        if dev is not None:
            info = dev.info()
            capacity = int(info.get("native_duo_per_cu_last", 0)) * int(info.get("num_cus", 0))
            if "service" in info:
                capacity = int(info["service"]["blocks"])
        rec = dict(kind="steady_final" if final else "steady_status", rank=fs.ctx.rank, wall_s=round(wall, 3),
                   evaluations=st.evaluations, evals_per_s=round(st.evaluations / wall, 2),
                   device_busy=round(busy / wall, 4),
                   new_shape_fraction=round(st.new_shapes / max(1, st.evaluations), 4),
                   native_fraction=round(st.native / max(1, st.evaluations), 4), host_fallback=st.fallback,
                   shed=st.shed, abandoned=st.abandoned, polish_batches=st.polish_batches,
                   polish_evals=st.polish_evals, polish_improved=st.polish_improved, polish_idle=st.polish_idle,
                   coupled=st.coupled,
                   coupler_evals=(fs.coupler.evaluated if fs.coupler is not None else 0),
                   # MFMA behavioural screen of the coupler's linear families: drawn / replayed
                   coupler_screened=(sum(i.screened for i in fs.coupler.islands.values()) if fs.coupler else 0),
                   coupler_screen_kept=(sum(i.screen_kept for i in fs.coupler.islands.values()) if fs.coupler else 0),
                   all_evals_per_s=round((st.evaluations + st.polish_evals) / wall, 2),
                   inflight=inflight, inflight_mean=round(st.inflight_sum / max(1e-9, st.inflight_n), 1),
                   resident_capacity=capacity,
                   occupancy=round(inflight / capacity, 4) if capacity else None,
                   occupancy_mean=round(st.inflight_sum / max(1e-9, st.inflight_n) / capacity, 4) if capacity else None,
                   queued=len(ready),
                   # device cost of the children (program service: s_memtime cycles
                   # per replay) and what the selection did with it
                   mcycles_per_child=round(st.cost_sum / max(1, st.cost_n) / 1e6, 3), cost_rejected=st.cost_rejected,
                   rollovers=st.rollovers, rollover_s=round(st.rollover_s, 2), mem_used_mb=info.get("mem_used_mb"),
                   stragglers=stragglers, cost_anchor_mcycles=round(self.cost_anchor / 1e6, 3),
                   event_capped=st.event_capped, max_events=self.max_events,
                   producer_tasks=len(tasks), produced=st.produced,
                   children_per_s=round(st.produced / wall, 2),
                   llm_inflight=min(len(tasks), self.producers) * self.task_size if self.llm_concurrency else None,
                   producer_ms_per_child=round(1e3 * st.producer_cpu_s / max(1, st.produced), 3),
                   # producers' CPU / wall while on a task (< 1: preempted, the host's
                   # cores are short) and the fraction of the run they were on tasks
                   producer_cpu_share=round(st.producer_cpu_s / max(1e-9, st.producer_wall_s), 3),
                   producer_busy=round(st.producer_wall_s / max(1e-9, wall * self.producers), 3),
                   # mean producer task: submit -> collected, and its own wall time (the
                   # difference: queueing in the pool + hand-off to / from the worker)
                   task_turnaround_ms=round(1e3 * st.task_turnaround_s / max(1, st.task_n), 2),
                   task_wall_ms=round(1e3 * st.producer_wall_s / max(1, st.task_n), 2),
                   task_gap_ms=round(1e3 * st.producer_gap_s / max(1, st.task_n), 2),
                   main_cpu_frac=round((time.process_time() - self._cpu0) / wall, 3), rejected=st.rejected, jit_s=round(st.jit_s, 3),
                   generation=fs.generation, best=round(fs.best[1], 6), best_global=round(best_global, 6),
                   islands=[round(s.best_score, 6) for s in fs.islands], migrations=st.migrations,
                   resets=fs.resets, distinct_island_bests=len({s.best_policy for s in fs.islands}),
                   collective_wait_s=round(self.channel.wait_s, 4),
                   main_phase_s={k: round(v, 3) for k, v in self.phase.items()},
                   jit={k: (round(v, 3) if isinstance(v, float) else v)
                        for k, v in (getattr(getattr(fs.evaluator.device, "native_compiler", None), "stats", None)
                                     or {}).items()},
                   collective_wait_frac=round(self.channel.wait_s / wall, 5),
                   engines={k: v for k, v in fs.evaluator.stats.items() if k in
                            ("device_native", "device", "cpu_vm", "object", "shed", "compile_errors", "jit_shapes",
                             "native_timeout", "native_invariant", "native_event_cap")})
        fs.log.write(**rec)
        st.history.append(rec)
        if fs.verbose and fs.ctx.is_main and not final:
            import json
            print(json.dumps(rec), flush=True)
        return rec


__all__ = ["SteadyStateSearch", "SteadyStats"]
