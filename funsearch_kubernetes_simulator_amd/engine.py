"""`evaluate()`: score policy programs on the fastest exact engine available.

Routing per program (every path yields the reference's score bit-for-bit; the
device's `**`, math.exp / log / pow are glibc's own algorithms, so they return
CPython's bits -- csrc/hip/glibc_math.h, checked at start-up by
`hip_engine.glibc_math_ok`):

1. compile to bytecode (`policy.compiler`); programs outside the native
   subset go straight to the object engine (CPython ``exec``, step 4);
2. MI355X (`ops.hip_engine`): natively compiled programs first
   (`policy.native_codegen` -> `ops.jit`, one k_replay_native wave per program,
   any batch size; compiled shapes are cached), then the device bytecode VM for
   what the native backend declines, when the batch is large enough to fill
   the chip;
3. native CPU VM (`ops.cpu_engine`): for no-GPU hosts, for programs the device
   reports as EXC_UNSUPPORTED (bigint / complex / trig) or
   EXC_BUDGET (per-call instruction budget), and for results whose exact-mean
   accumulator flagged `inexact`;
4. object engine (`simulator.KubernetesSimulator` + ``exec``), which *is* the
   reference semantics, for whatever the native engines cannot express; it
   runs under a wall-clock budget (``object_timeout_s``, default 600 s).

Scores follow `evaluate_policy_standalone` (`funsearch/funsearch_integration.py:30-64`):
any exception during the replay gives score 0.  `EvalResult.exc` tells which
exception class it was; `EvalResult.engine` which engine produced it.
"""

from __future__ import annotations

import atexit
import copy
import os
import threading
import time
from concurrent.futures import ProcessPoolExecutor
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from .core.arrays import Workload
from .core.traces import load_default_workload
from .policy.bytecode import Exc
from .policy.compiler import CompiledPolicy, try_compile
from .simulator.metrics import EvaluationResults

COLS = {name: i for i, name in enumerate(
    ("score", "avg_cpu", "avg_mem", "avg_gpu_count", "avg_gpu_milli", "frag", "n_snapshots",
     "n_frag_events", "n_events", "n_unplaced", "exc", "inexact", "trace_hash_hi"))}


@dataclass
class EvalResult:
    score: float
    exc: int = 0
    engine: str = ""
    results: Optional[EvaluationResults] = None
    n_events: int = 0
    detail: Dict[str, float] = field(default_factory=dict)
    #: device cycles of the replay (program service only; 0 elsewhere): what a
    #: program costs the search -- parent sampling and bloat control, never the score
    device_cycles: float = 0.0

    @property
    def ok(self) -> bool:
        return self.exc == 0


def _row_to_result(row: np.ndarray, engine: str) -> EvalResult:
    exc = int(row[COLS["exc"]])
    if exc:
        return EvalResult(0.0, exc, engine, n_events=int(row[COLS["n_events"]]))
    res = EvaluationResults(
        avg_cpu_utilization=float(row[COLS["avg_cpu"]]),
        avg_memory_utilization=float(row[COLS["avg_mem"]]),
        avg_gpu_count_utilization=float(row[COLS["avg_gpu_count"]]),
        avg_gpu_memory_utilization=float(row[COLS["avg_gpu_milli"]]),
        gpu_fragmentation_score=float(row[COLS["frag"]]),
        num_snapshots=int(row[COLS["n_snapshots"]]),
        num_fragmentation_events=int(row[COLS["n_frag_events"]]))
    return EvalResult(float(row[COLS["score"]]), 0, engine, res, int(row[COLS["n_events"]]),
                      {"n_unplaced": float(row[COLS["n_unplaced"]]), "trace_hash_hi": float(row[COLS["trace_hash_hi"]])})


# ---------------------------------------------------------------------------- object engine
class ReplayTimeout(Exception):
    """Raised inside an object-engine replay that exceeded its wall-clock budget."""


def object_engine_eval(code: str, workload: Workload, budget_s: float = 0.0) -> EvalResult:
    """Reference-semantics replay with CPython ``exec`` (the exact fallback).

    ``budget_s`` > 0 bounds the replay's wall-clock time with ``SIGALRM`` (as
    the reference's `SafeExecutor`, `funsearch/safe_execution.py:81-96`, does
    per call): a program that loops forever scores 0 with `Exc.BUDGET`
    instead of hanging the search.  Only effective in a process's main thread.
    """
    import signal
    import threading
    from .funsearch.scheduler import FunSearchScheduler
    from .simulator import DiscreteEventSimulator, KubernetesSimulator, SchedulingEvaluator
    armed = budget_s > 0 and threading.current_thread() is threading.main_thread()
    if armed:
        def _expire(signum, frame):
            raise ReplayTimeout(f"replay exceeded {budget_s} s")
        old = signal.signal(signal.SIGALRM, _expire)
        signal.setitimer(signal.ITIMER_REAL, budget_s)
    try:
        sched = FunSearchScheduler(code)
        cluster, pods = workload.to_objects()
        ev = SchedulingEvaluator(cluster, enabled=True)
        sim = KubernetesSimulator(cluster, pods, DiscreteEventSimulator(pods), sched, evaluator=ev)
        sim.run_schedule()
        res = ev.get_evaluation_results()
        return EvalResult(float(ev.get_policy_score(pods)), 0, "object", res, sim.events_processed)
    except Exception as exc:  # any exception aborts the replay -> score 0
        return EvalResult(0.0, _exc_code(exc), "object")
    finally:
        if armed:
            signal.setitimer(signal.ITIMER_REAL, 0)
            signal.signal(signal.SIGALRM, old)


def _exc_code(exc: BaseException) -> int:
    if isinstance(exc, ReplayTimeout):
        return int(Exc.BUDGET)
    if isinstance(exc, ZeroDivisionError):
        return int(Exc.ZERO_DIVISION)
    if isinstance(exc, OverflowError):
        return int(Exc.OVERFLOW)
    if isinstance(exc, IndexError):
        return int(Exc.INDEX)
    if isinstance(exc, NameError):
        return int(Exc.NAME)
    if isinstance(exc, TypeError):
        return int(Exc.TYPE)
    return int(Exc.VALUE)


def _object_worker(args):
    code, workload, budget_s = args
    return object_engine_eval(code, workload, budget_s)


# ---------------------------------------------------------------------------- evaluator
#: exception codes of a native-program row that hand the program to the next
#: engine: UNSUPPORTED / BUDGET as for every engine, TIMEOUT -- the two-wave
#: kernel ends a replay with it when one wave stops hearing from the other (a
#: bounded spin, replay_duo.hip.h), which depends on timing, not on the
#: program -- and INVARIANT, a failed accounting check, i.e. a kernel bug: the
#: program is re-scored by the next engine (so the score stays exact) but the
#: row is counted in ``stats["native_invariant"]`` and logged, never hidden
NATIVE_DEFER = (int(Exc.UNSUPPORTED), int(Exc.BUDGET), int(Exc.TIMEOUT), int(Exc.INVARIANT))


def _native_deferred(row, bump) -> bool:
    """True: this native-program row goes to the next engine (counted through `bump`)."""
    exc = int(row[COLS["exc"]])
    if exc == Exc.TIMEOUT:
        bump("native_timeout")
    elif exc == Exc.EVENTS:
        bump("native_event_cap")   # final: past the caller's replay event budget, not scored
    elif exc == Exc.INVARIANT:
        bump("native_invariant")
        import warnings
        warnings.warn("native replay failed its invariant check (kernel bug?); program re-scored on the CPU VM",
                      RuntimeWarning, stacklevel=3)
    return exc in NATIVE_DEFER or bool(row[COLS["inexact"]])


class Evaluator:
    """Batched exact evaluator bound to one workload.

    ``device``: ``"auto"`` (MI355X if visible, else CPU), ``"gpu"``/``int``
    (HIP device index; fails loudly if unavailable), or ``"cpu"``.
    """

    def __init__(self, workload: Optional[Workload] = None, device="auto", options: Optional[dict] = None,
                 cpu_threads: int = 0, object_workers: int = 0, n_slots: int = 4):
        self.workload = workload or load_default_workload()
        self.options = dict(options or {})
        from .ops.cpu_engine import default_threads
        self.cpu_threads = cpu_threads or default_threads()
        self.object_workers = object_workers or min(8, self.cpu_threads)
        # below this many programs a batch runs faster on the CPU VM (one replay per
        # core, ~0.1 s each) than as a handful of latency-bound device waves
        self.device_min_batch = int(self.options.pop("device_min_batch", 128))
        # natively compiled programs on the device (any batch size)
        self.native = bool(self.options.pop("native", True))
        # fault-injection hook: fail this fraction of program
        # evaluations as if the replay had raised -> score 0, like the reference
        self.fault_rate = float(self.options.pop("fault_rate", 0.0) or 0.0)
        # bytecode compiles of program batches in worker processes: the compiler is
        # pure Python (~4 ms per program), and pipelined islands otherwise queue on
        # the GIL for it (0: in-process)
        self.compile_workers = int(self.options.pop("compile_workers", 0) or 0)
        self._compile_pool = None
        self._compile_lock = threading.Lock()
        # counters are bumped from the dispatcher and from the fallback worker
        # threads (`fallback_async`): every update goes through `_bump`
        self._stats_lock = threading.Lock()
        fault_seed = int(self.options.pop("fault_seed", 0))
        self._fault_rng = np.random.default_rng(fault_seed)
        # the fallback threads draw from their own generator (under the stats
        # lock), so the dispatcher's fault sequence stays deterministic
        self._fallback_fault_rng = np.random.default_rng(fault_seed + 1)
        self.device = None
        want_gpu = device not in ("cpu", None)
        if want_gpu:
            from .ops import hip_engine
            idx = device if isinstance(device, int) else int(os.environ.get("LOCAL_RANK", 0))
            available = hip_engine.device_available()
            if available and not isinstance(device, int):
                idx %= hip_engine.native().device_count()   # ranks > GPUs (gloo rehearsal) share the cards
            if not available and device != "auto":
                raise RuntimeError("HIP device requested but none is visible")
            if available:
                try:
                    self.device = hip_engine.DeviceEvaluator(self.workload, idx, self.options, n_slots)
                except hip_engine.UnsupportedWorkload:
                    if device != "auto":
                        raise
        self.stats = {"device": 0, "device_native": 0, "cpu_vm": 0, "object": 0, "compile_errors": 0,
                      "jit_s": 0.0, "jit_shapes": 0, "native_timeout": 0, "native_invariant": 0}
        self._done: Dict[int, np.ndarray] = {}   # CPU stand-in for in-flight slots

    def _bump(self, key: str, n=1) -> None:
        with self._stats_lock:
            self.stats[key] = self.stats.get(key, 0) + n

    @property
    def backend(self) -> str:
        return "hip" if self.device is not None else "cpu"

    # -- built-in parametric families -------------------------------------------
    def evaluate_family(self, family: str, weights: np.ndarray) -> np.ndarray:
        """[P, 13] result table for P members of a built-in family."""
        if self.device is not None:
            return self.device.evaluate_builtin(family, weights)
        from .ops import cpu_engine
        return cpu_engine.simulate_builtin_batch(self.workload, family, weights,
                                                 cpu_engine.SimOptions(**self._cpu_opts()), self.cpu_threads)

    # asynchronous form: several family batches in flight (one HIP stream per slot)
    def submit_family(self, slot: int, family: str, weights: np.ndarray) -> None:
        if self.device is not None:
            self.device.submit_builtin(slot, family, weights)
        else:
            self._done[slot] = self.evaluate_family(family, weights)

    def wait(self, slot: int) -> np.ndarray:
        return self.device.wait(slot) if self.device is not None else self._done.pop(slot)

    def _cpu_opts(self) -> dict:
        from .ops.cpu_engine import DEFAULT_CALL_BUDGET
        keep = ("repush", "gpu_alloc", "snapshot_interval", "budget")   # (object_timeout_s: object engine only)
        opts = {k: v for k, v in self.options.items() if k in keep}
        opts.setdefault("budget", DEFAULT_CALL_BUDGET)
        return opts

    # -- programs ---------------------------------------------------------------------
    def compile_batch(self, codes: Sequence[str]) -> List[Optional[CompiledPolicy]]:
        """Bytecode for every program text (None: rejected), in worker processes
        when ``compile_workers`` > 0 and the batch has more than one program."""
        codes = list(codes)
        if self.compile_workers > 0 and len(codes) > 1:
            with self._compile_lock:
                if self._compile_pool is None:
                    import multiprocessing
                    # spawn: the workers never inherit the parent's HIP state
                    self._compile_pool = ProcessPoolExecutor(max_workers=self.compile_workers,
                                                             mp_context=multiprocessing.get_context("spawn"))
                    atexit.register(self._compile_pool.shutdown, wait=False, cancel_futures=True)
            chunk = max(1, len(codes) // (2 * self.compile_workers))
            results = list(self._compile_pool.map(try_compile, codes, chunksize=chunk))
        else:
            results = [try_compile(c) for c in codes]
        out = []
        for prog, _ in results:
            if prog is None:
                self._bump("compile_errors", 1)
            out.append(prog)
        return out

    def evaluate_programs(self, codes: Sequence[str], slot: int = 0) -> List[EvalResult]:
        """Scores of program texts (synchronous; device work on HIP slot `slot`)."""
        compiled = self.compile_batch(codes)
        out = self._evaluate_compiled(list(codes), compiled, native=self.native, slot=slot)
        if self.fault_rate > 0:
            for i in range(len(out)):
                if self._fault_rng.random() < self.fault_rate:
                    out[i] = EvalResult(0.0, int(Exc.VALUE), "fault-injection")
                    self._bump("faults")
        return out

    def _evaluate_compiled(self, codes: Sequence[str], compiled: List[Optional[CompiledPolicy]],
                           native: bool, slot: int = 0, host_only: bool = False,
                           object_ok: bool = True) -> List[EvalResult]:
        n = len(codes)
        out: List[Optional[EvalResult]] = [None] * n
        # 1) device: native code, then the bytecode VM
        pending = [i for i, p in enumerate(compiled) if p is not None]
        if self.device is not None and not host_only:
            exact = getattr(self.device, "math_exact", True)
            dev_idx = [i for i in pending if compiled[i].device_ok and (exact or not compiled[i].uses_libm)]
            if dev_idx and native:
                self._absorb_native(dev_idx, compiled, out, slot)
            dev_idx = [i for i in dev_idx if out[i] is None]
            if len(dev_idx) >= self.device_min_batch:
                tab = self.device.evaluate_programs([compiled[i] for i in dev_idx], slot=slot)
                for row, i in zip(tab, dev_idx):
                    if int(row[COLS["exc"]]) in (Exc.UNSUPPORTED, Exc.BUDGET) or row[COLS["inexact"]]:
                        continue
                    out[i] = _row_to_result(row, "hip")
                    self._bump("device", 1)
        # 2) native CPU VM
        cpu_idx = [i for i in pending if out[i] is None]
        if cpu_idx:
            from .ops import cpu_engine
            tab = cpu_engine.simulate_program_batch(self.workload, [compiled[i] for i in cpu_idx],
                                                    cpu_engine.SimOptions(**self._cpu_opts()), self.cpu_threads)
            for row, i in zip(tab, cpu_idx):
                if int(row[COLS["exc"]]) in (Exc.UNSUPPORTED, Exc.BUDGET) or row[COLS["inexact"]]:
                    continue
                out[i] = _row_to_result(row, "cpu")
                self._bump("cpu_vm", 1)
        # 3) object engine (exact by construction)
        rest = [i for i in range(n) if out[i] is None]
        if rest and not object_ok:
            # the caller sheds what only CPython can score (bigint / complex
            # intermediates): engine "shed", never a score
            for i in rest:
                out[i] = EvalResult(0.0, int(Exc.UNSUPPORTED), "shed")
                self._bump("shed")
            rest = []
        if rest:
            if self._object_engine_ok():
                budget_s = float(self.options.get("object_timeout_s", 600.0))
                jobs = [(codes[i], self.workload, budget_s) for i in rest]
                if host_only:
                    # a worker thread (async fallback): the wall-clock budget needs a
                    # process main thread, so the replays run in the spawned object pool
                    results = list(self._object_pool().map(_object_worker, jobs))
                elif len(rest) > 1 and self.object_workers > 1:
                    with ProcessPoolExecutor(max_workers=min(self.object_workers, len(rest))) as ex:
                        results = list(ex.map(_object_worker, jobs))
                else:
                    results = [_object_worker(j) for j in jobs]
            else:
                results = [EvalResult(0.0, int(Exc.UNSUPPORTED), "none") for _ in rest]
            for i, r in zip(rest, results):
                out[i] = r
                self._bump("object", 1)
        return out  # type: ignore[return-value]

    def score_compiled(self, progs: Sequence[CompiledPolicy], slot: int = 0) -> np.ndarray:
        """Scores of already-compiled programs (e.g. constant variants of one
        shape, funsearch/polish.py): one native device launch when a device is
        attached (programs it declines fall back to the CPU VM), else the CPU VM."""
        out = np.zeros(len(progs))
        rest = list(range(len(progs)))
        if self.device is not None and self.native and progs:
            self.device.submit_native(slot, progs)
            tab = self.device.wait(slot)
            ok = np.array([not _native_deferred(row, self._bump) for row in tab], dtype=bool)
            out[ok] = tab[ok, COLS["score"]]
            rest = [i for i in range(len(progs)) if not ok[i]]
            self._bump("device_native", int(ok.sum()))
        if rest:
            from .ops import cpu_engine
            tab = cpu_engine.simulate_program_batch(self.workload, [progs[i] for i in rest],
                                                    cpu_engine.SimOptions(**self._cpu_opts()), self.cpu_threads)
            for row, i in zip(tab, rest):
                exc = int(row[COLS["exc"]])
                out[i] = 0.0 if exc else row[COLS["score"]]
            self._bump("cpu_vm", len(rest))
        return out

    # -- asynchronous program batches (pipelined islands) ------------------------------
    def submit_programs(self, codes: Sequence[str], slot: int) -> "PendingPrograms":
        """Start evaluating `codes` on device slot `slot` (its own HIP stream):
        compiles to bytecode and, on a device, JIT-compiles the native shapes and
        launches them; returns at once.  `ready` / `collect` finish the batch
        (programs the native backend declines run on the next engine at collect
        time).  Without a device everything happens at collect time."""
        return self.submit_compiled(codes, self.compile_batch(list(codes)), slot, count_errors=False)

    def submit_compiled(self, codes: Sequence[str], compiled: Sequence[Optional[CompiledPolicy]],
                        slot: int, count_errors: bool = True) -> "PendingPrograms":
        """`submit_programs` for programs whose bytecode was produced elsewhere
        (the steady-state search compiles in its producer processes)."""
        return self.launch_prepared(self.prepare_compiled(codes, compiled, count_errors), slot)

    def prepare_compiled(self, codes: Sequence[str], compiled: Sequence[Optional[CompiledPolicy]],
                         count_errors: bool = True) -> "PendingPrograms":
        """The compile half of `submit_compiled`, callable from a worker thread:
        JIT-compiles and loads the batch's native shapes (held until the batch
        is collected or `discard_prepared`).  `launch_prepared` starts it."""
        pend = PendingPrograms(list(codes), -1)
        pend.compiled = list(compiled)
        if count_errors:
            self._bump("compile_errors", sum(p is None for p in pend.compiled))
        if self.device is not None and self.native:
            idx = [i for i, p in enumerate(pend.compiled) if p is not None and p.device_ok]
            if idx:
                t0 = time.perf_counter()
                batch = self.device.prepare_native([pend.compiled[i] for i in idx])
                pend.prepared = batch
                pend.native_idx = idx
                pend.jit_s = batch.compile_s
                pend.new_shapes = batch.compiled
                pend.submit_s = time.perf_counter() - t0
                self._bump("jit_s", batch.compile_s)
                self._bump("jit_shapes", batch.compiled)
        return pend

    def launch_prepared(self, pend: "PendingPrograms", slot: int) -> "PendingPrograms":
        """Launch a `prepare_compiled` batch on device slot `slot` (main thread)."""
        pend.slot = slot
        if pend.native_idx:
            t0 = time.perf_counter()
            self.device.submit_native(slot, [pend.compiled[i] for i in pend.native_idx], pend.prepared)
            pend.prepared = None
            pend.t_launch = time.perf_counter()
            pend.submit_s += pend.t_launch - t0
        return pend

    def discard_prepared(self, pend: "PendingPrograms") -> None:
        """Give back the modules of a prepared batch that will not be launched."""
        if pend.prepared is not None:
            self.device.release_native(pend.prepared)
            pend.prepared = None

    def ready(self, pend) -> bool:
        """Slot index (family batches) or `PendingPrograms`: finished?"""
        if isinstance(pend, int):
            return self.device.ready(pend) if self.device is not None else True
        return not pend.native_idx or self.device.ready(pend.slot)

    def collect(self, pend: "PendingPrograms", defer_fallback: bool = False) -> List[Optional[EvalResult]]:
        """Results of a submitted batch.  Programs the device did not score
        (declined, deferred) run on the host engines here -- or, with
        `defer_fallback`, are left as None and listed in ``pend.fallback_idx``
        for `fallback_async` (the steady-state dispatcher must not block on a
        CPython replay)."""
        n = len(pend.codes)
        out: List[Optional[EvalResult]] = [None] * n
        if pend.native_idx:
            tab = self.device.wait(pend.slot)
            pend.t_done = time.perf_counter()
            for row, i in zip(tab, pend.native_idx):
                if _native_deferred(row, self._bump):
                    continue
                out[i] = _row_to_result(row, "hip-native")
                self._bump("device_native", 1)
        rest = [i for i in range(n) if out[i] is None]
        if rest and defer_fallback:
            pend.fallback_idx = rest
            if self.fault_rate > 0:
                for i in range(n):
                    if out[i] is not None and self._fault_rng.random() < self.fault_rate:
                        out[i] = EvalResult(0.0, int(Exc.VALUE), "fault-injection")
                        self._bump("faults")
            return out
        if rest:
            sub = self._evaluate_compiled([pend.codes[i] for i in rest], [pend.compiled[i] for i in rest],
                                          native=False, slot=pend.slot)
            for i, r in zip(rest, sub):
                out[i] = r
        if self.fault_rate > 0:
            for i in range(n):
                if self._fault_rng.random() < self.fault_rate:
                    out[i] = EvalResult(0.0, int(Exc.VALUE), "fault-injection")
                    self._bump("faults")
        return out  # type: ignore[return-value]

    def collect_partial(self, pend: "PendingPrograms") -> Tuple[List[Tuple[int, EvalResult]], bool]:
        """Streaming `collect` (device program service, `DeviceEvaluator.
        service_take`): the (index, result) pairs of the batch's programs that
        finished since the last call, and whether the batch is complete; on
        completion the programs the device did not score are listed in
        ``pend.fallback_idx`` (for `fallback_async`)."""
        got: List[Tuple[int, EvalResult]] = []
        complete = True
        if pend.native_idx:
            pos, rows, complete = self.device.service_take(pend.slot)
            for j, row in zip(pos, rows):
                i = pend.native_idx[int(j)]
                if _native_deferred(row, self._bump):
                    pend.deferred_idx.append(i)
                    continue
                r = _row_to_result(row, "hip-native")
                if len(row) > len(COLS):
                    r.device_cycles = float(row[len(COLS)])
                self._bump("device_native", 1)
                if self.fault_rate > 0 and self._fault_rng.random() < self.fault_rate:
                    r = EvalResult(0.0, int(Exc.VALUE), "fault-injection")
                    self._bump("faults")
                got.append((i, r))
        if complete:
            pend.t_done = time.perf_counter()
            native = set(pend.native_idx or ())
            pend.fallback_idx = sorted([i for i in range(len(pend.codes)) if i not in native] + pend.deferred_idx)
        return got, complete

    def fallback_async(self, pend: "PendingPrograms", object_ok: bool = True):
        """Score ``pend.fallback_idx`` on the host engines (CPU VM, then
        CPython unless `object_ok` is False) in a worker thread; the future
        yields (indices, results)."""
        idx = list(pend.fallback_idx)
        codes = [pend.codes[i] for i in idx]
        compiled = [pend.compiled[i] for i in idx]
        with self._compile_lock:
            if getattr(self, "_fallback_pool", None) is None:
                from concurrent.futures import ThreadPoolExecutor
                nice = int(getattr(self, "fallback_nice", 0))

                def lower_priority():
                    # a host fallback (a CPU-VM replay: seconds of a core for a large
                    # program) yields the cores to the threads that keep the GPU fed;
                    # nice is per thread on Linux and the VM's worker threads inherit it
                    if nice > 0 and hasattr(os, "setpriority") and hasattr(threading, "get_native_id"):
                        try:
                            os.setpriority(os.PRIO_PROCESS, threading.get_native_id(), nice)
                        except OSError:
                            pass
                self._fallback_pool = ThreadPoolExecutor(max_workers=2, thread_name_prefix="fks-fallback",
                                                         initializer=lower_priority)

        def job():
            res = self._evaluate_compiled(codes, compiled, native=False, host_only=True, object_ok=object_ok)
            if self.fault_rate > 0:
                for k in range(len(res)):
                    with self._stats_lock:
                        hit = self._fallback_fault_rng.random() < self.fault_rate
                    if hit:
                        res[k] = EvalResult(0.0, int(Exc.VALUE), "fault-injection")
            return idx, res
        return self._fallback_pool.submit(job)

    def _object_pool(self):
        """Persistent spawn pool for CPython replays started from worker threads."""
        with self._compile_lock:
            if getattr(self, "_obj_pool", None) is None:
                import multiprocessing
                self._obj_pool = ProcessPoolExecutor(max_workers=max(1, self.object_workers),
                                                     mp_context=multiprocessing.get_context("spawn"))
                atexit.register(self._obj_pool.shutdown, wait=False, cancel_futures=True)
        return self._obj_pool

    def _absorb_native(self, idx, compiled, out, slot: int) -> None:
        batch = self.device.submit_native(slot, [compiled[i] for i in idx])
        self._bump("jit_s", batch.compile_s)
        self._bump("jit_shapes", batch.compiled)
        tab = self.device.wait(slot)
        for row, i in zip(tab, idx):
            if _native_deferred(row, self._bump):
                continue
            out[i] = _row_to_result(row, "hip-native")
            self._bump("device_native", 1)

    def _object_engine_ok(self) -> bool:
        # the object engine implements only the reference's semantics
        return (self.options.get("repush", "first") == "first"
                and self.options.get("gpu_alloc", "best_fit") == "best_fit"
                and float(self.options.get("snapshot_interval", 0.05)) == 0.05)

    def scores(self, codes: Sequence[str]) -> List[float]:
        return [r.score for r in self.evaluate_programs(codes)]


@dataclass
class PendingPrograms:
    """A program batch in flight on one device slot (`Evaluator.submit_programs`)."""
    codes: List[str]
    slot: int
    compiled: List[Optional[CompiledPolicy]] = field(default_factory=list)
    native_idx: List[int] = field(default_factory=list)
    jit_s: float = 0.0
    submit_s: float = 0.0
    new_shapes: int = 0
    prepared: object = None          # NativeBatch compiled ahead, not launched yet
    t_launch: float = 0.0
    t_done: float = 0.0
    fallback_idx: List[int] = field(default_factory=list)
    deferred_idx: List[int] = field(default_factory=list)   # device rows deferred to the host (collect_partial)


_default: Dict[str, Evaluator] = {}


def evaluate(codes, device="auto", workload: Optional[Workload] = None, **options) -> List[float]:
    """Scores of policy programs (one program text or a list of them).

    Compatible with the reference's fitness: identical to running
    `evaluate_policy_standalone` on each program (exception -> 0)."""
    single = isinstance(codes, str)
    codes = [codes] if single else list(codes)
    if workload is None and not options:
        key = str(device)
        ev = _default.get(key)
        if ev is None:
            ev = _default[key] = Evaluator(None, device)
    else:
        ev = Evaluator(workload, device, options)
    scores = ev.scores(codes)
    return scores[0] if single else scores


def evaluate_detailed(codes: Sequence[str], device="auto", workload: Optional[Workload] = None,
                      **options) -> List[EvalResult]:
    return Evaluator(workload, device, options).evaluate_programs(list(codes))


def copy_workload(w: Workload) -> Workload:
    return copy.deepcopy(w)
