"""Python front-end of the MI355X replay engine (``_fks_hip``).

`DeviceEvaluator` turns a `Workload` into the device layout (pods relabelled
by id rank, node / GPU state padded to 64-lane passes, the initial event heap
heapified once on the host with CPython's own ``heapq``), uploads it to HBM
once, and evaluates batches of policies -- built-in families (weights as
data) or compiled bytecode programs -- with one k_replay workgroup per
policy.

On a GPU box the extension must load: there is no silent CPU fallback here
(callers that want one use `engine.evaluate`, which routes explicitly).
"""

from __future__ import annotations

import bisect
import heapq
import math
import os
import threading
import time
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from ..core.arrays import Workload
from ..policy.compiler import CompiledPolicy
from .cpu_engine import DEFAULT_CALL_BUDGET, FAMILY, RESULT_COLUMNS  # noqa: F401  (same table layout)

GMAX = 8
WEIGHTS_PER_POLICY = 16
LDS_BYTES_PER_CU = 160 * 1024
VREG_BYTES = 64 * 8  # one VM register: 64 lanes x 8 B

_mod = None


def native():
    """Load ``_fks_hip`` (torch first, so the process shares torch's HIP runtime)."""
    global _mod
    if _mod is None:
        try:
            import torch  # noqa: F401
        except Exception:
            pass
        if os.environ.get("FKS_NO_AUTOBUILD") != "1":
            from .build import build_hip
            build_hip()
        from . import _fks_hip  # noqa: F401
        from .build import verify
        verify(_fks_hip, "hip")    # refuses a binary built from other sources
        _mod = _fks_hip
    return _mod


_MATH_OK: Optional[bool] = None


_MATH_INFO: Dict[str, object] = {}


def math_selfcheck_info() -> dict:
    """Outcome of `glibc_math_ok` (which math path this process uses), for logs
    and the bench record."""
    glibc_math_ok()
    return dict(_MATH_INFO, ok=bool(_MATH_OK))


def glibc_math_ok(n: int = 200_000) -> bool:
    """The device's exp / log / pow (csrc/hip/glibc_math.h, glibc's own FMA
    algorithms and tables) equal this host's libm -- the one CPython calls --
    on `n` arguments per function, and on a sample checked through Python's
    `math` itself.  Checked once per process.  False (another libm build, a
    host without FMA): programs that call them are kept off the device and
    replayed by the CPU VM, which calls the host libm (`DeviceEvaluator`)."""
    global _MATH_OK
    if _MATH_OK is None:
        import math
        import random
        m = native()
        r = m.glibc_math_selfcheck(n, 7)
        ok = r["exp"] == 0 and r["log"] == 0 and r["pow"] == 0
        rng = random.Random(3)
        xs = np.array([rng.uniform(-700, 700) for _ in range(2000)])
        ys = np.array([rng.uniform(1e-3, 1e3) for _ in range(2000)])
        zs = np.array([rng.uniform(-20, 20) for _ in range(2000)])
        ok = ok and np.array_equal(m.gm_exp_batch(xs)[1], [math.exp(x) for x in xs]) \
            and np.array_equal(m.gm_log_batch(ys)[1], [math.log(y) for y in ys]) \
            and all(o == y ** z for o, y, z in zip(m.gm_pow_batch(ys, zs)[1], ys, zs) if y ** z != float("inf"))
        if not ok:
            import warnings
            warnings.warn(f"device exp/log/pow differ from this host's libm ({r}); programs using them run on "
                          "the CPU VM", RuntimeWarning)
        _MATH_OK = bool(ok)
        _MATH_INFO.update(checked_per_function=n, mismatches={k: int(r[k]) for k in ("exp", "log", "pow")},
                          device_math=("glibc-exact (device exp/log/pow == host libm)" if ok else
                                       "host fallback (programs using exp/log/pow replay on the CPU VM)"))
    return _MATH_OK


def device_available() -> bool:
    try:
        return native().device_count() > 0
    except Exception:
        return False


class UnsupportedWorkload(ValueError):
    """The workload exceeds a device-layout limit (the CPU engine handles it)."""


def _bits(n: int) -> int:
    return max(1, int(math.ceil(math.log2(max(2, n)))))


def snapshot_schedule(total_events: int, interval: float = 0.05, count: int = 4096):
    """Processed-event counts at which the reference evaluator snapshots.

    Replays `evaluator.py:55-67` exactly: snapshot k fires at the first event
    count c after the previous snapshot with ``c / total >= thr_k`` (IEEE
    division, the same as Python's int/int), and ``thr`` advances by repeated
    ``+= interval``.  Returns (fire counts, threshold after the last one)."""
    fire = np.zeros(count, dtype=np.int64)
    thr, prev = interval, 0
    for k in range(count):
        c = max(prev + 1, int(thr * total_events) - 2)
        while c - 1 > prev and (c - 1) / total_events >= thr:
            c -= 1
        while c / total_events < thr:
            c += 1
        fire[k] = c
        prev = c
        thr += interval
    return fire, thr


def prepare_device_workload(w: Workload, snapshot_interval: float = 0.05) -> Dict[str, object]:
    c, p = w.cluster, w.pods
    N, P = c.n_nodes, p.n_pods
    if N == 0 or P == 0:
        raise UnsupportedWorkload("empty workload")
    if N > 256:
        raise UnsupportedWorkload("more than 256 nodes")
    if c.max_gpus_per_node > GMAX:
        raise UnsupportedWorkload(f"more than {GMAX} GPUs on a node")
    if c.gpu_milli_total.size and (c.gpu_milli_total.max() >= 2 ** 20 or c.gpu_milli_total.min() < 0):
        raise UnsupportedWorkload("GPU milli totals outside [0, 2^20) (32-bit per-node sums on device)")
    if c.gpu_milli_total.size:
        # the kernels hold one GPU milli total per node (NodeRegs::gmt1)
        owner = np.repeat(np.arange(N), np.diff(c.gpu_start))
        first = c.gpu_milli_total[c.gpu_start[owner]]
        if not np.array_equal(first, c.gpu_milli_total):
            raise UnsupportedWorkload("GPUs of one node with different milli totals")
    if len(np.unique(p.pod_rank)) != P:
        raise UnsupportedWorkload("duplicate pod ids")
    if P >= 2 ** 20:
        raise UnsupportedWorkload("more than 2^20 pods (heap depth > 20 levels)")
    for name, arr in (("cpu", c.node_cpu_total), ("mem", c.node_mem_total), ("pcpu", p.pod_cpu),
                      ("pmem", p.pod_mem), ("dur", p.pod_dur), ("ctime", p.pod_ctime)):
        if arr.size and (arr.max() >= 2 ** 31 or arr.min() < -(2 ** 31)):
            raise UnsupportedWorkload(f"{name} outside int32")
    if p.pod_ctime.min() < 0 or p.pod_dur.min() < 0:
        raise UnsupportedWorkload("negative times")
    if p.pod_gmilli.max(initial=0) >= 2 ** 16 or p.pod_gmilli.min(initial=0) < 0 \
            or p.pod_ngpu.max(initial=0) >= 2 ** 8 or p.pod_ngpu.min(initial=0) < 0:
        raise UnsupportedWorkload("gpu request outside the packed pod record")
    npass = 1 if N <= 64 else (2 if N <= 128 else 4)
    if npass == 4 and c.gpu_milli_total.size and c.gpu_milli_total.max() >= 2 ** 16:
        # > 128 nodes: two GPUs' milli left share a register (16-bit halves, NodeRegs::kPack)
        raise UnsupportedWorkload("GPU milli totals >= 2^16 on a > 128-node cluster")
    NP = 64 * npass

    def pad(a, dtype):
        out = np.zeros(NP, dtype=dtype)
        out[:N] = a
        return out

    gml_total = np.zeros((NP, GMAX), dtype=np.int32)
    gml_left = np.zeros((NP, GMAX), dtype=np.int32)
    gmem_total = np.zeros((NP, GMAX), dtype=np.int64)
    for i in range(N):
        a, b = int(c.gpu_start[i]), int(c.gpu_start[i + 1])
        gml_total[i, :b - a] = c.gpu_milli_total[a:b]
        gml_left[i, :b - a] = c.gpu_milli_left[a:b]
        gmem_total[i, :b - a] = c.gpu_mem_total[a:b]

    gpu_pods = p.pod_ngpu > 0
    classes = np.unique(p.pod_gmilli[gpu_pods]).astype(np.int32)
    if classes.size > 256:
        raise UnsupportedWorkload("more than 256 distinct gpu_milli requests")
    if classes.size == 0:
        classes = np.zeros(1, dtype=np.int32)
    cls = np.searchsorted(classes, p.pod_gmilli).astype(np.int64)
    cls[~gpu_pods] = 0

    order = np.argsort(p.pod_rank, kind="stable")           # by rank
    rec = np.zeros((P, 4), dtype=np.int32)
    rec[:, 0] = p.pod_cpu[order]
    rec[:, 1] = p.pod_mem[order]
    rec[:, 2] = p.pod_dur[order]
    rec[:, 3] = (p.pod_gmilli[order].astype(np.int64) | (p.pod_ngpu[order].astype(np.int64) << 16)
                 | (cls[order] << 24)).astype(np.int64).astype(np.uint32).view(np.int32)

    rank_bits, node_bits = _bits(P), _bits(N)
    low_bits = 2 + node_bits + GMAX
    time_bits = 64 - rank_bits - low_bits
    if int(p.pod_ctime.max()) + int(p.pod_dur.max()) >= 2 ** min(time_bits, 62):
        raise UnsupportedWorkload("times exceed the packed key")
    items = [(int(t), int(r)) for t, r in zip(p.pod_ctime, p.pod_rank)]
    heapq.heapify(items)   # CPython's heapify on (time, rank): the reference's initial layout
    heap0 = np.array([(t << (rank_bits + low_bits)) | (r << low_bits) for t, r in items], dtype=np.uint64)

    used = dict(
        used_cpu=int((c.node_cpu_total - c.node_cpu_left).sum()),
        used_mem=int((c.node_mem_total - c.node_mem_left).sum()),
        used_gcnt=int((c.node_ngpus.astype(np.int64) - c.node_gpu_left).sum()),
        used_gmilli=int((c.gpu_milli_total.astype(np.int64) - c.gpu_milli_left).sum()),
    )
    fire, thr_after = snapshot_schedule(P, snapshot_interval)
    return dict(
        snap_fire=fire, thr_after_fire=float(thr_after),
        n_nodes=N, n_pods=P, n_classes=int(classes.size), npass=npass,
        cpu_total=pad(c.node_cpu_total, np.int32), cpu_left=pad(c.node_cpu_left, np.int32),
        mem_total=pad(c.node_mem_total, np.int32), mem_left=pad(c.node_mem_left, np.int32),
        gpu_left=pad(c.node_gpu_left, np.int32), ngpus=pad(c.node_ngpus, np.int32),
        gml_total=gml_total, gml_left=gml_left, gmem_total=gmem_total,
        pod=rec, pod_ctime=p.pod_ctime[order].astype(np.int32), heap0=heap0, class_value=classes,
        tot_cpu=int(c.node_cpu_total.sum()), tot_mem=int(c.node_mem_total.sum()),
        tot_gcnt=int(c.node_ngpus.sum()), tot_gmilli=int(c.gpu_milli_total.astype(np.int64).sum()),
        rank_bits=rank_bits, node_bits=node_bits, low_bits=low_bits, time_bits=time_bits, **used,
    )


def pack_programs(progs: Sequence[CompiledPolicy]):
    """Concatenate bytecode + constant pools for one device launch."""
    codes, offsets, lengths, kpay, koff, ktag = [], [], [], [], [], []
    pos = kpos = 0
    for prg in progs:
        offsets.append(pos)
        lengths.append(prg.n_insns)
        koff.append(kpos)
        codes.append(prg.code)
        pos += prg.n_insns
        for f, i, t in zip(prg.fconst, prg.iconst, prg.ctag):
            kpay.append(int(np.array(f, dtype=np.float64).view(np.int64)) if t == 1 else int(i))
            ktag.append(t)
        kpos += len(prg.ctag)
    return (b"".join(codes), np.array(offsets, np.int32), np.array(lengths, np.int32),
            np.array(kpay or [0], np.int64), np.array(koff, np.int32), np.array(ktag or [0], np.uint8))


class DeviceEvaluator:
    """A workload resident on one MI355X, evaluating policy batches."""

    def __init__(self, workload: Workload, device: int = 0, options: Optional[dict] = None, n_slots: int = 4):
        self.workload = workload
        self.device = device
        options = dict(options or {})
        interval = float(options.get("snapshot_interval", 0.05))
        self.layout = prepare_device_workload(workload, interval)
        self._eng = native().DeviceEngine(self.layout, device, n_slots)
        options["snapshot_interval"] = interval
        options.setdefault("budget", DEFAULT_CALL_BUDGET)
        self._eng.set_options(options)
        self.options = options

        self._jit = None
        self._jit_lock = threading.Lock()
        self._native_post: Dict[int, Tuple[int, np.ndarray]] = {}   # slot -> (P, native row indices)
        #: device exp / log / pow == host libm (else programs using them stay on the host)
        self.math_exact = glibc_math_ok()
        self._native_mods: Dict[int, tuple] = {}   # slot -> JIT modules its batch in flight calls into
        #: the resident program service (start_service): slot -> (P, native rows, first ring index)
        self._svc: Optional[dict] = None
        self._svc_post: Dict[int, Tuple[int, np.ndarray, int, np.ndarray]] = {}   # slot -> (P, rows, first, data slots)
        self._svc_taken: Dict[int, list] = {}   # slot -> [rows taken, declined rows reported] (service_take)
        self._svc_firsts: List[int] = []         # first index of every batch in flight (sorted) ...
        self._svc_keys: List[int] = []           # ... and its slot key
        self._svc_buf: Dict[int, list] = {}      # slot key -> [(offset, row)] polled, not taken yet
        self._svc_pumped = 0.0
        self._svc_orphans = 0                   # rows of forgotten batches (dropped)
        self._svc_lock = threading.Lock()

    def info(self) -> dict:
        d = dict(self._eng.info())
        if self._svc is not None:
            d["service"] = dict(self._eng.service_info())
        return d

    # -- resident program service (csrc/hip/replay_duo.hip.h native_service) ---------------
    #: slot ids of the service's callers start here (the engine's own stream
    #: slots, e.g. the family coupler's, stay below)
    SERVICE_SLOT_BASE = 64

    def start_service(self, slots: int = 16384, share: float = 1.0, idle_polls: int = 1 << 24) -> dict:
        """Launch the resident two-wave grid: from now on every native program
        batch (`submit_native`, any slot) is queued to it instead of launched
        as a kernel of its own, and a batch's `ready` / `wait` follow its own
        programs only -- a slow program no longer holds a launch's CU slots
        while the rest of them idle.  share: fraction of the two-wave kernel's
        resident capacity the grid takes (the rest stays free for other
        streams' kernels, e.g. the family coupler's row-kernel batches);
        slots: programs queued or running at most; idle_polls: polls with
        nothing published after which the whole grid drains (it is relaunched
        from the first unstarted program when more arrive)."""
        if self._svc is not None:
            return dict(self._svc)
        self.warm_native()
        nc = self.native_compiler
        # retired modules are parked (an unload would wait for the grid) until
        # stop_service; the steady search bounds them by rolling the grid over
        nc.defer_unloads = True
        self._svc = dict(self._eng.service_start(int(slots), float(share), int(idle_polls)))
        if not getattr(self, "_svc_atexit", False):
            # a grid left running at interpreter exit would hold every later
            # device-wide synchronisation (JIT module teardown) until its idle timeout
            import atexit
            import weakref
            ref = weakref.ref(self)
            atexit.register(lambda: ref() is not None and ref()._eng.service_stop())
            self._svc_atexit = True
        return dict(self._svc)

    def abort_service(self) -> None:
        """Replays in flight on the service end within ~1k events (their rows
        come back EXC_TIMEOUT, deferred like any timeout): for a run that is
        stopping and does not need them."""
        if self._svc is not None:
            self._eng.service_abort()

    def stop_service(self) -> None:
        """Drain and end the resident grid (batches still queued are waited for)."""
        if self._svc is None:
            return
        for slot in list(self._svc_post):
            self.wait(slot)
        self._eng.service_stop()
        self._svc = None
        nc = self.native_compiler
        nc.defer_unloads = False
        nc.flush_unloads()

    @property
    def service(self) -> Optional[dict]:
        return self._svc

    def warm_native(self) -> float:
        """First-use initialisation of the native program path -- the JIT's
        code-object skeleton load and layout probe, the first module load and
        launch -- done once, outside any measured batch; returns its seconds
        (0 when already done)."""
        if getattr(self, "_warm_s", None) is not None:
            return 0.0
        from ..models.library import reference_policies
        from ..policy.compiler import compile_policy
        t0 = time.perf_counter()
        prog = compile_policy(reference_policies()["first_fit"])
        self.submit_native(0, [prog])
        self.wait(0)
        bj = getattr(self.native_compiler, "_baseline", None)
        if bj is not None:
            from .gcnjit import compile_program
            code, _ = compile_program(prog)
            if code is not None:
                bj.verify_all(code)   # every code-object skeleton size, before replays fill the chip
        self._warm_s = time.perf_counter() - t0
        return self._warm_s

    # -- natively compiled programs (policy/native_codegen.py, ops/jit.py) ------------------
    @property
    def native_compiler(self):
        # Created once, under a lock: island threads submit their first batches
        # concurrently, and a second compiler instance would replace the first
        # one -- whose JIT modules (hipModuleUnload on collection) the first
        # thread's kernels are still executing.
        if self._jit is None:
            with self._jit_lock:
                if self._jit is None:
                    from .jit import NativeCompiler
                    self._jit = NativeCompiler(self._eng, self.device,
                                               budget=int(self.options.get("budget") or DEFAULT_CALL_BUDGET))
        return self._jit

    def prepare_native(self, progs: Sequence[CompiledPolicy]):
        """The compile half of `submit_native` (any thread): JIT-compile and load
        the shapes `progs` need and hold their modules.  The `NativeBatch` is then
        launched with `submit_native(slot, progs, batch)` or handed back with
        `release_native(batch)`."""
        batch = self.native_compiler.prepare(progs)
        if not self.math_exact:
            for i, p in enumerate(progs):
                if batch.ok[i] and p.uses_libm:
                    batch.ok[i] = False
                    batch.reasons[i] = "exp / log / pow: device math differs from this host's libm"
        return batch

    def release_native(self, batch) -> None:
        """A prepared batch that will not be launched."""
        self.native_compiler.release(batch.modules)

    def submit_native(self, slot: int, progs: Sequence[CompiledPolicy], batch=None):
        """Compile (shape-cached) and launch one k_replay_native wave per program on
        `slot`.  Programs the native backend cannot take (codegen / register limits)
        get an EXC_UNSUPPORTED row from `wait`, so callers fall back per program.
        `batch`: the result of `prepare_native(progs)` (compiled ahead on another
        thread).  Returns the `NativeBatch` (compile time, cache hits, reasons)."""
        if batch is None:
            batch = self.prepare_native(progs)
        idx = np.flatnonzero(batch.ok)
        prev = self._native_mods.pop(slot, None)
        if prev:    # a batch never waited for (the engine waits for it before restaging)
            self.native_compiler.release(prev)
        dump = os.environ.get("FKS_DUMP_BATCHES")
        if dump and idx.size:
            # diagnostics: every native launch's program texts, written before the launch
            import json
            with open(dump, "a") as f:
                f.write(json.dumps({"slot": slot, "t": time.time(), "P": int(idx.size),
                                    "codes": [progs[i].source for i in idx]}) + "\n")
        try:
            if self._svc is not None:
                with self._svc_lock:   # (indexes and their registration in one step: the list stays sorted)
                    if slot in self._svc_post:
                        raise RuntimeError(f"service slot {slot} still holds a batch")
                    first, dslots = -1, np.zeros(0, np.int32)
                    if idx.size:
                        first, dslots = self._eng.service_submit(batch.fn[idx], batch.kc, batch.koff[idx])
                        if first < 0:
                            held = sorted((v[2], v[1].size, k) for k, v in self._svc_post.items() if v[1].size)
                            raise RuntimeError(
                                f"program service full ({int(idx.size)} programs): batches held (first, n, slot) "
                                f"{held[:8]}, service {dict(self._eng.service_info())}")
                    self._svc_post[slot] = (len(progs), idx, first, np.asarray(dslots, np.int32))
                    if idx.size:
                        self._svc_firsts.append(int(first))
                        self._svc_keys.append(slot)
                    self._native_mods[slot] = batch.modules
                return batch
            else:
                self._native_post[slot] = (len(progs), idx)
                if idx.size:
                    self._eng.submit_native(slot, batch.fn[idx], batch.kc, batch.koff[idx])
        except BaseException:
            self.native_compiler.release(batch.modules)
            raise
        self._native_mods[slot] = batch.modules   # released once the batch is collected
        return batch

    def profile_native(self, progs: Sequence[CompiledPolicy]):
        """s_memtime phase-profiled native row-kernel launch: (table [P, 13], wave
        cycles [waves, 8] by ROW_PHASES); programs must all be native-compilable."""
        batch = self.native_compiler.prepare(progs)
        try:
            if not batch.ok.all():
                raise ValueError(f"not native: {batch.reasons}")
            return self._eng.profile_native(batch.fn, batch.kc, batch.koff)
        finally:
            self.native_compiler.release(batch.modules)

    def evaluate_native(self, progs: Sequence[CompiledPolicy]) -> np.ndarray:
        if not progs:
            return np.zeros((0, len(RESULT_COLUMNS)))
        self.submit_native(0, progs)
        return self.wait(0)

    def set_options(self, **opts) -> None:
        if "snapshot_interval" in opts and opts["snapshot_interval"] != self.options["snapshot_interval"]:
            raise ValueError("snapshot_interval is baked into the device schedule; build a new DeviceEvaluator")
        self.options.update(opts)
        self._eng.set_options(opts)

    @staticmethod
    def _builtin_args(family, weights, n=None):
        if isinstance(family, str):
            count = n if n is not None else (len(weights) if weights is not None else 1)
            fam = np.full(count, FAMILY[family], dtype=np.int32)
        else:
            fam = np.array([FAMILY[f] for f in family], dtype=np.int32)
        W = np.zeros((len(fam), WEIGHTS_PER_POLICY), dtype=np.float64)
        if weights is not None:
            weights = np.asarray(weights, dtype=np.float64).reshape(len(fam), -1)
            W[:, :weights.shape[1]] = weights
        return fam, W

    def evaluate_builtin(self, family: "str | Sequence[str]", weights: Optional[np.ndarray] = None,
                         n: Optional[int] = None) -> np.ndarray:
        return self._eng.evaluate_builtin(*self._builtin_args(family, weights, n))

    # -- asynchronous slots: several batches in flight on separate HIP streams --------------
    @property
    def n_slots(self) -> int:
        return self._eng.n_slots()

    def submit_builtin(self, slot: int, family: str, weights: np.ndarray) -> None:
        """Start a batch on `slot` (its own stream); returns immediately."""
        self._eng.submit_builtin(slot, *self._builtin_args(family, weights))

    def submit_programs(self, slot: int, progs: Sequence[CompiledPolicy]) -> None:
        self._eng.submit_programs(slot, *pack_programs(progs), max(p.nregs for p in progs))

    def wait(self, slot: int) -> np.ndarray:
        """[P, 13] result table of the batch in flight on `slot`."""
        if slot in self._svc_post:
            return self._service_wait(slot)
        post = self._native_post.pop(slot, None)
        if post is None:
            return self._eng.wait(slot)
        P, idx = post
        out = np.zeros((P, len(RESULT_COLUMNS)))
        out[:, 10] = 100.0   # EXC_UNSUPPORTED: not native -> the caller's next engine
        try:
            if idx.size:
                out[idx] = self._eng.wait(slot)
        finally:
            mods = self._native_mods.pop(slot, None)
            if mods:
                self.native_compiler.release(mods)
        return out

    #: seconds between two scans of the service's done flags (`_service_pump`)
    SERVICE_POLL_S = 0.001
    #: a whole-batch wait on the service gives up (with the service's state)
    #: after this long: the replay instruction budget ends any program long before
    SERVICE_WAIT_S = float(os.environ.get("FKS_SERVICE_WAIT_S", "900"))

    def _service_pump(self, min_interval_s: Optional[float] = None) -> None:
        """One `service_poll` (every finished program, all batches) at most
        every `min_interval_s`; rows are filed under their batches.  (Caller
        holds `_svc_lock`: island / coupler threads collect concurrently.)"""
        now = time.perf_counter()
        if now - self._svc_pumped < (self.SERVICE_POLL_S if min_interval_s is None else min_interval_s):
            return
        self._svc_pumped = now
        ids, rows, cyc = self._eng.service_poll()
        if not len(ids):
            return
        # rows carry the replay's device cycles as a 14th column (SERVICE_COST_COL)
        rows = np.concatenate([rows, np.asarray(cyc, np.float64).reshape(-1, 1)], axis=1)
        firsts = self._svc_firsts
        for k, ix in enumerate(ids.tolist()):
            j = bisect.bisect_right(firsts, ix) - 1
            key = self._svc_keys[j] if j >= 0 else None
            post = self._svc_post.get(key) if key is not None else None
            # a row of a batch that was forgotten before all its rows arrived
            # (an interrupted wait) bisects into the batch before it: it lies
            # past that batch's programs and is dropped, never filed under it
            if post is None or ix - firsts[j] >= post[1].size:
                self._svc_orphans += 1
                continue
            self._svc_buf.setdefault(key, []).append((ix - firsts[j], rows[k]))

    #: column of service_take rows holding the replay's device cycles (s_memtime
    #: from claim to result; 0 for rows the device did not replay)
    SERVICE_COST_COL = len(RESULT_COLUMNS)

    def service_take(self, slot: int):
        """Streaming collection from the program service: (positions, rows) of
        the programs of `slot`'s batch that finished since the last call
        (positions index the batch as submitted; programs the JIT declined come
        on the first call with EXC_UNSUPPORTED rows), and whether the batch is
        now complete (its modules released, the slot free).  Rows have the
        result columns plus the replay's device cycles (`SERVICE_COST_COL`)."""
        with self._svc_lock:
            P, idx, first, _ = self._svc_post[slot]
            taken = self._svc_taken.setdefault(slot, [0, False])
            pos_parts, row_parts = [], []
            if not taken[1]:
                taken[1] = True
                if idx.size < P:
                    rest = np.setdiff1d(np.arange(P), idx)
                    r = np.zeros((rest.size, len(RESULT_COLUMNS) + 1))
                    r[:, 10] = 100.0
                    pos_parts.append(rest)
                    row_parts.append(r)
            if idx.size:
                self._service_pump()
                got = self._svc_buf.pop(slot, None)
                if got:
                    pos_parts.append(idx[np.array([o for o, _ in got])])
                    row_parts.append(np.array([r for _, r in got]))
                    taken[0] += len(got)
            complete = taken[0] >= idx.size
            if complete:
                self._service_forget(slot)
        if not pos_parts:
            return np.zeros(0, np.int64), np.zeros((0, len(RESULT_COLUMNS) + 1)), complete
        return np.concatenate(pos_parts), np.concatenate(row_parts), complete

    def service_news(self) -> set:
        """After one scan of the done flags: the slots whose batches have
        something to take -- finished rows, or a first take still due (the
        rows of programs the device does not replay) -- so a caller with dozens
        of batches in flight visits only those."""
        with self._svc_lock:
            self._service_pump()
            news = set(self._svc_buf)
            news.update(s for s in self._svc_post if s not in self._svc_taken)
        return news

    def _service_forget(self, slot: int) -> None:
        P, idx, first, _ = self._svc_post.pop(slot)
        self._svc_taken.pop(slot, None)
        self._svc_buf.pop(slot, None)
        if idx.size:
            j = bisect.bisect_left(self._svc_firsts, first)
            del self._svc_firsts[j], self._svc_keys[j]
        mods = self._native_mods.pop(slot, None)
        if mods:
            self.native_compiler.release(mods)

    def _service_wait(self, slot: int) -> np.ndarray:
        """Whole-batch collection (`wait` on a service slot)."""
        P, idx, _, _ = self._svc_post[slot]
        out = np.zeros((P, len(RESULT_COLUMNS)))
        out[:, 10] = 100.0
        t0 = time.perf_counter()
        try:
            while idx.size:
                with self._svc_lock:
                    self._service_pump(0.0)
                    got = self._svc_buf.get(slot, [])
                    if len(got) >= idx.size:
                        for o, r in got:
                            out[idx[o]] = r[:len(RESULT_COLUMNS)]
                        break
                if time.perf_counter() - t0 > self.SERVICE_WAIT_S:
                    raise TimeoutError(f"program service: batch on slot {slot} incomplete after "
                                       f"{self.SERVICE_WAIT_S:.0f} s ({len(got)} of {idx.size} rows), "
                                       f"service {dict(self._eng.service_info())}")
                time.sleep(0.0002)
        finally:
            with self._svc_lock:
                self._service_forget(slot)
        return out

    def ready(self, slot: int) -> bool:
        svc = self._svc_post.get(slot)
        if svc is not None:
            # (whole batches: callers of ready() / wait() do not use service_take)
            with self._svc_lock:
                self._service_pump()
                return len(self._svc_buf.get(slot, ())) >= svc[1].size
        post = self._native_post.get(slot)
        if post is not None and post[1].size == 0:
            return True
        return self._eng.ready(slot)

    def evaluate_programs(self, progs: Sequence[CompiledPolicy], slot: Optional[int] = None) -> np.ndarray:
        """Device bytecode VM.  With `slot`, the batch runs on that slot's
        stream and buffers (callers in island worker threads pass their own
        slot, so two threads never stage into one slot)."""
        if not progs:
            return np.zeros((0, len(RESULT_COLUMNS)))
        if slot is not None:
            self.submit_programs(slot, progs)
            return self.wait(slot)
        nregs = max(p.nregs for p in progs)
        return self._eng.evaluate_programs(*pack_programs(progs), nregs)

    PHASES = ("pop", "delete", "score", "fail", "commit", "eval")

    def profile_builtin(self, family: str, weights: np.ndarray):
        """(result table, per-policy cycle counts [P, 8] by PHASES)."""
        fam = np.full(len(weights), FAMILY[family], dtype=np.int32)
        W = np.zeros((len(fam), WEIGHTS_PER_POLICY), dtype=np.float64)
        W[:, :np.asarray(weights).shape[1]] = weights
        return self._eng.profile(fam, W, None)

    ROW_PHASES = ("pop", "delete", "score", "fail", "commit", "eval", "next_policy")

    def profile_rows(self, family: str, weights: np.ndarray):
        """Row kernel, s_memtime build: (result table, per-wave cycles [waves, 8] by ROW_PHASES)."""
        return self._eng.profile_rows(*self._builtin_args(family, weights))

    def profile_programs(self, progs: Sequence[CompiledPolicy]):
        packed = pack_programs(progs) + (max(p.nregs for p in progs),)
        return self._eng.profile(None, None, packed)

    def stage_builtin_only(self, family: str, weights: np.ndarray) -> None:
        """Stage a batch on slot 0 for repeated timing launches (tools/)."""
        self._eng.stage_builtin_only(*self._builtin_args(family, weights))

    def launch_builtin_async(self) -> None:
        self._eng.launch_builtin_async()

    def synchronize(self) -> None:
        self._eng.synchronize()
