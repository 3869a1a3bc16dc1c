"""Run-time compiler of policy programs for the MI355X (native program backend).

Two tiers (``FKS_JIT_TIER`` / ``NativeCompiler(tier=...)``):

* ``baseline`` -- `ops.gcnjit`: bytecode -> gfx950 machine code generated in
  C++ without LLVM (~0.1-0.3 ms per program), a whole batch patched into one
  code-object skeleton and loaded with ``hipModuleLoadData``;
* ``llvm`` -- the pipeline below (~140 ms of clang + llc per program);
* ``auto`` -- baseline for every new shape, LLVM only for the shapes the
  baseline generator declines.

The default is ``baseline``: on the device, LLVM-tier code for a few evolved
programs (small float powers among GPU-list loops) gave rows that differ from
the CPU VM -- 9 of the first 256 evolved children at -O3, 1 at -O1 -- while the
host build of the same generated source and the baseline tier agree on all
of them.  Shapes the baseline declines (~0.1%) go to the host engines.

LLVM-tier pipeline per batch of new program *shapes* (bytecode + constant tags;
the constants themselves are data, `policy.native_codegen`):

  native_codegen.module_source  ->  clang -O3 -emit-llvm (gfx950, device
  only, no HIP headers, no device libraries)  ->  ``"amdgpu-agpr-alloc"="0"``
  on every function  ->  llc -O3  ->  resource check from the assembly's
  per-function ``.set <fn>.num_vgpr / numbered_sgpr / private_seg_size``
  symbols  ->  llvm-mc + ld.lld  ->  code object  ->
  ``_fks_hip.JitModule`` (hipModuleLoadData; the module's ``fks_rt_table``
  gets the extension's runtime-library addresses; ``fks_jit_table`` reports
  every program's device address).

The replay kernel (`k_replay_native`, csrc/hip/replay_kernels.hip) calls a
program through its address with an ordinary indirect call, so a compile never
touches the replay loop.  The caller allocates `JIT_VGPRS` / `JIT_SGPRS`
registers (its register floor); a program whose own use exceeds them, or whose
stack frame would not fit the dynamic stack, is reported unsupported and
evaluated by the VM / CPU engines instead.

Compiles of independent module chunks run in parallel subprocesses (the
clang processes release the GIL; at most 16 / ``LOCAL_WORLD_SIZE`` per rank),
every compiled shape is cached for the life of the process, so re-evaluating a
program -- or any program that differs from a compiled one only in its numeric
constants -- costs no compile at all, and LLVM-tier code objects persist in an
on-disk cache (``FKS_JIT_CACHE``, default ``~/.cache/fks_jit``; key: module
source + flags + toolchain identity) shared by the ranks of a host and by
``torchrun --max-restarts`` rounds.  In the ``auto`` tier a shape used in
``FKS_JIT_TIERUP`` batches (default 0: off) is recompiled by LLVM in a
background thread and swapped in when loaded (tier-up); no batch ever waits
for it.
"""

from __future__ import annotations

import math
import os
import re
import subprocess
import tempfile
import threading
import time
from concurrent.futures import ThreadPoolExecutor
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from .._paths import CSRC_DIR
from ..policy.compiler import CompiledPolicy
from ..policy.native_codegen import CodegenError, constant_blocks, module_source, shape_key

ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
CLANG = os.path.join(ROCM, "lib", "llvm", "bin", "clang")
LLD = os.path.join(ROCM, "lib", "llvm", "bin", "ld.lld")
LLC = os.path.join(ROCM, "lib", "llvm", "bin", "llc")
LLVM_MC = os.path.join(ROCM, "lib", "llvm", "bin", "llvm-mc")
_ATTR_RE = re.compile(r"^(attributes #\d+ = \{)", re.M)
ARCH = os.environ.get("FKS_OFFLOAD_ARCH", "gfx950")
JIT_INCLUDE = str(CSRC_DIR / "hip")
#: clang's optimisation level for generated programs (llc always runs -O3);
#: FKS_JIT_OPT overrides it for A/B runs
JIT_CLANG_OPT = os.environ.get("FKS_JIT_OPT", "-O3")
DEVICE_FLAGS = ["-x", "hip", "--offload-device-only", "-nogpulib", "-nogpuinc", JIT_CLANG_OPT, f"--offload-arch={ARCH}",
                "-std=c++17", "-DFKS_JIT", "-ffp-contract=off", "-fno-fast-math", "-Wno-unused-label",
                "-Wno-tautological-compare", f"-I{JIT_INCLUDE}"]
#: the runtime library's worst frame (fks_rt_binop/unop, measured from the
#: extension's assembly: <= 48 B) plus the replay kernel's call-site spills
RT_FRAME_BYTES = 256
STACK_LIMIT_BYTES = 1024   # HIP's default per-lane stack for dynamic-stack kernels


#: FKS_FEAS_SKIP=0 calls every program for every node (A/B of the feasibility-prologue skip)
_FEAS_SKIP = os.environ.get("FKS_FEAS_SKIP", "1") != "0"


def _shape_key(p) -> str:
    """The code cache key: shape_key, plus a mark when the baseline tier
    compiles the program's feasibility prologue out (gcnjit.elide_range) --
    that code is only valid where the kernels skip infeasible nodes, i.e. for
    programs whose function-table entry carries the prologue bit."""
    v = p.__dict__.get("_jit_key")
    if v is None:
        from .gcnjit import elide_range
        k = shape_key(p)
        v = p.__dict__["_jit_key"] = k + ":fp" if elide_range(p)[1] else k
    return v


def launch_key(p) -> str:
    """`_shape_key`, cached on the program: the producer processes of the steady
    search compute it (and the constant payload) before a child is pickled to
    the dispatcher, so the stager's per-program work is a dictionary lookup."""
    from ..policy.native_codegen import constant_payload
    constant_payload(p)
    return _shape_key(p)


class JitError(RuntimeError):
    """The toolchain failed on a module (a bug, not an unsupported program)."""


@dataclass
class Resources:
    vgprs: int = 0
    agprs: int = 0
    sgprs: int = 0
    private: int = 0

    def fits(self, vgpr_cap: int, sgpr_cap: int) -> Optional[str]:
        if self.vgprs > vgpr_cap:
            return f"{self.vgprs} VGPRs > {vgpr_cap}"
        if self.agprs:
            return f"uses {self.agprs} AGPRs"
        if self.sgprs > sgpr_cap:
            return f"{self.sgprs} SGPRs > {sgpr_cap}"
        if self.private + RT_FRAME_BYTES > STACK_LIMIT_BYTES:
            return f"{self.private} B stack frame"
        return None


_SET_RE = re.compile(r"^\s*\.set\s+(?:\.L)?(fks_prog_\d+)\.(num_vgpr|num_agpr|numbered_sgpr|private_seg_size),\s*(.+)$")


def _first_int(expr: str) -> int:
    """Own count of a resource symbol: ``max(52, amdgpu.max_num_vgpr)`` -> 52."""
    m = re.search(r"-?\d+", expr)
    return int(m.group(0)) if m else 0


def function_resources(asm: str) -> Dict[str, Resources]:
    out: Dict[str, Resources] = {}
    for line in asm.splitlines():
        m = _SET_RE.match(line)
        if not m:
            continue
        r = out.setdefault(m.group(1), Resources())
        v = _first_int(m.group(3))
        key = m.group(2)
        if key == "num_vgpr":
            r.vgprs = v
        elif key == "num_agpr":
            r.agprs = v
        elif key == "numbered_sgpr":
            r.sgprs = v
        else:
            r.private = v
    return out


@dataclass
class CompiledModule:
    image: bytes
    n: int
    resources: List[Optional[Resources]]
    compile_s: float
    handle: object = None            # _fks_hip.JitModule once loaded
    pointers: Optional[np.ndarray] = None
    cached: bool = False             # image came from the on-disk cache


#: wall-clock limit of one toolchain process (a pathological program must not
#: stall an island forever; the shape is then marked non-native)
TOOL_TIMEOUT_S = float(os.environ.get("FKS_JIT_TIMEOUT", "120"))


def _run(cmd: List[str], what: str) -> None:
    try:
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=TOOL_TIMEOUT_S)
    except subprocess.TimeoutExpired as exc:
        raise JitError(f"{what} timed out after {TOOL_TIMEOUT_S:.0f} s") from exc
    if r.returncode != 0:
        raise JitError(f"{what} failed ({r.returncode}): {r.stderr[-4000:]}")


def _cache_dir() -> Optional[str]:
    """On-disk code-object cache shared by every rank and every restart on a
    host (``FKS_JIT_CACHE``; ``off`` disables it)."""
    d = os.environ.get("FKS_JIT_CACHE", "")
    if d.lower() in ("off", "0", "none"):
        return None
    return d or os.path.join(os.environ.get("XDG_CACHE_HOME") or os.path.expanduser("~/.cache"), "fks_jit")


_TOOL_ID: Optional[str] = None


def _toolchain_id() -> str:
    """Identity of the LLVM toolchain (its binaries' size + mtime): a ROCm
    upgrade invalidates the cache."""
    global _TOOL_ID
    if _TOOL_ID is None:
        parts = []
        for t in (CLANG, LLC, LLVM_MC, LLD):
            try:
                st = os.stat(t)
                parts.append(f"{os.path.basename(t)}:{st.st_size}:{int(st.st_mtime)}")
            except OSError:
                parts.append(f"{os.path.basename(t)}:missing")
        _TOOL_ID = ";".join(parts)
    return _TOOL_ID


def _cache_key(src: str) -> str:
    import hashlib
    h = hashlib.sha256()
    for part in (src, " ".join(DEVICE_FLAGS), ARCH, _toolchain_id(), "v1"):
        h.update(part.encode("utf-8"))
        h.update(b"\0")
    return h.hexdigest()


def _cache_load(key: str, n: int) -> Optional[CompiledModule]:
    d = _cache_dir()
    if d is None:
        return None
    import json
    try:
        with open(os.path.join(d, key + ".json")) as f:
            meta = json.load(f)
        with open(os.path.join(d, key + ".co"), "rb") as f:
            image = f.read()
    except (OSError, ValueError):
        return None
    if meta.get("n") != n or len(image) != meta.get("bytes"):
        return None
    import hashlib
    if meta.get("sha256") != hashlib.sha256(image).hexdigest():
        return None    # corrupted / replaced image (the directory is shared): a miss, recompile
    res = [Resources(**r) if r is not None else None for r in meta["resources"]]
    return CompiledModule(image, n, res, 0.0, cached=True)


def _cache_store(key: str, mod: CompiledModule) -> None:
    """Atomic (tmp + rename): concurrent ranks writing the same key is harmless."""
    d = _cache_dir()
    if d is None:
        return
    import hashlib
    import json
    from dataclasses import asdict
    try:
        os.makedirs(d, exist_ok=True)
        for ext, data, mode in ((".co", mod.image, "wb"),
                                (".json", json.dumps({"n": mod.n, "bytes": len(mod.image),
                                                      "sha256": hashlib.sha256(mod.image).hexdigest(), "resources": [
                                    asdict(r) if r is not None else None for r in mod.resources]}), "w")):
            tmp = os.path.join(d, f".{key}{ext}.{os.getpid()}.{threading.get_ident()}")
            with open(tmp, mode) as f:
                f.write(data)
            os.replace(tmp, os.path.join(d, key + ext))   # the .json lands last: a reader sees both or neither
    except OSError:
        pass    # read-only home etc.: the cache is an optimisation


def compile_device_module(progs: Sequence[CompiledPolicy], workdir: Optional[str] = None) -> CompiledModule:
    """gfx950 code object holding ``fks_prog_<i>`` for every program (from
    the on-disk cache when this exact module was built before)."""
    t0 = time.perf_counter()
    src = module_source(progs, with_probes=False)
    key = _cache_key(src)
    hit = _cache_load(key, len(progs))
    if hit is not None:
        hit.compile_s = time.perf_counter() - t0
        return hit
    with tempfile.TemporaryDirectory(prefix="fksjit_", dir=workdir) as d:
        cpp, ll, asm, obj, co = (os.path.join(d, n) for n in ("m.hip", "m.ll", "m.s", "m.o", "m.co"))
        with open(cpp, "w") as f:
            f.write(src)
        _run([CLANG, *DEVICE_FLAGS, "-S", "-emit-llvm", cpp, "-o", ll], "clang -emit-llvm")
        # No accumulation registers anywhere in JIT code: the calling replay
        # kernel's AGPRs sit above its VGPRs, and a function that makes calls
        # would otherwise get a 64 VGPR + 64 AGPR split instead of 128 VGPRs.
        with open(ll) as f:
            ir = _ATTR_RE.sub(r'\1 "amdgpu-agpr-alloc"="0"', f.read())
        with open(ll, "w") as f:
            f.write(ir)
        _run([LLC, "-mtriple=amdgcn-amd-amdhsa", f"-mcpu={ARCH}", "-O3", ll, "-o", asm], "llc")
        with open(asm) as f:
            text = f.read()
        _run([LLVM_MC, "-triple=amdgcn-amd-amdhsa", f"-mcpu={ARCH}", "-filetype=obj", asm, "-o", obj], "llvm-mc")
        _run([LLD, "-shared", "--no-undefined", obj, "-o", co], "ld.lld")
        with open(co, "rb") as f:
            image = f.read()
    res = function_resources(text)
    mod = CompiledModule(image, len(progs), [res.get(f"fks_prog_{i}") for i in range(len(progs))],
                         time.perf_counter() - t0)
    _cache_store(key, mod)
    return mod


def compile_host_module(progs: Sequence[CompiledPolicy], path: str) -> str:
    """The same programs built for the host with g++ (``FKS_HOST_JIT``):
    exports ``fks_host_table`` / ``fks_host_count``.  Used by the codegen
    tests (CPU replays through the oracle engine) and as a CPU-native path."""
    src = module_source(progs, host=True)
    cpp = path + ".cpp"
    with open(cpp, "w") as f:
        f.write(src)
    _run([os.environ.get("CXX", "g++"), "-O2", "-std=c++17", "-DFKS_HOST_JIT", f"-I{JIT_INCLUDE}", "-shared", "-fPIC",
          "-ffp-contract=off", "-fno-fast-math", "-Wno-unused-label", "-x", "c++", cpp, "-o", path], "g++")
    return path


# ---------------------------------------------------------------------------- device cache
@dataclass
class NativeBatch:
    """Per-policy launch data of one batch (programs in input order)."""
    fn: np.ndarray                   # uint64 [P] device addresses | feasibility-prologue bit (0: not native)
    kc: np.ndarray                   # int64 concatenated constant blocks
    koff: np.ndarray                 # int32 [P]
    ok: np.ndarray                   # bool [P]
    reasons: Dict[int, str] = field(default_factory=dict)
    compile_s: float = 0.0           # wall time spent compiling for this batch
    compiled: int = 0                # new shapes compiled for this batch
    modules: Tuple[int, ...] = ()    # module ids the batch calls into (held until `release`)
    load_s: float = 0.0              # of compile_s: module loads


@dataclass
class _ModRec:
    """A loaded JIT module and the shapes that currently resolve into it."""
    handle: object                   # _fks_hip.JitModule
    shapes: set = field(default_factory=set)
    refs: int = 0                    # batches in flight calling into it
    last_use: int = 0                # prepare() sequence number of the last batch using it
    tier: str = "baseline"
    nbytes: int = 0                  # code-object bytes


class NativeCompiler:
    """Shape cache + parallel compiler + loader for one HIP device."""

    TIERS = ("auto", "baseline", "llvm")

    def __init__(self, engine, device: int = 0, workers: int = 0, budget: int = 1 << 22, max_chunk: int = 16,
                 tier: Optional[str] = None):
        from . import hip_engine
        self._hip = hip_engine.native()
        self._engine = engine            # _fks_hip.DeviceEngine (for the runtime table)
        self.device = device
        self.workers = workers or _default_workers()
        self.budget = int(budget)
        self.max_chunk = max_chunk
        self._rt = np.asarray(engine.native_rt_table(), dtype=np.uint64)
        self.vgpr_cap = int(self._hip.JIT_VGPRS)
        self.sgpr_cap = int(self._hip.JIT_SGPRS)
        self._shapes: Dict[str, Tuple[int, int]] = {}   # shape -> (module id, program index)
        self._ptr: Dict[str, int] = {}                  # shape -> device address of its code
        self._bad: Dict[str, str] = {}                  # shape -> reason it is not native
        self._modules: Dict[int, _ModRec] = {}         # live modules by id
        self._next_mod = 0
        self._seq = 0
        # bounded module lifetime: beyond this many live modules the least recently
        # used ones that no batch in flight calls into are unloaded (their shapes are
        # recompiled if they come back -- the baseline tier takes ~0.2 ms a shape).
        # A module is one batch's new shapes (~512 programs, a few MB of code), so
        # 2048 hold a long steady-state run in HBM: a 200 s config-3 run loads ~1,100
        # (round 5), and most of a retired module's shapes were one-off children --
        # `recompiled_shapes` counts the evicted shapes that did come back
        self.max_modules = int(os.environ.get("FKS_JIT_MAX_MODULES", "2048"))
        #: retired modules stay loaded until `flush_unloads` (set while the
        #: device's program service runs: an unload waits on the device)
        self.defer_unloads = False
        self._deferred: List[object] = []
        self._evicted: set = set()     # hashes of evicted shape keys (recompile accounting)
        self._lock = threading.Lock()
        self._inflight: Dict[str, threading.Event] = {}
        self._procs = threading.BoundedSemaphore(self.workers)
        # baseline by default: the LLVM tier's rows differed from the CPU VM on
        # 1-9 of 256 evolved children (-O1 / -O3) where the baseline's all agree
        self.tier = (tier or os.environ.get("FKS_JIT_TIER", "baseline")).lower()
        if self.tier not in self.TIERS:
            raise ValueError(f"unknown JIT tier {self.tier!r} (one of {self.TIERS})")
        if self.budget >= 1 << 31:
            raise ValueError("the per-call instruction budget must fit in int32 (baseline tier counter)")
        self._baseline = None
        if self.tier != "llvm":
            from .gcnjit import BaselineJit
            self._baseline = BaselineJit(self._hip, self._rt, device)
        self.stats = {"modules": 0, "shapes": 0, "compile_s": 0.0, "rejected": 0, "hits": 0,
                      "baseline_shapes": 0, "llvm_shapes": 0, "baseline_s": 0.0, "llvm_s": 0.0, "load_s": 0.0,
                      "disk_hits": 0, "tierup_queued": 0, "tierup_done": 0, "tierup_s": 0.0,
                      "live_modules": 0, "max_live_modules": 0, "retired_modules": 0, "evicted_shapes": 0,
                      "recompiled_shapes": 0, "unload_s": 0.0}
        # tier-up (auto tier): a baseline shape used in this many batches is
        # recompiled by the LLVM tier in the background (its code runs ~1.3x
        # faster on the device) and swapped in when ready; never on the
        # critical path of a batch.  Off by default (FKS_JIT_TIERUP=n enables
        # it): on 9 of the first 512 evolved children (data/populations,
        # small float powers next to GPU-list loops) the LLVM-tier rows differ
        # from the CPU VM on the device while the baseline rows and the host
        # build of the same LLVM-tier source agree (tools/scratch tier checks,
        # docs/REVIEW_RESPONSE.md round 5).
        self.tierup_after = int(os.environ.get("FKS_JIT_TIERUP", "0")) if self.tier == "auto" else 0
        self._uses: Dict[str, int] = {}
        self._tier_of: Dict[str, str] = {}
        self._tierup_pool: Optional[ThreadPoolExecutor] = None
        self._tierup_futs: List[object] = []

    def prepare(self, progs: Sequence[CompiledPolicy]) -> NativeBatch:
        """Compile every shape of `progs` not compiled yet (thread-safe: islands
        call this concurrently; a shape another thread is compiling is waited
        for, not compiled twice) and build the batch's launch data."""
        keys = [_shape_key(p) for p in progs]
        mine: Dict[str, CompiledPolicy] = {}
        others = []
        with self._lock:
            for k, p in zip(keys, progs):
                if k in self._shapes or k in self._bad or k in mine:
                    continue
                ev = self._inflight.get(k)
                if ev is not None:
                    others.append(ev)
                else:
                    mine[k] = p
            for k in mine:
                self._inflight[k] = threading.Event()
        t0 = time.perf_counter()
        load0 = self.stats["load_s"]
        try:
            if mine:
                self._compile_shapes(mine)
        finally:
            with self._lock:
                for k in mine:
                    self._inflight.pop(k).set()
        for ev in others:
            ev.wait()
        dt = time.perf_counter() - t0
        load_dt = self.stats["load_s"] - load0
        P = len(progs)
        fn = np.zeros(P, dtype=np.uint64)
        ok = np.zeros(P, dtype=bool)
        kc, koff = constant_blocks(progs, self.budget)
        reasons = {}
        used = set()
        retry = {}
        with self._lock:
            self._seq += 1
            for i, (k, p) in enumerate(zip(keys, progs)):
                loc = self._shapes.get(k)
                if loc is not None:
                    used.add(loc[0])
                    # bit 0: the program opens with the template's feasibility
                    # prologue, so the kernels call it for feasible nodes only
                    fn[i] = self._ptr[k] | (1 if _FEAS_SKIP and p.feasibility_prologue else 0)
                    ok[i] = True
                elif k in self._bad:
                    reasons[i] = self._bad[k]
                else:
                    retry[k] = p    # compiled, then retired by another thread before this batch held it
            for mid in used:         # held until release(): never retired while a batch may call it
                rec = self._modules[mid]
                rec.refs += 1
                rec.last_use = self._seq
            self.stats["hits"] += P - len(mine)
            up = self._tierup_candidates(keys, progs) if self.tierup_after else []
        if retry:
            # rare: recompile the retired shapes for this batch (their modules are gone)
            sub = self.prepare([retry[k] for k in retry])
            pos_of = {k: j for j, k in enumerate(retry)}
            for i, k in enumerate(keys):
                j = pos_of.get(k)
                if j is None:
                    continue
                if sub.ok[j]:
                    fn[i] = sub.fn[j] | (1 if _FEAS_SKIP and progs[i].feasibility_prologue else 0)
                    ok[i] = True
                else:
                    reasons[i] = sub.reasons.get(j, "not compiled")
            extra = sub.modules          # held by the inner prepare(): released with this batch
            dt += sub.compile_s
        else:
            extra = ()
        self._reap_tierup()
        for k, p in up:
            self._tierup_futs.append(self._tierup_executor().submit(self._tierup, k, p))
        self._retire()
        return NativeBatch(fn, kc, koff, ok, reasons, dt, len(mine), tuple(sorted(used)) + tuple(extra), load_dt)

    # -- module lifetime ---------------------------------------------------------------------
    def release(self, modules: Sequence[int]) -> None:
        """The batch that held `modules` (NativeBatch.modules) has completed."""
        with self._lock:
            for mid in modules:
                rec = self._modules.get(mid)
                if rec is not None:
                    rec.refs -= 1
        self._retire()

    def _add_module(self, handle, tier: str, nbytes: int = 0) -> int:
        """Register a loaded module (lock held); returns its id."""
        mid = self._next_mod
        self._next_mod += 1
        self._modules[mid] = _ModRec(handle, tier=tier, last_use=self._seq, nbytes=int(nbytes))
        self.stats["loaded_mb"] = round(self.stats.get("loaded_mb", 0.0) + nbytes / 2.0 ** 20, 3)
        self.stats["modules"] += 1
        self.stats["live_modules"] = len(self._modules)
        self.stats["max_live_modules"] = max(self.stats["max_live_modules"], len(self._modules))
        return mid

    def _map_shape(self, k: str, mid: int, idx: int, ptr: int) -> None:
        """shape k -> program idx of module mid (lock held)."""
        old = self._shapes.get(k)
        if old is not None and old[0] in self._modules:
            self._modules[old[0]].shapes.discard(k)
        self._shapes[k] = (mid, idx)
        self._ptr[k] = int(ptr)
        self._modules[mid].shapes.add(k)

    def _retire(self) -> None:
        """Unload the least recently used modules no batch in flight calls
        into, down to 3/4 of `max_modules`, once more than `max_modules` are
        live.  Their shapes leave the cache (a later batch recompiles them).
        No device-wide synchronisation: a module with no references has no
        launch that could still call into it."""
        if self.max_modules <= 0:
            return
        victims = []
        with self._lock:
            if len(self._modules) <= self.max_modules:
                return
            idle = sorted((rec.last_use, mid) for mid, rec in self._modules.items() if rec.refs <= 0)
            excess = len(self._modules) - max(1, (3 * self.max_modules) // 4)
            for _, mid in idle[:max(0, excess)]:
                rec = self._modules.pop(mid)
                for k in rec.shapes:
                    if self._shapes.get(k, (None,))[0] == mid:
                        del self._shapes[k]
                        self._ptr.pop(k, None)
                        self._tier_of.pop(k, None)
                        self._uses.pop(k, None)
                        self.stats["evicted_shapes"] += 1
                        self._evicted.add(hash(k))
                victims.append(rec)
            self.stats["retired_modules"] += len(victims)
            self.stats["live_modules"] = len(self._modules)
        if getattr(self, "defer_unloads", False):
            # a persistent grid is running (the program service): hipModuleUnload
            # waits on the device (~0.2 s per module measured, 107 s for one
            # retirement burst), so the modules stay loaded until `flush_unloads`
            # (the steady search rolls the grid over when too many are parked)
            with self._lock:
                self._deferred.extend(victims)
                self.stats["deferred_modules"] = len(self._deferred)
            return
        t0 = time.perf_counter()
        for rec in victims:
            rec.handle.unload()
        with self._lock:
            self.stats["unload_s"] += time.perf_counter() - t0
            self.stats["loaded_mb"] = round(self.stats.get("loaded_mb", 0.0) - sum(r.nbytes for r in victims) / 2.0 ** 20, 3)

    def flush_unloads(self) -> int:
        """Unload the modules retired while `defer_unloads` was set (call with
        no persistent kernel running); returns their number."""
        with self._lock:
            victims, self._deferred = getattr(self, "_deferred", []), []
            self.stats["deferred_modules"] = 0
        t0 = time.perf_counter()
        for rec in victims:
            rec.handle.unload()
        with self._lock:
            self.stats["unload_s"] += time.perf_counter() - t0
            self.stats["loaded_mb"] = round(self.stats.get("loaded_mb", 0.0) - sum(r.nbytes for r in victims) / 2.0 ** 20, 3)
            self.stats["flushed_modules"] = self.stats.get("flushed_modules", 0) + len(victims)
        return len(victims)

    @property
    def deferred(self) -> int:
        """Retired modules still loaded, waiting for `flush_unloads`."""
        return len(self._deferred)

    # -- background tier-up --------------------------------------------------------------
    def _tierup_candidates(self, keys, progs):
        """(key, program) of baseline shapes that just became hot (lock held)."""
        out, seen = [], set()
        for k, p in zip(keys, progs):
            if k in seen or self._tier_of.get(k) != "baseline":
                continue
            seen.add(k)
            n = self._uses.get(k, 0) + 1
            self._uses[k] = n
            if n == self.tierup_after:
                self._tier_of[k] = "tierup"
                self.stats["tierup_queued"] += 1
                out.append((k, p))
        return out

    def _tierup_executor(self) -> ThreadPoolExecutor:
        if self._tierup_pool is None:
            self._tierup_pool = ThreadPoolExecutor(max_workers=max(1, self.workers // 4),
                                                   thread_name_prefix="fks-tierup")
        return self._tierup_pool

    def _tierup(self, k: str, p: CompiledPolicy) -> bool:
        mod = self._compile_one([(k, p)])
        if isinstance(mod, Exception):
            return False
        res = mod.resources[0]
        if res is None or res.fits(self.vgpr_cap, self.sgpr_cap):
            return False    # the baseline code stays
        mod.handle = self._hip.JitModule(mod.image, self._rt, mod.n, self.device)
        mod.pointers = np.asarray(mod.handle.pointers(), dtype=np.uint64)
        with self._lock:
            if k not in self._shapes:     # retired meanwhile: nothing to upgrade
                mod.handle.unload()
                return False
            mi = self._add_module(mod.handle, "llvm")   # the baseline module stays loaded: batches in flight call it
            self._map_shape(k, mi, 0, int(mod.pointers[0]))
            self._tier_of[k] = "llvm"
            self.stats["tierup_done"] += 1
            self.stats["tierup_s"] += mod.compile_s
            self.stats["disk_hits"] += int(mod.cached)
        return True

    def _reap_tierup(self) -> None:
        """Drop finished tier-up futures; an exception in one (e.g. a failed
        module load in the worker) is counted and logged, not lost."""
        keep = []
        for f in self._tierup_futs:
            if not f.done():
                keep.append(f)
                continue
            exc = f.exception()
            if exc is not None:
                self.stats["tierup_errors"] = self.stats.get("tierup_errors", 0) + 1
                import warnings
                warnings.warn(f"background tier-up failed: {type(exc).__name__}: {exc}", RuntimeWarning)
        self._tierup_futs = keep

    def drain_tierup(self) -> None:
        """Wait for every queued background recompile (tests, benchmarks)."""
        while self._tierup_futs:
            self._tierup_futs.pop(0).result()

    def _compile_one(self, chunk):
        """CompiledModule, or the toolchain error (never raises: one bad
        program must not take down the batch or the search)."""
        with self._procs:   # bounds concurrent toolchain processes across all callers
            try:
                return compile_device_module([p for _, p in chunk])
            except (JitError, OSError) as exc:
                return exc

    def _compile_baseline(self, items):
        """Baseline tier: generate every shape (in parallel, C++ threads), load
        the batch as one module; returns the (key, program, reason) the
        generator declined."""
        from .gcnjit import compile_many
        t0 = time.perf_counter()
        codes, keys, declined = [], [], []
        for (k, p), (code, why) in zip(items, compile_many([p for _, p in items], self.workers)):
            if code is None:
                declined.append((k, p, why))
            else:
                codes.append(code)
                keys.append(k)
        t1 = time.perf_counter()
        with self._lock:
            self.stats["compile_s"] += t1 - t0
            self.stats["baseline_s"] += t1 - t0
        # one module per skeleton-sized chunk (thousands of long programs can
        # exceed the largest arena)
        for lo, hi in (self._baseline.chunks(codes) if codes else []):
            t1 = time.perf_counter()
            mod = self._baseline.load(codes[lo:hi], 0.0)
            t2 = time.perf_counter()
            with self._lock:
                mi = self._add_module(mod.handle, "baseline", mod.nbytes)
                self.stats["compile_s"] += t2 - t1
                self.stats["load_s"] += t2 - t1
                self.stats["probed_loads"] = self.stats.get("probed_loads", 0) + int(mod.probed)
                for j, k in enumerate(keys[lo:hi]):
                    if self._evicted and hash(k) in self._evicted:
                        self.stats["recompiled_shapes"] += 1
                    self._map_shape(k, mi, j, int(mod.pointers[j]))
                    self._tier_of[k] = "baseline"
                    self._uses.pop(k, None)
                    self.stats["shapes"] += 1
                    self.stats["baseline_shapes"] += 1
        return declined

    def _compile_shapes(self, new: Dict[str, CompiledPolicy]) -> None:
        items = list(new.items())
        if self._baseline is not None:
            declined = self._compile_baseline(items)
            if self.tier == "baseline":
                with self._lock:
                    rr = self.stats.setdefault("reject_reasons", {})
                    for k, _, why in declined:
                        self._bad[k] = why
                        self.stats["rejected"] += 1
                        r = why[:48]
                        rr[r] = rr.get(r, 0) + 1
                return
            items = [(k, p) for k, p, _ in declined]
            if not items:
                return
        self._compile_llvm(items)

    def _compile_llvm(self, items) -> None:
        # code generation first (cheap, in-process): shapes it cannot lower are rejected
        good = []
        for k, p in items:
            try:
                module_source([p], with_probes=False)
                good.append((k, p))
            except CodegenError as exc:
                with self._lock:
                    self._bad[k] = f"codegen: {exc}"
                    self.stats["rejected"] += 1
        if not good:
            return
        n_chunks = max(1, min(self.workers, len(good)))
        size = max(1, min(self.max_chunk, math.ceil(len(good) / n_chunks)))
        chunks = [good[i:i + size] for i in range(0, len(good), size)]
        with ThreadPoolExecutor(max_workers=min(self.workers, len(chunks))) as ex:
            mods = list(ex.map(self._compile_one, chunks))
        # a failed chunk: retry its programs one by one; the failing ones are
        # marked non-native (with the toolchain's message) and go to the VMs
        retry_ch, retry_mod = [], []
        for ch, mod in zip(chunks, mods):
            if not isinstance(mod, Exception):
                continue
            if len(ch) == 1:
                with self._lock:
                    self._bad[ch[0][0]] = f"llvm: {mod}"[:500]
                    self.stats["rejected"] += 1
                continue
            for item in ch:
                m1 = self._compile_one([item])
                if isinstance(m1, Exception):
                    with self._lock:
                        self._bad[item[0]] = f"llvm: {m1}"[:500]
                        self.stats["rejected"] += 1
                else:
                    retry_ch.append([item])
                    retry_mod.append(m1)
        pairs = [(ch, mod) for ch, mod in zip(chunks, mods) if not isinstance(mod, Exception)]
        pairs += list(zip(retry_ch, retry_mod))
        for ch, mod in pairs:
            mod.handle = self._hip.JitModule(mod.image, self._rt, mod.n, self.device)
            mod.pointers = np.asarray(mod.handle.pointers(), dtype=np.uint64)
            with self._lock:
                self.stats["compile_s"] += mod.compile_s
                self.stats["llvm_s"] += mod.compile_s
                self.stats["llvm_shapes"] += len(ch)
                self.stats["disk_hits"] += int(mod.cached)
                mi = self._add_module(mod.handle, "llvm")
                for j, (k, _) in enumerate(ch):
                    res = mod.resources[j]
                    why = "no resource record" if res is None else res.fits(self.vgpr_cap, self.sgpr_cap)
                    if why:
                        self._bad[k] = why
                        self.stats["rejected"] += 1
                    else:
                        self._map_shape(k, mi, j, int(mod.pointers[j]))
                        self._tier_of[k] = "llvm"
                        self.stats["shapes"] += 1


def _default_workers() -> int:
    """Toolchain processes per rank: the host's cores shared by the ranks on
    it (``LOCAL_WORLD_SIZE``), at most 16."""
    env = os.environ.get("FKS_JIT_WORKERS", "")
    if env.isdigit() and int(env) > 0:
        return int(env)
    from .cpu_engine import default_threads
    local = max(1, int(os.environ.get("LOCAL_WORLD_SIZE", "1") or 1))
    return max(1, min(16, default_threads() // local))


__all__ = ["CompiledModule", "JitError", "NativeBatch", "NativeCompiler", "Resources", "compile_device_module",
           "compile_host_module", "function_resources"]

