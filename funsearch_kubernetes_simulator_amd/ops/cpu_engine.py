"""Python front-end of the native CPU oracle engine (``_fks_cpu``).

The native module is built in-tree by `ops.build`; importing this module
builds it on demand when the toolchain is present (the CPU container and the
GPU box both have g++), and fails loudly otherwise.
"""

from __future__ import annotations

import os
from dataclasses import dataclass
from typing import Dict, Optional, Sequence

import numpy as np

from ..core.arrays import Workload
from ..policy.compiler import CompiledPolicy

_mod = None

#: Default VM instruction budget of one priority evaluation (one pod, all
#: nodes).  Runaway programs (``while True``) stop with EXC_BUDGET -- on the
#: GPU this guarantees every replay wave drains -- and the evaluator hands
#: them to the wall-clock-bounded object engine.
DEFAULT_CALL_BUDGET = 1 << 22


def default_threads() -> int:
    """Worker threads for the native CPU engine: the process's CPU share
    (OMP_NUM_THREADS / affinity) rather than every core of a shared machine."""
    env = os.environ.get("OMP_NUM_THREADS", "")
    if env.isdigit() and int(env) > 0:
        return int(env)
    try:
        return max(1, len(os.sched_getaffinity(0)))
    except (AttributeError, OSError):
        return os.cpu_count() or 1

FAMILY = {"first_fit": 0, "best_fit": 1, "random_linear": 2, "feature_linear": 3, "composite_linear": 4}


def native():
    """The loaded ``_fks_cpu`` extension (built if missing or stale)."""
    global _mod
    if _mod is None:
        if os.environ.get("FKS_NO_AUTOBUILD") != "1":
            from .build import build_cpu
            build_cpu()
        from . import _fks_cpu  # noqa: F401  (in-tree extension)
        from .build import verify
        verify(_fks_cpu, "cpu")    # refuses a binary built from other sources
        _mod = _fks_cpu
    return _mod


RESULT_COLUMNS = ("score", "avg_cpu", "avg_mem", "avg_gpu_count", "avg_gpu_milli", "frag",
                  "n_snapshots", "n_frag_events", "n_events", "n_unplaced", "exc", "inexact",
                  "trace_hash_hi")


def workload_dict(w: Workload) -> Dict[str, np.ndarray]:
    c, p = w.cluster, w.pods
    return dict(node_cpu_total=c.node_cpu_total, node_cpu_left=c.node_cpu_left,
                node_mem_total=c.node_mem_total, node_mem_left=c.node_mem_left,
                node_gpu_left=c.node_gpu_left, node_ngpus=c.node_ngpus, gpu_start=c.gpu_start,
                gpu_milli_total=c.gpu_milli_total, gpu_milli_left=c.gpu_milli_left,
                gpu_mem_total=c.gpu_mem_total, gpu_mem_left=c.gpu_mem_left,
                pod_cpu=p.pod_cpu, pod_mem=p.pod_mem, pod_ngpu=p.pod_ngpu, pod_gmilli=p.pod_gmilli,
                pod_ctime=p.pod_ctime, pod_dur=p.pod_dur, pod_rank=p.pod_rank)


_wl_cache: Dict[int, tuple] = {}


def native_workload(w: Workload):
    key = id(w)
    hit = _wl_cache.get(key)
    if hit is not None and hit[0] is w:
        return hit[1]
    nw = native().Workload(workload_dict(w))
    _wl_cache[key] = (w, nw)
    return nw


@dataclass
class SimOptions:
    repush: str = "first"           # "first" (reference) | "earliest"
    gpu_alloc: str = "best_fit"     # "best_fit" (reference) | "first_fit"
    snapshot_interval: float = 0.05
    truncate: bool = True           # FunSearchScheduler int(max(0, score))
    budget: int = DEFAULT_CALL_BUDGET  # VM instructions per priority evaluation (0 = unlimited)
    record_values: bool = False
    record_placements: bool = False
    check_invariants: int = 0       # verify resource accounting every K events + at the end (debug)
    record_states: bool = False     # per creation event: pod, decision, node/GPU state (analysis tools)

    def as_dict(self) -> dict:
        return dict(self.__dict__)


def simulate_builtin(w: Workload, family: str, weights: Sequence[float] = (),
                     options: Optional[SimOptions] = None) -> dict:
    return native().simulate_builtin(native_workload(w), FAMILY[family], list(map(float, weights)),
                                     (options or SimOptions()).as_dict())


def simulate_builtin_batch(w: Workload, family: str, weights: np.ndarray,
                           options: Optional[SimOptions] = None, threads: int = 0) -> np.ndarray:
    threads = threads or default_threads()
    return native().simulate_builtin_batch(native_workload(w), FAMILY[family],
                                           np.ascontiguousarray(weights, dtype=np.float64),
                                           (options or SimOptions()).as_dict(), threads)


def simulate_program(w: Workload, prog: CompiledPolicy, options: Optional[SimOptions] = None) -> dict:
    return native().simulate_program(native_workload(w), prog.code, prog.fconst, prog.iconst,
                                     prog.ctag, (options or SimOptions()).as_dict())


def simulate_program_batch(w: Workload, progs: Sequence[CompiledPolicy],
                           options: Optional[SimOptions] = None, threads: int = 0) -> np.ndarray:
    threads = threads or default_threads()
    return native().simulate_program_batch(native_workload(w), [p.code for p in progs],
                                           [p.fconst for p in progs], [p.iconst for p in progs],
                                           [p.ctag for p in progs], (options or SimOptions()).as_dict(),
                                           threads)


# ---------------------------------------------------------------------------- native programs on the CPU
_host_libs: dict = {}


def host_native_library(progs: Sequence[CompiledPolicy], workdir: Optional[str] = None):
    """g++ build of the programs' native code (policy/native_codegen.py, the
    same C++ the device JIT compiles) loaded with ctypes: (library, addresses)."""
    import ctypes
    import hashlib
    import tempfile
    from . import jit
    from ..policy.native_codegen import module_source
    key = hashlib.sha1(module_source(progs, host=True).encode()).hexdigest()
    if key not in _host_libs:
        d = workdir or tempfile.mkdtemp(prefix="fks_hostjit_")
        path = jit.compile_host_module(progs, os.path.join(d, f"m_{key[:12]}.so"))
        lib = ctypes.CDLL(path)
        n = ctypes.c_int.in_dll(lib, "fks_host_count").value
        table = (ctypes.c_void_p * n).in_dll(lib, "fks_host_table")
        _host_libs[key] = (lib, [int(table[i]) for i in range(n)])
    return _host_libs[key]


def simulate_native_batch(w: Workload, progs: Sequence[CompiledPolicy], options: Optional[SimOptions] = None,
                          threads: int = 0) -> np.ndarray:
    """Replays with host-compiled native programs: [P, 13] like the VM batch."""
    from ..policy.native_codegen import constant_block
    threads = threads or default_threads()
    opts = options or SimOptions()
    _, addrs = host_native_library(progs)
    blocks = [constant_block(p, opts.budget if opts.budget > 0 else DEFAULT_CALL_BUDGET) for p in progs]
    koff = np.cumsum([0] + [len(b) for b in blocks[:-1]]).astype(np.int32)
    return native().simulate_native_batch(native_workload(w), addrs, np.concatenate(blocks), koff, opts.as_dict(),
                                          threads)
