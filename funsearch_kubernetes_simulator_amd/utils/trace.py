"""roctx ranges for rocprofv3 `--marker-trace` timelines (no-ops without ROCm).

    with roctx_range("generation 12"):
        ...

The native engine marks every device batch itself ("fks.batch.builtin" /
"fks.batch.vm", submit -> completion); these host ranges add the search
structure around them (generations, migrations).
"""

from __future__ import annotations

import ctypes
import contextlib
import os

_lib = None
_loaded = False


def _roctx():
    global _lib, _loaded
    if not _loaded:
        _loaded = True
        for name in ("librocprofiler-sdk-roctx.so.1", "librocprofiler-sdk-roctx.so",
                     os.path.join("/opt/rocm/lib", "librocprofiler-sdk-roctx.so")):
            try:
                lib = ctypes.CDLL(name)
                lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
                lib.roctxMarkA.argtypes = [ctypes.c_char_p]
                _lib = lib
                break
            except OSError:
                continue
    return _lib


@contextlib.contextmanager
def roctx_range(name: str):
    lib = _roctx()
    if lib is None:
        yield
        return
    lib.roctxRangePushA(name.encode())
    try:
        yield
    finally:
        lib.roctxRangePop()


def roctx_mark(name: str) -> None:
    lib = _roctx()
    if lib is not None:
        lib.roctxMarkA(name.encode())


class ThreadSampler:
    """Where the host's threads spend their time (a run-time breakdown of the
    steady loop: dispatcher, stagers, fallbacks, coupler, native threads).

    Two measures, both cheap enough for a production run:

    * CPU seconds per OS thread (``psutil``), grouped by Python thread name
      (threads Python did not start -- the JIT's C++ workers, the HIP runtime's
      -- are grouped as ``native``);
    * a statistical profile: every ``interval_s`` the Python stack of every
      Python thread (``sys._current_frames``) is sampled and its innermost
      ``depth`` frames counted, so a thread's samples split into what it was
      running, including waits (``sleep``, ``wait``, lock acquisition) -- a
      thread that holds or waits for the GIL is visible here, not in CPU time.
    """

    def __init__(self, interval_s: float = 0.01, depth: int = 4):
        import threading
        self.interval_s = float(interval_s)
        self.depth = int(depth)
        self.samples: dict = {}       # thread name -> {frame key: count}
        self.totals: dict = {}        # thread name -> samples
        self._stop = threading.Event()
        self._thread = threading.Thread(target=self._run, name="fks-sampler", daemon=True)
        self._cpu0 = self._cpu_by_thread()
        self.t0 = None

    @staticmethod
    def _names() -> dict:
        import threading
        return {t.native_id: t.name for t in threading.enumerate() if t.native_id is not None}

    @staticmethod
    def _group(name: str) -> str:
        # pool workers: "fks-stage_0" -> "fks-stage"; "ThreadPoolExecutor-3_1" -> "ThreadPoolExecutor"
        base = name.rsplit("_", 1)[0] if "_" in name else name
        return base.split("-")[0] if base.startswith("ThreadPoolExecutor") else base

    def _cpu_by_thread(self) -> dict:
        try:
            import psutil
            return {t.id: t.user_time + t.system_time for t in psutil.Process().threads()}
        except Exception:   # (psutil missing or no /proc access)
            return {}

    def start(self) -> "ThreadSampler":
        import time
        self.t0 = time.time()
        self._names_seen = dict(self._names())
        self._thread.start()
        return self

    def _run(self) -> None:
        import sys
        import threading
        me = threading.get_ident()
        while not self._stop.wait(self.interval_s):
            by_ident = {t.ident: t.name for t in threading.enumerate()}
            self._names_seen.update(self._names())
            for ident, frame in sys._current_frames().items():
                if ident == me:
                    continue
                name = self._group(by_ident.get(ident, "?"))
                parts = []
                f = frame
                while f is not None and len(parts) < self.depth:
                    co = f.f_code
                    # the innermost frame with its line: where in a long loop body
                    ln = f":{f.f_lineno}" if not parts else ""
                    parts.append(f"{os.path.basename(co.co_filename)}:{co.co_name}{ln}")
                    f = f.f_back
                key = " < ".join(parts)
                d = self.samples.setdefault(name, {})
                d[key] = d.get(key, 0) + 1
                self.totals[name] = self.totals.get(name, 0) + 1

    def stop(self) -> None:
        self._stop.set()
        if self._thread.is_alive():
            self._thread.join(timeout=2.0)

    def report(self, top: int = 12) -> dict:
        """{wall_s, cpu_s: {group: seconds}, profile: {group: [(fraction, frames)]}}"""
        import time
        wall = time.time() - (self.t0 or time.time())
        cpu1 = self._cpu_by_thread()
        names = dict(self._names_seen)
        names.update(self._names())
        cpu: dict = {}
        for tid, t in cpu1.items():
            g = self._group(names.get(tid, "native"))
            cpu[g] = cpu.get(g, 0.0) + t - self._cpu0.get(tid, 0.0)
        prof = {}
        for name, d in self.samples.items():
            n = max(1, self.totals.get(name, 1))
            prof[name] = [(round(c / n, 4), k) for k, c in sorted(d.items(), key=lambda kv: -kv[1])[:top]]
        return {"wall_s": round(wall, 3), "cpu_s": {k: round(v, 2) for k, v in sorted(cpu.items(), key=lambda kv: -kv[1])},
                "samples": dict(self.totals), "profile": prof}
