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
