"""In-tree build of the native extensions.

* ``_fks_cpu``  - C++17 oracle engine + bytecode VM (g++, pybind11);
* ``_fks_hip``  - MI355X replay kernels (hipcc ``--offload-arch=gfx950``,
  pybind11 host side).  It links ``libamdhip64.so.7`` by SONAME so that, once
  ``torch`` is imported, the process shares torch's HIP runtime.

Both land next to this file so they travel with the repository snapshot to
the GPU box.  ``python -m funsearch_kubernetes_simulator_amd.ops.build``
rebuilds whatever is stale.

Provenance: every build embeds a SHA-256 of its sources and compile flags
(``FKS_SOURCE_HASH=<hex>`` in the binary, ``SOURCE_HASH`` on the module).
Staleness is that hash against the current tree -- not file times, which a
snapshot copy rewrites -- and `verify` refuses to load an extension built
from other sources.
"""

from __future__ import annotations

import hashlib
import os
import re
import subprocess
import sys
import sysconfig
from pathlib import Path
from typing import List

from .._paths import CSRC_DIR, NATIVE_DIR

ARCH = os.environ.get("FKS_OFFLOAD_ARCH", "gfx950")


def _py_includes() -> List[str]:
    import pybind11
    return [f"-I{pybind11.get_include()}", f"-I{sysconfig.get_paths()['include']}"]


def _ext_suffix() -> str:
    return sysconfig.get_config_var("EXT_SUFFIX") or ".so"


class StaleExtension(ImportError):
    """An extension binary was built from sources other than the tree's."""


def source_hash(sources: List[Path], flags: List[str]) -> str:
    h = hashlib.sha256()
    for src in sorted(sources):
        h.update(str(src.relative_to(CSRC_DIR)).encode())
        h.update(b"\0")
        h.update(src.read_bytes())
        h.update(b"\0")
    # include directories are machine paths (the GPU box runs the tree from
    # a scratch directory): only the other flags are part of the identity
    h.update(" ".join(f for f in flags if not f.startswith("-I")).encode())
    return h.hexdigest()


_MARK = re.compile(rb"FKS_SOURCE_HASH=([0-9a-f]{64})")


def embedded_hash(target: Path) -> str:
    """The source hash compiled into a built extension ('' if none)."""
    try:
        m = _MARK.search(target.read_bytes())
    except OSError:
        return ""
    return m.group(1).decode() if m else ""


def _stale(target: Path, want: str) -> bool:
    return not target.exists() or embedded_hash(target) != want


def _run(cmd: List[str]) -> None:
    print("[fks build]", " ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)


def _deps(*globs: str) -> List[Path]:
    out: List[Path] = []
    for g in globs:
        out.extend(sorted(CSRC_DIR.glob(g)))
    return out


CPU_FLAGS = ["-O3", "-std=c++17", "-shared", "-fPIC", "-fvisibility=hidden", "-ffp-contract=off", "-fno-fast-math",
             "-Wall", "-Wno-unused-function"]


def _cpu_sources() -> List[Path]:
    return _deps("cpu/*.cpp", "cpu/*.hpp", "include/fks/*.hpp", "jit/*", "hip/jit_abi.h", "hip/pyops_dev.h",
                 "hip/glibc_math.h", "hip/glibc_math_tables.inc", "hip/jit_env.h", "hip/exc_codes.h")


def cpu_hash() -> str:
    return source_hash(_cpu_sources(), CPU_FLAGS)


def build_cpu(force: bool = False) -> Path:
    target = NATIVE_DIR / f"_fks_cpu{_ext_suffix()}"
    want = cpu_hash()
    if force or _stale(target, want):
        cxx = os.environ.get("CXX", "g++")
        tmp = target.with_name(target.name + f".{os.getpid()}.tmp")
        cmd = [cxx, *CPU_FLAGS, f'-DFKS_SOURCE_HASH="{want}"', *_py_includes(), f"-I{CSRC_DIR / 'include'}",
               str(CSRC_DIR / "cpu" / "module.cpp"), str(CSRC_DIR / "jit" / "gcn_jit.cpp"), "-o", str(tmp),
               "-lpthread"]
        _run(cmd)
        os.replace(tmp, target)      # never a half-written .so next to the sources
    return target


#: Device translation units of _fks_hip: (object name, extra defines).  The
#: replay kernels are split per NPASS and kind so their many template
#: instances compile in parallel.
HIP_UNITS = [("module", "module.hip", [])] + [
    (f"replay_k{kind}_np{npass}", "replay_kernels.hip", [f"-DFKS_KIND={kind}", f"-DFKS_NPASS={npass}"])
    for kind, npasses in ((0, (1, 2, 4)), (1, (1, 2, 4)), (2, (1,)), (3, (1,)), (4, (1, 2, 4))) for npass in npasses]


def _hip_flags() -> List[str]:
    # occupancy knobs of the replay kernels (waves per SIMD), for A/B builds
    knobs = [f"-D{k}={os.environ[k]}" for k in ("FKS_LIGHT_WAVES", "FKS_HEAVY_WAVES", "FKS_ROW_WAVES", "FKS_ROW_HEAVY_WAVES", "FKS_NP4_WAVES", "FKS_DUO_SLEEP", "FKS_WAVE_FLAT") if os.environ.get(k)]
    return [f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-fvisibility=hidden", "-ffp-contract=off",
            "-fno-fast-math", "-munsafe-fp-atomics", "-Wno-unused-result", *knobs,
            *_py_includes(), f"-I{CSRC_DIR / 'include'}", f"-I{CSRC_DIR / 'hip'}"]


def _hip_sources() -> List[Path]:
    return _deps("hip/*.hip", "hip/*.h", "hip/*.inc", "hip/*.cpp", "include/fks/*.hpp")


def hip_hash() -> str:
    return source_hash(_hip_sources(), _hip_flags() + [repr(HIP_UNITS)])


def build_hip(force: bool = False, jobs: int = 0) -> Path:
    """Compile every HIP unit for gfx950 (in parallel) and link ``_fks_hip``."""
    from concurrent.futures import ThreadPoolExecutor
    target = NATIVE_DIR / f"_fks_hip{_ext_suffix()}"
    want = hip_hash()
    if not (force or _stale(target, want)):
        return target
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    obj_dir = NATIVE_DIR.parent.parent / "build" / "hip_obj"
    obj_dir.mkdir(parents=True, exist_ok=True)
    flags = _hip_flags()
    cmds, objs = [], []
    for name, src, defs in HIP_UNITS:
        obj = obj_dir / f"{name}.o"
        objs.append(obj)
        extra = [f'-DFKS_SOURCE_HASH="{want}"'] if name == "module" else []
        cmds.append([hipcc, *flags, *defs, *extra, "-c", str(CSRC_DIR / "hip" / src), "-o", str(obj)])
    jobs = jobs or min(len(cmds), int(os.environ.get("MAX_JOBS", "0")) or os.cpu_count() or 1, 16)
    with ThreadPoolExecutor(jobs) as ex:
        list(ex.map(_run, cmds))
    tmp = target.with_name(target.name + f".{os.getpid()}.tmp")
    _run([hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", *map(str, objs), "-o", str(tmp),
          "-L/opt/rocm/lib", "-lrocprofiler-sdk-roctx", "-Wl,-rpath,/opt/rocm/lib"])
    os.replace(tmp, target)
    return target


def verify(module, which: str) -> None:
    """Refuse an extension whose embedded source hash is not the tree's
    (``FKS_ALLOW_STALE=1`` skips the check, e.g. for a bisect)."""
    if os.environ.get("FKS_ALLOW_STALE") == "1" or not (CSRC_DIR / "cpu").exists():
        return
    want = cpu_hash() if which == "cpu" else hip_hash()
    got = getattr(module, "SOURCE_HASH", "")
    if got != want:
        raise StaleExtension(f"{module.__name__} was built from other sources (embedded {got[:12] or 'none'}, "
                             f"tree {want[:12]}): rebuild with `python -m funsearch_kubernetes_simulator_amd.ops.build`")


def build_all(force: bool = False) -> None:
    """Build what is stale, then check every binary carries its tree's hash."""
    targets = [(build_cpu, cpu_hash, NATIVE_DIR / f"_fks_cpu{_ext_suffix()}")]
    if (CSRC_DIR / "hip" / "module.hip").exists():
        targets.append((build_hip, hip_hash, NATIVE_DIR / f"_fks_hip{_ext_suffix()}"))
    for fn, hfn, target in targets:
        want = hfn()
        state = "compiled" if (force or _stale(target, want)) else "up to date (embedded source hash matches), reused"
        fn(force)
        got = embedded_hash(target)
        if got != want:
            raise StaleExtension(f"{target.name}: embedded source hash {got[:12] or 'none'} != tree {want[:12]}")
        print(f"[fks build] {target.name}: {state}; source hash {want[:16]}", flush=True)
    from .gcnjit import build_all_skeletons
    for path in build_all_skeletons(force):
        print(f"[fks build] {path.name}: baseline-JIT code-object skeleton", flush=True)


if __name__ == "__main__":
    build_all(force="--force" in sys.argv)
