"""In-tree build of the native extensions.

* ``_fks_cpu``  - C++17 oracle engine + bytecode VM (g++, pybind11);
* ``_fks_hip``  - MI355X replay kernels (hipcc ``--offload-arch=gfx950``,
  pybind11 host side).  It links ``libamdhip64.so.7`` by SONAME so that, once
  ``torch`` is imported, the process shares torch's HIP runtime.

Both land next to this file so they travel with the repository snapshot to
the GPU box.  ``python -m funsearch_kubernetes_simulator_amd.ops.build``
rebuilds whatever is stale (sources newer than the .so).
"""

from __future__ import annotations

import os
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


def _stale(target: Path, sources: List[Path]) -> bool:
    if not target.exists():
        return True
    t = target.stat().st_mtime
    return any(s.stat().st_mtime > t for s in sources)


def _run(cmd: List[str]) -> None:
    print("[fks build]", " ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)


def _deps(*globs: str) -> List[Path]:
    out: List[Path] = []
    for g in globs:
        out.extend(sorted(CSRC_DIR.glob(g)))
    return out


def build_cpu(force: bool = False) -> Path:
    target = NATIVE_DIR / f"_fks_cpu{_ext_suffix()}"
    srcs = _deps("cpu/*.cpp", "cpu/*.hpp", "include/fks/*.hpp", "jit/*", "hip/jit_abi.h", "hip/pyops_dev.h",
                 "hip/dd_math.h", "hip/jit_env.h", "hip/exc_codes.h")
    if force or _stale(target, srcs):
        cxx = os.environ.get("CXX", "g++")
        cmd = [cxx, "-O3", "-std=c++17", "-shared", "-fPIC", "-fvisibility=hidden",
               "-ffp-contract=off", "-fno-fast-math", "-Wall", "-Wno-unused-function",
               *_py_includes(), f"-I{CSRC_DIR / 'include'}", str(CSRC_DIR / "cpu" / "module.cpp"),
               str(CSRC_DIR / "jit" / "gcn_jit.cpp"), "-o", str(target), "-lpthread"]
        _run(cmd)
    return target


#: Device translation units of _fks_hip: (object name, extra defines).  The
#: replay kernels are split per NPASS and kind so their many template
#: instances compile in parallel.
HIP_UNITS = [("module", "module.hip", []), ("screen", "screen.hip", [])] + [
    (f"replay_k{kind}_np{npass}", "replay_kernels.hip", [f"-DFKS_KIND={kind}", f"-DFKS_NPASS={npass}"])
    for kind, npasses in ((0, (1, 2, 4)), (1, (1, 2, 4)), (2, (1,)), (3, (1,)), (4, (1, 2, 4))) for npass in npasses]


def _hip_flags() -> List[str]:
    # occupancy knobs of the replay kernels (waves per SIMD), for A/B builds
    knobs = [f"-D{k}={os.environ[k]}" for k in ("FKS_LIGHT_WAVES", "FKS_HEAVY_WAVES", "FKS_ROW_WAVES", "FKS_ROW_HEAVY_WAVES", "FKS_NP4_WAVES", "FKS_DUO_SLEEP") if os.environ.get(k)]
    return [f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-fvisibility=hidden", "-ffp-contract=off",
            "-fno-fast-math", "-munsafe-fp-atomics", "-Wno-unused-result", *knobs,
            *_py_includes(), f"-I{CSRC_DIR / 'include'}", f"-I{CSRC_DIR / 'hip'}"]


def build_hip(force: bool = False, jobs: int = 0) -> Path:
    """Compile every HIP unit for gfx950 (in parallel) and link ``_fks_hip``."""
    from concurrent.futures import ThreadPoolExecutor
    target = NATIVE_DIR / f"_fks_hip{_ext_suffix()}"
    srcs = _deps("hip/*.hip", "hip/*.h", "hip/*.cpp", "include/fks/*.hpp")
    if not (force or _stale(target, srcs)):
        return target
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    obj_dir = NATIVE_DIR.parent.parent / "build" / "hip_obj"
    obj_dir.mkdir(parents=True, exist_ok=True)
    flags = _hip_flags()
    cmds, objs = [], []
    for name, src, defs in HIP_UNITS:
        obj = obj_dir / f"{name}.o"
        objs.append(obj)
        cmds.append([hipcc, *flags, *defs, "-c", str(CSRC_DIR / "hip" / src), "-o", str(obj)])
    jobs = jobs or min(len(cmds), int(os.environ.get("MAX_JOBS", "0")) or os.cpu_count() or 1, 16)
    with ThreadPoolExecutor(jobs) as ex:
        list(ex.map(_run, cmds))
    _run([hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", *map(str, objs), "-o", str(target),
          "-L/opt/rocm/lib", "-lrocprofiler-sdk-roctx", "-Wl,-rpath,/opt/rocm/lib"])
    return target


def _report(target: Path, before: float) -> None:
    """One line per extension: compiled now, or reused (its sources are older)."""
    after = target.stat().st_mtime if target.exists() else -1.0
    state = "compiled" if after != before else "up to date (sources older than the .so), reused"
    print(f"[fks build] {target.name}: {state}", flush=True)


def build_all(force: bool = False) -> None:
    targets = [(build_cpu, NATIVE_DIR / f"_fks_cpu{_ext_suffix()}")]
    if (CSRC_DIR / "hip" / "module.hip").exists():
        targets.append((build_hip, NATIVE_DIR / f"_fks_hip{_ext_suffix()}"))
    for fn, target in targets:
        before = target.stat().st_mtime if target.exists() else -1.0
        fn(force)
        _report(target, before)


if __name__ == "__main__":
    build_all(force="--force" in sys.argv)
