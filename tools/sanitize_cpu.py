"""Host-sanitizer run of the native C++ engine (race/memory checking).

GPU AddressSanitizer is not available on the MI355X pool, so the memory and UB
checking runs on the host: ``csrc/cpu/selftest.cpp`` (CSV reader -> workload ->
built-in scorers + bytecode VM, with the invariant checker on) is built with
``-fsanitize=address,undefined -fno-sanitize-recover=all`` and run on the default
trace; the programs it replays (the reference's published policies, discovered
family champions, random composite programs) are compiled here and their scores
compared with the regular optimised extension, so the sanitized build must be
both clean and exact.

A ThreadSanitizer build (``--tsan``) runs the same policies as one threaded
batch over the shared workload, the way the ``simulate_*_batch`` entry points do.

    python tools/sanitize_cpu.py            # ASan + UBSan; exit 0 = clean and exact
    python tools/sanitize_cpu.py --tsan     # ThreadSanitizer on the threaded batch path
    python tools/sanitize_cpu.py --quick    # reference policies only (the CPU test suite)
"""
from __future__ import annotations

import argparse
import os
import re
import struct
import subprocess
import sys
import tempfile
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

SANITIZE = {
    "asan": ["-fsanitize=address,undefined", "-fno-sanitize-recover=all", "-fno-omit-frame-pointer"],
    "tsan": ["-fsanitize=thread", "-fno-omit-frame-pointer"],
}


def build(out: Path, kind: str = "asan") -> Path:
    exe = out / f"fks_selftest_{kind}"
    cmd = [os.environ.get("CXX", "g++"), "-std=c++17", "-O1", "-g", "-ffp-contract=off", *SANITIZE[kind],
           f"-I{ROOT / 'csrc/include'}", f"-I{ROOT / 'csrc/cpu'}", str(ROOT / "csrc/cpu/selftest.cpp"),
           "-o", str(exe), "-lpthread"]
    subprocess.run(cmd, check=True)
    return exe


def dump_programs(pdir: Path, quick: bool = False) -> dict:
    """Writes <name>.code / <name>.consts and returns {name: compiled policy}."""
    import numpy as np

    from funsearch_kubernetes_simulator_amd.models import families as fam
    from funsearch_kubernetes_simulator_amd.models import library
    from funsearch_kubernetes_simulator_amd.policy.bytecode import TAG_FLOAT
    from funsearch_kubernetes_simulator_amd.policy.compiler import compile_policy

    sources = dict(library.reference_policies())
    for name, rec in ({} if quick else library.discovered_policies()).items():
        sources[f"discovered_{name}"] = rec["code"]
    rng = np.random.default_rng(7)
    for family in (() if quick else ("composite_linear", "feature_linear")):
        for k, wts in enumerate(fam.SAMPLERS[family](2, rng)):
            sources[f"{family}_{k}"] = fam.to_program(family, wts)
    progs = {}
    for name, src in sources.items():
        safe = re.sub(r"[^A-Za-z0-9_.-]", "_", name)
        p = compile_policy(src)
        (pdir / f"{safe}.code").write_bytes(p.code)
        lines = []
        for tag, iv, fv in zip(p.ctag, p.iconst, p.fconst):
            payload = struct.unpack("<q", struct.pack("<d", fv))[0] if tag == TAG_FLOAT else int(iv)
            lines.append(f"{int(tag)} {payload}")
        (pdir / f"{safe}.consts").write_text("\n".join(lines) + "\n")
        progs[safe] = p
    return progs


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--tsan", action="store_true", help="ThreadSanitizer build instead of ASan+UBSan")
    ap.add_argument("--quick", action="store_true", help="reference policies only")
    ap.add_argument("--threads", type=int, default=4)
    args = ap.parse_args(argv)
    kind = "tsan" if args.tsan else "asan"
    from funsearch_kubernetes_simulator_amd.core.traces import load_default_workload
    from funsearch_kubernetes_simulator_amd.ops import cpu_engine as ce

    with tempfile.TemporaryDirectory() as td:
        td = Path(td)
        exe = build(td, kind)
        pdir = td / "progs"
        pdir.mkdir()
        progs = dump_programs(pdir, args.quick)
        env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:halt_on_error=1",
                   UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1", TSAN_OPTIONS="halt_on_error=1")
        r = subprocess.run([str(exe), str(ROOT / "data/traces"), str(pdir), str(args.threads)],
                           capture_output=True, text=True, env=env)
    print(r.stdout, end="")
    if r.returncode != 0 or any(t in r.stderr for t in ("runtime error", "ERROR: AddressSanitizer",
                                                          "WARNING: ThreadSanitizer")):
        print(r.stderr, file=sys.stderr)
        print(f"sanitized self-test FAILED (exit {r.returncode})")
        return 1
    w = load_default_workload()
    opts = ce.SimOptions(check_invariants=97)
    bad = 0
    got = {m.group(1): (int(m.group(2)), float(m.group(3)))
           for m in re.finditer(r"^program (\S+): exc (-?\d+) score (\S+)", r.stdout, re.M)}
    for name, p in progs.items():
        ref = ce.simulate_program(w, p, opts)
        if got.get(name) != (ref["exc"], ref["score"]):
            print(f"MISMATCH {name}: sanitized {got.get(name)} vs extension {(ref['exc'], ref['score'])}")
            bad += 1
    print(f"{len(progs)} programs compared, {bad} mismatches; {kind} clean")
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
