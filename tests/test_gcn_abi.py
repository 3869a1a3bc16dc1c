"""ABI of the baseline JIT's machine code (csrc/jit/gcn_lower.hpp), checked on
the disassembly of real programs: the generated function writes no
callee-saved register, and the runtime-library call sequence leaves the
inactive lanes of its SGPR-spill VGPR as it found them (v_writelane ignores
EXEC; an LLVM caller may keep values in those lanes across the call -- the
round-6 service mis-score, tests/test_gpu_service.py)."""
import json
import re
import shutil
import subprocess
from pathlib import Path

import numpy as np
import pytest

from funsearch_kubernetes_simulator_amd.ops import gcnjit
from funsearch_kubernetes_simulator_amd.policy.compiler import try_compile

from program_corpus import programs

MC = Path("/opt/rocm/lib/llvm/bin/llvm-mc")
POP = Path(__file__).resolve().parents[1] / "data" / "diag" / "r6i_population.json"

pytestmark = pytest.mark.skipif(not MC.exists() and shutil.which("llvm-mc") is None,
                                reason="llvm-mc (ROCm LLVM) not installed")


def _disasm(words: np.ndarray) -> list:
    txt = " ".join("0x%02x" % b for b in words.astype("<u4").tobytes())
    out = subprocess.run([str(MC) if MC.exists() else "llvm-mc", "-arch=amdgcn", "-mcpu=gfx950", "--disassemble"],
                         input=txt, capture_output=True, text=True, check=True)
    assert "invalid" not in out.stderr, out.stderr[:400]
    return [ln.strip() for ln in out.stdout.splitlines() if ln.strip() and not ln.strip().startswith(".")]


def _regs(operand: str, kind: str) -> list:
    m = re.fullmatch(kind + r"(\d+)", operand)
    if m:
        return [int(m.group(1))]
    m = re.fullmatch(kind + r"\[(\d+):(\d+)\]", operand)
    if m:
        return list(range(int(m.group(1)), int(m.group(2)) + 1))
    return []


def _callee_saved_v(r: int) -> bool:
    return r >= 40 and (r - 40) % 16 < 8          # v40-47, v56-63, ..., v120-127


def _callee_saved_s(r: int) -> bool:
    return 34 <= r <= 39 or (r >= 48 and (r - 48) % 16 < 8 and r <= 103)   # s34-39, s48-55, ..., s96-103


def _population():
    progs = [p for p in (try_compile(x["code"])[0] for x in json.load(open(POP))["programs"]) if p is not None]
    # the corpus too: a spread of shapes (loops, calls, tags, spills)
    return progs[::4] + programs()[:48]


def test_no_callee_saved_writes_and_spill_vgpr_restored():
    progs = _population()
    codes = gcnjit.compile_many(progs)
    calls = checked = 0
    for p, (code, why) in zip(progs, codes):
        if code is None:
            continue
        checked += 1
        lines = _disasm(code.words)
        for ln in lines:
            op, _, rest = ln.partition(" ")
            dst = rest.split(",")[0].strip() if rest else ""
            if op.startswith(("v_", "scratch_load", "ds_read", "global_load")) and not op.startswith(
                    ("v_readlane", "v_readfirstlane", "v_cmp")):
                assert not any(_callee_saved_v(r) for r in _regs(dst, "v")), ln
            if op.startswith(("s_", "v_readlane", "v_readfirstlane")) and not op.startswith(
                    ("s_cbranch", "s_waitcnt", "s_setpc", "s_nop", "s_branch")):
                assert not any(_callee_saved_s(r) for r in _regs(dst, "s")), ln
        # every runtime call: the spill VGPR's own contents stored before the
        # first v_writelane into it and reloaded (same slot) after the last readlane
        i = 0
        while i < len(lines):
            if not lines[i].startswith("v_writelane_b32"):
                i += 1
                continue
            calls += 1
            spill = lines[i].split()[1].rstrip(",")
            before = [ln for ln in lines[max(0, i - 64):i] if ln.startswith("scratch_store_dword")
                      and ln.split(",")[1].strip() == spill]
            assert before, ("spill VGPR not saved before v_writelane", spill, lines[i])
            slot = re.search(r"offset:(\d+)", before[-1])
            slot = slot.group(1) if slot else "0"
            j = i
            while j < len(lines) and not lines[j].startswith("v_readlane_b32"):
                j += 1
            while j < len(lines) and lines[j].startswith("v_readlane_b32"):
                j += 1
            after = lines[j] if j < len(lines) else ""
            m = re.search(r"offset:(\d+)", after)
            assert after.startswith("scratch_load_dword " + spill + ",") and (m.group(1) if m else "0") == slot, \
                ("spill VGPR not reloaded after the readlanes", spill, after)
            i = j
    assert checked >= 40 and calls >= 10, (checked, calls)
