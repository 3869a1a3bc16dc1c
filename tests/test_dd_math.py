"""Device exact math (csrc/hip/dd_math.h) on the host: the kernels' pow / exp /
log are __host__ __device__, so the C++ harness csrc/tools/dd_math_check.cpp
runs the very same arithmetic with g++ and compares it with glibc (what
CPython's `**`, math.exp and math.log call).

Finding recorded here (parity note): the device returns the *correctly
rounded* result; glibc's pow / exp / log are not correctly rounded (<= 0.52
ULP), so about 0.08% of pow / exp calls (a few per million for log) differ
from CPython by one ULP.  Every such difference is checked below to be a case
where the device value is the correctly rounded one.  A one-ULP difference
changes a replay only if it moves a node's `int(score)` across an integer or
flips a comparison whose sides are within one ULP; the device == CPU-VM replay
tests (which use glibc) have not hit one."""
import os
import re
import subprocess
from decimal import Decimal, getcontext

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def harness(tmp_path_factory):
    exe = str(tmp_path_factory.mktemp("dd") / "dd_math_check")
    r = subprocess.run(["g++", "-O2", "-std=c++17", "-DFKS_HOST_JIT", "-ffp-contract=off",
                        "-I", os.path.join(ROOT, "csrc", "hip"), os.path.join(ROOT, "csrc", "tools", "dd_math_check.cpp"),
                        "-o", exe], capture_output=True, text=True)
    if r.returncode != 0:
        pytest.skip(f"g++ unavailable: {r.stderr[-500:]}")
    return exe


def _cr(v: Decimal) -> float:
    return float(v)   # Decimal -> float is correctly rounded


def test_device_math_is_correctly_rounded_where_glibc_differs(harness):
    getcontext().prec = 80
    out = subprocess.run([harness, "200000", "7"], capture_output=True, text=True).stdout
    stats = {m.group(1): {k: float(v) for k, v in re.findall(r"(\w+)=([\d.]+)", m.group(0))}
             for m in re.finditer(r"^(pow|exp|log) calls=.*$", out, re.M)}
    assert set(stats) == {"pow", "exp", "log"}
    for name, st in stats.items():
        assert st["mismatches"] <= 0.002 * st["calls"], (name, st)   # glibc's own <= 0.52 ULP error
        assert st["defers"] <= 0.001 * st["calls"], (name, st)
    checked = 0
    for m in re.finditer(r"^pow mismatch x=(\S+) y=(\S+) dev=(\S+) glibc=(\S+)$", out, re.M):
        x, y, dev, gl = (float(g) for g in m.groups())
        assert dev == _cr((Decimal(y) * Decimal(x).ln()).exp()) and dev != gl
        checked += 1
    for m in re.finditer(r"^exp mismatch x=(\S+) dev=(\S+) glibc=(\S+)$", out, re.M):
        x, dev, gl = (float(g) for g in m.groups())
        assert dev == _cr(Decimal(x).exp()) and dev != gl
        checked += 1
    for m in re.finditer(r"^log mismatch x=(\S+) dev=(\S+) glibc=(\S+)$", out, re.M):
        x, dev, gl = (float(g) for g in m.groups())
        assert dev == _cr(Decimal(x).ln()) and dev != gl
        checked += 1
    assert checked > 0
