"""Host sanitizer builds of the native engine.

The C++ self-test (csrc/cpu/selftest.cpp) is compiled with AddressSanitizer +
UndefinedBehaviorSanitizer, and separately with ThreadSanitizer, and must run
clean AND reproduce the optimised extension's scores (golden first-fit /
best-fit values, the reference's published programs through the bytecode VM,
and a threaded batch over the shared workload).
"""
import shutil
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "tools"))

pytestmark = pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")


def test_asan_ubsan_selftest_clean_and_exact(capsys):
    import sanitize_cpu
    assert sanitize_cpu.main(["--quick"]) == 0
    out = capsys.readouterr().out
    assert "selftest ok" in out and "0 mismatches; asan clean" in out


@pytest.mark.slow
def test_tsan_threaded_batch_race_free(capsys):
    import sanitize_cpu
    assert sanitize_cpu.main(["--tsan", "--quick", "--threads", "4"]) == 0
    out = capsys.readouterr().out
    assert "0 differ from serial" in out and "tsan clean" in out
