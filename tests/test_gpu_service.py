"""The resident program service (k_native_service, csrc/hip/replay_duo.hip.h):
a persistent grid of two-wave workgroups replaying programs from a host ring
must give rows bit-identical to the per-batch two-wave launch -- across ring
wrap-around, interleaved batches, a program that runs out of loop budget, and
a stop / restart of the grid."""
import numpy as np
import pytest

from funsearch_kubernetes_simulator_amd.policy.bytecode import Exc
from funsearch_kubernetes_simulator_amd.policy.compiler import compile_policy

from program_corpus import programs

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev(default_workload):
    from funsearch_kubernetes_simulator_amd.ops import hip_engine as he
    if not he.device_available():
        pytest.fail("GPU test collected but no HIP device is visible")
    d = he.DeviceEvaluator(default_workload)
    yield d
    d.stop_service()


def _batched(dev, progs, size):
    return np.concatenate([dev.evaluate_native(progs[i:i + size]) for i in range(0, len(progs), size)])


def test_service_rows_equal_batch_rows(dev):
    progs = programs()[:96]
    want = _batched(dev, progs, 32)
    info = dev.start_service(slots=64, share=0.25)   # 64 data slots, a 128-entry queue: both wrap
    try:
        assert info["blocks"] >= 1 and info["slots"] == 64 and info["queue"] == 128
        base = dev.SERVICE_SLOT_BASE
        got = np.zeros_like(want)
        # four batches of 16 in flight at once (the whole ring), collected out of order
        order = [(k, progs[k * 16:(k + 1) * 16]) for k in range(6)]
        inflight = {}
        for k, chunk in order:
            if len(inflight) == 4:
                old = max(inflight)          # the newest first: done flags are per program
                got[old * 16:(old + 1) * 16] = dev.wait(base + inflight.pop(old))
            dev.submit_native(base + k % 8, chunk)
            inflight[k] = k % 8
        for k, s in inflight.items():
            got[k * 16:(k + 1) * 16] = dev.wait(base + s)
        for i in range(len(progs)):
            assert np.array_equal(got[i], want[i]), (i, got[i], want[i])
        sv = dev.info()["service"]
        # (the corpus holds programs only the host engines take: not published)
        assert sv["running"] and sv["unconsumed"] == 0 and 48 <= sv["published"] <= 96
    finally:
        dev.stop_service()
    assert dev.service is None


def test_service_budget_exhaustion_and_restart(dev):
    runaway = compile_policy("def priority_function(pod, node):\n    x = 0\n    while True:\n        x += 1\n    return x\n")
    good = [compile_policy("def priority_function(pod, node):\n    return node.cpu_milli_left\n")] * 3
    want = dev.evaluate_native(good)
    dev.native_compiler.budget = 2000
    try:
        b = dev.native_compiler.prepare([runaway])
        assert b.ok.all()
        dev.release_native(b)
    finally:
        dev.native_compiler.budget = 1 << 22
    for _ in range(2):                      # start, stop, start again
        dev.start_service(slots=256, share=0.5)
        try:
            tab = dev.evaluate_native([runaway] + good)
        finally:
            dev.stop_service()
        assert int(tab[0, 10]) == Exc.BUDGET, tab[0]
        for i in range(3):
            assert np.array_equal(tab[1 + i], want[i])
    # batch launches work again after the grid left
    assert np.array_equal(dev.evaluate_native(good), want)


def test_service_many_small_batches(dev):
    """More batches than ring slots over the run (indexes far past the ring),
    one and two programs at a time: the claim / publish / done handshake."""
    progs = programs()[:40]
    want = _batched(dev, progs, 40)
    dev.start_service(slots=64, share=1.0)
    try:
        got = []
        for rep in range(3):
            for i in range(0, len(progs), 2):
                got.append(dev.evaluate_native(progs[i:i + 2]))
        got = np.concatenate(got)
    finally:
        dev.stop_service()
    for rep in range(3):
        for i in range(len(progs)):
            assert np.array_equal(got[rep * len(progs) + i], want[i]), (rep, i)


def test_service_abort_ends_replays_in_flight(dev):
    """abort_service: the replays in flight end early with EXC_TIMEOUT rows
    (programs already done keep their rows); a restarted grid replays normally."""
    progs = programs()[:32]
    want = dev.evaluate_native(progs)
    dev.start_service(slots=256, share=0.5)
    try:
        dev.submit_native(dev.SERVICE_SLOT_BASE, progs)
        dev.abort_service()
        got = dev.wait(dev.SERVICE_SLOT_BASE)
    finally:
        dev.stop_service()
    for i in range(len(progs)):
        if int(got[i, 10]) == Exc.TIMEOUT and int(want[i, 10]) != Exc.TIMEOUT:
            continue   # aborted
        assert np.array_equal(got[i], want[i]), i
    assert (got[:, 10] == Exc.TIMEOUT).sum() >= 1
    dev.start_service(slots=256, share=0.5)
    try:
        again = dev.evaluate_native(progs)
    finally:
        dev.stop_service()
    assert np.array_equal(again, want)


def test_service_idle_drain_and_revive(dev):
    """A grid with a tiny idle limit drains between submissions -- all of it:
    the first workgroup to time out sets the device-wide stop mirror -- and a
    submission published while it drains (or after) is replayed by the
    relaunch from the first unstarted index.  (A workgroup that left alone
    after claiming an index, while the rest stayed resident, lost that index.)"""
    import time
    progs = programs()[:24]
    want = dev.evaluate_native(progs)
    dev.start_service(slots=128, share=0.5, idle_polls=256)
    try:
        got = []
        for k, pause in enumerate((0.0, 0.0005, 0.002, 0.0, 0.01, 0.05, 0.001, 0.2)):
            time.sleep(pause)
            got.append(dev.evaluate_native(progs[3 * k:3 * k + 3]))
        sv = dev.info()["service"]
    finally:
        dev.stop_service()
    got = np.concatenate(got)
    for i in range(len(progs)):
        assert np.array_equal(got[i], want[i]), i
    assert sv["launches"] >= 2 and sv["idle_polls"] == 256, sv


def test_service_event_budget(dev):
    """max_events: a replay past the budget ends with EXC_EVENTS (final, never
    deferred to the host); with the budget off the same programs replay in full,
    equal to the batch launch."""
    from funsearch_kubernetes_simulator_amd.engine import NATIVE_DEFER
    progs = programs()[:16]
    want = dev.evaluate_native(progs)
    native = [i for i in range(len(progs)) if int(want[i, 10]) not in NATIVE_DEFER]
    assert native
    dev.set_options(max_events=2048)
    try:
        dev.start_service(slots=256, share=0.5)
        try:
            capped = dev.evaluate_native(progs)
        finally:
            dev.stop_service()
    finally:
        dev.set_options(max_events=0)
    assert int(Exc.EVENTS) not in NATIVE_DEFER
    for i in native:
        if want[i, 8] > 2048 + 1024:        # n_events: over the budget -> capped
            assert int(capped[i, 10]) == Exc.EVENTS, (i, capped[i])
        else:
            assert np.array_equal(capped[i], want[i]), i
    assert dev.info()["max_events"] == 0


def test_service_rtcall_population_matches_vm(dev, default_workload):
    """Regression (round 6): an evolved population whose baseline-JIT code
    calls the runtime library with its feasibility prologue compiled out.  The
    RT-call sequence spilled SGPRs with v_writelane into a caller-saved VGPR
    without restoring that VGPR's inactive lanes; the service's caller keeps
    the zeroed score of the infeasible nodes there across the call, so 43 of
    these 80 programs placed pods on infeasible nodes (EXC_ALLOC, or 0.79
    against the true 0.4467) -- on the service only, the per-batch kernels'
    register allocation happened not to expose it."""
    import json
    from pathlib import Path

    from funsearch_kubernetes_simulator_amd.ops import cpu_engine as ce
    from funsearch_kubernetes_simulator_amd.policy.compiler import try_compile
    path = Path(__file__).resolve().parents[1] / "data" / "diag" / "r6i_population.json"
    progs = [p for p in (try_compile(x["code"])[0] for x in json.load(open(path))["programs"]) if p is not None]
    assert len(progs) == 80
    vm = np.asarray(ce.simulate_program_batch(default_workload, progs, threads=8))
    dev.start_service(slots=1024, share=0.875)
    try:
        got = dev.evaluate_native(progs)
    finally:
        dev.stop_service()
    bad = [i for i in range(len(progs)) if not (got[i, 0] == vm[i, 0] and got[i, 8] == vm[i, 8]
                                                and int(got[i, 10]) == int(vm[i, 10]))]
    assert not bad, [(i, got[i, [0, 8, 10]].tolist(), vm[i, [0, 8, 10]].tolist()) for i in bad[:8]]
