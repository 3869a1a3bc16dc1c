"""DeviceEvaluator's routing of native batches to the resident program service
(ops/hip_engine.py start_service / submit_native / ready / wait /
service_take), against a stand-in engine on the CPU that models the data
slots and done flags of csrc/hip/engine_host.hip.h (`service_poll`: every
finished program, filed under its batch): batches map to index ranges, rows the device did not take come back EXC_UNSUPPORTED, a
full service refuses, streaming collection returns finished rows early (a
straggler holds its own slot only), and modules are held until a batch is
complete.  The device side is covered by tests/test_gpu_service.py."""
import threading
import types

import numpy as np
import pytest

from funsearch_kubernetes_simulator_amd.ops import hip_engine as he


class _FakeEngine:
    def __init__(self, nslots):
        self.nslots, self.published = nslots, 0
        self.free = list(range(nslots))[::-1]
        self.row = {}           # slot -> fn value (the "result")
        self.held = {}          # slot -> index
        self.done = set()       # indexes finished on the "device"
        self.stopped = 0

    def service_start(self, slots, share, idle_polls=1 << 24):
        return {"blocks": 8, "slots": slots, "queue": 2 * slots, "per_cu": 8, "heap_top": 63, "lds": 1}

    def service_submit(self, fn, kc, koff):
        if len(self.free) < len(fn):
            return -1, np.zeros(0, np.int32)
        first = self.published
        slots = []
        for i, f in enumerate(fn):
            s = self.free.pop()
            self.row[s], self.held[s] = float(f), first + i
            slots.append(s)
        self.published += len(fn)
        return first, np.array(slots, np.int32)

    def service_poll(self):
        hit = sorted(s for s, ix in self.held.items() if ix in self.done)
        ids = np.array([self.held[s] for s in hit], np.int64)
        rows = np.zeros((len(hit), 13))
        for k, s in enumerate(hit):
            rows[k, 0] = self.row[s]
            self._free(s)
        return ids, rows, 1000 * (ids + 1)   # (device cycles)

    def _free(self, s):
        del self.held[s]
        self.free.append(s)

    def service_stop(self):
        self.stopped += 1

    def service_info(self):
        return {"blocks": 8, "unconsumed": self.nslots - len(self.free)}


class _FakeCompiler:
    max_modules = 2048
    defer_unloads = False

    def __init__(self):
        self.released = []

    def flush_unloads(self):
        return 0

    def prepare(self, progs):
        n = len(progs)
        ok = np.array([p != "host" for p in progs])
        return types.SimpleNamespace(ok=ok, fn=np.arange(1, n + 1, dtype=np.uint64) * 10,
                                     kc=np.zeros(4, np.int64), koff=np.zeros(n, np.int32),
                                     reasons=[""] * n, modules=("m", n))

    def release(self, mods):
        self.released.append(mods)


def _dev(nslots=8):
    d = object.__new__(he.DeviceEvaluator)
    d._eng = _FakeEngine(nslots)
    d._jit = _FakeCompiler()
    d.math_exact = True
    d._native_post, d._native_mods, d._svc, d._svc_post, d._svc_taken = {}, {}, None, {}, {}
    d._svc_firsts, d._svc_keys, d._svc_buf, d._svc_pumped, d._svc_orphans = [], [], {}, 0.0, 0
    d._svc_lock = threading.Lock()
    d.SERVICE_POLL_S = 0.0
    d._warm_s = 0.0
    d._svc_atexit = True
    return d


def test_service_routes_batches_by_slot():
    d = _dev()
    d.start_service(slots=8, share=1.0)
    base = d.SERVICE_SLOT_BASE
    d.submit_native(base, ["a", "host", "b"])        # native rows 0 and 2 -> indexes 0, 1
    d.submit_native(base + 1, ["c"])                 # index 2
    assert not d.ready(base) and not d.ready(base + 1)
    d._eng.done.update({2})
    assert d.ready(base + 1) and not d.ready(base)
    out1 = d.wait(base + 1)
    assert out1[0, 0] == 10.0
    d._eng.done.update({0, 1})
    out0 = d.wait(base)
    assert out0[0, 0] == 10.0 and out0[2, 0] == 30.0
    assert out0[1, 10] == 100.0                      # not taken by the device: EXC_UNSUPPORTED
    assert ("m", 1) in d._jit.released and ("m", 3) in d._jit.released
    with pytest.raises(RuntimeError):
        d.submit_native(base, ["x"] * 9)             # more programs than data slots
    d.stop_service()
    assert d._eng.stopped == 1 and d.service is None


def test_service_slot_reuse_before_collect_refused():
    d = _dev()
    d.start_service()
    d.submit_native(5, ["a"])
    with pytest.raises(RuntimeError):
        d.submit_native(5, ["b"])


def test_all_host_batch_is_ready_at_once():
    d = _dev()
    d.start_service()
    d.submit_native(3, ["host", "host"])
    assert d.ready(3)
    assert (d.wait(3)[:, 10] == 100.0).all()


def test_streaming_take_returns_finished_rows_early():
    """A straggler keeps its own data slot; the rest of its batch's rows and
    slots come back (and are reused by later batches) before it finishes."""
    d = _dev(nslots=4)
    d.start_service(slots=4)
    d.submit_native(0, ["a", "host", "b", "c"])      # indexes 0, 1, 2 in three data slots
    pos, rows, complete = d.service_take(0)          # nothing done yet: the declined row only
    assert list(pos) == [1] and rows[0, 10] == 100.0 and not complete
    d._eng.done.update({0, 2})                       # index 1 ("b") is the straggler
    pos, rows, complete = d.service_take(0)
    assert sorted(pos.tolist()) == [0, 3] and not complete
    assert sorted(rows[:, 0].tolist()) == [10.0, 40.0]
    d.submit_native(1, ["d", "e", "f"])              # reuses the two freed slots + the spare one
    d._eng.done.update({3, 4, 5})
    assert d.service_take(1)[2]
    pos, rows, complete = d.service_take(0)
    assert len(pos) == 0 and not complete
    d._eng.done.add(1)
    pos, rows, complete = d.service_take(0)
    assert pos.tolist() == [2] and rows[0, 0] == 30.0 and complete
    assert ("m", 4) in d._jit.released and 0 not in d._svc_post


def test_evaluator_collect_partial_streams_and_lists_fallbacks(default_workload):
    """`Evaluator.collect_partial`: finished native rows become results as they
    arrive; on completion the programs the device did not score (not native,
    or rows deferred to the host) are in ``fallback_idx``."""
    from funsearch_kubernetes_simulator_amd.engine import COLS, Evaluator, PendingPrograms

    class _Dev:
        def __init__(self):
            self.calls = 0

        def service_take(self, slot):
            self.calls += 1
            if self.calls == 1:   # native position 0 finished, scored
                r = np.zeros((1, 13)); r[0, COLS["score"]] = 0.5; r[0, COLS["n_events"]] = 7
                return np.array([0]), r, False
            r = np.zeros((1, 13)); r[0, COLS["exc"]] = 100.0   # position 1: declined -> host
            return np.array([1]), r, True

    ev = Evaluator(default_workload, device="cpu")
    ev.device = _Dev()
    pend = PendingPrograms(codes=["a", "b", "c"], slot=64, native_idx=[0, 2])
    got, complete = ev.collect_partial(pend)
    assert not complete and len(got) == 1 and got[0][0] == 0 and got[0][1].score == 0.5
    got, complete = ev.collect_partial(pend)
    assert complete and got == [] and pend.fallback_idx == [1, 2]


def test_service_news_and_cost_column():
    """service_news names the batches with rows to take (and first takes still
    due); taken rows carry the replay's device cycles in SERVICE_COST_COL."""
    d = _dev()
    d.start_service(slots=8)
    d.submit_native(0, ["a", "b"])          # indexes 0, 1
    d.submit_native(1, ["host"])            # nothing published: complete at its first take
    assert d.service_news() == {0, 1}
    pos, rows, complete = d.service_take(1)
    assert complete and list(pos) == [0] and rows.shape[1] == d.SERVICE_COST_COL + 1
    d.service_take(0)
    assert d.service_news() == set()
    d._eng.done.add(1)
    assert d.service_news() == {0}
    pos, rows, complete = d.service_take(0)
    assert list(pos) == [1] and rows[0, d.SERVICE_COST_COL] == 2000 and not complete


def test_rows_of_a_forgotten_batch_are_dropped():
    """A batch forgotten before all its rows arrived (an interrupted wait):
    its late rows are counted and dropped, never filed under the batch before
    it (they bisect into it)."""
    d = _dev()
    d.start_service(slots=8)
    d.submit_native(0, ["a", "b"])          # indexes 0, 1
    d.submit_native(1, ["c", "d"])          # indexes 2, 3
    with d._svc_lock:
        d._service_forget(1)
    d._eng.done.update({0, 2, 3})
    pos, rows, complete = d.service_take(0)
    assert list(pos) == [0] and not complete and d._svc_orphans == 2
    d._eng.done.add(1)
    pos, rows, complete = d.service_take(0)
    assert list(pos) == [1] and complete
