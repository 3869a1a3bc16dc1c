"""DeviceEvaluator's routing of native batches to the resident program service
(ops/hip_engine.py start_service / submit_native / ready / wait), against a
stand-in engine on the CPU: slots map to ring index ranges, rows the device
did not take come back EXC_UNSUPPORTED, the ring-full refusal surfaces, and
modules are held until the batch is collected.  The device side is covered by
tests/test_gpu_service.py."""
import types

import numpy as np
import pytest

from funsearch_kubernetes_simulator_amd.ops import hip_engine as he


class _FakeEngine:
    def __init__(self, ring):
        self.ring, self.published, self.rows, self.done = ring, 0, {}, set()
        self.started = self.stopped = 0

    def service_start(self, ring, share):
        self.started += 1
        return {"blocks": 8, "ring": ring, "per_cu": 8, "heap_top": 63, "lds": 1}

    def service_submit(self, fn, kc, koff):
        if self.published + len(fn) - min(self.rows or [self.published]) > self.ring:
            return -1
        first = self.published
        for i, f in enumerate(fn):
            self.rows[first + i] = float(f)
        self.published += len(fn)
        return first

    def service_ready(self, first, n):
        return all(first + i in self.done for i in range(n))

    def service_collect(self, first, n):
        out = np.zeros((n, 13))
        for i in range(n):
            out[i, 0] = self.rows.pop(first + i)
        return out

    def service_stop(self):
        self.stopped += 1

    def service_info(self):
        return {"blocks": 8}


class _FakeCompiler:
    def __init__(self):
        self.released = []

    def prepare(self, progs):
        n = len(progs)
        ok = np.array([p != "host" for p in progs])
        return types.SimpleNamespace(ok=ok, fn=np.arange(1, n + 1, dtype=np.uint64) * 10,
                                     kc=np.zeros(4, np.int64), koff=np.zeros(n, np.int32),
                                     reasons=[""] * n, modules=("m", n))

    def release(self, mods):
        self.released.append(mods)


def _dev(ring=8):
    d = object.__new__(he.DeviceEvaluator)
    d._eng = _FakeEngine(ring)
    d._jit = _FakeCompiler()
    d.math_exact = True
    d._native_post, d._native_mods, d._svc, d._svc_post = {}, {}, None, {}
    d._warm_s = 0.0
    return d


def test_service_routes_batches_by_slot():
    d = _dev()
    d.start_service(ring=8, share=1.0)
    base = d.SERVICE_SLOT_BASE
    d.submit_native(base, ["a", "host", "b"])        # native rows 0 and 2 -> ring indexes 0, 1
    d.submit_native(base + 1, ["c"])                 # ring index 2
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
        d.submit_native(base, ["x"] * 9)             # more than the ring holds
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
