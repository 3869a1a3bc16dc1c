"""Device primitives: DPP wave reductions and the wave-parallel heapq."""
import heapq

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def hip():
    from funsearch_kubernetes_simulator_amd.ops import hip_engine as he
    if not he.device_available():
        pytest.fail("GPU test collected but no HIP device is visible")
    return he.native()


def test_wave_ops(hip):
    rng = np.random.default_rng(3)
    for _ in range(5):
        v = rng.integers(0, 2 ** 62, 64, dtype=np.uint64)
        out = hip.test_wave_ops(v)
        assert out[0] == v.max()
        assert out[1] == (v.sum(dtype=np.uint64))
        sw = v.reshape(32, 2)[:, ::-1].reshape(-1)
        assert np.array_equal(out[2:66], sw)
        lo = (v & np.uint64(0xFFFFFFFF)).astype(np.uint32).view(np.int32).astype(np.int64)
        sh = out[66:130].view(np.int64)
        for lane in range(64):
            expect = -1 if lane % 16 == 0 else lo[lane - 1]
            assert sh[lane] == expect, lane


@pytest.mark.parametrize("seed", range(6))
def test_wave_heap_matches_heapq(hip, seed):
    rng = np.random.default_rng(seed)
    lb = 7
    n0 = int(rng.integers(1, 1500))
    keys = [(int(t) << lb) | int(k & 3) for k, t in enumerate(rng.integers(0, 10 ** 6, n0) * 4096 + np.arange(n0))]
    heapq.heapify(keys)
    ops, ref, popped = [], list(keys), []
    for step in range(1200):
        if ref and rng.random() < 0.5:
            popped.append(heapq.heappop(ref))
            ops.append(-1)
        else:
            x = ((int(rng.integers(0, 10 ** 6)) * 4096 + 2000 + step) << lb) | int(rng.integers(0, 4))
            heapq.heappush(ref, x)
            ops.append(x)
    out, pops = hip.test_heap(np.array(keys, dtype=np.uint64), np.array(ops, dtype=np.int64), lb)
    assert list(pops[:len(popped)]) == popped
    assert list(out) == ref
