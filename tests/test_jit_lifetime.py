"""Bounded JIT module lifetime (ops/jit.py NativeCompiler): reference-counted
modules, LRU retirement of modules no batch in flight calls into, eviction of
their shapes from the cache.  Host-only logic, exercised with stand-in module
handles (the GPU path is tests/test_gpu_native.py)."""
import threading

from funsearch_kubernetes_simulator_amd.ops.jit import NativeCompiler


class FakeHandle:
    def __init__(self):
        self.unloaded = False

    def unload(self):
        assert not self.unloaded
        self.unloaded = True


def _compiler(max_modules):
    nc = NativeCompiler.__new__(NativeCompiler)
    nc._lock = threading.Lock()
    nc._modules, nc._shapes, nc._ptr, nc._tier_of, nc._uses = {}, {}, {}, {}, {}
    nc._next_mod = nc._seq = 0
    nc.max_modules = max_modules
    nc._evicted = set()
    nc.stats = {"modules": 0, "live_modules": 0, "max_live_modules": 0, "retired_modules": 0,
                "evicted_shapes": 0, "recompiled_shapes": 0, "unload_s": 0.0}
    return nc


def _load(nc, keys):
    h = FakeHandle()
    with nc._lock:
        nc._seq += 1
        mid = nc._add_module(h, "baseline")
        for j, k in enumerate(keys):
            nc._map_shape(k, mid, j, 0x1000 * (mid + 1) + 256 * j)
            nc._tier_of[k] = "baseline"
    return mid, h


def _hold(nc, mids):
    with nc._lock:
        nc._seq += 1
        for m in mids:
            nc._modules[m].refs += 1
            nc._modules[m].last_use = nc._seq


def test_lru_retirement_skips_modules_in_flight():
    nc = _compiler(4)
    mods = [_load(nc, [f"s{i}a", f"s{i}b"]) for i in range(4)]
    _hold(nc, [mods[0][0]])                 # module 0: a batch in flight (and the most recent use)
    _load(nc, ["s4a"])                      # 5 live > 4
    nc._retire()
    # down to 3 live: the two least recently used idle modules (1, 2) go; 0 is held
    assert nc.stats["live_modules"] == 3 and nc.stats["retired_modules"] == 2
    assert mods[1][1].unloaded and mods[2][1].unloaded and not mods[0][1].unloaded
    assert "s1a" not in nc._shapes and "s2b" not in nc._shapes and "s0a" in nc._shapes
    assert nc.stats["evicted_shapes"] == 4
    assert hash("s1a") in nc._evicted and hash("s0a") not in nc._evicted   # recompile accounting
    nc.release([mods[0][0]])
    assert not mods[0][1].unloaded          # at the cap: nothing more to retire


def test_remapped_shape_is_not_evicted_with_its_old_module():
    nc = _compiler(1)
    m0, h0 = _load(nc, ["x", "y"])
    m1, h1 = _load(nc, ["x"])               # tier-up: x now lives in module 1
    assert nc._shapes["x"][0] == m1 and "x" not in nc._modules[m0].shapes
    _hold(nc, [m1])
    nc._retire()
    assert h0.unloaded and not h1.unloaded
    assert "x" in nc._shapes and "y" not in nc._shapes
