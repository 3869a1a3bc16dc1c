"""Natively compiled programs on the MI355X (k_replay_native + run-time JIT)
vs the CPU bytecode VM: full replays of the whole program corpus on the FULL
8,152-pod trace, bit-identical rows (score, means, counts, exception class,
event-trace hash)."""
import numpy as np
import pytest

from funsearch_kubernetes_simulator_amd.models.library import reference_policies, reference_scores
from funsearch_kubernetes_simulator_amd.ops import cpu_engine as ce
from funsearch_kubernetes_simulator_amd.policy.bytecode import Exc
from funsearch_kubernetes_simulator_amd.policy.compiler import compile_policy

from program_corpus import programs

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev(default_workload):
    from funsearch_kubernetes_simulator_amd.ops import hip_engine as he
    if not he.device_available():
        pytest.fail("GPU test collected but no HIP device is visible")
    return he.DeviceEvaluator(default_workload)


def test_reference_programs_native_exact(dev):
    ref = reference_scores()
    names = list(reference_policies())
    tab = dev.evaluate_native([compile_policy(reference_policies()[k]) for k in names])
    for k, row in zip(names, tab):
        assert row[10] == 0, (k, row)
        assert row[0] == ref[k], (k, row[0], ref[k])


def test_native_equals_cpu_vm_full_trace(dev, default_workload):
    progs = programs()
    nat = dev.evaluate_native(progs)
    vm = ce.simulate_program_batch(default_workload, progs, threads=16)
    compared = 0
    skipped = []
    for i, p in enumerate(progs):
        if int(nat[i, 10]) in (Exc.UNSUPPORTED, Exc.BUDGET) or int(vm[i, 10]) in (Exc.UNSUPPORTED, Exc.BUDGET):
            skipped.append((i, int(nat[i, 10]), int(vm[i, 10])))
            continue
        assert np.array_equal(nat[i], vm[i]), (i, p.source[-400:], nat[i], vm[i])
        compared += 1
    # only programs the engines defer by design (trig, bigint, near-tie math) may be skipped
    assert compared >= len(progs) - 4, skipped


@pytest.mark.parametrize("layout", [{"native_rows": 1, "native_duo": False}, {"native_rows": 1, "native_duo": True},
                                    {"native_rows": 4}, {"row_kernel": "off"}],
                         ids=["rows1", "duo", "rows4", "wave"])
def test_native_kernel_layouts_agree(dev, default_workload, layout):
    """Row kernel with one / four programs per wave, the two-wave (heap wave +
    scoring wave) kernel and the one-wave-per-program kernel: every row
    bit-identical to the CPU VM (score, means, counts, trace hash)."""
    progs = programs()[:24]
    vm = ce.simulate_program_batch(default_workload, progs, threads=16)
    dev.set_options(**layout)
    try:
        nat = dev.evaluate_native(progs)
        info = dev.info()
    finally:
        dev.set_options(native_rows=0, row_kernel="auto", native_duo=True)
    if "native_rows" in layout:
        want = 0 if layout.get("native_duo") else layout["native_rows"]   # 0: the two-wave kernel
        assert info["native_rows_last"] == want, info
    for i, p in enumerate(progs):
        if int(nat[i, 10]) in (Exc.UNSUPPORTED, Exc.BUDGET) or int(vm[i, 10]) in (Exc.UNSUPPORTED, Exc.BUDGET):
            continue
        assert np.array_equal(nat[i], vm[i]), (layout, i, nat[i], vm[i])


def test_shape_cache_reuses_compiled_code(dev):
    a = compile_policy("def priority_function(pod, node):\n    return 5000 - node.cpu_milli_left * 0.25\n")
    b = compile_policy("def priority_function(pod, node):\n    return 7000 - node.cpu_milli_left * 0.5\n")
    first = dev.native_compiler.prepare([a])
    second = dev.native_compiler.prepare([b])
    assert second.compiled == 0 and second.ok.all()
    assert first.fn[0] == second.fn[0]       # one function, different constant blocks
    tab = dev.evaluate_native([a, b])
    cpu = ce.simulate_program_batch(dev.workload, [a, b], threads=2)
    assert np.array_equal(tab, cpu)


def test_runaway_native_program_drains(dev):
    prog = compile_policy("def priority_function(pod, node):\n    x = 0\n    while True:\n        x += 1\n    return x\n")
    dev.native_compiler.budget = 2000
    try:
        fresh = dev.native_compiler.prepare([prog])
        assert fresh.ok.all()
        tab = dev.evaluate_native([prog])
    finally:
        dev.native_compiler.budget = 1 << 22
    assert int(tab[0, 10]) == Exc.BUDGET


def test_engine_routes_small_batches_to_native(default_workload):
    from funsearch_kubernetes_simulator_amd.engine import Evaluator
    ev = Evaluator(default_workload, device="gpu")
    res = ev.evaluate_programs(list(reference_policies().values())[:3])
    assert [r.engine for r in res] == ["hip-native"] * 3
    ref = reference_scores()
    assert [r.score for r in res] == [ref[k] for k in list(reference_policies())[:3]]


def test_concurrent_first_submits_share_one_compiler(default_workload):
    """Island threads start their first native batches at the same moment on a
    fresh evaluator (a resumed run evaluates nothing before them): they must
    share one JIT compiler -- a second instance would replace the first and
    unload the modules the first thread's kernels are running (a device fault
    at the first launch of every resumed config-3 run, before the fix)."""
    import threading
    from funsearch_kubernetes_simulator_amd.bench.programs import mutation_children
    from funsearch_kubernetes_simulator_amd.ops import hip_engine as he
    dev = he.DeviceEvaluator(default_workload, n_slots=4)
    batches = [mutation_children(6, seed=40 + k) for k in range(4)]
    barrier = threading.Barrier(4)
    compilers, out, errs = [None] * 4, [None] * 4, []

    def run(k):
        try:
            barrier.wait()
            dev.submit_native(k, batches[k])
            compilers[k] = dev.native_compiler
            out[k] = dev.wait(k)
        except Exception as exc:   # surfaced below
            errs.append(repr(exc))

    threads = [threading.Thread(target=run, args=(k,)) for k in range(4)]
    for t in threads:
        t.start()
    for t in threads:
        t.join()
    assert not errs, errs
    assert all(c is compilers[0] for c in compilers)
    for k in range(4):
        ok = out[k][:, 10] != Exc.UNSUPPORTED
        cpu = ce.simulate_program_batch(default_workload, batches[k])
        assert np.array_equal(out[k][ok], cpu[ok])


@pytest.mark.parametrize("top", [63, 1023, -1])
def test_duo_hbm_heap_tops_agree(dev, default_workload, top):
    """The two-wave kernel with its heap mostly in the HBM slice (LDS top of
    63 / 1,023 slots) and with the heap top sized for 2,048 programs in
    flight: rows bit-identical to the CPU VM."""
    progs = programs()[:24]
    vm = ce.simulate_program_batch(default_workload, progs, threads=16)
    opts = {"native_duo_top": top} if top >= 0 else {"native_inflight": 2048}
    dev.set_options(**opts)
    try:
        nat = dev.evaluate_native(progs)
        info = dev.info()
    finally:
        dev.set_options(native_duo_top=-1, native_inflight=0)
    assert info["native_rows_last"] == 0, info
    if top >= 0:
        assert info["native_duo_top_last"] == top, info
    else:
        # as many programs resident as the registers allow (or all 2,048)
        cap = info["native_duo_reg_cap"]
        assert info["native_duo_per_cu_last"] >= min(cap, 2048 // info["num_cus"]), info
    compared = 0
    for i in range(len(progs)):
        if int(nat[i, 10]) in (Exc.UNSUPPORTED, Exc.BUDGET) or int(vm[i, 10]) in (Exc.UNSUPPORTED, Exc.BUDGET):
            continue
        assert np.array_equal(nat[i], vm[i]), (top, i, nat[i], vm[i])
        compared += 1
    assert compared >= len(progs) - 4


def test_module_retirement_bounds_live_modules(default_workload):
    """Modules whose batches have completed are unloaded once more than
    `max_modules` are live (no device-wide sync); their shapes leave the cache
    and are recompiled when they come back, with identical rows.  Baseline
    modules after the first of each skeleton size load without a probe kernel."""
    from funsearch_kubernetes_simulator_amd.bench.programs import novel_children
    from funsearch_kubernetes_simulator_amd.ops import hip_engine as he
    from funsearch_kubernetes_simulator_amd.ops.jit import NativeCompiler
    d = he.DeviceEvaluator(default_workload)
    d._jit = NativeCompiler(d._eng, d.device, budget=int(d.options["budget"]), tier="baseline")
    nc = d.native_compiler
    nc.max_modules = 3
    progs = novel_children(32, seed=77)
    batches = [progs[4 * k:4 * (k + 1)] for k in range(8)]
    first = None
    for k, b in enumerate(batches):
        tab = d.evaluate_native(b)
        if k == 0:
            first = tab
        assert nc.stats["live_modules"] <= 3, nc.stats
    assert nc.stats["retired_modules"] >= 5 and nc.stats["evicted_shapes"] >= 20, nc.stats
    assert nc.stats["probed_loads"] == 1, nc.stats          # later loads: no probe kernel, no copy
    again = d.evaluate_native(batches[0])                    # evicted shapes: recompiled
    assert np.array_equal(again, first)
    cpu = ce.simulate_program_batch(default_workload, batches[0], threads=16)
    ok = (first[:, 10] != Exc.UNSUPPORTED) & (cpu[:, 10] != Exc.UNSUPPORTED)
    assert np.array_equal(first[ok], cpu[ok])
