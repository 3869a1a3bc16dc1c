"""Program JIT tiers on the MI355X: the baseline generator (csrc/jit, direct
gfx950 machine code), the LLVM tier and the background tier-up between them,
each bit-identical to the CPU VM on full replays of the 8,152-pod trace."""
import numpy as np
import pytest

from funsearch_kubernetes_simulator_amd.ops import cpu_engine as ce
from funsearch_kubernetes_simulator_amd.policy.bytecode import Exc

from program_corpus import programs

pytestmark = pytest.mark.gpu
DEFER = (int(Exc.UNSUPPORTED), int(Exc.BUDGET))


def _dev(workload, tier):
    from funsearch_kubernetes_simulator_amd.ops import hip_engine as he
    from funsearch_kubernetes_simulator_amd.ops.jit import NativeCompiler
    if not he.device_available():
        pytest.fail("GPU test collected but no HIP device is visible")
    dev = he.DeviceEvaluator(workload)
    dev._jit = NativeCompiler(dev._eng, dev.device, budget=int(dev.options["budget"]), tier=tier)
    return dev


def _assert_equal_rows(nat, vm, progs):
    compared = 0
    for i in range(len(progs)):
        if int(nat[i, 10]) in DEFER or int(vm[i, 10]) in DEFER:
            continue
        assert np.array_equal(nat[i], vm[i]), (i, progs[i].source[-300:], nat[i], vm[i])
        compared += 1
    return compared


@pytest.mark.parametrize("tier", ["baseline", "llvm"])
def test_jit_tier_equals_cpu_vm(default_workload, tier):
    from funsearch_kubernetes_simulator_amd.bench.programs import mutation_children
    progs = programs()[:16] + mutation_children(48, seed=23)
    dev = _dev(default_workload, tier)
    nat = dev.evaluate_native(progs)
    st = dev.native_compiler.stats
    assert st[f"{tier}_shapes"] > 0 and st["rejected"] == 0, st
    vm = ce.simulate_program_batch(default_workload, progs, threads=16)
    assert _assert_equal_rows(nat, vm, progs) >= len(progs) - 2


def test_tierup_swaps_in_llvm_code(default_workload):
    """auto tier: hot baseline shapes are recompiled by LLVM in the background
    and swapped in; rows stay bit-identical and the pointer changes."""
    from funsearch_kubernetes_simulator_amd.bench.programs import novel_children
    progs = novel_children(8, seed=31)      # distinct shapes: one pointer per tier-up
    dev = _dev(default_workload, "auto")
    nc = dev.native_compiler
    nc.tierup_after = 2
    a = dev.evaluate_native(progs)
    fn_a = nc.prepare(progs).fn.copy()      # second use: tier-up queued
    nc.drain_tierup()
    assert nc.stats["tierup_done"] == nc.stats["tierup_queued"] > 0, nc.stats
    fn_b = nc.prepare(progs).fn
    assert (fn_a != fn_b).sum() == nc.stats["tierup_done"]
    b = dev.evaluate_native(progs)
    assert np.array_equal(a, b)


def test_novel_batch_measurement_is_exact(default_workload):
    """bench.py's `program_path.novel`: distinct shapes, JIT included, rows
    bit-identical to the CPU VM on the same batch."""
    from funsearch_kubernetes_simulator_amd.bench.programs import measure_novel
    dev = _dev(default_workload, "auto")
    rec = measure_novel(dev, default_workload, n=64, compile_batches=1, seed=5, cpu_threads=16)
    assert rec["new_shapes"] == 64 and rec["native"] == 64 and rec["bit_identical"], rec
    assert rec["compared"] >= 60 and rec["compile_s_per_64_median"] < 1.0


@pytest.mark.parametrize("cap", [2, 3])
def test_spilled_registers_equal_cpu_vm(default_workload, cap):
    """Baseline code with virtual registers in per-lane scratch slots (the pool
    capped at `cap` pairs forces the spill path on ordinary programs): full
    device replays bit-identical to the CPU VM, runtime calls included (their
    save area sits above the slots on the kernel's stack)."""
    from funsearch_kubernetes_simulator_amd.bench.programs import mutation_children
    from funsearch_kubernetes_simulator_amd.ops import gcnjit
    m = ce.native()
    progs = programs()[:24] + mutation_children(24, seed=29)
    m.gcn_set_pair_cap(cap)
    try:
        codes = [(p, gcnjit.compile_program(p)[0]) for p in progs]
        spilled = [p for p, c in codes if c is not None and c.info["spills"] > 0]
        assert len(spilled) >= 8, len(spilled)
        dev = _dev(default_workload, "baseline")
        assert dev.info()["stack_bytes"] >= 2048
        nat = dev.evaluate_native(spilled)
    finally:
        m.gcn_set_pair_cap(0)
    vm = ce.simulate_program_batch(default_workload, spilled, threads=16)
    assert _assert_equal_rows(nat, vm, spilled) >= len(spilled) - 2
