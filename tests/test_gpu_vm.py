"""Device bytecode VM vs CPU VM: full replays of many programs on sub-traces."""
import numpy as np
import pytest

from funsearch_kubernetes_simulator_amd.core.arrays import Workload
from funsearch_kubernetes_simulator_amd.models import families as fam
from funsearch_kubernetes_simulator_amd.models.library import reference_policies, seed_policies
from funsearch_kubernetes_simulator_amd.ops import cpu_engine as ce
from funsearch_kubernetes_simulator_amd.policy.bytecode import Exc
from funsearch_kubernetes_simulator_amd.policy.compiler import CompileError, compile_policy

from program_corpus import programs as corpus_programs

pytestmark = pytest.mark.gpu


def _programs():
    return corpus_programs()


@pytest.mark.parametrize("mode", ["lds", "hbm"])
def test_device_vm_equals_cpu_vm(default_workload, mode):
    from funsearch_kubernetes_simulator_amd.ops import hip_engine as he
    if not he.device_available():
        pytest.fail("GPU test collected but no HIP device is visible")
    w = default_workload
    sub = Workload(w.cluster, w.pods.subset(np.arange(1000, 1600)))
    dev = he.DeviceEvaluator(sub, options={"heap_mode": mode})
    progs = _programs()
    gpu = dev.evaluate_programs(progs)
    cpu = ce.simulate_program_batch(sub, progs, threads=8)
    deferred = []
    for i, p in enumerate(progs):
        if int(gpu[i, 10]) == Exc.UNSUPPORTED:
            deferred.append(i)   # deferred to the host by design (trig, near-tie math, bigint)
            continue
        assert np.array_equal(gpu[i], cpu[i]), (i, p.source[-300:], gpu[i], cpu[i])
    # the deferred programs are named in the failure message (the engine re-runs them on the CPU VM)
    assert len(deferred) <= 6, [(i, progs[i].source[-200:]) for i in deferred]


def test_device_vm_runaway_program_drains(default_workload):
    """A non-terminating candidate must not hang the GPU: the per-call budget ends its wave."""
    from funsearch_kubernetes_simulator_amd.ops import hip_engine as he
    w = default_workload
    sub = Workload(w.cluster, w.pods.subset(np.arange(0, 64)))
    dev = he.DeviceEvaluator(sub, options={"budget": 100000})
    prog = compile_policy("def priority_function(pod, node):\n    x = 0\n    while True:\n        x += 1\n"
                          "    return 1\n")
    tab = dev.evaluate_programs([prog] * 4)
    assert np.all(tab[:, 10] == Exc.BUDGET)


def test_device_vm_wide_register_file(default_workload):
    """Programs with > 32 virtual registers take the VGPR + LDS register-file kernel."""
    from funsearch_kubernetes_simulator_amd.ops import hip_engine as he
    body = "".join(f"    v{i} = node.cpu_milli_left * {i + 1} + pod.cpu_milli\n" for i in range(40))
    total = " + ".join(f"v{i}" for i in range(40))
    code = ("def priority_function(pod, node):\n"
            "    if pod.cpu_milli > node.cpu_milli_left or pod.memory_mib > node.memory_mib_left:\n"
            "        return 0\n"
            "    if pod.num_gpu > 0 and sum(1 for g in node.gpus if g.gpu_milli_left >= pod.gpu_milli) < pod.num_gpu:\n"
            "        return 0\n" + body + f"    return ({total}) % 1000 + 1\n")
    prog = compile_policy(code)
    assert prog.nregs > 32
    w = default_workload
    sub = Workload(w.cluster, w.pods.subset(np.arange(0, 800)))
    dev = he.DeviceEvaluator(sub)
    gpu = dev.evaluate_programs([prog, prog])
    cpu = ce.simulate_program_batch(sub, [prog, prog], threads=2)
    assert np.array_equal(gpu, cpu)
