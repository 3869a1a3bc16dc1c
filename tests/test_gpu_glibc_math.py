"""The device build of glibc_math.h on the MI355X equals the host build (and
so CPython) bit for bit, and a pow / exp / log-heavy policy program replayed
natively on the device equals the CPU VM, which calls the host libm."""
import numpy as np
import pytest

from funsearch_kubernetes_simulator_amd.ops import cpu_engine as ce
from funsearch_kubernetes_simulator_amd.policy.compiler import compile_policy

pytestmark = pytest.mark.gpu


def test_device_equals_host_build():
    from funsearch_kubernetes_simulator_amd.ops import hip_engine as he
    if not he.device_available():
        pytest.fail("GPU test collected but no HIP device is visible")
    m = he.native()
    rng = np.random.default_rng(3)
    n = 1 << 20
    xs = np.concatenate([rng.uniform(-745, 709.7, n // 2), rng.uniform(-2, 2, n // 2)])
    lx = np.concatenate([rng.uniform(0, 100, n // 2), 1 + rng.uniform(-0.07, 0.07, n // 2)])
    px = np.concatenate([rng.uniform(1e-3, 3, n // 2), rng.uniform(1, 1e4, n // 2)])
    py = np.concatenate([rng.uniform(-30, 30, n // 2), rng.uniform(-300, 300, n // 2)])
    for fn, x, y, host in ((0, xs, xs, lambda: m.gm_exp_batch(xs)), (1, lx, lx, lambda: m.gm_log_batch(lx)),
                           (2, px, py, lambda: m.gm_pow_batch(px, py))):
        dst, dout = m.gm_device_batch(fn, x, y, 0)
        hst, hout = host()
        assert np.array_equal(dst, hst), fn
        assert np.array_equal(dout.view(np.uint64), hout.view(np.uint64)), fn


def test_pow_heavy_program_native_equals_cpu_vm(default_workload):
    from funsearch_kubernetes_simulator_amd.ops import hip_engine as he
    dev = he.DeviceEvaluator(default_workload)
    from funsearch_kubernetes_simulator_amd.policy.template import PolicyTemplate
    body = PolicyTemplate.fill_template(
        "c = (node.cpu_milli_left / max(1, node.cpu_milli_total)) ** 1.37\n"
        "    m = math.exp(-node.memory_mib_left / max(1.0, node.memory_mib_total * 1.9))\n"
        "    g = math.log(1.0 + node.gpu_left + pod.cpu_milli / 997.0) ** 0.71\n"
        "    score = 1000 * (c + m) * g * 7.3 + math.pow(2.0, g) * 3.1")
    progs = [compile_policy(body.replace("1.37", str(1.37 + 0.013 * k))) for k in range(16)]
    nat = dev.evaluate_native(progs)
    vm = ce.simulate_program_batch(default_workload, progs, threads=16)
    assert (nat[:, 10] == 0).all(), nat[:, 10]          # nothing deferred: no EXC_UNSUPPORTED rows
    assert np.array_equal(nat, vm)
