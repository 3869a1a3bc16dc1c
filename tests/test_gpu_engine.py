"""MI355X replay kernels vs the native CPU oracle (bit-exact)."""
import numpy as np
import pytest

from funsearch_kubernetes_simulator_amd.models import families as fam
from funsearch_kubernetes_simulator_amd.models.library import reference_policies, reference_scores
from funsearch_kubernetes_simulator_amd.ops import cpu_engine as ce
from funsearch_kubernetes_simulator_amd.policy.compiler import compile_policy

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev(default_workload):
    from funsearch_kubernetes_simulator_amd.ops import hip_engine as he
    if not he.device_available():
        pytest.fail("GPU test collected but no HIP device is visible")
    return he.DeviceEvaluator(default_workload)


def test_builtin_ff_bf_exact(dev):
    tab = dev.evaluate_builtin(["first_fit", "best_fit"] * 8)
    scores = reference_scores()
    assert np.all(tab[0::2, 0] == scores["first_fit"])
    assert np.all(tab[1::2, 0] == scores["best_fit"])
    assert list(tab[0, 6:9]) == [47, 3152, 19456]
    assert list(tab[1, 6:9]) == [40, 79, 16383]


def test_random_linear_matches_cpu(dev, default_workload):
    rng = np.random.default_rng(7)
    P = 256
    w = np.stack([rng.uniform(1000, 5000, P), rng.uniform(1e-4, 1e-2, P),
                  rng.uniform(1e-5, 1e-3, P), rng.uniform(10, 1000, P)], axis=1)
    gpu = dev.evaluate_builtin("random_linear", w)
    cpu = ce.simulate_builtin_batch(default_workload, "random_linear", w)
    assert np.array_equal(gpu, cpu)


def test_feature_linear_matches_cpu(dev, default_workload):
    rng = np.random.default_rng(11)
    P = 128
    w = rng.normal(0, 1000, size=(P, 12))
    gpu = dev.evaluate_builtin("feature_linear", w)
    cpu = ce.simulate_builtin_batch(default_workload, "feature_linear", w)
    assert np.array_equal(gpu, cpu)


def test_composite_linear_matches_cpu(dev, default_workload):
    w = fam.sample_composite_linear(128, np.random.default_rng(12))
    gpu = dev.evaluate_builtin("composite_linear", w)
    cpu = ce.simulate_builtin_batch(default_workload, "composite_linear", w)
    assert np.array_equal(gpu, cpu)


def test_vm_reference_programs_exact(dev, default_workload):
    names = list(reference_policies())
    progs = [compile_policy(reference_policies()[n]) for n in names]
    tab = dev.evaluate_programs(progs)
    for i, n in enumerate(names):
        assert tab[i, 0] == reference_scores()[n], n
        cpu = ce.simulate_program(default_workload, progs[i])
        assert tab[i, 12] == float(cpu["trace_hash"] >> 11), n


def test_async_slots_match_sync(dev, default_workload):
    """Batches in flight on separate streams give the same tables as round trips."""
    rng = np.random.default_rng(5)
    a = fam.sample_composite_linear(96, rng)
    b = fam.sample_random_linear(80, rng)
    dev.submit_builtin(1, "composite_linear", a)
    dev.submit_builtin(2, "random_linear", b)
    tb = dev.wait(2)
    ta = dev.wait(1)
    assert np.array_equal(ta, dev.evaluate_builtin("composite_linear", a))
    assert np.array_equal(tb, dev.evaluate_builtin("random_linear", b))
    assert dev.ready(1) and dev.ready(2)


@pytest.mark.parametrize("top", [0, 3, 7, 63, 127, 511, 1023, 2047])
def test_hbm_heap_with_lds_top_matches_cpu(default_workload, top):
    """Heap slots split between LDS (top levels) and HBM give the CPU oracle's tables."""
    from funsearch_kubernetes_simulator_amd.ops import hip_engine as he
    dev = he.DeviceEvaluator(default_workload, options={"heap_mode": "hbm", "heap_top": top, "row_kernel": "off"})
    assert not dev._eng.would_use_rows(64)
    w = fam.sample_composite_linear(64, np.random.default_rng(top))
    assert np.array_equal(dev.evaluate_builtin("composite_linear", w),
                          ce.simulate_builtin_batch(default_workload, "composite_linear", w))


@pytest.mark.parametrize("mode", ["lds", "hbm"])
def test_device_invariant_checker(default_workload, mode):
    """k_check_invariants: resource accounting holds on device replays and does not perturb them."""
    from funsearch_kubernetes_simulator_amd.ops import hip_engine as he
    w = fam.sample_composite_linear(32, np.random.default_rng(3))
    plain = he.DeviceEvaluator(default_workload, options={"heap_mode": mode}).evaluate_builtin("composite_linear", w)
    dev = he.DeviceEvaluator(default_workload, options={"heap_mode": mode, "check_invariants": 61})
    checked = dev.evaluate_builtin("composite_linear", w)
    assert np.all(checked[:, 10] == 0)
    assert np.array_equal(checked, plain)


def test_scaled_synthetic_256_nodes_matches_cpu():
    """Config-5 shape (256 nodes -> 4 node slots per lane, HBM heap): device == CPU oracle."""
    from funsearch_kubernetes_simulator_amd.core import synthetic_workload
    from funsearch_kubernetes_simulator_amd.ops import hip_engine as he
    w = synthetic_workload(n_nodes=256, n_pods=24000, seed=5)
    dev = he.DeviceEvaluator(w)
    assert dev.info()["npass"] == 4
    for family in ("first_fit", "best_fit", "random_linear", "composite_linear"):
        W = fam.SAMPLERS[family](48, np.random.default_rng(1)) if family in fam.SAMPLERS else None
        gpu = dev.evaluate_builtin(family, W, n=48)
        cpu = ce.simulate_builtin_batch(w, family, fam.pad_weights(W) if W is not None else np.zeros((48, 16)))
        assert np.array_equal(gpu, cpu), family


def test_config5_full_shape_matches_cpu():
    """BASELINE config 5 at its full shape (65,536 pods / 256 nodes: NPASS = 4,
    HBM heaps of 64k entries): device == CPU oracle for built-in, linear-family
    and natively compiled reference programs."""
    from funsearch_kubernetes_simulator_amd.core import synthetic_workload
    from funsearch_kubernetes_simulator_amd.ops import hip_engine as he
    w = synthetic_workload(n_nodes=256, n_pods=65536, seed=0)
    dev = he.DeviceEvaluator(w)
    assert dev.info()["npass"] == 4
    for family in ("first_fit", "best_fit", "composite_linear"):
        W = fam.SAMPLERS[family](8, np.random.default_rng(11)) if family in fam.SAMPLERS else None
        gpu = dev.evaluate_builtin(family, W, n=8)
        cpu = ce.simulate_builtin_batch(w, family, fam.pad_weights(W) if W is not None else np.zeros((8, 16)))
        assert np.array_equal(gpu, cpu), family
        assert np.all(gpu[:, 8] > 65536)   # every pod replayed (creations + deletions + retries)
    from funsearch_kubernetes_simulator_amd.models.library import reference_policies
    from funsearch_kubernetes_simulator_amd.policy.compiler import compile_policy
    progs = [compile_policy(c) for c in reference_policies().values()]
    assert np.array_equal(dev.evaluate_native(progs), ce.simulate_program_batch(w, progs))


@pytest.mark.parametrize("repush", ["first", "earliest"])
def test_wave_duo_256_nodes_matches_one_wave(repush):
    """256-node clusters on the two-wave kernel (heap wave + scoring wave,
    replay_wave_duo.hip.h) give the one-wave kernel's rows bit for bit, trace
    hash included (the same events in the same order), for every family and
    a mixed batch, under either repush rule."""
    from funsearch_kubernetes_simulator_amd.core import synthetic_workload
    from funsearch_kubernetes_simulator_amd.ops import hip_engine as he
    w = synthetic_workload(n_nodes=256, n_pods=24000, seed=7)
    opts = {"trace_hash": True, "repush": repush}
    one = he.DeviceEvaluator(w, options={**opts, "wave_duo": False})
    duo = he.DeviceEvaluator(w, options={**opts, "wave_duo": True})
    assert duo.info()["wave_duo"] and not one.info()["wave_duo"]
    for family in ("first_fit", "best_fit", "random_linear", "feature_linear", "composite_linear"):
        W = fam.SAMPLERS[family](40, np.random.default_rng(3)) if family in fam.SAMPLERS else None
        a = one.evaluate_builtin(family, W, n=40)
        b = duo.evaluate_builtin(family, W, n=40)
        assert np.array_equal(a, b), family
        assert np.all(b[:, 10] == 0) and np.all(b[:, 8] > 24000), family
    names = ["first_fit", "best_fit"] * 10
    assert np.array_equal(one.evaluate_builtin(names), duo.evaluate_builtin(names))
    if repush == "first":
        W = fam.SAMPLERS["composite_linear"](16, np.random.default_rng(9))
        assert np.array_equal(duo.evaluate_builtin("composite_linear", W, n=16),
                              ce.simulate_builtin_batch(w, "composite_linear", fam.pad_weights(W)))


# ---- row kernel: 4 policies per wave (clusters of <= 16 nodes) --------------------------

def test_row_kernel_is_default_for_16_nodes(dev):
    assert dev.info()["row_kernel_ok"] and dev._eng.would_use_rows(4096)


@pytest.mark.parametrize("top", [1, 63, 511, 4095])
def test_row_kernel_matches_cpu(default_workload, top):
    """Row kernel with heaps split between LDS and HBM at every depth == CPU oracle;
    P = 37 leaves a partly empty last wave."""
    from funsearch_kubernetes_simulator_amd.ops import hip_engine as he
    dev = he.DeviceEvaluator(default_workload, options={"row_kernel": "on", "row_heap_top": top})
    assert dev._eng.would_use_rows(37)
    w = fam.sample_composite_linear(37, np.random.default_rng(100 + top))
    assert np.array_equal(dev.evaluate_builtin("composite_linear", w),
                          ce.simulate_builtin_batch(default_workload, "composite_linear", w))


@pytest.mark.parametrize("waves,flat", [(4, True), (5, True), (4, False)])
def test_row_composite_reciprocal_path_matches_cpu(default_workload, waves, flat):
    """The composite row instances (host-verified reciprocal divisions, no zero-weight tests,
    one member per threshold pair, double-valued argmax; 4 / 5 waves per SIMD; flat or
    exec-masked LDS/HBM heap accesses) == CPU oracle, including zero weights and a
    huge-weight row that overflows."""
    from funsearch_kubernetes_simulator_amd.ops import hip_engine as he
    dev = he.DeviceEvaluator(default_workload, options={"row_kernel": "on", "row_composite_waves": waves,
                                                        "row_flat": flat})
    info = dev.info()
    assert info["fast_div"] == 1 and info["cap_recips"] and info["frag_recip"]
    assert info["row_composite_waves"] == waves and info["row_flat"] == flat
    w = fam.sample_composite_linear(70, np.random.default_rng(31 + waves))
    w[1, ::2] = 0.0
    w[2, :] = -0.0
    w[3, 13] = 1e308
    gpu = dev.evaluate_builtin("composite_linear", w)
    assert np.array_equal(gpu, ce.simulate_builtin_batch(default_workload, "composite_linear", w))


def test_row_composite_nonfinite_weights_take_mixed_instance(default_workload):
    """inf * 0.0 is NaN: a composite batch with a non-finite weight runs the generic instance
    (engine_host stage_builtin) and still equals the CPU oracle."""
    from funsearch_kubernetes_simulator_amd.ops import hip_engine as he
    dev = he.DeviceEvaluator(default_workload, options={"row_kernel": "on"})
    w = fam.sample_composite_linear(8, np.random.default_rng(5))
    w[0, 2] = np.inf
    w[1, 9] = np.nan
    w[2, 15] = -np.inf
    gpu = dev.evaluate_builtin("composite_linear", w)
    assert np.array_equal(gpu, ce.simulate_builtin_batch(default_workload, "composite_linear", w))
    assert (gpu[:3, 10] != 0).all()


def test_row_kernel_mixed_families_and_exceptions(default_workload):
    """Mixed-family batch (one kernel, divergent scorers per row) incl. rows that raise."""
    from funsearch_kubernetes_simulator_amd.ops import hip_engine as he
    rng = np.random.default_rng(9)
    names = ["first_fit", "best_fit", "random_linear", "feature_linear", "composite_linear"] * 6
    W = np.zeros((len(names), 16))
    for i, n in enumerate(names):
        if n in fam.SAMPLERS:
            W[i] = fam.pad_weights(fam.SAMPLERS[n](1, rng))[0]
    W[3, :12] = 1e308          # feature_linear overflow -> OverflowError (score 0, exception column)
    rows = he.DeviceEvaluator(default_workload, options={"row_kernel": "on"}).evaluate_builtin(names, W)
    wave = he.DeviceEvaluator(default_workload, options={"row_kernel": "off"}).evaluate_builtin(names, W)
    assert np.array_equal(rows, wave)
    assert rows[3, 10] != 0
    for n in set(names):
        idx = [i for i, m in enumerate(names) if m == n]
        assert np.array_equal(rows[idx], ce.simulate_builtin_batch(default_workload, n, W[idx])), n


def test_row_kernel_deep_heap_synthetic():
    """16 nodes, 40,000 pods: 16-level heaps (4 pop rounds) in the row kernel == CPU oracle."""
    from funsearch_kubernetes_simulator_amd.core import synthetic_workload
    from funsearch_kubernetes_simulator_amd.ops import hip_engine as he
    w = synthetic_workload(n_nodes=16, n_pods=40000, seed=3)
    w.pods.pod_ctime[:] = w.pods.pod_ctime * 5   # 5x the pods over 5x the time: the 16 nodes keep up
    dev = he.DeviceEvaluator(w, options={"row_kernel": "on"})
    for family in ("best_fit", "random_linear"):
        W = fam.SAMPLERS[family](12, np.random.default_rng(2)) if family in fam.SAMPLERS else None
        gpu = dev.evaluate_builtin(family, W, n=12)
        cpu = ce.simulate_builtin_batch(w, family, fam.pad_weights(W) if W is not None else np.zeros((12, 16)))
        assert np.array_equal(gpu, cpu), family
