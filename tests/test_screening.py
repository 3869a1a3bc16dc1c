"""MFMA surrogate screening: numpy reference semantics (CPU) and the k_screen_linear kernel (GPU)."""
import numpy as np
import pytest

from funsearch_kubernetes_simulator_amd.ops import screening as scr


def _integer_problem(S=37, Np=64, N=50, P=70, seed=0):
    rng = np.random.default_rng(seed)
    X = rng.integers(-4, 5, size=(S, Np, scr.KP)).astype(np.float32)
    X[:, :, 16] = 0.0
    X[:, N:, 16] = scr.INFEASIBLE          # padding rows
    X[:, :, 17] = 0.0
    W = rng.integers(-3, 4, size=(P, 16)).astype(np.float64)
    R = rng.integers(0, 9, size=(S, Np)).astype(np.float32)
    Rfail = rng.integers(-5, 0, size=S).astype(np.float32)
    return X.reshape(S * Np, scr.KP), scr.weights_matrix(W), R.reshape(-1), Rfail, Np, W


def test_screen_numpy_matches_bruteforce():
    X, Wt, R, Rfail, Np, W = _integer_problem()
    S = X.shape[0] // Np
    fit = scr.screen_numpy(X, Wt, R, Rfail, Np, chunk=5)
    for p in range(W.shape[0]):
        tot = 0.0
        for s in range(S):
            y = X[s * Np:(s + 1) * Np] @ Wt[:, p]
            best, bv = 0, -np.inf
            for n in range(Np):          # strict '>' scan: the first node wins ties
                if y[n] > bv:
                    best, bv = n, y[n]
            tot += R[s * Np + best] if bv > 0 else Rfail[s]
        assert fit[p] == pytest.approx(tot)


def test_screener_builds_on_default_trace(default_workload):
    sc = scr.Screener(default_workload, device="cpu")
    assert sc.X.shape == (sc.states.n_states * 32, scr.KP)
    from funsearch_kubernetes_simulator_amd.models import families as fam
    f = sc.score(fam.sample_composite_linear(8, np.random.default_rng(0)))
    assert f.shape == (8,) and np.all(np.isfinite(f))


@pytest.mark.gpu
def test_mfma_output_layout():
    from funsearch_kubernetes_simulator_amd.ops import hip_engine as he
    if not he.device_available():
        pytest.fail("GPU test collected but no HIP device is visible")
    out = he.native().mfma_probe(0)
    A = np.array([[i + 100 * k for k in range(2)] for i in range(32)], dtype=np.float64)
    B = np.array([[j + 1000 * k for j in range(32)] for k in range(2)], dtype=np.float64)
    D = A @ B
    for lane in range(64):
        col, half = lane % 32, lane // 32
        for r in range(16):
            row = 8 * (r // 4) + 4 * half + r % 4
            assert out[lane, r] == D[row, col], (lane, r)


@pytest.mark.gpu
def test_k_screen_linear_exact_on_integer_data():
    from funsearch_kubernetes_simulator_amd.ops import hip_engine as he
    X, Wt, R, Rfail, Np, W = _integer_problem(S=301, Np=64, N=50, P=200, seed=3)
    dev = he.native().screen_linear(X, Wt, R, Rfail, Np, 0)
    ref = scr.screen_numpy(X, Wt, R, Rfail, Np)
    assert np.array_equal(dev[:W.shape[0]], ref[:W.shape[0]])


@pytest.mark.gpu
def test_screener_device_matches_numpy(default_workload):
    from funsearch_kubernetes_simulator_amd.models import families as fam
    sc = scr.Screener(default_workload, device="auto")
    assert sc.device is not None
    W = fam.sample_composite_linear(96, np.random.default_rng(1))
    dev = sc.score(W)
    ref = scr.screen_numpy(sc.X, scr.weights_matrix(W), sc.R, sc.Rfail, sc.Np)[:96]
    # fp32 accumulation order differs (MFMA vs BLAS): near-ties may flip a few decisions
    assert np.allclose(dev, ref, rtol=2e-3, atol=2.0)
