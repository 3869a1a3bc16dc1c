"""k_score_linear_mfma (csrc/hip/screen_mfma.hip.h) on the MI355X: the MFMA
tile decisions against the f32 / f64 host reference of the same rule, and
the kernel's signature fold against its host twin."""
import numpy as np
import pytest

from funsearch_kubernetes_simulator_amd.models.families import sample_feature_linear
from funsearch_kubernetes_simulator_amd.ops import screen

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def states(default_workload):
    from funsearch_kubernetes_simulator_amd.core.arrays import Workload
    from funsearch_kubernetes_simulator_amd.ops import hip_engine as he
    if not he.device_available():
        pytest.fail("GPU test collected but no HIP device is visible")
    c, p = default_workload.to_objects()
    w = Workload.from_objects(c, p[:3000])
    w0 = sample_feature_linear(1, np.random.default_rng(3))[0]
    return screen.record_states(w, w0, every=4, max_states=256)


def test_mfma_decisions_match_reference(states):
    st = states
    W = sample_feature_linear(1000, np.random.default_rng(7))
    sig, dec, ms = screen.screen(st, W, want_dec=True)
    assert dec.shape == (1000, st.S) and sig.shape == (1000,)
    ref32 = screen.decisions_reference(st, W, dtype=np.float32)
    ref64 = screen.decisions_reference(st, W, dtype=np.float64)
    # f32 accumulation order differs from numpy's only at near-ties
    assert (dec == ref32).mean() > 0.999, (dec == ref32).mean()
    assert (dec == ref64).mean() > 0.995, (dec == ref64).mean()
    assert np.array_equal(sig, screen.signature(dec, screen.chunks_for(1000, st.S)))
    # a signature does not depend on the batch it was computed in
    one, _, _ = screen.screen(st, W[7:8])
    assert one[0] == sig[7]


def test_mfma_exact_on_integer_data(states):
    """Integer features and weights (exact in f32): every decision equals the
    f64 reference, so the fragment maps and the tie rule are right."""
    st = states
    rng = np.random.default_rng(11)
    st2 = screen.States(np.round(st.feats * 8.0), st.feasible, st.chosen)
    W = rng.integers(-20, 21, size=(96, 12)).astype(np.float64)
    W[:, 0] = 500.0
    sig, dec, _ = screen.screen(st2, W, want_dec=True)
    assert np.array_equal(dec, screen.decisions_reference(st2, W))
    dup = np.concatenate([W, W[:5]])
    sig2, _, _ = screen.screen(st2, dup)
    assert np.array_equal(sig2[96:], sig2[:5])
