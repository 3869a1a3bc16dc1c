"""Behavioural screening of linear-family candidates (ops/screen.py): the
host twins of `k_score_linear_mfma`'s layouts and decision rule.  The GPU
test (tests/test_gpu_screen.py) checks the kernel against these."""
import numpy as np
import pytest

from funsearch_kubernetes_simulator_amd.models.families import N_FEATURES, sample_composite_linear, sample_feature_linear
from funsearch_kubernetes_simulator_amd.ops import screen


@pytest.fixture(scope="module")
def states(default_workload):
    from funsearch_kubernetes_simulator_amd.core.arrays import Workload
    c, p = default_workload.to_objects()
    w = Workload.from_objects(c, p[:1500])          # a sub-trace: quick on the object engine
    w0 = sample_feature_linear(1, np.random.default_rng(3))[0]
    return w0, screen.record_states(w, w0, every=4, max_states=128)


@pytest.fixture(scope="module")
def composite_states(default_workload):
    w0 = sample_composite_linear(1, np.random.default_rng(5))[0]
    return w0, screen.record_states(default_workload, w0, family="composite_linear", every=8, max_states=96)


def test_recorded_decisions_match_the_replay(states):
    """The recording policy's own fp64 decisions on its recorded states are the
    nodes the object engine chose there: features, feasibility and the
    max(1, int(score)) first-maximum rule agree with the replay."""
    w0, st = states
    assert st.S == 128 and st.feats.shape == (128, 16, N_FEATURES)
    dec = screen.decisions_reference(st, w0[None, :])[0]
    chosen = np.where(st.chosen < 0, 255, st.chosen)
    assert np.array_equal(dec, chosen.astype(np.uint8))


def test_composite_recorded_decisions_match_the_replay(composite_states):
    w0, st = composite_states
    assert st.S == 96 and st.feats.shape[2] == 16
    dec = screen.decisions_reference(st, w0[None, :])[0]
    assert np.array_equal(dec, np.where(st.chosen < 0, 255, st.chosen).astype(np.uint8))


def test_layouts_round_trip(states):
    """arrange_states / arrange_weights: the MFMA fragment maps (A lane l =
    row l & 15, k l >> 4; B lane l = k l >> 4, col l & 15) reproduce w . f."""
    _, st = states
    W = sample_feature_linear(37, np.random.default_rng(1))
    X = screen.arrange_states(st)
    Wt, P = screen.arrange_weights(W, N_FEATURES)
    assert X.shape == (st.S, screen.STEPS, 64) and Wt.shape == (3, screen.STEPS, 64) and P == 37
    # emulate the 16x16x4 tiles: D[row][col] = sum_t sum_k A_t[row][k] B_t[k][col]
    lanes = np.arange(64)
    s, tile = 5, 1
    D = np.zeros((16, 16))
    for t in range(screen.STEPS):
        A = np.zeros((16, 4)); B = np.zeros((4, 16))
        A[lanes & 15, lanes >> 4] = X[s, t]
        B[lanes >> 4, lanes & 15] = Wt[tile, t]
        D += A @ B
    want = st.feats[s] @ W[16:32, :N_FEATURES].T + np.where(st.feasible[s], 0.0, screen.MASK)[:, None]
    assert np.allclose(D, want.astype(np.float32), rtol=1e-5, atol=1e-3 * np.abs(want).max())


def test_signatures_and_unique(states):
    _, st = states
    W = sample_feature_linear(8, np.random.default_rng(2))
    W = np.concatenate([W, W[:3]])                  # three exact duplicates
    dec = screen.decisions_reference(st, W)
    sig = screen.signature(dec, screen.chunks_for(len(W), st.S))
    assert len(set(sig.tolist())) <= 8
    keep = screen.unique_by_signature(sig)
    assert list(keep[:len(keep)]) == sorted(keep) and all(k < 8 for k in keep)
    assert len(screen.unique_by_signature(sig, exclude=[sig[0]])) == len(keep) - 1


def test_param_island_screen_keeps_new_behaviours(composite_states):
    """ParamIsland with a screener: a generation draws factor x candidates and
    returns only behaviourally new ones (not an elite's signature, no two
    alike), in the order drawn."""
    from funsearch_kubernetes_simulator_amd.funsearch.param_islands import make_islands
    _, st = composite_states
    isl = make_islands(1, "composite_linear", 64, 8, seed=4)[0]
    w = isl.propose()
    isl.update(w, np.linspace(0.3, 0.5, len(w)))
    isl.screener = lambda W: screen.signature(screen.decisions_reference(st, W))
    isl.screen_factor = 4
    out = isl.propose()
    assert 0 < len(out) <= 64 and isl.screened == 256 and isl.screen_kept == len(out)
    sig = isl.screener(out)
    assert len(set(sig.tolist())) == len(out)
    assert not set(sig.tolist()) & set(isl.screener(isl.elites).tolist())


def test_signature_independent_of_batch(states):
    """A candidate's signature is the same alone or inside a larger batch (the
    island compares its elites' signatures with a batch's)."""
    _, st = states
    W = sample_feature_linear(40, np.random.default_rng(9))
    dec = screen.decisions_reference(st, W)
    full = screen.signature(dec, screen.chunks_for(40, st.S))
    one = screen.signature(dec[3:4], screen.chunks_for(1, st.S))
    assert one[0] == full[3]
