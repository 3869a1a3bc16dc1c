"""Host model of the wave kernel's placement argmax (csrc/hip/replay.hip.h,
creation branch of replay_one).

The kernel keeps, per lane, the best score over its NPASS node slots (strict
`>`, so the lowest slot wins a tie) plus its first exception, runs ONE wave
max, and takes the lowest slot whose ballot (lane best == max and lane slot ==
that slot) is non-empty.  This must pick exactly the node the pass-by-pass
argmax picks (node = slot * 64 + lane; strict `>` across passes, first lane
within a pass; a score of 0 never places), and report the exception of the
first raising node in node order.
"""

import numpy as np
import pytest

WAVE = 64


def pass_by_pass(scores, exc):
    """The previous formulation: one wave max per slot, stop at the first slot with an exception."""
    best, node = 0, -1
    for ps in range(scores.shape[0]):
        bad = np.nonzero(exc[ps])[0]
        if len(bad):
            return None, int(exc[ps, bad[0]])
        m = int(scores[ps].max())
        if m > best:
            best, node = m, ps * WAVE + int(np.nonzero(scores[ps] == m)[0][0])
    return node, 0


def one_max(scores, exc):
    """The kernel's formulation, lane by lane."""
    npass = scores.shape[0]
    lbest = np.zeros(WAVE, dtype=np.uint64)
    lst = np.zeros(WAVE, dtype=np.int64)          # bits 0-1 slot of lbest, 2-3 slot of first exc, 8+ exc code
    for ps in range(npass):
        s = scores[ps].astype(np.uint64)
        first = (exc[ps] != 0) & ((lst >> 8) == 0)
        lst = np.where(first, lst | (exc[ps].astype(np.int64) << 8) | (ps << 2), lst)
        better = s > lbest
        lbest = np.where(better, s, lbest)
        lst = np.where(better, (lst & ~3) | ps, lst)
    if np.any((lst >> 8) != 0):
        for ps in range(npass):
            b = np.nonzero(((lst >> 8) != 0) & (((lst >> 2) & 3) == ps))[0]
            if len(b):
                return None, int(lst[b[0]] >> 8)
    m = lbest.max()
    node = -1
    if m > 0:
        for ps in range(npass - 1, -1, -1):
            b = np.nonzero((lbest == m) & ((lst & 3) == ps))[0]
            if len(b):
                node = ps * WAVE + int(b[0])
    return node, 0


@pytest.mark.parametrize("npass", [1, 2, 4])
def test_one_max_matches_pass_by_pass(npass):
    rng = np.random.default_rng(npass)
    for trial in range(3000):
        hi = int(rng.choice([2, 5, 1000, 2**62]))
        scores = rng.integers(0, hi, size=(npass, WAVE), dtype=np.int64)
        if trial % 7 == 0:
            scores[:] = 0                                     # nothing fits
        if trial % 5 == 0:                                    # ties across slots and lanes
            scores[rng.integers(0, npass), rng.integers(0, WAVE)] = scores.max()
        exc = np.zeros((npass, WAVE), dtype=np.int64)
        if trial % 11 == 0:
            k = rng.integers(1, 4)
            exc[rng.integers(0, npass, k), rng.integers(0, WAVE, k)] = rng.integers(1, 6, k)
        assert one_max(scores, exc) == pass_by_pass(scores, exc), trial
