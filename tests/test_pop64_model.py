"""Host model of the two-wave kernel's 64-lane pop (csrc/hip/replay_duo.hip.h
`pop_reinsert64`): each round lane j < 63 is node j (BFS order) of the 6-level
subtree under the path end; the path is found from ballots of per-lane
"go right" / "has children" bits and ancestor masks, entries above `last` move
up, `last` lands on the first path entry greater than it.  The model runs the
same lane-parallel logic with Python lists and must leave the heap array
exactly as CPython's heapq.heappop does (the kernel itself is checked end to
end on the device: test_gpu_native.py)."""
import heapq
import random


def _masks():
    anc, dirm = [0] * 64, [0] * 64
    for j in range(64):
        x = j
        while 0 < x < 63:
            a = (x - 1) >> 1
            anc[j] |= 1 << a
            if x % 2 == 0:
                dirm[j] |= 1 << a
            x = a
    return anc, dirm


ANC, DIR = _masks()


def _depth(j):
    return (j + 1).bit_length() - 1


def pop_reinsert64(h, n, last):
    """h: heap array whose root was popped and whose last entry (`last`) was
    removed (len(h) == n); re-inserts `last` like heapq._siftup."""
    pos, target = 0, -1
    for _ in range(4):
        if 2 * pos + 1 >= n:
            break
        valid, go_r, vals, qs = [False] * 64, [False] * 64, [None] * 64, [0] * 64
        for j in range(64):
            k = _depth(j)
            q = ((pos + 1) << k) - 1 + (j - ((1 << k) - 1))
            c = 2 * q + 1
            qs[j] = q
            valid[j] = j < 63 and c < n
            if valid[j]:
                vl = h[c]
                vr = h[c + 1] if c + 1 < n else None
                go_r[j] = c + 1 < n and not (vl < vr)
                vals[j] = vr if go_r[j] else vl
        m = sum(1 << j for j in range(64) if go_r[j])
        ex = sum(1 << j for j in range(64) if valid[j])
        on = [valid[j] and (ex & ANC[j]) == ANC[j] and ((m ^ DIR[j]) & ANC[j]) == 0 for j in range(64)]
        onm = sum(1 << j for j in range(64) if on[j])
        jd = onm.bit_length() - 1
        kd = _depth(jd)
        qd = ((pos + 1) << kd) - 1 + (jd - ((1 << kd) - 1))
        nxt = 2 * qd + 1 + ((m >> jd) & 1)
        g = [j for j in range(64) if on[j] and last < vals[j]]
        jl = g[0] if g else 64
        for j in range(64):
            if on[j] and j < jl:
                h[qs[j]] = vals[j]
        if g:
            kk = _depth(jl)
            target = ((pos + 1) << kk) - 1 + (jl - ((1 << kk) - 1))
            break
        pos = nxt
        if kd + 1 < 6:
            break
    if target < 0:
        target = pos
    h[target] = last


def test_pop64_matches_heapq():
    rng = random.Random(5)
    for trial in range(60):
        size = rng.choice([2, 3, 7, 63, 64, 65, 200, 1000, 5000])
        keys = rng.sample(range(10 * size + 10), size)   # unique keys, like the kernels' (time, rank) keys
        ref = list(keys)
        heapq.heapify(ref)
        mine = list(ref)
        for _ in range(min(size, 150)):
            heapq.heappop(ref)
            last = mine.pop()
            n = len(mine)
            if n > 0:
                pop_reinsert64(mine, n, last)
            assert mine == ref, trial
            if rng.random() < 0.5:   # interleave pushes like the replay does
                item = rng.randrange(10 * size + 10, 20 * size + 20) * 2 + 1
                heapq.heappush(ref, item)
                heapq.heappush(mine, item)
