"""Asynchronous ring migration between ranks, with a consistent early stop.

The reference has one population and no ranks.  Here every
rank holds ``islands.per_rank`` islands and, every ``migrate_every``
generations, each island's best programs move to the next island of a global
ring.  A blocking all-gather at that point would put every rank in lockstep
with the slowest one (its slowest replay plus its JIT), so a migration is
*posted* instead:

* `post` starts an async all-gather (RCCL on its own stream / gloo thread) of
  this rank's payload -- a 16-byte header ``[best score, stop vote]`` followed
  by the migrant blob (`dist.pack_migrants`: compressed, length-prefixed,
  template bodies only, drops logged) -- and returns at once;
* `poll` finishes gathers that have completed, in posting order, and blocks
  only when a rank is ``lookahead`` migrations ahead of its slowest peer;
  every finished gather yields the incoming migrants per local island and
  the global best (so no per-generation all-reduce is needed);
* **stop**: a rank that wants to stop (threshold reached, wall time up) sets
  its vote in its next payload.  Every rank sees the same gathered votes, so
  all decide to stop at the same migration ``m``; each then posts the gathers
  its peers may already have started (through ``m + lookahead * every``) and
  the ranks leave with equal collective sequences.

* **stop delay**: a stop takes effect ``lookahead * every`` generations after
  the migration whose gather first carries a vote (or a best over the
  threshold), so a run may continue up to ``(lookahead + 1) * every``
  generations past the generation that reached the threshold.
* **no migrations, several ranks** (``migrate_every = 0``): the channel still
  runs, as a *stop-only* channel -- every generation an async all-gather of
  the 16-byte header plus an empty blob -- so ranks never stop on their own
  local best (a rank leaving early would sit in the final champion gather
  while its peers run on, and time out as a "lost" peer).

`wait_s` accumulates the wall time a rank spent blocked in collectives (the
"collective wait" of the multi-rank logs); `max_stall_s` is the longest single
block and `max_gather_s` the longest post-to-completion time of a gather.
"""

from __future__ import annotations

import time
from collections import deque
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Tuple

import numpy as np

from ..parallel import dist

HEADER_BYTES = 16


@dataclass
class MigrationResult:
    generation: int
    bests: List[float]
    votes: int
    incoming: Dict[int, List[Tuple[str, float]]] = field(default_factory=dict)   # local island -> migrants


class MigrationChannel:
    def __init__(self, fs, every: int, start: int, lookahead: int = 2):
        self.fs = fs
        self.every = int(every)
        #: False: a stop-only channel (several ranks, no migrations configured)
        self.migrate = self.every > 0
        if not self.every and fs.ctx.distributed:
            self.every = 1
        self.next = start + self.every if self.every else None
        self.lookahead = max(1, int(lookahead))
        self.pending: deque = deque()
        self.stop_at: Optional[int] = None
        self.best_global = float(fs.best[1])
        self.wait_s = 0.0
        self.max_stall_s = 0.0          # longest single time blocked in a post or a wait
        self.max_gather_s = 0.0         # longest post -> completion of a gather
        self.last_gather_s = 0.0
        self.completed = 0

    # ---------------------------------------------------------------------------------------
    @property
    def active(self) -> bool:
        """Collectives to agree on (several ranks and migrations on)."""
        return self.every > 0 and self.fs.ctx.distributed

    @property
    def stopping(self) -> bool:
        return self.stop_at is not None

    def payload(self, vote: bool) -> np.ndarray:
        hdr = np.array([self.fs.best[1], 1.0 if vote else 0.0], dtype=np.float64)
        blob = self.fs.migrant_blob() if self.migrate else np.zeros(8, dtype=np.uint8)   # length 0: no migrants
        return np.concatenate([hdr.view(np.uint8), blob])

    def post(self, generation: int, vote: bool) -> None:
        t = time.perf_counter()
        try:
            self.pending.append((generation, dist.all_gather_array_async(self.payload(vote)), t))
        except Exception as exc:      # a dead peer: carry on alone (islands.elastic)
            self.fs.rank_lost("migrate", exc)
            self.pending.clear()
        dt = time.perf_counter() - t
        self.wait_s += dt
        self.max_stall_s = max(self.max_stall_s, dt)

    def post_due(self, g_min: int, vote: bool) -> int:
        """Post every migration whose generation the slowest local island has
        reached (or, once stopping, every one through ``stop_at``)."""
        n = 0
        while self.next is not None:
            if self.stop_at is not None:
                if self.next > self.stop_at:
                    break
            elif g_min < self.next or len(self.pending) > self.lookahead:
                # never more than lookahead + 1 gathers in flight: a peer that
                # decides to stop at the oldest one posts exactly that many more
                break
            self.post(self.next, vote)
            self.next += self.every
            n += 1
        return n

    def poll(self, threshold: float, block: bool = False) -> List[MigrationResult]:
        out = []
        while self.pending:
            g, h, t_post = self.pending[0]
            must = block or self.stop_at is not None or len(self.pending) > self.lookahead
            if not must and not h.done():
                break
            t = time.perf_counter()
            try:
                glob = h.wait()
            except Exception as exc:
                self.wait_s += time.perf_counter() - t
                self.pending.clear()
                self.fs.rank_lost("migrate", exc)
                break
            t_done = time.perf_counter()
            self.wait_s += t_done - t
            self.max_stall_s = max(self.max_stall_s, t_done - t)
            self.last_gather_s = t_done - t_post
            self.max_gather_s = max(self.max_gather_s, self.last_gather_s)
            self.pending.popleft()
            hdr = [np.frombuffer(glob[r, :HEADER_BYTES].tobytes(), np.float64) for r in range(glob.shape[0])]
            bests = [float(x[0]) for x in hdr]
            votes = int(sum(x[1] > 0 for x in hdr))
            self.best_global = max([self.best_global] + bests)
            res = MigrationResult(g, bests, votes, self.fs.incoming_migrants(glob[:, HEADER_BYTES:]))
            self.completed += 1
            # decided from this gather alone: every rank sees the same bytes
            if self.stop_at is None and (votes or max(bests) >= threshold):
                self.stop_at = g + self.lookahead * self.every
            out.append(res)
        return out

    def drained(self) -> bool:
        """Nothing in flight and, when stopping, every agreed gather posted."""
        return not self.pending and (self.stop_at is None or self.next is None or self.next > self.stop_at)


__all__ = ["MigrationChannel", "MigrationResult", "HEADER_BYTES"]
