"""Event queue of the object-level (reference-compatible) simulator.

Semantics follow `simulator/event_simulator.py:1-58` of the reference, which
the exact engines (native CPU, HIP) reproduce bit-for-bit:

* heap items are ``(time, Event)`` tuples driven by CPython ``heapq``; ties on
  time fall through to ``Event.__lt__``, which compares ``pod_id`` strings;
* the heap starts as every pod's CREATION in trace order, then ``heapify``;
* a DELETION is pushed at ``creation_time + duration_time``;
* a failed placement re-queues the pod one tick after the **first DELETION in
  heap-array order** (not the earliest one) and mutates
  ``pod.creation_time``; with no DELETION pending the pod is dropped.

The quirky repush rule changes the policy ranking (SURVEY §2.4 rule 5), so it
is the default.  ``repush="earliest"`` selects the earliest pending deletion
instead (opt-in variant, not reference behaviour).
"""

from __future__ import annotations

import heapq
from dataclasses import dataclass
from enum import Enum
from typing import List, Tuple

from ..core.model import Pod


class EventType(str, Enum):
    """``StrEnum``-compatible event kind (values match ``enum.auto()`` on a
    StrEnum: the lower-cased member name)."""

    CREATION = "creation"
    DELETION = "deletion"

    def __str__(self) -> str:  # StrEnum prints the value
        return self.value


@dataclass
class Event:
    event_type: EventType
    pod: Pod

    def __lt__(self, other: "Event") -> bool:
        return self.pod.pod_id < other.pod.pod_id


HeapItem = Tuple[int, Event]


class DiscreteEventSimulator:
    """Min-heap of pending pod events."""

    def __init__(self, pod_list: List[Pod], repush: str = "first"):
        if repush not in ("first", "earliest"):
            raise ValueError("repush must be 'first' (reference) or 'earliest'")
        self.repush_mode = repush
        self.event_heap: List[HeapItem] = [(p.creation_time, Event(EventType.CREATION, p))
                                           for p in pod_list]
        heapq.heapify(self.event_heap)

    # -- queue primitives ------------------------------------------------------
    def pop_event(self) -> HeapItem:
        return heapq.heappop(self.event_heap)

    def peak_event(self) -> HeapItem:
        return self.event_heap[0]

    def finished_events(self) -> bool:
        return not self.event_heap

    def __len__(self) -> int:
        return len(self.event_heap)

    # -- scheduling hooks ------------------------------------------------------
    def push_deletion_event(self, pod: Pod) -> None:
        heapq.heappush(self.event_heap,
                       (pod.creation_time + pod.duration_time, Event(EventType.DELETION, pod)))

    def _retry_anchor(self):
        """Time of the deletion the retry is anchored to, or ``None``."""
        if self.repush_mode == "first":
            return next((t for t, ev in self.event_heap if ev.event_type == EventType.DELETION), None)
        times = [t for t, ev in self.event_heap if ev.event_type == EventType.DELETION]
        return min(times) if times else None

    def repush_creation_event(self, pod: Pod) -> bool:
        """Re-queue ``pod`` one tick after a pending deletion.

        Returns False when nothing is pending (the pod is then dropped, as in
        the reference, which leaves it unassigned forever)."""
        anchor = self._retry_anchor()
        if anchor is None:
            return False
        pod.creation_time = anchor + 1
        heapq.heappush(self.event_heap, (pod.creation_time, Event(EventType.CREATION, pod)))
        return True
