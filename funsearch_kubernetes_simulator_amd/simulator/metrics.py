"""Fitness evaluation: utilisation snapshots, GPU fragmentation, policy score.

Reference contract (`simulator/evaluator.py:27-164`, SURVEY §2.4 rules 6-8):

* snapshots live in *event-count* space: after every processed event
  ``progress = processed / total_events`` (``total_events`` = the initial
  heap size = #pods) and a snapshot is taken when ``progress >= threshold``,
  after which ``threshold += interval`` in IEEE double (one snapshot per
  event at most);
* a snapshot holds four used/total ratios: CPU, memory, GPU count
  (``len(node.gpus) - gpu_left``) and GPU milli;
* fragmentation is sampled only when a placement fails:
  ``min(gpu_milli)`` over waiting GPU pods, then the free milli of every GPU
  with ``0 < left < min`` over the cluster's total GPU milli (0.0 when the
  waiting set holds no GPU pod);
* means are ``statistics.mean`` (exact rational mean, correctly rounded) and
  ``score = clamp01(mean of the 4 utilisations - min(0.1, mean frag))``,
  forced to 0 when any pod never got a node.

The native engines compute the same means with an exact fixed-point
accumulator (`csrc/include/fks/exact_mean.hpp`); `exact_mean` here is the
pure-Python twin used by tests.
"""

from __future__ import annotations

import statistics
from dataclasses import dataclass
from fractions import Fraction
from typing import Iterable, List, Optional, Sequence

from ..core.model import Cluster, Pod


@dataclass
class UtilizationSnapshot:
    cpu_utilization: float
    memory_utilization: float
    gpu_count_utilization: float
    gpu_memory_utilization: float
    event_progress: float


@dataclass
class EvaluationResults:
    avg_cpu_utilization: float
    avg_memory_utilization: float
    avg_gpu_count_utilization: float
    avg_gpu_memory_utilization: float
    gpu_fragmentation_score: float
    num_snapshots: int
    num_fragmentation_events: int

    def as_dict(self) -> dict:
        return dict(self.__dict__)


def exact_mean(values: Iterable[float]) -> float:
    """Correctly rounded mean of doubles (same value as ``statistics.mean``)."""
    vals = list(values)
    if not vals:
        raise statistics.StatisticsError("mean requires at least one data point")
    return float(sum(map(Fraction, vals)) / len(vals))


def combine_policy_score(results: Optional[EvaluationResults], all_placed: bool) -> float:
    """The scalar fitness (`evaluator.py:101-127`)."""
    if not results:
        return 0.0
    if not all_placed:
        return 0
    overall = (results.avg_cpu_utilization + results.avg_memory_utilization
               + results.avg_gpu_count_utilization + results.avg_gpu_memory_utilization) / 4.0
    penalty = min(0.1, results.gpu_fragmentation_score)
    return max(0.0, min(1.0, overall - penalty))


def _ratio(num: int, den: int) -> float:
    return num / den if den > 0 else 0.0


class SchedulingEvaluator:
    """Collects snapshots / fragmentation samples while a replay runs."""

    def __init__(self, cluster: Cluster, enabled: bool = True, snapshot_interval: float = 0.05):
        self.enabled = enabled
        self.snapshot_interval = snapshot_interval
        nodes = list(cluster.nodes_dict.values())
        self.total_cpu = sum(n.cpu_milli_total for n in nodes)
        self.total_memory = sum(n.memory_mib_total for n in nodes)
        self.total_gpu_count = sum(len(n.gpus) for n in nodes)
        self.total_gpu_memory = sum(g.gpu_milli_total for n in nodes for g in n.gpus)
        self.utilization_snapshots: List[UtilizationSnapshot] = []
        self.fragmentation_events: List[float] = []
        self.total_events = 0
        self.events_processed = 0
        self.next_snapshot_threshold = snapshot_interval

    def initialize(self, total_events: int) -> None:
        if not self.enabled:
            return
        self.total_events = total_events
        self.events_processed = 0
        self.next_snapshot_threshold = self.snapshot_interval

    # -- hooks called by the simulator ---------------------------------------
    def record_event_processed(self, cluster: Cluster) -> None:
        if not self.enabled:
            return
        self.events_processed += 1
        progress = self.events_processed / self.total_events if self.total_events > 0 else 0
        if progress >= self.next_snapshot_threshold:
            self.utilization_snapshots.append(self._snapshot(cluster, progress))
            self.next_snapshot_threshold += self.snapshot_interval

    def record_fragmentation_event(self, cluster: Cluster, waiting_pods: Sequence[Pod]) -> None:
        if not self.enabled or not waiting_pods:
            return
        self.fragmentation_events.append(self._fragmentation(cluster, waiting_pods))

    # -- results ----------------------------------------------------------------
    def get_evaluation_results(self) -> Optional[EvaluationResults]:
        if not self.enabled or not self.utilization_snapshots:
            return None
        snaps = self.utilization_snapshots
        frag = statistics.mean(self.fragmentation_events) if self.fragmentation_events else 0.0
        return EvaluationResults(
            avg_cpu_utilization=statistics.mean(s.cpu_utilization for s in snaps),
            avg_memory_utilization=statistics.mean(s.memory_utilization for s in snaps),
            avg_gpu_count_utilization=statistics.mean(s.gpu_count_utilization for s in snaps),
            avg_gpu_memory_utilization=statistics.mean(s.gpu_memory_utilization for s in snaps),
            gpu_fragmentation_score=frag,
            num_snapshots=len(snaps),
            num_fragmentation_events=len(self.fragmentation_events),
        )

    def get_policy_score(self, pods: Sequence[Pod]) -> float:
        res = self.get_evaluation_results()
        if not res:
            return 0.0
        return combine_policy_score(res, all(p.assigned_node != "" for p in pods))

    # -- internals ---------------------------------------------------------------
    def _snapshot(self, cluster: Cluster, progress: float) -> UtilizationSnapshot:
        cpu = mem = cnt = milli = 0
        for n in cluster.nodes_dict.values():
            cpu += n.cpu_milli_total - n.cpu_milli_left
            mem += n.memory_mib_total - n.memory_mib_left
            cnt += len(n.gpus) - n.gpu_left
            for g in n.gpus:
                milli += g.gpu_milli_total - g.gpu_milli_left
        return UtilizationSnapshot(_ratio(cpu, self.total_cpu), _ratio(mem, self.total_memory),
                                   _ratio(cnt, self.total_gpu_count),
                                   _ratio(milli, self.total_gpu_memory), progress)

    def _fragmentation(self, cluster: Cluster, waiting_pods: Sequence[Pod]) -> float:
        needs = [p.gpu_milli for p in waiting_pods if p.num_gpu > 0]
        if not needs:
            return 0.0
        floor_need = min(needs)
        stranded = sum(g.gpu_milli_left for n in cluster.nodes_dict.values() for g in n.gpus
                       if 0 < g.gpu_milli_left < floor_need)
        return _ratio(stranded, self.total_gpu_memory)

    # naming parity with the reference's private helpers
    _take_utilization_snapshot = _snapshot
    _calculate_gpu_fragmentation = _fragmentation
