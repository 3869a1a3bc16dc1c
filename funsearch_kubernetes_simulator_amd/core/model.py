"""Mutable cluster / workload objects used by the Python-facing API.

These are the object-graph views of the cluster and the pod trace.  Field
names and constructor order are the compatibility contract with the
reference's `simulator/entities.py:4-43` (GPU, Node, Cluster, Pod), because
user policies are written against exactly these attribute names
(`pod.cpu_milli`, `node.gpus[i].gpu_milli_left`, ...).

The hot simulation paths never touch these objects: the native CPU engine and
the HIP replay kernel work on flat structure-of-arrays buffers produced by
:mod:`funsearch_kubernetes_simulator_amd.core.arrays`.  Converting between the
two views is explicit (`ClusterArrays.from_objects` / `to_objects`).
"""

from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, Iterator, List


@dataclass
class GPU:
    """One accelerator inside a node.

    ``gpu_milli_*`` is the compute share (1000 = a whole GPU) that the
    placement logic debits; ``memory_mib_*`` is carried for policies but is
    never debited (reference behaviour).
    """

    memory_mib_left: int
    memory_mib_total: int
    gpu_milli_left: int
    gpu_milli_total: int

    @property
    def gpu_milli_used(self) -> int:
        return self.gpu_milli_total - self.gpu_milli_left


@dataclass
class Node:
    """A machine.  ``gpu_left`` counts whole unassigned GPUs (debited by
    ``pod.num_gpu`` on placement), independently of the per-GPU milli shares."""

    node_id: str
    cpu_milli_left: int
    cpu_milli_total: int
    memory_mib_left: int
    memory_mib_total: int
    gpu_left: int
    gpus: List[GPU]

    def is_active(self) -> bool:
        """True when anything is allocated on the node (used for ``max_nodes``)."""
        return (self.cpu_milli_left < self.cpu_milli_total
                or self.memory_mib_left < self.memory_mib_total
                or self.gpu_left < len(self.gpus))


@dataclass
class Cluster:
    """Ordered collection of nodes.  Iteration order (dict insertion order,
    i.e. the CSV row order) is the order in which a scheduler sees nodes and
    therefore the tie-break order of the placement argmax."""

    nodes_dict: Dict[str, Node]

    def __iter__(self) -> Iterator[Node]:
        return iter(self.nodes_dict.values())

    def __len__(self) -> int:
        return len(self.nodes_dict)

    @property
    def num_gpus(self) -> int:
        return sum(len(n.gpus) for n in self.nodes_dict.values())


@dataclass
class Pod:
    """One workload request from the trace.

    ``creation_time`` is mutated by the simulator when a placement fails and
    the pod is re-queued; ``assigned_node`` / ``assigned_gpus`` record the
    placement (``""`` / ``[]`` while unplaced).
    """

    pod_id: str
    cpu_milli: int
    memory_mib: int
    num_gpu: int
    gpu_milli: int
    gpu_spec: str
    creation_time: int
    duration_time: int
    assigned_node: str = ""
    assigned_gpus: List[int] = field(default_factory=list)

    @property
    def deletion_time(self) -> int:
        return self.creation_time + self.duration_time

    @property
    def is_placed(self) -> bool:
        return self.assigned_node != ""
