"""Object-level cluster simulator (reference-compatible, pure Python).

This engine is the *semantic ground truth* for arbitrary Python scorers: it
calls ``scheduler(pod, node)`` on live entity objects exactly like the
reference's `simulator/main.py:28-278`, so anything a policy can observe
(node order, in-place mutation, exceptions) behaves identically.  It is also
the fallback the batched engines use for programs the policy compiler cannot
lower.  The fast paths are `ops.cpu_engine` (native oracle) and
`ops.hip_engine` (MI355X replay kernel), which must agree with this class
bit-for-bit.

Placement rules (SURVEY §2.4 rules 3-5):

* creation: score every node in cluster order, keep the strictly greatest
  score above 0 (first node wins ties);
* success: debit cpu / memory / whole-GPU count, pick GPUs best-fit (stable
  ascending ``gpu_milli_left`` among GPUs with enough milli), push the
  deletion;
* failure: add to ``waiting_pods`` (once), sample fragmentation, re-queue.
"""

from __future__ import annotations

from typing import Callable, List, Optional

from ..core.model import GPU, Cluster, Node, Pod
from .events import DiscreteEventSimulator, Event, EventType
from .metrics import SchedulingEvaluator

PodNodeScorer = Callable[[Pod, Node], int]


def print_cluster_state(cluster: Cluster, step: str) -> None:
    print(f"\n--- Cluster State: {step} ---")
    for node_id, node in cluster.nodes_dict.items():
        print(f"{node_id}:")
        print(f"  CPU: {node.cpu_milli_total - node.cpu_milli_left}/{node.cpu_milli_total} milli")
        print(f"  Memory: {node.memory_mib_total - node.memory_mib_left}/{node.memory_mib_total} MiB")
        print(f"  GPUs: {len(node.gpus) - node.gpu_left}/{len(node.gpus)}")
        for i, gpu in enumerate(node.gpus):
            print(f"    GPU{i}: {gpu.gpu_milli_total - gpu.gpu_milli_left}/{gpu.gpu_milli_total} milli")


def pick_gpus_best_fit(node: Node, pod: Pod) -> List[int]:
    """Indices of the ``pod.num_gpu`` tightest-fitting GPUs (stable order)."""
    if pod.num_gpu == 0:
        return []
    fits = [i for i, g in enumerate(node.gpus) if g.gpu_milli_left >= pod.gpu_milli]
    if len(fits) < pod.num_gpu:
        raise ValueError(f"Not enough GPUs available on node {node.node_id}")
    fits.sort(key=lambda i: node.gpus[i].gpu_milli_left)     # list.sort is stable
    return fits[:pod.num_gpu]


def pick_gpus_first_fit(node: Node, pod: Pod) -> List[int]:
    """Indices of the first ``pod.num_gpu`` GPUs with enough milli."""
    if pod.num_gpu == 0:
        return []
    fits = [i for i, g in enumerate(node.gpus) if g.gpu_milli_left >= pod.gpu_milli][:pod.num_gpu]
    if len(fits) < pod.num_gpu:
        raise ValueError(f"Not enough GPUs available on node {node.node_id}")
    return fits


class KubernetesSimulator:
    def __init__(self, cluster: Cluster, pod_list: List[Pod],
                 event_simulator: DiscreteEventSimulator, scheduler: PodNodeScorer,
                 validate_invariants: bool = False,
                 evaluator: Optional[SchedulingEvaluator] = None,
                 gpu_alloc: str = "best_fit", track_max_nodes: bool = True):
        self.cluster = cluster
        self.pod_list = pod_list
        self.event_simulator = event_simulator
        self.scheduler = scheduler
        self.validate_invariants = validate_invariants
        self.evaluator = evaluator
        self.max_nodes = 0
        self.waiting_pods: List[Pod] = []
        self.events_processed = 0
        self.track_max_nodes = track_max_nodes
        if gpu_alloc not in ("best_fit", "first_fit"):
            raise ValueError("gpu_alloc must be 'best_fit' or 'first_fit'")
        self._alloc = pick_gpus_best_fit if gpu_alloc == "best_fit" else pick_gpus_first_fit
        if evaluator:
            evaluator.initialize(len(event_simulator.event_heap))

    # -- main loop -----------------------------------------------------------
    def run_schedule(self) -> None:
        nodes = list(self.cluster.nodes_dict.values())
        queue, ev_hook = self.event_simulator, self.evaluator
        while not queue.finished_events():
            _, event = queue.pop_event()
            if event.event_type == EventType.DELETION:
                self._handle_deletion(event)
            else:
                self._handle_creation(event)
            self.events_processed += 1
            if ev_hook:
                ev_hook.record_event_processed(self.cluster)
            if self.track_max_nodes:
                busy = sum(1 for n in nodes if n.is_active())
                if busy > self.max_nodes:
                    self.max_nodes = busy

    # -- event handlers -------------------------------------------------------
    def _handle_deletion(self, event: Event) -> None:
        pod = event.pod
        if pod.assigned_node == "":
            raise ValueError("Invalid node id, pod was never assigned node yet being deleted")
        node = self.cluster.nodes_dict[pod.assigned_node]
        node.cpu_milli_left += pod.cpu_milli
        node.memory_mib_left += pod.memory_mib
        node.gpu_left += pod.num_gpu
        for gi in pod.assigned_gpus:
            node.gpus[gi].gpu_milli_left += pod.gpu_milli
        if self.validate_invariants:
            self._validate_cluster_invariants()

    def _select_node(self, pod: Pod) -> Optional[Node]:
        best_score, best = 0, None
        for node in self.cluster.nodes_dict.values():
            s = self.scheduler(pod, node)
            if s > best_score:
                best_score, best = s, node
        return best

    def _handle_creation(self, event: Event) -> None:
        pod = event.pod
        node = self._select_node(pod)
        if node is None:
            if pod not in self.waiting_pods:
                self.waiting_pods.append(pod)
            if self.evaluator:
                self.evaluator.record_fragmentation_event(self.cluster, self.waiting_pods)
            self.event_simulator.repush_creation_event(pod)
            return
        node.cpu_milli_left -= pod.cpu_milli
        node.memory_mib_left -= pod.memory_mib
        node.gpu_left -= pod.num_gpu
        picked = self._alloc(node, pod)
        for gi in picked:
            node.gpus[gi].gpu_milli_left -= pod.gpu_milli
        pod.assigned_node = node.node_id
        pod.assigned_gpus = picked
        if pod in self.waiting_pods:
            self.waiting_pods.remove(pod)
        self.event_simulator.push_deletion_event(pod)
        if self.validate_invariants:
            self._validate_cluster_invariants()

    # reference-named helpers (callable directly, e.g. by tests)
    def _allocate_gpus_best_fit(self, node: Node, pod: Pod) -> List[int]:
        picked = pick_gpus_best_fit(node, pod)
        for gi in picked:
            node.gpus[gi].gpu_milli_left -= pod.gpu_milli
        return picked

    def _allocate_gpus_first_fit(self, node: Node, pod: Pod) -> List[int]:
        picked = pick_gpus_first_fit(node, pod)
        for gi in picked:
            node.gpus[gi].gpu_milli_left -= pod.gpu_milli
        return picked

    # -- debugging -------------------------------------------------------------
    def _validate_cluster_invariants(self) -> None:
        """Resource accounting checks (`simulator/main.py:201-272`).

        "In use" means: pods that hold a node and whose pending event is still
        queued (i.e. their deletion has not fired yet)."""
        nodes = self.cluster.nodes_dict
        for nid, n in nodes.items():
            for what, left, total in (("CPU", n.cpu_milli_left, n.cpu_milli_total),
                                      ("memory", n.memory_mib_left, n.memory_mib_total),
                                      ("GPU count", n.gpu_left, len(n.gpus))):
                if left < 0:
                    raise ValueError(f"Node {nid} has negative {what} remaining: {left}")
                if left > total:
                    raise ValueError(f"Node {nid} {what} remaining exceeds total: {left} > {total}")
            for i, g in enumerate(n.gpus):
                if not 0 <= g.gpu_milli_left <= g.gpu_milli_total:
                    raise ValueError(f"Node {nid} GPU {i} milli out of range: {g.gpu_milli_left}")
        for p in self.pod_list:
            if p.assigned_node != "" and p.assigned_node not in nodes:
                raise ValueError(f"Pod {p.pod_id} assigned to non-existent node: {p.assigned_node}")
        live = [ev.pod for _, ev in self.event_simulator.event_heap if ev.pod.assigned_node != ""]
        for nid, n in nodes.items():
            mine = [p for p in live if p.assigned_node == nid]
            used = (sum(p.cpu_milli for p in mine), sum(p.memory_mib for p in mine),
                    sum(p.num_gpu for p in mine))
            if used[0] + n.cpu_milli_left != n.cpu_milli_total:
                raise ValueError(f"Node {nid} CPU accounting error: used({used[0]}) + "
                                 f"remaining({n.cpu_milli_left}) != total({n.cpu_milli_total})")
            if used[1] + n.memory_mib_left != n.memory_mib_total:
                raise ValueError(f"Node {nid} memory accounting error: used({used[1]}) + "
                                 f"remaining({n.memory_mib_left}) != total({n.memory_mib_total})")
            if used[2] + n.gpu_left != len(n.gpus):
                raise ValueError(f"Node {nid} GPU accounting error: used({used[2]}) + "
                                 f"remaining({n.gpu_left}) != total({len(n.gpus)})")
            per_gpu = [0] * len(n.gpus)
            for p in mine:
                for gi in (p.assigned_gpus if p.num_gpu > 0 else ()):
                    per_gpu[gi] += p.gpu_milli
            for i, g in enumerate(n.gpus):
                if per_gpu[i] + g.gpu_milli_left != g.gpu_milli_total:
                    raise ValueError(f"Node {nid} GPU {i} milli accounting error: used({per_gpu[i]}) + "
                                     f"remaining({g.gpu_milli_left}) != total({g.gpu_milli_total})")

    def get_evaluation_results(self):
        return self.evaluator.get_evaluation_results() if self.evaluator else None


GPUType = GPU  # re-export convenience
