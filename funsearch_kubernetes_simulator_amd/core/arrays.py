"""Structure-of-arrays views of a cluster and a pod trace.

This is the representation every engine consumes: the native CPU oracle
(``csrc/cpu``), and the HIP replay kernel (``csrc/hip``), which uploads these
arrays to HBM once and keeps them resident across all evaluations.

Layout (all little-endian, C-contiguous numpy arrays):

* nodes, in cluster iteration order (this order is the placement tie-break):
  ``node_cpu_total/left``, ``node_mem_total/left`` (int64),
  ``node_gpu_left`` (int32, the node-level whole-GPU counter),
  ``node_ngpus`` (int32, ``len(node.gpus)``), ``gpu_start`` (int32 prefix,
  length n_nodes + 1);
* GPUs, concatenated per node: ``gpu_milli_total/left`` (int32),
  ``gpu_mem_total/left`` (int64);
* pods, in trace order (this order seeds the event heap):
  ``pod_cpu``, ``pod_mem`` (int64), ``pod_ngpu``, ``pod_gmilli`` (int32),
  ``pod_ctime``, ``pod_dur`` (int64) and ``pod_rank`` (int32) = dense rank of
  ``pod_id`` in string order, which is the event tie-break key of the
  reference (`simulator/event_simulator.py:16-17`).
"""

from __future__ import annotations

from dataclasses import dataclass, field
from typing import List, Sequence

import numpy as np

from .model import GPU, Cluster, Node, Pod


def dense_rank(keys: Sequence[str]) -> np.ndarray:
    """Dense rank of each key under Python ``str`` ordering (equal keys share
    a rank, exactly like the reference's ``Event.__lt__`` tie semantics)."""
    uniq = sorted(set(keys))
    pos = {k: i for i, k in enumerate(uniq)}
    return np.fromiter((pos[k] for k in keys), dtype=np.int32, count=len(keys))


@dataclass
class ClusterArrays:
    node_ids: List[str]
    node_cpu_total: np.ndarray
    node_cpu_left: np.ndarray
    node_mem_total: np.ndarray
    node_mem_left: np.ndarray
    node_gpu_left: np.ndarray
    node_ngpus: np.ndarray
    gpu_start: np.ndarray
    gpu_milli_total: np.ndarray
    gpu_milli_left: np.ndarray
    gpu_mem_total: np.ndarray
    gpu_mem_left: np.ndarray

    @property
    def n_nodes(self) -> int:
        return len(self.node_ids)

    @property
    def n_gpus(self) -> int:
        return int(self.gpu_start[-1])

    @property
    def max_gpus_per_node(self) -> int:
        return int(self.node_ngpus.max()) if self.n_nodes else 0

    @classmethod
    def from_objects(cls, cluster: Cluster) -> "ClusterArrays":
        nodes = list(cluster.nodes_dict.values())
        ngpus = np.array([len(n.gpus) for n in nodes], dtype=np.int32)
        start = np.zeros(len(nodes) + 1, dtype=np.int32)
        np.cumsum(ngpus, out=start[1:])
        gpus = [g for n in nodes for g in n.gpus]

        def i64(xs):
            return np.array(list(xs), dtype=np.int64)

        def i32(xs):
            return np.array(list(xs), dtype=np.int32)

        return cls(
            node_ids=[n.node_id for n in nodes],
            node_cpu_total=i64(n.cpu_milli_total for n in nodes),
            node_cpu_left=i64(n.cpu_milli_left for n in nodes),
            node_mem_total=i64(n.memory_mib_total for n in nodes),
            node_mem_left=i64(n.memory_mib_left for n in nodes),
            node_gpu_left=i32(n.gpu_left for n in nodes),
            node_ngpus=ngpus,
            gpu_start=start,
            gpu_milli_total=i32(g.gpu_milli_total for g in gpus),
            gpu_milli_left=i32(g.gpu_milli_left for g in gpus),
            gpu_mem_total=i64(g.memory_mib_total for g in gpus),
            gpu_mem_left=i64(g.memory_mib_left for g in gpus),
        )

    def to_objects(self) -> Cluster:
        nodes = {}
        for i, nid in enumerate(self.node_ids):
            a, b = int(self.gpu_start[i]), int(self.gpu_start[i + 1])
            gpus = [GPU(int(self.gpu_mem_left[j]), int(self.gpu_mem_total[j]),
                        int(self.gpu_milli_left[j]), int(self.gpu_milli_total[j]))
                    for j in range(a, b)]
            nodes[nid] = Node(nid, int(self.node_cpu_left[i]), int(self.node_cpu_total[i]),
                              int(self.node_mem_left[i]), int(self.node_mem_total[i]),
                              int(self.node_gpu_left[i]), gpus)
        return Cluster(nodes)


@dataclass
class PodArrays:
    pod_ids: List[str]
    pod_cpu: np.ndarray
    pod_mem: np.ndarray
    pod_ngpu: np.ndarray
    pod_gmilli: np.ndarray
    pod_ctime: np.ndarray
    pod_dur: np.ndarray
    pod_rank: np.ndarray
    gpu_spec: List[str] = field(default_factory=list)

    @property
    def n_pods(self) -> int:
        return len(self.pod_ids)

    @classmethod
    def from_objects(cls, pods: Sequence[Pod]) -> "PodArrays":
        ids = [p.pod_id for p in pods]
        return cls(
            pod_ids=ids,
            pod_cpu=np.array([p.cpu_milli for p in pods], dtype=np.int64),
            pod_mem=np.array([p.memory_mib for p in pods], dtype=np.int64),
            pod_ngpu=np.array([p.num_gpu for p in pods], dtype=np.int32),
            pod_gmilli=np.array([p.gpu_milli for p in pods], dtype=np.int32),
            pod_ctime=np.array([p.creation_time for p in pods], dtype=np.int64),
            pod_dur=np.array([p.duration_time for p in pods], dtype=np.int64),
            pod_rank=dense_rank(ids),
            gpu_spec=[p.gpu_spec for p in pods],
        )

    def to_objects(self) -> List[Pod]:
        specs = self.gpu_spec or [""] * self.n_pods
        return [Pod(self.pod_ids[i], int(self.pod_cpu[i]), int(self.pod_mem[i]),
                    int(self.pod_ngpu[i]), int(self.pod_gmilli[i]), specs[i],
                    int(self.pod_ctime[i]), int(self.pod_dur[i]), "", [])
                for i in range(self.n_pods)]

    def subset(self, idx: np.ndarray) -> "PodArrays":
        """A sub-trace (pods re-ranked among themselves)."""
        idx = np.asarray(idx)
        ids = [self.pod_ids[i] for i in idx]
        specs = [self.gpu_spec[i] for i in idx] if self.gpu_spec else []
        return PodArrays(ids, self.pod_cpu[idx].copy(), self.pod_mem[idx].copy(),
                         self.pod_ngpu[idx].copy(), self.pod_gmilli[idx].copy(),
                         self.pod_ctime[idx].copy(), self.pod_dur[idx].copy(),
                         dense_rank(ids), specs)


@dataclass
class Workload:
    """A (cluster, trace) pair in SoA form -- the unit the engines replay."""

    cluster: ClusterArrays
    pods: PodArrays
    name: str = "workload"

    @classmethod
    def from_objects(cls, cluster: Cluster, pods: Sequence[Pod], name: str = "workload") -> "Workload":
        return cls(ClusterArrays.from_objects(cluster), PodArrays.from_objects(pods), name)

    def to_objects(self):
        return self.cluster.to_objects(), self.pods.to_objects()

    def fingerprint(self) -> str:
        """Content hash used to key device-resident uploads and caches."""
        import hashlib
        h = hashlib.sha1()
        c, p = self.cluster, self.pods
        for a in (c.node_cpu_total, c.node_cpu_left, c.node_mem_total, c.node_mem_left,
                  c.node_gpu_left, c.node_ngpus, c.gpu_milli_total, c.gpu_milli_left,
                  p.pod_cpu, p.pod_mem, p.pod_ngpu, p.pod_gmilli, p.pod_ctime, p.pod_dur,
                  p.pod_rank):
            h.update(np.ascontiguousarray(a).tobytes())
        return h.hexdigest()
