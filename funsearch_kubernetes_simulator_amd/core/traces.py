"""OpenB trace ingestion: CSV / k8s-YAML readers and a synthetic generator.

`TraceParser` keeps the reference's public surface
(`benchmarks/parser.py:9-122`: ``parse_nodes``, ``parse_cluster``,
``parse_pods``, ``parse_workload``, ``get_available_{node,pod}_files`` and the
same default file names) and its observable quirks:

* every GPU gets ``gpu_milli = 1000`` and ``memory_mib`` from
  ``gpu_mem_mapping.json``; a model missing from the mapping yields
  ``gpus == []`` while ``gpu_left`` still equals the CSV count
  (`parser.py:39,56`);
* ``duration = deletion_time - creation_time``; an empty ``gpu_milli`` is 0;
* the ``multigpu*`` CSVs lack the time columns and raise ``KeyError`` like the
  reference does.

Beyond the reference it offers `load_workload` (straight to SoA arrays, no
object graph), a reader for the bundled-but-unused Kubernetes Node YAML, and
`synthetic_workload` for the scaled 65,536-pod / 256-node configuration.
"""

from __future__ import annotations

import csv
import json
import re
from pathlib import Path
from typing import Dict, List, Optional, Tuple

import numpy as np

from .._paths import DEFAULT_NODE_FILE, DEFAULT_POD_FILE, resolve_traces_dir
from .arrays import ClusterArrays, PodArrays, Workload, dense_rank
from .model import GPU, Cluster, Node, Pod

GPU_MILLI_PER_CARD = 1000


def _read_rows(path: Path) -> List[Dict[str, str]]:
    with open(path, newline="") as fh:
        return list(csv.DictReader(fh))


class TraceParser:
    """Reads OpenB node / pod CSVs into entity objects."""

    def __init__(self, traces_dir: "str | None" = "benchmarks/traces"):
        self.traces_dir = resolve_traces_dir(traces_dir)
        self.csv_dir = self.traces_dir / "csv"
        self.gpu_mem_mapping = self._load_gpu_memory_mapping()

    def _load_gpu_memory_mapping(self) -> Dict[str, int]:
        with open(self.traces_dir / "gpu_mem_mapping.json") as fh:
            return {str(k): int(v) for k, v in json.load(fh).items()}

    # -- nodes ---------------------------------------------------------------
    def _node_from_row(self, row: Dict[str, str]) -> Node:
        count = int(row["gpu"])
        model = row["model"]
        gpus: List[GPU] = []
        if count > 0 and model in self.gpu_mem_mapping:
            mem = self.gpu_mem_mapping[model]
            gpus = [GPU(mem, mem, GPU_MILLI_PER_CARD, GPU_MILLI_PER_CARD) for _ in range(count)]
        cpu, mem_mib = int(row["cpu_milli"]), int(row["memory_mib"])
        return Node(row["sn"], cpu, cpu, mem_mib, mem_mib, count, gpus)

    def parse_nodes(self, node_file: str = "openb_node_list_all_node.csv") -> Dict[str, Node]:
        nodes: Dict[str, Node] = {}
        for row in _read_rows(self.csv_dir / node_file):
            node = self._node_from_row(row)
            nodes[node.node_id] = node      # dict semantics: a repeated sn keeps its first slot
        return nodes

    def parse_cluster(self, node_file: str = "openb_node_list_gpu_node.csv") -> Cluster:
        return Cluster(nodes_dict=self.parse_nodes(node_file))

    # -- pods ----------------------------------------------------------------
    @staticmethod
    def _pod_from_row(row: Dict[str, str]) -> Pod:
        gm = row["gpu_milli"]
        spec = row["gpu_spec"]          # KeyError on multigpu*.csv, as in the reference
        created = int(row["creation_time"])
        return Pod(pod_id=row["name"], cpu_milli=int(row["cpu_milli"]),
                   memory_mib=int(row["memory_mib"]), num_gpu=int(row["num_gpu"]),
                   gpu_milli=int(gm) if gm else 0, gpu_spec=spec or "",
                   creation_time=created, duration_time=int(row["deletion_time"]) - created,
                   assigned_node="", assigned_gpus=[])

    def parse_pods(self, pod_file: str = "openb_pod_list_default.csv") -> List[Pod]:
        return [self._pod_from_row(r) for r in _read_rows(self.csv_dir / pod_file)]

    # -- listing / convenience -----------------------------------------------
    def get_available_node_files(self) -> List[str]:
        return sorted(p.name for p in self.csv_dir.glob("openb_node_list_*.csv"))

    def get_available_pod_files(self) -> List[str]:
        return sorted(p.name for p in self.csv_dir.glob("openb_pod_list_*.csv"))

    def parse_workload(self, node_file: str = DEFAULT_NODE_FILE,
                       pod_file: str = DEFAULT_POD_FILE) -> Tuple[Cluster, List[Pod]]:
        return self.parse_cluster(node_file), self.parse_pods(pod_file)

    def load_workload(self, node_file: str = DEFAULT_NODE_FILE,
                      pod_file: str = DEFAULT_POD_FILE, native: Optional[bool] = None) -> Workload:
        """Parse straight into SoA arrays (what the engines consume).

        ``native`` (default: when the C++ extension is built) reads the CSVs with
        the C++ loader (csrc/cpu/trace_io.hpp) without building the object
        graph; the result is identical to the object path."""
        name = f"{Path(node_file).stem}/{Path(pod_file).stem}"
        if native is None or native:
            try:
                from ..ops.cpu_engine import native as _native
                mod = _native()
            except Exception:
                if native:
                    raise
                mod = None
            if mod is not None:
                return self._load_native(mod, node_file, pod_file, name)
        cluster, pods = self.parse_workload(node_file, pod_file)
        return Workload.from_objects(cluster, pods, name=name)

    def _load_native(self, mod, node_file: str, pod_file: str, name: str) -> Workload:
        n = mod.load_node_csv(str(self.csv_dir / node_file), self.gpu_mem_mapping)
        p = mod.load_pod_csv(str(self.csv_dir / pod_file))
        ngpus = np.asarray(n["ngpus"], dtype=np.int32)
        start = np.zeros(ngpus.size + 1, dtype=np.int32)
        np.cumsum(ngpus, out=start[1:])
        G = int(start[-1])
        gmem = np.repeat(np.asarray(n["gpu_mem"], dtype=np.int64), ngpus)
        cpu, mem = np.asarray(n["cpu"], dtype=np.int64), np.asarray(n["mem"], dtype=np.int64)
        cluster = ClusterArrays(
            node_ids=list(n["sn"]), node_cpu_total=cpu, node_cpu_left=cpu.copy(),
            node_mem_total=mem, node_mem_left=mem.copy(),
            node_gpu_left=np.asarray(n["gpu_count"], dtype=np.int32), node_ngpus=ngpus, gpu_start=start,
            gpu_milli_total=np.full(G, GPU_MILLI_PER_CARD, dtype=np.int32),
            gpu_milli_left=np.full(G, GPU_MILLI_PER_CARD, dtype=np.int32),
            gpu_mem_total=gmem, gpu_mem_left=gmem.copy())
        ids = list(p["name"])
        pods = PodArrays(ids, np.asarray(p["cpu"], dtype=np.int64), np.asarray(p["mem"], dtype=np.int64),
                         np.asarray(p["ngpu"], dtype=np.int32), np.asarray(p["gmilli"], dtype=np.int32),
                         np.asarray(p["ctime"], dtype=np.int64), np.asarray(p["dur"], dtype=np.int64),
                         dense_rank(ids), list(p["gpu_spec"]))
        return Workload(cluster, pods, name=name)

    # -- Kubernetes Node YAML (bundled with the reference, unused there) ----
    def parse_node_yaml(self, yaml_file: str = "openb_node_list_gpu_node.yaml") -> Cluster:
        """Build a cluster from ``kind: Node`` documents (capacity section)."""
        import yaml

        path = self.traces_dir / "node_yaml" / yaml_file
        nodes: Dict[str, Node] = {}
        with open(path) as fh:
            for doc in yaml.safe_load_all(fh):
                if not doc or doc.get("kind") != "Node":
                    continue
                meta, cap = doc.get("metadata", {}), doc.get("status", {}).get("capacity", {})
                name = meta.get("name")
                model = (meta.get("labels") or {}).get("alibabacloud.com/gpu-card-model", "")
                row = {"sn": name, "cpu_milli": str(_k8s_cpu_milli(cap.get("cpu", "0"))),
                       "memory_mib": str(_k8s_mem_mib(cap.get("memory", "0"))),
                       "gpu": str(int(cap.get("alibabacloud.com/gpu-count", 0))), "model": model}
                node = self._node_from_row(row)
                nodes[node.node_id] = node
        return Cluster(nodes)


def _k8s_cpu_milli(q: str) -> int:
    q = str(q)
    return int(q[:-1]) if q.endswith("m") else int(float(q) * 1000)


_MEM_UNITS = {"Ki": 1 / 1024, "Mi": 1, "Gi": 1024, "Ti": 1024 * 1024}


def _k8s_mem_mib(q: str) -> int:
    m = re.fullmatch(r"(\d+)([KMGT]i)?", str(q))
    if not m:
        raise ValueError(f"unsupported memory quantity {q!r}")
    return int(int(m.group(1)) * _MEM_UNITS.get(m.group(2) or "Mi", 1))


def load_default_workload(traces_dir: Optional[str] = None) -> Workload:
    """The headline workload: 16-node / 64-GPU cluster x 8,152-pod OpenB trace."""
    return TraceParser(traces_dir).load_workload()


def synthetic_workload(n_nodes: int = 256, n_pods: int = 65536, seed: int = 0,
                       base: Optional[Workload] = None, jitter: int = 3600) -> Workload:
    """Scaled synthetic workload (BASELINE config 5).

    The cluster tiles the base cluster's node rows until ``n_nodes``; the pod
    trace replicates the base trace with +-``jitter`` seconds of creation-time
    noise (durations kept) until ``n_pods``, then sorts by creation time.
    Pod ids are ``syn-pod-%06d`` so string order equals index order.
    """
    base = base or load_default_workload()
    rng = np.random.default_rng(seed)
    bc, bp = base.cluster, base.pods
    sel = np.arange(n_nodes) % bc.n_nodes
    ngpus = bc.node_ngpus[sel]
    start = np.zeros(n_nodes + 1, dtype=np.int32)
    np.cumsum(ngpus, out=start[1:])
    gsel = np.concatenate([np.arange(bc.gpu_start[i], bc.gpu_start[i + 1]) for i in sel]) \
        if start[-1] else np.zeros(0, dtype=np.int64)
    cluster = ClusterArrays(
        node_ids=[f"syn-node-{i:04d}" for i in range(n_nodes)],
        node_cpu_total=bc.node_cpu_total[sel].copy(), node_cpu_left=bc.node_cpu_total[sel].copy(),
        node_mem_total=bc.node_mem_total[sel].copy(), node_mem_left=bc.node_mem_total[sel].copy(),
        node_gpu_left=bc.node_gpu_left[sel].copy(), node_ngpus=ngpus.astype(np.int32), gpu_start=start,
        gpu_milli_total=bc.gpu_milli_total[gsel].copy(), gpu_milli_left=bc.gpu_milli_total[gsel].copy(),
        gpu_mem_total=bc.gpu_mem_total[gsel].copy(), gpu_mem_left=bc.gpu_mem_total[gsel].copy())
    psel = np.arange(n_pods) % bp.n_pods
    ctime = bp.pod_ctime[psel] + rng.integers(-jitter, jitter + 1, size=n_pods)
    ctime = np.maximum(ctime, 0)
    order = np.argsort(ctime, kind="stable")
    psel, ctime = psel[order], ctime[order]
    ids = [f"syn-pod-{i:06d}" for i in range(n_pods)]
    pods = PodArrays(ids, bp.pod_cpu[psel].copy(), bp.pod_mem[psel].copy(), bp.pod_ngpu[psel].copy(),
                     bp.pod_gmilli[psel].copy(), ctime.astype(np.int64), bp.pod_dur[psel].copy(),
                     dense_rank(ids), [""] * n_pods)
    return Workload(cluster, pods, name=f"synthetic-{n_nodes}n-{n_pods}p-s{seed}")
