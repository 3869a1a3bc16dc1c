"""L0: entity model, SoA arrays and trace I/O."""
from .arrays import ClusterArrays, PodArrays, Workload, dense_rank
from .model import GPU, Cluster, Node, Pod
from .traces import TraceParser, load_default_workload, synthetic_workload

__all__ = ["GPU", "Node", "Cluster", "Pod", "ClusterArrays", "PodArrays", "Workload", "dense_rank",
           "TraceParser", "load_default_workload", "synthetic_workload"]
