"""Compat path for `benchmarks/parser.py` (reference); see core.traces.

``python -m funsearch_kubernetes_simulator_amd.benchmarks.parser`` prints the
same overview as the reference's demo ``main``.
"""
from ..core.traces import TraceParser  # noqa: F401


def main() -> None:
    parser = TraceParser()
    print("Available node files:", parser.get_available_node_files())
    print("Available pod files:", parser.get_available_pod_files())
    cluster, pods = parser.parse_workload()
    print(f"\nParsed cluster with {len(cluster.nodes_dict)} nodes")
    print(f"Parsed {len(pods)} pods")
    if cluster.nodes_dict:
        n = next(iter(cluster.nodes_dict.values()))
        print(f"\nSample node: {n.node_id}\n  CPU: {n.cpu_milli_total} milli\n"
              f"  Memory: {n.memory_mib_total} MiB\n  GPUs: {n.gpu_left}")
        if n.gpus:
            print(f"  GPU Memory: {n.gpus[0].memory_mib_total} MiB each")
    if pods:
        p = pods[0]
        print(f"\nSample pod: {p.pod_id}\n  CPU: {p.cpu_milli} milli\n  Memory: {p.memory_mib} MiB\n"
              f"  GPUs: {p.num_gpu}\n  Creation time: {p.creation_time}")


if __name__ == "__main__":
    main()
