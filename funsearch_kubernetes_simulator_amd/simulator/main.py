"""Compat path for `simulator/main.py` (reference); see .cluster_sim."""
from .cluster_sim import KubernetesSimulator, PodNodeScorer, print_cluster_state  # noqa: F401

__all__ = ["KubernetesSimulator", "PodNodeScorer", "print_cluster_state"]
