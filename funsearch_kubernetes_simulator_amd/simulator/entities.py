"""Compat path for `simulator/entities.py` (reference); see core.model."""
from ..core.model import GPU, Cluster, Node, Pod  # noqa: F401

__all__ = ["GPU", "Node", "Cluster", "Pod"]
