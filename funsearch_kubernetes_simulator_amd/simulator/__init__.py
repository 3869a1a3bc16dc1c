"""L1/L2 object-level simulator: event queue, cluster placement, evaluator."""
from .cluster_sim import KubernetesSimulator, print_cluster_state
from .events import DiscreteEventSimulator, Event, EventType
from .metrics import EvaluationResults, SchedulingEvaluator, UtilizationSnapshot

__all__ = ["KubernetesSimulator", "print_cluster_state", "DiscreteEventSimulator", "Event",
           "EventType", "SchedulingEvaluator", "EvaluationResults", "UtilizationSnapshot"]
