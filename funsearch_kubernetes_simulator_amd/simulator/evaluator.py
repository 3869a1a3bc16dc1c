"""Compat path for `simulator/evaluator.py` (reference); see .metrics."""
from .metrics import EvaluationResults, SchedulingEvaluator, UtilizationSnapshot  # noqa: F401

__all__ = ["SchedulingEvaluator", "EvaluationResults", "UtilizationSnapshot"]
