"""Compat path for `funsearch/safe_execution.py` (reference)."""
from ..policy.sandbox import SafeExecutor  # noqa: F401
from ..policy.template import PolicyTemplate  # noqa: F401
from .generator import LLMCodeGenerator  # noqa: F401

__all__ = ["SafeExecutor", "PolicyTemplate", "LLMCodeGenerator"]
