"""`FunSearchScheduler`: a policy program as a ``(pod, node) -> int`` scorer.

Reference semantics (`funsearch/funsearch_integration.py:67-101`): the program
is ``exec``-ed once in the restricted namespace; each call returns
``int(max(0, score))`` and *re-raises* any exception, which aborts the whole
replay (the reference's "fallback" path is dead code).
"""

from __future__ import annotations

from ..core.model import Node, Pod
from ..policy.sandbox import SafeExecutor, compile_priority_function


class FunSearchScheduler:
    def __init__(self, evolved_code: str, safe_executor: "SafeExecutor | None" = None):
        self.evolved_code = evolved_code
        self.safe_executor = safe_executor or SafeExecutor()
        self.fallback_print = True
        try:
            self._compiled_function = compile_priority_function(evolved_code, self.safe_executor)
        except Exception as exc:
            raise ValueError(f"Failed to compile evolved policy: {exc}")

    def __call__(self, pod: Pod, node: Node) -> int:
        try:
            return int(max(0, self._compiled_function(pod, node)))
        except Exception as exc:
            print(f"Evolved policy failed: {exc}")
            raise

    def _fallback_score(self, pod: Pod, node: Node) -> int:
        """Feasibility-only score (dead code in the reference, kept callable)."""
        if (pod.cpu_milli > node.cpu_milli_left or pod.memory_mib > node.memory_mib_left
                or pod.num_gpu > node.gpu_left):
            return 0
        if pod.num_gpu > 0 and sum(g.gpu_milli_left >= pod.gpu_milli for g in node.gpus) < pod.num_gpu:
            return 0
        return 1000 - node.cpu_milli_left
