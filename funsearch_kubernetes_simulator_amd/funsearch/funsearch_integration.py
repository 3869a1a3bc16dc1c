"""Compat path for `funsearch/funsearch_integration.py` (reference).

``python -m funsearch_kubernetes_simulator_amd.funsearch.funsearch_integration``
runs the reference-shaped loop (`SimpleFunSearch` + `save_top_policies(5)`,
top-5 saved on Ctrl-C).  The multi-island / multi-GPU loop is
`islands.run_funsearch` (CLI: ``python -m funsearch_kubernetes_simulator_amd.funsearch``).
"""

from __future__ import annotations

from typing import Optional, Tuple

from ..engine import Evaluator
from .scheduler import FunSearchScheduler  # noqa: F401
from .search import SimpleFunSearch  # noqa: F401

_standalone: Optional[Evaluator] = None


def evaluate_policy_standalone(policy_data: Tuple[int, str]) -> Tuple[int, str, Optional[float]]:
    """``(index, code) -> (index, code, score)``; any failure scores 0
    (reference `funsearch_integration.py:30-64`).  The workload is parsed once
    per process and stays resident on the device between calls."""
    global _standalone
    idx, code = policy_data
    try:
        if _standalone is None:
            _standalone = Evaluator()
        return idx, code, _standalone.evaluate_programs([code])[0].score
    except Exception:
        return idx, code, 0


def main(config_path: str = "configs/llm_config.json") -> None:
    funsearch = SimpleFunSearch(config_path)
    try:
        best_policy, best_score = funsearch.run_evolution()
        path = funsearch.save_top_policies(top_k=5)
        print("\nFinal Results:")
        print(f"Best Score: {best_score:.4f}")
        print(f"Top 5 policies saved to: {path}")
    except KeyboardInterrupt:
        print("\nEvolution interrupted by user")
        if funsearch.population:
            print(f"Current top policies saved to: {funsearch.save_top_policies(top_k=5)}")


if __name__ == "__main__":
    import sys
    main(*sys.argv[1:2])
