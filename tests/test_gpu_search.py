"""Program-level search on the MI355X: pipelined program islands evaluated by
the native backend while the family coupler runs its device family search on
its own HIP slot (funsearch/coupling.py)."""
import json

import pytest

pytestmark = pytest.mark.gpu


def test_coupled_islands_on_device(tmp_path):
    from funsearch_kubernetes_simulator_amd.funsearch.islands import IslandFunSearch
    from funsearch_kubernetes_simulator_amd.models.library import reference_scores
    from funsearch_kubernetes_simulator_amd.ops import hip_engine as he
    if not he.device_available():
        pytest.fail("GPU test collected but no HIP device is visible")
    cfg = {"llm": {"backend": "mutation", "seed": 3}, "safe_execution": {"timeout_seconds": 3},
           "funsearch": {"population_size": 8, "generations": 3, "early_stop_threshold": 1.0, "elite_size": 3,
                         "max_workers": 4, "policies_per_generation": 5},
           "device": {"kind": "auto", "min_batch": 1},
           "islands": {"per_rank": 2, "migrate_every": 0, "migrants": 1, "pipeline": True},
           "coupling": {"every": 1, "generations": 1, "candidates": 512, "elite": 8,
                        "families": ["random_linear", "feature_linear"]},
           "checkpoint": {}, "log_path": str(tmp_path / "log.jsonl")}
    fs = IslandFunSearch(cfg)
    assert fs.evaluator.backend == "hip" and fs.coupler.slot == fs._n_slots() - 1 >= 2
    code, score = fs.run(3)
    recs = [json.loads(l) for l in open(tmp_path / "log.jsonl")]
    cp = [r for r in recs if r["kind"] == "coupling"]
    assert cp and all(r["score"] == r["family_score"] for r in cp)   # device family score == program text score
    assert fs.evaluator.stats["device_native"] > 0
    assert score >= reference_scores()["best_fit"]
