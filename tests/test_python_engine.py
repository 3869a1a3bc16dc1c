"""Golden tests of the object-level (reference-semantics) engine."""
import copy

import pytest

from funsearch_kubernetes_simulator_amd.funsearch.scheduler import FunSearchScheduler
from funsearch_kubernetes_simulator_amd.models.library import reference_policies, reference_scores
from funsearch_kubernetes_simulator_amd.simulator import (DiscreteEventSimulator, KubernetesSimulator,
                                                         SchedulingEvaluator)

# snapshots / fragmentation events / events per replay measured on the reference
COUNTS = {"first_fit": (47, 3152, 19456), "best_fit": (40, 79, 16383),
          "funsearch_4901": (67, 11259, 27563), "funsearch_4816": (45, 2353, 18657),
          "funsearch_4800": (45, 2299, 18603)}


@pytest.mark.parametrize("name", list(COUNTS))
def test_reference_scores_exact(name, default_objects):
    cluster, pods = copy.deepcopy(default_objects)
    ev = SchedulingEvaluator(cluster)
    sim = KubernetesSimulator(cluster, pods, DiscreteEventSimulator(pods),
                              FunSearchScheduler(reference_policies()[name]), evaluator=ev)
    sim.run_schedule()
    res = ev.get_evaluation_results()
    assert ev.get_policy_score(pods) == reference_scores()[name]
    assert (res.num_snapshots, res.num_fragmentation_events, sim.events_processed) == COUNTS[name]


def test_invariants_prefix(default_objects):
    cluster, pods = copy.deepcopy(default_objects)
    pods = sorted(pods, key=lambda p: p.creation_time)[:400]
    sim = KubernetesSimulator(cluster, pods, DiscreteEventSimulator(pods),
                              FunSearchScheduler(reference_policies()["first_fit"]),
                              validate_invariants=True)
    sim.run_schedule()
    assert all(p.assigned_node for p in pods)
