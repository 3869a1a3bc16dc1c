import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device)")
    config.addinivalue_line("markers", "slow: long-running CPU test")


@pytest.fixture(scope="session")
def default_workload():
    from funsearch_kubernetes_simulator_amd.core import load_default_workload
    return load_default_workload()


@pytest.fixture(scope="session")
def default_objects():
    from funsearch_kubernetes_simulator_amd.core import TraceParser
    return TraceParser().parse_workload()
