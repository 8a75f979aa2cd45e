"""pytest setup: the ``gpu`` marker and the repo root on sys.path."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP kernels on cuda:0)")
    config.addinivalue_line("markers", "slow: long-running test")


@pytest.fixture(autouse=True)
def _reset_topology():
    from fleetx_amd.parallel import topology as topo
    from fleetx_amd.parallel.rng import model_parallel_random_seed
    topo.reset_hcg()
    model_parallel_random_seed(1234)
    yield
    topo.reset_hcg()
