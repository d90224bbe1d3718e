import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(REPO, "tests", "golden")
if REPO not in sys.path:
    sys.path.insert(0, REPO)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run with -m gpu on the GPU box)")


def golden(name):
    return np.load(os.path.join(GOLDEN, name), allow_pickle=False)


@pytest.fixture(scope="session")
def ik_weights():
    from temporal_inverse_kinematics_amd import synthetic as syn
    from oracle import stgcn as orc
    A = orc.graph_A("coco", "uniform", 2, 1)
    return syn.ik_state_dict(A, seed=0)
