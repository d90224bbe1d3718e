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


# The f16x3 arithmetic (3 f16 products, f16 range: not range-safe, see
# test_gpu_precision.py) and its fused kernel set are experimental: their GPU
# tests run only with TIK_TEST_F16X3=1.
F16X3 = bool(os.environ.get("TIK_TEST_F16X3"))
f16x3_only = pytest.mark.skipif(not F16X3, reason="f16x3 is experimental; TIK_TEST_F16X3=1 runs its tests")


def prec_params(*names):
    """pytest params for precision names, the f16x3 ones marked experimental."""
    return [pytest.param(n, marks=f16x3_only) if str(n).startswith("f16x3") else n for n in names]


def golden(name):
    return np.load(os.path.join(GOLDEN, name), allow_pickle=False)


@pytest.fixture(scope="session")
def ik_weights():
    from temporal_inverse_kinematics_amd import synthetic as syn
    from oracle import stgcn as orc
    A = orc.graph_A("coco", "uniform", 2, 1)
    return syn.ik_state_dict(A, seed=0)
