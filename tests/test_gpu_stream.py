"""Online IK (config #5) reproduces run_inference exactly, graph and eager."""
import numpy as np
import pytest

from conftest import golden

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("win,graph", [(64, True), (9, True), (9, False)])
def test_stream_matches_run_inference(win, graph):
    from temporal_inverse_kinematics_amd import _build
    _build.build()
    from temporal_inverse_kinematics_amd.inference import run_inference, synthetic_model
    from temporal_inverse_kinematics_amd.streaming import OnlineIK
    r = golden("run_inference.npz")
    seq = r["seq"][:100] if win == 64 else r["seq"]
    m = synthetic_model(win_size=win, device="cuda")
    ref = run_inference(m, seq)
    online = OnlineIK(m, use_graph=graph)
    got = online.run(seq)
    assert got.shape == ref.shape
    assert np.abs(got - ref).max() < 1e-5
    if seq.shape[0] == 231:
        assert np.abs(got - r[f"win{win}"]).max() < 1e-4
    # a second pass after reset gives the same answer
    again = online.run(seq)
    assert np.array_equal(again, got)
