"""Online IK (config #5) reproduces run_inference exactly, graph and eager."""
import numpy as np
import pytest

from conftest import golden

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("win,graph,online", [(64, True, "1"), (9, True, "1"), (9, False, "1"), (64, True, "0"),
                                              (9, False, "0")])
def test_stream_matches_run_inference(win, graph, online, monkeypatch):
    """Both steps: the dataflow kernel (default) and the layered forward (TIK_ONLINE=0)."""
    monkeypatch.setenv("TIK_ONLINE", online)
    from temporal_inverse_kinematics_amd import _build
    _build.build()
    from temporal_inverse_kinematics_amd.inference import run_inference, synthetic_model
    from temporal_inverse_kinematics_amd.streaming import OnlineIK
    r = golden("run_inference.npz")
    seq = r["seq"][:100] if win == 64 else r["seq"]
    m = synthetic_model(win_size=win, device="cuda")
    ref = run_inference(m, seq)
    online = OnlineIK(m, use_graph=graph)
    assert online.path == ("dataflow" if online_flag(online) else "layered")
    got = online.run(seq)
    assert got.shape == ref.shape
    assert np.abs(got - ref).max() < 1e-5
    if seq.shape[0] == 231:
        assert np.abs(got - r[f"win{win}"]).max() < 1e-4
    # a second pass after reset gives the same answer
    again = online.run(seq)
    assert np.array_equal(again, got)


def online_flag(_):
    import os
    return os.environ.get("TIK_ONLINE", "1") != "0"


def test_online_default_path_win64_full_sample_vs_golden():
    """the default online path (dataflow kernel, hipGraph
    replay) over the whole 231-frame sample at win_size 64 (T = 65) against the
    reference's own run_inference output (golden run_inference.npz:win64,
    inference.py:37-67 over data_amass.py:18-42 windows) at 1e-4."""
    import os
    assert os.environ.get("TIK_ONLINE", "1") != "0"
    from temporal_inverse_kinematics_amd import _build
    _build.build()
    from temporal_inverse_kinematics_amd.inference import synthetic_model
    from temporal_inverse_kinematics_amd.streaming import OnlineIK
    r = golden("run_inference.npz")
    assert r["seq"].shape[0] == 231
    m = synthetic_model(win_size=64, device="cuda")
    online = OnlineIK(m, use_graph=True)
    assert online.path == "dataflow" and online.win_size == 64
    got = online.run(r["seq"])
    assert got.shape == r["win64"].shape == (231, 66)
    assert np.abs(got - r["win64"]).max() < 1e-4


def _regressor_with_layers(layers, win, seed=7):
    """An IKPoseTrainer whose backbone has the given (cout, stride) blocks
    (the last one 256 channels for the 17 x 256 head), seeded synthetic weights."""
    import torch
    from temporal_inverse_kinematics_amd import synthetic as syn
    from temporal_inverse_kinematics_amd.models import IKPoseTrainer, PoseRegressor, default_hparams

    class Reg(PoseRegressor):
        LAYERS = layers

    class Trainer(IKPoseTrainer):
        def __init__(self, hp):
            torch.nn.Module.__init__(self)
            self.hparams = hp
            self.regressor = Reg(hp)

    model = Trainer(default_hparams(win))
    full, c = [], 3
    for cout, s in layers:
        full.append((c, cout, s))
        c = cout
    sd = syn.ik_state_dict(model.regressor.backbone.graph.A, seed=seed, layers=full)
    res = model.regressor.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()}, strict=False)
    assert not [k for k in res.missing_keys if "num_batches_tracked" not in k] and not res.unexpected_keys
    return model.cuda().eval()


@pytest.mark.parametrize("c1", [48, 80])
def test_online_identity_block_c_mod_32_eq_16(c1, monkeypatch):
    """in the dataflow kernel's temporal-conv task the block
    input x of an identity-residual layer is staged after the 3 C tap channels,
    and the K padding up to a multiple of 32 is zeroed. With C % 32 == 16
    (C = 48: 3 C = 144 -> 160) that padding overlapped x's first 16 channels,
    so the identity term read zeros. x now sits past the padding. Both identity
    blocks (layers 1 and 2) have C % 32 == 16; the dataflow step must equal the
    layered one (TIK_ONLINE=0)."""
    from temporal_inverse_kinematics_amd import _build
    _build.build()
    from temporal_inverse_kinematics_amd.streaming import OnlineIK
    layers = [(c1, 1), (c1, 1), (c1, 1), (128, 2), (128, 1), (128, 2), (256, 2), (256, 2)]
    m = _regressor_with_layers(layers, 64)
    seq = golden("run_inference.npz")["seq"][:40]
    monkeypatch.setenv("TIK_ONLINE", "0")
    ref = OnlineIK(m, use_graph=True).run(seq)
    monkeypatch.setenv("TIK_ONLINE", "1")
    s = OnlineIK(m, use_graph=True)
    assert s.path == "dataflow"
    got = s.run(seq)
    assert np.isfinite(ref).all()
    assert np.abs(got - ref).max() < 2e-5


@pytest.mark.parametrize("value", ["f16x3", "bf16", "FP32"])
def test_unknown_precision_env_fails(value, monkeypatch):
    """an unrecognised TIK_PRECISION (the retired f16x3
    included) fails the handle's creation instead of running bf16x3 silently."""
    import torch
    from temporal_inverse_kinematics_amd import _build
    _build.build()
    from temporal_inverse_kinematics_amd.inference import synthetic_model
    monkeypatch.setenv("TIK_PRECISION", value)
    m = synthetic_model(win_size=9, device="cuda")
    with pytest.raises(Exception, match="TIK_PRECISION"):
        with torch.no_grad():
            m(torch.zeros(1, 9, 17, 3, device="cuda"))


@pytest.mark.parametrize("win", [3, 21, 22, 23, 40, 64, 129])
def test_online_kernel_matches_layered(win, monkeypatch):
    """The dataflow step (only the frames pose row 0 depends on, fp32) against
    the layered step on the whole window, over window sizes around the 22-frame
    receptive field of row 0, including ones shorter than it."""
    from temporal_inverse_kinematics_amd import _build
    _build.build()
    from temporal_inverse_kinematics_amd.inference import synthetic_model
    from temporal_inverse_kinematics_amd.streaming import OnlineIK
    r = golden("run_inference.npz")
    seq = r["seq"][:50]
    m = synthetic_model(win_size=win, device="cuda")
    monkeypatch.setenv("TIK_ONLINE", "0")
    ref = OnlineIK(m, use_graph=True).run(seq)
    monkeypatch.setenv("TIK_ONLINE", "1")
    s = OnlineIK(m, use_graph=True)
    assert s.path == "dataflow"
    got = s.run(seq)
    assert np.abs(got - ref).max() < 2e-5
    # 300 more replays: counters and tickets are left clean by every launch
    for i in range(300):
        s.push(seq[i % seq.shape[0]])
    assert np.array_equal(s.run(seq), got)


@pytest.mark.parametrize("grid", ["1", "3", "64"])
def test_online_kernel_grid_sizes(grid, monkeypatch):
    """Any number of workgroups gives the same poses (tickets are taken in
    topological order, so even one workgroup runs every task)."""
    from temporal_inverse_kinematics_amd import _build
    _build.build()
    from temporal_inverse_kinematics_amd.inference import synthetic_model
    from temporal_inverse_kinematics_amd.streaming import OnlineIK
    r = golden("run_inference.npz")
    seq = r["seq"][:40]
    m = synthetic_model(win_size=64, device="cuda")
    base = OnlineIK(m, use_graph=False).run(seq)
    monkeypatch.setenv("TIK_ONLINE_GRID", grid)
    got = OnlineIK(m, use_graph=True).run(seq)
    assert np.array_equal(got, base)


def test_stream_survives_batch_calls_and_rebuilds():
    """a live OnlineIK must not share the handle's workspace.
    Create the stream FIRST, then run batch calls on the same model that grow
    the handle's workspace (and run on another torch stream), then rebuild the
    handle by changing a weight: the stream keeps giving the poses of the
    weights it was created with, and its graph never touches freed memory."""
    import torch
    from temporal_inverse_kinematics_amd import _build
    _build.build()
    from temporal_inverse_kinematics_amd.inference import run_inference, synthetic_model
    from temporal_inverse_kinematics_amd.streaming import OnlineIK
    from temporal_inverse_kinematics_amd import synthetic as syn
    r = golden("run_inference.npz")
    seq = r["seq"][:60]
    m = synthetic_model(win_size=9, device="cuda")
    online = OnlineIK(m, use_graph=True)
    first = online.run(seq)
    ref = run_inference(m, seq)
    assert np.abs(first - ref).max() < 1e-5
    # large batches on the handle: its workspace is reallocated several times,
    # one of them on a non-default torch stream while the online stream is idle
    x = torch.from_numpy(syn.synthetic_windows(700, 64, seed=3)).cuda()
    with torch.no_grad():
        m(x)
        s2 = torch.cuda.Stream()
        with torch.cuda.stream(s2):
            m(torch.from_numpy(syn.synthetic_windows(1500, 64, seed=4)).cuda())
        torch.cuda.synchronize()
    assert np.array_equal(online.run(seq), first)
    # a weight change rebuilds the handle (the old one is released); the
    # stream still holds the old model and still reproduces its poses
    with torch.no_grad():
        m.regressor.pose_regressor[3].bias.add_(1.0)
    moved = run_inference(m, seq)
    assert np.abs(moved - ref).max() > 0.5
    import gc
    gc.collect()
    assert np.array_equal(online.run(seq), first)
    # a new stream follows the new weights
    assert np.abs(OnlineIK(m, use_graph=True).run(seq) - moved).max() < 1e-5
    del online
    gc.collect()


def test_online_timeout_recovers():
    """a dependency timeout in the dataflow kernel (forced
    here through tik_debug_stream_inject_error) fails that push only: the
    frame is still appended (host and device frame counts stay in step), the
    error flag is cleared for the next launch, and the stream keeps matching
    run_inference afterwards; reset() clears everything."""
    from temporal_inverse_kinematics_amd import _build, _lib
    _build.build()
    from temporal_inverse_kinematics_amd.inference import run_inference, synthetic_model
    from temporal_inverse_kinematics_amd.streaming import OnlineIK
    r = golden("run_inference.npz")
    seq = r["seq"][:40]
    m = synthetic_model(win_size=9, device="cuda")
    ref = run_inference(m, seq)
    s = OnlineIK(m, use_graph=True)
    assert s.path == "dataflow"
    lib = _lib.load()
    s.reset()
    got = {}
    for i, fr in enumerate(seq):
        if i == 10:
            _lib.check(lib.tik_debug_stream_inject_error(s._s))
            with pytest.raises(RuntimeError):
                s.push(fr)
            continue
        p = s.push(fr)
        if p is not None:
            got[i - s.h] = p
    for i, p in got.items():
        if i != 10 - s.h:
            assert np.abs(p - ref[i]).max() < 1e-5, i
    assert np.array_equal(s.run(seq), OnlineIK(m, use_graph=True).run(seq))


@pytest.mark.parametrize("n_first", [7, 8])
def test_online_reset_restores_the_activation_tag(n_first):
    """The dataflow kernel hands activations over through the launch parity in
    their sign bit (online.hip): launch c writes tag c & 1, and a consumer waits
    for it. reset() restarts the frame count at 0, so it must also put every
    element back to tag 1 — after an odd number of pushes the buffer holds tag 0,
    which launch 0 would otherwise accept as fresh (stale rows, wrong poses)."""
    from temporal_inverse_kinematics_amd import _build
    _build.build()
    from temporal_inverse_kinematics_amd.inference import synthetic_model
    from temporal_inverse_kinematics_amd.streaming import OnlineIK
    r = golden("run_inference.npz")
    seq = r["seq"][:30]
    m = synthetic_model(win_size=64, device="cuda")
    ref = OnlineIK(m, use_graph=True).run(seq)
    s = OnlineIK(m, use_graph=True)
    s.reset()
    other = r["seq"][100:100 + n_first]
    for fr in other:
        s.push(fr)
    # run() resets, then replays seq from frame 0
    assert np.array_equal(s.run(seq), ref)


@pytest.mark.parametrize("online", ["1", "0"])
def test_stream_count_wrap(online, monkeypatch):
    """The device frame count stays below 2^30 (csrc/online.h stream_next_count):
    a stream moved to just below the wrap (tik_debug_stream_set_count, same ring
    slot and parity) keeps giving the poses of one that never wrapped, on the
    dataflow kernel and on the layered step."""
    monkeypatch.setenv("TIK_ONLINE", online)
    from temporal_inverse_kinematics_amd import _build, _lib
    _build.build()
    from temporal_inverse_kinematics_amd.inference import synthetic_model
    from temporal_inverse_kinematics_amd.streaming import OnlineIK
    r = golden("run_inference.npz")
    seq = r["seq"][:120]
    m = synthetic_model(win_size=64, device="cuda")
    a, b = OnlineIK(m, use_graph=True), OnlineIK(m, use_graph=True)
    a.reset()
    b.reset()
    for fr in seq[:80]:
        a.push(fr)
        b.push(fr)
    W = 2 * b.h + 1
    k = ((1 << 30) - 10 - 80) // (2 * W)
    lib = _lib.load()
    _lib.check(lib.tik_debug_stream_set_count(b._s, 80 + 2 * W * k))
    with pytest.raises(ValueError):   # not congruent modulo 2W
        _lib.check(lib.tik_debug_stream_set_count(b._s, 81 + 2 * W * k))
    for fr in seq[80:]:   # crosses 2^30 after ~10 pushes
        pa, pb = a.push(fr), b.push(fr)
        assert np.array_equal(pa, pb)
