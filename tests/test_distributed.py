"""The N>1 path on CPU: world_size-2 gloo processes shard a global batch
contiguously and all-gather the per-rank pose blocks in rank order (the
compute is injected: the HIP forward has no CPU path)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from temporal_inverse_kinematics_amd.distributed import gather_poses, shard_range, sharded_forward
    g = torch.arange(n * 4 * 66, dtype=torch.float32).reshape(n, 4, 66)
    seen = []

    def fwd(x):
        # PoseRegressor.forward's shape contract: (N,...) -> (N,...), N == 0 included
        seen.append(x.shape[0])
        return x * 2 + 1

    out = sharded_forward(fwd, g)
    ok = torch.equal(out, g * 2 + 1)
    lo, hi = shard_range(n, rank, world)
    ok = ok and seen == [hi - lo]
    if n % world == 0:
        local = g[lo:hi] + rank
        full = gather_poses(local)
        exp = torch.cat([g[shard_range(n, r, world)[0]:shard_range(n, r, world)[1]] + r for r in range(world)])
        ok = ok and torch.equal(full, exp)
    q.put((rank, bool(ok)))
    dist.destroy_process_group()


@pytest.mark.parametrize("n", [8, 7, 1])
def test_sharded_gather_gloo_ws2(n):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, n, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(60)
    assert res == {0: True, 1: True}


def test_shard_range_covers():
    from temporal_inverse_kinematics_amd.distributed import shard_range
    for n in [0, 1, 7, 8, 1023, 8192]:
        for w in [1, 2, 3, 8]:
            spans = [shard_range(n, r, w) for r in range(w)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(spans[i][1] == spans[i + 1][0] for i in range(w - 1))


def _worker_model(rank, world, port, q):
    """n < world with the real PoseRegressor: the rank with the empty shard
    gets an empty (0,T',66) result from forward (no library call) and still
    joins the all-gather; the other rank's forward is stubbed on CPU."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from temporal_inverse_kinematics_amd.distributed import sharded_forward
    from temporal_inverse_kinematics_amd.models import PoseRegressor, default_hparams
    m = PoseRegressor(default_hparams(win_size=64)).eval()
    x = torch.zeros((1, 64, 17, 3))

    def fwd(xs):
        if xs.shape[0] == 0:
            return m(xs)["poses"]
        return torch.full((xs.shape[0], m.backbone.out_frames(64), 66), 7.0)

    out = sharded_forward(fwd, x)
    q.put((rank, tuple(out.shape) == (1, 4, 66) and bool((out == 7.0).all())))
    dist.destroy_process_group()


def test_empty_shard_joins_gather_gloo_ws2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_model, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=180) for _ in procs)
    for p in procs:
        p.join(60)
    assert res == {0: True, 1: True}


def test_empty_batch_forward_cpu():
    from temporal_inverse_kinematics_amd.models import PoseRegressor, default_hparams
    m = PoseRegressor(default_hparams(win_size=64)).eval()
    y = m(torch.zeros((0, 64, 17, 3)))["poses"]
    assert tuple(y.shape) == (0, 4, 66)
    f = m.backbone_features(torch.zeros((0, 9, 17, 3)))
    assert tuple(f.shape) == (0, 1, 17 * 256)


def _pipe_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from temporal_inverse_kinematics_amd.distributed import PosesGatherPipeline, gather_poses
    pipe = PosesGatherPipeline()
    outs, refs = [], []
    for k in range(4):
        y = torch.full((3, 4, 66), float(10 * k + rank))
        refs.append(gather_poses(y))
        outs.append(pipe.push(y))
    pipe.drain()
    ok = all(torch.equal(a, b) for a, b in zip(outs, refs))
    q.put((rank, bool(ok)))
    dist.destroy_process_group()


def test_gather_pipeline_gloo_ws2():
    """The overlapped all-gather (bench.py's multi-GPU step) delivers every
    batch's gathered poses, in rank order, once the next push / drain returns."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_pipe_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(60)
    assert res == {0: True, 1: True}
