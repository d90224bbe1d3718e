"""Multi-GPU IK: windows are independent (data_amass.py:18-42 makes each window
self-contained), so a batch shards contiguously over ranks with no data-path
exchange; the one collective is the all-gather of the predicted SMPL-X pose
parameters to every rank (BASELINE.json config #3), RCCL over xGMI on the GPU
box (torch.distributed backend "nccl" = RCCL), gloo in the CPU tests.
"""
from __future__ import annotations

from typing import Callable, Optional

import torch
import torch.distributed as dist


def shard_range(n: int, rank: int, world: int):
    """Contiguous shard [lo, hi) of n items for `rank` (first n % world ranks get one more)."""
    base, rem = divmod(n, world)
    lo = rank * base + min(rank, rem)
    return lo, lo + base + (1 if rank < rem else 0)


def gather_poses(local: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """All-gather equal-size per-rank pose blocks (B,T',66) into rank order (world*B,T',66)."""
    if not dist.is_initialized() or dist.get_world_size() == 1:
        return local if out is None else out.copy_(local)
    world = dist.get_world_size()
    if out is None:
        out = torch.empty((world * local.shape[0],) + tuple(local.shape[1:]), device=local.device, dtype=local.dtype)
    if dist.get_backend() == "gloo":
        parts = list(out.chunk(world, 0))
        dist.all_gather(parts, local.contiguous())
    else:
        dist.all_gather_into_tensor(out, local.contiguous())
    return out


def sharded_forward(forward: Callable[[torch.Tensor], torch.Tensor], windows: torch.Tensor) -> torch.Tensor:
    """Run `forward` on this rank's contiguous shard of `windows` (global batch,
    identical on every rank) and all-gather the results in global order.
    Uneven shards are padded to the largest shard for the collective and
    trimmed afterwards. A rank whose shard is empty (fewer windows than
    ranks) still joins the collective: `forward` must map an empty batch to
    an empty (0, ...) result, as PoseRegressor.forward does."""
    if not dist.is_initialized() or dist.get_world_size() == 1 or windows.shape[0] == 0:
        return forward(windows)
    world, rank = dist.get_world_size(), dist.get_rank()
    n = windows.shape[0]
    lo, hi = shard_range(n, rank, world)
    y = forward(windows[lo:hi])
    cap = -(-n // world)
    pad = torch.zeros((cap,) + tuple(y.shape[1:]), device=y.device, dtype=y.dtype)
    pad[: hi - lo] = y
    full = gather_poses(pad)
    parts = [full[r * cap: r * cap + (shard_range(n, r, world)[1] - shard_range(n, r, world)[0])] for r in range(world)]
    return torch.cat(parts, 0)


class PosesGatherPipeline:
    """Overlaps the pose all-gather of batch k with the forward of batch k+1.

    push(y) issues the all-gather of this rank's block y asynchronously (RCCL
    runs it on its own stream after the forward that produced y) into `out`
    (or a fresh (world*B,...) tensor) and then makes the caller's stream wait
    for the PREVIOUS batch's gather, so that gather ran concurrently with this
    batch's forward. drain() waits for the last one. Each gathered tensor is
    complete once the next push() (or drain()) has returned; push returns the
    tensor its gather writes. The local blocks stay referenced until their
    gather is waited on."""

    def __init__(self):
        self._pending = []

    def push(self, local: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
        if not dist.is_initialized() or dist.get_world_size() == 1:
            return local if out is None else out.copy_(local)
        world = dist.get_world_size()
        if out is None:
            out = torch.empty((world * local.shape[0],) + tuple(local.shape[1:]), device=local.device, dtype=local.dtype)
        local = local.contiguous()
        if dist.get_backend() == "gloo":
            work = dist.all_gather(list(out.chunk(world, 0)), local, async_op=True)
        else:
            work = dist.all_gather_into_tensor(out, local, async_op=True)
        self._pending.append((work, local, out))
        while len(self._pending) > 1:
            w, _, _ = self._pending.pop(0)
            w.wait()
        return out

    def drain(self) -> None:
        while self._pending:
            w, _, _ = self._pending.pop(0)
            w.wait()
