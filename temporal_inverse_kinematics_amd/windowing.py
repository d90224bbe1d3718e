"""Temporal windowing — drop-in for `sample_window` and `InferenceDataset`
(`mmskeleton/datasets/data_amass.py:18-42, 221-236`), plus the on-device
batched gather (`tik_window_gather`) the inference path uses.
"""
from __future__ import annotations

import numpy as np
import torch

from . import _lib


def sample_window(arr, idx, h_win_size):
    """2h+1 frames centred at idx, edge-padded (host numpy).

    Same ValueError condition as data_amass.py:27-29, and the same short
    window the reference returns when a window overruns both ends.
    """
    F = arr.shape[0]
    h = h_win_size
    pad_l = pad_r = 0
    if h > idx > F - h:
        raise ValueError(f"h_win_size > idx > arr.shape[0] - h_win_size: {h} > {idx} > {F} - {h}")
    if idx < h:
        pad_l = h - idx
    elif idx > F - h - 1:
        pad_r = idx - (F - h) + 1
    pads = [[0, 0] for _ in range(arr.ndim)]
    pads[0] = [pad_l, pad_r]
    if pad_l or pad_r:
        arr = np.pad(arr, pads, "edge")
    return arr[idx + pad_l - h: idx + pad_l + h + 1]


class InferenceDataset(torch.utils.data.Dataset):
    """data_amass.py:221-236 — item idx = (root-relative window, idx)."""

    def __init__(self, input_3d_poses: np.ndarray, win_size: int, relative_pose=True):
        self.poses_3d = input_3d_poses
        self.half_win_size = win_size // 2
        self.relative_pose = relative_pose

    def __len__(self):
        return self.poses_3d.shape[0]

    def __getitem__(self, idx):
        w = sample_window(self.poses_3d, idx, self.half_win_size)
        if self.relative_pose:
            roots = 0.5 * (w[:, 11, :] + w[:, 12, :])
            w = w - roots[:, np.newaxis, :]
        return w, idx


def gather_windows(seq: torch.Tensor, win_size: int, idx0: int = 0, n: int | None = None,
                   relative_pose: bool = True, root=(11, 12), out: torch.Tensor | None = None) -> torch.Tensor:
    """All InferenceDataset items [idx0, idx0+n) at once on the GPU:
    seq (F,V,3) device -> (n, 2h+1, V, 3) device, h = win_size//2."""
    _lib.require_gpu(seq)
    F, V, C = seq.shape
    if C != 3:
        raise ValueError("expected (F,V,3) keypoints")
    h = win_size // 2
    n = F - idx0 if n is None else n
    if out is None:
        out = torch.empty((n, 2 * h + 1, V, 3), device=seq.device, dtype=torch.float32)
    _lib.check(_lib.load().tik_window_gather(seq.data_ptr(), F, V, idx0, n, h, root[0], root[1],
                                             int(relative_pose), out.data_ptr(), _lib.stream_of(seq)),
               "sample_window")
    return out
