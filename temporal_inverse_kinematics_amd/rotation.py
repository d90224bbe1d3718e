"""Rotation conversions on the GPU — drop-in for
`common/kornia_geometry_conversion.angle_axis_to_rotation_matrix` (:125-201)."""
from __future__ import annotations

import torch

from . import _lib


def angle_axis_to_rotation_matrix(angle_axis: torch.Tensor) -> torch.Tensor:
    """(N,3) -> (N,3,3); Taylor branch for theta^2 <= 1e-6, as kornia."""
    if not isinstance(angle_axis, torch.Tensor):
        raise TypeError("Input type is not a torch.Tensor. Got {}".format(type(angle_axis)))
    if not angle_axis.shape[-1] == 3:
        raise ValueError("Input size must be a (*, 3) tensor. Got {}".format(angle_axis.shape))
    aa = angle_axis.reshape(-1, 3).contiguous()
    _lib.require_gpu(aa)
    R = torch.empty((aa.shape[0], 3, 3), device=aa.device, dtype=torch.float32)
    _lib.check(_lib.load().tik_aa_to_rotmat(aa.data_ptr(), aa.shape[0], R.data_ptr(), _lib.stream_of(aa)),
               "angle_axis_to_rotation_matrix")
    return R
