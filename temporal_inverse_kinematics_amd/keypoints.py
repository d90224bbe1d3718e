"""Keypoint format maps — drop-in for `common/keypoints_util.py:5-60` plus the
moveai_3d → COCO conversion of `inference.run_test` (`inference.py:121-133`)."""
from __future__ import annotations

from typing import List

import numpy as np
import torch

_COCO_FROM_SMPLX = ["nose", "left_eye", "right_eye", "left_ear", "right_ear", "left_shoulder",
                    "right_shoulder", "left_elbow", "right_elbow", "left_wrist", "right_wrist", "left_hip",
                    "right_hip", "left_knee", "right_knee", "left_ankle", "right_ankle"]
_COCO_FROM_MOVEAI = [None, None, None, "L_Ear", "R_Ear", "L_Shoulder", "R_Shoulder", "L_Elbow", "R_Elbow",
                     "L_Wrist", "R_Wrist", "L_Hip", "R_Hip", "L_Knee", "R_Knee", "L_Ankle", "R_Ankle"]


def generate_smplx_to_coco_mappings(smplx_kps_names: List[str]) -> List[int]:
    """keypoints_util.py:5-24"""
    return [smplx_kps_names.index(n) for n in _COCO_FROM_SMPLX]


def generate_moveai3d_to_coco_mappings(mvai_3d_joint_names: List[str]) -> List[int]:
    """keypoints_util.py:27-46 (nose/eyes have no moveai joint: -1)."""
    return [-1 if n is None else mvai_3d_joint_names.index(n) for n in _COCO_FROM_MOVEAI]


def convert_seq_keypoints(in_seq_kps, mappings, do_copy=False):
    """keypoints_util.py:49-60: (B,J,C) -> (B,len(mappings),C) f32, -1 -> zeros."""
    m = np.asarray(mappings)
    out = np.zeros((in_seq_kps.shape[0], len(m), in_seq_kps.shape[2]), dtype=np.float32)
    ok = m >= 0
    out[:, ok] = in_seq_kps[:, m[ok]]
    return out


def moveai3d_to_coco(joints_3d: np.ndarray, joint_names: List[str]) -> np.ndarray:
    """inference.py:121-133: gather, head points from the ears, axis swap (x,y,z)->(x,z,-y)."""
    kps = convert_seq_keypoints(joints_3d, generate_moveai3d_to_coco_mappings(joint_names))
    kps[:, 0] = 0.5 * (joints_3d[:, -1] + joints_3d[:, -2])
    kps[:, 1] = joints_3d[:, -2]
    kps[:, 2] = joints_3d[:, -1]
    y = kps[:, :, 1].copy()
    kps[:, :, 1] = kps[:, :, 2]
    kps[:, :, 2] = -y
    return kps


def moveai3d_to_coco_device(joints_3d: torch.Tensor, joint_names: List[str]) -> torch.Tensor:
    """moveai3d_to_coco on the GPU (tik_moveai_to_coco, one gather kernel):
    joints_3d (F,J,3) fp32 device -> (F,17,3) device, bit-identical to the host
    version."""
    from . import _lib
    _lib.require_gpu(joints_3d)
    if joints_3d.dim() != 3 or joints_3d.shape[2] != 3:
        raise ValueError(f"expected (F,J,3) joints, got {tuple(joints_3d.shape)}")
    F, J, _ = joints_3d.shape
    m = (_lib.ctypes.c_int * 17)(*generate_moveai3d_to_coco_mappings(joint_names))
    out = torch.empty((F, 17, 3), device=joints_3d.device, dtype=torch.float32)
    _lib.check(_lib.load().tik_moveai_to_coco(joints_3d.data_ptr(), F, J, m, out.data_ptr(),
                                              _lib.stream_of(joints_3d)), "moveai3d_to_coco_device")
    return out
