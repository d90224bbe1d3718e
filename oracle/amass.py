"""ORACLE — CPU restatement of AmassDataset's training-data generation
(mmskeleton/datasets/data_amass.py:87-218). TEST INFRASTRUCTURE ONLY: only
tests/ and the CPU-baseline leg of bench_train_data.py may import it.

* regenerate_data's root-orientation augmentation uses scipy.spatial.transform
  exactly as the reference does (data_amass.py:184-190): scipy is the
  reference's own dependency and is importable here, so this part is pinned
  to the library itself.
* __getitem__ (data_amass.py:125-154): sample_window (oracle/stgcn.py, pinned
  to the reference's golden windows), convert_smplx (:45-55), root-relative
  (:133-135), _aug_3d_keypoints (:65-84) with the reference's float32
  arithmetic, target = poses window [-1:, :66].
* The keypoint noise: the reference draws it from numpy's global generator
  (np.random.multivariate_normal with a diagonal covariance whose diagonal is
  sigma, i.e. std = sqrt(sigma)); the GPU path draws the same distribution
  from a counter-based generator keyed by (seed, dataset index, value index)
  so that any batching gives the same numbers. counter_normal below restates
  that generator (splitmix64 + Box-Muller) so the GPU noise is checked value
  by value; the distribution itself is checked statistically.
"""
from __future__ import annotations

from typing import Dict, List

import numpy as np

from .stgcn import sample_window

# keypoints_util.py:5-24 over smplx.joint_names.JOINT_NAMES (first 60 names; golden
# tests/golden/keypoints.npz pins the mapping): COCO-17 <- SMPL-X joint index
SMPLX_TO_COCO = [55, 57, 56, 59, 58, 16, 17, 18, 19, 20, 21, 1, 2, 4, 5, 7, 8]


def coco_kps_sigma() -> np.ndarray:
    """data_amass.py:58-62"""
    return np.array([.26, .25, .25, .35, .35, .79, .79, .72, .72, .62, .62, 1.07, 1.07, .87, .87, .89, .89],
                    dtype=np.float32) * 0.1


_M64 = (1 << 64) - 1


def splitmix64(x: np.ndarray) -> np.ndarray:
    x = (np.asarray(x, dtype=np.uint64) + np.uint64(0x9E3779B97F4A7C15)) & np.uint64(_M64)
    x = ((x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)) & np.uint64(_M64)
    x = ((x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)) & np.uint64(_M64)
    return x ^ (x >> np.uint64(31))


def counter_normal(seed: int, uid: int, n: np.ndarray) -> np.ndarray:
    """Standard normals number n of item uid's stream (train_data.hip counter_normal)."""
    with np.errstate(over="ignore"):
        key = splitmix64(np.uint64(seed) ^ splitmix64(np.uint64(uid)))
        n = np.asarray(n, dtype=np.uint64)
        a = splitmix64(key + np.uint64(2) * n)
        b = splitmix64(key + np.uint64(2) * n + np.uint64(1))
    u1 = ((a >> np.uint64(11)) + np.uint64(1)).astype(np.float64) * 2.0 ** -53
    u2 = (b >> np.uint64(11)).astype(np.float64) * 2.0 ** -53
    return np.sqrt(-2.0 * np.log(u1)) * np.cos(6.283185307179586 * u2)


def rotate_root_z(poses: np.ndarray, angle: float) -> np.ndarray:
    """data_amass.py:185-190 (scipy Rotation, float64) -> float32 pose rows."""
    from scipy.spatial import transform
    out = np.array(poses, dtype=np.float32, copy=True)
    org = transform.Rotation.from_rotvec(np.asarray(poses[:, :3], dtype=np.float64))
    aug = transform.Rotation.from_rotvec(np.array([0.0, 0.0, 1.0]) * angle)
    out[:, :3] = (aug * org).as_rotvec()
    return out


def convert_smplx(kps: np.ndarray, mappings: List[int]) -> np.ndarray:
    """data_amass.py:45-55"""
    out = np.zeros((kps.shape[0], len(mappings), kps.shape[2]), dtype=np.float32)
    for t, s in enumerate(mappings):
        out[:, t, :] = kps[:, s, :]
    return out


def noise_sigma(win: np.ndarray, kps_sigmas: np.ndarray) -> np.ndarray:
    """data_amass.py:69-76: the (17, 3) covariance diagonal of a window's keypoint noise."""
    sizes = np.max(win, axis=1) - np.min(win, axis=1)
    mean_size = np.mean(sizes, axis=0)
    return np.array([s * kps_sigmas * 0.003 for s in mean_size]).T


def getitem(joints: np.ndarray, poses: np.ndarray, betas: np.ndarray, local_idx: int, h: int, uid: int,
            relative: bool = True, add_noise: bool = True, seed: int = 0) -> Dict[str, np.ndarray]:
    """data_amass.py:125-154 for one sequence (joints (F,144,3) float32 from the FK)."""
    kp = sample_window(joints, local_idx, h)
    kp = convert_smplx(kp, SMPLX_TO_COCO)
    if relative:
        roots = 0.5 * (kp[:, 11, :] + kp[:, 12, :])
        kp = kp - roots[:, np.newaxis, :]
    if add_noise:
        sig = noise_sigma(kp, coco_kps_sigma())
        W = kp.shape[0]
        n = np.arange(W * 17 * 3).reshape(W, 17, 3)
        z = counter_normal(seed, uid, n)
        kp = kp + (np.sqrt(sig.astype(np.float64))[None] * z).astype(np.float32)
    ps = sample_window(poses, local_idx, h)
    return {"keypoints_3d": kp.astype(np.float32), "poses": ps[-1:, :66].astype(np.float32),
            "betas": np.asarray(betas, np.float32)}
