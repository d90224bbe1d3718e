"""Training-data generation on the GPU — drop-in for `AmassDataset`
(`mmskeleton/datasets/data_amass.py:87-218`), SURVEY.md §8f row 4 (the data
half of the training path).

Per epoch (`prepare_epoch_training_data` / `on_epoch_end`, :112-123) every
sequence is re-augmented and pushed through the SMPL-X FK (:176-218): the
root orientation is rotated about z by 2*pi*RandomState(epoch).rand()
(`tik_rotate_root_z`, float64 like scipy's Rotation), optionally a shape from
the shape DB replaces the betas (:192-208, the reference's own RNG calls), and
the FK joints of all frames (`tik_fk_forward`, joints only, no translation)
stay on the device, all sequences back to back. An item (:125-154) is the
edge-padded window of the COCO-17 keypoints (SMPL-X -> COCO gather), made
root-relative, with per-joint Gaussian noise, plus the target pose row;
`get_batch` builds any set of items in one launch (`tik_train_windows`).

Noise: the reference samples np.random.multivariate_normal from numpy's
global state; here the same distribution comes from a counter-based generator
keyed by (noise_seed, epoch, dataset index), so batches are reproducible and
independent of how items are grouped (the tests restate it on the CPU).
"""
from __future__ import annotations

import ctypes
from pathlib import Path
from typing import Dict, List, Optional

import numpy as np
import torch

from . import _lib

# keypoints_util.py:5-24 over smplx.joint_names.JOINT_NAMES (pinned by the golden
# mapping in tests/golden/keypoints.npz): COCO-17 <- SMPL-X FK joint index
SMPLX_TO_COCO = [55, 57, 56, 59, 58, 16, 17, 18, 19, 20, 21, 1, 2, 4, 5, 7, 8]


def coco_kps_sigma() -> np.ndarray:
    """data_amass.py:58-62"""
    return np.array([.26, .25, .25, .35, .35, .79, .79, .72, .72, .62, .62, 1.07, 1.07, .87, .87, .89, .89],
                    dtype=np.float32) * 0.1


def _load_sequence(p) -> Dict[str, object]:
    """An AMASS npz (poses, betas, gender[, trans]) or an in-memory dict."""
    if isinstance(p, dict):
        return dict(p)
    d = np.load(str(p), allow_pickle=False)
    out = {}
    for k in d.files:
        v = d[k]
        out[k] = v.item() if v.ndim == 0 else v
    return out


def rotate_root_z(poses: torch.Tensor, angle: float) -> torch.Tensor:
    """In place on device pose rows (F, >=3): root aa <- rotvec(R_z(angle) R(root))."""
    _lib.require_gpu(poses)
    if poses.dim() != 2 or poses.shape[1] < 3 or not poses.is_contiguous() or poses.dtype != torch.float32:
        raise ValueError("expected contiguous float32 (F, >=3) pose rows")
    _lib.check(_lib.load().tik_rotate_root_z(poses.data_ptr(), poses.shape[0], poses.shape[1], float(angle),
                                             _lib.stream_of(poses)), "rotate_root_z")
    return poses


def fk_joints(model, poses: torch.Tensor, betas: np.ndarray, apply_root_rot: bool = True) -> torch.Tensor:
    """smpl_util.py:22-82 with apply_trans=False, on device rows: (F, >=66) -> joints (F, J, 3)."""
    F = poses.shape[0]
    P = torch.zeros((F, 156), device=poses.device, dtype=torch.float32)
    w = min(156, poses.shape[1])
    P[:, :w] = poses[:, :w]
    full = torch.zeros((F, 55, 3), device=poses.device)
    if apply_root_rot:
        full[:, 0] = P[:, :3]
    full[:, 1:22] = P[:, 3:66].reshape(F, 21, 3)
    full[:, 25:40] = P[:, 66:111].reshape(F, 15, 3)
    full[:, 40:55] = P[:, 111:156].reshape(F, 15, 3)
    b = torch.from_numpy(np.asarray(betas, np.float32)[:model.num_betas][None]).to(poses.device)
    with torch.no_grad():
        joints, _ = model.full_forward(full, b.expand(F, -1).contiguous(), None, None, return_verts=False)
    return joints


class AmassDataset(torch.utils.data.Dataset):
    """data_amass.py:87-218. `amass_paths`: AMASS npz files or dicts with
    poses (F, >=66), betas, gender. Items are numpy dicts like the reference;
    `get_batch(indices)` returns device tensors for a whole batch."""

    def __init__(self, smplx_models, amass_paths: List, window_size: int, keypoint_format: str, device="cuda",
                 add_gaussian_noise=True, shape_db_path: Optional[Path] = None, aug_shape=True,
                 aug_root_orientation=True, noise_seed: int = 0):
        self.origin_amass_paths = amass_paths
        self.device = torch.device(device)
        self.smplx_models = smplx_models
        self.half_win_size = window_size // 2
        self.relative_pose = True
        self.add_gaussian_noise = add_gaussian_noise
        self.kps_noise_sigmas = coco_kps_sigma()
        self.aug_root_orientation = aug_root_orientation
        self.aug_shape = aug_shape
        self.noise_seed = int(noise_seed)
        self.epoch = 0
        self.smplx_shape_db = None
        if shape_db_path is not None:
            db = np.load(str(shape_db_path), allow_pickle=False)
            # (betas, gender) pairs: the reference's object array is stored here as two arrays
            self.smplx_shape_db = list(zip(db["betas"], [str(g) for g in db["genders"]]))
        if keypoint_format == "coco":
            self.target_kps_mapping = list(SMPLX_TO_COCO)
        else:
            raise ValueError("unsupported keypoint format")
        self.data_paths = []
        self.data_anims = []
        self.index_mappings = []
        self.prepare_epoch_training_data(0)

    # ---------------------------------------------------------------- epochs
    def prepare_epoch_training_data(self, epoch_idx):
        self.epoch = int(epoch_idx)
        self.data_anims = self.regenerate_data(epoch_idx)
        self.index_mappings = self.generate_index_file_mapping()
        self._pack()

    def on_epoch_end(self, epoch_idx):
        self.prepare_epoch_training_data(epoch_idx)

    def regenerate_data(self, random_seed) -> List[Dict[str, object]]:
        """data_amass.py:176-218 with the FK joints kept on the device."""
        data_s = []
        rand_stt = np.random.RandomState(seed=random_seed)
        shape_rand_stt = np.random.RandomState(seed=random_seed)
        for apath in self.origin_amass_paths:
            data = _load_sequence(apath)
            poses = torch.from_numpy(np.ascontiguousarray(np.asarray(data["poses"], np.float32))).to(self.device)
            if self.aug_root_orientation:
                aug_angle = 2.0 * np.pi * rand_stt.rand()
                rotate_root_z(poses, aug_angle)
            if self.aug_shape and self.smplx_shape_db is not None:
                shape_idx = int(shape_rand_stt.randint(0, len(self.smplx_shape_db), 1)[0])
                beta, gender = self.smplx_shape_db[shape_idx]
                gender = "female" if "female" in gender else ("male" if "male" in gender else "neutral")
                aug_beta = beta + 0.4 * np.random.rand() * beta   # the reference's global-RNG draw
                data["betas"] = np.asarray(aug_beta, np.float32)
                data["gender"] = gender
            data["betas"] = np.asarray(data["betas"], np.float32)
            model = self.smplx_models[str(data["gender"])]
            data["poses"] = poses
            data["keypoints_3d"] = fk_joints(model, poses, data["betas"], apply_root_rot=True)
            data_s.append(data)
        return data_s

    def count_samples(self):
        return sum(int(d["keypoints_3d"].shape[0]) for d in self.data_anims)

    def generate_index_file_mapping(self):
        """data_amass.py:163-174: item -> (sequence, first item of that sequence)."""
        mappings = []
        off = 0
        for i, d in enumerate(self.data_anims):
            n = int(d["poses"].shape[0])
            mappings += [(i, off)] * n
            off += n
        return mappings

    def _pack(self):
        """All sequences' joints / pose rows back to back on the device (one gather per batch)."""
        if not self.data_anims:
            self._joints = self._poses = None
            self._starts = np.zeros(0, np.int64)
            self._lens = np.zeros(0, np.int64)
            self._cum = np.zeros(0, np.int64)
            self._betas = None
            return
        lens = np.array([int(d["poses"].shape[0]) for d in self.data_anims], np.int64)
        pw = max(66, max(int(d["poses"].shape[1]) for d in self.data_anims))
        self._joints = torch.cat([d["keypoints_3d"] for d in self.data_anims], 0).contiguous()
        poses = torch.zeros((int(lens.sum()), pw), device=self.device, dtype=torch.float32)
        r = 0
        for d, n in zip(self.data_anims, lens):
            poses[r:r + n, :d["poses"].shape[1]] = d["poses"]
            r += n
        self._poses = poses
        self._starts = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.int64)
        self._lens = lens
        self._cum = np.cumsum(lens)
        self._betas = torch.from_numpy(np.stack([np.asarray(d["betas"], np.float32) for d in self.data_anims])).to(self.device)

    @property
    def noise_key(self) -> int:
        """The noise generator's seed for this epoch (train_data.hip counter_normal)."""
        return (self.noise_seed * 1000003 + self.epoch) & 0xFFFFFFFFFFFFFFFF

    # ---------------------------------------------------------------- items
    def __len__(self):
        return len(self.index_mappings)

    def _items(self, indices: np.ndarray):
        h = self.half_win_size
        indices = np.asarray(indices, np.int64)
        if indices.size and (indices.min() < 0 or indices.max() >= len(self)):
            raise IndexError("dataset index out of range")
        seq = np.searchsorted(self._cum, indices, side="right")
        local = indices - self._starts[seq]
        F = self._lens[seq]
        # sample_window's ValueError (data_amass.py:27-29) and its short window
        bad = (h > local) & (local > F - h)
        if bad.any():
            i = int(np.argmax(bad))
            raise ValueError(f"h_win_size > idx > arr.shape[0] - h_win_size: {h} > {local[i]} > {F[i]} - {h}")
        short = (local - h < 0) & (local + h > F - 1) & (local <= F - h)
        if short.any():
            raise ValueError(f"window at idx {int(local[np.argmax(short)])} overruns both ends of a "
                             f"{int(F[np.argmax(short)])}-frame sequence (the reference returns a short window)")
        return seq, local, F

    def get_batch(self, indices) -> Dict[str, torch.Tensor]:
        """Items `indices` at once: keypoints_3d (B, 2h+1, 17, 3), poses (B, 1, 66), betas (B, nb) on the device."""
        idx = np.asarray(indices, np.int64).reshape(-1)
        seq, local, F = self._items(idx)
        B, W = idx.size, 2 * self.half_win_size + 1
        win = torch.empty((B, W, 17, 3), device=self.device, dtype=torch.float32)
        tgt = torch.empty((B, 1, 66), device=self.device, dtype=torch.float32)
        if B:
            meta = torch.from_numpy(np.stack([self._starts[seq], F, local, idx, seq]).astype(np.int32)).to(self.device)
            cmap = (ctypes.c_int * 17)(*self.target_kps_mapping)
            sig = (ctypes.c_float * 17)(*[float(s) for s in self.kps_noise_sigmas])
            seed = self.noise_key
            _lib.check(_lib.load().tik_train_windows(
                self._joints.data_ptr(), self._joints.shape[1], self._poses.data_ptr(), self._poses.shape[1],
                meta[0].data_ptr(), meta[1].data_ptr(), meta[2].data_ptr(), meta[3].data_ptr(), B,
                self.half_win_size, ctypes.addressof(cmap), ctypes.addressof(sig), int(self.relative_pose),
                int(self.add_gaussian_noise), seed, win.data_ptr(), tgt.data_ptr(), _lib.stream_of(win)),
                "AmassDataset.get_batch")
        betas = (self._betas.index_select(0, meta[4].long()) if B
                 else torch.zeros((0, 10), device=self.device, dtype=torch.float32))
        return {"keypoints_3d": win, "poses": tgt, "betas": betas}

    def __getitem__(self, idx):
        b = self.get_batch([idx])
        return {"keypoints_3d": b["keypoints_3d"][0].cpu().numpy(), "poses": b["poses"][0].cpu().numpy(),
                "betas": b["betas"][0].cpu().numpy()}
