"""Deterministic synthetic weights, windows and SMPL-X-shaped constants.

The reference's trained checkpoint (`data/models/checkpoint_epoch=98.ckpt`) and
the SMPL-X model files are not available (`/root/reference/.MISSING_LARGE_BLOBS:2`,
`common/smpl_util.py:9-11`), so every parity test and benchmark runs on weights
drawn from a counter-based PRNG that is re-implemented here and in the golden
fixture generator: the 12.7 MB weight blob never has to be committed.

PRNG: splitmix64 over a per-tensor 64-bit key (FNV-1a of the tensor name xor a
seed), element i uses counter ``key + (i+1) * 0x9E3779B97F4A7C15``; the top 53
bits give a double in [0, 1).

Weight naming follows the reference state dict of ``PoseRegressor``
(`pose_trainer.py:66-92`, `st_gcn_aaai18.py:52-111,161-206`) — that key list
is the weight ABI the C library consumes (`include/tik.h`).
"""
from __future__ import annotations

import hashlib
import os
from dataclasses import dataclass, field
from typing import Dict, List, Tuple

import numpy as np

_MASK = np.uint64(0xFFFFFFFFFFFFFFFF)
_GOLDEN = np.uint64(0x9E3779B97F4A7C15)


def _fnv1a64(text: str) -> int:
    h = 0xCBF29CE484222325
    for b in text.encode("utf-8"):
        h ^= b
        h = (h * 0x100000001B3) & 0xFFFFFFFFFFFFFFFF
    return h


def splitmix_uniform(key: str, n: int, seed: int = 0) -> np.ndarray:
    """n doubles in [0,1) from splitmix64, keyed by (key, seed)."""
    base = np.uint64((_fnv1a64(key) ^ (seed * 0xD1B54A32D192ED03)) & 0xFFFFFFFFFFFFFFFF)
    with np.errstate(over="ignore"):
        ctr = np.arange(1, n + 1, dtype=np.uint64)
        z = base + ctr * _GOLDEN
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return (z >> np.uint64(11)).astype(np.float64) * (1.0 / 9007199254740992.0)


def uniform(key: str, shape, lo: float, hi: float, seed: int = 0) -> np.ndarray:
    n = int(np.prod(shape)) if len(shape) else 1
    u = splitmix_uniform(key, n, seed)
    return (lo + (hi - lo) * u).reshape(shape).astype(np.float32)


# --------------------------------------------------------------------------
# Architecture of the reference IK model (pose_trainer.py:76-92)
# --------------------------------------------------------------------------
# (in_channels, out_channels, temporal_stride); all layers is_residual=True.
IK_LAYERS: List[Tuple[int, int, int]] = [
    (3, 64, 1), (64, 64, 1), (64, 128, 2), (128, 128, 1),
    (128, 128, 1), (128, 128, 2), (128, 256, 2), (256, 256, 2),
]
TEMPORAL_KERNEL = 3          # pose_trainer.py:85
POSE_DIM = 22 * 3            # pose_trainer.py:88
HIDDEN = 512                 # pose_trainer.py:89
NUM_JOINTS = 17              # COCO layout, graph.py:76-85


def residual_kind(cin: int, cout: int, stride: int, residual: bool = True) -> str:
    """'zero' | 'iden' | 'conv', as chosen at st_gcn_aaai18.py:191-204."""
    if not residual:
        return "zero"
    if cin == cout and stride == 1:
        return "iden"
    return "conv"


def out_frames(T: int, layers=IK_LAYERS, kt: int = TEMPORAL_KERNEL) -> int:
    """Temporal length after the backbone (conv (kt,1), stride s, pad (kt-1)/2)."""
    pad = (kt - 1) // 2
    for _, _, s in layers:
        T = (T + 2 * pad - kt) // s + 1
    return T


@dataclass
class HParams:
    """The hparams the reference model reads (pose_trainer.py:204-230)."""
    win_size: int = 9
    kps_channel: int = 3
    graph_layout: str = "coco"
    max_hop: int = 2
    dilation: int = 1
    n_out_joints: int = 22
    n_out_channels: int = 3
    extra: Dict = field(default_factory=dict)


def _bn_params(prefix: str, c: int, seed: int) -> Dict[str, np.ndarray]:
    return {
        prefix + ".weight": uniform(prefix + ".weight", (c,), 0.8, 1.2, seed),
        prefix + ".bias": uniform(prefix + ".bias", (c,), -0.1, 0.1, seed),
        prefix + ".running_mean": uniform(prefix + ".running_mean", (c,), -0.1, 0.1, seed),
        prefix + ".running_var": uniform(prefix + ".running_var", (c,), 0.5, 1.5, seed),
    }


def _conv_params(prefix: str, cout: int, cin: int, kt: int, seed: int) -> Dict[str, np.ndarray]:
    bound = np.sqrt(3.0 / (cin * kt))   # LeCun-uniform: keeps activations O(1)
    return {
        prefix + ".weight": uniform(prefix + ".weight", (cout, cin, kt, 1), -bound, bound, seed),
        prefix + ".bias": uniform(prefix + ".bias", (cout,), -bound, bound, seed),
    }


def block_state_dict(prefix: str, cin: int, cout: int, stride: int, kt: int = TEMPORAL_KERNEL,
                     K: int = 1, residual: bool = True, seed: int = 0) -> Dict[str, np.ndarray]:
    """State dict of one StGcnBlock (st_gcn_aaai18.py:161-206) under `prefix`."""
    sd: Dict[str, np.ndarray] = {}
    sd.update(_conv_params(prefix + "gcn.conv", cout * K, cin, 1, seed))
    sd.update(_bn_params(prefix + "tcn.0", cout, seed))
    sd.update(_conv_params(prefix + "tcn.2", cout, cout, kt, seed))
    sd.update(_bn_params(prefix + "tcn.3", cout, seed))
    if residual_kind(cin, cout, stride, residual) == "conv":
        sd.update(_conv_params(prefix + "residual.0", cout, cin, 1, seed))
        sd.update(_bn_params(prefix + "residual.1", cout, seed))
    return sd


def ik_state_dict(A: np.ndarray, seed: int = 0, layers=IK_LAYERS) -> Dict[str, np.ndarray]:
    """Full PoseRegressor state dict (keys without the PL `regressor.` prefix).

    A: (K, V, V) graph adjacency (the `backbone.A` buffer, st_gcn_aaai18.py:61-65).
    """
    K, V, _ = A.shape
    sd: Dict[str, np.ndarray] = {"backbone.A": A.astype(np.float32)}
    sd.update(_bn_params("backbone.data_bn", layers[0][0] * V, seed))
    for l, (cin, cout, s) in enumerate(layers):
        sd.update(block_state_dict(f"backbone.st_gcn_networks.{l}.", cin, cout, s, K=K, seed=seed))
        sd[f"backbone.edge_importance.{l}"] = uniform(f"backbone.edge_importance.{l}", (K, V, V), 0.5, 1.5, seed)
    feat = V * layers[-1][1]
    b0 = np.sqrt(3.0 / feat)
    sd["pose_regressor.0.weight"] = uniform("pose_regressor.0.weight", (HIDDEN, feat), -b0, b0, seed)
    sd["pose_regressor.0.bias"] = uniform("pose_regressor.0.bias", (HIDDEN,), -b0, b0, seed)
    b3 = np.sqrt(6.0 / HIDDEN)
    sd["pose_regressor.3.weight"] = uniform("pose_regressor.3.weight", (POSE_DIM, HIDDEN), -b3, b3, seed)
    sd["pose_regressor.3.bias"] = uniform("pose_regressor.3.bias", (POSE_DIM,), -b3, b3, seed)
    return sd


def state_dict_sha256(sd: Dict[str, np.ndarray]) -> str:
    h = hashlib.sha256()
    for k in sorted(sd):
        h.update(k.encode())
        h.update(np.ascontiguousarray(sd[k], dtype=np.float32).tobytes())
    return h.hexdigest()


# --------------------------------------------------------------------------
# Synthetic AMASS-shaped windows
# --------------------------------------------------------------------------
_DATA_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "data")
SAMPLE_COCO_PATH = os.path.join(_DATA_DIR, "dance_contemporary_coco.npy")


def load_sample_coco() -> np.ndarray:
    """The reference's sample sequence converted to COCO-17, (231,17,3) f32.

    Produced by `tests/golden/make_golden.py` with the reference's own
    moveai→COCO conversion (`inference.py:121-133`).
    """
    return np.load(SAMPLE_COCO_PATH, allow_pickle=False)


def synthetic_windows(B: int, T: int, seed: int = 0, start: int = 0,
                      seq: np.ndarray | None = None, noise: float = 0.01) -> np.ndarray:
    """B windows (B,T,17,3) f32: random T-frame crops of the sample sequence
    (edge-padded), a random rotation about the vertical (z) axis
    (mirrors data_amass.py:184-190), N(0, noise) jitter, root-relative per frame
    (data_amass.py:232-235). Window b uses generator (seed, start+b) so any
    contiguous shard [start, start+B) of a global batch is reproducible alone.
    """
    if seq is None:
        seq = load_sample_coco()
    F = seq.shape[0]
    out = np.empty((B, T, seq.shape[1], 3), dtype=np.float32)
    for b in range(B):
        rng = np.random.default_rng([seed, start + b])
        c = int(rng.integers(-(T // 2), F - T // 2))
        idx = np.clip(np.arange(c, c + T), 0, F - 1)
        w = seq[idx].astype(np.float64)
        ang = rng.uniform(0.0, 2.0 * np.pi)
        ca, sa = np.cos(ang), np.sin(ang)
        R = np.array([[ca, -sa, 0.0], [sa, ca, 0.0], [0.0, 0.0, 1.0]])
        w = w @ R.T + rng.normal(0.0, noise, size=w.shape)
        root = 0.5 * (w[:, 11] + w[:, 12])
        out[b] = (w - root[:, None, :]).astype(np.float32)
    return out


# --------------------------------------------------------------------------
# Synthetic SMPL-X-shaped constants
# --------------------------------------------------------------------------
SMPLX_PARENTS = np.array(
    [-1, 0, 0, 0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 9, 9, 12, 13, 14, 16, 17, 18, 19, 15, 15, 15,
     20, 25, 26, 20, 28, 29, 20, 31, 32, 20, 34, 35, 20, 37, 38, 21, 40, 41, 21, 43, 44,
     21, 46, 47, 21, 49, 50, 21, 52, 53], dtype=np.int32)
SMPLX_NUM_JOINTS = 55
SMPLX_NUM_VERTS = 10475
SMPLX_NUM_BETAS = 10
SMPLX_NUM_EXPR = 10
# 21 vertex-picked joints (nose, r/l eye, r/l ear, feet, fingertips); the
# first five ids are the public smplx vertex_ids['smplx'] values.
SMPLX_EXTRA_VERTS = np.array(
    [9120, 9929, 9448, 616, 6, 5770, 5780, 8846, 8463, 8474, 8635, 5361, 4933, 5058, 5169,
     5286, 8079, 7669, 7794, 7905, 8022], dtype=np.int32)
SMPLX_NUM_LMK = 51


def synthetic_smplx_constants(seed: int = 1, num_verts: int = SMPLX_NUM_VERTS,
                              num_faces: int = 20908) -> Dict[str, np.ndarray]:
    """SMPL-X-shaped constants drawn from numpy PCG64(seed).

    Shapes follow the public SMPL-X model files: v_template (V,3), shapedirs
    (V,3,10), exprdirs (V,3,10), posedirs (486, V*3) [smplx stores it
    transposed to (P, V*3) at load time], J_regressor (55,V) non-negative with
    rows summing to 1, lbs_weights (V,55) softmax rows with <=4 dominant joints,
    faces (F,3), landmark faces/barycentrics for the 51 static face landmarks,
    the dynamic-contour tables (79 bins x 17) and the flat_hand_mean=False
    pose mean (55,3).
    """
    rng = np.random.default_rng(seed)
    V, J = num_verts, SMPLX_NUM_JOINTS
    c: Dict[str, np.ndarray] = {}
    c["v_template"] = rng.normal(0.0, 0.3, (V, 3)).astype(np.float32)
    c["shapedirs"] = rng.normal(0.0, 0.01, (V, 3, SMPLX_NUM_BETAS)).astype(np.float32)
    c["exprdirs"] = rng.normal(0.0, 0.01, (V, 3, SMPLX_NUM_EXPR)).astype(np.float32)
    c["posedirs"] = rng.normal(0.0, 0.001, ((J - 1) * 9, V * 3)).astype(np.float32)
    jr = np.zeros((J, V), dtype=np.float64)
    for j in range(J):
        idx = rng.choice(V, size=20, replace=False)
        jr[j, idx] = rng.uniform(0.1, 1.0, 20)
    jr /= jr.sum(axis=1, keepdims=True)
    c["J_regressor"] = jr.astype(np.float32)
    logits = rng.normal(0.0, 1.0, (V, J))
    top = np.argsort(-logits, axis=1)[:, :4]
    w = np.full((V, J), -30.0)
    np.put_along_axis(w, top, np.take_along_axis(logits, top, axis=1) * 2.0, axis=1)
    w = np.exp(w - w.max(axis=1, keepdims=True))
    c["lbs_weights"] = (w / w.sum(axis=1, keepdims=True)).astype(np.float32)
    c["faces"] = rng.integers(0, V, (num_faces, 3)).astype(np.int32)
    c["lmk_faces_idx"] = rng.integers(0, num_faces, (SMPLX_NUM_LMK,)).astype(np.int32)
    bc = rng.uniform(0.05, 1.0, (SMPLX_NUM_LMK, 3))
    c["lmk_bary_coords"] = (bc / bc.sum(axis=1, keepdims=True)).astype(np.float32)
    c["parents"] = SMPLX_PARENTS.copy()
    c["extra_verts"] = np.minimum(SMPLX_EXTRA_VERTS, V - 1).astype(np.int32)
    # flat_hand_mean=False: the hand mean pose is added to the hand joints
    pm = np.zeros((SMPLX_NUM_JOINTS, 3))
    pm[25:] = rng.normal(0.0, 0.2, (30, 3))
    c["pose_mean"] = pm.astype(np.float32)
    # 17 dynamic face-contour landmarks, one (face, barycentric) set per
    # y-rotation bin (79 bins: 0..39 and the negative-angle bins 40..78)
    c["dynamic_lmk_faces_idx"] = rng.integers(0, num_faces, (79, 17)).astype(np.int32)
    db = rng.uniform(0.05, 1.0, (79, 17, 3))
    c["dynamic_lmk_bary_coords"] = (db / db.sum(axis=2, keepdims=True)).astype(np.float32)
    return c


def synthetic_fk_inputs(B: int, seed: int = 1) -> Tuple[np.ndarray, np.ndarray]:
    """full_pose (B,55,3) ~ N(0,0.3) with a uniform-sphere*pi global orient,
    betas (B,10) ~ N(0,1)."""
    rng = np.random.default_rng([seed, 7])
    pose = rng.normal(0.0, 0.3, (B, SMPLX_NUM_JOINTS, 3))
    d = rng.normal(size=(B, 3))
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    pose[:, 0] = d * rng.uniform(0.0, np.pi, (B, 1))
    betas = rng.normal(0.0, 1.0, (B, SMPLX_NUM_BETAS))
    return pose.astype(np.float32), betas.astype(np.float32)
