"""ORACLE — CPU restatement of SMPL-X forward kinematics + LBS. TEST INFRASTRUCTURE ONLY.

The reference calls the third-party `smplx` package (vchoutas/smplx) at
common/smpl_util.py:13-18 (smplx.create(model_type='smplx', use_pca=False,
use_face_contour=True, batch_size=...)) and :67-69 (SMPLX.forward). smplx is
not vendored in /root/reference, not installed here, and its version is not
pinned (README.md:14 names a requirements.txt that does not exist), so this
restates its published algorithm (smplx/lbs.py: lbs, blend_shapes,
vertices2joints, batch_rodrigues, batch_rigid_transform, vertices2landmarks,
find_dynamic_lmk_idx_and_bcoords, rot_mat_to_euler; smplx/body_models.py:
SMPLX.forward, VertexJointSelector) in numpy float64.

PARITY UNPINNED for everything past the rotation step: no reference test,
fixture or model file pins the kinematic chain, LBS or landmarks (SURVEY.md
§8c). The axis-angle -> rotation step is pinned: smplx's batch_rodrigues
agrees with the reference's kornia copy (golden kornia.npz) to ~1.5e-6.
"""
from __future__ import annotations

from typing import Dict, Optional

import numpy as np

NECK_IDX = 12


def batch_rodrigues(rot_vecs):
    """smplx lbs.batch_rodrigues: angle = ||v + 1e-8||, K skew of v/angle,
    R = I + sin K + (1 - cos) K^2."""
    v = np.asarray(rot_vecs, dtype=np.float64).reshape(-1, 3)
    angle = np.linalg.norm(v + 1e-8, axis=1, keepdims=True)
    d = v / angle
    c, s = np.cos(angle)[:, :, None], np.sin(angle)[:, :, None]
    rx, ry, rz = d[:, 0], d[:, 1], d[:, 2]
    z = np.zeros_like(rx)
    K = np.stack([z, -rz, ry, rz, z, -rx, -ry, rx, z], 1).reshape(-1, 3, 3)
    return np.eye(3)[None] + s * K + (1 - c) * (K @ K)


def rot_mat_to_euler(R):
    sy = np.sqrt(R[:, 0, 0] ** 2 + R[:, 1, 0] ** 2)
    return np.arctan2(-R[:, 2, 0], sy)


def neck_kin_chain(parents):
    chain, i = [], NECK_IDX
    while i != -1:
        chain.append(i)
        i = int(parents[i])
    return chain


def smplx_forward(c: Dict[str, np.ndarray], full_pose, betas=None, expression=None, transl=None,
                  return_verts=True):
    """SMPLX.forward for pose2rot, use_pca=False, use_face_contour=True.

    c: constants (synthetic.synthetic_smplx_constants layout, plus optional
    'pose_mean' (55,3), 'dynamic_lmk_faces_idx' (79,17), 'dynamic_lmk_bary_coords' (79,17,3)).
    full_pose: (B,55,3) [global, 21 body, jaw, leye, reye, 15 lhand, 15 rhand].
    Returns joints (B, 55+21+51[+17], 3) and vertices (B,V,3).
    """
    pose = np.asarray(full_pose, dtype=np.float64).reshape(-1, 55, 3)
    B = pose.shape[0]
    if "pose_mean" in c:
        pose = pose + c["pose_mean"].astype(np.float64).reshape(1, 55, 3)
    nb = c["shapedirs"].shape[2]
    ne = c["exprdirs"].shape[2]
    beta = np.zeros((B, nb)) if betas is None else np.asarray(betas, np.float64)
    expr = np.zeros((B, ne)) if expression is None else np.asarray(expression, np.float64)
    shape_components = np.concatenate([beta, expr], 1)
    shapedirs = np.concatenate([c["shapedirs"], c["exprdirs"]], 2).astype(np.float64)
    # lbs()
    v_shaped = c["v_template"].astype(np.float64)[None] + np.einsum("bl,mkl->bmk", shape_components, shapedirs)
    J = np.einsum("bik,ji->bjk", v_shaped, c["J_regressor"].astype(np.float64))
    R = batch_rodrigues(pose.reshape(-1, 3)).reshape(B, 55, 3, 3)
    pose_feature = (R[:, 1:] - np.eye(3)).reshape(B, -1)
    v_posed = v_shaped + (pose_feature @ c["posedirs"].astype(np.float64)).reshape(B, -1, 3)
    parents = c["parents"].astype(np.int64)
    rel = J.copy()
    rel[:, 1:] -= J[:, parents[1:]]
    T = np.zeros((B, 55, 4, 4))
    T[:, :, :3, :3] = R
    T[:, :, :3, 3] = rel
    T[:, :, 3, 3] = 1.0
    G = np.zeros_like(T)
    G[:, 0] = T[:, 0]
    for i in range(1, 55):
        G[:, i] = G[:, parents[i]] @ T[:, i]
    posed_joints = G[:, :, :3, 3].copy()
    A = G.copy()
    A[:, :, :3, 3] -= np.einsum("bjkl,bjl->bjk", G[:, :, :3, :3], J)
    W = c["lbs_weights"].astype(np.float64)
    Tv = np.einsum("vj,bjkl->bvkl", W, A)
    verts = np.einsum("bvkl,bvl->bvk", Tv[:, :, :3, :3], v_posed) + Tv[:, :, :3, 3]
    # landmarks (vertices2landmarks)
    faces = c["faces"].astype(np.int64)
    lf = np.broadcast_to(c["lmk_faces_idx"].astype(np.int64), (B, len(c["lmk_faces_idx"])))
    lb = np.broadcast_to(c["lmk_bary_coords"].astype(np.float64), (B,) + c["lmk_bary_coords"].shape)
    if "dynamic_lmk_faces_idx" in c:
        chain = neck_kin_chain(parents)
        rel_rot = np.broadcast_to(np.eye(3), (B, 3, 3)).copy()
        for j in chain:
            rel_rot = R[:, j] @ rel_rot
        y = np.round(np.minimum(-rot_mat_to_euler(rel_rot) * 180.0 / np.pi, 39)).astype(np.int64)
        neg = (y < 0).astype(np.int64)
        mask = (y < -39).astype(np.int64)
        negv = mask * 78 + (1 - mask) * (39 - y)
        y = neg * negv + (1 - neg) * y
        lf = np.concatenate([lf, c["dynamic_lmk_faces_idx"].astype(np.int64)[y]], 1)
        lb = np.concatenate([lb, c["dynamic_lmk_bary_coords"].astype(np.float64)[y]], 1)
    tri = verts[np.arange(B)[:, None, None], faces[lf]]            # (B, L, 3 verts, 3)
    landmarks = np.einsum("blfi,blf->bli", tri, lb)
    extra = verts[:, c["extra_verts"].astype(np.int64)]
    joints = np.concatenate([posed_joints, extra, landmarks], 1)
    if transl is not None:
        t = np.asarray(transl, np.float64)[:, None, :]
        joints = joints + t
        verts = verts + t
    return (joints, verts) if return_verts else joints
