"""SMPL-X FK check — drop-in for `common/smpl_util.py` (`load_smplx_models`
:8-19, `run_smpl_inference` :22-82) and for the `smplx.SMPLX` model object
those functions drive (`smplx.create(model_type='smplx', use_pca=False,
use_face_contour=True, batch_size=...)`; `.forward(global_orient, body_pose,
betas, left_hand_pose, right_hand_pose, transl, ...)` -> `.joints`
(B,144,3), `.vertices` (B,10475,3); `.faces`, `.batch_size`).

All arithmetic runs in libtik.so (tik_fk_*): the kinematic chain (one wave
per body), the blend-shape GEMM and the skinning (bf16x3 split MFMA, fp32 range,
by default; exact fp32 MFMA with precision="fp32"), the landmark gather.
The fixed `batch_size` of smplx (which forces the reference to zero-pad
chunks, smpl_util.py:49-56) is kept as an attribute only: any batch runs.
Model files: SMPLX_{MALE,FEMALE,NEUTRAL}.npz (licensed, not shipped) are read
with numpy allow_pickle=False; `load_smplx_models(None|'synthetic', ...)`
builds the seeded synthetic SMPL-X-shaped constants instead.
"""
from __future__ import annotations

import os
from types import SimpleNamespace
from typing import Dict, Optional

import numpy as np
import torch

from . import _lib
from . import synthetic as syn

NUM_BETAS = 10
NUM_EXPR = 10


def constants_from_npz(path: str, num_betas: int = NUM_BETAS, num_expr: int = NUM_EXPR,
                       flat_hand_mean: bool = False) -> Dict[str, np.ndarray]:
    """SMPL-X model file -> the tensor set tik_fk_create takes (public smplx
    body_models SMPL/SMPLX.__init__ conventions, the loader smpl_util.py:13-18
    drives through smplx.create): posedirs (V,3,486) -> (486,3V), parents =
    kintree_table[0], hand mean pose when flat_hand_mean=False, and the shape
    and expression bases by the file's component count —
      * >= 400 components (SMPL-X v1.1: 300 shape + 100 expression):
        shapedirs[..., :min(num_betas, 300)], exprdirs = shapedirs[..., 300:300+min(num_expr, 100)];
      * fewer (the 20-component layout: 10 shape + 10 expression):
        shapedirs[..., :min(num_betas, 10)], exprdirs = shapedirs[..., 10:10+min(num_expr, 10)]."""
    d = np.load(path, allow_pickle=False)
    sd = d["shapedirs"]
    V = d["v_template"].shape[0]
    if sd.ndim != 3 or sd.shape[:2] != (V, 3):
        raise ValueError(f"shapedirs must be (V, 3, components), got {sd.shape}")
    if sd.shape[-1] < 400:   # 10 shape + 10 expression components (smplx: SHAPE_SPACE_DIM + EXPRESSION_SPACE_DIM)
        nb, e0, ne = min(num_betas, 10), 10, min(num_expr, 10)
    else:
        nb, e0, ne = min(num_betas, 300), 300, min(num_expr, 100)
    if sd.shape[-1] < e0 + ne:
        raise ValueError(f"shapedirs has {sd.shape[-1]} components: no expression basis at [{e0}, {e0 + ne})")
    c = {
        "v_template": d["v_template"].astype(np.float32),
        "shapedirs": sd[:, :, :nb].astype(np.float32),
        "exprdirs": sd[:, :, e0:e0 + ne].astype(np.float32),
        "posedirs": np.reshape(d["posedirs"], [-1, d["posedirs"].shape[-1]]).T.astype(np.float32),
        "J_regressor": d["J_regressor"].astype(np.float32),
        "lbs_weights": d["weights"].astype(np.float32),
        "faces": d["f"].astype(np.int32),
        "lmk_faces_idx": d["lmk_faces_idx"].astype(np.int32),
        "lmk_bary_coords": d["lmk_bary_coords"].astype(np.float32),
        "extra_verts": syn.SMPLX_EXTRA_VERTS.copy(),
    }
    par = d["kintree_table"][0].astype(np.int64)
    par[0] = -1
    c["parents"] = par.astype(np.int32)
    pm = np.zeros((55, 3), np.float32)
    if not flat_hand_mean:
        pm[25:40] = d["hands_meanl"].reshape(15, 3)
        pm[40:55] = d["hands_meanr"].reshape(15, 3)
    c["pose_mean"] = pm
    if "dynamic_lmk_faces_idx" in d.files:
        c["dynamic_lmk_faces_idx"] = d["dynamic_lmk_faces_idx"].astype(np.int32)
        c["dynamic_lmk_bary_coords"] = d["dynamic_lmk_bary_coords"].astype(np.float32)
    assert c["posedirs"].shape == (486, 3 * V)
    return c


class SMPLX:
    """The smplx.SMPLX object the reference drives (pose2rot, use_pca=False)."""

    NUM_BODY_JOINTS = 21

    def __init__(self, constants: Dict[str, np.ndarray], batch_size: int = 1, device="cuda",
                 use_face_contour: bool = True, gender: str = "neutral", precision: Optional[str] = None):
        self.batch_size = batch_size
        self.device = torch.device(device)
        self.gender = gender
        self.faces = constants["faces"].astype(np.int64)
        self.num_betas = constants["shapedirs"].shape[2]
        self.num_expression_coeffs = constants["exprdirs"].shape[2] if "exprdirs" in constants else 0
        lib = _lib.load()
        named = [(k, np.asarray(v, dtype=np.float32)) for k, v in constants.items()]
        arr, keep = _lib.pack_tensors(named)
        h = _lib.ctypes.c_void_p()
        _lib.check(lib.tik_fk_create(arr, len(named), int(use_face_contour), _lib.ctypes.byref(h)), "SMPLX")
        self._h = h.value
        self._destroy = lib.tik_fk_destroy
        if precision is not None:
            _lib.check(lib.tik_fk_set_precision(self._h, _lib.precision_code(precision)))
        # the GEMM arithmetic in use (library default bf16x3 unless TIK_PRECISION says otherwise)
        env = os.environ.get("TIK_PRECISION")
        self.precision = precision if precision is not None else ("fp32" if env in ("fp32", "f32") else "bf16x3")
        self.num_joints = _lib.check(lib.tik_fk_num_joints(self._h))
        self.num_verts = _lib.check(lib.tik_fk_num_verts(self._h))

    def __del__(self):
        try:
            if getattr(self, "_h", None):
                self._destroy(self._h)
        except Exception:
            pass

    def to(self, device):
        if torch.device(device).type != "cuda":
            raise RuntimeError("the SMPL-X FK runs on the GPU only (no CPU fallback)")
        return self

    def full_forward(self, full_pose: torch.Tensor, betas=None, expression=None, transl=None,
                     return_verts: bool = True, out=None):
        """full_pose (B,55,3) device -> (joints (B,J,3), vertices (B,V,3) or None).
        out: optional preallocated (joints, vertices) float32 tensors of those
        shapes to write into (a serving loop's output buffers; vertices may be None)."""
        fp = full_pose.reshape(-1, 55, 3).contiguous()
        B = fp.shape[0]
        args = [t.contiguous() if t is not None else None for t in (betas, expression, transl)]
        _lib.require_gpu(fp, *args)
        if out is not None:
            joints, verts = out
            if joints.shape != (B, self.num_joints, 3) or not joints.is_contiguous() or joints.dtype != torch.float32:
                raise ValueError("out joints must be a contiguous float32 (B, num_joints, 3) tensor")
            if return_verts and verts is None:
                raise ValueError("return_verts=True needs an out vertices tensor (out=(joints, verts))")
            if verts is not None and (verts.shape != (B, self.num_verts, 3) or not verts.is_contiguous()
                                      or verts.dtype != torch.float32):
                raise ValueError("out vertices must be a contiguous float32 (B, num_verts, 3) tensor")
            if not return_verts:
                verts = None
            _lib.require_gpu(joints, verts)
        else:
            joints = torch.empty((B, self.num_joints, 3), device=fp.device, dtype=torch.float32)
            verts = torch.empty((B, self.num_verts, 3), device=fp.device, dtype=torch.float32) if return_verts else None
        _lib.check(_lib.load().tik_fk_forward(self._h, fp.data_ptr(), _lib.ptr(args[0]), _lib.ptr(args[1]),
                                              _lib.ptr(args[2]), B, joints.data_ptr(), _lib.ptr(verts),
                                              _lib.stream_of(fp)), "SMPLX.forward")
        return joints, verts

    def __call__(self, global_orient=None, body_pose=None, betas=None, left_hand_pose=None, right_hand_pose=None,
                 transl=None, expression=None, jaw_pose=None, leye_pose=None, reye_pose=None, return_verts=True):
        ref = next(t for t in (body_pose, global_orient, left_hand_pose, right_hand_pose, betas) if t is not None)
        B = ref.shape[0]
        dev = ref.device

        def part(t, n):
            return torch.zeros((B, n * 3), device=dev) if t is None else t.reshape(B, n * 3).float()

        full = torch.cat([part(global_orient, 1), part(body_pose, 21), part(jaw_pose, 1), part(leye_pose, 1),
                          part(reye_pose, 1), part(left_hand_pose, 15), part(right_hand_pose, 15)], 1)
        j, v = self.full_forward(full, betas, expression, transl, return_verts)
        return SimpleNamespace(joints=j, vertices=v, full_pose=full)


def load_smplx_models(smplx_dir, device, batch_size):
    """smpl_util.py:8-19 -> {'male','female','neutral'} SMPLX objects."""
    out = {}
    for gender in ("male", "female", "neutral"):
        if smplx_dir in (None, "synthetic"):
            c = syn.synthetic_smplx_constants(seed={"male": 1, "female": 2, "neutral": 3}[gender])
        else:
            c = constants_from_npz(os.path.join(str(smplx_dir), f"SMPLX_{gender.upper()}.npz"))
        out[gender] = SMPLX(c, batch_size=batch_size, device=device, gender=gender)
    return out


def run_smpl_inference(data, smplx_models, device, apply_trans=True, apply_root_rot=True, apply_shape=True,
                       return_mesh=False):
    """smpl_util.py:22-82: poses (F,>=66) [+ trans, betas] -> joints (F,144,3) [, verts].

    All F frames go through one call (no fixed-size zero-padded chunks);
    pose columns past the array's width are treated as zero. The joints come
    back un-padded (smpl_util.py:72-74). The meshes keep the reference's
    padding: it appends every chunk's body.vertices without the [:org_bsize]
    slice (smpl_util.py:76-77), so it returns ceil(F / batch_size) *
    batch_size meshes, the extra ones the bodies of all-zero inputs; here
    those rows are solved from zero inputs too. Pinned by
    tests/test_smpl_orchestration.py against the reference's own function."""
    model = smplx_models[str(data["gender"])]
    poses = np.asarray(data["poses"], dtype=np.float32)
    F = poses.shape[0]
    bs = max(1, int(getattr(model, "batch_size", 1) or 1))
    R = F + ((-F) % bs if return_mesh else 0)   # rows solved: + the reference's mesh padding
    if poses.shape[1] < 156:
        poses = np.concatenate([poses, np.zeros((F, 156 - poses.shape[1]), np.float32)], 1)
    P = torch.zeros((R, 156), device=device)
    P[:F] = torch.from_numpy(np.ascontiguousarray(poses[:, :156])).to(device)
    full = torch.zeros((R, 55, 3), device=device)
    if apply_root_rot:
        full[:, 0] = P[:, :3]
    full[:, 1:22] = P[:, 3:66].reshape(R, 21, 3)
    full[:, 25:40] = P[:, 66:111].reshape(R, 15, 3)
    full[:, 40:55] = P[:, 111:156].reshape(R, 15, 3)
    trans = None
    if apply_trans:
        trans = torch.zeros((R, 3), device=device)
        trans[:F] = torch.from_numpy(np.asarray(data["trans"], np.float32)).to(device)
    betas = None
    if apply_shape:
        b = np.asarray(data["betas"], np.float32)[:model.num_betas][None]
        betas = torch.zeros((R, b.shape[1]), device=device)
        betas[:F] = torch.from_numpy(np.tile(b, (F, 1))).to(device)
    with torch.no_grad():
        joints, verts = model.full_forward(full, betas, None, trans, return_verts=return_mesh)
    j = joints[:F].cpu().numpy()
    if return_mesh:
        return j, verts.cpu().numpy()
    return j
