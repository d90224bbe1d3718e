"""Entry point — drop-in for `inference.py` (`run_inference` :37-67, `run_test`
:110-149). Windows are gathered on the GPU (tik_window_gather) and the whole
sequence is solved in large batches by the fused HIP forward; like the
reference, each window's output frame 0 is the solution for frame idx
(inference.py:58-66, h_w_size = 0).

CLI (README.md:24-26):
    python -m temporal_inverse_kinematics_amd.inference <moveai_3d.npz> [SMPLX_DIR]
        [--ckpt model.ckpt] [--win-size 64] [--out poses.npy]
Without --ckpt the seeded synthetic weights are used (the trained checkpoint
is not distributed with the reference: .MISSING_LARGE_BLOBS:2).
"""
from __future__ import annotations

import argparse
import sys

import numpy as np
import torch

from . import keypoints as kp
from .windowing import gather_windows

MAX_WINDOWS_PER_CALL = 8192


def run_inference(model, seq_3d_kps: np.ndarray) -> np.ndarray:
    """(F,17,3) keypoints -> (F,66) f32 SMPL-X body pose (inference.py:37-67)."""
    win = model.hparams.win_size
    dev = model.device
    if isinstance(seq_3d_kps, torch.Tensor):
        seq = seq_3d_kps.to(dev, torch.float32).contiguous()
    else:
        seq = torch.as_tensor(np.ascontiguousarray(seq_3d_kps, dtype=np.float32), device=dev)
    F = seq.shape[0]
    out = np.empty((F, 66), dtype=np.float32)
    with torch.no_grad():
        for s in range(0, F, MAX_WINDOWS_PER_CALL):
            n = min(MAX_WINDOWS_PER_CALL, F - s)
            windows = gather_windows(seq, win, idx0=s, n=n, relative_pose=True)
            poses = model(windows)["poses"]
            out[s:s + n] = poses[:, 0].float().cpu().numpy()
    return out


def synthetic_model(win_size: int = 64, device="cuda", seed: int = 0, precision=None):
    """IKPoseTrainer with the seeded synthetic weights of synthetic.ik_state_dict."""
    from . import synthetic as syn
    from .models import IKPoseTrainer, default_hparams
    model = IKPoseTrainer(default_hparams(win_size))
    sd = syn.ik_state_dict(model.regressor.backbone.graph.A, seed=seed)
    model.regressor.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()}, strict=False)
    model.regressor.tik_precision = precision
    return model.to(device).eval()


def run_test(npz_path: str, smplx_dir: str | None = None, ckpt: str | None = None, win_size: int = 64,
             device="cuda"):
    """inference.run_test:110-145: moveai npz -> COCO -> IK -> (optional) SMPL-X FK."""
    d = np.load(npz_path, allow_pickle=False)
    # the moveai_3d -> COCO conversion on the device (one gather kernel, bit-identical to the host form)
    seq = kp.moveai3d_to_coco_device(torch.as_tensor(np.ascontiguousarray(d["joints_3d"], dtype=np.float32),
                                                     device=device), d["joint_3d_names"].tolist())
    if ckpt:
        from .models import IKPoseTrainer
        model = IKPoseTrainer.load_from_checkpoint(ckpt).to(device).eval()
    else:
        model = synthetic_model(win_size, device)
    poses = run_inference(model, seq)
    result = {"coco": seq.cpu().numpy(), "poses": poses}
    if smplx_dir:
        from .smplx_fk import load_smplx_models, run_smpl_inference
        models = load_smplx_models(smplx_dir, device, 9)
        sample = np.zeros((poses.shape[0], 156), dtype=np.float32)
        sample[:, :66] = poses
        joints, verts = run_smpl_inference({"poses": sample, "gender": "male"}, models, device,
                                           apply_trans=False, apply_shape=False, return_mesh=True)
        result.update(joints=joints, vertices=verts)
    return result


def main(argv=None):
    p = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    p.add_argument("npz")
    p.add_argument("smplx_dir", nargs="?")
    p.add_argument("--ckpt")
    p.add_argument("--win-size", type=int, default=64)
    p.add_argument("--out")
    a = p.parse_args(argv)
    r = run_test(a.npz, a.smplx_dir, a.ckpt, a.win_size)
    if a.out:
        np.save(a.out, r["poses"])
    print(f"solved {r['poses'].shape[0]} frames -> poses {r['poses'].shape}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
