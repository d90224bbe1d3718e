"""Pin run_smpl_inference's ORCHESTRATION to the reference.

Runs only in the build container, where /root/reference is mounted read-only:
    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_smpl.py

It imports the reference's own common/smpl_util.py (run_smpl_inference,
smpl_util.py:22-82) with `smplx` replaced by a RECORDING stub: `create()`
returns a model object with the fixed `batch_size` smplx has, which records
the keyword arguments of every call (global_orient, body_pose, betas,
left/right_hand_pose, transl; None recorded as smplx's zero default) and
returns joints / vertices as a fixed linear function of them (float64
weights, no smplx arithmetic: the FK itself is pinned elsewhere, as far as it
can be without smplx). Cases: F = 20 frames with batch_size 9 (two full
chunks and a zero-padded one of 2 frames) and F = 18 (an exact multiple)
under every apply_trans / apply_root_rot / apply_shape / return_mesh
combination, on a neutral body with 16 betas in the data (the reference
keeps [:10]).

Output tests/golden/smpl_orchestration.npz (numpy arrays only):
  inputs   poses (20,156), trans (20,3), betas (16,)
  per case "<F>|<t><r><s><m>|...":
    call_rows   rows of every smplx call (the padded batch size, 9)
    args        the recorded per-row arguments of all calls, concatenated
                (169 = 3 global + 63 body + 45 lhand + 45 rhand + 10 betas + 3 transl)
    joints      run_smpl_inference's return (F, 8, 3) [verts (F, 5, 3) when m]
  W_joints (169, 24), W_verts (169, 15): the stub's linear maps
"""
import os
import sys
import types

import numpy as np

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
NJ_OUT, NV_OUT = 8, 5   # the stub's joint / vertex counts (smplx: 144 / 10475)


def stub_weights():
    rng = np.random.default_rng(2024)
    return rng.normal(0, 1, (169, NJ_OUT * 3)), rng.normal(0, 1, (169, NV_OUT * 3))


def args_vector(B, global_orient, body_pose, betas, lhand, rhand, transl):
    """(B,169) float64: the per-row arguments, None -> smplx's zero default."""
    def part(t, n):
        return np.zeros((B, n)) if t is None else np.asarray(t, np.float64).reshape(B, n)
    return np.concatenate([part(global_orient, 3), part(body_pose, 63), part(lhand, 45), part(rhand, 45),
                           part(betas, 10), part(transl, 3)], 1)


def main():
    import torch

    calls = []
    Wj, Wv = stub_weights()

    class RecordingSMPLX:
        def __init__(self, batch_size):
            self.batch_size = batch_size

        def to(self, device):
            return self

        def __call__(self, global_orient=None, body_pose=None, betas=None, left_hand_pose=None,
                     right_hand_pose=None, transl=None, **kw):
            assert not kw, kw
            B = self.batch_size
            np_ = lambda t: None if t is None else t.detach().cpu().numpy()
            a = args_vector(B, np_(global_orient), np_(body_pose), np_(betas), np_(left_hand_pose),
                            np_(right_hand_pose), np_(transl))
            calls.append(a)
            return types.SimpleNamespace(joints=torch.from_numpy((a @ Wj).reshape(B, NJ_OUT, 3).astype(np.float32)),
                                         vertices=torch.from_numpy((a @ Wv).reshape(B, NV_OUT, 3).astype(np.float32)))

    smplx = types.ModuleType("smplx")
    smplx.create = lambda **kw: RecordingSMPLX(kw["batch_size"])
    sys.modules["smplx"] = smplx
    sys.path.insert(0, REF)
    from common import smpl_util   # the reference module itself

    rng = np.random.default_rng(7)
    poses = rng.normal(0, 0.4, (20, 156)).astype(np.float32)
    trans = rng.normal(0, 1.0, (20, 3)).astype(np.float32)
    betas = rng.normal(0, 1.0, (16,)).astype(np.float32)
    out = {"poses": poses, "trans": trans, "betas": betas, "W_joints": Wj, "W_verts": Wv}
    models = smpl_util.load_smplx_models("unused", "cpu", batch_size=9)
    for F in (20, 18):
        data = {"gender": "neutral", "poses": poses[:F], "trans": trans[:F], "betas": betas}
        for t in (0, 1):
            for r in (0, 1):
                for s in (0, 1):
                    for m in (0, 1):
                        calls.clear()
                        res = smpl_util.run_smpl_inference(data, models, "cpu", apply_trans=bool(t),
                                                           apply_root_rot=bool(r), apply_shape=bool(s),
                                                           return_mesh=bool(m))
                        key = f"{F}|{t}{r}{s}{m}|"
                        out[key + "call_rows"] = np.array([c.shape[0] for c in calls], np.int32)
                        out[key + "args"] = np.concatenate(calls, 0).astype(np.float32)   # exact: float32 inputs
                        if m:
                            out[key + "joints"], out[key + "verts"] = res
                        else:
                            out[key + "joints"] = res
    np.savez_compressed(os.path.join(HERE, "smpl_orchestration.npz"), **out)
    print("wrote", os.path.join(HERE, "smpl_orchestration.npz"), len(out), "arrays")


if __name__ == "__main__":
    main()
