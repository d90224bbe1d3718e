"""Generate the golden fixtures under tests/golden/ from the REFERENCE itself.

Runs only in the build container, where /root/reference is mounted read-only:
    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py

It imports the reference's own Python (model, operators, windowing, kornia
rotation, keypoint maps) with stubs for third-party modules the reference
imports but that are absent here: pytorch_lightning,
torchvision, smplx, trimesh, imageio and the pyrender-based viewers. None of
the stubbed modules is on the computation path that the fixtures record.
Weights come from the PRNG in temporal_inverse_kinematics_amd/synthetic.py, so
the fixtures hold only inputs, outputs and the weight-blob sha256.

Outputs (all .npz, numpy arrays only, no pickles):
  graph.npz            Graph(...).A for several layouts/strategies  (graph.py:25-133)
  windowing.npz        sample_window / InferenceDataset cases       (data_amass.py:18-42,221-236)
  blocks.npz           StGcnBlock outputs, 3 residual kinds         (st_gcn_aaai18.py:136-214)
  gconv.npz            ConvTemporalGraphical, K=5 (spatial), t_kernel 1/3       (gconv_origin.py:36-65)
  model.npz            PoseRegressor outputs, T=64/65/9             (pose_trainer.py:66-133)
  run_inference.npz    inference.run_inference on the sample        (inference.py:37-67)
  kornia.npz           angle_axis_to_rotation_matrix                (kornia_geometry_conversion.py:125-201)
  keypoints.npz        moveai→COCO and SMPL-X→COCO maps             (keypoints_util.py:5-60)
and the data file temporal_inverse_kinematics_amd/data/dance_contemporary_coco.npy
(the sample sequence after inference.run_test's conversion, inference.py:121-133).
"""
import os
import sys
import types

import numpy as np
import torch

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)

from temporal_inverse_kinematics_amd import synthetic as syn  # noqa: E402


def _install_stubs():
    def mod(name, **attrs):
        m = types.ModuleType(name)
        m.__dict__.update(attrs)
        sys.modules[name] = m
        return m

    # bare packages: bypass the eager mmskeleton/__init__.py:1-3 import chain
    for name, path in [("mmskeleton", "mmskeleton"), ("mmskeleton.ops", "mmskeleton/ops"),
                       ("mmskeleton.models", "mmskeleton/models"),
                       ("mmskeleton.models.backbones", "mmskeleton/models/backbones"),
                       ("mmskeleton.datasets", "mmskeleton/datasets")]:
        m = mod(name)
        m.__path__ = [os.path.join(REF, path)]

    mod("torchvision")
    mod("torchvision.transforms")
    mod("torchvision.datasets", MNIST=object)

    class LightningModule(torch.nn.Module):
        @property
        def device(self):
            return next(self.parameters()).device

        def __setattr__(self, k, v):
            if k == "hparams":
                object.__setattr__(self, k, v)
            else:
                super().__setattr__(k, v)

    pl = mod("pytorch_lightning", _logger=None, LightningModule=LightningModule)
    mod("pytorch_lightning.core", LightningModule=LightningModule)
    pl.core = sys.modules["pytorch_lightning.core"]
    mod("smplx", create=None)
    mod("smplx.joint_names", JOINT_NAMES=[])
    mod("trimesh")
    mod("imageio", get_writer=None)
    mod("common.mesh_viewer", MeshViewer=None)
    mod("common.sphere", points_to_spheres=None)
    mod("common.draw_util", draw_3d_pose=None)
    sys.path.insert(0, REF)


def _load_state(module, sd):
    own = module.state_dict()
    new = {}
    for k, v in own.items():
        if k.endswith("num_batches_tracked"):
            new[k] = v
            continue
        assert k in sd, f"missing synthetic tensor for {k}"
        assert tuple(sd[k].shape) == tuple(v.shape), (k, sd[k].shape, v.shape)
        new[k] = torch.from_numpy(np.ascontiguousarray(sd[k]))
    extra = set(sd) - set(own)
    assert not extra, f"synthetic tensors not in reference module: {sorted(extra)}"
    module.load_state_dict(new)


def main():
    _install_stubs()
    torch.manual_seed(0)
    torch.set_num_threads(8)
    from mmskeleton.ops.st_gcn import ConvTemporalGraphical, Graph
    import mmskeleton.models.backbones.st_gcn_aaai18 as stg
    sys.modules["mmskeleton.models"].StgGcn18 = stg.StgGcn18
    sys.modules["mmskeleton.models"].StgLayerConfig = stg.StgLayerConfig
    sys.modules["mmskeleton.models"].StgConfig = stg.StgConfig
    import mmskeleton.datasets.data_amass as da
    sys.modules["mmskeleton.datasets"].AmassDataset = da.AmassDataset
    import pose_trainer
    import inference
    from common import kornia_geometry_conversion as kgc
    from common import keypoints_util as ku

    out = {}

    # ---- graph --------------------------------------------------------------
    g = {}
    for layout in ["coco", "openpose", "ntu-rgb+d", "ntu_edge"]:
        for strategy in ["uniform", "distance", "spatial"]:
            for max_hop in [1, 2]:
                G = Graph(layout=layout, strategy=strategy, max_hop=max_hop, dilation=1)
                g[f"{layout}|{strategy}|{max_hop}"] = G.A.astype(np.float64)
                g[f"{layout}|{strategy}|{max_hop}|hop"] = np.where(np.isinf(G.hop_dis), -1, G.hop_dis)
    np.savez_compressed(os.path.join(HERE, "graph.npz"), **g)

    # ---- windowing ------------------------------------------------------------
    w = {}
    arr = np.arange(10, dtype=np.float32)[:, None, None] * np.ones((1, 17, 3), np.float32)
    for idx in [0, 3, 5, 9]:
        w[f"sw|10|{idx}|4"] = da.sample_window(arr, idx, 4)
    arr20 = (np.arange(20 * 17 * 3, dtype=np.float32).reshape(20, 17, 3)) * 0.01
    for idx in [0, 1, 10, 18, 19]:
        try:
            w[f"sw|20|{idx}|8"] = da.sample_window(arr20, idx, 8)
        except ValueError:
            w[f"sw|20|{idx}|8|err"] = np.array(1)
    for idx in [10, 5]:
        try:
            w[f"sw|20|{idx}|32"] = da.sample_window(arr20, idx, 32)
        except ValueError:
            w[f"sw|20|{idx}|32|err"] = np.array(1)
    w["arr20"] = arr20
    arr10 = arr20[:10]
    for idx in [2, 3, 8, 9, 7]:  # short sequence: windows overrun both ends
        try:
            w[f"sw|10b|{idx}|8"] = da.sample_window(arr10, idx, 8)
        except ValueError:
            w[f"sw|10b|{idx}|8|err"] = np.array(1)
    rs = np.random.default_rng(3).normal(size=(30, 17, 3)).astype(np.float32)
    w["ids_in"] = rs
    ds = da.InferenceDataset(rs, win_size=9, relative_pose=True)
    w["ids_items"] = np.stack([ds[i][0] for i in range(len(ds))])
    np.savez_compressed(os.path.join(HERE, "windowing.npz"), **w)

    # ---- keypoint maps + the converted sample -----------------------------------
    d = np.load(os.path.join(REF, "data/sample_3d_poses/dance_contemporary.npz"), allow_pickle=False)
    mv = d["joints_3d"]
    names = d["joint_3d_names"].tolist()
    m = ku.generate_moveai3d_to_coco_mappings(names)
    seq = ku.convert_seq_keypoints(mv, m)
    # inference.run_test:126-133 (head keypoints and axis swap)
    seq[:, 0] = 0.5 * (mv[:, -1] + mv[:, -2])
    seq[:, 1] = mv[:, -2]
    seq[:, 2] = mv[:, -1]
    y = seq[:, :, 1].copy()
    z = seq[:, :, 2].copy()
    seq[:, :, 1] = z
    seq[:, :, 2] = -y
    os.makedirs(os.path.dirname(syn.SAMPLE_COCO_PATH), exist_ok=True)
    np.save(syn.SAMPLE_COCO_PATH, seq.astype(np.float32))
    smplx_names = ([f"j{i}" for i in range(55)] + ["nose", "right_eye", "left_eye", "right_ear", "left_ear"])
    # the public smplx JOINT_NAMES order for the first 60 names that the COCO map touches
    body = ["pelvis", "left_hip", "right_hip", "spine1", "left_knee", "right_knee", "spine2",
            "left_ankle", "right_ankle", "spine3", "left_foot", "right_foot", "neck", "left_collar",
            "right_collar", "head", "left_shoulder", "right_shoulder", "left_elbow", "right_elbow",
            "left_wrist", "right_wrist"]
    smplx_names[:22] = body
    np.savez_compressed(os.path.join(HERE, "keypoints.npz"),
                        moveai_names=np.array(names), moveai_to_coco=np.array(m),
                        moveai_joints=mv, coco_seq=seq.astype(np.float32),
                        smplx_names=np.array(smplx_names),
                        smplx_to_coco=np.array(ku.generate_smplx_to_coco_mappings(smplx_names)))

    # ---- kornia aa -> rotmat ------------------------------------------------------
    rng = np.random.default_rng(11)
    aa = rng.normal(0.0, 1.0, (1000, 3)).astype(np.float32)
    aa[:200] *= 2.0
    aa[0] = 0.0
    aa[1:40] = rng.normal(0.0, 1.0, (39, 3)).astype(np.float32) * 3e-4  # theta^2 <= 1e-6 Taylor branch
    aa[40:50] = rng.normal(0.0, 1.0, (10, 3)).astype(np.float32) * 6e-4  # near the branch threshold
    R = kgc.angle_axis_to_rotation_matrix(torch.from_numpy(aa)).numpy()
    np.savez_compressed(os.path.join(HERE, "kornia.npz"), aa=aa, R=R)

    # ---- ConvTemporalGraphical (generic operator) --------------------------------
    gc = {}
    Gs = Graph(layout="coco", strategy="spatial", max_hop=2, dilation=1)
    A3 = torch.tensor(Gs.A, dtype=torch.float32)
    for tag, (cin, cout, tk, ts, tp, td, bias) in {
        "k5_t1": (5, 7, 1, 1, 0, 1, True),
        "k5_t3": (6, 4, 3, 2, 1, 1, True),
        "k5_t3d2": (4, 8, 3, 1, 2, 2, False),
    }.items():
        op = ConvTemporalGraphical(cin, cout, A3.shape[0], t_kernel_size=tk, t_stride=ts,
                                   t_padding=tp, t_dilation=td, bias=bias)
        K = A3.shape[0]
        sd = {"conv.weight": syn.uniform(f"gconv.{tag}.w", (cout * K, cin, tk, 1), -0.4, 0.4)}
        if bias:
            sd["conv.bias"] = syn.uniform(f"gconv.{tag}.b", (cout * K,), -0.2, 0.2)
        _load_state(op, sd)
        x = torch.from_numpy(syn.uniform(f"gconv.{tag}.x", (3, cin, 11, 17), -1.0, 1.0))
        with torch.no_grad():
            y, _ = op(x, A3)
        gc[f"{tag}|x"] = x.numpy()
        gc[f"{tag}|y"] = y.numpy()
        for k, v in sd.items():
            gc[f"{tag}|{k}"] = v
        gc[f"{tag}|cfg"] = np.array([cin, cout, tk, ts, tp, td, int(bias)])
    gc["A"] = Gs.A.astype(np.float32)
    np.savez_compressed(os.path.join(HERE, "gconv.npz"), **gc)

    # ---- StGcnBlock: one per residual kind -----------------------------------------
    Gc = Graph(layout="coco", strategy="uniform", max_hop=2, dilation=1)
    A = torch.tensor(Gc.A, dtype=torch.float32)
    bl = {}
    for tag, (cin, cout, s) in {"conv_l0": (3, 64, 1), "iden_l1": (64, 64, 1),
                                "conv_s2_l2": (64, 128, 2), "zero": (16, 16, 1)}.items():
        residual = tag != "zero"
        blk = stg.StGcnBlock(cin, cout, (3, 1), stride=s, residual=residual)
        sd = syn.block_state_dict("", cin, cout, s, residual=residual, seed=5)
        _load_state(blk, sd)
        blk.eval()
        imp = torch.from_numpy(syn.uniform(f"block.{tag}.imp", (1, 17, 17), 0.5, 1.5))
        for T in [9, 16]:
            x = torch.from_numpy(syn.uniform(f"block.{tag}.x{T}", (2, cin, T, 17), -1.0, 1.0))
            with torch.no_grad():
                y, _ = blk(x, A * imp)
            bl[f"{tag}|T{T}|x"] = x.numpy()
            bl[f"{tag}|T{T}|y"] = y.numpy()
        bl[f"{tag}|imp"] = imp.numpy()
        bl[f"{tag}|cfg"] = np.array([cin, cout, s, int(residual)])
    bl["A"] = Gc.A.astype(np.float32)
    np.savez_compressed(os.path.join(HERE, "blocks.npz"), **bl)

    # ---- full PoseRegressor -----------------------------------------------------------
    hp = syn.HParams(win_size=64)
    net = pose_trainer.PoseRegressor(hp)
    sd = syn.ik_state_dict(Gc.A, seed=0)
    _load_state(net, sd)
    net.eval()
    md = {"weights_sha256": np.array(syn.state_dict_sha256(sd))}
    for (N, T, seed) in [(4, 64, 100), (2, 65, 101), (8, 9, 102), (3, 17, 103)]:
        x = syn.synthetic_windows(N, T, seed=seed)
        with torch.no_grad():
            feats = net.backbone(torch.from_numpy(x))
            y = net(torch.from_numpy(x))["poses"]
        md[f"T{T}|x"] = x
        md[f"T{T}|feat"] = feats.numpy()
        md[f"T{T}|y"] = y.numpy()
    np.savez_compressed(os.path.join(HERE, "model.npz"), **md)

    # ---- inference.run_inference on the converted sample --------------------------------
    ri = {"seq": seq.astype(np.float32)}

    class _Model(torch.nn.Module):
        def __init__(self, reg, win):
            super().__init__()
            self.regressor = reg
            self.hparams = types.SimpleNamespace(win_size=win)

        @property
        def device(self):
            return torch.device("cpu")

        def forward(self, x):
            return self.regressor(x)

    for win in [64, 9]:
        with torch.no_grad():
            ri[f"win{win}"] = inference.run_inference(_Model(net, win), seq.astype(np.float32))
    np.savez_compressed(os.path.join(HERE, "run_inference.npz"), **ri)
    print("wrote fixtures; weights sha256", md["weights_sha256"])


if __name__ == "__main__":
    main()
