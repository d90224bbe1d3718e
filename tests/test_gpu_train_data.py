"""AmassDataset training-data generation on the GPU (data
half) against oracle/amass.py: the root-orientation augmentation against
scipy's Rotation (the reference's own dependency), the item windows against
the oracle's __getitem__ restatement on the same FK joints (noise value by
value through the restated counter generator; its distribution statistically),
and the FK-generated keypoints against the numpy SMPL-X oracle (parity
unpinned beyond the rotation step, as for the FK itself: tol 1e-4)."""
import numpy as np
import pytest
import torch

from oracle import amass as oa
from oracle import smplx_lbs as sl

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def models():
    from temporal_inverse_kinematics_amd import _build
    _build.build()
    from temporal_inverse_kinematics_amd.smplx_fk import load_smplx_models
    return load_smplx_models(None, "cuda", batch_size=9)


def _sequences(lens, seed=0):
    rng = np.random.default_rng(seed)
    out = []
    for i, F in enumerate(lens):
        t = np.linspace(0, 2 * np.pi, F, dtype=np.float32)[:, None]
        base = rng.normal(0, 0.3, (1, 156)).astype(np.float32)
        amp = rng.normal(0, 0.2, (1, 156)).astype(np.float32)
        poses = (base + amp * np.sin(t + i)).astype(np.float32)
        out.append({"poses": poses, "betas": rng.normal(0, 1, 10).astype(np.float32),
                    "gender": ["male", "female", "neutral"][i % 3]})
    return out


def test_rotate_root_z_matches_scipy():
    from temporal_inverse_kinematics_amd import _build
    _build.build()
    from temporal_inverse_kinematics_amd.training_data import rotate_root_z
    rng = np.random.default_rng(3)
    aa = rng.normal(0, 1.5, (500, 66)).astype(np.float32)
    aa[:20, :3] *= 1e-4                        # small-angle series branch
    aa[20:40, :3] = aa[20:40, :3] / np.linalg.norm(aa[20:40, :3], axis=1, keepdims=True) * 3.14159
    aa[40, :3] = 0.0
    for angle in [0.0, 0.3, 2.0 * np.pi * 0.77, np.pi]:
        g = rotate_root_z(torch.from_numpy(aa.copy()).cuda(), angle).cpu().numpy()
        r = oa.rotate_root_z(aa, angle)
        assert np.array_equal(g[:, 3:], aa[:, 3:])
        # rotvecs near pi may flip sign as a whole (same rotation): compare rotations
        from scipy.spatial import transform
        Rg = transform.Rotation.from_rotvec(g[:, :3].astype(np.float64)).as_matrix()
        Rr = transform.Rotation.from_rotvec(r[:, :3].astype(np.float64)).as_matrix()
        assert np.abs(Rg - Rr).max() < 2e-6, angle
        ok = np.linalg.norm(r[:, :3], axis=1) < 3.1
        assert np.abs(g[ok, :3] - r[ok, :3]).max() < 2e-6, angle


@pytest.mark.parametrize("noise", [False, True])
def test_items_match_oracle(models, noise):
    from temporal_inverse_kinematics_amd.training_data import AmassDataset
    seqs = _sequences([80, 131, 65, 200])
    ds = AmassDataset(models, seqs, window_size=64, keypoint_format="coco", add_gaussian_noise=noise, noise_seed=7)
    n = len(ds)
    assert n == 80 + 131 + 65 + 200
    idx = np.array([0, 1, 31, 32, 33, 48, 79, 80, 100, 210, 211, 240, 275, 276, 300, n - 1])
    b = ds.get_batch(idx)
    kp, ps = b["keypoints_3d"].cpu().numpy(), b["poses"].cpu().numpy()
    off = np.concatenate([[0], np.cumsum([80, 131, 65, 200])])
    for r, i in enumerate(idx):
        s = int(np.searchsorted(off, i, side="right") - 1)
        d = ds.data_anims[s]
        ref = oa.getitem(d["keypoints_3d"].cpu().numpy(), d["poses"].cpu().numpy(), d["betas"], int(i - off[s]),
                         32, int(i), add_noise=noise, seed=ds.noise_key)
        assert np.abs(kp[r] - ref["keypoints_3d"]).max() < 2e-6, i
        assert np.array_equal(ps[r], ref["poses"]), i
        assert np.array_equal(b["betas"][r].cpu().numpy(), ref["betas"])
    # any grouping of the items gives the same numbers
    b2 = ds.get_batch(idx[::-1])
    assert torch.equal(b2["keypoints_3d"], b["keypoints_3d"].flip(0))
    one = ds[int(idx[5])]
    assert np.array_equal(one["keypoints_3d"], kp[5])


def test_noise_distribution(models):
    """(noisy - clean) / sqrt(sigma) ~ N(0, 1) per coordinate (the reference's
    multivariate normal with a diagonal covariance sigma)."""
    from temporal_inverse_kinematics_amd.training_data import AmassDataset
    seqs = _sequences([400, 300])
    dn = AmassDataset(models, seqs, 64, "coco", add_gaussian_noise=True, noise_seed=1)
    dc = AmassDataset(models, seqs, 64, "coco", add_gaussian_noise=False)
    idx = np.arange(len(dn))
    a = dn.get_batch(idx)["keypoints_3d"].cpu().numpy().astype(np.float64)
    c = dc.get_batch(idx)["keypoints_3d"].cpu().numpy().astype(np.float64)
    sig = np.stack([oa.noise_sigma(w.astype(np.float32), oa.coco_kps_sigma()) for w in c])   # (B,17,3)
    z = (a - c) / np.sqrt(sig)[:, None]
    assert abs(z.mean()) < 0.01 and abs(z.std() - 1.0) < 0.01, (z.mean(), z.std())
    assert np.abs(np.corrcoef(z[..., 0].ravel(), z[..., 1].ravel())[0, 1]) < 0.01


def test_fk_keypoints_vs_oracle(models):
    """regenerate_data: rotated root + FK joints against scipy + the numpy SMPL-X oracle."""
    from temporal_inverse_kinematics_amd import synthetic as syn
    from temporal_inverse_kinematics_amd.training_data import AmassDataset
    seqs = _sequences([50, 70], seed=5)
    ds = AmassDataset(models, seqs, 16, "coco", add_gaussian_noise=False)
    rs = np.random.RandomState(0)
    for i, s in enumerate(seqs):
        angle = 2.0 * np.pi * rs.rand()
        rot = oa.rotate_root_z(s["poses"], angle)
        consts = syn.synthetic_smplx_constants(seed={"male": 1, "female": 2, "neutral": 3}[s["gender"]])
        full = np.zeros((rot.shape[0], 55, 3), np.float32)
        full[:, 0] = rot[:, :3]
        full[:, 1:22] = rot[:, 3:66].reshape(-1, 21, 3)
        full[:, 25:40] = rot[:, 66:111].reshape(-1, 15, 3)
        full[:, 40:55] = rot[:, 111:156].reshape(-1, 15, 3)
        jr = sl.smplx_forward(consts, full, np.tile(s["betas"][None], (rot.shape[0], 1)), return_verts=False)
        jg = ds.data_anims[i]["keypoints_3d"].cpu().numpy()
        assert np.abs(jg - jr).max() < 1e-4, i
    # and the epoch hook re-augments with the next epoch's angles
    first = ds.data_anims[0]["keypoints_3d"].clone()
    ds.on_epoch_end(1)
    assert not torch.equal(first, ds.data_anims[0]["keypoints_3d"])


def test_short_sequences_raise_like_sample_window(models):
    from temporal_inverse_kinematics_amd.training_data import AmassDataset
    ds = AmassDataset(models, _sequences([20]), 64, "coco", add_gaussian_noise=False)
    with pytest.raises(ValueError):
        ds.get_batch([5])
