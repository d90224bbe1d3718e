"""Diagnostic: the persistent temporal-conv kernel switched on one layer at a
time (TIK_XPT bit l); prints max |poses - per-tile kernel| per layer mask and
the first rows / columns of the backbone features that differ.
    python tests/diag/xpt_layers.py [N] [T]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from temporal_inverse_kinematics_amd import synthetic as syn  # noqa: E402
from temporal_inverse_kinematics_amd.inference import synthetic_model  # noqa: E402


def model(**env):
    old = {k: os.environ.get(k) for k in env}
    os.environ.update({k: str(v) for k, v in env.items()})
    try:
        m = synthetic_model(win_size=64, device="cuda", precision="bf16x3").regressor
        m.tik_handle()
    finally:
        for k, v in old.items():
            if v is None:
                del os.environ[k]
            else:
                os.environ[k] = v
    return m


N = int(sys.argv[1]) if len(sys.argv) > 1 else 4
T = int(sys.argv[2]) if len(sys.argv) > 2 else 64
x = torch.from_numpy(syn.synthetic_windows(N, T, seed=5)).cuda()
ref = model(TIK_SPLIT=0)
with torch.no_grad():
    yr = ref(x)["poses"].clone()
    fr = ref.backbone_features(x).clone()
for mask in ([1 << l for l in range(8)] + [255] if os.environ.get("ALL") else [128]):
    m = model(TIK_SPLIT=0, TIK_XPT=mask)
    with torch.no_grad():
        y = m(x)["poses"]
        f = m.backbone_features(x)
    d = (f - fr).abs().reshape(-1, f.shape[-1])
    bad = (d > 0).nonzero()
    print(f"mask {mask:3d}: max|dposes| {float((y - yr).abs().max()):.3e} max|dfeat| {float(d.max()):.3e} "
          f"bad feat elems {bad.shape[0]}" + (f" first {bad[:3].tolist()}" if bad.shape[0] else ""), flush=True)

# last layer only: which output rows / channels of layer 7 differ (rows = frame*17 + joint)
m = model(TIK_SPLIT=0, TIK_XPT=128)
with torch.no_grad():
    f = m.backbone_features(x)
d = (f - fr).abs().reshape(-1, 17, f.shape[-1] // 17).reshape(-1, f.shape[-1] // 17)   # rows x channels
rows = (d > 0).any(dim=1).nonzero().flatten().tolist()
cols = (d > 0).any(dim=0).nonzero().flatten().tolist()
print("layer-7 rows with a diff:", len(rows), "of", d.shape[0], "first", rows[:24], flush=True)
print("  row % 16 histogram:", [sum(1 for r in rows if r % 16 == k) for k in range(16)], flush=True)
print("  row % 128 first:", sorted(set(r % 128 for r in rows))[:40], flush=True)
print("channels with a diff:", len(cols), "first", cols[:24], flush=True)
print("  per-row bad counts (first 20 rows):", [(int(r), int((d[r] > 0).sum())) for r in rows[:20]], flush=True)
