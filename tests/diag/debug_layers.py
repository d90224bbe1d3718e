"""Layer-by-layer GPU vs oracle comparison (debug aid)."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np, torch
from oracle import stgcn as orc
from temporal_inverse_kinematics_amd import synthetic as syn
from temporal_inverse_kinematics_amd.models import StGcnBlock

A = orc.graph_A("coco", "uniform", 2, 1)
for (cin, cout, s, res, T, N) in [(64, 64, 1, True, 9, 2), (16, 16, 1, False, 9, 1), (64, 64, 1, False, 4, 1),
                                  (8, 16, 1, False, 1, 1), (3, 64, 1, True, 9, 2), (64, 128, 2, True, 16, 2),
                                  (128, 128, 1, True, 32, 3), (256, 256, 2, True, 8, 2)]:
    sd = syn.block_state_dict("", cin, cout, s, residual=res, seed=5)
    imp = syn.uniform("imp", (1, 17, 17), 0.5, 1.5)
    Ae = A * imp
    x = syn.uniform("x", (N, cin, T, 17), -1, 1)
    blk = StGcnBlock(cin, cout, (3, 1), stride=s, residual=res)
    blk.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()}, strict=False)
    blk = blk.cuda().eval()
    with torch.no_grad():
        y, _ = blk(torch.from_numpy(x).cuda(), torch.from_numpy(Ae.astype(np.float32)).cuda())
    y = y.cpu().numpy()
    ref = orc.stgcn_block(x.astype(np.float64), Ae, sd, "", cin, cout, s, res)
    err = np.abs(y - ref)
    print(f"block cin={cin} cout={cout} s={s} res={res} T={T}: max err {err.max():.3e} "
          f"(max|ref| {np.abs(ref).max():.2f}); worst at {np.unravel_index(err.argmax(), err.shape)}")
    if err.max() > 1e-3 and T <= 9:
        # gcn-only check: z = relu(bn(mix(conv(x))))
        z = orc.gconv(x.astype(np.float64), Ae[None], sd["gcn.conv.weight"], sd["gcn.conv.bias"], 1)
        z = np.maximum(orc.batchnorm(z, sd, "tcn.0"), 0)
        print("   z range", np.abs(z).max())
