"""Max |poses(XB0+XB1) - poses(layered)|, and with only one of the whole-block kernels."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import torch
from temporal_inverse_kinematics_amd import synthetic as syn
from test_gpu_ik import _model_with_env

x = torch.from_numpy(syn.synthetic_windows(64, 64, seed=5)).cuda()
outs = {}
for name, env in (("layered", dict(TIK_XBLK=0)), ("xblock", dict())):
    m = _model_with_env("bf16x3", TIK_SPLIT=0, **env)
    with torch.no_grad():
        outs[name] = m(x)["poses"].clone()
d = (outs["xblock"] - outs["layered"]).abs()
print("max diff", float(d.max()), "equal", bool(torch.equal(outs["xblock"], outs["layered"])), "n differing", int((d > 0).sum()), "of", d.numel())
