"""Per-phase timing of the whole-block kernel (TIK_STB_TRACE hook) at the bench size."""
import os
import sys

os.environ["TIK_STB_TRACE"] = "1"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from temporal_inverse_kinematics_amd import synthetic as syn  # noqa: E402
from temporal_inverse_kinematics_amd.inference import synthetic_model  # noqa: E402

m = synthetic_model(win_size=64, device="cuda", precision="f16x3")
x = torch.from_numpy(syn.synthetic_windows(1024, 64, seed=0)).cuda()
with torch.no_grad():
    for _ in range(3):
        m(x)
    torch.cuda.synchronize()
