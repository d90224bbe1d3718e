"""Per-phase timing of the xgemm launches of one IK forward (TIK_X_TRACE=1 must
be set in the environment): prints one XTRACE line per launch (stderr)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from temporal_inverse_kinematics_amd import synthetic as syn  # noqa: E402
from temporal_inverse_kinematics_amd.inference import synthetic_model  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
m = synthetic_model(win_size=64, device="cuda")
x = torch.from_numpy(syn.synthetic_windows(B, 64, seed=0)).cuda()
with torch.no_grad():
    m(x)
    torch.cuda.synchronize()
    print("---- traced forward", file=sys.stderr)
    m(x)
    torch.cuda.synchronize()
