"""FK step time: default stream vs a created stream, full_forward vs the C
call with preallocated outputs (where do the ~10 us inter-kernel gaps come from)."""
import ctypes, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from temporal_inverse_kinematics_amd import _build, _lib, synthetic as syn
from temporal_inverse_kinematics_amd.smplx_fk import SMPLX

_build.build()
B = 4096
c = syn.synthetic_smplx_constants(seed=1)
m = SMPLX(c, batch_size=B)
pose, betas = syn.synthetic_fk_inputs(B, seed=1)
P, Bt = torch.from_numpy(pose).cuda(), torch.from_numpy(betas).cuda()
J = torch.empty((B, m.num_joints, 3), device="cuda")
Vt = torch.empty((B, m.num_verts, 3), device="cuda")
lib = _lib.load()


def run(fn, stream, steps=10):
    with torch.cuda.stream(stream):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(steps):
            fn()
        e1.record()
        torch.cuda.synchronize()
    return e0.elapsed_time(e1) / steps


def ff():
    m.full_forward(P, Bt)


def ffo():
    m.full_forward(P, Bt, out=(J, Vt))


def direct():
    _lib.check(lib.tik_fk_forward(m._h, P.data_ptr(), Bt.data_ptr(), None, None, B, J.data_ptr(), Vt.data_ptr(),
                                  torch.cuda.current_stream().cuda_stream))


s = torch.cuda.Stream()
for rep in range(2):
    print(f"[pass {rep}]")
    print(f"direct      default stream {run(direct, torch.cuda.default_stream()):.4f} ms")
    print(f"full_forward out= default  {run(ffo, torch.cuda.default_stream()):.4f} ms")
    print(f"full_forward default stream {run(ff, torch.cuda.default_stream()):.4f} ms")
    print(f"direct      created stream {run(direct, s):.4f} ms")
    print(f"direct x50  default stream {run(direct, torch.cuda.default_stream(), 50):.4f} ms")
