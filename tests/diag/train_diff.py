"""Per-tensor gradient / update differences of the GPU training step vs the oracle (diagnostic)."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np, torch
from oracle import stgcn as orc, train as otr
from temporal_inverse_kinematics_amd import synthetic as syn
from temporal_inverse_kinematics_amd.models import IKPoseTrainer, default_hparams
from temporal_inverse_kinematics_amd.trainer import GpuTrainer
N, T = int(sys.argv[1]) if len(sys.argv) > 1 else 8, int(sys.argv[2]) if len(sys.argv) > 2 else 9
sd = syn.ik_state_dict(orc.graph_A("coco", "uniform", 2, 1), seed=0)
m = IKPoseTrainer(default_hparams(win_size=T))
own = m.regressor.state_dict()
m.regressor.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items() if k in own}, strict=False)
Tp = T
for s in m.regressor.backbone.strides: Tp = (Tp - 1) // s + 1
rng = np.random.default_rng(1)
x = syn.synthetic_windows(N, T, seed=3)
tgt = rng.normal(0, 0.5, (N, Tp, 66)).astype(np.float32)
mask = (rng.random((N * Tp, 512)) < 0.3).astype(np.float32)
if len(sys.argv) > 3 and sys.argv[3] == "golden":
    gz = np.load("tests/golden/train.npz")
    x, tgt, mask = gz["x"][0], gz["target"][0], gz["mask"][0]
lr_ref, g_ref, s_ref = otr.train_steps(sd, [(x, tgt, mask)])
tr = GpuTrainer(m, lr=1e-4)
loss = float(tr.step(torch.from_numpy(x).cuda(), torch.from_numpy(tgt).cuda(), torch.from_numpy(mask).cuda()))
print("loss", loss, lr_ref)
G = {k: v.cpu().numpy() for k, v in tr.grads().items()}
S = {k: v.cpu().numpy() for k, v in tr.state_dict().items() if not k.endswith("tracked")}
for k in otr.param_names():
    g, r = G[k], g_ref[k]
    e = np.abs(g - r).max() / (np.abs(r).max() + 1e-30)
    d = S[k].astype(np.float64) - sd[k]; dr = s_ref[k].astype(np.float64) - sd[k]
    flag = " <<<" if e > 2e-3 else ""
    print(f"{k:50s} grad rel {e:.2e} |r|max {np.abs(r).max():.3e} delta maxdiff {np.abs(d-dr).max():.2e}{flag}")
for k, v in s_ref.items():
    if "running" in k:
        e = np.abs(S[k] - v).max()
        if e > 1e-5: print("BUF", k, e)
for k in ("backbone.data_bn.weight", "backbone.data_bn.bias"):
    e = np.abs(G[k] - g_ref[k])
    print(k, "per-channel abs err", np.array2string(e, precision=1, max_line_width=200))
    print(k, "ref", np.array2string(g_ref[k], precision=3, max_line_width=200))
# per-block outputs and input gradients vs the oracle (TIK_TRAIN_DEBUG=1)
if os.environ.get("TIK_TRAIN_DEBUG"):
    from temporal_inverse_kinematics_amd import _lib
    P, Bf = otr.split_state(sd)
    taps = []
    y = otr.forward(P, Bf, torch.from_numpy(x), torch.from_numpy(mask), taps=taps)
    torch.nn.functional.mse_loss(y, torch.from_numpy(tgt)).backward()
    cins = [4, 64, 64, 128, 128, 128, 128, 256]
    tins = [T]
    for s_ in m.regressor.backbone.strides: tins.append((tins[-1] - 1) // s_ + 1)
    for l, h in enumerate(taps):
        o_ref = h.detach().permute(0, 2, 3, 1).contiguous().numpy()          # (N,T',V,C)
        o = torch.empty(o_ref.size, device="cuda")
        _lib.check(_lib.load().tik_trainer_debug(tr._h.h, 0, l, o.data_ptr(), o.numel(), 0))
        eo = np.abs(o.cpu().numpy().reshape(o_ref.shape) - o_ref).max()
        msg = f"L{l} out err {eo:.2e}"
        if l + 1 < len(taps):
            gref = taps[l].grad.permute(0, 2, 3, 1).contiguous().numpy()     # grad of block l output = input grad of l+1
            gd = torch.empty(gref.size, device="cuda")
            _lib.check(_lib.load().tik_trainer_debug(tr._h.h, 1, l + 1, gd.data_ptr(), gd.numel(), 0))
            gg = gd.cpu().numpy().reshape(gref.shape)
            e = np.abs(gg - gref)
            msg += f"  dOut err {e.max():.2e} (max|ref| {np.abs(gref).max():.2e}); worst at {np.unravel_index(e.argmax(), e.shape)}"
            msg += f" frame-err {np.array2string(e.max(axis=(0,2,3)), precision=1)}"
        print(msg)
# one block's backward intermediates (TIK_TRAIN_DEBUG_LAYER=l) vs torch autograd of that block alone
if os.environ.get("TIK_TRAIN_DEBUG_LAYER"):
    from temporal_inverse_kinematics_amd import _lib
    L = int(os.environ["TIK_TRAIN_DEBUG_LAYER"])
    import torch.nn.functional as F
    P, Bf = otr.split_state(sd)
    taps = []
    y = otr.forward(P, Bf, torch.from_numpy(x), torch.from_numpy(mask), taps=taps)
    torch.nn.functional.mse_loss(y, torch.from_numpy(tgt)).backward()
    dO = taps[L].grad.detach()
    Xin = taps[L - 1].detach().clone().requires_grad_(True)
    cin, cout, s_ = otr.IK_LAYERS[L]
    p = f"backbone.st_gcn_networks.{L}."
    P2, B2 = otr.split_state(sd)
    Ae = B2["backbone.A"] * P2[f"backbone.edge_importance.{L}"]
    res = Xin if (cin == cout and s_ == 1) else None
    Yt = F.conv2d(Xin, P2[p + "gcn.conv.weight"], P2[p + "gcn.conv.bias"]); Yt.retain_grad()
    Zt = torch.einsum("nctv,vw->nctw", Yt, Ae[0]); Zt.retain_grad()
    Ht = F.relu(F.batch_norm(Zt, None, None, P2[p + "tcn.0.weight"], P2[p + "tcn.0.bias"], training=True)); Ht.retain_grad()
    Ut = F.conv2d(Ht, P2[p + "tcn.2.weight"], P2[p + "tcn.2.bias"], stride=(s_, 1), padding=(1, 0)); Ut.retain_grad()
    St = F.batch_norm(Ut, None, None, P2[p + "tcn.3.weight"], P2[p + "tcn.3.bias"], training=True) + res
    St.retain_grad()
    Ot = F.relu(St)
    Ot.backward(dO)
    def cl(t): return t.detach().permute(0, 2, 3, 1).contiguous().numpy()
    refs = {2: cl(Ut), 3: cl(Ht), 4: cl(Zt), 5: cl(Yt), 10: cl(St.grad), 11: cl(Ut.grad), 12: cl(Ht.grad), 13: cl(Zt.grad), 14: cl(Yt.grad)}
    names = {2: "U", 3: "H", 4: "Z", 5: "Y", 10: "gS", 11: "dU", 12: "dH", 13: "dZ", 14: "dY"}
    for w, r in refs.items():
        o = torch.empty(r.size, device="cuda")
        _lib.check(_lib.load().tik_trainer_debug(tr._h.h, w, L, o.data_ptr(), o.numel(), 0))
        e = np.abs(o.cpu().numpy().reshape(r.shape) - r)
        print(f"B{L} {names[w]:8s} err {e.max():.2e} max|ref| {np.abs(r).max():.2e} frame-err {np.array2string(e.max(axis=(0,2,3)), precision=1)}")
    # gS consistency: GPU gS vs dO(gpu dump) * (O(gpu dump) > 0)
    co = otr.IK_LAYERS[L][1]
    def dump(w, lay, n):
        o = torch.empty(n, device="cuda")
        _lib.check(_lib.load().tik_trainer_debug(tr._h.h, w, lay, o.data_ptr(), n, 0))
        return o.cpu().numpy()
    r = refs[10]
    gS = dump(10, L, r.size).reshape(r.shape)
    dOg = dump(1, L + 1, r.size).reshape(r.shape)
    Og = dump(0, L, r.size).reshape(r.shape)
    mine = dOg * (Og > 0)
    print("B gS vs dO*(O>0) (gpu dumps):", np.abs(gS - mine).max(), " ref vs same:", np.abs(r - mine).max())
    bad = np.argwhere(np.abs(gS - r) > 1e-4)[:8]
    for b in bad:
        b = tuple(b)
        print("B  at", b, "gS", gS[b], "ref", r[b], "dO", dOg[b], "O", Og[b], "O_ref", cl(Ot)[b])
