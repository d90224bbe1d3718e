"""Max |xtws - XT128| of the poses and backbone features (TIK_XTWS=255 vs 0)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch


def model(**env):
    from temporal_inverse_kinematics_amd.inference import synthetic_model
    os.environ.update({k: str(v) for k, v in env.items()})
    m = synthetic_model(win_size=64, device="cuda").regressor
    m.tik_handle()
    return m


def main():
    from temporal_inverse_kinematics_amd import _build, synthetic as syn
    _build.build()
    xw = model(TIK_SPLIT=0, TIK_XTWS=255)
    tl = model(TIK_SPLIT=0, TIK_XTWS=0)
    for n, T in [(1024, 64), (3, 16), (7, 128), (257, 32)]:
        x = torch.from_numpy(syn.synthetic_windows(n, T, seed=n * 7 + T)).cuda()
        with torch.no_grad():
            a, b = xw(x)["poses"].clone(), tl(x)["poses"]
            fa, fb = xw.backbone_features(x), tl.backbone_features(x)
        print(n, T, "poses equal", torch.equal(a, b), float((a - b).abs().max()),
              "features equal", torch.equal(fa, fb), float((fa - fb).abs().max()), flush=True)


if __name__ == "__main__":
    main()
