// trainer.cpp — C ABI of the training step: IKPoseTrainer.training_step
// (pose_trainer.py:146-155) + the Lightning backward + torch.optim.Adam step
// (configure_optimizers, pose_trainer.py:196-197), on the device.
//
// One step = train-mode forward (BatchNorm on batch statistics with the
// running-stat update, the head's Dropout(0.7), st_gcn_aaai18.py:119-133,
// 208-214, pose_trainer.py:89-92,94-133), nn.MSELoss against the target
// poses (PoseLosses, pose_trainer.py:42-50), the backward of every
// operation, and one Adam update of every parameter (lr = hparams.lr,
// betas (0.9, 0.999), eps 1e-8, no weight decay).
//
// Parameters live in ONE flat fp32 buffer in the reference's tensor layouts
// (so Adam is one launch and a state-dict export is a copy); after every
// update the GEMM-side layouts are re-derived on the device (temporal taps
// innermost for the forward, transposed / tap-flipped for the input
// gradients, A_eff = A * edge_importance). GEMMs (forward convs, input
// gradients) run on the fp32 implicit-GEMM kernel (cgemm.hip); weight
// gradients on train.hip's row-split MFMA kernel; BatchNorm, graph mix,
// activation and loss kernels in train.hip.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/tik.h"
#include "cgemm.h"
#include "common.h"
#include "misc.h"
#include "train.h"

using namespace tik_host;

namespace {

constexpr int V = 17;
constexpr int HIDDEN = 512;
constexpr float DROPOUT_P = 0.7f;   // pose_trainer.py:91
enum { RES_I = 1, RES_C = 2 };

struct TEntry {          // one exported state-dict tensor
    std::string name;
    std::vector<int64_t> shape;
    long long off = 0, numel = 0;
    int kind = 0;        // 0 parameter (flat P / grad / Adam state), 1 buffer (flat B)
};

struct TLayer {
    int cin = 0, cinp = 0, cout = 0, stride = 1, res = RES_I;
    // parameter offsets (flat P) and buffer offsets (flat B)
    long long wg = -1, bg = -1, g1 = -1, b1 = -1, wt = -1, bt = -1, g2 = -1, b2 = -1, wr = -1, br = -1, g3 = -1,
              b3 = -1, E = -1;
    long long rm1 = -1, rv1 = -1, rm2 = -1, rv2 = -1, rm3 = -1, rv3 = -1;
    DevBuf wgf, wgb, wtf, wtb, wrf, wrb, aeff;     // derived GEMM layouts
    DevBuf Y, Z, H, U, Q, O;                        // saved activations
    DevBuf st1, st2, st3;                           // [4][C] mean, invstd, scale, shift
    int tin = 0, tout = 0;
};

int round4(int c) { return (c + 3) & ~3; }

tik::Seg seg32(const float* src, const float* w, int cin, int ld, int kt, int stride, int pad, int tin, int ldw) {
    tik::Seg s{src, w, cin, ld, kt, stride, pad, tin, ldw};
    return s;
}

}  // namespace

struct tik_trainer {
    std::vector<TEntry> ents;
    std::vector<TLayer> L;
    DevBuf P, G, M, Vv, B;
    long long np = 0, nb = 0;
    long long dg = -1, db = -1, rm0 = -1, rv0 = -1, A = -1;       // data_bn + adjacency
    bool zero_pending = false;                                     // gA/gB reallocated: zero them on the step's stream
    long long w1 = -1, b1 = -1, w2 = -1, b2 = -1;                  // head
    int feat = 0, pose_dim = 0;
    DevBuf w1b, w2b;                                               // W1^T [feat][512], W2^T [512][ldp]
    int ldp = 0;                                                   // pose_dim rounded to 4
    // workspace
    int N = 0, T = 0;
    DevBuf x4, x0, st0, k, Ph, Dh, Oh, dOh, dD, mask, loss, partf, gA, gB, tS, tU, tQ, tH, tZ, tY, col, up;
    DevArray<double> partd;
    DevIBuf cmap0;
    long long partf_cap = 0, partd_cap = 0;
    long long steps = 0;
    DevArray<unsigned char> perm;   // weight re-layout descriptors (tik::PermDesc)
    int nperm = 0;
    long long perm_blocks = 0;
    std::vector<DevBuf> dbg_dx;   // TIK_TRAIN_DEBUG=1: each block's input gradient of the last step
    DevBuf dbg_b[5];              // TIK_TRAIN_DEBUG_LAYER=l: that block's gS, dU, dH (post-ReLU), dZ, dY
    float lr = 1e-4f, beta1 = 0.9f, beta2 = 0.999f, eps = 1e-8f, momentum = 0.1f;
};

namespace {

int add_entry(tik_trainer* t, const TensorMap& m, const std::string& name, int kind, long long* off,
              std::vector<float>& hp, std::vector<float>& hb, bool required = true) {
    const HostTensor* h = find(m, name);
    if (!h) {
        if (required) return fail(TIK_E_MISSING, "tik_trainer_create: missing tensor '%s'", name.c_str());
        *off = -1;
        return TIK_OK;
    }
    TEntry e;
    e.name = name;
    e.shape = h->shape;
    e.numel = (long long)h->v.size();
    e.kind = kind;
    std::vector<float>& dst = kind == 0 ? hp : hb;
    e.off = (long long)dst.size();
    dst.insert(dst.end(), h->v.begin(), h->v.end());
    *off = e.off;
    t->ents.push_back(std::move(e));
    return TIK_OK;
}

const HostTensor* shape_of(const TensorMap& m, const std::string& k) { return find(m, k); }

// GEMM-side layouts from the flat parameters (after create and every update):
// one batched launch over a descriptor table built once (pointers are fixed)
int derive(tik_trainer* t, hipStream_t st) {
    if (!t->perm.p) {
        const float* P = t->P.p;
        std::vector<tik::PermDesc> d;
        auto add = [&](float* dst, const float* src, const float* src2, int d0, int d1, int d2, long long ds0,
                       long long ds1, long long ds2, long long soff, long long ss0, long long ss1, long long ss2) {
            tik::PermDesc q{dst, src, src2, d0, d1, d2, ds0, ds1, ds2, soff, ss0, ss1, ss2, 0};
            d.push_back(q);
        };
        for (TLayer& l : t->L) {
            const int ci = l.cin, cp = l.cinp, co = l.cout;
            // wgf[co][cp] <- W[co][ci]; wgb[ci][co] <- W[co][ci]
            add(l.wgf.p, P + l.wg, nullptr, co, ci, 1, cp, 1, 0, 0, ci, 1, 0);
            add(l.wgb.p, P + l.wg, nullptr, ci, co, 1, co, 1, 0, 0, 1, ci, 0);
            // wtf[co][tap][c] <- W[co][c][tap]; wtb[c][tap'][co] <- W[co][c][2 - tap']
            add(l.wtf.p, P + l.wt, nullptr, co, 3, co, 3LL * co, co, 1, 0, 3LL * co, 1, 3);
            add(l.wtb.p, P + l.wt, nullptr, co, 3, co, 3LL * co, co, 1, 2, 3, -1, 3LL * co);
            if (l.res == RES_C) {
                add(l.wrf.p, P + l.wr, nullptr, co, ci, 1, cp, 1, 0, 0, ci, 1, 0);
                add(l.wrb.p, P + l.wr, nullptr, ci, co, 1, co, 1, 0, 0, 1, ci, 0);
            }
            // A_eff = A * edge_importance (st_gcn_aaai18.py:129)
            add(l.aeff.p, t->B.p + t->A, P + l.E, V * V, 1, 1, 1, 0, 0, 0, 1, 0, 0);
        }
        // W1^T [feat][512] <- W1[512][feat]; W2^T [512][ldp] <- W2[pose][512]
        add(t->w1b.p, P + t->w1, nullptr, t->feat, HIDDEN, 1, HIDDEN, 1, 0, 0, 1, t->feat, 0);
        add(t->w2b.p, P + t->w2, nullptr, HIDDEN, t->pose_dim, 1, t->ldp, 1, 0, 0, 1, HIDDEN, 0);
        t->perm_blocks = tik::permute_batch_blocks(d.data(), (int)d.size());
        t->nperm = (int)d.size();
        std::vector<unsigned char> bytes(d.size() * sizeof(tik::PermDesc));
        memcpy(bytes.data(), d.data(), bytes.size());
        int rc;
        if ((rc = t->perm.upload(bytes))) return rc;
    }
    HIP_TRY(tik::launch_permute_batch(reinterpret_cast<const tik::PermDesc*>(t->perm.p), t->nperm, t->perm_blocks, st));
    return TIK_OK;
}

int reserve(tik_trainer* t, int N, int T) {
    if (N == t->N && T == t->T) return TIK_OK;
    int rc;
    long long big = 0, colsz = 0;
    int tin = T;
    for (TLayer& l : t->L) {
        l.tin = tin;
        l.tout = (tin - 1) / l.stride + 1;
        const long long pin = (long long)N * l.tin * V, pout = (long long)N * l.tout * V;
        if ((rc = l.Y.reserve(pin * l.cout)) || (rc = l.Z.reserve(pin * l.cout)) || (rc = l.H.reserve(pin * l.cout)) ||
            (rc = l.U.reserve(pout * l.cout)) || (rc = l.O.reserve(pout * l.cout)))
            return rc;
        if (l.res == RES_C && (rc = l.Q.reserve(pout * l.cout))) return rc;
        big = std::max(big, pin * std::max(l.cout, l.cinp));
        colsz = std::max(colsz, std::max(pout * 3LL * l.cout, pout * (long long)l.cinp));
        tin = l.tout;
    }
    const long long rows_h = (long long)N * tin;
    const long long p0 = (long long)N * T * V;
    t->partf_cap = std::max<long long>(8LL << 20, 64LL * rows_h * HIDDEN);
    t->partd_cap = 2LL * 1024 * 1024;
    if ((rc = t->x4.reserve(p0 * 4)) || (rc = t->x0.reserve(p0 * 4)) || (rc = t->Ph.reserve(rows_h * HIDDEN)) ||
        (rc = t->Dh.reserve(rows_h * HIDDEN)) || (rc = t->Oh.reserve(rows_h * t->ldp)) ||
        (rc = t->dOh.reserve(rows_h * t->ldp)) || (rc = t->dD.reserve(rows_h * HIDDEN)) ||
        (rc = t->mask.reserve(rows_h * HIDDEN)) || (rc = t->partf.reserve(t->partf_cap)) ||
        (rc = t->partd.reserve(t->partd_cap)) || (rc = t->gA.reserve(big)) || (rc = t->gB.reserve(big)) ||
        (rc = t->tS.reserve(big)) || (rc = t->tU.reserve(big)) || (rc = t->tQ.reserve(big)) ||
        (rc = t->tH.reserve(big)) || (rc = t->tZ.reserve(big)) || (rc = t->tY.reserve(big)) ||
        (rc = t->col.reserve(colsz)) || (rc = t->up.reserve(big)))
        return rc;
    // the gradient ping-pong buffers start zeroed (stream-ordered, in step()); their
    // padding column (layer 0's 4th input channel) is never read: bn_bwd_finalize
    // zeroes it through cmap0 = -1
    t->zero_pending = true;
    t->N = N;
    t->T = T;
    return TIK_OK;
}

// fp32 implicit GEMM: 128x128 tiles when they fill the chip (>= 256
// workgroups) and the output is wider than 64 channels, else 64x64 tiles (the
// training batches are 10-40k rows: 128x128 tiles would leave CUs idle, and
// half of each tile would be empty on the 64-channel blocks)
int gemm(const tik::CgemmArgs& a, hipStream_t st) {
    const long long t128 = (long long)((a.M + 127) / 128) * ((a.Nc + 127) / 128);
    const int cfg = (a.Nc > 64 && t128 >= 256) ? tik::CFG_T128x128 : tik::CFG_H64x64;
    HIP_TRY(tik::launch_cgemm(a, cfg, st, tik::PREC_F32));
    return TIK_OK;
}

// train-mode BatchNorm statistics of X [R][C] -> stat, running stats updated
int bn_stats(tik_trainer* t, const float* X, long long R, int C, const int* cmap, long long g, long long b,
             long long rm, long long rv, float* stat, hipStream_t st) {
    int nc = 0;
    HIP_TRY(tik::launch_colstats(X, nullptr, nullptr, R, C, t->partd.p, (int)(t->partd_cap / (2LL * C)), &nc, st));
    HIP_TRY(tik::launch_bn_fwd_finalize(t->partd.p, nc, R, C, cmap, t->P.p + g, t->P.p + b, t->B.p + rm, t->B.p + rv,
                                        t->momentum, BN_EPS, stat, st));
    return TIK_OK;
}

// BatchNorm backward: grads of gamma/beta into G, dx into out (when non-null)
// (Mr: the output of a ReLU between this BatchNorm and Gr, whose backward is folded in)
int bn_back(tik_trainer* t, const float* Gr, const float* X, long long R, int C, const int* cmap, long long g,
            long long b, const float* stat, float* out, hipStream_t st, const float* Mr = nullptr) {
    int nc = 0;
    HIP_TRY(tik::launch_colstats(X, Gr, stat, R, C, t->partd.p, (int)(t->partd_cap / (2LL * C)), &nc, st, Mr));
    HIP_TRY(tik::launch_bn_bwd_finalize(t->partd.p, nc, R, C, cmap, t->P.p + g, stat, t->G.p + g, t->G.p + b,
                                        t->k.p, st));
    if (out) HIP_TRY(tik::launch_bn_bwd_apply(out, Gr, X, stat, t->k.p, R, C, st, Mr));
    return TIK_OK;
}

int colsum(tik_trainer* t, const float* X, long long R, int C, float* dst, hipStream_t st) {
    int nc = 0;
    HIP_TRY(tik::launch_colstats(X, nullptr, nullptr, R, C, t->partd.p, (int)(t->partd_cap / (2LL * C)), &nc, st));
    HIP_TRY(tik::launch_colsum_finalize(t->partd.p, nc, C, dst, st));
    return TIK_OK;
}

int wgrad(tik_trainer* t, const float* A, int lda, const float* Bm, int ldb, int M, int Nn, long long R, float* C,
          int ldc, hipStream_t st, const tik::WgradTaps& g = tik::WgradTaps()) {
    HIP_TRY(tik::launch_wgrad(A, lda, Bm, ldb, M, Nn, R, C, ldc, t->partf.p, t->partf_cap, st, g));
    return TIK_OK;
}

int forward_block(tik_trainer* t, TLayer& l, const float* X, int ldx, hipStream_t st) {
    const int N = t->N, co = l.cout;
    const long long pin = (long long)N * l.tin * V, pout = (long long)N * l.tout * V;
    float* P = t->P.p;
    int rc;
    // gcn 1x1 conv + bias (gconv_origin.py:61), then the graph mix (:64)
    tik::CgemmArgs g{};
    g.M = (int)pin; g.Nc = co; g.V = V; g.tout = l.tin;
    g.seg[0] = seg32(X, l.wgf.p, l.cinp, ldx, 1, 1, 0, l.tin, l.cinp);
    g.nseg = 1; g.bias = P + l.bg; g.out = l.Y.p; g.ldo = co; g.act = tik::ACT_NONE;
    if ((rc = gemm(g, st))) return rc;
    HIP_TRY(tik::launch_mix(l.Z.p, l.Y.p, l.aeff.p, 0, (long long)N * l.tin, co, st));
    // tcn.0 BatchNorm (batch statistics) + tcn.1 ReLU (st_gcn_aaai18.py:178-179)
    if ((rc = bn_stats(t, l.Z.p, pin, co, nullptr, l.g1, l.b1, l.rm1, l.rv1, l.st1.p, st))) return rc;
    HIP_TRY(tik::launch_affine(l.H.p, l.Z.p, l.st1.p + 2 * co, l.st1.p + 3 * co, nullptr, nullptr, nullptr, pin, co, 1,
                               st));
    // tcn.2 temporal conv (3x1, stride s, pad 1) + bias (:180-185)
    tik::CgemmArgs u{};
    u.M = (int)pout; u.Nc = co; u.V = V; u.tout = l.tout;
    u.seg[0] = seg32(l.H.p, l.wtf.p, co, co, 3, l.stride, 1, l.tin, 3 * co);
    u.nseg = 1; u.bias = P + l.bt; u.out = l.U.p; u.ldo = co; u.act = tik::ACT_NONE;
    if ((rc = gemm(u, st))) return rc;
    if ((rc = bn_stats(t, l.U.p, pout, co, nullptr, l.g2, l.b2, l.rm2, l.rv2, l.st2.p, st))) return rc;
    // residual (:191-204) and the block's ReLU (:212-214)
    if (l.res == RES_C) {
        tik::CgemmArgs q{};
        q.M = (int)pout; q.Nc = co; q.V = V; q.tout = l.tout;
        q.seg[0] = seg32(X, l.wrf.p, l.cinp, ldx, 1, l.stride, 0, l.tin, l.cinp);
        q.nseg = 1; q.bias = P + l.br; q.out = l.Q.p; q.ldo = co; q.act = tik::ACT_NONE;
        if ((rc = gemm(q, st))) return rc;
        if ((rc = bn_stats(t, l.Q.p, pout, co, nullptr, l.g3, l.b3, l.rm3, l.rv3, l.st3.p, st))) return rc;
        HIP_TRY(tik::launch_affine(l.O.p, l.U.p, l.st2.p + 2 * co, l.st2.p + 3 * co, l.Q.p, l.st3.p + 2 * co,
                                   l.st3.p + 3 * co, pout, co, 1, st));
    } else {
        HIP_TRY(tik::launch_affine(l.O.p, l.U.p, l.st2.p + 2 * co, l.st2.p + 3 * co, X, nullptr, nullptr, pout, co, 1,
                                   st));
    }
    return TIK_OK;
}

// dO: gradient of the block output [pout][co]; X: block input [pin][ldx];
// dX: its gradient [pin][ldx] (ldx = cinp; padding columns left untouched)
int backward_block(tik_trainer* t, TLayer& l, const float* X, int ldx, const float* dO, float* dX, hipStream_t st) {
    const int N = t->N, co = l.cout, ci = l.cin;
    const long long pin = (long long)N * l.tin * V, pout = (long long)N * l.tout * V;
    float* Gd = t->G.p;
    int rc;
    // block ReLU: materialized (gS) only where the identity residual passes it
    // on; otherwise folded into the two BatchNorm backward passes
    const float* gS = dO;
    const float* mO = l.O.p;
    if (l.res == RES_I) {
        HIP_TRY(tik::launch_relu_bwd(t->tS.p, dO, l.O.p, pout * co, st));
        gS = t->tS.p;
        mO = nullptr;
    }
    // tcn.3 BatchNorm -> dU ; residual BatchNorm -> dQ
    if ((rc = bn_back(t, gS, l.U.p, pout, co, nullptr, l.g2, l.b2, l.st2.p, t->tU.p, st, mO))) return rc;
    if (l.res == RES_C && (rc = bn_back(t, gS, l.Q.p, pout, co, nullptr, l.g3, l.b3, l.st3.p, t->tQ.p, st, mO)))
        return rc;
    // tcn.2: bias and weight gradients (im2col of H, [ci][tap] = the torch weight layout)
    if ((rc = colsum(t, t->tU.p, pout, co, Gd + l.bt, st))) return rc;
    {
        // implicit im2col of H through the conv's row map (C % 64 == 0 for every block)
        tik::WgradTaps g;
        g.C = co; g.kt = 3; g.s = l.stride; g.pad = 1; g.tin = l.tin; g.tout = l.tout; g.V = V;
        if (co % 64 == 0) {
            if ((rc = wgrad(t, t->tU.p, co, l.H.p, co, co, 3 * co, pout, Gd + l.wt, 3 * co, st, g))) return rc;
        } else {
            HIP_TRY(tik::launch_im2col(t->col.p, l.H.p, co, co, 3, l.stride, 1, N, l.tin, l.tout, V, st));
            if ((rc = wgrad(t, t->tU.p, co, t->col.p, 3 * co, co, 3 * co, pout, Gd + l.wt, 3 * co, st))) return rc;
        }
    }
    // residual conv: bias and weight gradients
    if (l.res == RES_C) {
        if ((rc = colsum(t, t->tQ.p, pout, co, Gd + l.br, st))) return rc;
        if (l.stride == 1) {
            if ((rc = wgrad(t, t->tQ.p, co, X, ldx, co, ci, pout, Gd + l.wr, ci, st))) return rc;
        } else if (ci % 64 == 0 && ldx == ci) {   // strided rows of X read in place (tap mode, kt = 1)
            tik::WgradTaps g;
            g.C = ci; g.kt = 1; g.s = l.stride; g.pad = 0; g.tin = l.tin; g.tout = l.tout; g.V = V;
            if ((rc = wgrad(t, t->tQ.p, co, X, ldx, co, ci, pout, Gd + l.wr, ci, st, g))) return rc;
        } else {
            HIP_TRY(tik::launch_im2col(t->col.p, X, ldx, l.cinp, 1, l.stride, 0, N, l.tin, l.tout, V, st));
            if ((rc = wgrad(t, t->tQ.p, co, t->col.p, l.cinp, co, ci, pout, Gd + l.wr, ci, st))) return rc;
        }
    }
    // tcn.2 input gradient: the transposed conv = stride-1 conv of the
    // (zero-upsampled) dU with the tap-flipped, transposed weights
    const float* du = t->tU.p;
    if (l.stride != 1) {
        HIP_TRY(tik::launch_upsample(t->up.p, t->tU.p, co, l.stride, N, l.tin, l.tout, V, st));
        du = t->up.p;
    }
    tik::CgemmArgs h{};
    h.M = (int)pin; h.Nc = co; h.V = V; h.tout = l.tin;
    h.seg[0] = seg32(du, l.wtb.p, co, co, 3, 1, 1, l.tin, 3 * co);
    h.nseg = 1; h.out = t->tH.p; h.ldo = co; h.act = tik::ACT_NONE;
    if ((rc = gemm(h, st))) return rc;
    // tcn.1 ReLU (folded) + tcn.0 BatchNorm -> dZ
    if ((rc = bn_back(t, t->tH.p, l.Z.p, pin, co, nullptr, l.g1, l.b1, l.st1.p, t->tZ.p, st, l.H.p))) return rc;
    // graph mix: dY = mix(dZ, A_eff^T); edge-importance gradient
    HIP_TRY(tik::launch_mix(t->tY.p, t->tZ.p, l.aeff.p, 1, (long long)N * l.tin, co, st));
    HIP_TRY(tik::launch_mix_grad(l.Y.p, t->tZ.p, (long long)N * l.tin, co, t->B.p + t->A, Gd + l.E, t->partd.p,
                                 (int)(t->partd_cap / 289), st));
    // gcn conv: bias and weight gradients
    if ((rc = colsum(t, t->tY.p, pin, co, Gd + l.bg, st))) return rc;
    if ((rc = wgrad(t, t->tY.p, co, X, ldx, co, ci, pin, Gd + l.wg, ci, st))) return rc;
    // input gradient: dY Wg (+ the residual conv's transposed 1x1, or the identity residual)
    tik::CgemmArgs x{};
    x.M = (int)pin; x.Nc = ci; x.V = V; x.tout = l.tin;
    x.seg[0] = seg32(t->tY.p, l.wgb.p, co, co, 1, 1, 0, l.tin, co);
    x.nseg = 1;
    if (l.res == RES_C) {
        const float* dq = t->tQ.p;
        if (l.stride != 1) {
            HIP_TRY(tik::launch_upsample(t->up.p, t->tQ.p, co, l.stride, N, l.tin, l.tout, V, st));
            dq = t->up.p;
        }
        x.seg[1] = seg32(dq, l.wrb.p, co, co, 1, 1, 0, l.tin, co);
        x.nseg = 2;
    } else {
        x.resid = t->tS.p; x.ldr = co;
    }
    x.out = dX; x.ldo = ldx; x.act = tik::ACT_NONE;
    if ((rc = gemm(x, st))) return rc;
    static const int dbg_layer = getenv("TIK_TRAIN_DEBUG_LAYER") ? atoi(getenv("TIK_TRAIN_DEBUG_LAYER")) : -1;
    if (&l == &t->L[dbg_layer < 0 ? 0 : dbg_layer] && dbg_layer >= 0) {
        const float* src[5] = {t->tS.p, t->tU.p, t->tH.p, t->tZ.p, t->tY.p};
        const long long n[5] = {pout * co, pout * co, pin * co, pin * co, pin * co};
        for (int j = 0; j < 5; ++j) {
            if ((rc = t->dbg_b[j].reserve(n[j]))) return rc;
            HIP_TRY(hipMemcpyAsync(t->dbg_b[j].p, src[j], n[j] * sizeof(float), hipMemcpyDeviceToDevice, st));
        }
    }
    return TIK_OK;
}

int step(tik_trainer* t, const float* x, int N, int T, const float* target, const float* user_mask,
         unsigned long long seed, float* loss_out, hipStream_t st) {
    int rc;
    if ((rc = reserve(t, N, T))) return rc;
    if (t->zero_pending) {
        HIP_TRY(hipMemsetAsync(t->gA.p, 0, t->gA.n * sizeof(float), st));
        HIP_TRY(hipMemsetAsync(t->gB.p, 0, t->gB.n * sizeof(float), st));
        t->zero_pending = false;
    }
    (void)hipGetLastError();
    const long long R0 = (long long)N * T, p0 = R0 * V;
    float* P = t->P.p;
    float* Gd = t->G.p;
    // data_bn (BatchNorm1d over the V*C channels, st_gcn_aaai18.py:119-125) on
    // 4-channel padded rows: column 4v+c is channel v*3+c
    HIP_TRY(tik::launch_pad_channels(x, p0, 3, 4, t->x4.p, st));
    if ((rc = bn_stats(t, t->x4.p, R0, 4 * V, t->cmap0.p, t->dg, t->db, t->rm0, t->rv0, t->st0.p, st))) return rc;
    HIP_TRY(tik::launch_affine(t->x0.p, t->x4.p, t->st0.p + 2 * 4 * V, t->st0.p + 3 * 4 * V, nullptr, nullptr, nullptr,
                               R0, 4 * V, 0, st));
    // backbone
    const float* X = t->x0.p;
    int ldx = 4;
    for (TLayer& l : t->L) {
        if ((rc = forward_block(t, l, X, ldx, st))) return rc;
        X = l.O.p;
        ldx = l.cout;
    }
    // head: Linear -> LeakyReLU -> Dropout(0.7) -> Linear (pose_trainer.py:89-92)
    const int Tp = t->L.back().tout;
    const long long rows = (long long)N * Tp;
    const float* feat = t->L.back().O.p;
    tik::CgemmArgs h{};
    h.M = (int)rows; h.Nc = HIDDEN; h.V = 1; h.tout = (int)rows;
    h.seg[0] = seg32(feat, P + t->w1, t->feat, t->feat, 1, 1, 0, (int)rows, t->feat);
    h.nseg = 1; h.bias = P + t->b1; h.out = t->Ph.p; h.ldo = HIDDEN; h.act = tik::ACT_NONE;
    h.ksplit = tik::splitk_for(h, 64, 64, 16, 64);
    h.partial = t->partf.p;
    HIP_TRY(tik::launch_cgemm(h, tik::CFG_H64x64, st, tik::PREC_F32));
    const float* mask = user_mask;
    if (!mask) {
        HIP_TRY(tik::launch_dropout_mask(t->mask.p, rows * HIDDEN, 1.f - DROPOUT_P, seed, st));
        mask = t->mask.p;
    }
    const float scale = 1.f / (1.f - DROPOUT_P);
    HIP_TRY(tik::launch_leaky_dropout(t->Dh.p, t->Ph.p, mask, scale, rows * HIDDEN, st));
    tik::CgemmArgs o{};
    o.M = (int)rows; o.Nc = t->pose_dim; o.V = 1; o.tout = (int)rows;
    o.seg[0] = seg32(t->Dh.p, P + t->w2, HIDDEN, HIDDEN, 1, 1, 0, (int)rows, HIDDEN);
    o.nseg = 1; o.bias = P + t->b2; o.out = t->Oh.p; o.ldo = t->ldp; o.act = tik::ACT_NONE;
    o.ksplit = tik::splitk_for(o, 64, 64, 16, 64);
    o.partial = t->partf.p;
    HIP_TRY(tik::launch_cgemm(o, tik::CFG_H64x64, st, tik::PREC_F32));
    // MSE loss (PoseLosses, pose_trainer.py:42-50) and its gradient
    HIP_TRY(tik::launch_mse(t->Oh.p, t->ldp, target, rows, t->pose_dim, t->dOh.p, loss_out, st));
    // head backward
    if ((rc = colsum(t, t->dOh.p, rows, t->ldp, t->tS.p, st))) return rc;
    HIP_TRY(hipMemcpyAsync(Gd + t->b2, t->tS.p, t->pose_dim * sizeof(float), hipMemcpyDeviceToDevice, st));
    if ((rc = wgrad(t, t->dOh.p, t->ldp, t->Dh.p, HIDDEN, t->pose_dim, HIDDEN, rows, Gd + t->w2, HIDDEN, st))) return rc;
    tik::CgemmArgs d{};
    d.M = (int)rows; d.Nc = HIDDEN; d.V = 1; d.tout = (int)rows;
    d.seg[0] = seg32(t->dOh.p, t->w2b.p, t->ldp, t->ldp, 1, 1, 0, (int)rows, t->ldp);
    d.nseg = 1; d.out = t->dD.p; d.ldo = HIDDEN; d.act = tik::ACT_NONE;
    d.ksplit = tik::splitk_for(d, 64, 64, 16, 64);
    d.partial = t->partf.p;
    HIP_TRY(tik::launch_cgemm(d, tik::CFG_H64x64, st, tik::PREC_F32));
    HIP_TRY(tik::launch_leaky_dropout_bwd(t->dD.p, t->dD.p, t->Ph.p, mask, scale, rows * HIDDEN, st));
    if ((rc = colsum(t, t->dD.p, rows, HIDDEN, Gd + t->b1, st))) return rc;
    if ((rc = wgrad(t, t->dD.p, HIDDEN, feat, t->feat, HIDDEN, t->feat, rows, Gd + t->w1, t->feat, st))) return rc;
    float* gOut = t->gA.p;
    float* gIn = t->gB.p;
    tik::CgemmArgs f{};
    f.M = (int)rows; f.Nc = t->feat; f.V = 1; f.tout = (int)rows;
    f.seg[0] = seg32(t->dD.p, t->w1b.p, HIDDEN, HIDDEN, 1, 1, 0, (int)rows, HIDDEN);
    f.nseg = 1; f.out = gOut; f.ldo = t->feat; f.act = tik::ACT_NONE;
    if ((rc = gemm(f, st))) return rc;
    // backbone backward
    for (int i = (int)t->L.size() - 1; i >= 0; --i) {
        TLayer& l = t->L[i];
        const float* Xi = i > 0 ? t->L[i - 1].O.p : t->x0.p;
        const int ldi = i > 0 ? t->L[i - 1].cout : 4;
        if ((rc = backward_block(t, l, Xi, ldi, gOut, gIn, st))) return rc;
        static const bool dbg = getenv("TIK_TRAIN_DEBUG") != nullptr;
        if (dbg) {
            t->dbg_dx.resize(t->L.size());
            const size_t n = (size_t)N * l.tin * V * ldi;
            if ((rc = t->dbg_dx[i].reserve(n))) return rc;
            HIP_TRY(hipMemcpyAsync(t->dbg_dx[i].p, gIn, n * sizeof(float), hipMemcpyDeviceToDevice, st));
        }
        std::swap(gOut, gIn);
    }
    // data_bn gamma / beta gradients (no input gradient: x is data)
    if ((rc = bn_back(t, gOut, t->x4.p, R0, 4 * V, t->cmap0.p, t->dg, t->db, t->st0.p, nullptr, st))) return rc;
    // Adam
    t->steps += 1;
    const double bc1 = 1.0 - std::pow((double)t->beta1, (double)t->steps);
    const double bc2 = 1.0 - std::pow((double)t->beta2, (double)t->steps);
    HIP_TRY(tik::launch_adam(P, Gd, t->M.p, t->Vv.p, t->np, t->lr, t->beta1, t->beta2, t->eps, bc1, bc2, st));
    return derive(t, st);
}

}  // namespace

extern "C" {

int tik_trainer_create(const tik_tensor* tensors, int n_tensors, float lr, tik_trainer_t* out) {
    if (!tensors || n_tensors <= 0 || !out || !(lr > 0.f)) return fail(TIK_E_INVALID, "tik_trainer_create: bad arguments");
    *out = nullptr;
    const TensorMap m = to_map(tensors, n_tensors);
    auto* t = new tik_trainer();
    t->lr = lr;
    std::vector<float> hp, hb;
    int rc = TIK_OK;
    auto fin = [&](int r) {
        if (r) delete t;
        return r;
    };
    const HostTensor* strides = find(m, "tik.strides");
    if (!strides) return fin(fail(TIK_E_MISSING, "tik_trainer_create: missing 'tik.strides'"));
    const std::string bb = "backbone.";
    if ((rc = add_entry(t, m, bb + "data_bn.weight", 0, &t->dg, hp, hb)) ||
        (rc = add_entry(t, m, bb + "data_bn.bias", 0, &t->db, hp, hb)) ||
        (rc = add_entry(t, m, bb + "data_bn.running_mean", 1, &t->rm0, hp, hb)) ||
        (rc = add_entry(t, m, bb + "data_bn.running_var", 1, &t->rv0, hp, hb)) ||
        (rc = add_entry(t, m, bb + "A", 1, &t->A, hp, hb)))
        return fin(rc);
    if (find(m, bb + "data_bn.weight")->v.size() != 3 * V || find(m, bb + "A")->v.size() != V * V)
        return fin(fail(TIK_E_INVALID, "tik_trainer_create: expected 17 joints x 3 channels and a (1,17,17) A"));
    const int nl = (int)strides->v.size();
    int cin = 3;
    for (int i = 0; i < nl; ++i) {
        const std::string p = bb + "st_gcn_networks." + std::to_string(i) + ".";
        const HostTensor* wg = shape_of(m, p + "gcn.conv.weight");
        if (!wg || wg->shape.size() < 2) return fin(fail(TIK_E_MISSING, "tik_trainer_create: missing '%sgcn.conv.weight'", p.c_str()));
        TLayer l;
        l.cin = cin;
        l.cinp = round4(cin);
        l.cout = (int)wg->shape[0];
        l.stride = (int)strides->v[i];
        if (wg->shape[1] != cin || l.cout % 4 || l.cout > 256 || l.stride < 1)
            return fin(fail(TIK_E_INVALID, "tik_trainer_create: layer %d: gcn weight (%lld,%lld) vs %d input channels", i,
                            (long long)wg->shape[0], (long long)wg->shape[1], cin));
        l.res = find(m, p + "residual.0.weight") ? RES_C : RES_I;
        if (l.res == RES_I && (cin != l.cout || l.stride != 1))
            return fin(fail(TIK_E_INVALID, "tik_trainer_create: layer %d: identity residual needs cin == cout, stride 1", i));
        if ((rc = add_entry(t, m, p + "gcn.conv.weight", 0, &l.wg, hp, hb)) ||
            (rc = add_entry(t, m, p + "gcn.conv.bias", 0, &l.bg, hp, hb)) ||
            (rc = add_entry(t, m, p + "tcn.0.weight", 0, &l.g1, hp, hb)) ||
            (rc = add_entry(t, m, p + "tcn.0.bias", 0, &l.b1, hp, hb)) ||
            (rc = add_entry(t, m, p + "tcn.0.running_mean", 1, &l.rm1, hp, hb)) ||
            (rc = add_entry(t, m, p + "tcn.0.running_var", 1, &l.rv1, hp, hb)) ||
            (rc = add_entry(t, m, p + "tcn.2.weight", 0, &l.wt, hp, hb)) ||
            (rc = add_entry(t, m, p + "tcn.2.bias", 0, &l.bt, hp, hb)) ||
            (rc = add_entry(t, m, p + "tcn.3.weight", 0, &l.g2, hp, hb)) ||
            (rc = add_entry(t, m, p + "tcn.3.bias", 0, &l.b2, hp, hb)) ||
            (rc = add_entry(t, m, p + "tcn.3.running_mean", 1, &l.rm2, hp, hb)) ||
            (rc = add_entry(t, m, p + "tcn.3.running_var", 1, &l.rv2, hp, hb)))
            return fin(rc);
        if (find(m, p + "tcn.2.weight")->v.size() != (size_t)l.cout * l.cout * 3)
            return fin(fail(TIK_E_INVALID, "tik_trainer_create: layer %d: tcn.2.weight must be (%d,%d,3,1)", i, l.cout, l.cout));
        if (l.res == RES_C &&
            ((rc = add_entry(t, m, p + "residual.0.weight", 0, &l.wr, hp, hb)) ||
             (rc = add_entry(t, m, p + "residual.0.bias", 0, &l.br, hp, hb)) ||
             (rc = add_entry(t, m, p + "residual.1.weight", 0, &l.g3, hp, hb)) ||
             (rc = add_entry(t, m, p + "residual.1.bias", 0, &l.b3, hp, hb)) ||
             (rc = add_entry(t, m, p + "residual.1.running_mean", 1, &l.rm3, hp, hb)) ||
             (rc = add_entry(t, m, p + "residual.1.running_var", 1, &l.rv3, hp, hb))))
            return fin(rc);
        cin = l.cout;
        t->L.push_back(std::move(l));
    }
    for (int i = 0; i < nl; ++i)
        if ((rc = add_entry(t, m, bb + "edge_importance." + std::to_string(i), 0, &t->L[i].E, hp, hb))) return fin(rc);
    if ((rc = add_entry(t, m, "pose_regressor.0.weight", 0, &t->w1, hp, hb)) ||
        (rc = add_entry(t, m, "pose_regressor.0.bias", 0, &t->b1, hp, hb)) ||
        (rc = add_entry(t, m, "pose_regressor.3.weight", 0, &t->w2, hp, hb)) ||
        (rc = add_entry(t, m, "pose_regressor.3.bias", 0, &t->b2, hp, hb)))
        return fin(rc);
    const HostTensor* W1 = find(m, "pose_regressor.0.weight");
    const HostTensor* W2 = find(m, "pose_regressor.3.weight");
    t->feat = V * cin;
    t->pose_dim = (int)W2->shape[0];
    t->ldp = round4(t->pose_dim);
    if (W1->shape[0] != HIDDEN || W1->shape[1] != t->feat || W2->shape[1] != HIDDEN)
        return fin(fail(TIK_E_INVALID, "tik_trainer_create: head shapes (%lld,%lld),(%lld,%lld) vs feature %d",
                        (long long)W1->shape[0], (long long)W1->shape[1], (long long)W2->shape[0],
                        (long long)W2->shape[1], t->feat));
    t->np = (long long)hp.size();
    t->nb = (long long)hb.size();
    std::vector<float> zeros(hp.size(), 0.f);
    if ((rc = t->P.upload(hp)) || (rc = t->B.upload(hb)) || (rc = t->G.upload(zeros)) || (rc = t->M.upload(zeros)) ||
        (rc = t->Vv.upload(zeros)))
        return fin(rc);
    std::vector<int> cm(4 * V);
    for (int c = 0; c < 4 * V; ++c) cm[c] = (c % 4 < 3) ? (c / 4) * 3 + c % 4 : -1;
    if ((rc = t->cmap0.upload(cm))) return fin(rc);
    int kmax = 4 * V;
    for (TLayer& l : t->L) {
        kmax = std::max(kmax, l.cout);
        std::vector<float> zf((size_t)l.cout * l.cinp, 0.f);
        if ((rc = l.wgf.upload(zf)) || (rc = l.wgb.reserve((size_t)l.cin * l.cout)) ||
            (rc = l.wtf.reserve(3ULL * l.cout * l.cout)) || (rc = l.wtb.reserve(3ULL * l.cout * l.cout)) ||
            (rc = l.aeff.reserve(V * V)) || (rc = l.st1.reserve(4 * l.cout)) || (rc = l.st2.reserve(4 * l.cout)) ||
            (rc = l.st3.reserve(4 * l.cout)))
            return fin(rc);
        if (l.res == RES_C && ((rc = l.wrf.upload(zf)) || (rc = l.wrb.reserve((size_t)l.cin * l.cout)))) return fin(rc);
    }
    std::vector<float> zw2((size_t)HIDDEN * t->ldp, 0.f);
    if ((rc = t->w1b.reserve((size_t)t->feat * HIDDEN)) || (rc = t->w2b.upload(zw2)) || (rc = t->st0.reserve(4 * 4 * V)) ||
        (rc = t->k.reserve(3 * kmax)) || (rc = t->loss.reserve(1)))
        return fin(rc);
    if ((rc = derive(t, nullptr))) return fin(rc);
    HIP_TRY(hipDeviceSynchronize());
    *out = t;
    return TIK_OK;
}

int tik_trainer_destroy(tik_trainer_t t) {
    if (t) {
        (void)hipDeviceSynchronize();
        delete t;
    }
    return TIK_OK;
}

int tik_trainer_step(tik_trainer_t t, const float* x, int N, int T, const float* target, const float* dropout_mask,
                     unsigned long long seed, float* loss, void* stream) {
    if (!t || !x || !target || N <= 0 || T <= 0) return fail(TIK_E_INVALID, "tik_trainer_step: bad arguments");
    // every float4 launcher indexes rows x channels / 4 in 32 bits: check the widest
    // activation up front, before any kernel updates running statistics
    int maxc = 4;
    for (const TLayer& l : t->L) maxc = std::max(maxc, std::max(l.cinp, l.cout));
    if ((long long)N * T * V * maxc / 4 > (1LL << 31) - 1 || (long long)N * T * V * 4 > (1LL << 31) - 1)
        return fail(TIK_E_INVALID, "tik_trainer_step: batch of %d x %d frames too large", N, T);
    if (N * T < 2) return fail(TIK_E_INVALID, "tik_trainer_step: BatchNorm needs more than one value per channel");
    hipStream_t st = (hipStream_t)stream;
    int rc = step(t, x, N, T, target, dropout_mask, seed, loss ? loss : t->loss.p, st);
    return rc;
}

int tik_trainer_out_frames(tik_trainer_t t, int T) {
    if (!t || T <= 0) return fail(TIK_E_INVALID, "tik_trainer_out_frames: bad arguments");
    for (const TLayer& l : t->L) T = (T - 1) / l.stride + 1;
    return T;
}

int tik_trainer_count(tik_trainer_t t) {
    if (!t) return fail(TIK_E_INVALID, "tik_trainer_count: null handle");
    return (int)t->ents.size();
}

int tik_trainer_tensor(tik_trainer_t t, int i, char* name, int name_len, int64_t* shape4, int* ndim, int* kind) {
    if (!t || i < 0 || i >= (int)t->ents.size()) return fail(TIK_E_INVALID, "tik_trainer_tensor: bad index");
    const TEntry& e = t->ents[i];
    if (name && name_len > 0) snprintf(name, (size_t)name_len, "%s", e.name.c_str());
    if (ndim) *ndim = (int)e.shape.size();
    if (shape4)
        for (size_t d = 0; d < e.shape.size() && d < 4; ++d) shape4[d] = e.shape[d];
    if (kind) *kind = e.kind;
    return TIK_OK;
}

// what: 0 value, 1 gradient of the last step, 2 Adam exp_avg, 3 Adam exp_avg_sq (parameters only)
int tik_trainer_read(tik_trainer_t t, int i, int what, float* dst, void* stream) {
    if (!t || i < 0 || i >= (int)t->ents.size() || !dst || what < 0 || what > 3)
        return fail(TIK_E_INVALID, "tik_trainer_read: bad arguments");
    const TEntry& e = t->ents[i];
    if (e.kind == 1 && what != 0) return fail(TIK_E_INVALID, "tik_trainer_read: '%s' is a buffer", e.name.c_str());
    const float* base = e.kind == 1 ? t->B.p : (what == 0 ? t->P.p : what == 1 ? t->G.p : what == 2 ? t->M.p : t->Vv.p);
    HIP_TRY(hipMemcpyAsync(dst, base + e.off, e.numel * sizeof(float), hipMemcpyDeviceToDevice, (hipStream_t)stream));
    return TIK_OK;
}

long long tik_trainer_steps(tik_trainer_t t) { return t ? t->steps : -1; }

// Debug / test hook on the last step's saved state: which = 0 block `layer`'s
// output, 2 its tcn conv output U, 3 its ReLU(BN(mix)) H, 4 the mix output Z,
// 5 the gcn conv output Y (channels-last rows), 6 the head's first Linear
// output; 1 the block's input gradient and 10..14 its gS (identity-residual blocks),
// dU, dH (before the ReLU backward, which is folded into the BatchNorm pass), dZ, dY
// (recorded with TIK_TRAIN_DEBUG=1 / TIK_TRAIN_DEBUG_LAYER=l). Copies
// min(n, size) floats to the device pointer dst.
int tik_trainer_debug(tik_trainer_t t, int which, int layer, float* dst, long long n, void* stream) {
    if (!t || layer < 0 || layer >= (int)t->L.size() || !dst || n < 0) return fail(TIK_E_INVALID, "tik_trainer_debug: bad arguments");
    const TLayer& l = t->L[layer];
    const DevBuf* b = which == 0 ? &l.O : which == 1 ? (layer < (int)t->dbg_dx.size() ? &t->dbg_dx[layer] : nullptr)
                    : which == 2 ? &l.U : which == 3 ? &l.H : which == 4 ? &l.Z : which == 5 ? &l.Y
                    : which == 6 ? &t->Ph
                    : (which >= 10 && which < 15) ? &t->dbg_b[which - 10] : nullptr;
    if (!b || !b->p) return fail(TIK_E_INVALID, "tik_trainer_debug: buffer not recorded");
    const size_t m = std::min<size_t>((size_t)n, b->n);
    HIP_TRY(hipMemcpyAsync(dst, b->p, m * sizeof(float), hipMemcpyDeviceToDevice, (hipStream_t)stream));
    return TIK_OK;
}

}  // extern "C"
