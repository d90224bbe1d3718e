// api.cpp — the C ABI of libtik.so (include/tik.h): weight folding/packing,
// handle-owned workspace, and the launch sequence of the IK forward pass.
//
// Forward of PoseRegressor (pose_trainer.py:94-133) on channels-last data:
//   xb  = data_bn(x)                                      st_gcn_aaai18.py:119-125
//   per block l (st_gcn_aaai18.py:208-214):
//     z   = ReLU( mix_A( x . Wg'^T ) + bias2[w][c] )      gcn + tcn.0 BN + ReLU (folded)
//     out = ReLU( sum_tap z[s t'+tap-1] . Wt'_tap^T + res + bT )   tcn.2 + tcn.3 BN + residual
//   feat = out_7 viewed (N*T', 17*256)                    st_gcn_aaai18.py:131-132
//   poses = (LeakyReLU(feat . W0^T + b0)) . W3^T + b3      pose_trainer.py:89-92
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/tik.h"
#include "cgemm.h"
#include "misc.h"
#include "online.h"
#include "common.h"
#include "xblock.h"
#include "xgemm.h"
#include "xgraph.h"
#include "xtws.h"

namespace tik_host {
thread_local std::string g_err;

bool guard_mode() {
    static const bool on = getenv("TIK_GUARD") && getenv("TIK_GUARD")[0] == '1';
    return on;
}
static std::mutex g_guard_mu;
static std::map<void*, size_t> g_guard_bufs;   // base -> payload bytes
void guard_register(void* base, size_t bytes) {
    std::lock_guard<std::mutex> l(g_guard_mu);
    g_guard_bufs[base] = bytes;
}
void guard_unregister(void* base) {
    std::lock_guard<std::mutex> l(g_guard_mu);
    g_guard_bufs.erase(base);
}
}
using namespace tik_host;

namespace {

int round4(int c) { return (c + 3) & ~3; }

tik::Seg mkseg(const float* src, const float* w, const SplitW3& s3, int cin, int ld, int kt, int stride, int pad,
               int tin, int ldw) {
    tik::Seg s{src, w, cin, ld, kt, stride, pad, tin, ldw};
    s.cin8 = s3.cin8; s.ldw8 = s3.ldw8;
    for (int i = 0; i < 3; ++i) s.wb[i] = s3.p[i].p;
    return s;
}

// eval BatchNorm -> (scale, shift)
int bn_fold(const TensorMap& m, const std::string& pre, int C, std::vector<float>& sc, std::vector<float>& sh) {
    const HostTensor* g = find(m, pre + ".weight");
    const HostTensor* b = find(m, pre + ".bias");
    const HostTensor* mu = find(m, pre + ".running_mean");
    const HostTensor* var = find(m, pre + ".running_var");
    if (!g || !b || !mu || !var) return fail(TIK_E_MISSING, "missing BatchNorm tensors under '%s'", pre.c_str());
    if ((int)g->v.size() != C || (int)b->v.size() != C || (int)mu->v.size() != C || (int)var->v.size() != C)
        return fail(TIK_E_INVALID, "BatchNorm '%s' expects %d channels", pre.c_str(), C);
    sc.resize(C);
    sh.resize(C);
    for (int c = 0; c < C; ++c) {
        const double s = (double)g->v[c] / std::sqrt((double)var->v[c] + (double)BN_EPS);
        sc[c] = (float)s;
        sh[c] = (float)((double)b->v[c] - (double)mu->v[c] * s);
    }
    return TIK_OK;
}

enum ResKind { RES_ZERO = 0, RES_IDEN = 1, RES_CONV = 2 };

// debug (TIK_X_TRACE=1): launch an xgemm with per-workgroup phase stamps and
// print the averages (s_memtime cycles) to stderr; synchronizes the stream
hipError_t launch_xgemm_traced(tik::XArgs a, int bn, int epi, hipStream_t st, const char* label) {
    static const bool on = getenv("TIK_X_TRACE") != nullptr;
    if (!on) return tik::launch_xgemm(a, bn, epi, st);
    const int rt = tik::xgemm_tile_rows(epi, a.nw);
    const long long nwg = (long long)((a.M + rt - 1) / rt) * ((a.Nc + bn - 1) / bn);
    unsigned long long* d = nullptr;
    hipError_t e = hipMalloc(&d, nwg * 8 * 8);
    if (e != hipSuccess) return e;
    (void)hipMemset(d, 0, nwg * 8 * 8);
    a.trace = d;
    e = tik::launch_xgemm(a, bn, epi, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    std::vector<unsigned long long> h(nwg * 8);
    if (e == hipSuccess) e = hipMemcpy(h.data(), d, h.size() * 8, hipMemcpyDeviceToHost);
    (void)hipFree(d);
    double s[6] = {0, 0, 0, 0, 0, 0}, n = 0, ks = 0;
    for (long long w = 0; w < nwg; ++w) {
        if (!h[8 * w + 7]) continue;
        n += 1; ks = (double)h[8 * w + 6];
        for (int k = 0; k < 6; ++k) s[k] += (double)h[8 * w + k];
    }
    n = std::max(1.0, n);
    fprintf(stderr, "XTRACE %-10s wg %6.0f ksteps %3.0f | cycles/wg: prologue %7.0f main %8.0f iden %6.0f epi %7.0f | "
            "barrier %7.0f vmwait %7.0f | main/kstep %6.0f\n", label, n, ks, s[0] / n, s[1] / n, s[2] / n, s[3] / n,
            s[4] / n, s[5] / n, s[1] / n / std::max(1.0, ks));
    return e;
}

thread_local Profiler* g_prof = nullptr;   // set for the duration of a profiled call

// debug (TIK_CHECKSUM=1): after every annotated launch, synchronise and
// record a checksum of its output buffer (tik_debug_checksums)
static bool checksum_mode() {
    static const bool on = getenv("TIK_CHECKSUM") != nullptr;
    return on;
}
static std::string g_cks;
static unsigned long long* g_cks_dev = nullptr;

struct ProfScope {
    int i;
    hipStream_t st;
    const char* lab;
    const void* op = nullptr;
    size_t obytes = 0;
    void out(const void* p, size_t bytes) { op = p; obytes = bytes; }
    ProfScope(const char* label, double flops, double bytes, hipStream_t s) : st(s), lab(label) {
        i = g_prof ? g_prof->begin(label, flops, bytes, s) : -1;
    }
    ~ProfScope() {
        if (g_prof) g_prof->end(i, st);
        if (checksum_mode() && op) {
            if (!g_cks_dev) (void)hipMalloc(&g_cks_dev, 8);
            unsigned long long h = 0;
            (void)hipMemsetAsync(g_cks_dev, 0, 8, st);
            (void)tik::launch_checksum(op, obytes, g_cks_dev, st);
            (void)hipMemcpyAsync(&h, g_cks_dev, 8, hipMemcpyDeviceToHost, st);
            (void)hipStreamSynchronize(st);
            char b[160];
            snprintf(b, sizeof(b), "%s:%llx;", lab, h);
            g_cks += b;
        }
    }
};

// One StGcnBlock with BN folded into packed fp32 weights.
static hipError_t launch_xgraph_traced(tik::XGraphArgs a, int ncu, hipStream_t st, const char* label) {
    static const bool on = getenv("TIK_X_TRACE") != nullptr;
    if (!on) return tik::launch_xgraph(a, ncu, st);
    unsigned long long* d = nullptr;
    hipError_t e = hipMalloc(&d, (size_t)ncu * 16 * 8);
    if (e != hipSuccess) return e;
    (void)hipMemset(d, 0, (size_t)ncu * 16 * 8);
    a.trace = d;
    e = tik::launch_xgraph(a, ncu, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    std::vector<unsigned long long> h((size_t)ncu * 16);
    if (e == hipSuccess) e = hipMemcpy(h.data(), d, h.size() * 8, hipMemcpyDeviceToHost);
    (void)hipFree(d);
    double s0[8] = {0}, s4[8] = {0}, n = 0;
    for (int w = 0; w < ncu; ++w) {
        if (!h[16 * w + 6]) continue;
        n += 1;
        for (int k = 0; k < 8; ++k) { s0[k] += (double)h[16 * w + k]; s4[k] += (double)h[16 * w + 8 + k]; }
    }
    const double ns = std::max(1.0, s0[6]);
    fprintf(stderr, "XGTRACE %-8s wgs %4.0f steps/wg %5.1f total/wg %8.0f | per step, wave0: bar %6.0f mfma0-3 %6.0f split %6.0f load %6.0f mfma4-16 %6.0f epi %6.0f"
            " | wave4: bar %6.0f mfma0-3 %6.0f split %6.0f load %6.0f mfma4-16 %6.0f epi %6.0f\n", label, n, s0[6] / std::max(1.0, n),
            s0[7] / std::max(1.0, n), s0[0] / ns, s0[1] / ns, s0[2] / ns, s0[3] / ns, s0[4] / ns, s0[5] / ns, s4[0] / ns, s4[1] / ns,
            s4[2] / ns, s4[3] / ns, s4[4] / ns, s4[5] / ns);
    return e;
}

struct Layer {
    int cin = 0, cinp = 0, cout = 0, stride = 1, res = RES_IDEN, V = 17, index = 0;
    DevBuf wg;      // [cout][cinp]          gcn conv scaled by tcn.0 BN
    DevBuf bias2;   // [V][cout]             sc1*bg*colsum(A)[w] + sh1
    DevBuf amix;    // [V][V]                A_eff[v][w]
    DevBuf wt;      // [cout][3*cout]        tcn conv scaled by tcn.3 BN, k = tap*cout + ci
    DevBuf wr;      // [cout][cinp]          residual conv scaled by residual.1 BN
    DevBuf biasT;   // [cout]                tcn bias (+ residual bias) folded
    SplitW3 s3g, s3t, s3r;  // bf16 planes p0+p1+p2 of wg, wt, wr (cgemm.hip: tik_stgcn_block_fwd, small batches)
    DevBuf wr0;             // [cout][cin] residual conv for a raw-input first layer (cin <= 4)
    DevHBuf xg, xt;         // bf16x3 tiles of the gcn (cin % 32 == 0) and of tcn (+ residual conv) (xgemm.hip)
    DevHBuf xtw;            // weight-stationary temporal conv (xtws.hip, 128 -> 128, stride 1, identity residual)
    DevHBuf xgw;            // weight-stationary gcn kernel (xgraph.hip, 128 / 256 output channels): gcn planes in the MFMA register layout
    DevHBuf xbg, xbt;       // whole-block kernel (xblock.hip, 64 channels, stride 1): gcn / tcn planes in the MFMA register layout
    int xg_bn = 0, xt_bn = 0, xg_ks = 0, xt_ks = 0;
    int xgwon = 1;          // gcn on xgraph.hip where packed (TIK_XGW bit mask of layers; 0 = the XG tiles)
    int xtwson = 1;         // temporal conv on xtws.hip where packed (TIK_XTWS bit mask of layers; 0 = XT128)
    int xfgon = 1;          // the next block's gcn inside this block's xtws launch where possible (TIK_XFG bit mask)
    float* xtrash = nullptr;   // store target of rows past M (persistent kernel), owned by the model
    bool mix_sparse = false;

    int build(const TensorMap& m, const std::string& pre, int cin_, int cout_, int stride_, int residual,
              const std::vector<float>& A_eff, int V_) {
        cin = cin_; cout = cout_; stride = stride_; V = V_;
        cinp = round4(cin);
        if (cout % 4 != 0) return fail(TIK_E_INVALID, "out_channels must be a multiple of 4 (got %d)", cout);
        res = !residual ? RES_ZERO : ((cin == cout && stride == 1) ? RES_IDEN : RES_CONV);
        const HostTensor* Wg = find(m, pre + "gcn.conv.weight");
        const HostTensor* bg = find(m, pre + "gcn.conv.bias");
        if (!Wg) return fail(TIK_E_MISSING, "missing '%sgcn.conv.weight'", pre.c_str());
        if ((int64_t)Wg->v.size() != (int64_t)cout * cin)
            return fail(TIK_E_INVALID, "'%sgcn.conv.weight' must be (%d,%d,1,1) (spatial kernel K=1 only)", pre.c_str(), cout, cin);
        std::vector<float> sc1, sh1, sc2, sh2;
        int rc;
        if ((rc = bn_fold(m, pre + "tcn.0", cout, sc1, sh1))) return rc;
        if ((rc = bn_fold(m, pre + "tcn.3", cout, sc2, sh2))) return rc;
        std::vector<double> colsum(V, 0.0);
        for (int v = 0; v < V; ++v)
            for (int w = 0; w < V; ++w) colsum[w] += A_eff[v * V + w];
        std::vector<float> hwg((size_t)cout * cinp, 0.f), hb2((size_t)V * cout);
        for (int co = 0; co < cout; ++co)
            for (int ci = 0; ci < cin; ++ci) hwg[(size_t)co * cinp + ci] = sc1[co] * Wg->v[(size_t)co * cin + ci];
        for (int w = 0; w < V; ++w)
            for (int co = 0; co < cout; ++co) {
                const double b = bg ? bg->v[co] : 0.0;
                hb2[(size_t)w * cout + co] = (float)((double)sc1[co] * b * colsum[w] + sh1[co]);
            }
        const HostTensor* Wt = find(m, pre + "tcn.2.weight");
        const HostTensor* bt = find(m, pre + "tcn.2.bias");
        if (!Wt) return fail(TIK_E_MISSING, "missing '%stcn.2.weight'", pre.c_str());
        if ((int64_t)Wt->v.size() != (int64_t)cout * cout * TK)
            return fail(TIK_E_INVALID, "'%stcn.2.weight' must be (%d,%d,3,1)", pre.c_str(), cout, cout);
        std::vector<float> hwt((size_t)cout * TK * cout), hbt(cout);
        for (int co = 0; co < cout; ++co) {
            for (int tap = 0; tap < TK; ++tap)
                for (int ci = 0; ci < cout; ++ci)
                    hwt[(size_t)co * TK * cout + tap * cout + ci] = sc2[co] * Wt->v[((size_t)co * cout + ci) * TK + tap];
            hbt[co] = (float)((double)sc2[co] * (bt ? bt->v[co] : 0.0) + sh2[co]);
        }
        std::vector<float> wr_host;   // folded residual conv [cout][cinp] (RES_CONV)
        if (res == RES_CONV) {
            const HostTensor* Wr = find(m, pre + "residual.0.weight");
            const HostTensor* br = find(m, pre + "residual.0.bias");
            if (!Wr) return fail(TIK_E_MISSING, "missing '%sresidual.0.weight'", pre.c_str());
            if ((int64_t)Wr->v.size() != (int64_t)cout * cin)
                return fail(TIK_E_INVALID, "'%sresidual.0.weight' must be (%d,%d,1,1)", pre.c_str(), cout, cin);
            std::vector<float> scr, shr;
            if ((rc = bn_fold(m, pre + "residual.1", cout, scr, shr))) return rc;
            std::vector<float> hwr((size_t)cout * cinp, 0.f);
            for (int co = 0; co < cout; ++co) {
                for (int ci = 0; ci < cin; ++ci) hwr[(size_t)co * cinp + ci] = scr[co] * Wr->v[(size_t)co * cin + ci];
                hbt[co] += (float)((double)scr[co] * (br ? br->v[co] : 0.0) + shr[co]);
            }
            wr_host = hwr;
            if ((rc = wr.upload(hwr)) || (rc = s3r.build(hwr, cout, 1, cinp, cinp)))
                return rc;
            if (cin <= 4) {
                std::vector<float> h0((size_t)cout * cin);
                for (int co = 0; co < cout; ++co)
                    for (int ci = 0; ci < cin; ++ci) h0[(size_t)co * cin + ci] = hwr[(size_t)co * cinp + ci];
                if ((rc = wr0.upload(h0))) return rc;
            }
        }
        {   // bf16x3 tiles for xgemm.hip
            const int bn = cout >= 128 ? 128 : 64;
            if (cin % 32 == 0) {
                const tik::XPackSeg g{hwg.data(), cinp, 1, cin};
                if ((rc = xg.upload(tik::xgemm_pack(&g, 1, cout, bn)))) return rc;
                xg_bn = bn; xg_ks = cin / 32;
            }
            if (cout % 32 == 0) {
                tik::XPackSeg t[2] = {{hwt.data(), TK * cout, TK, cout}, {wr_host.data(), cinp, 1, cin}};
                const int ns = (res == RES_CONV && cin % 32 == 0) ? 2 : 1;
                if ((rc = xt.upload(tik::xgemm_pack(t, ns, cout, bn)))) return rc;
                xt_bn = bn; xt_ks = TK * cout / 32 + (ns == 2 ? cin / 32 : 0);
            }
            if (cout == 128 && cin == 128 && stride == 1 && res == RES_IDEN && V == 17)   // xtws.hip
                if ((rc = xtw.upload(tik::xblock_pack_weights(hwt.data(), cout, TK * cout, TK, cout)))) return rc;
            if ((cout == 128 || cout == 256) && (cin == 64 || cin == 128 || cin == 256) && V == 17)   // xgraph.hip
                if ((rc = xgw.upload(tik::xblock_pack_weights(hwg.data(), cout, cinp, 1, cin)))) return rc;
            if (cout == 64 && stride == 1 && V == 17) {   // xblock.hip
                if ((rc = xbt.upload(tik::xblock_pack_weights(hwt.data(), cout, TK * cout, TK, cout)))) return rc;
                if (cin == 64 && (rc = xbg.upload(tik::xblock_pack_weights(hwg.data(), cout, cinp, 1, cin)))) return rc;
            }
        }
        std::vector<float> ha(A_eff.begin(), A_eff.end());
        mix_sparse = tik::fits_coco_hop2(ha.data(), V);
        if ((rc = wg.upload(hwg)) || (rc = bias2.upload(hb2)) || (rc = amix.upload(ha)) || (rc = wt.upload(hwt)) ||
            (rc = biasT.upload(hbt)) || (rc = s3g.build(hwg, cout, 1, cinp, cinp)) ||
            (rc = s3t.build(hwt, cout, TK, cout, TK * cout)))
            return rc;
        return TIK_OK;
    }

    static int tout(int tin, int s) { return (tin - 1) / s + 1; }   // kt=3, pad=1

    // x: rows (N*tin*V) of ld floats (>= cinp, %4); z: workspace N*tin*V*cout;
    // out: rows (N*tout*V) of cout floats.
    int forward(const float* x, int ld, int N, int tin, float* z, float* out, hipStream_t st, int prec,
                float* part = nullptr) const {
        const int to = tout(tin, stride);
        tik::CgemmArgs g{};
        g.M = N * tin * V; g.Nc = cout; g.V = V; g.tout = tin;
        g.seg[0] = mkseg(x, wg.p, s3g, cinp, ld, 1, 1, 0, tin, cinp);
        g.nseg = 1;
        g.bias = bias2.p; g.out = z; g.ldo = cout; g.amix = amix.p; g.act = tik::ACT_RELU;
        g.mix_sparse = mix_sparse ? 1 : 0;
        const double px_in = (double)N * tin * V, px_out = (double)N * to * V;
        {
            const std::string lab = "G272x64.L" + std::to_string(index);
            ProfScope p(lab.c_str(), 2.0 * px_in * cin * cout + 2.0 * V * px_in * cout,
                        4.0 * (px_in * cin + px_in * cout + (double)cout * cin + (double)V * (V + cout)), st);
            HIP_TRY(tik::launch_cgemm(g, tik::CFG_G272x64, st, prec));
        }

        tik::CgemmArgs t{};
        t.M = N * to * V; t.Nc = cout; t.V = V; t.tout = to;
        t.seg[0] = mkseg(z, wt.p, s3t, cout, cout, TK, stride, 1, tin, TK * cout);
        t.nseg = 1;
        if (res == RES_CONV) {
            t.seg[1] = mkseg(x, wr.p, s3r, cinp, ld, 1, stride, 0, tin, cinp);
            t.nseg = 2;
        } else if (res == RES_IDEN) {
            t.resid = x; t.ldr = ld;
        }
        t.bias = biasT.p; t.out = out; t.ldo = cout; t.act = tik::ACT_RELU;
        const bool big = cout >= 128;
        double fl = 2.0 * px_out * TK * cout * cout, by = 4.0 * (px_in * cout + px_out * cout + (double)TK * cout * cout);
        if (res == RES_CONV) { fl += 2.0 * px_out * cin * cout; by += 4.0 * (px_out * cin + (double)cin * cout); }
        if (res == RES_IDEN) by += 4.0 * px_out * cout;
        {
            // 64-channel layers: 256x64 tiles for fp32; 128x64 for bf16x3 (two register
            // staging sets of a 256-row tile would cost a wave per SIMD)
            const int cfg = big ? tik::CFG_T128x128 : (prec == tik::PREC_F32 ? tik::CFG_T256x64 : tik::CFG_T128x64);
            const std::string lab = std::string(big ? "T128x128.L" : (cfg == tik::CFG_T256x64 ? "T256x64.L" : "T128x64.L")) +
                                    std::to_string(index);
            if (part) {   // small batches: split K over more workgroups (latency path)
                t.ksplit = tik::splitk_for(t, cfg == tik::CFG_T256x64 ? 256 : 128, big ? 128 : 64,
                                           prec == tik::PREC_F32 ? 16 : 32, 64);
                t.partial = part;
            }
            ProfScope p(lab.c_str(), fl, by, st);
            HIP_TRY(tik::launch_cgemm(t, cfg, st, prec));
        }
        return TIK_OK;
    }

    bool x_ok() const { return xt.p && (xg.p || (index == 0 && cin <= 4 && res == RES_CONV && wr0.p)); }

    // the temporal conv runs on xtws.hip (input rows x of ld floats, tin frames per window)
    bool xtws_path(bool raw, int ld, int tin) const {
        return xtwson && xtw.p && xtrash && !raw && res == RES_IDEN && stride == 1 && ld >= cout && ld % 4 == 0 && tin % 8 == 0;
    }
    // block `nx`'s spatial half can run inside this block's xtws launch (xtws.hip FG:
    // 128 -> 128 gcn planes on xgraph.hip's layout; TIK_XFG bit mask of this layer)
    bool fuses_gcn_of(const Layer& nx) const {
        return xfgon && xtw.p && nx.xgwon && nx.xgw.p && nx.cin == cout && cout == 128 && nx.cout == 128 && nx.V == 17;
    }

    // bf16x3 on fp32 activations (xgemm.hip). x: fp32 rows [N*tin*V][ld];
    // z: workspace; out: [N*tout*V][cout]. Layer 0 from the raw keypoints
    // (cin <= 4): xraw = (N,T,V,C0) keypoints, its data_bn'd copy goes to xb4
    // ([rows][4]) for the residual conv in the temporal conv's epilogue.
    //
    // zin: this block's z, already made by the previous block's fused launch (no G
    // launch here); gn / zn: the next block, whose z this block's xtws launch makes
    // into zn (fuses_gcn_of(*gn) and xtws_path; the caller checks both)
    int forward_x(const float* x, int ld, int N, int tin, float* z, float* out, hipStream_t st, int ncu,
                  const float* xraw = nullptr, const float* bn_sc = nullptr, const float* bn_sh = nullptr,
                  float* xb4 = nullptr, const float* zin = nullptr, const Layer* gn = nullptr, float* zn = nullptr) const {
        const int to = tout(tin, stride);
        const long long rin = (long long)N * tin * V, rout = (long long)N * to * V;
        const double px_in = (double)rin, px_out = (double)rout;
        if (zin) {
            z = const_cast<float*>(zin);
        } else if (xraw) {
            ProfScope p("G0f_raw.L0", 2.0 * px_in * cin * cout + 2.0 * V * px_in * cout, 4.0 * (px_in * cin + px_in * cout), st);
            HIP_TRY(tik::launch_gcn0_f32(xraw, (int)rin, V, cin, bn_sc, bn_sh, wg.p, cinp, bias2.p, amix.p, mix_sparse ? 1 : 0,
                                         cout, z, cout, xb4, st));
        } else if (xgwon && xgw.p && xtrash) {
            tik::XGraphArgs g{};
            g.nframes = N * tin; g.x = x; g.ldx = ld; g.cin = cin; g.cout = cout; g.wp = xgw.p;
            g.bias2 = bias2.p; g.amix = amix.p; g.mix_sparse = mix_sparse ? 1 : 0; g.out = z; g.ldo = cout;
            g.nts = 1; g.trash = xtrash;
            const std::string lab = "XGW.L" + std::to_string(index);
            ProfScope p(lab.c_str(), 2.0 * px_in * cin * cout + 2.0 * V * px_in * cout,
                        4.0 * (px_in * cin + px_in * cout + (double)cout * cin + (double)V * (V + cout)), st);
            p.out(z, (size_t)rin * cout * 4);
            HIP_TRY(launch_xgraph_traced(g, ncu, st, lab.c_str()));
        } else {
            tik::XArgs g{};
            g.M = (int)rin; g.Nc = cout; g.V = V; g.tout = tin;
            g.seg[0] = tik::XSeg{x, ld, cin, 1, 1, 0, tin, rin};
            g.nseg = 1; g.wp = xg.p; g.ksteps = xg_ks;
            g.bias = bias2.p; g.amix = amix.p; g.mix_sparse = mix_sparse ? 1 : 0; g.out = z; g.ldo = cout; g.act = tik::ACT_RELU;
            g.nw = 4; g.nts = 1;
            const std::string lab = std::string(xg_bn == 128 ? "XG128.L" : "XG64.L") + std::to_string(index);
            ProfScope p(lab.c_str(), 2.0 * px_in * cin * cout + 2.0 * V * px_in * cout,
                        4.0 * (px_in * cin + px_in * cout + (double)cout * cin + (double)V * (V + cout)), st);
            p.out(z, (size_t)rin * cout * 4);
            HIP_TRY(launch_xgemm_traced(g, xg_bn, tik::EPI_GRAPH, st, lab.c_str()));
        }
        if (xtws_path(xraw != nullptr, ld, tin)) {
            tik::XTConvArgs c{};
            c.M = (int)rout; c.T = tin; c.z = z; c.ldz = cout; c.x = x; c.ldx = ld; c.wp = xtw.p; c.bias = biasT.p;
            c.out = out; c.ldo = cout; c.nts = 1; c.trash = xtrash;
            double fl = 2.0 * px_out * TK * cout * cout, by = 4.0 * (px_in * cout + 2.0 * px_out * cout + (double)TK * cout * cout);
            if (gn) {   // + block l+1's gcn: its algorithmic FLOPs, its z written (out is not re-read)
                c.wg = gn->xgw.p; c.bias2 = gn->bias2.p; c.amix = gn->amix.p; c.mix_sparse = gn->mix_sparse ? 1 : 0;
                c.zout = zn; c.ldzo = gn->cout;
                fl += 2.0 * px_out * gn->cin * gn->cout + 2.0 * V * px_out * gn->cout;
                by += 4.0 * (px_out * gn->cout + (double)gn->cout * gn->cin + (double)V * (V + gn->cout));
            }
            const std::string lab = (gn ? "XTWG.L" : "XTW.L") + std::to_string(index);
            ProfScope p(lab.c_str(), fl, by, st);
            p.out(out, (size_t)rout * cout * 4);
            HIP_TRY(tik::launch_xtws(c, ncu, st));
            return TIK_OK;
        }
        tik::XArgs t{};
        t.M = (int)rout; t.Nc = cout; t.V = V; t.tout = to;
        t.seg[0] = tik::XSeg{z, cout, cout, TK, stride, 1, tin, rin};
        t.nseg = 1;
        double fl = 2.0 * px_out * TK * cout * cout, by = 4.0 * (px_in * cout + px_out * cout + (double)TK * cout * cout);
        if (xraw) {
            t.rx = xb4; t.rxc = cin; t.rw = wr0.p;
            fl += 2.0 * px_out * cin * cout; by += 4.0 * px_out * 4;
        } else if (res == RES_CONV) {
            t.seg[1] = tik::XSeg{x, ld, cin, 1, stride, 0, tin, rin};
            t.nseg = 2;
            fl += 2.0 * px_out * cin * cout; by += 4.0 * (px_out * cin + (double)cin * cout);
        } else if (res == RES_IDEN) {
            t.idn = tik::XSeg{x, ld, cin, 1, 1, 0, to, rin};
            by += 4.0 * px_out * cout;
        }
        t.wp = xt.p; t.ksteps = tik::xgemm_ksteps(t);
        if (tik::xgemm_kmain(t) != xt_ks) return fail(TIK_E_INVALID, "layer %d: xgemm K steps %d != packed %d", index, tik::xgemm_kmain(t), xt_ks);
        t.bias = biasT.p; t.out = out; t.ldo = cout; t.act = tik::ACT_RELU;
        t.nw = 4; t.epi_lds = 1; t.idn_epi = 1; t.nts = 1;
        t.trash = xtrash;
        // the 64-column temporal convs (6 K steps per tile) on the persistent kernel: it hides
        // the first-DMA prologue that is a large share of such short tiles
        const bool pt = xt_bn == 64 && xtrash && cout % xt_bn == 0;
        const std::string lab = std::string(xt_bn == 128 ? (pt ? "XP128.L" : "XT128.L") : (pt ? "XP64.L" : "XT64.L")) +
                                std::to_string(index);
        ProfScope p(lab.c_str(), fl, by, st);
        p.out(out, (size_t)rout * cout * 4);
        if (pt) {
            t.trash = xtrash;
            HIP_TRY(tik::launch_xgemm_pt(t, xt_bn, ncu, st));
        } else {
            HIP_TRY(launch_xgemm_traced(t, xt_bn, tik::EPI_BIAS, st, lab.c_str()));
        }
        return TIK_OK;
    }
};

}  // namespace

// ----------------------------------------------------------------------------
struct tik_model {
    int V = 17, C0 = 3, feat = 0, hidden = 0, pose_dim = 0;
    std::vector<Layer> layers;
    DevBuf bn_sc, bn_sh;           // data_bn (V*C0)
    DevBuf w0, b0, w3, b3;         // head
    SplitW3 s30, s33;
    DevHBuf xh0;                   // bf16x3 tiles of pose_regressor.0 for xgemm.hip (feat % 32 == 0)
    int xhead_ks = 4;              // xgemm head: K slices, fixed so a window's poses do not depend on the batch size
    int prec = 2;
    // ws[0]: the handle's workspace; ws[1] + a private stream: large batches run
    // as two parts on two streams, so one part's HBM-bound launches run beside
    // the other's MFMA-bound ones. Online-IK streams own their workspaces (stream.cpp).
    static constexpr int MAXSPLIT = 2;
    Workspace ws[MAXSPLIT];
    hipStream_t aux[MAXSPLIT - 1] = {};
    hipEvent_t ev_fork = nullptr, ev_join[MAXSPLIT - 1] = {};
    bool split = true;                 // TIK_SPLIT=0: one stream
    int nsplit = 2;                    // parts of a split batch
    std::atomic<int> refs{1};          // the handle + every live online-IK stream
    ~tik_model() {
        if (ev_fork) (void)hipEventDestroy(ev_fork);
        for (auto e : ev_join) if (e) (void)hipEventDestroy(e);
        for (auto a : aux) if (a) (void)hipStreamDestroy(a);
    }
    int x_chunk_max = 0;               // test hook (TIK_X_CHUNK): cap on windows per sub-batch
    bool xblk = true;                  // blocks 0 and 1 as whole-block kernels (xblock.hip; TIK_XBLK=0: layered G + T)
    int ncu = 256;                     // compute units (persistent grids)
    DevHBuf trash;                     // scratch line for the persistent kernels' stores of invalid rows
    Profiler prof;
    bool profiling = false;
};

struct ProfGuard {
    ProfGuard(tik_model* m) { g_prof = (m && m->profiling) ? &m->prof : nullptr; }
    ~ProfGuard() { g_prof = nullptr; }
};

struct tik_block {
    Layer layer;
    DevBuf xp, z;   // padded-input and z workspace
    int prec = 2;
};

// handle settings read from the environment (each selects a test-pinned
// alternative of the default path) and the device facts the launches need;
// the same for full and backbone-only handles
static void apply_env(tik_model* md) {
    if (const char* e = getenv("TIK_X_CHUNK")) md->x_chunk_max = atoi(e);
    if (const char* e = getenv("TIK_XBLK")) md->xblk = e[0] != '0';
    int dev = 0, ncu = 0;
    if (hipGetDevice(&dev) == hipSuccess && hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && ncu > 0)
        md->ncu = ncu;
    for (auto& L : md->layers) {
        if (const char* w = getenv("TIK_XGW")) L.xgwon = (atoi(w) >> L.index) & 1;
        if (const char* w = getenv("TIK_XTWS")) L.xtwson = (atoi(w) >> L.index) & 1;
        if (const char* w = getenv("TIK_XFG")) L.xfgon = (atoi(w) >> L.index) & 1;
        L.xtrash = reinterpret_cast<float*>(md->trash.p);
    }
    if (const char* e = getenv("TIK_SPLIT")) md->split = e[0] != '0';
}

extern "C" {

const char* tik_last_error(void) { return g_err.c_str(); }

int tik_debug_checksums(char* buf, int len) {
    if (!checksum_mode()) return fail(TIK_E_INVALID, "TIK_CHECKSUM is not set");
    const int n = (int)g_cks.size();
    if (buf && len > 0) {
        strncpy(buf, g_cks.c_str(), len - 1);
        buf[len - 1] = 0;
    }
    g_cks.clear();
    return n;
}

int tik_debug_check_guards(void) {
    if (!guard_mode()) return fail(TIK_E_INVALID, "TIK_GUARD=1 is not set");
    HIP_TRY(hipDeviceSynchronize());
    std::lock_guard<std::mutex> l(g_guard_mu);
    std::vector<unsigned char> h(GUARD_BYTES);
    int bad = 0;
    std::string rep;
    for (const auto& kv : g_guard_bufs) {
        const char* base = static_cast<const char*>(kv.first);
        for (int side = 0; side < 2; ++side) {
            const char* gp = side == 0 ? base : base + GUARD_BYTES + kv.second;
            HIP_TRY(hipMemcpy(h.data(), gp, GUARD_BYTES, hipMemcpyDeviceToHost));
            size_t first = GUARD_BYTES, last = 0, cnt = 0;
            for (size_t i = 0; i < GUARD_BYTES; ++i)
                if (h[i] != 0xA5) { first = std::min(first, i); last = i; ++cnt; }
            if (cnt) {
                ++bad;
                char b[256];
                snprintf(b, sizeof(b), "[buf %p payload %zu B: %s guard, %zu bytes changed at +%zu..+%zu] ", (const void*)(base + GUARD_BYTES),
                         kv.second, side == 0 ? "front" : "back", cnt, first, last);
                rep += b;
                HIP_TRY(hipMemset(const_cast<char*>(gp), 0xA5, GUARD_BYTES));
            }
        }
    }
    g_err = rep;
    return bad;
}
const char* tik_version(void) { return "tik 0.4.0 (gfx950; bf16x3 split MFMA (default, fp32 range), exact fp32 MFMA)"; }

int tik_model_create(const tik_tensor* tensors, int n_tensors, tik_model_t* out) {
    if (!tensors || n_tensors <= 0 || !out) return fail(TIK_E_INVALID, "tik_model_create: null argument");
    *out = nullptr;
    TensorMap m = to_map(tensors, n_tensors);
    const HostTensor* A = find(m, "backbone.A");
    if (!A) return fail(TIK_E_MISSING, "missing 'backbone.A'");
    if (A->shape.size() != 3 || A->shape[1] != A->shape[2])
        return fail(TIK_E_INVALID, "'backbone.A' must be (K,V,V)");
    if (A->shape[0] != 1) return fail(TIK_E_INVALID, "only the 'uniform' graph strategy (K=1) is supported by the fused path");
    auto* md = new tik_model();
    md->V = (int)A->shape[1];
    if (md->V != 17) { delete md; return fail(TIK_E_INVALID, "fused path is built for V=17 (coco), got %d", (int)A->shape[1]); }
    const int V = md->V;
    int rc;
    // data_bn
    {
        std::vector<float> sc, sh;
        const HostTensor* g = find(m, "backbone.data_bn.weight");
        if (!g) { delete md; return fail(TIK_E_MISSING, "missing 'backbone.data_bn.weight'"); }
        md->C0 = (int)g->v.size() / V;
        if (md->C0 * V != (int)g->v.size() || md->C0 > 4) { delete md; return fail(TIK_E_INVALID, "data_bn size %zu not V*C (C<=4)", g->v.size()); }
        if ((rc = bn_fold(m, "backbone.data_bn", V * md->C0, sc, sh))) { delete md; return rc; }
        if ((rc = md->bn_sc.upload(sc)) || (rc = md->bn_sh.upload(sh))) { delete md; return rc; }
    }
    int cin = md->C0;
    for (int l = 0;; ++l) {
        const std::string pre = "backbone.st_gcn_networks." + std::to_string(l) + ".";
        const HostTensor* Wg = find(m, pre + "gcn.conv.weight");
        if (!Wg) break;
        const int cout = (int)Wg->shape[0];
        if ((int)Wg->shape[1] != cin) { delete md; return fail(TIK_E_INVALID, "layer %d: in_channels %d != previous out %d", l, (int)Wg->shape[1], cin); }
        // Temporal strides are architecture, not weights: the IK config of
        // pose_trainer.py:76-83 unless the caller passes a "tik.strides" tensor.
        static const int ik_strides[8] = {1, 1, 2, 1, 1, 2, 2, 2};
        int stride = l < 8 ? ik_strides[l] : 1;
        if (const HostTensor* s = find(m, "tik.strides")) {
            if (l >= (int)s->v.size()) { delete md; return fail(TIK_E_INVALID, "'tik.strides' has no entry for layer %d", l); }
            stride = (int)s->v[l];
        }
        const HostTensor* Wr = find(m, pre + "residual.0.weight");
        if ((Wr != nullptr) != (cin != cout || stride != 1)) {
            delete md;
            return fail(TIK_E_INVALID, "layer %d: residual conv presence does not match (cin=%d, cout=%d, stride=%d)", l, cin, cout, stride);
        }
        const HostTensor* imp = find(m, "backbone.edge_importance." + std::to_string(l));
        std::vector<float> Ae(V * V);
        for (int i = 0; i < V * V; ++i) Ae[i] = A->v[i] * (imp ? imp->v[i] : 1.0f);
        md->layers.emplace_back();
        md->layers.back().index = l;
        if ((rc = md->layers.back().build(m, pre, cin, cout, stride, 1, Ae, V))) { delete md; return rc; }
        cin = cout;
    }
    if (md->layers.empty()) { delete md; return fail(TIK_E_MISSING, "no 'backbone.st_gcn_networks.*' layers"); }
    const HostTensor* W0 = find(m, "pose_regressor.0.weight");
    const HostTensor* B0 = find(m, "pose_regressor.0.bias");
    const HostTensor* W3 = find(m, "pose_regressor.3.weight");
    const HostTensor* B3 = find(m, "pose_regressor.3.bias");
    md->feat = V * cin;
    if ((rc = precision_from_env(md->prec))) { delete md; return rc; }
    if (!W0 && !B0 && !W3 && !B3) {
        // backbone-only handle (StgGcn18 state dict, st_gcn_aaai18.py:32-133):
        // tik_backbone_forward only; tik_ik_forward refuses it
        if ((rc = md->trash.upload(std::vector<unsigned short>(4096, 0)))) {
            delete md;
            return rc;
        }
        apply_env(md);
        *out = md;
        return TIK_OK;
    }
    if (!W0 || !B0 || !W3 || !B3) { delete md; return fail(TIK_E_MISSING, "missing pose_regressor.{0,3}.{weight,bias}"); }
    md->hidden = (int)W0->shape[0];
    md->pose_dim = (int)W3->shape[0];
    if ((int)W0->shape[1] != md->feat || (int)W3->shape[1] != md->hidden) { delete md; return fail(TIK_E_INVALID, "head shapes do not match backbone features %d", md->feat); }
    if (md->hidden % 4) { delete md; return fail(TIK_E_INVALID, "hidden size must be a multiple of 4"); }
    if ((rc = md->trash.upload(std::vector<unsigned short>(4096, 0)))) {
        delete md;
        return rc;
    }
    apply_env(md);
    if ((rc = md->w0.upload(W0->v)) || (rc = md->b0.upload(B0->v)) || (rc = md->w3.upload(W3->v)) || (rc = md->b3.upload(B3->v)) ||
        (rc = md->s30.build(W0->v, md->hidden, 1, md->feat, md->feat)) ||
        (rc = md->s33.build(W3->v, md->pose_dim, 1, md->hidden, md->hidden))) {
        delete md;
        return rc;
    }
    if (md->feat % 32 == 0) {
        const tik::XPackSeg h{W0->v.data(), md->feat, 1, md->feat};
        if ((rc = md->xh0.upload(tik::xgemm_pack(&h, 1, md->hidden, 128)))) { delete md; return rc; }
    }
    *out = md;
    return TIK_OK;
}

int tik_model_destroy(tik_model_t m) {
    if (m) model_release(m);   // freed now, or when its last online-IK stream is destroyed
    return TIK_OK;
}

int tik_model_out_frames(tik_model_t m, int T) {
    if (!m || T <= 0) return fail(TIK_E_INVALID, "bad model/T");
    for (const Layer& L : m->layers) T = Layer::tout(T, L.stride);
    return T;
}

}  // extern "C"

static bool use_xblk(const tik_model* m);

namespace tik_host {
// Bytes per pixel (frame x joint) of block 0's output when blocks 0 and 1 run
// whole (xblock.hip): 64 channels as three bf16 planes, written into the z
// workspace (blocks01_x), so z must hold N*T*V of them whatever the widths of
// the later layers.
constexpr size_t XB0_P3_FLOATS = 64 * 3 * 2 / 4;

int model_reserve_ws(tik_model* m, Workspace& w, int N, int T) {
    const size_t V = m->V;
    size_t zmax = 0, amax = 0;
    int t = T;
    for (const Layer& L : m->layers) {
        zmax = std::max(zmax, (size_t)N * t * V * L.cout);
        t = Layer::tout(t, L.stride);
        amax = std::max(amax, (size_t)N * t * V * L.cout);
    }
    if (use_xblk(m)) zmax = std::max(zmax, (size_t)N * T * V * XB0_P3_FLOATS);
    // the second z buffer: the next block's z made inside a fused xtws launch
    size_t z2max = 0;
    t = T;
    for (size_t l = 0; l + 1 < m->layers.size(); ++l) {
        const Layer& L = m->layers[l];
        t = Layer::tout(t, L.stride);
        if (L.index > 0 && L.stride == 1 && L.fuses_gcn_of(m->layers[l + 1])) z2max = std::max(z2max, (size_t)N * t * V * m->layers[l + 1].cout);
    }
    t = T;
    for (const Layer& L : m->layers) t = Layer::tout(t, L.stride);
    int rc;
    if (z2max && (rc = w.z2.reserve(z2max))) return rc;
    // split-K partials: ksplit * tiles <= 256 + 128 launches of <= 128x128 tiles
    // (cgemm), or up to 8 K slices of the xgemm head's hidden rows
    if ((rc = w.xb.reserve((size_t)N * T * V * 4)) || (rc = w.z.reserve(zmax)) ||
        (rc = w.a0.reserve(amax)) || (rc = w.a1.reserve(amax)) || (rc = w.hid.reserve((size_t)N * t * m->hidden)) ||
        (rc = w.part.reserve(std::max((size_t)384 * 128 * 128, (size_t)8 * N * t * m->hidden))))
        return rc;
    return TIK_OK;
}

void model_retain(tik_model* m) { m->refs.fetch_add(1); }
int model_pose_dim(const tik_model* m) { return m->pose_dim; }
void model_release(tik_model* m) {
    if (m->refs.fetch_sub(1) == 1) delete m;
}

int model_online_fill(tik_model* m, tik::OnlineArgs& a) {
    static_assert((int)tik::ONR_ZERO == RES_ZERO && (int)tik::ONR_IDEN == RES_IDEN && (int)tik::ONR_CONV == RES_CONV, "");
    const int nl = (int)m->layers.size();
    if (m->V != 17 || m->C0 != 3 || nl > tik::ONL_MAXL) return fail(TIK_E_INVALID, "online kernel: V=17, 3 input channels, <= %d layers", tik::ONL_MAXL);
    if (m->pose_dim <= 0) return fail(TIK_E_INVALID, "online kernel: backbone-only handle (no pose_regressor weights)");
    a.nl = nl;
    for (int l = 0; l < nl; ++l) {
        const Layer& L = m->layers[l];
        if (L.cout % 16 || L.cout > tik::ONL_MAXC || L.cinp > tik::ONL_MAXC || (l > 0 && L.cinp != L.cin))
            return fail(TIK_E_INVALID, "online kernel: layer %d channels %d -> %d", l, L.cin, L.cout);
        tik::OnlineLayer& o = a.L[l];
        o.cin = L.cin; o.cinp = L.cinp; o.cout = L.cout; o.stride = L.stride; o.res = L.res;
        o.wg = L.wg.p; o.bias2 = L.bias2.p; o.amix = L.amix.p; o.wt = L.wt.p; o.wr = L.wr.p; o.biasT = L.biasT.p;
    }
    if (m->feat % 4 || m->feat > tik::ONL_MAXHC * 256 || m->hidden % 16 || m->hidden > tik::ONL_MAXHC * 256 ||
        m->pose_dim > 256)   // head tasks: one thread per pose value, W3 columns in LDS
        return fail(TIK_E_INVALID, "online kernel: head %d -> %d", m->feat, m->hidden);
    a.w0 = m->w0.p; a.b0 = m->b0.p; a.w3 = m->w3.p; a.b3 = m->b3.p;
    a.feat = m->feat; a.hidden = m->hidden; a.pose_dim = m->pose_dim;
    a.bn_sc = m->bn_sc.p; a.bn_sh = m->bn_sh.p;
    return TIK_OK;
}
}  // namespace tik_host

extern "C" {

int tik_model_reserve(tik_model_t m, int N, int T) {
    if (!m || N <= 0 || T <= 0) return fail(TIK_E_INVALID, "tik_model_reserve: bad arguments");
    return model_reserve_ws(m, m->ws[0], N, T);
}

struct WsPtrs {
    float *xb, *z, *a0, *a1, *hid, *part;
    int ncu;   // persistent grids: the CUs this part runs on
    float* z2;   // the second z buffer of fused xtws launches (null: none reserved)
};
static WsPtrs ptrs_of(const Workspace& w, int ncu) {
    return WsPtrs{w.xb.p, w.z.p, w.a0.p, w.a1.p, w.hid.p, w.part.p, ncu, w.z2.n ? w.z2.p : nullptr};
}
// the workspaces and aux streams of the parts 1 .. np-1 of a split batch
static int reserve_parts(tik_model* m, int np, int N, int T) {
    int rc;
    if (!m->ev_fork) HIP_TRY(hipEventCreateWithFlags(&m->ev_fork, hipEventDisableTiming));
    for (int k = 1; k < np; ++k) {
        if ((rc = model_reserve_ws(m, m->ws[k], N, T))) return rc;
        if (!m->aux[k - 1]) {
            HIP_TRY(hipStreamCreateWithFlags(&m->aux[k - 1], hipStreamNonBlocking));
            HIP_TRY(hipEventCreateWithFlags(&m->ev_join[k - 1], hipEventDisableTiming));
        }
    }
    return TIK_OK;
}

// Backbone on fp32 activations (both precisions; split-K for small batches).
static int backbone(tik_model_t m, const float* x, int N, int T, float** feat_out, int* tout, hipStream_t st,
                    const WsPtrs& w) {
    const int V = m->V;
    {
        const double px = (double)N * T * V;
        ProfScope p("data_bn", 2.0 * px * m->C0, 4.0 * px * (m->C0 + 4), st);
        HIP_TRY(tik::launch_data_bn(x, N * T * V, V, m->C0, m->bn_sc.p, m->bn_sh.p, w.xb, st));
    }
    const float* cur = w.xb;
    int ld = 4, t = T, rc;
    float* bufs[2] = {w.a0, w.a1};
    int which = 0;
    for (const Layer& L : m->layers) {
        float* o = bufs[which];
        if ((rc = L.forward(cur, ld, N, t, w.z, o, st, m->prec, w.part))) return rc;
        cur = o; ld = L.cout; t = Layer::tout(t, L.stride); which ^= 1;
    }
    *feat_out = const_cast<float*>(cur);
    *tout = t;
    return TIK_OK;
}

static bool use_x(const tik_model* m) {
    if (m->prec != tik::PREC_BF16X3 || m->C0 > 4) return false;
    for (const Layer& L : m->layers)
        if (!L.x_ok() || (L.index == 0) != (L.cin <= 4)) return false;
    return true;
}

// Windows per xgemm call: every fp32 activation tensor the DMA reads stays
// below 2 GiB (32-bit buffer offsets), block 0's bf16x3-plane output of the
// whole-block path included.
static int x_chunk(const tik_model* m, int T) {
    long long worst = 1;
    int t = T;
    for (const Layer& L : m->layers) {
        worst = std::max(worst, (long long)t * m->V * L.cout * 4);   // z
        t = Layer::tout(t, L.stride);
        worst = std::max(worst, (long long)t * m->V * L.cout * 4);   // out
    }
    if (use_xblk(m)) worst = std::max(worst, (long long)T * m->V * (long long)(XB0_P3_FLOATS * 4));
    const long long lim = (1LL << 31) - (1LL << 20);
    const int c = (int)std::max(1LL, lim / worst);
    return m->x_chunk_max > 0 ? std::min(c, m->x_chunk_max) : c;
}

// Backbone on fp32 activations with the bf16x3 xgemm kernels. Layer 0 runs
// from the raw keypoints (data_bn folded into its gcn kernel).
// debug (TIK_X_TRACE=1 with a -DTIK_XTRACE build): per-phase sums of the whole-block kernels
static hipError_t launch_xblock_traced(tik::XBlkArgs a, bool raw, int ncu, hipStream_t st, const char* label) {
    static const bool on = getenv("TIK_X_TRACE") != nullptr;
    if (!on) return tik::launch_xblock(a, raw, ncu, st);
    unsigned long long* d = nullptr;
    hipError_t e = hipMalloc(&d, (size_t)ncu * 24 * 8);
    if (e != hipSuccess) return e;
    (void)hipMemset(d, 0, (size_t)ncu * 24 * 8);
    a.trace = d;
    e = tik::launch_xblock(a, raw, ncu, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    std::vector<unsigned long long> h((size_t)ncu * 24);
    if (e == hipSuccess) e = hipMemcpy(h.data(), d, h.size() * 8, hipMemcpyDeviceToHost);
    (void)hipFree(d);
    double s0[8] = {0}, s4[8] = {0}, nt = 0;
    for (int w = 0; w < ncu; ++w) {
        if (!h[24 * w + 9]) continue;
        nt += (double)h[24 * w + 8];
        for (int k = 0; k < 8; ++k) { s0[k] += (double)h[24 * w + k]; s4[k] += (double)h[24 * w + 12 + k]; }
    }
    nt = std::max(1.0, nt);
    fprintf(stderr, "XBTRACE %-8s tiles %6.0f | per tile, wave0: start %6.0f G+mix %6.0f zbar %6.0f res %6.0f bar+dma %6.0f T %6.0f endbar %6.0f"
            " | wave4: start %6.0f G+mix %6.0f zbar %6.0f res %6.0f bar+dma %6.0f T %6.0f endbar %6.0f\n", label, nt,
            s0[0] / nt, s0[1] / nt, s0[2] / nt, (s0[3] + s0[6]) / nt, s0[7] / nt, s0[4] / nt, s0[5] / nt, s4[0] / nt, s4[1] / nt,
            s4[2] / nt, (s4[3] + s4[6]) / nt, s4[7] / nt, s4[4] / nt, s4[5] / nt);
    return e;
}

static bool use_xblk(const tik_model* m) {
    if (!m->xblk || m->layers.size() < 2 || m->C0 > 4) return false;
    const Layer& L0 = m->layers[0];
    const Layer& L1 = m->layers[1];
    return L0.cout == 64 && L0.stride == 1 && L0.res == RES_CONV && L0.cin == m->C0 && L0.wr0.p && L0.xbt.p &&
           L1.cin == 64 && L1.cout == 64 && L1.stride == 1 && L1.res == RES_IDEN && L1.xbt.p && L1.xbg.p && m->V == 17;
}

// Blocks 0 and 1 as whole-block kernels (xblock.hip): block 0 from the raw
// keypoints writes its output as bf16x3 planes into the z workspace, block 1
// reads them and writes fp32 rows to `out`.
static int blocks01_x(tik_model_t m, const float* x, int N, int T, float* out, hipStream_t st, const WsPtrs& w) {
    const Layer& L0 = m->layers[0];
    const Layer& L1 = m->layers[1];
    const double px = (double)N * T * m->V;
    unsigned short* p3 = reinterpret_cast<unsigned short*>(w.z);
    tik::XBlkArgs b{};
    b.nframes = N * T; b.T = T;
    b.xraw = x; b.c0 = m->C0; b.bn_sc = m->bn_sc.p; b.bn_sh = m->bn_sh.p; b.wg0 = L0.wg.p; b.ldwg0 = L0.cinp; b.rw = L0.wr0.p;
    b.wtp = L0.xbt.p; b.bias2 = L0.bias2.p; b.amix = L0.amix.p; b.mix_sparse = L0.mix_sparse ? 1 : 0; b.bias = L0.biasT.p;
    b.out_p3 = p3; b.trash = L0.xtrash;
    {
        ProfScope p("XB0.L0", 2.0 * px * (L0.cin * 64 + 17 * 64) + 2.0 * px * (TK * 64 * 64 + L0.cin * 64), px * (4.0 * m->C0 + 384.0), st);
        p.out(p3, (size_t)px * 384);
        HIP_TRY(launch_xblock_traced(b, true, w.ncu, st, "XB0.L0"));
    }
    tik::XBlkArgs c{};
    c.nframes = N * T; c.T = T; c.xp3 = p3;
    c.wgp = L1.xbg.p; c.wtp = L1.xbt.p; c.bias2 = L1.bias2.p; c.amix = L1.amix.p; c.mix_sparse = L1.mix_sparse ? 1 : 0;
    c.bias = L1.biasT.p; c.out_f = out; c.trash = L1.xtrash;
    {
        ProfScope p("XB1.L1", 2.0 * px * (64 * 64 + 17 * 64) + 2.0 * px * TK * 64 * 64, px * (384.0 + 256.0), st);
        p.out(out, (size_t)px * 256);
        HIP_TRY(launch_xblock_traced(c, false, w.ncu, st, "XB1.L1"));
    }
    return TIK_OK;
}

static int backbone_x(tik_model_t m, const float* x, int N, int T, float** feat_out, int* tout, hipStream_t st,
                      const WsPtrs& w) {
    const float* cur = nullptr;
    int ld = 0, t = T, rc;
    float* bufs[2] = {w.a0, w.a1};
    int which = 0;
    const bool xblk = use_xblk(m);
    if (xblk) {
        if ((rc = blocks01_x(m, x, N, T, w.a1, st, w))) return rc;
        cur = w.a1; ld = 64;
    }
    // zin: the current block's z when the previous launch made it (xtws FG); the z
    // buffers alternate (w.z, w.z2), since a fused launch reads z(l) halo rows of
    // neighbouring tiles while it writes z(l+1)
    const float* zin = nullptr;
    float* zbuf[2] = {w.z, w.z2};
    int zw = 0;
    const int nl = (int)m->layers.size();
    for (int l = 0; l < nl; ++l) {
        const Layer& L = m->layers[l];
        if (xblk && L.index < 2) continue;
        float* o = bufs[which];
        const Layer* gn = nullptr;
        if (l + 1 < nl && w.z2 && L.index > 0 && L.xtws_path(false, ld, t) && L.fuses_gcn_of(m->layers[l + 1])) gn = &m->layers[l + 1];
        float* zc = zin ? const_cast<float*>(zin) : zbuf[zw];
        float* zn = zbuf[zc == zbuf[0] ? 1 : 0];
        if (L.index == 0) rc = L.forward_x(nullptr, 0, N, t, zc, o, st, w.ncu, x, m->bn_sc.p, m->bn_sh.p, w.xb);
        else rc = L.forward_x(cur, ld, N, t, zc, o, st, w.ncu, nullptr, nullptr, nullptr, nullptr, zin, gn, zn);
        if (rc) return rc;
        zin = gn ? zn : nullptr;
        zw = zc == zbuf[0] ? 0 : 1;
        cur = o; ld = L.cout; t = Layer::tout(t, L.stride); which ^= 1;
    }
    *feat_out = const_cast<float*>(cur);
    *tout = t;
    return TIK_OK;
}

int tik_backbone_forward(tik_model_t m, const float* x, int N, int T, float* feat, void* stream) {
    if (!m || !x || !feat || N <= 0 || T <= 0) return fail(TIK_E_INVALID, "tik_backbone_forward: bad arguments");
    hipStream_t st = (hipStream_t)stream;
    ProfGuard pg(m);
    int to, rc;
    if (use_x(m)) {
        const int chunk = std::min(N, x_chunk(m, T));
        if ((rc = tik_model_reserve(m, chunk, T))) return rc;
        for (int n0 = 0; n0 < N; n0 += chunk) {
            const int n = std::min(chunk, N - n0);
            float* f;
            if ((rc = backbone_x(m, x + (size_t)n0 * T * m->V * m->C0, n, T, &f, &to, st, ptrs_of(m->ws[0], m->ncu)))) return rc;
            HIP_TRY(hipMemcpyAsync(feat + (size_t)n0 * to * m->feat, f, sizeof(float) * (size_t)n * to * m->feat,
                                   hipMemcpyDeviceToDevice, st));
        }
        return TIK_OK;
    }
    if ((rc = tik_model_reserve(m, N, T))) return rc;
    float* f;
    if ((rc = backbone(m, x, N, T, &f, &to, st, ptrs_of(m->ws[0], m->ncu)))) return rc;
    HIP_TRY(hipMemcpyAsync(feat, f, sizeof(float) * (size_t)N * to * m->feat, hipMemcpyDeviceToDevice, st));
    return TIK_OK;
}

static int head3_splitk(tik_model_t m, const float* hid, int rows, float* poses, float* part, hipStream_t st, int ks = 0);

// Head on fp32 features with split-K (few rows: the K = 4352 loop spread over
// workgroups instead of run serially by the handful of row tiles).
static int head_splitk(tik_model_t m, const float* f, int rows, float* poses, float* hid, float* part, hipStream_t st) {
    tik::CgemmArgs h{};
    h.M = rows; h.Nc = m->hidden; h.V = 1; h.tout = rows;
    h.seg[0] = mkseg(f, m->w0.p, m->s30, m->feat, m->feat, 1, 1, 0, rows, m->feat);
    h.nseg = 1; h.bias = m->b0.p; h.out = hid; h.ldo = m->hidden; h.act = tik::ACT_LEAKY;
    h.ksplit = tik::splitk_for(h, 64, 64, m->prec == tik::PREC_F32 ? 16 : 32, 64);
    h.partial = part;
    {
        ProfScope pr("H64x64.head0", 2.0 * rows * m->feat * m->hidden,
                     4.0 * ((double)rows * (m->feat + m->hidden) + (double)m->feat * m->hidden), st);
        HIP_TRY(tik::launch_cgemm(h, tik::CFG_H64x64, st, m->prec));
    }
    return head3_splitk(m, hid, rows, poses, part, st);
}

// the head's second layer (hidden -> pose_dim, pose_trainer.py:92) with split-K
// (ks > 0: that many K slices whatever the row count)
static int head3_splitk(tik_model_t m, const float* hid, int rows, float* poses, float* part, hipStream_t st, int ks) {
    tik::CgemmArgs p{};
    p.M = rows; p.Nc = m->pose_dim; p.V = 1; p.tout = rows;
    p.seg[0] = mkseg(hid, m->w3.p, m->s33, m->hidden, m->hidden, 1, 1, 0, rows, m->hidden);
    p.nseg = 1; p.bias = m->b3.p; p.out = poses; p.ldo = m->pose_dim; p.act = tik::ACT_NONE;
    p.ksplit = ks > 0 ? ks : tik::splitk_for(p, 64, 64, m->prec == tik::PREC_F32 ? 16 : 32, 64);
    p.partial = part;
    {
        ProfScope pr("H64x64.head3", 2.0 * rows * m->hidden * m->pose_dim,
                     4.0 * ((double)rows * (m->hidden + m->pose_dim) + (double)m->hidden * m->pose_dim), st);
        HIP_TRY(tik::launch_cgemm(p, tik::CFG_H64x64, st, m->prec));
    }
    return TIK_OK;
}

// Head of the bf16x3 path: pose_regressor.0 (feat -> hidden, LeakyReLU,
// pose_trainer.py:89-91) on xgemm.hip, its K = feat loop split into a fixed
// number of slices (the frames are few: 4096 rows at B = 1024, 128 tiles) and
// the slices summed in a fixed order by the reduce kernel (+ bias, LeakyReLU);
// then pose_regressor.3 with split-K as head_splitk.
static int head_x(tik_model_t m, const float* f, int rows, float* poses, const WsPtrs& w, hipStream_t st) {
    if (!m->xh0.p || m->xhead_ks <= 0) return head_splitk(m, f, rows, poses, w.hid, w.part, st);
    tik::XArgs h{};
    h.M = rows; h.Nc = m->hidden; h.V = 1; h.tout = rows;
    h.seg[0] = tik::XSeg{f, m->feat, m->feat, 1, 1, 0, rows, rows};
    h.nseg = 1; h.wp = m->xh0.p; h.ksteps = tik::xgemm_ksteps(h);
    h.nw = 4; h.epi_lds = 1;
    {   // K slices: the fixed count (4: 512 workgroups at 4096 rows), each non-empty
        const int kper = (h.ksteps + m->xhead_ks - 1) / m->xhead_ks;
        h.ksplit = (h.ksteps + kper - 1) / kper;
    }
    if (h.ksplit > 1) {
        h.out = w.part; h.act = tik::ACT_NONE;
    } else {
        h.out = w.hid; h.bias = m->b0.p; h.act = tik::ACT_LEAKY;
    }
    h.ldo = m->hidden;
    {
        ProfScope pr("XH128.head0", 2.0 * rows * m->feat * m->hidden,
                     4.0 * ((double)rows * (m->feat + (double)h.ksplit * m->hidden) + (double)m->feat * m->hidden), st);
        HIP_TRY(tik::launch_xgemm(h, 128, tik::EPI_BIAS, st));
    }
    if (h.ksplit > 1) {
        ProfScope pr("XR.head0", (double)rows * m->hidden * h.ksplit, 4.0 * (double)rows * m->hidden * (h.ksplit + 1), st);
        HIP_TRY(tik::launch_xgemm_splitk_reduce(w.part, h.ksplit, rows, m->hidden, m->b0.p, tik::ACT_LEAKY, w.hid,
                                                m->hidden, st));
    }
    // pose_regressor.3: a fixed K split too (4 slices of 128), so no row's
    // arithmetic depends on the batch size
    return head3_splitk(m, w.hid, rows, poses, w.part, st, std::min(4, std::max(1, m->hidden / 128)));
}

}  // extern "C"

namespace tik_host {
int model_forward_ws(tik_model* m, const float* x, int N, int T, float* poses, hipStream_t st, Workspace& ws,
                     bool allow_split) {
    float* f;
    int to, rc;
    if (use_x(m)) {
        const int chunk = std::min(N, x_chunk(m, T));
        if ((rc = model_reserve_ws(m, ws, chunk, T))) return rc;
        const int To = tik_model_out_frames(m, T);
        // large batches: np parts on np streams (the caller's + handle-owned
        // ones, fork/join by events), so one part's HBM-bound graph launches
        // run beside another part's MFMA-bound temporal convs (not while
        // profiling: per-launch events would time overlapping kernels)
        const bool split = allow_split && m->split && !m->profiling && (long long)std::min(N, chunk) * T >= 32768 && N >= 2;
        const int np = split ? std::min(m->nsplit, std::min(N, chunk)) : 1;
        if (split && (rc = reserve_parts(m, np, (std::min(N, chunk) + np - 1) / np, T))) return rc;
        auto part = [&](const float* xs, int n, float* ps, hipStream_t s, const WsPtrs& w) -> int {
            float* fs;
            int r;
            if ((r = backbone_x(m, xs, n, T, &fs, &to, s, w))) return r;
            return head_x(m, fs, n * to, ps, w, s);
        };
        for (int n0 = 0; n0 < N; n0 += chunk) {
            const int n = std::min(chunk, N - n0);
            const float* xs = x + (size_t)n0 * T * m->V * m->C0;
            float* ps = poses + (size_t)n0 * To * m->pose_dim;
            if (split && n >= np && (long long)n * T >= 32768) {
                HIP_TRY(hipEventRecord(m->ev_fork, st));
                for (int k = 1; k < np; ++k) HIP_TRY(hipStreamWaitEvent(m->aux[k - 1], m->ev_fork, 0));
                for (int k = 0; k < np; ++k) {
                    const int a0 = (int)((long long)n * k / np), a1 = (int)((long long)n * (k + 1) / np);
                    if ((rc = part(xs + (size_t)a0 * T * m->V * m->C0, a1 - a0, ps + (size_t)a0 * To * m->pose_dim,
                                   k == 0 ? st : m->aux[k - 1], ptrs_of(k == 0 ? ws : m->ws[k], m->ncu))))
                        return rc;
                }
                for (int k = 1; k < np; ++k) {
                    HIP_TRY(hipEventRecord(m->ev_join[k - 1], m->aux[k - 1]));
                    HIP_TRY(hipStreamWaitEvent(st, m->ev_join[k - 1], 0));
                }
            } else if ((rc = part(xs, n, ps, st, ptrs_of(ws, m->ncu)))) {
                return rc;
            }
        }
        return TIK_OK;
    }
    if ((rc = model_reserve_ws(m, ws, N, T))) return rc;
    const WsPtrs w = ptrs_of(ws, m->ncu);
    if ((rc = backbone(m, x, N, T, &f, &to, st, w))) return rc;
    return head_splitk(m, f, N * to, poses, w.hid, w.part, st);
}
}  // namespace tik_host

extern "C" {

int tik_ik_forward(tik_model_t m, const float* x, int N, int T, float* poses, void* stream) {
    if (!m || !x || !poses || N <= 0 || T <= 0) return fail(TIK_E_INVALID, "tik_ik_forward: bad arguments");
    if (m->pose_dim <= 0) return fail(TIK_E_INVALID, "tik_ik_forward: backbone-only handle (no pose_regressor weights)");
    ProfGuard pg(m);
    return model_forward_ws(m, x, N, T, poses, (hipStream_t)stream, m->ws[0], true);
}

int tik_model_set_precision(tik_model_t m, int prec) {
    if (!m || (prec != tik::PREC_F32 && prec != tik::PREC_BF16X3))
        return fail(TIK_E_INVALID, "tik_model_set_precision: precision must be 0 (fp32) or 2 (bf16x3), got %d", prec);
    m->prec = prec;
    return TIK_OK;
}

int tik_model_get_precision(tik_model_t m) {
    if (!m) return fail(TIK_E_INVALID, "null model");
    return m->prec;
}

int tik_block_set_precision(tik_block_t b, int prec) {
    if (!b || (prec != tik::PREC_F32 && prec != tik::PREC_BF16X3))
        return fail(TIK_E_INVALID, "tik_block_set_precision: precision must be 0 (fp32) or 2 (bf16x3), got %d", prec);
    b->prec = prec;
    return TIK_OK;
}

int tik_model_profile(tik_model_t m, int max_launches) {
    if (!m || max_launches < 0) return fail(TIK_E_INVALID, "tik_model_profile: bad arguments");
    m->profiling = max_launches > 0;
    return max_launches > 0 ? m->prof.enable(max_launches) : (m->prof.clear(), TIK_OK);
}

int tik_model_profile_count(tik_model_t m) {
    if (!m) return fail(TIK_E_INVALID, "null model");
    return (int)m->prof.recs.size();
}

int tik_model_profile_read(tik_model_t m, int i, char* label, int label_len, float* ms, double* flops,
                           double* bytes) {
    if (!m) return fail(TIK_E_INVALID, "tik_model_profile_read: null model");
    return m->prof.read(i, label, label_len, ms, flops, bytes);
}

// ---------------------------------------------------------------------------- block API
int tik_block_create(const tik_tensor* tensors, int n_tensors, int in_channels, int out_channels, int stride,
                     int residual, const float* A_eff_host, int V, tik_block_t* out) {
    if (!tensors || !A_eff_host || !out || in_channels <= 0 || out_channels <= 0 || stride <= 0 || V <= 0)
        return fail(TIK_E_INVALID, "tik_block_create: bad arguments");
    if (V != 17) return fail(TIK_E_INVALID, "fused block kernel is built for V=17 (coco layout), got V=%d", V);
    TensorMap m = to_map(tensors, n_tensors);
    auto* b = new tik_block();
    std::vector<float> Ae(A_eff_host, A_eff_host + V * V);
    int rc = precision_from_env(b->prec);
    if (rc) { delete b; return rc; }
    rc = b->layer.build(m, "", in_channels, out_channels, stride, residual, Ae, V);
    if (rc) { delete b; return rc; }
    *out = b;
    return TIK_OK;
}

int tik_block_destroy(tik_block_t b) {
    delete b;
    return TIK_OK;
}

int tik_stgcn_block_fwd(tik_block_t b, const float* x, int N, int T, float* out, void* stream) {
    if (!b || !x || !out || N <= 0 || T <= 0) return fail(TIK_E_INVALID, "tik_stgcn_block_fwd: bad arguments");
    hipStream_t st = (hipStream_t)stream;
    const Layer& L = b->layer;
    const size_t rows = (size_t)N * T * L.V;
    int rc;
    const float* xin = x;
    if (L.cin != L.cinp) {
        if ((rc = b->xp.reserve(rows * L.cinp))) return rc;
        HIP_TRY(tik::launch_pad_channels(x, (long long)rows, L.cin, L.cinp, b->xp.p, st));
        xin = b->xp.p;
    }
    if ((rc = b->z.reserve(rows * L.cout))) return rc;
    return L.forward(xin, L.cinp, N, T, b->z.p, out, st, b->prec);
}

// ---------------------------------------------------------------------------- ops
int tik_gconv_fwd(const float* x, int N, int Cin, int T, int V, const float* A, int K, const float* W,
                  const float* b, int Cout, int t_kernel, int t_stride, int t_padding, int t_dilation, float* out,
                  void* stream) {
    if (!x || !A || !W || !out || N <= 0 || Cin <= 0 || T <= 0 || V <= 0 || K <= 0 || Cout <= 0 || t_kernel <= 0 ||
        t_stride <= 0 || t_padding < 0 || t_dilation <= 0)
        return fail(TIK_E_INVALID, "tik_gconv_fwd: bad arguments");
    const int To = (T + 2 * t_padding - t_dilation * (t_kernel - 1) - 1) / t_stride + 1;
    if (To <= 0) return fail(TIK_E_INVALID, "tik_gconv_fwd: empty temporal output");
    if ((size_t)K * Cout * V * sizeof(float) > 160 * 1024)
        return fail(TIK_E_INVALID, "tik_gconv_fwd: K*Cout*V=%d exceeds the per-frame LDS tile", K * Cout * V);
    HIP_TRY(tik::launch_gconv(x, N, Cin, T, V, A, K, W, b, Cout, t_kernel, t_stride, t_padding, t_dilation, To, out,
                              (hipStream_t)stream));
    return TIK_OK;
}

int tik_aa_to_rotmat(const float* aa, int n, float* R, void* stream) {
    if (!aa || !R || n < 0) return fail(TIK_E_INVALID, "tik_aa_to_rotmat: bad arguments");
    HIP_TRY(tik::launch_aa_to_rotmat(aa, n, R, (hipStream_t)stream));
    return TIK_OK;
}

int tik_moveai_to_coco(const float* joints, int F, int J, const int* map17_host, float* out, void* stream) {
    if (!joints || !map17_host || !out || F < 0 || J < 2) return fail(TIK_E_INVALID, "tik_moveai_to_coco: bad arguments");
    for (int c = 0; c < 17; ++c)
        if (map17_host[c] < -1 || map17_host[c] >= J)
            return fail(TIK_E_INVALID, "tik_moveai_to_coco: map entry %d = %d out of range for %d joints", c, map17_host[c], J);
    HIP_TRY(tik::launch_moveai_to_coco(joints, F, J, map17_host, out, (hipStream_t)stream));
    return TIK_OK;
}

int tik_window_gather(const float* seq, int F, int V, int idx0, int n_idx, int h, int root_a, int root_b,
                      int relative, float* windows, void* stream) {
    if (!seq || !windows || F <= 0 || V <= 0 || n_idx < 0 || h < 0 || idx0 < 0 || idx0 + n_idx > F)
        return fail(TIK_E_INVALID, "tik_window_gather: bad arguments");
    if (relative && (root_a < 0 || root_a >= V || root_b < 0 || root_b >= V))
        return fail(TIK_E_INVALID, "tik_window_gather: root joints out of range");
    // data_amass.py:27-29 raises when h > idx > F - h; a window that overruns
    // both ends of a short sequence comes back shorter than 2h+1 there.
    for (int i = idx0; i < idx0 + n_idx; ++i) {
        if (h > i && i > F - h)
            return fail(TIK_E_INVALID, "h_win_size > idx > arr.shape[0] - h_win_size: %d > %d > %d - %d", h, i, F, h);
        if (i - h < 0 && i + h > F - 1 && i <= F - h)
            return fail(TIK_E_INVALID, "window at idx %d overruns both ends (reference returns a short window)", i);
    }
    HIP_TRY(tik::launch_window_gather(seq, F, V, idx0, n_idx, h, root_a, root_b, relative, windows,
                                      (hipStream_t)stream));
    return TIK_OK;
}

}  // extern "C"
