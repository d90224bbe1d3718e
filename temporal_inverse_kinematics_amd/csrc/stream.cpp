// stream.cpp — online (stride-1 sliding-window) IK with a hipGraph-captured step
// (BASELINE.json config #5). The reference solves a recorded sequence offline,
// one window per frame (inference.run_inference, inference.py:37-67; windows
// from data_amass.py:18-42, 221-236). Online, frame c can be solved once frame
// c+h has arrived: each push of frame k runs the window centred at c = k-h
// (frames k-2h..k, left edge clamped like sample_window's edge padding) and
// returns pose row 0 of the model output, i.e. exactly run_inference's frame c.
// Flushing the last h frames = pushing the last frame h more times (right edge
// padding). Default step: ONE dataflow kernel (online.hip) that reads the
// frame from pinned host memory, appends it to the ring, computes only the
// frames pose row 0 depends on, and writes the pose to pinned host memory.
// Fallback step (TIK_ONLINE=0, or a model that kernel does not cover): ring
// append, window gather, the layered IK forward on the whole window, the pose
// copy. Either is one hipGraph replay on a private stream when use_graph.
#include <hip/hip_runtime.h>

#include "../../include/tik.h"
#include "common.h"
#include "misc.h"
#include "online.h"

#include <algorithm>
#include <chrono>
#include <cstring>

using namespace tik_host;

struct tik_stream {
    tik_model_t model = nullptr;   // retained: the handle may be destroyed first
    Workspace ws;                  // private: batch calls on the handle never touch it
    int h = 0, W = 0, V = 17, tout = 0, pose_dim = 66;
    hipStream_t st = nullptr;
    hipGraph_t graph = nullptr;
    hipGraphExec_t exec = nullptr;
    DevBuf ring, window, poses, frame_in, pose_out;
    DevIBuf count;
    float* host_frame = nullptr;   // pinned
    float* host_pose = nullptr;    // pinned; [pose_dim] = the online kernel's error flag
    volatile int* host_done = nullptr;   // pinned, coherent: the dataflow kernel's frame count after each step
    long long pushed = 0;
    int dcount = 0;                       // mirror of the device frame count (stream_next_count)
    // the dataflow step (online.hip)
    bool online = false;
    int onl_grid = 0;
    DevBuf onl_act;                       // every activation of the step
    DevIBuf onl_cnt;                      // completion counters, ticket, done, err
    DevArray<tik::OnlineArgs> onl_args;   // the kernel's argument block
    DevArray<unsigned long long> onl_trace;   // TIK_ONLINE_TRACE=1
    std::vector<DevHBuf> onl_wtp, onl_wgp;   // per layer: temporal conv / gcn weights as bf16x3 MFMA planes
    std::vector<DevBuf> onl_wtf, onl_wgf;    // per layer: the same, fp32, K zero-padded to 32
    int onl_ntasks = 0;
    ~tik_stream() {
        if (st) (void)hipStreamSynchronize(st);
        if (exec) (void)hipGraphExecDestroy(exec);
        if (graph) (void)hipGraphDestroy(graph);
        if (host_frame) (void)hipHostFree(host_frame);
        if (host_pose) (void)hipHostFree(host_pose);
        if (host_done) (void)hipHostFree(const_cast<int*>(host_done));
        if (st) (void)hipStreamDestroy(st);
        if (model) model_release(model);
    }
};

static int cu_count() {
    int dev = 0, c = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || c <= 0) return 256;
    return c;
}

// frames each layer must compute for pose row 0, buffers, task list (online.h)
static int setup_online(tik_stream* s) {
    tik::OnlineArgs a{};
    int rc = model_online_fill(s->model, a);
    if (rc) return rc;
    const int nl = a.nl;
    // the temporal conv tasks' weights (online.hip onl_tconv): K = [tap 0 | tap 1 | tap 2 |
    // residual conv] per output channel, zero-padded to steps of 32, as bf16x3 planes in the
    // MFMA B-operand lane layout and as fp32 rows
    s->onl_wtp.resize(nl); s->onl_wtf.resize(nl); s->onl_wgp.resize(nl); s->onl_wgf.resize(nl);
    // rows [cout][Kt] -> fp32 rows zero-padded to K32 steps of 32 + bf16x3 planes [cout/16][K32][3][64][8]
    auto pack = [](const std::vector<float>& w, int cout, int Kt, int K32, std::vector<float>& wf, std::vector<unsigned short>& wp) {
        wf.assign((size_t)cout * 32 * K32, 0.f);
        for (int co = 0; co < cout; ++co)
            for (int k = 0; k < Kt; ++k) wf[(size_t)co * 32 * K32 + k] = w[(size_t)co * Kt + k];
        wp.assign((size_t)(cout / 16) * K32 * 3 * 64 * 8, 0);
        for (int cg = 0; cg < cout / 16; ++cg)
            for (int sk = 0; sk < K32; ++sk)
                for (int ln = 0; ln < 64; ++ln)
                    for (int e = 0; e < 8; ++e) {
                        unsigned short h[3];
                        split_bf16x3(wf[(size_t)(16 * cg + (ln & 15)) * 32 * K32 + 32 * sk + 8 * (ln >> 4) + e], h[0], h[1], h[2]);
                        for (int pl = 0; pl < 3; ++pl) wp[((((size_t)cg * K32 + sk) * 3 + pl) * 64 + ln) * 8 + e] = h[pl];
                    }
    };
    for (int l = 0; l < nl; ++l) {
        tik::OnlineLayer& L = a.L[l];
        const int C = L.cout, cinp = L.cinp, rconv = L.res == tik::ONR_CONV;
        const int Kt = 3 * C + (rconv ? cinp : 0), K32 = (Kt + 31) / 32, G32 = (cinp + 31) / 32;
        std::vector<float> wt((size_t)C * 3 * C), wr(rconv ? (size_t)C * cinp : 0), wg((size_t)C * cinp), w((size_t)C * Kt), wf;
        std::vector<unsigned short> wp;
        HIP_TRY(hipMemcpy(wt.data(), L.wt, wt.size() * sizeof(float), hipMemcpyDeviceToHost));
        if (rconv) HIP_TRY(hipMemcpy(wr.data(), L.wr, wr.size() * sizeof(float), hipMemcpyDeviceToHost));
        HIP_TRY(hipMemcpy(wg.data(), L.wg, wg.size() * sizeof(float), hipMemcpyDeviceToHost));
        for (int co = 0; co < C; ++co)
            for (int k = 0; k < Kt; ++k) w[(size_t)co * Kt + k] = k < 3 * C ? wt[(size_t)co * 3 * C + k] : wr[(size_t)co * cinp + (k - 3 * C)];
        pack(w, C, Kt, K32, wf, wp);
        if ((rc = s->onl_wtp[l].upload(wp)) || (rc = s->onl_wtf[l].upload(wf))) return rc;
        L.k32 = K32; L.wtp = s->onl_wtp[l].p; L.wtf = s->onl_wtf[l].p;
        pack(wg, C, cinp, G32, wf, wp);
        if ((rc = s->onl_wgp[l].upload(wp)) || (rc = s->onl_wgf[l].upload(wf))) return rc;
        L.gk32 = G32; L.wgp = s->onl_wgp[l].p; L.wgf = s->onl_wgf[l].p;
    }
    int t = s->W;
    for (int l = 0; l < nl; ++l) {
        a.L[l].tin = t;
        t = (t - 1) / a.L[l].stride + 1;
    }
    int need = 1;   // the last layer's output frames: row 0
    for (int l = nl - 1; l >= 0; --l) {
        tik::OnlineLayer& L = a.L[l];
        L.n_out = need;
        L.n_in = std::min(L.tin, L.stride * (need - 1) + 2);
        need = L.n_in;
    }
    size_t tot = (size_t)(a.hidden / 16) * a.pose_dim + ((a.pose_dim + 3) & ~3);
    for (int l = 0; l < nl; ++l) tot += (size_t)(a.L[l].n_in + a.L[l].n_out) * 17 * a.L[l].cout;
    if ((rc = s->onl_act.reserve(tot))) return rc;
    float* q = s->onl_act.p;
    for (int l = 0; l < nl; ++l) {
        tik::OnlineLayer& L = a.L[l];
        L.x = l == 0 ? nullptr : a.L[l - 1].out;
        L.z = q; q += (size_t)L.n_in * 17 * L.cout;
        L.out = q; q += (size_t)L.n_out * 17 * L.cout;
    }
    a.hpart = q; q += (size_t)(a.hidden / 16) * a.pose_dim;
    a.pose = q;
    a.act = s->onl_act.p;
    a.act_bytes = (unsigned)(tot * sizeof(float));
    // every G / T output carries its launch's tag (online.hip): start at tag 1, for launch 0
    HIP_TRY(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(s->onl_act.p), (int)0x80000000u, s->onl_act.n, s->st));
    int np = 0, task = 0, cb = 0;
    auto add = [&](int kind, int layer, int nf, int ng) {
        a.ph[np++] = tik::OnlinePhase{kind, layer, nf, ng, task, cb};
        task += nf * ng;
        if (kind == tik::ONP_H) ++cb;   // the head's one counter (G / T hand over tagged data)
    };
    for (int l = 0; l < nl; ++l) {
        add(tik::ONP_G, l, a.L[l].n_in, a.L[l].cout / 16);
        add(tik::ONP_T, l, a.L[l].n_out, a.L[l].cout / 16);
    }
    add(tik::ONP_H, nl - 1, 1, a.hidden / 16);
    a.nph = np;
    a.ntasks = task;
    if ((rc = s->onl_cnt.reserve(cb + 3))) return rc;
    HIP_TRY(hipMemsetAsync(s->onl_cnt.p, 0, sizeof(int) * (cb + 3), s->st));
    // the initial tags and scheduling words are in place before the first step on this
    // (non-blocking) stream: the memsets ran on it, and the host waits here
    HIP_TRY(hipStreamSynchronize(s->st));
    a.cnt = s->onl_cnt.p; a.ncnt = cb;
    a.ticket = a.cnt + cb; a.done = a.cnt + cb + 1; a.err = a.cnt + cb + 2;
    a.ring = s->ring.p; a.W = s->W; a.h = s->h; a.ra = 11; a.rb = 12; a.relative = 1;
    a.count = s->count.p;
    void* dp = nullptr;
    HIP_TRY(hipHostGetDevicePointer(&dp, s->host_frame, 0));
    a.frame = static_cast<const float*>(dp);
    HIP_TRY(hipHostGetDevicePointer(&dp, s->host_pose, 0));
    a.pose_host = static_cast<float*>(dp);
    HIP_TRY(hipHostGetDevicePointer(&dp, const_cast<int*>(s->host_done), 0));
    a.done_host = static_cast<int*>(dp);
    a.trace = nullptr;
    if (const char* e = getenv("TIK_ONLINE_TRACE"); e && e[0] == '1') {
        if ((rc = s->onl_trace.reserve((size_t)8 * task))) return rc;
        a.trace = s->onl_trace.p;
    }
    s->onl_ntasks = task;
    if ((rc = s->onl_args.upload(std::vector<tik::OnlineArgs>{a}))) return rc;
    // one workgroup per CU (89 KB of LDS each). With per-frame counters half the CUs was best
    // (143 us at 128 vs 151 us at 256); with tagged data the wider grid wins: p50 81 us at 128,
    // 74 at 160, 70 at 192, 67 at 256 (profiles/r05_og_ab_online_grid.txt)
    int grid = std::max(1, cu_count());
    if (const char* e = getenv("TIK_ONLINE_GRID")) grid = std::max(1, std::min(cu_count(), atoi(e)));   // test hook
    s->onl_grid = grid;
    s->online = true;
    return TIK_OK;
}

static int record_step(tik_stream* s) {
    if (s->online) {
        HIP_TRY(tik::launch_online(s->onl_args.p, s->onl_grid, s->st));
        return TIK_OK;
    }
    HIP_TRY(hipMemcpyAsync(s->frame_in.p, s->host_frame, sizeof(float) * s->V * 3, hipMemcpyHostToDevice, s->st));
    HIP_TRY(tik::launch_stream_push(s->ring.p, s->W, s->V * 3, s->count.p, s->frame_in.p, s->st));
    HIP_TRY(tik::launch_stream_window(s->ring.p, s->W, s->V, s->count.p, s->h, 11, 12, 1, s->window.p, s->st));
    int rc = model_forward_ws(s->model, s->window.p, 1, s->W, s->poses.p, s->st, s->ws, false);
    if (rc) return rc;
    HIP_TRY(hipMemcpyAsync(s->host_pose, s->poses.p, sizeof(float) * s->pose_dim, hipMemcpyDeviceToHost, s->st));
    return TIK_OK;
}

extern "C" {

int tik_stream_create(tik_model_t model, int win_size, int use_graph, tik_stream_t* out) {
    if (!model || win_size <= 0 || !out) return fail(TIK_E_INVALID, "tik_stream_create: bad arguments");
    *out = nullptr;
    if (model_pose_dim(model) <= 0) return fail(TIK_E_INVALID, "tik_stream_create: backbone-only model handle");
    auto* s = new tik_stream();
    model_retain(model);
    s->model = model;
    s->h = win_size / 2;
    s->W = 2 * s->h + 1;
    s->tout = tik_model_out_frames(model, s->W);
    int rc = 0;
    if (s->tout <= 0 || (rc = model_reserve_ws(model, s->ws, 1, s->W)) || (rc = s->ring.reserve((size_t)s->W * s->V * 3)) ||
        (rc = s->window.reserve((size_t)s->W * s->V * 3)) || (rc = s->poses.reserve((size_t)s->tout * s->pose_dim)) ||
        (rc = s->frame_in.reserve((size_t)s->V * 3)) || (rc = s->count.reserve(1))) {
        delete s;
        return rc ? rc : fail(TIK_E_INVALID, "bad window");
    }
    auto bail = [&](const char* what, hipError_t e) { delete s; return fail(TIK_E_HIP, "%s: %s", what, hipGetErrorString(e)); };
    hipError_t e;
    if ((e = hipStreamCreateWithFlags(&s->st, hipStreamNonBlocking)) != hipSuccess) return bail("hipStreamCreate", e);
    if ((e = hipHostMalloc(&s->host_frame, sizeof(float) * s->V * 3, hipHostMallocDefault)) != hipSuccess) return bail("hipHostMalloc", e);
    if ((e = hipHostMalloc(&s->host_pose, sizeof(float) * (s->pose_dim + 1), hipHostMallocCoherent)) != hipSuccess) return bail("hipHostMalloc", e);
    s->host_pose[s->pose_dim] = 0.f;
    {
        void* hd = nullptr;
        if ((e = hipHostMalloc(&hd, sizeof(int), hipHostMallocCoherent)) != hipSuccess) return bail("hipHostMalloc", e);
        s->host_done = static_cast<volatile int*>(hd);
        *s->host_done = 0;
    }
    if ((e = hipMemsetAsync(s->count.p, 0, sizeof(int), s->st)) != hipSuccess) return bail("hipMemset", e);
    if ((e = hipMemsetAsync(s->ring.p, 0, sizeof(float) * s->W * s->V * 3, s->st)) != hipSuccess) return bail("hipMemset", e);
    if ((e = hipStreamSynchronize(s->st)) != hipSuccess) return bail("hipStreamSynchronize", e);
    {
        const char* env = getenv("TIK_ONLINE");
        if (!(env && env[0] == '0') && setup_online(s) != TIK_OK) s->online = false;   // layered fallback
    }
    if (use_graph) {
        if ((e = hipStreamBeginCapture(s->st, hipStreamCaptureModeThreadLocal)) != hipSuccess) return bail("hipStreamBeginCapture", e);
        rc = record_step(s);
        hipGraph_t g = nullptr;
        e = hipStreamEndCapture(s->st, &g);
        if (rc) { if (g) (void)hipGraphDestroy(g); delete s; return rc; }
        if (e != hipSuccess) return bail("hipStreamEndCapture", e);
        s->graph = g;
        if ((e = hipGraphInstantiate(&s->exec, g, nullptr, nullptr, 0)) != hipSuccess) return bail("hipGraphInstantiate", e);
    }
    *out = s;
    return TIK_OK;
}

int tik_stream_destroy(tik_stream_t s) {
    delete s;
    return TIK_OK;
}

int tik_stream_path(tik_stream_t s) {
    if (!s) return fail(TIK_E_INVALID, "null stream");
    return s->online ? 1 : 0;
}

int tik_debug_stream_trace(tik_stream_t s, long long* out, int cap) {
    if (!s || !s->online || !s->onl_trace.p) return fail(TIK_E_INVALID, "no online trace (TIK_ONLINE_TRACE=1 at tik_stream_create)");
    const int n = std::min(cap / 8, s->onl_ntasks);
    // a push returns once the pose is in host memory, while the launch's tail (the last
    // tasks' end marks, the scheduling bookkeeping) may still run on the non-blocking
    // stream, which a null-stream copy does not wait for
    HIP_TRY(hipStreamSynchronize(s->st));
    if (out && n > 0) HIP_TRY(hipMemcpy(out, s->onl_trace.p, sizeof(long long) * 8 * n, hipMemcpyDeviceToHost));
    return s->onl_ntasks;
}

int tik_stream_reset(tik_stream_t s) {
    if (!s) return fail(TIK_E_INVALID, "null stream");
    HIP_TRY(hipMemsetAsync(s->count.p, 0, sizeof(int), s->st));
    // the dataflow kernel's scheduling state: completion counters, ticket, done, err
    if (s->online) {
        HIP_TRY(hipMemsetAsync(s->onl_cnt.p, 0, sizeof(int) * s->onl_cnt.n, s->st));
        // count restarts at 0: the activations go back to tag 1 (online.hip)
        HIP_TRY(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(s->onl_act.p), (int)0x80000000u, s->onl_act.n, s->st));
    }
    HIP_TRY(hipStreamSynchronize(s->st));
    s->host_pose[s->pose_dim] = 0.f;
    *s->host_done = 0;
    s->pushed = 0;
    s->dcount = 0;
    return TIK_OK;
}

int tik_debug_stream_inject_error(tik_stream_t s) {
    if (!s || !s->online) return fail(TIK_E_INVALID, "tik_debug_stream_inject_error: not a dataflow-kernel stream");
    // err is the last of the scheduling words (setup_online: cnt[cb + 2])
    const int one = 1;
    HIP_TRY(hipMemcpyAsync(s->onl_cnt.p + (s->onl_cnt.n - 1), &one, sizeof(int), hipMemcpyHostToDevice, s->st));
    HIP_TRY(hipStreamSynchronize(s->st));
    return TIK_OK;
}

int tik_debug_stream_set_count(tik_stream_t s, int count) {
    if (!s) return fail(TIK_E_INVALID, "null stream");
    const long long period = 2LL * s->W;
    if (count < 0 || count >= (1 << 30) || ((long long)count - s->dcount) % period != 0)
        return fail(TIK_E_INVALID, "tik_debug_stream_set_count: %d is not the current count %d modulo %lld (or out of range)",
                    count, s->dcount, period);
    HIP_TRY(hipStreamSynchronize(s->st));
    HIP_TRY(hipMemcpy(s->count.p, &count, sizeof(int), hipMemcpyHostToDevice));
    s->dcount = count;
    return TIK_OK;
}

int tik_stream_push(tik_stream_t s, const float* frame_host, float* pose_host) {
    if (!s || !frame_host) return fail(TIK_E_INVALID, "tik_stream_push: bad arguments");
    memcpy(s->host_frame, frame_host, sizeof(float) * s->V * 3);
    if (s->exec) {
        HIP_TRY(hipGraphLaunch(s->exec, s->st));
    } else {
        int rc = record_step(s);
        if (rc) return rc;
    }
    bool seen = false;
    if (s->online) {
        // the dataflow kernel's last head task writes the new frame count to pinned
        // host memory after the pose: spin on it (sooner than the completion signal
        // hipStreamSynchronize waits for); the stream stays ordered for the next step
        const int want = tik::stream_next_count(s->dcount, s->W);
        const auto t0 = std::chrono::steady_clock::now();
        for (long it = 0;; ++it) {
            if (*s->host_done == want) { seen = true; break; }
            if ((it & 1023) == 1023 && std::chrono::steady_clock::now() - t0 > std::chrono::seconds(2)) break;
        }
    }
    if (!seen) HIP_TRY(hipStreamSynchronize(s->st));
    ++s->pushed;   // the step appended the frame to the device ring either way
    s->dcount = tik::stream_next_count(s->dcount, s->W);
    if (s->online && s->host_pose[s->pose_dim] != 0.f) {
        s->host_pose[s->pose_dim] = 0.f;
        return fail(TIK_E_HIP, "tik_stream_push: the online kernel timed out waiting on a dependency "
                               "(this frame's pose is invalid; the stream stays usable)");
    }
    const int valid = s->pushed > s->h;   // frame pushed-1-h >= 0 solved
    if (valid && pose_host) memcpy(pose_host, s->host_pose, sizeof(float) * s->pose_dim);
    return valid;
}

}  // extern "C"
