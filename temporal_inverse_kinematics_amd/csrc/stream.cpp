// stream.cpp — online (stride-1 sliding-window) IK with a hipGraph-captured step
// (BASELINE.json config #5). The reference solves a recorded sequence offline,
// one window per frame (inference.run_inference, inference.py:37-67; windows
// from data_amass.py:18-42, 221-236). Online, frame c can be solved once frame
// c+h has arrived: each push of frame k runs the window centred at c = k-h
// (frames k-2h..k, left edge clamped like sample_window's edge padding) and
// returns pose row 0 of the model output, i.e. exactly run_inference's frame c.
// Flushing the last h frames = pushing the last frame h more times (right edge
// padding). The whole step — ring append, window gather, the ~20 kernels of the
// IK forward, the pose copy — is one hipGraph replay on a private stream.
#include <hip/hip_runtime.h>

#include "../../include/tik.h"
#include "common.h"
#include "misc.h"

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
    float* host_pose = nullptr;    // pinned
    long long pushed = 0;
    ~tik_stream() {
        if (st) (void)hipStreamSynchronize(st);
        if (exec) (void)hipGraphExecDestroy(exec);
        if (graph) (void)hipGraphDestroy(graph);
        if (host_frame) (void)hipHostFree(host_frame);
        if (host_pose) (void)hipHostFree(host_pose);
        if (st) (void)hipStreamDestroy(st);
        if (model) model_release(model);
    }
};

static int record_step(tik_stream* s) {
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
    if ((e = hipHostMalloc(&s->host_pose, sizeof(float) * s->pose_dim, hipHostMallocDefault)) != hipSuccess) return bail("hipHostMalloc", e);
    if ((e = hipMemsetAsync(s->count.p, 0, sizeof(int), s->st)) != hipSuccess) return bail("hipMemset", e);
    if ((e = hipMemsetAsync(s->ring.p, 0, sizeof(float) * s->W * s->V * 3, s->st)) != hipSuccess) return bail("hipMemset", e);
    if ((e = hipStreamSynchronize(s->st)) != hipSuccess) return bail("hipStreamSynchronize", e);
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

int tik_stream_reset(tik_stream_t s) {
    if (!s) return fail(TIK_E_INVALID, "null stream");
    HIP_TRY(hipMemsetAsync(s->count.p, 0, sizeof(int), s->st));
    HIP_TRY(hipStreamSynchronize(s->st));
    s->pushed = 0;
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
    HIP_TRY(hipStreamSynchronize(s->st));
    ++s->pushed;
    const int valid = s->pushed > s->h;   // frame pushed-1-h >= 0 solved
    if (valid && pose_host) memcpy(pose_host, s->host_pose, sizeof(float) * s->pose_dim);
    return valid;
}

}  // extern "C"
