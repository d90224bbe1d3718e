// online.h — the online-IK step as ONE dataflow kernel (online.hip).
//
// The stream returns pose row 0 of the window's output (stream.cpp), and with
// 3x1 temporal convs row 0 only sees the first frames of every layer: output
// frame t of a stride-s layer reads input frames s*t-1 .. s*t+1. Walking that
// back from the head gives each layer's needed frame count (n_out, n_in; 1,
// 2, 4, 8, 9, 10, 20, 21, 22 input frames for the IK net at any window of at
// least 22 frames). The step computes exactly those frames as a list of small
// tasks in topological order:
//   G_L(f, 16 channels): gcn 1x1 conv + 17x17 graph mix + bias + ReLU (layer 0
//          builds its input rows itself: window gather with the left-edge
//          clamp, root-relative, data_bn; the pushed frame is read from pinned
//          host memory and appended to the ring by task 0)
//   T_L(t, 16 channels): 3x1 temporal conv + residual + bias + ReLU
//   H(16 hidden units + their share of the pose; the last H task sums the shares
//          and writes the pose straight to pinned host memory)
// Workgroups take task tickets in order and wait only for the activation
// elements a task reads (tagged with the launch's parity, online.hip; no
// grid-wide barrier), so the layers pipeline frame by frame; a task's weights
// are loaded before it waits.
#pragma once
#include <hip/hip_runtime.h>

namespace tik {

// The stream's frame count after one more push. It stays below 2^30: past it, a
// multiple of 2W is subtracted (W = the odd ring size), which keeps the ring slot
// (count % W), the launch parity (count & 1, online.hip's activation tag) and the
// window's frame offsets, and stays far above the left-edge clamp (count >= 2^29).
// Device kernels and the host's mirror of the count use the same rule.
__host__ __device__ inline int stream_next_count(int c, int W) {
    const int n = c + 1;
    return n >= (1 << 30) ? n - 2 * W * ((1 << 29) / (2 * W)) : n;
}

constexpr int ONL_MAXL = 12;        // layers
constexpr int ONL_MAXC = 256;       // channels per layer
constexpr int ONL_MAXHC = 17;       // head K chunks of 4 per lane: K <= 17 * 4 * 64 = 4352 = 17 joints x ONL_MAXC
enum { ONP_G = 1, ONP_T = 2, ONP_H = 3 };
enum { ONR_ZERO = 0, ONR_IDEN = 1, ONR_CONV = 2 };

struct OnlineLayer {
    int cin, cinp, cout, stride, res;
    int tin;           // the layer's real input frame count (zero padding past it)
    int n_in, n_out;   // frames computed: z (gcn) / out (temporal conv)
    const float *wg, *bias2, *amix, *wt, *wr, *biasT;   // the fp32 folded weights of api.cpp's Layer
    int gk32;                    // gcn K = cinp in steps of 32
    const unsigned short* wgp;   // gcn weight planes [cout/16][gk32][3][64][8] (stream-owned)
    const float* wgf;            // gcn weights fp32, [cout][32 gk32] zero-padded (joint 16)
    int k32;                     // temporal conv K = 3 cout (+ cinp, residual conv) in steps of 32
    const unsigned short* wtp;   // its bf16x3 planes [cout/16][k32][3][64 lanes][8] (stream-owned)
    const float* wtf;            // the same weights fp32, [cout][32 k32] zero-padded (joint 16)
    const float* x;    // input rows [n_in][17][cinp] (layer 0: built in place from the ring)
    float *z, *out;    // [n_in][17][cout], [n_out][17][cout]
};

struct OnlinePhase {
    int kind, layer, nframes, ngroups, task0, cbase;   // cbase: the phase's counter (the head's: tasks done)
};

struct OnlineArgs {
    int nl, nph, ntasks;
    OnlineLayer L[ONL_MAXL];
    OnlinePhase ph[2 * ONL_MAXL + 3];
    // input: ring of W frames (V*3 floats), count of frames pushed so far
    float* ring;
    int W, h, ra, rb, relative;
    int* count;
    const float* frame;   // the pushed frame (pinned host memory)
    const float *bn_sc, *bn_sh;
    // head
    const float *w0, *b0, *w3, *b3;
    int feat, hidden, pose_dim;
    float* hpart;         // [hidden / 16][pose_dim]: each head task's share of pose_regressor.3
    float* pose;          // device copy of the pose row
    float* pose_host;     // pinned host copy
    int* done_host;       // pinned host word: the frame count after this step, written last (the host spins on it)
    // scheduling state: zero at launch, left zero by the last workgroup out
    int* ticket;
    int* done;
    int* cnt;
    int ncnt;
    int* err;             // sticky: a dependency wait timed out
    unsigned long long* trace;   // debug (TIK_ONLINE_TRACE=1): per task 7 time stamps + the workgroup
    float* act;           // the one buffer every inter-task activation lives in (z, out, hpart, pose)
    unsigned act_bytes;
};

hipError_t launch_online(const OnlineArgs* dev_args, int grid, hipStream_t st);

}  // namespace tik
