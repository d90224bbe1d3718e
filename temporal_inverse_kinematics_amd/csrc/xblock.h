// xblock.h — the first two ST-GCN blocks as whole-block kernels (xblock.hip).
#pragma once
#include <hip/hip_runtime.h>

#include <vector>

namespace tik {

struct XBlkArgs {
    int nframes;                 // N * T frames of the batch (flattened; taps stop at window edges)
    int T;                       // frames per window
    // block 1 (raw = false): the block input as P3 planes [rows][3][64] bf16 (block 0's output)
    const unsigned short* xp3;
    // block 0 (raw = true): raw keypoints [rows][c0], data_bn scale/shift [17][c0],
    // gcn weights (tcn.0 BN folded) [64][ldwg0], residual conv (BN folded) [64][c0]
    const float* xraw;
    int c0;
    const float* bn_sc;
    const float* bn_sh;
    const float* wg0;
    int ldwg0;
    const float* rw;
    const unsigned short* wgp;   // block 1: gcn weight planes (xblock_pack_weights, kt 1)
    const unsigned short* wtp;   // temporal conv weight planes (xblock_pack_weights, kt 3)
    const float* bias2;          // [17][64]: sc1 * bg * colsum(A)[w] + sh1
    const float* amix;           // [17][17] A_eff[v][w]
    int mix_sparse;
    const float* bias;           // [64]: tcn bias (+ residual bias), BN folded
    float* out_f;                // block 1: fp32 [rows][64]
    unsigned short* out_p3;      // block 0: P3 planes [rows][3][64]
    float* trash;                // >= 64 B: store target of pixels past the batch
    unsigned long long* trace;   // debug (-DTIK_XTRACE build): 24 phase sums per workgroup, or null
};

// raw: block 0 from the keypoints (writes P3); else block 1 from P3 (writes fp32).
// One 512-thread workgroup per CU (ncu), persistent over tiles of 10 output frames.
hipError_t launch_xblock(const XBlkArgs& a, bool raw, int ncu, hipStream_t st);
int xblock_frames_per_tile();
// fp32 weights w[co][tap * cin + ci] (row stride ldw) -> bf16x3 planes in the
// MFMA A-operand register layout [co/16][tap * cin/32 + kb][plane][lane][8]
std::vector<unsigned short> xblock_pack_weights(const float* w, int cout, int ldw, int kt, int cin);

}  // namespace tik
