// xtws.h — the temporal half of a 128-channel stride-1 ST-GCN block with
// identity residual (tcn conv 3x1 + folded BN + residual + ReLU) as one
// persistent, weight-stationary launch (xtws.hip), optionally fused with the
// spatial half of the NEXT block (its gcn 1x1 conv + graph mix + BN + ReLU).
#pragma once
#include <hip/hip_runtime.h>

namespace tik {

struct XTConvArgs {
    int M;                       // output rows = input rows (N * T * 17, stride 1)
    int T;                       // frames per window (taps never cross a window)
    const float* z;              // conv input, fp32 rows [M][ldz], 128 channels
    int ldz;
    const float* x;              // identity residual, fp32 rows [M][ldx], 128 channels
    int ldx;
    const unsigned short* wp;    // tcn.2 weights (BN folded), xblock_pack_weights(w, 128, 3 * 128, 3, 128)
    const float* bias;           // [128]
    float* out;                  // [M][ldo]
    int ldo;
    int nts;                     // nontemporal stores
    float* trash;                // >= 4 KB: store target of rows past M (branch-free epilogue)
    int tune;                    // diagnostic builds (-DTIK_XTUNE) only: bits switch parts off (1 loads, 2 split, 4 MFMAs, 8 stores;
                                 // FG: 16 gcn MFMAs, 32 gcn split, 64 mix + z stores); 0
    unsigned long long* trace;   // diagnostic builds (-DTIK_XTRACE), FG: per workgroup, waves 0 and 4, 8 phase sums each
    // the next block's spatial half on this block's output tile (wg != nullptr:
    // the fused launch): zout = ReLU(bias2 + sum_v A[v][w] (out . Wg'^T)[v]),
    // 128 -> 128 channels (st_gcn_aaai18.py:211 of block l + 1, gconv_origin.py:56-65)
    const unsigned short* wg;    // gcn planes of block l + 1, xblock_pack_weights(w, 128, ldw, 1, 128)
    const float* bias2;          // [17][128] of block l + 1
    const float* amix;           // [17][17] A_eff[v][w] of block l + 1
    int mix_sparse;              // A_eff fits the COCO hop <= 2 pattern (the mix unrolls it)
    float* zout;                 // [M][ldzo]: block l + 1's z (must not alias z: other tiles read z's halo rows)
    int ldzo;
};

// weight-stationary (weights in VGPRs), 8-frame
// tiles whose 10-frame halo is split once per K block for all 3 taps
// (T % 8 == 0; the same packed weights, wp; the accumulation runs (K block,
// tap): equal to XT128 up to fp32 rounding of that order). With wg set, each
// tile's output rows (still in LDS) also go through block l + 1's gcn conv and
// graph mix (the products, K order and mix order of xgraph.hip: zout is bit
// for bit what launch_xgraph makes from out)
bool xtws_ok(const XTConvArgs& a);
hipError_t launch_xtws(const XTConvArgs& a, int ncu, hipStream_t st);

}  // namespace tik
