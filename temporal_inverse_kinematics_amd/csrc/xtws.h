// xtws.h — the temporal half of a 128-channel stride-1 ST-GCN block with
// identity residual (tcn conv 3x1 + folded BN + residual + ReLU) as one
// persistent, weight-stationary launch (xtws.hip).
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
    int tune;                    // diagnostic builds (-DTIK_XTUNE) only: bits switch parts off (1 loads, 2 split, 4 MFMAs, 8 stores); 0
};

// weight-stationary (weights in VGPRs), 8-frame
// tiles whose 10-frame halo is split once per K block for all 3 taps
// (T % 8 == 0; the same packed weights, wp; the accumulation runs (K block,
// tap): equal to XT128 up to fp32 rounding of that order)
bool xtws_ok(const XTConvArgs& a);
hipError_t launch_xtws(const XTConvArgs& a, int ncu, hipStream_t st);

}  // namespace tik
