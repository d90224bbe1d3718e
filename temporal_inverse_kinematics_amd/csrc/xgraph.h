// xgraph.h — the gcn half of an ST-GCN block as one persistent weight-stationary launch (xgraph.hip).
#pragma once
#include <hip/hip_runtime.h>

namespace tik {

struct XGraphArgs {
    int nframes;                 // frames of the batch (N * T, flattened)
    const float* x;              // block input, fp32 rows [nframes * 17][ldx]
    int ldx;
    int cin, cout;               // 64 / 128 / 256 -> 128 / 256
    const unsigned short* wp;    // gcn weight planes (tcn.0 BN folded), xblock_pack_weights(w, cout, ldw, 1, cin)
    const float* bias2;          // [17][cout]
    const float* amix;           // [17][17] A_eff[v][w]
    int mix_sparse;
    float* out;                  // z, fp32 rows [nframes * 17][ldo]
    int ldo;
    int nts;                     // nontemporal stores
    float* trash;                // >= 16 B: store target of frames past the batch
    int tune;
    unsigned long long* trace;   // diagnostic builds (-DTIK_XTRACE): per workgroup, waves 0 and 4, 8 counters each                    // diagnostic builds (-DTIK_XTUNE) only: bits switch parts off (1 x loads, 2 split, 4 MFMAs, 8 stores, 16 mix)
};

bool xgraph_ok(const XGraphArgs& a);
// one 512-thread workgroup per CU (ncu), persistent over (16-frame group, 128-channel pass) tiles
hipError_t launch_xgraph(const XGraphArgs& a, int ncu, hipStream_t st);

}  // namespace tik
