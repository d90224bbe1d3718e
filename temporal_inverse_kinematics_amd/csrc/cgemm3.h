// cgemm3.h — the f16x3 implicit-GEMM path on split activations.
//
// Same contraction as cgemm.h (rows r = (n*tout + t')*V + w, temporal taps,
// up to two K segments), but every operand is stored pre-split as two f16
// planes (hi = f16(x), lo = f16(x - hi)): activations [rows][ld] halves with
// the lo plane `plane` halves after the hi plane; weights [Nc][kt*cin8].
// Operands reach LDS by direct global->LDS DMA (global_load_lds_dwordx4) in a
// 3-stage ring: no VGPR staging, no conversion VALU, two chunks of prefetch.
#pragma once
#include <hip/hip_runtime.h>

#include "cgemm.h"

namespace tik {

struct Seg3 {
    const unsigned short* src;   // hi plane; lo plane at src + plane
    long long plane;
    int cin8, ld, kt, stride, pad, tin;   // cin8 % 8 == 0, ld % 8 == 0 (halves)
    const unsigned short* whi;   // [Nc][ldw8] weights, k = tap*cin8 + ci
    const unsigned short* wlo;
    int ldw8;
};

struct Cgemm3Args {
    int M, Nc, V, tout;
    Seg3 seg[2];
    int nseg;
    const float* bias;            // EPI_BIAS [Nc]; EPI_GRAPH [V][Nc]
    const unsigned short* resid;  // identity residual, split planes [M][ldr]
    long long resid_plane;
    int ldr;
    unsigned short* out_h;        // split output planes [M][ldo] (or null)
    long long out_plane;
    float* out_f;                 // fp32 output [M][ldo] (or null)
    int ldo;
    const float* amix;            // EPI_GRAPH [V][V]
    int act;
    int mix_sparse;
    const unsigned short* zeros;  // >= 16 B of zeros: source of padded rows
    int tune;                     // tuning experiments (0 = production): 1 plain tile order
                                  // instead of the XCD-aware one
    unsigned long long* trace;    // tuning only: per-workgroup {start, loop end, end, hw_id, xcc_id}
};

enum Cgemm3Cfg {
    C3_T128x128 = 0,   // tcn / residual, C >= 128
    C3_T128x64 = 1,    // tcn, C = 64
    C3_G272x64 = 2,    // gcn + graph mix (16 frames x 17 joints)
    C3_H64x64 = 3,     // head Linear layers
    C3_T128x128_S3 = 4, C3_T128x128_S4 = 5, C3_T256x128_W8 = 6, C3_T256x64_W8 = 7, C3_T128x64_S4 = 8,
    C3_G272x128_W8 = 9, C3_G272x64_S2 = 10,
    C3_DBG_T128x128_DMA = 11, C3_DBG_T128x128_MFMA = 12, C3_DBG_T128x64_DMA = 13, C3_DBG_T128x64_MFMA = 14,
    C3_NCFG = 15,
};

hipError_t launch_cgemm3(const Cgemm3Args& a, int cfg, hipStream_t st);

// stride-1 temporal conv + residual with a frame halo in LDS (tconv.hip):
// seg[0] kt=3/stride 1/pad 1, optional seg[1] kt=1 (residual conv), V=17,
// Nc % 64 == 0; bn = 64 or 128 output columns per tile
bool tconv_halo_ok(const Cgemm3Args& a);
hipError_t launch_tconv_halo(const Cgemm3Args& a, int bn, hipStream_t st);

// fp32 [rows][C] (row stride lds floats) -> split planes [rows][Cp] (zero-filled C..Cp)
hipError_t launch_split(const float* x, long long rows, int C, int lds, int Cp, unsigned short* hi, long long plane,
                        hipStream_t st);
// split planes [rows][ld] -> fp32 [rows][C]
hipError_t launch_merge(const unsigned short* hi, long long plane, long long rows, int C, int ld, float* y,
                        hipStream_t st);
// data_bn on load, straight to split planes with 8 channels (st_gcn_aaai18.py:119-125)
hipError_t launch_data_bn_split(const float* x, int n_px, int V, int C, const float* scale, const float* shift,
                                unsigned short* hi, long long plane, hipStream_t st);

}  // namespace tik
