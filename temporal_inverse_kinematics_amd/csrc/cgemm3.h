// cgemm3.h — the f16x3 implicit-GEMM path on split-block activations.
//
// Same contraction as cgemm.h (rows r = (n*tout + t')*V + w, temporal taps,
// up to two K segments), but every operand is stored pre-split in the
// SPLIT-BLOCK ("SB") layout: channels in blocks of 32, each block 64 halves =
// [hi(x) for its 32 channels | lo(x) = f16(x - hi) for the same 32], i.e. one
// full 128-B line per row per block. Channel c of row r:
//     hi at r*ld + (c/32)*64 + c%32,   lo at that + 32.
// Weights use the same blocks along K: [Nc][tap][block][64]. Operands reach
// LDS by direct global->LDS DMA (global_load_lds_dwordx4), each wave
// instruction moving 8 full rows x 128 B.
#pragma once
#include <hip/hip_runtime.h>

#include "cgemm.h"

namespace tik {

struct Seg3 {
    const unsigned short* src;   // SB activations [rows][ld]
    int nblk;                    // 32-channel blocks per tap (K = kt * nblk * 32)
    int ld;                      // halves per activation row (>= 64 * nblk)
    int kt, stride, pad, tin;
    const unsigned short* w;     // SB weights [Nc][ldw], ldw = kt * nblk * 64
    int ldw;
};

struct Cgemm3Args {
    int M, Nc, V, tout;
    Seg3 seg[2];
    int nseg;
    const float* bias;            // EPI_BIAS [Nc]; EPI_GRAPH [V][Nc]
    const unsigned short* resid;  // identity residual, SB [M][ldr]
    int ldr;
    unsigned short* out_h;        // SB output [M][ldo] (or null)
    int ldo;
    float* out_f;                 // fp32 output [M][ldf] (or null)
    int ldf;
    // small residual conv on a 4-float-per-row input (layer 0, EPI_BIAS):
    // res[r][c] = sum_{k < rxc} rx[r][k] * rw[c][k]; rx [M][4] fp32 (data_bn applied), rxc <= 4
    const float* rx;
    int rxc;
    const float* rw;
    const float* amix;            // EPI_GRAPH [V][V]
    int act;
    int mix_sparse;
    const unsigned short* zeros;  // >= 128 B of zeros: source of padded rows
    // TG_128x128_G7 (tgemm.hip): the NEXT block's gcn (1x1 conv + graph mix +
    // folded BN + ReLU) on this launch's output tile; null g_w = off
    const unsigned short* g_w;    // SB weights of the next gcn [g_nc][g_ldw], K = Nc
    int g_ldw, g_nc;
    const float* g_bias2;         // [V][g_nc]
    const float* g_amix;          // [V][V]
    int g_mix_sparse;
    unsigned short* g_out;        // SB z of the next block [M][g_ldo]
    int g_ldo;
    unsigned short* trash;        // TW_128 (tgw.hip): >= 4 KB scratch line for the stores of invalid rows
    int tune;                     // tuning experiments (0 = production): 1 plain tile order
                                  // instead of the XCD-aware one
    unsigned long long* trace;    // tuning only: per-workgroup {start, loop end, end, wait clk, barrier|loop clk}
};

enum Cgemm3Cfg {
    C3_T128x128 = 0,   // tcn / residual, C >= 128
    C3_T128x64 = 1,    // tcn, C = 64
    C3_G272x64 = 2,    // gcn + graph mix (16 frames x 17 joints)
    C3_H64x64 = 3,     // head Linear layers
    C3_T128x128_S3 = 4, C3_T128x128_S4 = 5, C3_T256x128_W8 = 6, C3_T256x64_W8 = 7, C3_T128x64_S4 = 8,
    C3_G272x128_W8 = 9, C3_G272x64_S2 = 10,
    C3_DBG_T128x128_DMA = 11, C3_DBG_T128x128_MFMA = 12, C3_DBG_T128x64_DMA = 13, C3_DBG_T128x64_MFMA = 14,
    C3_T128x128_W8 = 15, C3_T128x64_W8 = 16, C3_DBG_W8_DMA = 17, C3_DBG_W8_MFMA = 18,
    C3_NCFG = 19,
};

hipError_t launch_cgemm3(const Cgemm3Args& a, int cfg, hipStream_t st);

// bias-epilogue GEMM with split DMA rings (tgemm.hip): A ring NSA deep, B ring 2
enum TgemmCfg {
    TG_128x128 = 0,      // 8 waves, A ring 3
    TG_128x64 = 1,       // 8 waves, A ring 3
    TG_128x128_A4 = 2,   // A ring 4 (one workgroup per CU)
    TG_128x64_A4 = 3,
    TG_64x64 = 4,        // head Linear layers, 4 waves
    TG_128x128_G7 = 5,   // 7-frame tiles (119 of 128 rows) + the next block's gcn in the epilogue
};
hipError_t launch_tgemm(const Cgemm3Args& a, int cfg, hipStream_t st);

// weight-stationary persistent T + next gcn (tgw.hip, TW_128): stride 1, identity
// residual, 128 -> 128 -> 128, V = 17; one workgroup per CU over contiguous tile runs
bool tgw_ok(const Cgemm3Args& a);
hipError_t launch_tgw(const Cgemm3Args& a, hipStream_t st);

// weight-stationary persistent gcn (gpw.hip, GP_*): 1x1 conv + graph mix + bias +
// ReLU for 64->128, 128->256, 256->256, V = 17; the next tile's x DMA'd behind the current
bool gpw_ok(const Cgemm3Args& a);
hipError_t launch_gpw(const Cgemm3Args& a, hipStream_t st);

// stride-1 temporal conv + residual with a frame halo in LDS (tconv.hip):
// seg[0] kt=3/stride 1/pad 1, optional seg[1] kt=1 (residual conv), V=17,
// Nc % 64 == 0; bn = 64 or 128 output columns per tile
bool tconv_halo_ok(const Cgemm3Args& a);
hipError_t launch_tconv_halo(const Cgemm3Args& a, int bn, hipStream_t st);

// layer 0 spatial half straight from the raw keypoints (layer0.hip):
// z = ReLU(mix_A(data_bn(x) . Wg'^T) + bias2) -> SB [rows][ldo]; x [rows][C0], C0 <= 4;
// also writes xb4 = data_bn(x) as [rows][4] fp32 (the residual conv's input)
hipError_t launch_gcn0(const float* x, int rows, int V, int C0, const float* bn_sc, const float* bn_sh,
                       const float* wg, int ldwg, const float* bias2, const float* amix, int mix_sparse, int Cout,
                       unsigned short* out, int ldo, float* xb4, hipStream_t st);

// the same with z as fp32 rows [rows][ldo] (bf16x3 path)
hipError_t launch_gcn0_f32(const float* x, int rows, int V, int C0, const float* bn_sc, const float* bn_sh,
                           const float* wg, int ldwg, const float* bias2, const float* amix, int mix_sparse, int Cout,
                           float* out, int ldo, float* xb4, hipStream_t st);

// SB activations [rows][ld] -> fp32 [rows][C]
// One whole stride-1, identity-residual ST-GCN block per workgroup
// (stblock.hip): z = ReLU(mix(x Wg') + bias2) stays in LDS, then
// out = ReLU(tcn(z) + bias + x). x / out: SB rows (n, t, v) of nwin windows x T frames.
struct StbArgs {
    const unsigned short* x;
    int ldx;
    int nwin, T;
    const unsigned short* wg;   // SB [Cout][Cin/32][64]
    int ldwg;
    const float* bias2;         // [17][Cout]
    const float* amix;          // [17][17], input joint v -> output joint w at v*17+w
    int mix_sparse;
    const unsigned short* wt;   // SB [Cout][3][Cout/32][64]
    int ldwt;
    const float* bias;          // [Cout]
    int resid;                  // 1: + x (identity residual)
    unsigned short* out;
    int ldo;
    unsigned long long* trace;  // optional: 6 s_memrealtime stamps per workgroup (phase boundaries)
    // raw-input first block (launch_stblock0): z from the keypoints in VALU, residual conv from them too
    const float* xraw;          // [rows][c0] keypoints
    int c0;                     // <= 4 input channels
    const float* bn_sc;         // data_bn per (joint, channel) [17][c0]
    const float* bn_sh;
    const float* wg0;           // fp32 gcn weights (tcn.0 BN folded) [Cout][ldwg0]
    int ldwg0;
    const float* rw;            // fp32 residual conv (BN folded) [Cout][c0]
};
bool stblock_ok(int cin, int cout);
hipError_t launch_stblock(const StbArgs& a, int cin, int cout, hipStream_t st);
// the whole FIRST block from the raw keypoints (Cout = 64, stride 1, residual conv)
hipError_t launch_stblock0(const StbArgs& a, int cout, hipStream_t st);


hipError_t launch_merge(const unsigned short* sb, long long rows, int C, int ld, float* y, hipStream_t st);
// data_bn on load, straight to one SB block per pixel (C <= 32 channels, rest zero) (st_gcn_aaai18.py:119-125)
hipError_t launch_data_bn_split(const float* x, int n_px, int V, int C, const float* scale, const float* shift,
                                unsigned short* sb, hipStream_t st);

inline int sb_blocks(int c) { return (c + 31) / 32; }

}  // namespace tik
