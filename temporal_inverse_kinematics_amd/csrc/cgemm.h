// cgemm.h — the implicit-GEMM temporal-convolution kernel family (fp32 MFMA).
//
// One kernel computes every dense contraction of the IK path on
// channels-last activations act[(n*T + t)*V + v][c]:
//   out[r][co] = epi( sum_seg sum_tap sum_ci  src_seg[row(r,tap)][ci] * W_seg[co][tap*cin_seg + ci] )
// with r = (n*tout + t')*V + w and row(r,tap) = (n*tin + s*t' + tap - pad)*V + w
// (zero when the source frame is outside [0, tin): the temporal zero padding
// of Conv2d((kt,1), stride (s,1), padding (pad,0))).
//   * gcn 1x1 conv          gconv_origin.py:49-60        (seg: kt=1)
//   * tcn 3x1 conv + BN     st_gcn_aaai18.py:180-187     (seg: kt=3, pad=1, stride s)
//   * residual 1x1 conv+BN  st_gcn_aaai18.py:198-204     (second seg: kt=1, stride s)
//   * head Linear layers    pose_trainer.py:89-92        (V=1, tout=M)
// Epilogues: bias (+ identity residual) + {none, ReLU, LeakyReLU}; or the
// graph epilogue: per-frame V-mix  z[w] = sum_v A[v][w] y[v]  (the einsum of
// gconv_origin.py:64) + folded BN bias + ReLU (st_gcn_aaai18.py:178-179);
// or the skinning epilogue of SMPL-X LBS (rows = body*16 + transform entry,
// cols = vertices): verts[b][v] = T_v(b)[:3,:3] v_posed[b][v] + T_v(b)[:3,3] (+ transl).
#pragma once
#include <hip/hip_runtime.h>

namespace tik {

enum { ACT_NONE = 0, ACT_RELU = 1, ACT_LEAKY = 2 };
enum { EPI_BIAS = 0, EPI_GRAPH = 1, EPI_SKIN = 2 };
enum { PREC_F32 = 0, PREC_BF16X3 = 2 };   // see cgemm.hip (1 was the retired f16x3 split)

struct Seg {
    const float* src;   // rows of `ld` floats, cin used (cin % 4 == 0)
    const float* w;     // [Nc][ldw], k = tap*cin + ci                 (PREC_F32)
    int cin, ld, kt, stride, pad, tin, ldw;
    int cin8 = 0, ldw8 = 0;                // cin rounded up to 8; row stride of the planes in bf16 elements
    const unsigned short* wb[3] = {nullptr, nullptr, nullptr};   // bf16 planes, w = p0+p1+p2 (PREC_BF16X3):
                                                                  // [Nc][ldw8], k = tap*cin8 + ci
};

struct CgemmArgs {
    int M, Nc, V, tout;
    Seg seg[2];
    int nseg;
    const float* bias;   // EPI_BIAS: [Nc];  EPI_GRAPH: [V][Nc]
    const float* resid;  // EPI_BIAS identity residual [M][ldr] or null
    int ldr;
    float* out;
    int ldo;
    const float* amix;   // EPI_GRAPH: [V][V], A_eff[v][w]
    int act;
    int mix_sparse = 0;  // EPI_GRAPH: A_eff's nonzeros lie inside the COCO hop<=2 pattern
    int ksplit = 1;      // EPI_BIAS: split K over gridDim.z workgroups (small-batch latency)
    float* partial = nullptr;   // [ksplit][M][Nc] workspace when ksplit > 1
    // EPI_SKIN: resid = v_posed [B][ldr], out = verts [B][ldo], bias = transl [B][3] or null
};

// Tile configurations.
enum CgemmCfg {
    CFG_T128x128 = 0,   // BM=128, BN=128, waves 2x2 : tcn/residual of 128/256-channel layers
    CFG_T128x64 = 1,    // BM=128, BN=64,  waves 2x2 : tcn of 64-channel layers
    CFG_G272x64 = 2,    // BM=272 (16 frames x 17 joints), BN=64, waves 1x4 : gcn + V-mix
    CFG_H64x128 = 3,    // BM=64,  BN=128, waves 2x2 : head Linear layers
    CFG_S128x128 = 4,   // BM=128 (8 bodies x 16), BN=128 vertices, waves 2x2 : LBS skinning
    CFG_T256x64 = 5,    // BM=256, BN=64,  waves 4x1 : tcn of 64-channel layers
    CFG_H64x64 = 6,     // BM=64,  BN=64,  waves 2x2 : head (more workgroups)
};

// true when every nonzero of A (V x V, row-major A[v][w]) lies in the COCO-17
// hop<=2 pattern the sparse graph epilogue unrolls
bool fits_coco_hop2(const float* A, int V);

// split-K factor for a small launch (fewer than 128 output tiles), 1 otherwise
int splitk_for(const CgemmArgs& a, int BM, int BN, int bk, int max_split);

hipError_t launch_cgemm(const CgemmArgs& a, int cfg, hipStream_t st, int prec = PREC_F32);

}  // namespace tik
