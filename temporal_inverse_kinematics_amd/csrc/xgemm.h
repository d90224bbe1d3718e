// xgemm.h — the bf16x3 implicit-GEMM kernels of the IK forward (xgemm.hip).
//
// Arithmetic: every fp32 operand x = p0 + p1 + p2 (three bf16 planes, round to
// nearest even on exact fp32 residuals: exact for normal fp32, fp32's 8-bit
// exponent), out = sum of the six products p_i q_j with i + j <= 2 on
// v_mfma_f32_16x16x32_bf16, fp32 accumulation (the dropped ones are <= 2^-24
// relative each). Activations stay fp32 in HBM (4 B per element, as an fp32
// implementation): they reach LDS by direct global->LDS DMA as fp32 rows and
// are split in registers when each wave reads its A fragment (every wave owns
// distinct rows, so every element is split once per K step). Weights are
// split once on the host and packed per (column tile, K step) in exactly the
// LDS image order, so their DMA is a linear copy.
//
// Contraction (same row conventions as cgemm.h): rows r = (n*tout + t')*V + w;
// segment s, tap k reads source row (n*tin + stride*t' + k - pad)*V + w, zero
// outside [0, tin). K step = (segment, 32-channel block, tap): the taps of a
// block are adjacent, so the rows two taps share (stride 2: tap 2 of frame t is
// tap 0 of frame t + 1) are re-read from L2 two steps later, not from MALL/HBM
// a whole tap pass later.
#pragma once
#include <hip/hip_runtime.h>

#include <vector>

#include "cgemm.h"   // EPI_*, ACT_*

namespace tik {

struct XSeg {
    const float* src;     // fp32 rows [rows_in][ld]
    int ld;               // floats per row (multiple of 4)
    int cin;              // channels (multiple of 32)
    int kt, stride, pad, tin;
    long long rows_in;    // rows of src (the DMA bound: reads past it return zeros)
};

struct XArgs {
    int M, Nc, V, tout;
    XSeg seg[2];
    int nseg;
    const unsigned short* wp;   // packed weight tiles (xgemm_pack), [Nc/BN][kmain][3][BN*32] bf16
    int ksteps;                 // K steps of all segments (xgemm_ksteps)
    // identity residual (EPI_BIAS): idn.src = the block input rows, read at the
    // output row (kt 1, stride 1, pad 0); null = none. Added inside the K loop
    // as idn.cin/32 extra K steps against the identity (x = p0 + p1 + p2, three
    // MFMAs with a constant 1.0 operand: an exact add), so its rows stream
    // through the DMA ring with the other operands instead of the epilogue
    XSeg idn;
    const float* bias;          // EPI_BIAS: [Nc]; EPI_GRAPH: [V][Nc]
    const float* rx;            // EPI_BIAS small residual conv input [M][4] fp32 (layer 0; or null)
    int rxc;
    const float* rw;            // its weights [Nc][rxc]
    const float* amix;          // EPI_GRAPH [V][V], A_eff[v][w]
    int mix_sparse;
    const float* resid;         // EPI_SKIN: v_posed [M/16][ldr] (bodies x 3V), out = verts [M/16][ldo], bias = transl [M/16][3] or null
    int ldr;
    float* out;                 // fp32 [M][ldo]
    float* trash;               // xgemm_pt: >= BN floats, the store target of rows past M
    int nts;                    // nontemporal output stores (EPI_BIAS / EPI_GRAPH; the backbone's layer outputs)
    int skin_rows;              // EPI_SKIN on xgemm_pt: GEMM rows per body, 16 (A_j rows 4r+c incl. [0 0 0 1]; 0 = 16) or 12 (3x4 only)
    int ldo;
    int act;
    // split K (EPI_BIAS, one kt-1 segment, no residual, bias or activation):
    // blockIdx.z = k slice; slice z writes its raw partial sums to
    // out + z * M * ldo, and xgemm_splitk_reduce finishes (0 or 1: no split)
    int ksplit;
    int idn_epi;  // with epi_lds: the identity residual added in the epilogue from row-major loads (no K steps)
    int epi_lds;  // EPI_BIAS: stage the C tile through LDS for whole-line row-major stores (else float4 stores from registers)
    int gm;     // xgemm_kernel tile order: >1 = groups of gm row tiles, columns outer within a group (the B operand
                // is shared by the gm row tiles running together: for a large B, e.g. the FK blend shapes); else rows outer
    int nw;     // waves per workgroup: 4 (or 0: two 128-row workgroups per CU) or 8 (one 256-row workgroup)
    int tune;   // experiments only (0 = production): 1 skip the A DMA, 2 skip the B DMA, 8 skip the split
    unsigned long long* trace;   // debug (TIK_X_TRACE): 8 s_memtime stamps/sums per workgroup, or null
};

// K steps with packed weight tiles (the segments), and all K steps (+ identity)
__host__ __device__ inline int xgemm_kmain(const XArgs& a) {
    int k = 0;
    for (int s = 0; s < a.nseg; ++s) k += a.seg[s].kt * (a.seg[s].cin / 32);
    return k;
}
__host__ __device__ inline int xgemm_ksteps(const XArgs& a) { return xgemm_kmain(a) + (a.idn.src ? a.idn.cin / 32 : 0); }

// epi: EPI_BIAS (cgemm.h: bias + residual + activation), EPI_GRAPH (graph
// mix over the 17 joints + bias2[w][c] + ReLU) or EPI_SKIN (SMPL-X skinning:
// rows = body * 16 + transform entry, columns = vertices); bn: 64 or 128 output columns per tile
hipError_t launch_xgemm(const XArgs& a, int bn, int epi, hipStream_t st);
// the persistent EPI_BIAS variant (xgemm_pt_kernel): <= 2 workgroups per CU
// (ncu = compute units) walk the tiles with one DMA pipeline across tiles.
// Needs Nc % bn == 0, >= 2 K steps, a.trash; identity residual read in the
// epilogue (no identity K steps); bit-identical to launch_xgemm with epi_lds.
// epi: EPI_BIAS or EPI_SKIN (bn 128, bias = translations (B,3), zeros if none).
hipError_t launch_xgemm_pt(const XArgs& a, int bn, int ncu, hipStream_t st, int epi = EPI_BIAS);
int xgemm_tile_rows(int epi, int nw);   // output rows per workgroup (whole frames for EPI_GRAPH)
// out[r][c] = act(sum_z part[z][r][c] + bias[c]) for the ksplit partials of a
// split-K launch (part: [ksplit][M][Nc], fixed summation order: deterministic)
hipError_t launch_xgemm_splitk_reduce(const float* part, int ksplit, int M, int Nc, const float* bias, int act,
                                      float* out, int ldo, hipStream_t st);

// layer 0's spatial half straight from the raw keypoints (layer0.hip; the
// layered path, TIK_XBLK=0): z = ReLU(mix_A(data_bn(x) . Wg'^T) + bias2) as fp32
// rows [rows][ldo]; x [rows][C0], C0 <= 4; also writes xb4 = data_bn(x) as
// [rows][4] fp32 (XArgs::rx, the residual conv's input)
hipError_t launch_gcn0_f32(const float* x, int rows, int V, int C0, const float* bn_sc, const float* bn_sh,
                           const float* wg, int ldwg, const float* bias2, const float* amix, int mix_sparse, int Cout,
                           float* out, int ldo, float* xb4, hipStream_t st);

// Host packing of the weights of up to two segments (segment s: fp32
// W_s[n][tap * cin_s + c], row stride ldw_s) into the tile layout above,
// bf16x3-split, with the LDS bank swizzle applied. n >= Nc and c >= cin_s are zero.
struct XPackSeg {
    const float* w;
    int ldw, kt, cin;
};
std::vector<unsigned short> xgemm_pack(const XPackSeg* segs, int nseg, int Nc, int bn);

}  // namespace tik
