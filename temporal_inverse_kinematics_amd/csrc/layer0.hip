// layer0.hip — the first ST-GCN block's spatial half straight from the raw
// keypoints: data_bn (st_gcn_aaai18.py:119-125) + gcn 1x1 conv C0 -> Cout +
// 17x17 graph mix + folded tcn.0 BN + ReLU, written as fp32 rows (the layered
// bf16x3 path, TIK_XBLK=0; the default runs block 0 whole in xblock.hip).
//
// With C0 = 3 input channels the 1x1 conv is 3 MACs per output: a GEMM
// (K padded to 32) would spend its MFMAs on zeros and force the input into a
// padded 16-B-per-pixel operand.
// Here the graph mix runs first, on the 4-channel data_bn'd keypoints, once per
// (frame, joint) (dev_common.h l0_mix_in), then each thread computes (frame, 4
// output channels) for all 17 joints in fp32 VALU: bound by the z write
// (Cout x 4 B per pixel).
// Layer 0's residual conv (3 -> Cout) is folded into the temporal-conv
// epilogue the same way (XArgs::rx: the data_bn'd keypoints as 16-B rows, xb4).
#include "dev_common.h"
#include "xgemm.h"

namespace tik {

template <int SPARSE>
__global__ __launch_bounds__(256) void gcn0_kernel(const float* __restrict__ x, int rows, int C0,
                                                   const float* __restrict__ sc, const float* __restrict__ sh,
                                                   const float* __restrict__ wg, int ldwg, const float* __restrict__ bias2,
                                                   const float* __restrict__ amix, int Cout,
                                                   float* __restrict__ out, int ldo, float* __restrict__ xb4) {
    constexpr int VT = 17;
    const int G = Cout / 4;            // channel groups per frame
    const int FPB = 256 / G;           // frames per workgroup
    __shared__ __attribute__((aligned(16))) float xs[256 / 4 * VT * 4];   // up to 64 frames x 17 joints x 4 channels
    const int tid = threadIdx.x;
    const int nframes = rows / VT;
    const int f0 = blockIdx.x * FPB;
    for (int i = tid; i < FPB * VT * 4; i += 256) {
        const int c = i & 3, p = i >> 2;           // pixel within the block's frames
        const int v = p % VT, fr = f0 + p / VT;
        float val = 0.f;
        if (c < C0 && fr < nframes) val = fmaf(x[((size_t)fr * VT + v) * C0 + c], sc[v * C0 + c], sh[v * C0 + c]);
        xs[i] = val;
        if (fr < nframes) xb4[((size_t)fr * VT + v) * 4 + c] = val;
    }
    // the mix matrix in registers (amv[k] lane l = A[64 k + l], read back with
    // v_readlane): wave-uniform operands, no broadcast LDS reads in the mix
    constexpr int NAM = (VT * VT + 63) / 64;
    float amv[NAM];
#pragma unroll
    for (int k = 0; k < NAM; ++k) amv[k] = 64 * k + (tid & 63) < VT * VT ? amix[64 * k + (tid & 63)] : 0.f;
    __syncthreads();

    // mix first (dev_common.h l0_mix_in): u[f][w] for the block's frames x 17 joints,
    // once each: wave wv takes the joints w = wv (mod 4) (wave-uniform, so the mix
    // coefficients are v_readlane operands), lane = frame
    __shared__ f32x4 us[256 / 4 * VT];
    {
        const int wv = __builtin_amdgcn_readfirstlane(tid >> 6), fl = tid & 63;
        for (int fb = 0; fb < FPB; fb += 64)
            if (fb + fl < FPB) {
#pragma unroll
                for (int wj = 0; wj < VT; ++wj)
                    if ((wj & 3) == wv) us[(fb + fl) * VT + wj] = l0_mix_in<SPARSE != 0>(xs + (fb + fl) * VT * 4, amv, wj);
            }
    }
    __syncthreads();
    const int f = tid / G, g = tid - f * G;
    const int frame = f0 + f;
    if (f >= FPB || frame >= nframes) return;
    const int co = 4 * g;
    float w[4][4];
#pragma unroll
    for (int e = 0; e < 4; ++e)
#pragma unroll
        for (int c = 0; c < 4; ++c) w[e][c] = c < C0 ? wg[(co + e) * ldwg + c] : 0.f;
    // all bias loads ahead of the stores
    f32x4 b[VT];
#pragma unroll
    for (int wj = 0; wj < VT; ++wj) b[wj] = *reinterpret_cast<const f32x4*>(bias2 + wj * Cout + co);
#pragma unroll
    for (int wj = 0; wj < VT; ++wj)
        *reinterpret_cast<f32x4*>(out + ((size_t)frame * VT + wj) * ldo + co) = l0_conv_relu(us[f * VT + wj], w, b[wj]);
}

hipError_t launch_gcn0_f32(const float* x, int rows, int V, int C0, const float* bn_sc, const float* bn_sh,
                           const float* wg, int ldwg, const float* bias2, const float* amix, int mix_sparse, int Cout,
                           float* out, int ldo, float* xb4, hipStream_t st) {
    if (rows <= 0) return hipSuccess;
    if (V != 17 || rows % 17 || C0 < 1 || C0 > 4 || ldwg < C0 || Cout % 4 || Cout / 4 > 256 || 256 % (Cout / 4) ||
        ldo < Cout || ldo % 4)
        return hipErrorInvalidValue;
    const int fpb = 256 / (Cout / 4);
    const int nframes = rows / 17;
    (void)hipGetLastError();
    const dim3 grid((nframes + fpb - 1) / fpb), blk(256);
    if (mix_sparse)
        hipLaunchKernelGGL(gcn0_kernel<1>, grid, blk, 0, st, x, rows, C0, bn_sc, bn_sh, wg, ldwg, bias2, amix, Cout, out,
                           ldo, xb4);
    else
        hipLaunchKernelGGL(gcn0_kernel<0>, grid, blk, 0, st, x, rows, C0, bn_sc, bn_sh, wg, ldwg, bias2, amix, Cout, out,
                           ldo, xb4);
    return hipGetLastError();
}

}  // namespace tik
