// layer0.hip — the first ST-GCN block's spatial half straight from the raw
// keypoints: data_bn (st_gcn_aaai18.py:119-125) + gcn 1x1 conv C0 -> Cout +
// 17x17 graph mix + folded tcn.0 BN + ReLU, written as split-block rows.
//
// With C0 = 3 input channels the 1x1 conv is 3 MACs per output: a GEMM
// (K padded to 32) would spend its MFMAs on zeros and force the input into a
// 128-B-per-pixel split block (142 MB at B=1024 instead of the 13 MB input).
// Here each thread computes (frame, 4 output channels) for all 17 joints in
// fp32 VALU: the kernel is bound by the z write (Cout x 4 B per pixel).
// Layer 0's residual conv (3 -> Cout) is folded into the temporal-conv
// epilogue the same way (Cgemm3Args::rx, cgemm3_dev.h epi_resid).
#include "cgemm3_dev.h"

namespace tik {

// F32OUT: z as fp32 rows [rows][ldo] (the bf16x3 path, xgemm.hip) instead of split blocks
template <int SPARSE, bool F32OUT = false>
__global__ __launch_bounds__(256) void gcn0_kernel(const float* __restrict__ x, int rows, int C0,
                                                   const float* __restrict__ sc, const float* __restrict__ sh,
                                                   const float* __restrict__ wg, int ldwg, const float* __restrict__ bias2,
                                                   const float* __restrict__ amix, int Cout,
                                                   unsigned short* __restrict__ out, int ldo, float* __restrict__ xb4,
                                                   float* __restrict__ outf = nullptr) {
    constexpr int VT = 17;
    const int G = Cout / 4;            // channel groups per frame
    const int FPB = 256 / G;           // frames per workgroup
    __shared__ float xs[256 / 4 * VT * 4];   // up to 64 frames x 17 joints x 4 channels
    const int tid = threadIdx.x;
    TIK_FENCE_BEGIN();
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

    const int f = tid / G, g = tid - f * G;
    const int frame = f0 + f;
    if (f >= FPB || frame >= nframes) return;
    const int co = 4 * g;
    float w[4][4];
#pragma unroll
    for (int e = 0; e < 4; ++e)
#pragma unroll
        for (int c = 0; c < 4; ++c) w[e][c] = c < C0 ? wg[(co + e) * ldwg + c] : 0.f;
    f32x4 y[VT];
#pragma unroll
    for (int v = 0; v < VT; ++v) {
        const float* xp = xs + (f * VT + v) * 4;
#pragma unroll
        for (int e = 0; e < 4; ++e) y[v][e] = xp[0] * w[e][0] + xp[1] * w[e][1] + xp[2] * w[e][2] + xp[3] * w[e][3];
    }
    // all bias loads ahead of the stores
    f32x4 b[VT];
#pragma unroll
    for (int wj = 0; wj < VT; ++wj) b[wj] = *reinterpret_cast<const f32x4*>(bias2 + wj * Cout + co);
    unsigned short* obase = out + (size_t)frame * VT * ldo + sbc(co);
#pragma unroll
    for (int wj = 0; wj < VT; ++wj) {
        f32x4 z = b[wj];
#pragma unroll
        for (int v = 0; v < VT; ++v)
            if (!SPARSE || ((coco_hop2_mask3(wj) >> v) & 1u)) {
                const float av = __builtin_bit_cast(
                    float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, amv[(v * VT + wj) / 64]), (v * VT + wj) % 64));
                z += av * y[v];
            }
#pragma unroll
        for (int e = 0; e < 4; ++e) z[e] = z[e] > 0.f ? z[e] : 0.f;
        if constexpr (F32OUT) {
            *reinterpret_cast<f32x4*>(outf + ((size_t)frame * VT + wj) * ldo + co) = z;
        } else {
            f16x4 h, l;
            split4(z, h, l);
            unsigned short* o = obase + (size_t)wj * ldo;
            *reinterpret_cast<f16x4*>(o) = h;
            *reinterpret_cast<f16x4*>(o + 32) = l;
        }
    }
    TIK_FENCE_END();
}

hipError_t launch_gcn0(const float* x, int rows, int V, int C0, const float* bn_sc, const float* bn_sh,
                       const float* wg, int ldwg, const float* bias2, const float* amix, int mix_sparse, int Cout,
                       unsigned short* out, int ldo, float* xb4, hipStream_t st) {
    if (rows <= 0) return hipSuccess;
    if (V != 17 || rows % 17 || C0 < 1 || C0 > 4 || ldwg < C0 || Cout % 4 || Cout / 4 > 256 || 256 % (Cout / 4) ||
        (256 / (Cout / 4)) * 17 * 4 > 256 / 4 * 17 * 4 || ldo < 64 * sb_blocks(Cout) || ldo % 8)
        return hipErrorInvalidValue;
    const int fpb = 256 / (Cout / 4);
    const int nframes = rows / 17;
    (void)hipGetLastError();
    const dim3 grid((nframes + fpb - 1) / fpb), blk(256);
    if (mix_sparse)
        hipLaunchKernelGGL(gcn0_kernel<1>, grid, blk, 0, st, x, rows, C0, bn_sc, bn_sh, wg, ldwg, bias2, amix, Cout, out, ldo, xb4);
    else
        hipLaunchKernelGGL(gcn0_kernel<0>, grid, blk, 0, st, x, rows, C0, bn_sc, bn_sh, wg, ldwg, bias2, amix, Cout, out, ldo, xb4);
    return hipGetLastError();
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
        hipLaunchKernelGGL((gcn0_kernel<1, true>), grid, blk, 0, st, x, rows, C0, bn_sc, bn_sh, wg, ldwg, bias2, amix, Cout,
                           nullptr, ldo, xb4, out);
    else
        hipLaunchKernelGGL((gcn0_kernel<0, true>), grid, blk, 0, st, x, rows, C0, bn_sc, bn_sh, wg, ldwg, bias2, amix, Cout,
                           nullptr, ldo, xb4, out);
    return hipGetLastError();
}

}  // namespace tik
