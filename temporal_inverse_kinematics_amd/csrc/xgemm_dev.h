// xgemm_dev.h — device pieces shared by the bf16x3 GEMM kernels (xgemm.hip,
// xgraph.hip, xblock.hip, xtconv.hip): the fp32 -> three-bf16-plane split, the A-image swizzle, the
// epilogue store, and the LDS ring geometry of a tile configuration.
#pragma once
#include <hip/hip_runtime.h>

#include "cgemm.h"
#include "dev_common.h"
#include "xgemm.h"

namespace tik {

typedef __bf16 xbf16x8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ void xsplit8(const f32x4 lo, const f32x4 hi, xbf16x8& p0, xbf16x8& p1, xbf16x8& p2) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
        const float x = e < 4 ? lo[e] : hi[e - 4];
        const __bf16 b0 = (__bf16)x;
        const float r1 = x - (float)b0;
        const __bf16 b1 = (__bf16)r1;
        p0[e] = b0;
        p1[e] = b1;
        p2[e] = (__bf16)(r1 - (float)b1);
    }
}

// part q (0..3) of xsplit8: elements 2q, 2q + 1 (the same arithmetic), so a
// fragment's split can be spread over four MFMA groups
__device__ __forceinline__ void xsplit8_part(const f32x4 lo, const f32x4 hi, xbf16x8& p0, xbf16x8& p1, xbf16x8& p2, int q) {
#pragma unroll
    for (int e = 2 * q; e < 2 * q + 2; ++e) {
        const float x = e < 4 ? lo[e] : hi[e - 4];
        const __bf16 b0 = (__bf16)x;
        const float r1 = x - (float)b0;
        const __bf16 b1 = (__bf16)r1;
        p0[e] = b0;
        p1[e] = b1;
        p2[e] = (__bf16)(r1 - (float)b1);
    }
}

// epilogue stores of output tiles: nontemporal for the backbone's layer
// outputs (XArgs::nts; same-box A/B +0.9 % IK frames/s), plain for split-K
// partials and the FK GEMMs (re-read at once; NT measured slower there)
__device__ __forceinline__ void xst4(float* p, const f32x4 v, bool nt) {
    if (nt) __builtin_nontemporal_store(v, reinterpret_cast<f32x4*>(p));
    else *reinterpret_cast<f32x4*>(p) = v;
}

__device__ __forceinline__ int xa_swz(int r) { return (r >> 1) & 7; }

// EPI_SKIN: body b and transform row k of a lane's 4 GEMM rows rb .. rb + 3
// (rb % 4 == 0, so they never straddle bodies). 16 rows per body: k == 3 is
// the [0 0 0 1] row (not stored); 12 rows per body: the 3x4 part only
__device__ __forceinline__ void xskin_row(int rb, int srows, int& b, int& k) {
    const int q = rb >> 2;
    if (srows == 12) {
        b = q / 3;
        k = q - 3 * b;
    } else {
        b = q >> 2;
        k = q & 3;
    }
}

template <int BN, int EPI, int NW_>
struct XCfg {
    // NW waves of 32 rows (two 16-row fragments) each: NW = 8 is one 256-row
    // workgroup per CU (two waves per SIMD); NW = 4 a 128-row workgroup of
    // <= 80 KB LDS, two per CU, so one workgroup's prologue and epilogue run
    // under the other's main loop
    static constexpr int NW = NW_, NT = 64 * NW, BM = 32 * NW, FM = 2, FN = BN / 16, RW = 32;
    static constexpr bool TR = EPI == EPI_BIAS;   // transposed MFMA: each lane ends with 4 channels of a row
    static constexpr int ABYTES = BM * 128;
    static constexpr int PLANE = BN * 64;
    static constexpr int BBYTES = 3 * PLANE;
    // A rows are DMA'd and consumed by the same wave (wave w fills and reads rows
    // 32w..32w+31), so the A ring needs no barrier: 2 slots, issued 2 steps ahead
    // (a slot is free once its step's fragments were split, one step early).
    // B (weights) is shared by all waves, one barrier per step: issued LB steps
    // ahead into NSB = LB + 1 slots (LB = 1 for the two-per-CU tile: its wait for
    // B(k+1) sits after step k's MFMAs, so the DMA has a whole step to land)
    static constexpr int LB = NW == 8 ? 2 : 1;
    static constexpr int NSA = 2, NSB = LB + 1;
    static constexpr int RING = NSA * ABYTES + NSB * BBYTES;
    static constexpr int NIA = ABYTES / 1024 / NW;   // A DMA instructions per wave per stage
    static constexpr int NIB_TOT = BBYTES / 1024;
    static constexpr int NIBW = (NIB_TOT + NW - 1) / NW;   // B DMA instructions per wave per stage (at most)
    static constexpr int RT = EPI == EPI_GRAPH ? BM / 17 * 17 : BM;   // valid rows per tile (whole frames for the mix)
    static constexpr int LDCG = BN + 4;
    // C tile (+ the bias2 slice for the graph mix)
    static constexpr int CT = EPI == EPI_GRAPH ? BM * LDCG * 4 + 17 * BN * 4 : (EPI == EPI_SKIN ? 0 : BM * LDCG * 4);
    static constexpr int SMEM = RING > CT ? RING : CT;
    static constexpr int WG_PER_CU = NW == 8 ? 1 : 2;
    static_assert(NIA * 1024 * NW == ABYTES && NIA * 8 == RW, "A DMA split");
    static_assert(SMEM * WG_PER_CU <= 160 * 1024, "LDS");
};

}  // namespace tik
