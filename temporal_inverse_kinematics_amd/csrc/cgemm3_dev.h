// cgemm3_dev.h — device helpers shared by the split-activation f16x3 kernels
// (cgemm3.hip, tconv.hip): vector types, the 64-B-row LDS swizzle, f16 hi/lo
// splitting, and the bias/residual/activation epilogue of a staged C tile.
#pragma once
#include <hip/hip_runtime.h>

#include "cgemm3.h"

namespace tik {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));

__host__ __device__ constexpr unsigned coco_hop2_mask3(int w) {
    constexpr unsigned m[17] = {0x1Fu,   0x3Fu,   0x5Fu,   0x8EFu,   0x1177u, 0x3BFAu, 0x5DFCu, 0xAE8u,  0x1570u,
                                0x2A0u,  0x540u,  0xF8E8u, 0x17970u, 0xB820u, 0x15840u, 0xA800u, 0x15000u};
    return m[w];
}

__device__ __forceinline__ int sw3(int r) { return (0x1230 >> (4 * ((r >> 2) & 3))) & 3; }
__device__ __forceinline__ int swz3(int r, int c) { return r * 64 + ((c ^ sw3(r)) << 4); }

__device__ __forceinline__ void split4(const f32x4 v, f16x4& h, f16x4& l) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        h[e] = (_Float16)v[e];
        l[e] = (_Float16)(v[e] - (float)h[e]);
    }
}

__device__ __forceinline__ f32x4 merge4(const unsigned short* hi, long long plane) {
    const f16x4 h = *reinterpret_cast<const f16x4*>(hi);
    const f16x4 l = *reinterpret_cast<const f16x4*>(hi + plane);
    f32x4 v;
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] = (float)h[e] + (float)l[e];
    return v;
}

template <int N>
__device__ __forceinline__ void wait_vm() {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// Bias epilogue of a BM x BN fp32 tile staged in LDS (row stride LDC floats):
// v = act(C + bias + residual) -> split planes and/or fp32. bv = this
// thread's 4 bias values (columns n0 + 4*(tid % (BN/4)) ...), zero past Nc.
template <int BM, int BN, int NT, int LDC>
__device__ __forceinline__ void epi_bias(const Cgemm3Args& a, const float* Cs, const f32x4 bv, int r0, int n0, int tid) {
    constexpr int C4 = BN / 4;
    static_assert(NT % C4 == 0, "epilogue mapping");
    constexpr int RS = NT / C4;          // rows between one thread's items
    constexpr int KI = BM / RS;          // items per thread
    const int c4 = tid % C4, lr0 = tid / C4;
    const int col = n0 + 4 * c4;
    const bool vec = (a.ldo % 4 == 0) && (!a.resid || a.ldr % 4 == 0) && col + 3 < a.Nc;
    if (vec) {
        // all residual loads first, then branch-free math and the stores
        // (a data-dependent branch between stores makes the compiler wait
        // for every outstanding store: vmcnt counts stores too)
        f16x4 rh[KI], rl[KI];
#pragma unroll
        for (int k = 0; k < KI; ++k) { rh[k] = f16x4{}; rl[k] = f16x4{}; }
        if (a.resid) {
#pragma unroll
            for (int k = 0; k < KI; ++k) {
                const int row = r0 + lr0 + k * RS;
                if (row < a.M) {
                    const unsigned short* rp = a.resid + (size_t)row * a.ldr + col;
                    rh[k] = *reinterpret_cast<const f16x4*>(rp);
                    rl[k] = *reinterpret_cast<const f16x4*>(rp + a.resid_plane);
                }
            }
        }
        const float slope = a.act == ACT_RELU ? 0.f : (a.act == ACT_LEAKY ? 0.01f : 1.f);
#pragma unroll
        for (int k = 0; k < KI; ++k) {
            const int lr = lr0 + k * RS, row = r0 + lr;
            if (row >= a.M) continue;
            f32x4 v = *reinterpret_cast<const f32x4*>(Cs + lr * LDC + 4 * c4) + bv;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                v[e] += (float)rh[k][e] + (float)rl[k][e];
                v[e] = v[e] > 0.f ? v[e] : slope * v[e];
            }
            if (a.out_h) {
                f16x4 h, l;
                split4(v, h, l);
                unsigned short* o = a.out_h + (size_t)row * a.ldo + col;
                *reinterpret_cast<f16x4*>(o) = h;
                *reinterpret_cast<f16x4*>(o + a.out_plane) = l;
            }
            if (a.out_f) *reinterpret_cast<f32x4*>(a.out_f + (size_t)row * a.ldo + col) = v;
        }
    } else {
        for (int k = 0; k < KI; ++k) {
            const int lr = lr0 + k * RS, row = r0 + lr;
            if (row >= a.M) continue;
            for (int e = 0; e < 4 && col + e < a.Nc; ++e) {
                float v = Cs[lr * LDC + 4 * c4 + e] + bv[e];
                if (a.resid) {
                    const unsigned short* rp = a.resid + (size_t)row * a.ldr + col + e;
                    v += (float)__builtin_bit_cast(_Float16, rp[0]) + (float)__builtin_bit_cast(_Float16, rp[a.resid_plane]);
                }
                if (a.act == ACT_RELU) v = v > 0.f ? v : 0.f;
                else if (a.act == ACT_LEAKY) v = v > 0.f ? v : 0.01f * v;
                if (a.out_h) {
                    const _Float16 h = (_Float16)v;
                    const _Float16 l = (_Float16)(v - (float)h);
                    a.out_h[(size_t)row * a.ldo + col + e] = __builtin_bit_cast(unsigned short, h);
                    a.out_h[(size_t)row * a.ldo + col + e + a.out_plane] = __builtin_bit_cast(unsigned short, l);
                }
                if (a.out_f) a.out_f[(size_t)row * a.ldo + col + e] = v;
            }
        }
    }
}

}  // namespace tik
