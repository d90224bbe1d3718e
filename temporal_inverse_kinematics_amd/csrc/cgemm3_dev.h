// cgemm3_dev.h — device helpers shared by the split-block f16x3 kernels
// (cgemm3.hip, tconv.hip): vector types, the 128-B-row LDS swizzle of the
// split-block image, f16 hi/lo splitting, and the bias/residual/activation
// epilogue of a staged C tile.
#pragma once
#include <hip/hip_runtime.h>

#include "cgemm3.h"

namespace tik {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));

__host__ __device__ constexpr unsigned coco_hop2_mask3(int w) {
    constexpr unsigned m[17] = {0x1Fu,   0x3Fu,   0x5Fu,   0x8EFu,   0x1177u, 0x3BFAu, 0x5DFCu, 0xAE8u,  0x1570u,
                                0x2A0u,  0x540u,  0xF8E8u, 0x17970u, 0xB820u, 0x15840u, 0xA800u, 0x15000u};
    return m[w];
}

// LDS image of one K block: 128-B rows (8 x 16-B units: hi k 0-7, 8-15,
// 16-23, 24-31, then lo likewise); unit u of row r sits at u ^ ((r >> 1) & 7).
// A 16-row fragment read (ds_read_b128, fixed unit) then touches 16 distinct
// 16-B bank slots: conflict-free.
__device__ __forceinline__ int sbf(int r) { return (r >> 1) & 7; }
__device__ __forceinline__ int sbo(int r, int u) { return r * 128 + ((u ^ sbf(r)) << 4); }

// element offset of channel c (4-aligned group start) in an SB row
__device__ __forceinline__ int sbc(int c) { return ((c >> 5) << 6) + (c & 31); }

__device__ __forceinline__ void split4(const f32x4 v, f16x4& h, f16x4& l) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        h[e] = (_Float16)v[e];
        l[e] = (_Float16)(v[e] - (float)h[e]);
    }
}

// ---- buffer_load ... lds (raw buffer, stride 0): offsets at or past
// num_records read as zeros, which implements every padded / out-of-range row
typedef int i32x4 __attribute__((ext_vector_type(4)));
__device__ void tik_llvm_raw_buffer_load_lds(i32x4 rsrc, __attribute__((address_space(3))) unsigned* lds, int size,
                                             int voffset, int soffset, int offset, int aux)
    __asm("llvm.amdgcn.raw.buffer.load.lds");

__device__ __forceinline__ i32x4 buf_rsrc(const void* p, unsigned bytes) {
    const unsigned long long a = reinterpret_cast<unsigned long long>(p);
    i32x4 r;
    r[0] = __builtin_amdgcn_readfirstlane((int)(unsigned)a);
    r[1] = __builtin_amdgcn_readfirstlane((int)((unsigned)(a >> 32) & 0xffffu));   // stride 0
    r[2] = __builtin_amdgcn_readfirstlane((int)bytes);
    r[3] = 0x00020000;
    return r;
}

// 16 B per lane from rsrc + voff + soff into LDS at dst (wave-uniform base; lane l -> dst + 16 l)
__device__ __forceinline__ void dma16(const i32x4 r, void* dst, unsigned voff, int soff) {
#ifndef TIK_DMA_AUX
#define TIK_DMA_AUX 0
#endif
    tik_llvm_raw_buffer_load_lds(r, (__attribute__((address_space(3))) unsigned*)dst, 16, (int)voff, soff, 0, TIK_DMA_AUX);
}

constexpr unsigned DMA_OOB = 0x80000000u;

// debug build hook (-DTIK_KFENCE): explicit agent-scope acquire at kernel
// start / release at kernel end of the DMA-path kernels
#ifdef TIK_KFENCE
#define TIK_FENCE_BEGIN() __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent")
#define TIK_FENCE_END() __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent")
#else
#define TIK_FENCE_BEGIN() ((void)0)
#define TIK_FENCE_END() ((void)0)
#endif

template <int N>
__device__ __forceinline__ void wait_vm() {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// s_waitcnt vmcnt(n) for a wave-uniform n in [0, 63]
__device__ __forceinline__ void wait_vm_dyn(int n) {
    switch (n) {
#define TIK_VMW(k) \
    case k: asm volatile("s_waitcnt vmcnt(" #k ")" ::: "memory"); break;
        TIK_VMW(0) TIK_VMW(1) TIK_VMW(2) TIK_VMW(3) TIK_VMW(4) TIK_VMW(5) TIK_VMW(6) TIK_VMW(7)
        TIK_VMW(8) TIK_VMW(9) TIK_VMW(10) TIK_VMW(11) TIK_VMW(12) TIK_VMW(13) TIK_VMW(14) TIK_VMW(15)
        TIK_VMW(16) TIK_VMW(17) TIK_VMW(18) TIK_VMW(19) TIK_VMW(20) TIK_VMW(21) TIK_VMW(22) TIK_VMW(23)
        TIK_VMW(24) TIK_VMW(25) TIK_VMW(26) TIK_VMW(27) TIK_VMW(28) TIK_VMW(29) TIK_VMW(30) TIK_VMW(31)
        TIK_VMW(32) TIK_VMW(33) TIK_VMW(34) TIK_VMW(35) TIK_VMW(36) TIK_VMW(37) TIK_VMW(38) TIK_VMW(39)
        TIK_VMW(40) TIK_VMW(41) TIK_VMW(42) TIK_VMW(43) TIK_VMW(44) TIK_VMW(45) TIK_VMW(46) TIK_VMW(47)
        TIK_VMW(48) TIK_VMW(49) TIK_VMW(50) TIK_VMW(51) TIK_VMW(52) TIK_VMW(53) TIK_VMW(54) TIK_VMW(55)
        TIK_VMW(56) TIK_VMW(57) TIK_VMW(58) TIK_VMW(59) TIK_VMW(60) TIK_VMW(61) TIK_VMW(62) TIK_VMW(63)
#undef TIK_VMW
        default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
}

__device__ __forceinline__ void lds_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
}

// Bias epilogue of a BM x BN fp32 tile staged in LDS (row stride LDC floats):
// v = act(C + bias + residual) -> SB output and/or fp32. bv = this thread's 4
// bias values (columns n0 + 4*(tid % (BN/4)) ...), zero past Nc. The
// residual is loaded by epi_resid (the caller issues it early, during the
// last K step, so its latency hides behind the MFMAs); the math between the
// stores is branch-free (a data-dependent branch between stores makes the
// compiler wait for every outstanding store: vmcnt counts stores too).
template <int BM, int BN, int NT>
struct EpiMap {
    static constexpr int C4 = BN / 4;
    static_assert(NT % C4 == 0, "epilogue mapping");
    static constexpr int RS = NT / C4;   // rows between one thread's items
    static constexpr int KI = BM / RS;   // items per thread
};

// Residual operand of the EPI_BIAS epilogue, loaded before the C-tile staging
// and consumed after it: the loads stay in flight across the staging (no
// conversion here — converting would force a vmcnt wait before the barrier).
// rr[k] holds the raw 16 bytes of item k: the identity residual's SB hi (dwords
// 0-1) and lo (dwords 2-3) halves, or one [M][4] fp32 row of a.rx.
template <int BM, int BN, int NT>
__device__ __forceinline__ void epi_resid(const Cgemm3Args& a, int r0, int n0, int tid, f32x4* rr) {
    using E = EpiMap<BM, BN, NT>;
    const int c4 = tid % E::C4, lr0 = tid / E::C4;
    const int col = n0 + 4 * c4;
#pragma unroll
    for (int k = 0; k < E::KI; ++k) rr[k] = f32x4{0.f, 0.f, 0.f, 0.f};
    if (col + 3 >= a.Nc) return;
    if (a.resid) {   // identity residual: SB hi + lo
#pragma unroll
        for (int k = 0; k < E::KI; ++k) {
            const int row = r0 + lr0 + k * E::RS;
            if (row < a.M) {
                const unsigned short* rp = a.resid + (size_t)row * a.ldr + sbc(col);
                const f32x2 h = *reinterpret_cast<const f32x2*>(rp);
                const f32x2 l = *reinterpret_cast<const f32x2*>(rp + 32);
                rr[k] = f32x4{h[0], h[1], l[0], l[1]};
            }
        }
    } else if (a.rx) {   // small residual conv input: [M][4] fp32 rows
#pragma unroll
        for (int k = 0; k < E::KI; ++k) {
            const int row = r0 + lr0 + k * E::RS;
            if (row < a.M) rr[k] = *reinterpret_cast<const f32x4*>(a.rx + (size_t)row * 4);
        }
    }
}

template <int BM, int BN, int NT, int LDC>
__device__ __forceinline__ void epi_bias(const Cgemm3Args& a, const float* Cs, const f32x4 bv, int r0, int n0, int tid,
                                         const f32x4* rr) {
    using E = EpiMap<BM, BN, NT>;
    constexpr int C4 = E::C4, RS = E::RS, KI = E::KI;
    const int c4 = tid % C4, lr0 = tid / C4;
    const int col = n0 + 4 * c4;
    const float slope = a.act == ACT_RELU ? 0.f : (a.act == ACT_LEAKY ? 0.01f : 1.f);
    if (col + 3 < a.Nc) {
        // residual-conv weights (a.rx mode; identity mode: w = 0 and rr read as SB halves)
        const bool conv = a.resid == nullptr && a.rx != nullptr;
        float w[4][4];
#pragma unroll
        for (int e = 0; e < 4; ++e)
#pragma unroll
            for (int c = 0; c < 4; ++c) w[e][c] = conv && c < a.rxc ? a.rw[(col + e) * a.rxc + c] : 0.f;
#pragma unroll
        for (int k = 0; k < KI; ++k) {
            const int lr = lr0 + k * RS, row = r0 + lr;
            if (row >= a.M) continue;
            f32x4 v = *reinterpret_cast<const f32x4*>(Cs + lr * LDC + 4 * c4) + bv;
            const f16x4 h = __builtin_bit_cast(f16x4, f32x2{rr[k][0], rr[k][1]});
            const f16x4 l = __builtin_bit_cast(f16x4, f32x2{rr[k][2], rr[k][3]});
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                v[e] += conv ? rr[k][0] * w[e][0] + rr[k][1] * w[e][1] + rr[k][2] * w[e][2] + rr[k][3] * w[e][3]
                             : (float)h[e] + (float)l[e];
                v[e] = v[e] > 0.f ? v[e] : slope * v[e];
            }
            if (a.out_h) {
                f16x4 h, l;
                split4(v, h, l);
                unsigned short* o = a.out_h + (size_t)row * a.ldo + sbc(col);
                *reinterpret_cast<f16x4*>(o) = h;
                *reinterpret_cast<f16x4*>(o + 32) = l;
            }
            if (a.out_f) {
                float* of = a.out_f + (size_t)row * a.ldf + col;
                if ((a.ldf & 3) == 0) {
                    *reinterpret_cast<f32x4*>(of) = v;
                } else {
#pragma unroll
                    for (int e = 0; e < 4; ++e) of[e] = v[e];
                }
            }
        }
    } else if (col < a.Nc) {
        // ragged last column group (fp32 outputs only, e.g. the 66 pose values)
        for (int k = 0; k < KI; ++k) {
            const int lr = lr0 + k * RS, row = r0 + lr;
            if (row >= a.M) continue;
            for (int e = 0; e < 4 && col + e < a.Nc; ++e) {
                float v = Cs[lr * LDC + 4 * c4 + e] + bv[e];
                if (a.resid) {
                    const unsigned short* rp = a.resid + (size_t)row * a.ldr + sbc(col + e);
                    v += (float)__builtin_bit_cast(_Float16, rp[0]) + (float)__builtin_bit_cast(_Float16, rp[32]);
                }
                v = v > 0.f ? v : slope * v;
                if (a.out_h) {
                    const _Float16 h = (_Float16)v;
                    const _Float16 l = (_Float16)(v - (float)h);
                    a.out_h[(size_t)row * a.ldo + sbc(col + e)] = __builtin_bit_cast(unsigned short, h);
                    a.out_h[(size_t)row * a.ldo + sbc(col + e) + 32] = __builtin_bit_cast(unsigned short, l);
                }
                if (a.out_f) a.out_f[(size_t)row * a.ldf + col + e] = v;
            }
        }
    }
}

}  // namespace tik
