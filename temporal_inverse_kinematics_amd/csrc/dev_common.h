// dev_common.h — device helpers shared by the gfx950 kernels: vector types,
// the COCO-17 hop<=2 adjacency mask of the graph mix, direct global->LDS
// buffer DMA (buffer_load ... lds, out-of-range offsets read zeros), counted
// vmcnt waits and the LDS barrier.
#pragma once
#include <hip/hip_runtime.h>

namespace tik {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

// column w of the COCO-17 hop<=2 adjacency (Graph('coco','uniform',max_hop=2),
// mmskeleton/ops/st_gcn/graph.py:76-133): bit v set <=> A[v][w] != 0 (107 entries)
__host__ __device__ constexpr unsigned coco_hop2_mask3(int w) {
    constexpr unsigned m[17] = {0x1Fu,   0x3Fu,   0x5Fu,   0x8EFu,   0x1177u, 0x3BFAu, 0x5DFCu, 0xAE8u,  0x1570u,
                                0x2A0u,  0x540u,  0xF8E8u, 0x17970u, 0xB820u, 0x15840u, 0xA800u, 0x15000u};
    return m[w];
}

// ---- layer 0's spatial half, mix first: with C0 <= 4 input channels the
// 17 x 17 graph mix commutes with the 1x1 conv (both linear; the conv bias is
// inside bias2), so z[w] = bias2[w] + (sum_v A[v][w] x[v]) . Wg', mixing 4
// channels once per (frame, joint) instead of 64 per output. Shared by the layered
// kernel (layer0.hip) and the whole-block kernel (xblock.hip), which must agree
// bit for bit. x4: the frame's 17 data_bn'd keypoints as 4 floats each (4th = 0);
// amv: A_eff across the wave (lane l of amv[k] = A[64 k + l], v_readlane).
template <bool SPARSE>
__device__ __forceinline__ f32x4 l0_mix_in(const float* x4, const float (&amv)[5], int wj) {
    f32x4 u = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int v = 0; v < 17; ++v)
        if (!SPARSE || ((coco_hop2_mask3(wj) >> v) & 1u)) {
            const float av = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, amv[(v * 17 + wj) / 64]), (v * 17 + wj) % 64));
            const f32x4 xv = *reinterpret_cast<const f32x4*>(x4 + 4 * v);
            u = f32x4{fmaf(av, xv[0], u[0]), fmaf(av, xv[1], u[1]), fmaf(av, xv[2], u[2]), fmaf(av, xv[3], u[3])};
        }
    return u;
}
// the 1x1 conv of a mixed joint for 4 output channels + bias2, ReLU
__device__ __forceinline__ f32x4 l0_conv_relu(const f32x4 u, const float (&w)[4][4], const f32x4 b) {
    f32x4 z;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        const float s = fmaf(u[3], w[e][3], fmaf(u[2], w[e][2], fmaf(u[1], w[e][1], fmaf(u[0], w[e][0], b[e]))));
        z[e] = s > 0.f ? s : 0.f;
    }
    return z;
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

// dma16 as inline asm: invisible to the compiler's vmcnt bookkeeping (no wait before
// later accesses of the LDS it writes, not counted either); the caller orders every
// use with an explicit wait_vm (loads, stores and DMAs retire vmcnt in issue order)
__device__ __forceinline__ void dma16_asm(const i32x4 r, void* dst, unsigned voff) {
    const unsigned m = (unsigned)(unsigned long long)(__attribute__((address_space(3))) unsigned char*)dst;
    asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds" ::"s"(m), "v"(voff), "s"(r) : "memory", "m0");
}

constexpr unsigned DMA_OOB = 0x80000000u;

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

}  // namespace tik
