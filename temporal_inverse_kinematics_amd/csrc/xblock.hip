// xblock.hip — the first two ST-GCN blocks (64 channels, stride 1) as WHOLE
// blocks in bf16x3: the spatial half's output z never leaves the CU.
//
// Layered, a block is two launches: G (x -> z) and T (z, x -> out), five
// activation streams through HBM (read x, write z, read z + taps, read x,
// write out). Here one persistent workgroup per CU walks tiles of F = 10
// output frames (12 input frames: one halo frame each side for the taps):
//   block 0 (RAW): z0 = ReLU(mix(data_bn(keypoints) . Wg0') + bias2) in fp32
//     VALU (layer0.hip's gcn0 arithmetic) straight into the LDS z image;
//   block 1: G = x . Wg1' on MFMA from an LDS x image of the tile's 12 input
//     frames (DMA'd during the previous tile's T), transposed so that pixel
//     block j is joint j of the 12 frames: each lane ends with 4 channels of
//     one frame for ALL 17 joints and the graph mix runs in registers;
//   then T (3 taps) on MFMA from the z image (tap k of output pixel p is z row
//   p + 17 k, or the zero row past a window edge), + bias, + the residual
//   (block 0: the 3 -> 64 conv of the data_bn'd keypoints; block 1: x, read
//   from the x image before the next tile's DMA overwrites it), ReLU.
// Block 0 writes its output as three bf16 planes per element ("P3": row =
// [p0 x 64 | p1 x 64 | p2 x 64], x = p0 + p1 + p2 exactly), so block 1 DMAs
// MFMA-ready operands and never splits them (its four channel-group waves all
// read every pixel: split on read, each would split every element again).
// Block 1 writes fp32 rows for the layered layers that follow.
// Weights live in registers for the whole launch (weight-stationary): wave w
// owns output channels 16 (w & 3) .. +15, its Wt' planes (3 taps x 2 K blocks
// x 3 planes = 72 VGPRs) and Wg' planes (24) preloaded in the MFMA operand
// layout by xblock_pack_weights. Same products and K order as the layered
// xgemm path (bf16x3: the six p_i q_j with i + j <= 2, fp32 accumulation).
// HBM per pixel: block 0 reads 12 B and writes 384 B (was 256 + 12 + 768 B);
// block 1 reads 384 B and writes 256 B (was 256 x 5 B).
#include <algorithm>
#include <type_traits>

#include "xgemm_dev.h"
#include "xblock.h"
#include "common.h"

namespace tik {

namespace xb {
constexpr int V = 17, C = 64, F = 10, FIN = F + 2;
constexpr int ROWB = 3 * C * 2;                        // 384 B per P3 row
constexpr int ZROWS = FIN * V, ZR = ZROWS;             // z image rows + the zero row
constexpr int ZBYTES = (ZROWS + 1) * ROWB;             // 78,720
constexpr int XUNITS = ZROWS * 24, XINST = (XUNITS + 63) / 64;   // 16-B units of the x image, DMA instructions
constexpr int XBYTES = XINST * 1024;                   // 78,848 (padded to whole DMA instructions)
constexpr int B2BYTES = V * C * 4;                     // bias2 for the mix
constexpr int KPBYTES = FIN * V * 4 * 4;               // RAW: data_bn'd keypoints, 4 floats per pixel
constexpr int SMEM1 = ZBYTES + XBYTES + B2BYTES;       // block 1
constexpr int UBYTES = FIN * V * 16;                   // RAW: the mixed keypoints u[f][w] (4 floats)
constexpr int SMEM0 = ZBYTES + KPBYTES + UBYTES;       // block 0
constexpr int TPX = F * V, TBLK = (TPX + 15) / 16;     // 170 output pixels in 11 blocks of 16
static_assert(SMEM1 <= 163840, "LDS");
}  // namespace xb

// unit u (16 B: 8 channels of one plane segment) of P3 image row R sits at u ^ (R & 7)
__device__ __forceinline__ int xb_unit(int R, int plane, int u) { return R * xb::ROWB + plane * 128 + ((u ^ (R & 7)) << 4); }
// block 1's x image (joint-major, row R = FIN j + f): unit u at u ^ ((R + j) & 7). Its G reads
// (16 frames of one joint) stay conflict-free, and the residual reads (consecutive pixels: joints
// j, j + 1, ... of one frame, rows FIN apart, which R & 7 put on 2 bank groups: 6x conflicts on
// average) spread over all 8 units (1.9x)
__device__ __forceinline__ int xb_xunit(int R, int j, int plane, int u) { return R * xb::ROWB + plane * 128 + ((u ^ ((R + j) & 7)) << 4); }

template <bool RAW>
__global__ __launch_bounds__(512, 1) void xblock_kernel(XBlkArgs a) {
    using namespace xb;
    __shared__ __attribute__((aligned(16))) unsigned char smem[RAW ? SMEM0 : SMEM1];
    unsigned char* const zimg = smem;
    unsigned char* const ximg = smem + ZBYTES;            // block 1: x image; block 0: keypoint image
    float* const b2s = reinterpret_cast<float*>(smem + ZBYTES + XBYTES);

    // tid / lane / g are re-made opaque every tile (asm below): hoisted out of the
    // tile loop, every lane-derived address would stay live across it and spill
    int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    int g = lane >> 4;
    const int cg = wave & 3, ph = wave >> 2;              // channel group (16 channels), T pixel half
    const int QO = a.nframes, T = a.T;
    const int ntiles = (QO + F - 1) / F;
    int t_begin, t_end;
    {   // persistent: a contiguous run of tiles per workgroup, runs ordered per XCD
        const int nwg = gridDim.x, bid = blockIdx.x;
        const int per = nwg >> 3, rem = nwg & 7, x = bid & 7, k = bid >> 3;
        const int s = x < rem ? x * (per + 1) + k : rem * (per + 1) + (x - rem) * per + k;
        t_begin = (int)((long long)s * ntiles / nwg);
        t_end = (int)((long long)(s + 1) * ntiles / nwg);
    }
    if (t_begin >= t_end) return;

    // ---- weights in registers (MFMA A operand: lane l = output channel 16 cg + (l & 15), K group l >> 4).
    // Wt' (72 VGPRs) stays resident: with the gcn split by joint halves a wave
    // holds 9 joints' accumulators during G (36 VGPRs), so Wt' fits beside them
    // (it was re-loaded every tile before, ~2k cycles of L2 traffic per tile)
    xbf16x8 wt[3][2][3];   // [tap][K block][plane]
    auto load_wt = [&]() __attribute__((always_inline)) {
        const unsigned short* wp = a.wtp;
        asm volatile("" : "+s"(wp));   // opaque: not hoisted out of the tile loop
#pragma unroll
        for (int k = 0; k < 3; ++k)
#pragma unroll
            for (int kb = 0; kb < 2; ++kb)
#pragma unroll
                for (int p = 0; p < 3; ++p)
                    wt[k][kb][p] = *reinterpret_cast<const xbf16x8*>(wp + ((((size_t)cg * 6 + k * 2 + kb) * 3 + p) * 64 + lane) * 8);
    };
    xbf16x8 wg[RAW ? 1 : 2][3];
    if constexpr (!RAW) {
#pragma unroll
        for (int kb = 0; kb < 2; ++kb)
#pragma unroll
            for (int p = 0; p < 3; ++p)
                wg[kb][p] = *reinterpret_cast<const xbf16x8*>(a.wgp + ((((size_t)cg * 2 + kb) * 3 + p) * 64 + lane) * 8);
    }
    // A_eff in 5 VGPRs across the wave (read back with v_readlane: wave-uniform operands)
    float amv[5];
#pragma unroll
    for (int k = 0; k < 5; ++k) amv[k] = 64 * k + lane < V * V ? a.amix[64 * k + lane] : 0.f;
    // this lane's 4 output channels of T and their bias
    int cho = 16 * cg + 4 * g;
    const f32x4 bv = *reinterpret_cast<const f32x4*>(a.bias + cho);
    float rw[4][4];   // block 0: residual conv weights of the 4 channels
#pragma unroll
    for (int e = 0; e < 4; ++e)
#pragma unroll
        for (int c = 0; c < 4; ++c) rw[e][c] = RAW && c < a.c0 ? a.rw[(cho + e) * a.c0 + c] : 0.f;

    // ---- LDS constants: the zero row; block 1: bias2
    for (int i = tid; i < ROWB / 16; i += 512) *reinterpret_cast<f32x4*>(zimg + ZR * ROWB + 16 * i) = f32x4{0.f, 0.f, 0.f, 0.f};
    if constexpr (!RAW)
        for (int i = tid; i < V * C; i += 512) b2s[i] = a.bias2[i];

    // ---- block 1: the x image of a tile (joint-major rows R = 12 j + f, f = input frame q0 - 1 + f)
    const i32x4 rX = buf_rsrc(RAW ? nullptr : (const void*)a.xp3, RAW ? 0u : (unsigned)((long long)QO * V * ROWB));
    // the tile-invariant part of each DMA lane's source offset, made once: (frame f of
    // the 12, joint j, plane, swizzled unit) -> byte offset from the tile's first input
    // frame row | f << 24 | bit 31 = past the image (the per-tile work is then an add
    // and a range check instead of two divisions per instruction)
    constexpr int NXI = (XINST + 7) / 8;   // DMA instructions per wave
    unsigned xpre[NXI];
#pragma unroll
    for (int i = 0; i < NXI; ++i) {
        const int ins = wave + 8 * i;
        const int U = ins * 64 + lane;
        const int R = U / 24, k = U - R * 24, plane = k >> 3, up = k & 7;
        const int j = R / FIN, f = R - j * FIN;
        xpre[i] = U < XUNITS && ins < XINST ? (unsigned)((f * V + j) * ROWB + plane * 128 + ((up ^ ((R + j) & 7)) << 4)) | ((unsigned)f << 24)
                                            : 0x80000000u;
    }
    auto issue_x = [&](int tile) __attribute__((always_inline)) {
        const int q0 = tile * F;
#pragma unroll
        for (int i = 0; i < NXI; ++i) {
            const int ins = wave + 8 * i;
            if (ins >= XINST) break;
            const unsigned c = xpre[i];
            const int q = q0 - 1 + (int)((c >> 24) & 0x7F);
            const bool ok = !(c >> 31) && q >= 0 && q < QO;
            const unsigned off = ok ? (unsigned)((long long)(q0 - 1) * V * ROWB) + (c & 0xFFFFFFu) : DMA_OOB;
            // nt cache policy (aux 2): XB1 -1.6 % (profiles/r06_ab_xblock_nt_dma.txt)
            tik_llvm_raw_buffer_load_lds(rX, (__attribute__((address_space(3))) unsigned*)(ximg + ins * 1024), 16, (int)off, 0, 0, 2);
        }
    };
    // ---- block 0: raw keypoints of a tile, loaded a tile ahead into registers
    constexpr int KNE = RAW ? (FIN * V * 4 + 511) / 512 : 1;
    float kx[KNE], ksc[KNE], ksh[KNE];
    bool kok[KNE];
    auto load_kp = [&](int tile) __attribute__((always_inline)) {
#pragma unroll
        for (int jj = 0; jj < KNE; ++jj) {
            const int i = tid + 512 * jj, c = i & 3, p = i >> 2;
            const int v = p % V, fr = tile * F - 1 + p / V;
            kok[jj] = RAW && i < FIN * V * 4 && c < a.c0 && fr >= 0 && fr < QO;
            kx[jj] = kok[jj] ? a.xraw[((size_t)fr * V + v) * a.c0 + c] : 0.f;
        }
    };
    if constexpr (RAW) {
#pragma unroll
        for (int jj = 0; jj < KNE; ++jj) {
            const int i = tid + 512 * jj, c = i & 3, v = (i >> 2) % V;
            const bool ok = i < FIN * V * 4 && c < a.c0;
            ksc[jj] = ok ? a.bn_sc[v * a.c0 + c] : 0.f;
            ksh[jj] = ok ? a.bn_sh[v * a.c0 + c] : 0.f;
        }
        load_kp(t_begin);
    } else {
        // LDS writes above before the first DMA (an LDS access behind an LDS-DMA
        // gets a compiler vmcnt(0): possible alias)
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        issue_x(t_begin);
    }

    // T: this wave's output pixel blocks (ph 0: blocks 0-5, ph 1: 6-10)
    constexpr int NB = (TBLK + 1) / 2;   // 6
    const int blk0 = ph * NB;
    const int nblk = ph == 0 ? NB : TBLK - NB;

#ifdef TIK_XTRACE
    const bool tr = a.trace != nullptr && (wave == 0 || wave == 4);
#else
    constexpr bool tr = false;
#endif
    unsigned long long ph_[8] = {0, 0, 0, 0, 0, 0, 0, 0}, tlast = 0;   // 6 res reads, 7 barrier + next-tile DMA issue (block 1)
    auto stamp = [&](int i) __attribute__((always_inline)) {
        if (tr) {
            const unsigned long long t = __builtin_amdgcn_s_memtime();
            if (i >= 0) ph_[i] += t - tlast;
            tlast = t;
        }
    };
    load_wt();
    // the compiler's own wait for the Wt' loads goes here (an opaque use), not
    // inside the tile loop behind DMAs it would have to count
#pragma unroll
    for (int k = 0; k < 3; ++k)
#pragma unroll
        for (int kb = 0; kb < 2; ++kb)
#pragma unroll
            for (int p = 0; p < 3; ++p) asm volatile("" : "+v"(wt[k][kb][p]));
    for (int tile = t_begin; tile < t_end; ++tile) {
        const int q0 = tile * F;
        stamp(-1);
        asm volatile("" : "+v"(tid), "+v"(lane));
        g = lane >> 4;
        cho = 16 * cg + 4 * g;
        // ================= 1. z image of the tile's 12 input frames
        if constexpr (RAW) {
            // data_bn(keypoints) -> keypoint image (the previous tile's T finished reading it)
            float* kps = reinterpret_cast<float*>(ximg);
#pragma unroll
            for (int jj = 0; jj < KNE; ++jj) {
                const int i = tid + 512 * jj;
                if (i < FIN * V * 4) kps[i] = kok[jj] ? fmaf(kx[jj], ksc[jj], ksh[jj]) : 0.f;
            }
            __syncthreads();
            stamp(0);
            if (tile + 1 < t_end) load_kp(tile + 1);   // lands under this tile's work
            // the graph mix first, on the 4-channel keypoints (dev_common.h l0_mix_in, as the
            // layered gcn0_kernel): u[f][w] once per (frame, joint); wave wv takes the joints
            // w = wv (mod 8) (wave-uniform: v_readlane coefficients), lane = frame
            f32x4* const us = reinterpret_cast<f32x4*>(ximg + KPBYTES);
            {
                const int fl = lane;
                if (fl < FIN) {
#pragma unroll
                    for (int wj = 0; wj < V; ++wj)
                        if ((wj & 7) == wave) {
                            if (a.mix_sparse) us[fl * V + wj] = l0_mix_in<true>(kps + fl * V * 4, amv, wj);
                            else us[fl * V + wj] = l0_mix_in<false>(kps + fl * V * 4, amv, wj);
                        }
                }
            }
            __syncthreads();
            // then the 1x1 conv + bias2 + ReLU, split into the z image: thread (frame f,
            // channel quad c4) of a joint half: waves 0-3 joints 0-8, waves 4-7 joints 9-16
            const int f = tid & 15, c4 = (tid >> 4) & 15, half = wave >> 2, co = 4 * c4;
            if (f < FIN) {
                float w[4][4];
#pragma unroll
                for (int e = 0; e < 4; ++e)
#pragma unroll
                    for (int c = 0; c < 4; ++c) w[e][c] = c < a.c0 ? a.wg0[(co + e) * a.ldwg0 + c] : 0.f;
                auto conv_half = [&](auto w0c, auto w1c) __attribute__((always_inline)) {
                    constexpr int W0 = decltype(w0c)::value, W1 = decltype(w1c)::value;
#pragma unroll
                    for (int wj = W0; wj < W1; ++wj) {
                        const f32x4 z = l0_conv_relu(us[f * V + wj], w, *reinterpret_cast<const f32x4*>(a.bias2 + wj * C + co));
                        // split into the three planes of z image row f * 17 + wj, channels co .. co + 3
                        xbf16x8 p0, p1, p2;
                        xsplit8(z, z, p0, p1, p2);
                        const int R = f * V + wj, u = co >> 3, o = (co & 7) * 2;
                        typedef __bf16 xbf16x4 __attribute__((ext_vector_type(4)));
                        *reinterpret_cast<xbf16x4*>(zimg + xb_unit(R, 0, u) + o) = xbf16x4{p0[0], p0[1], p0[2], p0[3]};
                        *reinterpret_cast<xbf16x4*>(zimg + xb_unit(R, 1, u) + o) = xbf16x4{p1[0], p1[1], p1[2], p1[3]};
                        *reinterpret_cast<xbf16x4*>(zimg + xb_unit(R, 2, u) + o) = xbf16x4{p2[0], p2[1], p2[2], p2[3]};
                    }
                };
                using I0 = std::integral_constant<int, 0>;
                using I9 = std::integral_constant<int, 9>;
                using I17 = std::integral_constant<int, 17>;
                if (half) conv_half(I9{}, I17{});
                else conv_half(I0{}, I9{});
            }
        } else {
            // x image landed (every wave waits for its own DMA share, then the barrier)
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            stamp(0);
            // G transposed, split by joint halves: waves 0-3 joints 0-8, waves 4-7 joints
            // 9-16 (channel group cg = wave & 3 on both); the halves swap accumulators
            // through the z image (free until the mix writes it), then each half mixes
            // its own output joints. Same MFMAs and mix order as one wave doing all 17.
            auto run_half = [&](auto jhc) __attribute__((always_inline)) {
                constexpr int JH = decltype(jhc)::value, J0 = JH ? 9 : 0, J1 = JH ? V : 9;
                f32x4 acc[V];
#pragma unroll
                for (int j = 0; j < V; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
                const int fs = lane & 15, fr = fs < FIN ? fs : fs - FIN;
                // pixel block j = joint j of the tile's frames (lane & 15 = frame slot;
                // slots 12-15 re-read slots 0-3: broadcast, discarded). Operand ring: step
                // s + XPF's planes are read while step s's MFMAs run
                constexpr int XPF = 2, S0 = 2 * J0, S1 = 2 * J1;
                xbf16x8 xb[XPF + 1][3];
                auto rd = [&](int s, xbf16x8 (&d)[3]) __attribute__((always_inline)) {
                    const int R = (s >> 1) * FIN + fr, kb = s & 1;
#pragma unroll
                    for (int p = 0; p < 3; ++p) d[p] = *reinterpret_cast<const xbf16x8*>(ximg + xb_xunit(R, s >> 1, p, 4 * kb + g));
                };
#pragma unroll
                for (int s = S0; s < S0 + XPF; ++s) rd(s, xb[(s - S0) % (XPF + 1)]);
#pragma unroll
                for (int s = S0; s < S1; ++s) {
                    const int j = s >> 1, kb = s & 1;
                    if (s + XPF < S1) rd(s + XPF, xb[(s + XPF - S0) % (XPF + 1)]);
                    __builtin_amdgcn_sched_barrier(0);
                    const xbf16x8(&x)[3] = xb[(s - S0) % (XPF + 1)];
                    // (w0,x2) (w1,x1) (w2,x0) (w0,x1) (w1,x0) (w0,x0): xgemm's product order
                    acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wg[kb][0], x[2], acc[j], 0, 0, 0);
                    acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wg[kb][1], x[1], acc[j], 0, 0, 0);
                    acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wg[kb][2], x[0], acc[j], 0, 0, 0);
                    acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wg[kb][0], x[1], acc[j], 0, 0, 0);
                    acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wg[kb][1], x[0], acc[j], 0, 0, 0);
                    acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wg[kb][0], x[0], acc[j], 0, 0, 0);
                    __builtin_amdgcn_sched_barrier(0);
                }
                // exchange: [joint][cg][lane] f32x4 in the z image rows (69.6 KB, below the zero row)
                f32x4* xch = reinterpret_cast<f32x4*>(zimg);
#pragma unroll
                for (int j = J0; j < J1; ++j) xch[(j * 4 + cg) * 64 + lane] = acc[j];
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                __builtin_amdgcn_s_barrier();
#pragma unroll
                for (int j = 0; j < V; ++j)
                    if (j < J0 || j >= J1) acc[j] = xch[(j * 4 + cg) * 64 + lane];
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                __builtin_amdgcn_s_barrier();   // every wave's exchange reads done before the z image writes
                // graph mix in registers: lane = frame fs, channels cho .. cho + 3, output
                // joints J0 .. J1 (xgemm.hip xmix_store's order: bias2, then v ascending)
                if (fs < FIN) {
                    auto mix_half = [&](auto sparse) __attribute__((always_inline)) {
                        constexpr bool SP = decltype(sparse)::value;
#pragma unroll
                        for (int w = J0; w < J1; ++w) {
                            f32x4 z = *reinterpret_cast<const f32x4*>(b2s + w * C + cho);
#pragma unroll
                            for (int v = 0; v < V; ++v)
                                if (!SP || ((coco_hop2_mask3(w) >> v) & 1u)) {
                                    const float av = __builtin_bit_cast(
                                        float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, amv[(v * V + w) / 64]), (v * V + w) % 64));
                                    z += av * acc[v];
                                }
#pragma unroll
                            for (int e = 0; e < 4; ++e) z[e] = z[e] > 0.f ? z[e] : 0.f;
                            xbf16x8 p0, p1, p2;
                            xsplit8(z, z, p0, p1, p2);
                            const int R = fs * V + w, u = cho >> 3, o = (cho & 7) * 2;
                            typedef __bf16 xbf16x4 __attribute__((ext_vector_type(4)));
                            *reinterpret_cast<xbf16x4*>(zimg + xb_unit(R, 0, u) + o) = xbf16x4{p0[0], p0[1], p0[2], p0[3]};
                            *reinterpret_cast<xbf16x4*>(zimg + xb_unit(R, 1, u) + o) = xbf16x4{p1[0], p1[1], p1[2], p1[3]};
                            *reinterpret_cast<xbf16x4*>(zimg + xb_unit(R, 2, u) + o) = xbf16x4{p2[0], p2[1], p2[2], p2[3]};
                        }
                    };
                    if (a.mix_sparse) mix_half(std::true_type{});
                    else mix_half(std::false_type{});
                }
            };
            // (both halves run the same number of s_barrier)
            if (ph == 0) run_half(std::integral_constant<int, 0>{});
            else run_half(std::integral_constant<int, 1>{});
        }
        stamp(1);
        __syncthreads();   // z image complete
        stamp(2);

        // ================= 2. the residual of this wave's output pixels (before the
        // next tile's data overwrites its source), then the next tile's x image
        // output pixel p = 17 fo + joint (fo = local output frame), channels cho .. +3
        f32x4 res[NB];
#pragma unroll
        for (int b = 0; b < NB; ++b) {
            const int p = (blk0 + b) * 16 + (lane & 15);
            const int fo = p / V, jt = p - fo * V;
            res[b] = f32x4{0.f, 0.f, 0.f, 0.f};
            if (b < nblk && p < TPX) {
                if constexpr (RAW) {
                    const float* xp = reinterpret_cast<const float*>(ximg) + ((fo + 1) * V + jt) * 4;
                    res[b] = f32x4{xp[0], xp[1], xp[2], xp[3]};   // data_bn'd keypoints (residual conv input)
                } else {
                    const int R = jt * FIN + fo + 1, u = cho >> 3, o = (cho & 7) * 2;
                    typedef __bf16 xbf16x4 __attribute__((ext_vector_type(4)));
                    const xbf16x4 h0 = *reinterpret_cast<const xbf16x4*>(ximg + xb_xunit(R, jt, 0, u) + o);
                    const xbf16x4 h1 = *reinterpret_cast<const xbf16x4*>(ximg + xb_xunit(R, jt, 1, u) + o);
                    const xbf16x4 h2 = *reinterpret_cast<const xbf16x4*>(ximg + xb_xunit(R, jt, 2, u) + o);
#pragma unroll
                    for (int e = 0; e < 4; ++e) res[b][e] = ((float)h0[e] + (float)h1[e]) + (float)h2[e];   // exact: x = p0 + p1 + p2
                }
            }
        }
        if constexpr (!RAW) {
            // every wave done with the x image (LDS reads; T's register operands are
            // resident, so nothing in T waits on this DMA); s_barrier alone:
            // __syncthreads' release fence would wait for the previous T's stores
            stamp(6);
            lds_barrier();
            if (tile + 1 < t_end) issue_x(tile + 1);
            stamp(7);
        }
        stamp(3);

        // ================= 3. T: 3 taps x 2 K blocks from the z image, this wave's pixel
        // blocks, as one flattened (block, K step) loop so the operand ring runs across blocks
        int rows[NB][3];
#pragma unroll
        for (int b = 0; b < NB; ++b) {
            const int p = (blk0 + b) * 16 + (lane & 15);
            const int fo = p / V, jt = p - fo * V;
            const int q = q0 + fo, tw = q % T;
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                const bool ok = b < nblk && p < TPX && q < QO && tw + k - 1 >= 0 && tw + k - 1 < T;
                rows[b][k] = ok ? (fo + k) * V + jt : ZR;
            }
        }
        {
            constexpr int ZPF = 2, NS = 6 * NB;
            xbf16x8 zb[ZPF + 1][3];
            auto rdz = [&](int i, xbf16x8 (&d)[3]) __attribute__((always_inline)) {
                const int b = i / 6, s = i % 6, k = s % 3, kb = s / 3;
#pragma unroll
                for (int pl = 0; pl < 3; ++pl) d[pl] = *reinterpret_cast<const xbf16x8*>(zimg + xb_unit(rows[b][k], pl, 4 * kb + g));
            };
#pragma unroll
            for (int i = 0; i < ZPF; ++i) rdz(i, zb[i]);
            f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int i = 0; i < NS; ++i) {   // K step s = (K block s / 3, tap s % 3): xgemm's K order
                const int b = i / 6, s = i % 6;
                if (b >= nblk) break;
                if (i + ZPF < NS) rdz(i + ZPF, zb[(i + ZPF) % (ZPF + 1)]);
                __builtin_amdgcn_sched_barrier(0);
                const xbf16x8(&z)[3] = zb[i % (ZPF + 1)];
                const xbf16x8(&w)[3] = wt[s % 3][s / 3];
                acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[0], z[2], acc, 0, 0, 0);
                acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[1], z[1], acc, 0, 0, 0);
                acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[2], z[0], acc, 0, 0, 0);
                acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[0], z[1], acc, 0, 0, 0);
                acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[1], z[0], acc, 0, 0, 0);
                acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[0], z[0], acc, 0, 0, 0);
                __builtin_amdgcn_sched_barrier(0);
                if (s < 5) continue;
                // epilogue of block b: lane = pixel p, channels cho .. cho + 3
                const int p = (blk0 + b) * 16 + (lane & 15);
                const int fo = p / V;
                const int q = q0 + fo;
                const long long row = (long long)q0 * V + p;
                const bool st = p < TPX && q < QO;
                f32x4 v = acc;
                acc = f32x4{0.f, 0.f, 0.f, 0.f};
                if constexpr (RAW) {
                    v += bv;
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        v[e] += res[b][0] * rw[e][0] + res[b][1] * rw[e][1] + res[b][2] * rw[e][2] + res[b][3] * rw[e][3];
                        v[e] = v[e] > 0.f ? v[e] : 0.f;
                    }
                    xbf16x8 p0, p1, p2;
                    xsplit8(v, v, p0, p1, p2);
                    typedef __bf16 xbf16x4 __attribute__((ext_vector_type(4)));
                    unsigned short* o = st ? a.out_p3 + row * (3 * C) + cho : reinterpret_cast<unsigned short*>(a.trash);
                    *reinterpret_cast<xbf16x4*>(o) = xbf16x4{p0[0], p0[1], p0[2], p0[3]};
                    *reinterpret_cast<xbf16x4*>(o + C) = xbf16x4{p1[0], p1[1], p1[2], p1[3]};
                    *reinterpret_cast<xbf16x4*>(o + 2 * C) = xbf16x4{p2[0], p2[1], p2[2], p2[3]};
                } else {
                    v += res[b];   // (acc + x) + bias: xgemm's identity-epilogue order
                    v += bv;
#pragma unroll
                    for (int e = 0; e < 4; ++e) v[e] = v[e] > 0.f ? v[e] : 0.f;
                    float* o = st ? a.out_f + row * C + cho : a.trash;
                    *reinterpret_cast<f32x4*>(o) = v;
                }
            }
        }
        // every wave done reading the z image (and, block 0, the keypoint image)
        // before the next tile writes them
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        stamp(4);
        __syncthreads();
        stamp(5);
    }
    if (tr && lane == 0) {
        unsigned long long* o = a.trace + 24 * (size_t)blockIdx.x + (wave == 4 ? 12 : 0);
        for (int i = 0; i < 8; ++i) o[i] = ph_[i];
        o[8] = t_end - t_begin; o[9] = 1;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

hipError_t launch_xblock(const XBlkArgs& a, bool raw, int ncu, hipStream_t st) {
    if (a.nframes <= 0) return hipSuccess;
    if (a.T <= 0 || !a.wtp || !a.amix || !a.bias || !a.trash || ncu <= 0) return hipErrorInvalidValue;
    if (raw && (!a.xraw || a.c0 < 1 || a.c0 > 4 || !a.bn_sc || !a.bn_sh || !a.wg0 || a.ldwg0 < a.c0 || !a.rw || !a.out_p3 || !a.bias2))
        return hipErrorInvalidValue;
    if (!raw && (!a.xp3 || !a.wgp || !a.bias2 || !a.out_f)) return hipErrorInvalidValue;
    if (!raw && (long long)a.nframes * xb::V * xb::ROWB >= (1LL << 31)) return hipErrorInvalidValue;   // 32-bit DMA offsets
    const int ntiles = (a.nframes + xb::F - 1) / xb::F;
    const int grid = std::min(ntiles, ncu);
    (void)hipGetLastError();
    if (raw) hipLaunchKernelGGL(xblock_kernel<true>, dim3(grid), dim3(512), 0, st, a);
    else hipLaunchKernelGGL(xblock_kernel<false>, dim3(grid), dim3(512), 0, st, a);
    return hipGetLastError();
}

int xblock_frames_per_tile() { return xb::F; }

std::vector<unsigned short> xblock_pack_weights(const float* w, int cout, int ldw, int kt, int cin) {
    // [cg][tap * (cin/32) + kb][plane][lane][8]: lane l = channel 16 cg + (l & 15), K = 32 kb + 8 (l >> 4) + e
    const int nkb = cin / 32, ns = kt * nkb, ncg = cout / 16;
    std::vector<unsigned short> out((size_t)ncg * ns * 3 * 64 * 8, 0);
    for (int c = 0; c < ncg; ++c)
        for (int tap = 0; tap < kt; ++tap)
            for (int kb = 0; kb < nkb; ++kb)
                for (int l = 0; l < 64; ++l)
                    for (int e = 0; e < 8; ++e) {
                        const int co = 16 * c + (l & 15), ci = 32 * kb + 8 * (l >> 4) + e;
                        unsigned short p[3];
                        tik_host::split_bf16x3(w[(size_t)co * ldw + (size_t)tap * cin + ci], p[0], p[1], p[2]);
                        const int s = tap * nkb + kb;
                        for (int pl = 0; pl < 3; ++pl) out[((((size_t)c * ns + s) * 3 + pl) * 64 + l) * 8 + e] = p[pl];
                    }
    return out;
}

}  // namespace tik
