// xgemm.hip — bf16x3 implicit GEMM on fp32 activations (see xgemm.h).
//
// Tile: BM = 32 NW rows x BN columns. Default NW = 4: a 128-row, 256-thread
// workgroup of <= 80 KB LDS, TWO per CU, so one workgroup's prologue (first
// DMA round trip) and epilogue run under the other's main loop (one 256-row
// 8-wave workgroup per CU measured 3-9 % slower; removed). Wave w owns
// rows 32w..32w+31 (two 16-row fragments) and ALL BN columns, so each A
// element is read from LDS and split into bf16 planes exactly once per K
// step, in registers, by the wave that uses it (no split pass, no extra LDS);
// the weight planes are read by every wave.
//
// LDS, per stage: the A image (BM rows x 32 fp32 = 128 B per row) and the B
// image (3 planes x BN columns x 32 bf16 = 64 B per column), both written by
// LDS-DMA (buffer_load ... lds, 16 B per lane). A: 2 slots, each wave DMAs
// its own rows 2 steps ahead (no barrier); B: LB + 1 slots, LB steps ahead,
// one barrier per K step.
//  * A row r, logical floats [8g+4h, 8g+4h+4) (g = k group of the MFMA
//    operand, h = half) at 16-B unit (g + 4h) ^ ((r >> 1) & 7): the two
//    ds_read_b128 of a fragment read are conflict-free in every lane group.
//    The DMA lane that fills unit p of row r fetches the logical unit
//    (p ^ swz(r)), so the swizzle costs nothing.
//  * B column n, k group g at unit g ^ ((-(n >> 2)) & 3) of its 64-B row:
//    conflict-free ds_read_b128 per plane; applied on the host (xgemm_pack).
// Rows past the batch, and taps outside the window (the temporal zero
// padding), DMA from an out-of-range offset of the buffer resource: zeros.
// Inside a step: the next step's A fragments are read first, then per column
// block the next block's weight reads are issued before this block's 6 FM
// MFMAs, and fragment i's split for the next step runs between block i's MFMAs.
//
// Epilogues:
//  * EPI_BIAS (transposed MFMA, so a lane holds 4 channels of a row): + bias
//    (+ the layer-0 residual conv on 4-float rows) -> activation -> float4
//    stores straight from registers; the identity residual is added before,
//    as extra K steps of exact fp32 adds from the DMA'd block-input rows.
//  * EPI_GRAPH: tiles of whole frames (7 or 15: 119 / 255 rows) staged through
//    LDS; z[f][w] = sum_v A[v][w] y[f][v] (the einsum of gconv_origin.py:61-63;
//    COCO hop<=2 pattern unrolled when A_eff fits it) + bias2[w][c], ReLU
//    (st_gcn_aaai18.py:178-179).
#include <algorithm>
#include <cstdlib>
#include <type_traits>

#include "cgemm.h"
#include "dev_common.h"
#include "common.h"
#include "xgemm.h"
#include "xgemm_dev.h"

namespace tik {

// graph mix of one frame, output joints [W0, W1): z[w] = sum_v A[v][w] y[v] +
// bias2[w], ReLU, stored. w and v are compile-time, so the sparse COCO
// pattern unrolls and the A entries are wave-uniform scalar loads.
// A_eff entry i from the 5 VGPRs that hold it across the wave (lane i % 64 of amv[i / 64])
__device__ __forceinline__ float xam(const float (&amv)[5], int i) {
    return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, amv[i / 64]), i % 64));
}

// bias2 is the tile's [17][BN] slice staged in LDS (a global load between the
// stores would wait for every store before it: vmcnt counts both)
template <int W0, int W1, bool SPARSE, int BN>
__device__ __forceinline__ void xmix_store(const f32x4 (&y)[17], const float (&amv)[5],
                                           const float* __restrict__ bias2s, int lcol, float* __restrict__ o,
                                           int ldo, bool nt) {
#pragma unroll
    for (int w = W0; w < W1; ++w) {
        f32x4 z = *reinterpret_cast<const f32x4*>(bias2s + w * BN + lcol);
        if constexpr (SPARSE) {
#pragma unroll
            for (int v = 0; v < 17; ++v)
                if ((coco_hop2_mask3(w) >> v) & 1u) z += xam(amv, v * 17 + w) * y[v];
        } else {
#pragma unroll
            for (int v = 0; v < 17; ++v) z += xam(amv, v * 17 + w) * y[v];
        }
#pragma unroll
        for (int e = 0; e < 4; ++e) z[e] = z[e] > 0.f ? z[e] : 0.f;
        xst4(o + (size_t)w * ldo, z, nt);
    }
}

// SK: a split-K launch (XArgs::ksplit > 1; its own instantiation, so the
// profiler tells it from the backbone's EPI_BIAS launches)
template <int BN, int EPI, int NW_, bool SK>
__global__ __launch_bounds__(64 * NW_, NW_ == 8 ? 1 : 2) void xgemm_kernel(XArgs a) {
    using C = XCfg<BN, EPI, NW_>;
    constexpr int NW = C::NW, NT = C::NT, FM = C::FM, FN = C::FN, NIA = C::NIA, NSA = C::NSA, NSB = C::NSB,
                  RT = C::RT, RW = C::RW, LB = C::LB, BM = C::BM;
    constexpr bool TR = C::TR;
    __shared__ __attribute__((aligned(16))) unsigned char smem[C::SMEM];   // the only LDS object

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    // phase stamps only in a -DTIK_XTRACE build: a runtime check puts a scalar
    // branch around every stamp of the K loop
#ifdef TIK_XTRACE
    const bool tr = a.trace != nullptr;
#else
    constexpr bool tr = false;
#endif
#ifdef TIK_XTUNE
    const int tune = a.tune;
#else
    constexpr int tune = 0;   // experiment bits (XArgs::tune) only in a -DTIK_XTUNE build
#endif
    unsigned long long t0 = tr ? __builtin_amdgcn_s_memtime() : 0, t_bar = 0, t_vm = 0, t1 = 0, t2 = 0, t3 = 0;
    int r0, ntile;
    {   // XCD-aware tile order: consecutive workgroup ids go to different XCDs,
        // so give each XCD a contiguous run of tiles (rows shared by neighbours stay in its L2)
        const int nwg = gridDim.x * gridDim.y, bid = blockIdx.y * gridDim.x + blockIdx.x;
        const int per = nwg >> 3, rem = nwg & 7, x = bid & 7, k = bid >> 3;
        const int swz = x < rem ? x * (per + 1) + k : rem * (per + 1) + (x - rem) * per + k;
        if (a.gm > 1) {   // groups of gm row tiles; within a group the gm rows of one column tile are adjacent
            const int gy = gridDim.y, g = swz / (a.gm * gy), w = swz - g * a.gm * gy;
            const int left = gridDim.x - g * a.gm, ge = left < a.gm ? left : a.gm;
            r0 = (g * a.gm + w % ge) * RT;
            ntile = w / ge;
        } else {
            r0 = (swz / gridDim.y) * RT;
            ntile = swz % gridDim.y;
        }
    }
    const int n0 = ntile * BN;
    const int V = a.V;
    // EPI_GRAPH: this tile's bias2[17][n0 .. n0 + BN) slice, loaded now so its
    // latency hides under the K loop (staged in LDS by the epilogue)
    constexpr int NB2 = EPI == EPI_GRAPH ? (17 * BN / 4 + NT - 1) / NT : 0;
    f32x4 b2r[NB2 > 0 ? NB2 : 1];
#pragma unroll
    for (int u = 0; u < NB2; ++u) {
        const int q = tid + u * NT, w = q / (BN / 4), c = 4 * (q - w * (BN / 4));
        b2r[u] = q < 17 * BN / 4 && n0 + c + 3 < a.Nc ? *reinterpret_cast<const f32x4*>(a.bias + w * a.Nc + n0 + c)
                                                       : f32x4{0.f, 0.f, 0.f, 0.f};
    }

    // ---- A DMA roles: instruction j of this wave fills rows (wave*NIA + j)*8 + lane/8, unit lane&7
    // (rows RW wave .. RW wave + RW - 1: exactly the rows this wave computes)
    int a_n[NIA], a_t[NIA], a_w[NIA], a_uo[NIA];
    bool a_ok[NIA];
#pragma unroll
    for (int j = 0; j < NIA; ++j) {
        const int rr = (wave * NIA + j) * 8 + (lane >> 3);
        const int row = r0 + rr;
        const int pl = (lane & 7) ^ xa_swz(rr);            // logical unit: g = pl & 3, h = pl >> 2
        a_uo[j] = 32 * (pl & 3) + 16 * (pl >> 2);         // its byte offset in the 128-B K block
        a_ok[j] = rr < RT && row < a.M;
        const int q = a_ok[j] ? row / V : 0;
        a_w[j] = a_ok[j] ? row - q * V : 0;
        a_n[j] = q / a.tout;
        a_t[j] = q - a_n[j] * a.tout;
    }
    // K steps with weight tiles (the identity steps follow); a split-K slice
    // runs packed steps kb .. kb + kmain of its single kt-1 segment
    const int kall = xgemm_kmain(a);
    int kb = 0, kmain = kall;
    if (SK) {
        const int kper = (kall + a.ksplit - 1) / a.ksplit;
        kb = blockIdx.z * kper;
        kmain = min(kper, kall - kb);
    }
    // the identity residual read in the LDS epilogue (row-major whole lines) instead of as K steps
    const bool idn_epi = TR && a.epi_lds && a.idn_epi && a.idn.src;
    const int K = SK || idn_epi ? kmain : a.ksteps;
    // B DMA: a stage's B image is one contiguous packed block; instruction q (of NIB_TOT) copies 1 KB
    const i32x4 rB = buf_rsrc(a.wp, (unsigned)((size_t)gridDim.y * kall * C::BBYTES));
    const int nbw = (C::NIB_TOT - wave + NW - 1) / NW;   // this wave's B instructions per stage (NIBW or NIBW - 1)

    // The A cursor walks (segment, 32-channel block, tap); segment slot 0 =
    // seg[0], 1 = seg[1] (or the identity when nseg == 1), 2 = the identity.
    // The per-step advance reads the blocks and taps of each slot from one
    // packed 64-bit scalar (8 bits each; a select chain over separate values
    // becomes a scratch lookup table, a dynamically indexed XSeg a kernel-argument
    // load, every step); the segment's geometry is re-read only when the tap changes.
    const bool two = a.nseg > 1;
    const unsigned long long nbkt =
        (unsigned long long)((a.seg[0].cin >> 5) | (a.seg[0].kt << 8)) |
        ((unsigned long long)(two ? (a.seg[1].cin >> 5) | (a.seg[1].kt << 8) : (a.idn.cin >> 5) | (a.idn.kt << 8)) << 16) |
        ((unsigned long long)((a.idn.cin >> 5) | (a.idn.kt << 8)) << 32);
    int ca_seg = 0, ca_tap = 0, ca_blk = kb, ca_k = 0, cb_k = 0;
    auto advance_a = [&]() __attribute__((always_inline)) {
        const unsigned f = (unsigned)(nbkt >> (16 * ca_seg));
        ++ca_k;
        if (++ca_tap >= (int)((f >> 8) & 255u)) {   // taps innermost: a block's 3 taps read overlapping rows back to back
            ca_tap = 0;
            if (++ca_blk >= (int)(f & 255u)) { ca_blk = 0; ++ca_seg; }
        }
    };
    // per row, at the segment's change: its tap-0 input frame and byte offset;
    // per step, tap k's offset is base + k frames, valid when the frame is in range
    int a_t0[NIA], a_base[NIA];
    int sg_tin = 0, sg_fb = 0, cur_seg = -1;   // the segment's frames, bytes per frame (V rows)
    i32x4 rA;
    auto prepare = [&]() __attribute__((always_inline)) {
        if (ca_seg == cur_seg) return;
        cur_seg = ca_seg;
        const XSeg sg = ca_seg == 0 ? a.seg[0] : (ca_seg == 1 && two ? a.seg[1] : a.idn);
        rA = buf_rsrc(sg.src, (unsigned)(sg.rows_in * sg.ld * 4));
        sg_tin = sg.tin;
        sg_fb = V * sg.ld * 4;
#pragma unroll
        for (int j = 0; j < NIA; ++j) {
            const int t0 = sg.stride * a_t[j] - sg.pad;
            a_t0[j] = a_ok[j] ? t0 : -(1 << 29);   // a dead row fails every tap
            a_base[j] = ((a_n[j] * sg.tin + t0) * V + a_w[j]) * sg.ld * 4 + (int)a_uo[j];
        }
    };
    auto a_slot = [&](int s) __attribute__((always_inline)) { return smem + s * C::ABYTES; };
    auto b_slot = [&](int s) __attribute__((always_inline)) { return smem + NSA * C::ABYTES + s * C::BBYTES; };
    auto issue_a = [&]() __attribute__((always_inline)) {   // the A cursor's step, into its ring slot
        prepare();
        unsigned char* A = a_slot(ca_k % NSA);
        const int soA = __builtin_amdgcn_readfirstlane(ca_blk * 128);
        const int tap = ca_tap, tb = tap * sg_fb;
        if (!(tune & 1))
#pragma unroll
            for (int j = 0; j < NIA; ++j)
                dma16(rA, A + (wave * NIA + j) * 1024,
                      (unsigned)(a_t0[j] + tap) < (unsigned)sg_tin ? (unsigned)(a_base[j] + tb) : DMA_OOB, soA);
        advance_a();
    };
    auto issue_b = [&]() __attribute__((always_inline)) {   // weight step cb_k (main steps only)
        unsigned char* B = b_slot(cb_k % NSB);
        const int soB = __builtin_amdgcn_readfirstlane((ntile * kall + kb + cb_k) * C::BBYTES);
        if (!(tune & 2))
#pragma unroll
            for (int q = 0; q < C::NIBW; ++q)
                if (q < C::NIBW - 1 || wave + q * NW < C::NIB_TOT)
                    dma16(rB, B + (wave + q * NW) * 1024, (unsigned)((wave + q * NW) * 1024 + lane * 16), soB);
        ++cb_k;
    };
    // vmcnt accounting: at step k this wave issues B(k + LB) (nbw instructions,
    // NIBW or NIBW - 1) then A(k + 2) (NIA); waits count the younger ones
    auto nA = [&](int k) __attribute__((always_inline)) { return k < K ? NIA : 0; };
    auto nB = [&](int k) __attribute__((always_inline)) { return k < kmain ? nbw : 0; };
    auto wait_steady = [&]() __attribute__((always_inline)) {   // NIA + this wave's full B share outstanding
        if constexpr (C::NIB_TOT % NW == 0) wait_vm<NIA + C::NIBW>();   // every wave issues NIBW
        else if (nbw == C::NIBW) wait_vm<NIA + C::NIBW>();
        else wait_vm<NIA + C::NIBW - 1>();
    };

    f32x4 acc[FM][FN];
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int g = lane >> 4;
    const int bsw = (-((lane & 15) >> 2)) & 3;
    const int boff = (lane & 15) * 64 + ((g ^ bsw) << 4);
    auto mma = [&](const xbf16x8& x, const xbf16x8& w, f32x4& c) __attribute__((always_inline)) {
        // TR: C^T = W . X^T, so lane l holds row (l & 15), channels 4(l >> 4) .. +3
        c = TR ? __builtin_amdgcn_mfma_f32_16x16x32_bf16(w, x, c, 0, 0, 0)
               : __builtin_amdgcn_mfma_f32_16x16x32_bf16(x, w, c, 0, 0, 0);
    };
    // this wave's A fragments of a step: fp32 rows -> three bf16 planes
    auto read_a = [&](int k, f32x4 (&lo)[FM], f32x4 (&hi)[FM]) __attribute__((always_inline)) {
        const unsigned char* A = a_slot(k % NSA);
#pragma unroll
        for (int i = 0; i < FM; ++i) {
            const int r = wave * RW + i * 16 + (lane & 15);
            lo[i] = *reinterpret_cast<const f32x4*>(A + r * 128 + ((g ^ xa_swz(r)) << 4));
            hi[i] = *reinterpret_cast<const f32x4*>(A + r * 128 + (((g + 4) ^ xa_swz(r)) << 4));
        }
    };
    xbf16x8 c0[FM], c1[FM], c2[FM];   // the current step's split A
    f32x4 alo[FM], ahi[FM];

    // ---- main steps: the split of step k+1 runs under step k's MFMAs
    // issue order: B(0) A(0) [B(1)] A(1) | per step k: B(k+LB) A(k+2), so a wait
    // for this wave's A(k) (in issue order) also retires its B(k)
    issue_b();
    issue_a();
    if (LB == 2 && 1 < kmain) issue_b();
    if (1 < K) issue_a();
    wait_vm_dyn(nA(1) + (LB == 2 ? nB(1) : 0));   // A(0) and B(0) landed
    if (tr) t1 = __builtin_amdgcn_s_memtime();
    {
        read_a(0, alo, ahi);
#pragma unroll
        for (int i = 0; i < FM; ++i) xsplit8(alo[i], ahi[i], c0[i], c1[i], c2[i]);
    }
    // one main step: MFMAs of step k on the split held in cur, with step k+1's A
    // reads and split into nxt interleaved between them (the loop below runs it
    // twice per iteration with the two register sets swapped: no copies)
    xbf16x8 d0[FM], d1[FM], d2[FM];
    // ST (steady, k + 2 < kmain: B(k+LB) and A(k+2) both exist): no conditions,
    // compile-time waits; the last steps take the general path
    auto main_step = [&](int k, auto steady, xbf16x8 (&u0)[FM], xbf16x8 (&u1)[FM], xbf16x8 (&u2)[FM], xbf16x8 (&v0)[FM],
                         xbf16x8 (&v1)[FM], xbf16x8 (&v2)[FM]) __attribute__((always_inline)) {
        constexpr bool ST = decltype(steady)::value;
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        const unsigned long long tb0 = tr ? __builtin_amdgcn_s_memtime() : 0;
        __builtin_amdgcn_s_barrier();   // every wave's B(k) landed; every wave done reading B(k-1)
        if (tr) t_bar += __builtin_amdgcn_s_memtime() - tb0;
        if (ST || k + LB < kmain) issue_b();
        if (ST || k + 2 < K) issue_a();
        // this wave's A(k+1) landed (B(k+LB), A(k+2) may still fly); past the last
        // step the read + split below run on a stale slot and are discarded
        auto wait_a_next = [&]() __attribute__((always_inline)) {
            const unsigned long long tv0 = tr ? __builtin_amdgcn_s_memtime() : 0;
            if (ST || k + 2 < kmain) wait_steady();
            else wait_vm_dyn(nB(k + LB) + nA(k + 2));
            if (tr) t_vm += __builtin_amdgcn_s_memtime() - tv0;
        };
#ifndef TIK_XORDER
        wait_a_next();
#endif
        const unsigned char* B = b_slot(k % NSB) + boff;
        // Software pipeline inside the step: the A reads of step k+1 and the
        // first weight block's reads, then per column block j the next block's
        // reads are issued BEFORE the 6 FM MFMAs of j (so no read is waited on
        // right after its issue), and a quarter of one fragment's split of step
        // k+1 runs between block j's MFMAs, one VALU per MFMA (round 6: the whole
        // split in blocks 0-1, and one step of each unrolled pair had its split
        // sunk past all its MFMAs to the next step's start, 80 VALU in a row;
        // spread and pinned, XT128 runs 6-10 % faster). sched_barriers keep the
        // blocks in this order.
        xbf16x8 bb[2][3];
        __builtin_amdgcn_sched_barrier(0);
#ifdef TIK_XORDER
        // B(k) is ready at the barrier: its first block's reads go out before the
        // wait for A(k+1), so they overlap that wait and the first MFMAs need not
        // wait for the A reads
#pragma unroll
        for (int p = 0; p < 3; ++p) bb[0][p] = *reinterpret_cast<const xbf16x8*>(B + p * C::PLANE);
        wait_a_next();
        read_a(k + 1, alo, ahi);
#else
        read_a(k + 1, alo, ahi);
#pragma unroll
        for (int p = 0; p < 3; ++p) bb[0][p] = *reinterpret_cast<const xbf16x8*>(B + p * C::PLANE);
#endif
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int j = 0; j < FN; ++j) {
            if (j + 1 < FN)
#pragma unroll
                for (int p = 0; p < 3; ++p)
                    bb[(j + 1) & 1][p] = *reinterpret_cast<const xbf16x8*>(B + p * C::PLANE + (j + 1) * 16 * 64);
            const xbf16x8(&b)[3] = bb[j & 1];
#pragma unroll
            for (int i = 0; i < FM; ++i) {
                mma(u2[i], b[0], acc[i][j]);
                mma(u1[i], b[1], acc[i][j]);
                mma(u0[i], b[2], acc[i][j]);
                mma(u1[i], b[0], acc[i][j]);
                mma(u0[i], b[1], acc[i][j]);
                mma(u0[i], b[0], acc[i][j]);
            }
            // the next step's split in 4 * FM parts spread evenly over the FN column blocks
            constexpr int PPJ = (4 * FM + FN - 1) / FN;
#pragma unroll
            for (int pp = 0; pp < PPJ; ++pp) {
                const int p = j * PPJ + pp;
                if (p < 4 * FM && !(tune & 8)) {
                    xsplit8_part(alo[p >> 2], ahi[p >> 2], v0[p >> 2], v1[p >> 2], v2[p >> 2], p & 3);
                    // pin the finished fragment here (left alone, the split of one step of a pair
                    // was sunk past its MFMAs to the next step's start)
                    if ((p & 3) == 3) asm volatile("" : "+v"(v0[p >> 2]), "+v"(v1[p >> 2]), "+v"(v2[p >> 2]));
                }
            }
            if (j + 1 < FN) __builtin_amdgcn_sched_group_barrier(0x100, 3, 0);
#pragma unroll
            for (int q = 0; q < 6 * FM; ++q) {
                __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                __builtin_amdgcn_sched_group_barrier(0x002, 1, 0);
            }
            __builtin_amdgcn_sched_barrier(0);
        }
        if constexpr (LB == 1) {   // B(k+1) landed before the next step's barrier (only A(k+2) younger)
            const unsigned long long tv0 = tr ? __builtin_amdgcn_s_memtime() : 0;
            if (ST) wait_vm<NIA>();
            else wait_vm_dyn(nA(k + 2));
            if (tr) t_vm += __builtin_amdgcn_s_memtime() - tv0;
        }
    };
    const std::true_type steady{};
    const std::false_type general{};
    int k = 0;
    for (; k + 3 < kmain; k += 2) {   // both steps of the pair steady
        main_step(k, steady, c0, c1, c2, d0, d1, d2);
        main_step(k + 1, steady, d0, d1, d2, c0, c1, c2);
    }
    for (; k < kmain; k += 2) {
        main_step(k, general, c0, c1, c2, d0, d1, d2);
        if (k + 1 < kmain) main_step(k + 1, general, d0, d1, d2, c0, c1, c2);
    }
    if (tr) t2 = __builtin_amdgcn_s_memtime();
    // ---- identity residual steps (TR): acc += x, exact fp32 adds from this wave's rows
    if constexpr (TR) {
        for (int k = kmain; k < K; ++k) {
            wait_vm_dyn(k + 1 < K ? NIA : 0);   // A(k) landed (only A(k+1) was issued after it)
            const unsigned char* A = a_slot(k % NSA);
            const int blk = k - kmain;
            const int jb = (32 * blk - n0) / 16;   // first local column block of these channels
            f32x4 xv[FM][2];
#pragma unroll
            for (int i = 0; i < FM; ++i) {
                const int r = wave * RW + i * 16 + (lane & 15);
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    // channels 32 blk + 16h + 4g .. +3 = logical floats [8 g' + 4 h', +4)
                    const int gp = 2 * h + (g >> 1), hp = g & 1;
                    xv[i][h] = *reinterpret_cast<const f32x4*>(A + r * 128 + (((gp + 4 * hp) ^ xa_swz(r)) << 4));
                }
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            if (k + 2 < K) issue_a();   // into the slot just read
#pragma unroll
            for (int j = 0; j < FN; ++j) {
                const int h = j - jb;
#pragma unroll
                for (int i = 0; i < FM; ++i)
                    if (h == 0) acc[i][j] += xv[i][0];
                    else if (h == 1) acc[i][j] += xv[i][1];
            }
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (tr) t3 = __builtin_amdgcn_s_memtime();
    auto trace_out = [&]() __attribute__((always_inline)) {
        if (tr && tid == 0) {
            unsigned long long* o = a.trace + 8 * (size_t)(blockIdx.y * gridDim.x + blockIdx.x);
            o[0] = t1 - t0; o[1] = t2 - t1; o[2] = t3 - t2; o[3] = __builtin_amdgcn_s_memtime() - t3;
            o[4] = t_bar; o[5] = t_vm; o[6] = kmain; o[7] = 1;
        }
    };

    if constexpr (TR) {
        const float slope = a.act == ACT_RELU ? 0.f : (a.act == ACT_LEAKY ? 0.01f : 1.f);
        float* const outp = SK ? a.out + (size_t)blockIdx.z * a.M * a.ldo : a.out;
        if (a.epi_lds) {
            // ---- EPI_BIAS through LDS: each wave stages its own 32 rows (no barrier
            // between its writes and reads) and stores them row-major, so every
            // store instruction writes whole 128-B lines (RPI rows x BN x 4 B)
            // instead of 16 half lines (one 64-B piece per row)
            constexpr int LDC = BN + 4, LPR = BN / 4, RPI = 64 / LPR, NQ = RW / RPI;
            constexpr int NQR = BN == 64 ? NQ : 1;
            float* Cs = reinterpret_cast<float*>(smem);
            const int cl = 4 * (lane % LPR), col = n0 + cl, rsub = lane / LPR;
            const bool cok = col + 3 < a.Nc;
            // global operands before the first store (vmcnt counts loads and stores in order)
            const f32x4 bv = a.bias && cok ? *reinterpret_cast<const f32x4*>(a.bias + col) : f32x4{0.f, 0.f, 0.f, 0.f};
            float rw[4][4];
            f32x4 xr[NQR];
#pragma unroll
            for (int e = 0; e < 4; ++e)
#pragma unroll
                for (int c = 0; c < 4; ++c) rw[e][c] = BN == 64 && a.rx && c < a.rxc && col + e < a.Nc ? a.rw[(col + e) * a.rxc + c] : 0.f;
#pragma unroll
            for (int q = 0; q < NQR; ++q) {
                const int lr = wave * RW + q * RPI + rsub;
                xr[q] = BN == 64 && a.rx && lr < RT && r0 + lr < a.M ? *reinterpret_cast<const f32x4*>(a.rx + (size_t)(r0 + lr) * 4)
                                                                      : f32x4{0.f, 0.f, 0.f, 0.f};
            }
            constexpr int NQI = TR ? NQ : 1;
            f32x4 xi[NQI];
            if (idn_epi) {   // the identity residual rows (block input = output row, same channels)
#pragma unroll
                for (int q = 0; q < NQI; ++q) {
                    const int lr = wave * RW + q * RPI + rsub;
                    xi[q] = cok && lr < RT && r0 + lr < a.M
                                ? __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(a.idn.src + (size_t)(r0 + lr) * a.idn.ld + col))
                                : f32x4{0.f, 0.f, 0.f, 0.f};
                }
            }
            __syncthreads();   // every wave done reading the ring (the B slots are shared)
#pragma unroll
            for (int i = 0; i < FM; ++i)
#pragma unroll
                for (int j = 0; j < FN; ++j)
                    *reinterpret_cast<f32x4*>(Cs + (wave * RW + 16 * i + (lane & 15)) * LDC + 16 * j + 4 * g) = acc[i][j];
#pragma unroll
            for (int q = 0; q < NQ; ++q) {
                const int lr = wave * RW + q * RPI + rsub;
                f32x4 v = *reinterpret_cast<const f32x4*>(Cs + lr * LDC + cl);
                if (idn_epi) v += xi[q % NQI];   // same order as the K-step adds: (acc + x) + bias
                v += bv;
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    if (BN == 64 && a.rx) v[e] += xr[q % NQR][0] * rw[e][0] + xr[q % NQR][1] * rw[e][1] + xr[q % NQR][2] * rw[e][2] + xr[q % NQR][3] * rw[e][3];
                    v[e] = v[e] > 0.f ? v[e] : slope * v[e];
                }
                if (lr < RT && r0 + lr < a.M) {
                    if (cok) {
                        xst4(outp + (size_t)(r0 + lr) * a.ldo + col, v, a.nts);
                    } else {
                        for (int e = 0; e < 4 && col + e < a.Nc; ++e) {
                            float t = *(Cs + lr * LDC + cl + e) + (a.bias ? a.bias[col + e] : 0.f);
                            if (a.rx)
                                for (int c = 0; c < a.rxc; ++c) t = fmaf(xr[q % NQR][c], a.rw[(col + e) * a.rxc + c], t);
                            outp[(size_t)(r0 + lr) * a.ldo + col + e] = t > 0.f ? t : slope * t;
                        }
                    }
                }
            }
            trace_out();
            return;
        }
        // ---- EPI_BIAS from registers: acc[i][j] lane l = row wave*32 + 16i + (l & 15),
        // channels n0 + 16j + 4(l >> 4) .. +3: float4 operands and stores, no LDS
        int rows[FM];
        bool rok[FM];
#pragma unroll
        for (int i = 0; i < FM; ++i) {
            const int lr = wave * RW + i * 16 + (lane & 15);
            rok[i] = lr < RT && r0 + lr < a.M;
            rows[i] = rok[i] ? r0 + lr : 0;
        }
        f32x4 xr[FM];
#pragma unroll
        for (int i = 0; i < FM; ++i) {
            xr[i] = f32x4{0.f, 0.f, 0.f, 0.f};
            if (a.rx) xr[i] = *reinterpret_cast<const f32x4*>(a.rx + (size_t)rows[i] * 4);
        }
        // every global operand is loaded before the first store: a load issued
        // after a store waits for that store too (vmcnt counts both, in order)
        f32x4 bvs[FN];
#pragma unroll
        for (int j = 0; j < FN; ++j) {
            const int col = n0 + 16 * j + 4 * g;
            bvs[j] = a.bias && col + 3 < a.Nc ? *reinterpret_cast<const f32x4*>(a.bias + col) : f32x4{0.f, 0.f, 0.f, 0.f};
        }
        // layer 0's residual conv weights (BN 64 tiles only, launch_xgemm checks)
        constexpr int FNR = BN == 64 ? FN : 1;
        float rws[FNR][4][4];
#pragma unroll
        for (int j = 0; j < FNR; ++j)
#pragma unroll
            for (int e = 0; e < 4; ++e)
#pragma unroll
                for (int c = 0; c < 4; ++c) {
                    const int col = n0 + 16 * j + 4 * g + e;
                    rws[j][e][c] = BN == 64 && a.rx && c < a.rxc && col < a.Nc ? a.rw[col * a.rxc + c] : 0.f;
                }
#pragma unroll
        for (int j = 0; j < FN; ++j) {
            const int col = n0 + 16 * j + 4 * g;
            if (col >= a.Nc) continue;
            if (col + 3 < a.Nc) {
                const f32x4 bv = bvs[j];
                float rw[4][4];
#pragma unroll
                for (int e = 0; e < 4; ++e)
#pragma unroll
                    for (int c = 0; c < 4; ++c) rw[e][c] = rws[j % FNR][e][c];
#pragma unroll
                for (int i = 0; i < FM; ++i) {
                    f32x4 v = acc[i][j] + bv;
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        v[e] += xr[i][0] * rw[e][0] + xr[i][1] * rw[e][1] + xr[i][2] * rw[e][2] + xr[i][3] * rw[e][3];
                        v[e] = v[e] > 0.f ? v[e] : slope * v[e];
                    }
                    if (rok[i]) xst4(outp + (size_t)rows[i] * a.ldo + col, v, a.nts);
                }
            } else {
#pragma unroll
                for (int i = 0; i < FM; ++i) {
                    if (!rok[i]) continue;
                    for (int e = 0; e < 4 && col + e < a.Nc; ++e) {
                        float t = acc[i][j][e] + (a.bias ? a.bias[col + e] : 0.f);
                        if (a.rx)
                            for (int c = 0; c < a.rxc; ++c) t = fmaf(xr[i][c], a.rw[(col + e) * a.rxc + c], t);
                        t = t > 0.f ? t : slope * t;
                        outp[(size_t)rows[i] * a.ldo + col + e] = t;
                    }
                }
            }
        }
    } else if constexpr (EPI == EPI_SKIN) {
        // ---- SMPL-X skinning (lbs): rows = body * 16 + transform entry e of
        // T_v(b) = sum_j W[v][j] A_j(b); a 16-row fragment is one body and lane
        // group g holds entries 4g..4g+3 = transform row g of vertex n0 + 16j +
        // (lane & 15). verts[b][3v + g] = T[g][:3] . v_posed[b][3v..] + T[g][3]
        // (+ transl[b][g]), the fma chain of cgemm.hip's EPI_SKIN.
        // Every global operand is loaded before the first store.
        const int vl = lane & 15;
        float vpr[FM][FN][3], tb[FM];
        int bdy[FM];
#pragma unroll
        for (int i = 0; i < FM; ++i) {
            bdy[i] = (r0 + wave * RW + 16 * i) >> 4;
            const bool bok = g < 3 && bdy[i] * 16 < a.M;
            tb[i] = bok && a.bias ? a.bias[bdy[i] * 3 + g] : 0.f;
#pragma unroll
            for (int j = 0; j < FN; ++j) {
                const int v = n0 + 16 * j + vl;
                const float* vp = a.resid + (size_t)bdy[i] * a.ldr + 3 * v;
#pragma unroll
                for (int c = 0; c < 3; ++c) vpr[i][j][c] = bok && v < a.Nc ? vp[c] : 0.f;
            }
        }
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
            for (int j = 0; j < FN; ++j) {
                const int v = n0 + 16 * j + vl;
                if (g < 3 && bdy[i] * 16 < a.M && v < a.Nc) {
                    const f32x4 t = acc[i][j];
                    const float x = fmaf(t[0], vpr[i][j][0], fmaf(t[1], vpr[i][j][1], fmaf(t[2], vpr[i][j][2], t[3])));
                    a.out[(size_t)bdy[i] * a.ldo + 3 * v + g] = x + tb[i];
                }
            }
    } else {
        // ---- EPI_GRAPH: the C tile through LDS, then the graph mix per frame
        float* Cs = reinterpret_cast<float*>(smem);
        const int crow = wave * RW + 4 * g;
        const int ccol = lane & 15;
        __syncthreads();   // every wave done with the K loop's LDS
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
            for (int j = 0; j < FN; ++j)
#pragma unroll
                for (int e = 0; e < 4; ++e) Cs[(crow + i * 16 + e) * C::LDCG + j * 16 + ccol] = acc[i][j][e];
        float* b2s = Cs + BM * C::LDCG;   // bias2[w][n0 .. n0 + BN) (loaded at kernel start)
#pragma unroll
        for (int u = 0; u < NB2; ++u) {
            const int q = tid + u * NT;
            if (q < 17 * BN / 4) *reinterpret_cast<f32x4*>(b2s + 4 * q) = b2r[u];
        }
        // A_eff in 5 VGPRs across the wave, read back with v_readlane (global loads
        // would be re-issued after every store, which may alias them)
        float amv[5];
#pragma unroll
        for (int k = 0; k < 5; ++k) amv[k] = 64 * k + lane < 17 * 17 ? a.amix[64 * k + lane] : 0.f;
        __syncthreads();
        // the first half of the waves produce joints 0-8, the second joints 9-16 (wave-uniform split,
        // so each half's joint loop is compile-time); item = (frame, 4 columns)
        constexpr int C4 = BN / 4;
        const int nframes = a.M / 17, f0 = r0 / 17;
        const bool second = wave >= NW / 2;
#pragma unroll 1
        for (int it = tid & (NT / 2 - 1); it < RT / 17 * C4; it += NT / 2) {
            const int f = it / C4, c4 = it - f * C4;
            const int col = n0 + 4 * c4;
            if (f0 + f >= nframes || col >= a.Nc) continue;
            f32x4 y[17];
#pragma unroll
            for (int v = 0; v < 17; ++v) y[v] = *reinterpret_cast<const f32x4*>(Cs + (f * 17 + v) * C::LDCG + 4 * c4);
            float* o = a.out + (size_t)(f0 + f) * 17 * a.ldo + col;
            if (a.mix_sparse) {
                if (second) xmix_store<9, 17, true, BN>(y, amv, b2s, 4 * c4, o, a.ldo, a.nts);
                else xmix_store<0, 9, true, BN>(y, amv, b2s, 4 * c4, o, a.ldo, a.nts);
            } else {
                if (second) xmix_store<9, 17, false, BN>(y, amv, b2s, 4 * c4, o, a.ldo, a.nts);
                else xmix_store<0, 9, false, BN>(y, amv, b2s, 4 * c4, o, a.ldo, a.nts);
            }
        }
    }
    trace_out();
}

// ---------------------------------------------------------------------------
// Persistent temporal-conv kernel (EPI_BIAS, 4 waves, two workgroups per CU):
// each workgroup walks tiles b, b + G, b + 2G, ... and its DMA pipeline runs
// ACROSS tiles — the next tile's first A and B stages are issued during the
// current tile's last two K steps, and its step-0 A split runs under the
// current tile's last MFMAs — so no tile pays a prologue (the first DMA round
// trip) and the epilogue's stores drain under the next tile's K loop.
// Epilogue (from the registers of the finished tile): global operands first
// (bias, identity-residual rows, layer 0's residual-conv rows), then per
// quarter of its 32 rows each wave stages 8 rows in the free B slot and
// stores them row-major (whole 128-B lines). Rows past M store to a_trash, so
// every wave issues the same count of vector-memory ops per tile and the
// vmcnt waits stay exact. Same arithmetic, in the same order, as
// xgemm_kernel with the LDS epilogue: bit-identical output.
// EPI: EPI_BIAS (temporal convs) or EPI_SKIN (SMPL-X skinning, the epilogue
// of xgemm_kernel's EPI_SKIN from registers, non-transposed MFMA);
// IDN: identity residual (block input rows); RX: layer 0's residual conv rows
template <int BN, int EPI, bool IDN, bool RX>
__global__ __launch_bounds__(256, 2) void xgemm_pt_kernel(XArgs a) {
    constexpr bool SKIN = EPI == EPI_SKIN;
    using C = XCfg<BN, EPI_BIAS, 4>;   // the same ring (EPI_SKIN needs no C tile)
    constexpr int NW = 4, FM = C::FM, FN = C::FN, NIA = C::NIA, NIBW = C::NIBW, RW = C::RW, BM = C::BM;
    static_assert(C::NIB_TOT % NW == 0 && C::LB == 1 && C::NSA == 2 && C::NSB == 2, "pt pipeline");
    constexpr int LDC = BN + 4, LPR = BN / 4, RPI = 64 / LPR, NQ = 8 / RPI;   // staging: 8 rows per quarter
    static_assert(9 * LDC * 4 * NW <= C::BBYTES, "staging (8 rows + a dummy row per wave) fits one B slot");
    __shared__ __attribute__((aligned(16))) unsigned char smem[C::SMEM];

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int g = lane >> 4;
    const int V = a.V;
    const int ntn = (a.Nc + BN - 1) / BN;               // column tiles (EPI_BIAS: Nc % BN == 0)
    const int ntot = ((a.M + BM - 1) / BM) * ntn;       // tiles
    const int G = gridDim.x, b = blockIdx.x;
    const int my = b < ntot ? (ntot - 1 - b) / G + 1 : 0;
    if (my == 0) return;
    const int K = xgemm_kmain(a);                       // K steps per tile (all with weights)
    const int total = my * K;
    // tile i of this workgroup -> (first row, column tile): XCD-aware order over
    // the linear id b + i G (G % 8 == 0: the XCD of the id is the workgroup's)
    auto tile_of = [&](int i, int& r0, int& nt) __attribute__((always_inline)) {
        const int L = b + i * G;
        const int per = ntot >> 3, rem = ntot & 7, x = L & 7, k = L >> 3;
        const int swz = x < rem ? x * (per + 1) + k : rem * (per + 1) + (x - rem) * per + k;
        r0 = (swz / ntn) * BM;
        nt = swz - (swz / ntn) * ntn;
    };

    // ---- A cursor: tile ia, (segment, block, tap) within it, global step ga
    int a_n[NIA], a_t[NIA], a_w[NIA], a_uo[NIA];
    bool a_ok[NIA];
#pragma unroll
    for (int j = 0; j < NIA; ++j) {
        const int rr = (wave * NIA + j) * 8 + (lane >> 3);
        const int pl = (lane & 7) ^ xa_swz(rr);
        a_uo[j] = 32 * (pl & 3) + 16 * (pl >> 2);
    }
    auto set_rows = [&](int r0) __attribute__((always_inline)) {
#pragma unroll
        for (int j = 0; j < NIA; ++j) {
            const int row = r0 + (wave * NIA + j) * 8 + (lane >> 3);
            a_ok[j] = row < a.M;
            const int q = a_ok[j] ? row / V : 0;
            a_w[j] = a_ok[j] ? row - q * V : 0;
            a_n[j] = q / a.tout;
            a_t[j] = q - a_n[j] * a.tout;
        }
    };
    const bool two = a.nseg > 1;
    const unsigned nbk = (unsigned)((a.seg[0].cin >> 5) | (a.seg[0].kt << 8)) |
                         ((unsigned)(two ? (a.seg[1].cin >> 5) | (a.seg[1].kt << 8) : 0) << 16);
    int ia = 0, ca_seg = 0, ca_tap = 0, ca_blk = 0, ga = 0;
    {
        int r0, nt;
        tile_of(0, r0, nt);
        set_rows(r0);
    }
    unsigned a_off[NIA];
    i32x4 rA;
    bool a_stale = true;
    auto prepare = [&]() __attribute__((always_inline)) {
        if (!a_stale) return;
        const XSeg sg = ca_seg == 0 ? a.seg[0] : a.seg[1];
        rA = buf_rsrc(sg.src, (unsigned)(sg.rows_in * sg.ld * 4));
#pragma unroll
        for (int j = 0; j < NIA; ++j) {
            const int t = sg.stride * a_t[j] + ca_tap - sg.pad;
            a_off[j] = (a_ok[j] && t >= 0 && t < sg.tin)
                           ? (unsigned)(((a_n[j] * sg.tin + t) * V + a_w[j]) * sg.ld * 4 + a_uo[j])
                           : DMA_OOB;
        }
        a_stale = false;
    };
    auto a_slot = [&](int s) __attribute__((always_inline)) { return smem + s * C::ABYTES; };
    auto b_slot = [&](int s) __attribute__((always_inline)) { return smem + 2 * C::ABYTES + s * C::BBYTES; };
    auto issue_a = [&]() __attribute__((always_inline)) {
        prepare();
        unsigned char* A = a_slot(ga & 1);
        const int soA = __builtin_amdgcn_readfirstlane(ca_blk * 128);
#pragma unroll
        for (int j = 0; j < NIA; ++j) dma16(rA, A + (wave * NIA + j) * 1024, a_off[j], soA);
        ++ga;
        const unsigned f = nbk >> (16 * ca_seg);
        const int seg = ca_seg, tap = ca_tap;
        if (++ca_tap >= (int)((f >> 8) & 255u)) {
            ca_tap = 0;
            if (++ca_blk >= (int)(f & 255u)) {
                ca_blk = 0;
                if (++ca_seg >= a.nseg) {   // the tile's last K step: on to the next tile
                    ca_seg = 0;
                    if (++ia < my) {
                        int r0, nt;
                        tile_of(ia, r0, nt);
                        set_rows(r0);
                    }
                }
            }
        }
        a_stale = ca_seg != seg || ca_tap != tap || (ca_blk == 0 && ca_tap == 0);
    };
    // ---- B cursor: tile ib (its column tile ntb), K step kbi, global step gb
    int ib = 0, kbi = 0, gb = 0, ntb;
    {
        int r0;
        tile_of(0, r0, ntb);
    }
    const i32x4 rB = buf_rsrc(a.wp, (unsigned)((size_t)ntn * K * C::BBYTES));
    auto issue_b = [&]() __attribute__((always_inline)) {
        unsigned char* Bd = b_slot(gb & 1);
        const int soB = __builtin_amdgcn_readfirstlane((ntb * K + kbi) * C::BBYTES);
#pragma unroll
        for (int q = 0; q < NIBW; ++q)
            dma16(rB, Bd + (wave + q * NW) * 1024, (unsigned)((wave + q * NW) * 1024 + lane * 16), soB);
        ++gb;
        if (++kbi == K) {
            kbi = 0;
            if (++ib < my) {
                int r0;
                tile_of(ib, r0, ntb);
            }
        }
    };

    // ---- epilogue operands that do not change per tile
    const float slope = a.act == ACT_RELU ? 0.f : (a.act == ACT_LEAKY ? 0.01f : 1.f);
    const int cl = 4 * (lane % LPR), rsub = lane / LPR;
    constexpr bool has_i = IDN, has_x = BN == 64 && RX;   // the bias is always there (the launch checks)
    float rw[4][4];   // layer 0's residual conv (one column tile: the launch checks)
#pragma unroll
    for (int e = 0; e < 4; ++e)
#pragma unroll
        for (int c = 0; c < 4; ++c) rw[e][c] = has_x && c < a.rxc ? a.rw[(cl + e) * a.rxc + c] : 0.f;
    // vector-memory ops per wave (all unconditional): the epilogue operand loads,
    // issued at the start of a tile's last K step (before its DMAs), and the
    // epilogue's stores
    // (EPI_SKIN: per lane FM x FN v_posed triples + FM translations; FM x FN scalar stores)
    constexpr int NXL = SKIN ? FM * FN + FM : 1 + 4 * NQ * ((has_i ? 1 : 0) + (has_x ? 1 : 0));
    constexpr int NST = SKIN ? FM * FN : 4 * NQ;
    // early (during the last K step): 64 more live VGPRs there; the 128-column
    // identity variant would spill, so it loads at the epilogue start instead
    constexpr bool EARLY = !(BN == 128 && IDN);
    f32x4 bv, xi[4][NQ], xr[4][NQ];
    float vpr[SKIN ? FM : 1][SKIN ? FN : 1][3], tb[SKIN ? FM : 1];
    auto load_epi = [&](int ic) __attribute__((always_inline)) {
        int r0, nt;
        tile_of(ic, r0, nt);
        if constexpr (SKIN) {
            // lane = vertex n0 + 16 j + (lane & 15), rows r0 + 32 wave + 16 i + 4 g .. +3
            // = transform row k of body b (xskin_row; k == 3 and rows / vertices past
            // the end load valid dummies and store to a_trash)
            const int sr = a.skin_rows == 12 ? 12 : 16, nbody = a.M / sr;
#pragma unroll
            for (int i = 0; i < FM; ++i) {
                int b, k;
                xskin_row(r0 + wave * RW + 16 * i + 4 * g, sr, b, k);
                const int bb = b < nbody ? b : 0;
                tb[i] = a.bias[bb * 3 + (k < 3 ? k : 0)];
#pragma unroll
                for (int j = 0; j < FN; ++j) {
                    const int v = nt * BN + 16 * j + (lane & 15);
                    const float* vp = a.resid + (size_t)bb * a.ldr + 3 * (v < a.Nc ? v : 0);
                    __builtin_memcpy(&vpr[i][j][0], vp, 12);   // one 12-B load
                }
            }
            return;
        }
        const int col = nt * BN + cl;
        bv = *reinterpret_cast<const f32x4*>(a.bias + col);
#pragma unroll
        for (int q = 0; q < 4; ++q)
#pragma unroll
            for (int rr = 0; rr < NQ; ++rr) {
                const int row = r0 + wave * RW + 16 * (q >> 1) + 8 * (q & 1) + rr * RPI + rsub;
                const int rc = row < a.M ? row : 0;   // rows past M read row 0 (discarded)
                if constexpr (has_i) xi[q][rr] = *reinterpret_cast<const f32x4*>(a.idn.src + (size_t)rc * a.idn.ld + col);
                if constexpr (has_x) xr[q][rr] = *reinterpret_cast<const f32x4*>(a.rx + (size_t)rc * 4);
            }
    };

    f32x4 acc[FM][FN];
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int bsw = (-((lane & 15) >> 2)) & 3;
    const int boff = (lane & 15) * 64 + ((g ^ bsw) << 4);
    auto mma = [&](const xbf16x8& x, const xbf16x8& w, f32x4& c) __attribute__((always_inline)) {
        // EPI_BIAS transposed (lane = row (l & 15), 4 channels); EPI_SKIN not (lane = vertex, 4 entries)
        c = SKIN ? __builtin_amdgcn_mfma_f32_16x16x32_bf16(x, w, c, 0, 0, 0)
                 : __builtin_amdgcn_mfma_f32_16x16x32_bf16(w, x, c, 0, 0, 0);
    };
    auto read_a = [&](int s, f32x4 (&lo)[FM], f32x4 (&hi)[FM]) __attribute__((always_inline)) {
        const unsigned char* A = a_slot(s & 1);
#pragma unroll
        for (int i = 0; i < FM; ++i) {
            const int r = wave * RW + i * 16 + (lane & 15);
            lo[i] = *reinterpret_cast<const f32x4*>(A + r * 128 + ((g ^ xa_swz(r)) << 4));
            hi[i] = *reinterpret_cast<const f32x4*>(A + r * 128 + (((g + 4) ^ xa_swz(r)) << 4));
        }
    };

    // epilogue of the finished tile ic (its last K step used B slot `slot`)
    auto epilogue = [&](int ic, int slot) __attribute__((always_inline)) {
        int r0, nt;
        tile_of(ic, r0, nt);
        if constexpr (SKIN) {
            const int sr = a.skin_rows == 12 ? 12 : 16, nbody = a.M / sr;
#pragma unroll
            for (int i = 0; i < FM; ++i) {
                int b, k;
                xskin_row(r0 + wave * RW + 16 * i + 4 * g, sr, b, k);
#pragma unroll
                for (int j = 0; j < FN; ++j) {
                    const int v = nt * BN + 16 * j + (lane & 15);
                    const f32x4 t = acc[i][j];
                    const float x = fmaf(t[0], vpr[i][j][0], fmaf(t[1], vpr[i][j][1], fmaf(t[2], vpr[i][j][2], t[3])));
                    float* dst = k < 3 && b < nbody && v < a.Nc ? a.out + (size_t)b * a.ldo + 3 * v + k : a.trash + lane;
                    *dst = x + tb[i];
                    acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
                }
            }
            return;
        }
        const int col = nt * BN + cl;
        // bv, xi, xr: loaded by load_epi at the start of the tile's last K step (EARLY) or now
        if constexpr (!EARLY) load_epi(ic);
        float* st = reinterpret_cast<float*>(b_slot(slot)) + wave * 9 * LDC;
        // every wave done reading B slot `slot` (the last K step's weights); no
        // __syncthreads: its release fence would wait for every DMA in flight
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int i = q >> 1, h = q & 1;
            // every lane writes (the other half's lanes to a dummy 9th row): with a
            // divergent `if` here hipcc sank the following read into the masked block
            const int wr = ((lane & 15) >> 3) == h ? (lane & 7) : 8;
#pragma unroll
            for (int j = 0; j < FN; ++j) *reinterpret_cast<f32x4*>(st + wr * LDC + 16 * j + 4 * g) = acc[i][j];
#pragma unroll
            for (int rr = 0; rr < NQ; ++rr) {
                const int lr = rr * RPI + rsub;
                const int row = r0 + wave * RW + 16 * i + 8 * h + lr;
                f32x4 v = *reinterpret_cast<const f32x4*>(st + lr * LDC + cl);
                if constexpr (has_i) v += xi[q][rr];   // (acc + x) + bias, as xgemm_kernel
                v += bv;
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    if constexpr (has_x) v[e] += xr[q][rr][0] * rw[e][0] + xr[q][rr][1] * rw[e][1] + xr[q][rr][2] * rw[e][2] + xr[q][rr][3] * rw[e][3];
                    v[e] = v[e] > 0.f ? v[e] : slope * v[e];
                }
                float* dst = row < a.M ? a.out + (size_t)row * a.ldo + col : a.trash + cl;
                xst4(dst, v, a.nts);
            }
        }
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
            for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    };

    xbf16x8 c0[FM], c1[FM], c2[FM], d0[FM], d1[FM], d2[FM];
    f32x4 alo[FM], ahi[FM];
    // prologue (the first tile only): B(0) A(0) A(1)
    issue_b();
    issue_a();
    if (total > 1) issue_a();
    if (total > 1) wait_vm<NIA>();
    else wait_vm<0>();
    read_a(0, alo, ahi);
#pragma unroll
    for (int i = 0; i < FM; ++i) xsplit8(alo[i], ahi[i], c0[i], c1[i], c2[i]);

    int k = 0, ic = 0;   // the computing tile and its K step
    // global step s: MFMAs of (tile ic, step k) on the split in u, with step
    // s+1's A read and split into v (which may be the next tile's step 0)
    auto step = [&](int s, auto steady, xbf16x8 (&u0)[FM], xbf16x8 (&u1)[FM], xbf16x8 (&u2)[FM], xbf16x8 (&v0)[FM],
                    xbf16x8 (&v1)[FM], xbf16x8 (&v2)[FM]) __attribute__((always_inline)) {
        constexpr bool ST = decltype(steady)::value;   // s + 2 < total: B(s+1) and A(s+2) exist
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();   // every wave's B(s) landed; every wave done with B(s-1) / the staging
        const bool last = k == K - 1;
        if (EARLY && last) load_epi(ic);   // the epilogue's global operands, a whole K step ahead
        if (ST || s + 1 < total) issue_b();
        if (ST || s + 2 < total) issue_a();
        // A(s+1) landed: younger are B(s+1), A(s+2), plus the epilogue loads just
        // issued (a tile's last step) or the stores of the epilogue that ended the
        // previous tile (its first step)
        if (ST) {
            if (EARLY && last) wait_vm<NIA + NIBW + NXL>();
            else if (k == 0 && s > 0) wait_vm<NIA + NIBW + NST + (EARLY ? 0 : NXL)>();
            else wait_vm<NIA + NIBW>();
        } else {
            wait_vm<0>();
        }
        const unsigned char* Bp = b_slot(s & 1) + boff;
        xbf16x8 bb[2][3];
        __builtin_amdgcn_sched_barrier(0);
        read_a(s + 1, alo, ahi);
#pragma unroll
        for (int p = 0; p < 3; ++p) bb[0][p] = *reinterpret_cast<const xbf16x8*>(Bp + p * C::PLANE);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int j = 0; j < FN; ++j) {
            if (j + 1 < FN)
#pragma unroll
                for (int p = 0; p < 3; ++p)
                    bb[(j + 1) & 1][p] = *reinterpret_cast<const xbf16x8*>(Bp + p * C::PLANE + (j + 1) * 16 * 64);
            const xbf16x8(&bq)[3] = bb[j & 1];
#pragma unroll
            for (int i = 0; i < FM; ++i) {
                mma(u2[i], bq[0], acc[i][j]);
                mma(u1[i], bq[1], acc[i][j]);
                mma(u0[i], bq[2], acc[i][j]);
                mma(u1[i], bq[0], acc[i][j]);
                mma(u0[i], bq[1], acc[i][j]);
                mma(u0[i], bq[0], acc[i][j]);
            }
            if (j < FM) xsplit8(alo[j], ahi[j], v0[j], v1[j], v2[j]);
            if (j == FN - 1)
#pragma unroll
                for (int i = FN; i < FM; ++i) xsplit8(alo[i], ahi[i], v0[i], v1[i], v2[i]);
            if (j + 1 < FN) __builtin_amdgcn_sched_group_barrier(0x100, 3, 0);
#pragma unroll
            for (int q = 0; q < 6 * FM; ++q) {
                __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                __builtin_amdgcn_sched_group_barrier(0x002, 2, 0);
            }
            __builtin_amdgcn_sched_barrier(0);
        }
        // B(s+1) landed before the next barrier (only A(s+2) younger)
        if (ST) wait_vm<NIA>();
        else wait_vm<0>();
        if (++k == K) {
            epilogue(ic, s & 1);
            k = 0;
            ++ic;
        }
    };
    const std::true_type steady{};
    const std::false_type general{};
    int s = 0;
    for (; s + 3 < total; s += 2) {
        step(s, steady, c0, c1, c2, d0, d1, d2);
        step(s + 1, steady, d0, d1, d2, c0, c1, c2);
    }
    for (; s < total; s += 2) {
        step(s, general, c0, c1, c2, d0, d1, d2);
        if (s + 1 < total) step(s + 1, general, d0, d1, d2, c0, c1, c2);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

hipError_t launch_xgemm_pt(const XArgs& a, int bn, int ncu, hipStream_t st, int epi) {
    if (a.M <= 0 || a.Nc <= 0) return hipSuccess;
    const int kall = xgemm_kmain(a);
    const bool skin = epi == EPI_SKIN;
    if (epi != EPI_BIAS && !skin) return hipErrorInvalidValue;
    if (skin && (a.skin_rows != 0 && a.skin_rows != 12 && a.skin_rows != 16)) return hipErrorInvalidValue;
    const int srows = skin && a.skin_rows == 12 ? 12 : 16;
    if (skin && (bn != 128 || a.M % srows || !a.resid || a.ldr < 3 * a.Nc || a.ldo < 3 * a.Nc || a.idn.src || a.rx))
        return hipErrorInvalidValue;
    if ((bn != 64 && bn != 128) || !a.wp || !a.out || !a.trash || !a.bias || (!skin && (a.ldo % 4 || a.Nc % bn)) || a.nseg < 1 || a.nseg > 2 ||
        kall < 2 || a.ksplit > 1 || (a.nw != 0 && a.nw != 4))
        return hipErrorInvalidValue;
    for (int s = 0; s <= a.nseg; ++s) {
        const XSeg& g = s < a.nseg ? a.seg[s] : a.idn;
        if (s == a.nseg && !g.src) break;
        // the K cursors pack cin/32 and kt into 8 bits each
        if (!g.src || g.cin % 32 || g.cin / 32 > 255 || g.kt < 1 || g.kt > 255 || g.ld % 4 || g.ld < g.cin ||
            g.rows_in * g.ld * 4 >= (1LL << 31))
            return hipErrorInvalidValue;
    }
    if (a.idn.src && (a.idn.kt != 1 || a.idn.stride != 1 || a.idn.pad != 0 || a.idn.tin != a.tout || a.idn.cin != a.Nc))
        return hipErrorInvalidValue;
    if (a.rx && (bn != 64 || a.Nc != bn || a.rxc < 0 || a.rxc > 4 || !a.rw || a.idn.src)) return hipErrorInvalidValue;
    if ((long long)(skin ? a.M / srows : a.M) * a.ldo >= (1LL << 31) * 1LL * 4) return hipErrorInvalidValue;
    const long long ntot = (long long)((a.M + 127) / 128) * ((a.Nc + bn - 1) / bn);
    long long G = std::min<long long>(ntot, 2LL * ncu);
    if (G > 8) G &= ~7LL;   // a multiple of 8: tile id b + i G stays on the workgroup's XCD
    (void)hipGetLastError();
    const dim3 grid((unsigned)G), blk(256);
    if (skin) {
        hipLaunchKernelGGL((xgemm_pt_kernel<128, EPI_SKIN, false, false>), grid, blk, 0, st, a);
    } else if (bn == 128) {
        if (a.idn.src) hipLaunchKernelGGL((xgemm_pt_kernel<128, EPI_BIAS, true, false>), grid, blk, 0, st, a);
        else hipLaunchKernelGGL((xgemm_pt_kernel<128, EPI_BIAS, false, false>), grid, blk, 0, st, a);
    } else {
        if (a.rx) hipLaunchKernelGGL((xgemm_pt_kernel<64, EPI_BIAS, false, true>), grid, blk, 0, st, a);
        else if (a.idn.src) hipLaunchKernelGGL((xgemm_pt_kernel<64, EPI_BIAS, true, false>), grid, blk, 0, st, a);
        else hipLaunchKernelGGL((xgemm_pt_kernel<64, EPI_BIAS, false, false>), grid, blk, 0, st, a);
    }
    return hipGetLastError();
}

int xgemm_tile_rows(int epi, int nw) {
    const int bm = 32 * (nw == 8 ? 8 : 4);
    return epi == EPI_GRAPH ? bm / 17 * 17 : bm;
}

hipError_t launch_xgemm(const XArgs& a, int bn, int epi, hipStream_t st) {
    if (a.M <= 0 || a.Nc <= 0) return hipSuccess;
    if ((bn != 64 && bn != 128) || (epi != EPI_BIAS && epi != EPI_GRAPH && epi != EPI_SKIN) || !a.wp || !a.out ||
        (epi != EPI_SKIN && a.ldo % 4) ||
        a.nseg < 1 || a.nseg > 2 || a.ksteps != xgemm_ksteps(a) || xgemm_kmain(a) <= 0)
        return hipErrorInvalidValue;
    for (int s = 0; s <= a.nseg; ++s) {
        const XSeg& g = s < a.nseg ? a.seg[s] : a.idn;
        if (s == a.nseg && !g.src) break;
        // the K cursors pack cin/32 and kt into 8 bits each
        if (!g.src || g.cin % 32 || g.cin / 32 > 255 || g.kt < 1 || g.kt > 255 || g.ld % 4 || g.ld < g.cin ||
            g.rows_in * g.ld * 4 >= (1LL << 31))
            return hipErrorInvalidValue;
    }
    if (epi == EPI_GRAPH && (a.V != 17 || a.M % 17 || !a.amix || !a.bias || a.idn.src)) return hipErrorInvalidValue;
    if (a.rx && (bn != 64 || epi != EPI_BIAS || a.rxc < 0 || a.rxc > 4)) return hipErrorInvalidValue;
    if (a.idn.src && (a.idn.kt != 1 || a.idn.stride != 1 || a.idn.pad != 0 || a.idn.tin != a.tout || a.idn.cin != a.Nc))
        return hipErrorInvalidValue;
    if (epi == EPI_SKIN && (a.M % 16 || (a.skin_rows && a.skin_rows != 16) || !a.resid || a.ldr < 3 * a.Nc || a.ldo < 3 * a.Nc || a.idn.src || a.rx))
        return hipErrorInvalidValue;
    if ((long long)(epi == EPI_SKIN ? a.M / 16 : a.M) * a.ldo >= (1LL << 31) * 1LL * 4) return hipErrorInvalidValue;
    const int nw = 4, rt = xgemm_tile_rows(epi, nw);
    if (a.nw != 0 && a.nw != 4) return hipErrorInvalidValue;
    const int ks = a.ksplit > 1 ? a.ksplit : 1;
    if (ks > 1) {   // one kt-1 segment, raw partials, every slice non-empty
        const int kall = xgemm_kmain(a), kper = (kall + ks - 1) / ks;
        if (epi != EPI_BIAS || a.nseg != 1 || a.seg[0].kt != 1 || a.idn.src || a.rx || a.bias || a.act != ACT_NONE ||
            (ks - 1) * kper >= kall || a.trace)
            return hipErrorInvalidValue;
    }
    const dim3 grid((a.M + rt - 1) / rt, (a.Nc + bn - 1) / bn, ks), blk(64 * nw);
    (void)hipGetLastError();
#define XL(BN_, EPI_, NW__) hipLaunchKernelGGL((xgemm_kernel<BN_, EPI_, NW__, false>), grid, blk, 0, st, a)
    if (ks > 1) {
        if (bn == 128) hipLaunchKernelGGL((xgemm_kernel<128, EPI_BIAS, 4, true>), grid, blk, 0, st, a);
        else return hipErrorInvalidValue;
    } else if (epi == EPI_SKIN) {
        if (bn == 128) XL(128, EPI_SKIN, 4);
        else XL(64, EPI_SKIN, 4);
    } else {
        if (bn == 128) { if (epi == EPI_BIAS) XL(128, EPI_BIAS, 4); else XL(128, EPI_GRAPH, 4); }
        else { if (epi == EPI_BIAS) XL(64, EPI_BIAS, 4); else XL(64, EPI_GRAPH, 4); }
    }
#undef XL
    return hipGetLastError();
}

__global__ __launch_bounds__(256) void xgemm_splitk_reduce_kernel(const float* __restrict__ part, int ksplit, int M,
                                                                  int Nc, const float* __restrict__ bias, float slope,
                                                                  float* __restrict__ out, int ldo) {
    const int c4 = Nc / 4;
    const long long n = (long long)M * c4, plane = (long long)M * Nc;
    for (long long i = blockIdx.x * 256LL + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
        const int r = (int)(i / c4), c = 4 * (int)(i - (long long)r * c4);
        const float* p = part + (size_t)r * Nc + c;
        f32x4 v = bias ? *reinterpret_cast<const f32x4*>(bias + c) : f32x4{0.f, 0.f, 0.f, 0.f};
        f32x4 s = *reinterpret_cast<const f32x4*>(p);
        for (int z = 1; z < ksplit; ++z) s += *reinterpret_cast<const f32x4*>(p + z * plane);
        v = s + v;
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = v[e] > 0.f ? v[e] : slope * v[e];
        *reinterpret_cast<f32x4*>(out + (size_t)r * ldo + c) = v;
    }
}

hipError_t launch_xgemm_splitk_reduce(const float* part, int ksplit, int M, int Nc, const float* bias, int act,
                                      float* out, int ldo, hipStream_t st) {
    if (M <= 0) return hipSuccess;
    if (!part || !out || ksplit < 1 || Nc % 4 || ldo % 4) return hipErrorInvalidValue;
    const float slope = act == ACT_RELU ? 0.f : (act == ACT_LEAKY ? 0.01f : 1.f);
    const long long n = (long long)M * (Nc / 4);
    const int grid = (int)std::min<long long>((n + 255) / 256, 4096);
    (void)hipGetLastError();
    hipLaunchKernelGGL(xgemm_splitk_reduce_kernel, dim3(grid), dim3(256), 0, st, part, ksplit, M, Nc, bias, slope, out, ldo);
    return hipGetLastError();
}

std::vector<unsigned short> xgemm_pack(const XPackSeg* segs, int nseg, int Nc, int bn) {
    int ks = 0;
    for (int s = 0; s < nseg; ++s) ks += segs[s].kt * ((segs[s].cin + 31) / 32);
    const int ntiles = (Nc + bn - 1) / bn;
    const size_t tile = (size_t)3 * bn * 32;   // halves per (column tile, K step)
    std::vector<unsigned short> out((size_t)ntiles * ks * tile, 0);
    for (int nt = 0; nt < ntiles; ++nt) {
        int k = 0;
        for (int s = 0; s < nseg; ++s) {
            const XPackSeg& sg = segs[s];
            const int nb = (sg.cin + 31) / 32;
            for (int b = 0; b < nb; ++b)
                for (int tap = 0; tap < sg.kt; ++tap, ++k) {
                    unsigned short* base = out.data() + ((size_t)nt * ks + k) * tile;
                    for (int n = 0; n < bn; ++n) {
                        const int col = nt * bn + n;
                        if (col >= Nc) continue;
                        for (int kk = 0; kk < 32; ++kk) {
                            const int c = b * 32 + kk;
                            if (c >= sg.cin) continue;
                            const float w = sg.w[(size_t)col * sg.ldw + (size_t)tap * sg.cin + c];
                            unsigned short p[3];
                            tik_host::split_bf16x3(w, p[0], p[1], p[2]);
                            const int gg = kk >> 3, sw = (-(n >> 2)) & 3;
                            const size_t off = (size_t)n * 32 + (size_t)((gg ^ sw) * 8) + (kk & 7);
                            for (int pl = 0; pl < 3; ++pl) base[(size_t)pl * bn * 32 + off] = p[pl];
                        }
                    }
                }
        }
    }
    return out;
}

}  // namespace tik
