// tgemm.hip — the bias-epilogue f16x3 implicit GEMM (temporal conv +
// residual, head Linear) with SPLIT DMA rings: the activation operand A
// (first-touch rows, HBM/MALL latency) is fetched NSA-1 K steps ahead, the
// weight operand B (L2-resident, short latency) one step ahead.
//
// cgemm3.hip keeps one stage (A and B together) in flight per workgroup;
// its K loop was measured to be bound by that single ~2 µs DMA round trip
// (DMA-only runs took 87 % of the full kernel time). With a 3-deep A ring and
// a 2-deep B ring, 48 KB per workgroup (96 KB per CU) stay in flight and the
// critical A rows get two K steps of lead, in the same 80 KB of LDS that lets
// two workgroups share a CU.
//
// Issue order per K step is B(ch+1) then A(ch+2), so the counted wait at step
// ch — vmcnt(NIA_w) — retires A(ch) and B(ch) and leaves only A(ch+1) in
// flight (vmcnt retires in issue order).
//
// FG > 0 (TG_128x128_G7): tiles of FG whole output frames (17 FG of the 128
// MFMA rows) with all 128 output channels, and the NEXT ST-GCN block's
// spatial half fused into the epilogue: the output tile is split once more
// into an LDS image that is the A operand of the next gcn 1x1 conv (its K =
// this tile's 128 channels), followed by the 17x17 graph mix, so the next
// block's z is written here and its separate G launch (a full re-read of
// this output from HBM) disappears. Everything stays inside the 80 KB of
// LDS that keeps two workgroups per CU.
#include <type_traits>

#include "cgemm3_dev.h"

namespace tik {

template <int BM, int BN, int WM, int WN, int NSA, int FG = 0>
__global__ __launch_bounds__(64 * WM * WN, WM * WN / 2) void tgemm_kernel(Cgemm3Args a) {
    constexpr int FM = BM / WM / 16, FN = BN / WN / 16;
    constexpr int NW = WM * WN, NT = 64 * NW;
    static_assert(FM * WM * 16 == BM && FN * WN * 16 == BN, "tile");
    constexpr int NIA = BM / 8 / NW, NIB = BN / 8 / NW;   // DMA instructions per wave per stage
    static_assert(NIA * 8 * NW == BM && NIB * 8 * NW == BN, "DMA split");
    constexpr int NSB = 2;
    constexpr int ASLOT = BM * 128, BSLOT = BN * 128;
    constexpr int RING = NSA * ASLOT + NSB * BSLOT;
    constexpr int LDC = BN + 4;
    constexpr int CTILE = BM * LDC * 4;
    constexpr int SMEM = RING > CTILE ? RING : CTILE;
    __shared__ __attribute__((aligned(16))) unsigned char smem[SMEM];   // the only LDS object

    const int tid = threadIdx.x, lane = tid & 63;
    TIK_FENCE_BEGIN();
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave / WN, wn = wave % WN;
    int r0, n0;
    {   // XCD-aware tile order (cgemm3.hip)
        const int nwg = gridDim.x * gridDim.y, bid = blockIdx.y * gridDim.x + blockIdx.x;
        const int per = nwg >> 3, rem = nwg & 7, x = bid & 7, k = bid >> 3;
        const int swz = (a.tune & 1) ? bid : x < rem ? x * (per + 1) + k : rem * (per + 1) + (x - rem) * per + k;
        r0 = (swz / gridDim.y) * (FG > 0 ? FG * 17 : BM);
        n0 = (swz % gridDim.y) * BN;
    }
    const int V = a.V;
    const unsigned long long ts0 = a.trace ? __builtin_amdgcn_s_memrealtime() : 0;

    // ---- DMA roles. A instruction j of this wave: A image rows (wave*NIA+j)*8 ..+7;
    // B instruction j: B image rows (wave*NIB+j)*8 ..+7; lane l writes unit l&7 of row l>>3.
    int a_n[NIA], a_t[NIA], a_w[NIA], a_ck[NIA];
    bool a_ok[NIA];
#pragma unroll
    for (int j = 0; j < NIA; ++j) {
        const int rr = (wave * NIA + j) * 8 + (lane >> 3);
        const int row = r0 + rr;
        a_ck[j] = (lane & 7) ^ sbf(rr);
        a_ok[j] = (FG == 0 || rr < FG * 17) && row < a.M;   // rows past the frames: zero DMA
        const int q = a_ok[j] ? row / V : 0;
        a_w[j] = a_ok[j] ? row - q * V : 0;
        a_n[j] = q / a.tout;
        a_t[j] = q - a_n[j] * a.tout;
    }
    int b_col[NIB], b_ck[NIB];
#pragma unroll
    for (int j = 0; j < NIB; ++j) {
        const int rr = (wave * NIB + j) * 8 + (lane >> 3);
        b_ck[j] = (lane & 7) ^ sbf(rr);
        b_col[j] = n0 + rr < a.Nc ? n0 + rr : -1;
    }
    f32x4 bv = {0.f, 0.f, 0.f, 0.f};
    {
        const int col = n0 + 4 * (tid % (BN / 4));
#pragma unroll
        for (int e = 0; e < 4; ++e)
            if (a.bias && col + e < a.Nc) bv[e] = a.bias[col + e];
    }

    const int ktotal = a.seg[0].kt * a.seg[0].nblk + (a.nseg > 1 ? a.seg[1].kt * a.seg[1].nblk : 0);
    const int nwin = a.M / (V * a.tout);

    // Two independent K cursors (A runs one step ahead of B). Each keeps its
    // own (segment, tap, block) and its own per-lane offsets.
    struct Cur { int seg, tap, blk; };
    auto step = [&](Cur& c) {
        const int nb = c.seg == 0 ? a.seg[0].nblk : a.seg[1].nblk;
        const int kt = c.seg == 0 ? a.seg[0].kt : a.seg[1].kt;
        if (++c.blk >= nb) { c.blk = 0; if (++c.tap >= kt) { c.tap = 0; ++c.seg; } }
    };
    Cur ca{0, 0, 0}, cb{0, 0, 0};
    unsigned a_off[NIA], b_off[NIB];
    i32x4 rA = buf_rsrc(a.seg[0].src, (unsigned)(nwin * a.seg[0].tin * V * a.seg[0].ld * 2));
    i32x4 rB = buf_rsrc(a.seg[0].w, (unsigned)(a.Nc * a.seg[0].ldw * 2));
    int a_seg_cached = -1, a_tap_cached = -1, b_seg_cached = -1;
    auto a_prepare = [&]() {   // per-lane A offsets for cursor ca's (segment, tap)
        if (ca.seg == a_seg_cached && ca.tap == a_tap_cached) return;
        const Seg3 sg = ca.seg == 0 ? a.seg[0] : a.seg[1];
        if (ca.seg != a_seg_cached) rA = buf_rsrc(sg.src, (unsigned)(nwin * sg.tin * V * sg.ld * 2));
#pragma unroll
        for (int j = 0; j < NIA; ++j) {
            const int t = sg.stride * a_t[j] + ca.tap - sg.pad;
            a_off[j] = (a_ok[j] && t >= 0 && t < sg.tin)
                           ? (unsigned)((((a_n[j] * sg.tin + t) * V + a_w[j]) * sg.ld + 8 * a_ck[j]) * 2)
                           : DMA_OOB;
        }
        a_seg_cached = ca.seg; a_tap_cached = ca.tap;
    };
    auto b_prepare = [&]() {
        if (cb.seg == b_seg_cached) return;
        const Seg3 sg = cb.seg == 0 ? a.seg[0] : a.seg[1];
        rB = buf_rsrc(sg.w, (unsigned)(a.Nc * sg.ldw * 2));
#pragma unroll
        for (int j = 0; j < NIB; ++j)
            b_off[j] = b_col[j] >= 0 ? (unsigned)((b_col[j] * sg.ldw + 8 * b_ck[j]) * 2) : DMA_OOB;
        b_seg_cached = cb.seg;
    };
    auto issue_a = [&](int slot) {   // A stage of cursor ca, then advance it
        a_prepare();
        unsigned char* dst = smem + slot * ASLOT + wave * NIA * 1024;
        // soffset through readfirstlane: the cursor is uniform but not provably so,
        // and a VGPR soffset makes hipcc wrap every DMA in a waterfall loop
        const int soA = __builtin_amdgcn_readfirstlane(ca.blk * 128);
#pragma unroll
        for (int j = 0; j < NIA; ++j) dma16(rA, dst + j * 1024, a_off[j], soA);
        step(ca);
    };
    auto issue_b = [&](int slot) {
        b_prepare();
        const int nb = cb.seg == 0 ? a.seg[0].nblk : a.seg[1].nblk;
        unsigned char* dst = smem + NSA * ASLOT + slot * BSLOT + wave * NIB * 1024;
        const int soB = __builtin_amdgcn_readfirstlane((cb.tap * nb + cb.blk) * 128);
#pragma unroll
        for (int j = 0; j < NIB; ++j) dma16(rB, dst + j * 1024, b_off[j], soB);
        step(cb);
    };

    f32x4 acc[FM][FN];
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int arow = wm * FM * 16 + (lane & 15);
    const int brow = wn * FN * 16 + (lane & 15);
    const int g = lane >> 4;
    auto compute = [&](int as, int bs) {
        const unsigned char* A = smem + as * ASLOT;
        const unsigned char* B = smem + NSA * ASLOT + bs * BSLOT;
        f16x8 bh[FN], bl[FN];
#pragma unroll
        for (int j = 0; j < FN; ++j) {
            bh[j] = *reinterpret_cast<const f16x8*>(B + sbo(brow + j * 16, g));
            bl[j] = *reinterpret_cast<const f16x8*>(B + sbo(brow + j * 16, 4 + g));
        }
#pragma unroll
        for (int i = 0; i < FM; ++i) {
            const f16x8 ah = *reinterpret_cast<const f16x8*>(A + sbo(arow + i * 16, g));
            const f16x8 al = *reinterpret_cast<const f16x8*>(A + sbo(arow + i * 16, 4 + g));
#pragma unroll
            for (int j = 0; j < FN; ++j) {
                acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(al, bh[j], acc[i][j], 0, 0, 0);
                acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bl[j], acc[i][j], 0, 0, 0);
                acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bh[j], acc[i][j], 0, 0, 0);
            }
        }
    };

    unsigned long long tw_vm = 0, tw_bar = 0;
    const unsigned long long tl0 = a.trace ? __builtin_amdgcn_s_memtime() : 0;
    if (ktotal > 0) {
        // prologue: B(0); A(0) .. A(NSA-2)
        issue_b(0);
#pragma unroll
        for (int s = 0; s < NSA - 1; ++s)
            if (s < ktotal) issue_a(s);
        for (int ch = 0; ch < ktotal; ++ch) {
            const unsigned long long w0 = a.trace ? __builtin_amdgcn_s_memtime() : 0;
            // in flight (issue order): A(ch) .. | B(ch) | A(ch+1) .. A(ch+NSA-2):
            // retire everything up to B(ch), leave the younger A stages
            const int younger = min(NSA - 2, ktotal - 1 - ch);
            if (NSA >= 3 && younger >= 1 && !(a.tune & 2)) wait_vm<(NSA >= 3 ? NIA : 0)>();
            else wait_vm<0>();
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            const unsigned long long w1 = a.trace ? __builtin_amdgcn_s_memtime() : 0;
            __builtin_amdgcn_s_barrier();
            if (a.trace) {
                const unsigned long long w2 = __builtin_amdgcn_s_memtime();
                tw_vm += w1 - w0; tw_bar += w2 - w1;
            }
            if (ch + 1 < ktotal) issue_b((ch + 1) % NSB);
            if (ch + NSA - 1 < ktotal) issue_a((ch + NSA - 1) % NSA);
            compute(ch % NSA, ch % NSB);
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    const unsigned long long ts1 = a.trace ? __builtin_amdgcn_s_memrealtime() : 0;
    const unsigned long long tl1 = a.trace ? __builtin_amdgcn_s_memtime() : 0;


    unsigned long long tp[6] = {0, 0, 0, 0, 0, 0};   // FG phase stamps (trace only)
    if constexpr (FG == 0) {
        f32x4 res[EpiMap<BM, BN, NT>::KI];
        epi_resid<BM, BN, NT>(a, r0, n0, tid, res);
        const int crow0 = wm * FM * 16 + 4 * (lane >> 4);
        const int ccol0 = wn * FN * 16 + (lane & 15);
        float* Cs = reinterpret_cast<float*>(smem);
    #pragma unroll
        for (int i = 0; i < FM; ++i)
    #pragma unroll
            for (int j = 0; j < FN; ++j)
    #pragma unroll
                for (int e = 0; e < 4; ++e) Cs[(crow0 + i * 16 + e) * LDC + ccol0 + j * 16] = acc[i][j][e];
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        epi_bias<BM, BN, NT, LDC>(a, Cs, bv, r0, n0, tid, res);
    } else {
        // ===== fused epilogue: out = act(C + bias + residual) -> HBM and the LDS
        // split image; z' = ReLU(mix_A(out . Wg'^T) + bias2') -> HBM. The gcn GEMM
        // uses cgemm3's f16x3 products in cgemm3's K order (bit-identical z').
        constexpr int RT = FG * 17;
        constexpr int IMGB = BM * 128;   // one 32-channel split-block image of the tile
        constexpr int NKB = BN / 32;     // K blocks of the next gcn
        constexpr int BOFF = CTILE;      // bias2' [17][BN] fp32 past the C tile
        using E = EpiMap<BM, BN, NT>;
        static_assert(BN == 128 && NT == 512 && RT <= BM && NKB * IMGB <= CTILE && BOFF + 17 * BN * 4 <= SMEM,
                      "fused graph epilogue");
        // constants: A_eff' in registers (v_readlane), bias2' staged into LDS
        constexpr int NAM = (17 * 17 + 63) / 64;
        float amv[NAM];
#pragma unroll
        for (int k = 0; k < NAM; ++k) amv[k] = 64 * k + lane < 17 * 17 ? a.g_amix[64 * k + lane] : 0.f;
        constexpr int NBQ = (17 * BN + NT - 1) / NT;
        float bq[NBQ];
#pragma unroll
        for (int q = 0; q < NBQ; ++q) bq[q] = tid + NT * q < 17 * BN ? a.g_bias2[tid + NT * q] : 0.f;
        f32x4 res[E::KI];
        epi_resid<BM, BN, NT>(a, r0, 0, tid, res);
        const int crow0 = wm * FM * 16 + 4 * (lane >> 4);
        const int ccol0 = wn * FN * 16 + (lane & 15);
        float* Cs = reinterpret_cast<float*>(smem);
        float* b2s = reinterpret_cast<float*>(smem + BOFF);
        // (1) C tile -> LDS
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
            for (int j = 0; j < FN; ++j)
#pragma unroll
                for (int e = 0; e < 4; ++e) Cs[(crow0 + i * 16 + e) * LDC + ccol0 + j * 16] = acc[i][j][e];
#pragma unroll
        for (int q = 0; q < NBQ; ++q)
            if (tid + NT * q < 17 * BN) b2s[tid + NT * q] = bq[q];
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        if (a.trace) tp[0] = __builtin_amdgcn_s_memrealtime();
        // B operand of the next gcn: its SB weights (L2-resident) for this wave's
        // columns, in two halves of K issued ahead of the work that hides them
        // (the first here, over the residual wait; the second over the image store)
        f16x8 gh[NKB][FN], gl[NKB][FN];
        auto load_g = [&](int kb0, int kb1) {
#pragma unroll
            for (int kb = kb0; kb < kb1; ++kb)
#pragma unroll
                for (int j = 0; j < FN; ++j) {
                    const unsigned short* p = a.g_w + (size_t)(brow + j * 16) * a.g_ldw + kb * 64 + 8 * g;
                    gh[kb][j] = *reinterpret_cast<const f16x8*>(p);
                    gl[kb][j] = *reinterpret_cast<const f16x8*>(p + 32);
                }
        };
        load_g(0, NKB / 2);
        __builtin_amdgcn_sched_barrier(0);
        // (2) this thread's output items
        const int c4 = tid % E::C4, lr0 = tid / E::C4, col = 4 * c4;
        const float slope = a.act == ACT_RELU ? 0.f : (a.act == ACT_LEAKY ? 0.01f : 1.f);
        f32x4 vv[E::KI];
#pragma unroll
        for (int k = 0; k < E::KI; ++k) {
            const int lr = lr0 + k * E::RS;
            f32x4 v = *reinterpret_cast<const f32x4*>(Cs + lr * LDC + col) + bv;
            const f16x4 h = __builtin_bit_cast(f16x4, f32x2{res[k][0], res[k][1]});
            const f16x4 l = __builtin_bit_cast(f16x4, f32x2{res[k][2], res[k][3]});
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                v[e] += (float)h[e] + (float)l[e];
                v[e] = v[e] > 0.f ? v[e] : slope * v[e];
            }
            const bool ok = lr < RT && r0 + lr < a.M;
            vv[k] = ok ? v : f32x4{0.f, 0.f, 0.f, 0.f};
        }
        load_g(NKB / 2, NKB);
        __builtin_amdgcn_sched_barrier(0);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();   // every C read done: the image goes over it
        // (3) the split image (zero rows past the tile's frames)
        {
            unsigned char* ib = smem + (col >> 5) * IMGB;
            const int uh = (col & 31) >> 3, sub = (col & 7) * 2;
#pragma unroll
            for (int k = 0; k < E::KI; ++k) {
                const int lr = lr0 + k * E::RS;
                f16x4 h, l;
                split4(vv[k], h, l);
                *reinterpret_cast<f16x4*>(ib + sbo(lr, uh) + sub) = h;
                *reinterpret_cast<f16x4*>(ib + sbo(lr, 4 + uh) + sub) = l;
            }
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        if (a.trace) tp[1] = __builtin_amdgcn_s_memrealtime();
        // (4) the next block's gcn 1x1 conv on the tile
        f32x4 acc2[FM][FN];
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
            for (int j = 0; j < FN; ++j) acc2[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kb = 0; kb < NKB; ++kb) {
            const unsigned char* A = smem + kb * IMGB;
#pragma unroll
            for (int i = 0; i < FM; ++i) {
                const f16x8 ah = *reinterpret_cast<const f16x8*>(A + sbo(arow + i * 16, g));
                const f16x8 al = *reinterpret_cast<const f16x8*>(A + sbo(arow + i * 16, 4 + g));
#pragma unroll
                for (int j = 0; j < FN; ++j) {
                    acc2[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(al, gh[kb][j], acc2[i][j], 0, 0, 0);
                    acc2[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, gl[kb][j], acc2[i][j], 0, 0, 0);
                    acc2[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, gh[kb][j], acc2[i][j], 0, 0, 0);
                }
            }
        }
        if (a.trace) tp[2] = __builtin_amdgcn_s_memrealtime();
        // (5) this block's output to HBM from the image, in whole 128-B lines
        constexpr int NU = NKB * BM * 8 / NT;   // 16-B units per thread
#pragma unroll
        for (int q = 0; q < NU; ++q) {
            const int idx = tid + NT * q;
            const int b = idx / (BM * 8), rem = idx % (BM * 8), r = rem >> 3, u = rem & 7;
            const f32x4 d = *reinterpret_cast<const f32x4*>(smem + b * IMGB + sbo(r, u));
            if (r < RT && r0 + r < a.M) *reinterpret_cast<f32x4*>(a.out_h + (size_t)(r0 + r) * a.ldo + b * 64 + u * 8) = d;
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();   // image reads done
        // (6) gcn output -> LDS
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
            for (int j = 0; j < FN; ++j)
#pragma unroll
                for (int e = 0; e < 4; ++e) Cs[(crow0 + i * 16 + e) * LDC + ccol0 + j * 16] = acc2[i][j][e];
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        if (a.trace) tp[3] = __builtin_amdgcn_s_memrealtime();
        // (7) graph mix + bias2' + ReLU -> z' (frame, 4 channels) per lane; even
        // waves joints 0-8, odd waves 9-16 (wave-uniform joint ranges)
        const int item = (wave >> 1) * 64 + lane, f = item >> 5, cq = item & 31;
        const int frame0 = r0 / 17;
        if (f < FG && frame0 + f < a.M / 17) {
            f32x4 y[17];
#pragma unroll
            for (int v = 0; v < 17; ++v) y[v] = *reinterpret_cast<const f32x4*>(Cs + (f * 17 + v) * LDC + 4 * cq);
            unsigned short* ob = a.g_out + (size_t)(frame0 + f) * 17 * a.g_ldo + sbc(4 * cq);
            auto mixr = [&](auto w0c, auto w1c, auto sp) {
                constexpr int W0 = decltype(w0c)::value, W1 = decltype(w1c)::value;
                constexpr bool SP = decltype(sp)::value;
#pragma unroll
                for (int w = W0; w < W1; ++w) {
                    f32x4 z = *reinterpret_cast<const f32x4*>(b2s + w * BN + 4 * cq);
#pragma unroll
                    for (int v = 0; v < 17; ++v)
                        if (!SP || ((coco_hop2_mask3(w) >> v) & 1u)) {
                            const float av = __builtin_bit_cast(
                                float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, amv[(v * 17 + w) / 64]), (v * 17 + w) % 64));
                            z += av * y[v];
                        }
#pragma unroll
                    for (int e = 0; e < 4; ++e) z[e] = z[e] > 0.f ? z[e] : 0.f;
                    f16x4 h, l;
                    split4(z, h, l);
                    *reinterpret_cast<f16x4*>(ob + (size_t)w * a.g_ldo) = h;
                    *reinterpret_cast<f16x4*>(ob + (size_t)w * a.g_ldo + 32) = l;
                }
            };
            using I0 = std::integral_constant<int, 0>;
            using I9 = std::integral_constant<int, 9>;
            using I17 = std::integral_constant<int, 17>;
            if (wave & 1) {
                if (a.g_mix_sparse) mixr(I9{}, I17{}, std::true_type{});
                else mixr(I9{}, I17{}, std::false_type{});
            } else {
                if (a.g_mix_sparse) mixr(I0{}, I9{}, std::true_type{});
                else mixr(I0{}, I9{}, std::false_type{});
            }
        }
        if (a.trace) tp[4] = __builtin_amdgcn_s_memrealtime();
    }

    if (a.trace) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (tid == 0 && FG > 0) {   // start, loop end, C staged, image ready, gcn done, z' staged, mix done, end
            unsigned long long* t = a.trace + 8 * ((size_t)blockIdx.y * gridDim.x + blockIdx.x);
            t[0] = ts0; t[1] = ts1;
            for (int k = 0; k < 5; ++k) t[2 + k] = tp[k];
            t[7] = __builtin_amdgcn_s_memrealtime();
        } else if (tid == 0) {
            unsigned long long* t = a.trace + 5 * ((size_t)blockIdx.y * gridDim.x + blockIdx.x);
            t[0] = ts0; t[1] = ts1; t[2] = __builtin_amdgcn_s_memrealtime();
            t[3] = tw_vm;
            t[4] = tw_bar | ((unsigned long long)(tl1 - tl0) << 32);
        }
    }
    TIK_FENCE_END();
}

template <int BM, int BN, int WM, int WN, int NSA, int FG = 0>
static hipError_t launch_t(const Cgemm3Args& a, hipStream_t st) {
    constexpr int RT = FG > 0 ? FG * 17 : BM;   // output rows per tile
    const dim3 g((a.M + RT - 1) / RT, (a.Nc + BN - 1) / BN), blk(64 * WM * WN);
    hipLaunchKernelGGL((tgemm_kernel<BM, BN, WM, WN, NSA, FG>), g, blk, 0, st, a);
    return hipGetLastError();
}

hipError_t launch_tgemm(const Cgemm3Args& a, int cfg, hipStream_t st) {
    if (a.M <= 0 || a.Nc <= 0) return hipSuccess;
    for (int s = 0; s < a.nseg; ++s)
        if (a.seg[s].nblk <= 0 || a.seg[s].ld % 8 || a.seg[s].ld < 64 * a.seg[s].nblk || !a.seg[s].w ||
            a.seg[s].ldw < a.seg[s].kt * a.seg[s].nblk * 64)
            return hipErrorInvalidValue;
    if (a.out_h && (a.ldo % 8 || a.ldo < 64 * sb_blocks(a.Nc))) return hipErrorInvalidValue;
    (void)hipGetLastError();
    switch (cfg) {
        case TG_128x128: return launch_t<128, 128, 2, 4, 3>(a, st);
        case TG_128x64: return launch_t<128, 64, 4, 2, 3>(a, st);
        case TG_128x128_A4: return launch_t<128, 128, 2, 4, 4>(a, st);
        case TG_128x64_A4: return launch_t<128, 64, 4, 2, 4>(a, st);
        case TG_64x64: return launch_t<64, 64, 2, 2, 3>(a, st);
        case TG_128x128_G7:
            // whole frames, all 128 channels in one tile, the next gcn 128 -> 128
            if (a.V != 17 || a.Nc != 128 || a.M % 17 || !a.out_h || !a.g_w || !a.g_bias2 || !a.g_amix || !a.g_out ||
                a.g_nc != 128 || a.g_ldw < 64 * 4 || a.g_ldw % 8 || a.g_ldo < 64 * 4 || a.g_ldo % 8 || a.rx)
                return hipErrorInvalidValue;
            return launch_t<128, 128, 2, 4, 3, 7>(a, st);
        default: return hipErrorInvalidValue;
    }
}

}  // namespace tik
