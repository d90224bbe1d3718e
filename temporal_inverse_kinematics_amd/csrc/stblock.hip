// stblock.hip — one whole ST-GCN block per workgroup, for the stride-1
// identity-residual 64-channel blocks (st_gcn_aaai18.py st_gcn.forward:
// gcn -> tcn -> + x -> ReLU; models.py StbBlock): the spatial half's output
// z never leaves the CU.
//
// The layered path runs a block as two kernels, G (x -> z) and T
// (z, x -> out): five activation streams through HBM per block (read x,
// write z, read z, read x, write out). Here one workgroup owns F = 14
// consecutive output frames (all 64 channels) and
//   1. G: streams x for the 16 input frames (one halo frame each side, the
//      temporal taps) and Wg through LDS-DMA. The x image is JOINT-MAJOR
//      (image row 16 v + f = joint v of frame f), and y = x Wg' is computed
//      transposed (MFMA A = Wg rows, B = pixel rows): pixel block j is joint
//      j of the 16 frames, so each lane of waves 0-3 ends holding y for one
//      frame (lane & 15), 4 channels and ALL 17 joints;
//   2. mix in registers: z = ReLU(mix_A(y) + bias2) per lane (17x17, fp32,
//      the COCO 2-hop sparsity unrolled), written once, split, into the
//      frame-major z image (row 17 f + w) — no y pass through LDS;
//   3. T: the 3-tap temporal conv with A read straight from the resident z
//      image (tap k of output row m is z row m + 17 k, or the zero row when
//      the tap leaves the window) and Wt streamed through the ring;
//   4. epilogue: C tile staged over the (dead) z image, + bias + x, ReLU,
//      split-block stores.
// HBM traffic per block: read x (+2 halo frames per 14, L2 hits for the
// neighbour tiles), re-read x for the residual (L2-hot), write out.
#include <cstdlib>
#include <type_traits>

#include "cgemm3_dev.h"

namespace tik {

template <int CIN, int COUT, int FIN>
struct StbGeo {
    static constexpr int V = 17;
    static constexpr int F = FIN - 2;   // output frames per tile
    static constexpr int PX = FIN * V, PXB = V, PXR = PX;   // pixel block j = joint j of the FIN frames
    static constexpr int ZR = PX, ZROWS = PX + 1;          // zero row of each z block image
    static constexpr int TR = F * V, TRB = (TR + 15) / 16;
    static constexpr int NKG = CIN / 32, NKB = COUT / 32, NKT = 3 * NKB;
    static constexpr int ZB = ZROWS * 128, ZBYTES = NKB * ZB;
    static constexpr int XS = PXR * 128, WS = COUT * 128;
    static constexpr int GSLOT = XS + WS, RING = 2 * GSLOT;
    static constexpr int TSLOTS = RING / WS < NKT ? RING / WS : NKT;
    static constexpr int LDC = COUT + 4;
    static constexpr int CT = TRB * 16 * LDC * 4;
    static constexpr int SMEM = ZBYTES + RING;
    static_assert(FIN == 16, "joint-major pixel blocks: 16 frames per block");
    static_assert(COUT == 64, "G: one 16-channel block per wave for waves 0-3");
    static_assert(CT <= ZBYTES, "C tile must fit over the z image");
    static_assert(SMEM <= 163840, "LDS");
    static_assert(TSLOTS == NKT, "T: the whole Wt resident in the ring (no per-chunk waits)");
};

// RAW: the first block straight from the raw keypoints (layer0.hip's gcn0
// math in VALU writes the z image; data_bn'd keypoints of the tile's 16
// frames stay in LDS for the 3 -> Cout residual conv of the epilogue): the
// block reads 12 B and writes 256 B per pixel, against the 256 + 768 B of
// the gcn0 + temporal-conv pair.
template <int CIN, int COUT, int FIN, bool RAW = false>
__global__ __launch_bounds__(512) void stblock_kernel(StbArgs a, int ntiles) {
    using G = StbGeo<CIN, COUT, FIN>;
    constexpr int V = 17;
    // RAW: data_bn'd keypoints, 4 floats per pixel; otherwise bias2 [17][COUT] (the same 4,352 B)
    constexpr int XSB = RAW ? FIN * V * 4 * 4 : V * COUT * 4;
    constexpr int BSB = RAW ? COUT * 4 : 0;   // RAW: the epilogue bias in LDS
    static_assert(G::SMEM + XSB + BSB <= 163840, "LDS");
    __shared__ __attribute__((aligned(16))) unsigned char smem[G::SMEM + XSB + BSB];   // the only LDS object
    unsigned char* const zimg = smem;
    unsigned char* const ring = smem + G::ZBYTES;

    const int tid = threadIdx.x, lane = tid & 63;
    TIK_FENCE_BEGIN();
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int g = lane >> 4;
    const int QO = a.nwin * a.T;   // frames (flat, input = output for stride 1)
    const int M = QO * V;          // rows
    // persistent: one workgroup per CU walks a contiguous run of tiles (runs
    // ordered per XCD, so the halo frames neighbouring tiles share are L2 hits)
    int t_begin, t_end;
    {
        const int nwg = gridDim.x, bid = blockIdx.x;
        const int per = nwg >> 3, rem = nwg & 7, x = bid & 7, k = bid >> 3;
        const int s = x < rem ? x * (per + 1) + k : rem * (per + 1) + (x - rem) * per + k;
        t_begin = (int)((long long)s * ntiles / nwg);
        t_end = (int)((long long)(s + 1) * ntiles / nwg);
    }
    unsigned long long trs[5] = {0, 0, 0, 0, 0};   // debug: phase sums over this workgroup's tiles

    // The mix matrix goes to registers before any DMA is issued (an LDS read
    // after an LDS-DMA gets a compiler vmcnt(0): possible alias):
    // amv[k] lane l = A[64 k + l], read back with v_readlane (wave-uniform).
    constexpr int NAM = (V * V + 63) / 64;
    float amv[NAM];
#pragma unroll
    for (int k = 0; k < NAM; ++k) amv[k] = 64 * k + lane < V * V ? a.amix[64 * k + lane] : 0.f;

    // ---- DMA roles (lane l of an instruction writes unit l&7 of image row l>>3)
    constexpr int NXI = G::PXR / 8, NXJ = (NXI + 7) / 8;   // x instructions per chunk / per wave (max)
    constexpr int NWJ = COUT / 64;                          // Wg / Wt instructions per wave per chunk
    unsigned xoff[NXJ];
    auto set_xoff = [&](int tl) {   // x rows of tile tl (input frames tl*F-1 .. tl*F+F)
        const int f0 = tl * G::F - 1;
#pragma unroll
        for (int j = 0; j < NXJ; ++j) {
            const int idx = wave + 8 * j;
            const int rr = idx * 8 + (lane >> 3);   // image row: joint rr / 16, frame rr % 16
            const int ck = (lane & 7) ^ sbf(rr);
            const long long gr = (long long)(f0 + (rr & 15)) * V + (rr >> 4);
            xoff[j] = (idx < NXI && f0 + (rr & 15) >= 0 && gr < M) ? (unsigned)((gr * a.ldx + 8 * ck) * 2) : DMA_OOB;
        }
    };
    const int nxj = (NXI - wave + 7) / 8;   // x instructions of this wave
    unsigned wgoff[NWJ], wtoff[NWJ];
#pragma unroll
    for (int j = 0; j < NWJ; ++j) {
        const int rr = (wave * NWJ + j) * 8 + (lane >> 3);
        const int ck = (lane & 7) ^ sbf(rr);
        wgoff[j] = (unsigned)((rr * a.ldwg + 8 * ck) * 2);
        wtoff[j] = (unsigned)((rr * a.ldwt + 8 * ck) * 2);
    }
    const i32x4 rX = buf_rsrc(a.x, (unsigned)((long long)M * a.ldx * 2));
    const i32x4 rWg = buf_rsrc(a.wg, (unsigned)(COUT * a.ldwg * 2));
    const i32x4 rWt = buf_rsrc(a.wt, (unsigned)(COUT * a.ldwt * 2));

    auto issue_g = [&](int kb, int slot) {
        unsigned char* xs = ring + slot * G::GSLOT;
#pragma unroll
        for (int j = 0; j < NXJ; ++j)
            if (wave + 8 * j < NXI) dma16(rX, xs + (wave + 8 * j) * 1024, xoff[j], kb * 128);
#pragma unroll
        for (int j = 0; j < NWJ; ++j) dma16(rWg, xs + G::XS + (wave * NWJ + j) * 1024, wgoff[j], kb * 128);
    };
    auto issue_t = [&](int c, int slot) {
        unsigned char* ws = ring + slot * G::WS;
#pragma unroll
        for (int j = 0; j < NWJ; ++j) dma16(rWt, ws + (wave * NWJ + j) * 1024, wtoff[j], c * 128);
    };

    float* const xsf = reinterpret_cast<float*>(smem + G::SMEM);
    // RAW: this thread's keypoint elements i = tid + 512 j of a tile's 16 x 17 x 4
    // image (pixel i/4, channel i%4): data_bn scale / shift are tile-invariant, the
    // raw values are loaded a tile ahead (kx) during the previous tile's epilogue
    constexpr int KNE = RAW ? (FIN * V * 4 + 511) / 512 : 1;
    float kx[KNE], ksc[KNE], ksh[KNE];
    bool kok[KNE];
    auto load_kp = [&](int tl) {
        int t_ = tid;   // opaque: the per-element joint / frame offsets are not hoisted out of the tile loop
        asm volatile("" : "+v"(t_));
#pragma unroll
        for (int j = 0; j < KNE; ++j) {
            const int i = t_ + 512 * j, c = i & 3, p = i >> 2;
            const int v = p % V, fr = tl * G::F - 1 + p / V;
            kok[j] = RAW && i < FIN * V * 4 && c < a.c0 && fr >= 0 && fr < QO;
            kx[j] = kok[j] ? a.xraw[((size_t)fr * V + v) * a.c0 + c] : 0.f;
        }
    };
    if constexpr (RAW) {
#pragma unroll
        for (int j = 0; j < KNE; ++j) {
            const int i = tid + 512 * j, c = i & 3, v = (i >> 2) % V;
            const bool ok = i < FIN * V * 4 && c < a.c0;
            ksc[j] = ok ? a.bn_sc[v * a.c0 + c] : 0.f;
            ksh[j] = ok ? a.bn_sh[v * a.c0 + c] : 0.f;
        }
        if (t_begin < t_end) load_kp(t_begin);
        float* bsl = reinterpret_cast<float*>(smem + G::SMEM + XSB);
        if (tid < COUT) bsl[tid] = a.bias[tid];
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // written before the first DMA
        // RAW never uses the ring for anything else: the whole Wt stays resident
        // for every tile of the run (the first T's wait covers it)
#pragma unroll
        for (int c = 0; c < G::NKT; ++c) issue_t(c, c);
    }
    // the first tile's x image (and Wg); later tiles' are prefetched during the
    // previous tile's epilogue
    // non-RAW: bias2 in LDS for the whole run, written before any DMA is in flight
    // (an LDS access behind an LDS-DMA gets a compiler vmcnt(0): possible alias)
    float* const b2s = reinterpret_cast<float*>(smem + G::SMEM);
    if constexpr (!RAW) {
        for (int i = tid; i < V * COUT; i += 512) b2s[i] = a.bias2[i];
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    if (!RAW && t_begin < t_end) {
        set_xoff(t_begin);
        issue_g(0, 0);
        if (G::NKG > 1) issue_g(1, 1);
    }
    // this thread's epilogue bias (4 channels): non-RAW keeps it for the whole
    // run (a load inside the tile would queue behind the x prefetch), RAW
    // (no registers to spare) loads it in each epilogue
    const f32x4 bv_run = RAW ? f32x4{0.f, 0.f, 0.f, 0.f} : *reinterpret_cast<const f32x4*>(a.bias + 4 * (tid % (COUT / 4)));
    for (int tile = t_begin; tile < t_end; ++tile) {
    // every wave is done with the previous tile's epilogue LDS reads (C tile over the
    // z image, RAW keypoint image) before this tile writes them (zero rows, keypoints)
    if (tile != t_begin) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
    }
    // re-materialised every tile: hoisted out of the tile loop, the mix's v_readlane
    // values and the lane-derived addresses would stay live across it and spill
#pragma unroll
    for (int k = 0; k < NAM; ++k) asm volatile("" : "+v"(amv[k]));
    int lt_ = lane;
    asm volatile("" : "+v"(lt_));
    const int lane = lt_, g = lt_ >> 4;
    unsigned long long tr[6];
    if (a.trace) tr[0] = __builtin_amdgcn_s_memrealtime();
    const int q0 = tile * G::F;   // first output frame
    const int r0 = q0 * V;        // first output row
    const int fi0 = q0 - 1;       // first input frame of the z image
    // epilogue operands: the identity residual x of this tile's rows (raw split
    // halves: hi dwords 0-1, lo 2-3), read from the LDS x image at the end of G
    // (it holds exactly these rows: output frame q0 + t is image frame t + 1), and
    // the bias
    constexpr int C4 = COUT / 4, RS = 512 / C4, KI = (G::TR + RS - 1) / RS;
    const int c4 = tid % C4, lr0 = tid / C4, col = 4 * c4;
    f32x4 rr[KI];
    auto resid_from_image = [&]() {
        const unsigned char* X = ring + (col >> 5) * G::GSLOT;
        const int cc = col & 31, u = cc >> 3, bo = (cc & 7) * 2;
#pragma unroll
        for (int k = 0; k < KI; ++k) {
            const int lr = lr0 + k * RS;
            const int tl = lr / V, v = lr - tl * V, ir = 16 * v + tl + 1;
            const bool ok = a.resid && lr < G::TR && r0 + lr < M;
            const f32x2 h = *reinterpret_cast<const f32x2*>(X + sbo(ok ? ir : 0, u) + bo);
            const f32x2 l = *reinterpret_cast<const f32x2*>(X + sbo(ok ? ir : 0, 4 + u) + bo);
            rr[k] = ok ? f32x4{h[0], h[1], l[0], l[1]} : f32x4{0.f, 0.f, 0.f, 0.f};
        }
    };
    if constexpr (RAW) {
        // ================= 1'. G from the raw keypoints. Thread (frame f, channels
        // co..co+3) of a joint half: waves 0-3 joints 0-8, waves 4-7 joints 9-16; every
        // thread forms y for all 17 joints (the mix input), each half mixes its joints.
        const int f = tid & 15, co = 4 * ((tid >> 4) & 15), half = wave >> 2;
        const int w0 = half ? 9 : 0;
        // weights and bias2' (L2 hits), re-loaded every tile through opaque pointers:
        // hoisted out of the tile loop they would stay live across it and spill
        const float* wg0p = a.wg0;
        const float* b2p = a.bias2;
        asm volatile("" : "+s"(wg0p), "+s"(b2p));
        float w[4][4];
#pragma unroll
        for (int e = 0; e < 4; ++e)
#pragma unroll
            for (int c = 0; c < 4; ++c) w[e][c] = c < a.c0 ? wg0p[(co + e) * a.ldwg0 + c] : 0.f;
        f32x4 b[9];
#pragma unroll
        for (int k = 0; k < 9; ++k) b[k] = w0 + k < V ? *reinterpret_cast<const f32x4*>(b2p + (w0 + k) * COUT + co) : f32x4{0.f, 0.f, 0.f, 0.f};
        // data_bn(x) of the 16 frames -> LDS (the raw keypoints were loaded during the
        // previous tile's epilogue)
#pragma unroll
        for (int j = 0; j < KNE; ++j) {
            const int i = tid + 512 * j;
            if (i < FIN * V * 4) xsf[i] = kok[j] ? fmaf(kx[j], ksc[j], ksh[j]) : 0.f;
        }
        if (tid < G::NKB * 8)   // zero rows (taps past a window edge)
            *reinterpret_cast<f32x4*>(zimg + (tid >> 3) * G::ZB + G::ZR * 128 + (tid & 7) * 16) = f32x4{0.f, 0.f, 0.f, 0.f};
        __syncthreads();
        {
            f32x4 y[V];
#pragma unroll
            for (int v = 0; v < V; ++v) {
                const float* xp = xsf + (f * V + v) * 4;
#pragma unroll
                for (int e = 0; e < 4; ++e) y[v][e] = xp[0] * w[e][0] + xp[1] * w[e][1] + xp[2] * w[e][2] + xp[3] * w[e][3];
            }
            const int cc = co & 31;
            unsigned char* zb = zimg + (co >> 5) * G::ZB + (cc & 4) * 2;
            const int uh = cc >> 3;
            auto mix_range = [&](auto w0c, auto w1c, auto sparse_tag) {
                constexpr int W0 = decltype(w0c)::value, W1 = decltype(w1c)::value;
                constexpr bool SP = decltype(sparse_tag)::value;
#pragma unroll
                for (int wj = W0; wj < W1; ++wj) {
                    f32x4 z = b[wj - W0];
#pragma unroll
                    for (int v = 0; v < V; ++v)
                        if (!SP || ((coco_hop2_mask3(wj) >> v) & 1u)) {
                            const float av = __builtin_bit_cast(
                                float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, amv[(v * V + wj) / 64]), (v * V + wj) % 64));
                            z += av * y[v];
                        }
#pragma unroll
                    for (int e = 0; e < 4; ++e) z[e] = z[e] > 0.f ? z[e] : 0.f;
                    f16x4 h, l;
                    split4(z, h, l);
                    const int row = f * V + wj;
                    *reinterpret_cast<f16x4*>(zb + sbo(row, uh)) = h;
                    *reinterpret_cast<f16x4*>(zb + sbo(row, 4 + uh)) = l;
                }
            };
            using I0 = std::integral_constant<int, 0>;
            using I9 = std::integral_constant<int, 9>;
            using I17 = std::integral_constant<int, 17>;
            if (half) {
                if (a.mix_sparse) mix_range(I9{}, I17{}, std::true_type{});
                else mix_range(I9{}, I17{}, std::false_type{});
            } else {
                if (a.mix_sparse) mix_range(I0{}, I9{}, std::true_type{});
                else mix_range(I0{}, I9{}, std::false_type{});
            }
        }
        if (a.trace) tr[1] = tr[2] = __builtin_amdgcn_s_memrealtime();
        // the resident Wt landed (only the first tile waits on it; the previous
        // epilogue's stores are long done) and the z image is complete
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        if (a.trace) tr[3] = __builtin_amdgcn_s_memrealtime();
    } else {
        // ================= 1. G: y^T = Wg'^T x^T; waves 0-3 own channel block `wave`, all 17 joints
        const bool gw = wave < 4;
        f32x4 accg[V];
    #pragma unroll
        for (int j = 0; j < V; ++j) accg[j] = f32x4{0.f, 0.f, 0.f, 0.f};

    #pragma unroll
        for (int kb = 0; kb < G::NKG; ++kb) {
            if (kb + 1 < G::NKG) {   // chunk kb+1 may stay in flight
                if (nxj == NXJ) wait_vm<NXJ + NWJ>();
                else wait_vm<(NXJ > 0 ? NXJ - 1 : 0) + NWJ>();
            } else {
                wait_vm<0>();
            }
            __builtin_amdgcn_s_barrier();
            if (gw) {
                const unsigned char* X = ring + (kb & 1) * G::GSLOT;
                const unsigned char* W = X + G::XS;
                const int r = wave * 16 + (lane & 15);
                const f16x8 ah = *reinterpret_cast<const f16x8*>(W + sbo(r, g));
                const f16x8 al = *reinterpret_cast<const f16x8*>(W + sbo(r, 4 + g));
                // B fragments read GPD joints ahead of their MFMAs (read right before
                // use, every fragment exposed the LDS latency)
                constexpr int GPD = 3;
                f16x8 pbh[GPD + 1], pbl[GPD + 1];
                auto ldb = [&](int j) {
                    const int rx = j * 16 + (lane & 15);
                    pbh[j % (GPD + 1)] = *reinterpret_cast<const f16x8*>(X + sbo(rx, g));
                    pbl[j % (GPD + 1)] = *reinterpret_cast<const f16x8*>(X + sbo(rx, 4 + g));
                };
    #pragma unroll
                for (int j = 0; j < GPD; ++j) ldb(j);
    #pragma unroll
                for (int j = 0; j < V; ++j) {
                    if (j + GPD < V) ldb(j + GPD);
                    // fence the scheduler: under this kernel's register pressure it
                    // otherwise sinks every read to right before its MFMA
                    __builtin_amdgcn_sched_barrier(0);
                    const f16x8 bh = pbh[j % (GPD + 1)], bl = pbl[j % (GPD + 1)];
                    accg[j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(al, bh, accg[j], 0, 0, 0);
                    accg[j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bl, accg[j], 0, 0, 0);
                    accg[j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bh, accg[j], 0, 0, 0);
                    __builtin_amdgcn_sched_barrier(0);
                }
            }
            if (kb + 2 < G::NKG) {
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                __builtin_amdgcn_s_barrier();
                issue_g(kb + 2, kb & 1);
            }
        }
        // bias2 of this lane's 4 channels for all joints, from LDS before the Wt
        // DMAs below (no DMA in flight: no alias wait)
        const int mc = wave * 16 + 4 * g;   // mix channels mc .. mc+3 (waves 0-3)
        f32x4 b2r[V];
    #pragma unroll
        for (int w = 0; w < V; ++w)
            b2r[w] = gw ? *reinterpret_cast<const f32x4*>(b2s + w * COUT + mc) : f32x4{0.f, 0.f, 0.f, 0.f};
        resid_from_image();
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        if (a.trace) tr[1] = __builtin_amdgcn_s_memrealtime();
        // the ring is free: the whole Wt loads during the mix
    #pragma unroll
        for (int c = 0; c < G::NKT; ++c) issue_t(c, c);
        if (a.trace) tr[2] = __builtin_amdgcn_s_memrealtime();

        // ================= 2. mix in registers: z[w] = ReLU(bias2[w] + sum_v A[v][w] y[v])
        if (gw) {
            const int f = lane & 15, cc = mc & 31;
            unsigned char* zb = zimg + (mc >> 5) * G::ZB + (cc & 4) * 2;
            const int uh = cc >> 3;
            auto mix_all = [&](auto sparse_tag) {
                constexpr bool SP = decltype(sparse_tag)::value;
    #pragma unroll
                for (int w = 0; w < V; ++w) {
                    f32x4 z = b2r[w];
    #pragma unroll
                    for (int v = 0; v < V; ++v)
                        if (!SP || ((coco_hop2_mask3(w) >> v) & 1u)) {
                            const float av = __builtin_bit_cast(
                                float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, amv[(v * V + w) / 64]), (v * V + w) % 64));
                            z += av * accg[v];
                        }
    #pragma unroll
                    for (int e = 0; e < 4; ++e) z[e] = z[e] > 0.f ? z[e] : 0.f;
                    f16x4 h, l;
                    split4(z, h, l);
                    const int row = f * V + w;
                    *reinterpret_cast<f16x4*>(zb + sbo(row, uh)) = h;
                    *reinterpret_cast<f16x4*>(zb + sbo(row, 4 + uh)) = l;
                }
            };
            if (a.mix_sparse) mix_all(std::true_type{});
            else mix_all(std::false_type{});
        } else if (tid - 256 < G::NKB * 8) {   // zero rows (taps past a window edge)
            const int i = tid - 256;
            *reinterpret_cast<f32x4*>(zimg + (i >> 3) * G::ZB + G::ZR * 128 + (i & 7) * 16) = f32x4{0.f, 0.f, 0.f, 0.f};
        }
        // the whole Wt landed and the z image is complete
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        if (a.trace) tr[3] = __builtin_amdgcn_s_memrealtime();
    }

    // ================= 3. T: out = z (*) Wt over 3 taps, A from the resident z image
    constexpr int NCGT = COUT / 64, WR = 8 / NCGT, NRB = (G::TRB + WR - 1) / WR;
    const int cgt = wave % NCGT, wr = wave / NCGT;
    int aoh[NRB][3], aol[NRB][3];
#pragma unroll
    for (int i = 0; i < NRB; ++i) {
        const int rb = wr + WR * i;
        const int m = rb * 16 + (lane & 15);
        const int tl = m / V, v = m - tl * V;
        const int q = q0 + tl;
        const bool okm = rb < G::TRB && m < G::TR && q < QO;
        const int to = okm ? q % a.T : 0;
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            const int ti = to + k - 1;
            const int zr = (okm && ti >= 0 && ti < a.T) ? (tl + k) * V + v : G::ZR;
            aoh[i][k] = sbo(zr, g);
            aol[i][k] = sbo(zr, 4 + g);
        }
    }
    f32x4 acct[NRB][4];
#pragma unroll
    for (int i = 0; i < NRB; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acct[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

#pragma unroll
    for (int c = 0; c < G::NKT; ++c) {
        const int tap = c / G::NKB, kb = c % G::NKB;
        const unsigned char* B = ring + c * G::WS;
        const unsigned char* A = zimg + kb * G::ZB;
        f16x8 bh[4], bl[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int r = cgt * 64 + j * 16 + (lane & 15);
            bh[j] = *reinterpret_cast<const f16x8*>(B + sbo(r, g));
            bl[j] = *reinterpret_cast<const f16x8*>(B + sbo(r, 4 + g));
        }
#pragma unroll
        for (int i = 0; i < NRB; ++i) {
            if (wr + WR * i < G::TRB) {
                const f16x8 ah = *reinterpret_cast<const f16x8*>(A + aoh[i][tap]);
                const f16x8 al = *reinterpret_cast<const f16x8*>(A + aol[i][tap]);
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    acct[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(al, bh[j], acct[i][j], 0, 0, 0);
                    acct[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bl[j], acct[i][j], 0, 0, 0);
                    acct[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bh[j], acct[i][j], 0, 0, 0);
                }
            }
        }
    }

    if (a.trace) tr[4] = __builtin_amdgcn_s_memrealtime();
    // ================= 4. epilogue: + bias + x, ReLU, split-block stores
    float rw[4][4];  // RAW: residual conv weights of this thread's 4 channels
#pragma unroll
    for (int e = 0; e < 4; ++e)
#pragma unroll
        for (int c = 0; c < 4; ++c) rw[e][c] = (RAW && c < a.c0) ? a.rw[(col + e) * a.c0 + c] : 0.f;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();   // every wave is done reading z: the C tile goes over it
    // ... and done with the ring: the next tile's x image (and Wg) streams in behind this epilogue
    if (!RAW && tile + 1 < t_end) {
        set_xoff(tile + 1);
        issue_g(0, 0);
        if (G::NKG > 1) issue_g(1, 1);
    }
    if (RAW && tile + 1 < t_end) load_kp(tile + 1);
    float* Cs = reinterpret_cast<float*>(zimg);
#pragma unroll
    for (int i = 0; i < NRB; ++i) {
        if (wr + WR * i < G::TRB) {
            const int crow = (wr + WR * i) * 16 + 4 * g;
#pragma unroll
            for (int j = 0; j < 4; ++j)
#pragma unroll
                for (int e = 0; e < 4; ++e) Cs[(crow + e) * G::LDC + cgt * 64 + j * 16 + (lane & 15)] = acct[i][j][e];
        }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();   // LDS only: the residual loads stay in flight
    const f32x4 bv = RAW ? *reinterpret_cast<const f32x4*>(smem + G::SMEM + XSB + 4 * col) : bv_run;
#pragma unroll
    for (int k = 0; k < KI; ++k) {
        const int lr = lr0 + k * RS, row = r0 + lr;
        if (lr >= G::TR || row >= M) continue;
        f32x4 v = *reinterpret_cast<const f32x4*>(Cs + lr * G::LDC + col) + bv;
        if constexpr (RAW) {   // 3 -> Cout residual conv of data_bn(x) (output frame = z image frame + 1)
            const f32x4 xb = *reinterpret_cast<const f32x4*>(xsf + (lr + V) * 4);
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                v[e] += xb[0] * rw[e][0] + xb[1] * rw[e][1] + xb[2] * rw[e][2] + xb[3] * rw[e][3];
                v[e] = v[e] > 0.f ? v[e] : 0.f;
            }
        } else {
            const f16x4 h = __builtin_bit_cast(f16x4, f32x2{rr[k][0], rr[k][1]});
            const f16x4 l = __builtin_bit_cast(f16x4, f32x2{rr[k][2], rr[k][3]});
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                v[e] += (float)h[e] + (float)l[e];
                v[e] = v[e] > 0.f ? v[e] : 0.f;
            }
        }
        f16x4 oh, ol;
        split4(v, oh, ol);
        unsigned short* o = a.out + (size_t)row * a.ldo + sbc(col);
        *reinterpret_cast<f16x4*>(o) = oh;
        *reinterpret_cast<f16x4*>(o + 32) = ol;
    }
    if (a.trace) {
        tr[5] = __builtin_amdgcn_s_memrealtime();
#pragma unroll
        for (int k = 0; k < 5; ++k) trs[k] += tr[k + 1] - tr[k];
    }
    }   // tile loop
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (a.trace && tid == 0) {   // cumulative phase sums: trace[6 w + k+1] - trace[6 w + k] = phase k
        unsigned long long c = 0;
        a.trace[6 * blockIdx.x] = 0;
        for (int k = 0; k < 5; ++k) {
            c += trs[k];
            a.trace[6 * blockIdx.x + k + 1] = c;
        }
    }
    TIK_FENCE_END();
}

bool stblock_ok(int cin, int cout) { return cin == 64 && cout == 64; }

// persistent grid: one workgroup per CU (156 KB of LDS), at most one per tile
static int stb_grid(int ntiles) {
    static const bool one_tile = getenv("TIK_STB_ONE_TILE") != nullptr;   // tuning hook: a workgroup per tile
    if (one_tile) return ntiles;
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (cus <= 0) cus = 256;
    return ntiles < cus ? ntiles : cus;
}

hipError_t launch_stblock(const StbArgs& a, int cin, int cout, hipStream_t st) {
    if (a.nwin <= 0 || a.T <= 0) return hipSuccess;
    if (!stblock_ok(cin, cout) || !a.x || !a.wg || !a.wt || !a.bias || !a.bias2 || !a.amix || !a.out)
        return hipErrorInvalidValue;
    const long long M = (long long)a.nwin * a.T * 17;
    if (a.ldx < 64 * (cin / 32) || a.ldo < 64 * (cout / 32) || a.ldx % 8 || a.ldo % 8 || a.ldwg < 64 * (cin / 32) ||
        a.ldwt < 3 * 64 * (cout / 32) || a.ldwg % 8 || a.ldwt % 8 || M * a.ldx * 2 >= 0x80000000LL)
        return hipErrorInvalidValue;
    (void)hipGetLastError();
    using G = StbGeo<64, 64, 16>;
    const int QO = a.nwin * a.T;
    const int ntiles = (QO + G::F - 1) / G::F;
    hipLaunchKernelGGL((stblock_kernel<64, 64, 16>), dim3(stb_grid(ntiles)), dim3(512), 0, st, a, ntiles);
    return hipGetLastError();
}

hipError_t launch_stblock0(const StbArgs& a, int cout, hipStream_t st) {
    if (a.nwin <= 0 || a.T <= 0) return hipSuccess;
    if (cout != 64 || !a.xraw || a.c0 < 1 || a.c0 > 4 || !a.bn_sc || !a.bn_sh || !a.wg0 || a.ldwg0 < a.c0 || !a.rw ||
        !a.wt || !a.bias || !a.bias2 || !a.amix || !a.out)
        return hipErrorInvalidValue;
    if (a.ldo < 64 * (cout / 32) || a.ldo % 8 || a.ldwt < 3 * 64 * (cout / 32) || a.ldwt % 8)
        return hipErrorInvalidValue;
    StbArgs b = a;
    b.x = nullptr; b.ldx = 64; b.wg = a.wt; b.ldwg = 64; b.resid = 0;   // unused by the raw G phase
    (void)hipGetLastError();
    using G = StbGeo<64, 64, 16>;
    const int QO = a.nwin * a.T;
    const int ntiles = (QO + G::F - 1) / G::F;
    hipLaunchKernelGGL((stblock_kernel<64, 64, 16, true>), dim3(stb_grid(ntiles)), dim3(512), 0, st, b, ntiles);
    return hipGetLastError();
}

}  // namespace tik
