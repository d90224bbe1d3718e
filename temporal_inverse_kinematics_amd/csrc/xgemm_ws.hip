// xgemm_ws.hip — the temporal conv (EPI_BIAS) as ONE persistent,
// warp-specialized launch: bf16x3 arithmetic and results identical to
// xgemm_kernel<128, EPI_BIAS> with the identity residual loaded in the
// epilogue (same products, same K order, same (acc + x) + bias order).
//
// Why: the two-workgroups-per-CU kernel runs both workgroups of a CU in
// lockstep, so their prologues (the first DMA round trip, ~5.8k cycles) and
// epilogues (~16.6k cycles of residual loads and stores) never overlap the
// other's K loop: 37 % of an XT128 tile is spent outside the MFMA loop
// (DESIGN.md §2). A persistent kernel hides the prologue, but when the waves
// that issue the DMAs also store the epilogue, every DMA wait also waits for
// those stores (vmcnt counts loads, LDS-DMA and stores of a wave in order).
// Here the roles are split:
//   * 4 LOADER waves issue every LDS-DMA of the K stream (A: the rows of each
//     K step through the tap / segment row map; B: the packed bf16x3 weight
//     planes), three stages ahead, into a 4-stage ring that fills the CU's
//     160 KB of LDS, across tile boundaries; they wait only on their own
//     DMAs (exact counts);
//   * 4 MFMA waves (one per SIMD, 32 rows x 128 columns each) read, split and
//     multiply; at a tile's last K step they issue the epilogue's residual
//     and bias loads, and after it store the tile straight from the
//     accumulators — fire and forget: none of their waits is on a DMA.
// One s_barrier per K step orders the ring (stage s and s+1 landed, every
// MFMA wave done with stage s-1, whose slot the loaders refill next).
// One 512-thread workgroup per CU; tiles b, b + G, ... of the launch
// (G a multiple of 8: each workgroup stays on its XCD's contiguous run).
#include "xgemm_dev.h"

namespace tik {

// S: ring stages (4: the whole LDS, DMAs issued three stages ahead; 3: two)
template <bool IDN, int S>
__global__ __launch_bounds__(512, 1) void xgemm_ws_kernel(XArgs a) {
    constexpr int BN = 128, NWM = 4, BM = 128, FM = 2, FN = BN / 16, RW = 32;
    constexpr int P = S - 1;                              // stages in flight ahead of the computing one
    constexpr int ABYTES = BM * 128, PLANE = BN * 64, BBYTES = 3 * PLANE;
    constexpr int NIA = RW * 128 / 1024;                  // A DMA instructions per loader wave per stage (4)
    constexpr int NIB = BBYTES / 1024 / NWM;              // B DMA instructions per loader wave per stage (6)
    constexpr int NPS = NIA + NIB;
    static_assert(S * (ABYTES + BBYTES) <= 160 * 1024 && BBYTES % (1024 * NWM) == 0, "ring");
    __shared__ __attribute__((aligned(16))) unsigned char smem[S * (ABYTES + BBYTES)];

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int g = lane >> 4;
    const int V = a.V;
#ifdef TIK_XTUNE
    // diagnostic build only: parts switched off (1 A DMA, 2 B DMA, 4 MFMAs, 8 split, 16 epilogue stores)
    const int tune = a.tune;
#else
    constexpr int tune = 0;
#endif
#ifdef TIK_XTRACE
    // diagnostic build only: per-workgroup phase sums (s_memtime cycles) of MFMA wave 0 and loader wave 0
    const bool tr = a.trace != nullptr;
#else
    constexpr bool tr = false;
#endif
    unsigned long long ph[4] = {0, 0, 0, 0}, tnow = tr ? __builtin_amdgcn_s_memtime() : 0, tstart = tnow;
    auto stamp = [&](int i) __attribute__((always_inline)) {
        if (tr) {
            const unsigned long long t = __builtin_amdgcn_s_memtime();
            ph[i] += t - tnow;
            tnow = t;
        }
    };
    auto trace_out = [&](int base) __attribute__((always_inline)) {
        if (tr && lane == 0) {
            unsigned long long* o = a.trace + 16 * (size_t)blockIdx.x + base;
            o[0] = ph[0]; o[1] = ph[1]; o[2] = ph[2]; o[3] = ph[3];
            o[4] = __builtin_amdgcn_s_memtime() - tstart; o[5] = 1;
        }
    };
    const int ntn = a.Nc / BN;                            // column tiles (Nc % 128 == 0: the launch checks)
    const int ntot = ((a.M + BM - 1) / BM) * ntn;
    const int G = gridDim.x, b = blockIdx.x;
    const int my = b < ntot ? (ntot - 1 - b) / G + 1 : 0;
    if (my == 0) return;
    const int K = xgemm_kmain(a);                         // K steps per tile
    const int total = my * K;
    auto tile_of = [&](int i, int& r0, int& nt) __attribute__((always_inline)) {
        const int L = b + i * G;
        const int per = ntot >> 3, rem = ntot & 7, x = L & 7, k = L >> 3;
        const int swz = x < rem ? x * (per + 1) + k : rem * (per + 1) + (x - rem) * per + k;
        r0 = (swz / ntn) * BM;
        nt = swz - (swz / ntn) * ntn;
    };
    auto a_slot = [&](int s) __attribute__((always_inline)) { return smem + (s % S) * ABYTES; };
    auto b_slot = [&](int s) __attribute__((always_inline)) { return smem + S * ABYTES + (s % S) * BBYTES; };

    if (wave >= NWM) {
        // =========================== loader wave lw: fills rows 32 lw .. 32 lw + 31
        // of every A stage (the rows MFMA wave lw reads) and 6 of the 24 KB of B
        const int lw = wave - NWM;
        int a_n[NIA], a_t[NIA], a_w[NIA], a_uo[NIA];
        bool a_ok[NIA];
#pragma unroll
        for (int j = 0; j < NIA; ++j) {
            const int rr = (lw * NIA + j) * 8 + (lane >> 3);
            const int pl = (lane & 7) ^ xa_swz(rr);
            a_uo[j] = 32 * (pl & 3) + 16 * (pl >> 2);
        }
        auto set_rows = [&](int r0) __attribute__((always_inline)) {
#pragma unroll
            for (int j = 0; j < NIA; ++j) {
                const int row = r0 + (lw * NIA + j) * 8 + (lane >> 3);
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
        int ia = 0, ca_seg = 0, ca_tap = 0, ca_blk = 0, kbi = 0, ntb = 0, gs = 0;
        {
            int r0;
            tile_of(0, r0, ntb);
            set_rows(r0);
        }
        unsigned a_off[NIA];
        i32x4 rA;
        bool a_stale = true;
        const i32x4 rB = buf_rsrc(a.wp, (unsigned)((size_t)ntn * K * BBYTES));
        // one stage: this wave's A rows of K step (ca_seg, ca_tap, ca_blk) of tile ia
        // and its share of the step's weight image; then advance the cursor
        auto issue = [&]() __attribute__((always_inline)) {
            if (a_stale) {
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
            }
            unsigned char* A = a_slot(gs);
            const int soA = __builtin_amdgcn_readfirstlane(ca_blk * 128);
            if (!(tune & 1))
#pragma unroll
                for (int j = 0; j < NIA; ++j) dma16(rA, A + (lw * NIA + j) * 1024, a_off[j], soA);
            unsigned char* Bd = b_slot(gs);
            const int soB = __builtin_amdgcn_readfirstlane((ntb * K + kbi) * BBYTES);
            if (!(tune & 2))
#pragma unroll
                for (int q = 0; q < NIB; ++q)
                    dma16(rB, Bd + (lw + q * NWM) * 1024, (unsigned)((lw + q * NWM) * 1024 + lane * 16), soB);
            ++gs;
            const unsigned f = nbk >> (16 * ca_seg);
            const int seg = ca_seg, tap = ca_tap;
            if (++ca_blk >= (int)(f & 255u)) {
                ca_blk = 0;
                if (++ca_tap >= (int)((f >> 8) & 255u)) {
                    ca_tap = 0;
                    if (++ca_seg >= a.nseg) ca_seg = 0;
                }
            }
            if (++kbi == K) {   // the tile's last K step: on to the next tile
                kbi = 0;
                if (++ia < my) {
                    int r0;
                    tile_of(ia, r0, ntb);
                    set_rows(r0);
                }
            }
            a_stale = ca_seg != seg || ca_tap != tap || kbi == 0;
        };
        // prologue: stages 0 .. P-1 in flight; stage 0 landed before the first barrier
        for (int i = 0; i < P; ++i)
            if (i < total) issue();
        if (tune) wait_vm<0>();
        else if (S == 4 && 2 < total) wait_vm<2 * NPS>();
        else if (1 < total) wait_vm<NPS>();
        else wait_vm<0>();
        __builtin_amdgcn_s_barrier();
        stamp(3);
        for (int s = 0; s < total; ++s) {
            // stage s + 1 landed (stages s + 2 .. s + P - 1 may still fly)
            if (tune) wait_vm_dyn(S == 4 && s + 2 < total ? ((tune & 1) ? 0 : NIA) + ((tune & 2) ? 0 : NIB) : 0);
            else if (S == 4 && s + 2 < total) wait_vm<NPS>();
            else wait_vm<0>();
            stamp(0);
            __builtin_amdgcn_s_barrier();
            stamp(1);
            // stage s + P into the slot of stage s - 1: every MFMA wave finished
            // reading it before this barrier (B(s-1) in step s-1, A(s-1) in step s-2)
            if (s + P < total) issue();
            stamp(2);
        }
        if (lw == 0) trace_out(8);   // loader: vmcnt wait, barrier wait, issue, prologue, total
        return;
    }

    // =========================== MFMA wave w: rows 32 w .. 32 w + 31, all 128 columns
    const int w = wave;
    const float slope = a.act == ACT_RELU ? 0.f : (a.act == ACT_LEAKY ? 0.01f : 1.f);
    f32x4 acc[FM][FN];
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int bsw = (-((lane & 15) >> 2)) & 3;
    const int boff = (lane & 15) * 64 + ((g ^ bsw) << 4);
    auto mma = [&](const xbf16x8& x, const xbf16x8& wt, f32x4& c) __attribute__((always_inline)) {
        // transposed: C^T = W . X^T, so lane l holds row (l & 15), channels 4 (l >> 4) .. +3
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wt, x, c, 0, 0, 0);
    };
    auto read_a = [&](int s, f32x4 (&lo)[FM], f32x4 (&hi)[FM]) __attribute__((always_inline)) {
        const unsigned char* A = a_slot(s);
#pragma unroll
        for (int i = 0; i < FM; ++i) {
            const int r = w * RW + i * 16 + (lane & 15);
            lo[i] = *reinterpret_cast<const f32x4*>(A + r * 128 + ((g ^ xa_swz(r)) << 4));
            hi[i] = *reinterpret_cast<const f32x4*>(A + r * 128 + (((g + 4) ^ xa_swz(r)) << 4));
        }
    };
    // epilogue operands of tile ic, issued at the start of its last K step so
    // their latency hides under that step's MFMAs. The tile's 128 bias values sit
    // in 2 VGPRs across the wave (lane l: columns l and 64 + l) and reach the
    // lanes that need them by ds_bpermute in the epilogue (32 VGPRs of per-lane
    // bias beside the residual rows would not fit)
    float bw[2];
    f32x4 xi[IDN ? FM : 1][IDN ? FN : 1];
    auto load_epi = [&](int ic) __attribute__((always_inline)) {
        int r0, nt;
        tile_of(ic, r0, nt);
        bw[0] = a.bias[nt * BN + lane];
        bw[1] = a.bias[nt * BN + 64 + lane];
        if constexpr (IDN) {
#pragma unroll
            for (int i = 0; i < FM; ++i) {
                const int row = r0 + w * RW + 16 * i + (lane & 15);
                const int rc = row < a.M ? row : 0;   // rows past M read row 0 (not stored)
#pragma unroll
                for (int j = 0; j < FN; ++j)
                    xi[i][j] = *reinterpret_cast<const f32x4*>(a.idn.src + (size_t)rc * a.idn.ld + nt * BN + 16 * j + 4 * g);
            }
        }
    };
    // the finished tile ic from the accumulators: (acc + x) + bias, activation,
    // float4 stores (rows past M go to the trash line: no branch between stores)
    auto epilogue = [&](int ic) __attribute__((always_inline)) {
        int r0, nt;
        tile_of(ic, r0, nt);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's epilogue loads (its older stores too)
#pragma unroll
        for (int i = 0; i < FM; ++i) {
            const int row = r0 + w * RW + 16 * i + (lane & 15);
#pragma unroll
            for (int j = 0; j < FN; ++j) {
                f32x4 v = acc[i][j];
                if constexpr (IDN) v += xi[i][j];
                f32x4 bvj;
#pragma unroll
                for (int e = 0; e < 4; ++e) {   // column 16 j + 4 g + e: lane (16 j + 4 g + e) % 64 of bw[j / 4]
                    const int c = 16 * j + 4 * g + e;
                    bvj[e] = __builtin_bit_cast(float, __builtin_amdgcn_ds_bpermute(4 * (c & 63), __builtin_bit_cast(int, bw[j / 4])));
                }
                v += bvj;
#pragma unroll
                for (int e = 0; e < 4; ++e) v[e] = v[e] > 0.f ? v[e] : slope * v[e];
                float* dst = row < a.M ? a.out + (size_t)row * a.ldo + nt * BN + 16 * j + 4 * g : a.trash + 4 * g;
                if (!(tune & 16)) xst4(dst, v, a.nts);
                acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
            }
        }
    };

    xbf16x8 c0[FM], c1[FM], c2[FM], d0[FM], d1[FM], d2[FM];
    f32x4 alo[FM], ahi[FM];
    __builtin_amdgcn_s_barrier();   // stage 0 landed
    read_a(0, alo, ahi);
#pragma unroll
    for (int i = 0; i < FM; ++i) xsplit8(alo[i], ahi[i], c0[i], c1[i], c2[i]);

    int k = 0, ic = 0;   // the computing tile and its K step
    // global step s: MFMAs of (tile ic, step k) on the split in u; step s+1's A
    // (possibly the next tile's step 0) read and split into v between them
    auto step = [&](int s, xbf16x8 (&u0)[FM], xbf16x8 (&u1)[FM], xbf16x8 (&u2)[FM], xbf16x8 (&v0)[FM],
                    xbf16x8 (&v1)[FM], xbf16x8 (&v2)[FM]) __attribute__((always_inline)) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        stamp(3);
        __builtin_amdgcn_s_barrier();   // stages s and s+1 landed; every wave done with stage s-1
        stamp(0);
        const bool last = k == K - 1;
        if (last) load_epi(ic);
        const unsigned char* Bp = b_slot(s) + boff;
        xbf16x8 bb[2][3];
        __builtin_amdgcn_sched_barrier(0);
        read_a(s + 1, alo, ahi);   // past the last stage: a stale slot, discarded
#pragma unroll
        for (int p = 0; p < 3; ++p) bb[0][p] = *reinterpret_cast<const xbf16x8*>(Bp + p * PLANE);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int j = 0; j < FN; ++j) {
            if (j + 1 < FN)
#pragma unroll
                for (int p = 0; p < 3; ++p)
                    bb[(j + 1) & 1][p] = *reinterpret_cast<const xbf16x8*>(Bp + p * PLANE + (j + 1) * 16 * 64);
            const xbf16x8(&bq)[3] = bb[j & 1];
#pragma unroll
            for (int i = 0; i < FM; ++i) {
                if (!(tune & 4)) {
                    mma(u2[i], bq[0], acc[i][j]);
                    mma(u1[i], bq[1], acc[i][j]);
                    mma(u0[i], bq[2], acc[i][j]);
                    mma(u1[i], bq[0], acc[i][j]);
                    mma(u0[i], bq[1], acc[i][j]);
                    mma(u0[i], bq[0], acc[i][j]);
                } else {
                    acc[i][j][0] += (float)u0[i][0] * (float)bq[0][0];   // keep the reads live
                }
            }
            if (j < FM && !(tune & 8)) {
                xsplit8(alo[j], ahi[j], v0[j], v1[j], v2[j]);
                // pin the split here, between this step's MFMA groups: without it the
                // compiler sinks the whole chain past the next barrier, in front of the
                // next step's first MFMA (one MFMA wave per SIMD: nothing covers it)
                asm volatile("" : "+v"(v0[j]), "+v"(v1[j]), "+v"(v2[j]));
            }
            if (j + 1 < FN) __builtin_amdgcn_sched_group_barrier(0x100, 3, 0);
#pragma unroll
            for (int q = 0; q < 6 * FM; ++q) {
                __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                __builtin_amdgcn_sched_group_barrier(0x002, 2, 0);
            }
            __builtin_amdgcn_sched_barrier(0);
        }
        stamp(1);
        if (last) epilogue(ic);
        stamp(2);
        // branch-free cursor update (a pointer select between k and ic would put both in scratch)
        ic += last ? 1 : 0;
        k = last ? 0 : k + 1;
    };
    int s = 0;
    for (; s + 1 < total; s += 2) {
        step(s, c0, c1, c2, d0, d1, d2);
        step(s + 1, d0, d1, d2, c0, c1, c2);
    }
    if (s < total) step(s, c0, c1, c2, d0, d1, d2);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (w == 0) trace_out(0);   // MFMA: barrier wait, compute, epilogue, lgkm wait, total
}

bool xgemm_ws_ok(const XArgs& a) {
    return a.Nc % 128 == 0 && xgemm_kmain(a) >= 1 && a.ksplit <= 1 && !a.rx && a.trash && a.bias && a.ldo % 4 == 0 &&
           a.nseg >= 1 && a.nseg <= 2;
}

hipError_t launch_xgemm_ws(const XArgs& a, int ncu, hipStream_t st, int stages) {
    if (a.M <= 0 || a.Nc <= 0) return hipSuccess;
    if (!xgemm_ws_ok(a) || !a.wp || !a.out || ncu <= 0) return hipErrorInvalidValue;
    for (int s = 0; s <= a.nseg; ++s) {
        const XSeg& g = s < a.nseg ? a.seg[s] : a.idn;
        if (s == a.nseg && !g.src) break;
        // the K cursor packs cin/32 and kt into 8 bits each
        if (!g.src || g.cin % 32 || g.cin / 32 > 255 || g.kt < 1 || g.kt > 255 || g.ld % 4 || g.ld < g.cin ||
            g.rows_in * g.ld * 4 >= (1LL << 31))
            return hipErrorInvalidValue;
    }
    if (a.idn.src && (a.idn.kt != 1 || a.idn.stride != 1 || a.idn.pad != 0 || a.idn.tin != a.tout || a.idn.cin != a.Nc))
        return hipErrorInvalidValue;
    if ((long long)a.M * a.ldo >= (1LL << 31) * 1LL * 4) return hipErrorInvalidValue;
    const long long ntot = (long long)((a.M + 127) / 128) * (a.Nc / 128);
    long long G = std::min<long long>(ntot, (long long)ncu);
    if (G > 8) G &= ~7LL;   // a multiple of 8: tile id b + i G stays on the workgroup's XCD
    (void)hipGetLastError();
    if (stages == 3) {
        if (a.idn.src) hipLaunchKernelGGL((xgemm_ws_kernel<true, 3>), dim3((unsigned)G), dim3(512), 0, st, a);
        else hipLaunchKernelGGL((xgemm_ws_kernel<false, 3>), dim3((unsigned)G), dim3(512), 0, st, a);
    } else {
        if (a.idn.src) hipLaunchKernelGGL((xgemm_ws_kernel<true, 4>), dim3((unsigned)G), dim3(512), 0, st, a);
        else hipLaunchKernelGGL((xgemm_ws_kernel<false, 4>), dim3((unsigned)G), dim3(512), 0, st, a);
    }
    return hipGetLastError();
}

}  // namespace tik
