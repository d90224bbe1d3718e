// tconv.hip — the stride-1 temporal conv (tcn.2, kernel 3, pad 1) of an
// ST-GCN block with its residual, on split f16 activations, with a frame
// HALO instead of three shifted operand copies.
//
// A 128-row output tile covers at most 9 frames of the 17-joint graph; its
// three temporal taps read input frames q-1, q, q+1, i.e. at most 11 frames
// (187 rows). cgemm3 streams those rows three times (once per tap); here each
// 32-channel chunk of the halo is DMA'd into LDS once and the three taps read
// it at row offsets -17, 0, +17. Taps that fall outside the sample's window
// (zero padding of the reference conv, st_gcn_aaai18.py tcn) read a zero row
// of the halo image. The residual conv (1x1, same frames) reuses the halo
// machinery with the centre tap only. Epilogue as cgemm3 (bias, residual,
// ReLU, split store).
//
// Pipeline (one chunk in flight, two blocks per CU): iteration it = (group g
// = channel chunk of a segment, tap k). Per iteration the B tile (weights of
// tap k for this chunk) is DMA'd into a 2-deep ring; per group the halo is
// DMA'd into a 2-deep ring one iteration ahead of its first use.
#include "cgemm3_dev.h"

namespace tik {

template <int BN, int WM, int WN>
__global__ __launch_bounds__(64 * WM * WN) void tconv_halo_kernel(Cgemm3Args a) {
    constexpr int BM = 128, NW = WM * WN, NT = 64 * NW;
    constexpr int FM = BM / WM / 16, FN = BN / WN / 16;
    constexpr int HMAX = 192;             // halo rows in the image (>= 11 frames x 17)
    constexpr int ZR = HMAX - 1;          // a row that is always zero-filled
    constexpr int ASLOT = HMAX * 128;     // split-block rows: 128 B = 32 channels hi | lo
    constexpr int BSLOT = BN * 128;
    constexpr int NIA = HMAX / 8 / NW;    // halo DMA wave-instructions (8 rows each) per wave
    constexpr int NIB = BN / 8 / NW;      // weight DMA wave-instructions per wave
    static_assert(NIA * 8 * NW == HMAX && NIB * 8 * NW == BN, "DMA split");
    constexpr int LDC = BN + 4;
    constexpr int CTILE = BM * LDC * 4;
    constexpr int RING = 2 * ASLOT + 2 * BSLOT;
    constexpr int SMEM = RING > CTILE ? RING : CTILE;
    __shared__ __attribute__((aligned(16))) unsigned char smem[SMEM];

    const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave / WN, wn = wave % WN;
    const int V = a.V, M = a.M, tin = a.tout;
    int r0, n0;
    {   // XCD-aware tile order (cgemm3.hip)
        const int nwg = gridDim.x * gridDim.y, bid = blockIdx.y * gridDim.x + blockIdx.x;
        const int per = nwg >> 3, rem = nwg & 7, x = bid & 7, k = bid >> 3;
        const int swz = x < rem ? x * (per + 1) + k : rem * (per + 1) + (x - rem) * per + k;
        r0 = (swz / gridDim.y) * BM;
        n0 = (swz % gridDim.y) * BN;
    }
    const unsigned long long ts0 = a.trace ? __builtin_amdgcn_s_memrealtime() : 0;

    // halo frames [F0, F0 + HR/V) of the flattened (sample, frame) axis
    const int Q = M / V;
    const int q0 = r0 / V, q1 = (min(r0 + BM, M) - 1) / V;
    const int F0 = max(q0 - 1, 0), F1 = min(q1 + 1, Q - 1);
    const int HR = (F1 - F0 + 1) * V;

    // per-lane A-fragment halo rows: centre-tap row hr1[i]; taps 0 / 2 are
    // hr1 -/+ V when that frame lies inside the sample (bit 2i / 2i+1 of
    // tapok), else the zero row. Kept as scalars per fragment and combined
    // arithmetically each iteration: an indexed [tap][i] table is lowered to
    // scratch memory, whose loads would queue behind the in-flight DMAs.
    const int g = lane >> 4;
    int hr1[FM];
    unsigned tapok = 0;
#pragma unroll
    for (int i = 0; i < FM; ++i) {
        const int r = r0 + wm * FM * 16 + i * 16 + (lane & 15);
        const int q = r / V, w = r - q * V, t = q % tin;
        hr1[i] = r < M ? (q - F0) * V + w : ZR;
        if (r < M && t >= 1) tapok |= 1u << (2 * i);
        if (r < M && t + 1 < tin) tapok |= 2u << (2 * i);
    }

    // DMA roles: instruction j covers 8 image rows; lane l writes unit l & 7 of
    // row l >> 3 and fetches the source unit the swizzle puts there
    int a_row[NIA], a_ck[NIA];
#pragma unroll
    for (int j = 0; j < NIA; ++j) {
        const int hrow = (wave * NIA + j) * 8 + (lane >> 3);
        a_ck[j] = (lane & 7) ^ sbf(hrow);
        a_row[j] = hrow < HR ? F0 * V + hrow : -1;
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

    // iteration space: segment 0 (taps 0,1,2 per chunk), segment 1 (centre tap)
    const int G0 = a.seg[0].nblk;
    const int G1 = a.nseg > 1 ? a.seg[1].nblk : 0;
    const int NIT = 3 * G0 + G1;

    // buffer_load ... lds: per-segment resources (SGPRs), per-lane row offsets
    // fixed per segment (VGPRs), the K-block and tap parts in soffset; rows past
    // the halo / Nc get an offset past num_records and read as zeros
    constexpr unsigned OOB = DMA_OOB;
    const Seg3& S0 = a.seg[0];
    const Seg3& S1 = a.seg[1];
    const i32x4 rA0 = buf_rsrc(S0.src, (unsigned)(M * S0.ld * 2));
    const i32x4 rB0 = buf_rsrc(S0.w, (unsigned)(a.Nc * S0.ldw * 2));
    i32x4 rA1 = rA0, rB1 = rB0;
    if (a.nseg > 1) {
        rA1 = buf_rsrc(S1.src, (unsigned)(M * S1.ld * 2));
        rB1 = buf_rsrc(S1.w, (unsigned)(a.Nc * S1.ldw * 2));
    }
    unsigned ha0[NIA], ha1[NIA], wb0[NIB], wb1[NIB];
#pragma unroll
    for (int j = 0; j < NIA; ++j) {
        ha0[j] = a_row[j] >= 0 ? (a_row[j] * S0.ld + 8 * a_ck[j]) * 2 : OOB;
        ha1[j] = a_row[j] >= 0 ? (a_row[j] * S1.ld + 8 * a_ck[j]) * 2 : OOB;
    }
#pragma unroll
    for (int j = 0; j < NIB; ++j) {
        wb0[j] = b_col[j] >= 0 ? (b_col[j] * S0.ldw + 8 * b_ck[j]) * 2 : OOB;
        wb1[j] = b_col[j] >= 0 ? (b_col[j] * S1.ldw + 8 * b_ck[j]) * 2 : OOB;
    }
    auto issue_halo = [&](int grp, int slot, int j0, int j1) {
        const bool s1 = grp >= G0;
        const int so = 128 * (s1 ? grp - G0 : grp);
        unsigned char* dst = smem + slot * ASLOT + wave * NIA * 1024;
#pragma unroll
        for (int j = j0; j < j1; ++j) {
            if (s1) dma16(rA1, dst + j * 1024, ha1[j], so);
            else dma16(rA0, dst + j * 1024, ha0[j], so);
        }
    };
    auto issue_w = [&](int grp, int tap, int slot, int j0, int j1) {
        const bool s1 = grp >= G0;
        unsigned char* dst = smem + 2 * ASLOT + slot * BSLOT + wave * NIB * 1024;
#pragma unroll
        for (int j = j0; j < j1; ++j) {
            if (s1) dma16(rB1, dst + j * 1024, wb1[j], 128 * (grp - G0));
            else dma16(rB0, dst + j * 1024, wb0[j], 128 * (tap * S0.nblk + grp));
        }
    };

    f32x4 acc[FM][FN];
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int brow = wn * FN * 16 + (lane & 15);
    auto compute = [&](int aslot, int bslot, int tap) {
        const unsigned char* Aimg = smem + aslot * ASLOT;
        const unsigned char* Bimg = smem + 2 * ASLOT + bslot * BSLOT;
        f16x8 bh[FN], bl[FN];
#pragma unroll
        for (int j = 0; j < FN; ++j) {
            bh[j] = *reinterpret_cast<const f16x8*>(Bimg + sbo(brow + j * 16, g));
            bl[j] = *reinterpret_cast<const f16x8*>(Bimg + sbo(brow + j * 16, 4 + g));
        }
#pragma unroll
        for (int i = 0; i < FM; ++i) {
            int hr = hr1[i];
            if (tap != 1) hr = ((tapok >> (2 * i + (tap >> 1))) & 1u) ? hr + (tap - 1) * V : ZR;
            const f16x8 ah = *reinterpret_cast<const f16x8*>(Aimg + sbo(hr, g));
            const f16x8 al = *reinterpret_cast<const f16x8*>(Aimg + sbo(hr, 4 + g));
#pragma unroll
            for (int j = 0; j < FN; ++j) {
                acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(al, bh[j], acc[i][j], 0, 0, 0);
                acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bl[j], acc[i][j], 0, 0, 0);
                acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bh[j], acc[i][j], 0, 0, 0);
            }
        }
    };

    // (group, tap) of iteration it: groups < G0 have 3 taps, the rest 1 (centre)
    auto it_group = [&](int it) { return it < 3 * G0 ? it / 3 : G0 + (it - 3 * G0); };
    auto it_tap = [&](int it) { return it < 3 * G0 ? it % 3 : 1; };
    unsigned long long tw_vm = 0, tw_bar = 0;
    const unsigned long long tl0 = a.trace ? __builtin_amdgcn_s_memtime() : 0;
    if (NIT > 0) {
        issue_halo(0, 0, 0, NIA);
        issue_w(0, it_tap(0), 0, 0, NIB);
        for (int it = 0; it < NIT; ++it) {
            const unsigned long long w0 = a.trace ? __builtin_amdgcn_s_memtime() : 0;
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            const unsigned long long w1 = a.trace ? __builtin_amdgcn_s_memtime() : 0;
            __builtin_amdgcn_s_barrier();
            if (a.trace) {
                const unsigned long long w2 = __builtin_amdgcn_s_memtime();
                tw_vm += w1 - w0; tw_bar += w2 - w1;
            }
            const int grp = it_group(it);
            if (it + 1 < NIT) {
                const int gn = it_group(it + 1);
                if (gn != grp) issue_halo(gn, gn & 1, 0, NIA);
                issue_w(gn, it_tap(it + 1), (it + 1) & 1, 0, NIB);
            }
            compute(grp & 1, it & 1, it_tap(it));
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    const unsigned long long ts1 = a.trace ? __builtin_amdgcn_s_memrealtime() : 0;
    const unsigned long long tl1 = a.trace ? __builtin_amdgcn_s_memtime() : 0;

    const int crow0 = wm * FM * 16 + 4 * (lane >> 4);
    const int ccol0 = wn * FN * 16 + (lane & 15);
    float* Cs = reinterpret_cast<float*>(smem);
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
#pragma unroll
            for (int e = 0; e < 4; ++e) Cs[(crow0 + i * 16 + e) * LDC + ccol0 + j * 16] = acc[i][j][e];
    __syncthreads();
    f32x4 res[EpiMap<BM, BN, NT>::KI];
    epi_resid<BM, BN, NT>(a, r0, n0, tid, res);
    epi_bias<BM, BN, NT, LDC>(a, Cs, bv, r0, n0, tid, res);

    if (a.trace) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (tid == 0) {
            unsigned long long* t = a.trace + 5 * ((size_t)blockIdx.y * gridDim.x + blockIdx.x);
            t[0] = ts0; t[1] = ts1; t[2] = __builtin_amdgcn_s_memrealtime();
            t[3] = tw_vm;    // wave 0: cycles in the DMA wait
            t[4] = tw_bar | ((unsigned long long)(tl1 - tl0) << 32);   // barrier cycles | loop cycles << 32
        }
    }
}

bool tconv_halo_ok(const Cgemm3Args& a) {
    const Seg3& s0 = a.seg[0];
    if (a.V != 17 || a.M % a.V || s0.kt != 3 || s0.stride != 1 || s0.pad != 1 || s0.tin != a.tout) return false;
    if (a.nseg > 1) {
        const Seg3& s1 = a.seg[1];
        if (s1.kt != 1 || s1.stride != 1 || s1.pad != 0 || s1.tin != a.tout) return false;
    }
    return a.zeros && (a.Nc % 64 == 0);
}

hipError_t launch_tconv_halo(const Cgemm3Args& a, int bn, hipStream_t st) {
    if (a.M <= 0 || a.Nc <= 0) return hipSuccess;
    if (!tconv_halo_ok(a) || (bn != 64 && bn != 128)) return hipErrorInvalidValue;
    for (int s = 0; s < a.nseg; ++s)
        if (a.seg[s].nblk <= 0 || a.seg[s].ld % 8 || a.seg[s].ld < 64 * a.seg[s].nblk || !a.seg[s].w) return hipErrorInvalidValue;
    if (a.out_h && (a.ldo % 8 || a.ldo < 64 * sb_blocks(a.Nc))) return hipErrorInvalidValue;
    (void)hipGetLastError();
    // 8 waves (4 per SIMD with two workgroups per CU) hide the barrier and
    // LDS latencies of the 1-chunk-in-flight ring better than 4
    const dim3 grid((a.M + 127) / 128, (a.Nc + bn - 1) / bn), blk(512);
    if (bn == 128) hipLaunchKernelGGL((tconv_halo_kernel<128, 2, 4>), grid, blk, 0, st, a);
    else hipLaunchKernelGGL((tconv_halo_kernel<64, 4, 2>), grid, blk, 0, st, a);
    return hipGetLastError();
}

}  // namespace tik
