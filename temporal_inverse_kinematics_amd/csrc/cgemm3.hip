// cgemm3.hip — f16x3 implicit GEMM with direct global->LDS DMA staging.
//
// Each stage holds, as 64-B rows (32 halves of K) with the swizzle of
// cgemm.hip (16-B chunk c of row r at c ^ SW[(r>>2)&3]), the image
// [A_hi | A_lo | B_hi | B_lo]. Every row chunk is one 16-B
// global_load_lds_dwordx4: lane l of a wave-instruction writes LDS bytes
// [16l, 16l+16) of that instruction's 1 KiB slice, so the swizzle is applied
// on the per-lane SOURCE address (the chunk a lane fetches), never on the
// LDS destination. Padded/out-of-range rows fetch from a zero buffer.
//
// Ring of NSTAGE stages; iteration ch: wait for this wave's DMAs of stage ch
// (counted vmcnt leaves stage ch+1 in flight), s_barrier (everyone's stage ch
// landed, everyone finished reading stage ch-1), issue stage ch+NSTAGE-1 into
// the slot stage ch-1 used, then the MFMAs of stage ch:
//   acc += a_lo.b_hi + a_hi.b_lo + a_hi.b_hi   (v_mfma_f32_16x16x32_f16)
// Epilogues write split planes (or fp32 for the network's final outputs).
#include <type_traits>

#include "cgemm3_dev.h"

namespace tik {

// DBG (tuning only, scripts/kbench.hip): 1 = DMA without MFMA, 2 = MFMA without DMA
template <int BM, int BN, int WM, int WN, int EPI, int VT, int NSTAGE, int DBG = 0>
__global__ __launch_bounds__(64 * WM * WN) void cgemm3_kernel(Cgemm3Args a) {
    constexpr int FM = BM / WM / 16;
    constexpr int FN = BN / WN / 16;
    constexpr int NW = WM * WN;                 // waves per workgroup
    constexpr int NT = 64 * NW;
    static_assert(FM * WM * 16 == BM && FN * WN * 16 == BN && (NW == 4 || NW == 8), "tile");
    constexpr int R = BM + BN;                  // 128-B image rows per stage (A rows, then B rows)
    static_assert(R % 8 == 0, "image rows");
    constexpr int NIT = R / 8;                  // DMA wave-instructions (8 rows each) per stage
    constexpr int NI = (NIT + NW - 1) / NW;     // ... per wave (the last waves may issue fewer)
    constexpr int PN = NIT % NI;                // count of a partial wave (0: none)
    constexpr int STAGEB = NIT * 1024;
    constexpr int LDC = BN + 4;
    constexpr int CTILE = BM * LDC * 4;
    constexpr int SMEM = NSTAGE * STAGEB > CTILE ? NSTAGE * STAGEB : CTILE;
    // epilogue constants staged once, so the epilogue issues no global load
    // behind its own stores (unknown aliasing would serialise each item).
    // ALL LDS lives in one __shared__ array: a second __shared__ object beside
    // the DMA ring makes hipcc wait vmcnt(0) before the first ds_read of every
    // k-step, i.e. for the stage just issued, which serialises DMA and MFMA.
    constexpr int NB = (EPI == EPI_GRAPH) ? VT * BN : BN;
    constexpr int NBA = (NB + 3) & ~3;
    __shared__ __attribute__((aligned(16))) unsigned char smem[SMEM + 4 * NBA];
    float* bias_s = reinterpret_cast<float*>(smem + SMEM);

    const int tid = threadIdx.x;
    TIK_FENCE_BEGIN();
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave / WN, wn = wave % WN;
    // XCD-aware tile order: workgroups are dealt round-robin over the 8 XCDs
    // (each with its own L2); give every XCD a contiguous run of tiles, column
    // tiles of the same rows adjacent, so halo rows and column-tile re-reads
    // hit that XCD's L2 (bijective for any grid size)
    int r0, n0;
    {
        const int nwg = gridDim.x * gridDim.y, bid = blockIdx.y * gridDim.x + blockIdx.x;
        const int per = nwg >> 3, rem = nwg & 7, x = bid & 7, k = bid >> 3;
        const int swz = (a.tune & 1) ? bid : x < rem ? x * (per + 1) + k : rem * (per + 1) + (x - rem) * per + k;
        r0 = (swz / gridDim.y) * BM;
        n0 = (swz % gridDim.y) * BN;
    }
    const int V = (VT > 0) ? VT : a.V;
    const unsigned long long ts0 = a.trace ? __builtin_amdgcn_s_memrealtime() : 0;

    // ---- per-lane DMA roles: instruction j covers image rows 8*(wave*NI+j) .. +7;
    // lane l writes 16-B unit (l & 7) of row (l >> 3), fetching the source unit
    // that the swizzle puts there
    int kind[NI], ck[NI], an[NI], at[NI], aw[NI], bcol[NI];
#pragma unroll
    for (int j = 0; j < NI; ++j) {
        const int r = (wave * NI + j) * 8 + (lane >> 3);
        int rr = r, k = 2;   // 0 A, 1 B, 2 pad
        if (r < BM) { k = 0; }
        else if (r < R) { k = 1; rr = r - BM; }
        ck[j] = (lane & 7) ^ sbf(r);
        an[j] = at[j] = aw[j] = 0;
        bcol[j] = -1;
        if (k == 0) {
            const int row = r0 + rr;
            if (row < a.M) {
                const int q = row / V;
                aw[j] = row - q * V;
                an[j] = q / a.tout;
                at[j] = q - an[j] * a.tout;
            } else {
                k = 2;
            }
        } else if (k == 1) {
            bcol[j] = n0 + rr;
            if (bcol[j] >= a.Nc) k = 2;
        }
        kind[j] = k;
    }

    for (int i = threadIdx.x; i < NB; i += NT) {
        const int w = i / BN, col = n0 + i % BN;
        bias_s[i] = (a.bias && col < a.Nc) ? a.bias[w * a.Nc + col] : 0.f;
    }
    // A_eff in registers (amv[k] lane l = A[64 k + l], read back with v_readlane):
    // the mix reads no broadcast LDS constants (layer0.hip: such reads returned
    // wrong elements when other kernels shared the CU)
    constexpr int NAM = (EPI == EPI_GRAPH) ? (VT * VT + 63) / 64 : 1;
    float amv[NAM];
#pragma unroll
    for (int k = 0; k < NAM; ++k) amv[k] = (EPI == EPI_GRAPH && 64 * k + lane < VT * VT) ? a.amix[64 * k + lane] : 0.f;

    int ktotal = a.seg[0].kt * a.seg[0].nblk;
    if (a.nseg > 1) ktotal += a.seg[1].kt * a.seg[1].nblk;

    // DMA by buffer_load ... lds: a buffer resource per operand (SGPRs), the
    // per-lane row part of the byte offset in a VGPR (recomputed only when the
    // segment or tap changes), the K-block part in the uniform soffset. An
    // invalid row (temporal zero padding, past M / Nc) gets an offset past
    // num_records: the hardware returns zeros.
    constexpr unsigned OOB = DMA_OOB;
    int kindu[NI];
#pragma unroll
    for (int j = 0; j < NI; ++j) kindu[j] = __builtin_amdgcn_readfirstlane(kind[j] == 2 && (wave * NI + j) * 8 < BM ? 0 : kind[j]);
    const int nwin = a.M / (V * a.tout);   // samples in the batch (rows are (n, t', w))
    int seg = 0, tap = 0, c0 = 0;
    unsigned voff[NI];
    i32x4 rsA, rsB;
    int ldwb = 0, nblkb = 0;   // weight row stride and blocks of the current segment (halves)
    // segment fields by constant index only: a runtime-indexed kernarg struct
    // becomes vector loads + vmcnt(0) waits that would drain the DMA ring
    auto set_seg = [&]() {
        const Seg3 sg = (seg == 0) ? a.seg[0] : a.seg[1];
        rsA = buf_rsrc(sg.src, (unsigned)(nwin * sg.tin * V * sg.ld * 2));
        rsB = buf_rsrc(sg.w, (unsigned)(a.Nc * sg.ldw * 2));
        ldwb = sg.ldw; nblkb = sg.nblk;
    };
    auto set_tap = [&]() {
        const Seg3 sg = (seg == 0) ? a.seg[0] : a.seg[1];
#pragma unroll
        for (int j = 0; j < NI; ++j) {
            unsigned v = OOB;
            if (kindu[j] == 0) {
                const int t = sg.stride * at[j] + tap - sg.pad;
                if (kind[j] == 0 && t >= 0 && t < sg.tin) v = ((((an[j] * sg.tin + t) * V + aw[j]) * sg.ld) + 8 * ck[j]) * 2;
            } else if (kindu[j] == 1) {
                v = (kind[j] == 1) ? (bcol[j] * sg.ldw + 8 * ck[j]) * 2 : OOB;
            }
            voff[j] = v;
        }
    };
    const int nb_0 = a.seg[0].nblk * 64, nb_1 = a.seg[1].nblk * 64, kt_0 = a.seg[0].kt, kt_1 = a.seg[1].kt;
    auto advance = [&]() {
        c0 += 64;
        if (c0 >= (seg == 0 ? nb_0 : nb_1)) {
            c0 = 0;
            const int seg0 = seg;
            if (++tap >= (seg == 0 ? kt_0 : kt_1)) { tap = 0; ++seg; }
            if (seg < a.nseg) {
                if (seg != seg0) set_seg();
                set_tap();
            }
        }
    };
    auto issue = [&](int slot) {
        unsigned char* dst = smem + slot * STAGEB + wave * NI * 1024;
        const int soA = c0 * 2, soB = (tap * nblkb * 64 + c0) * 2;
#pragma unroll
        for (int j = 0; j < NI; ++j) {
            if (DBG != 2 && (NIT % NW == 0 || wave * NI + j < NIT)) {
                if (kindu[j] == 1) dma16(rsB, dst + j * 1024, voff[j], soB);
                else dma16(rsA, dst + j * 1024, voff[j], soA);
            }
        }
    };

    f32x4 acc[FM][FN];
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    const int arow = wm * FM * 16 + (lane & 15);
    const int brow = wn * FN * 16 + (lane & 15);
    const int g = lane >> 4;
    auto compute = [&](int slot) {
        if (DBG == 1) return;
        const unsigned char* img = smem + slot * STAGEB;
        f16x8 bh[FN], bl[FN];
#pragma unroll
        for (int j = 0; j < FN; ++j) {
            const int r = BM + brow + j * 16;
            bh[j] = *reinterpret_cast<const f16x8*>(img + sbo(r, g));
            bl[j] = *reinterpret_cast<const f16x8*>(img + sbo(r, 4 + g));
        }
#pragma unroll
        for (int i = 0; i < FM; ++i) {
            const int r = arow + i * 16;
            const f16x8 ah = *reinterpret_cast<const f16x8*>(img + sbo(r, g));
            const f16x8 al = *reinterpret_cast<const f16x8*>(img + sbo(r, 4 + g));
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
    if constexpr (NSTAGE == 1) {
      if (ktotal > 0) {
        // single stage (LDS-bound tiles): DMA of chunk ch+1 waits for compute(ch);
        // a second resident workgroup per CU supplies the overlap
        set_seg();
        set_tap();
        issue(0);
        advance();
        for (int ch = 0; ch < ktotal; ++ch) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __builtin_amdgcn_s_barrier();
            compute(0);
            if (ch + 1 < ktotal) {
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                __builtin_amdgcn_s_barrier();
                issue(0);
                advance();
            }
        }
      }
    } else if (ktotal > 0) {
        set_seg();
        set_tap();
        issue(0);
        advance();
#pragma unroll
        for (int s = 1; s < NSTAGE - 1; ++s)
            if (s < ktotal) { issue(s); advance(); }
        for (int ch = 0; ch < ktotal; ++ch) {
            // this wave's DMAs for stage ch are done when at most the younger
            // stages' NI-instruction groups are still outstanding
            const int ahead = min(NSTAGE - 2, ktotal - 1 - ch);
            const unsigned long long w0 = a.trace ? __builtin_amdgcn_s_memtime() : 0;
            // this wave's DMA count per stage: NI, PN (one partial wave) or 0
            const int myn = min(NI, max(0, NIT - wave * NI));
            if (a.tune & 2) {
                wait_vm<0>();
            } else if (NSTAGE >= 4 && ahead >= 2) {
                if (myn == NI) wait_vm<(NSTAGE >= 4 ? 2 * NI : 0)>();
                else if (myn == PN) wait_vm<(NSTAGE >= 4 ? 2 * PN : 0)>();
                else wait_vm<0>();
            } else if (NSTAGE >= 3 && ahead >= 1) {
                if (myn == NI) wait_vm<(NSTAGE >= 3 ? NI : 0)>();
                else if (myn == PN) wait_vm<(NSTAGE >= 3 ? PN : 0)>();
                else wait_vm<0>();
            } else {
                wait_vm<0>();
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            const unsigned long long w1 = a.trace ? __builtin_amdgcn_s_memtime() : 0;
            __builtin_amdgcn_s_barrier();
            if (a.trace) {
                const unsigned long long w2 = __builtin_amdgcn_s_memtime();
                tw_vm += w1 - w0; tw_bar += w2 - w1;
            }
            if (ch + NSTAGE - 1 < ktotal) {
                issue((ch + NSTAGE - 1) % NSTAGE);
                advance();
            }
            compute(ch % NSTAGE);
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    const unsigned long long ts1 = a.trace ? __builtin_amdgcn_s_memrealtime() : 0;
    const unsigned long long tl1 = a.trace ? __builtin_amdgcn_s_memtime() : 0;

    // ---- epilogues (C tile staged through LDS) -----------------------------
    // identity residual (EPI_BIAS): loads issued before the C-tile staging so
    // their latency overlaps it
    constexpr int KIE = (EPI == EPI_BIAS) ? EpiMap<BM, BN, NT>::KI : 1;
    f32x4 res[KIE];
    if constexpr (EPI == EPI_BIAS) epi_resid<BM, BN, NT>(a, r0, n0, tid, res);
    const int crow0 = wm * FM * 16 + 4 * (lane >> 4);
    const int ccol0 = wn * FN * 16 + (lane & 15);
    float* Cs = reinterpret_cast<float*>(smem);
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
#pragma unroll
            for (int e = 0; e < 4; ++e) Cs[(crow0 + i * 16 + e) * LDC + ccol0 + j * 16] = acc[i][j][e];
    // LDS-only barrier: __syncthreads() would also drain the residual loads
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();

    if constexpr (EPI == EPI_BIAS) {
        const f32x4 bv = *reinterpret_cast<const f32x4*>(bias_s + 4 * (tid % (BN / 4)));
        epi_bias<BM, BN, NT, LDC>(a, Cs, bv, r0, n0, tid, res);
    } else {
        // graph epilogue: frame-aligned tile; (frame, 4 channels) per thread;
        // A_eff and the bias come from LDS, the sparse/dense choice is hoisted
        static_assert(VT == 17 && BN % 4 == 0 && BM % VT == 0, "graph epilogue is built for the 17-joint COCO graph");
        constexpr int FR = BM / VT;
        constexpr int C4 = BN / 4;
        const int frame0 = r0 / VT;
        const int nframes = a.M / VT;
        auto mix = [&](auto sparse) {
            for (int p = tid; p < FR * C4; p += NT) {
                const int c4 = p % C4;
                const int f = p / C4;
                const int col = n0 + 4 * c4;
                if (frame0 + f >= nframes || col >= a.Nc) continue;
                f32x4 y[VT];
#pragma unroll
                for (int v = 0; v < VT; ++v) y[v] = *reinterpret_cast<const f32x4*>(Cs + (f * VT + v) * LDC + 4 * c4);
                const size_t obase = (size_t)(frame0 + f) * VT * a.ldo;
                const bool full = col + 3 < a.Nc;
#pragma unroll
                for (int w = 0; w < VT; ++w) {
                    f32x4 z = *reinterpret_cast<const f32x4*>(bias_s + w * BN + 4 * c4);
#pragma unroll
                    for (int v = 0; v < VT; ++v)
                        if (!decltype(sparse)::value || ((coco_hop2_mask3(w) >> v) & 1u)) {
                            const float av = __builtin_bit_cast(
                                float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, amv[(v * VT + w) / 64]), (v * VT + w) % 64));
                            z += av * y[v];
                        }
#pragma unroll
                    for (int e = 0; e < 4; ++e) z[e] = z[e] > 0.f ? z[e] : 0.f;
                    if (full) {
                        f16x4 h, l;
                        split4(z, h, l);
                        unsigned short* o = a.out_h + obase + (size_t)w * a.ldo + sbc(col);
                        *reinterpret_cast<f16x4*>(o) = h;
                        *reinterpret_cast<f16x4*>(o + 32) = l;
                    } else {
                        for (int e = 0; e < 4 && col + e < a.Nc; ++e) {
                            const _Float16 h = (_Float16)z[e];
                            const _Float16 l = (_Float16)(z[e] - (float)h);
                            unsigned short* o = a.out_h + obase + (size_t)w * a.ldo + sbc(col + e);
                            o[0] = __builtin_bit_cast(unsigned short, h);
                            o[32] = __builtin_bit_cast(unsigned short, l);
                        }
                    }
                }
            }
        };
        if (a.mix_sparse) mix(std::true_type{});
        else mix(std::false_type{});
    }
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
    TIK_FENCE_END();
}

template <int BM, int BN, int WM, int WN, int EPI, int VT, int NSTAGE, int DBG = 0>
static hipError_t launch3(const Cgemm3Args& a, hipStream_t st) {
    const dim3 g((a.M + BM - 1) / BM, (a.Nc + BN - 1) / BN), blk(64 * WM * WN);
    hipLaunchKernelGGL((cgemm3_kernel<BM, BN, WM, WN, EPI, VT, NSTAGE, DBG>), g, blk, 0, st, a);
    return hipGetLastError();
}

hipError_t launch_cgemm3(const Cgemm3Args& a, int cfg, hipStream_t st) {
    if (a.M <= 0 || a.Nc <= 0) return hipSuccess;
    if (!a.zeros) return hipErrorInvalidValue;
    for (int s = 0; s < a.nseg; ++s)
        if (a.seg[s].nblk <= 0 || a.seg[s].ld % 8 || a.seg[s].ld < 64 * a.seg[s].nblk || !a.seg[s].w ||
            a.seg[s].ldw < a.seg[s].kt * a.seg[s].nblk * 64)
            return hipErrorInvalidValue;
    if (a.out_h && (a.ldo % 8 || a.ldo < 64 * sb_blocks(a.Nc))) return hipErrorInvalidValue;
    (void)hipGetLastError();
    switch (cfg) {
        case C3_T128x128: return launch3<128, 128, 2, 2, EPI_BIAS, 0, 2>(a, st);
        case C3_T128x64: return launch3<128, 64, 2, 2, EPI_BIAS, 0, 3>(a, st);
        case C3_G272x64:
            if (a.V != 17) return hipErrorInvalidValue;
            return launch3<272, 64, 1, 4, EPI_GRAPH, 17, 1>(a, st);
        case C3_H64x64: return launch3<64, 64, 2, 2, EPI_BIAS, 0, 3>(a, st);
        // tuning candidates (scripts/kbench.hip)
        case C3_T128x128_S3: return launch3<128, 128, 2, 2, EPI_BIAS, 0, 3>(a, st);
        case C3_T128x128_S4: return launch3<128, 128, 2, 2, EPI_BIAS, 0, 4>(a, st);
        case C3_T256x128_W8: return launch3<256, 128, 4, 2, EPI_BIAS, 0, 3>(a, st);
        case C3_T256x64_W8: return launch3<256, 64, 4, 2, EPI_BIAS, 0, 3>(a, st);
        case C3_T128x64_S4: return launch3<128, 64, 2, 2, EPI_BIAS, 0, 4>(a, st);
        case C3_G272x128_W8:
            if (a.V != 17) return hipErrorInvalidValue;
            return launch3<272, 128, 1, 8, EPI_GRAPH, 17, 3>(a, st);
        case C3_DBG_T128x128_DMA: return launch3<128, 128, 2, 2, EPI_BIAS, 0, 2, 1>(a, st);
        case C3_DBG_T128x128_MFMA: return launch3<128, 128, 2, 2, EPI_BIAS, 0, 2, 2>(a, st);
        case C3_DBG_T128x64_DMA: return launch3<128, 64, 2, 2, EPI_BIAS, 0, 3, 1>(a, st);
        case C3_DBG_T128x64_MFMA: return launch3<128, 64, 2, 2, EPI_BIAS, 0, 3, 2>(a, st);
        case C3_T128x128_W8: return launch3<128, 128, 2, 4, EPI_BIAS, 0, 2>(a, st);
        case C3_T128x64_W8: return launch3<128, 64, 4, 2, EPI_BIAS, 0, 3>(a, st);
        case C3_DBG_W8_DMA: return launch3<128, 128, 2, 4, EPI_BIAS, 0, 2, 1>(a, st);
        case C3_DBG_W8_MFMA: return launch3<128, 128, 2, 4, EPI_BIAS, 0, 2, 2>(a, st);
        case C3_G272x64_S2:
            if (a.V != 17) return hipErrorInvalidValue;
            return launch3<272, 64, 1, 4, EPI_GRAPH, 17, 2>(a, st);
        default: return hipErrorInvalidValue;
    }
}

// ---------------------------------------------------------------- conversions
__global__ void merge_kernel(const unsigned short* __restrict__ sb, long long rows, int C, int ld, float* __restrict__ y) {
    const long long p = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= rows * C) return;
    const long long r = p / C;
    const int c = (int)(p - r * C);
    const unsigned short* q = sb + (size_t)r * ld + ((c >> 5) << 6) + (c & 31);
    y[p] = (float)__builtin_bit_cast(_Float16, q[0]) + (float)__builtin_bit_cast(_Float16, q[32]);
}

// x (px, C<=32) -> one SB block per pixel: per-(v,c) eval BN (channel v*C + c)
__global__ void data_bn_split_kernel(const float* __restrict__ x, int n_px, int V, int C, const float* __restrict__ scale,
                                     const float* __restrict__ shift, unsigned short* __restrict__ sb) {
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= n_px) return;
    const int v = p % V;
    f16x8 h = {}, l = {};
    for (int c = 0; c < C && c < 8; ++c) {
        const float t = fmaf(x[(size_t)p * C + c], scale[v * C + c], shift[v * C + c]);
        h[c] = (_Float16)t;
        l[c] = (_Float16)(t - (float)h[c]);
    }
    f16x8* o = reinterpret_cast<f16x8*>(sb + (size_t)p * 64);
    const f16x8 z = {};
    o[0] = h; o[1] = z; o[2] = z; o[3] = z;
    o[4] = l; o[5] = z; o[6] = z; o[7] = z;
}

hipError_t launch_merge(const unsigned short* sb, long long rows, int C, int ld, float* y, hipStream_t st) {
    const long long n = rows * C;
    if (n <= 0) return hipSuccess;
    (void)hipGetLastError();
    hipLaunchKernelGGL(merge_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, sb, rows, C, ld, y);
    return hipGetLastError();
}

hipError_t launch_data_bn_split(const float* x, int n_px, int V, int C, const float* scale, const float* shift,
                                unsigned short* sb, hipStream_t st) {
    if (n_px <= 0) return hipSuccess;
    if (C > 8) return hipErrorInvalidValue;
    (void)hipGetLastError();
    hipLaunchKernelGGL(data_bn_split_kernel, dim3((n_px + 255) / 256), dim3(256), 0, st, x, n_px, V, C, scale, shift, sb);
    return hipGetLastError();
}

}  // namespace tik
