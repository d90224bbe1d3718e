// cgemm.hip — implicit-GEMM temporal convolution on gfx950 MFMA.
//
// Block = 256 threads = 4 waves; tile BM rows x BN output channels; K is
// walked in chunks of BK input channels per (segment, tap). Operands are
// staged global -> registers -> LDS (register prefetch of chunk i+1 while
// chunk i computes), A and B both stored [row][k] in LDS with padded rows so
// one ds_read_b128 feeds one MFMA operand. Two precisions:
//
//  PREC_F32   v_mfma_f32_16x16x4_f32 (exact f32 fma chain, 64 FLOP/clk/SIMD).
//             BK=16; the 4 k of a ds_read_b128 are consumed k-permuted: MFMA
//             step j takes k = {j, 4+j, 8+j, 12+j} from the 4 lane groups,
//             identically for A and B, so the sum is unchanged.
//  PREC_F16X3 v_mfma_f32_16x16x32_f16 on a 2-term split of both operands,
//             x = x_hi + x_lo (x_hi = f16(x), x_lo = f16(x - x_hi)), fp32
//             accumulate of  a_lo.b_hi + a_hi.b_lo + a_hi.b_hi  (a_lo.b_lo,
//             2^-22 relative, dropped): ~fp32 accuracy at 16/3 the f32-MFMA
//             rate. BK=32. Activations are split when staged into LDS;
//             weights arrive pre-split (host) as f16 pairs.
//
// Both share the C/D layout (lane holds rows 4*(lane>>4)+e, column lane&15),
// hence the epilogues.
#include "cgemm.h"

namespace tik {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));

template <int PREC> struct PrecCfg;
template <> struct PrecCfg<PREC_F32> { static constexpr int BK = 16, LDK = 20, ESZ = 4, PLANES = 1; };
template <> struct PrecCfg<PREC_F16X3> { static constexpr int BK = 32, LDK = 40, ESZ = 2, PLANES = 2; };

template <int BM, int BN, int WM, int WN, int EPI, int VT, int PREC, int NBUF>
__global__ __launch_bounds__(256) void cgemm_kernel(CgemmArgs a) {
    constexpr int FM = BM / WM / 16;
    constexpr int FN = BN / WN / 16;
    static_assert(FM * WM * 16 == BM && FN * WN * 16 == BN && WM * WN == 4, "tile");
    using PC = PrecCfg<PREC>;
    constexpr int BK = PC::BK, LDK = PC::LDK;
    // bytes of one staging buffer: (A planes + B planes) rows x LDK elements
    constexpr int ROWB = LDK * PC::ESZ;
    constexpr int BUFB = (BM + BN) * PC::PLANES * ROWB;
    constexpr int STAGE = NBUF * BUFB;
    constexpr int LDC = BN + 1;
    constexpr int CTILE = (EPI == EPI_GRAPH) ? BM * LDC * 4 : 0;
    constexpr int SMEM = STAGE > CTILE ? STAGE : CTILE;
    __shared__ __attribute__((aligned(16))) unsigned char smem[SMEM];

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const int wm = wave / WN, wn = wave % WN;
    const int r0 = blockIdx.x * BM;
    const int n0 = blockIdx.y * BN;
    const int V = (VT > 0) ? VT : a.V;

    // ---- per-thread staging assignment ---------------------------------
    // A: BM rows x BK fp32 = BM*KQ float4 slots (KQ = BK/4)
    constexpr int KQ = BK / 4;
    constexpr int NA4 = BM * KQ;
    constexpr int LA = (NA4 + 255) / 256;
    // B: F32: BN*KQ float4 slots; F16X3: BN*(2*BK/8) 16-B slots (hi and lo planes)
    constexpr int BQ = (PREC == PREC_F32) ? KQ : 2 * BK / 8;
    constexpr int NB4 = BN * BQ;
    constexpr int LB = (NB4 + 255) / 256;
    int a_q[LA], a_lrow[LA], a_n[LA], a_t[LA], a_w[LA];
    bool a_live[LA];
#pragma unroll
    for (int i = 0; i < LA; ++i) {
        const int idx = tid + i * 256;
        a_lrow[i] = idx / KQ;
        a_q[i] = idx % KQ;
        const int r = r0 + a_lrow[i];
        a_live[i] = (idx < NA4) && (r < a.M);
        const int rr = a_live[i] ? r : 0;
        const int q = rr / V;
        a_w[i] = rr - q * V;
        a_n[i] = q / a.tout;
        a_t[i] = q - a_n[i] * a.tout;
    }
    int b_q[LB], b_lrow[LB];
    bool b_live[LB];
#pragma unroll
    for (int i = 0; i < LB; ++i) {
        const int idx = tid + i * 256;
        b_lrow[i] = idx / BQ;
        b_q[i] = idx % BQ;
        b_live[i] = (idx < NB4) && (n0 + b_lrow[i] < a.Nc);
    }

    int nchunk = 0;
    for (int s = 0; s < a.nseg; ++s) nchunk += a.seg[s].kt * ((a.seg[s].cin + BK - 1) / BK);

    f32x4 ra[LA], rb[LB];
    auto load_chunk = [&](int seg, int tap, int c0) {
        const Seg& sg = a.seg[seg];
#pragma unroll
        for (int i = 0; i < LA; ++i) {
            f32x4 v = {0.f, 0.f, 0.f, 0.f};
            const int c = c0 + 4 * a_q[i];
            const int t = sg.stride * a_t[i] + tap - sg.pad;
            if (a_live[i] && c < sg.cin && t >= 0 && t < sg.tin) {
                const size_t row = ((size_t)a_n[i] * sg.tin + t) * V + a_w[i];
                v = *reinterpret_cast<const f32x4*>(sg.src + row * sg.ld + c);
            }
            ra[i] = v;
        }
#pragma unroll
        for (int i = 0; i < LB; ++i) {
            f32x4 v = {0.f, 0.f, 0.f, 0.f};
            if constexpr (PREC == PREC_F32) {
                const int c = c0 + 4 * b_q[i];
                if (b_live[i] && c < sg.cin)
                    v = *reinterpret_cast<const f32x4*>(sg.w + (size_t)(n0 + b_lrow[i]) * sg.ldw + tap * sg.cin + c);
            } else {
                const int part = b_q[i] & 3;
                const int c = c0 + 8 * part;
                if (b_live[i] && c < sg.cin8) {
                    const unsigned short* base = (b_q[i] < 4) ? sg.whi : sg.wlo;
                    v = *reinterpret_cast<const f32x4*>(base + (size_t)(n0 + b_lrow[i]) * sg.ldw8 + tap * sg.cin8 + c);
                }
            }
            rb[i] = v;
        }
    };
    auto store_chunk = [&](int buf) {
        unsigned char* base = smem + buf * BUFB;
        if constexpr (PREC == PREC_F32) {
            float* As = reinterpret_cast<float*>(base);
            float* Bs = As + BM * LDK;
#pragma unroll
            for (int i = 0; i < LA; ++i)
                if (tid + i * 256 < NA4) *reinterpret_cast<f32x4*>(As + a_lrow[i] * LDK + 4 * a_q[i]) = ra[i];
#pragma unroll
            for (int i = 0; i < LB; ++i)
                if (tid + i * 256 < NB4) *reinterpret_cast<f32x4*>(Bs + b_lrow[i] * LDK + 4 * b_q[i]) = rb[i];
        } else {
            _Float16* Ahi = reinterpret_cast<_Float16*>(base);
            _Float16* Alo = Ahi + BM * LDK;
            _Float16* Bhi = Alo + BM * LDK;
            _Float16* Blo = Bhi + BN * LDK;
#pragma unroll
            for (int i = 0; i < LA; ++i)
                if (tid + i * 256 < NA4) {
                    const f32x4 x = ra[i];
                    f16x4 h, l;
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        h[e] = (_Float16)x[e];
                        l[e] = (_Float16)(x[e] - (float)h[e]);
                    }
                    *reinterpret_cast<f16x4*>(Ahi + a_lrow[i] * LDK + 4 * a_q[i]) = h;
                    *reinterpret_cast<f16x4*>(Alo + a_lrow[i] * LDK + 4 * a_q[i]) = l;
                }
#pragma unroll
            for (int i = 0; i < LB; ++i)
                if (tid + i * 256 < NB4) {
                    _Float16* dst = (b_q[i] < 4) ? Bhi : Blo;
                    *reinterpret_cast<f32x4*>(dst + b_lrow[i] * LDK + 8 * (b_q[i] & 3)) = rb[i];
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
    auto compute = [&](int buf) {
        const unsigned char* base = smem + buf * BUFB;
        if constexpr (PREC == PREC_F32) {
            const float* As = reinterpret_cast<const float*>(base);
            const float* Bs = As + BM * LDK;
            const int kof = 4 * (lane >> 4);
            f32x4 fb[FN];
#pragma unroll
            for (int j = 0; j < FN; ++j) fb[j] = *reinterpret_cast<const f32x4*>(Bs + (brow + j * 16) * LDK + kof);
#pragma unroll
            for (int i = 0; i < FM; ++i) {
                const f32x4 fa = *reinterpret_cast<const f32x4*>(As + (arow + i * 16) * LDK + kof);
#pragma unroll
                for (int k = 0; k < 4; ++k)
#pragma unroll
                    for (int j = 0; j < FN; ++j)
                        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[k], fb[j][k], acc[i][j], 0, 0, 0);
            }
        } else {
            const _Float16* Ahi = reinterpret_cast<const _Float16*>(base);
            const _Float16* Alo = Ahi + BM * LDK;
            const _Float16* Bhi = Alo + BM * LDK;
            const _Float16* Blo = Bhi + BN * LDK;
            const int kof = 8 * (lane >> 4);
            f16x8 bh[FN], bl[FN];
#pragma unroll
            for (int j = 0; j < FN; ++j) {
                bh[j] = *reinterpret_cast<const f16x8*>(Bhi + (brow + j * 16) * LDK + kof);
                bl[j] = *reinterpret_cast<const f16x8*>(Blo + (brow + j * 16) * LDK + kof);
            }
#pragma unroll
            for (int i = 0; i < FM; ++i) {
                const f16x8 ah = *reinterpret_cast<const f16x8*>(Ahi + (arow + i * 16) * LDK + kof);
                const f16x8 al = *reinterpret_cast<const f16x8*>(Alo + (arow + i * 16) * LDK + kof);
#pragma unroll
                for (int j = 0; j < FN; ++j) {
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(al, bh[j], acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bl[j], acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bh[j], acc[i][j], 0, 0, 0);
                }
            }
        }
    };

    int seg = 0, tap = 0, c0 = 0;
    auto advance = [&]() {
        c0 += BK;
        if (c0 >= a.seg[seg].cin) {
            c0 = 0;
            if (++tap >= a.seg[seg].kt) { tap = 0; ++seg; }
        }
    };

    load_chunk(seg, tap, c0);
    if constexpr (NBUF == 2) {
        store_chunk(0);
        __syncthreads();
        for (int ch = 0; ch < nchunk; ++ch) {
            const int buf = ch & 1;
            const bool more = ch + 1 < nchunk;
            if (more) {
                advance();
                load_chunk(seg, tap, c0);
            }
            compute(buf);
            if (more) store_chunk(buf ^ 1);
            __syncthreads();
        }
    } else {
        for (int ch = 0; ch < nchunk; ++ch) {
            store_chunk(0);
            __syncthreads();
            if (ch + 1 < nchunk) {
                advance();
                load_chunk(seg, tap, c0);
            }
            compute(0);
            __syncthreads();
        }
    }

    // ---- epilogue ---------------------------------------------------------
    // 16x16 C/D layout: lane holds rows 4*(lane>>4)+e, column lane&15.
    const int crow0 = wm * FM * 16 + 4 * (lane >> 4);
    const int ccol0 = wn * FN * 16 + (lane & 15);
    if constexpr (EPI == EPI_BIAS) {
#pragma unroll
        for (int j = 0; j < FN; ++j) {
            const int col = n0 + ccol0 + j * 16;
            if (col >= a.Nc) continue;
            const float bj = a.bias ? a.bias[col] : 0.f;
#pragma unroll
            for (int i = 0; i < FM; ++i)
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const int row = r0 + crow0 + i * 16 + e;
                    if (row >= a.M) continue;
                    float v = acc[i][j][e] + bj;
                    if (a.resid) v += a.resid[(size_t)row * a.ldr + col];
                    if (a.act == ACT_RELU) v = v > 0.f ? v : 0.f;
                    else if (a.act == ACT_LEAKY) v = v > 0.f ? v : 0.01f * v;
                    a.out[(size_t)row * a.ldo + col] = v;
                }
        }
    } else if constexpr (EPI == EPI_SKIN) {
        // rows r = b*16 + e, e = 4*row + col of the 3x4 transform T_v(b); lane
        // group g = lane>>4 holds e = 4g..4g+3, i.e. transform row g (g < 3).
        const int g = lane >> 4;
        if (g < 3) {
#pragma unroll
            for (int i = 0; i < FM; ++i) {
                const int b = (r0 + wm * FM * 16 + i * 16) >> 4;
                if (b * 16 >= a.M) continue;
                const float tb = a.bias ? a.bias[b * 3 + g] : 0.f;
                const float* vp = a.resid + (size_t)b * a.ldr;
                float* vo = a.out + (size_t)b * a.ldo;
#pragma unroll
                for (int j = 0; j < FN; ++j) {
                    const int v = n0 + ccol0 + j * 16;
                    if (v >= a.Nc) continue;
                    const f32x4 t = acc[i][j];
                    const float x = fmaf(t[0], vp[3 * v], fmaf(t[1], vp[3 * v + 1], fmaf(t[2], vp[3 * v + 2], t[3])));
                    vo[3 * v + g] = x + tb;
                }
            }
        }
    } else {
        // graph epilogue: BM = F frames * V joints, frame-aligned tiles.
        float* Cs = reinterpret_cast<float*>(smem);
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
            for (int j = 0; j < FN; ++j)
#pragma unroll
                for (int e = 0; e < 4; ++e)
                    Cs[(crow0 + i * 16 + e) * LDC + ccol0 + j * 16] = acc[i][j][e];
        __syncthreads();
        static_assert(VT > 0 && BM % VT == 0, "graph epilogue needs whole frames");
        constexpr int FR = BM / VT;
        constexpr int PAIRS = FR * BN;
        const int frame0 = r0 / VT;
        const int nframes = a.M / VT;
        for (int p = tid; p < PAIRS; p += 256) {
            const int c = p % BN;
            const int f = p / BN;
            const int col = n0 + c;
            if (frame0 + f >= nframes || col >= a.Nc) continue;
            float y[VT];
#pragma unroll
            for (int v = 0; v < VT; ++v) y[v] = Cs[(f * VT + v) * LDC + c];
            float* o = a.out + (size_t)(frame0 + f) * VT * a.ldo + col;
#pragma unroll
            for (int w = 0; w < VT; ++w) {
                float z = 0.f;
#pragma unroll
                for (int v = 0; v < VT; ++v) z = fmaf(a.amix[v * VT + w], y[v], z);
                z += a.bias[w * a.Nc + col];
                o[(size_t)w * a.ldo] = z > 0.f ? z : 0.f;
            }
        }
    }
}

template <int BM, int BN, int WM, int WN, int EPI, int VT>
static hipError_t launch_t(const CgemmArgs& a, int prec, hipStream_t st) {
    const dim3 g((a.M + BM - 1) / BM, (a.Nc + BN - 1) / BN), blk(256);
    // the graph tile (BM=272) keeps one staging buffer in f16x3 so that two
    // workgroups fit a CU's 160 KiB of LDS
    constexpr int NB16 = (BM > 128) ? 1 : 2;
    if (prec == PREC_F16X3)
        hipLaunchKernelGGL((cgemm_kernel<BM, BN, WM, WN, EPI, VT, PREC_F16X3, NB16>), g, blk, 0, st, a);
    else
        hipLaunchKernelGGL((cgemm_kernel<BM, BN, WM, WN, EPI, VT, PREC_F32, 2>), g, blk, 0, st, a);
    return hipGetLastError();
}

hipError_t launch_cgemm(const CgemmArgs& a, int cfg, hipStream_t st, int prec) {
    if (a.M <= 0 || a.Nc <= 0) return hipSuccess;
    if (prec == PREC_F16X3)
        for (int s = 0; s < a.nseg; ++s)
            if (!a.seg[s].whi || !a.seg[s].wlo) return hipErrorInvalidValue;
    (void)hipGetLastError();   // drop a stale error left by earlier runtime calls (not ours)
    switch (cfg) {
        case CFG_T128x128: return launch_t<128, 128, 2, 2, EPI_BIAS, 0>(a, prec, st);
        case CFG_T128x64: return launch_t<128, 64, 2, 2, EPI_BIAS, 0>(a, prec, st);
        case CFG_G272x64:
            if (a.V != 17) return hipErrorInvalidValue;
            return launch_t<272, 64, 1, 4, EPI_GRAPH, 17>(a, prec, st);
        case CFG_H64x128: return launch_t<64, 128, 2, 2, EPI_BIAS, 0>(a, prec, st);
        case CFG_S128x128: return launch_t<128, 128, 2, 2, EPI_SKIN, 0>(a, prec, st);
        default: return hipErrorInvalidValue;
    }
}

}  // namespace tik
