// cgemm.hip — implicit-GEMM temporal convolution on gfx950 fp32 MFMA
// (v_mfma_f32_16x16x4_f32: exact f32 fma chain, 64 FLOP/clk/SIMD).
//
// Block = 256 threads = 4 waves; tile BM rows x BN output channels; K is
// walked in chunks of 16 input channels per (segment, tap). Operands are
// staged global -> registers -> LDS (double-buffered, one barrier per chunk),
// A and B both stored [row][k] with a padded 20-float row so one
// ds_read_b128 gives a lane 4 consecutive k. The 16x16x4 MFMA consumes them
// k-permuted: MFMA step j takes k = {j, 4+j, 8+j, 12+j} from the four lane
// groups, identically for A and B, so the sum is unchanged.
#include "cgemm.h"

namespace tik {

typedef float f32x4 __attribute__((ext_vector_type(4)));

static constexpr int BK = 16;
static constexpr int LDK = 20;   // padded LDS row, floats (80 B, 16-B aligned)

template <int BM, int BN, int WM, int WN, int EPI, int VT>
__global__ __launch_bounds__(256) void cgemm_kernel(CgemmArgs a) {
    constexpr int FM = BM / WM / 16;
    constexpr int FN = BN / WN / 16;
    static_assert(FM * WM * 16 == BM && FN * WN * 16 == BN && WM * WN == 4, "tile");
    constexpr int STAGE = 2 * (BM + BN) * LDK;
    constexpr int LDC = BN + 1;
    constexpr int CTILE = (EPI == EPI_GRAPH) ? BM * LDC : 0;
    constexpr int SMEM = STAGE > CTILE ? STAGE : CTILE;
    __shared__ __attribute__((aligned(16))) float smem[SMEM];

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const int wm = wave / WN, wn = wave % WN;
    const int r0 = blockIdx.x * BM;
    const int n0 = blockIdx.y * BN;
    const int V = (VT > 0) ? VT : a.V;

    // ---- per-thread staging assignment ---------------------------------
    constexpr int NA4 = BM * 4, NB4 = BN * 4;   // float4 slots per chunk
    constexpr int LA = (NA4 + 255) / 256, LB = (NB4 + 255) / 256;
    int a_q[LA], a_lrow[LA], a_n[LA], a_t[LA], a_w[LA];
    bool a_live[LA];
#pragma unroll
    for (int i = 0; i < LA; ++i) {
        const int idx = tid + i * 256;
        a_lrow[i] = idx >> 2;
        a_q[i] = idx & 3;
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
        b_lrow[i] = idx >> 2;
        b_q[i] = idx & 3;
        b_live[i] = (idx < NB4) && (n0 + b_lrow[i] < a.Nc);
    }

    // ---- chunk schedule: (seg, tap, c0) ---------------------------------
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
            const int c = c0 + 4 * b_q[i];
            if (b_live[i] && c < sg.cin)
                v = *reinterpret_cast<const f32x4*>(sg.w + (size_t)(n0 + b_lrow[i]) * sg.ldw +
                                                    tap * sg.cin + c);
            rb[i] = v;
        }
    };
    auto store_chunk = [&](int buf) {
        float* As = smem + buf * (BM + BN) * LDK;
        float* Bs = As + BM * LDK;
#pragma unroll
        for (int i = 0; i < LA; ++i)
            if (tid + i * 256 < NA4)
                *reinterpret_cast<f32x4*>(As + a_lrow[i] * LDK + 4 * a_q[i]) = ra[i];
#pragma unroll
        for (int i = 0; i < LB; ++i)
            if (tid + i * 256 < NB4)
                *reinterpret_cast<f32x4*>(Bs + b_lrow[i] * LDK + 4 * b_q[i]) = rb[i];
    };

    f32x4 acc[FM][FN];
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    int seg = 0, tap = 0, c0 = 0;
    auto advance = [&]() {
        c0 += BK;
        if (c0 >= a.seg[seg].cin) {
            c0 = 0;
            if (++tap >= a.seg[seg].kt) { tap = 0; ++seg; }
        }
    };

    load_chunk(seg, tap, c0);
    store_chunk(0);
    __syncthreads();
    const int arow = wm * FM * 16 + (lane & 15);
    const int brow = wn * FN * 16 + (lane & 15);
    const int kof = 4 * (lane >> 4);
    for (int ch = 0; ch < nchunk; ++ch) {
        const int buf = ch & 1;
        const bool more = ch + 1 < nchunk;
        if (more) {
            advance();
            load_chunk(seg, tap, c0);
        }
        const float* As = smem + buf * (BM + BN) * LDK;
        const float* Bs = As + BM * LDK;
        f32x4 fa[FM], fb[FN];
#pragma unroll
        for (int i = 0; i < FM; ++i)
            fa[i] = *reinterpret_cast<const f32x4*>(As + (arow + i * 16) * LDK + kof);
#pragma unroll
        for (int j = 0; j < FN; ++j)
            fb[j] = *reinterpret_cast<const f32x4*>(Bs + (brow + j * 16) * LDK + kof);
#pragma unroll
        for (int k = 0; k < 4; ++k)
#pragma unroll
            for (int i = 0; i < FM; ++i)
#pragma unroll
                for (int j = 0; j < FN; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[i][k], fb[j][k], acc[i][j], 0, 0, 0);
        if (more) store_chunk(buf ^ 1);
        __syncthreads();
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
        float* Cs = smem;
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

hipError_t launch_cgemm(const CgemmArgs& a, int cfg, hipStream_t st) {
    if (a.M <= 0 || a.Nc <= 0) return hipSuccess;
    const dim3 blk(256);
    (void)hipGetLastError();   // drop a stale error left by earlier runtime calls (not ours)
    switch (cfg) {
        case CFG_T128x128: {
            dim3 g((a.M + 127) / 128, (a.Nc + 127) / 128);
            hipLaunchKernelGGL((cgemm_kernel<128, 128, 2, 2, EPI_BIAS, 0>), g, blk, 0, st, a);
            break;
        }
        case CFG_T128x64: {
            dim3 g((a.M + 127) / 128, (a.Nc + 63) / 64);
            hipLaunchKernelGGL((cgemm_kernel<128, 64, 2, 2, EPI_BIAS, 0>), g, blk, 0, st, a);
            break;
        }
        case CFG_G272x64: {
            if (a.V != 17) return hipErrorInvalidValue;
            dim3 g((a.M + 271) / 272, (a.Nc + 63) / 64);
            hipLaunchKernelGGL((cgemm_kernel<272, 64, 1, 4, EPI_GRAPH, 17>), g, blk, 0, st, a);
            break;
        }
        case CFG_S128x128: {
            dim3 g((a.M + 127) / 128, (a.Nc + 127) / 128);
            hipLaunchKernelGGL((cgemm_kernel<128, 128, 2, 2, EPI_SKIN, 0>), g, blk, 0, st, a);
            break;
        }
        case CFG_H64x128: {
            dim3 g((a.M + 63) / 64, (a.Nc + 127) / 128);
            hipLaunchKernelGGL((cgemm_kernel<64, 128, 2, 2, EPI_BIAS, 0>), g, blk, 0, st, a);
            break;
        }
        default:
            return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

}  // namespace tik
