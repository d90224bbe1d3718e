// cgemm.hip — implicit-GEMM temporal convolution on gfx950 MFMA.
//
// Block = 256 threads = 4 waves; tile BM rows x BN output channels; K is
// walked in chunks of BK input channels per (segment, tap). Operands are
// staged global -> registers -> LDS (register prefetch of chunk i+1 while
// chunk i computes), A and B both stored [row][k] in LDS as unpadded 64-B rows
// of four 16-B chunks, chunk c of row r stored at c ^ SW[(r>>2)&3] with
// SW = {0,3,2,1}: the 16-lane groups of a ds_read_b128 (lane l reads row l&15,
// chunk l>>4) then hit 16 distinct 4-bank slots (conflict-free). One
// ds_read_b128 feeds one MFMA operand. Two precisions:
//
//  PREC_F32   v_mfma_f32_16x16x4_f32 (exact f32 fma chain, 64 FLOP/clk/SIMD).
//             BK=16; the 4 k of a ds_read_b128 are consumed k-permuted: MFMA
//             step j takes k = {j, 4+j, 8+j, 12+j} from the 4 lane groups,
//             identically for A and B, so the sum is unchanged.
//  PREC_BF16X3 v_mfma_f32_16x16x32_bf16 on x = p0 + p1 + p2 (three bf16
//             planes, fp32 range), the six products p_i q_j with i + j <= 2,
//             fp32 accumulation. BK=32. Activations are split when staged into
//             LDS; weights arrive pre-split (host, SplitW3).
//
// Both share the C/D layout (lane holds rows 4*(lane>>4)+e, column lane&15),
// hence the epilogues.
#include "cgemm.h"

namespace tik {

typedef float f32x4 __attribute__((ext_vector_type(4)));

// column w of the COCO-17 hop<=2 adjacency (Graph('coco','uniform',max_hop=2),
// mmskeleton/ops/st_gcn/graph.py:76-133): bit v set <=> A[v][w] != 0 (107 entries)
__host__ __device__ constexpr unsigned coco_hop2_mask(int w) {
    constexpr unsigned m[17] = {0x1Fu,   0x3Fu,   0x5Fu,   0x8EFu,   0x1177u, 0x3BFAu, 0x5DFCu, 0xAE8u,  0x1570u,
                                0x2A0u,  0x540u,  0xF8E8u, 0x17970u, 0xB820u, 0x15840u, 0xA800u, 0x15000u};
    return m[w];
}

template <int PREC> struct PrecCfg;
template <> struct PrecCfg<PREC_F32> { static constexpr int BK = 16, LDK = 16, ESZ = 4, PLANES = 1; };
template <> struct PrecCfg<PREC_BF16X3> { static constexpr int BK = 32, LDK = 32, ESZ = 2, PLANES = 3; };

typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

// x = p0 + p1 + p2, p_i = bf16_rn(residual): v_cvt_pk_bf16_f32 (round to
// nearest even) on the exact fp32 residuals
__device__ __forceinline__ void split3(const f32x4 x, bf16x4& p0, bf16x4& p1, bf16x4& p2) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        p0[e] = (__bf16)x[e];
        const float r1 = x[e] - (float)p0[e];
        p1[e] = (__bf16)r1;
        p2[e] = (__bf16)(r1 - (float)p1[e]);
    }
}

// byte offset of 16-B chunk c of 64-B row r in a swizzled [rows][64 B] image
__device__ __forceinline__ int swz_off(int r, int c) { return r * 64 + ((c ^ ((0x1230 >> (4 * ((r >> 2) & 3))) & 3)) << 4); }

template <int BM, int BN, int WM, int WN, int EPI, int VT, int PREC, int NBUF>
__global__ __launch_bounds__(256) void cgemm_kernel(CgemmArgs a) {
    constexpr int FM = BM / WM / 16;
    constexpr int FN = BN / WN / 16;
    static_assert(FM * WM * 16 == BM && FN * WN * 16 == BN && WM * WN == 4, "tile");
    using PC = PrecCfg<PREC>;
    constexpr int BK = PC::BK, LDK = PC::LDK;
    // bytes of one staging buffer: (A planes + B planes) rows x LDK elements
    constexpr int ROWB = 64;   // BK elements of ESZ bytes: 16 fp32 or 32 halves
    static_assert(LDK * PC::ESZ == ROWB, "64-B rows");
    constexpr int BUFB = (BM + BN) * PC::PLANES * ROWB;
    constexpr int STAGE = NBUF * BUFB;
    constexpr int LDC = BN + 4;   // fp32 C tile row (epilogue), 16-B aligned
    constexpr int CTILE = (EPI == EPI_SKIN) ? 0 : BM * LDC * 4;
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
    // B: F32: BN*KQ float4 slots; BF16X3: BN*(PLANES*BK/8) 16-B slots (one run per plane)
    constexpr int BQ = (PREC == PREC_F32) ? KQ : PC::PLANES * BK / 8;
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

    int ktotal = a.seg[0].kt * ((a.seg[0].cin + BK - 1) / BK);
    if (a.nseg > 1) ktotal += a.seg[1].kt * ((a.seg[1].cin + BK - 1) / BK);
    // split-K (EPI_BIAS only): workgroup z takes chunks [kbeg, kend) and writes raw partial sums
    int kbeg = 0, nchunk = ktotal;
    if (a.ksplit > 1) {
        const int per = (ktotal + a.ksplit - 1) / a.ksplit;
        kbeg = blockIdx.z * per;
        nchunk = min(ktotal, kbeg + per) - kbeg;
        if (nchunk < 0) nchunk = 0;
    }

    // Load cursor (seg, tap, c0) and per-thread source pointers for the current
    // (seg, tap): row addresses are computed once per tap, not per chunk.
    int seg = 0, tap = 0, c0 = 0;
    const float* a_ptr[LA];
    const unsigned char* b_ptr[LB];
    int cin_cur = 0, bcin_cur = 0;
    // segment fields by constant index only (a runtime-indexed kernarg struct
    // turns into vector loads + vmcnt(0) waits in the main loop)
    auto set_tap = [&]() {
        const Seg sg = (seg == 0) ? a.seg[0] : a.seg[1];
        cin_cur = sg.cin;
#pragma unroll
        for (int i = 0; i < LA; ++i) {
            const int t = sg.stride * a_t[i] + tap - sg.pad;
            a_ptr[i] = nullptr;
            if (a_live[i] && t >= 0 && t < sg.tin)
                a_ptr[i] = sg.src + (((size_t)a_n[i] * sg.tin + t) * V + a_w[i]) * sg.ld + 4 * a_q[i];
        }
        if constexpr (PREC == PREC_F32) {
            bcin_cur = sg.cin;
#pragma unroll
            for (int i = 0; i < LB; ++i)
                b_ptr[i] = b_live[i] ? reinterpret_cast<const unsigned char*>(
                                           sg.w + (size_t)(n0 + b_lrow[i]) * sg.ldw + tap * sg.cin + 4 * b_q[i])
                                     : nullptr;
        } else {
            bcin_cur = sg.cin8;
#pragma unroll
            for (int i = 0; i < LB; ++i) {
                const unsigned short* base = (b_q[i] < 4) ? sg.wb[0] : (b_q[i] < 8 ? sg.wb[1] : sg.wb[2]);
                b_ptr[i] = b_live[i] ? reinterpret_cast<const unsigned char*>(
                                           base + (size_t)(n0 + b_lrow[i]) * sg.ldw8 + tap * sg.cin8 + 8 * (b_q[i] & 3))
                                     : nullptr;
            }
        }
    };
    const int cin_0 = a.seg[0].cin, cin_1 = a.seg[1].cin, kt_0 = a.seg[0].kt, kt_1 = a.seg[1].kt;
    auto advance = [&]() {
        c0 += BK;
        if (c0 >= (seg == 0 ? cin_0 : cin_1)) {
            c0 = 0;
            if (++tap >= (seg == 0 ? kt_0 : kt_1)) { tap = 0; ++seg; }
            if (seg < a.nseg) set_tap();
        }
    };
    auto load_into = [&](f32x4 (&ra_)[LA], f32x4 (&rb_)[LB]) {
#pragma unroll
        for (int i = 0; i < LA; ++i) {
            f32x4 v = {0.f, 0.f, 0.f, 0.f};
            if (a_ptr[i] && c0 + 4 * a_q[i] < cin_cur) v = *reinterpret_cast<const f32x4*>(a_ptr[i] + c0);
            ra_[i] = v;
        }
#pragma unroll
        for (int i = 0; i < LB; ++i) {
            f32x4 v = {0.f, 0.f, 0.f, 0.f};
            const int cq = (PREC == PREC_F32) ? 4 * b_q[i] : 8 * (b_q[i] & 3);
            if (b_ptr[i] && c0 + cq < bcin_cur) v = *reinterpret_cast<const f32x4*>(b_ptr[i] + c0 * PC::ESZ);
            rb_[i] = v;
        }
    };
    f32x4 ra[LA], rb[LB], ra1[LA], rb1[LB];
    auto store_from = [&](int buf, const f32x4 (&ra)[LA], const f32x4 (&rb)[LB]) {
        unsigned char* base = smem + buf * BUFB;
        if constexpr (PREC == PREC_F32) {
            unsigned char* As = base;
            unsigned char* Bs = As + BM * 64;
#pragma unroll
            for (int i = 0; i < LA; ++i)
                if (tid + i * 256 < NA4) *reinterpret_cast<f32x4*>(As + swz_off(a_lrow[i], a_q[i])) = ra[i];
#pragma unroll
            for (int i = 0; i < LB; ++i)
                if (tid + i * 256 < NB4) *reinterpret_cast<f32x4*>(Bs + swz_off(b_lrow[i], b_q[i])) = rb[i];
        } else if constexpr (PREC == PREC_BF16X3) {
            unsigned char* A0 = base;
            unsigned char* B0 = A0 + 3 * BM * 64;
#pragma unroll
            for (int i = 0; i < LA; ++i)
                if (tid + i * 256 < NA4) {
                    bf16x4 p0, p1, p2;
                    split3(ra[i], p0, p1, p2);
                    const int off = swz_off(a_lrow[i], a_q[i] >> 1) + 8 * (a_q[i] & 1);
                    *reinterpret_cast<bf16x4*>(A0 + off) = p0;
                    *reinterpret_cast<bf16x4*>(A0 + BM * 64 + off) = p1;
                    *reinterpret_cast<bf16x4*>(A0 + 2 * BM * 64 + off) = p2;
                }
#pragma unroll
            for (int i = 0; i < LB; ++i)
                if (tid + i * 256 < NB4)
                    *reinterpret_cast<f32x4*>(B0 + (b_q[i] >> 2) * BN * 64 + swz_off(b_lrow[i], b_q[i] & 3)) = rb[i];
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
        const int g = lane >> 4;
        if constexpr (PREC == PREC_F32) {
            const unsigned char* As = base;
            const unsigned char* Bs = As + BM * 64;
            f32x4 fb[FN];
#pragma unroll
            for (int j = 0; j < FN; ++j) fb[j] = *reinterpret_cast<const f32x4*>(Bs + swz_off(brow + j * 16, g));
#pragma unroll
            for (int i = 0; i < FM; ++i) {
                const f32x4 fa = *reinterpret_cast<const f32x4*>(As + swz_off(arow + i * 16, g));
#pragma unroll
                for (int k = 0; k < 4; ++k)
#pragma unroll
                    for (int j = 0; j < FN; ++j)
                        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[k], fb[j][k], acc[i][j], 0, 0, 0);
            }
        } else if constexpr (PREC == PREC_BF16X3) {
            // six products a_i.b_j, i + j <= 2 (the dropped ones are <= 2^-24
            // relative each), smallest first, one fp32 accumulator
            const unsigned char* A0 = base;
            const unsigned char* B0 = A0 + 3 * BM * 64;
            bf16x8 b0[FN], b1[FN], b2[FN];
#pragma unroll
            for (int j = 0; j < FN; ++j) {
                const int off = swz_off(brow + j * 16, g);
                b0[j] = *reinterpret_cast<const bf16x8*>(B0 + off);
                b1[j] = *reinterpret_cast<const bf16x8*>(B0 + BN * 64 + off);
                b2[j] = *reinterpret_cast<const bf16x8*>(B0 + 2 * BN * 64 + off);
            }
#pragma unroll
            for (int i = 0; i < FM; ++i) {
                const int off = swz_off(arow + i * 16, g);
                const bf16x8 a0 = *reinterpret_cast<const bf16x8*>(A0 + off);
                const bf16x8 a1 = *reinterpret_cast<const bf16x8*>(A0 + BM * 64 + off);
                const bf16x8 a2 = *reinterpret_cast<const bf16x8*>(A0 + 2 * BM * 64 + off);
#pragma unroll
                for (int j = 0; j < FN; ++j) {
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a2, b0[j], acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1, b1[j], acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0, b2[j], acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1, b0[j], acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0, b1[j], acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0, b0[j], acc[i][j], 0, 0, 0);
                }
            }
        }
    };

    // position the load cursor at chunk kbeg
    {
        int rem = kbeg;
        while (seg < a.nseg) {
            const int nc = ((seg == 0 ? cin_0 : cin_1) + BK - 1) / BK;
            const int segc = (seg == 0 ? kt_0 : kt_1) * nc;
            if (rem < segc) { tap = rem / nc; c0 = (rem % nc) * BK; break; }
            rem -= segc;
            ++seg;
        }
    }
    if (nchunk > 0) set_tap();
    if (nchunk <= 0) {
        // empty K range: contributes zeros
    } else if constexpr (NBUF == 2) {
        // two register sets + two LDS buffers: the global loads of chunk ch+2
        // are issued before chunk ch computes and land in LDS after chunk ch+1
        // computes (two compute phases of latency cover); one barrier per chunk
        load_into(ra, rb);
        advance();
        if (nchunk > 1) { load_into(ra1, rb1); advance(); }
        store_from(0, ra, rb);
        __syncthreads();
        for (int ch = 0; ch < nchunk; ++ch) {
            const bool odd = ch & 1;
            if (ch + 2 < nchunk) {
                if (odd) load_into(ra1, rb1);
                else load_into(ra, rb);
                advance();
            }
            compute(odd ? 1 : 0);
            if (ch + 1 < nchunk) {
                if (odd) store_from(0, ra, rb);
                else store_from(1, ra1, rb1);
            }
            __syncthreads();
        }
    } else {
        load_into(ra, rb);
        advance();
        for (int ch = 0; ch < nchunk; ++ch) {
            store_from(0, ra, rb);
            __syncthreads();
            if (ch + 1 < nchunk) { load_into(ra, rb); advance(); }
            compute(0);
            __syncthreads();
        }
    }

    // ---- epilogue ---------------------------------------------------------
    // 16x16 C/D layout: lane holds rows 4*(lane>>4)+e, column lane&15.
    const int crow0 = wm * FM * 16 + 4 * (lane >> 4);
    const int ccol0 = wn * FN * 16 + (lane & 15);
    if constexpr (EPI == EPI_BIAS) {
        // acc -> LDS C tile -> row-contiguous float4 epilogue (bias, residual, act)
        float* Cs = reinterpret_cast<float*>(smem);
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
            for (int j = 0; j < FN; ++j)
#pragma unroll
                for (int e = 0; e < 4; ++e)
                    Cs[(crow0 + i * 16 + e) * LDC + ccol0 + j * 16] = acc[i][j][e];
        __syncthreads();
        constexpr int C4 = BN / 4;
        const bool vec = (a.ldo % 4 == 0) && (!a.resid || a.ldr % 4 == 0);
        if (a.ksplit > 1) {   // raw partial sums [z][M][Nc]; the reduce kernel applies the epilogue
            float* part = a.partial + (size_t)blockIdx.z * a.M * a.Nc;
            for (int p = tid; p < BM * BN; p += 256) {
                const int lr = p / BN, c = p % BN;
                const int row = r0 + lr, col = n0 + c;
                if (row < a.M && col < a.Nc) part[(size_t)row * a.Nc + col] = Cs[lr * LDC + c];
            }
            return;
        }
        for (int p = tid; p < BM * C4; p += 256) {
            const int lr = p / C4, c4 = p % C4;
            const int row = r0 + lr, col = n0 + 4 * c4;
            if (row >= a.M || col >= a.Nc) continue;
            const f32x4 cv = *reinterpret_cast<const f32x4*>(Cs + lr * LDC + 4 * c4);
            if (vec && col + 3 < a.Nc) {
                f32x4 v = cv;
                if (a.bias) v += *reinterpret_cast<const f32x4*>(a.bias + col);
                if (a.resid) v += *reinterpret_cast<const f32x4*>(a.resid + (size_t)row * a.ldr + col);
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    if (a.act == ACT_RELU) v[e] = v[e] > 0.f ? v[e] : 0.f;
                    else if (a.act == ACT_LEAKY) v[e] = v[e] > 0.f ? v[e] : 0.01f * v[e];
                }
                *reinterpret_cast<f32x4*>(a.out + (size_t)row * a.ldo + col) = v;
            } else {
                for (int e = 0; e < 4 && col + e < a.Nc; ++e) {
                    float v = cv[e] + (a.bias ? a.bias[col + e] : 0.f);
                    if (a.resid) v += a.resid[(size_t)row * a.ldr + col + e];
                    if (a.act == ACT_RELU) v = v > 0.f ? v : 0.f;
                    else if (a.act == ACT_LEAKY) v = v > 0.f ? v : 0.01f * v;
                    a.out[(size_t)row * a.ldo + col + e] = v;
                }
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
        // graph epilogue: BM = F frames * V joints, frame-aligned tiles. One
        // thread per (frame, 4 channels): y[v] for the 17 joints from LDS,
        // z[w] = sum_v A[v][w] y[v] over the COCO hop<=2 pattern (107 of 289
        // entries, unrolled at compile time) when the layer's A fits it,
        // else dense; + bias2[w][c]; ReLU; float4 stores.
        static_assert(VT == 17 && BN % 4 == 0, "graph epilogue is built for the 17-joint COCO graph");
        float* Cs = reinterpret_cast<float*>(smem);
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
            for (int j = 0; j < FN; ++j)
#pragma unroll
                for (int e = 0; e < 4; ++e)
                    Cs[(crow0 + i * 16 + e) * LDC + ccol0 + j * 16] = acc[i][j][e];
        __syncthreads();
        constexpr int FR = BM / VT;
        constexpr int C4 = BN / 4;
        const int frame0 = r0 / VT;
        const int nframes = a.M / VT;
        for (int p = tid; p < FR * C4; p += 256) {
            const int c4 = p % C4;
            const int f = p / C4;
            const int col = n0 + 4 * c4;
            if (frame0 + f >= nframes || col >= a.Nc) continue;
            f32x4 y[VT];
#pragma unroll
            for (int v = 0; v < VT; ++v) y[v] = *reinterpret_cast<const f32x4*>(Cs + (f * VT + v) * LDC + 4 * c4);
            float* o = a.out + (size_t)(frame0 + f) * VT * a.ldo + col;
            const bool full = col + 3 < a.Nc;
#pragma unroll
            for (int w = 0; w < VT; ++w) {
                f32x4 z = {0.f, 0.f, 0.f, 0.f};
                if (a.mix_sparse) {
#pragma unroll
                    for (int v = 0; v < VT; ++v)
                        if ((coco_hop2_mask(w) >> v) & 1u) z += a.amix[v * VT + w] * y[v];
                } else {
#pragma unroll
                    for (int v = 0; v < VT; ++v) z += a.amix[v * VT + w] * y[v];
                }
                if (full) {
                    z += *reinterpret_cast<const f32x4*>(a.bias + w * a.Nc + col);
#pragma unroll
                    for (int e = 0; e < 4; ++e) z[e] = z[e] > 0.f ? z[e] : 0.f;
                    *reinterpret_cast<f32x4*>(o + (size_t)w * a.ldo) = z;
                } else {
                    for (int e = 0; e < 4 && col + e < a.Nc; ++e) {
                        const float t = z[e] + a.bias[w * a.Nc + col + e];
                        o[(size_t)w * a.ldo + e] = t > 0.f ? t : 0.f;
                    }
                }
            }
        }
    }
}

// split-K reduction + EPI_BIAS epilogue: out = act(sum_z partial[z] + bias (+ resid))
__global__ void splitk_reduce_kernel(CgemmArgs a) {
    const long long p = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= (long long)a.M * a.Nc) return;
    const int row = (int)(p / a.Nc), col = (int)(p % a.Nc);
    float v = 0.f;
    for (int z = 0; z < a.ksplit; ++z) v += a.partial[(size_t)z * a.M * a.Nc + p];
    if (a.bias) v += a.bias[col];
    if (a.resid) v += a.resid[(size_t)row * a.ldr + col];
    if (a.act == ACT_RELU) v = v > 0.f ? v : 0.f;
    else if (a.act == ACT_LEAKY) v = v > 0.f ? v : 0.01f * v;
    a.out[(size_t)row * a.ldo + col] = v;
}

template <int BM, int BN, int WM, int WN, int EPI, int VT>
static hipError_t launch_t(const CgemmArgs& a, int prec, hipStream_t st) {
    const dim3 g((a.M + BM - 1) / BM, (a.Nc + BN - 1) / BN, a.ksplit > 1 ? a.ksplit : 1), blk(256);
    // the graph tile (BM=272) keeps one staging buffer in bf16x3 so that two
    // workgroups fit a CU's 160 KiB of LDS
    constexpr int NB16 = (EPI == EPI_GRAPH) ? 1 : 2;
    if (prec == PREC_BF16X3)
        hipLaunchKernelGGL((cgemm_kernel<BM, BN, WM, WN, EPI, VT, PREC_BF16X3, NB16>), g, blk, 0, st, a);
    else
        hipLaunchKernelGGL((cgemm_kernel<BM, BN, WM, WN, EPI, VT, PREC_F32, 2>), g, blk, 0, st, a);
    if (EPI == EPI_BIAS && a.ksplit > 1) {
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
        const long long n = (long long)a.M * a.Nc;
        hipLaunchKernelGGL(splitk_reduce_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, a);
    }
    return hipGetLastError();
}

bool fits_coco_hop2(const float* A, int V) {
    if (V != 17) return false;
    for (int v = 0; v < 17; ++v)
        for (int w = 0; w < 17; ++w)
            if (A[v * 17 + w] != 0.f && !((coco_hop2_mask(w) >> v) & 1u)) return false;
    return true;
}

int splitk_for(const CgemmArgs& a, int BM, int BN, int bk, int max_split) {
    int k = 0;
    for (int s = 0; s < a.nseg; ++s) k += a.seg[s].kt * ((a.seg[s].cin + bk - 1) / bk);
    const int tiles = ((a.M + BM - 1) / BM) * ((a.Nc + BN - 1) / BN);
    if (tiles >= 128 || k < 8) return 1;
    int s = (256 + tiles - 1) / tiles;
    s = s > k / 2 ? k / 2 : s;
    return s > max_split ? max_split : (s < 1 ? 1 : s);
}

hipError_t launch_cgemm(const CgemmArgs& a, int cfg, hipStream_t st, int prec) {
    if (a.M <= 0 || a.Nc <= 0) return hipSuccess;
    if (a.ksplit > 1 && !a.partial) return hipErrorInvalidValue;
    if (prec != PREC_F32 && prec != PREC_BF16X3) return hipErrorInvalidValue;
    if (prec == PREC_BF16X3)
        for (int s = 0; s < a.nseg; ++s)
            if (!a.seg[s].wb[0] || !a.seg[s].wb[1] || !a.seg[s].wb[2]) return hipErrorInvalidValue;
    (void)hipGetLastError();   // drop a stale error left by earlier runtime calls (not ours)
    switch (cfg) {
        case CFG_T128x128: return launch_t<128, 128, 2, 2, EPI_BIAS, 0>(a, prec, st);
        case CFG_T128x64: return launch_t<128, 64, 2, 2, EPI_BIAS, 0>(a, prec, st);
        case CFG_G272x64:
            if (a.V != 17) return hipErrorInvalidValue;
            return launch_t<272, 64, 1, 4, EPI_GRAPH, 17>(a, prec, st);
        case CFG_H64x128: return launch_t<64, 128, 2, 2, EPI_BIAS, 0>(a, prec, st);
        case CFG_T256x64: return launch_t<256, 64, 4, 1, EPI_BIAS, 0>(a, prec, st);
        case CFG_H64x64: return launch_t<64, 64, 2, 2, EPI_BIAS, 0>(a, prec, st);
        case CFG_S128x128: return launch_t<128, 128, 2, 2, EPI_SKIN, 0>(a, prec, st);
        default: return hipErrorInvalidValue;
    }
}

}  // namespace tik
