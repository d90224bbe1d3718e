// xgemm.hip — bf16x3 implicit GEMM on fp32 activations (see xgemm.h).
//
// Tile: 256 rows x BN columns, 8 waves (512 threads), one workgroup per CU.
// Wave w owns rows 32w..32w+31 (two 16-row fragments) and ALL BN columns, so
// each A element is read from LDS and split into bf16 planes exactly once per
// K step, in registers, by the wave that uses it (no split pass, no extra
// LDS); the weight planes are read by every wave.
//
// LDS, per stage: the A image (256 rows x 32 fp32 = 128 B per row) and the B
// image (3 planes x BN columns x 32 bf16 = 64 B per column). Both are written
// by LDS-DMA (buffer_load ... lds, 16 B per lane), NST stages deep, one
// barrier per K step.
//  * A row r, logical floats [8g+4h, 8g+4h+4) (g = k group of the MFMA
//    operand, h = half) at 16-B unit (g + 4h) ^ ((r >> 1) & 7): the two
//    ds_read_b128 of a fragment read are conflict-free in every lane group.
//    The DMA lane that fills unit p of row r fetches the logical unit
//    (p ^ swz(r)), so the swizzle costs nothing.
//  * B column n, k group g at unit g ^ ((-(n >> 2)) & 3) of its 64-B row:
//    conflict-free ds_read_b128 per plane; applied on the host (xgemm_pack).
// Rows past the batch, and taps outside the window (the temporal zero
// padding), DMA from an out-of-range offset of the buffer resource: zeros.
//
// Epilogues stage the fp32 C tile through LDS (half the columns at a time)
// and store whole 16-B row segments:
//  * EPI_BIAS: + bias[c] (+ identity residual row, or the layer-0 residual
//    conv on 4-float rows) -> activation -> out.
//  * EPI_GRAPH: tiles of 15 whole frames (255 rows); z[f][w] = sum_v A[v][w]
//    y[f][v] (the einsum of gconv_origin.py:61-63; COCO hop<=2 pattern
//    unrolled when A_eff fits it) + bias2[w][c], ReLU (st_gcn_aaai18.py:178-179).
#include <algorithm>

#include "cgemm.h"
#include "cgemm3_dev.h"
#include "common.h"
#include "xgemm.h"

namespace tik {

typedef __bf16 xbf16x8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ void xsplit8(const f32x4 lo, const f32x4 hi, xbf16x8& p0, xbf16x8& p1, xbf16x8& p2) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
        const float x = e < 4 ? lo[e] : hi[e - 4];
        const __bf16 b0 = (__bf16)x;
        const float r1 = x - (float)b0;
        const __bf16 b1 = (__bf16)r1;
        p0[e] = b0;
        p1[e] = b1;
        p2[e] = (__bf16)(r1 - (float)b1);
    }
}

__device__ __forceinline__ int xa_swz(int r) { return (r >> 1) & 7; }

// graph mix of one frame, output joints [W0, W1): z[w] = sum_v A[v][w] y[v] +
// bias2[w], ReLU, stored. w and v are compile-time, so the sparse COCO
// pattern unrolls and the A entries are wave-uniform scalar loads.
// A_eff entry i from the 5 VGPRs that hold it across the wave (lane i % 64 of amv[i / 64])
__device__ __forceinline__ float xam(const float (&amv)[5], int i) {
    return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, amv[i / 64]), i % 64));
}

template <int W0, int W1, bool SPARSE>
__device__ __forceinline__ void xmix_store(const f32x4 (&y)[17], const float (&amv)[5],
                                           const float* __restrict__ bias2, int Nc, int col, float* __restrict__ o,
                                           int ldo) {
#pragma unroll
    for (int w = W0; w < W1; ++w) {
        f32x4 z = *reinterpret_cast<const f32x4*>(bias2 + w * Nc + col);
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
        *reinterpret_cast<f32x4*>(o + (size_t)w * ldo) = z;
    }
}

template <int BN, int EPI>
struct XCfg {
    static constexpr int NW = 8, NT = 512, BM = 256, FM = 2, FN = BN / 16;
    static constexpr int ABYTES = BM * 128;
    static constexpr int PLANE = BN * 64;
    static constexpr int BBYTES = 3 * PLANE;
    static constexpr int STAGE = ABYTES + BBYTES;
    static constexpr int NST = BN >= 128 ? 2 : 3;
    static constexpr int NIA = ABYTES / 1024 / NW;   // A DMA instructions per wave per stage
    static constexpr int NIB_TOT = BBYTES / 1024;
    static constexpr int RT = EPI == EPI_GRAPH ? 255 : 256;   // valid rows per tile
    static constexpr int HB = BN / 2;                         // epilogue columns per pass
    static constexpr int LDC = HB + 4;
    static constexpr int LDCG = BN + 4;                       // EPI_GRAPH: the whole tile at once
    static constexpr int CT = EPI == EPI_GRAPH ? BM * LDCG * 4 : BM * LDC * 4;
    static constexpr int SMEM = NST * STAGE > CT ? NST * STAGE : CT;
    static_assert(NIA * 1024 * NW == ABYTES, "A DMA split");
    static_assert(SMEM <= 160 * 1024, "LDS");
};

template <int BN, int EPI>
__global__ __launch_bounds__(512, 1) void xgemm_kernel(XArgs a) {
    using C = XCfg<BN, EPI>;
    constexpr int NW = C::NW, NT = C::NT, FM = C::FM, FN = C::FN, NIA = C::NIA, NST = C::NST, RT = C::RT;
    __shared__ __attribute__((aligned(16))) unsigned char smem[C::SMEM];   // the only LDS object

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    int r0, ntile;
    {   // XCD-aware tile order: consecutive workgroup ids go to different XCDs,
        // so give each XCD a contiguous run of tiles (rows shared by neighbours stay in its L2)
        const int nwg = gridDim.x * gridDim.y, bid = blockIdx.y * gridDim.x + blockIdx.x;
        const int per = nwg >> 3, rem = nwg & 7, x = bid & 7, k = bid >> 3;
        const int swz = x < rem ? x * (per + 1) + k : rem * (per + 1) + (x - rem) * per + k;
        r0 = (swz / gridDim.y) * RT;
        ntile = swz % gridDim.y;
    }
    const int n0 = ntile * BN;
    const int V = a.V;

    // ---- A DMA roles: instruction j of this wave fills rows (wave*NIA + j)*8 + lane/8, unit lane&7
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
    // B DMA: the stage's B image is one contiguous packed block; instruction q (of NIB_TOT) copies 1 KB
    const i32x4 rB = buf_rsrc(a.wp, (unsigned)((size_t)gridDim.y * a.ksteps * C::BBYTES));
    const int nb_w = (C::NIB_TOT - wave + NW - 1) / NW;   // this wave's B instructions per stage
    const int nper = NIA + nb_w;

    struct Cur { int seg, tap, blk, k; };
    Cur cur{0, 0, 0, 0};
    unsigned a_off[NIA];
    i32x4 rA = buf_rsrc(a.seg[0].src, (unsigned)(a.seg[0].rows_in * a.seg[0].ld * 4));
    int cached_seg = -1, cached_tap = -1;
    auto prepare = [&]() {
        if (cur.seg == cached_seg && cur.tap == cached_tap) return;
        const XSeg sg = cur.seg == 0 ? a.seg[0] : a.seg[1];
        if (cur.seg != cached_seg) rA = buf_rsrc(sg.src, (unsigned)(sg.rows_in * sg.ld * 4));
#pragma unroll
        for (int j = 0; j < NIA; ++j) {
            const int t = sg.stride * a_t[j] + cur.tap - sg.pad;
            a_off[j] = (a_ok[j] && t >= 0 && t < sg.tin)
                           ? (unsigned)(((a_n[j] * sg.tin + t) * V + a_w[j]) * sg.ld * 4 + a_uo[j])
                           : DMA_OOB;
        }
        cached_seg = cur.seg; cached_tap = cur.tap;
    };
    auto issue = [&](int slot) {   // stage of the cursor, then advance it
        prepare();
        unsigned char* A = smem + slot * C::STAGE;
        const int soA = __builtin_amdgcn_readfirstlane(cur.blk * 128);
#pragma unroll
        for (int j = 0; j < NIA; ++j) dma16(rA, A + (wave * NIA + j) * 1024, a_off[j], soA);
        const int soB = __builtin_amdgcn_readfirstlane((ntile * a.ksteps + cur.k) * C::BBYTES);
        for (int q = wave; q < C::NIB_TOT; q += NW) dma16(rB, A + C::ABYTES + q * 1024, (unsigned)(q * 1024 + lane * 16), soB);
        const int nb = (cur.seg == 0 ? a.seg[0].cin : a.seg[1].cin) / 32;
        const int kt = cur.seg == 0 ? a.seg[0].kt : a.seg[1].kt;
        ++cur.k;
        if (++cur.blk >= nb) { cur.blk = 0; if (++cur.tap >= kt) { cur.tap = 0; ++cur.seg; } }
    };

    f32x4 acc[FM][FN];
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int g = lane >> 4;
    const int bsw = (-((lane & 15) >> 2)) & 3;
    const int boff = (lane & 15) * 64 + ((g ^ bsw) << 4);
    auto compute = [&](int slot) {
        const unsigned char* A = smem + slot * C::STAGE;
        const unsigned char* B = A + C::ABYTES;
        xbf16x8 a0[FM], a1[FM], a2[FM];
#pragma unroll
        for (int i = 0; i < FM; ++i) {
            const int r = wave * 32 + i * 16 + (lane & 15);
            const f32x4 lo = *reinterpret_cast<const f32x4*>(A + r * 128 + ((g ^ xa_swz(r)) << 4));
            const f32x4 hi = *reinterpret_cast<const f32x4*>(A + r * 128 + (((g + 4) ^ xa_swz(r)) << 4));
            xsplit8(lo, hi, a0[i], a1[i], a2[i]);
        }
#pragma unroll
        for (int j = 0; j < FN; ++j) {
            const xbf16x8 b0 = *reinterpret_cast<const xbf16x8*>(B + j * 16 * 64 + boff);
            const xbf16x8 b1 = *reinterpret_cast<const xbf16x8*>(B + C::PLANE + j * 16 * 64 + boff);
            const xbf16x8 b2 = *reinterpret_cast<const xbf16x8*>(B + 2 * C::PLANE + j * 16 * 64 + boff);
#pragma unroll
            for (int i = 0; i < FM; ++i) {
                acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a2[i], b0, acc[i][j], 0, 0, 0);
                acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1[i], b1, acc[i][j], 0, 0, 0);
                acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0[i], b2, acc[i][j], 0, 0, 0);
                acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1[i], b0, acc[i][j], 0, 0, 0);
                acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0[i], b1, acc[i][j], 0, 0, 0);
                acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0[i], b0, acc[i][j], 0, 0, 0);
            }
        }
    };

    const int K = a.ksteps;
#pragma unroll
    for (int s = 0; s < NST - 1; ++s)
        if (s < K) issue(s);
    for (int k = 0; k < K; ++k) {
        // in flight: stages k .. k+younger; retire stage k (vmcnt retires in issue order)
        const int younger = min(NST - 2, K - 1 - k);
        wait_vm_dyn(younger * nper);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();   // every wave's stage-k DMA landed; every wave done with stage k-1
        if (k + NST - 1 < K) issue((k + NST - 1) % NST);
        compute(k % NST);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");

    // ---- epilogue: C tile through LDS
    float* Cs = reinterpret_cast<float*>(smem);
    const int crow = wave * 32 + 4 * g;
    const int ccol = lane & 15;
    if constexpr (EPI == EPI_GRAPH) {
        __syncthreads();   // every wave done with the K loop's LDS
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
            for (int j = 0; j < FN; ++j)
#pragma unroll
                for (int e = 0; e < 4; ++e) Cs[(crow + i * 16 + e) * C::LDCG + j * 16 + ccol] = acc[i][j][e];
        // A_eff in 5 VGPRs across the wave, read back with v_readlane (global loads
        // would be re-issued after every store, which may alias them)
        float amv[5];
#pragma unroll
        for (int k = 0; k < 5; ++k) amv[k] = 64 * k + lane < 17 * 17 ? a.amix[64 * k + lane] : 0.f;
        __syncthreads();
        // waves 0-3 produce joints 0-8, waves 4-7 joints 9-16 (wave-uniform split,
        // so each half's joint loop is compile-time); item = (frame, 4 columns)
        constexpr int C4 = BN / 4;
        const int nframes = a.M / 17, f0 = r0 / 17;
        const bool second = wave >= NW / 2;
#pragma unroll 1
        for (int it = tid & (NT / 2 - 1); it < 15 * C4; it += NT / 2) {
            const int f = it / C4, c4 = it - f * C4;
            const int col = n0 + 4 * c4;
            if (f0 + f >= nframes || col >= a.Nc) continue;
            f32x4 y[17];
#pragma unroll
            for (int v = 0; v < 17; ++v) y[v] = *reinterpret_cast<const f32x4*>(Cs + (f * 17 + v) * C::LDCG + 4 * c4);
            float* o = a.out + (size_t)(f0 + f) * 17 * a.ldo + col;
            if (a.mix_sparse) {
                if (second) xmix_store<9, 17, true>(y, amv, a.bias, a.Nc, col, o, a.ldo);
                else xmix_store<0, 9, true>(y, amv, a.bias, a.Nc, col, o, a.ldo);
            } else {
                if (second) xmix_store<9, 17, false>(y, amv, a.bias, a.Nc, col, o, a.ldo);
                else xmix_store<0, 9, false>(y, amv, a.bias, a.Nc, col, o, a.ldo);
            }
        }
        return;
    }
    const float slope = a.act == ACT_RELU ? 0.f : (a.act == ACT_LEAKY ? 0.01f : 1.f);
#pragma unroll
    for (int half = 0; half < 2; ++half) {
        __syncthreads();   // K loop done (first pass) / previous pass's reads done
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
            for (int jj = 0; jj < FN / 2; ++jj)
#pragma unroll
                for (int e = 0; e < 4; ++e)
                    Cs[(crow + i * 16 + e) * C::LDC + jj * 16 + ccol] = acc[i][half * (FN / 2) + jj][e];
        __syncthreads();
        const int cbase = n0 + half * C::HB;
        {
            // KI items per thread, all global operands loaded before any store
            constexpr int C4 = C::HB / 4, KI = C::BM * C4 / NT;
            static_assert(KI * NT == C::BM * C4, "epilogue mapping");
            const int c4 = tid % C4, lr0 = tid / C4, col = cbase + 4 * c4;
            const bool colv = col + 3 < a.Nc;
            f32x4 bv = {0.f, 0.f, 0.f, 0.f};
            if (a.bias && colv) bv = *reinterpret_cast<const f32x4*>(a.bias + col);
            f32x4 rv[KI];
#pragma unroll
            for (int k = 0; k < KI; ++k) {
                const int row = min(r0 + lr0 + k * (NT / C4), a.M - 1);
                rv[k] = f32x4{0.f, 0.f, 0.f, 0.f};
                if (a.resid && colv) rv[k] = *reinterpret_cast<const f32x4*>(a.resid + (size_t)row * a.ldr + col);
                else if (a.rx) rv[k] = *reinterpret_cast<const f32x4*>(a.rx + (size_t)row * 4);
            }
            float rw[4][4] = {};
            if (a.rx && colv)
#pragma unroll
                for (int e = 0; e < 4; ++e)
#pragma unroll
                    for (int c = 0; c < 4; ++c) rw[e][c] = c < a.rxc ? a.rw[(col + e) * a.rxc + c] : 0.f;
#pragma unroll
            for (int k = 0; k < KI; ++k) {
                const int lr = lr0 + k * (NT / C4), row = r0 + lr;
                if (lr >= RT || row >= a.M || col >= a.Nc) continue;
                f32x4 v = *reinterpret_cast<const f32x4*>(Cs + lr * C::LDC + 4 * c4);
                if (colv) {
                    v += bv;
                    if (a.rx) {
#pragma unroll
                        for (int e = 0; e < 4; ++e)
                            v[e] += rv[k][0] * rw[e][0] + rv[k][1] * rw[e][1] + rv[k][2] * rw[e][2] + rv[k][3] * rw[e][3];
                    } else {
                        v += rv[k];
                    }
#pragma unroll
                    for (int e = 0; e < 4; ++e) v[e] = v[e] > 0.f ? v[e] : slope * v[e];
                    *reinterpret_cast<f32x4*>(a.out + (size_t)row * a.ldo + col) = v;
                } else {
                    for (int e = 0; e < 4 && col + e < a.Nc; ++e) {
                        float t = v[e] + (a.bias ? a.bias[col + e] : 0.f);
                        if (a.resid) t += a.resid[(size_t)row * a.ldr + col + e];
                        if (a.rx)
                            for (int c = 0; c < a.rxc; ++c) t = fmaf(a.rx[(size_t)row * 4 + c], a.rw[(col + e) * a.rxc + c], t);
                        t = t > 0.f ? t : slope * t;
                        a.out[(size_t)row * a.ldo + col + e] = t;
                    }
                }
            }
        }
    }
}

hipError_t launch_xgemm(const XArgs& a, int bn, int epi, hipStream_t st) {
    if (a.M <= 0 || a.Nc <= 0) return hipSuccess;
    if ((bn != 64 && bn != 128) || (epi != EPI_BIAS && epi != EPI_GRAPH) || !a.wp || !a.out || a.ldo % 4 ||
        a.nseg < 1 || a.nseg > 2 || a.ksteps != xgemm_ksteps(a) || a.ksteps <= 0)
        return hipErrorInvalidValue;
    for (int s = 0; s < a.nseg; ++s) {
        const XSeg& g = a.seg[s];
        if (!g.src || g.cin % 32 || g.ld % 4 || g.ld < g.cin || g.rows_in * g.ld * 4 >= (1LL << 31)) return hipErrorInvalidValue;
    }
    if (epi == EPI_GRAPH && (a.V != 17 || a.M % 17 || !a.amix || !a.bias)) return hipErrorInvalidValue;
    if (epi == EPI_BIAS && a.resid && a.ldr % 4) return hipErrorInvalidValue;
    if ((long long)a.M * a.ldo >= (1LL << 31) * 1LL * 4) return hipErrorInvalidValue;
    const int rt = epi == EPI_GRAPH ? 255 : 256;
    const dim3 grid((a.M + rt - 1) / rt, (a.Nc + bn - 1) / bn), blk(512);
    (void)hipGetLastError();
    if (bn == 128) {
        if (epi == EPI_BIAS) hipLaunchKernelGGL((xgemm_kernel<128, EPI_BIAS>), grid, blk, 0, st, a);
        else hipLaunchKernelGGL((xgemm_kernel<128, EPI_GRAPH>), grid, blk, 0, st, a);
    } else {
        if (epi == EPI_BIAS) hipLaunchKernelGGL((xgemm_kernel<64, EPI_BIAS>), grid, blk, 0, st, a);
        else hipLaunchKernelGGL((xgemm_kernel<64, EPI_GRAPH>), grid, blk, 0, st, a);
    }
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
            for (int tap = 0; tap < sg.kt; ++tap)
                for (int b = 0; b < nb; ++b, ++k) {
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
