// gpw.hip — weight-stationary persistent gcn (GP_*): the spatial half of an
// ST-GCN block that no fused kernel carries (L2 64->128 and L6 128->256 of
// the IK net):
//   z = ReLU( mix_A( x . Wg'^T ) + bias2' )        (1x1 conv + 17x17 graph mix)
//
// Why: the G3_272x128 kernel spends most of each workgroup's life waiting for
// its first DMA (one 154 KB workgroup per CU, so nothing overlaps the load of
// a tile: per workgroup L2 9.7 us loop for 2 K steps + 5.5 us epilogue,
// TIK_G_TRACE). Here one workgroup per CU walks a contiguous run of FT-frame
// tiles and the x image of tile i+1 is DMA'd (into the other of two buffers)
// at the START of tile i, so its HBM latency hides behind tile i's MFMAs and
// graph mix. The weights never move: each wave keeps its output channels'
// f16 hi/lo Wg' in registers (transposed MFMA: A = weights, B = pixel rows),
// so an accumulator lane holds 4 consecutive channels of one pixel and the
// fp32 y tile goes to LDS in 16-B pieces. The mix is the G3 epilogue's (bias2'
// first, then the joints in order, COCO 2-hop sparsity unrolled, A_eff read
// back from registers with v_readlane), one (frame, 4 channels, joint half)
// item per thread, written split into an LDS z image over the dead y tile and
// stored as whole 128-B lines (the direct 8-B hi / lo stores of G3 write each
// line in two halves).
//
// Every wave issues a fixed number of vector-memory instructions per tile
// (its x DMAs and NSP line stores; invalid pieces go to a trash line), so the
// one vmcnt wait per tile is exact.
#include <cstdlib>
#include <type_traits>

#include "cgemm3_dev.h"

namespace tik {

template <int CIN, int COUT, int FT, int NW, int NBUF>
struct GpwGeo {
    static constexpr int V = 17;
    static constexpr int RT = FT * V;                 // pixel rows of a tile
    static constexpr int NF = (RT + 15) / 16;         // 16-row MFMA fragments
    static constexpr int ROWS = NF * 16;
    static constexpr int NKB = CIN / 32;              // K blocks
    static constexpr int CF = COUT / (16 * NW);       // 16-channel A fragments per wave
    static constexpr int XB = ROWS * 128;             // one K block image
    static constexpr int XBUF = NKB * XB;             // one tile's x image
    static constexpr int NI = NKB * ROWS / 8;         // DMA instructions per tile (8 rows each)
    static constexpr int LDY = COUT + 4;
    static constexpr int YOFF = NBUF * XBUF;
    static constexpr int B2OFF = YOFF + RT * LDY * 4;
    static constexpr int SMEM = B2OFF + V * COUT * 4;
    static constexpr int NQ = COUT / 4;               // channel quads
    static constexpr int ZROW = COUT * 4 + 16;        // z image row (split-block row + 16 B pad) = Y row
    static constexpr int PPR = COUT / 4;              // 16-B pieces per split-block row (4 B per channel)
    static constexpr int NSP = (RT * PPR + 64 * NW - 1) / (64 * NW);   // line-store pieces per thread
    static_assert(ZROW == LDY * 4, "the z image reuses the Y region");
    static_assert(CIN % 32 == 0 && CF * 16 * NW == COUT && (NBUF == 1 || NBUF == 2), "shape");
    static_assert(SMEM <= 163840, "LDS");
    static_assert(FT * NQ <= 32 * NW, "mix items: one per thread of a joint half");
};

template <int CIN, int COUT, int FT, int NW, int NBUF>
__global__ __launch_bounds__(64 * NW, 8 / NW) void gpw_kernel(Cgemm3Args a, int ntiles) {
    using G = GpwGeo<CIN, COUT, FT, NW, NBUF>;
    constexpr int NT = 64 * NW;
    constexpr int V = 17;
    __shared__ __attribute__((aligned(16))) unsigned char smem[G::SMEM];   // the only LDS object
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int M = a.M;

    // ---- this workgroup's contiguous run of tiles (runs ordered per XCD, as tgw.hip)
    int t_begin, t_end;
    {
        const int Gn = gridDim.x, bid = blockIdx.x;
        const int per = Gn >> 3, rem = Gn & 7, x = bid & 7, k = bid >> 3;
        const int s = x < rem ? x * (per + 1) + k : rem * (per + 1) + (x - rem) * per + k;
        t_begin = (int)((long long)s * ntiles / Gn);
        t_end = (int)((long long)(s + 1) * ntiles / Gn);
    }

    // ---- stationary operands: this wave's CF x 16 output channels
    const int g0 = lane >> 4;
    f16x8 wgh[G::CF][G::NKB], wgl[G::CF][G::NKB];
#pragma unroll
    for (int cf = 0; cf < G::CF; ++cf) {
        const int co = (wave * G::CF + cf) * 16 + (lane & 15);
#pragma unroll
        for (int kb = 0; kb < G::NKB; ++kb) {
            const unsigned short* p = a.seg[0].w + (size_t)co * a.seg[0].ldw + kb * 64 + 8 * g0;
            wgh[cf][kb] = *reinterpret_cast<const f16x8*>(p);
            wgl[cf][kb] = *reinterpret_cast<const f16x8*>(p + 32);
        }
    }
    constexpr int NAM = (V * V + 63) / 64;   // A_eff' in registers, read back with v_readlane
    float amv[NAM];
#pragma unroll
    for (int k = 0; k < NAM; ++k) amv[k] = 64 * k + lane < V * V ? a.amix[64 * k + lane] : 0.f;
    float* b2s = reinterpret_cast<float*>(smem + G::B2OFF);
    for (int i = tid; i < V * COUT; i += NT) b2s[i] = a.bias[i];
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
    for (int cf = 0; cf < G::CF; ++cf)
#pragma unroll
        for (int kb = 0; kb < G::NKB; ++kb) asm volatile("" : "+v"(wgh[cf][kb]), "+v"(wgl[cf][kb]));
#pragma unroll
    for (int k = 0; k < NAM; ++k) asm volatile("" : "+v"(amv[k]));
    lds_barrier();

    // ---- x DMA: instruction j = wave + NW m covers K block j / (ROWS / 8), rows 8 (j % (ROWS / 8)) ..
    constexpr int NIW = (G::NI + NW - 1) / NW;            // per wave (max)
    const int my_ni = (G::NI - wave + NW - 1) / NW;       // this wave's count (wave-uniform)
    const int ld = a.seg[0].ld;
    const i32x4 rX = buf_rsrc(a.seg[0].src, (unsigned)((long long)M * ld * 2));
    auto issue_x = [&](int tile, int buf) {
#pragma unroll
        for (int m = 0; m < NIW; ++m) {
            const int j = wave + NW * m;
            if (j < G::NI) {
                const int kb = j / (G::ROWS / 8), rg = j % (G::ROWS / 8);
                const int r = 8 * rg + (lane >> 3);
                const int R = tile * G::RT + r;
                const int ck = (lane & 7) ^ sbf(r);
                const unsigned off = (r < G::RT && R < M) ? (unsigned)(((long long)R * ld + kb * 64 + 8 * ck) * 2) : DMA_OOB;
                dma16(rX, smem + buf * G::XBUF + kb * G::XB + rg * 1024, off, 0);
            }
        }
    };

    // mix roles: joint half h (wave-uniform), item (frame f, channel quad q)
    const int h = wave & 1;
    constexpr int nst = G::NSP;   // stores per thread per tile (whole-line pieces)

    if (t_begin < t_end) issue_x(t_begin, 0);
    int prev_st = 0;
    // debug (a.trace): per-workgroup phase sums in s_memrealtime ticks
    unsigned long long tr_w = 0, tr_m = 0, tr_y = 0, tr_x = 0, tr_i = 0, tr_v = 0;
    for (int tile = t_begin; tile < t_end; ++tile) {
        const unsigned long long ts0 = a.trace ? __builtin_amdgcn_s_memrealtime() : 0;
        const int buf = NBUF == 2 ? (tile - t_begin) & 1 : 0;
        const bool nxt = tile + 1 < t_end;
        // NBUF 2: tile+1's image streams in during this whole tile (the other buffer
        // was last read by tile-1's MFMAs, which every wave finished before tile-1's mix)
        if (NBUF == 2 && nxt) issue_x(tile + 1, buf ^ 1);
        const unsigned long long tsa = a.trace ? __builtin_amdgcn_s_memrealtime() : 0;
        // this tile's image landed: younger are only tile+1's DMAs (NBUF 2) and tile-1's stores
        wait_vm_dyn((NBUF == 2 && nxt ? my_ni : 0) + prev_st);
        const unsigned long long tsb = a.trace ? __builtin_amdgcn_s_memrealtime() : 0;
        lds_barrier();
        const unsigned long long ts1 = a.trace ? __builtin_amdgcn_s_memrealtime() : 0;
        int lt = lane;   // opaque per tile: lane-derived addresses stay out of the loop-carried state
        asm volatile("" : "+v"(lt));
        const int l15 = lt & 15, g = lt >> 4;

        f32x4 acc[G::CF][G::NF];
#pragma unroll
        for (int cf = 0; cf < G::CF; ++cf)
#pragma unroll
            for (int i = 0; i < G::NF; ++i) acc[cf][i] = f32x4{0.f, 0.f, 0.f, 0.f};
        const unsigned char* X = smem + buf * G::XBUF;
#pragma unroll
        for (int kb = 0; kb < G::NKB; ++kb) {
#pragma unroll
            for (int i = 0; i < G::NF; ++i) {
                const int r = 16 * i + l15;
                const f16x8 bh = *reinterpret_cast<const f16x8*>(X + kb * G::XB + sbo(r, g));
                const f16x8 bl = *reinterpret_cast<const f16x8*>(X + kb * G::XB + sbo(r, 4 + g));
#pragma unroll
                for (int cf = 0; cf < G::CF; ++cf) {
                    acc[cf][i] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wgh[cf][kb], bl, acc[cf][i], 0, 0, 0);
                    acc[cf][i] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wgl[cf][kb], bh, acc[cf][i], 0, 0, 0);
                    acc[cf][i] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wgh[cf][kb], bh, acc[cf][i], 0, 0, 0);
                }
            }
        }
        const unsigned long long ts2 = a.trace ? __builtin_amdgcn_s_memrealtime() : 0;
        // y -> LDS [pixel][channel] fp32 (every wave is past the previous tile's mix reads:
        // the barrier above)
        float* Y = reinterpret_cast<float*>(smem + G::YOFF);
#pragma unroll
        for (int cf = 0; cf < G::CF; ++cf) {
            const int c0 = (wave * G::CF + cf) * 16 + 4 * g;
#pragma unroll
            for (int i = 0; i < G::NF; ++i) {
                const int p = 16 * i + l15;
                if (p < G::RT) *reinterpret_cast<f32x4*>(Y + p * G::LDY + c0) = acc[cf][i];
            }
        }
        lds_barrier();
        // NBUF 1: every wave is past its MFMA reads of the image: tile+1's streams in
        // during this tile's mix (and the other workgroup on the CU)
        if (NBUF == 1 && nxt) issue_x(tile + 1, 0);
        const unsigned long long ts3 = a.trace ? __builtin_amdgcn_s_memrealtime() : 0;

        // ---- graph mix + bias2' + ReLU -> split-block z rows
#pragma unroll
        for (int k = 0; k < NAM; ++k) asm volatile("" : "+v"(amv[k]));
        {
            const int it = (wave >> 1) * 64 + lt;   // 0 .. 32 NW - 1
            const int f = it / G::NQ, q = it % G::NQ;
            const bool fok = f < FT;
            const int fr = fok ? f : FT - 1;
            f32x4 y[V];
#pragma unroll
            for (int v = 0; v < V; ++v) y[v] = *reinterpret_cast<const f32x4*>(Y + (fr * V + v) * G::LDY + 4 * q);
            lds_barrier();   // every y read done: the z image goes over Y
            const int col = 4 * q;
            // z image: pixel rows of ZROW bytes = the split-block row (COUT/32 blocks of
            // [hi x32 | lo x32]) + 16 B of padding against bank conflicts
            unsigned char* zrow = smem + G::YOFF + (size_t)(fr * V) * G::ZROW + (col >> 5) * 128 + (col & 31) * 2;
            auto mixr = [&](auto w0c, auto w1c, auto sp) {
                constexpr int W0 = decltype(w0c)::value, W1 = decltype(w1c)::value;
                constexpr bool SP = decltype(sp)::value;
#pragma unroll
                for (int w = W0; w < W1; ++w) {
                    f32x4 z = *reinterpret_cast<const f32x4*>(b2s + w * COUT + col);
#pragma unroll
                    for (int v = 0; v < V; ++v)
                        if (!SP || ((coco_hop2_mask3(w) >> v) & 1u)) {
                            const float av = __builtin_bit_cast(
                                float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, amv[(v * V + w) / 64]), (v * V + w) % 64));
                            z += av * y[v];
                        }
#pragma unroll
                    for (int e = 0; e < 4; ++e) z[e] = z[e] > 0.f ? z[e] : 0.f;
                    f16x4 zh, zl;
                    split4(z, zh, zl);
                    if (fok) {   // rows of frames past the tile: not written
                        *reinterpret_cast<f16x4*>(zrow + w * G::ZROW) = zh;
                        *reinterpret_cast<f16x4*>(zrow + w * G::ZROW + 64) = zl;
                    }
                }
            };
            using I0 = std::integral_constant<int, 0>;
            using I9 = std::integral_constant<int, 9>;
            using I17 = std::integral_constant<int, 17>;
            if (h) {
                if (a.mix_sparse) mixr(I9{}, I17{}, std::true_type{});
                else mixr(I9{}, I17{}, std::false_type{});
            } else {
                if (a.mix_sparse) mixr(I0{}, I9{}, std::true_type{});
                else mixr(I0{}, I9{}, std::false_type{});
            }
            lds_barrier();
            // z -> HBM in whole 128-B lines: NSP 16-B pieces per thread (a wave writes
            // 64 consecutive pieces); pieces past the tile or the batch go to the trash line
            unsigned short* trash = a.trash + (((wave << 6) + lt) & 255) * 8;
#pragma unroll
            for (int j = 0; j < G::NSP; ++j) {
                const int pc = tid + NT * j;
                const int r = pc / G::PPR, u = pc % G::PPR;
                const bool ok = r < G::RT && (size_t)tile * G::RT + r < (size_t)M;
                const int rr = ok ? r : 0;
                const f32x4 d = *reinterpret_cast<const f32x4*>(smem + G::YOFF + (size_t)rr * G::ZROW + u * 16);
                unsigned short* o = ok ? a.out_h + ((size_t)tile * G::RT + r) * a.ldo + u * 8 : trash;
                *reinterpret_cast<f32x4*>(o) = d;
            }
        }
        prev_st = nst;
        if (a.trace) {
            const unsigned long long ts4 = __builtin_amdgcn_s_memrealtime();
            tr_w += ts1 - ts0; tr_m += ts2 - ts1; tr_y += ts3 - ts2; tr_x += ts4 - ts3; tr_i += tsa - ts0; tr_v += tsb - tsa;
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (a.trace && tid == 0) {   // {tiles, wait+barrier, MFMA, y staging, mix + stores}
        unsigned long long* t = a.trace + 8 * (size_t)blockIdx.x;
        t[0] = (unsigned long long)(t_end - t_begin);
        t[1] = tr_w; t[2] = tr_m; t[3] = tr_y; t[4] = tr_x; t[5] = tr_i; t[6] = tr_v;
    }
}

template <int CIN, int COUT, int FT, int NW, int NBUF>
static hipError_t launch_gpw_t(const Cgemm3Args& a, hipStream_t st) {
    const int ntiles = (a.M / 17 + FT - 1) / FT;
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    const int slots = cus * (8 / NW);   // resident workgroups
    const int grid = ntiles < slots ? ntiles : slots;
    (void)hipGetLastError();
    hipLaunchKernelGGL((gpw_kernel<CIN, COUT, FT, NW, NBUF>), dim3(grid), dim3(64 * NW), 0, st, a, ntiles);
    return hipGetLastError();
}

bool gpw_ok(const Cgemm3Args& a) {
    const int cin = a.seg[0].nblk * 32;
    // 256 -> 256 (L7) stays on G3: its 2-frame tiles measured slower (0.117 vs 0.101 ms)
    const bool shape = (cin == 64 && a.Nc == 128) || (cin == 128 && a.Nc == 256);
    return shape && a.V == 17 && a.M % 17 == 0 && a.nseg == 1 && a.seg[0].kt == 1 && a.seg[0].stride == 1 &&
           a.seg[0].pad == 0 && a.seg[0].ldw == a.seg[0].nblk * 64 && a.bias && a.amix && a.out_h && a.trash &&
           a.act == ACT_RELU && a.seg[0].ld % 8 == 0 && a.seg[0].ld >= 64 * a.seg[0].nblk && a.ldo % 8 == 0 &&
           a.ldo >= 64 * (a.Nc / 32) && (long long)a.M * a.seg[0].ld * 2 < (1LL << 31);
}

hipError_t launch_gpw(const Cgemm3Args& a, hipStream_t st) {
    if (a.M <= 0) return hipSuccess;
    if (!gpw_ok(a)) return hipErrorInvalidValue;
    const int cin = a.seg[0].nblk * 32;
    static const int var = getenv("TIK_GPW_VAR") ? atoi(getenv("TIK_GPW_VAR")) : 1;   // tuning hook
    if (cin == 64) return var ? launch_gpw_t<64, 128, 4, 4, 1>(a, st) : launch_gpw_t<64, 128, 8, 8, 2>(a, st);
    return launch_gpw_t<128, 256, 3, 8, 2>(a, st);
}

}  // namespace tik
