// xtws.hip — tcn conv (3 x 1 over frames, stride 1, 128 -> 128 channels) +
// folded BN + identity residual + ReLU of an ST-GCN block
// (st_gcn_aaai18.py:180-189), bf16x3 on MFMA, as one persistent,
// weight-stationary launch that splits every activation ONCE for all 3 taps.
//
// The tiled kernel (XT128) DMAs and splits the conv input three times (once per
// tap) and re-reads a 24 KB weight stage from L2 for every K step of every
// tile. Here (the xgraph.hip pattern applied to the temporal conv):
//   * weights in registers: wave w owns output channels 16w .. 16w + 15, all 3
//     taps x 128 input channels (144 VGPRs of bf16 planes, loaded once);
//   * tile = 8 consecutive frames of one window x 17 joints; per 32-channel K
//     block the 10-frame HALO (frames f0 - 1 .. f0 + 8, zeros outside the
//     window) is loaded into registers D blocks ahead and split once,
//     cooperatively, into a double-buffered LDS image of bf16 planes, one
//     barrier per K block; the three taps read it at frame offsets 0, 1, 2 —
//     each z element is loaded and split once per tile instead of three times;
//   * MFMA transposed (A = weights): pixel block j = joints (2j, 2j + 1) x the
//     tile's 8 frames (9 blocks; the 9th block's second joint is dead), each
//     lane ends with one pixel and 4 channels, so the epilogue runs on the
//     accumulators: (acc + x) + bias, ReLU, 16-B stores;
//   * the identity rows (this wave's 16 channels of the tile's 136 pixels) are
//     LDS-DMA'd into a per-wave slot at the start of the tile; the epilogue
//     writes its outputs over them and all waves then store whole 512-B rows;
//   * the next K block's split runs one 16-B unit at a time between the MFMA
//     items (the waves leave each barrier together).
// Measured (L3/L4, 1024 x 64 windows, same box): 0.265 ms vs 0.281-0.291 for
// XT128; components (-DTIK_XTUNE, before the row staging and the priority): no
// MFMAs 0.210, MFMAs + operand reads only 0.193 (the MFMA roof is 0.138).
// The default for L3/L4 (TIK_XTWS=0 restores XT128).
// Image row R = 10 jj + h (joint jj, halo frame h), 192 B: 3 planes x 4 units
// of 16 B (8 channels); unit u of joint jj at u ^ 2 (jj & 1): with the 48-dword
// row pitch, the ds_read_b128 of one (block, tap, plane) is conflict-free in
// every lane group (lanes of the two joints and the two frame halves land on
// distinct 4-bank slots).
// Products as xgemm (bf16x3, six products per K block), fp32 accumulation in
// the order (K block, tap), XT128's K order: the two are bitwise equal.
// FG (xtws_kernel<.., true>, round 6, the default for L3/L4): each tile's output
// rows, still in the slots, also go through block l + 1's gcn 1x1 conv + graph
// mix + BN + ReLU (XTWG; see "FG:" below and DESIGN.md §2a), bit for bit what
// launch_xgraph makes from `out`.
#include <algorithm>
#include <type_traits>

#include "xgemm_dev.h"
#include "xtws.h"

namespace tik {

namespace xw {
constexpr int V = 17, F = 8, H = F + 2;       // output frames per tile, halo frames
constexpr int ROWS = H * V;                   // 170 live image rows
constexpr int NU = ROWS * 8;                  // 16-B fp32 units of one K block (1360)
constexpr int PROWB = 192;                    // 3 planes x 32 channels x 2 B
constexpr int IMG = (ROWS + H) * PROWB;       // + the dead joint 17's rows (read by block 8, never written): 34,560
constexpr int NB = 9;                         // pixel blocks per tile
constexpr int NKB = 4;                        // 32-channel K blocks
constexpr int SLOTS = NB * 16 * 512;          // identity / output staging: 144 pixels x 128 channels (73,728)
// NW waves, each 16 CB = 128 / NW output channels; per-wave slot 144 x 64 CB B (+ 64: slots 16 banks apart)
// FG (the fused next-block gcn): + bias2 [17][128] of block l + 1 staged in LDS
template <int NW, bool FG>
struct Cfg {
    static constexpr int CB = 8 / NW, NT = 64 * NW, NLD = (NU + NT - 1) / NT;
    static constexpr int IDW = SLOTS / NW + 64;
    static constexpr int B2 = FG ? V * 128 * 4 + 320 * 4 : 0;   // + A_eff [17][17] (padded to 320)
    static constexpr int SMEM = 2 * IMG + NW * IDW + B2;
    static constexpr int NGU = F * V * 8;                 // the gcn split's 16-B fp32 units per K block (1088)
    static constexpr int NLG = (NGU + NT - 1) / NT;       // ... per thread (3, the last partial)
    static_assert(SMEM <= 160 * 1024, "LDS");
};
}  // namespace xw

__device__ __forceinline__ int xw_unit(int jj, int h, int p, int u) {
    return (10 * jj + h) * xw::PROWB + ((p * 4 + (u ^ ((jj & 1) << 1))) << 4);
}

__device__ f32x4 tik_llvm_raw_buffer_load_v4f32_xw(i32x4 rsrc, int voffset, int soffset, int aux)
    __asm("llvm.amdgcn.raw.buffer.load.v4f32");

typedef __bf16 xwbf16x4 __attribute__((ext_vector_type(4)));

#ifndef XW_D
#define XW_D 1     // K blocks of register prefetch
#endif
#ifndef XW_SPLIT_AT
#define XW_SPLIT_AT 0   // split unit i after item: 0 = (2 i + 1) NI / (2 NLD) (midpoints), 1 = i NI / NLD + 1
#endif

#ifndef XW_EPIBAR
#define XW_EPIBAR 1   // no barrier at a tile's first K block (the epilogue's serves), identity DMA at K block 1 (0: both at K block 0; 0.5 % slower)
#endif

#ifndef XW_XPF
#define XW_XPF 1   // operand read-ahead (items; 2 spills at 8 waves)
#endif

#ifndef XW_MIXW
#define XW_MIXW 7   // FG mix: waves 0-3 make joints 0 .. XW_MIXW - 1, waves 4-7 the rest (7: 55 vs 52 hop<=2 terms)
#endif

#ifdef TIK_XTUNE
#define XW_OFF(bit) (a.tune & (bit))
#else
#define XW_OFF(bit) false
#endif

template <int D, int NW, bool FG>
__global__ __launch_bounds__(64 * NW, 1) void xtws_kernel(XTConvArgs a) {
    using namespace xw;
    using C = Cfg<NW, FG>;
    constexpr int CB = C::CB, NT = C::NT, NLD = C::NLD, IDW = C::IDW;
    constexpr int NHD = (NU + NT - 1) / NT;   // FG: halo DMA instructions per wave
    // the two planes images and the rest (slots, FG's bias2 + A_eff) as separate LDS objects:
    // the compiler then knows an LDS-DMA into one image cannot alias reads of the other or of
    // the slots, and adds no vmcnt(0) before them
    __shared__ __attribute__((aligned(16))) unsigned char img0[IMG], img1[IMG], sl[C::SMEM - 2 * IMG];
    auto pimg = [&](int kb) __attribute__((always_inline)) { return (kb & 1) ? img1 : img0; };

    int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    unsigned char* const idw = sl + wave * IDW;
    const int T = a.T, tpw = T / F;
    const int ntiles = a.M / (V * T) * tpw;
    int t_begin, t_end;
    {   // persistent: a contiguous run of tiles per workgroup, runs ordered per XCD
        const int nwg = gridDim.x, bid = blockIdx.x;
        const int per = nwg >> 3, rem = nwg & 7, x = bid & 7, k = bid >> 3;
        const int s = x < rem ? x * (per + 1) + k : rem * (per + 1) + (x - rem) * per + k;
        t_begin = (int)((long long)s * ntiles / nwg);
        t_end = (int)((long long)(s + 1) * ntiles / nwg);
    }
    if (t_begin >= t_end) return;
    const int total = (t_end - t_begin) * NKB;
    // first output row of tile t (window w, frames f0 .. f0 + 7) and its first frame
    auto tile_geo = [&](int t, int& row0, int& f0) __attribute__((always_inline)) {
        const int w = t / tpw;
        f0 = (t - w * tpw) * F;
        row0 = (w * T + f0) * V;
    };

#ifdef TIK_XTRACE
    const bool tr = FG && a.trace != nullptr && (wave == 0 || wave == 4);
#else
    constexpr bool tr = false;
#endif
    // FG phases: 0 T K blocks, 1 T epilogue + out stores, 2 gcn split 0, 3-6 gcn K blocks, 7 y + mix
    unsigned long long ph_[8] = {0, 0, 0, 0, 0, 0, 0, 0}, tlast = 0;
    auto stamp = [&](int i) __attribute__((always_inline)) {
        if (tr) {
            const unsigned long long t = __builtin_amdgcn_s_memtime();
            if (i >= 0) ph_[i] += t - tlast;
            tlast = t;
        }
    };
    const i32x4 rZ = buf_rsrc(a.z, (unsigned)((long long)a.M * a.ldz * 4));
    const i32x4 rXI = buf_rsrc(a.x, (unsigned)((long long)a.M * a.ldx * 4));
    // ---- the halo rows of global step s (tile t_begin + s / 4, K block s % 4) into registers.
    // Unit U = NT i + tid: halo row m = U / 8 (frame f0 - 1 + m / 17, joint m % 17), channels 4 (U % 8) ..
    // Every lane issues NLD loads per step (out-of-range offsets read zeros): no branch, exact vmcnt
    f32x4 rb[D][NLD];
    auto load_unit = [&](int s, f32x4 (&r)[NLD], int i) __attribute__((always_inline)) {
        const int t = t_begin + s / NKB, kb = s - (s / NKB) * NKB;
        int row0, f0;
        tile_geo(t, row0, f0);
        const bool live = s < total;
        const int U = NT * i + tid, m = U >> 3, u = U & 7;
        const int fh = f0 - 1 + m / V;
        const bool ok = live && U < NU && fh >= 0 && fh < T && !XW_OFF(1);
        const unsigned off = ok ? (unsigned)((long long)(row0 - V + m) * a.ldz * 4 + kb * 128 + u * 16) : DMA_OOB;
        r[i] = tik_llvm_raw_buffer_load_v4f32_xw(rZ, (int)off, 0, 0);
    };
    auto load = [&](int s, f32x4 (&r)[NLD]) __attribute__((always_inline)) {
#pragma unroll
        for (int i = 0; i < NLD; ++i) load_unit(s, r, i);
    };
    // ---- split registers r (step s) into planes image (s & 1)
    // halo unit U (row m = U / 8: frame m / 17, joint m % 17; channels 4 (U % 8) ..) of x -> planes image P
    auto split_store = [&](unsigned char* P, int U, const f32x4 x) __attribute__((always_inline)) {
        const int m = U >> 3, u = U & 7;
        const int h = m / V, jj = m - h * V;
        xwbf16x4 p0, p1, p2;
#pragma unroll
        for (int e = 0; e < 4; ++e) {   // xsplit8's arithmetic, 4 channels
            const __bf16 b0 = (__bf16)x[e];
            const float r1 = x[e] - (float)b0;
            const __bf16 b1 = (__bf16)r1;
            p0[e] = b0;
            p1[e] = b1;
            p2[e] = (__bf16)(r1 - (float)b1);
        }
        const int hb = (u & 1) * 8;
        *reinterpret_cast<xwbf16x4*>(P + xw_unit(jj, h, 0, u >> 1) + hb) = p0;
        *reinterpret_cast<xwbf16x4*>(P + xw_unit(jj, h, 1, u >> 1) + hb) = p1;
        *reinterpret_cast<xwbf16x4*>(P + xw_unit(jj, h, 2, u >> 1) + hb) = p2;
    };
    auto split_unit = [&](int kb, const f32x4 (&r)[NLD], int i) __attribute__((always_inline)) {
        const int U = NT * i + tid;
        if (i + 1 < NLD || U < NU) split_store(pimg(kb), U, r[i]);
    };
    // FG: the halo rows of global step s as raw fp32 units (unit U at byte 16 U) into LDS at dst
    // by LDS-DMA: instruction k of wave w fills units 64 (NW k + w) + lane (every wave issues
    // the same count: out-of-range units read zeros into the dead tail)
    // (by inline asm: the compiler does not track these LDS writes, so it adds no vmcnt wait
    // before later accesses of dst, nor counts them; the caller waits with wait_vm)
    auto dma_halo = [&](int s, unsigned char* dst) __attribute__((always_inline)) {
        const int t = t_begin + s / NKB, kb = s - (s / NKB) * NKB;
        int row0, f0;
        tile_geo(t, row0, f0);
        const bool live = s < total;
#pragma unroll
        for (int k = 0; k < NHD; ++k) {
            const int U = 64 * (NW * k + wave) + lane, m = U >> 3, u = U & 7;
            const int fh = f0 - 1 + m / V;
            const bool ok = live && U < NU && fh >= 0 && fh < T;
            dma16_asm(rZ, dst + 1024 * (NW * k + wave), ok ? (unsigned)((long long)(row0 - V + m) * a.ldz * 4 + kb * 128 + u * 16) : DMA_OOB);
        }
    };
    auto split = [&](int s, const f32x4 (&r)[NLD]) __attribute__((always_inline)) {
#pragma unroll
        for (int i = 0; i < NLD; ++i) split_unit(s, r, i);
    };
    // ---- identity rows of tile t (this wave's 16 CB channels) into the wave's LDS slot,
    // pixel-major (64 CB B per pixel): instruction k covers pixels 16 k / CB .. (1 KB each)
    constexpr int PPI = 16 / CB;   // pixels per DMA instruction
    auto dma_ident = [&](int t) __attribute__((always_inline)) {
        int row0, f0;
        tile_geo(t, row0, f0);
        const bool live = t < t_end;
        const int pl = lane / (4 * CB), c = lane - pl * (4 * CB);
#pragma unroll
        for (int k = 0; k < NB * CB; ++k) {
            const int pix = k * PPI + pl, j = pix >> 4, pp = pix & 15;
            const int jj = 2 * j + (pp >> 3), fi = pp & 7;
            const bool ok = live && jj < V && !XW_OFF(1);
            const unsigned off = ok ? (unsigned)((long long)(row0 + fi * V + jj) * a.ldx * 4 + (16 * CB * wave + 4 * c) * 4) : DMA_OOB;
            dma16(rXI, idw + k * 1024, off, 0);
        }
    };

    // weights: [cg][tap * 4 + kb][plane][lane][8] (xblock_pack_weights), this wave's cg = CB wave + cb
    xbf16x8 w[3 * NKB][CB][3];
#pragma unroll
    for (int k = 0; k < 3 * NKB; ++k)
#pragma unroll
        for (int cb = 0; cb < CB; ++cb)
#pragma unroll
            for (int p = 0; p < 3; ++p)
                w[k][cb][p] = *reinterpret_cast<const xbf16x8*>(a.wp + ((((size_t)(CB * wave + cb) * 3 * NKB + k) * 3 + p) * 64 + lane) * 8);
    const int g = lane >> 4, px = lane & 15;
    f32x4 bv[CB];
#pragma unroll
    for (int cb = 0; cb < CB; ++cb) bv[cb] = *reinterpret_cast<const f32x4*>(a.bias + 16 * (CB * wave + cb) + 4 * g);
    // FG: block l + 1's bias2 [17][128] and A_eff in LDS (read by the mix, after many barriers)
    float* const b2s = reinterpret_cast<float*>(sl + NW * IDW);
    if constexpr (FG)
        for (int i = tid; i < V * 128 + 320; i += NT) b2s[i] = i < V * 128 ? a.bias2[i] : (i - V * 128 < V * V ? a.amix[i - V * 128] : 0.f);

    // prologue: step 0 -> planes[0]; steps 1 .. D into registers
    load(0, rb[0]);
    split(0, rb[0]);
#pragma unroll
    for (int d = 1; d <= D; ++d) load(d, rb[d % D]);

    f32x4 acc[NB][CB];
#pragma unroll
    for (int j = 0; j < NB; ++j)
#pragma unroll
        for (int cb = 0; cb < CB; ++cb) acc[j][cb] = f32x4{0.f, 0.f, 0.f, 0.f};

    // ---- FG: block l + 1's gcn (1x1 conv 128 -> 128 + graph mix + bias2 + ReLU,
    // st_gcn_aaai18.py:211, gconv_origin.py:56-65) on the tile's output rows, which the
    // epilogue left in the slots (fp32, this wave's 16 channels per slot, pixel-major).
    // Per 32-channel K block kb the rows are split once, cooperatively, into planes
    // image kb & 1 at the rows of halo frame f + 1 (where the T phase's tap 1 reads
    // them: the same operand reads), this wave's 16 output channels take 9 items x 6
    // products (weights from L2, two K blocks ahead), and the next K block's split runs
    // beside them. y then goes through the slots, and the mix runs per (frame, 4
    // channels) over compile-time joint halves. Products, K order and mix order are
    // xgraph.hip's: zout equals launch_xgraph's output from `out` bit for bit.
    xbf16x8 wga[3];
    auto load_wg = [&](int kb, xbf16x8 (&d)[3]) __attribute__((always_inline)) {
        // the base through an opaque register: loop-invariant loads would be hoisted out of
        // the tile loop and their 48 registers held across the T phase
        const unsigned short* wgp = a.wg;
        asm volatile("" : "+s"(wgp));
        if constexpr (FG)
#pragma unroll
            for (int p = 0; p < 3; ++p) {
                const auto* q = (const __attribute__((address_space(1))) xbf16x8*)(wgp + ((((size_t)wave * NKB + kb) * 3 + p) * 64 + lane) * 8);
                if (kb == NKB - 1)
                    // K block 3's planes by inline asm, waited for explicitly (wait_wg3) with the
                    // halo DMA issued after them still in flight; the compiler, not seeing that
                    // DMA, would wait with vmcnt(0)
                    asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(d[p]) : "v"(q) : "memory");
                else
                    // a global (not flat) load: a pending flat load makes every later vmcnt wait a vmcnt(0)
                    d[p] = *q;
            }
    };
    auto gsplit_unit = [&](int kb, int i) __attribute__((always_inline)) {
        const int U = NT * i + tid;
        if ((i + 1 < C::NLG || U < C::NGU) && !XW_OFF(32)) {
            const int m = U >> 3, u = U & 7;
            const int f = m / V, jj = m - f * V;
            const int pix = 16 * (jj >> 1) + 8 * (jj & 1) + f;
            const f32x4 x = *reinterpret_cast<const f32x4*>(sl + (2 * kb + (u >> 2)) * IDW + pix * 64 + (u & 3) * 16);
            xwbf16x4 p0, p1, p2;
#pragma unroll
            for (int e = 0; e < 4; ++e) {   // xsplit8's arithmetic, 4 channels
                const __bf16 b0 = (__bf16)x[e];
                const float r1 = x[e] - (float)b0;
                const __bf16 b1 = (__bf16)r1;
                p0[e] = b0;
                p1[e] = b1;
                p2[e] = (__bf16)(r1 - (float)b1);
            }
            unsigned char* P = pimg(kb);
            const int hb = (u & 1) * 8;
            *reinterpret_cast<xwbf16x4*>(P + xw_unit(jj, f + 1, 0, u >> 1) + hb) = p0;
            *reinterpret_cast<xwbf16x4*>(P + xw_unit(jj, f + 1, 1, u >> 1) + hb) = p1;
            *reinterpret_cast<xwbf16x4*>(P + xw_unit(jj, f + 1, 2, u >> 1) + hb) = p2;
        }
    };
    // K block kb's MFMAs (image kb & 1, weights wk); beside(j) runs after item j
    auto gmma = [&](int kb, const xbf16x8 (&wk)[3], auto&& beside) __attribute__((always_inline)) {
        asm volatile("" : "+v"(tid), "+v"(lane));
        const int g = lane >> 4, px = lane & 15, jb = px >> 3, fb = px & 7;
        const unsigned char* P = pimg(kb);
        constexpr int XPF = XW_XPF;
        xbf16x8 xr[XPF + 1][3];
        auto rd = [&](int j, xbf16x8 (&d)[3]) __attribute__((always_inline)) {
#pragma unroll
            for (int p = 0; p < 3; ++p) d[p] = *reinterpret_cast<const xbf16x8*>(P + xw_unit(2 * j + jb, fb + 1, p, g));
        };
#pragma unroll
        for (int j = 0; j < XPF; ++j) rd(j, xr[j]);
#pragma unroll
        for (int j = 0; j < NB; ++j) {
            if (j + XPF < NB) rd(j + XPF, xr[(j + XPF) % (XPF + 1)]);
            __builtin_amdgcn_sched_barrier(0);
            const xbf16x8(&x)[3] = xr[j % (XPF + 1)];
            if (XW_OFF(16)) {
                beside(j);
                continue;
            }
            // (w0,x2) (w1,x1) (w2,x0) (w0,x1) (w1,x0) (w0,x0): xgraph's product order
            acc[j][0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wk[0], x[2], acc[j][0], 0, 0, 0);
            acc[j][0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wk[1], x[1], acc[j][0], 0, 0, 0);
            acc[j][0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wk[2], x[0], acc[j][0], 0, 0, 0);
            acc[j][0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wk[0], x[1], acc[j][0], 0, 0, 0);
            acc[j][0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wk[1], x[0], acc[j][0], 0, 0, 0);
            acc[j][0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wk[0], x[0], acc[j][0], 0, 0, 0);
            __builtin_amdgcn_sched_barrier(0);
            beside(j);
        }
    };
    // the split units of one K block spread over the 9 items (after items 1, 4, 7)
    auto spread = [&](int kb) __attribute__((always_inline)) {
        return [&, kb](int j) __attribute__((always_inline)) {
#pragma unroll
            for (int i = 0; i < C::NLG; ++i)
                if (j == 3 * i + 1) {
                    gsplit_unit(kb, i);
                    __builtin_amdgcn_sched_barrier(0);
                }
        };
    };
    // s: the tile's last global T step (its next tile's K blocks are s + 1, s + 2)
    auto gcn_phase = [&](int s, int row0) __attribute__((always_inline)) {
        // the gcn K blocks carry nothing of the next tile (with the T weights resident the
        // register file is full): one weight register set, K block kb + 1's load issued
        // right after K block kb's MFMAs, its latency under the barrier and the split
        stamp(1);
        asm volatile("" : "+v"(tid), "+v"(lane));   // lane-derived addresses made here, not hoisted out of the tile loop
        load_wg(0, wga);
#pragma unroll
        for (int i = 0; i < C::NLG; ++i) gsplit_unit(0, i);
        lds_barrier();   // K block 0's planes landed
        stamp(2);
        gmma(0, wga, spread(1));
        load_wg(1, wga);
        lds_barrier();
        stamp(3);
        gmma(1, wga, spread(2));
        load_wg(2, wga);
        lds_barrier();
        stamp(4);
        gmma(2, wga, spread(3));
        load_wg(3, wga);
        lds_barrier();   // every image read of K block 2 done, the slots' out rows all split
        stamp(5);
        // the next tile's K block 0 as raw fp32 rows by LDS-DMA into image 0, free since K block
        // 2's reads (no registers: with the T weights resident the mix has none to spare); HBM
        // latency under K block 3's MFMAs and the mix
        dma_halo(s + 1, pimg(0));
        // K block 3's weights landed: only the halo DMA (NHD instructions per wave) is younger
        static_assert(NHD == 3, "wait_wg3");
        asm volatile("s_waitcnt vmcnt(3)" : "+v"(wga[0]), "+v"(wga[1]), "+v"(wga[2]));
        gmma(3, wga, [&](int) __attribute__((always_inline)) {});
        // y through the slots (this wave's 16 channels, pixel-major, as the T epilogue)
        asm volatile("" : "+v"(tid), "+v"(lane));
        {
            const int g = lane >> 4, px = lane & 15;
#pragma unroll
            for (int j = 0; j < NB; ++j) {
                *reinterpret_cast<f32x4*>(idw + (16 * j + px) * 64 + g * 16) = acc[j][0];
                acc[j][0] = f32x4{0.f, 0.f, 0.f, 0.f};
            }
        }
        lds_barrier();   // y complete; every image read done
        stamp(6);
        // the mix: thread (frame f, channels 4 c4 ..), waves 0-3 joints 0 .. XW_MIXW - 1, 4-7 the
        // rest (the COCO hop <= 2 terms split about evenly: 55 / 52 at 7)
        asm volatile("" : "+v"(tid), "+v"(lane));
        const int it = tid & 255, f = it >> 5, c4 = it & 31;
        // A_eff across the wave from LDS (5 VGPRs, v_readlane as xgraph.hip)
        float amv[5];
#pragma unroll
        for (int k = 0; k < 5; ++k) amv[k] = b2s[V * 128 + 64 * k + lane];
        auto mix = [&](auto W0c, auto W1c, auto sparse) __attribute__((always_inline)) {
            constexpr int W0 = decltype(W0c)::value, W1 = decltype(W1c)::value;
            constexpr bool SP = decltype(sparse)::value;
            // the joints this half reads (all of them for a dense A_eff)
            unsigned need = 0;
#pragma unroll
            for (int wj = W0; wj < W1; ++wj) need |= SP ? coco_hop2_mask3(wj) : 0x1FFFFu;
            f32x4 y[V];
#pragma unroll
            for (int v = 0; v < V; ++v)
                if ((need >> v) & 1u)
                    y[v] = *reinterpret_cast<const f32x4*>(sl + (c4 >> 2) * IDW + (16 * (v >> 1) + 8 * (v & 1) + f) * 64 + (c4 & 3) * 16);
#pragma unroll
            for (int wj = W0; wj < W1; ++wj) {
                f32x4 z = *reinterpret_cast<const f32x4*>(b2s + wj * 128 + 4 * c4);
#pragma unroll
                for (int v = 0; v < V; ++v)
                    if (!SP || ((coco_hop2_mask3(wj) >> v) & 1u)) {
                        const float av = __builtin_bit_cast(
                            float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, amv[(v * V + wj) / 64]), (v * V + wj) % 64));
                        z += av * y[v];
                    }
#pragma unroll
                for (int e = 0; e < 4; ++e) z[e] = z[e] > 0.f ? z[e] : 0.f;
                xst4(a.zout + (size_t)(row0 + f * V + wj) * a.ldzo + 4 * c4, z, a.nts);
            }
        };
        using I0 = std::integral_constant<int, 0>;
        using I9 = std::integral_constant<int, XW_MIXW>;
        using I17 = std::integral_constant<int, 17>;
        if (XW_OFF(64)) {
        } else if (wave >= NW / 2) {
            if (a.mix_sparse) mix(I9{}, I17{}, std::true_type{});
            else mix(I9{}, I17{}, std::false_type{});
        } else {
            if (a.mix_sparse) mix(I0{}, I9{}, std::true_type{});
            else mix(I0{}, I9{}, std::false_type{});
        }
        // the next tile's K block 1 into rb (split late in its K block 0); then its K block 0,
        // in place: every thread reads its raw units of image 0, a barrier, then writes their
        // planes into image 0 (the next tile's K block 0 barrier publishes them). This wave's
        // DMA is older than its z stores (>= min(XW_MIXW, 17 - XW_MIXW)) and those rb loads (NLD)
        load(s + 2, rb[0]);
        wait_vm<NLD + (XW_MIXW < V - XW_MIXW ? XW_MIXW : V - XW_MIXW)>();
        lds_barrier();
        asm volatile("" : "+v"(tid), "+v"(lane));
        // (units past NU read inside image 0 and are not used)
        f32x4 raw[NLD];
#pragma unroll
        for (int i = 0; i < NLD; ++i) raw[i] = *reinterpret_cast<const f32x4*>(pimg(0) + (NT * i + tid) * 16);
        lds_barrier();   // every raw unit read (lgkmcnt(0)) before any plane overwrites it
#pragma unroll
        for (int i = 0; i < NLD; ++i) {
            const int U = NT * i + tid;
            if (i + 1 < NLD || U < NU) split_store(pimg(0), U, raw[i]);
        }
        stamp(7);
    };

    // one K block; KB compile-time so the weights and the prefetch registers are statically indexed
    auto step = [&](int s, int t, auto KBc) __attribute__((always_inline)) {
        constexpr int kb = decltype(KBc)::value;
        constexpr int nb = (kb + 1) % D;   // registers holding step s+1 (s % D == kb % D: 4 % D == 0)
        asm volatile("" : "+v"(tid), "+v"(lane));   // lane-derived addresses: not hoisted across steps
        // every wave's split(s) landed; every wave done with step s-1's image (the one split(s+1) writes)
#if XW_EPIBAR
        // at a tile's first K block the previous tile's epilogue barrier (after this image's
        // split and the last reads of the other one) already holds, except at the run's start
        if (kb != 0 || t == t_begin || FG) lds_barrier();
        constexpr int KDMA = 1;
#else
        lds_barrier();
        constexpr int KDMA = 0;
#endif
        if constexpr (kb == KDMA) {
            // this tile's identity rows into the wave's slot (every wave is done with the
            // previous tile's outputs there: the barrier above)
            __builtin_amdgcn_sched_barrier(0);
            dma_ident(t);
            __builtin_amdgcn_sched_barrier(0);
        }
        const unsigned char* P = pimg(kb);   // s & 1 == kb & 1 (4 K blocks per tile)
        const int jb = px >> 3, fb = px & 7;
        // operand ring over the 27 (block, tap) items: item n + XPF's planes are read while item n's MFMAs run
        constexpr int NI = NB * 3, XPF = XW_XPF;
        xbf16x8 xr[XPF + 1][3];
        auto rd = [&](int n, xbf16x8 (&d)[3]) __attribute__((always_inline)) {
            const int j = n / 3, tap = n - 3 * (n / 3);
#pragma unroll
            for (int p = 0; p < 3; ++p) d[p] = *reinterpret_cast<const xbf16x8*>(P + xw_unit(2 * j + jb, fb + tap, p, g));
        };
        // FG: the next tile's K blocks 0 and 1 are split / loaded in the gcn phase (its
        // planes images are busy until then): K block 2 splits block 3 only, 3 nothing
        constexpr bool SPL = !FG || kb < NKB - 1, LDN = !FG || kb < NKB - 2;
        auto mfma_n = [&](int n, int unit) __attribute__((always_inline)) {
            if (n + XPF < NI) rd(n + XPF, xr[(n + XPF) % (XPF + 1)]);
            __builtin_amdgcn_sched_barrier(0);
            if (XW_OFF(4)) return;
            const int j = n / 3, tap = n - 3 * (n / 3);
            const xbf16x8(&x)[3] = xr[n % (XPF + 1)];
#pragma unroll
            for (int cb = 0; cb < CB; ++cb) {
                const xbf16x8(&wk)[3] = w[tap * NKB + kb][cb];
                // (w0,x2) (w1,x1) (w2,x0) (w0,x1) (w1,x0) (w0,x0): xgemm's product order
                acc[j][cb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wk[0], x[2], acc[j][cb], 0, 0, 0);
                acc[j][cb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wk[1], x[1], acc[j][cb], 0, 0, 0);
                acc[j][cb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wk[2], x[0], acc[j][cb], 0, 0, 0);
                acc[j][cb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wk[0], x[1], acc[j][cb], 0, 0, 0);
                acc[j][cb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wk[1], x[0], acc[j][cb], 0, 0, 0);
                acc[j][cb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wk[0], x[0], acc[j][cb], 0, 0, 0);
            }
            if (unit >= 0) {
                // a split unit after the item's MFMAs in program order, its VALU then
                // scheduled between them (its LDS writes and load anywhere)
                if (!XW_OFF(2)) split_unit(kb + 1, rb[nb], unit);
                if (LDN) load_unit(s + 1 + D, rb[nb], unit);
#pragma unroll
                for (int q = 0; q < 6 * CB; ++q) {
                    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                    __builtin_amdgcn_sched_group_barrier(0x002, 4, 0);
                }
            }
            __builtin_amdgcn_sched_barrier(0);
        };
#pragma unroll
        for (int n = 0; n < XPF; ++n) rd(n, xr[n]);
        // the next K block's split, one 16-B unit at a time, spread over this block's
        // MFMA items (waves leave the barrier together: a split in one piece would
        // idle the MFMA pipe), each unit's register slot reloaded right after (past
        // the run: zeros, never read)
#pragma unroll
        for (int n = 0; n < NI; ++n) {
            int unit = -1;
#pragma unroll
            for (int i = 0; i < NLD; ++i)
                // FG K block 0: its rb was loaded just before the tile, so its split units go late
                if (SPL && n == (FG && kb == 0 ? NI / 2 + (i * NI) / (2 * NLD) : XW_SPLIT_AT ? i * NI / NLD + 1 : ((2 * i + 1) * NI) / (2 * NLD)) + 1)
                    unit = i;
            mfma_n(n, unit);
        }
        if constexpr (kb == NKB - 1) {
            // ---- epilogue: (acc + x) + bias, ReLU. The identity DMA of this tile was issued
            // before the register loads of its K blocks KDMA .. 3: at most that many may stay in flight
            if constexpr (FG) {
                stamp(0);
                wait_vm<0>();   // the identity DMA landed (the K-block loads since were consumed)
            } else {
                wait_vm<(NKB - KDMA) * NLD>();
            }
#pragma unroll
            for (int j = 0; j < NB; ++j)
#pragma unroll
                for (int cb = 0; cb < CB; ++cb) {
                    f32x4* sl = reinterpret_cast<f32x4*>(idw + (16 * j + px) * (64 * CB) + (4 * cb + g) * 16);
                    f32x4 v = acc[j][cb] + *sl;
                    v += bv[cb];
#pragma unroll
                    for (int e = 0; e < 4; ++e) v[e] = v[e] > 0.f ? v[e] : 0.f;
                    *sl = v;   // the output replaces the identity in the slot
                    acc[j][cb] = f32x4{0.f, 0.f, 0.f, 0.f};
                }
            // whole output rows from the slots: 32 lanes x 16 B = one 512-B row
            lds_barrier();
            int row0, f0;
            tile_geo(t, row0, f0);
#pragma unroll
            for (int i = 0; i < NB * 16 * 32 / NT; ++i) {
                const int q = tid + NT * i, pix = q >> 5, cu = q & 31;
                const int j = pix >> 4, pp = pix & 15, jj = 2 * j + (pp >> 3);
                const int ws = cu / (4 * CB), pc = cu - ws * (4 * CB);
                const f32x4 v = *reinterpret_cast<const f32x4*>(sl + ws * IDW + pix * (64 * CB) + pc * 16);
                float* o = jj < V ? a.out + (size_t)(row0 + (pp & 7) * V + jj) * a.ldo + cu * 4 : a.trash + (tid & 255) * 4;
                if (!XW_OFF(8)) xst4(o, v, a.nts);
            }
        }
    };
    // static priority for the younger half of the workgroup (waves 4-7 lose VALU arbitration
    // to their older SIMD partners on every segment: MI355X_MICROARCH.md, two waves per SIMD):
    // 0.265 vs 0.272 ms on L3. 8 waves only (the condition must be wave-uniform: readfirstlane)
    if (NW == 8 && __builtin_amdgcn_readfirstlane(threadIdx.x) >= 256) __builtin_amdgcn_s_setprio(1);
    stamp(-1);
    auto tphase = [&](int t) __attribute__((always_inline)) {
        const int s0 = (t - t_begin) * NKB;
        step(s0, t, std::integral_constant<int, 0>{});
        step(s0 + 1, t, std::integral_constant<int, 1>{});
        step(s0 + 2, t, std::integral_constant<int, 2>{});
        step(s0 + 3, t, std::integral_constant<int, 3>{});
    };
    if constexpr (FG) {
        // the loop body is [gcn phase of tile t, T phase of tile t + 1]: the registers the gcn
        // phase loads for the next tile are used in the same iteration, so the loop header (a
        // control-flow merge) does not wait for them, or for every store, with vmcnt(0)
        tphase(t_begin);
        for (int t = t_begin; t < t_end; ++t) {
            int row0, f0;
            tile_geo(t, row0, f0);
            gcn_phase((t - t_begin) * NKB + NKB - 1, row0);
            if (t + 1 < t_end) tphase(t + 1);
        }
    } else {
        for (int t = t_begin; t < t_end; ++t) tphase(t);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#ifdef TIK_XTRACE
    if (tr && lane == 0) {
        unsigned long long* o = a.trace + 16 * (size_t)blockIdx.x + (wave == 4 ? 8 : 0);
#pragma unroll
        for (int i = 0; i < 8; ++i) o[i] = ph_[i];
        if (wave == 0) o[7] |= (unsigned long long)(t_end - t_begin) << 48;
    }
#endif
}

bool xtws_ok(const XTConvArgs& a) {
    return a.T > 0 && a.T % xw::F == 0 && a.ldz % 4 == 0 && a.ldz >= 128 && a.ldx % 4 == 0 && a.ldx >= 128 &&
           a.ldo % 4 == 0 && a.ldo >= 128;
}

hipError_t launch_xtws(const XTConvArgs& a, int ncu, hipStream_t st) {
    if (a.M <= 0) return hipSuccess;
    if (!xtws_ok(a) || !a.z || !a.x || !a.wp || !a.bias || !a.out || !a.trash || ncu <= 0 || a.M % (17 * a.T) != 0)
        return hipErrorInvalidValue;
    if (a.wg && (!a.bias2 || !a.amix || !a.zout || a.ldzo % 4 || a.ldzo < 128 || a.zout == a.z)) return hipErrorInvalidValue;
    // the buffer offsets are 32-bit: launches of whole windows, < 2 GiB of conv input and identity rows each
    const long long win = 17LL * a.T, win_bytes = win * std::max(std::max(a.ldz, a.ldx), a.wg ? a.ldzo : 0) * 4;
    if (win_bytes >= (1LL << 31)) return hipErrorInvalidValue;
    const long long wper = std::max(1LL, ((1LL << 31) - 1) / win_bytes);
    const long long rows_per = wper * win;
    (void)hipGetLastError();
    for (long long r0 = 0; r0 < a.M; r0 += rows_per) {
        XTConvArgs c = a;
        c.M = (int)std::min(rows_per, (long long)a.M - r0);
        c.z = a.z + (size_t)r0 * a.ldz;
        c.x = a.x + (size_t)r0 * a.ldx;
        c.out = a.out + (size_t)r0 * a.ldo;
        if (a.wg) c.zout = a.zout + (size_t)r0 * a.ldzo;
        const int ntiles = (int)(c.M / win) * (a.T / xw::F);
        // 8 waves (two per SIMD, 16 channels each); 4 waves of 32 channels (one per SIMD, the weights
        // through AGPRs: v_accvgpr_read before every MFMA group) measured 0.364 vs 0.288 ms
        if (a.wg) hipLaunchKernelGGL((xtws_kernel<XW_D, 8, true>), dim3(std::min(ntiles, ncu)), dim3(512), 0, st, c);
        else hipLaunchKernelGGL((xtws_kernel<XW_D, 8, false>), dim3(std::min(ntiles, ncu)), dim3(512), 0, st, c);
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

}  // namespace tik
