// tgw.hip — weight-stationary persistent temporal conv + next gcn (TW_128):
// the stride-1, identity-residual 128->128 ST-GCN blocks whose successor is a
// 128->128 block (L3 -> L4, L4 -> L5 of the IK net).
//
// Per output tile of 7 whole frames (119 pixels, 17 joints):
//   out = ReLU( sum_tap z[t+tap-1] . Wt'_tap^T + bias + x )        (this block's T)
//   z'  = ReLU( mix_A( out . Wg'^T ) + bias2' )                     (next block's G)
// computed TRANSPOSED (MFMA A operand = weights, B operand = pixels), so
//  * each wave owns 16 output channels and keeps their f16 hi/lo weights —
//    all 12 (tap, block) K steps of Wt' — in registers for the whole launch:
//    no weight traffic in the K loop (the round-1 TG3 kernel streamed 192 KB
//    of Wt' from L2 per 119-row tile); the next gcn's 32 KB of Wg' come from
//    L2 into registers once per tile, behind the tile's DMAs;
//  * an accumulator lane holds 4 consecutive channels of one pixel, which is
//    one 8-byte piece of a split-block row: bias + residual + ReLU + the hi/lo
//    split happen in registers, no fp32 C-tile staging.
// The z operand of a tile is ONE frame-halo image per 32-channel block (frames
// q0-1 .. q0+7, 160 rows): tap k of pixel p reads image row p + 17k, or a
// zero row when the tap leaves the pixel's window (Conv2d zero padding), so
// each z row is DMA'd once per tile instead of once per tap.
//
// Persistent: one 512-thread workgroup per CU walks a contiguous run of tiles
// (runs laid out per XCD). The four block slots of the NEXT tile are DMA'd as
// soon as every wave is past the current tile's last tap (the epilogue's first
// barrier), and its residual tile x in tap 0, so HBM keeps streaming through
// the epilogue.
// Every wave issues a fixed number of vector-memory instructions per tile
// (slot DMA, residual DMA, 8 gcn-weight loads, 8 + 8 whole-line stores;
// invalid rows go to a trash line), which makes every counted vmcnt wait
// exact (tests/test_isa.py checks the counts in the generated code).
//
// Arithmetic is cgemm3/tgemm's f16x3 (a_lo b_hi + a_hi b_lo + a_hi b_hi, fp32
// accumulate) in the same K order, and the mix adds bias2' then the joints in
// order, like the TG_128x128_G7 epilogue it replaces.
#include <cstdlib>
#include <type_traits>

#include "cgemm3_dev.h"

namespace tik {

namespace tw {
constexpr int FG = 7;                       // output frames per tile
constexpr int RT = FG * 17;                 // 119 output pixels per tile
constexpr int NPF = 8;                      // 16-pixel MFMA fragments (128 pixel slots)
constexpr int IMG_ROWS = 160;               // DMA'd halo rows per block slot (>= (FG + 2) * 17 = 153)
constexpr int ZROW = IMG_ROWS;              // the slot's zero row
constexpr int SLOT = (IMG_ROWS + 1) * 128;  // 20,608 B
constexpr int EOFF = 4 * SLOT;              // E region: residual image, then next-gcn image, then Y
constexpr int EB = 128 * 128;               // one 128-row block image
constexpr int LDY = 132;                    // Y (fp32 gcn output) row stride in floats
constexpr int B2OFF = EOFF + 4 * EB;        // bias2' [17][128] fp32
constexpr int SMEM = B2OFF + 17 * 128 * 4;  // 156,672 B: one workgroup per CU
constexpr int NR = 8;                       // residual DMA instructions per wave per tile
constexpr int NS = 8 + 8;                   // stores per wave per tile (out lines + z' lines)
static_assert(RT * LDY * 4 <= 4 * EB, "Y fits the E region");
static_assert(SMEM <= 160 * 1024, "LDS");
}  // namespace tw

template <int PD, int PG>
__global__ __launch_bounds__(512, 2) void tgw_kernel(Cgemm3Args a, int ntiles) {
    using namespace tw;
    __shared__ __attribute__((aligned(16))) unsigned char smem[SMEM];   // the only LDS object
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int M = a.M, nfo = a.M / 17, T = a.tout;
    // debug (a.trace): per-workgroup phase sums over its tiles, in s_memrealtime ticks
    unsigned long long tr_loop = 0, tr_epi1 = 0, tr_epi2 = 0, tr_epi3 = 0, tr_wait = 0, tr_bar = 0;
    const unsigned long long ts_start = a.trace ? __builtin_amdgcn_s_memrealtime() : 0;

    // ---- this workgroup's contiguous run of tiles (runs ordered per XCD)
    int t_begin, t_end;
    {
        const int G = gridDim.x, bid = blockIdx.x;
        const int per = G >> 3, rem = G & 7, x = bid & 7, k = bid >> 3;
        const int s = x < rem ? x * (per + 1) + k : rem * (per + 1) + (x - rem) * per + k;
        t_begin = (int)((long long)s * ntiles / G);
        t_end = (int)((long long)(s + 1) * ntiles / G);
    }

    // ---- stationary operands: this wave's 16 output channels
    const int co = 16 * wave + (lane & 15), g0 = lane >> 4;
    f16x8 wth[12], wtl[12];
#pragma unroll
    for (int s = 0; s < 12; ++s) {   // K step s = tap * 4 + block: SB weights [Nc][tap][block][64]
        const unsigned short* p = a.seg[0].w + (size_t)co * a.seg[0].ldw + s * 64 + 8 * g0;
        wth[s] = *reinterpret_cast<const f16x8*>(p);
        wtl[s] = *reinterpret_cast<const f16x8*>(p + 32);
    }
    const f32x4 bv = *reinterpret_cast<const f32x4*>(a.bias + 16 * wave + 4 * g0);   // this lane's 4 output channels
    constexpr int NAM = (17 * 17 + 63) / 64;   // A_eff' in registers, read back with v_readlane
    float amv[NAM];
#pragma unroll
    for (int k = 0; k < NAM; ++k) amv[k] = 64 * k + lane < 17 * 17 ? a.g_amix[64 * k + lane] : 0.f;
    float* b2s = reinterpret_cast<float*>(smem + B2OFF);
    for (int i = tid; i < 17 * 128; i += 512) b2s[i] = a.g_bias2[i];
    if (tid < 32) *reinterpret_cast<f32x4*>(smem + (tid >> 3) * SLOT + ZROW * 128 + (tid & 7) * 16) = f32x4{0.f, 0.f, 0.f, 0.f};
    // every register load retired before the first DMA, and visibly so to the
    // compiler (the empty asm redefines each value), so it never inserts a
    // vmcnt wait for them inside the pipelined loop
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
    for (int s = 0; s < 12; ++s) asm volatile("" : "+v"(wth[s]), "+v"(wtl[s]));
    f32x4 bias_t = bv;
    asm volatile("" : "+v"(bias_t));
#pragma unroll
    for (int k = 0; k < NAM; ++k) asm volatile("" : "+v"(amv[k]));
    lds_barrier();

    // ---- DMA roles. Slot: 20 instructions of 8 rows (waves 0-3: 3, waves 4-7: 2).
    // Residual image: 4 blocks x 16 instructions, 8 per wave (wave w: block w/2).
    const int na = wave < 4 ? 3 : 2;
    const int jj0 = wave < 4 ? 3 * wave : 12 + 2 * (wave - 4);
    const int ldz = a.seg[0].ld, ldr = a.ldr;
    const i32x4 rZ = buf_rsrc(a.seg[0].src, (unsigned)((long long)M * ldz * 2));
    const i32x4 rX = buf_rsrc(a.resid, (unsigned)((long long)M * ldr * 2));
    unsigned zoff[3];
    auto prep_slots = [&](int tile) {   // tile < 0: a dummy (all rows zero-filled)
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            const int rr = 8 * (jj0 + j) + (lane >> 3);
            const int R = (tile * FG - 1) * 17 + rr;
            const int ck = (lane & 7) ^ sbf(rr);
            zoff[j] = (tile >= 0 && R >= 0 && R < M) ? (unsigned)(((long long)R * ldz + 8 * ck) * 2) : DMA_OOB;
        }
    };
    auto issue_slot = [&](int blk) {
        unsigned char* dst = smem + blk * SLOT + jj0 * 1024;
        dma16(rZ, dst, zoff[0], blk * 128);
        dma16(rZ, dst + 1024, zoff[1], blk * 128);
        if (na == 3) dma16(rZ, dst + 2048, zoff[2], blk * 128);
    };
    auto issue_resid = [&](int tile, int j0, int nj) {   // residual DMA instructions j0 .. j0+nj-1
        const int b = wave >> 1;
        unsigned char* dst = smem + EOFF + b * EB + (wave & 1) * 8 * 1024;
#pragma unroll
        for (int j = j0; j < j0 + nj; ++j) {
            const int rg = (wave & 1) * 8 + j;
            const int rr = 8 * rg + (lane >> 3);
            const int R = tile * FG * 17 + rr;
            const int ck = (lane & 7) ^ sbf(rr);
            const unsigned off = (tile >= 0 && R < M) ? (unsigned)(((long long)R * ldr + b * 64 + 8 * ck) * 2) : DMA_OOB;
            dma16(rX, dst + j * 1024, off, 0);
        }
    };

    // ---- prologue: the first tile's four slots
    if (t_begin < t_end) {
        prep_slots(t_begin);
#pragma unroll
        for (int blk = 0; blk < 4; ++blk) issue_slot(blk);
    }
    int prev_stores = 0;   // vector-memory ops issued after a tile's slot DMAs (the last epilogue's stores)
    for (int tile = t_begin; tile < t_end; ++tile) {
        const int q0 = tile * FG;
        const int nxt = tile + 1 < t_end ? tile + 1 : -1;
        const unsigned long long ts0 = a.trace ? __builtin_amdgcn_s_memrealtime() : 0;
        // lane-derived offsets and row strides are re-derived from opaque copies every
        // tile: hoisted out of the tile loop they would stay live across the K loop
        // (dozens of VGPRs of per-joint and per-fragment addresses) and spill
        int lt = lane, ldo = a.ldo, gldo = a.g_ldo;
        asm volatile("" : "+v"(lt), "+s"(ldo), "+s"(gldo));
        const int l15 = lt & 15, g = lt >> 4;
        const int c0 = 16 * wave + 4 * g;   // this lane's 4 output channels (accumulator rows)
        const int cb = c0 >> 5, cc = c0 & 31, uh = cc >> 3, sub = (cc & 7) * 2;   // c0's place in a split-block row
        unsigned short* trash = a.trash + (((wave << 6) + lt) & 255) * 8;
        // B operand rows of this tile: tap k of pixel p = image row p + 17k, or
        // the zero row when the tap leaves the pixel's window; bit 3i+k of tmask
        // marks a valid (fragment i, tap k) row of this lane
        unsigned tmask = 0;
#pragma unroll
        for (int i = 0; i < NPF; ++i) {
            const int p = 16 * i + l15, f = p / 17;
            const int q = q0 + f;
            const int t = q % T;
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                const bool ok = p < RT && q < nfo && t + k - 1 >= 0 && t + k - 1 < T;
                tmask |= (ok ? 1u : 0u) << (3 * i + k);
            }
        }
        prep_slots(nxt);

        f32x4 acc[NPF];
#pragma unroll
        for (int i = 0; i < NPF; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
        // all four slots of this tile landed (younger: the last epilogue's stores); and every
        // wave is past the last epilogue's reads of the E region (the residual DMA target)
        wait_vm_dyn(prev_stores);
        lds_barrier();
        // K loop, fully unrolled over (tap, block, fragment) with the B reads PD
        // fragments ahead of their MFMAs (a read consumed right away exposes the
        // LDS latency; measured: loop at ~2x the MFMA time)
        f16x8 wgh[4], wgl[4];
        int bo[2][NPF];   // B row offsets of the current and the next tap (the block slot is an immediate)
        auto tap_offsets = [&](int tap, int* o) {
#pragma unroll
            for (int i = 0; i < NPF; ++i) o[i] = sbo(((tmask >> (3 * i + tap)) & 1u) ? 16 * i + l15 + 17 * tap : ZROW, g);
        };
        tap_offsets(0, bo[0]);
        constexpr int NSTEP = 3 * 4 * NPF;   // (tap, block, fragment) triples
        f16x8 pbh[PD + 1], pbl[PD + 1];
        auto load_b = [&](int n) {
            const int tap = n / (4 * NPF), blk = (n / NPF) % 4, i = n % NPF;
            const unsigned char* B = smem + blk * SLOT;
            const int o = bo[tap & 1][i];
            pbh[n % (PD + 1)] = *reinterpret_cast<const f16x8*>(B + o);
            pbl[n % (PD + 1)] = *reinterpret_cast<const f16x8*>(B + (o ^ 64));
        };
#pragma unroll
        for (int n = 0; n < PD; ++n) load_b(n);
#pragma unroll
        for (int tap = 0; tap < 3; ++tap) {
#pragma unroll
            for (int blk = 0; blk < 4; ++blk) {
#pragma unroll
                for (int i = 0; i < NPF; ++i) {
                    const int n = (tap * 4 + blk) * NPF + i;
                    if (blk == 0 && i == 0 && tap + 1 < 3) tap_offsets(tap + 1, bo[(tap + 1) & 1]);
                    if (n + PD < NSTEP) load_b(n + PD);
                    const int s = tap * 4 + blk;
                    const f16x8 bh = pbh[n % (PD + 1)], bl = pbl[n % (PD + 1)];
                    acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wth[s], bl, acc[i], 0, 0, 0);
                    acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wtl[s], bh, acc[i], 0, 0, 0);
                    acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wth[s], bh, acc[i], 0, 0, 0);
                    // keep the prefetch distance: the two reads of fragment n+2 go between
                    // fragment n's three MFMAs (the scheduler would sink them to their use)
                    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                    __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
                    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                    __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
                    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                    // this tile's residual image: 2 DMA instructions per block of tap 0,
                    // their issue cost hidden among the MFMAs
                    if (tap == 0 && (i == 1 || i == 5)) issue_resid(tile, 2 * blk + (i == 5), 1);
                    // the next gcn's weights for this wave's 16 channels (L2-resident),
                    // loaded during tap 2: live only from here to the epilogue's gcn
                    if (tap == 2 && blk == 0 && i == 0) {
                        const unsigned short* pg = a.g_w + (size_t)(16 * wave + l15) * a.g_ldw + 8 * g;
#pragma unroll
                        for (int kb = 0; kb < 4; ++kb) {
                            wgh[kb] = *reinterpret_cast<const f16x8*>(pg + kb * 64);
                            wgl[kb] = *reinterpret_cast<const f16x8*>(pg + kb * 64 + 32);
                        }
                    }
                }
            }
        }
        const unsigned long long ts1 = a.trace ? __builtin_amdgcn_s_memrealtime() : 0;

        // ===== epilogue
        // (1) this tile's residual image and the gcn weights landed (the youngest loads)
        wait_vm_dyn(0);
#pragma unroll
        for (int kb = 0; kb < 4; ++kb) asm volatile("" : "+v"(wgh[kb]), "+v"(wgl[kb]));
        const unsigned long long tsw = a.trace ? __builtin_amdgcn_s_memrealtime() : 0;
        lds_barrier();   // ... for every wave; and every wave is done with the four slots
        // the next tile's four blocks stream in behind the whole epilogue (issued
        // inside the next-gcn loop they landed later: TW 0.359 -> 0.353 ms)
#pragma unroll
        for (int kb = 0; kb < 4; ++kb) issue_slot(kb);
        const unsigned long long tsb = a.trace ? __builtin_amdgcn_s_memrealtime() : 0;
        // (2) out = ReLU(C + bias + x) -> the split image of out, IN PLACE of the residual
        // image: each (pixel, 4-channel) piece is read and rewritten by the same lane
        // (all reads first: one LDS round trip, not one per fragment)
        {
            unsigned char* rb = smem + EOFF + cb * EB;
            f16x4 rh[NPF], rl[NPF];
#pragma unroll
            for (int i = 0; i < NPF; ++i) {
                const int p = 16 * i + l15;
                rh[i] = *reinterpret_cast<const f16x4*>(rb + sbo(p, uh) + sub);
                rl[i] = *reinterpret_cast<const f16x4*>(rb + sbo(p, 4 + uh) + sub);
            }
#pragma unroll
            for (int i = 0; i < NPF; ++i) {
                const int p = 16 * i + l15;
                f32x4 v = acc[i] + bias_t;
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    v[e] += (float)rh[i][e] + (float)rl[i][e];
                    v[e] = v[e] > 0.f ? v[e] : 0.f;
                }
                f16x4 oh, ol;
                split4(v, oh, ol);
                *reinterpret_cast<f16x4*>(rb + sbo(p, uh) + sub) = oh;
                *reinterpret_cast<f16x4*>(rb + sbo(p, 4 + uh) + sub) = ol;
            }
        }
        lds_barrier();
        const unsigned long long ts2 = a.trace ? __builtin_amdgcn_s_memrealtime() : 0;
        // (5) the next block's gcn 1x1 conv on the tile
        f32x4 acc2[NPF];
#pragma unroll
        for (int i = 0; i < NPF; ++i) acc2[i] = f32x4{0.f, 0.f, 0.f, 0.f};
        {
            // B reads two fragments ahead of their MFMAs, as in the K loop
            f16x8 gbh[PG + 1], gbl[PG + 1];
            auto load_g = [&](int n) {
                const unsigned char* B = smem + EOFF + (n / NPF) * EB;
                const int p = 16 * (n % NPF) + l15;
                gbh[n % (PG + 1)] = *reinterpret_cast<const f16x8*>(B + sbo(p, g));
                gbl[n % (PG + 1)] = *reinterpret_cast<const f16x8*>(B + sbo(p, 4 + g));
            };
#pragma unroll
            for (int n = 0; n < PG; ++n) load_g(n);
#pragma unroll
            for (int kb = 0; kb < 4; ++kb) {
#pragma unroll
                for (int i = 0; i < NPF; ++i) {
                    const int n = kb * NPF + i;
                    if (n + PG < 4 * NPF) load_g(n + PG);
                    const f16x8 bh = gbh[n % (PG + 1)], bl = gbl[n % (PG + 1)];
                    acc2[i] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wgh[kb], bl, acc2[i], 0, 0, 0);
                    acc2[i] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wgl[kb], bh, acc2[i], 0, 0, 0);
                    acc2[i] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wgh[kb], bh, acc2[i], 0, 0, 0);
                    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                    __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
                    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                    __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
                    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                }
            }
        }
        // (4) out -> HBM in whole 128-B lines (8 per thread; rows past the tile to the trash line)
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            const int idx = (wave << 6) + lt + 512 * q;
            const int b = idx >> 10, r = (idx & 1023) >> 3, u = idx & 7;
            const f32x4 d = *reinterpret_cast<const f32x4*>(smem + EOFF + b * EB + sbo(r, u));
            const bool ok = r < RT && q0 * 17 + r < M;
            unsigned short* o = ok ? a.out_h + (size_t)(q0 * 17 + r) * ldo + b * 64 + u * 8 : trash;
            *reinterpret_cast<f32x4*>(o) = d;
        }
        lds_barrier();   // image reads done (gcn and out lines)
        // (6) gcn output -> Y [pixel][channel] fp32
        {
            float* Y = reinterpret_cast<float*>(smem + EOFF);
#pragma unroll
            for (int i = 0; i < NPF; ++i) {
                const int p = 16 * i + l15;
                if (p < RT) *reinterpret_cast<f32x4*>(Y + p * LDY + c0) = acc2[i];
            }
        }
        lds_barrier();
        const unsigned long long ts3 = a.trace ? __builtin_amdgcn_s_memrealtime() : 0;
        // (7) graph mix + bias2' + ReLU -> z' (frame f, channels 4cq..4cq+3 per lane;
        // even waves joints 0-8, odd waves 9-16 and one trash pair: 18 stores each)
        {
            // re-materialise A_eff' each tile: its v_readlane values would otherwise be
            // hoisted out of the tile loop into ~150 live SGPRs
#pragma unroll
            for (int k = 0; k < NAM; ++k) asm volatile("" : "+v"(amv[k]));
            const float* Y = reinterpret_cast<const float*>(smem + EOFF);
            const int item = (wave >> 1) * 64 + lt, f = item >> 5, cq = item & 31;
            const int fr = f < FG ? f : FG - 1;
            f32x4 y[17];
#pragma unroll
            for (int v = 0; v < 17; ++v) y[v] = *reinterpret_cast<const f32x4*>(Y + (fr * 17 + v) * LDY + 4 * cq);
            lds_barrier();   // every Y read done: the z' image goes over Y
            unsigned char* zb = smem + EOFF + ((4 * cq) >> 5) * EB;
            const int zu = ((4 * cq) & 31) >> 3, zs = ((4 * cq) & 7) * 2;
            auto mixr = [&](auto w0c, auto w1c, auto sp) {
                constexpr int W0 = decltype(w0c)::value, W1 = decltype(w1c)::value;
                constexpr bool SP = decltype(sp)::value;
#pragma unroll
                for (int w = W0; w < W1; ++w) {
                    f32x4 z = *reinterpret_cast<const f32x4*>(b2s + w * 128 + 4 * cq);
#pragma unroll
                    for (int v = 0; v < 17; ++v)
                        if (!SP || ((coco_hop2_mask3(w) >> v) & 1u)) {
                            const float av = __builtin_bit_cast(
                                float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, amv[(v * 17 + w) / 64]), (v * 17 + w) % 64));
                            z += av * y[v];
                        }
#pragma unroll
                    for (int e = 0; e < 4; ++e) z[e] = z[e] > 0.f ? z[e] : 0.f;
                    f16x4 h, l;
                    split4(z, h, l);
                    const int r = fr * 17 + w;   // image row (frames past the tile rewrite frame 6's rows: never stored)
                    if (f < FG) {
                        *reinterpret_cast<f16x4*>(zb + sbo(r, zu) + zs) = h;
                        *reinterpret_cast<f16x4*>(zb + sbo(r, 4 + zu) + zs) = l;
                    }
                }
            };
            using I0 = std::integral_constant<int, 0>;
            using I9 = std::integral_constant<int, 9>;
            using I17 = std::integral_constant<int, 17>;
            if (wave & 1) {
                if (a.g_mix_sparse) mixr(I9{}, I17{}, std::true_type{});
                else mixr(I9{}, I17{}, std::false_type{});
            } else {
                if (a.g_mix_sparse) mixr(I0{}, I9{}, std::true_type{});
                else mixr(I0{}, I9{}, std::false_type{});
            }
            lds_barrier();
            // z' -> HBM in whole 128-B lines (8 per thread; rows past the tile to the trash line)
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                const int idx = (wave << 6) + lt + 512 * q;
                const int b = idx >> 10, r = (idx & 1023) >> 3, u = idx & 7;
                const f32x4 d = *reinterpret_cast<const f32x4*>(smem + EOFF + b * EB + sbo(r, u));
                const bool ok = r < RT && q0 * 17 + r < M;
                unsigned short* o = ok ? a.g_out + (size_t)(q0 * 17 + r) * gldo + b * 64 + u * 8 : trash;
                *reinterpret_cast<f32x4*>(o) = d;
            }
        }
        prev_stores = NS;
        if (a.trace) {
            const unsigned long long ts4 = __builtin_amdgcn_s_memrealtime();
            tr_loop += ts1 - ts0; tr_epi1 += ts2 - ts1; tr_epi2 += ts3 - ts2; tr_epi3 += ts4 - ts3;
            tr_wait += tsw - ts1; tr_bar += tsb - tsw;
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (a.trace && tid == 0) {   // {tiles, loop, epilogue to image, to Y, mix + z', span, E1 wait, E1 barrier}
        unsigned long long* tr = a.trace + 8 * (size_t)blockIdx.x;
        tr[0] = (unsigned long long)(t_end - t_begin);
        tr[1] = tr_loop; tr[2] = tr_epi1; tr[3] = tr_epi2; tr[4] = tr_epi3;
        tr[5] = __builtin_amdgcn_s_memrealtime() - ts_start;
        tr[6] = tr_wait; tr[7] = tr_bar;
    }
}

static int cu_count() {
    static int n[64] = {0};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
    if (!n[dev]) {
        int c = 0;
        if (hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || c <= 0) c = 256;
        n[dev] = c;
    }
    return n[dev];
}

bool tgw_ok(const Cgemm3Args& a) {
    return a.V == 17 && a.Nc == 128 && a.M % 17 == 0 && a.nseg == 1 && a.seg[0].kt == 3 && a.seg[0].stride == 1 &&
           a.seg[0].pad == 1 && a.seg[0].nblk == 4 && a.seg[0].ldw == 12 * 64 && a.seg[0].tin == a.tout &&
           a.resid && a.out_h && a.g_w && a.g_nc == 128 && a.g_ldw >= 4 * 64 && a.g_bias2 && a.g_amix && a.g_out &&
           a.trash && !a.rx && a.act == ACT_RELU && a.seg[0].ld % 8 == 0 && a.seg[0].ld >= 256 && a.ldr % 8 == 0 &&
           a.ldr >= 256 && a.ldo % 8 == 0 && a.ldo >= 256 && a.g_ldo % 8 == 0 && a.g_ldo >= 256 &&
           (long long)a.M * a.seg[0].ld * 2 < (1LL << 31) && (long long)a.M * a.ldr * 2 < (1LL << 31);
}

hipError_t launch_tgw(const Cgemm3Args& a, hipStream_t st) {
    if (a.M <= 0) return hipSuccess;
    if (!tgw_ok(a)) return hipErrorInvalidValue;
    const int ntiles = (a.M / 17 + tw::FG - 1) / tw::FG;
    const int grid = ntiles < cu_count() ? ntiles : cu_count();
    (void)hipGetLastError();
    // B operand reads three fragments ahead of their MFMAs (measured: two ahead 0.355 ms, three 0.352 ms)
    // next-gcn B reads: two fragments ahead (three measured 0.342 vs 0.340 ms)
    hipLaunchKernelGGL((tgw_kernel<3, 2>), dim3(grid), dim3(512), 0, st, a, ntiles);
    return hipGetLastError();
}

}  // namespace tik
