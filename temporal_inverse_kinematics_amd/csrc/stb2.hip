// stb2.hip — persistent, weight-stationary whole ST-GCN block (B3_64P): the
// stride-1, identity-residual 64 -> 64 block (L1 of the IK net), as
// stblock.hip's B3_64 computes it, restructured for overlap:
//
//   * one 512-thread workgroup per CU walks a contiguous run of 14-frame
//     tiles (runs laid out per XCD);
//   * the weights live in registers for the whole launch, read TRANSPOSED as
//     the MFMA A operand: G' (waves 0-3, 16 output channels each, K = 64: 16
//     VGPRs) and T' (every wave, 16 output channels, K = 3 x 64: 48 VGPRs) —
//     no Wt ring, no per-tile weight DMA;
//   * the next tile's x image (joint-major, 16 frames x 17 joints x 64
//     channels, split blocks) is DMA'd as soon as G has consumed the current
//     one (its issue hidden among the first tap's MFMAs), so it streams
//     during the temporal conv and the epilogue; the identity residual comes
//     from L2 into registers, issued just before that DMA;
//   * T's B operand is the resident z image (tap k of pixel p = z row
//     p + 17 k, the zero row past a window edge), read two fragments ahead of
//     the MFMAs; out leaves as whole 128-B lines from an LDS image.
// Every wave issues a fixed number of vector-memory instructions per tile
// (16 residual loads, 9 x-image DMAs, 8 line stores; invalid rows clamped or
// sent to a trash line), so each counted vmcnt wait is exact (pinned by
// tests/test_isa.py). Arithmetic, K orders and the mix order are B3_64's:
// bit-identical output.
#include <type_traits>

#include "cgemm3_dev.h"

namespace tik {

namespace s2 {
constexpr int V = 17, FIN = 16, F = FIN - 2;   // input (halo) / output frames per tile
constexpr int PX = FIN * V;                    // 272 input pixels: x image row 16 v + f (joint-major)
constexpr int TR = F * V;                      // 238 output pixels
constexpr int NTF = (TR + 15) / 16;            // 15 output fragments
constexpr int XROWS = 288;                     // x image rows per block (DMA: 36 instructions)
constexpr int XB = XROWS * 128;                // one x block image
constexpr int ZROW = PX;                       // zero row of a z block image
constexpr int ZB = (PX + 1) * 128;             // one z block image (frame-major rows 17 f + w)
constexpr int XOFF = 0, ZOFF = 2 * XB, B2OFF = ZOFF + 2 * ZB;
constexpr int SMEM = B2OFF + V * 64 * 4;       // 147,968 B: one workgroup per CU
constexpr int NX = 2 * XROWS / 8 / 8;          // x DMA instructions per wave per tile (9)
constexpr int NRL = 16;                        // residual loads per wave per tile (8 fragments x hi, lo)
constexpr int NST = 8;                         // line stores per wave per tile
static_assert(NX * 8 * 8 == 2 * XROWS, "x image DMA split");
static_assert(2 * 256 * 128 <= 2 * ZB, "out image over the z image");
static_assert(SMEM <= 160 * 1024, "LDS");
}  // namespace s2

__global__ __launch_bounds__(512, 2) void stb2_kernel(StbArgs a, int ntiles) {
    using namespace s2;
    __shared__ __attribute__((aligned(16))) unsigned char smem[SMEM];   // the only LDS object
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int QO = a.nwin * a.T, M = QO * V;
    // debug (a.trace): per-workgroup phase sums over its tiles, in s_memrealtime ticks
    unsigned long long tr_g = 0, tr_mix = 0, tr_t = 0, tr_epi = 0;
    const unsigned long long ts_start = a.trace ? __builtin_amdgcn_s_memrealtime() : 0;

    int t_begin, t_end;   // this workgroup's contiguous run of tiles (runs ordered per XCD)
    {
        const int G = gridDim.x, bid = blockIdx.x;
        const int per = G >> 3, rem = G & 7, x = bid & 7, k = bid >> 3;
        const int s = x < rem ? x * (per + 1) + k : rem * (per + 1) + (x - rem) * per + k;
        t_begin = (int)((long long)s * ntiles / G);
        t_end = (int)((long long)(s + 1) * ntiles / G);
    }

    // ---- stationary operands. cb = this wave's 16-channel block; G on waves 0-3 only.
    const int cb = wave & 3;
    f16x8 wgh[2], wgl[2], wth[6], wtl[6];
    {
        const int co = 16 * cb + (lane & 15), g0 = lane >> 4;
#pragma unroll
        for (int kb = 0; kb < 2; ++kb) {
            const unsigned short* p = a.wg + (size_t)co * a.ldwg + kb * 64 + 8 * g0;
            wgh[kb] = *reinterpret_cast<const f16x8*>(p);
            wgl[kb] = *reinterpret_cast<const f16x8*>(p + 32);
        }
#pragma unroll
        for (int s = 0; s < 6; ++s) {   // K step s = tap * 2 + block: SB weights [Cout][tap][block][64]
            const unsigned short* p = a.wt + (size_t)co * a.ldwt + s * 64 + 8 * g0;
            wth[s] = *reinterpret_cast<const f16x8*>(p);
            wtl[s] = *reinterpret_cast<const f16x8*>(p + 32);
        }
    }
    f32x4 bias_t = *reinterpret_cast<const f32x4*>(a.bias + 16 * cb + 4 * (lane >> 4));
    constexpr int NAM = (V * V + 63) / 64;   // A_eff in registers, read back with v_readlane
    float amv[NAM];
#pragma unroll
    for (int k = 0; k < NAM; ++k) amv[k] = 64 * k + lane < V * V ? a.amix[64 * k + lane] : 0.f;
    float* b2s = reinterpret_cast<float*>(smem + B2OFF);
    for (int i = tid; i < V * 64; i += 512) b2s[i] = a.bias2[i];
    if (tid < 16) *reinterpret_cast<f32x4*>(smem + ZOFF + (tid >> 3) * ZB + ZROW * 128 + (tid & 7) * 16) = f32x4{0.f, 0.f, 0.f, 0.f};
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) asm volatile("" : "+v"(wgh[kb]), "+v"(wgl[kb]));
#pragma unroll
    for (int s = 0; s < 6; ++s) asm volatile("" : "+v"(wth[s]), "+v"(wtl[s]));
    asm volatile("" : "+v"(bias_t));
#pragma unroll
    for (int k = 0; k < NAM; ++k) asm volatile("" : "+v"(amv[k]));
    lds_barrier();

    // ---- x image DMA: 2 blocks x 36 instructions of 8 rows, 9 per wave
    const i32x4 rX = buf_rsrc(a.x, (unsigned)((long long)M * a.ldx * 2));
    auto issue_x = [&](int tile) {   // tile < 0: a dummy (zero fill)
        const int fi0 = tile * F - 1;
#pragma unroll
        for (int j = 0; j < NX; ++j) {
            const int idx = wave * NX + j, blk = idx / (XROWS / 8), rg = idx % (XROWS / 8);
            const int rr = rg * 8 + (lane >> 3), ck = (lane & 7) ^ sbf(rr);
            const int f = rr & 15, v = rr >> 4;
            const long long gr = (long long)(fi0 + f) * V + v;
            const unsigned off = (tile >= 0 && rr < PX && fi0 + f >= 0 && gr < M)
                                     ? (unsigned)((gr * a.ldx + blk * 64 + 8 * ck) * 2) : DMA_OOB;
            dma16(rX, smem + XOFF + blk * XB + rg * 1024, off, 0);
        }
    };

    if (t_begin < t_end) issue_x(t_begin);
    int prev_st = 0;   // stores issued after the last x DMA
    for (int tile = t_begin; tile < t_end; ++tile) {
        const int q0 = tile * F;
        const int nxt = tile + 1 < t_end ? tile + 1 : -1;
        const unsigned long long ts0 = a.trace ? __builtin_amdgcn_s_memrealtime() : 0;
        // lane-derived offsets re-derived per tile from an opaque copy (hoisted, they stay live and spill)
        int lt = lane, ldo = a.ldo, ldx = a.ldx;
        asm volatile("" : "+v"(lt), "+s"(ldo), "+s"(ldx));
        const int l15 = lt & 15, g = lt >> 4;
        unsigned short* trash = a.trash + (((wave << 6) + lt) & 255) * 8;

        // (1) x(tile) landed (younger: the last tile's stores)
        wait_vm_dyn(prev_st);
        lds_barrier();
        // (2) G: y^T = Wg'^T x^T on waves 0-3 (channel block = wave): fragment j = joint j of the
        // 16 frames, lane -> frame l15, channels 4g..4g+3 of the block; B3_64's product order
        f32x4 accg[V];
#pragma unroll
        for (int j = 0; j < V; ++j) accg[j] = f32x4{0.f, 0.f, 0.f, 0.f};
        if (wave < 4) {
            f16x8 gbh[3], gbl[3];
            auto load_x = [&](int n) {   // n = kb * 17 + joint
                const unsigned char* X = smem + XOFF + (n / V) * XB;
                const int rx = (n % V) * 16 + l15;
                gbh[n % 3] = *reinterpret_cast<const f16x8*>(X + sbo(rx, g));
                gbl[n % 3] = *reinterpret_cast<const f16x8*>(X + sbo(rx, 4 + g));
            };
            load_x(0);
            load_x(1);
#pragma unroll
            for (int kb = 0; kb < 2; ++kb) {
#pragma unroll
                for (int j = 0; j < V; ++j) {
                    const int n = kb * V + j;
                    if (n + 2 < 2 * V) load_x(n + 2);
                    const f16x8 bh = gbh[n % 3], bl = gbl[n % 3];
                    accg[j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wgl[kb], bh, accg[j], 0, 0, 0);
                    accg[j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wgh[kb], bl, accg[j], 0, 0, 0);
                    accg[j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wgh[kb], bh, accg[j], 0, 0, 0);
                    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                    __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
                    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                    __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
                    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                }
            }
        }
        lds_barrier();   // every read of x(tile) done: the image may take x(tile+1)
        const unsigned long long ts1 = a.trace ? __builtin_amdgcn_s_memrealtime() : 0;
        const int half = wave >> 2, c0 = 16 * cb + 4 * g;
        // (4) mix in registers (waves 0-3): z[w] = ReLU(bias2[w] + sum_v A[v][w] y[v]) -> z image
        if (wave < 4) {
            const int mc = 16 * cb + 4 * g, cc = mc & 31;
            unsigned char* zb = smem + ZOFF + (mc >> 5) * ZB + (cc & 4) * 2;
            const int uh = cc >> 3;
            auto mix_all = [&](auto sparse_tag) {
                constexpr bool SP = decltype(sparse_tag)::value;
#pragma unroll
                for (int w = 0; w < V; ++w) {
                    f32x4 z = *reinterpret_cast<const f32x4*>(b2s + w * 64 + mc);
#pragma unroll
                    for (int v = 0; v < V; ++v)
                        if (!SP || ((coco_hop2_mask3(w) >> v) & 1u)) {
                            const float av = __builtin_bit_cast(
                                float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, amv[(v * V + w) / 64]), (v * V + w) % 64));
                            z += av * accg[v];
                        }
#pragma unroll
                    for (int e = 0; e < 4; ++e) z[e] = z[e] > 0.f ? z[e] : 0.f;
                    f16x4 h, l;
                    split4(z, h, l);
                    const int row = l15 * V + w;
                    *reinterpret_cast<f16x4*>(zb + sbo(row, uh)) = h;
                    *reinterpret_cast<f16x4*>(zb + sbo(row, 4 + uh)) = l;
                }
            };
            if (a.mix_sparse) mix_all(std::true_type{});
            else mix_all(std::false_type{});
        }
        lds_barrier();
        const unsigned long long ts2 = a.trace ? __builtin_amdgcn_s_memrealtime() : 0;
        // (5) T (transposed): this wave's 16 channels x fragments 8 half .. 8 half + 7 (< 15);
        // tap k of pixel p = z row p + 17 k, or the zero row past the window edge
        unsigned tmask = 0;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int fr = 8 * half + i, p = 16 * fr + l15, f = p / V;
            const int q = q0 + f, t = q % a.T;
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                const bool ok = fr < NTF && p < TR && q < QO && t + k - 1 >= 0 && t + k - 1 < a.T;
                tmask |= (ok ? 1u : 0u) << (3 * i + k);
            }
        }
        f32x4 acc[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
        // this tile's identity residual (L2-hot: x was just DMA'd) and then x(tile+1): issued
        // inside the tap-0 MFMAs below, their issue cost hidden; every load is issued (rows clamped)
        f32x2 rh[8], rl[8];
        auto load_resid = [&](int i) {
            const int p = 16 * (8 * half + i) + l15;
            const int R = min(q0 * V + min(p, TR - 1), M - 1);
            const unsigned short* rp = a.x + (size_t)R * ldx + sbc(c0);
            rh[i] = *reinterpret_cast<const f32x2*>(rp);
            rl[i] = *reinterpret_cast<const f32x2*>(rp + 32);
        };
        int bo[2][8];
        auto tap_offsets = [&](int tap, int* o) {
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const int p = 16 * (8 * half + i) + l15;
                o[i] = sbo(((tmask >> (3 * i + tap)) & 1u) ? p + V * tap : ZROW, g);
            }
        };
        tap_offsets(0, bo[0]);
        constexpr int NSTEP = 3 * 2 * 8;   // (tap, block, fragment)
        f16x8 pbh[3], pbl[3];
        auto load_b = [&](int n) {
            const int tap = n / 16, kb = (n / 8) % 2, i = n % 8;
            const unsigned char* B = smem + ZOFF + kb * ZB;
            const int o = bo[tap & 1][i];
            pbh[n % 3] = *reinterpret_cast<const f16x8*>(B + o);
            pbl[n % 3] = *reinterpret_cast<const f16x8*>(B + (o ^ 64));
        };
        load_b(0);
        load_b(1);
#pragma unroll
        for (int tap = 0; tap < 3; ++tap) {
#pragma unroll
            for (int kb = 0; kb < 2; ++kb) {
#pragma unroll
                for (int i = 0; i < 8; ++i) {
                    const int n = (tap * 2 + kb) * 8 + i;
                    if (kb == 0 && i == 0 && tap + 1 < 3) tap_offsets(tap + 1, bo[(tap + 1) & 1]);
                    if (n + 2 < NSTEP) load_b(n + 2);
                    const int s = tap * 2 + kb;
                    const f16x8 bh = pbh[n % 3], bl = pbl[n % 3];
                    acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wth[s], bl, acc[i], 0, 0, 0);
                    acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wtl[s], bh, acc[i], 0, 0, 0);
                    acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wth[s], bh, acc[i], 0, 0, 0);
                    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                    __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
                    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                    __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
                    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                    if (tap == 0 && kb == 0) load_resid(i);
                    if (tap == 0 && kb == 1 && i == 7) issue_x(nxt);
                }
            }
        }
        lds_barrier();   // every z read done: the out image goes over the z image
        const unsigned long long ts3 = a.trace ? __builtin_amdgcn_s_memrealtime() : 0;
        // (6) out = ReLU(C + bias + x) -> split image (residual loads landed: younger = x(tile+1))
        wait_vm_dyn(NX);
        {
            const int ob = c0 >> 5, cc = c0 & 31, uh = cc >> 3, sub = (cc & 7) * 2;
            unsigned char* ib = smem + ZOFF + ob * ZB;
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const int p = 16 * (8 * half + i) + l15;
                f32x4 v = acc[i] + bias_t;
                const f16x4 h = __builtin_bit_cast(f16x4, rh[i]);
                const f16x4 l = __builtin_bit_cast(f16x4, rl[i]);
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    v[e] += (float)h[e] + (float)l[e];
                    v[e] = v[e] > 0.f ? v[e] : 0.f;
                }
                f16x4 oh, ol;
                split4(v, oh, ol);
                if (p < 256) {
                    *reinterpret_cast<f16x4*>(ib + sbo(p, uh) + sub) = oh;
                    *reinterpret_cast<f16x4*>(ib + sbo(p, 4 + uh) + sub) = ol;
                }
            }
        }
        lds_barrier();
        // (7) out -> HBM in whole 128-B lines (8 per thread; rows past the tile to the trash line)
#pragma unroll
        for (int q = 0; q < NST; ++q) {
            const int idx = (wave << 6) + lt + 512 * q;
            const int b = idx >> 11, r = (idx & 2047) >> 3, u = idx & 7;
            const f32x4 d = *reinterpret_cast<const f32x4*>(smem + ZOFF + b * ZB + sbo(r, u));
            const bool ok = r < TR && q0 * V + r < M;
            unsigned short* o = ok ? a.out + (size_t)(q0 * V + r) * ldo + b * 64 + u * 8 : trash;
            *reinterpret_cast<f32x4*>(o) = d;
        }
        prev_st = NST;
        if (a.trace) {
            const unsigned long long ts4 = __builtin_amdgcn_s_memrealtime();
            tr_g += ts1 - ts0; tr_mix += ts2 - ts1; tr_t += ts3 - ts2; tr_epi += ts4 - ts3;
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (a.trace && tid == 0) {   // {tiles, wait+G, residual+x DMA+mix, T, epilogue, span}
        unsigned long long* tr = a.trace + 6 * (size_t)blockIdx.x;
        tr[0] = (unsigned long long)(t_end - t_begin);
        tr[1] = tr_g; tr[2] = tr_mix; tr[3] = tr_t; tr[4] = tr_epi;
        tr[5] = __builtin_amdgcn_s_memrealtime() - ts_start;
    }
}

static int cu_count2() {
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

hipError_t launch_stb2(const StbArgs& a, hipStream_t st) {
    if (a.nwin <= 0 || a.T <= 0) return hipSuccess;
    const long long M = (long long)a.nwin * a.T * 17;
    if (!a.x || !a.wg || !a.wt || !a.bias || !a.bias2 || !a.amix || !a.out || !a.trash || !a.resid || a.ldx % 8 ||
        a.ldx < 128 || a.ldo % 8 || a.ldo < 128 || a.ldwg < 128 || a.ldwt < 384 || a.ldwg % 8 || a.ldwt % 8 ||
        M * a.ldx * 2 >= 0x80000000LL)
        return hipErrorInvalidValue;
    const int ntiles = (a.nwin * a.T + s2::F - 1) / s2::F;
    const int grid = ntiles < cu_count2() ? ntiles : cu_count2();
    (void)hipGetLastError();
    hipLaunchKernelGGL(stb2_kernel, dim3(grid), dim3(512), 0, st, a, ntiles);
    return hipGetLastError();
}

}  // namespace tik
