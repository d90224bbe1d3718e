// xtconv.hip — tcn conv (3 x 1 over frames, stride 1, 128 -> 128 channels) +
// folded BN + identity residual + ReLU of an ST-GCN block
// (st_gcn_aaai18.py:180-189: tcn = BN-ReLU-Conv(3x1)-BN-Dropout, + residual,
// ReLU), bf16x3 on MFMA, as one persistent launch with the weights RESIDENT.
//
// The tiled kernel (xgemm_kernel, XT128) streams a 24 KB weight stage from L2
// into LDS for every K step of every 128 x 128 tile and pays a DMA round trip
// and an LDS-staged epilogue per tile. Here a workgroup owns one 64-channel
// half of the output for a contiguous range of rows: its 147 KB of weight
// planes (64 channels x 3 taps x 128 channels x 3 bf16 planes) are loaded into
// LDS once, and then every wave runs on its own — no barrier after the weight
// load:
//   * a wave takes blocks of 32 output rows (two 16-row MFMA fragments) and
//     walks the 12 K steps (tap-major, 32 channels per step: xgemm's K order);
//   * its A operand comes straight from HBM/L2 into registers (8 consecutive
//     channels of its pixel row per lane), 3 steps ahead, and is split into the
//     three bf16 planes in registers (no LDS round trip for activations), one
//     step ahead: step s+1's split runs between step s's MFMAs, so no MFMA
//     waits on the VALU chain of its own operands;
//   * taps outside the window read zeros (out-of-range buffer offsets);
//   * the epilogue works on the accumulators: (acc + x) + bias, ReLU, 16-B
//     stores; the residual rows are loaded 4 steps before the block ends.
// MFMA transposed (A = weights: lane = pixel (l & 15), 4 channels 4 (l >> 4)),
// products (w0,x2) (w1,x1) (w2,x0) (w0,x1) (w1,x0) (w0,x0) as xgemm: the same
// bits as the XT128 path.
#include <algorithm>

#include "xgemm_dev.h"
#include "xtconv.h"

namespace tik {

namespace xtc {
constexpr int V = 17, NS = 12, NCB = 4, RB = 32, D = 3;
constexpr int WBYTES = NCB * NS * 3 * 1024;   // 147,456
static_assert(NS % D == 0, "prefetch ring indices are static per step");
}  // namespace xtc

__device__ f32x4 tik_llvm_raw_buffer_load_v4f32_xtc(i32x4 rsrc, int voffset, int soffset, int aux)
    __asm("llvm.amdgcn.raw.buffer.load.v4f32");

#ifdef TIK_XTUNE
#define XTC_OFF(bit) (a.tune & (bit))
#else
#define XTC_OFF(bit) false
#endif

__global__ __launch_bounds__(512, 1) void xtconv_kernel(XTConvArgs a) {
    using namespace xtc;
    __shared__ __attribute__((aligned(16))) unsigned char wsm[WBYTES];
    int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int G = gridDim.x, b = blockIdx.x;
    // workgroups b and b + 8 run on the same XCD: the two column halves of one row range
    const int nk = G >> 3, xcd = b & 7, k = b >> 3, half = k & 1;
    const int NR = G >> 1, rid = xcd * (nk >> 1) + (k >> 1);
    const int M = a.M;
    const int nblk = (M + RB - 1) / RB;
    const int b0 = (int)((long long)rid * nblk / NR), b1 = (int)((long long)(rid + 1) * nblk / NR);

    // ---- this half's weight planes into LDS (cg 4 half .. 4 half + 3 are contiguous)
    {
        const f32x4* src = reinterpret_cast<const f32x4*>(a.wp) + (size_t)half * (WBYTES / 16);
        f32x4* dst = reinterpret_cast<f32x4*>(wsm);
#pragma unroll 6
        for (int i = tid; i < WBYTES / 16; i += 512) dst[i] = src[i];
    }
    const int g = lane >> 4, l15 = lane & 15;
    const int col0 = half * 64 + 4 * g;   // + 16 cb
    f32x4 bv[NCB];
#pragma unroll
    for (int cb = 0; cb < NCB; ++cb) bv[cb] = *reinterpret_cast<const f32x4*>(a.bias + col0 + 16 * cb);
    __syncthreads();

    const int nmy = b1 - b0 > wave ? (b1 - b0 - wave + 7) / 8 : 0;
    if (nmy == 0) return;
    const int total = nmy * NS;
    const i32x4 rZ = buf_rsrc(a.z, (unsigned)((long long)M * a.ldz * 4));

    // per block: the byte offsets of this lane's two pixel rows for the 3 taps (OOB: zeros)
    auto offsets = [&](int ib, unsigned (&o)[3][2]) __attribute__((always_inline)) {
        const int blk = b0 + wave + 8 * ib;
        const bool live = ib < nmy;
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int px = blk * RB + 16 * i + l15;
            const int t = (px / V) % a.T;
#pragma unroll
            for (int tap = 0; tap < 3; ++tap) {
                const bool ok = live && px < M && t + tap - 1 >= 0 && t + tap - 1 < a.T;
                o[tap][i] = ok ? (unsigned)((long long)(px + (tap - 1) * V) * a.ldz * 4 + 32 * g) : DMA_OOB;
            }
        }
    };
    unsigned oc[3][2], on[3][2];   // this block's / the next block's
    f32x4 ra[D][2][2];
    auto load = [&](const unsigned (&o)[3][2], int s, f32x4 (&r)[2][2]) __attribute__((always_inline)) {
        const int tap = s / 4, kb = s % 4;
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const unsigned off = o[tap][i];
            const int so = kb * 128;
            if (XTC_OFF(1)) {
                r[i][0] = f32x4{1.f, 1.f, 1.f, 1.f};
                r[i][1] = r[i][0];
                continue;
            }
            r[i][0] = tik_llvm_raw_buffer_load_v4f32_xtc(rZ, (int)off, so, 0);
            r[i][1] = tik_llvm_raw_buffer_load_v4f32_xtc(rZ, (int)off, so + 16, 0);
        }
    };
    offsets(0, oc);
    offsets(1, on);
#pragma unroll
    for (int s = 0; s < D; ++s) load(oc, s, ra[s]);
    // bf16 planes of the A fragments, double buffered by step parity
    xbf16x8 xp[2][2][3];
#pragma unroll
    for (int i = 0; i < 2; ++i) xsplit8(ra[0][i][0], ra[0][i][1], xp[0][i][0], xp[0][i][1], xp[0][i][2]);
    load(oc, D, ra[0]);

    f32x4 acc[2][NCB];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int cb = 0; cb < NCB; ++cb) acc[i][cb] = f32x4{0.f, 0.f, 0.f, 0.f};

    for (int ib = 0; ib < nmy; ++ib) {
        asm volatile("" : "+v"(tid), "+v"(lane));   // lane-derived values: recomputed per block (register pressure)
        const int blk = b0 + wave + 8 * ib;
        f32x4 xr[2][NCB];
#pragma unroll
        for (int s = 0; s < NS; ++s) {
            // step s's planes were split during step s-1; step s+1's rows (ring slot
            // (s+1) % D, loaded D steps ago) are split between this step's MFMAs, then
            // the slot takes step s+1+D's rows
            const xbf16x8(&x0)[2][3] = xp[s & 1];
            auto split_next = [&](int i) __attribute__((always_inline)) {
                if (XTC_OFF(2)) return;
                xsplit8(ra[(s + 1) % D][i][0], ra[(s + 1) % D][i][1], xp[(s + 1) & 1][i][0], xp[(s + 1) & 1][i][1],
                        xp[(s + 1) & 1][i][2]);
            };
            if (s == NS - D) {   // the residual rows of this block (clamped rows past M: discarded)
#pragma unroll
                for (int i = 0; i < 2; ++i) {
                    const int px = blk * RB + 16 * i + l15;
                    const int pr = px < M ? px : 0;
#pragma unroll
                    for (int cb = 0; cb < NCB; ++cb)
                        xr[i][cb] = *reinterpret_cast<const f32x4*>(a.x + (size_t)pr * a.ldx + col0 + 16 * cb);
                }
            }
            // MFMAs: column block cb's weight planes (ring of two)
            const unsigned char* W = wsm + (size_t)s * 3 * 1024 + lane * 16;
            xbf16x8 wb[2][3];
#pragma unroll
            for (int p = 0; p < 3; ++p) wb[0][p] = *reinterpret_cast<const xbf16x8*>(W + p * 1024);
#pragma unroll
            for (int cb = 0; cb < NCB; ++cb) {
                if (cb + 1 < NCB)
#pragma unroll
                    for (int p = 0; p < 3; ++p)
                        wb[(cb + 1) & 1][p] = *reinterpret_cast<const xbf16x8*>(W + (size_t)(cb + 1) * NS * 3 * 1024 + p * 1024);
                __builtin_amdgcn_sched_barrier(0);
                const xbf16x8(&w)[3] = wb[cb & 1];
#pragma unroll
                for (int i = 0; i < 2; ++i) {
                    if (XTC_OFF(4)) break;
                    const xbf16x8(&x)[3] = x0[i];
                    acc[i][cb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[0], x[2], acc[i][cb], 0, 0, 0);
                    acc[i][cb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[1], x[1], acc[i][cb], 0, 0, 0);
                    acc[i][cb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[2], x[0], acc[i][cb], 0, 0, 0);
                    acc[i][cb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[0], x[1], acc[i][cb], 0, 0, 0);
                    acc[i][cb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[1], x[0], acc[i][cb], 0, 0, 0);
                    acc[i][cb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[0], x[0], acc[i][cb], 0, 0, 0);
                }
                // the next step's split, one fragment per column block, under these MFMAs
                if (cb < 2) split_next(cb);
                if (cb == 1) {   // ring slot (s+1) % D is free: step s+1+D's rows
                    if (s + 1 + D < NS) load(oc, s + 1 + D, ra[(s + 1) % D]);
                    else load(on, s + 1 + D - NS, ra[(s + 1) % D]);
                }
                __builtin_amdgcn_sched_barrier(0);
            }
        }
        // ---- epilogue: (acc + x) + bias, ReLU (xgemm's identity-epilogue order)
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int px = blk * RB + 16 * i + l15;
#pragma unroll
            for (int cb = 0; cb < NCB; ++cb) {
                f32x4 v = acc[i][cb] + xr[i][cb];
                v += bv[cb];
#pragma unroll
                for (int e = 0; e < 4; ++e) v[e] = v[e] > 0.f ? v[e] : 0.f;
                float* o = px < M ? a.out + (size_t)px * a.ldo + col0 + 16 * cb : a.trash + (tid & 255) * 4;
                if (!XTC_OFF(8)) xst4(o, v, a.nts);
                acc[i][cb] = f32x4{0.f, 0.f, 0.f, 0.f};
            }
        }
#pragma unroll
        for (int tap = 0; tap < 3; ++tap)
#pragma unroll
            for (int i = 0; i < 2; ++i) oc[tap][i] = on[tap][i];
        offsets(ib + 2, on);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

bool xtconv_ok(const XTConvArgs& a) {
    return a.T > 0 && a.ldz % 4 == 0 && a.ldz >= 128 && a.ldx % 4 == 0 && a.ldx >= 128 && a.ldo % 4 == 0 && a.ldo >= 128;
}

hipError_t launch_xtconv(const XTConvArgs& a, int ncu, hipStream_t st) {
    if (a.M <= 0) return hipSuccess;
    if (!xtconv_ok(a) || !a.z || !a.x || !a.wp || !a.bias || !a.out || !a.trash || a.M % (17 * a.T) != 0) return hipErrorInvalidValue;
    // the buffer offsets are 32-bit: launches of whole windows, < 2 GiB of conv input rows each
    const long long win = 17LL * a.T, win_bytes = win * a.ldz * 4;
    const long long wper = std::max(1LL, ((1LL << 31) - 1) / win_bytes);
    const long long rows_per = wper * win;
    if (win_bytes >= (1LL << 31)) return hipErrorInvalidValue;
    int grid = std::max(16, (ncu / 16) * 16);   // 8 XCDs x an even number per XCD
    (void)hipGetLastError();
    for (long long r0 = 0; r0 < a.M; r0 += rows_per) {
        XTConvArgs c = a;
        c.M = (int)std::min(rows_per, (long long)a.M - r0);
        c.z = a.z + (size_t)r0 * a.ldz;
        c.x = a.x + (size_t)r0 * a.ldx;
        c.out = a.out + (size_t)r0 * a.ldo;
        hipLaunchKernelGGL(xtconv_kernel, dim3(grid), dim3(512), 0, st, c);
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

}  // namespace tik
