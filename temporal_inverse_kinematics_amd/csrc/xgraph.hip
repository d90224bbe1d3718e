// xgraph.hip — the spatial half of an ST-GCN block (gcn 1x1 conv + the 17 x 17
// graph mix + folded BN + ReLU: st_gcn_aaai18.py:178-179, gconv_origin.py:56-65)
// as one persistent, weight-stationary bf16x3 launch.
//
// The tiled G kernel (xgemm_kernel<EPI_GRAPH>) spends half its time outside
// the MFMA loop: the first DMA round trip of every tile and an epilogue that
// stages the whole C tile through LDS so the mix can gather the 17 joints of a
// frame across waves. Here:
//   * weights in registers: wave w owns 16 output channels (its Wg' planes in
//     the MFMA operand layout, xblock_pack_weights), so no weight DMA at all;
//   * MFMA transposed with JOINT-MAJOR pixel blocks (block j = joint j of the
//     tile's 16 frames): each lane ends with y for one frame, 4 channels and
//     all 17 joints, so the mix + bias2 + ReLU run in registers, no C tile;
//   * the fp32 rows of one K step (16 frames x 17 joints x 32 channels) arrive
//     by LDS-DMA in a staging slot and are split ONCE, cooperatively, into an
//     LDS image of bf16 planes that all eight waves read (split on read, each
//     wave would split every element again); the planes image is double-
//     buffered, so step k+1's split runs beside step k's MFMAs, and the DMA of
//     step k+2 lands during step k+1 — across tile boundaries (persistent).
// Products, K order and mix order as the tiled kernel (bf16x3 six products,
// fp32 accumulation; bias2 then v ascending).
// Tiles: (16-frame group, pass): a 256-channel output runs as two passes of
// 128 channels (eight waves x 16). Frames are flattened over windows (a 1x1
// conv has no temporal taps, so tiles may straddle windows).
#include <algorithm>
#include <type_traits>

#include "xgemm_dev.h"
#include "xgraph.h"

namespace tik {

namespace xg {
constexpr int V = 17, FR = 16, PX = FR * V;          // frames per tile, pixels (272)
constexpr int SBYTES = PX * 128;                     // fp32 staging of one K step (32 channels)
constexpr int SINST = SBYTES / 1024;                 // 34 DMA instructions
constexpr int PROWB = 3 * 32 * 2;                    // planes image row: 3 planes x 32 channels x 2 B
constexpr int PBYTES = PX * PROWB;                   // 52,224
constexpr int NCHUNK = PX * 4;                       // split work items: 8-channel chunks
}  // namespace xg

// planes image: row R = 16 j + f (joint-major), unit (plane p, K group u) at
// p * 4 + (u ^ ((R >> 1) & 3)): conflict-free b128 reads of 16 consecutive rows
__device__ __forceinline__ int xg_unit(int R, int p, int u) { return R * xg::PROWB + ((p * 4 + (u ^ ((R >> 1) & 3))) << 4); }

template <int NK>
__global__ __launch_bounds__(512, 1) void xgraph_kernel(XGraphArgs a) {
    using namespace xg;
    constexpr int B2MAX = V * 256 * 4;
    __shared__ __attribute__((aligned(16))) unsigned char smem[SBYTES + 2 * PBYTES + B2MAX];
    unsigned char* const stg = smem;
    float* const b2s = reinterpret_cast<float*>(smem + SBYTES + 2 * PBYTES);
    auto pimg = [&](int s) __attribute__((always_inline)) { return smem + SBYTES + (s & 1) * PBYTES; };

    int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int QO = a.nframes, M = QO * V;
    const int npass = a.cout / 128;
    const int nfg = (QO + FR - 1) / FR;
    const int ntiles = nfg * npass;
    int t_begin, t_end;
    {   // persistent: a contiguous run of tiles per workgroup, runs ordered per XCD
        const int nwg = gridDim.x, bid = blockIdx.x;
        const int per = nwg >> 3, rem = nwg & 7, x = bid & 7, k = bid >> 3;
        const int s = x < rem ? x * (per + 1) + k : rem * (per + 1) + (x - rem) * per + k;
        t_begin = (int)((long long)s * ntiles / nwg);
        t_end = (int)((long long)(s + 1) * ntiles / nwg);
    }
    if (t_begin >= t_end) return;
    const int total = (t_end - t_begin) * NK;   // global K steps of this workgroup
    // tile -> (frame group, pass): passes innermost, so a frame group's x rows
    // are read twice back to back (the second time from L2)
    auto tile_fg = [&](int t) __attribute__((always_inline)) { return t / npass; };
    auto tile_pass = [&](int t) __attribute__((always_inline)) { return t - (t / npass) * npass; };

    // bias2 [17][cout] and A_eff in VGPRs (v_readlane) before any DMA
    for (int i = tid; i < V * a.cout; i += 512) b2s[i] = a.bias2[i];
    float amv[5];
#pragma unroll
    for (int k = 0; k < 5; ++k) amv[k] = 64 * k + lane < V * V ? a.amix[64 * k + lane] : 0.f;
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");

    // ---- the fp32 rows of global step s (tile t_begin + s / NK, K block s % NK) into the staging slot
    const i32x4 rX = buf_rsrc(a.x, (unsigned)((long long)M * a.ldx * 4));
    auto issue = [&](int s) __attribute__((always_inline)) {
        const int t = t_begin + s / NK, kb = s - (s / NK) * NK;
        const int q0 = tile_fg(t) * FR;
#pragma unroll
        for (int i = 0; i < (SINST + 7) / 8; ++i) {
            const int ins = wave + 8 * i;
            if (ins >= SINST) break;
            const int U = ins * 64 + lane;            // staging unit: row U / 8 (R = 16 j + f), unit U % 8
            const int R = U >> 3, u = U & 7, j = R >> 4, f = R & 15, q = q0 + f;
            const unsigned off = q < QO ? (unsigned)(((long long)q * V + j) * a.ldx * 4 + kb * 128 + u * 16) : DMA_OOB;
            dma16(rX, stg + ins * 1024, off, 0);
        }
    };
    // ---- split this wave's staging rows (the rows its own DMA instructions
    // fill: ins = wave + 8 i) into planes image (s & 1); chunk = 8 channels of a row
    auto split = [&](int s) __attribute__((always_inline)) {
        unsigned char* P = pimg(s);
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            const int ins = wave + 8 * (2 * i + (lane >> 5));
            if (ins < SINST) {
                const int R = 8 * ins + ((lane & 31) >> 2), u = lane & 3;
                const f32x4 lo = *reinterpret_cast<const f32x4*>(stg + R * 128 + u * 32);
                const f32x4 hi = *reinterpret_cast<const f32x4*>(stg + R * 128 + u * 32 + 16);
                xbf16x8 p0, p1, p2;
                xsplit8(lo, hi, p0, p1, p2);
                *reinterpret_cast<xbf16x8*>(P + xg_unit(R, 0, u)) = p0;
                *reinterpret_cast<xbf16x8*>(P + xg_unit(R, 1, u)) = p1;
                *reinterpret_cast<xbf16x8*>(P + xg_unit(R, 2, u)) = p2;
            }
        }
    };

    // weights of this wave's 16 channels for the current pass (re-loaded when the pass changes)
    xbf16x8 w[NK][3];
    auto load_w = [&](int pass) __attribute__((always_inline)) {
        const int cg = pass * 8 + wave;
        const unsigned short* wp = a.wp;
#pragma unroll
        for (int kb = 0; kb < NK; ++kb)
#pragma unroll
            for (int p = 0; p < 3; ++p)
                w[kb][p] = *reinterpret_cast<const xbf16x8*>(wp + ((((size_t)cg * NK + kb) * 3 + p) * 64 + lane) * 8);
    };

    // prologue: weights; step 0 -> staging -> planes[0]; step 1 into the staging
    // rows. A wave only ever reads the staging rows its own DMA fills, so the
    // staging needs no barrier: each wave refills its rows right after its split.
    load_w(tile_pass(t_begin));
    issue(0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    split(0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (1 < total) issue(1);

    f32x4 acc[V];
#pragma unroll
    for (int j = 0; j < V; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
    // vector-memory ops this wave issued after its DMA of the next step (weight
    // loads, epilogue stores): they may stay in flight at that DMA's wait
    int n_after = 0;
    auto wait_after = [&](int n) __attribute__((always_inline)) {   // n in {0, V, 3 NK, 3 NK + V}
        if (n == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        else if (n == V) asm volatile("s_waitcnt vmcnt(17)" ::: "memory");
        else if (n == 3 * NK) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(3 * NK) : "memory");
        else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(3 * NK + V) : "memory");
    };

    // one K step; KB compile-time so the weights stay in registers (a runtime
    // index into w[][] puts the array in scratch)
    auto step = [&](int s, int t, int pass, auto KBc) __attribute__((always_inline)) {
        constexpr int kb = decltype(KBc)::value;
        asm volatile("" : "+v"(tid), "+v"(lane));   // lane-derived addresses: not hoisted across steps (spills)
        const int g = lane >> 4, f = lane & 15;
        // every wave's split(s) landed; every wave done with step s-1's planes (the buffer split(s+1) writes).
        // s_barrier alone: __syncthreads' release fence would wait for the DMA in flight
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        // MFMAs of step s (planes s & 1), the split of step s+1 (planes (s+1) & 1) beside them
        const unsigned char* P = pimg(s);
        xbf16x8 xb[2][3];
        auto rd = [&](int j, xbf16x8 (&d)[3]) __attribute__((always_inline)) {
#pragma unroll
            for (int p = 0; p < 3; ++p) d[p] = *reinterpret_cast<const xbf16x8*>(P + xg_unit(16 * j + f, p, g));
        };
        auto mfma_j = [&](int j) __attribute__((always_inline)) {
            if (j + 1 < V) rd(j + 1, xb[(j + 1) & 1]);
            const xbf16x8(&x)[3] = xb[j & 1];
            // (w0,x2) (w1,x1) (w2,x0) (w0,x1) (w1,x0) (w0,x0): xgemm's product order
            acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[kb][0], x[2], acc[j], 0, 0, 0);
            acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[kb][1], x[1], acc[j], 0, 0, 0);
            acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[kb][2], x[0], acc[j], 0, 0, 0);
            acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[kb][0], x[1], acc[j], 0, 0, 0);
            acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[kb][1], x[0], acc[j], 0, 0, 0);
            acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[kb][0], x[0], acc[j], 0, 0, 0);
            __builtin_amdgcn_sched_barrier(0);
        };
        rd(0, xb[0]);
#pragma unroll
        for (int j = 0; j < 4; ++j) mfma_j(j);
        if (s + 1 < total) {
            // this wave's rows of step s+1 landed (DMA issued one step ago): split them beside the MFMAs
            wait_after(n_after);
            n_after = 0;
            split(s + 1);
        }
#pragma unroll
        for (int j = 4; j < 8; ++j) mfma_j(j);
        if (s + 2 < total) {
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // the split's staging reads done
            issue(s + 2);
        }
#pragma unroll
        for (int j = 8; j < V; ++j) mfma_j(j);
        if (kb == NK - 1 && s + 1 < total && tile_pass(t + 1) != pass) {
            load_w(tile_pass(t + 1));   // the next tile's pass: behind the DMA, ahead of the stores
            n_after += NK * 3;
        }
        if constexpr (kb == NK - 1) {
            // ---- epilogue: the graph mix in registers (lane: frame f, channels co .. co + 3, all 17 joints)
            const int co = pass * 128 + 16 * wave + 4 * g;
            const int q = tile_fg(t) * FR + f;
            auto mix_all = [&](auto sparse) __attribute__((always_inline)) {
                constexpr bool SP = decltype(sparse)::value;
#pragma unroll
                for (int wj = 0; wj < V; ++wj) {
                    f32x4 z = *reinterpret_cast<const f32x4*>(b2s + wj * a.cout + co);
#pragma unroll
                    for (int v = 0; v < V; ++v)
                        if (!SP || ((coco_hop2_mask3(wj) >> v) & 1u)) {
                            const float av = __builtin_bit_cast(
                                float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, amv[(v * V + wj) / 64]), (v * V + wj) % 64));
                            z += av * acc[v];
                        }
#pragma unroll
                    for (int e = 0; e < 4; ++e) z[e] = z[e] > 0.f ? z[e] : 0.f;
                    float* o = q < QO ? a.out + ((size_t)q * V + wj) * a.ldo + co : a.trash;
                    xst4(o, z, a.nts);
                }
            };
            if (a.mix_sparse) mix_all(std::true_type{});
            else mix_all(std::false_type{});
            n_after += V;
#pragma unroll
            for (int j = 0; j < V; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
        }
    };
    for (int t = t_begin; t < t_end; ++t) {
        const int s0 = (t - t_begin) * NK, pass = tile_pass(t);
        step(s0, t, pass, std::integral_constant<int, 0>{});
        step(s0 + 1, t, pass, std::integral_constant<int, 1>{});
        if constexpr (NK > 2) {
            step(s0 + 2, t, pass, std::integral_constant<int, 2>{});
            step(s0 + 3, t, pass, std::integral_constant<int, 3>{});
        }
        if constexpr (NK > 4) {
            step(s0 + 4, t, pass, std::integral_constant<int, 4>{});
            step(s0 + 5, t, pass, std::integral_constant<int, 5>{});
            step(s0 + 6, t, pass, std::integral_constant<int, 6>{});
            step(s0 + 7, t, pass, std::integral_constant<int, 7>{});
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

bool xgraph_ok(const XGraphArgs& a) {
    return (a.cin == 64 || a.cin == 128 || a.cin == 256) && (a.cout == 128 || a.cout == 256) && a.ldx % 4 == 0 &&
           a.ldx >= a.cin && a.ldo % 4 == 0 && a.ldo >= a.cout;
}

hipError_t launch_xgraph(const XGraphArgs& a, int ncu, hipStream_t st) {
    if (a.nframes <= 0) return hipSuccess;
    if (!xgraph_ok(a) || !a.x || !a.wp || !a.bias2 || !a.amix || !a.out || !a.trash || ncu <= 0) return hipErrorInvalidValue;
    // the DMA offsets are 32-bit: launches of at most ~2 GiB of input rows each
    const long long row_bytes = 17LL * a.ldx * 4;
    const int chunk = (int)std::min<long long>(a.nframes, ((1LL << 31) - 1) / row_bytes / xg::FR * xg::FR);
    if (chunk <= 0) return hipErrorInvalidValue;
    (void)hipGetLastError();
    for (int q0 = 0; q0 < a.nframes; q0 += chunk) {
        XGraphArgs c = a;
        c.nframes = std::min(chunk, a.nframes - q0);
        c.x = a.x + (size_t)q0 * 17 * a.ldx;
        c.out = a.out + (size_t)q0 * 17 * a.ldo;
        const int ntiles = ((c.nframes + xg::FR - 1) / xg::FR) * (a.cout / 128);
        const int grid = std::min(ntiles, ncu);
        if (a.cin == 64) hipLaunchKernelGGL(xgraph_kernel<2>, dim3(grid), dim3(512), 0, st, c);
        else if (a.cin == 128) hipLaunchKernelGGL(xgraph_kernel<4>, dim3(grid), dim3(512), 0, st, c);
        else hipLaunchKernelGGL(xgraph_kernel<8>, dim3(grid), dim3(512), 0, st, c);
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

}  // namespace tik
