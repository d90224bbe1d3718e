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
//   * the fp32 rows of one K step (16 frames x 17 joints x 32 channels: 272
//     consecutive rows, 128 B each) are loaded into REGISTERS, D steps ahead
//     (D = 2: two steps, ~70 KB per CU, in flight — an HBM-bound kernel needs
//     that much to cover the loaded latency; an LDS staging slot would not
//     fit beside the planes images), and split ONCE, cooperatively, into an
//     LDS image of bf16 planes that all eight waves read (split on read, each
//     wave would split every element again); the planes image is double-
//     buffered, so step k+1's split runs beside step k's MFMAs, one barrier
//     per step, across tile boundaries (persistent).
// Products, K order and mix order as the tiled kernel (bf16x3 six products,
// fp32 accumulation; bias2 then v ascending): bit-identical poses.
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
constexpr int NU = PX * 8;                           // 16-B units of one K step (2176)
constexpr int NLD = (NU + 511) / 512;                // register loads per lane per step (5; the 5th on waves 0-1)
constexpr int PROWB = 3 * 32 * 2;                    // planes image row: 3 planes x 32 channels x 2 B
constexpr int PBYTES = PX * PROWB;                   // 52,224
}  // namespace xg

// planes image: row R = 16 j + f (joint-major), unit (plane p, K group u) at
// p * 4 + (u ^ ((R >> 1) & 3)): conflict-free b128 reads of 16 consecutive rows
__device__ __forceinline__ int xg_unit(int R, int p, int u) { return R * xg::PROWB + ((p * 4 + (u ^ ((R >> 1) & 3))) << 4); }

__device__ f32x4 tik_llvm_raw_buffer_load_v4f32(i32x4 rsrc, int voffset, int soffset, int aux)
    __asm("llvm.amdgcn.raw.buffer.load.v4f32");

typedef __bf16 xbf16x4 __attribute__((ext_vector_type(4)));

#ifdef TIK_XTUNE
#define XG_OFF(bit) (a.tune & (bit))
#else
#define XG_OFF(bit) false
#endif

template <int NK, int NP>
__global__ __launch_bounds__(512, 1) void xgraph_kernel(XGraphArgs a) {
    using namespace xg;
    constexpr int D = NK <= 4 ? 2 : 1;   // steps of prefetch in registers (NK = 8: the weights take 96 VGPRs)
    constexpr int B2MAX = V * 256 * 4;
    __shared__ __attribute__((aligned(16))) unsigned char smem[2 * PBYTES + B2MAX];
    float* const b2s = reinterpret_cast<float*>(smem + 2 * PBYTES);
    auto pimg = [&](int s) __attribute__((always_inline)) { return smem + (s & 1) * PBYTES; };

    int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int QO = a.nframes, M = QO * V;
    constexpr int npass = NP;
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

    // bias2 [17][cout] in LDS, A_eff in VGPRs (v_readlane)
    for (int i = tid; i < V * a.cout; i += 512) b2s[i] = a.bias2[i];
    float amv[5];
#pragma unroll
    for (int k = 0; k < 5; ++k) amv[k] = 64 * k + lane < V * V ? a.amix[64 * k + lane] : 0.f;

    // ---- the fp32 rows of global step s (tile t_begin + s / NK, K block s % NK):
    // unit U = 512 i + tid: group row m = U / 8 (frame m / 17, joint m % 17), channels 4 (U % 8) ..
    const i32x4 rX = buf_rsrc(a.x, (unsigned)((long long)M * a.ldx * 4));
    f32x4 rb[D][NLD];
    // Every wave issues NLD loads for every step, past the batch / the run as
    // out-of-range (zero) loads: no branch, so the compiler's vmcnt accounting
    // stays exact (at a merge it falls back to the fewest outstanding, i.e. vmcnt(0))
    auto load_unit = [&](int s, f32x4 (&r)[NLD], int i) __attribute__((always_inline)) {
        const int t = t_begin + s / NK, kb = s - (s / NK) * NK;
        const int q0 = tile_fg(t) * FR;
        const bool live = s < total;
        const int U = 512 * i + tid, m = U >> 3, u = U & 7;
        const int q = q0 + m / V;
        const unsigned off = live && U < NU && q < QO && !XG_OFF(1) ? (unsigned)(((long long)q0 * V + m) * a.ldx * 4 + kb * 128 + u * 16) : DMA_OOB;
        // nontemporal (aux 2: nt): XGW.L2 -3.5 %, the others within noise (profiles/r06_ab_xgraph_nt_loads2.txt)
        r[i] = tik_llvm_raw_buffer_load_v4f32(rX, (int)off, 0, 2);
    };
    auto load = [&](int s, f32x4 (&r)[NLD]) __attribute__((always_inline)) {
#pragma unroll
        for (int i = 0; i < NLD; ++i) load_unit(s, r, i);
    };
    // ---- split registers r (this lane's units of step s) into planes image (s & 1)
    auto split_unit = [&](int s, const f32x4 (&r)[NLD], int i) __attribute__((always_inline)) {
        unsigned char* P = pimg(s);
        const int U = 512 * i + tid;
        if (i + 1 < NLD || U < NU) {
            const int m = U >> 3, u = U & 7;
            const int R = 16 * (m % V) + m / V;
            xbf16x4 p0, p1, p2;
#pragma unroll
            for (int e = 0; e < 4; ++e) {   // xsplit8's arithmetic, 4 channels
                const float x = r[i][e];
                const __bf16 b0 = (__bf16)x;
                const float r1 = x - (float)b0;
                const __bf16 b1 = (__bf16)r1;
                p0[e] = b0;
                p1[e] = b1;
                p2[e] = (__bf16)(r1 - (float)b1);
            }
            const int h = (u & 1) * 8;
            *reinterpret_cast<xbf16x4*>(P + xg_unit(R, 0, u >> 1) + h) = p0;
            *reinterpret_cast<xbf16x4*>(P + xg_unit(R, 1, u >> 1) + h) = p1;
            *reinterpret_cast<xbf16x4*>(P + xg_unit(R, 2, u >> 1) + h) = p2;
        }
    };
    auto split = [&](int s, const f32x4 (&r)[NLD]) __attribute__((always_inline)) {
#pragma unroll
        for (int i = 0; i < NLD; ++i) split_unit(s, r, i);
    };

    // weights of this wave's 16 channels for the current pass. Two passes (256
    // channels): K block kb's planes are re-loaded for the next tile's pass right
    // after step kb's MFMAs, a whole tile before their next use
    xbf16x8 w[NK][3];
    auto load_wk = [&](int pass, int kb) __attribute__((always_inline)) {
        const int cg = pass * 8 + wave;
#pragma unroll
        for (int p = 0; p < 3; ++p)
            w[kb][p] = *reinterpret_cast<const xbf16x8*>(a.wp + ((((size_t)cg * NK + kb) * 3 + p) * 64 + lane) * 8);
    };
    auto load_w = [&](int pass) __attribute__((always_inline)) {
#pragma unroll
        for (int kb = 0; kb < NK; ++kb) load_wk(pass, kb);
    };

    // prologue: weights; step 0 -> planes[0]; steps 1 .. D into registers
    load(0, rb[0]);
    load_w(tile_pass(t_begin));
    split(0, rb[0]);
#pragma unroll
    for (int d = 1; d <= D; ++d) load(d, rb[d % D]);

    f32x4 acc[V];
#pragma unroll
    for (int j = 0; j < V; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};

#ifdef TIK_XTRACE
    const bool tr = a.trace != nullptr && (wave == 0 || wave == 4);
#else
    constexpr bool tr = false;
#endif
    // phases: 0 barrier, 1 MFMAs j < 4, 2 split, 3 loads, 4 MFMAs j >= 4, 5 epilogue
    unsigned long long ph_[6] = {0, 0, 0, 0, 0, 0}, tlast = 0, tstart = 0;
    auto stamp = [&](int i) __attribute__((always_inline)) {
        if (tr) {
            const unsigned long long t = __builtin_amdgcn_s_memtime();
            if (i >= 0) ph_[i] += t - tlast;
            else tstart = t;
            tlast = t;
        }
    };
    stamp(-1);

    // one K step; KB compile-time so the weights and the prefetch registers are
    // statically indexed (s % D == KB % D: NK is even)
    auto step = [&](int s, int t, int pass, auto KBc) __attribute__((always_inline)) {
        constexpr int kb = decltype(KBc)::value;
        constexpr int nb = (kb + 1) % D;   // registers holding step s+1
        asm volatile("" : "+v"(tid), "+v"(lane));   // lane-derived addresses: not hoisted across steps (spills)
        const int g = lane >> 4, f = lane & 15;
        // every wave's split(s) landed; every wave done with step s-1's planes (the buffer split(s+1) writes)
        lds_barrier();
        stamp(0);
        const unsigned char* P = pimg(s);
        // operand ring: joint j + XPF's planes are read while joint j's MFMAs run
        // (a sched_barrier between the reads and the MFMAs: left alone, the
        // scheduler sinks the reads next to their use and exposes the LDS latency)
        constexpr int XPF = 2;
        xbf16x8 xb[XPF + 1][3];
        auto rd = [&](int j, xbf16x8 (&d)[3]) __attribute__((always_inline)) {
#pragma unroll
            for (int p = 0; p < 3; ++p) d[p] = *reinterpret_cast<const xbf16x8*>(P + xg_unit(16 * j + f, p, g));
        };
        auto mfma_j = [&](int j) __attribute__((always_inline)) {
            if (j + XPF < V) rd(j + XPF, xb[(j + XPF) % (XPF + 1)]);
            __builtin_amdgcn_sched_barrier(0);
            if (XG_OFF(4)) return;
            const xbf16x8(&x)[3] = xb[j % (XPF + 1)];
            // (w0,x2) (w1,x1) (w2,x0) (w0,x1) (w1,x0) (w0,x0): xgemm's product order
            acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[kb][0], x[2], acc[j], 0, 0, 0);
            acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[kb][1], x[1], acc[j], 0, 0, 0);
            acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[kb][2], x[0], acc[j], 0, 0, 0);
            acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[kb][0], x[1], acc[j], 0, 0, 0);
            acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[kb][1], x[0], acc[j], 0, 0, 0);
            acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[kb][0], x[0], acc[j], 0, 0, 0);
            __builtin_amdgcn_sched_barrier(0);
        };
#pragma unroll
        for (int j = 0; j < XPF; ++j) rd(j, xb[j]);
        if constexpr (NP == 2) {
            // two-pass (256-channel) layers: the next step's split one unit every third joint
            // from joint 1 on, each unit's register slot reloaded right after it (past the run:
            // zeros, never read); the asm keeps the unit's VALU and LDS writes there. XGW.L7
            // -4 %, L6 -1 %; the HBM-bound one-pass layers are 0.5 % faster with the block below
#pragma unroll
            for (int j = 0; j < V; ++j) {
                mfma_j(j);
                if (j % 3 == 1 && j / 3 < NLD) {
                    const int i = j / 3;
                    if (!XG_OFF(2)) split_unit(s + 1, rb[nb], i);
                    load_unit(s + 1 + D, rb[nb], i);
                    asm volatile("" ::: "memory");
                    __builtin_amdgcn_sched_barrier(0);
                }
                if (j == 3) {
                    stamp(1);
                    stamp(2);
                    stamp(3);
                }
            }
        } else {
#pragma unroll
            for (int j = 0; j < 4; ++j) mfma_j(j);
            stamp(1);
            if (!XG_OFF(2)) split(s + 1, rb[nb]);   // VALU + LDS writes beside the MFMAs (past the run: zeros, never read)
            stamp(2);
            load(s + 1 + D, rb[nb]);
            stamp(3);
#pragma unroll
            for (int j = 4; j < V; ++j) mfma_j(j);
        }
        stamp(4);
        if constexpr (NP == 2) load_wk(tile_pass(t + 1), kb);
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
                        if (XG_OFF(16)) {
                            if (v == wj) z += acc[v];
                        } else if (!SP || ((coco_hop2_mask3(wj) >> v) & 1u)) {
                            const float av = __builtin_bit_cast(
                                float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, amv[(v * V + wj) / 64]), (v * V + wj) % 64));
                            z += av * acc[v];
                        }
#pragma unroll
                    for (int e = 0; e < 4; ++e) z[e] = z[e] > 0.f ? z[e] : 0.f;
                    float* o = q < QO ? a.out + ((size_t)q * V + wj) * a.ldo + co : a.trash;
                    if (!XG_OFF(8)) xst4(o, z, a.nts);
                }
            };
            if (a.mix_sparse) mix_all(std::true_type{});
            else mix_all(std::false_type{});
#pragma unroll
            for (int j = 0; j < V; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
            stamp(5);
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
#ifdef TIK_XTRACE
    if (tr && lane == 0) {
        unsigned long long* o = a.trace + 16 * (size_t)blockIdx.x + (wave == 4 ? 8 : 0);
#pragma unroll
        for (int i = 0; i < 6; ++i) o[i] = ph_[i];
        o[6] = (unsigned long long)total;
        o[7] = tlast - tstart;
    }
#endif
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
        const bool two = a.cout == 256;
        if (a.cin == 64) hipLaunchKernelGGL((two ? xgraph_kernel<2, 2> : xgraph_kernel<2, 1>), dim3(grid), dim3(512), 0, st, c);
        else if (a.cin == 128) hipLaunchKernelGGL((two ? xgraph_kernel<4, 2> : xgraph_kernel<4, 1>), dim3(grid), dim3(512), 0, st, c);
        else hipLaunchKernelGGL((two ? xgraph_kernel<8, 2> : xgraph_kernel<8, 1>), dim3(grid), dim3(512), 0, st, c);
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

}  // namespace tik
