// online.hip — the online-IK step (BASELINE.json config #5) as one dataflow
// kernel; see online.h for the task list and why only the first frames of
// each layer are computed.
//
// Arithmetic: the gcn and temporal-conv tasks in bf16x3 on
// v_mfma_f32_16x16x32_bf16 (the staged fp32 rows split into three bf16 planes
// in registers, the weights pre-split per stream, six products, fp32
// accumulation: fp32-class like the batch path; round 5 — the one-CU exact fp32
// MFMA rate bounded the 256-channel tasks at 1.8 us); joint 16, the graph mix
// and the head in fp32 VALU FMAs. Every task is one 1024-thread
// workgroup (16 waves: 4 per SIMD, so LDS and memory latency overlap); the
// task's weights are loaded into registers BEFORE it waits for its inputs,
// and the input rows are staged into LDS with coalesced 16-B loads. A task's
// 17 joints x 16 channels are one 16 x 16 MFMA block (joints 0-15) + joint 16
// on the VALU; its K (input channels, x 3 taps, + the residual conv) is split
// over the 16 waves, and the 16 partial blocks are summed through LDS in a
// fixed order (deterministic for any grid).
// (Round 2's VALU version spent 2-3 us per temporal-conv task in its FMAs and
// the 64-way reduction, profiles/r02_v2_online_trace.txt.)
//
// Synchronisation (cross-XCD: each XCD has its own L2). Every activation a
// task hands to another task is stored and loaded with device-scope cache
// policy (sc1: written through to / read from the device coherence point), the
// encoding the compiler uses for agent-scope atomic loads and stores; the
// weights stay ordinary cached loads (read-only for the whole launch). The
// activations are ReLU outputs, so their sign bit carries the launch's parity
// and a consumer polls the elements it reads until all carry it: no producer
// waits for its stores, no completion counters (round 5: a per-frame counter
// cost a store acknowledgement + counter update + counter poll + data load per
// dependency, ~1.5 us of the ~3.5 us per hop). No L2 write-back or invalidate:
// a first version with agent-scope release/acquire fences (buffer_wbl2 /
// buffer_inv per task) spent most of its time in them (213 us per step).
// Tickets are taken in topological order, so the smallest unfinished taken
// task always has its inputs complete: no deadlock, whatever the residency.
// Every wait is bounded (0.5 s): a timeout sets *err and the task proceeds,
// so the grid always drains; the host reports the error.
#include "online.h"
#include "xgemm_dev.h"

namespace tik {

namespace onl {
constexpr int NT = 1024;
constexpr int LDP = 4;                                    // row padding (floats): MFMA A reads conflict-free
constexpr int SMF = 4 * 17 * (ONL_MAXC + LDP);            // staged rows, floats (70,720 B)
constexpr int RED = 16 * 272;                              // the 16 waves' partial 17 x 16 blocks (after SMF)
constexpr int SMT = SMF + RED + 272;                       // + y[17][16]
constexpr unsigned long long TIMEOUT = 50000000ull;      // s_memrealtime ticks (100 MHz)
}  // namespace onl

__device__ __forceinline__ int cnt_load(int* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }

// device-coherent access to the activation buffer (raw buffer ops, cpol sc1)
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
constexpr int CPOL_SC1 = 16;
struct Act {
    __amdgpu_buffer_rsrc_t r;
    const char* base;
};
__device__ __forceinline__ Act act_of(const OnlineArgs* __restrict__ A) {
    return Act{__builtin_amdgcn_make_buffer_rsrc(A->act, 0, (int)A->act_bytes, 0x00020000), reinterpret_cast<const char*>(A->act)};
}
__device__ __forceinline__ int act_off(const Act& b, const float* p) { return (int)(reinterpret_cast<const char*>(p) - b.base); }
__device__ __forceinline__ void st1c(const Act& b, float* p, const float v) {
    __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v), b.r, act_off(b, p), 0, CPOL_SC1);
}
__device__ void onl_mark(const OnlineArgs* __restrict__ A, int task, int k);

// ---- tagged activations. Every G / T output is a ReLU value (>= +0), so its sign
// bit is free: launch c stores v | (c & 1) << 31, and a consumer polls the data itself
// until each element carries this launch's tag. A dependency costs one trip through
// memory (no store acknowledgement before a completion count, no count poll, no
// data load after it). Every launch runs the same task list and so rewrites every
// element it reads; the buffer starts at tag 1 (setup, reset) for launch 0.
__device__ __forceinline__ u32x4 ld4raw(const Act& b, const float* p) {
    return __builtin_amdgcn_raw_buffer_load_b128(b.r, act_off(b, p), 0, CPOL_SC1);
}
__device__ __forceinline__ bool tag_ok(const u32x4 r, const unsigned E) {
    return ((((r.x ^ E) | (r.y ^ E)) | ((r.z ^ E) | (r.w ^ E))) >> 31) == 0;
}
// r: the first load of p; polls until tagged E (or the error flag / a timeout), untags
__device__ __forceinline__ float4 onl_fin4(const OnlineArgs* __restrict__ A, const Act& b, const float* p, const unsigned E, u32x4 r) {
    if (!tag_ok(r, E)) {
        const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
        for (int it = 1;; ++it) {
            asm volatile("" ::: "memory");
            r = ld4raw(b, p);
            if (tag_ok(r, E)) break;
            if ((it & 63) == 0 && (cnt_load(A->err) || __builtin_amdgcn_s_memrealtime() - t0 > onl::TIMEOUT)) {
                __hip_atomic_fetch_or(A->err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                break;
            }
        }
    }
    const unsigned m = 0x7fffffffu;
    return make_float4(__builtin_bit_cast(float, r.x & m), __builtin_bit_cast(float, r.y & m), __builtin_bit_cast(float, r.z & m),
                       __builtin_bit_cast(float, r.w & m));
}
__device__ __forceinline__ void st1t(const Act& b, float* p, const float v, const unsigned E) {
    __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v) | E, b.r, act_off(b, p), 0, CPOL_SC1);
}

// debug trace: slot k of task `task` (thread 0 only): 0 ticket, 1 inputs requested,
// 2 inputs staged, 3 products, 4 reduced, 5 stored, 6 task end
__device__ void onl_mark(const OnlineArgs* __restrict__ A, int task, int k) {
    if (A->trace) A->trace[8 * (size_t)task + k] = __builtin_amdgcn_s_memrealtime();
}

// the prefetched operand is in registers here (the compiler otherwise sinks
// the load to its first use, after the dependency wait)
__device__ __forceinline__ void onl_hold(float& x) { asm volatile("" : "+v"(x)); }
__device__ __forceinline__ void onl_hold(float4& x) { asm volatile("" : "+v"(x.x), "+v"(x.y), "+v"(x.z), "+v"(x.w)); }

__device__ __forceinline__ float fma4(const float4 a, const float4 b, float c) {
    c = fmaf(a.x, b.x, c);
    c = fmaf(a.y, b.y, c);
    c = fmaf(a.z, b.z, c);
    return fmaf(a.w, b.w, c);
}

// ---- the layer-0 input rows of window frame k, computed where they are used
// (no input task, no round trip): window gather with the left-edge clamp,
// root-relative, data_bn -> 17 rows of 4 floats at dst, row stride ld4 float4s (threads 0-16).
// The pushed frame is read from pinned host memory; older frames from the ring,
// which task 0 of the launch appends the pushed frame to (online_kernel).
__device__ void onl_raw_rows(const OnlineArgs* __restrict__ A, int k, float4* dst, int ld4) {
    const int v = threadIdx.x;
    if (v >= 17) return;
    const int last = cnt_load(A->count);   // frames pushed before this one = the pushed frame's index
    const int W = A->W, nv = 17 * 3, ra = A->ra, rb = A->rb;
    int fi = last - 2 * A->h + k;
    fi = fi < 0 ? 0 : fi;
    const float* src = fi == last ? A->frame : A->ring + (size_t)(fi % W) * nv;
    float o[3];
#pragma unroll
    for (int e = 0; e < 3; ++e) {
        float x = src[v * 3 + e];
        if (A->relative) x -= 0.5f * (src[ra * 3 + e] + src[rb * 3 + e]);
        o[e] = fmaf(x, A->bn_sc[v * 3 + e], A->bn_sh[v * 3 + e]);
    }
    dst[v * ld4] = make_float4(o[0], o[1], o[2], 0.f);
}

// MFMA roles of a G / T task: wave w takes the K steps (32 input channels each)
// w, w + 16, ... Per step, six bf16x3 products on v_mfma_f32_16x16x32_bf16 cover
// joints 0-15: A = the staged fp32 rows split into three bf16 planes in registers
// (lane: joint l & 15, K elements 8 (l >> 4) .. + 7), B = the host-split weight
// planes (lane: output channel c0 + (l & 15), the same K elements), D lane l =
// joints 4 (l >> 4) + e, channel c0 + (l & 15). Joint 16 is 8 fp32 FMAs per step
// on the fp32 copy of the same weights (lane: channel l & 15, K elements 8 (l >> 4)
// ..), its 4 lane-group partials summed across the lane groups before the wave's
// partials go to LDS (a second 16-row MFMA block for one joint would double the
// MFMA time).
typedef float onl_f32x4 __attribute__((ext_vector_type(4)));
constexpr int ONL_KSL = 16;   // K slices (one per wave)

// the 16 waves' partials (acc: joints 0-15; p16: joint 16 of lane l's channel and K
// element) -> y[v][co] at sm[SMF + RED + 16 v + co], summed in a fixed order; the
// partials have their own LDS (no barrier for the staged rows' last reads). With
// sync_y the y block is visible to every thread on return (the gcn mix reads all
// 17 joints); without, thread tid < 272 reads only its own y[tid].
__device__ __forceinline__ void onl_reduce_mfma(const onl_f32x4 acc, float p16, float* sm, bool sync_y) {
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    p16 += __shfl_xor(p16, 16);
    p16 += __shfl_xor(p16, 32);
    float* red = sm + onl::SMF;   // [16 waves][17 joints][16 co]
#pragma unroll
    for (int e = 0; e < 4; ++e) red[wave * 272 + (4 * (lane >> 4) + e) * 16 + (lane & 15)] = acc[e];
    if (lane < 16) red[wave * 272 + 16 * 16 + lane] = p16;
    __syncthreads();
    if (tid < 272) {
        float s = 0.f;
#pragma unroll
        for (int k = 0; k < ONL_KSL; ++k) s += red[k * 272 + tid];
        sm[onl::SMF + onl::RED + tid] = s;
    }
    if (sync_y) __syncthreads();
}

// ---- G_L(f, 16 channels): z = ReLU(bias2 + sum_v A[v][w] (x . wg^T)[v])
__device__ void onl_gcn(const OnlineArgs* __restrict__ A, int p, int idx, float* sm, int task, const unsigned E) {
    const OnlinePhase& ph = A->ph[p];
    const OnlineLayer& L = A->L[ph.layer];
    int tid = threadIdx.x;
    asm volatile("" : "+v"(tid));   // lane-derived offsets are made per task, not hoisted across the task loop (spills)
    const int lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int ksl = wave, kk = lane >> 4, ri = lane & 15;
    const int f = idx / ph.ngroups, cg = idx - f * ph.ngroups;
    const int cinp = L.cinp, K4 = cinp >> 2, cout = L.cout, c0 = cg * 16;
    const int K32 = L.gk32;                                  // K = cinp in steps of 32 (zero-padded)
    const int LD = (cinp > 32 * K32 ? cinp : 32 * K32) + 4;  // staged row: an odd number of 16-B units
    static_assert(ONL_MAXC / 32 <= ONL_KSL, "gcn K steps: at most one per wave");
    // operands that do not depend on the input: this wave's weight planes (bf16x3, MFMA B
    // operand) and fp32 values (joint 16), mix column, bias
    const int sk = ksl;
    xbf16x8 w[3];
#pragma unroll
    for (int pl = 0; pl < 3; ++pl)
        w[pl] = sk < K32 ? *reinterpret_cast<const xbf16x8*>(L.wgp + ((((size_t)cg * K32 + sk) * 3 + pl) * 64 + lane) * 8) : xbf16x8{};
    const float* wgr = L.wgf + (size_t)(c0 + ri) * 32 * K32 + 32 * sk + 8 * kk;
    f32x4 wf0 = sk < K32 ? *reinterpret_cast<const f32x4*>(wgr) : f32x4{0.f, 0.f, 0.f, 0.f};
    f32x4 wf1 = sk < K32 ? *reinterpret_cast<const f32x4*>(wgr + 4) : f32x4{0.f, 0.f, 0.f, 0.f};
    const int wo = tid >> 4, co = tid & 15;   // mix output (wo, co) of threads 0-271
    float am[17], b = 0.f;
#pragma unroll
    for (int v = 0; v < 17; ++v) am[v] = tid < 272 ? L.amix[v * 17 + wo] : 0.f;
    if (tid < 272) b = L.bias2[wo * cout + c0 + co];
#pragma unroll
    for (int pl = 0; pl < 3; ++pl) asm volatile("" : "+v"(w[pl]));
    asm volatile("" : "+v"(wf0), "+v"(wf1));
    onl_hold(b);
#pragma unroll
    for (int v = 0; v < 17; ++v) onl_hold(am[v]);
    float4* s4 = reinterpret_cast<float4*>(sm);
    const Act ab = act_of(A);
    if (tid == 0) onl_mark(A, task, 1);
    if (ph.layer == 0) {
        onl_raw_rows(A, f, s4, LD / 4);
    } else {   // the previous temporal conv's frame f, all 17 x cinp loads in flight at once
        constexpr int NL = (17 * ONL_MAXC / 4 + onl::NT - 1) / onl::NT;
        const float* xr = L.x + (size_t)f * 17 * cinp;
        u32x4 r[NL];
#pragma unroll
        for (int j = 0; j < NL; ++j) {
            const int i = tid + j * onl::NT;
            if (i < 17 * K4) r[j] = ld4raw(ab, xr + 4 * i);
        }
#pragma unroll
        for (int j = 0; j < NL; ++j) {
            const int i = tid + j * onl::NT;
            if (i < 17 * K4) {
                const int v = i / K4;
                s4[v * (LD / 4) + (i - v * K4)] = onl_fin4(A, ab, xr + 4 * i, E, r[j]);
            }
        }
    }
    // the K padding past cinp (layer 0: 4 -> 32) reads zeros
    for (int i = tid; i < 17 * (32 * K32 - cinp); i += onl::NT) {
        const int v = i / (32 * K32 - cinp);
        sm[v * LD + cinp + (i - v * (32 * K32 - cinp))] = 0.f;
    }
    __syncthreads();
    if (tid == 0) onl_mark(A, task, 2);
    // bf16x3 products on v_mfma_f32_16x16x32_bf16 (rows split into planes in registers), joint 16 in fp32 FMAs
    onl_f32x4 acc[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
    float p16 = 0.f;
    if (sk < K32) {
        const float* xa = sm + ri * LD + 32 * sk + 8 * kk;
        const float* x16 = sm + 16 * LD + 32 * sk + 8 * kk;
        const f32x4 lo = *reinterpret_cast<const f32x4*>(xa), hi = *reinterpret_cast<const f32x4*>(xa + 4);
        xbf16x8 x0, x1, x2;
        xsplit8(lo, hi, x0, x1, x2);
        acc[0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x2, w[0], acc[0], 0, 0, 0);
        acc[1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x1, w[1], acc[1], 0, 0, 0);
        acc[0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x0, w[2], acc[0], 0, 0, 0);
        acc[1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x1, w[0], acc[1], 0, 0, 0);
        acc[0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x0, w[1], acc[0], 0, 0, 0);
        acc[1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x0, w[0], acc[1], 0, 0, 0);
        const f32x4 l16 = *reinterpret_cast<const f32x4*>(x16), h16 = *reinterpret_cast<const f32x4*>(x16 + 4);
#pragma unroll
        for (int e = 0; e < 4; ++e) p16 = fmaf(l16[e], wf0[e], p16);
#pragma unroll
        for (int e = 0; e < 4; ++e) p16 = fmaf(h16[e], wf1[e], p16);
    }
    if (tid == 0) onl_mark(A, task, 3);
    onl_reduce_mfma(acc[0] + acc[1], p16, sm, true);
    if (tid == 0) onl_mark(A, task, 4);
    const float* y = sm + onl::SMF + onl::RED;
    if (tid < 272) {
        float s = b;
#pragma unroll
        for (int v = 0; v < 17; ++v) s = fmaf(am[v], y[v * 16 + co], s);
        st1t(ab, L.z + (size_t)(f * 17 + wo) * cout + c0 + co, s > 0.f ? s : 0.f, E);
    }
    if (tid == 0) onl_mark(A, task, 5);
}

// ---- T_L(t, 16 channels): out = ReLU(sum_tap z[s t + tap - 1] . wt_tap^T + bias + residual)
// where the block input x sits in a staged T row: at 3 C for the residual conv (its K
// segment), past the K padding 32 K32 for the identity term (inside [3 C, 32 K32) the
// padding is zeroed; C % 32 == 16 puts 16 floats of padding there)
__device__ __forceinline__ int onl_tconv_xoff(int C, bool rconv, int K32) {
    return rconv || 32 * K32 < 3 * C ? 3 * C : 32 * K32;
}
// staged T row length (floats): the K range and the staged x, + 4 (an odd number of
// 16-B units: the 16 rows' ds_read_b128 hit distinct banks)
__device__ __forceinline__ int onl_tconv_ld(int xoff, int cinp, int K32) {
    const int k = xoff + cinp > 32 * K32 ? xoff + cinp : 32 * K32;
    return k + 4;
}

// Staged operand rows, one per joint, in K order: [z tap 0 (C) | tap 1 | tap 2 | block
// input x (cinp: the residual conv's K segment, or the identity term past the K padding)],
// so K step sk reads floats 4 sk .. of the row (no per-step tap decode between the MFMAs)
__device__ void onl_tconv(const OnlineArgs* __restrict__ A, int p, int idx, float* sm, int task, const unsigned E) {
    const OnlinePhase& ph = A->ph[p];
    const OnlineLayer& L = A->L[ph.layer];
    int tid = threadIdx.x;
    asm volatile("" : "+v"(tid));   // lane-derived offsets are made per task, not hoisted across the task loop (spills)
    const int lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int ksl = wave, kk = lane >> 4, ri = lane & 15;
    const int t = idx / ph.ngroups, cg = idx - t * ph.ngroups;
    const int C = L.cout, C4 = C >> 2, cinp4 = L.cinp >> 2;
    const bool rconv = L.res == ONR_CONV;
    const int c0 = cg * 16;
    const int s = L.stride, tin = L.tin, fx = s * t;
    // K = 3 C (+ cinp: the residual conv) in steps of 32 (L.k32, zero-padded)
    const int K32 = L.k32, Kt = 3 * C + (rconv ? L.cinp : 0);
    const int XO = onl_tconv_xoff(C, rconv, K32), XO4 = XO / 4;   // staged block input (floats)
    const int LK = onl_tconv_ld(XO, L.cinp, K32), LK4 = LK / 4;   // staged row (floats)
    constexpr int NS = (4 * ONL_MAXC / 32 + ONL_KSL - 1) / ONL_KSL;   // K steps per wave (at most): 2
    // this wave's weights: bf16x3 planes of K step sk (MFMA B operand: lane = channel
    // c0 + (lane & 15), K 8 (lane >> 4) ..) and the same 8 fp32 values for joint 16
    xbf16x8 w[NS][3];
    f32x4 wf[NS][2];
#pragma unroll
    for (int q = 0; q < NS; ++q) {
        const int sk = ksl + ONL_KSL * q;
#pragma unroll
        for (int pl = 0; pl < 3; ++pl)
            w[q][pl] = sk < K32 ? *reinterpret_cast<const xbf16x8*>(L.wtp + ((((size_t)cg * K32 + sk) * 3 + pl) * 64 + lane) * 8)
                                : xbf16x8{};
        const float* wr = L.wtf + (size_t)(c0 + ri) * 32 * K32 + 32 * sk + 8 * kk;
        wf[q][0] = sk < K32 ? *reinterpret_cast<const f32x4*>(wr) : f32x4{0.f, 0.f, 0.f, 0.f};
        wf[q][1] = sk < K32 ? *reinterpret_cast<const f32x4*>(wr + 4) : f32x4{0.f, 0.f, 0.f, 0.f};
    }
    const float bt = L.biasT[c0 + (tid & 15)];
#pragma unroll
    for (int q = 0; q < NS; ++q) {
#pragma unroll
        for (int pl = 0; pl < 3; ++pl) asm volatile("" : "+v"(w[q][pl]));
        asm volatile("" : "+v"(wf[q][0]), "+v"(wf[q][1]));
    }
    // staging: the block input rows (the previous layer's temporal conv, frame fx) and
    // the three z frames, every load in flight at once; each element is then polled
    // until it carries this launch's tag (usually only the newest frame's)
    float4* s4 = reinterpret_cast<float4*>(sm);
    const int nz = 17 * C4;
    const Act ab = act_of(A);
    constexpr int NL = (17 * ONL_MAXC / 4 + onl::NT - 1) / onl::NT;   // loads per thread per row block
    const bool xin = L.res != ONR_ZERO && ph.layer > 0;
    const float* xrow = xin ? L.x + (size_t)fx * 17 * L.cinp : L.z;
    if (tid == 0) onl_mark(A, task, 1);
    u32x4 rx[NL], rz[3][NL];
#pragma unroll
    for (int j = 0; j < NL; ++j) {
        const int i = tid + j * onl::NT;
        if (xin && i < 17 * cinp4) rx[j] = ld4raw(ab, xrow + 4 * i);
    }
#pragma unroll
    for (int tap = 0; tap < 3; ++tap) {
        const int fr = fx + tap - 1;
        const bool live = fr >= 0 && fr < tin;
#pragma unroll
        for (int j = 0; j < NL; ++j) {
            const int i = tid + j * onl::NT;
            if (live && i < nz) rz[tap][j] = ld4raw(ab, L.z + ((size_t)fr * nz + i) * 4);
        }
    }
    if (L.res != ONR_ZERO && ph.layer == 0) onl_raw_rows(A, fx, s4 + XO4, LK4);
#pragma unroll
    for (int j = 0; j < NL; ++j) {
        const int i = tid + j * onl::NT;
        if (xin && i < 17 * cinp4) {
            const int v = i / cinp4;
            s4[v * LK4 + XO4 + (i - v * cinp4)] = onl_fin4(A, ab, xrow + 4 * i, E, rx[j]);
        }
    }
#pragma unroll
    for (int tap = 0; tap < 3; ++tap) {
        const int fr = fx + tap - 1;
        const bool live = fr >= 0 && fr < tin;
#pragma unroll
        for (int j = 0; j < NL; ++j) {
            const int i = tid + j * onl::NT;
            if (i < nz) {
                const int v = i / C4;
                s4[v * LK4 + tap * C4 + (i - v * C4)] =
                    live ? onl_fin4(A, ab, L.z + ((size_t)fr * nz + i) * 4, E, rz[tap][j]) : make_float4(0.f, 0.f, 0.f, 0.f);
            }
        }
    }
    // the K padding past Kt (layer 0: 196 -> 224) reads zeros (disjoint from the staged x)
    for (int i = tid; i < 17 * (32 * K32 - Kt); i += onl::NT) {
        const int v = i / (32 * K32 - Kt);
        sm[v * LK + Kt + (i - v * (32 * K32 - Kt))] = 0.f;
    }
    __syncthreads();
    if (tid == 0) onl_mark(A, task, 2);
    // identity residual of this thread's output (v = tid / 16, threads 0-271),
    // read before the reduction reuses the LDS
    const float res = (L.res == ONR_IDEN && tid < 272) ? sm[(tid >> 4) * LK + XO + c0 + (tid & 15)] : 0.f;
    // bf16x3 products on v_mfma_f32_16x16x32_bf16 (A = the staged rows, split into three
    // bf16 planes in registers: lane = joint lane & 15, K 8 (lane >> 4) ..; six products,
    // fp32 accumulation), joint 16 in fp32 FMAs
    const float* ra = sm + ri * LK + 8 * kk;
    const float* r16 = sm + 16 * LK + 8 * kk;
    onl_f32x4 acc[4] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
    float p16 = 0.f;
#pragma unroll
    for (int q = 0; q < NS; ++q) {
        const int sk = ksl + ONL_KSL * q;
        if (sk < K32) {
            const f32x4 lo = *reinterpret_cast<const f32x4*>(ra + 32 * sk), hi = *reinterpret_cast<const f32x4*>(ra + 32 * sk + 4);
            xbf16x8 x0, x1, x2;
            xsplit8(lo, hi, x0, x1, x2);
            onl_f32x4& a0 = acc[2 * q], &a1 = acc[2 * q + 1];
            a0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x2, w[q][0], a0, 0, 0, 0);
            a1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x1, w[q][1], a1, 0, 0, 0);
            a0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x0, w[q][2], a0, 0, 0, 0);
            a1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x1, w[q][0], a1, 0, 0, 0);
            a0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x0, w[q][1], a0, 0, 0, 0);
            a1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x0, w[q][0], a1, 0, 0, 0);
            const f32x4 l16 = *reinterpret_cast<const f32x4*>(r16 + 32 * sk), h16 = *reinterpret_cast<const f32x4*>(r16 + 32 * sk + 4);
#pragma unroll
            for (int e = 0; e < 4; ++e) p16 = fmaf(l16[e], wf[q][0][e], p16);
#pragma unroll
            for (int e = 0; e < 4; ++e) p16 = fmaf(h16[e], wf[q][1][e], p16);
        }
    }
    const onl_f32x4 accs = (acc[0] + acc[1]) + (acc[2] + acc[3]);
    if (tid == 0) onl_mark(A, task, 3);
    onl_reduce_mfma(accs, p16, sm, false);
    if (tid == 0) onl_mark(A, task, 4);
    if (tid < 272) {
        const float r = sm[onl::SMF + onl::RED + tid] + bt + res;
        st1t(ab, L.out + (size_t)(t * 17 + (tid >> 4)) * C + c0 + (tid & 15), r > 0.f ? r : 0.f, E);
    }
    if (tid == 0) onl_mark(A, task, 5);
}

// ---- the head: task idx = hidden units 16 idx .. 16 idx + 15 (one per wave) of
// pose_regressor.0 + LeakyReLU, and right away their share of pose_regressor.3:
// part[idx][o] = sum_u W3[o][16 idx + u] h[16 idx + u] (threads o < pose_dim, the 16
// W3 columns prefetched). The last head task to finish (its counter add returns
// ngroups - 1) sums the parts in task order, + b3, and writes the pose: no
// separate second-layer task and dependency hop.
__device__ void onl_head(const OnlineArgs* __restrict__ A, int p, int idx, float* sm, int task, const unsigned E) {
    const OnlinePhase& ph = A->ph[p];
    int tid = threadIdx.x;
    asm volatile("" : "+v"(tid));
    const int u = tid >> 6, lane = tid & 63;
    const int j = 16 * idx + u;                         // hidden unit of this wave
    const int nout = A->hidden, npose = A->pose_dim;
    const int K4 = A->feat >> 2;
    const float4* w4 = reinterpret_cast<const float4*>(A->w0 + (size_t)(j < nout ? j : 0) * 4 * K4);
    float4 w[ONL_MAXHC];
#pragma unroll
    for (int i = 0; i < ONL_MAXHC; ++i) {
        const int k = lane + 64 * i;
        w[i] = (k < K4 && j < nout) ? w4[k] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
    const float b = j < nout ? A->b0[j] : 0.f;
    // this task's 16 columns of W3, staged in LDS (the reduction area) before the wait
    float* hs = sm + onl::SMF;          // [16] hidden values, then [npose][16] W3 columns
    float* hw3 = hs + 16;
    for (int i = tid; i < 16 * npose; i += onl::NT) hw3[i] = A->w3[(size_t)(i >> 4) * nout + 16 * idx + (i & 15)];
#pragma unroll
    for (int i = 0; i < ONL_MAXHC; ++i) onl_hold(w[i]);
    if (tid == 0) onl_mark(A, task, 1);
    float4* s4 = reinterpret_cast<float4*>(sm);
    const Act ab = act_of(A);
    const float* in = A->L[A->nl - 1].out;   // the (17*C) feature of frame 0
    {
        constexpr int NL = (ONL_MAXHC * 64 + onl::NT - 1) / onl::NT;
        u32x4 r[NL];
#pragma unroll
        for (int j = 0; j < NL; ++j) {
            const int i = tid + j * onl::NT;
            if (i < K4) r[j] = ld4raw(ab, in + 4 * i);
        }
#pragma unroll
        for (int j = 0; j < NL; ++j) {
            const int i = tid + j * onl::NT;
            if (i < K4) s4[i] = onl_fin4(A, ab, in + 4 * i, E, r[j]);
        }
    }
    __syncthreads();
    if (tid == 0) onl_mark(A, task, 2);
    float acc = 0.f;
#pragma unroll
    for (int i = 0; i < ONL_MAXHC; ++i) {
        const int k = lane + 64 * i;
        if (k < K4) acc = fma4(w[i], s4[k], acc);
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off);
    __shared__ int s_lastp;
    if (lane == 0) {
        const float r = acc + b;
        hs[u] = j < nout ? (r > 0.f ? r : 0.01f * r) : 0.f;
    }
    __syncthreads();
    if (tid < npose) {
        float q = 0.f;
#pragma unroll
        for (int e = 0; e < 16; ++e) q = fmaf(hw3[16 * tid + e], hs[e], q);
        st1c(ab, A->hpart + (size_t)idx * npose + tid, q);
    }
    // stores complete in every wave, then count this task; the last one finishes the pose
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
        onl_mark(A, task, 5);
        s_lastp = __hip_atomic_fetch_add(A->cnt + ph.cbase, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == ph.ngroups - 1;
    }
    __syncthreads();
    if (!s_lastp) return;
    const int c = cnt_load(A->count);
    if (tid < npose) {
        float r = A->b3[tid];
        for (int k0 = 0; k0 < ph.ngroups; k0 += 32) {   // 32 loads in flight, summed in task order
            float v[32];
#pragma unroll
            for (int k = 0; k < 32; ++k)
                v[k] = k0 + k < ph.ngroups ? __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                                                 ab.r, act_off(ab, A->hpart + (size_t)(k0 + k) * npose + tid), 0, CPOL_SC1))
                                           : 0.f;
#pragma unroll
            for (int k = 0; k < 32; ++k)
                if (k0 + k < ph.ngroups) r += v[k];
        }
        A->pose[tid] = r;
        __hip_atomic_store(A->pose_host + tid, r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    if (tid == 0)
        __hip_atomic_store(A->pose_host + npose, cnt_load(A->err) ? 1.f : 0.f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    // the pose and flag stores (system scope, to pinned host memory) complete in
    // every wave before the host is told (no L2 write-back fence: ~23 us
    // measured); the rest of the launch's bookkeeping (counters, count, ticket) is
    // on the device and ordered before the next launch by the stream
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) __hip_atomic_store(A->done_host, stream_next_count(c, A->W), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ __launch_bounds__(1024) void online_kernel(const OnlineArgs* __restrict__ A) {
    __shared__ float4 sm4[onl::SMT / 4];
    __shared__ int s_task, s_last;
    float* sm = reinterpret_cast<float*>(sm4);
    const int tid = threadIdx.x;
    // this launch's activation tag (count: frames pushed before it, bumped by the previous launch's last workgroup)
    const unsigned E = (unsigned)(cnt_load(A->count) & 1) << 31;
    for (;;) {
        if (tid == 0) s_task = __hip_atomic_fetch_add(A->ticket, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __syncthreads();
        const int task = s_task;
        if (task >= A->ntasks) break;
        if (tid == 0) onl_mark(A, task, 0);
        int p = 0;
        while (p + 1 < A->nph && task >= A->ph[p + 1].task0) ++p;
        const int idx = task - A->ph[p].task0;
        if (task == 0) {
            // the pushed frame into the ring. Slot count % W holds frame count - W,
            // which no task of this launch reads (frames count - 2h .. count - 1 come
            // from the ring, frame count from pinned host memory). Task 0 is in every
            // head task's dependency cone and waits for the load before its own
            // output stores, so the frame has been read before the host is signalled
            // and may overwrite its frame buffer.
            const int c = cnt_load(A->count);
            if (tid < 17 * 3) A->ring[(size_t)(c % A->W) * 17 * 3 + tid] = A->frame[tid];
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        switch (A->ph[p].kind) {
            case ONP_G: onl_gcn(A, p, idx, sm, task, E); break;
            case ONP_T: onl_tconv(A, p, idx, sm, task, E); break;
            default: onl_head(A, p, idx, sm, task, E); break;
        }
        if (tid == 0 && A->trace) {
            onl_mark(A, task, 6);
            A->trace[8 * (size_t)task + 7] = blockIdx.x;
        }
        __syncthreads();   // s_task is rewritten next
    }
    // the last workgroup out leaves the scheduling state zero for the next launch
    if (tid == 0) s_last = __hip_atomic_fetch_add(A->done, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == (int)gridDim.x - 1;
    __syncthreads();
    if (s_last) {
        for (int i = tid; i < A->ncnt; i += onl::NT) A->cnt[i] = 0;
        if (tid == 0) {
            // every task has read the count (the ring append and the host signal are
            // the last head task's)
            A->count[0] = stream_next_count(cnt_load(A->count), A->W);
            A->ticket[0] = 0;
            A->done[0] = 0;
            // the last head task already published the flag to pose_host; a timeout
            // must not leak into the next launch's waits
            A->err[0] = 0;
        }
    }
}

hipError_t launch_online(const OnlineArgs* dev_args, int grid, hipStream_t st) {
    if (grid <= 0) return hipErrorInvalidValue;
    (void)hipGetLastError();
    hipLaunchKernelGGL(online_kernel, dim3(grid), dim3(onl::NT), 0, st, dev_args);
    return hipGetLastError();
}

}  // namespace tik
