// online.hip — the online-IK step (BASELINE.json config #5) as one dataflow
// kernel; see online.h for the task list and why only the first frames of
// each layer are computed.
//
// Arithmetic: the gcn and temporal-conv tasks on the exact fp32 MFMA
// (v_mfma_f32_16x16x4_f32: fp32 products, fp32 accumulation, like the
// oracle); the head in fp32 VALU FMAs. Every task is one 1024-thread
// workgroup (16 waves: 4 per SIMD, so LDS and memory latency overlap); the
// task's weights are loaded into registers BEFORE it waits for its inputs,
// and the input rows are staged into LDS with coalesced 16-B loads. A task's
// 17 joints x 16 channels are two 16 x 16 MFMA blocks; its K (input channels,
// x 3 taps, + the residual conv) is split over 8 wave pairs, and the 8 partial
// blocks are summed through LDS in a fixed order (deterministic for any grid).
// (Round 2's VALU version spent 2-3 us per temporal-conv task in its FMAs and
// the 64-way reduction, profiles/r02_v2_online_trace.txt.)
//
// Synchronisation (cross-XCD: each XCD has its own L2). Every activation a
// task hands to another task is stored and loaded with device-scope cache
// policy (sc1: written through to / read from the device coherence point), the
// encoding the compiler uses for agent-scope atomic loads and stores; the
// weights stay ordinary cached loads (read-only for the whole launch). A
// producer waits for its stores (vmcnt(0) in every wave) and then bumps the
// frame's completion counter (device-scope atomic); a consumer polls the
// counter and only then issues its loads. No L2 write-back or invalidate: a
// first version with agent-scope release/acquire fences (buffer_wbl2 /
// buffer_inv per task) spent most of its time in them (213 us per step).
// Tickets are taken in topological order, so the smallest unfinished taken
// task always has its inputs complete: no deadlock, whatever the residency.
// Every wait is bounded (0.5 s): a timeout sets *err and the task proceeds,
// so the grid always drains; the host reports the error.
#include "online.h"

namespace tik {

namespace onl {
constexpr int NT = 1024;
constexpr int LDP = 4;                                    // row padding (floats): MFMA A reads conflict-free
constexpr int SMF = 4 * 17 * (ONL_MAXC + LDP);            // staged rows, floats (70,720 B)
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
__device__ __forceinline__ float4 ld4c(const Act& b, const float* p) {
    return __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(b.r, act_off(b, p), 0, CPOL_SC1));
}
__device__ __forceinline__ void st4c(const Act& b, float* p, const float4 v) {
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), b.r, act_off(b, p), 0, CPOL_SC1);
}
__device__ __forceinline__ void st1c(const Act& b, float* p, const float v) {
    __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v), b.r, act_off(b, p), 0, CPOL_SC1);
}

// thread 0 only: wait until *cnt[ci] >= target
__device__ void onl_wait(const OnlineArgs* __restrict__ A, int ci, int target) {
    int* p = A->cnt + ci;
    if (cnt_load(p) >= target) return;
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    while (cnt_load(p) < target) {
        if (cnt_load(A->err)) return;
        __builtin_amdgcn_s_sleep(1);
        if (__builtin_amdgcn_s_memrealtime() - t0 > onl::TIMEOUT) {
            __hip_atomic_fetch_or(A->err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            return;
        }
    }
}

// all threads: this task's stores are complete and visible device-wide, then count it
__device__ void onl_mark(const OnlineArgs* __restrict__ A, int task, int k);
__device__ void onl_release(const OnlineArgs* __restrict__ A, int ci, int task) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        onl_mark(A, task, 5);
        __hip_atomic_fetch_add(A->cnt + ci, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

// debug trace: slot k of task `task` (thread 0 only)
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
// which the last workgroup of the launch appends the pushed frame to.
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

// MFMA roles of a G / T task: wave w takes the K steps (4 input channels each)
// w, w + 16, ... One v_mfma_f32_16x16x4_f32 per step covers joints 0-15: A = the
// staged rows (lane: joint l & 15, K element l >> 4), B = the weights (lane: output
// channel c0 + (l & 15), K element l >> 4), D lane l = joints 4 (l >> 4) + e,
// channel c0 + (l & 15). Joint 16 is one VALU FMA per step on the same B register
// (lane: channel l & 15, K element l >> 4), its 4 K elements summed across the
// lane groups before the wave's partials go to LDS (a second 16-row MFMA block
// for one joint would double the MFMA time).
typedef float onl_f32x4 __attribute__((ext_vector_type(4)));
constexpr int ONL_KSL = 16;   // K slices (one per wave)

// the 16 waves' partials (acc: joints 0-15; p16: joint 16 of lane l's channel and K
// element) -> y[v][co] at sm[16 * 272 + 16 v + co] (threads 0-271 read it), summed in a fixed order
__device__ __forceinline__ void onl_reduce_mfma(const onl_f32x4 acc, float p16, float* sm) {
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    p16 += __shfl_xor(p16, 16);
    p16 += __shfl_xor(p16, 32);
    __syncthreads();   // every staged-row read done: the LDS is reused
    float* red = sm;   // [16 waves][17 joints][16 co]
#pragma unroll
    for (int e = 0; e < 4; ++e) red[wave * 272 + (4 * (lane >> 4) + e) * 16 + (lane & 15)] = acc[e];
    if (lane < 16) red[wave * 272 + 16 * 16 + lane] = p16;
    __syncthreads();
    if (tid < 272) {
        float s = 0.f;
#pragma unroll
        for (int k = 0; k < ONL_KSL; ++k) s += red[k * 272 + tid];
        sm[16 * 272 + tid] = s;
    }
    __syncthreads();
}

// ---- G_L(f, 16 channels): z = ReLU(bias2 + sum_v A[v][w] (x . wg^T)[v])
__device__ void onl_gcn(const OnlineArgs* __restrict__ A, int p, int idx, float* sm, int task) {
    const OnlinePhase& ph = A->ph[p];
    const OnlineLayer& L = A->L[ph.layer];
    int tid = threadIdx.x;
    asm volatile("" : "+v"(tid));   // lane-derived offsets are made per task, not hoisted across the task loop (spills)
    const int lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int ksl = wave, kk = lane >> 4, ri = lane & 15;
    const int f = idx / ph.ngroups, cg = idx - f * ph.ngroups;
    const int cinp = L.cinp, K4 = cinp >> 2, cout = L.cout, c0 = cg * 16;
    const int LD = cinp + onl::LDP;
    constexpr int NS = ONL_MAXC / 4 / ONL_KSL;   // K steps per wave (at most)
    static_assert(ONL_MAXC / 4 <= NS * ONL_KSL, "gcn K steps");
    // operands that do not depend on the input: this wave's weight column, mix column, bias
    float w[NS];
#pragma unroll
    for (int q = 0; q < NS; ++q) {
        const int sk = ksl + ONL_KSL * q;
        w[q] = sk < K4 ? L.wg[(size_t)(c0 + ri) * cinp + 4 * sk + kk] : 0.f;
    }
    const int wo = tid >> 4, co = tid & 15;   // mix output (wo, co) of threads 0-271
    float am[17], b = 0.f;
#pragma unroll
    for (int v = 0; v < 17; ++v) am[v] = tid < 272 ? L.amix[v * 17 + wo] : 0.f;
    if (tid < 272) b = L.bias2[wo * cout + c0 + co];
#pragma unroll
    for (int q = 0; q < NS; ++q) onl_hold(w[q]);
    onl_hold(b);
#pragma unroll
    for (int v = 0; v < 17; ++v) onl_hold(am[v]);
    if (tid == 0) {
        if (ph.layer > 0) {   // the previous temporal conv's frame f
            const OnlinePhase& pp = A->ph[p - 1];
            onl_wait(A, pp.cbase + f, pp.ngroups);
        }
        onl_mark(A, task, 1);
    }
    __syncthreads();
    float4* s4 = reinterpret_cast<float4*>(sm);
    const Act ab = act_of(A);
    if (ph.layer == 0) {
        onl_raw_rows(A, f, s4, LD / 4);
    } else {
        const float* xr = L.x + (size_t)f * 17 * cinp;
        for (int i = tid; i < 17 * K4; i += onl::NT) {
            const int v = i / K4;
            s4[v * (LD / 4) + (i - v * K4)] = ld4c(ab, xr + 4 * i);
        }
    }
    __syncthreads();
    if (tid == 0) onl_mark(A, task, 2);
    const float* xa = sm + ri * LD + kk;
    const float* x16 = sm + 16 * LD + kk;
    onl_f32x4 acc[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
    float p16 = 0.f;
#pragma unroll
    for (int q = 0; q < NS; ++q) {
        const int sk = ksl + ONL_KSL * q;
        if (sk < K4) {
            acc[q & 1] = __builtin_amdgcn_mfma_f32_16x16x4f32(xa[4 * sk], w[q], acc[q & 1], 0, 0, 0);
            p16 = fmaf(x16[4 * sk], w[q], p16);
        }
    }
    if (tid == 0) onl_mark(A, task, 3);
    onl_reduce_mfma(acc[0] + acc[1], p16, sm);
    if (tid == 0) onl_mark(A, task, 4);
    const float* y = sm + 16 * 272;
    if (tid < 272) {
        float s = b;
#pragma unroll
        for (int v = 0; v < 17; ++v) s = fmaf(am[v], y[v * 16 + co], s);
        st1c(ab, L.z + (size_t)(f * 17 + wo) * cout + c0 + co, s > 0.f ? s : 0.f);
    }
    onl_release(A, ph.cbase + f, task);
}

// ---- T_L(t, 16 channels): out = ReLU(sum_tap z[s t + tap - 1] . wt_tap^T + bias + residual)
// Staged operand rows, one per joint, in K order: [z tap 0 (C) | tap 1 | tap 2 | block
// input x (cinp: the residual conv's K segment, or the identity term)], so K step sk
// reads floats 4 sk .. of the row (no per-step tap decode between the MFMAs)
__device__ void onl_tconv(const OnlineArgs* __restrict__ A, int p, int idx, float* sm, int task) {
    const OnlinePhase& ph = A->ph[p];
    const OnlinePhase& pg = A->ph[p - 1];   // this layer's gcn
    const OnlineLayer& L = A->L[ph.layer];
    int tid = threadIdx.x;
    asm volatile("" : "+v"(tid));   // lane-derived offsets are made per task, not hoisted across the task loop (spills)
    const int lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int ksl = wave, kk = lane >> 4, ri = lane & 15;
    const int t = idx / ph.ngroups, cg = idx - t * ph.ngroups;
    const int C = L.cout, C4 = C >> 2, K4t = 3 * C4, cinp4 = L.cinp >> 2;
    const bool rconv = L.res == ONR_CONV;
    const int K4 = K4t + (rconv ? cinp4 : 0), c0 = cg * 16;
    const int s = L.stride, tin = L.tin, fx = s * t;
    const int LK = 3 * C + L.cinp + onl::LDP, LK4 = LK / 4;   // staged row (floats)
    constexpr int NS = (3 * ONL_MAXC + ONL_MAXC) / 4 / ONL_KSL;   // K steps per wave (at most): 16
    // this wave's weights: K step sk < K4t is tap sk / C4, channels 4 (sk % C4) ..; then the residual conv
    float w[NS];
    const float* wt = L.wt + (size_t)(c0 + ri) * 3 * C;
    const float* wr = rconv ? L.wr + (size_t)(c0 + ri) * L.cinp : L.wt;
#pragma unroll
    for (int q = 0; q < NS; ++q) {
        const int sk = ksl + ONL_KSL * q;
        w[q] = sk < K4t ? wt[4 * sk + kk] : (sk < K4 ? wr[4 * (sk - K4t) + kk] : 0.f);
    }
    const float bt = L.biasT[c0 + (tid & 15)];
#pragma unroll
    for (int q = 0; q < NS; ++q) onl_hold(w[q]);
    if (tid == 0) {
#pragma unroll
        for (int tap = 0; tap < 3; ++tap) {
            const int fr = fx + tap - 1;
            if (fr >= 0 && fr < tin) onl_wait(A, pg.cbase + fr, pg.ngroups);
        }
        onl_mark(A, task, 1);
    }
    __syncthreads();
    float4* s4 = reinterpret_cast<float4*>(sm);
    const int nz = 17 * C4;
    const Act ab = act_of(A);
    for (int i = tid; i < 3 * nz; i += onl::NT) {
        const int tap = i >= 2 * nz ? 2 : (i >= nz ? 1 : 0);
        const int fr = fx + tap - 1, r = i - tap * nz, v = r / C4;
        s4[v * LK4 + tap * C4 + (r - v * C4)] =
            (fr >= 0 && fr < tin) ? ld4c(ab, L.z + ((size_t)fr * nz + r) * 4) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
    const float* xrow = L.x + (size_t)fx * 17 * L.cinp;
    if (ph.layer == 0 && L.res != ONR_ZERO)
        onl_raw_rows(A, fx, s4 + 3 * C4, LK4);
    else if (L.res != ONR_ZERO)   // residual rows: the conv's K segment, or the identity term
        for (int i = tid; i < 17 * cinp4; i += onl::NT) {
            const int v = i / cinp4;
            s4[v * LK4 + 3 * C4 + (i - v * cinp4)] = ld4c(ab, xrow + 4 * i);
        }
    __syncthreads();
    if (tid == 0) onl_mark(A, task, 2);
    // identity residual of this thread's output (v = tid / 16, threads 0-271),
    // read before the reduction reuses the LDS
    const float res = (L.res == ONR_IDEN && tid < 272) ? sm[(tid >> 4) * LK + 3 * C + c0 + (tid & 15)] : 0.f;
    const float* ra = sm + ri * LK + kk;
    const float* r16 = sm + 16 * LK + kk;
    // four independent accumulation chains (the MFMA's dependent latency), summed in a fixed order
    onl_f32x4 acc[4] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
    float p16 = 0.f;
#pragma unroll
    for (int q = 0; q < NS; ++q) {
        const int sk = ksl + ONL_KSL * q;
        if (sk < K4) {
            acc[q & 3] = __builtin_amdgcn_mfma_f32_16x16x4f32(ra[4 * sk], w[q], acc[q & 3], 0, 0, 0);
            p16 = fmaf(r16[4 * sk], w[q], p16);
        }
    }
    const onl_f32x4 accs = (acc[0] + acc[1]) + (acc[2] + acc[3]);
    if (tid == 0) onl_mark(A, task, 3);
    onl_reduce_mfma(accs, p16, sm);
    if (tid == 0) onl_mark(A, task, 4);
    if (tid < 272) {
        const float r = sm[16 * 272 + tid] + bt + res;
        st1c(ab, L.out + (size_t)(t * 17 + (tid >> 4)) * C + c0 + (tid & 15), r > 0.f ? r : 0.f);
    }
    onl_release(A, ph.cbase + t, task);
}

// ---- H0 (16 hidden units, one per wave) and H1 (16 pose values, one per wave)
template <bool FIRST>
__device__ void onl_head(const OnlineArgs* __restrict__ A, int p, int idx, float* sm, int task) {
    const OnlinePhase& ph = A->ph[p];
    const OnlinePhase& pp = A->ph[p - 1];
    int tid = threadIdx.x;
    asm volatile("" : "+v"(tid));
    const int u = tid >> 6, lane = tid & 63;
    const int j = 16 * idx + u;                         // output index
    const int nout = FIRST ? A->hidden : A->pose_dim;
    const int K4 = (FIRST ? A->feat : A->hidden) >> 2;
    const float4* w4 = reinterpret_cast<const float4*>((FIRST ? A->w0 : A->w3) + (size_t)(j < nout ? j : 0) * 4 * K4);
    float4 w[ONL_MAXHC];
#pragma unroll
    for (int i = 0; i < ONL_MAXHC; ++i) {
        const int k = lane + 64 * i;
        w[i] = (k < K4 && j < nout) ? w4[k] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
    const float b = j < nout ? (FIRST ? A->b0 : A->b3)[j] : 0.f;
#pragma unroll
    for (int i = 0; i < ONL_MAXHC; ++i) onl_hold(w[i]);
    if (tid == 0) {
        onl_wait(A, pp.cbase, pp.ngroups);   // T_last frame 0 / all of H0
        onl_mark(A, task, 1);
    }
    __syncthreads();
    float4* s4 = reinterpret_cast<float4*>(sm);
    const Act ab = act_of(A);
    const float* in = FIRST ? A->L[A->nl - 1].out : A->hid;
    for (int i = tid; i < K4; i += onl::NT) s4[i] = ld4c(ab, in + 4 * i);   // the (17*C) feature of frame 0 / the hidden vector
    __syncthreads();
    float acc = 0.f;
#pragma unroll
    for (int i = 0; i < ONL_MAXHC; ++i) {
        const int k = lane + 64 * i;
        if (k < K4) acc = fma4(w[i], s4[k], acc);
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off);
    if (!FIRST && idx == 0 && tid == 0)
        __hip_atomic_store(A->pose_host + A->pose_dim, cnt_load(A->err) ? 1.f : 0.f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if (lane == 0 && j < nout) {
        float r = acc + b;
        if (FIRST) {
            st1c(ab, A->hid + j, r > 0.f ? r : 0.01f * r);
        } else {
            A->pose[j] = r;
            __hip_atomic_store(A->pose_host + j, r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
    if (FIRST) {
        onl_release(A, ph.cbase, task);
    } else {
        // the pose stores (system scope, to pinned host memory) complete before this
        // workgroup's done count, which the last workgroup waits for before it
        // signals the host (no L2 write-back fence: ~23 us measured)
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
    }
}

__global__ __launch_bounds__(1024) void online_kernel(const OnlineArgs* __restrict__ A) {
    __shared__ float4 sm4[onl::SMF / 4];
    __shared__ int s_task, s_last;
    float* sm = reinterpret_cast<float*>(sm4);
    const int tid = threadIdx.x;
    for (;;) {
        if (tid == 0) s_task = __hip_atomic_fetch_add(A->ticket, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __syncthreads();
        const int task = s_task;
        if (task >= A->ntasks) break;
        if (tid == 0) onl_mark(A, task, 0);
        int p = 0;
        while (p + 1 < A->nph && task >= A->ph[p + 1].task0) ++p;
        const int idx = task - A->ph[p].task0;
        switch (A->ph[p].kind) {
            case ONP_G: onl_gcn(A, p, idx, sm, task); break;
            case ONP_T: onl_tconv(A, p, idx, sm, task); break;
            case ONP_H0: onl_head<true>(A, p, idx, sm, task); break;
            default: onl_head<false>(A, p, idx, sm, task); break;
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
        // every task has read the ring and the count: append the pushed frame
        const int c = cnt_load(A->count);
        for (int i = tid; i < 17 * 3; i += onl::NT) A->ring[(size_t)(c % A->W) * 17 * 3 + i] = A->frame[i];
        if (tid == 0) {
            A->count[0] = c + 1;
            A->ticket[0] = 0;
            A->done[0] = 0;
            // the H1 task (done: every task has run) already published the flag to
            // pose_host; a timeout must not leak into the next launch's waits
            A->err[0] = 0;
            // every read of the pushed frame and every pose store is done: tell the
            // host (it spins on this word instead of waiting for the kernel's end)
            __hip_atomic_store(A->done_host, c + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
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
