// online.hip — the online-IK step (BASELINE.json config #5) as one dataflow
// kernel; see online.h for the task list and why only the first frames of
// each layer are computed.
//
// Arithmetic: fp32 FMAs in VALU (exact fp32 products, like the oracle).
// Every task is one 1024-thread workgroup (16 waves: 4 per SIMD, so LDS and
// memory latency overlap); the task's weight chunks are loaded into registers
// BEFORE it waits for its inputs, and the input rows are staged into LDS with
// coalesced 16-B loads. (A first 256-thread version spent 4-8 us per
// temporal-conv task in its one-wave-per-SIMD compute loop.)
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
constexpr int SMF = 3 * 17 * ONL_MAXC + 17 * ONL_MAXC;   // staged rows, floats (69,632 B)
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
// root-relative, data_bn -> 17 rows of 4 floats at dst (threads 0-16).
// The pushed frame is read from pinned host memory; older frames from the ring,
// which the last workgroup of the launch appends the pushed frame to.
__device__ void onl_raw_rows(const OnlineArgs* __restrict__ A, int k, float4* dst) {
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
    dst[v] = make_float4(o[0], o[1], o[2], 0.f);
}

// Thread roles of a G / T task: 1024 threads = 16 output channels (co = tid & 15)
// x 64 K slices of 4-float chunks (ks = tid >> 4: chunks ks, ks + 64, ...);
// every thread accumulates all 17 joints of its channel over its slice.
// Partial sums -> y[v][co] (LDS): the 4 slices of a wave by permlane swaps,
// the 16 waves through LDS, in a fixed order (deterministic for any grid).
__device__ __forceinline__ void onl_reduce17(float (&acc)[17], float* sm) {
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
#pragma unroll
    for (int v = 0; v < 17; ++v) {   // lane rows 0+1, 2+3, then (0+1)+(2+3): VALU swaps, no LDS
        // inline asm: hipcc's permlane swap builtins return the pair's second value
        // as a copy of the first when both feed one add (wrong code, seen in the ISA)
        float x = acc[v], y = acc[v];
        asm volatile("s_nop 1\n\tv_permlane16_swap_b32 %0, %1" : "+v"(x), "+v"(y));
        float u = x + y, w = x + y;
        asm volatile("s_nop 1\n\tv_permlane32_swap_b32 %0, %1" : "+v"(u), "+v"(w));
        acc[v] = u + w;
    }
    __syncthreads();   // every staged-row read done: the LDS is reused
    float* red = sm;   // [16 waves][17 v][16 co]
    if (lane < 16) {
#pragma unroll
        for (int v = 0; v < 17; ++v) red[(wave * 17 + v) * 16 + lane] = acc[v];
    }
    __syncthreads();
    if (tid < 272) {
        float s = 0.f;
#pragma unroll
        for (int k = 0; k < 16; ++k) s += red[k * 272 + tid];
        sm[16 * 272 + tid] = s;   // y[v][co] at tid = 16 v + co
    }
    __syncthreads();
}

// ---- G_L(f, 16 channels): z = ReLU(bias2 + sum_v A[v][w] (x . wg^T)[v])
__device__ void onl_gcn(const OnlineArgs* __restrict__ A, int p, int idx, float* sm, int task) {
    const OnlinePhase& ph = A->ph[p];
    const OnlineLayer& L = A->L[ph.layer];
    const int tid = threadIdx.x, co = tid & 15, ks = tid >> 4;
    const int f = idx / ph.ngroups, cg = idx - f * ph.ngroups;
    const int cinp = L.cinp, K4 = cinp >> 2, cout = L.cout, c0 = cg * 16;
    static_assert(ONL_MAXC / 4 <= 64, "one gcn weight chunk per thread");
    // operands that do not depend on the input: weight chunk, mix column, bias
    float4 w = ks < K4 ? reinterpret_cast<const float4*>(L.wg + (size_t)(c0 + co) * cinp)[ks]
                             : make_float4(0.f, 0.f, 0.f, 0.f);
    const int wo = tid >> 4;   // mix output (wo, co) of threads 0-271
    float am[17], b = 0.f;
#pragma unroll
    for (int v = 0; v < 17; ++v) am[v] = tid < 272 ? L.amix[v * 17 + wo] : 0.f;
    if (tid < 272) b = L.bias2[wo * cout + c0 + co];
    onl_hold(w);
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
        onl_raw_rows(A, f, s4);
    } else {
        const float* xr = L.x + (size_t)f * 17 * cinp;
        for (int i = tid; i < 17 * K4; i += onl::NT) s4[i] = ld4c(ab, xr + 4 * i);
    }
    __syncthreads();
    if (tid == 0) onl_mark(A, task, 2);
    float acc[17];
#pragma unroll
    for (int v = 0; v < 17; ++v) acc[v] = ks < K4 ? fma4(w, s4[v * K4 + ks], 0.f) : 0.f;
    if (tid == 0) onl_mark(A, task, 3);
    onl_reduce17(acc, sm);
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
__device__ void onl_tconv(const OnlineArgs* __restrict__ A, int p, int idx, float* sm, int task) {
    const OnlinePhase& ph = A->ph[p];
    const OnlinePhase& pg = A->ph[p - 1];   // this layer's gcn
    const OnlineLayer& L = A->L[ph.layer];
    const int tid = threadIdx.x, co = tid & 15, ks = tid >> 4;
    const int t = idx / ph.ngroups, cg = idx - t * ph.ngroups;
    const int C = L.cout, C4 = C >> 2, K4t = 3 * C4, cinp4 = L.cinp >> 2;
    const int K4 = K4t + (L.res == ONR_CONV ? cinp4 : 0), c0 = cg * 16;
    const int s = L.stride, tin = L.tin, fx = s * t;
    constexpr int NW = (3 * ONL_MAXC + ONL_MAXC) / 4 / 64;   // 4 chunks per thread
    float4 w[NW];
    const float4* wt4 = reinterpret_cast<const float4*>(L.wt + (size_t)(c0 + co) * 3 * C);
    const float4* wr4 = reinterpret_cast<const float4*>(L.res == ONR_CONV ? L.wr + (size_t)(c0 + co) * L.cinp : L.wt);
#pragma unroll
    for (int i = 0; i < NW; ++i) {
        const int j = ks + 64 * i;
        w[i] = j < K4t ? wt4[j] : (j < K4 ? wr4[j - K4t] : make_float4(0.f, 0.f, 0.f, 0.f));
    }
    const float bt = L.biasT[c0 + co];
#pragma unroll
    for (int i = 0; i < NW; ++i) onl_hold(w[i]);
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
        const int fr = fx + tap - 1;
        s4[i] = (fr >= 0 && fr < tin) ? ld4c(ab, L.z + ((size_t)fr * nz + (i - tap * nz)) * 4) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
    float4* xs4 = s4 + 3 * nz;
    const float* xs = reinterpret_cast<const float*>(xs4);
    const float* xrow = L.x + (size_t)fx * 17 * L.cinp;
    if (ph.layer == 0 && L.res != ONR_ZERO)
        onl_raw_rows(A, fx, xs4);
    else if (L.res != ONR_ZERO)   // residual rows: the conv's K segment, or the identity term
        for (int i = tid; i < 17 * cinp4; i += onl::NT) xs4[i] = ld4c(ab, xrow + 4 * i);
    __syncthreads();
    if (tid == 0) onl_mark(A, task, 2);
    // identity residual of this thread's output (v = tid / 16, threads 0-271),
    // read before the reduction reuses the LDS
    const float res = (L.res == ONR_IDEN && tid < 272) ? xs[(tid >> 4) * C + c0 + co] : 0.f;
    float acc[17];
#pragma unroll
    for (int v = 0; v < 17; ++v) acc[v] = 0.f;
#pragma unroll
    for (int i = 0; i < NW; ++i) {
        const int j = ks + 64 * i;
        if (j < K4t) {
            const int tap = j >= 2 * C4 ? 2 : (j >= C4 ? 1 : 0);
            const float4* zr = s4 + tap * nz + (j - tap * C4);
#pragma unroll
            for (int v = 0; v < 17; ++v) acc[v] = fma4(w[i], zr[v * C4], acc[v]);
        } else if (j < K4) {
            const float4* xr = xs4 + (j - K4t);
#pragma unroll
            for (int v = 0; v < 17; ++v) acc[v] = fma4(w[i], xr[v * cinp4], acc[v]);
        }
    }
    if (tid == 0) onl_mark(A, task, 3);
    onl_reduce17(acc, sm);
    if (tid == 0) onl_mark(A, task, 4);
    if (tid < 272) {
        const float r = sm[16 * 272 + tid] + bt + res;
        st1c(ab, L.out + (size_t)(t * 17 + (tid >> 4)) * C + c0 + co, r > 0.f ? r : 0.f);
    }
    onl_release(A, ph.cbase + t, task);
}

// ---- H0 (16 hidden units, one per wave) and H1 (16 pose values, one per wave)
template <bool FIRST>
__device__ void onl_head(const OnlineArgs* __restrict__ A, int p, int idx, float* sm, int task) {
    const OnlinePhase& ph = A->ph[p];
    const OnlinePhase& pp = A->ph[p - 1];
    const int tid = threadIdx.x, u = tid >> 6, lane = tid & 63;
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
    if (!FIRST && idx == 0 && tid == 0) A->pose_host[A->pose_dim] = cnt_load(A->err) ? 1.f : 0.f;
    if (lane == 0 && j < nout) {
        float r = acc + b;
        if (FIRST) {
            st1c(ab, A->hid + j, r > 0.f ? r : 0.01f * r);
        } else {
            A->pose[j] = r;
            A->pose_host[j] = r;
        }
    }
    if (FIRST) onl_release(A, ph.cbase, task);
    else __syncthreads();
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
