// mfmabench.hip — cycles per v_mfma_f32_16x16x32_bf16 for dependent chains
// (srcC = the previous MFMA's result) against interleaved independent
// accumulators, at 1 and 2 waves per SIMD. Numbers only.
//   hipcc --offload-arch=gfx950 -O3 scripts/mfmabench.hip -o build/mfmabench
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

// MODE 0: 2 accumulators, 6-long chains back to back (a a a a a a b b b b b b)
// MODE 1: 2 accumulators interleaved (a b a b ...)
// MODE 2: 4 accumulators, chains of 6 interleaved round-robin (a b c d a b c d ...), 24 per iteration -> scaled
// MODE 3: 1 accumulator, 12-long chain
template <int MODE>
__global__ __launch_bounds__(512) void k(const bf16x8* in, float* out, int iters, unsigned long long* cyc) {
    bf16x8 x0 = in[threadIdx.x & 63], x1 = in[64 + (threadIdx.x & 63)], x2 = in[128 + (threadIdx.x & 63)];
    f32x4 a = {0, 0, 0, 0}, b = a, c = a, d = a;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; ++it) {
        if (MODE == 0) {
#pragma unroll
            for (int q = 0; q < 6; ++q) {
                a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x0, x1, a, 0, 0, 0);
                __builtin_amdgcn_sched_barrier(0);
            }
#pragma unroll
            for (int q = 0; q < 6; ++q) {
                b = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x1, x2, b, 0, 0, 0);
                __builtin_amdgcn_sched_barrier(0);
            }
        } else if (MODE == 1) {
#pragma unroll
            for (int q = 0; q < 6; ++q) {
                a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x0, x1, a, 0, 0, 0);
                __builtin_amdgcn_sched_barrier(0);
                b = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x1, x2, b, 0, 0, 0);
                __builtin_amdgcn_sched_barrier(0);
            }
        } else if (MODE == 2) {
#pragma unroll
            for (int q = 0; q < 3; ++q) {
                a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x0, x1, a, 0, 0, 0);
                b = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x1, x2, b, 0, 0, 0);
                c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x2, x0, c, 0, 0, 0);
                d = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x0, x2, d, 0, 0, 0);
            }
        } else {
#pragma unroll
            for (int q = 0; q < 12; ++q) {
                a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x0, x1, a, 0, 0, 0);
                __builtin_amdgcn_sched_barrier(0);
            }
        }
        __builtin_amdgcn_sched_barrier(0);
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * blockDim.x + threadIdx.x] = a[0] + b[1] + c[2] + d[3];
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

int main() {
    bf16x8* in;
    float* out;
    unsigned long long* cyc;
    std::vector<unsigned short> h(192 * 8, 0x3f80);
    if (hipMalloc(&in, 192 * 16) || hipMalloc(&out, 256 * 512 * 4) || hipMalloc(&cyc, 256 * 8)) return 1;
    if (hipMemcpy(in, h.data(), 192 * 16, hipMemcpyHostToDevice)) return 1;
    const int iters = 2000;
    for (int waves : {4, 8}) {
        for (int mode = 0; mode < 4; ++mode) {
            for (int rep = 0; rep < 2; ++rep) {
                dim3 g(256), b(64 * waves);
                hipEvent_t e0, e1;
                if (hipEventCreate(&e0) || hipEventCreate(&e1) || hipEventRecord(e0, 0)) return 1;
                if (mode == 0) hipLaunchKernelGGL(k<0>, g, b, 0, 0, in, out, iters, cyc);
                if (mode == 1) hipLaunchKernelGGL(k<1>, g, b, 0, 0, in, out, iters, cyc);
                if (mode == 2) hipLaunchKernelGGL(k<2>, g, b, 0, 0, in, out, iters, cyc);
                if (mode == 3) hipLaunchKernelGGL(k<3>, g, b, 0, 0, in, out, iters, cyc);
                if (hipEventRecord(e1, 0) || hipDeviceSynchronize()) return 1;
                float ms = 0;
                if (hipEventElapsedTime(&ms, e0, e1)) return 1;
                const double tf = 2.0 * 16 * 16 * 32 * 12.0 * iters * waves * 256 / (ms * 1e-3) / 1e12;
                std::vector<unsigned long long> c(256);
                if (hipMemcpy(c.data(), cyc, 256 * 8, hipMemcpyDeviceToHost)) return 1;
                double s = 0;
                for (auto v : c) s += (double)v;
                s /= 256;
                // s_memtime runs at 100 MHz on gfx9 parts: report raw ticks per MFMA of one wave and per SIMD
                printf("waves/CU %d mode %d: memtime ticks per iteration (12 MFMAs/wave) %.3f  kernel %.3f ms  %.1f TFLOP/s (dense bf16 peak ~2516)\n",
                       waves, mode, s / iters, ms, tf);
            }
        }
    }
    return 0;
}
