// gapbench.hip — the idle time between two dependent kernels on one stream, by
// the first kernel's output store flavour (plain / nontemporal / sc1 / sc0 sc1 by
// inline asm) and size, and by launch shape (LDS bytes, workgroup size, grid) of
// a busy-waiting kernel. Read the gaps from `rocprofv3 --kernel-trace`.
//   hipcc --offload-arch=gfx950 -O3 scripts/gapbench.hip -o build/gapbench
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef float f4 __attribute__((ext_vector_type(4)));

template <int MODE>
__global__ __launch_bounds__(256) void writer(f4* __restrict__ o, size_t n4, float v) {
    for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n4; i += (size_t)gridDim.x * 256) {
        const f4 x = f4{v, v + 1.f, v + 2.f, v + 3.f};
        if (MODE == 0) o[i] = x;
        else if (MODE == 1) __builtin_nontemporal_store(x, o + i);
        else if (MODE == 2) asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(o + i), "v"(x) : "memory");
        else asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1" ::"v"(o + i), "v"(x) : "memory");
    }
}
__global__ void tiny(float* o) { if (threadIdx.x == 0) o[blockIdx.x] += 1.f; }

// busy kernel: every workgroup sleeps ~iters * 64 clocks, touches its LDS, writes one float
__global__ __launch_bounds__(512) void busy(float* o, int iters) {
    extern __shared__ float lds[];
    lds[threadIdx.x] = (float)threadIdx.x;
    for (int i = 0; i < iters; ++i) __builtin_amdgcn_s_sleep(1);
    __syncthreads();
    if (threadIdx.x == 0) o[blockIdx.x & 4095] = lds[(threadIdx.x + 1) % blockDim.x];
}

int main(int argc, char** argv) {
    const size_t mb = argc > 1 ? atoi(argv[1]) : 256;
    const size_t n4 = mb * (1 << 20) / 16;
    f4* o;
    float* t;
    if (hipMalloc(&o, n4 * 16) != hipSuccess || hipMalloc(&t, 16384 * 4) != hipSuccess) return 1;
    hipStream_t st;
    if (hipStreamCreate(&st) != hipSuccess) return 1;
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&busy), hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    for (int rep = 0; rep < 3; ++rep) {
        for (int m = 0; m < 5; ++m) {
            for (int k = 0; k < 4; ++k) {
                if (m == 0) hipLaunchKernelGGL(writer<0>, dim3(1024), dim3(256), 0, st, o, n4, 1.f);
                if (m == 1) hipLaunchKernelGGL(writer<1>, dim3(1024), dim3(256), 0, st, o, n4, 1.f);
                if (m == 2) hipLaunchKernelGGL(writer<2>, dim3(1024), dim3(256), 0, st, o, n4, 1.f);
                if (m == 3) hipLaunchKernelGGL(writer<3>, dim3(1024), dim3(256), 0, st, o, n4, 1.f);
                if (m == 4) hipLaunchKernelGGL(tiny, dim3(256), dim3(64), 0, st, t);
                hipLaunchKernelGGL(tiny, dim3(256), dim3(64), 0, st, t);
            }
        }
        // launch shapes: (grid, block, lds bytes)
        const int shapes[][3] = {{256, 512, 0}, {256, 512, 150 * 1024}, {256, 256, 80 * 1024}, {2048, 256, 0}, {4096, 512, 64 * 1024}, {32, 256, 80 * 1024}};
        for (auto& s : shapes)
            for (int k = 0; k < 4; ++k) hipLaunchKernelGGL(busy, dim3(s[0]), dim3(s[1]), s[2], st, t, 2000);
    }
    if (hipStreamSynchronize(st) != hipSuccess) return 1;
    printf("done %zu MB\n", mb);
    return 0;
}
