// dmabench.hip — ceiling of the operand paths the GEMMs use: global->LDS DMA
// (global_load_lds_dwordx4) vs global->VGPR (global_load_dwordx4), from an
// L2-resident buffer and from HBM, at 1-4 resident 256-thread workgroups/CU.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 scripts/dmabench.hip -o build/dmabench
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                                \
    do {                                                                                     \
        hipError_t e_ = (x);                                                                 \
        if (e_ != hipSuccess) {                                                              \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));        \
            exit(1);                                                                         \
        }                                                                                    \
    } while (0)

__device__ __forceinline__ void dma16(const unsigned char* g, unsigned char* l) {
    __builtin_amdgcn_global_load_lds(g, l, 16, 0, 0);
}

template <int NI, int LDSKB>
__global__ __launch_bounds__(256) void ldsdma_probe(const unsigned char* __restrict__ src, size_t mask, int iters,
                                                  int* sink) {
    __shared__ __attribute__((aligned(16))) unsigned char smem[LDSKB * 1024];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    size_t off = ((size_t)blockIdx.x * 256 * NI * 16 + (size_t)wave * NI * 1024 + lane * 16) & mask;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int j = 0; j < NI; ++j) {
            dma16(src + ((off + j * 1024) & mask), smem + ((wave * NI + j) * 1024) % (LDSKB * 1024));
        }
        off = (off + (size_t)gridDim.x * 256 * NI * 16) & mask;
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NI) : "memory");
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0 && smem[lane] == 123 && smem[1000] == 77) sink[0] = 1;
}

// fragment-shaped: each wave-instruction reads 16 rows x 64 B (4 lanes per row)
// of rows ROWB bytes apart, i.e. half lines, like a BK=32 f16 operand tile
template <int NI, int ROWB>
__global__ __launch_bounds__(256) void frag_probe(const unsigned char* __restrict__ src, size_t mask, int iters, int* sink) {
    __shared__ __attribute__((aligned(16))) unsigned char smem[32 * 1024];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    // block covers 256*NI/4... rows: instruction j -> rows 16*(wave*NI+j) + lane/4, chunk lane%4
    size_t rowbase = (size_t)blockIdx.x * 64 * NI;   // rows per block per iteration
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int j = 0; j < NI; ++j) {
            const size_t row = rowbase + (size_t)(wave * NI + j) * 16 + (lane >> 2);
            dma16(src + ((row * ROWB + (lane & 3) * 16) & mask), smem + ((wave * NI + j) * 1024) % (32 * 1024));
        }
        rowbase += (size_t)gridDim.x * 64 * NI;
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NI) : "memory");
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0 && smem[lane] == 123 && smem[1000] == 77) sink[0] = 1;
}

template <int NI>
__global__ __launch_bounds__(256) void vgpr_probe(const unsigned char* __restrict__ src, size_t mask, int iters,
                                                  int* sink) {
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    size_t off = ((size_t)blockIdx.x * 256 * NI * 16 + (size_t)wave * NI * 1024 + lane * 16) & mask;
    uint4 acc = {0, 0, 0, 0};
    for (int it = 0; it < iters; ++it) {
        uint4 v[NI];
#pragma unroll
        for (int j = 0; j < NI; ++j) v[j] = *reinterpret_cast<const uint4*>(src + ((off + j * 1024) & mask));
#pragma unroll
        for (int j = 0; j < NI; ++j) { acc.x ^= v[j].x; acc.y ^= v[j].y; acc.z ^= v[j].z; acc.w ^= v[j].w; }
        off = (off + (size_t)gridDim.x * 256 * NI * 16) & mask;
    }
    if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u) sink[0] = 1;
}


template <typename F>
static double run(F launch, double bytes) {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    launch();
    CK(hipEventRecord(e0, 0));
    for (int i = 0; i < 5; ++i) launch();
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    return bytes * 5 / (ms / 1e3) / 1e12;
}

int main() {
    const size_t big = (size_t)1 << 30;
    unsigned char* buf;
    int* sink;
    CK(hipMalloc(&buf, big));
    CK(hipMemset(buf, 1, big));
    CK(hipMalloc(&sink, 4));
    const int iters = 64;
    for (size_t span : {(size_t)1 << 21, (size_t)1 << 22, (size_t)1 << 23, (size_t)1 << 25, (size_t)1 << 27, (size_t)1 << 29, big}) {
        const size_t mask = span - 1;
        for (int wg_per_cu : {2}) {
            const int grid = 256 * wg_per_cu;
            const double bytes8 = (double)grid * 256 * 8 * 16 * iters;
            // LDS image 32 KB per workgroup (so 4 fit per CU)
            auto k8 = ldsdma_probe<8, 32>;
            auto k4 = ldsdma_probe<4, 32>;
            auto kr = vgpr_probe<8>;
            double d8 = run([&] { hipLaunchKernelGGL(k8, dim3(grid), dim3(256), 0, 0, buf, mask, iters, sink); }, bytes8);
            double d4 = run([&] { hipLaunchKernelGGL(k4, dim3(grid), dim3(256), 0, 0, buf, mask, iters, sink); }, bytes8 / 2);
            double r8 = run([&] { hipLaunchKernelGGL(kr, dim3(grid), dim3(256), 0, 0, buf, mask, iters, sink); }, bytes8);
            auto kf = frag_probe<8, 256>;
            // useful bytes: 64 B per row; the rows are 256 B apart
            double f8 = run([&] { hipLaunchKernelGGL(kf, dim3(grid), dim3(256), 0, 0, buf, mask, iters, sink); }, bytes8);
            printf("span %5zu MB  wg/CU %d:  lds-dma NI=8 %6.2f TB/s  NI=4 %6.2f TB/s   reg NI=8 %6.2f TB/s  frag(16x64B) %6.2f TB/s\n",
                   span >> 20, wg_per_cu, d8, d4, r8, f8);
        }
    }
    CK(hipDeviceSynchronize());
    return 0;
}
